"""cantorrl_amd: MI355X-native batched dynamic-hedging environment.

The hot path of bcosm/CantorRL (`HedgingEnv.step`, src/env/hedging_env_v2.py)
as HIP kernels behind a C ABI (include/hedge_env.h, libhedgeenv.so), with the
reference's Python interface on top:

* `HedgingVecEnv` -- N envs on one GPU, SB3 VecEnv interface (vec_env.py)
* `HedgingEnv`    -- the single-env gym API with the reference ctor (env.py)
"""
__version__ = "0.1.0"


def __getattr__(name):
    if name == "HedgingVecEnv":
        from .vec_env import HedgingVecEnv
        return HedgingVecEnv
    if name == "HedgingEnv":
        from .env import HedgingEnv
        return HedgingEnv
    raise AttributeError(name)
