"""Monitor's episode statistics at the drop-in boundary, pinned to the reference's own rewards.

SB3's Monitor wraps each HedgingEnv *inside* the VecEnv (train_ppo_v2.py:119): it appends
float(reward) of the env's own f64 step reward (hedging_env_v2.py:262,294) and reports
info["episode"] = {"r": round(sum, 6), "l": len, "t": ..., + info_keywords} on the step that
ends the episode.  The replay goldens hold the unmodified reference env's f64 rewards
(oracle/make_golden.py), so Monitor's "r" is round(sum of the golden rewards over the
episode, 6) exactly -- for HedgingVecEnv(monitor_keywords=...) and for DeviceVecNormalize's
device Monitor sums alike.
"""
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden_files
from oracle.hedging_oracle import load_golden

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

MON = ("per_share_step_pnl", "raw_pnl_deviation_abs", "transaction_costs_total")


def _venv(d, cfg, **kw):
    from cantorrl_amd.vec_env import HedgingVecEnv
    n = int(d["n_envs"])
    env = HedgingVecEnv(n, tables=(d["paths"], d["volatilities"], d["call_prices_atm"], d["put_prices_atm"]),
                        variant=int(d["variant"]), monitor_keywords=MON, **kw, **cfg)
    env.seed_envs([int(d["seed_base"]) + i for i in range(n)])
    return env


def _same(a, b):
    return a == b or (math.isnan(a) and math.isnan(b))


@pytest.mark.parametrize("fname", golden_files())
def test_monitor_episode_return_equals_reference_reward_sum(fname):
    """HedgingVecEnv (the SB3 NumPy path) over a reference golden: every finished episode's
    info["episode"]["r"] is round(sum of the reference's f64 rewards, 6), "l" its length, and
    each info keyword the reference's value on the terminal step."""
    cfg, d = load_golden(os.path.join(GOLDEN, fname))
    env = _venv(d, cfg, info_keys=MON)
    n = env.num_envs
    env.reset()
    acc = np.zeros(n)             # Monitor.rewards summed in step order (f64, as Python's sum)
    length = np.zeros(n, np.int64)
    finished = 0
    for s in range(int(d["n_steps"])):
        env.step_async(d["actions"][s])
        obs, rew, done, infos = env.step_wait()
        assert np.array_equal(done, d["terminated"][s]), s
        acc += d["reward"][s]
        length += 1
        for i in range(n):
            ep = infos[i].get("episode")
            if not done[i]:
                assert ep is None
                continue
            assert _same(ep["r"], round(float(acc[i]), 6)), (fname, s, i, ep["r"], acc[i])
            assert ep["l"] == length[i]
            for k in MON:
                assert _same(ep[k], float(d["info_" + k][s][i])), (fname, s, i, k)
            finished += 1
        acc[done] = 0.0
        length[done] = 0
    assert finished > 0
    env.close()


@pytest.mark.parametrize("fname", ["g1_v2_train.npz", "g1_v1_defaults.npz"])
@pytest.mark.parametrize("training", [True, False])
def test_device_vecnormalize_monitor_sums_equal_reference_reward_sum(fname, training):
    """DeviceVecNormalize's device Monitor sums (he_vecnorm_apply, or the eval step fused
    into he_step) over a reference golden: the episode return is the exact f64 sum of the
    reference's rewards (reported rounded to 6 decimals), the length its step count."""
    from cantorrl_amd.vec_normalize import DeviceVecNormalize
    cfg, d = load_golden(os.path.join(GOLDEN, fname))
    env = _venv(d, cfg, info_keys=(), return_numpy=False)
    vn = DeviceVecNormalize(env, training=training, norm_reward=training, gamma=0.99)
    n = env.num_envs
    vn.reset_tensors()
    acc = np.zeros(n)
    length = np.zeros(n, np.int64)
    finished = 0
    for s in range(int(d["n_steps"])):
        _, _, term, _ = vn.step_tensors(torch.from_numpy(d["actions"][s]).to(env.device), info=False)
        done = term.cpu().numpy().astype(bool)
        assert np.array_equal(done, d["terminated"][s]), s
        acc += d["reward"][s]
        length += 1
        if done.any():
            er, el = vn._ep_ret_done.cpu().numpy(), vn._ep_len_done.cpu().numpy()
            for i in np.nonzero(done)[0]:
                assert er[i] == acc[i] or (np.isnan(er[i]) and np.isnan(acc[i])), (fname, s, i, er[i], acc[i])
                assert el[i] == length[i]
                finished += 1
        acc[done] = 0.0
        length[done] = 0
    assert finished > 0
    vn.close()
