"""VecNormalize oracle (SB3 2.6.0 restatement) properties and the C ABI entry checks
that run without a GPU."""
import ctypes

import numpy as np

from oracle.vecnorm_oracle import RunningMeanStd, VecNormalizeOracle


def test_running_mean_std_merges_like_concatenation():
    rng = np.random.default_rng(0)
    batches = [rng.normal(3.0, 2.0, size=(n, 4)) for n in (5, 17, 64, 1)]
    r = RunningMeanStd(epsilon=1e-12, shape=(4,), moments="f64")
    for b in batches:
        r.update(b)
    allx = np.concatenate(batches)
    np.testing.assert_allclose(r.mean, allx.mean(axis=0), rtol=1e-12)
    np.testing.assert_allclose(r.var, allx.var(axis=0), rtol=1e-9)
    assert abs(r.count - len(allx)) < 1e-9


def test_sb3_moments_are_f32_batch_statistics():
    """moments='sb3' keeps NumPy's f32 batch mean/var of f32 obs (SB3's literal calls)."""
    rng = np.random.default_rng(1)
    obs = rng.normal(1.0, 0.01, size=(4096, 13)).astype(np.float32)
    a = RunningMeanStd(shape=(13,), moments="sb3")
    b = RunningMeanStd(shape=(13,), moments="f64")
    a.update(obs)
    b.update(obs)
    np.testing.assert_allclose(a.mean, b.mean, rtol=1e-5)
    np.testing.assert_allclose(a.var, b.var, rtol=1e-2)


def test_vecnormalize_oracle_step_semantics():
    rng = np.random.default_rng(2)
    n = 8
    vn = VecNormalizeOracle(n, obs_dim=3, gamma=0.9)
    o0 = rng.normal(size=(n, 3)).astype(np.float32)
    out = vn.reset(o0)
    assert out.dtype == np.float32 and np.all(np.abs(out) <= 10.0)
    rew = rng.normal(size=n).astype(np.float32)
    done = np.zeros(n, bool)
    done[3] = True
    o1 = rng.normal(size=(n, 3)).astype(np.float32)
    obs_n, rew_n, tobs_n, eps = vn.step(o1, rew, done, terminal_obs=o1)
    assert set(tobs_n) == {3} and set(eps) == {3}
    assert eps[3] == (float(rew[3]), 1)
    # Monitor sums the envs' own f64 rewards when given (train_ppo_v2.py:119: Monitor wraps
    # each env inside the VecEnv), not the VecEnv's f32 buffer
    vn2 = VecNormalizeOracle(n, obs_dim=3, gamma=0.9)
    vn2.reset(o0)
    env_rew = rew.astype(np.float64) + 1e-9   # not representable in f32
    _, _, _, eps2 = vn2.step(o1, rew, done, terminal_obs=o1, env_rewards=env_rew)
    assert eps2[3] == (env_rew[3], 1) and eps2[3][0] != float(rew[3])
    assert vn.returns[3] == 0.0 and vn.returns[0] == rew[0]
    # frozen statistics in eval mode
    vn.training = False
    m = vn.obs_rms.mean.copy()
    vn.step(o1, rew, done)
    np.testing.assert_array_equal(vn.obs_rms.mean, m)


def test_vecnorm_abi_rejects_bad_arguments():
    from cantorrl_amd import _lib
    lib = _lib.load()
    assert lib.he_vecnorm_stats_len(13) == 30
    assert lib.he_vecnorm_scratch_bytes(1 << 20, 13) > 0
    p = _lib.HeVecnormParams()
    p.obs_dim, p.gamma, p.clip_obs, p.clip_reward, p.epsilon = 13, 0.99, 10.0, 10.0, 1e-8
    assert lib.he_vecnorm_step(ctypes.byref(p), 0, *([None] * 15), None) == _lib.HE_OK      # n = 0: no-op
    assert lib.he_vecnorm_step(ctypes.byref(p), 4, *([None] * 15), None) == _lib.HE_EINVAL  # NULL buffers
    # Monitor buffers without the f64 rewards they sum: refused before anything is launched
    fake = [ctypes.c_void_p(4096)] * 14
    for fn in (lib.he_vecnorm_step, lib.he_vecnorm_apply):
        assert fn(ctypes.byref(p), 4, *fake, None, None) == _lib.HE_EINVAL
    p.obs_dim = 7
    assert lib.he_vecnorm_reset(ctypes.byref(p), 4, *([None] * 5), None) == _lib.HE_EINVAL
    assert lib.he_vecnorm_init(None, 13, None) == _lib.HE_EINVAL
