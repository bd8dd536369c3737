"""DeviceVecNormalize (he_vecnorm_step / he_vecnorm_reset) against the SB3 2.6.0
restatement, on raw obs / rewards / dones produced by the env on the GPU."""
import numpy as np
import pytest
import torch

from oracle.vecnorm_oracle import VecNormalizeOracle

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
KW = dict(loss_type="abs", pnl_penalty_weight=0.001, lambda_cost=0.0001, theta_weight=0.0002, slippage_bps=1.0)
GEN = dict(s0=496.48001098632812, variance=0.029028, mu=0.04, dt=1 / 252, episode_length=12)


MON = ("per_share_step_pnl",)


def _env(n, monitor=True):
    """Monitor on: the step also writes the f64 reward (info reward_step) that Monitor sums."""
    from cantorrl_amd.vec_env import HedgingVecEnv
    return HedgingVecEnv(n, mode="gbm", generate=GEN, seed=7, device=DEV, return_numpy=False, info_keys=(),
                         monitor_keywords=MON if monitor else None, **KW)


def _run(n, steps, training=True, norm_reward=True, gamma=0.95):
    from cantorrl_amd.vec_normalize import DeviceVecNormalize
    env = _env(n)
    vn = DeviceVecNormalize(env, training=training, norm_reward=norm_reward, gamma=gamma)
    ref = VecNormalizeOracle(n, training=training, norm_reward=norm_reward, gamma=gamma, moments="f64")
    sb3 = VecNormalizeOracle(n, training=training, norm_reward=norm_reward, gamma=gamma, moments="sb3")
    obs = vn.reset_tensors()
    raw = env._obs.cpu().numpy()
    np.testing.assert_allclose(obs.cpu().numpy(), ref.reset(raw), rtol=0, atol=2e-6)
    sb3.reset(raw)
    rng = np.random.default_rng(0)
    for k in range(steps):
        a = torch.as_tensor(rng.uniform(-1, 1, size=(n, 2)).astype(np.float32), device=DEV)
        o, r, term, _ = vn.step_tensors(a)
        raw_o, raw_r = env._obs.cpu().numpy(), env._rew.cpu().numpy()
        raw_r64 = env._rew64.cpu().numpy()
        assert np.array_equal(raw_r, raw_r64.astype(np.float32))
        done = term.cpu().numpy().astype(bool)
        tobs = env._tobs.cpu().numpy()
        eo, er, et, eps = ref.step(raw_o, raw_r, done, tobs, env_rewards=raw_r64)
        so, sr, _, _ = sb3.step(raw_o, raw_r, done, tobs)
        np.testing.assert_allclose(o.cpu().numpy(), eo, rtol=0, atol=2e-6, err_msg=f"obs step {k}")
        np.testing.assert_allclose(r.cpu().numpy(), er.astype(np.float32), rtol=1e-6, atol=1e-7)
        # SB3's literal calls take the batch mean / var of the f32 obs in f32 (NumPy
        # reduces axis 0 row by row): that alone moves normalized values by up to ~1e-3
        # at n = 1000 (measured 6.3e-4) and by 0.17 at n = 70,000 -- SB3's own rounding,
        # which the f64 moments here do not have.  Compared at small n only; the f64
        # restatement above is the tight check.
        if n <= 4096:
            np.testing.assert_allclose(o.cpu().numpy(), so, rtol=0, atol=2e-3)
            np.testing.assert_allclose(r.cpu().numpy(), sr.astype(np.float32), rtol=1e-4, atol=1e-6)
        if done.any():
            to = vn.terminal_obs_tensor.cpu().numpy()
            erd, eld = vn._ep_ret_done.cpu().numpy(), vn._ep_len_done.cpu().numpy()
            for i, t in et.items():
                np.testing.assert_allclose(to[i], t, rtol=0, atol=2e-6)
                assert erd[i] == eps[i][0] and eld[i] == eps[i][1]
    rms, ret = vn.obs_rms, vn.ret_rms
    np.testing.assert_allclose(rms.mean, ref.obs_rms.mean, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(rms.var, ref.obs_rms.var, rtol=1e-8, atol=1e-14)
    assert abs(rms.count - ref.obs_rms.count) < 1e-6
    np.testing.assert_allclose(ret.var, ref.ret_rms.var, rtol=1e-9)
    np.testing.assert_allclose(vn.returns, ref.returns, rtol=1e-12, atol=1e-15)
    return vn


@pytest.mark.parametrize("n", [1000, 70000])
def test_device_vecnormalize_matches_restatement(n):
    _run(n, 30)


def test_device_vecnormalize_eval_mode_freezes_stats():
    vn = _run(512, 14, training=False, norm_reward=False)
    r = vn.obs_rms
    np.testing.assert_array_equal(r.mean, np.zeros(13))
    np.testing.assert_array_equal(r.var, np.ones(13))


def test_sb3_api_and_save_load(tmp_path):
    from cantorrl_amd.vec_env import HedgingVecEnv
    from cantorrl_amd.vec_normalize import DeviceVecNormalize
    env = HedgingVecEnv(64, mode="gbm", generate=GEN, seed=3, device=DEV,
                        monitor_keywords=("per_share_step_pnl",), **KW)
    vn = DeviceVecNormalize(env, gamma=0.9)
    obs = vn.reset()
    assert obs.shape == (64, 13) and obs.dtype == np.float32
    seen = 0
    for _ in range(13):
        obs, rew, done, infos = vn.step(np.zeros((64, 2), np.float32))
        for i in np.nonzero(done)[0]:
            ep = infos[i]["episode"]
            assert ep["l"] == 12 and "per_share_step_pnl" in ep
            assert infos[i]["terminal_observation"].shape == (13,)
            seen += 1
    assert seen == 64
    vn.save(str(tmp_path / "vn.npz"))
    vn2 = DeviceVecNormalize.load(str(tmp_path / "vn.npz"), env)
    np.testing.assert_array_equal(vn2.obs_rms.mean, vn.obs_rms.mean)
    np.testing.assert_array_equal(vn2.ret_rms.var, vn.ret_rms.var)
    o = vn.get_original_obs()
    np.testing.assert_allclose(vn.normalize_obs(o), np.clip((o - vn.obs_rms.mean) / np.sqrt(vn.obs_rms.var + 1e-8),
                                                            -10, 10).astype(np.float32))
    vn.close()


def test_stats_assignment_pkl_path_and_stale_infos(tmp_path):
    """`eval_env.obs_rms = train_env.obs_rms` (train_ppo_v2.py:208,309)
    copies the statistics in; save/load round-trip under the reference's ".pkl" names
    (train_ppo_v2.py:343-350,437-450); an info view read after later steps shows its own
    step."""
    import os
    from cantorrl_amd.vec_env import HedgingVecEnv
    from cantorrl_amd.vec_normalize import DeviceVecNormalize
    mk = lambda: HedgingVecEnv(32, mode="gbm", generate=dict(episode_length=6), seed=3,  # noqa: E731
                               info_keys=("call_contracts", "per_share_step_pnl"),
                               monitor_keywords=("per_share_step_pnl",), **KW)
    train, ev = DeviceVecNormalize(mk()), DeviceVecNormalize(mk(), training=False, norm_reward=False)
    train.reset()
    for _ in range(9):
        train.step(np.full((32, 2), 0.3, np.float32))
    ev.obs_rms = train.obs_rms
    ev.ret_rms = train.ret_rms
    np.testing.assert_array_equal(ev.obs_rms.mean, train.obs_rms.mean)
    np.testing.assert_array_equal(ev.obs_rms.var, train.obs_rms.var)
    assert ev.obs_rms.count == train.obs_rms.count and ev.ret_rms.var == train.ret_rms.var
    path = str(tmp_path / "final_vecnormalize.pkl")
    train.save(path)
    assert os.path.exists(path) and not os.path.exists(path + ".npz")
    back = DeviceVecNormalize.load(path, mk())
    np.testing.assert_array_equal(back.obs_rms.mean, train.obs_rms.mean)
    # infos of step t read after step t+1 (the actions move the positions every step)
    ev.reset()
    _, _, _, na = ev.step(np.full((32, 2), 1.0, np.float32))
    _, _, _, nb = ev.step(np.full((32, 2), 1.0, np.float32))
    assert na[3]["call_contracts"] == 15 and nb[3]["call_contracts"] == 30
    venv = ev.venv
    venv.reset()
    _, _, _, ia = venv.step(np.full((32, 2), 1.0, np.float32))
    _, _, _, ib = venv.step(np.full((32, 2), 1.0, np.float32))
    assert ia[5]["call_contracts"] == 15 and ib[5]["call_contracts"] == 30
    for e in (train, ev, back):
        e.close()


def test_info_views_freeze_lazily_and_generate_seeding_takes_one_seed():
    """a device-path info view costs no copy when it is read (or dropped)
    before the next step, and is frozen (still showing its own step) when it is not; in
    generate modes seed_envs takes exactly one seed instead of silently keeping seeds[0]."""
    from cantorrl_amd.vec_env import HedgingVecEnv
    from cantorrl_amd.vec_normalize import DeviceVecNormalize
    for wrap in (False, True):
        env = HedgingVecEnv(32, mode="gbm", generate=dict(episode_length=6), seed=3, device=DEV,
                            return_numpy=False, info_keys=("call_contracts",), **KW)
        e = DeviceVecNormalize(env) if wrap else env
        e.reset()
        one = torch.full((32, 2), 1.0, device=DEV)
        e.step_async(one)
        ra = e.step_wait()[3]
        assert ra[4]["call_contracts"] == 15 and ra._snap is None  # read live, no copy
        e.step_async(one)
        ka = e.step_wait()[3]           # kept, unread, across the next steps
        e.step_async(one)
        kb = e.step_wait()[3]
        assert ka._snap is not None and kb._snap is None
        e.step_async(one)
        e.step_wait()
        assert ka[4]["call_contracts"] == 30 and kb[4]["call_contracts"] == 45
        with pytest.raises(ValueError, match="one seed"):
            env.seed_envs([1, 2, 3])
        env.seed_envs([5])
        assert len(env.seed(11)) == 32 and env._pending_seeds == [11]
        env.reset()
        e.close()


def test_nonfinite_counter():
    """check_finite: he_count_nonfinite after each step counts non-finite obs/reward
    values on the device.  Replay tables with a NaN mark column (as the shipped
    paths_options.npz has at t = 1) produce them; clean tables do not."""
    from cantorrl_amd.vec_env import HedgingVecEnv
    rng = np.random.default_rng(0)
    P_, T1 = 8, 21
    S = 100 * np.exp(np.cumsum(rng.normal(0, 0.01, size=(P_, T1)), axis=1))
    v = np.full((P_, T1), 0.04)
    C = np.full((P_, T1 - 1), 2.0)
    Pu = np.full((P_, T1 - 1), 1.5)
    clean = HedgingVecEnv(16, tables=(S, v, C, Pu), device=DEV, seed=0, return_numpy=False, info_keys=(),
                          check_finite=True)
    C2 = C.copy()
    C2[:, 1] = np.nan
    dirty = HedgingVecEnv(16, tables=(S, v, C2, Pu), device=DEV, seed=0, return_numpy=False, info_keys=(),
                          check_finite=True)
    for e in (clean, dirty):
        e.reset_tensors()
        for _ in range(25):
            e.step_tensors(torch.zeros((16, 2), device=DEV))
    assert clean.nonfinite_count() == 0
    assert dirty.nonfinite_count() > 0
    clean.close()
    dirty.close()


@pytest.mark.parametrize("info", [False, True])
def test_fused_moments_equal_separate_launch(info, monkeypatch):
    """he_vecnorm_attach + he_vecnorm_apply (the moments in he_step's own launch, or after
    an info step in a separate one) against he_vecnorm_step: the same normalized obs and
    rewards to f32 rounding, the same statistics to 1e-12 (the sums' shift differs: the
    old running mean against the batch's row 0)."""
    from cantorrl_amd.vec_env import HedgingVecEnv
    from cantorrl_amd.vec_normalize import DeviceVecNormalize
    outs = []
    for fused in ("1", "0"):
        monkeypatch.setenv("CANTORRL_VN_FUSED", fused)
        env = HedgingVecEnv(3000, mode="gbm", generate=GEN, seed=11, device=DEV, return_numpy=False,
                            info_keys=("cash",) if info else (), monitor_keywords=MON if info else None, **KW)
        vn = DeviceVecNormalize(env, gamma=0.97)
        assert vn._fusable == (fused == "1")
        vn.reset_tensors()
        g = torch.Generator(device=DEV)
        g.manual_seed(3)
        got = []
        for k in range(30):
            a = torch.rand((3000, 2), device=DEV, generator=g) * 2 - 1
            o, r, t, _ = vn.step_tensors(a)
            got.append((o.clone(), r.clone()))
            if k == 12:  # eval steps in between detach and re-attach
                vn.training = False
                vn.step_tensors(a)
                vn.training = True
        torch.cuda.synchronize()
        outs.append((got, vn.obs_rms, vn.ret_rms, vn.returns.copy()))
        vn.close()
    (ga, ra, qa, ta), (gb, rb, qb, tb) = outs
    for k, ((oa, wa), (ob, wb)) in enumerate(zip(ga, gb)):
        torch.testing.assert_close(oa, ob, rtol=0, atol=2e-6, msg=f"obs step {k}")
        torch.testing.assert_close(wa, wb, rtol=1e-6, atol=1e-7, msg=f"reward step {k}")
    np.testing.assert_allclose(ra.mean, rb.mean, rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(ra.var, rb.var, rtol=1e-10, atol=1e-16)
    np.testing.assert_allclose(qa.var, qb.var, rtol=1e-10)
    np.testing.assert_array_equal(ta, tb)


@pytest.mark.parametrize("info,norm_reward,n", [(False, False, 3000), (False, True, 70000), (True, False, 700),
                                                (True, True, 70000)])
def test_fused_eval_step_equals_separate_launch(info, norm_reward, n, monkeypatch):
    """he_vecnorm_attach_eval (the whole eval VecNormalize step inside he_step's launch, or
    he_vecnorm_apply run by he_step itself after an info step) against he_step +
    he_vecnorm_step with the statistics frozen: obs, rewards, normalized terminal obs,
    Monitor sums and returns bit for bit (the same per-element arithmetic), over episode
    ends (T = 12) and a partial last workgroup (n = 700, 70000).  Monitor is on: the fused
    launch (info=False) adds the f64 reward from its registers, the separate launch reads the
    step's info reward_step -- the same sums."""
    from cantorrl_amd.vec_env import HedgingVecEnv
    from cantorrl_amd.vec_normalize import DeviceVecNormalize
    outs = []
    for fused in ("1", "0"):
        monkeypatch.setenv("CANTORRL_VN_FUSED", fused)
        env = HedgingVecEnv(n, mode="gbm", generate=GEN, seed=11, device=DEV, return_numpy=False,
                            info_keys=("cash",) if info else (), monitor_keywords=MON, **KW)
        vn = DeviceVecNormalize(env, gamma=0.97, norm_reward=norm_reward)
        vn.reset_tensors()
        g = torch.Generator(device=DEV)
        g.manual_seed(5)
        for k in range(6):   # training steps: non-trivial statistics and returns
            vn.step_tensors(torch.rand((n, 2), device=DEV, generator=g) * 2 - 1)
        vn.training = False
        got = []
        for k in range(26):
            o, r, t, _ = vn.step_tensors(torch.rand((n, 2), device=DEV, generator=g) * 2 - 1, info=info)
            m = t.bool()
            got += [o.clone(), r.clone(), t.clone(), vn.terminal_obs_tensor[m].clone(), vn._ep_ret.clone(),
                    vn._ep_len.clone(), vn._ep_ret_done.clone(), vn._ep_len_done.clone(), vn._returns.clone()]
        torch.cuda.synchronize()
        outs.append(got)
        vn.close()
    for k, (a, b) in enumerate(zip(*outs)):
        assert torch.equal(a, b), k


def test_two_wrappers_on_one_env_and_inner_steps():
    """the fused moments are armed per step (he_vecnorm_attach is one-shot).
    Two DeviceVecNormalize on one env, the first dropped after the second has stepped, and
    the inner env stepped directly in between: each wrapper's returns and statistics equal
    a wrapper that alone saw exactly its own steps (the separate-launch path)."""
    import gc
    from cantorrl_amd.vec_normalize import DeviceVecNormalize
    n = 2000
    g = torch.Generator(device=DEV)
    g.manual_seed(5)
    acts = [torch.rand((n, 2), device=DEV, generator=g) * 2 - 1 for _ in range(12)]

    def drive(env, wrappers, plan):
        # plan: ("a" | "b" | "inner", action index); returns the last normalized outputs per wrapper
        for who, k in plan:
            if who == "inner":
                env.step_tensors(acts[k])
            else:
                wrappers[who].step_tensors(acts[k])
        torch.cuda.synchronize()

    plan = [("a", 0), ("b", 1), ("inner", 2), ("a", 3), ("b", 4), ("b", 5), ("inner", 6), ("b", 7)]
    env = _env(n)
    a, b = DeviceVecNormalize(env, gamma=0.9), DeviceVecNormalize(env, gamma=0.8)
    a.reset_tensors()
    b._returns.zero_()
    drive(env, {"a": a, "b": b}, plan[:5])
    ra = a.returns.copy()
    del a
    gc.collect()
    drive(env, {"b": b}, plan[5:])
    rb, sb = b.returns.copy(), b.obs_rms
    env.close()
    # the same env trajectory with separate-launch wrappers (nothing fused, nothing shared)
    import os
    os.environ["CANTORRL_VN_FUSED"] = "0"
    try:
        env2 = _env(n)
        a2, b2 = DeviceVecNormalize(env2, gamma=0.9), DeviceVecNormalize(env2, gamma=0.8)
        a2.reset_tensors()
        b2._returns.zero_()
        drive(env2, {"a": a2, "b": b2}, plan)
        np.testing.assert_allclose(ra, a2.returns, rtol=1e-12, atol=1e-15)  # a stepped at 0 and 3 only
        np.testing.assert_allclose(rb, b2.returns, rtol=1e-12, atol=1e-15)
        np.testing.assert_allclose(sb.mean, b2.obs_rms.mean, rtol=1e-12, atol=1e-14)
        np.testing.assert_allclose(sb.var, b2.obs_rms.var, rtol=1e-10, atol=1e-16)
        assert abs(sb.count - b2.obs_rms.count) < 1e-9
        env2.close()
    finally:
        del os.environ["CANTORRL_VN_FUSED"]


@pytest.mark.parametrize("fused", ["1", "0"])
def test_zero_epsilon_constant_column_clips(fused, monkeypatch):
    """epsilon = 0 with a zero variance (a constant column) makes 1/sqrt(var + eps)
    infinite.  Every element of that column is then (x - mean) / 0 = +-inf, clipped to
    +-clip_obs as SB3's f64 expression does -- not NaN (the f32 split terms were inf - inf);
    the other columns keep their normalization.  Eval arm fused into he_step and the separate
    apply launch."""
    from cantorrl_amd.vec_env import HedgingVecEnv
    from cantorrl_amd.vec_normalize import DeviceVecNormalize, _RmsView
    monkeypatch.setenv("CANTORRL_VN_FUSED", fused)
    n = 300
    env = HedgingVecEnv(n, mode="gbm", generate=GEN, seed=4, device=DEV, return_numpy=False, info_keys=(), **KW)
    vn = DeviceVecNormalize(env, training=False, norm_reward=False, epsilon=0.0)
    mean, var = np.zeros(13), np.ones(13)
    mean[0], var[0] = 1000.0, 0.0      # no obs equals the mean: every element clips to -10
    mean[5], var[5] = -1000.0, 0.0     # ... to +10
    vn.obs_rms = _RmsView(mean, var, 10.0)
    vn.reset_tensors()
    for _ in range(3):
        o, _, _, _ = vn.step_tensors(torch.zeros((n, 2), device=DEV))
    got = o.cpu().numpy()
    raw = env._obs.cpu().numpy()
    assert np.isfinite(got).all()
    assert (got[:, 0] == -10.0).all() and (got[:, 5] == 10.0).all()
    rest = [c for c in range(13) if c not in (0, 5)]
    exp = np.clip((raw[:, rest] - mean[rest]) / np.sqrt(var[rest]), -10, 10)
    np.testing.assert_allclose(got[:, rest], exp, rtol=0, atol=2e-6)
    vn.close()
