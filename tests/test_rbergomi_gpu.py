"""rBergomi generator on the GPU: the HIP kernels fed the reference's own draws
against the reference goldens, and the Philox path through size-independent
properties (Black-Scholes limit, sharding identity, determinism, NPZ replay)."""
import math
import os

import numpy as np
import pytest

from oracle import rbergomi_oracle as orc

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
DEV = "cuda:0"

# Tolerances.  Same draws, same algorithm, different f64 libm (device exp / pow /
# sqrt vs glibc), a direct convolution in place of two FFTs and the option price
# chain in log space: ~1e-15 relative per value, ~1e-13 after 252 chained price
# steps.  MC marks are means of max(S - K, 0) over 8-48 paths, where a 1e-13 change
# of S moves a near-the-money payoff by 1e-13 S absolute: an absolute floor of
# 1e-10 S0.
PATH_RTOL = 1e-12
MARK_RTOL = 1e-10


def _rb():
    from cantorrl_amd import rbergomi
    return rbergomi


def _history():
    # data/historical_prices.csv of the reference, as recorded in the golden file
    return np.load(os.path.join(GOLD, "rb_estimate.npz"))["hist__prices"]


def _bs(S, K, T, r, sig):
    d1 = (math.log(S / K) + (r + 0.5 * sig * sig) * T) / (sig * math.sqrt(T))
    d2 = d1 - sig * math.sqrt(T)
    N = lambda x: 0.5 * math.erfc(-x / math.sqrt(2))  # noqa: E731
    c = S * N(d1) - K * math.exp(-r * T) * N(d2)
    return c, c - S + K * math.exp(-r * T)


@pytest.fixture(params=["valu", "mfma"])
def mc_kernel_kind(request, monkeypatch):
    """The reference-draw parity through both MC pricers of the reference tenor."""
    monkeypatch.setenv("RB_MC_MFMA", "1" if request.param == "mfma" else "0")
    return request.param


def test_pricer_reference_draws_match_golden(mc_kernel_kind):
    rb = _rb()
    g = np.load(os.path.join(GOLD, "rb_price.npz"))
    S0, K, xi, H, eta, rho = (g[k] for k in ("S0", "K", "xi", "H", "eta", "rho"))
    n_mc, seed = int(g["n_mc"]), int(g["seed"])
    for i, T in enumerate(g["tenors"]):
        d = orc.ReferenceDraws(seed + i)
        n = int(T / orc.DT)
        Wc = Wp = np.zeros((len(S0), n_mc, 2, 2))
        if n > 0:
            Mo = orc.next_pow2(n + 1)
            Wc = orc.z_to_w(d.complex_normal((len(S0), n_mc, Mo)))
            Wp = orc.z_to_w(d.complex_normal((len(S0), n_mc, Mo)))
        for kind, W in (("call", Wc), ("put", Wp)):
            got = rb.price_rbergomi_option(S0, K, T, orc.R, xi, H, eta, rho, kind, n_mc, orc.DT, device=DEV, W=W)
            ref = g[f"{kind}_{i}"]
            np.testing.assert_allclose(got.cpu().numpy(), ref, rtol=MARK_RTOL, atol=1e-10 * S0.max(),
                                       err_msg=f"{kind} tenor {T}")


def test_generator_reference_draws_match_golden(mc_kernel_kind):
    """Every stage fed the draws the reference consumed: params from the unit
    normals, paths from W_main, and each day's marks from that day's W (call, put)."""
    import torch
    rb = _rb()
    g = np.load(os.path.join(GOLD, "rb_generate.npz"))
    P, n_mc, seed = int(g["num_paths"]), int(g["n_mc"]), int(g["seed"])
    base = tuple(g["base"])
    d = orc.ReferenceDraws(seed)
    unit = np.stack([d.normal(0.0, 1.0, P) for _ in range(5)])
    Zm = d.complex_normal((P, 256))
    cfg = rb.make_config(P, seed=seed)
    params = rb.sample_params(cfg, base, DEV, unit_normals=unit)
    ref_params = np.stack(orc.perturb_params(base, [s * u for s, u in zip(orc.PERTURB_STD, unit)]))
    np.testing.assert_array_equal(params.cpu().numpy(), ref_params)
    paths, vol = rb.simulate_paths(cfg, params, DEV, W=orc.z_to_w(Zm))
    np.testing.assert_allclose(vol.cpu().numpy(), g["volatilities"], rtol=PATH_RTOL, atol=0)
    np.testing.assert_allclose(paths.cpu().numpy(), g["paths"], rtol=PATH_RTOL, atol=0)
    # marks: day j prices at S_{j-1}, K = round(S_{j-1}), xi = v_{j-1} (:404-451)
    d = orc.ReferenceDraws(seed)
    T = 252
    Wc = np.zeros((T, P, n_mc, 32, 2))
    Wp = np.zeros_like(Wc)
    for j in range(T):
        Wc[j] = orc.z_to_w(d.complex_normal((P, n_mc, 32)))
        Wp[j] = orc.z_to_w(d.complex_normal((P, n_mc, 32)))
    S = paths[:, :T].T.reshape(-1)          # day-major, as the W arrays
    v = vol[:, :T].T.reshape(-1)
    pr = params.cpu().numpy()
    rep = lambda x: np.tile(x, T)           # noqa: E731
    for kind, W, key in (("call", Wc, "call_prices_atm"), ("put", Wp, "put_prices_atm")):
        got = rb.price_rbergomi_option(S, torch.round(S), orc.T_OPTION_TENOR, orc.R, v, rep(pr[2]), rep(pr[3]),
                                       rep(pr[4]), kind, n_mc, orc.DT, device=DEV, W=W.reshape(T * P, n_mc, 32, 2))
        got = got.cpu().numpy().reshape(T, P).T
        np.testing.assert_allclose(got, g[key], rtol=MARK_RTOL, atol=1e-10 * g["paths"].max(), err_msg=key)


def test_pricer_edge_inputs_follow_reference(mc_kernel_kind):
    """S0 <= 0, xi < 0 and NaN inputs through the oracle restatement (same draws)."""
    rb = _rb()
    rng = np.random.default_rng(4)
    S0 = np.array([0.0, -5.0, 100.0, np.nan, 1e-9, 50.0])
    K = np.array([1.0, 1.0, 100.0, 100.0, 0.0, 50.0])
    xi = np.array([0.04, 0.04, -0.01, 0.04, 0.04, 0.0])
    H = np.full(6, 0.2)
    eta = np.full(6, 1.5)
    rho = np.full(6, -0.5)
    Z = rng.normal(size=(6, 16, 32)) + 1j * rng.normal(size=(6, 16, 32))
    for kind in ("call", "put"):
        ref = orc.price_options(S0, K, 30 / 252, 0.04, xi, H, eta, rho, kind, Z, 1 / 252)
        got = rb.price_rbergomi_option(S0, K, 30 / 252, 0.04, xi, H, eta, rho, kind, 16, 1 / 252, device=DEV,
                                       W=orc.z_to_w(Z)).cpu().numpy()
        np.testing.assert_allclose(got, ref, rtol=MARK_RTOL, atol=1e-12, equal_nan=True, err_msg=kind)


@pytest.mark.parametrize("normals", ["f64", "f32"])
def test_pricer_philox_black_scholes_limit(normals):
    """eta -> 0 freezes the variance at xi: the Euler step is then exact GBM, so the
    MC price converges to Black-Scholes.  200k paths: 4 standard errors."""
    rb = _rb()
    n_mc = 200000
    S0 = np.array([100.0, 100.0, 496.48, 80.0])
    K = np.array([100.0, 105.0, 496.0, 90.0])
    xi = np.array([0.04, 0.09, 0.029, 0.01])
    T = 30 / 252
    for kind, col in (("call", 0), ("put", 1)):
        got = rb.price_rbergomi_option(S0, K, T, 0.04, xi, np.full(4, 0.3), np.full(4, 1e-9), np.full(4, -0.7),
                                       kind, n_mc, 1 / 252, device=DEV, normals=normals).cpu().numpy()
        for i in range(4):
            want = _bs(S0[i], K[i], T, 0.04, math.sqrt(xi[i]))[col]
            se = S0[i] * math.sqrt(xi[i] * T) / math.sqrt(n_mc)   # payoff sd <= S sigma sqrt(T)
            assert abs(got[i] - want) < 4 * se, (kind, i, got[i], want, se)


def test_generate_shards_equal_rows_and_is_deterministic():
    rb = _rb()
    hist = _history()
    kw = dict(n_mc=64, device=DEV, seed=9)
    full = rb.generate_paths_and_options(hist, 8, **kw)
    part = rb.generate_paths_and_options(hist, 3, path_offset=5, **kw)
    again = rb.generate_paths_and_options(hist, 8, **kw)
    for k in ("params", "paths", "volatilities", "call_prices_atm", "put_prices_atm"):
        a, b = full[k].cpu().numpy(), part[k].cpu().numpy()
        sub = a[:, 5:8] if k == "params" else a[5:8]
        np.testing.assert_array_equal(sub, b, err_msg=k)
        np.testing.assert_array_equal(a, again[k].cpu().numpy(), err_msg=k)


def test_generate_properties():
    import torch
    rb = _rb()
    hist = _history()
    res = rb.generate_paths_and_options(hist, 256, n_mc=512, device=DEV)
    base = np.array(res["base_params"])
    np.testing.assert_allclose(base, orc.estimate_base_params(hist), rtol=1e-12)
    S, v = res["paths"], res["volatilities"]
    C, Pp = res["call_prices_atm"], res["put_prices_atm"]
    assert S.shape == (256, 253) and C.shape == (256, 252)
    for t in (S, v, C, Pp):
        assert bool(torch.isfinite(t).all())
    assert bool((S >= 1e-8).all()) and bool((v > 0).all()) and bool((C >= 0).all()) and bool((Pp >= 0).all())
    pr = res["params"].cpu().numpy()
    assert (pr[2] >= 0.01).all() and (pr[2] <= 0.49).all() and (pr[4] >= -0.99).all() and (pr[4] <= -0.01).all()
    np.testing.assert_array_equal(S[:, 0].cpu().numpy(), pr[0])
    # ATM marks: C - P against S - K e^{-rT}, a loose check (independent MC draws
    # for C and P, and the reference's scheme is not an exact martingale)
    Sd = S[:, :252]
    par = (C - Pp - (Sd - torch.round(Sd) * math.exp(-0.04 * 30 / 252))) / Sd
    assert abs(float(par.mean())) < 1e-3 and float(par.abs().max()) < 0.05
    # the perturbed S0 are N(S0 base, 1 %)
    assert abs(pr[0].mean() / base[0] - 1) < 0.01 * 4 / 16


def test_npz_round_trip_into_replay_env(tmp_path):
    from cantorrl_amd.vec_env import HedgingVecEnv
    rb = _rb()
    res = rb.generate_paths_and_options(_history(), 16, n_mc=32, device=DEV)
    f = tmp_path / "rb.npz"
    rb.save_npz(str(f), res)
    z = np.load(f)
    assert set(z.files) == {"paths", "volatilities", "call_prices_atm", "put_prices_atm"}
    assert z["paths"].dtype == np.float64 and z["call_prices_atm"].shape == (16, 252)
    env = HedgingVecEnv(4, str(f), device=DEV, seed=0)
    obs = env.reset()
    assert obs.shape == (4, 13)
    for _ in range(3):
        obs, rew, done, _info = env.step(np.zeros((4, 2), np.float32))
    assert np.isfinite(obs).all() and np.isfinite(rew).all()
    env.close()


def test_inf_on_generated_dataset(tmp_path):
    """src/agents/test_inf.py on our own rBergomi data: the v1 env with its parameters
    (tcpc 0.05, lambda 1.0, 10,000 shares, 200 contracts) replays the generated NPZ
    under random actions; every reward and obs stays finite (here 2,048 envs x 600
    steps = 1.2M env-steps instead of 10k)."""
    import torch
    from cantorrl_amd.vec_env import HedgingVecEnv
    rb = _rb()
    res = rb.generate_paths_and_options(_history(), 64, n_mc=256, device=DEV, seed=5)
    f = tmp_path / "paths_rbergomi_options.npz"
    rb.save_npz(str(f), res)
    env = HedgingVecEnv(2048, str(f), variant=1, device=DEV, seed=0, return_numpy=False, info_keys=(), check_finite=True,
                        transaction_cost_per_contract=0.05, lambda_cost=1.0, shares_to_hedge=10_000,
                        max_contracts_held_per_type=200)
    env.reset_tensors()
    g = torch.Generator(device=DEV).manual_seed(1)
    bad = 0
    for _ in range(600):
        a = torch.rand((2048, 2), generator=g, device=DEV) * 2 - 1
        obs, rew, term, _ = env.step_tensors(a)
        bad += int((~torch.isfinite(rew)).sum()) + int((~torch.isfinite(obs)).sum())
    assert env.nonfinite_count() == 0      # the device-side counter agrees
    env.close()
    assert bad == 0


def test_chunked_mark_launches_equal_a_shard():
    """rb_price_atm_marks launches 8,192 paths at a time: rows on both sides of the
    chunk boundary equal the same rows generated as a small shard."""
    rb = _rb()
    kw = dict(n_mc=2, device=DEV, seed=13)
    big = rb.generate_paths_and_options(_history(), 8200, **kw)
    part = rb.generate_paths_and_options(_history(), 12, path_offset=8186, **kw)
    for k in ("call_prices_atm", "put_prices_atm", "paths"):
        np.testing.assert_array_equal(big[k][8186:8198].cpu().numpy(), part[k].cpu().numpy(), err_msg=k)


def test_mc_box_muller_extreme_uniforms():
    """the MC pricer's Box-Muller (rbergomi.hip mc_box_muller: v_rcp_f64 + Newton,
    x rsq(x) + Newton) over the whole range u01 produces, [2^-53, 1 - 2^-53] -- the ends
    included, where -2 log u is 73.5 and 2.2e-16 -- against the f64 formula
    sqrt(-2 log u1) (cos, sin)(2 pi u2) on the host: finite everywhere, within 1e-13 relative
    of the radius (the tests of the distribution hold the rest)."""
    import torch
    rb = _rb()
    lib = rb.load()
    lo, hi = 2.0 ** -53, 1.0 - 2.0 ** -53
    rng = np.random.default_rng(3)
    u1 = np.concatenate([[lo, hi, hi, 0.5, 0.70710678118654752, 0.7071067811865476], np.nextafter(hi, 0) - rng.uniform(0, 1e-12, 32),
                         lo * (1 + rng.uniform(0, 8, 32)), rng.uniform(lo, hi, 4000)])
    u2 = np.concatenate([[0.25, 0.0, hi, lo, 0.5, 0.125], rng.uniform(0, 1, u1.size - 6)])
    d = [torch.as_tensor(x, device=DEV) for x in (u1, u2)]
    z1, z2 = torch.empty_like(d[0]), torch.empty_like(d[0])
    st = lib.rb_device_mc_box_muller(d[0].data_ptr(), d[1].data_ptr(), u1.size, z1.data_ptr(), z2.data_ptr(),
                                     torch.cuda.current_stream().cuda_stream)
    assert st == 0, lib.rb_last_error()
    g1, g2 = z1.cpu().numpy(), z2.cpu().numpy()
    assert np.isfinite(g1).all() and np.isfinite(g2).all()
    r = np.sqrt(-2.0 * np.log(u1))
    np.testing.assert_allclose(np.hypot(g1, g2), r, rtol=1e-13, atol=0)
    e1, e2 = r * np.cos(2 * np.pi * u2), r * np.sin(2 * np.pi * u2)
    np.testing.assert_allclose(g1, e1, rtol=0, atol=1e-13 * r.max())
    np.testing.assert_allclose(g2, e2, rtol=0, atol=1e-13 * r.max())


@pytest.mark.parametrize("normals", ["f64", "f32"])
def test_mfma_pricer_equals_valu_pricer(normals, monkeypatch):
    """The reference tenor's MC pricer on the matrix cores (mc_mfma_kernel, RB_MC_MFMA=1: the
    fractional convolution as v_mfma_f64_16x16x4_f64, the Euler chain composed over 4 lanes)
    against mc_kernel (the default) on the same Philox normals: the same marks up to the summation
    order (~1e-16 relative per value); n_mc = 1000 leaves a partial last tile of paths, and the
    ATM generator (rb_price_atm_marks) is compared too."""
    rb = _rb()
    rng = np.random.default_rng(11)
    n = 40
    S0 = rng.uniform(50, 600, n)
    S0[:3] = (0.0, -1.0, 1e-9)
    K = np.round(S0 * rng.uniform(0.9, 1.1, n))
    xi = rng.uniform(0.005, 0.09, n)
    H, eta, rho = rng.uniform(0.03, 0.45, n), rng.uniform(0.5, 3.0, n), rng.uniform(-0.95, -0.05, n)
    hist = _history()
    out = {}
    for valu in ("0", "1"):
        monkeypatch.setenv("RB_MC_MFMA", "1" if valu == "0" else "0")
        got = [rb.price_rbergomi_option(S0, K, 30 / 252, 0.04, xi, H, eta, rho, kind, 1000, 1 / 252, device=DEV,
                                        normals=normals, seed=21).cpu().numpy() for kind in ("call", "put")]
        res = rb.generate_paths_and_options(hist, 6, n_mc=300, device=DEV, seed=3, normals=normals)
        out[valu] = got + [res["call_prices_atm"].cpu().numpy(), res["put_prices_atm"].cpu().numpy()]
    for a, b in zip(out["0"], out["1"]):
        assert np.isfinite(a).all()
        np.testing.assert_allclose(a, b, rtol=1e-11, atol=1e-11 * 600)
