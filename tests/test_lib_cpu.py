"""CPU-side checks of libhedgeenv (no GPU): it loads, exports every symbol the
header declares, and its host builds of the RNG code match NumPy/gymnasium."""
import os
import re

import numpy as np
import pytest

from conftest import GOLDEN, REPO
from _compare import assert_same
from cantorrl_amd import _lib
from oracle.hedging_oracle import philox_words


def header_symbols():
    txt = open(os.path.join(REPO, "include", "hedge_env.h")).read()
    return sorted(set(re.findall(r"^\S[^;(]*?\b(he_\w+)\s*\(", txt, flags=re.M)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 18, syms
    for s in syms:
        assert hasattr(lib, s), f"libhedgeenv does not export {s}"
    assert set(syms) == set(_lib.EXPORTS)
    assert b"gfx950" in lib.he_version()


def test_library_is_gfx950_code_object():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_config_init_matches_reference_defaults():
    lib = _lib.load()
    c = _lib.HeConfig()
    assert lib.he_config_init(c, 2) == 0
    assert (c.transaction_cost_per_contract, c.lambda_cost, c.pnl_penalty_weight) == (0.65, 1.0, 0.01)
    assert (c.theta_weight, c.slippage_bps, c.initial_cash) == (0.0, 0.0, 0.0)
    assert (c.shares_to_hedge, c.max_contracts_held_per_type, c.max_trade_per_step) == (10000, 200, 15)
    assert c.record_metrics == 1 and c.loss_type == _lib.HE_LOSS_ABS
    assert c.option_tenor_years == 30 / 252 and c.risk_free_rate == 0.04
    assert lib.he_config_init(c, 1) == 0 and c.transaction_cost_per_contract == 0.05
    assert lib.he_config_init(c, 3) != 0


def test_create_rejects_bad_config_without_gpu():
    lib = _lib.load()
    c = _lib.HeConfig()
    lib.he_config_init(c, 2)
    c.max_contracts_held_per_type = 40000
    h = _lib.ctypes.c_void_p()
    st = lib.he_create(c, _lib.ctypes.byref(h))
    assert st == _lib.HE_EINVAL
    assert b"max_contracts_held_per_type" in lib.he_last_error(h)
    lib.he_destroy(h)


def test_create_rejects_bad_mark_without_gpu():
    """he_config.mark (ABI v3): an he_mark, and generate modes only (replay reads its marks
    from the table)."""
    lib = _lib.load()
    for mode, mark, msg in ((_lib.HE_MODE_GBM, 7, b"bad mark"),
                            (_lib.HE_MODE_REPLAY, _lib.HE_MARK_FIXED_EUROPEAN, b"replay mode")):
        c = _lib.HeConfig()
        lib.he_config_init(c, 2)
        assert c.mark == _lib.HE_MARK_ROLLING_ATM and c.abi_version == _lib.HE_ABI_VERSION == 4
        c.mode, c.mark = mode, mark
        h = _lib.ctypes.c_void_p()
        assert lib.he_create(c, _lib.ctypes.byref(h)) == _lib.HE_EINVAL
        assert msg in lib.he_last_error(h)
        lib.he_destroy(h)


@pytest.mark.parametrize("seed", [0, 1, 7, 42, 12345, 2 ** 32 - 1, 2 ** 32, 2 ** 40 + 3, 2 ** 63 + 11])
def test_pcg64_seed_state_matches_numpy(seed):
    st = np.random.PCG64(np.random.SeedSequence(seed)).state["state"]
    hi, lo, ihi, ilo = _lib.pcg64_seed_state(seed)
    assert (hi << 64) | lo == st["state"]
    assert (ihi << 64) | ilo == st["inc"]


def test_episode_draws_match_gymnasium_golden():
    z = np.load(os.path.join(GOLDEN, "g7_episode_index.npz"))
    for a, P in enumerate(z["P"]):
        for s in z["seeds"]:
            got = _lib.host_episode_draws(int(s), int(P), z["draws"].shape[2])
            assert_same(got, z["draws"][a, s], f"P={P} seed={s}")


def test_episode_draws_many_seeds_vs_numpy():
    for s in range(200):
        g = np.random.Generator(np.random.PCG64(np.random.SeedSequence(s)))
        exp = np.array([g.integers(100000) for _ in range(20)])
        assert_same(_lib.host_episode_draws(s, 100000, 20), exp, f"seed {s}")


def test_host_philox_matches_oracle_and_kat():
    # Random123 / rocRAND KAT: ctr=0, key=0
    assert _lib.host_philox(0, 0, 0) == (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)
    rng = np.random.default_rng(3)
    for _ in range(50):
        seed, g, n = (int(x) for x in rng.integers(0, 2 ** 62, 3))
        exp = tuple(int(np.asarray(w).item()) for w in philox_words(seed, g, n))
        assert _lib.host_philox(seed, g, n) == exp


@pytest.mark.parametrize("b", [10000.0, 252.0, 25.0 + 1e-9, 625.0 + 1e-9, 496.4800109863281 + 1e-9, 1.0, 3.0,
                               0.1, 7.5e-3])
def test_reciprocal_division_is_ieee_division(b):
    # step_kernel divides P&L by shares_to_hedge, the reward term by its constant
    # denominator and (T - t) by 252 through q + (a - b q) / b with q = a * RN(1/b)
    rng = np.random.default_rng(int(b * 1000) % 2 ** 32)
    a = np.concatenate([
        rng.standard_normal(200_000) * 10.0 ** rng.integers(-12, 12, 200_000),
        np.round(rng.uniform(-1e6, 1e6, 100_000), 2),             # cent-valued P&L
        np.arange(0, 253, dtype=np.float64),                       # T - t
        [0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, -5e-324, 1e-310, 1.7e308, -1.7e308],
    ])
    got = _lib.host_div_by(a, b)
    with np.errstate(over="ignore"):
        exp = a / b
    assert_same(got, exp, "div_by")
    assert np.array_equal(np.signbit(got), np.signbit(exp))


@pytest.mark.parametrize("b", [25.0, 496.48001098632812, 200.0, 252.0, 40.0, 7.0, 0.3, 1.99999988, 1e-3, 3e5])
def test_reciprocal_division_f32_is_ieee_division(b):
    # obs quotients by per-handle constants (max(S0, 25), max_contracts_held, T) go
    # through div_byf; tools/div_check.c checks all 2^32 numerators for the defaults
    b = np.float32(b)
    rng = np.random.default_rng(int(b * 1000) % 2 ** 32)
    bits = rng.integers(0, 2 ** 32, 1_000_000, dtype=np.uint64).astype(np.uint32)
    a = np.concatenate([
        bits.view(np.float32),
        np.arange(-400, 401, dtype=np.float32),                    # positions, T - t
        rng.uniform(0, 2000, 200_000).astype(np.float32),           # prices
        np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45, 1e-38, 3.4e38], np.float32),
    ])
    got = _lib.host_div_byf(a, b)
    with np.errstate(over="ignore", under="ignore", invalid="ignore"):
        exp = a / b
    assert_same(got, exp, "div_byf")
    assert np.array_equal(np.signbit(got), np.signbit(exp))


def test_box_muller_within_ulps_of_libm():
    # generate-mode normals: fast log/sincos (he_math.h box_muller) vs NumPy's
    # rad*cos(2 pi u2): the oracle's definition; the difference is the libm argument
    # rounding of 2*pi*u2 plus a few ulp
    rng = np.random.default_rng(1)
    k1 = rng.integers(0, 2 ** 52, 400_000, dtype=np.uint64)
    k2 = rng.integers(0, 2 ** 52, 400_000, dtype=np.uint64)
    u1 = np.concatenate([(k1.astype(np.float64) + 0.5) * 2.0 ** -52, [0.5 * 2.0 ** -52, 1 - 0.5 * 2.0 ** -52, 0.5]])
    u2 = np.concatenate([(k2.astype(np.float64) + 0.5) * 2.0 ** -52, [0.5 * 2.0 ** -52, 1 - 0.5 * 2.0 ** -52, 0.25]])
    z1, z2 = _lib.host_box_muller(u1, u2)
    rad = np.sqrt(-2.0 * np.log(u1))
    ang = 2.0 * np.pi * u2
    assert np.all(np.abs(z1 - rad * np.cos(ang)) <= 8 * np.spacing(rad))
    assert np.all(np.abs(z2 - rad * np.sin(ang)) <= 8 * np.spacing(rad))


def test_rocrand_oracle_equals_host_philox_and_numpy():
    """SURVEY 8(c)'s RNG oracle: rocRAND's own Philox4x32-10, host-compiled from its ROCm 7.2
    header (oracle/rocrand_words.cpp), equals libhedgeenv's host build and the NumPy
    restatement word for word over the whole 64-bit (seed, env id, step) range."""
    from _rng_oracles import coordinates, rocrand_words
    rng = np.random.default_rng(11)
    for seed in (0, 42, 2 ** 32 - 1, 2 ** 32, int(rng.integers(0, 2 ** 63)), 2 ** 64 - 1):
        gid, n = coordinates(rng, 4000)
        ref = rocrand_words(seed, gid, n)
        npw = np.stack([np.asarray(w, np.uint32) for w in philox_words(seed, gid, n)], axis=1)
        assert np.array_equal(ref, npw), seed
        for k in range(0, gid.size, 97):
            assert _lib.host_philox(seed, int(gid[k]), int(n[k])) == tuple(int(x) for x in ref[k])
    # the Random123 / rocRAND known answer
    assert tuple(rocrand_words(0, [0], [0])[0]) == (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)


def test_exp_k_within_one_ulp():
    """he_math.h exp_k (the generate-mode price-advance exp, SGPR-constant polynomial):
    within 1 ulp of numpy's exp everywhere on |x| < 700, equal to it on the large majority
    of GBM increments (rbergomi_sim.py:459-463 arguments)."""
    import ctypes
    lib = _lib.load()
    rng = np.random.default_rng(5)
    gbm = -0.5 * 0.029028 / 252 + np.sqrt(0.029028 / 252) * rng.standard_normal(400_000)
    wide = rng.uniform(-699.0, 699.0, 400_000)
    for x, max_diff in ((gbm, 0.05), (wide, 0.08)):
        x = np.ascontiguousarray(x)
        out = np.empty_like(x)
        assert lib.he_host_math(0, x.ctypes.data, x.size, out.ctypes.data) == 0
        ref = np.exp(x)
        ulp = np.abs(out.view(np.int64) - ref.view(np.int64))
        assert ulp.max() <= 1, ulp.max()
        assert (ulp != 0).mean() < max_diff, (ulp != 0).mean()
    # edge cases take the library exp
    x = np.array([0.0, -0.0, 700.5, -745.0, 709.7, np.inf, -np.inf], np.float64)
    out = np.empty_like(x)
    assert lib.he_host_math(0, x.ctypes.data, x.size, out.ctypes.data) == 0
    assert np.array_equal(out[:2], [1.0, 1.0])
    assert np.allclose(out[2:5], np.exp(x[2:5]), rtol=1e-15) and out[5] == np.inf and out[6] == 0.0


def test_lockstep_math_equals_scalar_forms():
    """he_math.h's lockstep forms (exp_k_n, bs_call_put_n, box_muller_n: what the LDS
    producers evaluate for 4 market slots at once) give the scalar functions' bits (what the
    tile kernels and the host run), including the arguments that leave the fast paths:
    |x| >= 700 and NaN for exp, S < 64 (log ratio outside the series) and NaN for the
    marks, u at the quadrant and octave edges for Box-Muller."""
    lib = _lib.load()
    rng = np.random.default_rng(11)

    def run(op, x):
        x = np.ascontiguousarray(x, np.float64)
        out = np.empty_like(x)
        assert lib.he_host_math(op, x.ctypes.data, x.size, out.ctypes.data) == 0
        return out

    xe = np.concatenate([rng.normal(0, 0.02, 40001), rng.uniform(-720, 720, 4000),
                         [700.0, -700.0, 699.999, np.nan, np.inf, -np.inf, 0.0, -0.0]])
    assert np.array_equal(run(1, xe).view(np.int64), run(0, xe).view(np.int64))
    S = np.concatenate([496.48 * np.exp(rng.normal(0, 0.2, 40001)), rng.uniform(0.01, 80, 4000),
                        [63.5, 64.0, 64.4, 500.5, 499.5, 1e-8, 1e6, np.nan]])
    a, b = run(3, S), run(2, S)
    assert np.array_equal(np.isnan(a), np.isnan(b))
    ok = ~np.isnan(b)
    assert np.array_equal(a[ok].view(np.int64), b[ok].view(np.int64))
    u = rng.random(2 * 30001)
    u[:8] = [0.125, 0.25, 0.5, 0.75, 1 - 2 ** -53, 2 ** -53, 0.70710678118654752, 0.5 + 2 ** -40]
    assert np.array_equal(run(5, u).view(np.int64), run(4, u).view(np.int64))


def test_step_signal_entry_points_reject_null_without_gpu():
    """he_step_signal / he_signal_seq / he_signal_wait (the host-mapped step's completion word):
    argument errors come back as status codes, with no handle and no GPU."""
    lib = _lib.load()
    flag = (_lib.ctypes.c_uint32 * 1)()
    assert lib.he_step_signal(None, _lib.ctypes.addressof(flag)) == _lib.HE_EINVAL
    assert lib.he_signal_seq(None) == 0
    assert lib.he_signal_wait(None, _lib.ctypes.addressof(flag), None) == _lib.HE_EINVAL
