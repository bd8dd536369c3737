"""rBergomi generator, CPU side: the oracle against the reference goldens, the C++
estimator against the same goldens, the W-form identity the kernels rely on, and
the library's exports / config validation (no GPU calls)."""
import ctypes
import os

import numpy as np
import pytest

from oracle import rbergomi_oracle as orc

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    return np.load(os.path.join(GOLD, name))


# ------------------------------------------------------------------ oracle pinned
def test_oracle_estimator_matches_reference():
    g = _load("rb_estimate.npz")
    for name in g["names"]:
        p = g[f"{name}__prices"]
        base = np.array([float(x) for x in orc.estimate_base_params(p, 1 / 252)])
        np.testing.assert_array_equal(base, g[f"{name}__base"], err_msg=str(name))


def test_oracle_pricer_matches_reference_bitwise():
    g = _load("rb_price.npz")
    S0, K, xi, H, eta, rho = (g[k] for k in ("S0", "K", "xi", "H", "eta", "rho"))
    n_mc, seed = int(g["n_mc"]), int(g["seed"])
    for i, T in enumerate(g["tenors"]):
        d = orc.ReferenceDraws(seed + i)
        n = int(T / orc.DT)
        zc = zp = None
        if n > 0:
            Mo = orc.next_pow2(n + 1)
            zc = d.complex_normal((len(S0), n_mc, Mo))
            zp = d.complex_normal((len(S0), n_mc, Mo))
        np.testing.assert_array_equal(orc.price_options(S0, K, T, orc.R, xi, H, eta, rho, "call", zc, orc.DT),
                                      g[f"call_{i}"])
        np.testing.assert_array_equal(orc.price_options(S0, K, T, orc.R, xi, H, eta, rho, "put", zp, orc.DT),
                                      g[f"put_{i}"])


def test_oracle_generator_matches_reference_bitwise():
    g = _load("rb_generate.npz")
    o = orc.generate(tuple(g["base"]), int(g["num_paths"]), int(g["seed"]), n_mc=int(g["n_mc"]))
    for k in ("paths", "volatilities", "call_prices_atm", "put_prices_atm"):
        np.testing.assert_array_equal(o[k], g[k], err_msg=k)


def test_w_form_identity():
    """Re ifft(fft(lam) Z) = (lam (*) Re W) / sqrt(M) with W = ifft(Z) sqrt(M): the
    identity that lets the kernels draw W and convolve instead of two FFTs."""
    rng = np.random.default_rng(3)
    for n_steps in (30, 252, 20, 9):
        t = orc.time_grid(n_steps, orc.DT)
        H = rng.uniform(0.01, 0.49, 5)
        eta = rng.uniform(0.5, 2.5, 5)
        phi = orc.phi_fft(t, H)
        M = phi.shape[1]
        Z = rng.normal(size=(5, M)) + 1j * rng.normal(size=(5, M))
        X = orc.fractional_gaussian(phi, Z, H, eta, n_steps + 1)
        W = orc.z_to_w(Z)
        lam = np.zeros((5, M))
        lam[:, :n_steps + 1] = 0.5 * t[None, :] ** (2 * H[:, None])
        j = np.arange(n_steps + 1)
        conv = np.stack([np.array([np.sum(lam[b] * W[b, (jj - np.arange(M)) % M, 0]) for jj in j]) for b in range(5)])
        Xw = (np.sqrt(2 * H) * eta)[:, None] * (conv / np.sqrt(M))
        np.testing.assert_allclose(Xw, X, rtol=1e-12, atol=1e-14)
        # the increments are Re / Im of W exactly
        d1, d2 = orc.unit_increments(Z)
        np.testing.assert_array_equal(W[..., 0], d1)
        np.testing.assert_array_equal(W[..., 1], d2)


# ------------------------------------------------------------------ library (host entries only)
def _rb():
    from cantorrl_amd import rbergomi
    return rbergomi


def test_library_exports_and_defaults():
    rb = _rb()
    lib = rb.load()
    for s in rb.EXPORTS:
        assert hasattr(lib, s), s
    assert b"gfx950" in lib.rb_version()
    c = rb.make_config(10)
    assert (c.n_steps, c.seed, c.n_mc) == (252, 42, 5000)
    assert (c.r, c.dt, c.option_tenor) == (0.04, 1 / 252, 30 / 252)
    assert list(c.perturb_std) == [0.01, 0.20, 0.20, 0.20, 0.10]
    assert (c.clip_h_min, c.clip_h_max, c.clip_rho_min, c.clip_rho_max) == (0.01, 0.49, -0.99, -0.01)
    assert ctypes.sizeof(rb.RbConfig) == 4 * 2 + 8 * 3 + 8 * 3 + 4 * 2 + 8 * 5 + 8 * 6 + 4 * 4 + 8 * 4


def test_config_validation_errors():
    rb = _rb()
    lib = rb.load()
    c = rb.RbConfig()
    assert lib.rb_config_init(ctypes.byref(c), 99) == rb.RB_EINVAL
    assert b"abi_version" in lib.rb_last_error()
    c = rb.make_config(0)
    base = rb.RbBaseParams(100.0, 0.04, 0.1, 1.0, -0.7)
    assert lib.rb_sample_params(ctypes.byref(c), ctypes.byref(base), None, None, None) == rb.RB_OK  # n = 0
    c.n_steps = 0
    assert lib.rb_simulate_paths(ctypes.byref(c), None, None, None, None, None) == rb.RB_EINVAL
    assert b"n_steps" in lib.rb_last_error()
    c = rb.make_config(0, option_tenor=64 / 252)
    assert lib.rb_price_atm_marks(ctypes.byref(c), None, None, None, None, None, None) == rb.RB_EINVAL
    assert b"63 steps" in lib.rb_last_error()
    c = rb.make_config(0)
    assert lib.rb_price_options(ctypes.byref(c), 1, 5, *([None] * 9), None) == rb.RB_EINVAL


def test_cpp_estimator_matches_reference():
    rb = _rb()
    g = _load("rb_estimate.npz")
    for name in g["names"]:
        p = g[f"{name}__prices"]
        base = np.array(rb.estimate_base_params(p, 1 / 252))
        np.testing.assert_allclose(base, g[f"{name}__base"], rtol=1e-12, atol=0, err_msg=str(name))
        parts = np.array(rb.estimate_parts(p, 1 / 252))
        ref = g[f"{name}__parts"]
        fin = np.isfinite(ref)
        assert np.array_equal(fin, np.isfinite(parts)), name
        np.testing.assert_allclose(parts[fin], ref[fin], rtol=1e-12, atol=0, err_msg=str(name))


def test_cpp_estimator_edge_cases():
    rb = _rb()
    assert rb.estimate_base_params([], 1 / 252) == (100.0, 0.04, 0.1, 1.0, -0.7)
    assert rb.estimate_base_params([7.0, 8.0], 1 / 252) == (8.0, 0.04, 0.1, 1.0, -0.7)
    rng = np.random.default_rng(1)
    for n in (21, 22, 41, 44, 80, 161, 1000):
        p = 50 * np.exp(np.cumsum(rng.normal(0, 0.02, n)))
        np.testing.assert_allclose(rb.estimate_base_params(p), orc.estimate_base_params(p), rtol=1e-12, atol=0,
                                   err_msg=str(n))


def test_host_normals_are_the_env_box_muller():
    """rb_host_normals draws (seed, domain, sub, gid) blocks with the env's f64
    Box-Muller; a spot check of the stream's moments and determinism."""
    rb = _rb()
    lib = rb.load()
    out = np.zeros(200000)
    assert lib.rb_host_normals(42, 3, 5, 7, 0, out.size, out.ctypes.data) == 0
    assert abs(out.mean()) < 0.01 and abs(out.std() - 1) < 0.01
    again = np.zeros(1000)
    lib.rb_host_normals(42, 3, 5, 7, 0, again.size, again.ctypes.data)
    np.testing.assert_array_equal(again, out[:1000])
    other = np.zeros(1000)
    lib.rb_host_normals(42, 3, 5, 8, 0, other.size, other.ctypes.data)
    assert not np.array_equal(other, again)


def test_library_exports_every_header_symbol():
    import re
    txt = open(os.path.join(os.path.dirname(os.path.dirname(__file__)), "include", "rbergomi.h")).read()
    syms = sorted(set(re.findall(r"^\S[^;(]*?\b(rb_\w+)\s*\(", txt, flags=re.M)))
    rb = _rb()
    lib = rb.load()
    assert len(syms) >= 10, syms
    for s in syms:
        assert hasattr(lib, s), f"librbergomi does not export {s}"
    assert set(syms) == set(rb.EXPORTS)
