#!/usr/bin/env python3
"""Record rBergomi generator golden vectors by running the REFERENCE in this container.

TEST INFRASTRUCTURE ONLY (never shipped, never imported by the product path).

Imports `/root/reference/src/sim/rbergomi_sim.py` unmodified, with oracle/cupy_shim
standing in for the absent CuPy (NumPy underneath; cp.random = one NumPy PCG64
stream that oracle/rbergomi_oracle.ReferenceDraws replays).  Writes, as inputs +
expected outputs only:
  tests/golden/rb_estimate.npz  estimate_base_params + its parts on 8 price series
  tests/golden/rb_price.npz     price_rbergomi_option_gpu, 4 tenors x call/put
  tests/golden/rb_generate.npz  generate_paths_and_options, 3 paths, 8 MC paths
The normal draws are not stored: tests regenerate them from the recorded seeds.
Re-run:  python oracle/make_golden_rbergomi.py   (about a minute)
"""
import importlib
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = os.environ.get("CANTORRL_REFERENCE", "/root/reference")
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, os.path.join(HERE, "cupy_shim"))
sys.path.insert(0, REF)
sys.path.insert(0, REPO)


def series():
    """Price series for the estimator: the shipped history, its prefixes (every
    early-return branch of :174-195 and :82-130), and synthetic paths."""
    hist = np.loadtxt(os.path.join(REF, "data", "historical_prices.csv"), dtype=np.float64, delimiter=",")
    rng = np.random.default_rng(5)
    gbm = 100 * np.exp(np.cumsum(rng.normal(0, 0.01, 400)))
    # positively correlated returns / squared returns -> the rho > 0 branch (:169-170)
    up = np.concatenate([[100.0], 100 * np.exp(np.cumsum(np.abs(rng.normal(0, 0.02, 120)) - 0.012))])
    flat = np.full(50, 42.0)   # zero variance: xi / eta / rho defaults
    return {"hist": hist, "hist_15": hist[:15], "hist_30": hist[:30], "hist_45": hist[:45],
            "hist_300": hist[-300:], "gbm_400": gbm, "up_121": up, "flat_50": flat}


def main():
    rb = importlib.import_module("src.sim.rbergomi_sim")
    cp = importlib.import_module("cupy")
    from oracle import rbergomi_oracle as orc
    os.makedirs(OUT, exist_ok=True)

    # ---- estimation
    ser = series()
    est = {}
    for name, p in ser.items():
        est[f"{name}__prices"] = p
        est[f"{name}__base"] = np.array([float(x) for x in rb.estimate_base_params(p, 1 / 252)])
        r = rb.log_returns(p)
        est[f"{name}__parts"] = np.array([
            float(rb.estimate_xi(r, 1 / 252)) if len(r) > 0 else np.nan,
            float(rb.estimate_H(r)), float(rb.estimate_eta(r, 0.1)), float(rb.estimate_rho(r))])
        o = orc.estimate_base_params(p, 1 / 252)
        assert np.allclose(np.array([float(x) for x in o]), est[f"{name}__base"], rtol=1e-13, atol=0), name
    np.savez_compressed(os.path.join(OUT, "rb_estimate.npz"), names=np.array(list(ser)), **est)

    # ---- MC option pricer
    B, n_mc, seed = 6, 48, 7
    g = np.random.default_rng(11)
    S0 = np.array([496.48, 100.0, 250.3, 496.48, 1.5, 3000.0])
    K = np.round(S0 * np.array([1.0, 1.02, 0.97, 1.0, 1.0, 1.01]))
    xi = np.array([0.029, 0.04, 0.09, 1e-6, 0.2, 0.0])
    H = np.array([0.4656, 0.1, 0.01, 0.49, 0.25, 0.3])
    eta = np.array([1.985, 1.0, 2.5, 0.5, 1.2, 0.9])
    rho = np.array([-0.202, -0.7, -0.99, -0.01, -0.5, -0.3])
    pr = dict(S0=S0, K=K, xi=xi, H=H, eta=eta, rho=rho, n_mc=n_mc, seed=seed, r=rb.R, dt=rb.DT)
    tenors = [30 / 252, 20 / 252, 10 / 252, 0.5 / 252]
    pr["tenors"] = np.array(tenors)
    for i, T in enumerate(tenors):
        cp.random.seed(seed + i)
        c = rb.price_rbergomi_option_gpu(S0, K, T, rb.R, xi, H, eta, rho, "call", n_mc, rb.DT)
        p_ = rb.price_rbergomi_option_gpu(S0, K, T, rb.R, xi, H, eta, rho, "put", n_mc, rb.DT)
        pr[f"call_{i}"], pr[f"put_{i}"] = c, p_
        d = orc.ReferenceDraws(seed + i)
        n = int(T / rb.DT)
        if n > 0:
            Mo = orc.next_pow2(n + 1)
            zc = d.complex_normal((B, n_mc, Mo))
            zp = d.complex_normal((B, n_mc, Mo))
        else:
            zc = zp = None
        oc = orc.price_options(S0, K, T, rb.R, xi, H, eta, rho, "call", zc, rb.DT)
        op = orc.price_options(S0, K, T, rb.R, xi, H, eta, rho, "put", zp, rb.DT)
        assert np.array_equal(oc, c) and np.array_equal(op, p_), T
    np.savez_compressed(os.path.join(OUT, "rb_price.npz"), **pr)

    # ---- full generator (3 paths, 8 MC paths per option)
    P, n_mc_g, seed_g = 3, 8, 42
    hist = ser["hist"]
    rb.N_PATHS_OPTION_MC = n_mc_g
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as td:
        os.chdir(td)   # the reference checkpoints into ./ every day
        try:
            S, v, C, Pu = rb.generate_paths_and_options(hist, P, rb.R, rb.DT, seed_g)
        finally:
            os.chdir(cwd)
    base = np.array([float(x) for x in rb.estimate_base_params(hist, rb.DT)])
    o = orc.generate(tuple(base), P, seed_g, n_mc=n_mc_g)
    for k, a in (("paths", S), ("volatilities", v), ("call_prices_atm", C), ("put_prices_atm", Pu)):
        assert np.array_equal(o[k], a), k
    np.savez_compressed(os.path.join(OUT, "rb_generate.npz"), base=base, num_paths=P, n_mc=n_mc_g, seed=seed_g,
                        paths=S, volatilities=v, call_prices_atm=C, put_prices_atm=Pu)
    print("wrote rb_estimate / rb_price / rb_generate; oracle bit-identical to the reference on all")


if __name__ == "__main__":
    main()
