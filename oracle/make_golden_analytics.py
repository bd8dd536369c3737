#!/usr/bin/env python3
"""Record analytics golden vectors by running the REFERENCE in this container.

TEST INFRASTRUCTURE ONLY.  Imports /root/reference/src/tools/bs_delta.py and
src/sim/option_price_assignment.py unmodified (they need only NumPy / SciPy) and runs
them on the first 24 rows of the shipped data/paths.npy.  Writes
tests/golden/g11_analytics.npz: the input rows, the reference's vols / calls / puts /
pnl for them, and the same rows of the shipped data/paths_options.npz.
Re-run:  python oracle/make_golden_analytics.py
"""
import importlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = os.environ.get("CANTORRL_REFERENCE", "/root/reference")
sys.path.insert(0, REF)
sys.path.insert(0, REPO)


def main():
    from oracle import analytics_oracle as orc
    bsd = importlib.import_module("src.tools.bs_delta")
    opa = importlib.import_module("src.sim.option_price_assignment")
    paths = np.load(os.path.join(REF, "data", "paths.npy"))[:24]
    shipped = np.load(os.path.join(REF, "data", "paths_options.npz"))
    with np.errstate(invalid="ignore", divide="ignore"):
        vols = opa.calculate_annualized_vol_matrix(paths)
        n1 = paths.shape[1]
        T = np.clip(1 - np.arange(n1) / 252, 0, None)
        K = np.round(paths[:, 0])
        calls = np.zeros_like(paths)
        puts = np.zeros_like(paths)
        for t in range(n1):
            calls[:, t], puts[:, t] = opa.black_scholes_vectorized(paths[:, t], K, T[t], opa.RISK_FREE_RATE,
                                                                   vols[:, t])
    pnl = bsd.bs_delta_hedge(paths)
    ov, oc, op = orc.fixed_european_marks(paths)
    assert np.array_equal(np.isnan(oc), np.isnan(calls))
    for a, b in ((ov, vols), (oc, calls), (op, puts), (orc.bs_delta_hedge(paths), pnl)):
        assert np.array_equal(a, b, equal_nan=True)
    np.savez_compressed(os.path.join(REPO, "tests", "golden", "g11_analytics.npz"), paths=paths, vols=vols,
                        calls=calls, puts=puts, pnl=pnl, shipped_calls=shipped["calls"][:24],
                        shipped_puts=shipped["puts"][:24])
    print("wrote g11_analytics.npz; oracle bit-identical to the reference")


if __name__ == "__main__":
    main()
