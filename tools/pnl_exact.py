#!/usr/bin/env python3
"""Share of generate-mode P&L values equal bit for bit to the oracle's (the parity tests'
run_gbm_pair), for the GBM and Heston cases of tests/test_gpu_parity.py."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from test_gpu_parity import run_gbm_pair  # noqa: E402

cfg = dict(loss_type="abs", pnl_penalty_weight=0.001, lambda_cost=0.0001, theta_weight=0.0002, slippage_bps=1.0)
hes = dict(s0=496.48001098632812, variance=0.04, mu=0.04, dt=1 / 252, episode_length=30,
           heston_kappa=1.5, heston_theta=0.035, heston_xi=0.6, heston_rho=-0.7)
gbm = dict(s0=496.48001098632812, variance=0.029028, mu=0.04, dt=1 / 252, episode_length=40)
for name, gen, mode in (("gbm", gbm, "gbm"), ("heston", hes, "heston")):
    st = run_gbm_pair(256, 75, 11, cfg, gen, mode=mode)
    print(name, st, "%.4f" % (st["pnl_exact"] / st["pnl_total"]), flush=True)
