"""Time the rBergomi MC marks kernel (rb_price_atm_marks) on one GPU: options/s for
f64 and f32 normals at a bounded number of paths."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cantorrl_amd import rbergomi as rb  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 512
if len(sys.argv) > 2:          # A/B: an alternative build of librbergomi
    rb.load(sys.argv[2])
    print("lib", sys.argv[2])
dev = "cuda:0"
hist = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "rb_estimate.npz"))["hist__prices"]
base = rb.estimate_base_params(hist)
for normals in ("f32", "f64"):
    cfg = rb.make_config(P, normals=normals)
    params = rb.sample_params(cfg, base, dev)
    paths, vol = rb.simulate_paths(cfg, params, dev)
    rb.price_atm_marks(cfg, params, paths, vol, dev)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    reps = 2
    for _ in range(reps):
        c, p = rb.price_atm_marks(cfg, params, paths, vol, dev)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    n_opt = P * 252 * 2
    print(f"{normals}: {P} paths x 252 days x 2 = {n_opt} options, n_mc {cfg.n_mc}: {ms:.1f} ms  "
          f"{n_opt / ms * 1e3:.4g} options/s  {n_opt * cfg.n_mc * 30 / ms * 1e3:.4g} MC path-steps/s  "
          f"mean call {float(c.mean()):.4f} put {float(p.mean()):.4f}", flush=True)
