"""Offline path analytics of the reference on the GPU (libhedgeenv he_fixed_european_marks /
he_bs_delta_hedge; kernels in csrc/analytics.hip), with the reference's names:

  calculate_annualized_vol_matrix(paths)   src/sim/option_price_assignment.py:23-31
  process_price_paths(paths)               :33-52 -> (calls, puts), fixed-strike European marks
  bs_delta_hedge(paths)                    src/tools/bs_delta.py:36-55 -> daily delta-hedge P&L

`paths` is an [n_sims, n_steps + 1] array (NumPy or a torch tensor); results are f64
device tensors (NumPy in, NumPy out when return_numpy=True).  The expanding-window
realized volatility is a running scan, O(n_steps) per path instead of the
reference's O(n_steps^2).  No CPU fallback.
"""
import ctypes

import numpy as np
import torch

from . import _lib

RISK_FREE_RATE = 0.04
DT = 1 / 252


def _paths(paths, device):
    if isinstance(paths, torch.Tensor):
        return paths.to(device=device, dtype=torch.float64).contiguous(), False
    a = np.ascontiguousarray(paths, dtype=np.float64)
    if a.ndim != 2:
        raise ValueError("paths must be [n_sims, n_steps + 1]")
    return torch.as_tensor(a, device=device), True


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _check(st, what):
    if st != _lib.HE_OK:
        raise _lib.HedgeEnvError(f"{what} failed with status {st}")


def _out(t, to_numpy):
    return t.cpu().numpy() if to_numpy else t


def fixed_european_marks(paths, r=RISK_FREE_RATE, device="cuda", return_numpy=None):
    """(vols, calls, puts), each [n_sims, n_steps + 1] (option_price_assignment.py:23-52)."""
    lib = _lib.load()
    p, was_np = _paths(paths, device)
    n, c = p.shape
    vols, calls, puts = (torch.empty((n, c), dtype=torch.float64, device=p.device) for _ in range(3))
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    _check(lib.he_fixed_european_marks(ptr(p), n, c, float(r), ptr(vols), ptr(calls), ptr(puts), _stream(p.device)),
           "he_fixed_european_marks")
    to_np = was_np if return_numpy is None else return_numpy
    return _out(vols, to_np), _out(calls, to_np), _out(puts, to_np)


def calculate_annualized_vol_matrix(paths, device="cuda", return_numpy=None):
    return fixed_european_marks(paths, device=device, return_numpy=return_numpy)[0]


def process_price_paths(paths, r=RISK_FREE_RATE, device="cuda", return_numpy=None):
    """(calls, puts): what process_price_paths saves to paths_options.npz (:51)."""
    _, calls, puts = fixed_european_marks(paths, r, device, return_numpy)
    return calls, puts


def bs_delta_hedge(paths, r=RISK_FREE_RATE, dt=DT, device="cuda", return_numpy=None):
    """pnl [n_sims, n_steps + 1] of the daily BS delta hedge (bs_delta.py:36-55)."""
    lib = _lib.load()
    p, was_np = _paths(paths, device)
    n, c = p.shape
    pnl = torch.empty((n, c), dtype=torch.float64, device=p.device)
    _check(lib.he_bs_delta_hedge(ctypes.c_void_p(p.data_ptr()), n, c, float(r), float(dt),
                                 ctypes.c_void_p(pnl.data_ptr()), _stream(p.device)), "he_bs_delta_hedge")
    return _out(pnl, was_np if return_numpy is None else return_numpy)
