"""Rough-Bergomi path and rolling-ATM option-mark generator on MI355X.

Python face of librbergomi (include/rbergomi.h; kernels in csrc/rbergomi.hip).  It
mirrors /root/reference/src/sim/rbergomi_sim.py:
  estimate_base_params(prices, dt)                       :174-195 (host C++)
  price_rbergomi_option(...)                             :261-306 (price_rbergomi_option_gpu)
  generate_paths_and_options(prices, num_paths, r, dt, seed)   :309-499
  save_npz(path, result)                                 :528 (the replay NPZ format)
  main()                                                 :502-534
with the same argument meaning.  The normals come from Philox4x32-10 instead of
cuRAND (the reference's stream is not reproducible off its GPU), so runs are
reproducible per seed and identical for any sharding of the paths; every stage
also takes injected draws, which is how the tests run the reference's own.

There is no CPU fallback: without the in-tree library every entry raises.  The
checkpoint/resume machinery of the reference (:324-353, :470-489) exists because
its generator runs for hours; this one produces the 100,000-path set in one call.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# CANTORRL_RBERGOMI_LIB: an alternative build (e.g. the host-ASan build of tools/asan/run.sh)
LIB_PATH = os.environ.get("CANTORRL_RBERGOMI_LIB") or os.path.join(HERE, "lib", "librbergomi.so")
RB_ABI_VERSION = 1
RB_OK, RB_EINVAL, RB_EHIP = 0, 1, 3
OPTION_TYPES = {"call": 0, "put": 1}
NORMALS = {"f64": 0, "f32": 1}

# rbergomi_sim.py:8-40
INPUT_FILE = "./data/historical_prices.csv"
OUTPUT_FILE = "./data/paths_rbergomi_options_100k.npz"
R = 0.04
DT = 1 / 252
N_PATHS = 100000
N_STEPS = 252
SEED = 42
T_OPTION_TENOR = 30 / 252
N_PATHS_OPTION_MC = 5000


class RbergomiError(RuntimeError):
    pass


class RbBaseParams(ctypes.Structure):
    _fields_ = [("S0", ctypes.c_double), ("xi", ctypes.c_double), ("H", ctypes.c_double),
                ("eta", ctypes.c_double), ("rho", ctypes.c_double)]

    def astuple(self):
        return (self.S0, self.xi, self.H, self.eta, self.rho)


class RbConfig(ctypes.Structure):
    _fields_ = [
        ("abi_version", ctypes.c_int32),
        ("n_steps", ctypes.c_int32),
        ("n_paths", ctypes.c_int64),
        ("path_offset", ctypes.c_int64),
        ("seed", ctypes.c_uint64),
        ("r", ctypes.c_double),
        ("dt", ctypes.c_double),
        ("option_tenor", ctypes.c_double),
        ("n_mc", ctypes.c_int32),
        ("normals", ctypes.c_int32),
        ("perturb_std", ctypes.c_double * 5),
        ("min_xi_factor", ctypes.c_double),
        ("min_eta_factor", ctypes.c_double),
        ("clip_h_min", ctypes.c_double),
        ("clip_h_max", ctypes.c_double),
        ("clip_rho_min", ctypes.c_double),
        ("clip_rho_max", ctypes.c_double),
        ("reserved_i", ctypes.c_int32 * 4),
        ("reserved", ctypes.c_double * 4),
    ]


EXPORTS = ["rb_version", "rb_last_error", "rb_config_init", "rb_estimate_base_params", "rb_estimate_parts",
           "rb_sample_params", "rb_simulate_paths", "rb_price_options", "rb_price_atm_marks", "rb_generate",
           "rb_host_normals", "rb_device_mc_box_muller"]

_lib = None


def load(path=LIB_PATH):
    """Load librbergomi (once).  Raises if the in-tree library is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RbergomiError(f"{path} not found: build it with `python -m cantorrl_amd.build` "
                            "(hipcc --offload-arch=gfx950).  There is no CPU fallback.")
    try:
        import torch  # noqa: F401  (bind to torch's HIP runtime first, as _lib.py does)
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    vp, i32, i64, u32, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32, ctypes.c_uint64
    cfgp, basep = ctypes.POINTER(RbConfig), ctypes.POINTER(RbBaseParams)
    sig = {
        "rb_version": (ctypes.c_char_p, []),
        "rb_last_error": (ctypes.c_char_p, []),
        "rb_config_init": (i32, [cfgp, i32]),
        "rb_estimate_base_params": (i32, [vp, i64, ctypes.c_double, basep]),
        "rb_estimate_parts": (i32, [vp, i64, ctypes.c_double, vp]),
        "rb_sample_params": (i32, [cfgp, basep, vp, vp, vp]),
        "rb_simulate_paths": (i32, [cfgp, vp, vp, vp, vp, vp]),
        "rb_price_options": (i32, [cfgp, i64, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        "rb_price_atm_marks": (i32, [cfgp, vp, vp, vp, vp, vp, vp]),
        "rb_generate": (i32, [cfgp, basep, vp, vp, vp, vp, vp, vp]),
        "rb_host_normals": (i32, [u64, i32, u32, u64, u32, i64, vp]),
        "rb_device_mc_box_muller": (i32, [vp, vp, i64, vp, vp, vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype, f.argtypes = res, args
    _lib = lib
    return lib


def _check(status):
    if status != RB_OK:
        raise RbergomiError(load().rb_last_error().decode())


def make_config(num_paths, *, n_steps=N_STEPS, path_offset=0, seed=SEED, r=R, dt=DT, option_tenor=T_OPTION_TENOR,
                n_mc=N_PATHS_OPTION_MC, normals="f64"):
    lib = load()
    c = RbConfig()
    _check(lib.rb_config_init(ctypes.byref(c), RB_ABI_VERSION))
    c.n_paths, c.n_steps, c.path_offset, c.seed = int(num_paths), int(n_steps), int(path_offset), int(seed)
    c.r, c.dt, c.option_tenor, c.n_mc = float(r), float(dt), float(option_tenor), int(n_mc)
    c.normals = NORMALS[normals]
    return c


# ------------------------------------------------------------------ host estimator
def estimate_base_params(prices, dt=DT):
    """(S0, xi, H, eta, rho) from a price history (rbergomi_sim.py:174-195)."""
    p = np.ascontiguousarray(prices, dtype=np.float64).ravel()
    out = RbBaseParams()
    _check(load().rb_estimate_base_params(p.ctypes.data if p.size else None, p.size, float(dt), ctypes.byref(out)))
    return out.astuple()


def estimate_parts(prices, dt=DT):
    """(estimate_xi, estimate_H, estimate_eta, estimate_rho) of the log returns (:63-171)."""
    p = np.ascontiguousarray(prices, dtype=np.float64).ravel()
    out = np.zeros(4)
    _check(load().rb_estimate_parts(p.ctypes.data if p.size else None, p.size, float(dt), out.ctypes.data))
    return tuple(out)


# ------------------------------------------------------------------ device stages
def _torch():
    import torch
    return torch


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _dev_f64(x, device):
    torch = _torch()
    if isinstance(x, torch.Tensor):
        return x.to(device=device, dtype=torch.float64).contiguous()
    return torch.as_tensor(np.ascontiguousarray(x, dtype=np.float64), device=device)


def _stream(device):
    torch = _torch()
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def sample_params(cfg, base, device="cuda", unit_normals=None):
    """params [5, n] (rows S0, xi, H, eta, rho; :379-383).  unit_normals [5, n] or Philox."""
    torch = _torch()
    out = torch.empty((5, cfg.n_paths), dtype=torch.float64, device=device)
    b = RbBaseParams(*[float(x) for x in base])
    un = None if unit_normals is None else _dev_f64(unit_normals, device)
    _check(load().rb_sample_params(ctypes.byref(cfg), ctypes.byref(b), _ptr(un), _ptr(out), _stream(device)))
    return out


def simulate_paths(cfg, params, device="cuda", W=None):
    """(paths, volatilities) [n, n_steps + 1] (:385-400, :454-464).  W [n, M, 2] or Philox."""
    torch = _torch()
    n, T = cfg.n_paths, cfg.n_steps
    paths = torch.empty((n, T + 1), dtype=torch.float64, device=device)
    vol = torch.empty((n, T + 1), dtype=torch.float64, device=device)
    w = None if W is None else _dev_f64(W, device)
    _check(load().rb_simulate_paths(ctypes.byref(cfg), _ptr(params), _ptr(w), _ptr(paths), _ptr(vol),
                                    _stream(device)))
    return paths, vol


def price_rbergomi_option(S0, K, T, r, xi, H, eta, rho, option_type, n_mc, dt, *, device="cuda", seed=SEED,
                          index_offset=0, W=None, normals="f64"):
    """price_rbergomi_option_gpu (:261-306) for a batch of options; W [B, n_mc, M_opt, 2]
    (the reference's ifft(Z) sqrt(M)) or Philox (gid = index_offset + i, sub = type)."""
    torch = _torch()
    arrs = [_dev_f64(np.atleast_1d(x) if not isinstance(x, torch.Tensor) else x, device)
            for x in (S0, K, xi, H, eta, rho)]
    B = arrs[0].numel()
    cfg = make_config(1, seed=seed, r=r, dt=dt, option_tenor=T, n_mc=n_mc, normals=normals,
                      path_offset=index_offset)
    out = torch.empty(B, dtype=torch.float64, device=device)
    w = None if W is None else _dev_f64(W, device)
    _check(load().rb_price_options(ctypes.byref(cfg), B, OPTION_TYPES[option_type], *[_ptr(a) for a in arrs],
                                   _ptr(w), _ptr(out), _stream(device)))
    return out


def price_atm_marks(cfg, params, paths, vol, device="cuda"):
    """(call_prices_atm, put_prices_atm) [n, n_steps] (:404-451, every day at once)."""
    torch = _torch()
    call = torch.empty((cfg.n_paths, cfg.n_steps), dtype=torch.float64, device=device)
    put = torch.empty_like(call)
    _check(load().rb_price_atm_marks(ctypes.byref(cfg), _ptr(params), _ptr(paths), _ptr(vol), _ptr(call),
                                     _ptr(put), _stream(device)))
    return call, put


def generate_paths_and_options(historical_prices, num_paths=N_PATHS, r=R, dt=DT, seed=SEED, *, n_mc=N_PATHS_OPTION_MC,
                               option_tenor=T_OPTION_TENOR, n_steps=N_STEPS, path_offset=0, normals="f64",
                               device="cuda", base_params=None):
    """generate_paths_and_options (:309-499): dict of device f64 tensors `paths`,
    `volatilities` [n, n_steps + 1], `call_prices_atm`, `put_prices_atm` [n, n_steps],
    `params` [5, n].  path_offset selects rows [offset, offset + n) of the global set."""
    torch = _torch()
    base = base_params if base_params is not None else estimate_base_params(
        np.asarray(historical_prices, dtype=np.float64), dt)
    cfg = make_config(num_paths, n_steps=n_steps, path_offset=path_offset, seed=seed, r=r, dt=dt,
                      option_tenor=option_tenor, n_mc=n_mc, normals=normals)
    n, T = cfg.n_paths, cfg.n_steps
    f = dict(dtype=torch.float64, device=device)
    out = dict(params=torch.empty((5, n), **f), paths=torch.empty((n, T + 1), **f),
               volatilities=torch.empty((n, T + 1), **f), call_prices_atm=torch.empty((n, T), **f),
               put_prices_atm=torch.empty((n, T), **f))
    b = RbBaseParams(*[float(x) for x in base])
    _check(load().rb_generate(ctypes.byref(cfg), ctypes.byref(b), _ptr(out["params"]), _ptr(out["paths"]),
                              _ptr(out["volatilities"]), _ptr(out["call_prices_atm"]), _ptr(out["put_prices_atm"]),
                              _stream(device)))
    out["base_params"] = tuple(base)
    return out


def save_npz(path, result, compressed=True):
    """The reference's wire format (:528): paths, volatilities, call_prices_atm,
    put_prices_atm as f64 -- what HedgingEnv / HedgingVecEnv replay mode loads."""
    arrs = {k: result[k].detach().cpu().numpy() if hasattr(result[k], "detach") else np.asarray(result[k])
            for k in ("paths", "volatilities", "call_prices_atm", "put_prices_atm")}
    (np.savez_compressed if compressed else np.savez)(path, **arrs)


def load_history(path=INPUT_FILE):
    """:505-520: the first column of the CSV, [] when missing or unreadable."""
    try:
        p = np.loadtxt(path, dtype=np.float64, delimiter=",")
    except (OSError, ValueError):
        return np.array([])
    if p.ndim == 0:
        p = np.array([float(p)])
    elif p.ndim > 1:
        p = p[:, 0]
    return p


def main(argv=None):
    import argparse
    import time
    ap = argparse.ArgumentParser(description="rough-Bergomi paths + rolling-ATM MC marks (rbergomi_sim.py)")
    ap.add_argument("--input", default=INPUT_FILE)
    ap.add_argument("--output", default=OUTPUT_FILE)
    ap.add_argument("--paths", type=int, default=N_PATHS)
    ap.add_argument("--steps", type=int, default=N_STEPS)
    ap.add_argument("--n-mc", type=int, default=N_PATHS_OPTION_MC)
    ap.add_argument("--seed", type=int, default=SEED)
    ap.add_argument("--normals", choices=sorted(NORMALS), default="f64")
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args(argv)
    torch = _torch()
    t0 = time.time()
    res = generate_paths_and_options(load_history(a.input), a.paths, R, DT, a.seed, n_mc=a.n_mc, n_steps=a.steps,
                                     normals=a.normals, device=a.device)
    torch.cuda.synchronize()
    t1 = time.time()
    print("base params S0=%.2f xi=%.4f H=%.4f eta=%.4f rho=%.4f" % res["base_params"])
    print(f"generated {a.paths} paths x {a.steps} steps with {a.n_mc}-path MC marks in {t1 - t0:.2f} s")
    save_npz(a.output, res)
    print(f"saved {a.output} ({time.time() - t1:.1f} s)")


if __name__ == "__main__":
    main()
