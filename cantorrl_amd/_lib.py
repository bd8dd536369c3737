"""ctypes binding of libhedgeenv (include/hedge_env.h).

The shared library is built in-tree (`cantorrl_amd/lib/libhedgeenv.so`, see
`cantorrl_amd/build.py`).  There is no fallback: if the library cannot be
loaded, every constructor raises.  torch is imported first so that the HIP
runtime torch ships (SONAME libamdhip64.so.7) is the one the library binds to
-- one runtime per process, so torch streams and data_ptr()s are valid here.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# CANTORRL_HEDGEENV_LIB: an alternative build (diagnostic / A-B builds under tools/ab/)
LIB_PATH = os.environ.get("CANTORRL_HEDGEENV_LIB") or os.path.join(HERE, "lib", "libhedgeenv.so")

HE_ABI_VERSION = 4
HE_BOOK_MAX = 8
HE_OBS_DIM = 13
BOOK_TYPES = {"call": 0, "put": 1, "uo_call": 2}
HE_OK, HE_EINVAL, HE_ESHAPE, HE_EHIP, HE_ENOMEM, HE_ESTATE = range(6)
HE_MODE_REPLAY, HE_MODE_GBM, HE_MODE_HESTON = range(3)
HE_LOSS_MSE, HE_LOSS_ABS, HE_LOSS_CVAR, HE_LOSS_OTHER = range(4)
MODES = {"replay": HE_MODE_REPLAY, "gbm": HE_MODE_GBM, "heston": HE_MODE_HESTON}
# he_mark: rolling ATM (rbergomi_sim.py:418,437-446) or the fixed-strike European of
# option_price_assignment.py:10-21,33-49
HE_MARK_ROLLING_ATM, HE_MARK_FIXED_EUROPEAN = range(2)
MARKS = {"rolling_atm": HE_MARK_ROLLING_ATM, "fixed_european": HE_MARK_FIXED_EUROPEAN}


def loss_code(loss_type):
    """hedging_env_v2.py:246-253: "mse", "abs", "cvar", anything else = |x| branch."""
    return {"mse": HE_LOSS_MSE, "abs": HE_LOSS_ABS, "cvar": HE_LOSS_CVAR}.get(loss_type, HE_LOSS_OTHER)


class HeBookOption(ctypes.Structure):
    _fields_ = [
        ("type", ctypes.c_int32),
        ("expiry", ctypes.c_int32),
        ("strike", ctypes.c_double),
        ("barrier", ctypes.c_double),
        ("quantity", ctypes.c_double),
    ]


class HeConfig(ctypes.Structure):
    _fields_ = [
        ("abi_version", ctypes.c_int32),
        ("variant", ctypes.c_int32),
        ("mode", ctypes.c_int32),
        ("loss_type", ctypes.c_int32),
        ("n_envs", ctypes.c_int64),
        ("global_env_offset", ctypes.c_int64),
        ("transaction_cost_per_contract", ctypes.c_double),
        ("lambda_cost", ctypes.c_double),
        ("pnl_penalty_weight", ctypes.c_double),
        ("theta_weight", ctypes.c_double),
        ("slippage_bps", ctypes.c_double),
        ("initial_cash", ctypes.c_double),
        ("shares_to_hedge", ctypes.c_int64),
        ("max_contracts_held_per_type", ctypes.c_int32),
        ("max_trade_per_step", ctypes.c_int32),
        ("record_metrics", ctypes.c_int32),
        ("autoreset", ctypes.c_int32),
        ("risk_free_rate", ctypes.c_double),
        ("option_tenor_years", ctypes.c_double),
        ("episode_length", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("s0", ctypes.c_double),
        ("variance", ctypes.c_double),
        ("mu", ctypes.c_double),
        ("dt", ctypes.c_double),
        ("heston_kappa", ctypes.c_double),
        ("heston_theta", ctypes.c_double),
        ("heston_xi", ctypes.c_double),
        ("heston_rho", ctypes.c_double),
        ("market_block", ctypes.c_int32),
        ("market_prefetch", ctypes.c_int32),
        ("book_size", ctypes.c_int32),
        ("mark", ctypes.c_int32),
        ("book", HeBookOption * HE_BOOK_MAX),
        ("reserved", ctypes.c_double * 7),
    ]


POLICIES = {"no_hedge": 0, "delta_every_step": 1, "delta_threshold": 2}

# he_episode_record as a numpy structured dtype (64 B, include/hedge_env.h)
import numpy as _np  # noqa: E402
EPISODE_RECORD = _np.dtype([("env_id", "<i8"), ("length", "<i4"), ("reserved", "<i4"), ("reward_sum", "<f8"),
                            ("pnl_sum", "<f8"), ("abs_pnl_sum", "<f8"), ("cost_sum", "<f8"),
                            ("pnl_penalty_sum", "<f8"), ("cost_penalty_sum", "<f8"),
                            ("per_share_pnl_sum", "<f8"), ("reserved2", "<f8")])
assert EPISODE_RECORD.itemsize == 80

_P = ctypes.c_void_p
INFO_FIELDS = [
    ("step_pnl_total", "f8"), ("per_share_step_pnl", "f8"), ("raw_pnl_deviation_abs", "f8"),
    ("transaction_costs_total", "f8"), ("commission_cost", "f8"), ("slippage_cost", "f8"),
    ("reward_pnl_component", "f8"), ("transaction_cost_penalty", "f8"), ("theta_penalty", "f8"),
    ("reward_step", "f8"), ("portfolio_value", "f8"), ("cash", "f8"),
    ("call_contracts", "i4"), ("put_contracts", "i4"),
    ("scaled_float_call", "f4"), ("scaled_float_put", "f4"),
    ("requested_calls_rounded_clipped", "i4"), ("requested_puts_rounded_clipped", "i4"),
    ("actual_calls_traded", "i4"), ("actual_puts_traded", "i4"),
    ("initial_S0_for_episode", "f4"),
    ("current_stock_price", "f4"), ("current_volatility", "f4"),
    ("current_call_price", "f4"), ("current_put_price", "f4"), ("current_step", "i4"),
    ("current_episode_idx", "i4"),
]


class HeInfo(ctypes.Structure):
    _fields_ = [(name, _P) for name, _ in INFO_FIELDS]


EXPORTS = [
    "he_config_init", "he_create", "he_destroy", "he_last_error", "he_version", "he_load_paths",
    "he_seed", "he_reset", "he_reset_episodes", "he_step", "he_rollout", "he_num_envs", "he_episode_length",
    "he_num_episodes", "he_get_config", "he_state_size", "he_get_state", "he_set_state",
    "he_pcg64_seed_state", "he_host_episode_draws", "he_host_philox", "he_host_div_by", "he_host_div_byf", "he_time_next_step", "he_rollout_policy", "he_host_box_muller",
    "he_sync_market", "he_vecnorm_stats_len", "he_vecnorm_scratch_bytes", "he_vecnorm_init", "he_vecnorm_step",
    "he_vecnorm_apply", "he_vecnorm_attach", "he_vecnorm_attach_eval", "he_vecnorm_reset", "he_fixed_european_marks", "he_bs_delta_hedge", "he_count_nonfinite",
    "he_device_rng", "he_device_math", "he_host_math", "he_episode_summaries", "he_host_alloc", "he_host_free",
    "he_stream_wait", "he_step_signal", "he_signal_seq", "he_signal_wait",
]


class HeVecnormParams(ctypes.Structure):
    _fields_ = [
        ("obs_dim", ctypes.c_int32),
        ("training", ctypes.c_int32),
        ("norm_obs", ctypes.c_int32),
        ("norm_reward", ctypes.c_int32),
        ("gamma", ctypes.c_double),
        ("clip_obs", ctypes.c_double),
        ("clip_reward", ctypes.c_double),
        ("epsilon", ctypes.c_double),
        ("reserved", ctypes.c_int32 * 4),
    ]


class HeVecnormOut(ctypes.Structure):
    """include/hedge_env.h he_vecnorm_out: the eval VecNormalize step's buffers."""
    _fields_ = [(name, ctypes.c_void_p) for name in (
        "stats", "returns", "obs_out", "reward_out", "terminal_obs_out", "ep_return", "ep_length", "ep_return_done",
        "ep_length_done")]

_lib = None


class HedgeEnvError(RuntimeError):
    pass


def load(path=LIB_PATH):
    """Load libhedgeenv (once).  Raises if the in-tree library is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise HedgeEnvError(
            f"{path} not found: build it with `python -m cantorrl_amd.build` "
            "(hipcc --offload-arch=gfx950).  There is no CPU fallback.")
    try:
        import torch  # noqa: F401  (bind to torch's HIP runtime, see module doc)
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    vp, i32, i64, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
    sig = {
        "he_config_init": (i32, [ctypes.POINTER(HeConfig), i32]),
        "he_create": (i32, [ctypes.POINTER(HeConfig), ctypes.POINTER(vp)]),
        "he_destroy": (i32, [vp]),
        "he_last_error": (ctypes.c_char_p, [vp]),
        "he_version": (ctypes.c_char_p, []),
        "he_load_paths": (i32, [vp, vp, vp, vp, vp, i64, i64]),
        "he_seed": (i32, [vp, vp, vp, i64]),
        "he_reset": (i32, [vp, vp, i64, vp, ctypes.POINTER(HeInfo), vp]),
        "he_reset_episodes": (i32, [vp, vp, vp, i64, vp, ctypes.POINTER(HeInfo), vp]),
        "he_step": (i32, [vp, vp, vp, vp, vp, vp, vp, ctypes.POINTER(HeInfo), vp]),
        "he_rollout": (i32, [vp, i32, vp, vp, vp, vp, vp]),
        "he_rollout_policy": (i32, [vp, i32, i32, vp, vp, vp, vp, vp, i64, vp, vp]),
        "he_num_envs": (i64, [vp]),
        "he_episode_length": (i32, [vp]),
        "he_num_episodes": (i64, [vp]),
        "he_get_config": (i32, [vp, ctypes.POINTER(HeConfig)]),
        "he_state_size": (ctypes.c_size_t, [vp]),
        "he_get_state": (i32, [vp, vp, ctypes.c_size_t]),
        "he_set_state": (i32, [vp, vp, ctypes.c_size_t]),
        "he_pcg64_seed_state": (i32, [u64, ctypes.POINTER(ctypes.c_uint64 * 4)]),
        "he_host_episode_draws": (i32, [u64, u64, i64, vp]),
        "he_host_philox": (i32, [u64, u64, u64, ctypes.POINTER(ctypes.c_uint32 * 4)]),
        "he_host_div_by": (i32, [ctypes.c_void_p, i64, ctypes.c_double, ctypes.c_void_p]),
        "he_host_div_byf": (i32, [ctypes.c_void_p, i64, ctypes.c_float, ctypes.c_void_p]),
        "he_host_box_muller": (i32, [ctypes.c_void_p, ctypes.c_void_p, i64, ctypes.c_void_p, ctypes.c_void_p]),
        "he_time_next_step": (i32, [vp, vp, vp]),
        "he_sync_market": (i32, [vp, vp]),
        "he_vecnorm_stats_len": (i64, [i32]),
        "he_vecnorm_scratch_bytes": (i64, [i64, i32]),
        "he_vecnorm_init": (i32, [vp, i32, vp]),
        "he_vecnorm_step": (i32, [ctypes.POINTER(HeVecnormParams), i64] + [vp] * 15 + [vp]),
        "he_vecnorm_apply": (i32, [ctypes.POINTER(HeVecnormParams), i64] + [vp] * 15 + [vp]),
        "he_vecnorm_attach": (i32, [vp, ctypes.POINTER(HeVecnormParams), vp, vp, vp]),
        "he_vecnorm_attach_eval": (i32, [vp, ctypes.POINTER(HeVecnormParams), ctypes.POINTER(HeVecnormOut)]),
        "he_vecnorm_reset": (i32, [ctypes.POINTER(HeVecnormParams), i64] + [vp] * 5 + [vp]),
        "he_fixed_european_marks": (i32, [vp, i64, i32, ctypes.c_double, vp, vp, vp, vp]),
        "he_bs_delta_hedge": (i32, [vp, i64, i32, ctypes.c_double, ctypes.c_double, vp, vp]),
        "he_count_nonfinite": (i32, [vp, i64, vp, vp]),
        "he_device_rng": (i32, [u64, vp, vp, i64, vp, vp, vp]),
        "he_device_math": (i32, [i32, vp, i64, vp, vp]),
        "he_host_math": (i32, [i32, vp, i64, vp]),
        "he_episode_summaries": (i32, [vp, vp, vp]),
        "he_host_alloc": (i32, [ctypes.c_size_t, ctypes.POINTER(vp), ctypes.POINTER(vp)]),
        "he_host_free": (i32, [vp]),
        "he_stream_wait": (i32, [vp]),
        "he_step_signal": (i32, [vp, vp]),
        "he_signal_seq": (ctypes.c_uint32, [vp]),
        "he_signal_wait": (i32, [vp, vp, vp]),
    }
    ab = path != os.path.join(HERE, "lib", "libhedgeenv.so")  # an A/B build of an older tree
    for name, (res, args) in sig.items():
        if ab and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(lib, handle, status, what):
    if status != HE_OK:
        msg = lib.he_last_error(handle).decode() if handle else ""
        if status == HE_ESHAPE:
            raise ValueError(msg or "Data shapes are inconsistent.")
        raise HedgeEnvError(f"{what} failed (status {status}): {msg}")


def pcg64_seed_state(seed):
    """Host PCG64(SeedSequence(seed)) state as (state_hi, state_lo, inc_hi, inc_lo)."""
    lib = load()
    arr = (ctypes.c_uint64 * 4)()
    check(lib, None, lib.he_pcg64_seed_state(ctypes.c_uint64(seed), ctypes.byref(arr)), "he_pcg64_seed_state")
    return tuple(arr)


def host_episode_draws(seed, n_paths, count):
    """Host build of the device episode sampler (PCG64 + Lemire), for tests."""
    import numpy as np
    lib = load()
    out = np.zeros(count, np.int64)
    check(lib, None, lib.he_host_episode_draws(seed, n_paths, count, out.ctypes.data), "he_host_episode_draws")
    return out


def host_philox(seed, env_id, n):
    lib = load()
    arr = (ctypes.c_uint32 * 4)()
    check(lib, None, lib.he_host_philox(seed, env_id, n, ctypes.byref(arr)), "he_host_philox")
    return tuple(arr)


def host_div_by(a, b):
    """Host build of the step kernel's reciprocal-multiply division, for tests."""
    import numpy as np
    lib = load()
    a = np.ascontiguousarray(a, np.float64)
    out = np.empty_like(a)
    check(lib, None, lib.he_host_div_by(a.ctypes.data, a.size, float(b), out.ctypes.data), "he_host_div_by")
    return out


def host_div_byf(a, b):
    """Host build of the obs kernels' f32 reciprocal-multiply division, for tests."""
    import numpy as np
    lib = load()
    a = np.ascontiguousarray(a, np.float32)
    out = np.empty_like(a)
    check(lib, None, lib.he_host_div_byf(a.ctypes.data, a.size, float(b), out.ctypes.data), "he_host_div_byf")
    return out


def host_box_muller(u1, u2):
    """Host build of the generate-mode Box-Muller pair, for tests."""
    import numpy as np
    lib = load()
    u1 = np.ascontiguousarray(u1, np.float64)
    u2 = np.ascontiguousarray(u2, np.float64)
    z1 = np.empty_like(u1)
    z2 = np.empty_like(u1)
    check(lib, None, lib.he_host_box_muller(u1.ctypes.data, u2.ctypes.data, u1.size, z1.ctypes.data, z2.ctypes.data),
          "he_host_box_muller")
    return z1, z2
