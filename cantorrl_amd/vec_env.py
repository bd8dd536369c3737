"""HedgingVecEnv: N hedging envs on one MI355X behind the SB3 VecEnv interface.

Drop-in for the `create_vec_env(...)` swap point of the reference agents
(src/agents/train_ppo_v2.py:127-141): it exposes what SB3 2.6.0's
DummyVecEnv/SubprocVecEnv expose (num_envs, observation_space, action_space,
reset, step_async, step_wait, step, seed, close, get_attr, set_attr,
env_method, env_is_wrapped) with SB3's auto-reset semantics
(`info["terminal_observation"]`, `info["TimeLimit.truncated"]`), and Monitor's
`info["episode"]` when `monitor_keywords` is given (train_ppo_v2.py:119).

Every env's state lives on the device; one `he_step` launch advances all of
them.  `step_tensors` is the zero-copy path for GPU-resident learners.
"""
import os
import time
import weakref

import numpy as np
import torch

from . import _lib
from .spaces import Box

try:   # the C rows of an info view (csrc/info_rows.c, built with the HIP libraries)
    from .lib import _info_rows
except ImportError as e:  # no fallback: a missing build is an error, not a slow path
    raise ImportError(f"cantorrl_amd/lib/_info_rows is not built ({e}): run `python -m cantorrl_amd.build`")

OBS_LOW = np.array([0.1, -1.0, -1.0, -1.0, -1.0, 0.0, 0.0, -1.0, 0.0, -1.0, 0.0, -1.0, -1.0], np.float32)
OBS_HIGH = np.array([10.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 50.0, 1.0, 50.0, 1.0, 1.0], np.float32)

# HedgingEnv ctor keywords and defaults (hedging_env_v2.py:10-22, v1 hedging_env.py:10-20)
V2_DEFAULTS = dict(transaction_cost_per_contract=0.65, lambda_cost=1.0, pnl_penalty_weight=0.01,
                   theta_weight=0.0, slippage_bps=0.0, loss_type="abs", initial_cash=0.0,
                   shares_to_hedge=10000, max_contracts_held_per_type=200, max_trade_per_step=15,
                   profile_print_interval=0, record_metrics=True)
V1_DEFAULTS = {k: v for k, v in V2_DEFAULTS.items() if k not in ("theta_weight", "slippage_bps")}
V1_DEFAULTS["transaction_cost_per_contract"] = 0.05

GENERATE_DEFAULTS = dict(s0=496.48001098632812, variance=0.029028, mu=0.04, dt=1 / 252,
                         episode_length=252, heston_kappa=2.0, heston_theta=0.029028,
                         heston_xi=0.3, heston_rho=-0.7, mark="rolling_atm")

MONITOR_KEYWORDS = ("per_share_step_pnl", "raw_pnl_deviation_abs", "transaction_costs_total")
# host_io="auto": the NumPy step path (step_wait) of up to this many envs steps through
# host-mapped memory (he_host_alloc): no DMA, one launch, the kernel-raised completion word.
# The crossover (MI355X, step_async + step_wait with Monitor, profiles/r06h_host_io_scan.txt):
# 53 against 67 us at 8,192 envs, 105 against 79 us at 16,384 (the kernel's PCIe writes).
HOST_IO_MAX_ENVS = 8192

_TORCH_DT = {"f8": torch.float64, "f4": torch.float32, "i4": torch.int32}
_NP_DT = {torch.float64: np.float64, torch.float32: np.float32, torch.int32: np.int32}
_ROW_KIND = {np.dtype(np.float64): "d", np.dtype(np.float32): "f", np.dtype(np.int32): "i"}
# the current stream's raw handle (torch's own accessor; current_stream().cuda_stream builds a
# Stream object per call, a few us of every eager step)
_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None) or \
    (lambda idx: torch.cuda.current_stream(idx).cuda_stream)


def _align(x, a):
    return -(-x // a) * a


def load_npz_tables(data_file_path):
    """np.load + f32 cast + shape check exactly as hedging_env_v2.py:36-48."""
    try:
        data = np.load(data_file_path)
        S = data["paths"].astype(np.float32)
        v = data["volatilities"].astype(np.float32)
        C = data["call_prices_atm"].astype(np.float32)
        P = data["put_prices_atm"].astype(np.float32)
    except Exception as e:  # same exception contract as the reference
        raise FileNotFoundError(f"Could not load or parse data from {data_file_path}. Error: {e}")
    check_table_shapes(S, v, C, P)
    return S, v, C, P


def check_table_shapes(S, v, C, P):
    if not (S.ndim == 2 and S.shape == v.shape and S.shape[0] == C.shape[0] == P.shape[0]
            and S.shape[1] == C.shape[1] + 1 == P.shape[1] + 1):
        raise ValueError("Data shapes are inconsistent.")


class HedgingVecEnv:
    """Batched, device-resident `HedgingEnv` x n_envs.

    Replay mode (reference semantics): pass `data_file_path` (NPZ with paths,
    volatilities, call_prices_atm, put_prices_atm) or `tables=(S, v, C, P)`.
    Generate modes: `mode="gbm"` / `"heston"`, market in `generate=dict(...)`;
    `generate["mark"]` = "rolling_atm" (default: the 30-day ATM option re-struck every
    step, rbergomi_sim.py:418,437-446) or "fixed_european" (one option per episode at
    K = round(S0), T = max(1 - t/252, 0), option_price_assignment.py:10-21,33-49).
    `generate["book"]` = list of up to 8 dicts {type: "call"|"put"|"uo_call",
    strike, expiry (steps), quantity (contracts, < 0 short), barrier} is the
    per-env liability book (extension, include/hedge_env.h he_book_option).
    Remaining keywords are the reference HedgingEnv ctor keywords.
    """

    def __init__(self, n_envs, data_file_path=None, *, tables=None, variant=2, mode=None,
                 generate=None, device=None, seed=None, global_env_offset=0, autoreset=True,
                 return_numpy=True, info_keys=MONITOR_KEYWORDS, monitor_keywords=None, freeze_infos=True,
                 market_block=64, market_prefetch="auto", check_finite=False, host_io="auto", **env_kwargs):
        self.lib = _lib.load()
        self.num_envs = int(n_envs)
        self.variant = int(variant)
        if mode is None:
            mode = "replay" if (data_file_path is not None or tables is not None) else "gbm"
        self.mode = mode
        base = V2_DEFAULTS if self.variant == 2 else V1_DEFAULTS
        unknown = set(env_kwargs) - set(base)
        if unknown:
            raise TypeError(f"HedgingEnv() got unexpected keyword arguments {sorted(unknown)}")
        kw = dict(base, **env_kwargs)
        self.env_kwargs = kw
        gen = dict(GENERATE_DEFAULTS, **(generate or {}))
        book = list(gen.pop("book", None) or ())
        self.generate = gen
        self.book = book
        self.device = torch.device(device if device is not None else "cuda:0")
        if self.device.type != "cuda":
            raise _lib.HedgeEnvError("HedgingVecEnv runs on a HIP device (cuda:N); there is no CPU path")
        if not torch.cuda.is_available():
            raise _lib.HedgeEnvError("no HIP device visible: libhedgeenv needs an MI355X")
        dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.device = torch.device("cuda", dev_index)
        self._dev_index = dev_index

        cfg = _lib.HeConfig()
        _lib.check(self.lib, None, self.lib.he_config_init(cfg, self.variant), "he_config_init")
        cfg.mode = _lib.MODES[mode]
        cfg.loss_type = _lib.loss_code(kw["loss_type"])
        cfg.n_envs = self.num_envs
        cfg.global_env_offset = int(global_env_offset)
        cfg.transaction_cost_per_contract = float(kw["transaction_cost_per_contract"])
        cfg.lambda_cost = float(kw["lambda_cost"])
        cfg.pnl_penalty_weight = float(kw["pnl_penalty_weight"])
        cfg.theta_weight = float(kw.get("theta_weight", 0.0))
        cfg.slippage_bps = float(kw.get("slippage_bps", 0.0))
        cfg.initial_cash = float(kw["initial_cash"])
        cfg.shares_to_hedge = int(kw["shares_to_hedge"])
        cfg.max_contracts_held_per_type = int(kw["max_contracts_held_per_type"])
        cfg.max_trade_per_step = int(kw["max_trade_per_step"])
        cfg.record_metrics = 1 if kw["record_metrics"] else 0
        cfg.autoreset = 1 if autoreset else 0
        cfg.device = dev_index
        cfg.episode_length = int(gen["episode_length"])
        cfg.s0 = float(gen["s0"])
        cfg.variance = float(gen["variance"])
        cfg.mu = float(gen["mu"])
        cfg.dt = float(gen["dt"])
        cfg.heston_kappa = float(gen["heston_kappa"])
        cfg.heston_theta = float(gen["heston_theta"])
        cfg.heston_xi = float(gen["heston_xi"])
        cfg.heston_rho = float(gen["heston_rho"])
        cfg.market_block = int(market_block)
        mark = gen["mark"]
        if mark not in _lib.MARKS:
            raise ValueError(f"mark must be one of {sorted(_lib.MARKS)}, not {mark!r}")
        if mode == "replay" and mark != "rolling_atm":
            raise ValueError("replay mode reads its marks from the table (mark='rolling_atm')")
        cfg.mark = _lib.MARKS[mark]
        if book:
            if mode == "replay":
                raise ValueError("the liability book needs a generate mode (gbm / heston)")
            if len(book) > _lib.HE_BOOK_MAX:
                raise ValueError(f"at most {_lib.HE_BOOK_MAX} book options")
            cfg.book_size = len(book)
            for k, o in enumerate(book):
                typ = o["type"]
                cfg.book[k].type = _lib.BOOK_TYPES[typ] if isinstance(typ, str) else int(typ)
                cfg.book[k].expiry = int(o["expiry"])
                cfg.book[k].strike = float(o["strike"])
                cfg.book[k].barrier = float(o.get("barrier", 0.0))
                cfg.book[k].quantity = float(o["quantity"])
        if os.environ.get("CANTORRL_NO_PREFETCH"):
            market_prefetch = False
        # 0 auto (rollouts, or single steps from 131,072 envs), 1 never, 2 always
        cfg.market_prefetch = 0 if market_prefetch == "auto" else (2 if market_prefetch else 1)
        base_seed = int(seed if seed is not None else gen.get("seed", 42))
        cfg.seed = base_seed
        self._cfg = cfg
        handle = _lib.ctypes.c_void_p()
        st = self.lib.he_create(cfg, _lib.ctypes.byref(handle))
        self._h = handle
        _lib.check(self.lib, handle, st, "he_create")

        if mode == "replay":
            if tables is None:
                S, v, C, P = load_npz_tables(data_file_path)
            else:
                S, v, C, P = (np.ascontiguousarray(np.asarray(x).astype(np.float32)) for x in tables)
                check_table_shapes(S, v, C, P)
            S, v, C, P = (np.ascontiguousarray(x) for x in (S, v, C, P))
            st = self.lib.he_load_paths(self._h, S.ctypes.data, v.ctypes.data, C.ctypes.data,
                                        P.ctypes.data, S.shape[0], S.shape[1])
            _lib.check(self.lib, self._h, st, "he_load_paths")
            self.num_episodes = int(S.shape[0])
            self.episode_length = int(S.shape[1] - 1)
        else:
            self.num_episodes = None
            self.episode_length = int(gen["episode_length"])

        n = self.num_envs
        dev = self.device
        self._act = torch.zeros((n, 2), dtype=torch.float32, device=dev)
        self._tobs = torch.zeros((n, 13), dtype=torch.float32, device=dev)
        self.info_keys = tuple(info_keys or ())
        self.monitor_keywords = tuple(monitor_keywords) if monitor_keywords else None
        # Monitor sums the env's own f64 reward (it wraps each env inside the VecEnv,
        # train_ppo_v2.py:119; hedging_env_v2.py:262,294), so with monitor_keywords the step
        # also writes info["reward_step"] -- a hidden column unless the caller asked for it
        layout_keys = self.info_keys
        if self.monitor_keywords is not None and "reward_step" not in layout_keys:
            layout_keys = layout_keys + ("reward_step",)
        self._row_keys = self.info_keys
        self._info_t = {}
        self._info = _lib.HeInfo()
        known = dict(_lib.INFO_FIELDS)
        # ONE device buffer holds everything a host caller reads after a step:
        #   [obs f32 N x 13 | reward f32 N | terminated u8 N | truncated u8 N | info fields]
        # with every info field 256-B aligned.  step_wait copies the obs / reward / terminated
        # prefix to the host as one DMA and HedgingEnv.step the whole buffer (~7 KB at N = 1);
        # freezing an InfoView is one device copy of the info part, not one per key.
        o_rew, o_term = 52 * n, 56 * n
        o_trunc, end = o_term + n, o_term + 2 * n
        self._io_step_bytes = o_trunc            # obs + reward + terminated
        info0 = _align(end, 256)
        offs, tot = [], 0
        for k in layout_keys:
            if k not in known:
                raise KeyError(f"unknown info key {k!r}")
            dt = _TORCH_DT[known[k]]
            offs.append((k, dt, tot))
            tot += _align(n * torch.empty((), dtype=dt).element_size(), 256)
        self._io = torch.zeros(info0 + tot, dtype=torch.uint8, device=dev)
        self._obs = self._io[:o_rew].view(torch.float32).view(n, 13)
        self._rew = self._io[o_rew:o_term].view(torch.float32)
        self._term = self._io[o_term:o_trunc]
        self._trunc = self._io[o_trunc:end]
        self._io_info0 = info0
        self._info_flat = self._io[info0:]
        for k, dt, o in offs:
            t = self._info_flat[o:o + n * torch.empty((), dtype=dt).element_size()].view(dt)
            self._info_t[k] = t
            setattr(self._info, k, t.data_ptr())
        self._info_offs = offs
        self._ev = torch.cuda.Event()   # the one host wait of a host pull (_pull)
        self._step_args = (self._obs.data_ptr(), self._rew.data_ptr(), self._term.data_ptr(), self._trunc.data_ptr(),
                           self._tobs.data_ptr(), _lib.ctypes.byref(self._info) if self._info_t else None)
        # InfoView snapshots (see InfoView): freeze_infos=False skips them (a view read after
        # a later step then shows that step's values)
        self.freeze_infos = bool(freeze_infos)
        self.return_numpy = bool(return_numpy)
        self._rew64 = self._info_t.get("reward_step")   # the f64 rewards (Monitor's sums)
        self._pending_seeds = None
        self._live_view = None  # weakref to the newest InfoView (see InfoView)
        self._actions_pending = None
        # Monitor (monitor_keywords): each env's running sum of its f64 rewards on the device
        # (sum(float(r)) of Monitor.step, the same additions in the same order), and the
        # episode length as (steps so far - the step the env's episode began), so a step
        # that ends no episode costs the host nothing
        self._ep_ret = torch.zeros(n, dtype=torch.float64, device=dev)
        self._ep_start = np.zeros(n, np.int64)
        self._steps = 0
        # failure detection: device count of non-finite obs / reward values since
        # construction (he_count_nonfinite after every step when check_finite)
        self.check_finite = bool(check_finite)
        self._nonfinite = torch.zeros(1, dtype=torch.int64, device=dev)
        self._t_start = time.time()
        # the small-N host path (step_wait, HedgingEnv.step): actions in and every output out
        # through one host-mapped block the step kernel reads and writes itself (_HostIo);
        # Monitor's sums then live on the host too (the same f64 additions)
        if host_io == "auto":
            host_io = self.return_numpy and n <= HOST_IO_MAX_ENVS
        self._hio = _HostIo(self) if host_io else None
        self._ep_ret_h = np.zeros(n, np.float64)

        if self.return_numpy:
            # the host path's pinned blocks (step outputs, actions, the episode-end pull), made
            # now: a first hipHostMalloc costs milliseconds, inside a step it would be that step's
            self._warm_pinned([self._io_step_bytes] * 3 + [8 * n] * 2 + [52 * n, self._info_flat.numel(), 8 * n])
        if self.monitor_keywords is not None:
            # the Monitor sums' torch kernels, loaded now (a first launch loads the code object:
            # tens of ms, which the first episode end would otherwise pay)
            self._ep_ret.add_(self._rew64)
            self._ep_ret.masked_fill_(self._term.bool(), 0.0)
            self._ep_ret.zero_()
        self.action_space = Box(-1.0, 1.0, (2,), np.float32)
        self.observation_space = Box(OBS_LOW, OBS_HIGH, (13,), np.float32)
        # reference attribute names (hedging_env_v2.py:53-58) + the documented alias
        self.transaction_cost_per_contract = kw["transaction_cost_per_contract"]
        self.max_contracts_held = kw["max_contracts_held_per_type"]
        self.shares_held_fixed = kw["shares_to_hedge"]
        self.option_contract_multiplier = 100
        self.risk_free_rate = 0.04
        self.option_tenor_years = 30 / 252
        self.max_trade_per_step = kw["max_trade_per_step"]
        self._max_trade_per_step_internal = kw["max_trade_per_step"]
        self.loss_type = kw["loss_type"]
        self.record_metrics = kw["record_metrics"]

    # ------------------------------------------------------------------ plumbing
    @property
    def stream(self):
        """The caller's current stream on the env device (raw handle)."""
        return _raw_stream(self._dev_index)

    def _ptr(self, t):
        return t.data_ptr() if t is not None else None

    def _pull(self, srcs):
        """Device tensors -> numpy arrays in pinned host memory: one async copy each on the
        current stream (behind the step that wrote them), then ONE event wait.  The pinned
        blocks come from torch's caching host allocator, so each returned array owns its
        memory (nothing is overwritten by a later step) and allocation is a cache hit."""
        outs = []
        for t in srcs:
            h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
            h.copy_(t, non_blocking=True)
            outs.append(h)
        self._ev.record(torch.cuda.current_stream(self.device))
        self._ev.synchronize()
        return [h.numpy() for h in outs]

    @staticmethod
    def _warm_pinned(sizes):
        """Allocate pinned blocks of these byte sizes together and free them: torch's caching
        host allocator keeps them, so later pulls of those sizes are cache hits."""
        blocks = [torch.empty(max(int(b), 1), dtype=torch.uint8, pin_memory=True) for b in sizes]
        del blocks

    def _host_actions(self, actions):
        """Host actions -> self._act through a pinned staging block (an async DMA; a
        pageable source would make the copy synchronous)."""
        a = torch.as_tensor(actions, dtype=torch.float32).reshape(self.num_envs, 2)
        if not a.is_pinned():
            stage = torch.empty((self.num_envs, 2), dtype=torch.float32, pin_memory=True)
            stage.copy_(a)
            a = stage
        self._act.copy_(a, non_blocking=True)
        return self._act

    def _split_info(self, flat):
        """Host bytes of the info part of the io buffer -> {key: numpy array}."""
        n = self.num_envs
        return {k: flat[o:o + n * np.dtype(_NP_DT[dt]).itemsize].view(_NP_DT[dt]) for k, dt, o in self._info_offs}

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            torch.cuda.synchronize(self.device)
            self.lib.he_destroy(self._h)
            self._h = _lib.ctypes.c_void_p()
        hio = getattr(self, "_hio", None)
        if hio is not None:
            hio.free()
            self._hio = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ seeding
    def seed(self, seed=None):
        """SB3 semantics: env i gets seed + i, applied at the next reset()."""
        if seed is None:
            seed = int(np.random.randint(0, 2 ** 31 - 1))
        seeds = [int(seed) + i for i in range(self.num_envs)]
        # generate modes key every env's Philox stream by (seed, global id): one seed
        self._pending_seeds = seeds if self.mode == "replay" else seeds[:1]
        return seeds

    def seed_envs(self, seeds, env_ids=None):
        """Per-env reset(seed=...) re-seeding (replay).  Generate modes have one Philox
        key per handle (env i's stream is keyed by its global id): exactly one seed, and
        env_ids are refused (he_seed: HE_EINVAL)."""
        seeds = np.ascontiguousarray(np.asarray(seeds, dtype=np.uint64)).reshape(-1)
        if self.mode != "replay" and len(seeds) != 1:
            raise ValueError(f"{self.mode} mode takes one seed per handle (env i's Philox stream is "
                             f"keyed by the seed and its global id), got {len(seeds)}")
        ids = None if env_ids is None else np.ascontiguousarray(np.asarray(env_ids, dtype=np.int64))
        st = self.lib.he_seed(self._h, None if ids is None else ids.ctypes.data, seeds.ctypes.data,
                              len(seeds))
        _lib.check(self.lib, self._h, st, "he_seed")

    # ------------------------------------------------------------------ reset
    def _retire_view(self):
        """Freeze the newest InfoView (if still alive) before its buffers are overwritten."""
        r, self._live_view = self._live_view, None
        v = r() if r is not None else None
        if v is not None and self.freeze_infos:
            v._freeze()

    def _info_snapshot(self):
        """One device copy of every info field (the info part of the io buffer)."""
        return self._info_flat.clone()

    def _monitor_reset(self):
        self._ep_ret.zero_()
        self._ep_ret_h[:] = 0.0
        self._ep_start[:] = 0
        self._steps = 0

    def reset_tensors(self, env_ids=None, episode_idx=None):
        """Reset every env (or `env_ids`) and return the obs tensor.  episode_idx (replay mode):
        the episode row of each reset env, drawn by the caller (he_reset_episodes) instead of
        by the env's own PCG64 stream -- one per env in env_ids order (all envs when env_ids
        is None)."""
        self._retire_view()
        if self._pending_seeds is not None:
            self.seed_envs(self._pending_seeds)
            self._pending_seeds = None
        info = _lib.ctypes.byref(self._info) if self._info_t else None
        if episode_idx is not None:
            eps = np.ascontiguousarray(np.asarray(episode_idx, dtype=np.int64).reshape(-1))
            ids = None
            if env_ids is not None:
                ids = torch.as_tensor(env_ids, dtype=torch.int64, device=self.device).reshape(-1)
                if ids.numel() != eps.size:
                    raise ValueError(f"{eps.size} episode indices for {ids.numel()} envs")
            elif eps.size != self.num_envs:
                raise ValueError(f"{eps.size} episode indices for {self.num_envs} envs")
            st = self.lib.he_reset_episodes(self._h, None if ids is None else ids.data_ptr(),
                                            eps.ctypes.data, eps.size, self._obs.data_ptr(), info, self.stream)
            _lib.check(self.lib, self._h, st, "he_reset_episodes")
            if env_ids is None:
                self._monitor_reset()
            return self._obs
        if env_ids is None:
            st = self.lib.he_reset(self._h, None, self.num_envs, self._obs.data_ptr(), info, self.stream)
        else:
            ids = torch.as_tensor(env_ids, dtype=torch.int64, device=self.device)
            st = self.lib.he_reset(self._h, ids.data_ptr(), ids.numel(), self._obs.data_ptr(), info,
                                   self.stream)
        _lib.check(self.lib, self._h, st, "he_reset")
        if env_ids is None:
            self._monitor_reset()
        return self._obs

    def reset(self):
        obs = self.reset_tensors()
        return self._pull([obs])[0] if self.return_numpy else obs

    # ------------------------------------------------------------------ step
    def step_tensors(self, actions, terminal_obs=True, info=True):
        """Device path: actions [N,2] (tensor on the env device or array) ->
        (obs, reward, terminated, truncated) device tensors; no host sync."""
        if isinstance(actions, torch.Tensor) and actions.device == self.device \
                and actions.dtype == torch.float32 and actions.is_contiguous():
            act = actions
        elif isinstance(actions, torch.Tensor) and actions.is_cuda:
            self._act.copy_(actions.reshape(self.num_envs, 2), non_blocking=True)
            act = self._act
        else:
            act = self._host_actions(actions)
        self._retire_view()
        # the output pointers are fixed allocations: marshalled once (_step_args)
        o, r, t, tr, tob, inf = self._step_args
        st = self.lib.he_step(self._h, act.data_ptr(), o, r, t, tr, tob if terminal_obs else None,
                              inf if info else None, _raw_stream(self._dev_index))
        _lib.check(self.lib, self._h, st, "he_step")
        if self.check_finite:
            for t in (self._obs, self._rew):
                _lib.check(self.lib, self._h, self.lib.he_count_nonfinite(t.data_ptr(), t.numel(),
                                                                          self._nonfinite.data_ptr(), self.stream),
                           "he_count_nonfinite")
        return self._obs, self._rew, self._term, self._trunc

    def nonfinite_count(self):
        """Non-finite obs / reward values produced so far (check_finite=True); syncs."""
        return int(self._nonfinite.item())

    def step_async(self, actions):
        self._actions_pending = actions

    def step_wait(self):
        actions = self._actions_pending
        self._actions_pending = None
        if self._hio is not None and self.return_numpy:
            return self._step_wait_host(actions)
        obs, rew, term, _ = self.step_tensors(actions)
        self._steps += 1
        if not self.return_numpy:   # device results: Monitor's episodes are not reported
            return obs, rew, term.bool(), InfoView(self, None)
        if self.monitor_keywords is not None:
            self._ep_ret.add_(self._rew64)   # Monitor.step: the env's f64 reward
        # obs, reward and terminated are adjacent in the io buffer: one DMA, one wait
        n = self.num_envs
        h = self._pull([self._io[:self._io_step_bytes]])[0]
        obs_h = h[:52 * n].view(np.float32).reshape(n, 13)
        rew_h = h[52 * n:56 * n].view(np.float32)
        done_h = h[56 * n:57 * n].view(np.bool_)   # the kernels store 0 / 1
        infos = InfoView(self, done_h)
        if done_h.any():
            infos._materialize_done(done_h)
        return obs_h, rew_h, done_h, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def step_host(self, actions):
        """One he_step through the host-mapped block (host_io): the actions are written into
        it, the kernel reads them and writes obs / reward / flags / terminal obs / info fields
        back into it, and one stream wait ends the step.  Returns the block (_HostIo); its
        arrays hold this step's outputs until the next step_host."""
        z = self._hio
        np.copyto(z.act, np.asarray(actions, dtype=np.float32).reshape(self.num_envs, 2))
        self._retire_view()
        lib, h = self.lib, self._h
        stream = _raw_stream(self._dev_index)
        if not self.check_finite:
            # the step kernel raises the block's flag word after its outputs (he_step_signal):
            # the host reads it instead of waiting for the runtime's completion (~5 us less)
            _lib.check(lib, h, lib.he_step_signal(h, z.d_flag), "he_step_signal")
            _lib.check(lib, h, lib.he_step(h, *z.step_args, stream), "he_step")
            _lib.check(lib, h, lib.he_signal_wait(h, z.h_flag, stream), "he_signal_wait")
            return z
        _lib.check(lib, h, lib.he_step(h, *z.step_args, stream), "he_step")
        for p, c in ((z.d_obs, 13 * self.num_envs), (z.d_rew, self.num_envs)):
            _lib.check(lib, h, lib.he_count_nonfinite(p, c, self._nonfinite.data_ptr(), self.stream),
                       "he_count_nonfinite")
        _lib.check(lib, h, lib.he_stream_wait(stream), "he_stream_wait")
        return z

    def _step_wait_host(self, actions):
        """step_wait of the host_io path: the step's outputs are copied out of the mapped block
        once (private arrays: a later step never overwrites them), the info view starts with
        its host columns, and the Monitor sums are host f64 additions of the env's rewards."""
        z = self.step_host(actions)
        self._steps += 1
        n = self.num_envs
        h = z.io.copy()
        obs_h = h[:52 * n].view(np.float32).reshape(n, 13)
        rew_h = h[52 * n:56 * n].view(np.float32)
        done_h = h[56 * n:57 * n].view(np.bool_)   # the kernels store 0 / 1
        infos = InfoView(self, done_h)
        host = infos._host = self._split_info(h[self._io_info0:])
        mon = self.monitor_keywords is not None
        if mon:
            self._ep_ret_h += host["reward_step"]   # Monitor.step: the env's f64 reward
        if done_h.any():
            er = el = None
            if mon:
                er = self._ep_ret_h.copy()
                el = self._steps - self._ep_start
                self._ep_ret_h[done_h] = 0.0
                self._ep_start[done_h] = self._steps
            infos._ends = (z.tobs.copy(), er, el, round(time.time() - self._t_start, 6), mon)
        return obs_h, rew_h, done_h, infos

    def sync_market(self):
        """Join the library's market prefetch into the current stream (call before
        ending a hipGraph capture that contains steps)."""
        _lib.check(self.lib, self._h, self.lib.he_sync_market(self._h, self.stream), "he_sync_market")

    def rollout(self, actions, obs=None, reward=None, terminated=None):
        """K fused steps: actions [K,N,2] device tensor -> writes obs [K,N,13],
        reward [K,N], terminated [K,N] (allocated if None)."""
        K = int(actions.shape[0])
        n = self.num_envs
        dev = self.device
        if obs is None:
            obs = torch.empty((K, n, 13), dtype=torch.float32, device=dev)
        if reward is None:
            reward = torch.empty((K, n), dtype=torch.float32, device=dev)
        if terminated is None:
            terminated = torch.empty((K, n), dtype=torch.uint8, device=dev)
        actions = actions.to(device=dev, dtype=torch.float32).contiguous()
        st = self.lib.he_rollout(self._h, K, actions.data_ptr(), self._ptr(obs), self._ptr(reward),
                                 self._ptr(terminated), self.stream)
        _lib.check(self.lib, self._h, st, "he_rollout")
        return obs, reward, terminated

    def episode_summaries(self, out=None):
        """[N, 4] f32 device tensor: {return, sum of step P&L, sum of costs, length} of each
        env's most recently finished episode (he_episode_summaries; generate-mode rollouts
        and policy rollouts keep them)."""
        if out is None:
            out = torch.empty((self.num_envs, 4), dtype=torch.float32, device=self.device)
        _lib.check(self.lib, self._h, self.lib.he_episode_summaries(self._h, out.data_ptr(), self.stream),
                   "he_episode_summaries")
        return out

    def rollout_policy(self, k_steps, policy, actions_out=None, obs=None, reward=None, terminated=None,
                       records=None, record_count=None):
        """k_steps fused steps driven by a baseline policy evaluated on the device
        (he_rollout_policy): "no_hedge" / "delta_every_step" (baselines.py:74-103) or
        "delta_threshold" (delta_and_nothing.py:122-163).  Finished episodes append
        he_episode_record rows to `records` (uint8 device tensor [cap, 80]) at the
        index taken from `record_count` (int64 device tensor [1])."""
        pol = _lib.POLICIES[policy] if isinstance(policy, str) else int(policy)
        K = int(k_steps)
        cap = 0 if records is None else int(records.shape[0])
        st = self.lib.he_rollout_policy(self._h, K, pol, self._ptr(actions_out), self._ptr(obs), self._ptr(reward),
                                        self._ptr(terminated), self._ptr(records), cap, self._ptr(record_count),
                                        self.stream)
        _lib.check(self.lib, self._h, st, "he_rollout_policy")

    def evaluate_policy(self, policy, num_episodes, chunk=64, max_steps=None):
        """Run `policy` until `num_episodes` episodes finished (all envs stepping) and
        return the per-episode records as a numpy structured array (he_episode_record):
        the device-side evaluate_baseline_policy (baselines.py:32-72)."""
        dev = self.device
        cap = int(num_episodes) + self.num_envs
        recs = torch.zeros((cap, _lib.EPISODE_RECORD.itemsize), dtype=torch.uint8, device=dev)
        cnt = torch.zeros(1, dtype=torch.int64, device=dev)
        steps = 0
        limit = max_steps if max_steps is not None else (num_episodes // self.num_envs + 2) * (self.episode_length + 1)
        while True:
            self.rollout_policy(chunk, policy, records=recs, record_count=cnt)
            steps += chunk
            done = int(cnt.item())
            if done >= num_episodes or steps >= limit:
                break
        n = min(int(cnt.item()), cap)
        out = recs[:n].cpu().numpy().view(_lib.EPISODE_RECORD).reshape(n)
        return out[:num_episodes]

    # ------------------------------------------------------------------ attrs
    def _indices(self, indices):
        if indices is None:
            return range(self.num_envs)
        if isinstance(indices, int):
            return [indices]
        return indices

    def get_attr(self, attr_name, indices=None):
        val = getattr(self, attr_name)
        return [val for _ in self._indices(indices)]

    def set_attr(self, attr_name, value, indices=None):
        raise NotImplementedError("env attributes are fixed at construction (device-side config)")

    def env_method(self, method_name, *args, indices=None, **kwargs):
        if method_name in ("render", "close"):
            return [None for _ in self._indices(indices)]
        raise NotImplementedError(f"env_method({method_name!r}) is not supported")

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False for _ in self._indices(indices)]

    def get_state(self):
        size = self.lib.he_state_size(self._h)
        buf = np.empty(size, np.uint8)
        torch.cuda.synchronize(self.device)
        _lib.check(self.lib, self._h, self.lib.he_get_state(self._h, buf.ctypes.data, size), "he_get_state")
        return buf

    def set_state(self, buf):
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        torch.cuda.synchronize(self.device)
        _lib.check(self.lib, self._h, self.lib.he_set_state(self._h, buf.ctypes.data, buf.size), "he_set_state")

    def info_tensor(self, key):
        return self._info_t[key]


class _HostIo:
    """The host-mapped block of the small-N host path (he_host_alloc): the env's io layout
    [obs | reward | terminated | truncated | info fields] (as the device io buffer), then the
    actions [N, 2], the terminal obs [N, 13] and the step's completion flag (one u32), each 256-B
    aligned.  The step kernel reads the actions and writes everything else in place."""

    def __init__(self, venv):
        lib, n = venv.lib, venv.num_envs
        c = _lib.ctypes
        self.lib = lib
        io_b = venv._io.numel()
        a_off = _align(io_b, 256)
        t_off = _align(a_off + 8 * n, 256)
        f_off = _align(t_off + 52 * n, 256)   # the step's completion flag (he_step_signal)
        total = f_off + 4
        hp, dp = c.c_void_p(), c.c_void_p()
        _lib.check(lib, None, lib.he_host_alloc(total, c.byref(hp), c.byref(dp)), "he_host_alloc")
        self.host = hp.value
        base = np.frombuffer((c.c_uint8 * total).from_address(hp.value), np.uint8)
        d = dp.value
        self.io = base[:io_b]
        self.act = base[a_off:a_off + 8 * n].view(np.float32).reshape(n, 2)
        self.tobs = base[t_off:t_off + 52 * n].view(np.float32).reshape(n, 13)
        self.d_obs, self.d_rew = d, d + 52 * n
        self.d_flag, self.h_flag = d + f_off, hp.value + f_off
        self.info = _lib.HeInfo()
        for k, dt, o in venv._info_offs:
            setattr(self.info, k, d + venv._io_info0 + o)
        self.step_args = (d + a_off, d, d + 52 * n, d + 56 * n, d + 57 * n, d + t_off,
                          c.byref(self.info) if venv._info_offs else None)

    def free(self):
        if self.host:
            self.lib.he_host_free(self.host)
            self.host = None


class InfoView(_info_rows.Rows):
    """The step's `infos`: SB3's list of per-env info dicts, over the device info SoA.

    Rows come from the C module csrc/info_rows.c: a row answers row[k] / row.get(k) / k in row
    straight from the step's host columns, and becomes a plain dict only when something needs
    the whole mapping (keys, items, iteration, copy, an assignment -- SB3's VecNormalize writing
    a normalized terminal_observation).  SB3 reads every row every step (collect_rollouts'
    info.get("episode") / info.get("is_success")): that costs a few ms at 65,536 envs, where a
    dict per row costs 20+ (bench.py's sb3_loop line).  A done row's "terminal_observation"
    and Monitor "episode" are made when they are first read.

    The view reads the env's live info buffers, copied to the host on the first row access.
    It is the env's newest view until the env's next step or reset, which first freezes it
    when it is still alive and has not been read: a view read after later steps still shows
    its own step.  In SB3's loop (`obs, r, d, infos = env.step(a)`) the previous `infos` is
    still referenced while step() runs, so a step usually pays the freeze: ONE device copy
    of the info fields' flat buffer, not one per key.  freeze_infos=False (env constructor)
    drops the snapshots for callers that read infos before the next step.  The done rows'
    data (terminal obs, Monitor episode sums) is pulled by step_wait right away, from the
    live buffers, in the same single copy as the info fields."""

    def __init__(self, venv, done):
        self._v = venv
        self._done = done
        self._host = None
        self._snap = None
        self._ends = None   # done rows' host data (_materialize_done)
        venv._retire_view()
        venv._live_view = weakref.ref(self)

    def __len__(self):   # no host copy for len()
        return self._v.num_envs

    def _freeze(self):
        if self._host is None and self._snap is None and self._v._info_t:
            self._snap = self._v._info_snapshot()

    def _host_info(self, pulled=None):
        """Host copy of the view's info fields: ONE copy of the info bytes (live or frozen)."""
        if self._host is None:
            v = self._v
            if pulled is None:
                src = self._snap if self._snap is not None else v._info_flat
                pulled = v._pull([src])[0]
            self._host = v._split_info(pulled)
            self._snap = None
        return self._host

    def _load(self):
        """First row access (info_rows.c): attach the host columns to the C rows."""
        v = self._v
        h = self._host_info() if v._info_t else {}
        keys = tuple(k for k in v._row_keys if k in h)
        cols = tuple(h[k] for k in keys)
        kinds = "".join(_ROW_KIND[c.dtype] for c in cols).encode()
        ends = None
        done = None
        done_keys = ()
        if self._ends is not None:
            done = self._done
            mon = self._ends[4]
            done_keys = ("terminal_observation", "episode") if mon else ("terminal_observation",)
            ends = _episode_ends(self._ends, h, v.monitor_keywords)
        self._attach(keys, cols, kinds, v.num_envs, "TimeLimit.truncated", False, done, done_keys, ends)

    def _materialize_done(self, done):
        """Done rows (called by step_wait before any later step): this step's terminal obs,
        info fields and, with Monitor, episode sums come to the host now -- one pull -- and
        the rows' extra items are made when they are read."""
        v = self._v
        mon = v.monitor_keywords is not None
        srcs = [v._tobs]
        if self._host is None:
            srcs.append(self._snap if self._snap is not None else v._info_flat)
        if mon:
            srcs.append(v._ep_ret)
        got = v._pull(srcs)
        self._host_info(got[1] if self._host is None else None)
        er = el = None
        if mon:
            er = got[-1]
            el = v._steps - v._ep_start   # a new array: _ep_start moves on below
            v._ep_ret.masked_fill_(v._term.bool(), 0.0)   # the new episodes start at 0
            v._ep_start[np.nonzero(done)[0]] = v._steps
        self._ends = (got[0], er, el, round(time.time() - v._t_start, 6), mon)


def _episode_ends(ends, host, monitor_keywords):
    """ends(i) of a done row: {"terminal_observation", "episode"} (SB3 DummyVecEnv and
    Monitor.step: r = round(sum of the episode's f64 rewards, 6), l, t, + info_keywords).
    Holds the host arrays only (no reference back to the view)."""
    tobs, er, el, t, mon = ends

    def row_ends(i):
        d = {"terminal_observation": tobs[i].copy()}
        if mon:
            ep = {"r": round(float(er[i]), 6), "l": int(el[i]), "t": t}
            for k in monitor_keywords:
                ep[k] = host[k][i].item() if k in host else None
            d["episode"] = ep
        return d
    return row_ends


# the rows are mappings (isinstance(row, collections.abc.Mapping), dict(row), **row)
import collections.abc  # noqa: E402
collections.abc.MutableMapping.register(_info_rows.Row)
