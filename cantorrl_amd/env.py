"""HedgingEnv: the reference's single-env gym API on top of libhedgeenv.

Same constructor signature and defaults as bcosm/CantorRL's
`src/env/hedging_env_v2.py:10-22` (`HedgingEnv`) and `src/env/hedging_env.py:10-20`
(`HedgingEnvV1`), same `reset(seed, options) -> (obs, {})` /
`step(action) -> (obs, reward, terminated, truncated, info)` contract
(hedging_env_v2.py:145-294), same attribute names read by the reference's
baseline and benchmark scripts (src/agents/baselines.py:74-103,
src/benchmark/delta_and_nothing.py:70-88).  The env is a 1-env handle on the GPU
(no auto-reset: the caller resets, as with any gym env); use HedgingVecEnv for
batches.

Superset: `max_trade_per_step` is exposed as an attribute (the reference only
has `_max_trade_per_step_internal`, so its delta baseline raises AttributeError).
"""
import numpy as np
import torch

from . import _lib
from .vec_env import (HedgingVecEnv, OBS_HIGH, OBS_LOW)
from .spaces import Box

# the info fields HedgingEnv.step reads from the step's block, by dtype (hedging_env_v2.py:268-293)
_STEP_F8 = ["step_pnl_total", "per_share_step_pnl", "raw_pnl_deviation_abs", "transaction_costs_total",
            "commission_cost", "slippage_cost", "reward_pnl_component", "transaction_cost_penalty",
            "theta_penalty", "reward_step", "portfolio_value", "cash"]
_STEP_I4 = ["call_contracts", "put_contracts", "requested_calls_rounded_clipped", "requested_puts_rounded_clipped",
            "actual_calls_traded", "actual_puts_traded", "current_step"]
_STEP_F4 = ["scaled_float_call", "scaled_float_put", "current_stock_price", "current_volatility",
            "current_call_price", "current_put_price"]


class HedgingEnv:
    """hedging_env_v2.HedgingEnv, GPU-backed.  Extra keyword-only arguments select
    the market source: `data_file_path` (replay, reference semantics) or
    `mode="gbm"|"heston"` with `generate=dict(...)`."""

    metadata = {"render_modes": [], "render_fps": 1}
    _variant = 2

    def __init__(self, data_file_path=None,
                 transaction_cost_per_contract=0.65,
                 lambda_cost=1.0,
                 pnl_penalty_weight=0.01,
                 theta_weight=0.0,
                 slippage_bps=0.0,
                 loss_type="abs",
                 initial_cash=0.0,
                 shares_to_hedge=10000,
                 max_contracts_held_per_type=200,
                 max_trade_per_step=15,
                 profile_print_interval=0,
                 record_metrics=True,
                 *, mode=None, generate=None, device=None, tables=None):
        kw = dict(transaction_cost_per_contract=transaction_cost_per_contract, lambda_cost=lambda_cost,
                  pnl_penalty_weight=pnl_penalty_weight, theta_weight=theta_weight,
                  slippage_bps=slippage_bps, loss_type=loss_type, initial_cash=initial_cash,
                  shares_to_hedge=shares_to_hedge, max_contracts_held_per_type=max_contracts_held_per_type,
                  max_trade_per_step=max_trade_per_step, profile_print_interval=profile_print_interval,
                  record_metrics=record_metrics)
        self._init(data_file_path, kw, mode, generate, device, tables)

    def _init(self, data_file_path, kw, mode, generate, device, tables):
        keys = [k for k, _ in _lib.INFO_FIELDS]
        self._venv = HedgingVecEnv(1, data_file_path, tables=tables, variant=self._variant, mode=mode,
                                   generate=generate, device=device, autoreset=False, return_numpy=False,
                                   info_keys=keys, host_io=True, **kw)
        v = self._venv
        self.pnl_penalty_weight = kw["pnl_penalty_weight"]
        self.lambda_cost = kw["lambda_cost"]
        if self._variant == 2:
            self.theta_weight = kw["theta_weight"]
            self.slippage_bps = kw["slippage_bps"]
        self.loss_type = kw["loss_type"]
        self.record_metrics = kw["record_metrics"]
        self.initial_cash = kw["initial_cash"]
        self._max_trade_per_step_internal = kw["max_trade_per_step"]
        self.max_trade_per_step = kw["max_trade_per_step"]
        self.num_episodes = v.num_episodes
        self.episode_length = v.episode_length
        self.transaction_cost_per_contract = kw["transaction_cost_per_contract"]
        self.max_contracts_held = kw["max_contracts_held_per_type"]
        self.shares_held_fixed = kw["shares_to_hedge"]
        self.option_contract_multiplier = 100
        self.risk_free_rate = 0.04
        self.option_tenor_years = 30 / 252
        self.action_space = Box(low=-1.0, high=1.0, shape=(2,), dtype=np.float32)
        self.observation_space = Box(low=OBS_LOW, high=OBS_HIGH, shape=(13,), dtype=np.float32)
        self.current_episode_idx = -1
        self.current_step = 0
        self.initial_S0_for_episode = 1.0
        self._needs_reset = True
        self._terminated = False
        # host side of one step: the env's host-mapped block (HedgingVecEnv host_io,
        # he_host_alloc) -- the kernel reads the action from it and writes the obs, reward,
        # flags and every info field into it, read here through a structured dtype: one launch
        # and one stream wait per step, no DMA.  A reset (rare) writes the device io buffer and
        # comes back as one copy into a pinned mirror of the same layout.
        self._io_h = torch.zeros(v._io.numel(), dtype=torch.uint8, pin_memory=True)
        fields = {"names": ["obs", "reward", "terminated"], "formats": [("<f4", (13,)), "<f4", "u1"],
                  "offsets": [0, 52, 56]}
        for k, dt, o in v._info_offs:
            fields["names"].append(k)
            fields["formats"].append(np.dtype(dict(_lib.INFO_FIELDS)[k]))
            fields["offsets"].append(v._io_info0 + o)
        fields["itemsize"] = v._io.numel()
        rec_dt = np.dtype(fields)
        self._rec = self._io_h.numpy().view(rec_dt)   # shape (1,): a view, refreshed by each copy
        self._ev = torch.cuda.Event()
        # a step reads the mapped block by three gathers (f64, i32, f32 fields), whose numpy
        # scalars fill the info dict: ~45 structured-field reads cost more than the step itself
        offs = {k: v._io_info0 + o for k, dt, o in v._info_offs}
        self._g8 = np.array([offs[k] // 8 for k in _STEP_F8], np.intp)
        self._g4i = np.array([offs[k] // 4 for k in _STEP_I4], np.intp)
        self._g4f = np.array([offs[k] // 4 for k in _STEP_F4], np.intp)

    # ------------------------------------------------------------------ helpers
    def _fetch(self):
        """One copy of the io buffer into the pinned mirror, one wait -> the record."""
        v = self._venv
        self._io_h.copy_(v._io, non_blocking=True)
        self._ev.record(torch.cuda.current_stream(v.device))
        self._ev.synchronize()
        return self._rec[0]

    def _pull(self, h):
        self.current_stock_price = np.float32(h["current_stock_price"])
        self.current_volatility = np.float32(h["current_volatility"])
        self.current_call_price = np.float32(h["current_call_price"])
        self.current_put_price = np.float32(h["current_put_price"])
        self.current_step = int(h["current_step"])
        self.call_contracts_held = np.int64(h["call_contracts"])
        self.put_contracts_held = np.int64(h["put_contracts"])
        self.cash_balance = np.float64(h["cash"])
        return np.float32(h["initial_S0_for_episode"])

    # ------------------------------------------------------------------ gym API
    def reset(self, seed=None, options=None):
        """hedging_env_v2.py:145-173.  options={"episode_idx": k} (replay mode, an extension:
        the reference ignores options) starts episode row k instead of drawing it from
        np_random -- he_reset_episodes; the env's own stream is not advanced."""
        v = self._venv
        if seed is not None:
            v.seed_envs([int(seed)])
        ep = (options or {}).get("episode_idx")
        if ep is None:
            v.reset_tensors()
        else:
            v.reset_tensors(episode_idx=[int(ep)])
        h = self._fetch()
        o = h["obs"].copy()
        s0 = self._pull(h)
        small = bool(s0 == np.float32(1.0) and self.current_stock_price < np.float32(1e-6))
        self.initial_S0_for_episode = 1.0 if small else s0
        self.current_episode_idx = int(h["current_episode_idx"])
        self.S_t_minus_1 = self.current_stock_price
        self.v_t_minus_1 = self.current_volatility
        self.portfolio_value_t_minus_1 = (self.shares_held_fixed * self.current_stock_price) + 0 + \
            self.initial_cash
        self._needs_reset = False
        self._terminated = False
        return o, {}

    def step(self, action: np.ndarray):
        if self._needs_reset:
            raise RuntimeError("call reset() before step()")
        if self._terminated:
            # the reference indexes past the end of its path (hedging_env_v2.py:223)
            raise IndexError(f"index {self.episode_length + 1} is out of bounds for axis 0 with size "
                             f"{self.episode_length + 1}")
        a = np.asarray(action, dtype=np.float32).reshape(2)
        v = self._venv
        prev_S, prev_v = self.current_stock_price, self.current_volatility
        io = v.step_host(a).io
        o = io[:52].view(np.float32).copy()
        terminated = bool(io[56])
        # numpy scalars of the reference's dtypes: f64 P&L fields, int64 positions, f32 market
        pnl, ps, rab, tc, com, slip, rpc, tcp, thp, rew, pv, cash = io.view(np.float64)[self._g8]
        cc, pc, rqc, rqp, dc, dp, t = io.view(np.int32)[self._g4i].astype(np.int64)
        sfc, sfp, S, vv, C, P = io.view(np.float32)[self._g4f]
        self.current_stock_price, self.current_volatility = S, vv
        self.current_call_price, self.current_put_price = C, P
        self.current_step = int(t)
        self.call_contracts_held, self.put_contracts_held = cc, pc
        self.cash_balance = cash
        self._terminated = terminated
        self.S_t_minus_1, self.v_t_minus_1 = prev_S, prev_v
        self.portfolio_value_t_minus_1 = pv
        if self._variant == 2:
            info = {"step_pnl_total": pnl, "per_share_step_pnl": ps, "raw_pnl_deviation_abs": rab,
                    "transaction_costs_total": tc, "commission_cost": com, "slippage_cost": slip,
                    "reward_pnl_component": rpc, "transaction_cost_penalty": tcp, "theta_penalty": float(thp),
                    "reward_step": rew, "portfolio_value": pv}
        else:
            info = {"step_pnl_total": pnl, "per_share_step_pnl": ps, "raw_pnl_deviation_abs": rab,
                    "transaction_costs_total": tc, "reward_pnl_component": rpc, "transaction_cost_penalty": tcp,
                    "reward_step": rew, "portfolio_value": pv}
        info.update({
            "call_contracts": cc, "put_contracts": pc, "cash": cash,
            "raw_action_call": a[0], "raw_action_put": a[1],
            "scaled_float_call": sfc, "scaled_float_put": sfp,
            "requested_calls_rounded_clipped": rqc, "requested_puts_rounded_clipped": rqp,
            "actual_calls_traded": dc, "actual_puts_traded": dp,
            "loss_type_used": self.loss_type,
            "initial_S0_for_episode": self.initial_S0_for_episode,
        })
        return o, rew, terminated, False, info

    def render(self):
        pass

    def close(self):
        self._venv.close()


class HedgingEnvV1(HedgingEnv):
    """hedging_env.HedgingEnv (v1): no theta/slippage, $0.05 per contract."""

    _variant = 1

    def __init__(self, data_file_path=None,
                 transaction_cost_per_contract=0.05,
                 lambda_cost=1.0,
                 pnl_penalty_weight=0.01,
                 loss_type="abs",
                 initial_cash=0.0,
                 shares_to_hedge=10000,
                 max_contracts_held_per_type=200,
                 max_trade_per_step=15,
                 profile_print_interval=0,
                 record_metrics=True,
                 *, mode=None, generate=None, device=None, tables=None):
        kw = dict(transaction_cost_per_contract=transaction_cost_per_contract, lambda_cost=lambda_cost,
                  pnl_penalty_weight=pnl_penalty_weight, loss_type=loss_type, initial_cash=initial_cash,
                  shares_to_hedge=shares_to_hedge, max_contracts_held_per_type=max_contracts_held_per_type,
                  max_trade_per_step=max_trade_per_step, profile_print_interval=profile_print_interval,
                  record_metrics=record_metrics)
        self._init(data_file_path, kw, mode, generate, device, tables)
