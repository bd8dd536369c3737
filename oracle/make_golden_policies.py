#!/usr/bin/env python3
"""Record golden vectors of the reference BASELINE POLICIES, run in this container.

TEST INFRASTRUCTURE ONLY (never shipped, never imported by the product path).

Imports, unmodified, `src/agents/baselines.py` (policy_no_hedge,
policy_delta_every_step, :74-103) and `src/benchmark/delta_and_nothing.py`
(delta_hedging_action_selector, :122-163) from /root/reference, with
`oracle/gym_shim` for the absent gymnasium package.  Both read
`env.max_trade_per_step`, which the reference v1 env does not define (it keeps
`_max_trade_per_step_internal`, SURVEY.md section 4: the scripts raise
AttributeError as shipped); the generator sets that one attribute on each env
instance to the constructor's max_trade_per_step, nothing else.

16 v1 envs on the g1 tables (rolling-ATM marks, stochastic variance) are driven
DummyVecEnv-style: action = policy(current obs, env), step, on `terminated`
reset.  Output: tests/golden/g10_policy_*.npz (inputs, actions, obs, rewards,
info fields; no reference source).  Re-run: python oracle/make_golden_policies.py
"""
import importlib
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (sets up the shim + reference paths)

OUT = mg.OUT
KEYS = ["step_pnl_total", "raw_pnl_deviation_abs", "transaction_costs_total", "reward_pnl_component",
        "transaction_cost_penalty", "per_share_step_pnl", "call_contracts", "put_contracts", "portfolio_value"]


def d1_tables():
    rng = np.random.default_rng(20250629)
    paths = np.load(os.path.join(mg.REF, "data", "paths.npy"))
    S1 = paths[:24].copy()
    v1 = 0.029028 * np.exp(0.25 * np.cumsum(rng.normal(0, 0.1, size=S1.shape), axis=1))
    C1, Pu1 = mg.bs_rolling_atm(S1, v1)
    return S1, v1, C1, Pu1


def run(name, policy_name, env_kwargs, n_envs, n_steps, seed_base, data):
    base = importlib.import_module("src.agents.baselines")
    dn = importlib.import_module("src.benchmark.delta_and_nothing")
    Env = importlib.import_module("src.env.hedging_env").HedgingEnv
    S, v, C, Pm = data
    with np.errstate(all="ignore"), tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "data.npz")
        np.savez(path, paths=S, volatilities=v, call_prices_atm=C, put_prices_atm=Pm)
        envs = [Env(path, **env_kwargs) for _ in range(n_envs)]
    mt = env_kwargs.get("max_trade_per_step", 15)
    for e in envs:
        e.max_trade_per_step = mt   # the attribute the reference scripts read (see module doc)

    def act(o, e):
        if policy_name == "no_hedge":
            return base.policy_no_hedge(o, e)
        if policy_name == "delta_every_step":
            return base.policy_delta_every_step(o, e)
        state_info = {
            "S_t": e.current_stock_price, "v_t": e.current_volatility, "call_delta_atm": o[7],
            "put_delta_atm": o[9], "current_call_contracts": e.call_contracts_held,
            "current_put_contracts": e.put_contracts_held, "shares_to_hedge": e.shares_held_fixed,
            "option_contract_multiplier": e.option_contract_multiplier,
            "max_trade_per_step": e.max_trade_per_step}
        return dn.delta_hedging_action_selector(state_info)

    cur = []
    for i, e in enumerate(envs):
        o, _ = e.reset(seed=seed_base + i)
        cur.append(o)
    reset_obs = np.stack(cur).astype(np.float32)
    actions = np.zeros((n_steps, n_envs, 2), np.float32)
    obs = np.zeros((n_steps, n_envs, 13), np.float32)
    rew = np.zeros((n_steps, n_envs))
    term = np.zeros((n_steps, n_envs), bool)
    info = {k: np.zeros((n_steps, n_envs)) for k in KEYS}
    with np.errstate(all="ignore"):
        for s in range(n_steps):
            for i, e in enumerate(envs):
                a = np.asarray(act(cur[i], e), dtype=np.float32)
                actions[s, i] = a
                o, r, te, tr, inf = e.step(a)
                rew[s, i] = r
                term[s, i] = bool(te)
                for k in KEYS:
                    info[k][s, i] = inf[k]
                if te:
                    o, _ = e.reset()
                cur[i] = o
                obs[s, i] = o
    out = dict(variant=np.int64(1), n_envs=np.int64(n_envs), n_steps=np.int64(n_steps),
               seed_base=np.int64(seed_base), policy=np.array(policy_name),
               paths=S, volatilities=v, call_prices_atm=C, put_prices_atm=Pm,
               reset_obs=reset_obs, actions=actions, obs=obs, reward=rew, terminated=term,
               config_json=np.array(json.dumps(env_kwargs)))
    for k in KEYS:
        out["info_" + k] = info[k]
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
    print(f"{name}: {policy_name} envs={n_envs} steps={n_steps} episodes={int(term.sum())} "
          f"|a|max={np.nanmax(np.abs(actions)):.3f}")


def main():
    data = d1_tables()
    # baselines.py main (:124-138): w = lam = 0, abs loss, greeks only for delta policies
    bkw = dict(pnl_penalty_weight=0.0, lambda_cost=0.0, loss_type="abs")
    run("g10_policy_no_hedge", "no_hedge", dict(bkw, record_metrics=False), 16, 300, 300, data)
    run("g10_policy_delta_every_step", "delta_every_step", dict(bkw, record_metrics=True), 16, 600, 400, data)
    # delta_and_nothing.py (:20-28, :44-52)
    dkw = dict(transaction_cost_per_contract=0.05, lambda_cost=1.0, shares_to_hedge=10000,
               max_contracts_held_per_type=200, max_trade_per_step=15, profile_print_interval=10_000_000)
    run("g10_policy_delta_threshold", "delta_threshold", dkw, 16, 600, 500, data)
    # non-default limits: small position cap, other share count, tighter trade size
    run("g10_policy_delta_threshold_limits", "delta_threshold",
        dict(dkw, max_contracts_held_per_type=40, shares_to_hedge=3000, max_trade_per_step=6), 16, 300, 600, data)
    run("g10_policy_delta_every_step_limits", "delta_every_step",
        dict(bkw, record_metrics=True, max_contracts_held_per_type=40, shares_to_hedge=3000, max_trade_per_step=6),
        16, 300, 700, data)


if __name__ == "__main__":
    main()
