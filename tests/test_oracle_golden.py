"""Pin the CPU oracle against golden vectors recorded from the reference env.

Goldens: tests/golden/*.npz, produced by oracle/make_golden.py running
/root/reference/src/env/hedging_env{,_v2}.py unmodified (gymnasium shimmed).
Bar: bit-exact on every integer / f64 P&L / reward field and on the f32 obs.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden_files
from _compare import assert_same
from oracle.hedging_oracle import OracleVecEnv, load_golden, bs_price, bs_greeks

INFO_FIELDS = [
    "step_pnl_total", "per_share_step_pnl", "raw_pnl_deviation_abs", "transaction_costs_total",
    "commission_cost", "slippage_cost", "reward_pnl_component", "transaction_cost_penalty",
    "theta_penalty", "reward_step", "portfolio_value", "call_contracts", "put_contracts", "cash",
    "scaled_float_call", "scaled_float_put", "requested_calls_rounded_clipped",
    "requested_puts_rounded_clipped", "actual_calls_traded", "actual_puts_traded",
    "initial_S0_for_episode",
]


def run_oracle_on_golden(d, cfg):
    n = int(d["n_envs"])
    env = OracleVecEnv(n, variant=int(d["variant"]), mode="replay",
                       data=(d["paths"], d["volatilities"], d["call_prices_atm"], d["put_prices_atm"]),
                       **cfg)
    obs0 = env.reset(seeds=[int(d["seed_base"]) + i for i in range(n)])
    out = dict(reset_obs=obs0, ep_idx0=env.idx.copy())
    steps = int(d["n_steps"])
    obs = np.zeros((steps, n, 13), np.float32)
    tob = np.zeros((steps, n, 13), np.float32)
    rew = np.zeros((steps, n))
    term = np.zeros((steps, n), bool)
    ep = np.full((steps, n), -1, np.int64)
    info = {k: [] for k in INFO_FIELDS}
    for s in range(steps):
        o, r, te, to, inf = env.step(d["actions"][s])
        obs[s], rew[s], term[s], tob[s] = o, r, te, to
        ep[s] = np.where(te, env.idx, -1)
        for k in INFO_FIELDS:
            info[k].append(inf[k])
    out.update(obs=obs, terminal_obs=tob, reward=rew, terminated=term, ep_idx=ep)
    for k in INFO_FIELDS:
        out["info_" + k] = np.stack(info[k])
    return out


@pytest.mark.parametrize("fname", golden_files())
def test_oracle_matches_reference_golden(fname):
    cfg, d = load_golden(os.path.join(GOLDEN, fname))
    got = run_oracle_on_golden(d, cfg)
    assert_same(got["ep_idx0"], d["ep_idx0"], "ep_idx0")
    assert_same(got["reset_obs"], d["reset_obs"], "reset_obs")
    assert_same(got["terminated"], d["terminated"], "terminated")
    assert_same(got["ep_idx"], d["ep_idx"], "ep_idx")
    assert_same(got["reward"], d["reward"], "reward")
    for k in INFO_FIELDS:
        exp = d["info_" + k]
        g = got["info_" + k]
        assert_same(g.astype(exp.dtype), exp, "info_" + k)
    assert_same(got["obs"], d["obs"], "obs")
    assert_same(got["terminal_obs"], d["terminal_obs"], "terminal_obs")


def test_episode_index_streams_match_gymnasium_seeding():
    z = np.load(os.path.join(GOLDEN, "g7_episode_index.npz"))
    for a, P in enumerate(z["P"]):
        for s in z["seeds"]:
            g = np.random.Generator(np.random.PCG64(np.random.SeedSequence(int(s))))
            got = [g.integers(int(P)) for _ in range(z["draws"].shape[2])]
            assert_same(np.array(got), z["draws"][a, s], f"P={P} seed={s}")


def test_bs_price_matches_option_calculator():
    z = np.load(os.path.join(GOLDEN, "g9_black_scholes.npz"))
    c, p = bs_price(z["S"], z["K"], z["T"], float(z["r"]), z["sigma"])
    assert_same(c, z["call"], "call", rtol=1e-13, atol=1e-12)
    assert_same(p, z["put"], "put", rtol=1e-13, atol=1e-12)
    cd, pd, g, v = bs_greeks(z["S"], z["K"], z["T"], float(z["r"]), z["sigma"])
    assert_same(cd, z["call_delta"], "call_delta", rtol=1e-13)
    assert_same(pd, z["put_delta"], "put_delta", rtol=1e-13)
    assert_same(g, z["gamma"], "gamma", rtol=1e-12)
    assert_same(v, z["vega"], "vega", rtol=1e-12)


CLOSED_LOOPS = {"rolling_atm": "g12_closed_loop.npz", "fixed_european": "g13_closed_loop_fixed_european.npz"}


def load_closed_loop(mark="rolling_atm"):
    import json
    z = np.load(os.path.join(GOLDEN, CLOSED_LOOPS[mark]), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    return json.loads(str(d["gen_json"])), json.loads(str(d["config_json"])), d


@pytest.mark.parametrize("mark", sorted(CLOSED_LOOPS))
def test_oracle_generate_mode_matches_reference_closed_loop(mark):
    """G12 / G13: the oracle's generate mode (its own GBM market, made inside the env)
    equals the unmodified reference env replaying that market (oracle/make_golden.py
    --closed-loop / --closed-loop-fe): every obs, reward, done flag, terminal obs and info
    field, bit for bit, over 2 episodes x 16 envs.  G13's fixed-strike European marks were
    made by the reference's own black_scholes_vectorized (option_price_assignment.py:10-21),
    so it pins the oracle's mark function as well as the env mechanics."""
    gen, cfg, d = load_closed_loop(mark)
    assert gen.get("mark", "rolling_atm") == mark
    n, seed = int(d["n_envs"]), int(d["seed"])
    env = OracleVecEnv(n, mode="gbm", gen=dict(gen, seed=seed, env_offset=0), **cfg)
    env.seed_envs_at(np.arange(n), [seed] * n)
    assert_same(env.reset(), d["reset_obs"], "reset_obs")
    for s in range(int(d["n_steps"])):
        o, r, te, to, inf = env.step(d["actions"][s])
        assert_same(te, d["terminated"][s], f"terminated[{s}]")
        assert_same(r, d["reward"][s], f"reward[{s}]")
        assert_same(o, d["obs"][s], f"obs[{s}]")
        if te.any():
            assert_same(to[te], d["terminal_obs"][s][te], f"terminal_obs[{s}]")
        for k in INFO_FIELDS:
            assert_same(np.asarray(inf[k]).astype(d["info_" + k].dtype), d["info_" + k][s], f"info_{k}[{s}]")
