#!/usr/bin/env python3
"""Record golden vectors by running the REFERENCE env in this container.

TEST INFRASTRUCTURE ONLY (never shipped, never imported by the product path).

Imports `/root/reference/src/env/hedging_env_v2.py` / `hedging_env.py`,
`quantconnect/option_calculator.py` and `src/sim/option_price_assignment.py`
unmodified, with `oracle/gym_shim` standing in for the absent third-party
`gymnasium` 1.1.1 package (seeding restated from its published algorithm).
Each scenario drives 16 independent reference envs in a DummyVecEnv-style loop
(step every env, on `terminated` keep the terminal obs and call `reset()`),
mirroring SB3 2.6.0's auto-reset (`train_ppo_v2.py:127-141`).

Outputs `tests/golden/*.npz` (inputs + expected outputs only; no reference
source).  Re-run:  python oracle/make_golden.py
G12 (generate mode closed loop, the oracle's GBM market replayed through the
reference env):  python oracle/make_golden.py --closed-loop
G13 (the same with fixed-strike European marks made by the reference's own
black_scholes_vectorized):  python oracle/make_golden.py --closed-loop-fe
"""
import os
import sys
import tempfile
import importlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = os.environ.get("CANTORRL_REFERENCE", "/root/reference")
OUT = os.path.join(REPO, "tests", "golden")

sys.path.insert(0, os.path.join(HERE, "gym_shim"))
sys.path.insert(0, REF)
sys.path.insert(1, REPO)

INFO_KEYS = [
    "step_pnl_total", "per_share_step_pnl", "raw_pnl_deviation_abs",
    "transaction_costs_total", "commission_cost", "slippage_cost",
    "reward_pnl_component", "transaction_cost_penalty", "theta_penalty",
    "reward_step", "portfolio_value", "call_contracts", "put_contracts", "cash",
    "scaled_float_call", "scaled_float_put",
    "requested_calls_rounded_clipped", "requested_puts_rounded_clipped",
    "actual_calls_traded", "actual_puts_traded", "initial_S0_for_episode",
]
INT_KEYS = {"call_contracts", "put_contracts", "requested_calls_rounded_clipped",
            "requested_puts_rounded_clipped", "actual_calls_traded", "actual_puts_traded"}


def _ref_modules():
    v2 = importlib.import_module("src.env.hedging_env_v2")
    v1 = importlib.import_module("src.env.hedging_env")
    return {1: v1.HedgingEnv, 2: v2.HedgingEnv}


def bs_rolling_atm(S, v, tenor=30 / 252, r=0.04):
    """C/P columns t=0..T-1 = BS(S_t, K=round(S_t), tenor, r, sqrt(v_t)) using the
    reference OptionCalculator (quantconnect/option_calculator.py:11-27)."""
    oc = importlib.import_module("quantconnect.option_calculator").OptionCalculator()
    P_, T1 = S.shape
    C = np.zeros((P_, T1 - 1))
    Pu = np.zeros((P_, T1 - 1))
    for p in range(P_):
        for t in range(T1 - 1):
            s = np.float64(S[p, t])
            k = np.round(s)
            sig = np.sqrt(max(v[p, t], 0.0))
            C[p, t] = oc.black_scholes_price(s, k, tenor, r, sig, "call")
            Pu[p, t] = oc.black_scholes_price(s, k, tenor, r, sig, "put")
    return C, Pu


def make_actions(rng, n_steps, n_envs, kind):
    a = rng.uniform(-1.0, 1.0, size=(n_steps, n_envs, 2)).astype(np.float32)
    if kind == "random":
        return a
    if kind == "edge":
        # half-way points k/30 (a*15 lands on .5 -> round-half-even), |a|>1,
        # +-inf, NaN, huge finite, saturating runs to hit the +-max position clip
        grid = (np.arange(-32, 33, dtype=np.float32) / np.float32(30.0)).astype(np.float32)
        specials = np.array([np.nan, np.inf, -np.inf, 1.7, -1.7, 3e38, -3e38, 1e-30,
                             -0.0, 0.0, 1.0, -1.0, 0.1, 0.0333333, 0.9999999], np.float32)
        m = rng.uniform(size=a.shape)
        a = np.where(m < 0.35, rng.choice(grid, size=a.shape), a)
        a = np.where((m >= 0.35) & (m < 0.45), rng.choice(specials, size=a.shape), a)
        # saturating runs: envs 0..3 buy calls / sell puts for long stretches
        a[:, 0, 0] = 1.0
        a[:, 1, 1] = -1.0
        a[40:120, 2, :] = 1.0
        a[40:120, 3, :] = -1.0
        return a.astype(np.float32)
    raise ValueError(kind)


def run_scenario(name, variant, data, env_kwargs, n_envs, n_steps, seed_base, actions):
    envs_cls = _ref_modules()[variant]
    S, v, C, Pm = data
    with np.errstate(all="ignore"), tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "data.npz")
        np.savez(path, paths=S, volatilities=v, call_prices_atm=C, put_prices_atm=Pm)
        envs = [envs_cls(path, **env_kwargs) for _ in range(n_envs)]
    reset_obs = np.zeros((n_envs, 13), np.float32)
    ep_idx0 = np.zeros(n_envs, np.int64)
    for i, e in enumerate(envs):
        o, _ = e.reset(seed=seed_base + i)
        reset_obs[i] = o
        ep_idx0[i] = e.current_episode_idx
    obs = np.zeros((n_steps, n_envs, 13), np.float32)
    term_obs = np.full((n_steps, n_envs, 13), np.nan, np.float32)
    rew = np.zeros((n_steps, n_envs), np.float64)
    term = np.zeros((n_steps, n_envs), bool)
    ep_idx = np.full((n_steps, n_envs), -1, np.int64)
    info = {k: np.full((n_steps, n_envs), np.nan, np.float64) for k in INFO_KEYS}
    for k in INT_KEYS:
        info[k] = np.zeros((n_steps, n_envs), np.int64)
    for s in range(n_steps):
        for i, e in enumerate(envs):
            o, r, te, tr, inf = e.step(actions[s, i])
            assert tr is False
            rew[s, i] = r
            term[s, i] = bool(te)
            for k in INFO_KEYS:
                if k in inf:
                    info[k][s, i] = inf[k]
            if te:
                term_obs[s, i] = o
                o, _ = e.reset()
                ep_idx[s, i] = e.current_episode_idx
            obs[s, i] = o
    cfg = dict(env_kwargs)
    out = dict(
        variant=np.int64(variant), n_envs=np.int64(n_envs), n_steps=np.int64(n_steps),
        seed_base=np.int64(seed_base),
        paths=S, volatilities=v, call_prices_atm=C, put_prices_atm=Pm,
        actions=actions, reset_obs=reset_obs, ep_idx0=ep_idx0,
        obs=obs, terminal_obs=term_obs, reward=rew, terminated=term, ep_idx=ep_idx,
        config_json=np.array(__import__("json").dumps(cfg)),
    )
    for k in INFO_KEYS:
        out["info_" + k] = info[k]
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
    print(f"{name}: variant={variant} envs={n_envs} steps={n_steps} "
          f"resets={int(term.sum())} nan_rewards={int(np.isnan(rew).sum())}")


def closed_loop(n_envs=16, episodes=2, seed=42, mark="rolling_atm"):
    """G12: generate mode pinned to the reference env itself.

    The GBM market of generate mode, as the oracle restates it (Philox4x32-10 normals
    keyed by (seed, env id, episode * T + t), S_{t+1} = S_t exp((mu - v/2) dt +
    sqrt(v) sqrt(dt) z), rolling-ATM BS marks; SURVEY 8(d) inputs: S0 = 496.48,
    v = 0.029028, mu = 0.04, dt = 1/252, T = 252), is written per (env, episode) in the
    NPZ layout the reference loads (paths / volatilities / call_prices_atm /
    put_prices_atm, one path per file, so its episode draw integers(1) is always 0) and
    replayed through the UNMODIFIED hedging_env_v2.HedgingEnv with the train_ppo_v2.py
    reward settings, DummyVecEnv-style (terminal obs kept, the next episode's env
    reset).  episodes + 1 episodes of market are made: the last terminal step's
    post-reset obs is the next episode's reset obs."""
    from oracle.hedging_oracle import OracleVecEnv
    T = 252
    gen = dict(s0=496.48001098632812, variance=0.029028, mu=0.04, dt=1 / 252, episode_length=T)
    if mark != "rolling_atm":
        gen["mark"] = mark
    train = dict(loss_type="abs", pnl_penalty_weight=0.001, lambda_cost=0.0001,
                 theta_weight=0.0002, slippage_bps=1.0, record_metrics=True)  # train_ppo_v2.py:74-80
    orc = OracleVecEnv(n_envs, mode="gbm", gen=dict(gen, seed=seed, env_offset=0),
                       **{k: v for k, v in train.items()})
    orc.seed_envs_at(np.arange(n_envs), [seed] * n_envs)
    E = episodes + 1
    S = np.zeros((n_envs, E, T + 1))
    for e in range(E):
        orc.g_ep[:] = e
        orc.S64[:] = gen["s0"]
        S[:, e, 0] = gen["s0"]
        for t in range(T):
            orc.t[:] = t
            orc._gbm_advance(np.ones(n_envs, bool))
            S[:, e, t + 1] = orc.S64
    if mark == "fixed_european":
        # the reference's own black_scholes_vectorized (option_price_assignment.py:10-21) over
        # columns t = 0..T-1 as process_price_paths does (:33-49): K = np.round(S0),
        # T = np.clip(1 - t / 252, 0, None).  DELIBERATE DEVIATION: sigma is the market's own
        # volatility (the GBM's sqrt(v)), not process_price_paths' expanding-window realized
        # volatility (calculate_annualized_vol_matrix, :23-31: 0 at t = 0, clamped to 1e-8).
        # G13 therefore pins the black_scholes_vectorized formula and the env mechanics of
        # HE_MARK_FIXED_EUROPEAN, not the reference generator's realized-vol marks; those are
        # the analytics path's (he_fixed_european_marks, pinned by g11 to the reference).
        bsv = importlib.import_module("src.sim.option_price_assignment").black_scholes_vectorized
        Sf = S.reshape(n_envs * E, T + 1)
        K = np.round(Sf[:, 0])
        Tg = np.clip(1 - np.arange(T + 1) / 252, 0, None)
        sig = np.full(n_envs * E, np.sqrt(gen["variance"]))
        C = np.zeros((n_envs * E, T))
        P = np.zeros((n_envs * E, T))
        for t in range(T):
            C[:, t], P[:, t] = bsv(Sf[:, t], K, Tg[t], 0.04, sig)
        C = C.reshape(n_envs, E, T)
        P = P.reshape(n_envs, E, T)
    else:
        tt = np.broadcast_to(np.arange(T), (n_envs, E, T)).reshape(-1)
        C, P = orc._gbm_marks(S[..., :T].reshape(-1), None, tt)
        C = C.reshape(n_envs, E, T)
        P = P.reshape(n_envs, E, T)
    V = np.full((n_envs, E, T + 1), gen["variance"])
    cls = _ref_modules()[2]
    rng = np.random.default_rng(20251016)
    n_steps = episodes * T
    actions = make_actions(rng, n_steps, n_envs, "random")
    actions = (actions * np.float32(1.05)).astype(np.float32)  # past +-1 too (clip)

    def env_for(i, e):
        with tempfile.TemporaryDirectory() as td:
            path = os.path.join(td, "data.npz")
            np.savez(path, paths=S[i, e][None], volatilities=V[i, e][None], call_prices_atm=C[i, e][None],
                     put_prices_atm=P[i, e][None])
            env = cls(path, **train)
        o, _ = env.reset(seed=seed + i)
        return env, o

    with np.errstate(all="ignore"):
        envs, reset_obs, ep = [], np.zeros((n_envs, 13), np.float32), np.zeros(n_envs, np.int64)
        for i in range(n_envs):
            env, o = env_for(i, 0)
            envs.append(env)
            reset_obs[i] = o
        obs = np.zeros((n_steps, n_envs, 13), np.float32)
        term_obs = np.full((n_steps, n_envs, 13), np.nan, np.float32)
        rew = np.zeros((n_steps, n_envs), np.float64)
        term = np.zeros((n_steps, n_envs), bool)
        info = {k: np.full((n_steps, n_envs), np.nan, np.float64) for k in INFO_KEYS}
        for k in INT_KEYS:
            info[k] = np.zeros((n_steps, n_envs), np.int64)
        for s in range(n_steps):
            for i in range(n_envs):
                o, r, te, tr, inf = envs[i].step(actions[s, i])
                assert tr is False
                rew[s, i] = r
                term[s, i] = bool(te)
                for k in INFO_KEYS:
                    if k in inf:
                        info[k][s, i] = inf[k]
                if te:
                    term_obs[s, i] = o
                    ep[i] += 1
                    envs[i], o = env_for(i, ep[i])
                obs[s, i] = o
    out = dict(
        variant=np.int64(2), n_envs=np.int64(n_envs), n_steps=np.int64(n_steps), seed=np.int64(seed),
        gen_json=np.array(__import__("json").dumps(gen)), config_json=np.array(__import__("json").dumps(train)),
        market_S=S, market_C=C, market_P=P,
        actions=actions, reset_obs=reset_obs, obs=obs, terminal_obs=term_obs, reward=rew, terminated=term)
    for k in INFO_KEYS:
        out["info_" + k] = info[k]
    name = "g12_closed_loop" if mark == "rolling_atm" else "g13_closed_loop_fixed_european"
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
    print(f"{name}: envs={n_envs} steps={n_steps} resets={int(term.sum())}")


def main():
    if "--closed-loop" in sys.argv:
        closed_loop()
        return
    if "--closed-loop-fe" in sys.argv:
        closed_loop(mark="fixed_european")
        return
    os.makedirs(OUT, exist_ok=True)
    rng = np.random.default_rng(20250629)
    paths = np.load(os.path.join(REF, "data", "paths.npy"))
    opts = np.load(os.path.join(REF, "data", "paths_options.npz"))

    # D1: shipped GBM-like paths, stochastic variance, rolling-ATM BS marks
    P1 = 24
    S1 = paths[:P1].copy()
    v1 = 0.029028 * np.exp(0.25 * np.cumsum(rng.normal(0, 0.1, size=S1.shape), axis=1))
    C1, Pu1 = bs_rolling_atm(S1, v1)
    D1 = (S1, v1, C1, Pu1)

    # D2: shipped paths + shipped fixed-strike European marks (paths_options.npz),
    # column 1 is NaN there (ddof=1 on one return) -> NaN propagation
    P2 = 12
    D2 = (paths[:P2].copy(), np.full((P2, 253), 0.029028), opts["calls"][:P2, :252].copy(),
          opts["puts"][:P2, :252].copy())

    # D3: edge data, short episodes (T=20): S0<25, S0==0 (<1e-6), tiny S, v<=0,
    # integer S (S==K), S at x.5 (round-half-even), huge moves for the lag clip.
    T3 = 20
    P3 = 10
    S3 = np.abs(300 + np.cumsum(rng.normal(0, 4, size=(P3, T3 + 1)), axis=1))
    S3[0] = 10 + np.cumsum(rng.normal(0, 0.3, T3 + 1))          # S0 < 25
    S3[1, 0] = 0.0                                            # S0 < 1e-6 -> 1.0
    S3[2, 5:9] = [1e-7, 0.0, 2.5e-7, 0.4]                     # S <= 1e-6, K==0
    S3[3, :] = np.round(S3[3, :])                             # S == K
    S3[4, :] = np.floor(S3[4, :]) + 0.5                       # round half even
    S3[5, 3] = S3[5, 2] * 3.5                                 # lag return clip
    S3[5, 4] = 0.0                                            # S_prev == 0 next
    S3[6, 0] = 24.999
    v3 = np.abs(0.03 + rng.normal(0, 0.01, size=(P3, T3 + 1)))
    v3[7, 2:6] = [0.0, -0.01, 1e-12, 2.5]                     # v<=0 floor, lag v clip
    v3[8, :] = 1e-9
    C3, Pu3 = bs_rolling_atm(S3, np.maximum(v3, 0.0))
    D3 = (S3, v3, C3, Pu3)

    train = dict(loss_type="abs", pnl_penalty_weight=0.001, lambda_cost=0.0001,
                 theta_weight=0.0002, slippage_bps=1.0, record_metrics=True)  # train_ppo_v2.py:74-80
    a_rand = make_actions(rng, 300, 16, "random")
    a_edge = make_actions(rng, 300, 16, "edge")
    run_scenario("g1_v2_train", 2, D1, train, 16, 300, 12345, a_rand)
    run_scenario("g1_v2_defaults_edgeact", 2, D1, {}, 16, 300, 7, a_edge)
    run_scenario("g1_v1_defaults", 1, D1, {}, 16, 300, 1000, a_rand)
    run_scenario("g1_v1_edgeact", 1, D1, dict(transaction_cost_per_contract=0.35), 16, 300, 3, a_edge)
    run_scenario("g4_v2_mse", 2, D1, dict(train, loss_type="mse"), 16, 280, 11, a_rand[:280])
    run_scenario("g4_v2_cvar", 2, D1, dict(train, loss_type="cvar"), 8, 270, 12, a_edge[:270, :8])
    run_scenario("g4_v2_other", 2, D1, dict(train, loss_type="huber"), 8, 260, 13, a_rand[:260, :8])
    run_scenario("g3_v2_nometrics", 2, D1, dict(train, record_metrics=False), 8, 260, 14, a_edge[:260, :8])
    run_scenario("g8_v2_costs", 2, D1, dict(transaction_cost_per_contract=1.25, lambda_cost=0.5,
                                             pnl_penalty_weight=0.3, theta_weight=0.01, slippage_bps=7.5,
                                             initial_cash=12345.5, shares_to_hedge=7000,
                                             max_contracts_held_per_type=37, max_trade_per_step=9),
                 16, 300, 99, a_edge)
    run_scenario("g8_v2_zeroheld", 2, D1, dict(max_contracts_held_per_type=0, initial_cash=-250.25),
                 8, 260, 5, a_rand[:260, :8])
    run_scenario("g2_v2_fixedeuro_nan", 2, D2, train, 8, 260, 21, a_rand[:260, :8])
    run_scenario("g5_v2_edgedata", 2, D3, train, 16, 120, 31, a_edge[:120])
    run_scenario("g5_v2_edgedata_mse", 2, D3, dict(train, loss_type="mse", initial_cash=100.0),
                 16, 120, 41, a_rand[:120])
    run_scenario("g5_v1_edgedata", 1, D3, {}, 16, 120, 51, a_edge[:120])

    # G7: episode-index streams, Generator(PCG64(SeedSequence(seed))).integers(P)
    sd = importlib.import_module("gymnasium.utils.seeding")
    Ps = np.array([100000, 24, 1, 2, 3, 1000003, 2**31 + 11, 4294967295, 4294967296 + 7], np.int64)
    draws = np.zeros((len(Ps), 16, 64), np.int64)
    for a, P in enumerate(Ps):
        for s in range(16):
            g, _ = sd.np_random(s)
            draws[a, s] = [g.integers(int(P)) for _ in range(64)]
    np.savez_compressed(os.path.join(OUT, "g7_episode_index.npz"), P=Ps, seeds=np.arange(16), draws=draws)

    # BS formulas: OptionCalculator (scalar) and black_scholes_vectorized
    oc = importlib.import_module("quantconnect.option_calculator").OptionCalculator()
    opa = importlib.import_module("src.sim.option_price_assignment")
    n = 400
    S = np.concatenate([rng.uniform(1, 900, n - 8), [0.0, 1e-7, 100, 100, 100, 500, 250, 50]])
    K = np.round(S + rng.normal(0, 3, n))
    K[-8:] = [0, 0, 100, 0.0, 100, 500, 250, 60]
    T = rng.choice([30 / 252, 1.0, 1 / 252, 0.0, -0.1, 1e-7], n)
    T[-8:] = [30 / 252, 30 / 252, 0.0, 30 / 252, 30 / 252, 30 / 252, 1e-9, 30 / 252]
    sig = rng.uniform(0.01, 1.0, n)
    sig[-8:] = [0.2, 0.2, 0.2, 0.2, 0.0, 1e-9, 0.3, -0.1]
    r = 0.04
    with np.errstate(all="ignore"):
        call = np.array([oc.black_scholes_price(S[i], K[i], T[i], r, sig[i], "call") for i in range(n)])
        put = np.array([oc.black_scholes_price(S[i], K[i], T[i], r, sig[i], "put") for i in range(n)])
        gc = [oc.calculate_greeks(S[i], K[i], T[i], r, sig[i], "call") for i in range(n)]
        gp = [oc.calculate_greeks(S[i], K[i], T[i], r, sig[i], "put") for i in range(n)]
        vc, vp = opa.black_scholes_vectorized(S, np.where(K > 0, K, 1.0), T, r, sig)
    np.savez_compressed(
        os.path.join(OUT, "g9_black_scholes.npz"), S=S, K=K, T=T, sigma=sig, r=np.float64(r),
        call=call, put=put,
        call_delta=np.array([g["delta"] for g in gc]), put_delta=np.array([g["delta"] for g in gp]),
        gamma=np.array([g["gamma"] for g in gc]), vega=np.array([g["vega"] for g in gc]),
        vec_call=vc, vec_put=vp, vec_K=np.where(K > 0, K, 1.0))
    print("done")


if __name__ == "__main__":
    main()
