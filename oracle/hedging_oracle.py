"""CPU oracle: a vectorized NumPy restatement of the reference hedging env.

TEST INFRASTRUCTURE ONLY.  Only `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s `cpu_baseline` leg may import this module, and only as the
checker / the CPU baseline -- never as the product path.

It restates, over a batch of N independent envs, the exact per-element dtype
sequence of the reference (NumPy 2 / NEP 50 promotion, python scalars weak):

* `HedgingEnv.reset`       -- src/env/hedging_env_v2.py:145-173 (v1 :141-169)
* `HedgingEnv.step`        -- src/env/hedging_env_v2.py:175-294 (v1 :171-270)
* `_get_observation`       -- src/env/hedging_env_v2.py:109-143
* `_calculate_greeks`      -- src/env/hedging_env_v2.py:79-107
* `OptionCalculator.black_scholes_price`
                           -- quantconnect/option_calculator.py:11-27
* GBM price advance        -- src/sim/rbergomi_sim.py:454-464 (constant v)
* liability book (extension, BASELINE.json configs[3]/[4]; include/hedge_env.h
  he_book_option) -- Europeans in the option_calculator.py:11-27 form, the
  up-and-out call in Hull's closed form; parity unpinned by the reference (it has
  no book), checked against a Brownian-bridge Monte Carlo in tests/test_book_cpu.py

Replay mode consumes NPZ-layout tables (`paths`, `volatilities`,
`call_prices_atm`, `put_prices_atm`, hedging_env_v2.py:36-48) and draws the
episode index of every reset from `Generator(PCG64(SeedSequence(seed)))
.integers(P)` exactly as gymnasium seeding does (hedging_env_v2.py:146-150).

Generate mode (the north-star extension) produces the same market data the
reference would replay from an NPZ written by a GBM generator: S in f64
(advanced with Philox4x32-10 normals, counter layout in `philox_normals`),
variance constant, C/P = f64 Black-Scholes at K=round(S_t) (rolling ATM,
rbergomi_sim.py:418,437-446; gen["mark"] = "fixed_european": the fixed-strike
European of option_price_assignment.py:10-21,33-49, K = round(S0), T = 1 - t/252) --
then runs the identical env logic on the f32 casts (hedging_env_v2.py:38-41).

Pinned by: tests/golden/*.npz, recorded from the reference itself by
oracle/make_golden.py (see tests/test_oracle_golden.py).
"""
import json

import numpy as np
from scipy.special import ndtr

from oracle.analytics_oracle import black_scholes_vectorized

LOSS_CODES = {"mse": 0, "abs": 1, "cvar": 2}  # anything else -> 3 ("other", |x| branch)

V2_DEFAULTS = dict(transaction_cost_per_contract=0.65, lambda_cost=1.0, pnl_penalty_weight=0.01,
                   theta_weight=0.0, slippage_bps=0.0, loss_type="abs", initial_cash=0.0,
                   shares_to_hedge=10000, max_contracts_held_per_type=200, max_trade_per_step=15,
                   profile_print_interval=0, record_metrics=True)
V1_DEFAULTS = dict(V2_DEFAULTS, transaction_cost_per_contract=0.05)
del V1_DEFAULTS["theta_weight"], V1_DEFAULTS["slippage_bps"]

_NORM_PDF_C = np.sqrt(2 * np.pi)  # scipy.stats._continuous_distns._norm_pdf_C


def spow2(x):
    """Elementwise `x**2` with NumPy *scalar* semantics (libm pow/powf per element).

    The reference squares numpy scalars (`per_share_step_pnl**2`, `s0_floor**2`,
    `sigma**2`, hedging_env_v2.py:96,247), which calls libm pow()/powf(); array
    `**2` uses an exact x*x fast path and differs in ~0.1% of inputs by 1 ulp.
    """
    x = np.asarray(x)
    if x.ndim == 0:
        return x.dtype.type(x) ** 2
    t = x.dtype.type
    return np.array([t(v) ** 2 for v in x.ravel()], dtype=x.dtype).reshape(x.shape)

# --------------------------------------------------------------------------- #
# Philox4x32-10 (Salmon et al. 2011; rocRAND rocrand_philox4x32_10.h layout)    #
# --------------------------------------------------------------------------- #
_PH_M0, _PH_M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_PH_W0, _PH_W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
_M32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorized Philox4x32-10 block function; all args uint32 arrays/scalars."""
    c0, c1, c2, c3 = (np.asarray(x, np.uint32) for x in (c0, c1, c2, c3))
    k0 = np.asarray(k0, np.uint32).copy()
    k1 = np.asarray(k1, np.uint32).copy()
    with np.errstate(over="ignore"):
        for rnd in range(10):
            if rnd:
                k0 = (k0 + _PH_W0).astype(np.uint32)
                k1 = (k1 + _PH_W1).astype(np.uint32)
            p0 = _PH_M0 * c0.astype(np.uint64)
            p1 = _PH_M1 * c2.astype(np.uint64)
            hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & _M32).astype(np.uint32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & _M32).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
    return c0, c1, c2, c3


def philox_words(seed, env_ids, step_index):
    """4 uint32 words for (seed, global env id, env-step index n).

    Counter = (lo32(n), hi32(n), lo32(g), hi32(g)), key = (lo32(seed), hi32(seed));
    identical to rocRAND `rocrand_init(seed, subsequence=g, offset=4*n)` + `rocrand4` for
    n < 2^62 (every index an env reaches; rocRAND's offset 4n wraps beyond), checked word for
    word against rocRAND's own code (oracle/rocrand_words.cpp, tests/test_lib_cpu.py).
    """
    g = np.asarray(env_ids, np.uint64)
    n = np.asarray(step_index, np.uint64)
    n, g = np.broadcast_arrays(n, g)
    s = np.uint64(seed)
    return philox4x32_10((n & _M32).astype(np.uint32), (n >> np.uint64(32)).astype(np.uint32),
                         (g & _M32).astype(np.uint32), (g >> np.uint64(32)).astype(np.uint32),
                         np.uint32(s & _M32), np.uint32(s >> np.uint64(32)))


def u01_from_words(hi, lo):
    """(0,1) double from two uint32 words: ((hi:lo >> 12) + 0.5) * 2^-52 (exact)."""
    k = ((np.asarray(hi, np.uint64) << np.uint64(32)) | np.asarray(lo, np.uint64)) >> np.uint64(12)
    return (k.astype(np.float64) + 0.5) * (2.0 ** -52)


def philox_normals(seed, env_ids, step_index):
    """Two standard normals per (env, step) by Box-Muller in f64."""
    x0, x1, x2, x3 = philox_words(seed, env_ids, step_index)
    u1 = u01_from_words(x0, x1)
    u2 = u01_from_words(x2, x3)
    rad = np.sqrt(-2.0 * np.log(u1))
    ang = (2.0 * np.pi) * u2
    return rad * np.cos(ang), rad * np.sin(ang)


# --------------------------------------------------------------------------- #
# Black-Scholes (quantconnect/option_calculator.py:11-27), vectorized f64       #
# --------------------------------------------------------------------------- #
def bs_price(S, K, T, r, sigma, square=None):
    """`square` = how sigma**2 is formed: python-scalar pow (default, the reference's
    scalar call) or x*x (`square=np.square`, the per-env sigma of Heston marks)."""
    S, K, T, sigma = np.broadcast_arrays(*(np.asarray(x, np.float64) for x in (S, K, T, sigma)))
    with np.errstate(all="ignore"):
        sqT = np.sqrt(T)
        sig2 = spow2(sigma) if square is None else sigma * sigma
        d1 = (np.log(S / K) + (r + 0.5 * sig2) * T) / (sigma * sqT)
        d2 = d1 - sigma * sqT
        disc = np.exp(-r * T)
        call = S * ndtr(d1) - K * disc * ndtr(d2)
        put = K * disc * ndtr(-d2) - S * ndtr(-d1)
        # max(price, 0) with python semantics: max(nan, 0) -> nan, (0 > nan is False)
        call = np.where(call < 0, 0.0, call)
        put = np.where(put < 0, 0.0, put)
        intrinsic = (T <= 0) | (sigma <= 0)
        ic = np.where(S - K < 0, 0.0, S - K)
        ip = np.where(K - S < 0, 0.0, K - S)
        # python max(x, 0) returns x unless 0 > x (so nan/-0.0 stay)
        ic = np.where(np.isnan(S - K), S - K, ic)
        ip = np.where(np.isnan(K - S), K - S, ip)
    return np.where(intrinsic, ic, call), np.where(intrinsic, ip, put)


def bs_greeks(S, K, T, r, sigma):
    """OptionCalculator.calculate_greeks (option_calculator.py:29-59), vectorized."""
    S, K, T, sigma = np.broadcast_arrays(*(np.asarray(x, np.float64) for x in (S, K, T, sigma)))
    with np.errstate(all="ignore"):
        edge = (T <= 1e-6) | (sigma <= 1e-8) | (S <= 1e-6)
        Kc = np.maximum(K, 1e-6)
        d1 = (np.log(S / Kc) + (r + 0.5 * spow2(sigma)) * T) / (sigma * np.sqrt(T))
        pdf = np.exp(-d1 ** 2 / 2.0) / _NORM_PDF_C
        cd = np.where(edge, np.where(S > K, 1.0, 0.0), ndtr(d1))
        pd = np.where(edge, np.where(S < K, -1.0, 0.0), ndtr(d1) - 1.0)
        gamma = np.where(edge, 0.0, pdf / (S * sigma * np.sqrt(T)))
        vega = np.where(edge, 0.0, S * pdf * np.sqrt(T))
    return cd, pd, gamma, vega


# --------------------------------------------------------------------------- #
# Liability book (extension): restates cantorrl_amd/csrc/hedge_env.hip        #
# book_option / book_value                                                    #
# --------------------------------------------------------------------------- #
BOOK_TYPES = {"call": 0, "put": 1, "uo_call": 2}


def book_option_value(o, S, sig, tau, r, runmax):
    """One book option at (S, sig, tau) [f64 arrays]; runmax = episode max of S at the
    step dates (up-and-out monitor).  Intrinsic when tau <= 0 or sig <= 0."""
    typ = BOOK_TYPES[o["type"]] if isinstance(o["type"], str) else int(o["type"])
    K = float(o["strike"])
    H = float(o.get("barrier", 0.0))
    S, sig, tau, runmax = np.broadcast_arrays(*(np.asarray(x, np.float64) for x in (S, sig, tau, runmax)))
    with np.errstate(all="ignore"):
        intrinsic = (tau <= 0) | (sig <= 0)
        ic = np.where(S - K < 0, 0.0, S - K)
        ip = np.where(K - S < 0, 0.0, K - S)
        s2 = sig * sig
        sst = sig * np.sqrt(tau)
        d1 = (np.log(S / K) + (r + 0.5 * s2) * tau) / sst
        d2 = d1 - sst
        Kd = K * np.exp(-r * tau)
        if typ == 1:
            v = Kd * ndtr(-d2) - S * ndtr(-d1)
            v = np.where(v < 0, 0.0, v)
            return np.where(intrinsic, ip, v)
        v = S * ndtr(d1) - Kd * ndtr(d2)
        if typ == 2:
            lam = (r + 0.5 * s2) / s2
            ls = lam * sst
            lhs = np.log(H / S)
            x1 = np.log(S / H) / sst + ls
            y = np.log((H * H) / (S * K)) / sst + ls
            y1 = lhs / sst + ls
            p2l = np.exp((2.0 * lam) * lhs)
            p2l2 = np.exp((2.0 * lam - 2.0) * lhs)
            cui = (S * ndtr(x1) - Kd * ndtr(x1 - sst) - S * p2l * (ndtr(-y) - ndtr(-y1))
                   + Kd * p2l2 * (ndtr(-y + sst) - ndtr(-y1 + sst)))
            v = v - cui
        v = np.where(v < 0, 0.0, v)
        if typ == 2:
            v = np.where(H <= K, 0.0, v)
        v = np.where(intrinsic, ic, v)
        if typ == 2:
            v = np.where(runmax >= H, 0.0, v)
    return v


def book_value(book, S, var, t, runmax, r, dt):
    """sum_k q_k * 100 * V_k after step t of the episode (in book order, from 0.0)."""
    S = np.asarray(S, np.float64)
    sig = np.sqrt(np.maximum(np.asarray(var, np.float64), 0.0))
    B = np.zeros(S.shape)
    for o in book:
        tau = (int(o["expiry"]) - np.asarray(t, np.int64)) * dt
        B = B + (float(o["quantity"]) * 100.0) * book_option_value(o, S, sig, tau, r, runmax)
    return B


# --------------------------------------------------------------------------- #
# Baseline policies (restating src/agents/baselines.py:74-103 and              #
# src/benchmark/delta_and_nothing.py:122-163 over a batch, same dtypes)        #
# --------------------------------------------------------------------------- #
POLICIES = ("no_hedge", "delta_every_step", "delta_threshold")


def policy_actions(policy, obs, call, put, max_held, shares, mt):
    """Actions [N,2] f32 of `policy` on the current obs [N,13] f32 and positions."""
    obs = np.asarray(obs, np.float32)
    n = obs.shape[0]
    if policy == "no_hedge":
        return np.zeros((n, 2), np.float32)
    cd, pd = obs[:, 7], obs[:, 9]
    f100 = np.float32(100)
    with np.errstate(all="ignore"):
        if policy == "delta_every_step":
            # baselines.py:77-103: numpy f32 scalars with weak python ints / floats
            cur_call = obs[:, 3] * np.float32(max_held)
            cur_put = obs[:, 4] * np.float32(max_held)
            opt = (cur_call * cd + cur_put * pd) * f100
            target = -(np.float32(shares) + opt)
            use_c = np.abs(cd * f100) > np.float32(0.1)
            use_p = (~use_c) & (np.abs(pd * f100) > np.float32(0.1))
            tc = np.where(use_c, target / (cd * f100), np.float32(0))
            tp = np.where(use_p, target / (pd * f100), np.float32(0))
            m = np.float32(mt)
            return np.stack([np.clip(tc, -m, m), np.clip(tp, -m, m)], axis=1).astype(np.float32)
        if policy == "delta_threshold":
            # delta_and_nothing.py:122-163: np.int64 positions x f32 deltas -> f64
            cur = (np.asarray(call, np.int64) * cd.astype(np.float64)
                   + np.asarray(put, np.int64) * pd.astype(np.float64)) * 100
            need = -shares - cur
            thr = (np.float32(0.5) * np.abs(cd)) * f100
            skip = np.abs(need) < thr.astype(np.float64)
            rc = np.where((need > 0) & (np.abs(cd) > np.float32(1e-6)),
                          np.clip(need / (cd * f100).astype(np.float64), -mt, mt), 0.0)
            rp = np.where((need < 0) & (np.abs(pd) > np.float32(1e-6)),
                          np.clip(need / (pd * f100).astype(np.float64), -mt, mt), 0.0)
            rc = np.where(skip, 0.0, rc)
            rp = np.where(skip, 0.0, rp)
            return np.stack([rc, rp], axis=1).astype(np.float32)
    raise ValueError(policy)


# --------------------------------------------------------------------------- #
# The env batch                                                               #
# --------------------------------------------------------------------------- #
class OracleVecEnv:
    """N reference envs advanced in lock-step, DummyVecEnv-style auto-reset.

    mode="replay": data=(paths, volatilities, call_prices_atm, put_prices_atm).
    mode="gbm":    gen=dict(s0, variance, mu, dt, seed, episode_length, env_offset).
    """

    def __init__(self, n_envs, variant=2, mode="replay", data=None, gen=None, **kwargs):
        self.n = int(n_envs)
        self.variant = int(variant)
        self.mode = mode
        base = V2_DEFAULTS if self.variant == 2 else V1_DEFAULTS
        unknown = set(kwargs) - set(base)
        if unknown:
            raise TypeError(f"unexpected env kwargs {sorted(unknown)}")
        cfg = dict(base, **kwargs)
        self.cfg = cfg
        self.tcpc = cfg["transaction_cost_per_contract"]
        self.lam = cfg["lambda_cost"]
        self.w = cfg["pnl_penalty_weight"]
        self.theta = cfg.get("theta_weight", 0.0)
        self.slip = cfg.get("slippage_bps", 0.0)
        self.loss = cfg["loss_type"]
        self.initial_cash = cfg["initial_cash"]
        self.shares = cfg["shares_to_hedge"]
        self.max_held = cfg["max_contracts_held_per_type"]
        self.mt = cfg["max_trade_per_step"]
        self.record_metrics = cfg["record_metrics"]
        self.mult = 100
        self.r = 0.04
        self.tenor = 30 / 252
        if mode == "replay":
            S, v, C, P = data
            self.S_tab = np.asarray(S).astype(np.float32)
            self.v_tab = np.asarray(v).astype(np.float32)
            self.C_tab = np.asarray(C).astype(np.float32)
            self.P_tab = np.asarray(P).astype(np.float32)
            if not (self.S_tab.shape == self.v_tab.shape
                    and self.S_tab.shape[0] == self.C_tab.shape[0] == self.P_tab.shape[0]
                    and self.S_tab.shape[1] == self.C_tab.shape[1] + 1 == self.P_tab.shape[1] + 1):
                raise ValueError("Data shapes are inconsistent.")
            self.num_episodes = self.S_tab.shape[0]
            self.episode_length = self.S_tab.shape[1] - 1
        elif mode in ("gbm", "heston"):
            g = dict(gen)
            self.g_s0 = float(g["s0"])
            self.g_v = float(g["variance"])
            self.g_mu = float(g.get("mu", 0.04))
            self.g_dt = float(g.get("dt", 1 / 252))
            self.g_seed = int(g.get("seed", 42))
            self.g_offset = int(g.get("env_offset", 0))
            self.h_kappa = float(g.get("heston_kappa", 2.0))
            self.h_theta = float(g.get("heston_theta", 0.029028))
            self.h_xi = float(g.get("heston_xi", 0.3))
            self.h_rho = float(g.get("heston_rho", -0.7))
            self.episode_length = int(g.get("episode_length", 252))
            self.num_episodes = None
            self.g_ep = np.full(self.n, -1, np.int64)  # next reset starts episode 0
            self.S64 = np.zeros(self.n, np.float64)
            self.V64 = np.zeros(self.n, np.float64)
            self.book = list(g.get("book", None) or ())
            self.mark = g.get("mark", "rolling_atm")
            if self.mark not in ("rolling_atm", "fixed_european"):
                raise ValueError(self.mark)
            self.runmax = np.zeros(self.n, np.float64)
        else:
            raise ValueError(mode)
        self.rngs = [None] * self.n
        z = np.zeros(self.n)
        self.t = np.zeros(self.n, np.int64)
        self.idx = np.zeros(self.n, np.int64)
        self.S = z.astype(np.float32)
        self.v = z.astype(np.float32)
        self.C = z.astype(np.float32)
        self.P = z.astype(np.float32)
        self.S_prev = z.astype(np.float32)
        self.v_prev = z.astype(np.float32)
        self.S0 = z.astype(np.float32)          # initial_S0_for_episode (f32 view)
        self.S0_small = np.zeros(self.n, bool)  # S0<1e-6 -> python float 1.0
        self.call = np.zeros(self.n, np.int64)
        self.put = np.zeros(self.n, np.int64)
        self.cash = z.astype(np.float64)
        self.pv_prev = z.astype(np.float64)

    # ------------------------------------------------------------------ market
    def _gbm_marks(self, S64, V64, t):
        """C, P (f64) of the generated market at episode step t (int array)."""
        if self.mark == "fixed_european":
            # option_price_assignment.py:33-49: strike np.round(paths[:, 0]), expiry one year
            # after the episode start, T = np.clip(1 - t / 252, 0, None); the market's own
            # volatility in place of the realized one (GBM sqrt(v), Heston sqrt(max(v_t, 0)))
            K = np.round(np.full(len(S64), self.g_s0))
            T = np.clip(1 - np.asarray(t, np.int64) / 252, 0, None)
            v = V64 if self.mode == "heston" else np.full(len(S64), self.g_v)
            sig = np.sqrt(np.maximum(v, 0.0))
            return black_scholes_vectorized(S64, K, T, self.r, sig)
        K = np.round(S64)
        if self.mode == "heston":
            sig = np.sqrt(np.maximum(V64, 0.0))
            C, P = bs_price(S64, K, self.tenor, self.r, sig, square=np.square)
        else:
            sig = np.sqrt(self.g_v)
            C, P = bs_price(S64, K, self.tenor, self.r, sig)
        return C, P

    def _gbm_advance(self, mask):
        """S_{t+1} from S_t for masked envs (rbergomi_sim.py:454-464).

        GBM: constant v, one normal per step -- env-step n takes the cos (n even) or
        sin (n odd) half of the Box-Muller pair of Philox block n//2.  Heston:
        both halves of block n; full-truncation Euler on v driven by dw1, price
        driven by dW = rho*dw1 + sqrt(1-rho^2)*dw2 (rbergomi_sim.py:457)."""
        ids = np.nonzero(mask)[0]
        n_idx = (self.g_ep[ids] * self.episode_length + self.t[ids]).astype(np.uint64)
        gids = np.uint64(self.g_offset) + ids.astype(np.uint64)
        if self.mode == "heston":
            z0, z1 = philox_normals(self.g_seed, gids, n_idx)
        else:
            c, s = philox_normals(self.g_seed, gids, n_idx >> np.uint64(1))
            z0 = np.where((n_idx & np.uint64(1)) == 1, s, c)
        sqrt_dt = np.sqrt(self.g_dt)
        if self.mode == "heston":
            v = self.V64[ids]
            vp = np.maximum(v, 0.0)
            dw1 = sqrt_dt * z0
            dw2 = sqrt_dt * z1
            dW = self.h_rho * dw1 + np.sqrt(max(0.0, 1.0 - self.h_rho * self.h_rho)) * dw2
            drift = (self.g_mu - 0.5 * vp) * self.g_dt
            diff = np.sqrt(vp) * dW
            Snew = self.S64[ids] * np.exp(drift + diff)
            self.V64[ids] = (v + self.h_kappa * (self.h_theta - vp) * self.g_dt) + self.h_xi * np.sqrt(vp) * dw1
        else:
            v = self.g_v
            dW = sqrt_dt * z0
            drift = (self.g_mu - 0.5 * v) * self.g_dt
            diff = np.sqrt(np.maximum(0.0, v)) * dW
            Snew = self.S64[ids] * np.exp(drift + diff)
        self.S64[ids] = np.maximum(Snew, 1e-8)

    # ------------------------------------------------------------------ reset
    def seed_envs(self, seeds):
        """reset(seed=s_i) semantics: re-seed env i's episode generator."""
        for i, s in enumerate(seeds):
            if s is not None:
                self.rngs[i] = np.random.Generator(np.random.PCG64(np.random.SeedSequence(int(s))))

    def reset(self, env_ids=None, seeds=None, episode_idx=None):
        """episode_idx (replay): the rows of the reset envs (in env_ids order) given instead
        of drawn -- hedging_env_v2.py:150 with current_episode_idx supplied (he_reset_episodes);
        the envs' generators are not advanced."""
        ids = np.arange(self.n) if env_ids is None else np.asarray(env_ids)
        if seeds is not None:
            self.seed_envs_at(ids, seeds)
        mask = np.zeros(self.n, bool)
        mask[ids] = True
        given = None
        if episode_idx is not None:
            given = np.full(self.n, -1, np.int64)
            given[ids] = np.asarray(episode_idx, np.int64)
        self._reset_mask(mask, given)
        obs = self._obs()
        self.last_obs = obs.copy()
        self.ep_sums = np.zeros((self.n, 6))
        self.ep_len = np.zeros(self.n, np.int64)
        return obs[ids]

    def step_policy(self, policy):
        """One step with actions from a baseline policy on the current obs; returns the
        step outputs plus the actions and the records (env, length, 6 sums) of the
        episodes that ended (in env order)."""
        a = policy_actions(policy, self.last_obs, self.call, self.put, self.max_held, self.shares, self.mt)
        obs, rew, term, tobs, info = self.step(a)
        vals = (rew, info["step_pnl_total"], info["raw_pnl_deviation_abs"], info["transaction_costs_total"],
                info["reward_pnl_component"], info["transaction_cost_penalty"])
        for c, v in enumerate(vals):
            self.ep_sums[:, c] = self.ep_sums[:, c] + v
        self.ep_len += 1
        done = np.nonzero(term)[0]
        recs = [(int(i), int(self.ep_len[i]), *self.ep_sums[i]) for i in done]
        self.ep_sums[term] = 0.0
        self.ep_len[term] = 0
        return a, obs, rew, term, info, recs

    def seed_envs_at(self, ids, seeds):
        for i, s in zip(ids, seeds):
            if self.mode == "replay":
                self.rngs[i] = np.random.Generator(np.random.PCG64(np.random.SeedSequence(int(s))))
        if self.mode in ("gbm", "heston"):
            # generate mode: seed selects the Philox key for the whole batch
            self.g_seed = int(seeds[0])
            self.g_ep[:] = -1

    def _reset_mask(self, mask, given=None):
        ids = np.nonzero(mask)[0]
        if self.mode == "replay":
            for i in ids:
                if given is not None:
                    self.idx[i] = given[i]
                    continue
                if self.rngs[i] is None:
                    self.rngs[i] = np.random.Generator(np.random.PCG64(np.random.SeedSequence()))
                self.idx[i] = self.rngs[i].integers(self.num_episodes)
            row = self.idx[ids]
            S = self.S_tab[row, 0]
            v = self.v_tab[row, 0]
            C = self.C_tab[row, 0]
            P = self.P_tab[row, 0]
        else:
            self.g_ep[ids] += 1  # every reset starts the next episode of the env
            self.S64[ids] = self.g_s0
            self.V64[ids] = self.g_v
            S = self.S64[ids].astype(np.float32)
            v = np.full(len(ids), self.g_v).astype(np.float32)
            Cd, Pd = self._gbm_marks(self.S64[ids], self.V64[ids], np.zeros(len(ids), np.int64))
            C = Cd.astype(np.float32)
            P = Pd.astype(np.float32)
        self.t[ids] = 0
        self.S[ids], self.v[ids], self.C[ids], self.P[ids] = S, v, C, P
        small = S < 1e-6
        self.S0[ids] = np.where(small, np.float32(1.0), S)
        self.S0_small[ids] = small
        self.call[ids] = 0
        self.put[ids] = 0
        self.cash[ids] = self.initial_cash
        # (shares * S)[f32] + 0 + cash[weak -> f32]  (hedging_env_v2.py:167-168)
        pv0 = (np.float32(self.shares) * S + np.float32(0)) + np.float32(self.initial_cash)
        self.pv_prev[ids] = pv0.astype(np.float32).astype(np.float64)
        self.S_prev[ids] = S
        self.v_prev[ids] = v
        if self.mode != "replay" and self.book:
            self.runmax[ids] = self.g_s0
            self.pv_prev[ids] = self.pv_prev[ids] + book_value(self.book, np.full(len(ids), self.g_s0), self.g_v,
                                                               0, self.g_s0, self.r, self.g_dt)

    # ------------------------------------------------------------------ obs
    def _greeks(self):
        n = self.n
        z = np.zeros(n)
        if not self.record_metrics:
            return z, z, z, z
        S, v = self.S, self.v
        K = np.round(S)  # f32, half-even
        with np.errstate(all="ignore"):
            sigma = np.sqrt(np.maximum(v, np.float32(1e-8)))        # f32
            T = self.tenor
            Kc = np.maximum(K, np.float32(1e-6))                     # f32
            sst = sigma.astype(np.float64) * np.sqrt(T)              # f32*f64 -> f64
            num = np.log(S / Kc) + (np.float32(self.r) + np.float32(0.5) * spow2(sigma)) * np.float32(T)
            d1 = np.where(sst < 1e-9, np.sign(num).astype(np.float64) * 10.0,
                          num.astype(np.float64) / sst)
            cd = ndtr(d1)
            pd = ndtr(d1) - 1.0
            gden = S.astype(np.float64) * sst
            gam = np.where(np.abs(gden) < 1e-9, 0.0, np.exp(-d1 ** 2 / 2.0) / _NORM_PDF_C / gden)
        # branch S <= 1e-6 (hedging_env_v2.py:87-89)
        b1 = S <= 1e-6
        cd1 = np.where(K == 0, 0.5, np.where(K > 0, 0.0, 1.0))
        pd1 = np.where(K == 0, -0.5, np.where(K < 0, 0.0, -1.0))
        # branch T<=1e-6 or sigma<=1e-6 (:90-92)
        b2 = (~b1) & ((T <= 1e-6) | (sigma <= 1e-6))
        cd2 = np.where(S > K, 1.0, np.where(S == K, 0.5, 0.0))
        pd2 = np.where(S < K, -1.0, np.where(S == K, -0.5, 0.0))
        cd = np.where(b1, cd1, np.where(b2, cd2, cd))
        pd = np.where(b1, pd1, np.where(b2, pd2, pd))
        gam = np.where(b1 | b2, 0.0, gam)
        return cd, gam, pd, gam

    def _obs(self):
        n = self.n
        S0 = self.S0
        with np.errstate(all="ignore"):
            s0s = np.maximum(S0, np.float32(25.0))  # small-S0 envs: f64 25.0, same f32 quotient
            nS = self.S / s0s
            nC = self.C / s0s
            nP = self.P / s0s
            if self.max_held != 0:
                nch = self.call / self.max_held
                nph = self.put / self.max_held
            else:
                nch = np.zeros(n)
                nph = np.zeros(n)
            T = self.episode_length
            tte = (T - self.t) / T if T != 0 else np.zeros(n)
            cd, cg, pd, pg = self._greeks()
            zero_lag = (self.t == 0) | (self.S_prev == 0)
            lS = np.where(zero_lag, np.float32(0), (self.S - self.S_prev) / self.S_prev)
            lv = np.where(zero_lag, np.float32(0), self.v - self.v_prev)
            lS = np.clip(lS, np.float32(-1.0), np.float32(1.0)).astype(np.float32)
            lv = np.clip(lv, np.float32(-1.0), np.float32(1.0)).astype(np.float32)
        cols = [nS, nC, nP, nch, nph, self.v, tte, cd, cg, pd, pg, lS, lv]
        return np.stack([np.asarray(c).astype(np.float32) for c in cols], axis=1)

    # ------------------------------------------------------------------ step
    def step(self, actions):
        """One step of every env; auto-reset terminated envs (SB3 semantics).

        Returns obs[N,13] f32 (post-reset for done envs), reward[N] f64,
        terminated[N] bool, terminal_obs[N,13] (NaN rows where not done), info.
        """
        a = np.asarray(actions, np.float32).reshape(self.n, 2)
        mt = self.mt
        with np.errstate(all="ignore"):
            fc = a[:, 0] * np.float32(mt)
            fp = a[:, 1] * np.float32(mt)
            rqc = np.clip(np.rint(fc).astype(np.int64), -mt, mt)
            rqp = np.clip(np.rint(fp).astype(np.int64), -mt, mt)
        pc, pp = self.call, self.put
        self.call = np.clip(pc + rqc, -self.max_held, self.max_held).astype(np.int64)
        self.put = np.clip(pp + rqp, -self.max_held, self.max_held).astype(np.int64)
        dc = self.call - pc
        dp = self.put - pp
        with np.errstate(all="ignore"):
            commission = (np.abs(dc) + np.abs(dp)) * self.tcpc
            if self.variant == 2:
                slip_c = np.abs(dc) * self.C * self.mult * (self.slip / 10000.0)
                slip_p = np.abs(dp) * self.P * self.mult * (self.slip / 10000.0)
                slippage = slip_c + slip_p
                tc = commission + slippage
            else:
                slippage = np.full(self.n, np.nan)
                tc = commission.astype(np.float64)
            self.cash = self.cash - tc
        self.S_prev = self.S.copy()
        self.v_prev = self.v.copy()
        self.t = self.t + 1
        T = self.episode_length
        term = self.t >= T
        if self.mode == "replay":
            row = self.idx
            self.S = self.S_tab[row, self.t]
            self.v = self.v_tab[row, self.t]
            tc_idx = np.where(term, self.t - 1, self.t)
            self.C = self.C_tab[row, tc_idx]
            self.P = self.P_tab[row, tc_idx]
        else:
            self.t = self.t - 1
            self._gbm_advance(np.ones(self.n, bool))
            self.t = self.t + 1
            self.S = self.S64.astype(np.float32)
            if self.mode == "heston":
                self.v = self.V64.astype(np.float32)
            Cd, Pd = self._gbm_marks(self.S64, self.V64, self.t)
            self.C = np.where(term, self.C, Cd.astype(np.float32))
            self.P = np.where(term, self.P, Pd.astype(np.float32))
            if self.book:
                self.runmax = np.maximum(self.runmax, self.S64)
                var = self.V64 if self.mode == "heston" else self.g_v
                book = book_value(self.book, self.S64, var, self.t, self.runmax, self.r, self.g_dt)
        with np.errstate(all="ignore"):
            opt = (self.call * self.C * self.mult) + (self.put * self.P * self.mult)
            pv = (np.float32(self.shares) * self.S) + opt + self.cash
            if self.mode != "replay" and self.book:
                pv = pv + book
            pnl = pv - self.pv_prev
            ps = pnl / self.shares if self.shares != 0 else pnl
            raw = np.abs(ps)
            s0f32 = np.maximum(self.S0, np.float32(25.0))
            if self.loss == "mse":
                den = np.where(self.S0_small, 25.0 ** 2 + 1e-9,
                               (spow2(s0f32) + np.float32(1e-9)).astype(np.float64))
                term_v = spow2(ps) / den
            else:
                den = np.where(self.S0_small, 25.0 + 1e-9,
                               (s0f32 + np.float32(1e-9)).astype(np.float64))
                term_v = np.abs(ps) / den
            rpc = -self.w * term_v
            tcp = self.lam * tc
            tte_y = (T - self.t) / 252.0
            if self.variant == 2:
                thp = self.theta * tte_y
                reward = rpc - tcp - thp
            else:
                thp = np.full(self.n, np.nan)
                reward = rpc - tcp
        self.pv_prev = pv.copy()
        info = dict(step_pnl_total=pnl, per_share_step_pnl=ps, raw_pnl_deviation_abs=raw,
                    transaction_costs_total=tc, commission_cost=commission if self.variant == 2 else
                    np.full(self.n, np.nan), slippage_cost=slippage,
                    reward_pnl_component=rpc, transaction_cost_penalty=tcp, theta_penalty=thp,
                    reward_step=reward, portfolio_value=pv, call_contracts=self.call.copy(),
                    put_contracts=self.put.copy(), cash=self.cash.copy(),
                    scaled_float_call=fc, scaled_float_put=fp,
                    requested_calls_rounded_clipped=rqc, requested_puts_rounded_clipped=rqp,
                    actual_calls_traded=dc, actual_puts_traded=dp,
                    initial_S0_for_episode=np.where(self.S0_small, 1.0, self.S0.astype(np.float64)),
                    # the market after the step, before any autoreset (he_info current_*)
                    current_stock_price=self.S.copy(), current_call_price=self.C.copy(),
                    current_put_price=self.P.copy())
        obs = self._obs()
        terminal_obs = np.full_like(obs, np.nan)
        if term.any():
            terminal_obs[term] = obs[term]
            self._reset_mask(term)
            obs[term] = self._obs()[term]
        self.last_obs = obs.copy()
        return obs, reward, term, terminal_obs, info


def load_golden(path):
    """Load one golden scenario npz into (OracleVecEnv kwargs, arrays)."""
    z = np.load(path, allow_pickle=False)
    d = {k: z[k] for k in z.files}
    cfg = json.loads(str(d["config_json"]))
    return cfg, d
