"""CPU restatement of the reference's offline path analytics.

TEST INFRASTRUCTURE ONLY: the checker for cantorrl_amd.analytics (HIP kernels in
cantorrl_amd/csrc/analytics.hip).  Restates, with the reference's NumPy / math / scipy
calls in the same order:
  /root/reference/src/sim/option_price_assignment.py:10-52  (fixed-strike European marks)
  /root/reference/src/tools/bs_delta.py:11-55               (daily BS delta hedge P&L)
Pinned by the shipped data/paths_options.npz (the reference's own output for
data/paths.npy) and by tests/golden/g11_analytics.npz, recorded from the reference by
oracle/make_golden_analytics.py.
"""
import math

import numpy as np
from scipy.stats import norm

RISK_FREE_RATE = 0.04
DT = 1 / 252


def black_scholes_vectorized(S, K, T, r, sigma, epsilon=1e-8):       # option_price_assignment.py:10-21
    T_safe = np.where(T <= 0, 1e-8, T)
    sigma_safe = np.where(sigma < epsilon, epsilon, sigma)
    d1 = (np.log(S / K) + (r + 0.5 * sigma_safe ** 2) * T_safe) / (sigma_safe * np.sqrt(T_safe))
    d2 = d1 - sigma_safe * np.sqrt(T_safe)
    call = S * norm.cdf(d1) - K * np.exp(-r * T_safe) * norm.cdf(d2)
    put = K * np.exp(-r * T_safe) * norm.cdf(-d2) - S * norm.cdf(-d1)
    intrinsic_call = np.maximum(S - K * np.exp(-r * T), 0)
    intrinsic_put = np.maximum(K * np.exp(-r * T) - S, 0)
    return np.where(T <= 0, intrinsic_call, call), np.where(T <= 0, intrinsic_put, put)


def calculate_annualized_vol_matrix(paths):                            # :23-31
    n_sims, n_steps1 = paths.shape
    vols = np.zeros((n_sims, n_steps1))
    with np.errstate(invalid="ignore", divide="ignore"):
        for t in range(1, n_steps1):
            sl = paths[:, :t + 1]
            lr = np.log(sl[:, 1:] / sl[:, :-1])
            vols[:, t] = np.std(lr, axis=1, ddof=1) * math.sqrt(252)
    return vols


def fixed_european_marks(paths, r=RISK_FREE_RATE):                     # process_price_paths :33-52
    n_sims, n_steps1 = paths.shape
    strikes = np.round(paths[:, 0])
    T = np.clip(1 - np.arange(n_steps1) / 252, 0, None)
    vols = calculate_annualized_vol_matrix(paths)
    calls = np.zeros((n_sims, n_steps1))
    puts = np.zeros((n_sims, n_steps1))
    with np.errstate(invalid="ignore"):
        for t in range(n_steps1):
            calls[:, t], puts[:, t] = black_scholes_vectorized(paths[:, t], strikes, T[t], r, vols[:, t])
    return vols, calls, puts


def _bs_price(S, K, T, r, sigma, epsilon=1e-8):                        # bs_delta.py:11-18
    if sigma < epsilon or T <= 0:
        return max(S - K * math.exp(-r * T), 0)
    d1 = (math.log(S / K) + (r + 0.5 * sigma ** 2) * T) / (sigma * math.sqrt(T))
    d2 = d1 - sigma * math.sqrt(T)
    return S * norm.cdf(d1) - K * math.exp(-r * T) * norm.cdf(d2)


def _bs_delta(S, K, T, r, sigma, epsilon=1e-8):                        # :20-24
    if sigma < epsilon or T <= 0:
        return 1.0 if S > K else 0.0
    d1 = (math.log(S / K) + (r + 0.5 * sigma ** 2) * T) / (sigma * math.sqrt(T))
    return norm.cdf(d1)


def _ann_vol(prices):                                                  # :26-34
    if len(prices) < 2:
        return 0.0
    lr = np.log(prices[1:] / prices[:-1])
    sd = 0.0 if len(lr) < 2 else np.std(lr, ddof=1)
    return sd * math.sqrt(252)


def bs_delta_hedge(paths, r=RISK_FREE_RATE, dt=DT):                    # :36-55
    n_sims, n_steps1 = paths.shape
    T_total = n_steps1 * dt
    pnls = np.zeros((n_sims, n_steps1))
    for i in range(n_sims):
        prices = paths[i]
        K = prices[0]
        cash, prev = 0.0, 0.0
        for t in range(n_steps1):
            S = prices[t]
            T_remain = max(T_total - t * dt, 0.0)
            sigma = _ann_vol(prices[:t + 1])
            delta = _bs_delta(S, K, T_remain, r, sigma)
            cash -= (delta - prev) * S
            prev = delta
            pnls[i, t] = cash + prev * S - _bs_price(S, K, T_remain, r, sigma)
    return pnls
