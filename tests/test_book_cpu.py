"""Liability book (extension, BASELINE.json configs[3]/[4]): the oracle's pricer.

The reference has no book, so these pin the restatement independently: the
European entries equal the golden-pinned OptionCalculator form (bs_price), and the
up-and-out call's closed form (Hull, q = 0) matches a Brownian-bridge Monte Carlo
of the continuously monitored barrier.
"""
import numpy as np
import pytest

from _compare import assert_same
from oracle.hedging_oracle import OracleVecEnv, book_option_value, book_value, bs_price


def test_european_entries_are_the_option_calculator_form():
    rng = np.random.default_rng(0)
    S = rng.uniform(300, 700, 5000)
    sig = rng.uniform(0.05, 0.6, 5000)
    tau = rng.integers(-3, 300, 5000) / 252.0
    for typ, col in (("call", 0), ("put", 1)):
        got = book_option_value(dict(type=typ, strike=500.0), S, sig, tau, 0.04, S)
        exp = bs_price(S, 500.0, tau, 0.04, sig, square=np.square)[col]
        assert_same(got, exp, typ)


def _uo_mc(S0, K, H, r, sig, T, n=4_000_000, seed=1):
    """E[e^{-rT} (S_T - K)^+ 1{max S < H}] under GBM: terminal draw + the exact
    Brownian-bridge probability of not touching H in between."""
    rng = np.random.default_rng(seed)
    z = rng.standard_normal(n)
    ST = S0 * np.exp((r - 0.5 * sig * sig) * T + sig * np.sqrt(T) * z)
    alive = ST < H
    p_hit = np.exp(-2.0 * np.log(H / S0) * np.log(H / np.where(alive, ST, H)) / (sig * sig * T))
    pay = np.where(alive, np.maximum(ST - K, 0.0) * (1.0 - p_hit), 0.0) * np.exp(-r * T)
    return pay.mean(), pay.std() / np.sqrt(n)


@pytest.mark.parametrize("S0,K,H,sig,T", [(100.0, 100.0, 120.0, 0.2, 0.5), (496.48, 480.0, 560.0, 0.17, 1.0),
                                          (100.0, 90.0, 105.0, 0.3, 0.25)])
def test_up_and_out_closed_form_matches_brownian_bridge_mc(S0, K, H, sig, T):
    got = float(book_option_value(dict(type="uo_call", strike=K, barrier=H), S0, sig, T, 0.04, S0))
    mc, se = _uo_mc(S0, K, H, 0.04, sig, T)
    assert abs(got - mc) < 4 * se + 1e-4 * S0, (got, mc, se)


def test_up_and_out_limits():
    S = np.linspace(400, 560, 50)
    c = bs_price(S, 500.0, 0.5, 0.04, 0.2, square=np.square)[0]
    uo = book_option_value(dict(type="uo_call", strike=500.0, barrier=600.0), S, 0.2, 0.5, 0.04, S)
    assert np.all(uo <= c + 1e-9) and np.all(uo >= 0)
    far = book_option_value(dict(type="uo_call", strike=500.0, barrier=1e7), S, 0.2, 0.5, 0.04, S)
    np.testing.assert_allclose(far, c, rtol=1e-9, atol=1e-9)
    assert np.all(book_option_value(dict(type="uo_call", strike=500.0, barrier=480.0), S, 0.2, 0.5, 0.04, S) == 0)
    knocked = book_option_value(dict(type="uo_call", strike=500.0, barrier=600.0), S, 0.2, 0.5, 0.04, S * 0 + 600)
    assert np.all(knocked == 0)
    # at expiry: the call payoff while alive
    exp = book_option_value(dict(type="uo_call", strike=500.0, barrier=600.0), S, 0.2, 0.0, 0.04, S)
    assert_same(exp, np.maximum(S - 500.0, 0.0), "expiry payoff")


def test_oracle_portfolio_value_carries_the_book():
    book = [dict(type="call", strike=500.0, expiry=20, quantity=-30.0),
            dict(type="put", strike=480.0, expiry=8, quantity=-10.0),
            dict(type="uo_call", strike=490.0, barrier=510.0, expiry=30, quantity=-20.0)]
    gen = dict(s0=496.48001098632812, variance=0.029028, mu=0.04, dt=1 / 252, episode_length=12, seed=3)
    a = OracleVecEnv(64, mode="gbm", gen=dict(gen, book=book))
    b = OracleVecEnv(64, mode="gbm", gen=gen)
    for e in (a, b):
        e.seed_envs_at(np.arange(64), [3] * 64)
        e.reset()
    acts = np.random.default_rng(2).uniform(-1, 1, size=(30, 64, 2)).astype(np.float32)
    for s in range(30):
        *_, ia = a.step(acts[s])
        *_, ib = b.step(acts[s])
        B = book_value(book, a.S64, 0.029028, a.t, a.runmax, 0.04, 1 / 252)
        # envs that just reset report the pre-reset step; compare the book-free part
        np.testing.assert_allclose(ia["portfolio_value"] - ib["portfolio_value"],
                                   np.where(a.t == 0, ia["portfolio_value"] - ib["portfolio_value"], B),
                                   rtol=1e-12, atol=1e-6)
