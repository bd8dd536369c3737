"""The single-env drop-in (cantorrl_amd.env.HedgingEnv / HedgingEnvV1) replays
env 0 of every golden scenario exactly like the reference env object did:
same ctor keywords, reset(seed)/step contract, reward, info dict and attributes."""
import os
import tempfile

import numpy as np
import pytest

from conftest import GOLDEN, golden_files
from _compare import assert_same
from oracle.hedging_oracle import load_golden

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

GREEK_COLS = slice(7, 11)


def cmp_obs(got, exp, name):
    exact = [0, 1, 2, 3, 4, 5, 6, 11, 12]
    assert_same(got[exact], exp[exact], name)
    assert_same(got[GREEK_COLS], exp[GREEK_COLS], name + " greeks", rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("fname", golden_files())
def test_single_env_replays_golden_env0(fname):
    from cantorrl_amd.env import HedgingEnv, HedgingEnvV1
    cfg, d = load_golden(os.path.join(GOLDEN, fname))
    cls = HedgingEnv if int(d["variant"]) == 2 else HedgingEnvV1
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "paths.npz")
        np.savez(path, paths=d["paths"], volatilities=d["volatilities"],
                 call_prices_atm=d["call_prices_atm"], put_prices_atm=d["put_prices_atm"])
        env = cls(path, **cfg)
    mse = cfg.get("loss_type") == "mse"
    obs, info0 = env.reset(seed=int(d["seed_base"]))
    assert info0 == {} and obs.dtype == np.float32 and obs.shape == (13,)
    cmp_obs(obs, d["reset_obs"][0], "reset_obs")
    assert env.current_episode_idx == int(d["ep_idx0"][0])
    keys_v2 = 24 if int(d["variant"]) == 2 else 21
    for s in range(int(d["n_steps"])):
        obs, r, term, trunc, info = env.step(d["actions"][s, 0])
        assert trunc is False
        assert term == bool(d["terminated"][s, 0])
        assert len(info) == keys_v2
        assert_same(np.float64(r), d["reward"][s, 0], f"reward[{s}]", rtol=1e-12 if mse else 0.0)
        for k in ("per_share_step_pnl", "transaction_costs_total", "portfolio_value", "cash"):
            assert_same(np.float64(info[k]), d["info_" + k][s, 0], f"{k}[{s}]")
        for k in ("call_contracts", "put_contracts", "actual_calls_traded", "actual_puts_traded"):
            assert int(info[k]) == int(d["info_" + k][s, 0]), (k, s)
        assert env.call_contracts_held == d["info_call_contracts"][s, 0]
        if term:
            cmp_obs(obs, d["terminal_obs"][s, 0], f"terminal_obs[{s}]")
            with pytest.raises(IndexError):
                env.step(np.zeros(2, np.float32))
            obs, _ = env.reset()
            assert env.current_episode_idx == int(d["ep_idx"][s, 0])
        cmp_obs(obs, d["obs"][s, 0], f"obs[{s}]")
    env.close()


def test_single_env_generate_mode_and_attributes():
    from cantorrl_amd.env import HedgingEnv
    env = HedgingEnv(mode="gbm", generate=dict(episode_length=5), slippage_bps=2.0)
    obs, _ = env.reset(seed=3)
    assert env.current_step == 0 and env.max_trade_per_step == 15
    assert np.isclose(env.current_stock_price, 496.48, atol=1e-3)
    done = False
    n = 0
    while not done:
        obs, r, done, _, info = env.step(np.array([0.5, -0.5], np.float32))
        n += 1
    assert n == 5 and env.current_step == 5
    assert info["call_contracts"] == 5 * 8  # rint(0.5*15)=8 per step
    env.close()
