"""Baseline policies (baselines.py:74-103, delta_and_nothing.py:122-163): the oracle's
batched restatement replays the reference's own policy runs (tests/golden/g10_*,
recorded by oracle/make_golden_policies.py) bit for bit."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from _compare import assert_same
from oracle.hedging_oracle import OracleVecEnv

G10 = sorted(f for f in os.listdir(GOLDEN) if f.startswith("g10_policy_"))


def load(fname):
    z = np.load(os.path.join(GOLDEN, fname), allow_pickle=False)
    return {k: z[k] for k in z.files}


@pytest.mark.parametrize("fname", G10)
def test_oracle_policy_rollout_matches_reference(fname):
    d = load(fname)
    cfg = json.loads(str(d["config_json"]))
    n = int(d["n_envs"])
    env = OracleVecEnv(n, variant=1, mode="replay",
                       data=(d["paths"], d["volatilities"], d["call_prices_atm"], d["put_prices_atm"]), **cfg)
    obs0 = env.reset(seeds=[int(d["seed_base"]) + i for i in range(n)])
    assert_same(obs0, d["reset_obs"], "reset_obs")
    pol = str(d["policy"])
    for s in range(int(d["n_steps"])):
        a, obs, rew, term, info, _ = env.step_policy(pol)
        assert_same(a, d["actions"][s], f"actions[{s}]")
        assert_same(term, d["terminated"][s], f"terminated[{s}]")
        assert_same(rew, d["reward"][s], f"reward[{s}]")
        for k in ("step_pnl_total", "raw_pnl_deviation_abs", "transaction_costs_total", "call_contracts"):
            assert_same(np.asarray(info[k]).astype(np.float64), d["info_" + k][s], f"{k}[{s}]")
        assert_same(obs, d["obs"][s], f"obs[{s}]")
