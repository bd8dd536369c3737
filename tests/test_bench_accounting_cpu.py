"""bench.py's algorithmic-byte accounting, host logic only.

The roofline `achieved` figure is bytes per launch / measured launch time, so the byte
model has to follow the tile layout the library actually picks (hedge_env.hip
kGreeksInStepMinEnvs, Params::tile_greeks) and whether the market rides in the step
grid (step_market_kernel; not with a book).
"""
import importlib.util
import os

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_threshold_matches_library(bench):
    src = open(os.path.join(REPO, "cantorrl_amd", "csrc", "hedge_env.hip")).read()
    assert f"#define HE_GREEKS_IN_STEP_MIN_ENVS {bench.GREEKS_IN_STEP_MIN_ENVS}" in src


def test_tile_layout(bench, monkeypatch):
    monkeypatch.delenv("HE_GREEKS_IN_STEP_MIN_ENVS", raising=False)
    assert bench.tile_layout("gbm", 65536) == "gbm"
    assert bench.tile_layout("gbm", 262144) == "gbm_step"
    assert bench.tile_layout("heston", 1 << 20) == "heston"
    monkeypatch.setenv("HE_GREEKS_IN_STEP_MIN_ENVS", "0")
    assert bench.tile_layout("gbm", 1) == "gbm_step"


def test_per_step_bytes_add_up(bench):
    # rollout step: action 8 + post tile + obs 52 + reward 4 + terminated 1
    for lay, tile in (("gbm", 24), ("gbm_step", 12), ("heston", 32)):
        assert bench.ROLLOUT_BYTES_PER_ENV[lay] == 8 + tile + 52 + 4 + 1
        assert bench.MARKET_BYTES_PER_ENV[lay] == tile
    # he_step: state 16 + action 8 + tile slots read; state 16 + obs 52 + reward 4 + flags 2 written
    assert bench.STEP_BYTES_PER_ENV["gbm"] == 16 + 8 + 36 + 74
    assert bench.STEP_BYTES_PER_ENV["gbm_step"] == 16 + 8 + 24 + 74
    assert bench.STEP_BYTES_PER_ENV["heston"] == 16 + 8 + 48 + 74


def test_fused_launch_counts_the_market(bench, monkeypatch):
    n, rk = 65536, 64
    monkeypatch.setenv("HE_FUSED_MARKET", "1")
    r = bench.roofline("rollout", n, 0.1, rk, False, "gbm")
    step = n * (rk * 89 + 44)
    market = n * (rk * 24 + bench.MARKET_STATE_BYTES)
    assert r["bytes_per_launch"] == step + market == 481558528  # profiles/r01s21_bench.jsonl
    assert r["kernel"].startswith("step_market_kernel")
    # a book keeps the market on the side stream: the step kernel's bytes alone
    rb = bench.roofline("rollout", n, 0.1, rk, True, "gbm")
    assert rb["bytes_per_launch"] == n * (rk * (89 + 8) + 44)
    assert rb["kernel"].startswith("step_kernel")
    monkeypatch.setenv("HE_FUSED_MARKET", "0")
    r0 = bench.roofline("rollout", n, 0.1, rk, False, "gbm")
    assert r0["bytes_per_launch"] == step == 376176640  # profiles/r01s11_bench_all_configs.jsonl
    assert abs(r0["frac"] - r0["achieved"] / bench.HBM_PEAK_GBS) < 1e-4
