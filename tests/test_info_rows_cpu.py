"""The C info rows (cantorrl_amd/csrc/info_rows.c) behind HedgingVecEnv's `infos`: each row
must behave as the dict SB3's DummyVecEnv returns (train_ppo_v2.py:127-141) -- the env's info
keys (hedging_env_v2.py:268-293), "TimeLimit.truncated", and on a done row
"terminal_observation" / Monitor's "episode" (train_ppo_v2.py:119) -- for every way SB3 and the
reference's loops read or write it."""
import collections.abc
import copy
import gc
import json
import weakref

import numpy as np
import pytest

from cantorrl_amd.lib import _info_rows as R
import cantorrl_amd.vec_env  # noqa: F401  (registers Row as a MutableMapping)

N = 50
KEYS = ("per_share_step_pnl", "call_contracts", "scaled_float_call")


def _cols():
    rng = np.random.default_rng(0)
    return (rng.normal(size=N), np.arange(N, dtype=np.int32) - 7, rng.normal(size=N).astype(np.float32))


class _View(R.Rows):
    def __init__(self, done=None, monitor=True):
        self.loads = 0
        self.ends_calls = []
        self.cols = _cols()
        self.done = done
        self.monitor = monitor

    def _load(self):
        self.loads += 1
        calls, monitor = self.ends_calls, self.monitor   # no reference back to the view

        def ends(i):
            calls.append(i)
            d = {"terminal_observation": np.full(13, float(i), np.float32)}
            if monitor:
                d["episode"] = {"r": -0.5 * i, "l": 252, "t": 1.0}
            return d
        dk = ("terminal_observation", "episode") if self.monitor else ("terminal_observation",)
        self._attach(KEYS, self.cols, b"dif", N, "TimeLimit.truncated", False, self.done, dk, ends)


def _expected(v, i):
    c = v.cols
    return {KEYS[0]: float(c[0][i]), KEYS[1]: int(c[1][i]), KEYS[2]: float(c[2][i]), "TimeLimit.truncated": False}


def test_rows_read_like_dicts():
    v = _View()
    assert v.loads == 0 and not v._attached
    assert len(v) == N
    r = v[3]
    assert v.loads == 1 and v._attached
    exp = _expected(v, 3)
    assert r[KEYS[0]] == exp[KEYS[0]] and type(r[KEYS[1]]) is int and r[KEYS[1]] == -4
    assert r.get(KEYS[2]) == exp[KEYS[2]] and r.get("nope") is None and r.get("nope", 7) == 7
    assert r.get("episode") is None and r.get("terminal_observation") is None and r.get("is_success") is None
    assert KEYS[0] in r and "TimeLimit.truncated" in r and "episode" not in r
    assert r["TimeLimit.truncated"] is False
    with pytest.raises(KeyError):
        r["episode"]
    assert dict(r) == exp and r == exp and r.copy() == exp and list(r) == list(exp)
    assert list(r.keys()) == list(exp) and list(r.items()) == list(exp.items()) and len(r) == 4
    assert json.loads(json.dumps(dict(r))) == exp
    assert isinstance(r, collections.abc.Mapping) and isinstance(r, collections.abc.MutableMapping)
    assert {**r} == exp and copy.deepcopy(dict(r)) == exp
    assert repr(r) == repr(exp)


def test_rows_list_semantics():
    v = _View()
    assert v[-1] is v[N - 1] and v[0] is v[0]
    assert [x[KEYS[1]] for x in v[2:8:3]] == [-5, -2]
    assert len(list(v)) == N and [x[KEYS[1]] for x in v][:3] == [-7, -6, -5]
    assert [i for i, _ in enumerate(v)][-1] == N - 1
    with pytest.raises(IndexError):
        v[N]
    with pytest.raises(TypeError):
        v["a"]
    assert v.loads == 1   # one host attach for the view's whole life


def test_done_rows_extras_are_made_once_when_read():
    done = np.zeros(N, np.bool_)
    done[[4, 9]] = True
    v = _View(done)
    # SB3's per-step pass: every row's get("episode") / get("is_success")
    eps = [(i, info.get("episode")) for i, info in enumerate(v) if info.get("episode") is not None]
    assert [i for i, _ in eps] == [4, 9] and eps[1][1]["r"] == -4.5
    assert v.ends_calls == [4, 9]
    assert v[9].get("is_success") is None and "terminal_observation" in v[4]
    # SB3 VecNormalize normalizes the terminal obs in place: the write stays
    v[4]["terminal_observation"] = np.zeros(13)
    assert (v[4]["terminal_observation"] == 0).all()
    assert list(v[9]) == list(KEYS) + ["TimeLimit.truncated", "terminal_observation", "episode"]
    assert v.ends_calls == [4, 9]
    assert "episode" not in _View(done, monitor=False)[4]


def test_row_mutation_and_outliving_the_view():
    v = _View()
    r = v[5]
    r["x"] = 1
    r.update(y=2)
    assert v[5]["x"] == 1 and v[5]["y"] == 2 and r.pop("y") == 2 and "y" not in r
    assert r.setdefault("z", 3) == 3
    del r[KEYS[0]]
    assert KEYS[0] not in v[5]
    keep = v[7]
    w = weakref.ref(v)
    del v, r
    gc.collect()
    assert w() is None
    assert keep[KEYS[1]] == 0   # the row keeps its columns alive


def test_attach_validates():
    class Bad(R.Rows):
        def _load(self):
            pass
    with pytest.raises(RuntimeError, match="_attach"):
        Bad()[0]
    v = _View()
    with pytest.raises(ValueError):
        v._attach(KEYS, _cols()[:2], b"di", N, None, None, None, (), None)
    with pytest.raises(ValueError):
        v._attach(("a",), (np.zeros(3),), b"d", N, None, None, None, (), None)   # column too short
    with pytest.raises(ValueError):
        v._attach(("a",), (np.zeros(N),), b"q", N, None, None, None, (), None)
