"""Shared comparison helpers for parity tests (NaN-aware)."""
import numpy as np


def assert_same(got, exp, name, rtol=0.0, atol=0.0):
    got = np.asarray(got)
    exp = np.asarray(exp)
    assert got.shape == exp.shape, f"{name}: shape {got.shape} != {exp.shape}"
    if exp.dtype.kind in "biu":
        bad = got != exp
    else:
        g = got.astype(np.float64)
        e = exp.astype(np.float64)
        both_nan = np.isnan(g) & np.isnan(e)
        with np.errstate(invalid="ignore"):
            close = (g == e) | (np.abs(g - e) <= atol + rtol * np.abs(e))
        bad = ~(both_nan | close)
    if bad.any():
        idx = np.argwhere(bad)[:5]
        detail = ", ".join(f"{tuple(i)}: got {got[tuple(i)]!r} exp {exp[tuple(i)]!r}" for i in idx)
        raise AssertionError(f"{name}: {int(bad.sum())}/{bad.size} mismatches; {detail}")
