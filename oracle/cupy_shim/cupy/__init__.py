"""Stand-in for the absent `cupy` package, for golden-vector generation only.

TEST INFRASTRUCTURE ONLY.  `src/sim/rbergomi_sim.py` imports cupy at module level
(:4) and calls a small NumPy-compatible subset of it.  This shim maps that subset
onto NumPy so the reference functions run unmodified on the host; cupy's random
module is replaced by one NumPy PCG64 Generator whose draws the tests replay in the
same order (`oracle/rbergomi_oracle.py: ReferenceDraws`).
"""
import numpy as _np
from numpy import *  # noqa: F401,F403

fft = _np.fft
float64 = _np.float64
complex128 = _np.complex128


def asarray(a, dtype=None):
    return _np.asarray(a, dtype=dtype)


def asnumpy(a):
    return _np.asarray(a)


class _Random:
    def __init__(self):
        self.gen = _np.random.Generator(_np.random.PCG64(0))
        self.log = []   # calls, in order (for the replay check)

    def seed(self, s=None):
        self.gen = _np.random.Generator(_np.random.PCG64(s))
        self.log.append(("seed", s))

    def normal(self, loc=0.0, scale=1.0, size=None, dtype=_np.float64):
        self.log.append(("normal", loc, scale, size))
        return self.gen.normal(loc, scale, size)


random = _Random()


class _Stream:
    @staticmethod
    def synchronize():
        pass


class _Cuda:
    class Stream:
        null = _Stream()


cuda = _Cuda()
