"""Minimal stand-in for the third-party `gymnasium` 1.1.1 package (absent here).

TEST INFRASTRUCTURE ONLY: used by `oracle/make_golden.py` so the reference env
(`/root/reference/src/env/hedging_env{,_v2}.py`) can be imported unmodified in
this container to record golden vectors.  It restates only what the reference
touches: `gym.Env` (reset seeding + the `np_random` property), `spaces.Box`
and `utils.seeding.np_random`.  Seeding follows gymnasium 1.1.1's published
algorithm: Generator(PCG64(SeedSequence(seed))) (gymnasium/utils/seeding.py).
"""
import numpy as np

from . import spaces  # noqa: F401
from .utils import seeding  # noqa: F401
from . import utils  # noqa: F401


class Env:
    metadata = {"render_modes": []}
    _np_random = None
    _np_random_seed = None

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            self._np_random, self._np_random_seed = seeding.np_random(seed)

    @property
    def np_random(self):
        if self._np_random is None:
            self._np_random, self._np_random_seed = seeding.np_random()
        return self._np_random

    @np_random.setter
    def np_random(self, value):
        self._np_random = value
        self._np_random_seed = -1
