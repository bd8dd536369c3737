"""gymnasium 1.1.1 `utils.seeding.np_random`: Generator(PCG64(SeedSequence(seed)))."""
import numpy as np


def np_random(seed=None):
    if seed is not None and not (isinstance(seed, (int, np.integer)) and seed >= 0):
        raise ValueError(f"Seed must be a non-negative python integer, got {seed!r}")
    seed_seq = np.random.SeedSequence(seed)
    rng = np.random.Generator(np.random.PCG64(seed_seq))
    return rng, seed_seq.entropy
