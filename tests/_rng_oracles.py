"""Test helpers: the rocRAND Philox oracle (oracle/_build/librocrand_words.so, built by
oracle/build.py from rocRAND's own header) and triples of 64-bit RNG coordinates."""
import ctypes
import os

import numpy as np

from oracle import build as obuild


def rocrand_words(seed, gid, n):
    """rocrand_init(seed, gid[k], 4 n[k]) + rocrand4 for every k: uint32 [count, 4]."""
    path = obuild.ROCRAND_LIB
    if not os.path.exists(path):
        obuild.build()
    lib = ctypes.CDLL(path)
    f = lib.rocrand_philox_words
    f.restype = None
    f.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    gid = np.ascontiguousarray(gid, np.uint64)
    n = np.ascontiguousarray(n, np.uint64)
    out = np.zeros((gid.size, 4), np.uint32)
    f(ctypes.c_uint64(int(seed)), gid.ctypes.data, n.ctypes.data, gid.size, out.ctypes.data)
    return out


N_MAX = 2 ** 62  # the env-step index n = ep T + t < 2^32 2^30; rocRAND's offset 4 n wraps from 2^62


def coordinates(rng, count):
    """(env id, env-step index) pairs: ids over the whole 64-bit range, indices over
    [0, 2^62) (every index an env can reach), edges included."""
    edges = np.array([0, 1, 2 ** 32 - 1, 2 ** 32, 2 ** 63, 2 ** 64 - 1], np.uint64)
    nedge = np.array([0, 1, 2 ** 32 - 1, 2 ** 32, 2 ** 61, N_MAX - 1], np.uint64)
    gid = rng.integers(0, 2 ** 64 - 1, count, dtype=np.uint64, endpoint=True)
    n = rng.integers(0, N_MAX - 1, count, dtype=np.uint64, endpoint=True)
    gid[: edges.size] = edges
    n[: edges.size] = nedge[::-1]
    gid[edges.size: 2 * edges.size] = rng.integers(0, 1 << 22, edges.size, dtype=np.uint64)  # bench-sized ids
    n[edges.size: 2 * edges.size] = rng.integers(0, 1 << 20, edges.size, dtype=np.uint64)
    return gid, n
