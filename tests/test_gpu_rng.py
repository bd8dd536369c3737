"""The device's RNG words and math, bit for bit (he_device_rng / he_device_math):
device Philox4x32-10 == rocRAND's own (host-compiled) == the NumPy restatement; the
device Box-Muller pair == its host build; the device exp_k == its host build."""
import numpy as np
import pytest

from _compare import assert_same
from _rng_oracles import coordinates, rocrand_words
from oracle.hedging_oracle import philox_normals, philox_words

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("seed", [0, 42, 2 ** 32 + 7, 2 ** 64 - 1])
def test_device_philox_words_equal_rocrand(seed):
    from cantorrl_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(seed % (2 ** 32))
    gid, n = coordinates(rng, 200_000)
    g, m = _dev(gid.view(np.int64)), _dev(n.view(np.int64))
    words = torch.zeros((gid.size, 4), dtype=torch.int32, device="cuda")
    normals = torch.zeros((gid.size, 2), dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    assert lib.he_device_rng(seed, g.data_ptr(), m.data_ptr(), gid.size, words.data_ptr(), normals.data_ptr(), s) == 0
    torch.cuda.synchronize()
    dev = words.cpu().numpy().view(np.uint32)
    assert np.array_equal(dev, rocrand_words(seed, gid, n))
    npw = np.stack([np.asarray(w, np.uint32) for w in philox_words(seed, gid, n)], axis=1)
    assert np.array_equal(dev, npw)
    # Box-Muller: the device pair is the host build's, bit for bit, and the oracle's
    # libm form within a few ulp
    z = normals.cpu().numpy()
    u1 = ((((dev[:, 0].astype(np.uint64) << np.uint64(32)) | dev[:, 1].astype(np.uint64)) >> np.uint64(12))
          .astype(np.float64) + 0.5) * 2.0 ** -52
    u2 = ((((dev[:, 2].astype(np.uint64) << np.uint64(32)) | dev[:, 3].astype(np.uint64)) >> np.uint64(12))
          .astype(np.float64) + 0.5) * 2.0 ** -52
    h1, h2 = _lib.host_box_muller(u1, u2)
    assert np.array_equal(z[:, 0].view(np.int64), h1.view(np.int64))
    assert np.array_equal(z[:, 1].view(np.int64), h2.view(np.int64))
    o1, o2 = philox_normals(seed, gid, n)
    assert_same(z[:, 0], o1, "z1", rtol=1e-13, atol=1e-14)
    assert_same(z[:, 1], o2, "z2", rtol=1e-13, atol=1e-14)


def test_device_exp_equals_host_build():
    from cantorrl_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(9)
    x = np.concatenate([-0.5 * 0.029028 / 252 + np.sqrt(0.029028 / 252) * rng.standard_normal(500_000),
                        rng.uniform(-699.0, 699.0, 500_000), [0.0, -0.0, 700.5, -745.0, np.inf, -np.inf]])
    xd = _dev(x)
    out = torch.empty_like(xd)
    assert lib.he_device_math(0, xd.data_ptr(), x.size, out.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
    host = np.empty_like(x)
    assert lib.he_host_math(0, x.ctypes.data, x.size, host.ctypes.data) == 0
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.int64)[:-6], host.view(np.int64)[:-6])
    assert np.allclose(out.cpu().numpy()[-6:], host[-6:], rtol=1e-15)


@pytest.mark.parametrize("op", [1, 3, 5])
def test_device_lockstep_math_equals_scalar(op):
    """On the device, the lockstep forms the LDS producers run (op 1 exp_k_n, 3
    bs_call_put_n, 5 box_muller_n) give the scalar forms' bits (ops 0, 2, 4: the tile
    kernels' functions); exp and Box-Muller also equal the host build (he_device_math)."""
    from cantorrl_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(op)
    if op == 1:
        x = np.concatenate([rng.normal(0, 0.02, 100_001), rng.uniform(-699, 699, 1000)])
    elif op == 3:
        x = np.concatenate([496.48 * np.exp(rng.normal(0, 0.2, 100_001)), rng.uniform(0.01, 80, 1000)])
    else:
        x = rng.random(2 * 50_001)
    xd = _dev(x)
    st = torch.cuda.current_stream().cuda_stream
    lock, scal = torch.empty_like(xd), torch.empty_like(xd)
    assert lib.he_device_math(op, xd.data_ptr(), x.size, lock.data_ptr(), st) == 0
    assert lib.he_device_math(op - 1, xd.data_ptr(), x.size, scal.data_ptr(), st) == 0
    torch.cuda.synchronize()
    assert np.array_equal(lock.cpu().numpy().view(np.int64), scal.cpu().numpy().view(np.int64))
    if op != 3:  # exp_k and Box-Muller use no library transcendental: host == device
        host = np.empty_like(x)
        assert lib.he_host_math(op - 1, x.ctypes.data, x.size, host.ctypes.data) == 0
        assert np.array_equal(lock.cpu().numpy().view(np.int64), host.view(np.int64))


def test_device_rolling_atm_marks_bounded_against_host_build():
    """on the device log_ratio takes log(S / K) as the series in (S - K) * rcp(K), the
    log of the exact quotient, where the host build (and the reference's np.log(S / K)) takes the
    log of the rounded quotient S / K.  The f64 marks may therefore differ by a few f64 ulps
    (bounded here: 1e-12 relative to S, i.e. far below the f32 ulp of the mark); the f32 marks the
    env carries (hedging_env_v2.py:38 casts them) are the same bits, which is where the parity
    claim stands."""
    from cantorrl_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(31)
    x = np.concatenate([496.48 * np.exp(rng.normal(0, 0.2, 400_000)), rng.uniform(64.0, 4000.0, 100_000),
                        np.arange(64.0, 1200.0, 0.5) + 0.25])
    xd = _dev(x)
    dev = torch.empty_like(xd)
    assert lib.he_device_math(2, xd.data_ptr(), x.size, dev.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
    host = np.empty_like(x)
    assert lib.he_host_math(2, x.ctypes.data, x.size, host.ctypes.data) == 0
    torch.cuda.synchronize()
    d = dev.cpu().numpy()
    err = np.abs(d - host) / x
    assert err.max() < 1e-12, err.max()
    # after the f32 cast: equal, except where an f64 ulp or two straddles an f32 rounding
    # boundary (one f32 ulp, and rarely: a few in 10^7 draws expected)
    fd, fh = d.astype(np.float32), host.astype(np.float32)
    ulps = np.abs(fd.view(np.int32).astype(np.int64) - fh.view(np.int32).astype(np.int64))
    assert ulps.max() <= 1 and (ulps > 0).mean() < 1e-4, (ulps.max(), (ulps > 0).mean())
