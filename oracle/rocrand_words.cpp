// oracle/rocrand_words.cpp -- test infrastructure (an RNG oracle independent of this
// repo's Philox code): rocRAND's own Philox4x32-10, host-compiled from
// /opt/rocm/include/rocrand/rocrand_philox4x32_10.h (ROCm 7.2), for the bit-exactness
// tests of the device and host Philox words (tests/test_lib_cpu.py, tests/test_gpu_rng.py).
//
// words[4k..4k+3] = rocrand4 after rocrand_init(seed, subsequence = gid[k],
// offset = 4 n[k]): the layout libhedgeenv keys its generate-mode normals with
// (include/hedge_env.h he_host_philox; SURVEY.md 8(c) names this oracle).
#include <rocrand/rocrand_philox4x32_10.h>

#include <stdint.h>

extern "C" void rocrand_philox_words(uint64_t seed, const uint64_t* gid, const uint64_t* n, int64_t count,
                                     uint32_t* words) {
    for (int64_t k = 0; k < count; ++k) {
        rocrand_state_philox4x32_10 st;
        rocrand_init(seed, gid[k], 4ull * n[k], &st);
        const uint4 w = rocrand4(&st);
        words[4 * k] = w.x;
        words[4 * k + 1] = w.y;
        words[4 * k + 2] = w.z;
        words[4 * k + 3] = w.w;
    }
}
