// vecnorm.hip -- VecNormalize and Monitor statistics on the device (part of libhedgeenv;
// C ABI in include/hedge_env.h).
//
// The reference trains behind SB3 2.6.0's VecNormalize(norm_obs=True, norm_reward=True,
// gamma) (train_ppo_v2.py:204,305) and evaluates with the stats frozen (:450-453); every
// env is wrapped in Monitor(info_keywords=...) (:119).  On the host that is a NumPy
// pass over [N, 13] per step plus per-env Python lists -- the bottleneck once N is in
// the tens of thousands.  Here one step is ONE launch of vecnorm_kernel, one workgroup
// per CU at most (G <= 256 workgroups, every one resident):
//   1. per workgroup: exact two-pass f64 mean / M2 of its rows' obs columns and of the
//      updated running returns, written as a partial;
//   2. the last workgroup to arrive (atomic ticket) merges the G partials in workgroup
//      order (Chan et al.; sums as block reductions), applies
//      RunningMeanStd.update_from_moments and releases the others (a generation flag);
//   3. every workgroup normalizes its rows with the new statistics: obs / reward /
//      terminal obs, returns[done] = 0 and the Monitor episode sums.
// Deterministic for a given grid.  The waits are bounded (a spin that never sees the
// flag gives up and leaves the outputs unwritten, reported by the next he_vecnorm_step
// check) so a fault can never hang the device.  Eval mode (no statistics update) skips
// 1-2.  HBM-bound and tiny (68 B of obs + reward read and written per env): the point is
// to keep the statistics on the device within one launch, not the arithmetic.

#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include "../../include/hedge_env.h"

namespace {

constexpr int kD = HE_OBS_DIM;
constexpr int kVnThreads = 256;
constexpr int kVnMaxBlocks = 256;   // workgroups of one launch: all resident (one per CU at most)

// scratch layout: [blocks][kPart] doubles, then one u32 ticket
constexpr int kPart = 2 * kD + 3;   // count, mean[D], M2[D], ret_mean, ret_M2

struct VnArgs {
    int64_t n;
    int rows_per_block;
    int blocks;
    int training, norm_obs, norm_reward, upd_obs;
    double gamma, clip_obs, clip_rew, eps;
    const float* obs;
    const float* reward;
    const uint8_t* done;
    const float* tobs;
    double* returns;
    double* stats;
    double* part;
    unsigned int* ticket;
    float* obs_out;
    float* rew_out;
    float* tobs_out;
    double* ep_ret;
    int32_t* ep_len;
    double* ep_ret_done;
    int32_t* ep_len_done;
    int reset;   // he_vecnorm_reset: returns = 0 instead of the discounted update
};

// RunningMeanStd.update_from_moments (SB3 common/running_mean_std.py), f64
__device__ __forceinline__ void rms_update(double* mean, double* var, double* count, double bmean, double bvar,
                                           double bcount) {
    const double delta = bmean - *mean;
    const double tot = *count + bcount;
    const double new_mean = *mean + delta * bcount / tot;
    const double m_a = *var * *count;
    const double m_b = bvar * bcount;
    const double m2 = m_a + m_b + delta * delta * *count * bcount / tot;
    *mean = new_mean;
    *var = m2 / tot;
    *count = tot;
}

__device__ __forceinline__ double clipd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }

// Sum of v[0..NV) over the block into out[0..NV) (LDS): a wave-level butterfly per
// value, then one barrier and a 4-way sum -- two barriers for all NV values.
template <int NV>
__device__ __forceinline__ void block_sum(double* v, double (*sh)[NV], double* out) {
#pragma unroll
    for (int c = 0; c < NV; ++c) {
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) v[c] += __shfl_xor(v[c], m, 64);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int c = 0; c < NV; ++c) sh[w][c] = v[c];
    }
    __syncthreads();
    if (threadIdx.x < NV) {
        double t = 0.0;
#pragma unroll
        for (int i = 0; i < kVnThreads / 64; ++i) t += sh[i][threadIdx.x];
        out[threadIdx.x] = t;
    }
    __syncthreads();
}

constexpr long kVnSpinLimit = 1L << 20;  // ~1 s of polling: only a fault gets there

// Cross-workgroup data (partials, statistics, ticket, flag) moves through agent-scope
// relaxed atomics: sc1 loads and stores that go to the device coherence point, so no
// L2 writeback / invalidate (a __threadfence per workgroup costs more than the work --
// 17.7 us of the two-launch version was mostly those); "s_waitcnt vmcnt(0)" orders a
// workgroup's stores before its ticket.
__device__ __forceinline__ double ld_dev(const double* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_dev(double* p, double v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void stores_done() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__global__ void __launch_bounds__(kVnThreads) vecnorm_kernel(VnArgs a) {
    __shared__ double sh[kVnThreads / 64][kD + 2];
    __shared__ double smean[kD + 2];
    __shared__ double sm2[kD + 2];
    __shared__ double snorm[kD][2];   // per obs column: mean, sqrt(var + eps)
    __shared__ double srstd;
    __shared__ int sgo;
    const int b = blockIdx.x;
    const int64_t r0 = (int64_t)b * a.rows_per_block;
    const int64_t r1 = (r0 + a.rows_per_block < a.n) ? r0 + a.rows_per_block : a.n;
    const double cnt = (double)(r1 > r0 ? r1 - r0 : 0);
    const bool upd_ret = a.training && !a.reset;
    const bool sync = a.upd_obs || upd_ret;
    if (sync) {
        // the generation of this launch's release flag (stable: the previous launch on the
        // stream has finished; its last workgroup advanced it)
        unsigned int gen0 = 0;
        if (threadIdx.x == 0) gen0 = __hip_atomic_load(a.ticket + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // 1. pass 1: sums (and the running-return update)
        double v[kD + 1];
#pragma unroll
        for (int c = 0; c <= kD; ++c) v[c] = 0.0;
        for (int64_t r = r0 + threadIdx.x; r < r1; r += kVnThreads) {
            if (a.upd_obs) {
#pragma unroll
                for (int c = 0; c < kD; ++c) v[c] += (double)a.obs[r * kD + c];
            }
            if (upd_ret) {
                const double ret = a.returns[r] * a.gamma + (double)a.reward[r];   // VecNormalize._update_reward
                a.returns[r] = ret;
                v[kD] += ret;
            }
        }
        block_sum<kD + 1>(v, reinterpret_cast<double(*)[kD + 1]>(sh), smean);
        if (threadIdx.x <= kD) smean[threadIdx.x] = (cnt > 0.0) ? smean[threadIdx.x] / cnt : 0.0;
        __syncthreads();
        // pass 2: sums of squared deviations from the block means
#pragma unroll
        for (int c = 0; c <= kD; ++c) v[c] = 0.0;
        for (int64_t r = r0 + threadIdx.x; r < r1; r += kVnThreads) {
            if (a.upd_obs) {
#pragma unroll
                for (int c = 0; c < kD; ++c) {
                    const double d = (double)a.obs[r * kD + c] - smean[c];
                    v[c] += d * d;
                }
            }
            if (upd_ret) {
                const double d = a.returns[r] - smean[kD];
                v[kD] += d * d;
            }
        }
        block_sum<kD + 1>(v, reinterpret_cast<double(*)[kD + 1]>(sh), sm2);
        double* part = a.part + (int64_t)b * kPart;
        if (threadIdx.x <= kD) {
            const int c = threadIdx.x;
            st_dev(&part[(c < kD) ? 1 + c : 1 + 2 * kD], smean[c]);
            st_dev(&part[(c < kD) ? 1 + kD + c : 2 + 2 * kD], sm2[c]);
        }
        if (threadIdx.x == 0) st_dev(&part[0], cnt);
        stores_done();
        __syncthreads();
        // 2. the last workgroup to arrive merges and releases the others
        if (threadIdx.x == 0) {
            const unsigned int t = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sgo = (t == (unsigned)(a.blocks - 1)) ? 1 : 0;
        }
        __syncthreads();
        if (sgo) {
            // thread k holds partial k; the batch mean as sum n_k mean_k / n, then
            // M2 = sum M2_k + n_k (mean_k - mean)^2 -- block reductions in a fixed order
            const int k = threadIdx.x;
            const double* P = a.part + (int64_t)k * kPart;
            const bool has = k < a.blocks;
            const double n_k = has ? ld_dev(&P[0]) : 0.0;
            double mk[kD + 1], qk[kD + 1];
#pragma unroll
            for (int c = 0; c <= kD; ++c) {
                mk[c] = has ? ld_dev(&P[(c < kD) ? 1 + c : 1 + 2 * kD]) : 0.0;
                qk[c] = has ? ld_dev(&P[(c < kD) ? 1 + kD + c : 2 + 2 * kD]) : 0.0;
            }
            double w[kD + 2];
#pragma unroll
            for (int c = 0; c <= kD; ++c) w[c] = n_k * mk[c];
            w[kD + 1] = n_k;
            block_sum<kD + 2>(w, sh, smean);   // smean[0..kD] = sums, smean[kD + 1] = n
            const double n_a = smean[kD + 1];
#pragma unroll
            for (int c = 0; c <= kD; ++c) {
                const double d = mk[c] - smean[c] / n_a;
                w[c] = qk[c] + n_k * (d * d);
            }
            w[kD + 1] = 0.0;
            block_sum<kD + 2>(w, sh, sm2);
            const double obs_count0 = ld_dev(&a.stats[2 * kD]);
            __syncthreads();   // everyone has read the count before it is written
            const int c = threadIdx.x;
            if (c <= kD) {
                const double mean_a = smean[c] / n_a, m2_a = sm2[c];
                // np.mean / np.var(ddof=0) of the batch, then update_from_moments (:update)
                const int im = (c < kD) ? c : 2 * kD + 1, iv = (c < kD) ? kD + c : 2 * kD + 2;
                if ((c < kD && a.upd_obs) || (c == kD && upd_ret)) {
                    double mean = ld_dev(&a.stats[im]), var = ld_dev(&a.stats[iv]);
                    double count = (c < kD) ? obs_count0 : ld_dev(&a.stats[2 * kD + 3]);
                    rms_update(&mean, &var, &count, mean_a, m2_a / n_a, n_a);
                    st_dev(&a.stats[im], mean);
                    st_dev(&a.stats[iv], var);
                    if (c == 0) st_dev(&a.stats[2 * kD], count);
                    if (c == kD) st_dev(&a.stats[2 * kD + 3], count);
                }
            }
            stores_done();
            __syncthreads();
            if (threadIdx.x == 0) {
                __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // the next launch's
                stores_done();
                __hip_atomic_store(a.ticket + 1, gen0 + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        } else if (threadIdx.x == 0) {
            // relaxed polls (an acquire load per poll would invalidate this XCD's L2 every
            // time: 255 pollers thrash every cache); the statistics are read with sc1 loads
            long spins = 0;
            while (__hip_atomic_load(a.ticket + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen0) {
                if (++spins > kVnSpinLimit) {
                    sgo = -1;   // never released: leave the outputs alone
                    break;
                }
                __builtin_amdgcn_s_sleep(4);
            }
        }
        __syncthreads();
        if (sgo < 0) return;
    }
    // 3. normalize this workgroup's rows with the (new) statistics
    if (threadIdx.x < kD) {
        snorm[threadIdx.x][0] = ld_dev(&a.stats[threadIdx.x]);
        snorm[threadIdx.x][1] = sqrt(ld_dev(&a.stats[kD + threadIdx.x]) + a.eps);
    }
    if (threadIdx.x == 0) srstd = sqrt(ld_dev(&a.stats[2 * kD + 2]) + a.eps);
    __syncthreads();
    for (int64_t r = r0 + threadIdx.x; r < r1; r += kVnThreads) {
        const bool dn = a.done ? a.done[r] != 0 : false;
#pragma unroll
        for (int c = 0; c < kD; ++c) {
            const float x = a.obs[r * kD + c];
            a.obs_out[r * kD + c] =
                a.norm_obs ? (float)clipd(((double)x - snorm[c][0]) / snorm[c][1], -a.clip_obs, a.clip_obs) : x;
        }
        if (a.reset) {
            a.returns[r] = 0.0;
            continue;
        }
        const float rw = a.reward[r];
        a.rew_out[r] = a.norm_reward ? (float)clipd((double)rw / srstd, -a.clip_rew, a.clip_rew) : rw;
        if (dn && a.tobs && a.tobs_out) {
#pragma unroll
            for (int c = 0; c < kD; ++c) {
                const float x = a.tobs[r * kD + c];
                a.tobs_out[r * kD + c] =
                    a.norm_obs ? (float)clipd(((double)x - snorm[c][0]) / snorm[c][1], -a.clip_obs, a.clip_obs) : x;
            }
        }
        if (dn) a.returns[r] = 0.0;   // self.returns[dones] = 0
        if (a.ep_ret) {                 // Monitor: sum(rewards), len(rewards)
            const double er = a.ep_ret[r] + (double)rw;
            const int32_t el = a.ep_len[r] + 1;
            if (dn) {
                a.ep_ret_done[r] = er;
                a.ep_len_done[r] = el;
                a.ep_ret[r] = 0.0;
                a.ep_len[r] = 0;
            } else {
                a.ep_ret[r] = er;
                a.ep_len[r] = el;
            }
        }
    }
}

int blocks_for(int64_t n) {
    int64_t b = (n + kVnThreads - 1) / kVnThreads;   // one row per thread up to 65,536 envs
    if (b > kVnMaxBlocks) b = kVnMaxBlocks;
    return (int)(b < 1 ? 1 : b);
}

__global__ void init_kernel(double* stats) {
    const int i = threadIdx.x;
    if (i < kD) {
        stats[i] = 0.0;
        stats[kD + i] = 1.0;
    }
    if (i == 0) {
        stats[2 * kD] = 1e-4;
        stats[2 * kD + 1] = 0.0;
        stats[2 * kD + 2] = 1.0;
        stats[2 * kD + 3] = 1e-4;
    }
}

he_status launch(VnArgs& a, void* scratch, hipStream_t s) {
    a.blocks = blocks_for(a.n);
    a.rows_per_block = (int)((a.n + a.blocks - 1) / a.blocks);
    a.part = (double*)scratch;
    // {ticket, release generation}: zero-initialised by the caller's scratch (he_vecnorm_scratch_bytes)
    a.ticket = (unsigned int*)((char*)scratch + (size_t)kVnMaxBlocks * kPart * sizeof(double));
    hipLaunchKernelGGL(vecnorm_kernel, dim3(a.blocks), dim3(kVnThreads), 0, s, a);
    return hipGetLastError() == hipSuccess ? HE_OK : HE_EHIP;
}

bool params_ok(const he_vecnorm_params* p) {
    return p && p->obs_dim == kD && isfinite(p->gamma) && p->clip_obs >= 0.0 && p->clip_reward >= 0.0 &&
           p->epsilon >= 0.0;
}

VnArgs base_args(const he_vecnorm_params* p, int64_t n) {
    VnArgs a = {};
    a.n = n;
    a.training = p->training != 0;
    a.norm_obs = p->norm_obs != 0;
    a.norm_reward = p->norm_reward != 0;
    a.upd_obs = a.training && a.norm_obs;
    a.gamma = p->gamma;
    a.clip_obs = p->clip_obs;
    a.clip_rew = p->clip_reward;
    a.eps = p->epsilon;
    return a;
}

__global__ void __launch_bounds__(kVnThreads) nonfinite_kernel(const float* __restrict__ a, int64_t n,
                                                               unsigned long long* count) {
    unsigned long long c = 0;
    for (int64_t i = (int64_t)blockIdx.x * kVnThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kVnThreads)
        c += isfinite(a[i]) ? 0ull : 1ull;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) c += __shfl_xor(c, m, 64);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(count, c);
}

}  // namespace

extern "C" {

he_status he_count_nonfinite(const float* a, int64_t n, unsigned long long* count, void* stream) {
    if (n < 0 || !count || (n > 0 && !a)) return HE_EINVAL;
    if (n == 0) return HE_OK;
    int64_t blocks = (n + kVnThreads - 1) / kVnThreads;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(nonfinite_kernel, dim3((unsigned)blocks), dim3(kVnThreads), 0, (hipStream_t)stream, a, n, count);
    return hipGetLastError() == hipSuccess ? HE_OK : HE_EHIP;
}


int64_t he_vecnorm_stats_len(int32_t obs_dim) { return 2 * (int64_t)obs_dim + 4; }

int64_t he_vecnorm_scratch_bytes(int64_t n, int32_t obs_dim) {
    (void)n;
    (void)obs_dim;
    return (int64_t)kVnMaxBlocks * kPart * sizeof(double) + 256;
}

he_status he_vecnorm_init(double* stats, int32_t obs_dim, void* stream) {
    if (!stats || obs_dim != kD) return HE_EINVAL;
    hipLaunchKernelGGL(init_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, stats);
    return hipGetLastError() == hipSuccess ? HE_OK : HE_EHIP;
}

he_status he_vecnorm_step(const he_vecnorm_params* p, int64_t n, const float* obs, const float* reward,
                          const uint8_t* done, const float* terminal_obs, double* returns, double* stats,
                          void* scratch, float* obs_out, float* reward_out, float* terminal_obs_out,
                          double* ep_return, int32_t* ep_length, double* ep_return_done, int32_t* ep_length_done,
                          void* stream) {
    if (!params_ok(p) || n < 0) return HE_EINVAL;
    if (n == 0) return HE_OK;
    if (!obs || !reward || !returns || !stats || !scratch || !obs_out || !reward_out) return HE_EINVAL;
    if ((ep_return != nullptr) != (ep_length != nullptr) || (ep_return && (!ep_return_done || !ep_length_done || !done)))
        return HE_EINVAL;
    VnArgs a = base_args(p, n);
    a.obs = obs;
    a.reward = reward;
    a.done = done;
    a.tobs = terminal_obs;
    a.returns = returns;
    a.stats = stats;
    a.obs_out = obs_out;
    a.rew_out = reward_out;
    a.tobs_out = terminal_obs_out;
    a.ep_ret = ep_return;
    a.ep_len = ep_length;
    a.ep_ret_done = ep_return_done;
    a.ep_len_done = ep_length_done;
    return launch(a, scratch, (hipStream_t)stream);
}

he_status he_vecnorm_reset(const he_vecnorm_params* p, int64_t n, const float* obs, double* returns, double* stats,
                           void* scratch, float* obs_out, void* stream) {
    if (!params_ok(p) || n < 0) return HE_EINVAL;
    if (n == 0) return HE_OK;
    if (!obs || !returns || !stats || !scratch || !obs_out) return HE_EINVAL;
    VnArgs a = base_args(p, n);
    a.reset = 1;
    a.obs = obs;
    a.returns = returns;
    a.stats = stats;
    a.obs_out = obs_out;
    return launch(a, scratch, (hipStream_t)stream);
}

}  // extern "C"
