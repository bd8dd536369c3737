// vecnorm.hip -- VecNormalize and Monitor statistics on the device (part of libhedgeenv;
// C ABI in include/hedge_env.h).
//
// The reference trains behind SB3 2.6.0's VecNormalize(norm_obs=True, norm_reward=True,
// gamma) (train_ppo_v2.py:204,305) and evaluates with the stats frozen (:450-453); every
// env is wrapped in Monitor(info_keywords=...) (:119).  On the host that is a NumPy
// pass over [N, 13] per step plus per-env Python lists -- the bottleneck once N is in
// the tens of thousands.  Here one step is two launches:
//   moments_kernel  per block: exact two-pass f64 mean / M2 of the obs columns and of
//                   the updated running returns; the last block to finish (atomic
//                   ticket) merges the blocks in block order (Chan et al.) and applies
//                   RunningMeanStd.update_from_moments -- deterministic for a given grid
//   apply_kernel    obs / reward / terminal-obs normalization, returns[done] = 0 and
//                   the Monitor episode sums; one thread per env row
// HBM-bound and tiny (68 B of obs + reward read and written per env); the point is to
// keep the statistics on the device, not the arithmetic.

#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include "../../include/hedge_env.h"

namespace {

constexpr int kD = HE_OBS_DIM;
constexpr int kVnThreads = 256;
constexpr int kVnMaxBlocks = 64;    // the last block stages all partials in LDS and merges them serially

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

// Sum of s[0..kD] over the block into out[0..kD] (LDS): a wave-level butterfly per
// column, then one barrier and a 4-way sum -- two barriers for all 14 columns.
__device__ __forceinline__ void block_sum_cols(double* s, double (*sh)[kD + 1], double* out) {
#pragma unroll
    for (int c = 0; c <= kD; ++c) {
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) s[c] += __shfl_xor(s[c], m, 64);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int c = 0; c <= kD; ++c) sh[w][c] = s[c];
    }
    __syncthreads();
    if (threadIdx.x <= kD) {
        double t = 0.0;
#pragma unroll
        for (int i = 0; i < kVnThreads / 64; ++i) t += sh[i][threadIdx.x];
        out[threadIdx.x] = t;
    }
    __syncthreads();
}

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

__global__ void __launch_bounds__(kVnThreads) moments_kernel(VnArgs a) {
    __shared__ double sh[kVnThreads / 64][kD + 1];
    __shared__ double smean[kD + 1];
    __shared__ double sm2[kD + 1];
    __shared__ bool last;
    const int b = blockIdx.x;
    const int64_t r0 = (int64_t)b * a.rows_per_block;
    const int64_t r1 = (r0 + a.rows_per_block < a.n) ? r0 + a.rows_per_block : a.n;
    const double cnt = (double)(r1 > r0 ? r1 - r0 : 0);
    // pass 1: sums (and the running-return update)
    double s[kD + 1];
#pragma unroll
    for (int c = 0; c <= kD; ++c) s[c] = 0.0;
    for (int64_t r = r0 + threadIdx.x; r < r1; r += kVnThreads) {
        if (a.upd_obs) {
#pragma unroll
            for (int c = 0; c < kD; ++c) s[c] += (double)a.obs[r * kD + c];
        }
        if (a.training && !a.reset) {
            const double ret = a.returns[r] * a.gamma + (double)a.reward[r];   // VecNormalize._update_reward
            a.returns[r] = ret;
            s[kD] += ret;
        }
    }
    block_sum_cols(s, sh, smean);
    if (threadIdx.x <= kD) smean[threadIdx.x] = (cnt > 0.0) ? smean[threadIdx.x] / cnt : 0.0;
    __syncthreads();
    // pass 2: sums of squared deviations from the block means
#pragma unroll
    for (int c = 0; c <= kD; ++c) s[c] = 0.0;
    for (int64_t r = r0 + threadIdx.x; r < r1; r += kVnThreads) {
        if (a.upd_obs) {
#pragma unroll
            for (int c = 0; c < kD; ++c) {
                const double d = (double)a.obs[r * kD + c] - smean[c];
                s[c] += d * d;
            }
        }
        if (a.training && !a.reset) {
            const double d = a.returns[r] - smean[kD];
            s[kD] += d * d;
        }
    }
    block_sum_cols(s, sh, sm2);
    double* part = a.part + (int64_t)b * kPart;
    if (threadIdx.x <= kD) {
        const int c = threadIdx.x;
        part[(c < kD) ? 1 + c : 1 + 2 * kD] = smean[c];
        part[(c < kD) ? 1 + kD + c : 2 + 2 * kD] = sm2[c];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        part[0] = cnt;
        __threadfence();
        last = (atomicAdd(a.ticket, 1u) == (unsigned)(a.blocks - 1));
    }
    __syncthreads();
    if (!last) return;
    // the last block: stage every block's partials in LDS (parallel loads), then merge
    // them in block order, one thread per column; the D obs columns share one count,
    // read before anyone writes it
    __threadfence();
    __shared__ double sp[kVnMaxBlocks * kPart];
    {
        const volatile double* P = a.part;
        for (int k = threadIdx.x; k < a.blocks * kPart; k += kVnThreads) sp[k] = P[k];
    }
    const double obs_count0 = a.stats[2 * kD];
    __syncthreads();
    const int c = threadIdx.x;
    if (c <= kD) {
        // exact merge, two passes over the staged partials in block order: the batch
        // mean from the block sums, then M2 = sum_b M2_b + n_b (mean_b - mean)^2
        const int mi = (c < kD) ? 1 + c : 1 + 2 * kD;
        const int qi = (c < kD) ? 1 + kD + c : 2 + 2 * kD;
        // four interleaved accumulators (k mod 4), combined in a fixed order: the LDS
        // reads of a chain are independent, so the loop is not latency-bound
        double n4[4] = {0.0, 0.0, 0.0, 0.0}, s4[4] = {0.0, 0.0, 0.0, 0.0};
        int k = 0;
        for (; k + 4 <= a.blocks; k += 4) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const double n_b = sp[(k + u) * kPart];
                n4[u] += n_b;
                s4[u] = fma(n_b, sp[(k + u) * kPart + mi], s4[u]);
            }
        }
        for (; k < a.blocks; ++k) {
            const double n_b = sp[k * kPart];
            n4[0] += n_b;
            s4[0] = fma(n_b, sp[k * kPart + mi], s4[0]);
        }
        const double n_a = (n4[0] + n4[1]) + (n4[2] + n4[3]);
        const double mean_a = ((s4[0] + s4[1]) + (s4[2] + s4[3])) / n_a;
        double q4[4] = {0.0, 0.0, 0.0, 0.0};
        for (k = 0; k + 4 <= a.blocks; k += 4) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const double d = sp[(k + u) * kPart + mi] - mean_a;
                q4[u] += sp[(k + u) * kPart + qi] + sp[(k + u) * kPart] * (d * d);
            }
        }
        for (; k < a.blocks; ++k) {
            const double d = sp[k * kPart + mi] - mean_a;
            q4[0] += sp[k * kPart + qi] + sp[k * kPart] * (d * d);
        }
        const double m2_a = (q4[0] + q4[1]) + (q4[2] + q4[3]);
        // np.mean / np.var(ddof=0) of the batch, then update_from_moments (:update)
        if (c < kD) {
            if (a.upd_obs) {
                double cnt0 = obs_count0;
                rms_update(&a.stats[c], &a.stats[kD + c], &cnt0, mean_a, m2_a / n_a, n_a);
                if (c == 0) a.stats[2 * kD] = cnt0;
            }
        } else if (a.training && !a.reset) {
            rms_update(&a.stats[2 * kD + 1], &a.stats[2 * kD + 2], &a.stats[2 * kD + 3], mean_a, m2_a / n_a, n_a);
        }
    }
    if (threadIdx.x == 0) *a.ticket = 0u;   // ready for the next launch
}

__device__ __forceinline__ double clipd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }

__global__ void __launch_bounds__(kVnThreads) apply_kernel(VnArgs a) {
    __shared__ double sm[kD], ss[kD];
    __shared__ double rstd;
    if (threadIdx.x < kD) {
        sm[threadIdx.x] = a.stats[threadIdx.x];
        ss[threadIdx.x] = sqrt(a.stats[kD + threadIdx.x] + a.eps);
    }
    if (threadIdx.x == 0) rstd = sqrt(a.stats[2 * kD + 2] + a.eps);
    __syncthreads();
    const int64_t r = (int64_t)blockIdx.x * kVnThreads + threadIdx.x;
    if (r >= a.n) return;
    const bool dn = a.done ? a.done[r] != 0 : false;
#pragma unroll
    for (int c = 0; c < kD; ++c) {
        const float x = a.obs[r * kD + c];
        a.obs_out[r * kD + c] =
            a.norm_obs ? (float)clipd(((double)x - sm[c]) / ss[c], -a.clip_obs, a.clip_obs) : x;
    }
    if (a.reset) {
        a.returns[r] = 0.0;
        return;
    }
    const float rw = a.reward[r];
    a.rew_out[r] = a.norm_reward ? (float)clipd((double)rw / rstd, -a.clip_rew, a.clip_rew) : rw;
    if (dn && a.tobs && a.tobs_out) {
#pragma unroll
        for (int c = 0; c < kD; ++c) {
            const float x = a.tobs[r * kD + c];
            a.tobs_out[r * kD + c] =
                a.norm_obs ? (float)clipd(((double)x - sm[c]) / ss[c], -a.clip_obs, a.clip_obs) : x;
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

int blocks_for(int64_t n) {
    int64_t b = (n + 4 * kVnThreads - 1) / (4 * kVnThreads);   // >= 4 rows per thread
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
    a.ticket = (unsigned int*)((char*)scratch + (size_t)kVnMaxBlocks * kPart * sizeof(double));
    if (a.upd_obs || (a.training && !a.reset)) {
        hipLaunchKernelGGL(moments_kernel, dim3(a.blocks), dim3(kVnThreads), 0, s, a);
        if (hipGetLastError() != hipSuccess) return HE_EHIP;
    }
    hipLaunchKernelGGL(apply_kernel, dim3((unsigned)((a.n + kVnThreads - 1) / kVnThreads)), dim3(kVnThreads), 0, s,
                       a);
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
