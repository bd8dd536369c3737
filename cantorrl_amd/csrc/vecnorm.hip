// vecnorm.hip -- VecNormalize and Monitor statistics on the device (part of libhedgeenv;
// C ABI in include/hedge_env.h).
//
// The reference trains behind SB3 2.6.0's VecNormalize(norm_obs=True, norm_reward=True,
// gamma) (train_ppo_v2.py:204,305) and evaluates with the stats frozen (:450-453); every
// env is wrapped in Monitor(info_keywords=...) (:119).  On the host that is a NumPy
// pass over [N, 13] per step plus per-env Python lists -- the bottleneck once N is in
// the tens of thousands.  Here one step is two launches of G <= 256 workgroups, each
// owning a slice of 256 rows staged through LDS as flat coalesced copies:
//   vn_moments_kernel  one pass of f64 sums of d and d^2, d = x - shift (the batch's row 0
//                      for obs, the old running mean for the returns), over the slice's obs
//                      columns and updated running returns, stored as a partial (+ a
//                      snapshot of the old statistics and the shifts);
//   vn_apply_kernel    every workgroup merges all G partials itself (one block reduction in
//                      a fixed order, so the same result everywhere), applies
//                      RunningMeanStd.update_from_moments (workgroup 0 stores it), and
//                      normalizes its rows by (x - mean) * (1 / sqrt(var + eps)): obs /
//                      reward / terminal obs, returns[done] = 0 and the Monitor episode sums.
// Deterministic for a given grid; no atomics and no waiting between workgroups (the
// kernel boundary publishes the partials).  Eval mode (no statistics update) is the
// second launch alone.  68 B of obs + reward read and written per env.

#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include "../../include/hedge_env.h"
#include "vn_moments.h"

namespace {

using vn::kD;
using vn::kPart;
using vn::kVnChunk;
using vn::kVnMaxBlocks;
using vn::kVnThreads;
using vn::block_sum;
using vn::load_tile;

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
    float* obs_out;
    float* rew_out;
    float* tobs_out;
    double* ep_ret;
    int32_t* ep_len;
    double* ep_ret_done;
    int32_t* ep_len_done;
    const double* ep_reward;   // the env's f64 step rewards Monitor sums (he_info::reward_step)
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

struct VnRows {
    int64_t r0, r1;
    double cnt;
};
__device__ __forceinline__ VnRows rows_of(const VnArgs& a) {
    VnRows w;
    w.r0 = (int64_t)blockIdx.x * a.rows_per_block;
    w.r1 = (w.r0 + a.rows_per_block < a.n) ? w.r0 + a.rows_per_block : a.n;
    w.cnt = (double)(w.r1 > w.r0 ? w.r1 - w.r0 : 0);
    return w;
}

// Launch 1 (training): the moments partials of each workgroup's rows (vn_moments.h;
// the obs shift is the batch's row 0).  The kernel boundary publishes the partials to
// launch 2 -- no atomics, no waiting (a single launch with a grid-wide wait measured
// 25 us at 65,536 envs: four dependent device-coherent round trips between workgroups).
__device__ __forceinline__ vn::MomentsArgs moments_args(const VnArgs& a) {
    vn::MomentsArgs m = {};
    m.n = a.n;
    m.rows_per_block = a.rows_per_block;
    m.upd_obs = a.upd_obs;
    m.upd_ret = a.training && !a.reset;
    m.shift_mean = 0;
    m.gamma = a.gamma;
    m.obs = a.obs;
    m.reward = a.reward;
    m.returns = a.returns;
    m.stats = a.stats;
    m.part = a.part;
    return m;
}
__global__ void __launch_bounds__(kVnThreads) vn_moments_kernel(VnArgs a) {
    vn::moments_body(moments_args(a), blockIdx.x);
}

// A row's inputs besides its obs: reward, done flag, Monitor running sums and the f64
// reward Monitor adds (Monitor wraps each env inside the VecEnv, train_ppo_v2.py:119, so it
// sums the env's own f64 reward, hedging_env_v2.py:262,294 -- not the f32 VecEnv buffer).
struct RowIn {
    float rw;
    bool dn;
    double er;
    double rw64;
    int32_t el;
};
__device__ __forceinline__ RowIn row_in(const VnArgs& a, int64_t r) {
    RowIn in;
    in.rw = a.reward[r];
    in.dn = a.done ? a.done[r] != 0 : false;
    in.er = a.ep_ret ? a.ep_ret[r] : 0.0;
    in.rw64 = a.ep_ret ? a.ep_reward[r] : 0.0;
    in.el = a.ep_ret ? a.ep_len[r] : 0;
    return in;
}

constexpr int kMergeLanes = 8;   // lanes per merged value (vn_apply_kernel)
static_assert(kMergeLanes * kPart <= kVnThreads, "one merge lane group per value");
using vn::ColNorm;
using vn::col_norm;
using vn::norm_elem;

// Launch 2: every workgroup merges all the partials itself (one block reduction in a
// fixed order, so the same statistics everywhere; workgroup 0 stores them), then
// normalizes its rows: obs / reward / terminal obs, returns[done] = 0, Monitor sums.
// (2 or 4 rows per thread, so fewer workgroups read the partials, measured slower: rocprof
// 7.5 / 10.2 / 15.9 us at 65,536 envs, r03s32 -- the merge's reads are not what the launch
// waits on; each thread's rows are.)
__global__ void __launch_bounds__(kVnThreads) vn_apply_kernel(VnArgs a) {
    constexpr int R = 1;
    __shared__ double ssum[kPart];
    __shared__ ColNorm snorm[kD];     // per obs column (col_norm)
    __shared__ double srinv;
    __shared__ float tile[kVnChunk * kD];
    const VnRows w = rows_of(a);
    const float clip = (float)a.clip_obs;
    const bool upd_ret = a.training && !a.reset;
    const int t = threadIdx.x;
    const bool resident = w.r1 - w.r0 <= kVnChunk * R;
    const int nrows = (int)(w.r1 - w.r0);
    // the rows' loads first -- obs, and the row's reward, done flag and Monitor sums: they
    // are all in flight while the partials are merged (one memory round trip per launch)
    float xr[R * kD];
    const int nres = resident ? nrows * kD : 0;
    const float* src = a.obs + w.r0 * kD;
#pragma unroll
    for (int q = 0; q < R * kD; ++q) {
        const int k = t + q * kVnThreads;
        xr[q] = k < nres ? src[k] : 0.0f;
    }
    RowIn pin[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
        pin[j] = {};
        if (resident && !a.reset && t + j * kVnThreads < nrows) pin[j] = row_in(a, w.r0 + t + j * kVnThreads);
    }
    if (a.upd_obs || upd_ret) {
        // the merge, transposed: thread t < 8 kPart sums value c = t / 8 of the partials
        // b = t % 8, t % 8 + 8, ... (in b order), then a butterfly over its 8-lane group --
        // no block-wide LDS reduction (the row-major block_sum stored and re-read 61 KB)
        if (t < kMergeLanes * kPart) {
            const int c = t / kMergeLanes, j = t % kMergeLanes;
            const double* P = a.part + (size_t)c * kVnMaxBlocks;
            // every load issued before the first add (unrolled over the kVnMaxBlocks bound):
            // a rolled loop waited one round trip per partial
            double v[kVnMaxBlocks / kMergeLanes];
#pragma unroll
            for (int q = 0; q < kVnMaxBlocks / kMergeLanes; ++q) {
                const int b = j + q * kMergeLanes;
                v[q] = b < a.blocks ? P[b] : 0.0;
            }
            double x = 0.0;
#pragma unroll
            for (int q = 0; q < kVnMaxBlocks / kMergeLanes; ++q) x += v[q];
#pragma unroll
            for (int m = kMergeLanes / 2; m >= 1; m >>= 1) x += __shfl_xor(x, m, kMergeLanes);
            if (j == 0) ssum[c] = x;   // ssum[0] = n, [1 .. kD + 1] = S1, then S2
        }
        __syncthreads();
        const int c = t;
        if (c <= kD) {
            const double* old = a.part + kVnMaxBlocks * kPart;   // launch 1's snapshot
            const double n_a = ssum[0], s1 = ssum[1 + c], s2 = ssum[2 + kD + c];
            // np.mean / np.var(ddof=0) of the batch from the shifted sums, then
            // RunningMeanStd.update_from_moments
            const double mean_a = old[2 * kD + 4 + c] + s1 / n_a;
            const double m2 = s2 - s1 * (s1 / n_a);
            const double var_a = (m2 > 0.0 ? m2 : 0.0) / n_a;
            const int im = (c < kD) ? c : 2 * kD + 1, iv = (c < kD) ? kD + c : 2 * kD + 2;
            double mean = old[im], var = old[iv];
            if ((c < kD && a.upd_obs) || (c == kD && upd_ret)) {
                double count = (c < kD) ? old[2 * kD] : old[2 * kD + 3];
                rms_update(&mean, &var, &count, mean_a, var_a, n_a);
                if (blockIdx.x == 0) {
                    if (c == 0) a.stats[2 * kD] = count;
                    if (c == kD) a.stats[2 * kD + 3] = count;
                    a.stats[im] = mean;
                    a.stats[iv] = var;
                }
            }
            if (c < kD) {
                snorm[c] = col_norm(mean, var, a.eps);
            } else {
                srinv = 1.0 / sqrt(var + a.eps);
            }
        }
        __syncthreads();
    } else {
        if (t < kD) snorm[t] = col_norm(a.stats[t], a.stats[kD + t], a.eps);
        if (t == 0) srinv = 1.0 / sqrt(a.stats[2 * kD + 2] + a.eps);
        __syncthreads();
    }
    // the rows' own work (reward, returns, terminal obs, Monitor): thread t, row r0 + t
    auto row_work = [&](int64_t r, const RowIn& in) {
        if (a.reset) {
            a.returns[r] = 0.0;
            return;
        }
        const bool dn = in.dn;
        const float rw = in.rw;
        a.rew_out[r] = a.norm_reward ? (float)clipd((double)rw * srinv, -a.clip_rew, a.clip_rew) : rw;
        if (dn && a.tobs && a.tobs_out) {   // rare: per-row accesses
#pragma unroll
            for (int c = 0; c < kD; ++c) {
                const float x = a.tobs[r * kD + c];
                a.tobs_out[r * kD + c] = a.norm_obs ? norm_elem(x, snorm[c], clip) : x;
            }
        }
        if (dn) a.returns[r] = 0.0;   // self.returns[dones] = 0
        if (a.ep_ret) {                 // Monitor: sum(rewards) of the f64 rewards, len(rewards)
            const double er = in.er + in.rw64;
            const int32_t el = in.el + 1;
            if (dn) {
                a.ep_ret_done[r] = er;
                a.ep_len_done[r] = el;
            }
            a.ep_ret[r] = dn ? 0.0 : er;
            a.ep_len[r] = dn ? 0 : el;
        }
    };
    if (resident) {
        // the obs element-wise straight from the registers the loads landed in: element
        // k = t + 256 q of the slice is column k % 13 (the slice starts at a row boundary),
        // stepped by 256 % 13 = 9 per q without a division
        float* dst = a.obs_out + w.r0 * kD;
        int c = t % kD;
#pragma unroll
        for (int q = 0; q < R * kD; ++q) {
            const int k = t + q * kVnThreads;
            if (k < nres) dst[k] = a.norm_obs ? norm_elem(xr[q], snorm[c], clip) : xr[q];
            c += kVnThreads % kD;
            c = c >= kD ? c - kD : c;
        }
#pragma unroll
        for (int j = 0; j < R; ++j)
            if (t + j * kVnThreads < nrows) row_work(w.r0 + t + j * kVnThreads, pin[j]);
        return;
    }
    for (int64_t c0 = w.r0; c0 < w.r1; c0 += kVnChunk) {
        const int rows = (int)((w.r1 - c0) < kVnChunk ? (w.r1 - c0) : kVnChunk);
        load_tile(tile, a.obs, c0, rows);
        if (t < rows) {
            // the row in place in LDS, then stored back as a flat coalesced copy
            if (a.norm_obs) {
#pragma unroll
                for (int c = 0; c < kD; ++c) tile[t * kD + c] = norm_elem(tile[t * kD + c], snorm[c], clip);
            }
            row_work(c0 + t, a.reset ? RowIn{} : row_in(a, c0 + t));
        }
        __syncthreads();
        float* dst = a.obs_out + c0 * kD;
        const int nf = rows * kD;
        for (int k = t; k < nf; k += kVnThreads) dst[k] = tile[k];
        __syncthreads();
    }
}

int blocks_for(int64_t n) {
    int64_t b = (n + kVnChunk - 1) / kVnChunk;   // one row per thread up to 65,536 envs
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

he_status launch(VnArgs& a, void* scratch, hipStream_t s, bool moments = true) {
    a.blocks = blocks_for(a.n);
    a.rows_per_block = (int)((a.n + a.blocks - 1) / a.blocks);
    a.part = (double*)scratch;   // [kVnMaxBlocks][kPart] partials, then the old statistics
    if (moments && (a.upd_obs || (a.training && !a.reset))) {
        hipLaunchKernelGGL(vn_moments_kernel, dim3(a.blocks), dim3(kVnThreads), 0, s, a);
        if (hipGetLastError() != hipSuccess) return HE_EHIP;
    }
    hipLaunchKernelGGL(vn_apply_kernel, dim3(a.blocks), dim3(kVnThreads), 0, s, a);
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
    return ((int64_t)kVnMaxBlocks * kPart + 3 * kD + 5) * (int64_t)sizeof(double);  // partials + old statistics + shifts
}

he_status he_vecnorm_init(double* stats, int32_t obs_dim, void* stream) {
    if (!stats || obs_dim != kD) return HE_EINVAL;
    hipLaunchKernelGGL(init_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, stats);
    return hipGetLastError() == hipSuccess ? HE_OK : HE_EHIP;
}

static he_status vecnorm_step(const he_vecnorm_params* p, int64_t n, const float* obs, const float* reward,
                              const uint8_t* done, const float* terminal_obs, double* returns, double* stats,
                              void* scratch, float* obs_out, float* reward_out, float* terminal_obs_out,
                              double* ep_return, int32_t* ep_length, double* ep_return_done,
                              int32_t* ep_length_done, const double* ep_reward, void* stream, bool moments) {
    if (!params_ok(p) || n < 0) return HE_EINVAL;
    if (n == 0) return HE_OK;
    if (!obs || !reward || !returns || !stats || !scratch || !obs_out || !reward_out) return HE_EINVAL;
    if ((ep_return != nullptr) != (ep_length != nullptr) ||
        (ep_return && (!ep_return_done || !ep_length_done || !done || !ep_reward)))
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
    a.ep_reward = ep_reward;
    return launch(a, scratch, (hipStream_t)stream, moments);
}

he_status he_vecnorm_step(const he_vecnorm_params* p, int64_t n, const float* obs, const float* reward,
                          const uint8_t* done, const float* terminal_obs, double* returns, double* stats,
                          void* scratch, float* obs_out, float* reward_out, float* terminal_obs_out,
                          double* ep_return, int32_t* ep_length, double* ep_return_done, int32_t* ep_length_done,
                          const double* ep_reward, void* stream) {
    return vecnorm_step(p, n, obs, reward, done, terminal_obs, returns, stats, scratch, obs_out, reward_out,
                        terminal_obs_out, ep_return, ep_length, ep_return_done, ep_length_done, ep_reward, stream, true);
}

he_status he_vecnorm_apply(const he_vecnorm_params* p, int64_t n, const float* obs, const float* reward,
                           const uint8_t* done, const float* terminal_obs, double* returns, double* stats,
                           void* scratch, float* obs_out, float* reward_out, float* terminal_obs_out,
                           double* ep_return, int32_t* ep_length, double* ep_return_done, int32_t* ep_length_done,
                           const double* ep_reward, void* stream) {
    // training merges the fused partials, which cover <= 65,536 rows; frozen statistics read none
    if (p && p->training && n > (int64_t)kVnMaxBlocks * kVnThreads) return HE_EINVAL;
    return vecnorm_step(p, n, obs, reward, done, terminal_obs, returns, stats, scratch, obs_out, reward_out,
                        terminal_obs_out, ep_return, ep_length, ep_return_done, ep_length_done, ep_reward, stream, false);
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
