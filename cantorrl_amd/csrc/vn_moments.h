// vn_moments.h -- the first half of a VecNormalize step (SB3 2.6.0 VecNormalize.step_wait:
// obs_rms.update(obs), returns = returns * gamma + reward, ret_rms.update(returns);
// train_ppo_v2.py:204,305), shared by vecnorm.hip's vn_moments_kernel and by hedge_env.hip's
// step1_vn_kernel, which runs it as the epilogue of he_step on the rows its workgroup has
// just written (he_vecnorm_attach).
//
// Per workgroup of kVnThreads threads and up to rows_per_block rows: one pass of f64 sums
// S1 = sum d and S2 = sum d^2 with d = x - shift over the 13 obs columns and the updated
// running returns, stored as partial [kPart][kVnMaxBlocks] (count, S1[D + 1], S2[D + 1]);
// workgroup 0 also stores a snapshot of the old statistics and the shifts, which
// vn_apply_kernel (vecnorm.hip) reads after the kernel boundary.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hedge_env.h"

namespace vn {

constexpr int kD = HE_OBS_DIM;
constexpr int kVnThreads = 256;
constexpr int kVnMaxBlocks = 256;   // workgroups of a launch = partials merged per workgroup (one per thread)
constexpr int kVnChunk = kVnThreads;   // rows staged in LDS at a time (one per thread)
// scratch layout: [kPart][kVnMaxBlocks] doubles, then the 2 kD + 4 old statistics and
// the kD + 1 shifts of the sums
constexpr int kPart = 2 * kD + 3;   // count, S1[D + 1] (obs, returns), S2[D + 1]

struct MomentsArgs {
    int64_t n;
    int32_t rows_per_block;
    int32_t upd_obs, upd_ret;
    int32_t shift_mean;      // obs shift: 1 the old running mean (the fused epilogue: row 0 is
                             // another workgroup's output), 0 the batch's row 0
    double gamma;
    const float* obs;
    const float* reward;
    double* returns;
    const double* stats;
    double* part;
};

// Sum of v[0..NV) over the block into out[0..NV) (LDS), NV <= 32: every thread stores
// its NV values (row stride NV + 1), then TPV = 16 (NV <= 16) or 8 threads per value sum
// 256 / TPV rows each and finish with a butterfly inside their TPV-lane group -- against
// 6 shuffle levels per value (~180 LDS permutes per wave) of a butterfly over the whole
// wave.  The summation order is fixed.
template <int NV>
__device__ __forceinline__ void block_sum(const double* v, double* buf, double* out) {
    constexpr int TPV = NV <= 16 ? 16 : 8;
    static_assert(NV <= 32 && NV * TPV <= kVnThreads, "threads per value");
    constexpr int S = NV + 1;
    const int t = threadIdx.x;
#pragma unroll
    for (int c = 0; c < NV; ++c) buf[t * S + c] = v[c];
    __syncthreads();
    if (t < NV * TPV) {
        const int c = t / TPV, j = t % TPV;
        double x = 0.0;
#pragma unroll
        for (int k = 0; k < kVnThreads / TPV; ++k) x += buf[(j + TPV * k) * S + c];
#pragma unroll
        for (int m = TPV / 2; m >= 1; m >>= 1) x += __shfl_xor(x, m, TPV);
        if (j == 0) out[c] = x;
    }
    __syncthreads();
}

// Rows [c0, c0 + rows) of obs -> LDS tile, as a flat coalesced copy (the [N][13] rows are
// 52 B apart: per-row loads would touch 26 cache lines per wave instruction); the rows
// are then read from LDS with a stride of 13 words (odd: no bank conflicts).
__device__ __forceinline__ void load_tile(float* tile, const float* obs, int64_t c0, int rows) {
    const float* src = obs + c0 * kD;
    const int nf = rows * kD;
    for (int k = threadIdx.x; k < nf; k += kVnThreads) tile[k] = src[k];
    __syncthreads();
}

// The block sum of a workgroup's moments v, stored as its partial (+ workgroup 0: the
// snapshot of the old statistics and of the shifts).
__device__ __forceinline__ void store_partial(const MomentsArgs& a, int bid, const double* v, const double* sft,
                                             int64_t rows) {
    __shared__ double sh[kVnThreads * (kPart + 1)];
    __shared__ double ssum[kPart];
    const int t = threadIdx.x;
    block_sum<kPart - 1>(v, sh, ssum);
    double* part = a.part + bid;
    if (t < kPart - 1) part[(1 + t) * kVnMaxBlocks] = ssum[t];
    if (t == 0) part[0] = (double)rows;
    double* snap = a.part + kVnMaxBlocks * kPart;
    if (bid == 0 && t < 2 * kD + 4) snap[t] = a.stats[t];
    if (bid == 0 && t <= kD) snap[2 * kD + 4 + t] = sft[t];
}

// The moments of workgroup `bid`'s rows (blockDim.x == kVnThreads).
__device__ __forceinline__ void moments_body(const MomentsArgs& a, int bid) {
    __shared__ float tile[kVnChunk * kD];
    const int64_t r0 = (int64_t)bid * a.rows_per_block;
    const int64_t r1 = (r0 + a.rows_per_block < a.n) ? r0 + a.rows_per_block : a.n;
    const int t = threadIdx.x;
    double sft[kD + 1];
#pragma unroll
    for (int c = 0; c < kD; ++c) sft[c] = a.shift_mean ? a.stats[c] : (double)a.obs[c];
    sft[kD] = a.stats[2 * kD + 1];
    double v[kPart - 1];
#pragma unroll
    for (int c = 0; c < kPart - 1; ++c) v[c] = 0.0;
    for (int64_t c0 = r0; c0 < r1; c0 += kVnChunk) {
        const int rows = (int)((r1 - c0) < kVnChunk ? (r1 - c0) : kVnChunk);
        if (a.upd_obs) load_tile(tile, a.obs, c0, rows);
        if (t < rows) {
            if (a.upd_obs) {
#pragma unroll
                for (int c = 0; c < kD; ++c) {
                    const double d = (double)tile[t * kD + c] - sft[c];
                    v[c] += d;
                    v[kD + 1 + c] += d * d;
                }
            }
            if (a.upd_ret) {
                const int64_t r = c0 + t;
                const double ret = a.returns[r] * a.gamma + (double)a.reward[r];   // VecNormalize._update_reward
                a.returns[r] = ret;
                const double d = ret - sft[kD];
                v[kD] += d;
                v[2 * kD + 1] += d * d;
            }
        }
        __syncthreads();
    }
    store_partial(a, bid, v, sft, r1 > r0 ? r1 - r0 : 0);
}

// The same moments from rows already in LDS (step1_vn_kernel: the he_step workgroup's obs
// staging tile, row t at tile + t * kD, after a workgroup barrier), the thread's reward
// `rew` (its row r0 + t) and its running return before the update `ret_prev`, with no global
// round trip.  Obs shift: the old running mean (a.shift_mean).
// col_shift: this thread's column's shift (the old running mean of obs column t % (kD + 1),
// or of the returns), loaded by the caller before its step so it is not a round trip here.
__device__ __forceinline__ double load_col_shift(const MomentsArgs& a) {
    const int c = (int)(threadIdx.x % (kD + 1));
    return a.stats[c < kD ? c : 2 * kD + 1];
}
// Column-major over the LDS rows: thread t < kColThreads takes column c = t % (kD + 1)
// (13 obs columns, then the returns) and rows g, g + kColGroups, ... (g = t / (kD + 1)), summing
// d and d^2 of its rows in f64; the kColGroups group sums of each column are then added in group
// order by 2 (kD + 1) threads.  ~6 KB of LDS traffic per workgroup against the row-major
// block_sum's 57 KB (every thread's 28 values written, then read back): the fused epilogue's
// cost on the step kernel.  The summation order differs from moments_body's (row-major), so
// the statistics agree to rounding, not bit for bit (test_fused_moments_equal_separate_launch).
constexpr int kColGroups = kVnThreads / (kD + 1);            // 18
constexpr int kColThreads = kColGroups * (kD + 1);           // 252
__device__ __forceinline__ void moments_from_rows(const MomentsArgs& a, int bid, const float* tile, float rew,
                                                  double ret_prev, double col_shift) {
    __shared__ double rbuf[kVnThreads];
    __shared__ double red[kColGroups][kD + 1][2];
    const int64_t r0 = (int64_t)bid * a.rows_per_block;
    const int64_t r1 = (r0 + a.rows_per_block < a.n) ? r0 + a.rows_per_block : a.n;
    const int rows = (int)(r1 > r0 ? r1 - r0 : 0);
    const int t = threadIdx.x;
    if (a.upd_ret && t < rows) {
        const double ret = ret_prev * a.gamma + (double)rew;   // VecNormalize._update_reward
        a.returns[r0 + t] = ret;
        rbuf[t] = ret;
    }
    __syncthreads();
    if (t < kColThreads) {
        const int c = t % (kD + 1), g = t / (kD + 1);
        double s1 = 0.0, s2 = 0.0;
        if (c < kD ? a.upd_obs : a.upd_ret) {
            const double sh = col_shift;
            for (int r = g; r < rows; r += kColGroups) {
                const double x = (c < kD) ? (double)tile[r * kD + c] : rbuf[r];
                const double d = x - sh;
                s1 += d;
                s2 += d * d;
            }
        }
        red[g][c][0] = s1;
        red[g][c][1] = s2;
    }
    __syncthreads();
    if (t < 2 * (kD + 1)) {
        const int w = t / (kD + 1), c = t % (kD + 1);
        double x = 0.0;
#pragma unroll
        for (int g = 0; g < kColGroups; ++g) x += red[g][c][w];
        // partial layout: [count, S1[kD + 1], S2[kD + 1]] (S1[kD] / S2[kD]: the returns)
        a.part[(1 + w * (kD + 1) + c) * kVnMaxBlocks + bid] = x;
    }
    if (t == 0) a.part[bid] = (double)rows;
    double* snap = a.part + kVnMaxBlocks * kPart;
    if (bid == 0 && t < 2 * kD + 4) snap[t] = a.stats[t];
    if (bid == 0 && t <= kD) snap[2 * kD + 4 + t] = col_shift;   // thread t <= kD: column t
}

// ------------------------------------------------------------------ eval: the whole step fused
// VecNormalize.step_wait with the statistics frozen (training=False, train_ppo_v2.py:450-453):
// no moments, so nothing crosses workgroups and he_step's own launch can finish the step
// (step1_vne_kernel, he_vecnorm_attach_eval) -- the obs rows normalized from the step's LDS
// staging tile, the reward from the thread's register (f32 for VecNormalize, the f64 one for
// Monitor, which sums the env's own rewards: train_ppo_v2.py:119), returns[done] = 0, Monitor's sums and
// the normalized terminal obs of done rows.  The same per-element arithmetic as vecnorm.hip's
// apply (ColNorm, norm_elem): the same bits as he_step + he_vecnorm_apply.
struct ColNorm {
    float mh, mls, sh, sl;   // mean = mh + ml, s = 1 / sqrt(var + eps) = sh + sl, mls = RN(ml s)
};
__device__ __forceinline__ ColNorm col_norm(double mean, double var, double eps) {
    const double s = 1.0 / sqrt(var + eps);
    const float mh = (float)mean, sh = (float)s;
    // s past FLT_MAX (var + eps = 0, e.g. epsilon = 0 on a constant column): the split terms
    // would be inf - inf and 0 * inf = NaN for every element; with them 0 an element is
    // (x - mh) * inf = +-inf -> +-clip, as the f64 (x - mean) / sqrt(var + eps) clips (0 / 0
    // stays NaN, as in SB3)
    if (!(sh <= 3.402823466e38f)) return ColNorm{mh, 0.0f, sh, 0.0f};
    return ColNorm{mh, (float)((mean - (double)mh) * s), sh, (float)(s - (double)sh)};
}
// VecNormalize.normalize_obs of one element in f32 from the merged f64 statistics, converted
// once per column (col_norm): y = (x - mh) (sh + sl) - ml s.  x - mh is exact within a factor
// 2 of the mean (Sterbenz), else one rounding; the two FMAs round once more (the sl and ml s
// terms are corrections far below y's last bit).  About 1 f32 ulp of y against the f64
// (x - mean) / sqrt(var + eps) -- the tests allow 2e-6 absolute at |y| <= clip = 10, ~2 ulp.
// np.clip in f32 (NaN stays NaN).
__device__ __forceinline__ float norm_elem(float x, const ColNorm& n, float clip) {
    const float d = x - n.mh;
    const float r = fmaf(d, n.sh, fmaf(d, n.sl, -n.mls));
    return r < -clip ? -clip : (r > clip ? clip : r);
}
__device__ __forceinline__ double clip_d(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }

struct ApplyArgs {
    int32_t norm_obs, norm_reward;
    double clip_obs, clip_rew, eps;
    const double* stats;
    double* returns;
    float* obs_out;
    float* rew_out;
    float* tobs_out;
    double* ep_ret;       // Monitor sums (NULL: none)
    int32_t* ep_len;
    double* ep_ret_done;
    int32_t* ep_len_done;
};
// What a thread of the fused kernel loads before its step (off the epilogue's path): thread
// t < kD the statistics of obs column t, thread kD the returns' variance; its row's Monitor sums.
struct FrozenPre {
    double m, v, er;
    int32_t el;
};
__device__ __forceinline__ FrozenPre load_frozen(const ApplyArgs& a, int64_t r, bool live) {
    const int t = threadIdx.x;
    FrozenPre f{0.0, 1.0, 0.0, 0};
    if (t < kD) {
        f.m = a.stats[t];
        f.v = a.stats[kD + t];
    } else if (t == kD) {
        f.v = a.stats[2 * kD + 2];
    }
    if (a.ep_ret && live) {
        f.er = a.ep_ret[r];
        f.el = a.ep_len[r];
    }
    return f;
}
// The per-column constants in LDS, made before the step (their f64 square roots and divisions
// overlap the step's loads; the step's own barrier publishes them).
struct FrozenNorm {
    ColNorm cn[kD];
    double rinv;
};
__device__ __forceinline__ void prep_frozen(FrozenNorm& z, const ApplyArgs& a, const FrozenPre& f) {
    const int t = threadIdx.x;
    if (t < kD) z.cn[t] = col_norm(f.m, f.v, a.eps);
    if (t == kD) z.rinv = 1.0 / sqrt(f.v + a.eps);
}
// rows [r0, r0 + rows) of the workgroup, obs staged at tile (row t at tile + t kD), after a
// workgroup barrier that follows prep_frozen; thread t < rows owns row r0 + t: its reward, done
// flag and terminal obs row.
__device__ __forceinline__ void apply_frozen_rows(const ApplyArgs& a, const FrozenNorm& z, int64_t r0, int rows,
                                                  const float* tile, const FrozenPre& f, float rew, double rew64,
                                                  bool done, const float* tobs) {
    const ColNorm* cn = z.cn;
    const double rinv = z.rinv;
    const int t = threadIdx.x;
    const float clip = (float)a.clip_obs;
    // the obs as a flat coalesced copy: element k = t + 256 q is column k % 13 (rows start at a
    // row boundary), stepped by 256 % 13 = 9 per q without a division
    float* dst = a.obs_out + r0 * kD;
    const int nf = rows * kD;
    int c = t % kD;
#pragma unroll
    for (int q = 0; q < kD; ++q) {
        const int k = t + q * kVnThreads;
        if (k < nf) dst[k] = a.norm_obs ? norm_elem(tile[k], cn[c], clip) : tile[k];
        c += kVnThreads % kD;
        c = c >= kD ? c - kD : c;
    }
    if (t >= rows) return;
    const int64_t r = r0 + t;
    a.rew_out[r] = a.norm_reward ? (float)clip_d((double)rew * rinv, -a.clip_rew, a.clip_rew) : rew;
    if (done && tobs && a.tobs_out) {   // rare: per-row accesses (this thread stored the row)
#pragma unroll
        for (int k = 0; k < kD; ++k) {
            const float x = tobs[r * kD + k];
            a.tobs_out[r * kD + k] = a.norm_obs ? norm_elem(x, cn[k], clip) : x;
        }
    }
    if (done) a.returns[r] = 0.0;   // self.returns[dones] = 0
    if (a.ep_ret) {                 // Monitor: sum(rewards) of the env's f64 rewards, len(rewards)
        const double er = f.er + rew64;
        const int32_t el = f.el + 1;
        if (done) {
            a.ep_ret_done[r] = er;
            a.ep_len_done[r] = el;
        }
        a.ep_ret[r] = done ? 0.0 : er;
        a.ep_len[r] = done ? 0 : el;
    }
}

}  // namespace vn
