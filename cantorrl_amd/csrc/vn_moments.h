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
// `rew` (its row r0 + t) and its running return before the update `ret_prev`: the same
// operations on the same values as moments_body, with no global round trip.  Obs shift:
// the old running mean (a.shift_mean).
// sft: the shifts (the old running means of the obs columns and of the returns), loaded by
// the caller before its step so they are not a round trip here.
__device__ __forceinline__ void load_mean_shifts(const MomentsArgs& a, double* sft) {
#pragma unroll
    for (int c = 0; c < kD; ++c) sft[c] = a.stats[c];
    sft[kD] = a.stats[2 * kD + 1];
}
__device__ __forceinline__ void moments_from_rows(const MomentsArgs& a, int bid, const float* tile, float rew,
                                                  double ret_prev, const double* sft) {
    const int64_t r0 = (int64_t)bid * a.rows_per_block;
    const int64_t r1 = (r0 + a.rows_per_block < a.n) ? r0 + a.rows_per_block : a.n;
    const int t = threadIdx.x;
    double v[kPart - 1];
#pragma unroll
    for (int c = 0; c < kPart - 1; ++c) v[c] = 0.0;
    if (t < (int)(r1 - r0)) {
        if (a.upd_obs) {
#pragma unroll
            for (int c = 0; c < kD; ++c) {
                const double d = (double)tile[t * kD + c] - sft[c];
                v[c] += d;
                v[kD + 1 + c] += d * d;
            }
        }
        if (a.upd_ret) {
            const double ret = ret_prev * a.gamma + (double)rew;   // VecNormalize._update_reward
            a.returns[r0 + t] = ret;
            const double d = ret - sft[kD];
            v[kD] += d;
            v[2 * kD + 1] += d * d;
        }
    }
    store_partial(a, bid, v, sft, r1 > r0 ? r1 - r0 : 0);
}

}  // namespace vn
