// rbergomi.hip -- rough-Bergomi path and rolling-ATM option-mark generator for gfx950
// (librbergomi; C ABI in include/rbergomi.h).
//
// Reference: /root/reference/src/sim/rbergomi_sim.py.  The reference runs one CuPy
// pipeline per day: 196 mini-batches of [512 x 5000 x 32] complex128 arrays through
// two FFTs and a 30-step Python loop, per option type (:404-451).  Here the whole
// data set is three launches:
//   params_kernel  one thread per path: the five perturbations (:379-383)
//   paths_kernel   one workgroup per path, one thread per grid point: W from Philox,
//                  lam = t^(2H)/2, X = sqrt(2H) eta (lam (*) Re W)/sqrt(M) as an LDS
//                  circular convolution, v = xi exp(X + ma), the price increments in
//                  parallel and the price product in one lane (:385-400, :454-464)
//   mc_kernel      one workgroup per (path, day, type) option: every thread runs MC
//                  paths with W in registers and lam in SGPRs, then a workgroup sum
//                  (:261-306 for each day of :404-451)
// Why no FFT: see the header.  W = ifft(Z) sqrt(M) is i.i.d. complex normal, and
// Re ifft(fft(lam) Z) = (lam (*) Re W) / sqrt(M).  The convolution of a 32-point
// option grid is 30 x 32 FMAs per MC path with lam uniform across the workgroup.
//
// The kernels are VALU-bound (f64 exp / sqrt / pow and Philox); the inputs are a few
// scalars per option and the outputs 16 B per (path, day), so HBM is idle.

#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "../../include/rbergomi.h"
#include "he_math.h"

using he::box_muller;
using he::np_max;
using he::philox4x32_10;
using he::u01;
using he::u32x4;

namespace {

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

#define RB_HIP(call)                                                                     \
    do {                                                                                 \
        hipError_t e_ = (call);                                                          \
        if (e_ != hipSuccess) return fail(RB_EHIP, "%s: %s", #call, hipGetErrorString(e_)); \
    } while (0)

constexpr int kDomParams = 1, kDomMain = 2, kDomMc = 3;
constexpr int kMcThreads = 256;
constexpr int64_t kAtmChunk = 8192;   // rb_price_atm_marks: paths per launch
constexpr int kXc = 6;   // MC pricer: Euler steps per convolution chunk (divides the 30 of the reference tenor)

HE_HD u32x4 rb_ctr(uint32_t block, int dom, uint32_t sub, uint64_t gid) {
    return u32x4{block, ((uint32_t)dom << 24) | (sub & 0xFFFFFFu), (uint32_t)gid, (uint32_t)(gid >> 32)};
}

// Two f64 normals of one Philox block: the env's Box-Muller on 53-bit uniforms.
HE_HD void normal_pair(u32x4 c, uint32_t k0, uint32_t k1, double* a, double* b) {
    const u32x4 x = philox4x32_10(c, k0, k1);
    box_muller(u01(x.x, x.y), u01(x.z, x.w), a, b);
}

// The MC pricer's f64 normals (mc_kernel NORM 0, its hot loop: 31 Box-Muller pairs per MC
// path).  The env's box_muller (he_math.h) is pinned bit for bit to the oracle; these are
// only held to their distribution (test_pricer_philox_black_scholes_limit), so the two
// multi-instruction IEEE sequences go: s = (m - 1) / (m + 1) as (m - 1) times v_rcp_f64 with
// one Newton step (within 2.3e-15, profiles/r04s3_rcp_f64.txt), and sqrt(-2 log u) as
// x rsq(x) with one Newton-Raphson correction (u01 lies in [2^-53, 1 - 2^-53], so the argument
// -2 log u lies in [2^-52 = 2.2e-16, 73.5]: normal f64 numbers whose rsq is finite, no scaling
// or special cases; test_mc_box_muller_extreme_uniforms).  The series and the sin / cos
// polynomials are box_muller's.
__device__ __forceinline__ void mc_box_muller(double u1, double u2, double* z1, double* z2) {
    int e;
    double m = frexp(u1, &e);
    const bool lo = m < 0.70710678118654752;
    m = lo ? m + m : m;
    e = lo ? e - 1 : e;
    const double den = m + 1.0;
    double y = __builtin_amdgcn_rcp(den);
    y = fma(fma(-den, y, 1.0), y, y);
    const double s = (m - 1.0) * y;
    const double s2 = s * s;
    double p = 1.0 / 19.0;
    p = fma(p, s2, 1.0 / 17.0);
    p = fma(p, s2, 1.0 / 15.0);
    p = fma(p, s2, 1.0 / 13.0);
    p = fma(p, s2, 1.0 / 11.0);
    p = fma(p, s2, 1.0 / 9.0);
    p = fma(p, s2, 1.0 / 7.0);
    p = fma(p, s2, 1.0 / 5.0);
    p = fma(p, s2, 1.0 / 3.0);
    const double lm = (2.0 * s) + (2.0 * s) * (s2 * p);   // 2 atanh(s)
    const double ed = (double)e;
    const double lg = fma(ed, 6.93147180369123816490e-01, fma(ed, 1.90821492927058770002e-10, lm));
    const double x = -2.0 * lg;
    const double r0 = __builtin_amdgcn_rsq(x);
    const double g0 = x * r0, h0 = 0.5 * r0;
    const double rr0 = fma(-g0, h0, 0.5);
    const double rad = fma(g0, rr0, g0);
    double sn, cs;
    he::sincos_2pi_u(u2, &sn, &cs);
    *z1 = rad * cs;
    *z2 = rad * sn;
}
__device__ __forceinline__ void normal_pair_mc(u32x4 c, uint32_t k0, uint32_t k1, double* a, double* b) {
    const u32x4 x = philox4x32_10(c, k0, k1);
    mc_box_muller(u01(x.x, x.y), u01(x.z, x.w), a, b);
}

// np.clip(x, lo, hi) (NaN passes through)
HE_HD double np_clip(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }

int next_pow2(int n) {
    int p = 1;
    while (p < n) p <<= 1;
    return p;
}

// ------------------------------------------------------------------ params
struct Perturb {
    double std[5];
    double min_xi, min_eta, hlo, hhi, rlo, rhi;
};

__global__ void params_kernel(int64_t n, uint64_t off, uint32_t k0, uint32_t k1, rb_base_params b, Perturb q,
                              const double* __restrict__ unit, double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double z[6];
    if (unit) {
#pragma unroll
        for (int k = 0; k < 5; ++k) z[k] = unit[k * n + i];
    } else {
#pragma unroll
        for (int k = 0; k < 3; ++k) normal_pair(rb_ctr(k, kDomParams, 0, off + i), k0, k1, &z[2 * k], &z[2 * k + 1]);
    }
    // cp.random.normal(0.0, std, n) = 0.0 + std * z  (:379-383)
    out[i] = b.S0 * (1.0 + (0.0 + q.std[0] * z[0]));
    out[n + i] = b.xi * np_max(q.min_xi, 1.0 + (0.0 + q.std[1] * z[1]));
    out[2 * n + i] = np_clip(b.H * (1.0 + (0.0 + q.std[2] * z[2])), q.hlo, q.hhi);
    out[3 * n + i] = b.eta * np_max(q.min_eta, 1.0 + (0.0 + q.std[3] * z[3]));
    out[4 * n + i] = np_clip(b.rho * (1.0 + (0.0 + q.std[4] * z[4])), q.rlo, q.rhi);
}

// ------------------------------------------------------------------ main paths
struct PathArgs {
    int64_t n;
    uint64_t off;
    uint32_t k0, k1;
    int T, M;
    double inv_sqrt_m, r, dt, sdt, tstep, tstop;
    const double* params;
    const double* W;
    double* paths;
    double* vol;
};

// One workgroup of M threads per path; thread j owns grid point j.
__global__ void __launch_bounds__(1024) paths_kernel(PathArgs a) {
    extern __shared__ double sh[];
    double* w1 = sh;
    double* lam = sh + a.M;
    double* inc = sh + 2 * a.M;
    const int64_t p = blockIdx.x;
    const int j = threadIdx.x;
    const int T = a.T;
    const double S0 = a.params[p], xi = a.params[a.n + p], H = a.params[2 * a.n + p];
    const double eta = a.params[3 * a.n + p], rho = a.params[4 * a.n + p];
    double re, im;
    if (a.W) {
        re = a.W[(p * a.M + j) * 2];
        im = a.W[(p * a.M + j) * 2 + 1];
    } else {
        normal_pair(rb_ctr(j, kDomMain, 0, a.off + p), a.k0, a.k1, &re, &im);
    }
    // np.linspace(0, T dt, T + 1): j * step, the last point = stop (:385-386)
    const double t = (j == T) ? a.tstop : (double)j * a.tstep;
    const double pw = (j <= T) ? pow(t, 2.0 * H) : 0.0;
    w1[j] = re;
    lam[j] = (j <= T) ? 0.5 * pw : 0.0;   // rbergomi_lambda_gpu (:224-225), zero padded (:230)
    __syncthreads();
    if (j <= T) {
        double c = 0.0;
        for (int k = 0; k <= T; ++k) c = fma(lam[k], w1[(j - k) & (a.M - 1)], c);
        const double X = (sqrt(2.0 * H) * eta) * (c * a.inv_sqrt_m);        // :235-246
        const double ma = -0.5 * eta * eta * pw;                              // :254-256
        const double v = xi * exp(X + ma);
        a.vol[p * (T + 1) + j] = v;
        if (j < T) {                                                          // :454-462
            const double dW = rho * (a.sdt * re) + sqrt(np_max(0.0, 1.0 - rho * rho)) * (a.sdt * im);
            const double drift = (a.r - 0.5 * v) * a.dt;
            const double diff = sqrt(np_max(0.0, v)) * dW;
            inc[j] = exp(drift + diff);
        }
    }
    __syncthreads();
    if (j == 0) {   // S_j = max(S_{j-1} exp(.), 1e-8), in order (:463-464)
        double S = S0;
        for (int i = 0; i < T; ++i) {
            S = np_max(S * inc[i], 1e-8);
            lam[i] = S;
        }
    }
    __syncthreads();
    if (j <= T) a.paths[p * (T + 1) + j] = (j == 0) ? S0 : lam[j - 1];
}

// ------------------------------------------------------------------ MC option pricer
struct McArgs {
    int64_t n_opt;       // options (list) or paths (ATM)
    int64_t o_base;      // ATM: option index of blockIdx.x = 0 (chunked launches)
    uint64_t off;
    uint32_t k0, k1;
    int T;               // ATM: days per path
    int n;               // int(tenor / dt): Euler steps of one option
    int n_mc;
    int type;            // list mode
    double inv_sqrt_m, r, dt, sdt, tstep, tstop, disc, inv_n_mc;
    // list mode
    const double *S0, *K, *xi, *H, *eta, *rho, *W;
    double* price;
    // ATM mode
    const double *params, *paths, *vol;
    double *call, *put;
};

// Four f32-precision normals from one Philox block: uniforms ((x >> 8) + 1/2) 2^-24,
// Box-Muller with the hardware log2 / sin / cos (v_sin_f32 takes revolutions, so
// 2 pi u needs no range reduction).
__device__ __forceinline__ void normal_quad32(u32x4 c, uint32_t k0, uint32_t k1, double* z) {
    const u32x4 x = philox4x32_10(c, k0, k1);
    const float s = 5.9604644775390625e-08f;   // 2^-24
    const float u1 = ((float)(x.x >> 8) + 0.5f) * s, u2 = ((float)(x.y >> 8) + 0.5f) * s;
    const float u3 = ((float)(x.z >> 8) + 0.5f) * s, u4 = ((float)(x.w >> 8) + 0.5f) * s;
    const float m2ln2 = -1.3862943611198906f;   // -2 ln 2
    const float ra = __builtin_amdgcn_sqrtf(m2ln2 * __builtin_amdgcn_logf(u1));
    const float rb = __builtin_amdgcn_sqrtf(m2ln2 * __builtin_amdgcn_logf(u3));
    z[0] = (double)(ra * __builtin_amdgcn_cosf(u2));
    z[1] = (double)(ra * __builtin_amdgcn_sinf(u2));
    z[2] = (double)(rb * __builtin_amdgcn_cosf(u4));
    z[3] = (double)(rb * __builtin_amdgcn_sinf(u4));
}

// NORM: 0 Philox f64 normals, 1 Philox f32 normals, 2 W from memory (list mode).
// FULL: n == MO - 2 (30 steps on a 32-point grid, the reference's tenor), so the step
// guards are compile-time; otherwise n is tested per step.
template <int MO, int NORM, bool ATM, bool FULL>
__global__ void __launch_bounds__(kMcThreads) mc_kernel(McArgs a) {
    __shared__ double s_lam[MO];
    __shared__ double s_ma[MO];
    __shared__ double s_red[kMcThreads / 64];
    const int tid = threadIdx.x;
    const int64_t o = (ATM ? a.o_base : 0) + (int64_t)blockIdx.x;
    const int type = ATM ? (int)blockIdx.y : a.type;
    double S0, K, xi, H, eta, rho;
    uint64_t gid;
    uint32_t sub;
    if (ATM) {
        const int64_t p = o / a.T;
        const int d = (int)(o - p * a.T);
        S0 = a.paths[p * (a.T + 1) + d];
        xi = a.vol[p * (a.T + 1) + d];
        K = rint(S0);                       // cp.round (:409)
        H = a.params[2 * a.n_opt + p];
        eta = a.params[3 * a.n_opt + p];
        rho = a.params[4 * a.n_opt + p];
        gid = a.off + (uint64_t)p;
        sub = (uint32_t)(d * 2 + type);
    } else {
        S0 = a.S0[o];
        K = a.K[o];
        xi = a.xi[o];
        H = a.H[o];
        eta = a.eta[o];
        rho = a.rho[o];
        gid = a.off + (uint64_t)o;
        sub = (uint32_t)type;
    }
    double* out = ATM ? ((type == RB_CALL) ? a.call : a.put) : a.price;
    const int64_t oi = o;   // ATM: call / put [p][T] at o = p T + d
    if (a.n <= 0) {                     // :266-272
        if (tid == 0) {
            const double pay = (type == RB_CALL) ? np_max(S0 - K, 0.0) : np_max(K - S0, 0.0);
            out[oi] = pay * a.disc;
        }
        return;
    }
    // lam_k = t_k^(2H) / 2 and ma_k = -eta^2 t_k^(2H) / 2 on the option grid (:274-278, :254)
    if (tid < MO) {
        const int k = tid;
        const double t = (k == a.n) ? a.tstop : (double)k * a.tstep;
        const double pw = (k <= a.n) ? pow(t, 2.0 * H) : 0.0;
        s_lam[k] = (k <= a.n) ? 0.5 * pw : 0.0;
        s_ma[k] = -0.5 * eta * eta * pw;
    }
    __syncthreads();
    const double cx = sqrt(2.0 * H) * eta;
    const double rq = sqrt(np_max(0.0, 1.0 - rho * rho));
    const double sxi = sqrt(np_max(0.0, xi));
    // The price chain in log space: S_j = max(S_{j-1} e^a, 1e-8) is S0 e^L with
    // L_j = max(L_{j-1} + a, log(1e-8 / S0)) -- one exp per path instead of one per
    // step.  S0 <= 0 makes S_1 = 1e-8 whatever a is: restart from 1e-8 with L_1 = 0.
    // (A NaN S0 keeps s0_pos, so Lf and every L are NaN, as the reference's S.)
    const bool s0_pos = !(S0 <= 0.0);
    const double Sb = s0_pos ? S0 : 1e-8;
    const double Lf = s0_pos ? log(1e-8) - log(S0) : 0.0;
    double acc = 0.0;
    for (int m = tid; m < a.n_mc; m += kMcThreads) {
        // keep the lam / ma reads (LDS broadcasts) inside the loop: hoisted, they would
        // pin 2 (MO - 1) more VGPR pairs for the whole loop
        __asm__ volatile("" ::: "memory");
        // Re W in registers (every X_j reads all of it); Im W is drawn as the steps
        // consume it.  f64 normals: blocks [0, MO/2) give Re W pairs, [MO/2, MO) Im W
        // pairs; f32 normals: [0, MO/4) Re W quads, [MO/4, MO/2) Im W quads.
        double w1[MO];
        const double* wp = (NORM == 2) ? a.W + ((o * a.n_mc + m) * (int64_t)MO) * 2 : nullptr;
        if (NORM == 2) {
#pragma unroll
            for (int b = 0; b < MO; ++b) w1[b] = wp[2 * b];
        } else if (NORM == 0) {
#pragma unroll
            for (int b = 0; b < MO / 2; ++b) {
                __builtin_amdgcn_sched_barrier(0);
                normal_pair_mc(rb_ctr((uint32_t)(m * MO + b), kDomMc, sub, gid), a.k0, a.k1, &w1[2 * b], &w1[2 * b + 1]);
            }
        } else {
#pragma unroll
            for (int b = 0; b < MO / 4; ++b) {
                __builtin_amdgcn_sched_barrier(0);
                normal_quad32(rb_ctr((uint32_t)(m * (MO / 2) + b), kDomMc, sub, gid), a.k0, a.k1, &w1[4 * b]);
            }
        }
        // The steps in chunks of kXc: X_j = sum_k lam_k Re W_{(j - k) mod MO} for the
        // chunk's j, k outer (lam_k one LDS broadcast feeding kXc FMAs), then the chunk's
        // Euler steps.  Only kXc accumulators live beside Re W: 4 waves per SIMD.
        double L = 0.0;
        double w2q[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int j0 = 0; j0 < MO - 1; j0 += kXc) {
            if (FULL ? (j0 < MO - 2) : (j0 < a.n)) {
                __asm__ volatile("" ::: "memory");   // re-read lam per chunk (no CSE across chunks)
                __builtin_amdgcn_sched_barrier(0);   // and no interleaving of chunks: w1 + one chunk live
                double X[kXc];
#pragma unroll
                for (int q = 0; q < kXc; ++q) X[q] = 0.0;
#pragma unroll
                for (int k = 0; k < MO; ++k) {
                    const double lk = s_lam[k];
#pragma unroll
                    for (int q = 0; q < kXc; ++q) X[q] = fma(lk, w1[(j0 + q - k) & (MO - 1)], X[q]);
                }
#pragma unroll
                for (int q = 0; q < kXc; ++q) {   // Euler step j + 1 uses X_j, v_j, W_j (:285-295)
                    const int j = j0 + q;
                    if (FULL ? (j < MO - 2) : (j < MO - 1 && j < a.n)) {
                        double w2;
                        if (NORM == 2) {
                            w2 = wp[2 * j + 1];
                        } else if (NORM == 0) {
                            if ((j & 1) == 0)
                                normal_pair_mc(rb_ctr((uint32_t)(m * MO + MO / 2 + j / 2), kDomMc, sub, gid), a.k0,
                                            a.k1, &w2q[0], &w2q[1]);
                            w2 = w2q[j & 1];
                        } else {
                            if ((j & 3) == 0)
                                normal_quad32(rb_ctr((uint32_t)(m * (MO / 2) + MO / 4 + j / 4), kDomMc, sub, gid),
                                              a.k0, a.k1, w2q);
                            w2 = w2q[j & 3];
                        }
                        const double Xj = cx * (X[q] * a.inv_sqrt_m);
                        // v = xi e^(X + ma) and sqrt(v) = sqrt(xi) e^((X + ma) / 2): one exp
                        const double e = exp(0.5 * (Xj + s_ma[j]));
                        const double v = xi * (e * e);
                        const double dW = rho * (a.sdt * w1[j]) + rq * (a.sdt * w2);
                        const double drift = (a.r - 0.5 * v) * a.dt;
                        const double diff = (sxi * e) * dW;
                        L = np_max(L + (drift + diff), Lf);
                        if (j == 0 && !s0_pos) L = 0.0;
                    }
                }
            }
        }
        const double S = Sb * exp(L);
        acc += (type == RB_CALL) ? np_max(S - K, 0.0) : np_max(K - S, 0.0);   // :299-303
    }
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) acc += __shfl_xor(acc, s, 64);
    if ((tid & 63) == 0) s_red[tid >> 6] = acc;
    __syncthreads();
    if (tid == 0) {
        double sum = 0.0;
#pragma unroll
        for (int w = 0; w < kMcThreads / 64; ++w) sum += s_red[w];
        out[oi] = (sum / (double)a.n_mc) * a.disc;   // mean(payoff) exp(-r T) (:305)
    }
}

// ------------------------------------------------------------------ MC pricer, matrix cores
// mc_kernel's work for the reference tenor (30 Euler steps on the 32-point grid, MO = 32, FULL)
// with the fractional convolution on the f64 matrix pipe: for 16 MC paths at
// a time, X = T W with T[j][i] = lam_{(j - i) mod 32} the circulant of lam (a 32 x 32 constant of
// the option) and W = Re W of the 16 paths (32 x 16), as 2 row tiles x 8 k-steps of
// v_mfma_f64_16x16x4_f64 -- 960 f64 FMAs per MC path off the VALU, which keeps Philox, Box-Muller
// and the Euler steps.
//
// Layouts (v_mfma_f64_16x16x4_f64: lane l holds A[row l & 15][k l >> 4], B[k l >> 4][col l & 15],
// D[row (l >> 4) + 4 r][col l & 15], r = 0..3).  With g = l >> 4 and c = l & 15, lane l works on
// MC path base + c, and the rows and k of T are permuted so that every lane's operands and results
// are ITS OWN path's: k-step s, k = g <-> i = 8 g + s, and D row g + 4 r of row tile t <-> j =
// 8 g + 4 t + r.  So lane (g, c) draws Re W[8g .. 8g + 7] and Im W[8g .. 8g + 7] of path base + c
// (the same Philox blocks as mc_kernel: the same normals), feeds them as B, and receives X[8g ..
// 8g + 7]: the A fragment of (t, s) is lam[(8 (c & 3) + 4 t + (c >> 2) - 8 g - s) & 31], held in
// registers for the whole option.  No LDS, no transposes.
//
// The Euler chain L_{j+1} = max(L_j + a_j, Lf) of mc_kernel is then split over the 4 lanes of a
// path: each lane computes a_j of its 8 steps (their exp, drift, diffusion) and composes its 8
// steps into one map L -> max(L + s, b) (s = sum a, b = max(b + a, Lf), exact in real
// arithmetic: max distributes over +); the 4 maps, fetched by __shfl, are applied in order.  The
// sums' order is not mc_kernel's, so a mark moves by ~1e-16 relative: the reference-draw parity
// (tests/test_rbergomi_gpu.py, 1e-10) runs through this kernel.
typedef double v4d __attribute__((ext_vector_type(4)));

template <int NORM, bool ATM>
__global__ void __launch_bounds__(kMcThreads) mc_mfma_kernel(McArgs a) {
    constexpr int MO = 32;
    __shared__ double s_lam[MO];
    __shared__ double s_ma[MO];
    __shared__ double s_red[kMcThreads / 64];
    const int tid = threadIdx.x;
    const int64_t o = (ATM ? a.o_base : 0) + (int64_t)blockIdx.x;
    const int type = ATM ? (int)blockIdx.y : a.type;
    double S0, K, xi, H, eta, rho;
    uint64_t gid;
    uint32_t sub;
    if (ATM) {
        const int64_t p = o / a.T;
        const int d = (int)(o - p * a.T);
        S0 = a.paths[p * (a.T + 1) + d];
        xi = a.vol[p * (a.T + 1) + d];
        K = rint(S0);                       // cp.round (:409)
        H = a.params[2 * a.n_opt + p];
        eta = a.params[3 * a.n_opt + p];
        rho = a.params[4 * a.n_opt + p];
        gid = a.off + (uint64_t)p;
        sub = (uint32_t)(d * 2 + type);
    } else {
        S0 = a.S0[o];
        K = a.K[o];
        xi = a.xi[o];
        H = a.H[o];
        eta = a.eta[o];
        rho = a.rho[o];
        gid = a.off + (uint64_t)o;
        sub = (uint32_t)type;
    }
    double* out = ATM ? ((type == RB_CALL) ? a.call : a.put) : a.price;
    if (tid < MO) {   // lam_k and ma_k on the option grid (:274-278, :254), as mc_kernel
        const int k = tid;
        const double t = (k == a.n) ? a.tstop : (double)k * a.tstep;
        const double pw = (k <= a.n) ? pow(t, 2.0 * H) : 0.0;
        s_lam[k] = (k <= a.n) ? 0.5 * pw : 0.0;
        s_ma[k] = -0.5 * eta * eta * pw;
    }
    __syncthreads();
    const int lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, c = lane & 15;
    double A[2][8];   // the permuted circulant's fragments (see above)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int q = 0; q < 8; ++q) A[t][q] = s_lam[(8 * (c & 3) + 4 * t + (c >> 2) - 8 * g - q) & 31];
    double ma[8];     // ma_j of this lane's steps j = 8 g + q
#pragma unroll
    for (int q = 0; q < 8; ++q) ma[q] = s_ma[8 * g + q];
    const double cx = sqrt(2.0 * H) * eta;
    const double rq = sqrt(np_max(0.0, 1.0 - rho * rho));
    const double sxi = sqrt(np_max(0.0, xi));
    const bool s0_pos = !(S0 <= 0.0);
    const double Sb = s0_pos ? S0 : 1e-8;
    const double Lf = s0_pos ? log(1e-8) - log(S0) : 0.0;
    const double ninf = -__builtin_inf();
    double acc = 0.0;
    // every wave takes 16 paths per iteration: [base, base + 16), base = 16 wave + 64 k
    for (int base = 16 * wave; base < a.n_mc; base += 4 * 16) {
        const int m = base + c;
        const bool live = m < a.n_mc;
        double w1[8], w2[8];   // Re W, Im W at i = j = 8 g + q
        const double* wp = (NORM == 2 && live) ? a.W + ((o * a.n_mc + m) * (int64_t)MO) * 2 : nullptr;
        if (NORM == 2) {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                w1[q] = live ? wp[2 * (8 * g + q)] : 0.0;
                w2[q] = live ? wp[2 * (8 * g + q) + 1] : 0.0;
            }
        } else if (NORM == 0) {   // mc_kernel's blocks: Re pairs b = 4g .. 4g + 3, Im pairs 16 + 4g ..
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                __builtin_amdgcn_sched_barrier(0);
                normal_pair_mc(rb_ctr((uint32_t)(m * MO + 4 * g + b), kDomMc, sub, gid), a.k0, a.k1, &w1[2 * b],
                               &w1[2 * b + 1]);
            }
        } else {                  // Re quads 2g, 2g + 1; Im quads 8 + 2g, 9 + 2g
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                __builtin_amdgcn_sched_barrier(0);
                normal_quad32(rb_ctr((uint32_t)(m * (MO / 2) + 2 * g + b), kDomMc, sub, gid), a.k0, a.k1, &w1[4 * b]);
            }
        }
        if (NORM != 2 && !live) {
#pragma unroll
            for (int q = 0; q < 8; ++q) w1[q] = 0.0;
        }
        // X[8g + 4t + r] of path m: 16 MFMAs
        v4d X0 = {0.0, 0.0, 0.0, 0.0}, X1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            X0 = __builtin_amdgcn_mfma_f64_16x16x4f64(A[0][q], w1[q], X0, 0, 0, 0);
            X1 = __builtin_amdgcn_mfma_f64_16x16x4f64(A[1][q], w1[q], X1, 0, 0, 0);
        }
        if (NORM == 0) {   // Im W while the matrix pipe works
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                __builtin_amdgcn_sched_barrier(0);
                normal_pair_mc(rb_ctr((uint32_t)(m * MO + MO / 2 + 4 * g + b), kDomMc, sub, gid), a.k0, a.k1,
                               &w2[2 * b], &w2[2 * b + 1]);
            }
        } else if (NORM == 1) {
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                __builtin_amdgcn_sched_barrier(0);
                normal_quad32(rb_ctr((uint32_t)(m * (MO / 2) + MO / 4 + 2 * g + b), kDomMc, sub, gid), a.k0, a.k1,
                              &w2[4 * b]);
            }
        }
        // this lane's 8 Euler steps composed: L -> max(L + cs, cb)
        double cs = 0.0, cb = ninf;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int j = 8 * g + q;
            const double Xq = (q < 4) ? X0[q] : X1[q - 4];
            const double Xj = cx * (Xq * a.inv_sqrt_m);
            const double e = exp(0.5 * (Xj + ma[q]));
            const double v = xi * (e * e);
            const double dW = rho * (a.sdt * w1[q]) + rq * (a.sdt * w2[q]);
            const double drift = (a.r - 0.5 * v) * a.dt;
            const double diff = (sxi * e) * dW;
            const double st = drift + diff;
            const bool step = j < MO - 2;           // steps 0 .. 29; rows 30, 31 unused
            double ns = cs + st, nb = np_max(cb + st, Lf);
            if (j == 0 && !s0_pos) {                // S0 <= 0: S_1 = 1e-8 whatever a_0 (L_1 = 0)
                ns = ninf;
                nb = 0.0;
            }
            cs = step ? ns : cs;
            cb = step ? nb : cb;
        }
        // the path's 4 maps in step order
        double L = 0.0;
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const double sh = __shfl(cs, c + 16 * h, 64), bh = __shfl(cb, c + 16 * h, 64);
            L = np_max(L + sh, bh);
        }
        const double S = Sb * exp(L);
        const double pay = (type == RB_CALL) ? np_max(S - K, 0.0) : np_max(K - S, 0.0);   // :299-303
        acc += (g == 0 && live) ? pay : 0.0;
    }
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) acc += __shfl_xor(acc, s, 64);
    if ((tid & 63) == 0) s_red[tid >> 6] = acc;
    __syncthreads();
    if (tid == 0) {
        double sum = 0.0;
#pragma unroll
        for (int w = 0; w < kMcThreads / 64; ++w) sum += s_red[w];
        out[o] = (sum / (double)a.n_mc) * a.disc;   // mean(payoff) exp(-r T) (:305)
    }
}

// RB_MC_MFMA=1 (read per launch): the reference tenor through mc_mfma_kernel.  Not the default:
// measured slower than mc_kernel on MI355X (f64 normals 9.75e5 vs 1.02e6 options/s, f32
// 1.74e6 vs 2.02e6, profiles/r06m_rb_ab.txt) -- the f64 matrix pipe does the 960 FMAs per MC
// path at the vector rate, and splitting each path's Euler chain over 4 lanes (the 4 maps,
// the 8 shuffles, a final exp per lane, the NaN-safe max) costs more VALU issue than the
// convolution it takes off (2301 VALU instructions per lane per 16-path tile against 1884 for a
// quarter MC path of mc_kernel).  Kept as the tested alternative (test_mfma_pricer_equals_valu_pricer).
bool mc_mfma_enabled() {
    const char* e = getenv("RB_MC_MFMA");
    return e && e[0] == '1';
}

void launch_mc_mfma(const McArgs& a, int norm, bool atm, dim3 grid, hipStream_t s) {
    if (atm) {
        if (norm == RB_NORMALS_F32) hipLaunchKernelGGL((mc_mfma_kernel<1, true>), grid, dim3(kMcThreads), 0, s, a);
        else hipLaunchKernelGGL((mc_mfma_kernel<0, true>), grid, dim3(kMcThreads), 0, s, a);
    } else {
        if (a.W) hipLaunchKernelGGL((mc_mfma_kernel<2, false>), grid, dim3(kMcThreads), 0, s, a);
        else if (norm == RB_NORMALS_F32)
            hipLaunchKernelGGL((mc_mfma_kernel<1, false>), grid, dim3(kMcThreads), 0, s, a);
        else hipLaunchKernelGGL((mc_mfma_kernel<0, false>), grid, dim3(kMcThreads), 0, s, a);
    }
}

// ------------------------------------------------------------------ host helpers
int check_cfg(const rb_config* c) {
    if (!c) return fail(RB_EINVAL, "config is NULL");
    if (c->abi_version != RB_ABI_VERSION)
        return fail(RB_EINVAL, "abi_version %d != %d", c->abi_version, RB_ABI_VERSION);
    if (c->n_steps < 1 || c->n_steps > 1023) return fail(RB_EINVAL, "n_steps %d not in [1, 1023]", c->n_steps);
    if (c->n_paths < 0) return fail(RB_EINVAL, "n_paths < 0");
    if (c->path_offset < 0) return fail(RB_EINVAL, "path_offset < 0");
    if (!(c->dt > 0.0) || !isfinite(c->dt)) return fail(RB_EINVAL, "dt must be > 0");
    if (!isfinite(c->r)) return fail(RB_EINVAL, "r must be finite");
    if (!(c->option_tenor >= 0.0) || !isfinite(c->option_tenor)) return fail(RB_EINVAL, "option_tenor must be >= 0");
    if (c->n_mc < 1) return fail(RB_EINVAL, "n_mc must be >= 1");
    if (c->normals != RB_NORMALS_F64 && c->normals != RB_NORMALS_F32)
        return fail(RB_EINVAL, "normals %d unknown", c->normals);
    const double q = c->option_tenor / c->dt;
    if (q >= 64.0) return fail(RB_EINVAL, "int(option_tenor / dt) = %.0f: at most 63 steps per option", q);
    return RB_OK;
}

// Python int(T / dt) and the option grid of :273-274
struct OptGrid {
    int n, M;
    double tstep, tstop, inv_sqrt_m, disc;
};

OptGrid opt_grid(const rb_config* c) {
    OptGrid g;
    g.n = (int)(c->option_tenor / c->dt);
    g.M = next_pow2(g.n + 1);
    if (g.M < 2) g.M = 2;
    g.tstop = (double)g.n * c->dt;
    g.tstep = (g.n > 0) ? g.tstop / (double)g.n : 0.0;
    g.inv_sqrt_m = 1.0 / sqrt((double)next_pow2(g.n + 1));
    g.disc = exp(-c->r * c->option_tenor);
    return g;
}

McArgs mc_args(const rb_config* c, const OptGrid& g) {
    McArgs a;
    memset(&a, 0, sizeof(a));
    a.off = (uint64_t)c->path_offset;
    a.k0 = (uint32_t)c->seed;
    a.k1 = (uint32_t)(c->seed >> 32);
    a.T = c->n_steps;
    a.n = g.n;
    a.n_mc = c->n_mc;
    a.inv_sqrt_m = g.inv_sqrt_m;
    a.r = c->r;
    a.dt = c->dt;
    a.sdt = sqrt(c->dt);
    a.tstep = g.tstep;
    a.tstop = g.tstop;
    a.disc = g.disc;
    a.inv_n_mc = 1.0 / (double)c->n_mc;
    return a;
}

template <int MO, bool FULL>
void launch_mc_v(const McArgs& a, int norm, bool atm, dim3 grid, hipStream_t s) {
    if (atm) {
        if (norm == RB_NORMALS_F32) hipLaunchKernelGGL((mc_kernel<MO, 1, true, FULL>), grid, dim3(kMcThreads), 0, s, a);
        else hipLaunchKernelGGL((mc_kernel<MO, 0, true, FULL>), grid, dim3(kMcThreads), 0, s, a);
    } else {
        if (a.W) hipLaunchKernelGGL((mc_kernel<MO, 2, false, FULL>), grid, dim3(kMcThreads), 0, s, a);
        else if (norm == RB_NORMALS_F32)
            hipLaunchKernelGGL((mc_kernel<MO, 1, false, FULL>), grid, dim3(kMcThreads), 0, s, a);
        else hipLaunchKernelGGL((mc_kernel<MO, 0, false, FULL>), grid, dim3(kMcThreads), 0, s, a);
    }
}

template <int MO>
int launch_mc_mo(const McArgs& a, int norm, bool atm, dim3 grid, hipStream_t s) {
    if (MO == 32 && a.n == MO - 2) {
        if (mc_mfma_enabled()) launch_mc_mfma(a, norm, atm, grid, s);
        else launch_mc_v<MO, true>(a, norm, atm, grid, s);
    } else {
        launch_mc_v<MO, false>(a, norm, atm, grid, s);
    }
    RB_HIP(hipGetLastError());
    return RB_OK;
}

int launch_mc(const McArgs& a, int M, int norm, bool atm, dim3 grid, hipStream_t s) {
    switch (M) {
        case 2: return launch_mc_mo<2>(a, norm, atm, grid, s);
        case 4: return launch_mc_mo<4>(a, norm, atm, grid, s);
        case 8: return launch_mc_mo<8>(a, norm, atm, grid, s);
        case 16: return launch_mc_mo<16>(a, norm, atm, grid, s);
        case 32: return launch_mc_mo<32>(a, norm, atm, grid, s);
        case 64: return launch_mc_mo<64>(a, norm, atm, grid, s);
        default: return fail(RB_EINVAL, "option grid of %d points unsupported", M);
    }
}

// ------------------------------------------------------------------ host estimator
// numpy's pairwise summation (umath loops_utils: blocks of 128, 8 accumulators) so
// that np.sum / np.mean are followed as closely as the host allows.
double pairwise_sum(const double* a, int64_t n) {
    if (n < 8) {
        double res = 0.0;
        for (int64_t i = 0; i < n; ++i) res += a[i];
        return res;
    }
    if (n <= 128) {
        double r[8];
        for (int k = 0; k < 8; ++k) r[k] = a[k];
        int64_t i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int k = 0; k < 8; ++k) r[k] += a[i + k];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return pairwise_sum(a, n2) + pairwise_sum(a + n2, n - n2);
}

double np_sum(const std::vector<double>& v) { return pairwise_sum(v.data(), (int64_t)v.size()); }
double np_mean(const std::vector<double>& v) { return np_sum(v) / (double)v.size(); }

// np.var(v, ddof=1): mean, deviations squared, sum / (n - 1)   (:47-50 for n >= 2)
double np_var1(const std::vector<double>& v) {
    if (v.size() < 2) return 0.0;
    const double m = np_mean(v);
    std::vector<double> d(v.size());
    for (size_t i = 0; i < v.size(); ++i) {
        const double x = v[i] - m;
        d[i] = x * x;
    }
    return np_sum(d) / (double)(v.size() - 1);
}

std::vector<double> log_returns(const double* p, int64_t n) {   // :57-61
    std::vector<double> r;
    if (n < 2) return r;
    r.resize(n - 1);
    for (int64_t i = 0; i + 1 < n; ++i) r[i] = log(p[i + 1] / p[i]);
    return r;
}

const double XI_DEFAULT = 0.04, H_DEFAULT = 0.1, ETA_DEFAULT = 1.0, RHO_DEFAULT = -0.7, S0_DEFAULT = 100.0;

std::vector<double> detrend(const std::vector<double>& seg) {   // :67-80
    const size_t n = seg.size();
    if (n < 2) return seg;
    std::vector<double> t(n), a(n), b(n);
    for (size_t i = 0; i < n; ++i) t[i] = (double)(i + 1);
    const double tm = np_mean(t), ym = np_mean(seg);
    for (size_t i = 0; i < n; ++i) {
        a[i] = (t[i] - tm) * (seg[i] - ym);
        b[i] = (t[i] - tm) * (t[i] - tm);
    }
    const double num = np_sum(a), den = np_sum(b);
    if (fabs(den) < 1e-14) return seg;
    const double slope = num / den;
    const double icpt = ym - slope * tm;
    std::vector<double> out(n);
    for (size_t i = 0; i < n; ++i) out[i] = seg[i] - (slope * t[i] + icpt);
    return out;
}

double hurst_dfa(const std::vector<double>& x) {   // :82-130
    if (x.size() < 20) return H_DEFAULT;
    const double mu = np_mean(x);
    std::vector<double> data(x.size());
    double c = 0.0;
    for (size_t i = 0; i < x.size(); ++i) {
        c += x[i] - mu;   // np.cumsum of (data - mean), sequential
        data[i] = c;
    }
    std::vector<double> lw, lf;
    const int64_t wmin = 10, wmax = (int64_t)data.size() / 4;
    if (wmax < wmin) return H_DEFAULT;
    int64_t w = wmin;
    while (w <= wmax) {
        std::vector<double> fl;
        for (int64_t s = 0; s + w <= (int64_t)data.size(); s += w) {
            std::vector<double> seg(data.begin() + s, data.begin() + s + w);
            std::vector<double> d = detrend(seg);
            for (auto& e : d) e = e * e;
            const double rms = sqrt(np_mean(d));
            if (rms > 1e-8) fl.push_back(rms);
        }
        if (!fl.empty()) {
            const double mf = np_mean(fl);
            if (mf > 1e-8) {
                lw.push_back(log((double)w));
                lf.push_back(log(mf));
            }
        }
        if (w == wmax) break;
        if (w * 2 > wmax && w < wmax) w = wmax;
        else w *= 2;
    }
    const size_t n = lw.size();
    if (n < 2) return H_DEFAULT;
    std::vector<double> xx(n), xy(n);
    for (size_t i = 0; i < n; ++i) {
        xx[i] = lw[i] * lw[i];
        xy[i] = lw[i] * lf[i];
    }
    const double sx = np_sum(lw), sy = np_sum(lf), sxx = np_sum(xx), sxy = np_sum(xy);
    const double den = (double)n * sxx - sx * sx;
    if (fabs(den) < 1e-14) return H_DEFAULT;
    return np_clip(((double)n * sxy - sx * sy) / den, 0.01, 0.49);
}

double estimate_eta(const std::vector<double>& r, int window = 20) {   // :135-153
    if ((int64_t)r.size() < window + 1) return ETA_DEFAULT;
    std::vector<double> lrv;
    for (size_t i = window - 1; i < r.size(); ++i) {
        std::vector<double> sq(window);
        for (int k = 0; k < window; ++k) sq[k] = r[i - window + 1 + k] * r[i - window + 1 + k];
        lrv.push_back(log(np_mean(sq)));
    }
    if (lrv.size() < 2) return ETA_DEFAULT;
    std::vector<double> d(lrv.size() - 1);
    for (size_t i = 0; i + 1 < lrv.size(); ++i) d[i] = lrv[i + 1] - lrv[i];
    if (d.size() < 2) return ETA_DEFAULT;
    return sqrt(np_var1(d)) * sqrt(252.0);
}

double estimate_rho(const std::vector<double>& r) {   // :155-171
    if (r.size() < 2) return RHO_DEFAULT;
    const size_t n = r.size();
    std::vector<double> sq(n);
    for (size_t i = 0; i < n; ++i) sq[i] = r[i] * r[i];
    // np.cov(r, sq, ddof=1)[0, 1]: centred rows, dot product / (n - 1)
    const double mr = np_mean(r), ms = np_mean(sq);
    std::vector<double> pr(n);
    for (size_t i = 0; i < n; ++i) pr[i] = (r[i] - mr) * (sq[i] - ms);
    const double c = np_sum(pr) / (double)(n - 1);
    const double vr = np_var1(r), vs = np_var1(sq);
    if (vr == 0.0 || vs == 0.0) return RHO_DEFAULT;
    const double den = sqrt(vr * vs);
    double rho = (den != 0.0) ? c / den : 0.0;
    if (rho > 0.0) rho = -0.3;
    return np_clip(rho, -0.99, -0.01);
}

}  // namespace

// ================================================================== C ABI
// Test hook: mc_box_muller on caller-given uniforms (rb_device_mc_box_muller).
__global__ void mc_box_muller_kernel(const double* u1, const double* u2, int64_t n, double* z1, double* z2) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    double a, b;
    mc_box_muller(u1[i], u2[i], &a, &b);
    z1[i] = a;
    z2[i] = b;
}

extern "C" {

const char* rb_version(void) { return "librbergomi 0.1 (gfx950)"; }
const char* rb_last_error(void) { return g_err; }

int32_t rb_config_init(rb_config* c, int32_t abi_version) {
    if (!c) return fail(RB_EINVAL, "config is NULL");
    if (abi_version != RB_ABI_VERSION) return fail(RB_EINVAL, "abi_version %d != %d", abi_version, RB_ABI_VERSION);
    memset(c, 0, sizeof(*c));
    c->abi_version = RB_ABI_VERSION;
    c->n_steps = 252;
    c->n_paths = 100000;
    c->path_offset = 0;
    c->seed = 42;
    c->r = 0.04;
    c->dt = 1.0 / 252.0;
    c->option_tenor = 30.0 / 252.0;
    c->n_mc = 5000;
    c->normals = RB_NORMALS_F64;
    const double std[5] = {0.01, 0.20, 0.20, 0.20, 0.10};
    memcpy(c->perturb_std, std, sizeof(std));
    c->min_xi_factor = 0.5;
    c->min_eta_factor = 0.5;
    c->clip_h_min = 0.01;
    c->clip_h_max = 0.49;
    c->clip_rho_min = -0.99;
    c->clip_rho_max = -0.01;
    return RB_OK;
}

int32_t rb_estimate_parts(const double* prices, int64_t n, double dt, double out[4]) {
    if ((!prices && n > 0) || n < 0 || !out) return fail(RB_EINVAL, "bad arguments");
    const std::vector<double> r = log_returns(prices, n);
    out[0] = np_var1(r) / dt;
    out[1] = hurst_dfa(r);
    out[2] = estimate_eta(r);
    out[3] = estimate_rho(r);
    return RB_OK;
}

int32_t rb_estimate_base_params(const double* prices, int64_t n, double dt, rb_base_params* o) {
    if ((!prices && n > 0) || n < 0 || !o) return fail(RB_EINVAL, "bad arguments");
    if (n < 21) {   // :175-177
        *o = rb_base_params{n > 0 ? prices[n - 1] : S0_DEFAULT, XI_DEFAULT, H_DEFAULT, ETA_DEFAULT, RHO_DEFAULT};
        return RB_OK;
    }
    double p[4];
    rb_estimate_parts(prices, n, dt, p);
    o->S0 = prices[n - 1];
    o->xi = (!isfinite(p[0]) || p[0] <= 1e-6) ? XI_DEFAULT : p[0];
    o->H = !isfinite(p[1]) ? H_DEFAULT : p[1];
    o->eta = (!isfinite(p[2]) || p[2] <= 1e-6) ? ETA_DEFAULT : p[2];
    o->rho = !isfinite(p[3]) ? RHO_DEFAULT : p[3];
    return RB_OK;
}

int32_t rb_sample_params(const rb_config* c, const rb_base_params* b, const double* unit, double* params,
                         void* stream) {
    if (int e = check_cfg(c)) return e;
    if (!b || (!params && c->n_paths > 0)) return fail(RB_EINVAL, "base / params is NULL");
    if (c->n_paths == 0) return RB_OK;
    Perturb q;
    memcpy(q.std, c->perturb_std, sizeof(q.std));
    q.min_xi = c->min_xi_factor;
    q.min_eta = c->min_eta_factor;
    q.hlo = c->clip_h_min;
    q.hhi = c->clip_h_max;
    q.rlo = c->clip_rho_min;
    q.rhi = c->clip_rho_max;
    const int64_t n = c->n_paths;
    hipLaunchKernelGGL(params_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n,
                       (uint64_t)c->path_offset, (uint32_t)c->seed, (uint32_t)(c->seed >> 32), *b, q, unit, params);
    RB_HIP(hipGetLastError());
    return RB_OK;
}

int32_t rb_simulate_paths(const rb_config* c, const double* params, const double* W, double* paths, double* vol,
                          void* stream) {
    if (int e = check_cfg(c)) return e;
    if (c->n_paths == 0) return RB_OK;
    if (!params || !paths || !vol) return fail(RB_EINVAL, "params / paths / vol is NULL");
    PathArgs a;
    a.n = c->n_paths;
    a.off = (uint64_t)c->path_offset;
    a.k0 = (uint32_t)c->seed;
    a.k1 = (uint32_t)(c->seed >> 32);
    a.T = c->n_steps;
    a.M = next_pow2(c->n_steps + 1);
    a.inv_sqrt_m = 1.0 / sqrt((double)a.M);
    a.r = c->r;
    a.dt = c->dt;
    a.sdt = sqrt(c->dt);
    a.tstop = (double)c->n_steps * c->dt;             // np.linspace(0, N_STEPS * dt, N_STEPS + 1)
    a.tstep = a.tstop / (double)c->n_steps;
    a.params = params;
    a.W = W;
    a.paths = paths;
    a.vol = vol;
    const size_t lds = 3 * (size_t)a.M * sizeof(double);
    if (a.n > 0x7FFFFFFF) return fail(RB_EINVAL, "n_paths > 2^31 - 1 in one call");
    hipLaunchKernelGGL(paths_kernel, dim3((unsigned)a.n), dim3(a.M), lds, (hipStream_t)stream, a);
    RB_HIP(hipGetLastError());
    return RB_OK;
}

int32_t rb_price_options(const rb_config* c, int64_t n_opt, int32_t type, const double* S0, const double* K,
                         const double* xi, const double* H, const double* eta, const double* rho, const double* W,
                         double* price, void* stream) {
    if (int e = check_cfg(c)) return e;
    if (type != RB_CALL && type != RB_PUT) return fail(RB_EINVAL, "type %d unknown", type);
    if (n_opt < 0 || n_opt > 0x7FFFFFFF) return fail(RB_EINVAL, "n_options %lld out of range", (long long)n_opt);
    if (n_opt == 0) return RB_OK;
    if (!S0 || !K || !xi || !H || !eta || !rho || !price) return fail(RB_EINVAL, "an option array is NULL");
    const OptGrid g = opt_grid(c);
    McArgs a = mc_args(c, g);
    a.n_opt = n_opt;
    a.type = type;
    a.S0 = S0;
    a.K = K;
    a.xi = xi;
    a.H = H;
    a.eta = eta;
    a.rho = rho;
    a.W = W;
    a.price = price;
    return launch_mc(a, g.M, c->normals, false, dim3((unsigned)n_opt), (hipStream_t)stream);
}

int32_t rb_price_atm_marks(const rb_config* c, const double* params, const double* paths, const double* vol,
                           double* call, double* put, void* stream) {
    if (int e = check_cfg(c)) return e;
    if (c->n_paths == 0) return RB_OK;
    if (!params || !paths || !vol || !call || !put) return fail(RB_EINVAL, "an array is NULL");
    const OptGrid g = opt_grid(c);
    McArgs a = mc_args(c, g);
    a.n_opt = c->n_paths;
    a.params = params;
    a.paths = paths;
    a.vol = vol;
    a.call = call;
    a.put = put;
    // launches of kAtmChunk paths (x n_steps days x {call, put}): a few seconds each
    // at 5000 MC paths, and grids far below the 2^31 workgroup limit at any n_paths
    for (int64_t p0 = 0; p0 < c->n_paths; p0 += kAtmChunk) {
        const int64_t np = (c->n_paths - p0 < kAtmChunk) ? c->n_paths - p0 : kAtmChunk;
        a.o_base = p0 * (int64_t)c->n_steps;
        if (int e = launch_mc(a, g.M, c->normals, true, dim3((unsigned)(np * c->n_steps), 2), (hipStream_t)stream))
            return e;
    }
    return RB_OK;
}

int32_t rb_generate(const rb_config* c, const rb_base_params* b, double* params, double* paths, double* vol,
                    double* call, double* put, void* stream) {
    if (int e = rb_sample_params(c, b, nullptr, params, stream)) return e;
    if (int e = rb_simulate_paths(c, params, nullptr, paths, vol, stream)) return e;
    return rb_price_atm_marks(c, params, paths, vol, call, put, stream);
}

int32_t rb_host_normals(uint64_t seed, int32_t domain, uint32_t sub, uint64_t gid, uint32_t block0, int64_t n,
                        double* out) {
    if (!out || n < 0) return fail(RB_EINVAL, "bad arguments");
    for (int64_t i = 0; i < n; i += 2) {
        double z[2];
        normal_pair(rb_ctr(block0 + (uint32_t)(i / 2), domain, sub, gid), (uint32_t)seed, (uint32_t)(seed >> 32), &z[0],
                    &z[1]);
        out[i] = z[0];
        if (i + 1 < n) out[i + 1] = z[1];
    }
    return RB_OK;
}

int32_t rb_device_mc_box_muller(const double* u1, const double* u2, int64_t n, double* z1, double* z2, void* stream) {
    if (n < 0 || (n > 0 && (!u1 || !u2 || !z1 || !z2))) return fail(RB_EINVAL, "bad arguments");
    if (n == 0) return RB_OK;
    const int64_t blocks = (n + 255) / 256;
    if (blocks > 65535) return fail(RB_EINVAL, "n too large for the test hook");
    hipLaunchKernelGGL(mc_box_muller_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, u1, u2, n,
                       z1, z2);
    return hipGetLastError() == hipSuccess ? RB_OK : fail(RB_EHIP, "mc_box_muller_kernel launch failed");
}

}  // extern "C"
