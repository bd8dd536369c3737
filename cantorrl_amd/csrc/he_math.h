// he_math.h -- scalar building blocks of the hedging step, shared by the HIP
// kernels (__device__) and the host reference code (__host__).
//
// Every function restates one reference expression with the reference's
// dtype sequence (NumPy 2 / NEP 50: python scalars are weak, so f32 stays f32,
// int64 x f32 promotes to f64).  The library is compiled with
// -ffp-contract=off and correctly rounded f32 div/sqrt so that + - * / sqrt
// are bit-identical to NumPy's.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define HE_HD __host__ __device__ __forceinline__

namespace he {

// ---------------------------------------------------------------- constant FMAs
// a * b + c for a constant c (polynomial coefficients), bit-identical to fma(a, b, c).
// Left to itself the compiler emits v_fmac_f64 -- whose addend is its destination
// register, overwritten -- plus two v_mov per Horner step to re-materialise c: three
// VALU instructions.  The VOP3 v_fma_f64 reads c from an SGPR pair (s_mov, scalar
// unit, shared by every use in the block): one VALU instruction.
HE_HD double fma_k(double a, double b, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
    return r;
#else
    return fma(a, b, c);
#endif
}

// a * k + c for a constant multiplicand k (an SGPR pair), bit-identical to fma(a, k, c).
HE_HD double fma_kb(double a, double k, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(k), "v"(c));
    return r;
#else
    return fma(a, k, c);
#endif
}

// log(x) for the liability book's log S (hedge_env.hip book_value; its bar is 1e-5 on P&L, not
// bits): box_muller's reduction and atanh series (x = m 2^e, m in [sqrt2/2, sqrt2), s = (m - 1) /
// (m + 1), series to s^19) with s by v_rcp_f64 and two Newton steps instead of an IEEE division;
// within 2 ulp of the library log on positive finite x.  0, inf and NaN take the library's
// values by selects (the reduction runs on 1.0 there), so the caller stays branch-free.
HE_HD double log_book(double x) {
    const bool ok = x > 0.0 && x < __builtin_inf();   // frexp takes the denormals too
    const double xs = ok ? x : 1.0;
    int e;
    double m = frexp(xs, &e);
    const bool lo = m < 0.70710678118654752;
    m = lo ? m + m : m;
    e = lo ? e - 1 : e;
    const double den = m + 1.0;
#if defined(__HIP_DEVICE_COMPILE__)
    double y = __builtin_amdgcn_rcp(den);
#else
    double y = 1.0 / den;
#endif
    y = fma(fma(-den, y, 1.0), y, y);
    y = fma(fma(-den, y, 1.0), y, y);
    const double s = (m - 1.0) * y;
    const double s2 = s * s;
    double p = 1.0 / 19.0;
    p = fma_k(p, s2, 1.0 / 17.0);
    p = fma_k(p, s2, 1.0 / 15.0);
    p = fma_k(p, s2, 1.0 / 13.0);
    p = fma_k(p, s2, 1.0 / 11.0);
    p = fma_k(p, s2, 1.0 / 9.0);
    p = fma_k(p, s2, 1.0 / 7.0);
    p = fma_k(p, s2, 1.0 / 5.0);
    p = fma_k(p, s2, 1.0 / 3.0);
    const double lm = (2.0 * s) + (2.0 * s) * (s2 * p);
    const double ed = (double)e;
    const double r = fma(ed, 6.93147180369123816490e-01, fma(ed, 1.90821492927058770002e-10, lm));
    // log of 0 / inf / NaN or negatives: -inf / inf / NaN
    const double sp = (x == 0.0) ? -__builtin_inf() : (x > 0.0 ? __builtin_inf() : __builtin_nan(""));
    return ok ? r : sp;
}

// exp(x), f64, for the price advance exp((r - v/2) dt + sqrt(v) dW) (rbergomi_sim.py:459-463):
// x = k ln2 + r with k = rint(x / ln2), r by a two-constant Cody-Waite step (k ln2_hi exact
// for |k| < 2^21), e^r = (1 + r) + r^2 q(r) with q the Taylor series of (e^r - 1 - r) / r^2
// to r^15 (truncation < 2^-70 on |r| <= ln2 / 2) and the rounding error of 1 + r carried
// (Fast2Sum), then 2^k by v_ldexp.  Within 1 ulp of the correctly rounded value
// (tests/test_lib_cpu.py samples it against numpy); every constant an SGPR operand.  |x| >= 700 (over/underflow range) takes the library exp.
HE_HD double exp_k(double x) {
    if (!(fabs(x) < 700.0)) return exp(x);
    const double k = rint(x * 1.4426950408889634074);
    const double rh = fma_kb(-k, 6.93147180369123816490e-01, x);   // exact
    const double r = fma_kb(-k, 1.90821492927058770002e-10, rh);
    double q = 1.0 / 355687428096000.0;           // 1/17!, the r^15 coefficient of q
    q = fma_k(q, r, 1.0 / 20922789888000.0);      // 1/16!
    q = fma_k(q, r, 1.0 / 1307674368000.0);       // 1/15!
    q = fma_k(q, r, 1.0 / 87178291200.0);         // 1/14!
    q = fma_k(q, r, 1.0 / 6227020800.0);          // 1/13!
    q = fma_k(q, r, 1.0 / 479001600.0);           // 1/12!
    q = fma_k(q, r, 1.0 / 39916800.0);            // 1/11!
    q = fma_k(q, r, 1.0 / 3628800.0);             // 1/10!
    q = fma_k(q, r, 1.0 / 362880.0);
    q = fma_k(q, r, 1.0 / 40320.0);
    q = fma_k(q, r, 1.0 / 5040.0);
    q = fma_k(q, r, 1.0 / 720.0);
    q = fma_k(q, r, 1.0 / 120.0);
    q = fma_k(q, r, 1.0 / 24.0);
    q = fma_k(q, r, 1.0 / 6.0);
    q = fma_k(q, r, 0.5);
    // 1 + r + r^2 q with the rounding error of 1 + r kept (Fast2Sum: |1| >= |r|)
    const double s1 = 1.0 + r;
    const double e1 = (1.0 - s1) + r;              // exact
    return ldexp(s1 + fma(r * r, q, e1), (int)k);
}

// ---------------------------------------------------------------- numpy helpers
// np.maximum / np.minimum: NaN in either operand propagates.
HE_HD float np_maxf(float a, float b) { return (a != a) ? a : ((b != b) ? b : (a > b ? a : b)); }
HE_HD double np_max(double a, double b) { return (a != a) ? a : ((b != b) ? b : (a > b ? a : b)); }
// np.clip(x, lo, hi) for f32 with NaN propagation.
HE_HD float np_clipf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

// a / b, correctly rounded, from y = RN(1/b) precomputed on the host (Markstein:
// q = RN(a*y), r = a - b*q is exact by FMA, and RN(q + r*y) = RN(a/b) whenever the
// quotient and the dividend are clear of overflow and underflow).  Zero, tiny, huge
// and non-finite operands take the IEEE division.  Checked against a / b on 1.05e9
// pairs, 210 divisors (tests/test_lib_cpu.py repeats a sample through the host build).
HE_HD double div_by(double a, double b, double y) {
    double q = a * y;
    double aq = fabs(q), aa = fabs(a);
    // r = a - b q must be exact: keep q and a (so r ~ ulp(a)) clear of subnormals
    if (!(aq > 0x1p-960 && aq < 0x1p+960 && aa > 0x1p-960)) return a / b;
    double r = fma(-q, b, a);
    return fma(r, y, q);
}

// f32 a / b, correctly rounded, by the same Markstein step with y = RN_f32(1/b): the
// obs quotients by per-handle constants (max(S0, 25), max_contracts_held, T).  A
// true f32 division is ~11 instructions with two quarter-rate reciprocals; this is 3.
// Exhaustively checked over all 2^32 numerators for the default divisors
// (tools/div_check.c), sampled for random divisors in tests/test_lib_cpu.py.
HE_HD float div_byf(float a, float b, float y) {
    float q = a * y;
    float aq = fabsf(q), aa = fabsf(a);
    if (!(aq > 0x1p-100f && aq < 0x1p+100f && aa > 0x1p-100f)) return a / b;
    float r = fmaf(-q, b, a);
    return fmaf(r, y, q);
}

// div_by without its guard, for dividends that are 0 or normal with |a| < 2^900 and
// quotients clear of the subnormals (every FAST-configuration P&L and reward term: a
// difference of portfolio values is 0 or a multiple of ulp(pv), see fast_config):
// there q, r = a - b q (exact by FMA) and RN(q + r y) equal the guarded path bit for
// bit, a = +0 included.  Branch-free.
HE_HD double div_by_nb(double a, double b, double y) {
    const double q = a * y;
    return fma(fma(-q, b, a), y, q);
}

// Integer-valued a (|a| <= 2^24) by a constant 1 <= b <= 2^30: the Markstein step with
// no guard -- q = a*y can neither overflow nor fall near the subnormals, and a = 0
// gives +0 like +0 / b.  f32 (obs positions / max held, (T - t) / T) and f64 ((T - t)
// / 252) forms.
HE_HD float div_int_byf(float a, float b, float y) {
    const float q = a * y;
    return fmaf(fmaf(-q, b, a), y, q);
}
HE_HD double div_int_by(double a, double b, double y) {
    const double q = a * y;
    return fma(fma(-q, b, a), y, q);
}

// f32 a / b for any f32 a, branch-free: the f64 Markstein step on the f32 operands
// (an f32 quotient is never near the f64 subnormals or overflow, so RN64(a/b) is exact
// by the theorem) rounded once more to f32 -- RN32(RN64(a/b)) = RN32(a/b) since
// 53 >= 2*24 + 2.  Zero / inf / NaN dividends take a*y (same value and sign as a/b).
// y64 = RN64(1/b).
HE_HD float div_f32_by(float a, double b, double y64) {
    const double ad = (double)a;
    const double q = ad * y64;
    const double r = fma(-q, b, ad);
    const float res = (float)fma(r, y64, q);
    return (a == 0.0f || !(fabsf(a) <= 3.4028234663852886e38f)) ? (float)q : res;
}

// f32 a / b for an f32 b with y = RN32(1/b), when a and a / b are normal f32 numbers (the lean
// GBM obs prices over the constant max(S0, 25): S >= 1e-8, C, P >= 0): Markstein's step in f32,
// RN32(a/b) by the theorem (y within half an ulp of 1/b, a*y within one ulp of a/b) -- the value
// div_f32_by makes through f64.  Zero / inf / NaN dividends take a*y, as there.
HE_HD float div_f32_byf(float a, float b, float y) {
    const float q = a * y;
    const float res = fmaf(fmaf(-q, b, a), y, q);
    return (a == 0.0f || !(fabsf(a) <= 3.4028234663852886e38f)) ? q : res;
}

// np.rint(f32).astype(int64) then np.clip(., -mt, mt)  (hedging_env_v2.py:184-188).
// x86 cvttss2si maps NaN and |x| >= 2^63 to INT64_MIN, which the clip sends to -mt.
// Branch-free (selects only): the step kernels keep whole steps in one basic block.
HE_HD int32_t trade_round(float f, int32_t mt) {
    const float r = rintf(f);
    const bool ok = fabsf(r) < 9.2233720368547758e18f;  // false for NaN and |x| >= 2^63
    const float lo = -(float)mt, hi = (float)mt;
#if defined(__HIP_DEVICE_COMPILE__)
    // the clamp as one v_med3_f32 (lo <= hi; a NaN r is replaced by -mt either way): headline
    // 277.6 -> 274.1 us per launch, 3 of 3 same-box pairs (r05s27_ab_trade_med3.txt)
    return ok ? (int32_t)__builtin_amdgcn_fmed3f(r, lo, hi) : -mt;
#else
    const float c = r < lo ? lo : (r > hi ? hi : r);
    const int32_t v = ok ? (int32_t)c : 0;
    return ok ? v : -mt;
#endif
}

// ---------------------------------------------------------------- Philox4x32-10
// Salmon et al. (SC'11) / Random123; same block function as rocRAND's
// philox4x32_10.  Counter = (lo(n), hi(n), lo(g), hi(g)), key = (lo(seed), hi(seed)).
struct u32x4 { uint32_t x, y, z, w; };

HE_HD uint32_t mulhi32(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umulhi(a, b);
#else
    return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
#endif
}

HE_HD u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += W0; k1 += W1; }
        // one 32x32->64 product per multiplier (v_mad_u64_u32) instead of separate
        // quarter-rate mul_hi / mul_lo instructions
        const uint64_t p0 = (uint64_t)M0 * c.x, p1 = (uint64_t)M1 * c.z;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        u32x4 o;
        o.x = hi1 ^ c.y ^ k0;
        o.y = lo1;
        o.z = hi0 ^ c.w ^ k1;
        o.w = lo0;
        c = o;
    }
    return c;
}

// (0,1) double from two words: ((hi:lo >> 12) + 0.5) * 2^-52, exact.
HE_HD double u01(uint32_t hi, uint32_t lo) {
    uint64_t k = ((((uint64_t)hi) << 32) | (uint64_t)lo) >> 12;
    return ((double)k + 0.5) * 2.220446049250313e-16;
}

// ---------------------------------------------------------------- Box-Muller
// (sqrt(-2 log u1) cos(2 pi u2), sqrt(-2 log u1) sin(2 pi u2)) for u1, u2 in (0, 1)
// of the u01 form, in f64 within a few ulp of libm without libm's general-argument
// machinery (measured: 13 % of market_kernel with ocml log + sincos):
//  * log u1 = e ln2 + 2 atanh(s), s = (m-1)/(m+1), m in [sqrt2/2, sqrt2): the series to
//    s^19 (|s| <= 0.1716: next term < 2.4e-17 relative), ln2 split hi/lo;
//  * 2 pi u2 = (pi/2)(q + r), q = rint(4 u2), r = 4 u2 - q in [-1/2, 1/2] exactly (4 u2
//    is a fixed-point number), so sin/cos of (pi/2) r are two short even/odd
//    polynomials in r (Taylor to r^17 / r^16, truncation < 1e-19) and q picks the
//    quadrant -- no Cody-Waite reduction.
// sin / cos of 2 pi u for u in [0, 1) of the u01 form (box_muller's): 2 pi u = (pi/2)(q + r),
// q = rint(4 u), r = 4 u - q in [-1/2, 1/2] exactly, two short polynomials in r, q the quadrant
HE_HD void sincos_2pi_u(double u2, double* sin_out, double* cos_out) {
    const double x = 4.0 * u2;
    const double q = rint(x);
    const double r = x - q;
    const double rr = r * r;
    double sp = 6.066935731106192e-12;
    sp = fma_k(sp, rr, -6.688035109811464e-10);
    sp = fma_k(sp, rr, 5.692172921967924e-08);
    sp = fma_k(sp, rr, -3.598843235212084e-06);
    sp = fma_k(sp, rr, 0.00016044118478735975);
    sp = fma_k(sp, rr, -0.004681754135318687);
    sp = fma_k(sp, rr, 0.07969262624616703);
    sp = fma_k(sp, rr, -0.6459640975062462);
    sp = fma_k(sp, rr, 1.5707963267948966);
    const double sn = r * sp;
    double cp = 6.565963114979468e-11;
    cp = fma_k(cp, rr, -6.386603083791849e-09);
    cp = fma_k(cp, rr, 4.710874778818169e-07);
    cp = fma_k(cp, rr, -2.5202042373060596e-05);
    cp = fma_k(cp, rr, 0.0009192602748394263);
    cp = fma_k(cp, rr, -0.020863480763352957);
    cp = fma_k(cp, rr, 0.253669507901048);
    cp = fma_k(cp, rr, -1.2337005501361697);
    const double cs = fma_k(cp, rr, 1.0);
    // quadrant qi: (sin, cos) = (sn, cs), (cs, -sn), (-sn, -cs), (-cs, sn) -- as two
    // selects and two exact sign flips (a chained ?: on qi lowers to branches)
    const int qi = (int)q & 3;
    const bool swp = (qi & 1) != 0;
    const double s_ = swp ? cs : sn, c_ = swp ? sn : cs;
    *sin_out = (qi & 2) ? -s_ : s_;
    *cos_out = ((qi + 1) & 2) ? -c_ : c_;
}

// a / b by the correctly rounded f64 division's lowering without its v_div_scale / v_div_fixup:
// the same bits wherever those change nothing -- a and b finite, b normal and well inside the
// exponent range, a 0 or with an exponent within a few hundred of b's (bm_quot, the FAST replay
// reward's two quotients on an ordinary table: he_env::table_ordinary)
HE_HD double div_f64_core(double a, double b) {
#if defined(__HIP_DEVICE_COMPILE__)
    double r = __builtin_amdgcn_rcp(b);
    r = fma(r, fma(-b, r, 1.0), r);
    r = fma(r, fma(-b, r, 1.0), r);
    const double q = a * r;
    return fma(fma(-b, q, a), r, q);
#else
    return a / b;
#endif
}

// (m - 1) / (m + 1) for the Box-Muller log's mantissa m in [sqrt2/2, sqrt2): the correctly rounded
// f64 division's lowering (v_rcp_f64, two Newton steps, the quotient and one residual correction)
// without its v_div_scale / v_div_fixup, which never act on these operands (m - 1 is 0 or at least
// 2^-53, m + 1 within [1.7, 2.5]) -- the same operations, so the same bits (config 2 -0.4 %,
// r05s25_ab_bm_quot.txt)
HE_HD double bm_quot(double m) { return div_f64_core(m - 1.0, m + 1.0); }

// sqrt of the Box-Muller radius x = -2 log u, in [2.2e-16, 73.5] for the u01 draws: ocml's
// correctly rounded f64 sqrt (v_rsq_f64, then Goldschmidt and two residual corrections) without
// its range scaling and special-value selects, which never apply there -- the same operations,
// so the same bits (the host build's sqrt: test_device_philox_words_equal_rocrand); config 2
// -0.3 %, config 5 -0.4 %, 3 of 3 same-box pairs each (r05s24_ab_sqrt_bm.txt)
HE_HD double sqrt_bm(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = y * 0.5;
    const double r = fma(-h, g, 0.5);
    g = fma(g, r, g);
    double d = fma(-g, g, x);
    h = fma(h, r, h);
    g = fma(d, h, g);
    d = fma(-g, g, x);
    return fma(d, h, g);
#else
    return sqrt(x);
#endif
}

HE_HD void box_muller(double u1, double u2, double* z1, double* z2) {
    // log(u1)
    int e;
    double m = frexp(u1, &e);           // u1 = m 2^e, m in [1/2, 1)
    if (m < 0.70710678118654752) {      // -> [sqrt2/2, sqrt2)
        m = m + m;
        e -= 1;
    }
    const double s = bm_quot(m);
    const double s2 = s * s;
    double p = 1.0 / 19.0;
    p = fma_k(p, s2, 1.0 / 17.0);
    p = fma_k(p, s2, 1.0 / 15.0);
    p = fma_k(p, s2, 1.0 / 13.0);
    p = fma_k(p, s2, 1.0 / 11.0);
    p = fma_k(p, s2, 1.0 / 9.0);
    p = fma_k(p, s2, 1.0 / 7.0);
    p = fma_k(p, s2, 1.0 / 5.0);
    p = fma_k(p, s2, 1.0 / 3.0);
    const double lm = (2.0 * s) + (2.0 * s) * (s2 * p);   // 2 atanh(s)
    const double ed = (double)e;
    const double lg = fma(ed, 6.93147180369123816490e-01, fma(ed, 1.90821492927058770002e-10, lm));
    const double rad = sqrt_bm(-2.0 * lg);
    double sinv, cosv;
    sincos_2pi_u(u2, &sinv, &cosv);
    *z1 = rad * cosv;
    *z2 = rad * sinv;
}

// ---------------------------------------------------------------- normal cdf/pdf
// erf on |x| < 1/sqrt2 (the branch ndtr uses): Maclaurin series
// 2/sqrt(pi) * sum_n (-1)^n x^(2n+1) / (n! (2n+1)) to n = 15 -- alternating, so the
// truncation error < the n=16 term < 3e-20 |x|; 16 FMAs instead of ocml's
// ranged rational approximation (~2-3x the instructions).
HE_HD double erf_small(double x) {
    const double z = x * x;
    double p = -2.783516207210921354903762e-14;
    p = fma_k(p, z, 4.463224263286477344931894e-13);
    p = fma_k(p, z, -6.711366855164110377934626e-12);
    p = fma_k(p, z, 9.422759064650410970620214e-11);
    p = fma_k(p, z, -1.229055530171792735298289e-9);
    p = fma_k(p, z, 1.480719281587921723954605e-8);
    p = fma_k(p, z, -0.00000016365844691234924317393);
    p = fma_k(p, z, 0.000001646211436588924740161296);
    p = fma_k(p, z, -0.00001492565035840625097746242);
    p = fma_k(p, z, 0.0001205533298178966425102734);
    p = fma_k(p, z, -0.0008548327023450852832546658);
    p = fma_k(p, z, 0.005223977625442187842111847);
    p = fma_k(p, z, -0.02686617064513125175943235);
    p = fma_k(p, z, 0.1128379167095512573896159);
    p = fma_k(p, z, -0.376126389031837524632053);
    p = fma_k(p, z, 1.128379167095512573896159);
    return x * p;
}

// The same series for |x| < 1/4, to n = 8: the n=9 term < 0.25^19/(9! 19) = 5e-19 |x|
// relative to erf ~ 1.13 |x| -- below 2^-53.  Rolling-ATM marks have |d|/sqrt2 < 0.1.
HE_HD double erf_small4(double x) {
    const double z = x * x;
    double p = 0.000001646211436588924740161296;
    p = fma_k(p, z, -0.00001492565035840625097746242);
    p = fma_k(p, z, 0.0001205533298178966425102734);
    p = fma_k(p, z, -0.0008548327023450852832546658);
    p = fma_k(p, z, 0.005223977625442187842111847);
    p = fma_k(p, z, -0.02686617064513125175943235);
    p = fma_k(p, z, 0.1128379167095512573896159);
    p = fma_k(p, z, -0.376126389031837524632053);
    p = fma_k(p, z, 1.128379167095512573896159);
    return x * p;
}

// scipy.special.ndtr (cephes ndtr.c): erf branch inside |x| < 1/sqrt2.
HE_HD double ndtr(double a) {
    if (a != a) return a;
    const double SQRT1_2 = 0.70710678118654752440;
    double x = a * SQRT1_2;
    double z = fabs(x);
    double y;
    if (z < SQRT1_2) {
        y = 0.5 + 0.5 * erf_small(x);
    } else {
        y = 0.5 * erfc(z);
        if (x > 0) y = 1.0 - y;
    }
    return y;
}

// (ndtr(a), ndtr(-a)) from one erf/erfc evaluation, each bit-identical to a
// separate ndtr() call: erf_small is odd (x * P(x^2)), and for |x| >= 1/sqrt2 both
// branches evaluate erfc(|x|).
HE_HD void ndtr_pair(double a, double* pos, double* neg) {
    if (a != a) {
        *pos = *neg = a;
        return;
    }
    const double SQRT1_2 = 0.70710678118654752440;
    double x = a * SQRT1_2;
    double z = fabs(x);
    if (z < SQRT1_2) {
        double e = (z < 0.25) ? erf_small4(x) : erf_small(x);
        *pos = 0.5 + 0.5 * e;
        *neg = 0.5 + 0.5 * (-e);
    } else {
        double y = 0.5 * erfc(z);
        if (x > 0) {
            *pos = 1.0 - y;
            *neg = y;
        } else {
            *pos = y;
            *neg = 1.0 - y;
        }
    }
}

// scipy.stats.norm.pdf: exp(-x**2/2.0) / sqrt(2*pi)  (x**2 on an array = x*x)
// (division by 2.0 is exact scaling, so *0.5 is bit-identical; the division by
// sqrt(2 pi) becomes a multiply by 1/sqrt(2 pi): <= 1 ulp, far below the f32 cast)
HE_HD double norm_pdf(double x) {
    return exp(-(x * x) * 0.5) * 0.3989422804014327;
}

// ---------------------------------------------------------------- Black-Scholes
// OptionCalculator.black_scholes_price (quantconnect/option_calculator.py:11-27),
// f64.  `a` = (r + 0.5*sigma**2)*T, `b` = sigma*sqrt(T), `disc` = exp(-r*T) are
// precomputed with python-float semantics when sigma is constant.
// log(S / K) for the rolling-ATM strike K = round(S): the quotient is within
// 2^-7 of 1 whenever S >= 64, where log1p of y = S / K - 1 is a 9-term alternating
// series (truncation < y^10/10); elsewhere ocml log.  On the device y = (S - K) / K
// by v_rcp_f64 and two Newton steps (S - K exact by Sterbenz; y within a few ulps of
// y, which is tiny, against the 2^-53 absolute error of the rounded S / K - 1) instead
// of an IEEE f64 division: headline 288.0 -> 285.9 us per launch, 3 of 3 same-box
// pairs, every GPU test bit-identical (r05s14_ab_log_ratio_rcp.txt).
HE_HD double log_ratio(double S, double K) {
#if defined(__HIP_DEVICE_COMPILE__)
    double r = __builtin_amdgcn_rcp(K);
    r = fma(fma(-K, r, 1.0), r, r);
    r = fma(fma(-K, r, 1.0), r, r);
    const double y = (S - K) * r;
    if (!(fabs(y) < 0.0078125)) return log(S / K);
#else
    const double q = S / K;
    const double y = q - 1.0;
    if (!(fabs(y) < 0.0078125)) return log(q);
#endif
    double p = 1.0 / 9.0;
    p = fma_k(p, y, -1.0 / 8.0);
    p = fma_k(p, y, 1.0 / 7.0);
    p = fma_k(p, y, -1.0 / 6.0);
    p = fma_k(p, y, 1.0 / 5.0);
    p = fma_k(p, y, -1.0 / 4.0);
    p = fma_k(p, y, 1.0 / 3.0);
    p = fma_k(p, y, -0.5);
    p = fma_k(p, y, 1.0);
    return y * p;
}

struct BSConst {
    double a, b, disc;
    double inv_b;   // 1/b: the constant-sigma division becomes a multiply (<= 1 ulp)
    int intrinsic;  // T <= 0 or sigma <= 0
};

HE_HD void bs_call_put(double S, double K, const BSConst& c, double* call, double* put) {
    if (c.intrinsic) {
        double ic = S - K, ip = K - S;
        *call = (ic < 0.0) ? 0.0 : ic;
        *put = (ip < 0.0) ? 0.0 : ip;
        return;
    }
    double d1 = (log_ratio(S, K) + c.a) * c.inv_b;
    double d2 = d1 - c.b;
    double Kd = K * c.disc;
    double n1, m1, n2, m2;
    ndtr_pair(d1, &n1, &m1);
    ndtr_pair(d2, &n2, &m2);
    double cv = S * n1 - Kd * n2;
    double pv = Kd * m2 - S * m1;
    *call = (cv < 0.0) ? 0.0 : cv;   // python max(price, 0): NaN stays NaN
    *put = (pv < 0.0) ? 0.0 : pv;
}

// black_scholes_vectorized (src/sim/option_price_assignment.py:10-21) for one element,
// f64, the reference's operation order: T_safe = 1e-8 for T <= 0, sigma_safe = 1e-8 for
// sigma < 1e-8 (NaN stays NaN), no floor at 0, and the intrinsic value against the
// discounted strike K e^{-r T} when T <= 0.  ndtr(x) and ndtr(-x) from one erf / erfc
// evaluation (ndtr_pair: each bit-identical to its own ndtr call).  The fixed-strike
// European mark (he_mark HE_MARK_FIXED_EUROPEAN) and he_fixed_european_marks.
HE_HD void bs_vectorized(double S, double K, double T, double r, double sigma, double* call, double* put) {
    const double Ts = (T <= 0.0) ? 1e-8 : T;
    const double ss = (sigma < 1e-8) ? 1e-8 : sigma;
    const double sqT = sqrt(Ts);
    const double d1 = (log(S / K) + (r + 0.5 * (ss * ss)) * Ts) / (ss * sqT);
    const double d2 = d1 - ss * sqT;
    const double Kd = K * exp(-r * Ts);
    double n1, m1, n2, m2;
    ndtr_pair(d1, &n1, &m1);
    ndtr_pair(d2, &n2, &m2);
    double c = S * n1 - Kd * n2;
    double p = Kd * m2 - S * m1;
    if (T <= 0.0) {   // np.where(T <= 0, intrinsic, .)
        const double KT = K * exp(-r * T);
        c = np_max(S - KT, 0.0);
        p = np_max(KT - S, 0.0);
    }
    *call = c;
    *put = p;
}

// ---------------------------------------------------------------- lockstep forms
// The same functions over NN independent arguments at once, element for element the
// scalar version's operations in the scalar version's order (so the same bits), but with
// the loop over polynomial coefficients outside the loop over elements: a wave gets NN
// independent FMA chains to interleave instead of one dependent chain, and each f64
// constant is materialised in SGPRs once per coefficient for NN FMAs instead of once per
// FMA.  Used by the LDS producers, which evaluate several market slots per lane.
// Whether any lane of the wave holds `c` (device; the host build is one lane).  The lockstep
// fast paths below branch on it, so their common case is one straight-line block for the
// whole wave instead of an exec-mask branch per lane group (the general path gives the same
// bits for every lane, so which lanes take it does not matter).
#if defined(__HIP_DEVICE_COMPILE__) && !defined(HE_LOCK_LANEWISE)
__device__ __forceinline__ bool he_any_lane(bool c) { return __ballot(c) != 0ull; }
#else
HE_HD bool he_any_lane(bool c) { return c; }
#endif

template <int NN>
HE_HD void exp_k_n(const double* x, double* out) {
    double k[NN], r[NN], q[NN];
#pragma unroll
    for (int h = 0; h < NN; ++h) {
        const double xs = (fabs(x[h]) < 700.0) ? x[h] : 0.0;   // |x| >= 700 / NaN: library exp below
        k[h] = rint(xs * 1.4426950408889634074);
        const double rh = fma_kb(-k[h], 6.93147180369123816490e-01, xs);
        r[h] = fma_kb(-k[h], 1.90821492927058770002e-10, rh);
        q[h] = 1.0 / 355687428096000.0;
    }
    constexpr double C[16] = {1.0 / 20922789888000.0, 1.0 / 1307674368000.0, 1.0 / 87178291200.0,
                              1.0 / 6227020800.0,     1.0 / 479001600.0,     1.0 / 39916800.0,
                              1.0 / 3628800.0,        1.0 / 362880.0,        1.0 / 40320.0,
                              1.0 / 5040.0,           1.0 / 720.0,           1.0 / 120.0,
                              1.0 / 24.0,             1.0 / 6.0,             0.5,
                              0.0};
#pragma unroll
    for (int c = 0; c < 15; ++c)
#pragma unroll
        for (int h = 0; h < NN; ++h) q[h] = fma_k(q[h], r[h], C[c]);
#pragma unroll
    for (int h = 0; h < NN; ++h) {
        const double s1 = 1.0 + r[h];
        const double e1 = (1.0 - s1) + r[h];
        out[h] = ldexp(s1 + fma(r[h] * r[h], q[h], e1), (int)k[h]);
    }
    bool big = false;
#pragma unroll
    for (int h = 0; h < NN; ++h) big = big || !(fabs(x[h]) < 700.0);
    if (he_any_lane(big)) {   // |x| >= 700 / NaN somewhere in the wave: the library exp there
#pragma unroll
        for (int h = 0; h < NN; ++h) out[h] = (fabs(x[h]) < 700.0) ? out[h] : exp(x[h]);
    }
}

template <int NN>
HE_HD void philox4x32_10_n(u32x4* c, uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int rd = 0; rd < 10; ++rd) {
        if (rd) { k0 += W0; k1 += W1; }
#pragma unroll
        for (int h = 0; h < NN; ++h) {
            const uint64_t p0 = (uint64_t)M0 * c[h].x, p1 = (uint64_t)M1 * c[h].z;
            u32x4 o;
            o.x = (uint32_t)(p1 >> 32) ^ c[h].y ^ k0;
            o.y = (uint32_t)p1;
            o.z = (uint32_t)(p0 >> 32) ^ c[h].w ^ k1;
            o.w = (uint32_t)p0;
            c[h] = o;
        }
    }
}

template <int NN>
HE_HD void box_muller_n(const double* u1, const double* u2, double* z1, double* z2) {
    double s[NN], s2[NN], p[NN], ed[NN];
#pragma unroll
    for (int h = 0; h < NN; ++h) {
        int e;
        double m = frexp(u1[h], &e);
        const bool lo = m < 0.70710678118654752;
        m = lo ? m + m : m;
        ed[h] = (double)(lo ? e - 1 : e);
        s[h] = bm_quot(m);
        s2[h] = s[h] * s[h];
        p[h] = 1.0 / 19.0;
    }
    constexpr double PL[8] = {1.0 / 17.0, 1.0 / 15.0, 1.0 / 13.0, 1.0 / 11.0, 1.0 / 9.0, 1.0 / 7.0, 1.0 / 5.0, 1.0 / 3.0};
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
        for (int h = 0; h < NN; ++h) p[h] = fma_k(p[h], s2[h], PL[c]);
    double rad[NN], r[NN], rr[NN], sp[NN], cp[NN];
    int qi[NN];
#pragma unroll
    for (int h = 0; h < NN; ++h) {
        const double lm = (2.0 * s[h]) + (2.0 * s[h]) * (s2[h] * p[h]);
        const double lg = fma(ed[h], 6.93147180369123816490e-01, fma(ed[h], 1.90821492927058770002e-10, lm));
        rad[h] = sqrt_bm(-2.0 * lg);
        const double x = 4.0 * u2[h];
        const double q = rint(x);
        r[h] = x - q;
        rr[h] = r[h] * r[h];
        qi[h] = (int)q & 3;
        sp[h] = 6.066935731106192e-12;
        cp[h] = 6.565963114979468e-11;
    }
    constexpr double SP[8] = {-6.688035109811464e-10, 5.692172921967924e-08, -3.598843235212084e-06,
                              0.00016044118478735975, -0.004681754135318687, 0.07969262624616703,
                              -0.6459640975062462,    1.5707963267948966};
    constexpr double CP[8] = {-6.386603083791849e-09, 4.710874778818169e-07, -2.5202042373060596e-05,
                              0.0009192602748394263,  -0.020863480763352957, 0.253669507901048,
                              -1.2337005501361697,    1.0};
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
        for (int h = 0; h < NN; ++h) {
            sp[h] = fma_k(sp[h], rr[h], SP[c]);
            cp[h] = fma_k(cp[h], rr[h], CP[c]);
        }
#pragma unroll
    for (int h = 0; h < NN; ++h) {
        const double sn = r[h] * sp[h];
        const double cs = cp[h];
        const bool swp = (qi[h] & 1) != 0;
        const double s_ = swp ? cs : sn, c_ = swp ? sn : cs;
        const double sinv = (qi[h] & 2) ? -s_ : s_;
        const double cosv = ((qi[h] + 1) & 2) ? -c_ : c_;
        z1[h] = rad[h] * cosv;
        z2[h] = rad[h] * sinv;
    }
}

// ndtr_pair over NN arguments: the |x| < 1/4 series lockstep when every argument of the
// wave is there (rolling-ATM marks always are), else each through ndtr_pair.
template <int NN>
HE_HD void ndtr_pair_n(const double* a, double* pos, double* neg) {
    const double SQRT1_2 = 0.70710678118654752440;
    double x[NN], z[NN], p[NN];
    bool easy = true;
#pragma unroll
    for (int h = 0; h < NN; ++h) {
        x[h] = a[h] * SQRT1_2;
        easy = easy && (fabs(x[h]) < 0.25);   // NaN: false
        z[h] = x[h] * x[h];
        p[h] = 0.000001646211436588924740161296;
    }
    if (he_any_lane(!easy)) {   // device: wave-uniform (a scalar branch; the lockstep path stays straight-line)
#pragma unroll
        for (int h = 0; h < NN; ++h) ndtr_pair(a[h], pos + h, neg + h);
        return;
    }
    constexpr double E[8] = {-0.00001492565035840625097746242, 0.0001205533298178966425102734,
                             -0.0008548327023450852832546658,  0.005223977625442187842111847,
                             -0.02686617064513125175943235,    0.1128379167095512573896159,
                             -0.376126389031837524632053,      1.128379167095512573896159};
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
        for (int h = 0; h < NN; ++h) p[h] = fma_k(p[h], z[h], E[c]);
#pragma unroll
    for (int h = 0; h < NN; ++h) {
        const double e = x[h] * p[h];
        pos[h] = 0.5 + 0.5 * e;
        neg[h] = 0.5 + 0.5 * (-e);
    }
}

// log_ratio over NN (S, K) pairs: the log1p series lockstep when every quotient of the
// lane is within 2^-7 of 1 (S >= 64), else each through log_ratio.
template <int NN>
HE_HD void log_ratio_n(const double* S, const double* K, double* out) {
    double y[NN], p[NN];
    bool easy = true;
#pragma unroll
    for (int h = 0; h < NN; ++h) {
#if defined(__HIP_DEVICE_COMPILE__)
        double r = __builtin_amdgcn_rcp(K[h]);   // log_ratio's operations
        r = fma(fma(-K[h], r, 1.0), r, r);
        r = fma(fma(-K[h], r, 1.0), r, r);
        y[h] = (S[h] - K[h]) * r;
#else
        const double q = S[h] / K[h];
        y[h] = q - 1.0;
#endif
        easy = easy && (fabs(y[h]) < 0.0078125);
        p[h] = 1.0 / 9.0;
    }
    if (he_any_lane(!easy)) {
#pragma unroll
        for (int h = 0; h < NN; ++h) out[h] = log_ratio(S[h], K[h]);
        return;
    }
    constexpr double L[8] = {-1.0 / 8.0, 1.0 / 7.0, -1.0 / 6.0, 1.0 / 5.0, -1.0 / 4.0, 1.0 / 3.0, -0.5, 1.0};
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
        for (int h = 0; h < NN; ++h) p[h] = fma_k(p[h], y[h], L[c]);
#pragma unroll
    for (int h = 0; h < NN; ++h) out[h] = y[h] * p[h];
}

// bs_call_put over NN spots S with strikes K at the constant-sigma BSConst c.
template <int NN>
HE_HD void bs_call_put_n(const double* S, const double* K, const BSConst& c, double* call, double* put) {
    if (c.intrinsic) {
#pragma unroll
        for (int h = 0; h < NN; ++h) bs_call_put(S[h], K[h], c, call + h, put + h);
        return;
    }
    double lr[NN], d[2 * NN], nd[2 * NN], md[2 * NN];
    log_ratio_n<NN>(S, K, lr);
#pragma unroll
    for (int h = 0; h < NN; ++h) {
        d[h] = (lr[h] + c.a) * c.inv_b;
        d[NN + h] = d[h] - c.b;
    }
    ndtr_pair_n<NN>(d, nd, md);             // two groups of NN chains: 2 NN would spill
    ndtr_pair_n<NN>(d + NN, nd + NN, md + NN);
#pragma unroll
    for (int h = 0; h < NN; ++h) {
        const double Kd = K[h] * c.disc;
        const double cv = S[h] * nd[h] - Kd * nd[NN + h];
        const double pv = Kd * md[NN + h] - S[h] * md[h];
        call[h] = (cv < 0.0) ? 0.0 : cv;
        put[h] = (pv < 0.0) ? 0.0 : pv;
    }
}

// ---------------------------------------------------------------- PCG64 (numpy)
// numpy/random/src/pcg64: 128-bit LCG, XSL-RR output; next32 keeps the high
// half of a 64-bit draw buffered (has_uint32/uinteger).
struct Pcg64 {
    uint64_t sh, sl, ih, il;  // state hi/lo, inc hi/lo
    uint32_t has32, buf32;
};

HE_HD void pcg64_step(Pcg64& g) {
    const uint64_t MH = 0x2360ED051FC65DA4ull, ML = 0x4385DF649FCCF645ull;
#if defined(__HIP_DEVICE_COMPILE__)
    uint64_t lo = g.sl * ML;
    uint64_t hi = __umul64hi(g.sl, ML) + g.sl * MH + g.sh * ML;
#else
    unsigned __int128 p = (unsigned __int128)g.sl * ML;
    uint64_t lo = (uint64_t)p;
    uint64_t hi = (uint64_t)(p >> 64) + g.sl * MH + g.sh * ML;
#endif
    uint64_t nl = lo + g.il;
    uint64_t carry = nl < lo ? 1ull : 0ull;
    g.sl = nl;
    g.sh = hi + g.ih + carry;
}

HE_HD uint64_t pcg64_next64(Pcg64& g) {
    pcg64_step(g);
    uint64_t x = g.sh ^ g.sl;
    unsigned rot = (unsigned)(g.sh >> 58);
    return (x >> rot) | (x << ((64u - rot) & 63u));
}

HE_HD uint32_t pcg64_next32(Pcg64& g) {
    if (g.has32) {
        g.has32 = 0;
        return g.buf32;
    }
    uint64_t x = pcg64_next64(g);
    g.has32 = 1;
    g.buf32 = (uint32_t)(x >> 32);
    return (uint32_t)x;
}

HE_HD uint64_t mulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

// Generator.integers(P) for int64 (numpy random_bounded_uint64_fill, Lemire).
HE_HD int64_t pcg64_integers(Pcg64& g, uint64_t P) {
    uint64_t rng = P - 1;
    if (rng == 0) return 0;
    if (rng <= 0xFFFFFFFFull) {
        if (rng == 0xFFFFFFFFull) return (int64_t)pcg64_next32(g);
        uint32_t rng32 = (uint32_t)rng, excl = rng32 + 1u;
        uint64_t m = (uint64_t)pcg64_next32(g) * (uint64_t)excl;
        uint32_t left = (uint32_t)m;
        if (left < excl) {
            uint32_t thr = (0xFFFFFFFFu - rng32) % excl;
            while (left < thr) {
                m = (uint64_t)pcg64_next32(g) * (uint64_t)excl;
                left = (uint32_t)m;
            }
        }
        return (int64_t)(m >> 32);
    }
    uint64_t excl = rng + 1;
    uint64_t x = pcg64_next64(g);
    uint64_t left = x * excl, hi = mulhi64(x, excl);
    if (left < excl) {
        uint64_t thr = (~0ull - rng) % excl;
        while (left < thr) {
            x = pcg64_next64(g);
            left = x * excl;
            hi = mulhi64(x, excl);
        }
    }
    return (int64_t)hi;
}

}  // namespace he
