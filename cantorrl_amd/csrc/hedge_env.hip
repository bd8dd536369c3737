// hedge_env.hip -- libhedgeenv: the batched hedging environment for MI355X.
//
// Two kernels split the reference step (src/env/hedging_env_v2.py:175-294) along
// its data dependency:
//
//   market_kernel  (generate modes, once per M steps)  -- everything that does NOT
//       depend on the agent's actions: Philox4x32-10 normals, the GBM/Heston price
//       advance (rbergomi_sim.py:454-464), Black-Scholes rolling-ATM marks
//       (quantconnect/option_calculator.py:11-27) and the obs greeks
//       (hedging_env_v2.py:79-107).  Parallel over env x slot (4 slot-lanes per
//       env, 64 envs per workgroup, the sequential f64 price chain staged in LDS),
//       so it runs at >= 4 waves/SIMD even at 65,536 envs.  Output: an HBM tile
//       [M+1][N] of {S, v, C, P} and {delta_c, gamma, delta_p} in f32, exactly the
//       data the reference env would replay from an NPZ (hedging_env_v2.py:38-41).
//
//   step_kernel    (every step; K fused steps for he_rollout) -- the action-dependent
//       part: integer trade logic, commission + slippage, f64 mark-to-market P&L,
//       reward, 13-float obs, SB3 auto-reset.  One thread per env, struct-of-arrays
//       state, obs rows staged through LDS and written as 16-B stores, wave ballot
//       so waves with no terminating env skip the reset path.
//
// Replay mode reuses step_kernel: its market source is the loaded table
// [paths][T+1] {S, v, C, P} (+ greeks precomputed once at load time).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <new>
#include <type_traits>

#include "vn_moments.h"
#include <string>
#include <vector>

#include "../../include/hedge_env.h"
#include "he_math.h"

using namespace he;

namespace {

#define GLOBAL __attribute__((address_space(1)))
// Values a select picks from are pinned in VGPRs first (opaque), so the backend keeps the
// select instead of a divergent branch around their computation.
#define HE_OPAQUE1(a) asm volatile("" : "+v"(a))
#define HE_OPAQUE3(a, b, c) asm volatile("" : "+v"(a), "+v"(b), "+v"(c))
typedef float v2f __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld4(const GLOBAL v4f* p, int64_t k) {
    v4f x = p[k];
    return make_float4(x.x, x.y, x.z, x.w);
}
__device__ __forceinline__ float2 ld2(const GLOBAL v2f* p, int64_t k) {
    v2f x = p[k];
    return make_float2(x.x, x.y);
}
// GBM market tiles hold 12-B records (one dwordx3 per lane): tileA {S, C, P} (v is
// the handle's constant variance) and, below kGreeksInStepMinEnvs envs, tileB
// {call_delta, gamma, put_delta}.  The step kernel recomputes the lag return from S
// and the previous S, and from kGreeksInStepMinEnvs envs also the f32 obs greeks
// (greeks_fast, a function of S alone at constant v): the same f32 code the market
// kernel would run, so the same values.  Heston keeps 16-B {S, v, C, P} and
// {greeks, lag} records.
struct __attribute__((packed, aligned(4))) f3 {
    float x, y, z;
};
__device__ __forceinline__ float4 ld3A(const GLOBAL v4f* p, int64_t k, float v) {
    const GLOBAL f3* r = (const GLOBAL f3*)p + k;
    return make_float4(r->x, v, r->y, r->z);
}
__device__ __forceinline__ float4 ld3B(const GLOBAL v4f* p, int64_t k) {
    const GLOBAL f3* r = (const GLOBAL f3*)p + k;
    return make_float4(r->x, r->y, r->z, 0.0f);
}
__device__ __forceinline__ void st3(float4* p, int64_t k, float x, float y, float z) {
    GLOBAL f3* r = (GLOBAL f3*)p + k;
    r->x = x;
    r->y = y;
    r->z = z;
}

constexpr int kBlock = 256;      // step kernel: threads per workgroup (4 waves)
// step kernel: envs per wave (one per lane; 32 per wave, twice the waves, measured -10 % on the
// Gym-API path, r02s8)
constexpr int kEpw = 64;
constexpr int kEpb = (kBlock / 64) * kEpw; // step kernel: envs per workgroup
constexpr int kObs = HE_OBS_DIM;
constexpr int kMktEnvs = 32;     // market kernel: envs per workgroup (half a wave wide)
constexpr int kMktLanes = 8;     //                slot-lanes per env (4 waves, 16.6 KB LDS)
constexpr int kMaxBlock = 64;    // max market block length M
constexpr int kRolloutPrefetch = 4;  // rollout: steps of inputs in flight
// replay rollouts: steps of path rows in flight (config 6, same box: D = 4 585 us per 256-step
// launch, D = 8 574-576 us, r03s4)
constexpr int kReplayPrefetch = 8;
constexpr int kMktWaves = 2;  // market_kernel: min waves per SIMD (3 is faster alone, slower beside rollouts)
constexpr int64_t kPrefetchMinEnvs = 131072;  // auto prefetch for single steps from here
// GBM: obs greeks evaluated by the step kernel (no tileB) from this many envs.  A
// rollout wave at 65,536 envs (one wave per SIMD) pays the f32 greeks' dependent
// VALU latency in full (3.19e10 -> 2.88e10 env-steps/s), while at 1,048,576 envs the
// 12 bytes per env-step saved win (2.95e10 -> 3.68e10; MI355X, he_rollout K=64).
// (HE_GREEKS_IN_STEP_MIN_ENVS in the environment at he_create overrides it: tests, A/B)
constexpr int64_t kGreeksInStepMinEnvs = 262144;

// ------------------------------------------------------------------ parameters
// One option of the liability book (he_book_option), device copy: q100 = quantity*100.
struct BookOpt {
    int32_t type, expiry;
    double K, H, q100;
    double lnK, lnH, lnH2K;   // log K, log H, 2 log H - log K (host)
    double invK;              // 1 / K (host)
    double invH;              // 1 / H (host)
};

struct Params {
    int64_t n;
    int64_t goff;
    int32_t T;
    int32_t variant, loss, record_metrics, autoreset, mode;
    int32_t tile_greeks;    // GBM: the market kernel writes tileB {greeks} (else the step kernel evaluates them)
    int32_t mt, maxh;
    float mt_f, maxh_f, T_f;
    float inv_maxh_f, inv_T_f;  // RN_f32(1/x) for div_byf
    int32_t s0s_const;          // generate: max(S0, 25) is one constant for every env
    float s0s_f, inv_s0s_f;
    double s0s_d, inv_s0s_d;    // the same as f64 (div_f32_by)
    double inv_252;             // RN(1/252)
    float init_cash_f;
    double tcpc, slip_frac, lam, w, theta, initial_cash;
    double shares_d, inv_shares;  // inv_*: RN(1/x) for div_by
    float shares_f;
    int32_t shares_zero;
    // observation / greeks constants (hedging_env_v2.py:57-58)
    float r_f, tenor_f;
    double r_d, tenor_d, sqrt_tenor;
    int32_t tenor_small;    // tenor <= 1e-6
    // generate-mode market
    uint32_t key0, key1;
    double s0;
    double var;             // GBM variance (Heston v0)
    float var_f;
    double sqrt_var, drift, sqrt_dt, mu, dt;
    BSConst bs;             // constant-sigma BS constants (GBM)
    int32_t mark;           // he_mark of the generated C / P
    double fe_K;            // HE_MARK_FIXED_EUROPEAN: K = round(S0) (option_price_assignment.py:36)
    float g_sigma, g_num_drift;  // constant-variance greeks: sigma, (r+0.5 sigma**2)*T (f32)
    double g_sst;                // sigma*sqrt(T) (f64)
    double g_inv_sst;            // 1/(sigma*sqrt(T))
    float g_sst_f, g_inv_sst_f;  // f32 twins for greeks_fast
    float sqrt_tenor_f;
    double h_kappa, h_theta, h_xi, h_rho, h_sqrt1mrho2;
    int32_t den_const;      // generate: reward denominator of the shared S0 (all envs)
    double den, inv_den;
    int32_t M;              // market block length
    float4* tileA;          // [M+1][N] {S, v, C, P}; GBM: 12-B {S, C, P} records (ld3A)
    float4* tileB;          // [M+1][N] {call_delta, gamma, put_delta, lag}; GBM: 12-B {greeks} if tile_greeks
    float rstv[4 + kObs];   // reset market + obs (generate): {S0, v0, C0, P0, obs0[13]}, by value
    // replay
    const float4* rec;      // [n_paths][rstride] {S, v, C, P}, row t at rrow(p, path, t); C/P at T hold row T-1
    const float4* recg;     // [n_paths][rstride] {call_delta, gamma, put_delta, lag return}, same layout
    int64_t n_paths;
    int64_t rstride;        // rows per path in rec / recg: T + 1 + kRowOff rounded up to whole 128-B lines
    int32_t roff;           // row 0's slot in the path's stride (kRowOff)
    // liability book (generate modes)
    int32_t book_n;
    const BookOpt* book;    // device copy [book_n], read through the scalar cache
    const double* book_tab; // [m][4] = {sqrt(m dt), 1 / sqrt(m dt), exp(-r m dt), exp(r m dt)}, m = 0..max expiry
    int32_t book_rows;      // max expiry + 1
    double bk_sig, bk_isig, bk_s2, bk_lam;  // book_value's volatility terms at the constant variance
    double book_rst;        // book value of the reset market (t = 0, S0, v0)
    double* tileC;          // [M+1][N] f64 book value of every slot
#ifdef HE_TIMING
    uint64_t* tim;          // [5][8192][2]
#endif
};

// Replay table layout.  Row t of a path sits at slot kRowOff + t of a stride of whole 128-B
// lines (8 rows of 16 B), so rows 1..8, 9..16, ... -- the spans the LDS loaders read per
// 8-step block from an episode start, and their 4-row halves -- begin on a line whenever the
// block grid meets the episode at a multiple of 4 steps: always for T = 0 or 4 mod 8, e.g.
// the reference's T = 252, so no span straddles an extra line (1.15x traffic).
constexpr int32_t kRowOff = 7;
__host__ __device__ __forceinline__ int64_t replay_stride(int64_t T) { return ((T + 1 + kRowOff + 7) / 8) * 8; }
__device__ __forceinline__ int64_t rrow(const Params& p, int64_t path, int64_t t) {
    return path * p.rstride + p.roff + t;
}

struct State {
    uint32_t* t;
    uint32_t* pos;     // (uint16)call | (uint16)put << 16
    double* cash;
    int32_t* path;     // replay episode row
    float* s0;         // replay initial_S0_for_episode; -1 encodes the python 1.0 substitution
    uint64_t* pcg;     // replay [4][N]: state_hi, state_lo, inc_hi, inc_lo
    uint32_t* pcgb;    // replay [2][N]: has_uint32, uinteger
    double* acc;       // rollouts: [7][N] episode sums (reward, pnl, |ps|, tc, rpc, tcp, ps)
    uint32_t* acc_len; // rollouts: [N] episode length so far
    float* last;       // [4][N] the last finished episode {return, sum pnl, sum cost, length}
    double* sum;       // generate-mode rollouts: [3][N] running {return, sum pnl, sum cost}
    uint32_t* sum_len; // generate-mode rollouts: [N] running episode length
};

// Generate-mode market position of every env: `cur` = after the last generated
// block (or the reset state), `bak` = start of that block (for rewinds).
struct Market {
    uint32_t* ep;      // episode counter (0xFFFFFFFF before the first reset)
    uint32_t* t;       // step in episode, 0..T (T = terminal, next step resets)
    double* S;         // f64 price
    double* v;         // f64 variance (Heston)
    float* C;          // f32 marks at this position
    float* P;
    double* M;         // book: running max of S over the episode (barrier monitor)
};

// he_rollout_policy: device policy instead of an action input, episode records out
struct PolIo {
    int32_t policy;                 // he_policy
    float* act_out;                 // [K][N][2] or NULL
    he_episode_record* rec;         // [cap]
    int64_t cap;
    unsigned long long* count;
};

struct Io {
    const float* act;  // [K][N][2]
    float* obs;        // [K][N][13]
    float* rew;        // [K][N]
    uint8_t* term;     // [K][N]
    uint8_t* trunc;    // [N]
    float* tobs;       // [N][13]
    he_info info;
    PolIo pol;
    bool pol_on;
    bool sums;         // he_rollout: keep the episode summaries (State::sum / last)
    // he_step_signal (he_step only): the step's sequence number stored into `sig` (host-mapped)
    // after every output of the launch; `sig_cnt` counts the workgroups done (device word)
    uint32_t* sig;
    uint32_t* sig_cnt;
    uint32_t sig_seq;
};

struct Mkt {
    float S, v, C, P;
    double B;          // liability book value (0 without a book)
};

struct Env {
    uint32_t t;
    int32_t call, put;
    double cash;
    int32_t path;
    float s0;          // initial_S0_for_episode as f32 (1.0 when substituted)
    bool s0_small;
    // replay LDS steppers (EP): the episode's quotient constants (replay_episode_consts)
    double s0s_d, inv_s0s_d;  // max(S0, 25) of the obs prices (inf as DBL_MAX) and RN(1/.)
    float s0s_f, inv_s0s_f;   // the same in f32, RN32(1/.): the FAST replay obs (lds_replay_stepper)
    double den;               // the reward denominator
};

// The per-episode divisors of a replay env (hedging_env_v2.py:120-122 obs prices,
// :243-256 reward), computed at the episode's reset: max(S0, 25) of the obs prices with
// its RN reciprocal, so the obs take the correctly rounded Markstein quotient
// (div_f32_by, make_obs's value; an infinite max(S0, 25) is held as DBL_MAX, so
// div_f32_by gives a·0 = ±0 like a / inf), and step_env's reward denominator (FAST:
// loss != mse, a select-only expression).
template <bool FAST>
__device__ __forceinline__ double replay_den(const Params& p, float s0, bool small) {
    const float f = np_maxf(s0, 25.0f);
    const double da = small ? (25.0 + 1e-9) : (double)(f + 1e-9f);
    if (FAST) return da;
    const double dm = small ? (625.0 + 1e-9) : (double)(f * f + 1e-9f);
    return (p.loss == HE_LOSS_MSE) ? dm : da;
}
template <bool FAST = false>
__device__ __forceinline__ void replay_episode_consts(const Params& p, Env& e) {
    const float f = np_maxf(e.s0, 25.0f);
    const double fd = (double)f;
    e.s0s_d = (fd == __builtin_inf()) ? 1.7976931348623157e308 : fd;
    e.inv_s0s_d = 1.0 / fd;
    e.s0s_f = f;
    e.inv_s0s_f = 1.0f / f;
    e.den = replay_den<FAST>(p, e.s0, e.s0_small);
}


__device__ __forceinline__ int32_t unpack_lo(uint32_t p) { return (int32_t)(int16_t)(p & 0xFFFFu); }
__device__ __forceinline__ int32_t unpack_hi(uint32_t p) { return (int32_t)(int16_t)(p >> 16); }
__device__ __forceinline__ uint32_t pack_pos(int32_t c, int32_t q) {
    return ((uint32_t)(uint16_t)(int16_t)c) | (((uint32_t)(uint16_t)(int16_t)q) << 16);
}
__device__ __forceinline__ Mkt as_mkt(float4 r) { return Mkt{r.x, r.y, r.z, r.w}; }

// ------------------------------------------------------------------ greeks
// hedging_env_v2.py:79-107 on the f32 price S and variance v; returns the three
// f32 obs values (call_delta, gamma, put_delta).
template <bool CONST_VAR>
__device__ __forceinline__ float4 greeks(const Params& p, float S, float v) {
    double cd, gam, pd;
    float K = rintf(S);  // np.round: half-even
    if (S <= 1e-6f) {    // weak python 1e-6 compares as float32(1e-6)
        cd = (K == 0.0f) ? 0.5 : ((K > 0.0f) ? 0.0 : 1.0);
        pd = (K == 0.0f) ? -0.5 : ((K < 0.0f) ? 0.0 : -1.0);
        gam = 0.0;
    } else {
        float sigma, num_drift;
        double sst;
        if (CONST_VAR) {
            sigma = p.g_sigma;
            num_drift = p.g_num_drift;
            sst = p.g_sst;
        } else {
            sigma = sqrtf(np_maxf(v, 1e-8f));
            num_drift = (p.r_f + 0.5f * (sigma * sigma)) * p.tenor_f;
            sst = (double)sigma * p.sqrt_tenor;
        }
        if (p.tenor_small || sigma <= 1e-6f) {
            cd = (S > K) ? 1.0 : ((S == K) ? 0.5 : 0.0);
            pd = (S < K) ? -1.0 : ((S == K) ? -0.5 : 0.0);
            gam = 0.0;
        } else {
            float Kc = np_maxf(K, 1e-6f);
            float num = logf(S / Kc) + num_drift;
            double d1;
            if (sst < 1e-9) {
                float sg = (num > 0.0f) ? 1.0f : ((num < 0.0f) ? -1.0f : num);  // np.sign
                d1 = (double)(sg * 10.0f);
            } else {
                d1 = CONST_VAR ? (double)num * p.g_inv_sst : (double)num / sst;
            }
            double n1 = ndtr(d1);
            cd = n1;
            pd = n1 - 1.0;
            double gd = (double)S * sst;
            gam = (fabs(gd) < 1e-9) ? 0.0 : norm_pdf(d1) / gd;
        }
    }
    return make_float4((float)cd, (float)gam, (float)pd, 0.0f);
}

// Phi(-|d1|) for the f32 obs greeks, given ph = phi(d1) (which gamma needs anyway):
// ph * R(|d1|), R the Mills ratio sqrt(pi/2) erfcx(a/sqrt2), evaluated as w P(w) with
// w = 2 / (a + 2) and P a degree-10 least-squares fit over a in [0, 14] (phi underflows
// f32 beyond).  One rcp and 11 FMAs on top of the shared exp instead of erfcf's own
// exp and branchy rational approximations.  Error of the f32 evaluation: relative
// < 4.8e-7 where the tail is > 0.1, < 1.3e-6 below it, absolute < 2.2e-7 -- inside the
// obs tolerance (OBS_RTOL 1e-6, OBS_ATOL 1e-7) against the reference's f64 ndtr.
__device__ __forceinline__ float ncdf_tail(float d1, float ph) {
    const float a = fminf(fabsf(d1), 14.0f);
    const float w = 2.0f * __builtin_amdgcn_rcpf(a + 2.0f);
    float r = -2.690903097e-02f;
    r = fmaf(r, w, 6.361111253e-02f);
    r = fmaf(r, w, 2.313483953e-01f);
    r = fmaf(r, w, -1.219161630e+00f);
    r = fmaf(r, w, 2.182162046e+00f);
    r = fmaf(r, w, -1.785471797e+00f);
    r = fmaf(r, w, 4.304344356e-01f);
    r = fmaf(r, w, -1.690988056e-02f);
    r = fmaf(r, w, 3.958457112e-01f);
    r = fmaf(r, w, 4.983069301e-01f);
    r = fmaf(r, w, 5.000579357e-01f);
    return ph * (r * w);
}

// Generate-mode obs greeks (market_kernel): same branches and the same f32 d1
// numerator as greeks(), the rest in f32 instead of f64-then-cast.  N(d1) - 1 is
// taken as -N(-d1) (no cancellation, ncdf_tail sharing gamma's exp), 1/(S sigma sqrt T)
// through v_rcp_f32.  Within OBS_RTOL 1e-6 / OBS_ATOL 1e-7 of the reference's f64
// values (tests, columns 7-10) at well under a third of the cost of the f64 chain
// (measured: greeks were 32% of market_kernel; ncdf_tail in place of erfcf took
// 10-15 us off the headline launch, r04s3).  Replay tables and the reset obs keep
// greeks() (replay_greeks).
template <bool CONST_VAR>
__device__ __forceinline__ float4 greeks_fast(const Params& p, float S, float v) {
    float cd, gam, pd;
    const float K = rintf(S);
    if (S <= 1e-6f) {
        cd = (K == 0.0f) ? 0.5f : ((K > 0.0f) ? 0.0f : 1.0f);
        pd = (K == 0.0f) ? -0.5f : ((K < 0.0f) ? 0.0f : -1.0f);
        gam = 0.0f;
    } else {
        float sigma, num_drift, sstf;
        double sst;
        if (CONST_VAR) {
            sigma = p.g_sigma;
            num_drift = p.g_num_drift;
            sst = p.g_sst;
            sstf = p.g_sst_f;
        } else {
            sigma = sqrtf(np_maxf(v, 1e-8f));
            num_drift = (p.r_f + 0.5f * (sigma * sigma)) * p.tenor_f;
            sst = (double)sigma * p.sqrt_tenor;
            sstf = (float)sst;
        }
        if (p.tenor_small || sigma <= 1e-6f) {
            cd = (S > K) ? 1.0f : ((S == K) ? 0.5f : 0.0f);
            pd = (S < K) ? -1.0f : ((S == K) ? -0.5f : 0.0f);
            gam = 0.0f;
        } else {
            const float Kc = np_maxf(K, 1e-6f);
            const float num = logf(S / Kc) + num_drift;   // f32 in the reference too
            float d1;
            if (sst < 1e-9) {
                const float sg = (num > 0.0f) ? 1.0f : ((num < 0.0f) ? -1.0f : num);
                d1 = sg * 10.0f;
            } else {
                d1 = CONST_VAR ? num * p.g_inv_sst_f : num * __builtin_amdgcn_rcpf(sstf);
            }
            // N(d1) = Phi(d1) and N(d1) - 1 = -Phi(-d1): evaluate the small tail Phi(-|d1|)
            // (accurate) and take the other as 1 - tail (>= 1/2, no cancellation)
            const float ph = expf(-0.5f * (d1 * d1)) * 0.398942280401432678f;
            const float tail = ncdf_tail(d1, ph);
            cd = (d1 >= 0.0f) ? 1.0f - tail : tail;
            pd = (d1 >= 0.0f) ? -tail : tail - 1.0f;
            const float gd = S * sstf;
            gam = (fabsf(gd) < 1e-9f) ? 0.0f : ph * __builtin_amdgcn_rcpf(gd);
        }
    }
    return make_float4(cd, gam, pd, 0.0f);
}

// The obs greeks of a replay row (table_greeks_kernel at load, the replay LDS loaders per
// row): greeks(), the reference's f64 chain.  (greeks_fast at the row's own variance was
// A/B-tested: the loaders' busy cycles drop, config 6 does not move -- r03s18.)
__device__ __forceinline__ float4 replay_greeks(const Params& p, float S, float v) {
    return greeks<false>(p, S, v);
}

// greeks_fast<true> for the lean LDS obs stepper: the handle's sigma, tenor and sst are
// normal (lds_lean_config), so the uniform branches are gone, and the S <= 1e-6 case is
// a select over the main path's result (which it computes for every lane) instead of a
// divergent if/else.  Same operations and operands, so the same bits as greeks_fast<true>.
// The select operands are made opaque (asm): left alone, the backend turns the nested
// constant selects and the gamma quotient into exec-mask branches -- five per step in the
// obs stepper's block, which split the unrolled steps into separate basic blocks.
// a / b, f32, as the correctly rounded division's lowering computes it (v_rcp_f32, a Newton step,
// the quotient and two residual corrections) without its v_div_scale / v_div_fixup: those change
// nothing when a, b and a / b are normal and far from the exponent range's ends, as in the lean
// obs stepper's two quotients -- S / max(rint S, 1e-6) (within a factor 2 of 1 for S >= 0.5,
// below 5e5 under it) and (S - Sp) / Sp (0 or >= 2^-23 in magnitude) with S, Sp >= 1e-8.
// An inf dividend is NOT the IEEE quotient here (a - b q = inf - inf = NaN): callers keep the
// dividend finite (lag_return_lean caps it, greeks_lean's S / rint(S) is NaN for an inf S in IEEE
// too).  The lean LDS steppers against the
// tile kernels' IEEE divisions: bit for bit (test_lds_rollout_equals_tile_rollout and the suite);
// headline 280.8 -> 277.0 us per launch, 3 of 3 same-box pairs (r05s22_ab_div_core.txt).
__device__ __forceinline__ float div_f32_core(float a, float b) {
    float r = __builtin_amdgcn_rcpf(b);
    r = fmaf(fmaf(-b, r, 1.0f), r, r);
    float q = a * r;
    q = fmaf(fmaf(-b, q, a), r, q);
    return fmaf(fmaf(-b, q, a), r, q);
}

// logf for x >= FLT_MIN (or inf / NaN): ocml's logf -- v_log_f32, then the product with ln 2 in
// two parts -- without the denormal scaling it skips there (the same operations, the same bits;
// with expf_nonpos: headline 270.3 -> 267.4 us, 3 of 3 same-box pairs, r05s28_ab_log_exp.txt)
__device__ __forceinline__ float logf_normal(float x) {
    const float r = __builtin_amdgcn_logf(x);
    const float hi = r * 0x1.62e42ep-1f;
    float t = fmaf(r, 0x1.62e42ep-1f, -hi);
    t = fmaf(r, 0x1.efa39ep-25f, t);
    return (fabsf(r) < __builtin_inff()) ? hi + t : r;
}
// expf for x <= 0 (or NaN): ocml's expf without its overflow select (never taken there)
__device__ __forceinline__ float expf_nonpos(float x) {
    const float hi = x * 0x1.715476p+0f;
    float t = fmaf(x, 0x1.715476p+0f, -hi);
    const float k = rintf(hi);
    t = fmaf(x, 0x1.4ae0bep-26f, t);
    const float e = __builtin_amdgcn_exp2f((hi - k) + t);
    const float v = ldexpf(e, (int)k);
    return (x >= -0x1.9d1da0p+6f || x != x) ? v : 0.0f;
}

__device__ __forceinline__ float4 greeks_lean(float S, float num_drift, float inv_sst_f, float sstf) {
    const float K = rintf(S);
    const float Kc = np_maxf(K, 1e-6f);
    const float num = logf_normal(div_f32_core(S, Kc)) + num_drift;   // f32 in the reference too
    const float d1 = num * inv_sst_f;
    const float ph = expf_nonpos(-0.5f * (d1 * d1)) * 0.398942280401432678f;
    const float tail = ncdf_tail(d1, ph);
    float cd = (d1 >= 0.0f) ? 1.0f - tail : tail;
    float pd = (d1 >= 0.0f) ? -tail : tail - 1.0f;
    const float gd = S * sstf;
    float ge = ph * __builtin_amdgcn_rcpf(gd);
    float ct = (K == 0.0f) ? 0.5f : ((K > 0.0f) ? 0.0f : 1.0f);
    float pt = (K == 0.0f) ? -0.5f : ((K < 0.0f) ? 0.0f : -1.0f);
    HE_OPAQUE3(ge, ct, pt);
    float gam = (fabsf(gd) < 1e-9f) ? 0.0f : ge;
    const bool tiny = S <= 1e-6f;  // weak python 1e-6 compares as float32(1e-6)
    cd = tiny ? ct : cd;
    pd = tiny ? pt : pd;
    gam = tiny ? 0.0f : gam;
    return make_float4(cd, gam, pd, 0.0f);
}

// np.clip(n, -maxh, maxh) of the steppers' positions (maxh >= 0, he_create): one v_med3_i32 (the
// compiler made v_min_i32 + a compare + a select of it; headline 271.4 -> 268.7 us, 3 of 3
// same-box pairs, r05s30_ab_pos_med3.txt)
__device__ __forceinline__ int32_t clamp_pos(int32_t n, int32_t maxh) {
    int32_t r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(n), "v"(-maxh), "v"(maxh));
    return r;
}

// ------------------------------------------------------------------ observation
// S_t / S_{t-1} - 1 clipped to +-1, 0 when S_{t-1} == 0 (hedging_env_v2.py:129-136):
// a function of the market alone, so it is computed where the market is (market_kernel
// slots, replay table load) and travels in the .w lane of the greeks record.
__device__ __forceinline__ float lag_return(float S, float Sp) {
    float q = (S - Sp) / Sp;  // for every lane (opaque): a select, not a branch around the division
    HE_OPAQUE1(q);
    return (Sp == 0.0f) ? 0.0f : np_clipf(q, -1.0f, 1.0f);
}

// lag_return for the lean obs stepper (S, Sp >= 1e-8): the quotient by div_f32_core, its
// dividend capped at Sp -- every (S - Sp) / Sp >= 1 clips to 1 and Sp / Sp = 1 exactly, so the
// value is the same, and an infinite S (an f32 overflow of the f64 price) gives the reference's
// clip(inf) = 1 instead of div_f32_core's inf - inf = NaN; a NaN stays NaN (the compare is false)
__device__ __forceinline__ float lag_return_lean(float S, float Sp) {
    const float d = S - Sp;
    float q = div_f32_core((d > Sp) ? Sp : d, Sp);
    HE_OPAQUE1(q);
    return (Sp == 0.0f) ? 0.0f : np_clipf(q, -1.0f, 1.0f);
}

// hedging_env_v2.py:109-143.  m = market after the step, g = its greeks and, in g.w,
// lag_return(m.S, Sp); Sp/vp = S_t_minus_1 / v_t_minus_1.  Quotients by per-handle
// constants use div_byf (correctly rounded, 3 instructions).
// FAST: the hot configuration is known at compile time (see fast_config()):
// generate mode, record_metrics, max_contracts_held > 0, T > 0.
template <bool FAST = false, bool EP = false>
__device__ __forceinline__ void make_obs(const Params& p, const Env& e, const Mkt& m, float4 g, float Sp,
                                         float vp, float* o) {
    if (EP) {  // the episode's max(S0, 25) (replay_episode_consts)
        o[0] = div_f32_by(m.S, e.s0s_d, e.inv_s0s_d);
        o[1] = div_f32_by(m.C, e.s0s_d, e.inv_s0s_d);
        o[2] = div_f32_by(m.P, e.s0s_d, e.inv_s0s_d);
    } else if (FAST || p.s0s_const) {
        o[0] = div_f32_by(m.S, p.s0s_d, p.inv_s0s_d);
        o[1] = div_f32_by(m.C, p.s0s_d, p.inv_s0s_d);
        o[2] = div_f32_by(m.P, p.s0s_d, p.inv_s0s_d);
    } else {
        float s0s = np_maxf(e.s0, 25.0f);
        o[0] = m.S / s0s;
        o[1] = m.C / s0s;
        o[2] = m.P / s0s;
    }
    // int64/int -> f64 quotient cast to f32 == correctly rounded f32 quotient when
    // both operands are exact in f32 (|x| < 2^24) and 53 >= 2*24+2 (no double rounding)
    if (FAST || p.maxh != 0) {
        o[3] = div_int_byf((float)e.call, p.maxh_f, p.inv_maxh_f);
        o[4] = div_int_byf((float)e.put, p.maxh_f, p.inv_maxh_f);
    } else {
        o[3] = 0.0f;
        o[4] = 0.0f;
    }
    o[5] = m.v;
    o[6] = (FAST || p.T != 0) ? div_int_byf((float)(p.T - (int32_t)e.t), p.T_f, p.inv_T_f) : 0.0f;
    if (FAST || p.record_metrics) {
        o[7] = g.x;
        o[8] = g.y;
        o[9] = g.z;
        o[10] = g.y;
    } else {
        o[7] = o[8] = o[9] = o[10] = 0.0f;
    }
    const bool first = e.t == 0;  // reset obs
    o[11] = first ? 0.0f : g.w;
    o[12] = (first || Sp == 0.0f) ? 0.0f : np_clipf(m.v - vp, -1.0f, 1.0f);
}

// ------------------------------------------------------------------ marks
// f64 Black-Scholes marks of the market at episode step t, handed to the env as f32.
// HE_MARK_ROLLING_ATM: the 30-day option at K = round(S) (rbergomi_sim.py:418,437-446).
// HE_MARK_FIXED_EUROPEAN (FE = true: the kernel tests p.mark, a uniform branch): the
// episode's option struck at round(S0) with T = max(1 - t/252, 0) years left, through
// black_scholes_vectorized (option_price_assignment.py:10-21,36-38).
template <int MODE, bool FE = true>
__device__ __forceinline__ void marks(const Params& p, double S64, double var64, uint32_t t, float* C, float* P) {
    double c, q;
    if (FE && p.mark == HE_MARK_FIXED_EUROPEAN) {
        // np.clip(1 - time_grid / 252, 0, None): t / 252 correctly rounded (div_int_by)
        const double tau = 1.0 - div_int_by((double)t, 252.0, p.inv_252);
        const double sig = (MODE == HE_MODE_HESTON) ? sqrt(var64 < 0.0 ? 0.0 : var64) : p.sqrt_var;
        bs_vectorized(S64, p.fe_K, tau < 0.0 ? 0.0 : tau, p.r_d, sig, &c, &q);
        *C = (float)c;
        *P = (float)q;
        return;
    }
    double K = rint(S64);
    if (MODE == HE_MODE_HESTON) {
        BSConst h;
        double sig = sqrt(var64 < 0.0 ? 0.0 : var64);
        h.intrinsic = (p.tenor_d <= 0.0) || (sig <= 0.0);
        h.a = (p.r_d + 0.5 * (sig * sig)) * p.tenor_d;
        h.b = sig * p.sqrt_tenor;
        h.inv_b = 1.0 / h.b;
        h.disc = p.bs.disc;
        bs_call_put(S64, K, h, &c, &q);
    } else {
        bs_call_put(S64, K, p.bs, &c, &q);
    }
    *C = (float)c;
    *P = (float)q;
}

// ------------------------------------------------------------------ liability book
// Extension (he_book_option, BASELINE.json configs[3]/[4]).  Option o at the env's
// market S with volatility sig, tau years to expiry, runmax = max S over the episode
// at the step dates so far.  Europeans: the OptionCalculator.black_scholes_price form
// (option_calculator.py:11-27, intrinsic when tau <= 0 or sig <= 0).  Up-and-out call
// (q = 0, Hull, "Options, Futures and Other Derivatives", barrier options):
// c_uo = c - c_ui, worthless once S touched H at a step date or when H <= K.
// tab[m] = {sqrt(m dt), 1 / sqrt(m dt), exp(-r m dt), exp(r m dt)} (tau = m dt as in book_option)
__global__ void book_tab_kernel(double* tab, int32_t n, double dt, double r) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= n) return;
    const double tau = (double)m * dt;
    const double sq = sqrt(tau);
    tab[4 * m] = sq;
    tab[4 * m + 1] = 1.0 / sq;
    tab[4 * m + 2] = exp(-r * tau);
    tab[4 * m + 3] = exp(r * tau);
}

// Per env-step constants shared by the book's options: log S once (log(S/K) =
// log S - log K), 1/sigma, and lam of the barrier formula; per option the
// tau-dependent sqrt(tau), 1/sqrt(tau), exp(-r tau) and exp(r tau) come from a table
// indexed by the remaining steps m = expiry - t (tau = m dt, the same f64 product).
struct BookEnv {
    double S, lnS, sig, isig, s2, lam;
};

// The normal tail Q(a) = Phi(-a), a >= 0, as phi(a) R(a) with the Mills ratio
// R(a) = sqrt(pi/2) erfcx(a / sqrt 2) a degree-14 polynomial in u = A - B / (a + c), c = 5:
// the Chebyshev fit on a in [0, 38.6] (Q underflows past it) re-expanded in powers of u
// (coefficients below 0.39 in magnitude, so Horner loses nothing), 5.2e-11 relative on Q
// against scipy.special.ndtr (tools/mills_fit.py).  The producers of the book kernels are
// bound by VALU issue, so the degree is what costs: degree 16 (1.7e-12) against the former 20
// at c = 3.5 (2.6e-13) took config 4 8.77 -> 8.34 ms (r03s37); degree 14 against 16 config 4
// 6.85 -> 6.65 ms, config 5 1.53 -> 1.51 ms (r04t2_ab_mills_deg14.txt, book / full-size /
// randomised parity green), the book's P&L still far inside north_star's 1e-5.  Branch-free -- every lane of a wave
// runs the same instructions whatever its d -- and phi is the caller's: d1 and d2 of a
// Black-Scholes price share one exp (S phi(d1) = K e^{-r tau} phi(d2)).  Replaces two
// library erfc per pair, each with its own exp and range branches (the book is an
// extension without a reference; its bar is the oracle's P&L at 1e-5, test_gpu_parity.py).
constexpr double kMillsA = 1.2590673575129534, kMillsB = 11.295336787564768, kMillsC = 5.0;
constexpr double kMillsMax = 37.4;                       // phi(37.4) ~ 1e-304: the tail is 0 past it
constexpr double kInvSqrt2Pi = 0.39894228040143267794;
// the degree-14 polynomial of mills() in u
__device__ __forceinline__ double mills_u(double u) {
    double r = -2.8897932893921865e-07;
    r = fma_k(r, u, 9.2037477055214229e-08);
    r = fma_k(r, u, 4.205888988230914e-06);
    r = fma_k(r, u, -6.0256457018679174e-06);
    r = fma_k(r, u, -4.0951820297551139e-05);
    r = fma_k(r, u, 0.00016918165349102241);
    r = fma_k(r, u, 4.302225968256142e-05);
    r = fma_k(r, u, -0.0026776117165782177);
    r = fma_k(r, u, 0.013231545706850733);
    r = fma_k(r, u, -0.041271310285367596);
    r = fma_k(r, u, 0.097294624847109032);
    r = fma_k(r, u, -0.18472286911363267);
    r = fma_k(r, u, 0.29086958410834113);
    r = fma_k(r, u, -0.38520383403508307);
    r = fma_k(r, u, 0.2382000181985946);
    return r;
}
__device__ __forceinline__ double mills(double a) {
#if HE_BOOK_DIAG == 1
    return a * 0.25;  // diagnostic builds only (tools/gpu): the book without its tails
#endif
    const double d = a + kMillsC;                        // in [3.5, 41]: no special cases
    // v_rcp_f64 is within 4.7e-8 of 1 / d on [3.5, 43], one Newton step within 2.3e-15
    // (tools/probe/rcp_f64.hip, profiles/r04s3_rcp_f64.txt): u = A - B y then carries
    // ~5e-15 against the fit's 5e-11, so the second step (exact rounding) buys nothing
    double y = __builtin_amdgcn_rcp(d);
    y = fma(fma(-d, y, 1.0), y, y);
    return mills_u(fma(-kMillsB, y, kMillsA));
}
// mills() of an option's two tails with one reciprocal: 1 / (d1 d2) by v_rcp_f64 and one Newton
// step, then 1 / d1 = d2 / (d1 d2) and 1 / d2 = d1 / (d1 d2) (within 3e-15; the f64 reciprocal
// is a quarter-rate transcendental, two per option before): config 4 6.86 -> 6.82 ms, config 5
// 1.532 -> 1.524 ms, 3 of 3 same-box pairs (r04s9_ab_mills2.txt)
// SEQ: the two polynomials one after the other (the barrier formula's tail pairs: interleaved,
// they spilled the Heston producers' registers)
template <bool SEQ = false>
__device__ __forceinline__ void mills2(double a1, double a2, double* r1, double* r2) {
#if HE_BOOK_DIAG == 1
    *r1 = mills(a1);
    *r2 = mills(a2);
#else
    const double d1 = a1 + kMillsC, d2 = a2 + kMillsC;
    const double P = d1 * d2;
    double Y = __builtin_amdgcn_rcp(P);
    Y = fma(fma(-P, Y, 1.0), Y, Y);
    const double u2 = fma(-kMillsB, d1 * Y, kMillsA);
    *r1 = mills_u(fma(-kMillsB, d2 * Y, kMillsA));
    if (SEQ) __builtin_amdgcn_sched_barrier(0);
    *r2 = mills_u(u2);
#endif
}

// |d| clamped to the range of the fit, and its phi
__device__ __forceinline__ double tail_arg(double d) {
    const double a = fabs(d);
    return a < kMillsMax ? a : kMillsMax;                // NaN -> kMillsMax (the price is NaN anyway)
}
// exp(x) for the book's phi, x = -a^2 / 2 in [-700, 0] (a <= kMillsMax): exp_k's Cody-Waite
// reduction, then e^r as a degree-9 near-minimax polynomial on |r| <= ln2 / 2 (1.7e-14
// relative, a Lawson-weighted Chebyshev fit; the book's bar is 1e-5 on P&L) without the
// Fast2Sum or the range branch.  Round 4 against the degree-11 Taylor form (7e-15): config 4
// 6.65 -> 6.60 ms, config 5 1.503 -> 1.497 ms, 3 of 3 pairs (r04t3_ab_exp_minimax.txt; an A/B
// of the same change on an earlier tree was mixed, r04s3_ab_exp_book_minimax.txt).
__device__ __forceinline__ double exp_book(double x) {
    const double k = rint(x * 1.4426950408889634074);
    const double rh = fma_kb(-k, 6.93147180369123816490e-01, x);
    const double r = fma_kb(-k, 1.90821492927058770002e-10, rh);
    double q = 2.7474189376171111e-06;
    q = fma_k(q, r, 2.4883220877841942e-05);
    q = fma_k(q, r, 0.00019841609921119712);
    q = fma_k(q, r, 0.0013888804743864306);
    q = fma_k(q, r, 0.0083333330025783942);
    q = fma_k(q, r, 0.041666667017783966);
    q = fma_k(q, r, 0.16666666667764135);
    q = fma_k(q, r, 0.49999999999494837);
    q = fma_k(q, r, 0.99999999999990008);
    q = fma_k(q, r, 1.0000000000000104);
    return ldexp(q, (int)k);
}
// exp_book with exp_k's range guard, for the barrier formula's (H/S) powers (any sign,
// +-inf when S is 0 or inf): config 5 1.93 -> 1.89 ms per launch against exp_k (r03s44)
__device__ __forceinline__ double exp_book_g(double x) {
    if (!(fabs(x) < 700.0)) return exp(x);
    return exp_book(x);
}
// phi through exp_book: config 4 8.35 -> 7.74 ms, config 5 2.00 -> 1.94 ms against exp_k (r03s41)
__device__ __forceinline__ double phi_of(double a) { return exp_book(-0.5 * (a * a)) * kInvSqrt2Pi; }

// N(d) and N(-d) from the tail q = Q(|d|), as selects.  (0.5 -+ sign(d) (0.5 - q) is two
// instructions fewer per pair, but returns the small tail as 0.5 - (0.5 - q), an absolute
// 2^-54 error the barrier formula's (H/S)^(2 lam) factors push past the 1e-5 P&L bar, r03s40.)
__device__ __forceinline__ void ncdf_from_tail(double d, double q, double* pos, double* neg) {
    const bool p = d > 0.0;
    *pos = p ? 1.0 - q : q;
    *neg = p ? q : 1.0 - q;
}

// The value of a book option past its expiry (or at zero volatility): the intrinsic value, and a
// knocked-out up-and-out call 0 -- book_option's expressions for a lane that is not live.
__device__ __forceinline__ double book_option_intrinsic(const BookOpt& o, double S, double runmax) {
    double v;
    if (o.type == HE_BOOK_PUT) {
        const double ip = o.K - S;
        v = (ip < 0.0) ? 0.0 : ip;
    } else {
        const double ic = S - o.K;
        v = (ic < 0.0) ? 0.0 : ic;
        if (o.type == HE_BOOK_UO_CALL) v = (runmax >= o.H) ? 0.0 : v;
    }
    return (v < 0.0) ? 0.0 : v;
}

// One book option (branch-free in the lane-varying quantities: remaining steps, running max).
__device__ __forceinline__ double book_option(const Params& p, const BookOpt& o, const BookEnv& b, int32_t m,
                                              double runmax, const double* tab) {
    const double K = o.K, S = b.S, r = p.r_d;
    const bool live = m > 0 && b.sig > 0.0;             // tau = m dt > 0 (else intrinsic)
    // no lane of the wave before the option's expiry: its value is the intrinsic one on every lane,
    // so the pricer is skipped (the same bits).  Episodes of a fixed length keep a wave's envs in
    // step, so an option of the book past its expiry is past it on the whole wave (config 4's
    // expiries 63 / 126 / 189 / 252: 3 of 8 options expired at an average step).
    if (__ballot(live) == 0ull) return book_option_intrinsic(o, S, runmax);
    const int32_t mc = live ? m : 1;                    // a valid table row either way
    const double tau = (double)mc * p.dt;
    const double* e = tab + 4 * mc;
    const double sst = b.sig * e[0];
    const double isst = b.isig * e[1];
    const double d1 = ((b.lnS - o.lnK) + (r + 0.5 * b.s2) * tau) * isst;
    const double d2 = d1 - sst;
    const double Kd = K * e[2];
    const double SoKd = S * (o.invK * e[3]);            // S / (K e^{-r tau}) = phi(d2) / phi(d1)
    const double a1 = tail_arg(d1), a2 = tail_arg(d2);
    const double ph1 = phi_of(a1);
    double m1_, m2_;
    mills2(a1, a2, &m1_, &m2_);
    const double q1 = ph1 * m1_, q2 = (ph1 * SoKd) * m2_;
    double n1, m1, n2, m2;
    ncdf_from_tail(d1, q1, &n1, &m1);
    ncdf_from_tail(d2, q2, &n2, &m2);
    double v;
    if (o.type == HE_BOOK_PUT) {                         // o.type: uniform over the wave
        v = Kd * m2 - S * m1;
        const double ip = K - S;
        v = live ? v : ((ip < 0.0) ? 0.0 : ip);
    } else {
        v = S * n1 - Kd * n2;
        if (o.type == HE_BOOK_UO_CALL) {
            // c_uo = c - c_ui (Hull); the tails of x1 - sst, y - sst, y1 - sst from those of
            // x1, y, y1 (phi(x - sst) = phi(x) exp(x sst - sst^2 / 2))
            const double ls = b.lam * sst;
            const double lhs = o.lnH - b.lnS;                    // log(H / S)
            const double x1 = -lhs * isst + ls;                  // log(S / H) / sst + lam sst
            const double y = (o.lnH2K - b.lnS) * isst + ls;      // log(H^2 / (S K)) / sst + lam sst
            const double y1 = lhs * isst + ls;
            const double ert = e[3];                             // e^{r tau}
            // S / H as a product (one exp_book_g less per option and slot than exp(log S - log H):
            // the up-and-out call is the whole book of config 5); S = 0 or inf gives 0 or inf as
            // the exp did
            const double sh = S * o.invH;
            // H / S as 1 / (S / H): v_rcp_f64 and two Newton steps (1 ulp) instead of a second
            // exp_book; past |lhs| = 700 (S at 0 or inf) the library exp, as exp_book_g
            double hs;
            if (fabs(lhs) < 700.0) {
                double y = __builtin_amdgcn_rcp(sh);
                y = fma(fma(-sh, y, 1.0), y, y);
                hs = fma(fma(-sh, y, 1.0), y, y);
            } else {
                hs = exp(lhs);
            }
            const double p2l = exp_book_g((2.0 * b.lam) * lhs);  // (H/S)^(2 lam)
            const double p2l2 = p2l * (sh * sh);                 // (H/S)^(2 lam - 2)
            // the three tail pairs one after another (scheduling fences): interleaved, their
            // six Mills polynomials' live ranges spilled the Heston producers' registers.  The
            // expression is unchanged (same operations, same order): the same bits.
            __builtin_amdgcn_sched_barrier(0);
            double nx, mx, nx_, mx_, ny, my, ny_, my_, ny1, my1, ny1_, my1_;
            {
                const double ax = tail_arg(x1), ax_ = tail_arg(x1 - sst);
                const double px = phi_of(ax);
                double r_, r__;
                mills2<true>(ax, ax_, &r_, &r__);
                const double qx = px * r_, qx_ = (px * (sh * ert)) * r__;
                ncdf_from_tail(x1, qx, &nx, &mx);
                ncdf_from_tail(x1 - sst, qx_, &nx_, &mx_);
            }
            const double t1 = S * nx - Kd * nx_;
            __builtin_amdgcn_sched_barrier(0);
            {
                const double ay = tail_arg(y), ay_ = tail_arg(y - sst);
                const double py = phi_of(ay);
                double r_, r__;
                mills2<true>(ay, ay_, &r_, &r__);
                const double qy = py * r_, qy_ = (py * ((hs * hs) * (S * o.invK) * ert)) * r__;
                ncdf_from_tail(y, qy, &ny, &my);
                ncdf_from_tail(y - sst, qy_, &ny_, &my_);
            }
            __builtin_amdgcn_sched_barrier(0);
            {
                const double ay1 = tail_arg(y1), ay1_ = tail_arg(y1 - sst);
                const double py1 = phi_of(ay1);
                double r_, r__;
                mills2<true>(ay1, ay1_, &r_, &r__);
                const double qy1 = py1 * r_, qy1_ = (py1 * (hs * ert)) * r__;
                ncdf_from_tail(y1, qy1, &ny1, &my1);
                ncdf_from_tail(y1 - sst, qy1_, &ny1_, &my1_);
            }
            const double cui = t1 - S * p2l * (my - my1) + Kd * p2l2 * (my_ - my1_);
            v = v - cui;
            v = (runmax >= o.H || o.H <= K) ? 0.0 : v;          // knocked out / worthless
        }
        const double ic = S - K;
        v = live ? v : ((ic < 0.0) ? 0.0 : ic);
        if (o.type == HE_BOOK_UO_CALL) v = (runmax >= o.H) ? 0.0 : v;
    }
    return (v < 0.0) ? 0.0 : v;   // python max(price, 0)
}

// sum_k q_k * 100 * V_k after step t of the episode (variance var: GBM constant,
// Heston the env's v_t).  tab: the tau table, p.book_tab or its LDS copy.
template <bool CONST_VAR = false>
__device__ __forceinline__ double book_value(const Params& p, double S, double var, int32_t t, double runmax,
                                             const double* tab, const BookOpt* opts = nullptr) {
    BookEnv b;
    b.S = S;
    b.lnS = log_book(S);   // config 4 7.15 -> 7.04 ms, config 5 1.58 -> 1.55 ms against log (r04s7_ab_book_log.txt)
    if (CONST_VAR) {  // var == p.var: the host's values of the same expressions
        b.sig = p.bk_sig;
        b.isig = p.bk_isig;
        b.s2 = p.bk_s2;
        b.lam = p.bk_lam;
    } else {
        b.sig = sqrt(var < 0.0 ? 0.0 : var);
        // 1 / sigma by v_rcp_f64 and two Newton steps, lam = r / sigma^2 + 1/2 from it: no IEEE
        // division per slot (config 5 1.62 -> 1.58 ms with hs below, r04s7_ab_book_rcp.txt).  At
        // sigma = 0 both are NaN instead of inf: only the intrinsic-value branch is live there.
        double y = __builtin_amdgcn_rcp(b.sig);
        y = fma(fma(-b.sig, y, 1.0), y, y);
        y = fma(fma(-b.sig, y, 1.0), y, y);
        b.isig = y;
        b.s2 = b.sig * b.sig;
        b.lam = fma(p.r_d, y * y, 0.5);
    }
    double B = 0.0;
#if HE_BOOK_DIAG == 2
    return S * 1e-3;  // diagnostic builds only: no book pricing at all
#endif
    for (int k = 0; k < p.book_n; ++k) {
        BookOpt o;
        if (opts) {  // an LDS copy: the type and expiry back in SGPRs (uniform branches)
            o = opts[k];
            o.type = __builtin_amdgcn_readfirstlane(o.type);
            o.expiry = __builtin_amdgcn_readfirstlane(o.expiry);
        } else {
            o = p.book[k];
        }
        B = B + o.q100 * book_option(p, o, b, o.expiry - t, runmax, tab);
    }
    return B;
}
__device__ __forceinline__ double book_value(const Params& p, double S, double var, int32_t t, double runmax) {
    return book_value(p, S, var, t, runmax, p.book_tab);
}

// The Heston price advance's exp (market_body and the LDS producers, the same function) is
// the library exp: its P&L equals the oracle's bit for bit on the parity cases, as exp_k's
// does (tools/pnl_exact.py), and it is 1 % faster at config 5 (r02 g18).

// Box-Muller pair of the Philox block of (seed, global env id, env-step index n).
__device__ __forceinline__ void normals(const Params& p, int64_t gid, uint64_t n, double* z1, double* z2) {
    u32x4 ctr = {(uint32_t)n, (uint32_t)(n >> 32), (uint32_t)gid, (uint32_t)((uint64_t)gid >> 32)};
    u32x4 x = philox4x32_10(ctr, p.key0, p.key1);
    box_muller(u01(x.x, x.y), u01(x.z, x.w), z1, z2);
}

// The Box-Muller pairs of Philox blocks m0 .. m0 + B - 1 of env gid into z[2B] (cos, sin,
// cos, ...): normals() for B blocks in lockstep, the same bits.
template <int B>
__device__ __forceinline__ void philox_normals_n(const Params& p, int64_t gid, uint64_t m0, double* z) {
    u32x4 c[B];
    double u1[B], u2[B], z1[B], z2[B];
#pragma unroll
    for (int b = 0; b < B; ++b) {
        const uint64_t m = m0 + (uint64_t)b;
        c[b] = u32x4{(uint32_t)m, (uint32_t)(m >> 32), (uint32_t)gid, (uint32_t)((uint64_t)gid >> 32)};
    }
    philox4x32_10_n<B>(c, p.key0, p.key1);
#pragma unroll
    for (int b = 0; b < B; ++b) {
        u1[b] = u01(c[b].x, c[b].y);
        u2[b] = u01(c[b].z, c[b].w);
    }
    box_muller_n<B>(u1, u2, z1, z2);
#pragma unroll
    for (int b = 0; b < B; ++b) {
        z[2 * b] = z1[b];
        z[2 * b + 1] = z2[b];
    }
}

// ------------------------------------------------------------------ market kernel
// One workgroup = 64 envs x 4 slot-lanes.  Slot j (1..M) is the market after the
// j-th step from the block start; slot 0 is the block start itself.  With
// a = ep*T + t the step from position a uses Philox counter n = a and starts
// from S0 when t in {0, T} (autoreset), so every slot is a pure function of the
// block-start state.
template <int MODE, bool BOOK>
__device__ __forceinline__ void market_body(Params p, Market cur, Market bak, int32_t advance_only, int64_t bid) {
    constexpr bool HESTON = (MODE == HE_MODE_HESTON);
    __shared__ double shS[kMktEnvs][kMaxBlock + 1];
    __shared__ double shV[HESTON ? kMktEnvs : 1][HESTON ? kMaxBlock + 1 : 1];
    __shared__ double shM[BOOK ? kMktEnvs : 1][BOOK ? kMaxBlock + 1 : 1];  // running max of S
    const int lane = threadIdx.x & (kMktEnvs - 1);
    const int sub = threadIdx.x / kMktEnvs;
    const int64_t i = bid * kMktEnvs + lane;
    const bool live = i < p.n;
    const int M = p.M;
    const uint32_t T = (uint32_t)p.T;
    const int64_t gid = p.goff + i;
    // block-start position (advance_only: rewind from `bak`, else continue from `cur`)
    Market src = advance_only ? bak : cur;
    uint32_t ep0 = 0, t0 = 0;
    double S0v = 0.0, v0v = 0.0, M0v = 0.0;
    float C0v = 0.0f, P0v = 0.0f;
    if (live) {
        ep0 = src.ep[i];
        t0 = src.t[i];
        S0v = src.S[i];
        if (HESTON) v0v = src.v[i];
        if (BOOK) M0v = src.M[i];
        C0v = src.C[i];
        P0v = src.P[i];
    }
    const int nsteps = advance_only ? advance_only : M;
    const uint32_t t0m = (t0 >= T) ? 0u : t0;  // position modulo T
    const uint64_t a0 = (uint64_t)ep0 * T + t0m + ((t0 >= T) ? T : 0u);
    // phase 1 (all lanes, time-parallel): the random part of every step
    if (HESTON) {
        // two normals per step: Philox block n -> (z1, z2)
        for (int j = 1 + sub; j <= nsteps; j += kMktLanes) {
            if (!live) break;
            uint64_t n = a0 + (uint64_t)(j - 1);
            double z1, z2;
            normals(p, gid, n, &z1, &z2);
            double dw1 = p.sqrt_dt * z1, dw2 = p.sqrt_dt * z2;
            shV[lane][j] = dw1;
            shS[lane][j] = p.h_rho * dw1 + p.h_sqrt1mrho2 * dw2;  // rbergomi_sim.py:457
        }
    } else {
        // one normal per step: Philox block m = n/2 gives the Box-Muller pair of
        // steps 2m (cos branch) and 2m+1 (sin branch)
        const uint64_t m0 = a0 >> 1, m1 = (a0 + (uint64_t)nsteps - 1) >> 1;
        for (uint64_t m = m0 + (uint64_t)sub; m <= m1; m += kMktLanes) {
            if (!live) break;
            double z[2];
            normals(p, gid, m, &z[0], &z[1]);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                uint64_t n = 2 * m + (uint64_t)h;
                if (n < a0 || n >= a0 + (uint64_t)nsteps) continue;
                int j = (int)(n - a0) + 1;
                double dW = p.sqrt_dt * z[h];
                shS[lane][j] = exp_k(p.drift + p.sqrt_var * dW);  // rbergomi_sim.py:459-463
            }
        }
    }
    __syncthreads();
    // phase 2 (one lane per env): the sequential f64 chain
    if (sub == 0 && live) {
        double S = S0v, v = v0v, Mx = M0v;
        uint32_t tt = t0;
        uint32_t ep = ep0;
        shS[lane][0] = S;
        if (HESTON) shV[lane][0] = v;
        if (BOOK) shM[lane][0] = Mx;
        for (int j = 1; j <= nsteps; ++j) {
            if (tt == 0 || tt >= T) {  // autoreset: a new episode starts from S0
                if (tt >= T) ep += 1u;
                S = p.s0;
                if (HESTON) v = p.var;
                if (BOOK) Mx = p.s0;
                tt = 0;
            }
            if (HESTON) {
                double vp = v < 0.0 ? 0.0 : v;  // full truncation
                double dWS = shS[lane][j], dw1 = shV[lane][j];
                double drift = (p.mu - 0.5 * vp) * p.dt;
                double diff = sqrt(vp) * dWS;
                double Sn = S * exp(drift + diff);
                S = (Sn < 1e-8) ? 1e-8 : Sn;
                v = (v + p.h_kappa * (p.h_theta - vp) * p.dt) + p.h_xi * sqrt(vp) * dw1;
                shV[lane][j] = v;
            } else {
                double Sn = S * shS[lane][j];
                S = (Sn < 1e-8) ? 1e-8 : Sn;  // np.maximum(., 1e-8), NaN kept
            }
            shS[lane][j] = S;
            if (BOOK) {
                Mx = np_max(Mx, S);
                shM[lane][j] = Mx;
            }
            tt += 1u;
        }
        if (!advance_only) {  // keep the block start for rewinds
            bak.ep[i] = ep0;
            bak.t[i] = t0;
            bak.S[i] = S0v;
            if (HESTON) bak.v[i] = v0v;
            bak.C[i] = C0v;
            bak.P[i] = P0v;
            if (BOOK) bak.M[i] = M0v;
        }
        cur.ep[i] = ep;
        cur.t[i] = tt;
        cur.S[i] = S;
        if (HESTON) cur.v[i] = v;
        if (BOOK) cur.M[i] = Mx;
    }
    __syncthreads();
    // phase 3 (time-parallel): marks + greeks of every slot
    const int64_t N = p.n;
    // episode step of slot j: (t0m + j - 1) % T + 1, stepped by kMktLanes without a
    // divide per slot
    uint32_t tj = (t0m + (uint32_t)sub) % T + 1u;  // 1..T
    const uint32_t tstep = (uint32_t)kMktLanes % T;
    for (int j = 1 + sub; j <= nsteps; j += kMktLanes, tj += tstep, tj = (tj > T) ? tj - T : tj) {
        if (!live) break;
        double S64 = shS[lane][j];
        double v64 = HESTON ? shV[lane][j] : p.var;
        float C, P;
        if (tj < T) {
            marks<MODE>(p, S64, v64, tj, &C, &P);
        } else if (T == 1u) {  // lagged marks of t = T-1 = 0: the reset marks
            C = p.rstv[2];
            P = p.rstv[3];
        } else if (j == 1) {   // lagged marks of the block start
            C = C0v;
            P = P0v;
        } else {               // lagged marks of t = T-1: slot j-1 (hedging_env_v2.py:229-231)
            marks<MODE>(p, shS[lane][j - 1], HESTON ? shV[lane][j - 1] : p.var, T - 1u, &C, &P);
        }
        if (j == nsteps) {
            cur.C[i] = C;
            cur.P[i] = P;
        }
        if (advance_only) continue;
        float S32 = (float)S64;
        float v32 = HESTON ? (float)v64 : p.var_f;
        if (HESTON) p.tileA[(int64_t)j * N + i] = make_float4(S32, v32, C, P);
        else st3(p.tileA, (int64_t)j * N + i, S32, C, P);
        if (HESTON) {
            float4 g = p.record_metrics ? greeks_fast<false>(p, S32, v32) : make_float4(0.f, 0.f, 0.f, 0.f);
            // the step into slot j starts from the reset market (first step of an
            // episode) or from slot j-1
            const float Sp32 = (tj == 1u) ? p.rstv[0] : (float)shS[lane][j - 1];
            g.w = lag_return(S32, Sp32);
            p.tileB[(int64_t)j * N + i] = g;
        } else if (p.tile_greeks) {
            const float4 g = p.record_metrics ? greeks_fast<true>(p, S32, v32) : make_float4(0.f, 0.f, 0.f, 0.f);
            st3(p.tileB, (int64_t)j * N + i, g.x, g.y, g.z);
        }
        if (BOOK) p.tileC[(int64_t)j * N + i] = book_value(p, S64, v64, (int32_t)tj, shM[lane][j]);
    }
    if (!advance_only && sub == 0 && live) {
        float v32 = HESTON ? (float)v0v : p.var_f;
        if (HESTON) {
            p.tileA[i] = make_float4((float)S0v, v32, C0v, P0v);
            // greeks of the block start (the obs policy rollouts resume from); equal to
            // the previous block's last slot, same function of the same (S, v)
            p.tileB[i] = p.record_metrics ? greeks_fast<false>(p, (float)S0v, v32) : make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
            st3(p.tileA, i, (float)S0v, C0v, P0v);
            if (p.tile_greeks) {
                const float4 g = p.record_metrics ? greeks_fast<true>(p, (float)S0v, v32) : make_float4(0.f, 0.f, 0.f, 0.f);
                st3(p.tileB, i, g.x, g.y, g.z);
            }
        }
        // slot 0 = the block start; at t0 in {0, T} the next step starts from the reset
        // market and reads book_rst instead
        if (BOOK)
            p.tileC[i] = (t0 == 0u || t0 >= T) ? p.book_rst
                                                : book_value(p, S0v, HESTON ? v0v : p.var, (int32_t)t0, M0v);
    }
}

template <int MODE, bool BOOK>
__global__ __launch_bounds__(kMktEnvs * kMktLanes, kMktWaves) void market_kernel(Params p, Market cur, Market bak,
                                                                                     int32_t advance_only) {
    market_body<MODE, BOOK>(p, cur, bak, advance_only, blockIdx.x);
}

// Reset market constants + reset obs row (generate): rst = {S0, v0, C0, P0, obs0[13]}.
template <int MODE>
__global__ void init_reset_kernel(Params p, float* rst) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    p.s0s_const = 0;  // S0 is what this kernel computes: divide by the env's own max(S0, 25)
    float C, P;
    marks<MODE>(p, p.s0, p.var, 0u, &C, &P);
    Mkt m{(float)p.s0, p.var_f, C, P};
    Env e;
    e.t = 0;
    e.call = e.put = 0;
    e.cash = p.initial_cash;
    e.s0_small = m.S < 1e-6f;
    e.s0 = e.s0_small ? 1.0f : m.S;
    float4 g = p.record_metrics ? greeks<MODE == HE_MODE_GBM>(p, m.S, m.v) : make_float4(0.f, 0.f, 0.f, 0.f);
    rst[0] = m.S;
    rst[1] = m.v;
    rst[2] = C;
    rst[3] = P;
    make_obs(p, e, m, g, m.S, m.v, rst + 4);
    if (p.book_n) reinterpret_cast<double*>(rst)[10] = book_value(p, p.s0, p.var, 0, p.s0);  // rst[20..21]
}

// Replay: obs greeks of every table entry, once at load time.
__global__ __launch_bounds__(kBlock) void table_greeks_kernel(Params p, float4* recg, int64_t count) {
    int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= count) return;
    // k runs over the padded table: slots outside rows 0 .. T of a path are padding (zeros)
    const int64_t t = k % p.rstride - p.roff;
    if (t < 0 || t > (int64_t)p.T) {
        recg[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        return;
    }
    float4 r = p.rec[k];
    float4 g = p.record_metrics ? replay_greeks(p, r.x, r.y) : make_float4(0.f, 0.f, 0.f, 0.f);
    // row t >= 1 is stepped into from row t-1 of the same path; row 0 is only a reset obs
    g.w = (t == 0) ? 0.0f : lag_return(r.x, p.rec[k - 1].x);
    recg[k] = g;
}

// ------------------------------------------------------------------ step
struct StepOut {
    double reward;
    bool term;
    double pnl, ps, tc, commission, slippage, rpc, tcp, thp, pv;
    float fc, fp;
    int32_t rqc, rqp, dc, dp;
};

// hedging_env_v2.py:175-262 (v1: hedging_env.py:171-245).  pre/post: market before
// and after the advance (post C/P already lagged on the terminal step).
// ------------------------------------------------------------------ baseline policies
// The action of `policy` on the env's current obs (o3, o4, o7, o9 = obs[3], obs[4],
// obs[7], obs[9]) and positions, with the reference's dtype sequence.
__device__ __forceinline__ float2 policy_action(const Params& p, int policy, int32_t call, int32_t put, float o3,
                                                float o4, float cd, float pd) {
    const float mt = p.mt_f;
    if (policy == HE_POLICY_DELTA_EVERY_STEP) {
        // baselines.py:77-103, all f32 (numpy f32 scalars with weak python ints/floats)
        const float cur_call = o3 * p.maxh_f;                       // obs[3] * max_contracts_held
        const float cur_put = o4 * p.maxh_f;
        const float opt_delta = (cur_call * cd + cur_put * pd) * 100.0f;
        const float total = (float)p.shares_d + opt_delta;          // shares_held_fixed + ...
        const float target = -total;
        float tc = 0.0f, tp = 0.0f;
        if (fabsf(cd * 100.0f) > 0.1f) tc = target / (cd * 100.0f);
        else if (fabsf(pd * 100.0f) > 0.1f) tp = target / (pd * 100.0f);
        return make_float2(np_clipf(tc, -mt, mt), np_clipf(tp, -mt, mt));
    }
    if (policy == HE_POLICY_DELTA_THRESHOLD) {
        // delta_and_nothing.py:122-163: np.int64 positions x f32 deltas -> f64
        const double cur = ((double)call * (double)cd + (double)put * (double)pd) * 100.0;
        const double need = -p.shares_d - cur;                      // target - current
        const float thr = (0.5f * fabsf(cd)) * 100.0f;
        if (fabs(need) < (double)thr) return make_float2(0.0f, 0.0f);
        double rc = 0.0, rp = 0.0;
        const double mtd = (double)p.mt;
        if (need > 0.0) {
            if (fabsf(cd) > 1e-6f) {
                const double n = need / (double)(cd * 100.0f);
                rc = n < -mtd ? -mtd : (n > mtd ? mtd : n);
            }
        } else if (need < 0.0) {
            if (fabsf(pd) > 1e-6f) {
                const double n = need / (double)(pd * 100.0f);
                rp = n < -mtd ? -mtd : (n > mtd ? mtd : n);
            }
        }
        return make_float2((float)rc, (float)rp);
    }
    return make_float2(0.0f, 0.0f);  // HE_POLICY_NO_HEDGE (baselines.py:74-75)
}

// portfolio value of the pre-step state (hedging_env_v2.py:233-236): the previous
// step's pv, recomputed bit for bit (same operands, same order)
template <bool BOOK>
__device__ __forceinline__ double portfolio_value(const Params& p, const Env& e, const Mkt& m) {
    double optv = ((double)e.call * (double)m.C) * 100.0 + ((double)e.put * (double)m.P) * 100.0;
    double pv = ((double)(p.shares_f * m.S) + optv) + e.cash;
    if (BOOK) pv = pv + m.B;  // liability book (extension): after cash
    return pv;
}

// FAST: variant 2, loss != mse, shares_to_hedge != 0, generate mode (constant reward
// denominator) -- the branches on those flags compiled out (fast_config()).
// pv_last = portfolio_value(pre-step state), carried in registers across fused steps.
template <bool BOOK, bool FAST = false, bool EP = false>
__device__ __forceinline__ void step_env(const Params& p, Env& e, const Mkt& pre, const Mkt& post, float a0,
                                         float a1, double pv_last, StepOut& o) {
    double pv_prev;
    if (EP) {  // the replay LDS steppers: a select, no branch
        const float pv0 = (p.shares_f * pre.S + 0.0f) + p.init_cash_f;  // f32 (:167-168)
        pv_prev = (e.t == 0) ? (double)pv0 : pv_last;
    } else if (e.t == 0) {
        float pv0 = (p.shares_f * pre.S + 0.0f) + p.init_cash_f;  // f32 (:167-168)
        pv_prev = (double)pv0;
        if (BOOK) pv_prev = pv_prev + pre.B;
    } else {
        pv_prev = pv_last;
    }
    // (i)-(ii) integer trade logic (:181-200)
    float fc = a0 * p.mt_f;
    float fp = a1 * p.mt_f;
    int32_t rqc = trade_round(fc, p.mt);
    int32_t rqp = trade_round(fp, p.mt);
    int32_t nc = e.call + rqc, nq = e.put + rqp;
    nc = clamp_pos(nc, p.maxh);
    nq = clamp_pos(nq, p.maxh);
    int32_t dc = nc - e.call, dp = nq - e.put;
    e.call = nc;
    e.put = nq;
    // (iii) commission + slippage on the pre-advance marks (:203-213)
    int32_t adc = dc < 0 ? -dc : dc, adp = dp < 0 ? -dp : dp;
    double commission = (double)(adc + adp) * p.tcpc;
    double slippage = 0.0, tc;
    if (FAST || p.variant == 2) {
        double sc = (((double)adc * (double)pre.C) * 100.0) * p.slip_frac;
        double sp = (((double)adp * (double)pre.P) * 100.0) * p.slip_frac;
        slippage = sc + sp;
        tc = commission + slippage;
    } else {
        tc = commission;
    }
    e.cash = e.cash - tc;
    // (iv)-(v) advance (:216-231)
    e.t = e.t + 1;
    bool term = (int32_t)e.t >= p.T;
    // (vi) mark-to-market (:233-238)
    double pv = portfolio_value<BOOK>(p, e, post);
    double pnl = pv - pv_prev;
    // EP (the replay LDS steppers): the IEEE division, straight-line -- div_by's value without
    // its guard branch, so the unrolled steps of a block stay one basic block
    double ps = (!FAST && p.shares_zero) ? pnl : (EP ? pnl / p.shares_d : div_by(pnl, p.shares_d, p.inv_shares));
    // (vii) reward (:243-262)
    double term_v;
    const double num = (!FAST && p.loss == HE_LOSS_MSE) ? ps * ps : fabs(ps);
    if (EP) {  // the episode's denominator (replay_episode_consts)
        term_v = num / e.den;
    } else if (FAST || p.den_const) {
        term_v = div_by(num, p.den, p.inv_den);
    } else {
        float f = np_maxf(e.s0, 25.0f);
        double den;
        if (p.loss == HE_LOSS_MSE) den = e.s0_small ? (625.0 + 1e-9) : (double)(f * f + 1e-9f);
        else den = e.s0_small ? (25.0 + 1e-9) : (double)(f + 1e-9f);
        term_v = num / den;
    }
    double rpc = (-p.w) * term_v;
    double tcp = p.lam * tc;
    double thp = 0.0, reward;
    if (FAST || p.variant == 2) {
        // computed, not looked up: a table load indexed by t is a dependent round trip.
        // theta_weight 0 (the default): 0 * finite = +0 and x - +0 == x bit for bit
        if (FAST || p.theta != 0.0) thp = p.theta * div_int_by((double)(p.T - (int32_t)e.t), 252.0, p.inv_252);
        reward = (rpc - tcp) - thp;
    } else {
        reward = rpc - tcp;
    }
    o.reward = reward;
    o.term = term;
    o.pnl = pnl;
    o.ps = ps;
    o.tc = tc;
    o.commission = commission;
    o.slippage = slippage;
    o.rpc = rpc;
    o.tcp = tcp;
    o.thp = thp;
    o.pv = pv;
    o.fc = fc;
    o.fp = fp;
    o.rqc = rqc;
    o.rqp = rqp;
    o.dc = dc;
    o.dp = dp;
}

__device__ __forceinline__ void write_info(const he_info& inf, int64_t i, const StepOut& o, const Env& e,
                                           const Mkt& m, int variant) {
    const double nan = __builtin_nan("");
    if (inf.step_pnl_total) inf.step_pnl_total[i] = o.pnl;
    if (inf.per_share_step_pnl) inf.per_share_step_pnl[i] = o.ps;
    if (inf.raw_pnl_deviation_abs) inf.raw_pnl_deviation_abs[i] = fabs(o.ps);
    if (inf.transaction_costs_total) inf.transaction_costs_total[i] = o.tc;
    if (inf.commission_cost) inf.commission_cost[i] = variant == 2 ? o.commission : nan;
    if (inf.slippage_cost) inf.slippage_cost[i] = variant == 2 ? o.slippage : nan;
    if (inf.reward_pnl_component) inf.reward_pnl_component[i] = o.rpc;
    if (inf.transaction_cost_penalty) inf.transaction_cost_penalty[i] = o.tcp;
    if (inf.theta_penalty) inf.theta_penalty[i] = variant == 2 ? o.thp : nan;
    if (inf.reward_step) inf.reward_step[i] = o.reward;
    if (inf.portfolio_value) inf.portfolio_value[i] = o.pv;
    if (inf.cash) inf.cash[i] = e.cash;
    if (inf.call_contracts) inf.call_contracts[i] = e.call;
    if (inf.put_contracts) inf.put_contracts[i] = e.put;
    if (inf.scaled_float_call) inf.scaled_float_call[i] = o.fc;
    if (inf.scaled_float_put) inf.scaled_float_put[i] = o.fp;
    if (inf.requested_calls_rounded_clipped) inf.requested_calls_rounded_clipped[i] = o.rqc;
    if (inf.requested_puts_rounded_clipped) inf.requested_puts_rounded_clipped[i] = o.rqp;
    if (inf.actual_calls_traded) inf.actual_calls_traded[i] = o.dc;
    if (inf.actual_puts_traded) inf.actual_puts_traded[i] = o.dp;
    if (inf.initial_S0_for_episode) inf.initial_S0_for_episode[i] = e.s0;
    if (inf.current_stock_price) inf.current_stock_price[i] = m.S;
    if (inf.current_volatility) inf.current_volatility[i] = m.v;
    if (inf.current_call_price) inf.current_call_price[i] = m.C;
    if (inf.current_put_price) inf.current_put_price[i] = m.P;
    if (inf.current_step) inf.current_step[i] = (int32_t)e.t;
    if (inf.current_episode_idx) inf.current_episode_idx[i] = e.path;
}

// Write one wave's obs rows [wrow0, wrow0 + rows), staged in LDS as [rows][13] at
// wtile, to out (row-major [N][13]) with 16-B stores (wrow0 % 32 == 0: 16-B aligned).  Wave-local: the lanes of a
// wave issue their LDS writes and reads in program order, so no workgroup barrier.
// (compiler-only barriers around it: no hardware wait is needed)
__device__ __forceinline__ void flush_obs_wave(const float* wtile, float* out, int64_t wrow0, int rows, int lane) {
    asm volatile("" ::: "memory");
    GLOBAL float* dst = (GLOBAL float*)out + wrow0 * kObs;
    GLOBAL v4f* d4 = (GLOBAL v4f*)dst;
    const v4f* s4 = reinterpret_cast<const v4f*>(wtile);
    if (rows == 64) {
        // 64 rows = 208 float4: three per lane, a fourth on lanes 0-15
        d4[lane] = s4[lane];
        d4[lane + 64] = s4[lane + 64];
        d4[lane + 128] = s4[lane + 128];
        if (lane < 16) d4[lane + 192] = s4[lane + 192];
    } else if (rows > 0) {
        // a partial wave (the last rows of N): at most 4 float4 per lane and a 1-3 float
        // remainder, as predicated stores -- no loop carrying addresses (a loop here cost the
        // replay obs stepper its VGPR spills)
        const int nf = rows * kObs;
        const int nv = nf >> 2;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int k = lane + 64 * q;
            if (k < nv) d4[k] = s4[k];
        }
        if (lane < nf - (nv << 2)) dst[(nv << 2) + lane] = wtile[(nv << 2) + lane];
    }
    asm volatile("" ::: "memory");
}

// The episode's S0 of row e.path (hedging_env_v2.py:156-157: < 1e-6 -> 1.0).
__device__ __forceinline__ void replay_start(const Params& p, Env& e) {
    float S0 = p.rec[rrow(p, e.path, 0)].x;
    e.s0_small = S0 < 1e-6f;
    e.s0 = e.s0_small ? 1.0f : S0;
}

// replay reset (hedging_env_v2.py:145-173): draw the episode row from the env's
// PCG64 stream, exactly gymnasium's np_random.integers(num_episodes).
__device__ __forceinline__ void replay_reset(const Params& p, const State& s, int64_t i, Env& e) {
    const int64_t N = p.n;
    Pcg64 g;
    g.sh = s.pcg[i];
    g.sl = s.pcg[N + i];
    g.ih = s.pcg[2 * N + i];
    g.il = s.pcg[3 * N + i];
    g.has32 = s.pcgb[i];
    g.buf32 = s.pcgb[N + i];
    e.path = (int32_t)pcg64_integers(g, (uint64_t)p.n_paths);
    s.pcg[i] = g.sh;
    s.pcg[N + i] = g.sl;
    s.pcgb[i] = g.has32;
    s.pcgb[N + i] = g.buf32;
    replay_start(p, e);
}

__device__ __forceinline__ void env_reset_common(const Params& p, Env& e) {
    e.t = 0;
    e.call = 0;
    e.put = 0;
    e.cash = p.initial_cash;
}

// K fused steps from market slot `slot0` (generate) / the env's own path row (replay).
// Every load of step 0 is issued in a straight-line prologue before its first use
// (one memory round trip instead of two), and in generate mode the loads of step
// k+1 go out before the arithmetic of step k (software pipelining for rollouts).
#ifdef HE_TIMING
// Diagnostic builds (tools/step_ab.sh): per-wave timestamps of the last step_kernel
// at fixed points into p.tim[point][wave][2] = {s_memrealtime (100 MHz, points 0
// and 4 only), s_memtime (shader clock)}.
#define HE_TIM(k)                                                                          \
    do {                                                                                   \
        uint64_t rt_ = ((k) == 0 || (k) == 4) ? __builtin_amdgcn_s_memrealtime() : 0;       \
        uint64_t ct_ = __builtin_amdgcn_s_memtime();                                        \
        if ((threadIdx.x & 63) == 0) {                                                     \
            size_t w_ = (size_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);            \
            if (w_ < 8192) {                                                               \
                p.tim[((size_t)(k) * 8192 + w_) * 2] = rt_;                                \
                p.tim[((size_t)(k) * 8192 + w_) * 2 + 1] = ct_;                            \
            }                                                                              \
        }                                                                                  \
    } while (0)
#else
#define HE_TIM(k) \
    do {          \
    } while (0)
#endif

// SINGLE: the he_step instance (k_steps == 1 at compile time, straight-line code).
// tA/tB: the market source, tile buffer {S,v,C,P} / greeks (generate) or the
// replay table rec / recg.
// step1_vn_kernel's view of a he_step: the workgroup's obs rows in LDS after the step and
// this thread's reward, for the fused VecNormalize moments.
struct VnHook {
    const float* tile;
    float rew;
    double rew64;   // the f64 reward (Monitor's sums)
    bool term;
};

// he_step_signal: the end of an he_step launch, raised in host-mapped memory so the host can
// see the step's outputs without the runtime's completion path (~8 us of a small-N step,
// profiles/r06h_flag_probe.txt).  Every thread makes its own stores visible system-wide, the
// workgroup meets, and one thread per workgroup counts the workgroup done; the last one to count
// re-arms the counter for the next step and stores the sequence number with release semantics.
__device__ __forceinline__ void raise_step_signal(const Io& io) {
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t nwg = gridDim.x;
        const uint32_t prev =
            nwg == 1u ? 0u : __hip_atomic_fetch_add(io.sig_cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == nwg - 1u) {
            if (nwg > 1u) __hip_atomic_store(io.sig_cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(io.sig, io.sig_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

template <int MODE, bool INFO, bool SINGLE, bool BOOK, bool FAST, bool POL, bool GS>
__device__ __forceinline__ void step_body(const Params& pk, int64_t n_envs, const float4* tA, const float4* tB,
                                          const double* tC, State s, Io io, int k_steps_arg, int slot0,
                                          int64_t bid, VnHook* hook = nullptr) {
    constexpr bool REPLAY = (MODE == HE_MODE_REPLAY);
    constexpr bool CT = (MODE == HE_MODE_GBM);  // 12-B tile records (see ld3A)
    const int k_steps = SINGLE ? 1 : k_steps_arg;
    Params p = pk;
    HE_TIM(0);
    // latency-critical: win VALU/memory issue arbitration against the prefetching
    // market_kernel waves that share the SIMDs (they run at the default priority 0)
    __builtin_amdgcn_s_setprio(3);
    __shared__ __attribute__((aligned(16))) float tile[kEpb * kObs];
    if (hook) hook->tile = tile;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t wrow0 = bid * kEpb + wave * kEpw;  // first env of this wave
    const int64_t i = wrow0 + lane;
    const int64_t N = n_envs;
    const bool live = lane < kEpw && i < N;
    const int wrows = (int)((N - wrow0) < kEpw ? (N - wrow0 > 0 ? N - wrow0 : 0) : kEpw);
    const float2* act = reinterpret_cast<const float2*>(io.act);
    const Mkt rst{p.rstv[0], p.rstv[1], p.rstv[2], p.rstv[3], BOOK ? p.book_rst : 0.0};
    // Every kernel argument of the prologue's addresses and of the step arithmetic,
    // pinned in SGPRs by ONE asm: one scalar round trip to the kernarg segment.  Left
    // alone, the backend sinks some of these loads into the `live` branch or after
    // the first vector loads return, each a further serialized round trip (measured
    // 0.3 us apiece at 65,536 envs).  The pointers are laundered as global-address-
    // space pointers, or their loads would turn into flat loads.
    auto s_t = (const GLOBAL uint32_t*)s.t;
    auto s_pos = (const GLOBAL uint32_t*)s.pos;
    auto s_cash = (const GLOBAL double*)s.cash;
    auto gact = (const GLOBAL v2f*)act;
    auto mA = (const GLOBAL v4f*)tA;
    auto mB = (const GLOBAL v4f*)tB;
    auto mC = (const GLOBAL double*)tC;
    auto s_path = (const GLOBAL int32_t*)s.path;
    auto s_s0 = (const GLOBAL float*)s.s0;
    int32_t hot_i = REPLAY ? p.T : slot0;
    asm volatile("" : "+s"(s_t), "+s"(s_pos), "+s"(s_cash), "+s"(gact), "+s"(mA), "+s"(mB), "+s"(hot_i));
    if (BOOK) asm volatile("" : "+s"(mC));
    if (REPLAY) asm volatile("" : "+s"(s_path), "+s"(s_s0));
    const float var_f = p.var_f;
    auto ldA = [=](int64_t r) { return CT ? ld3A(mA, r, var_f) : ld4(mA, r); };
    constexpr bool tg = !(CT && GS);  // greeks from the tile (GS: gbm_greeks in this kernel)
    auto ldB = [=](int64_t r) {
        return CT ? (tg ? ld3B(mB, r) : make_float4(0.f, 0.f, 0.f, 0.f)) : ld4(mB, r);
    };
    // GBM: the obs greeks of market price S (the market kernel's Heston slot values)
    auto gbm_greeks = [&](float S) {
        return (FAST || p.record_metrics) ? greeks_fast<true>(p, S, var_f) : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    HE_TIM(1);
    Env e;
    Mkt pre;
    float4 postA, postB;
    double postC = 0.0;
    float2 a;
    if (live) {
        const uint32_t t0 = s_t[i];
        const uint32_t pk = s_pos[i];
        double cash = s_cash[i];
        a = POL ? make_float2(0.0f, 0.0f) : ld2(gact, i);
        if (REPLAY) {
            const int32_t T = hot_i;
            const int32_t path = s_path[i];
            const float s0 = s_s0[i];
            const uint32_t tt = t0 > (uint32_t)T ? (uint32_t)T : t0;
            const uint32_t tn = t0 + 1 > (uint32_t)T ? (uint32_t)T : t0 + 1;
            const int64_t r0 = rrow(p, path, 0);
            pre = as_mkt(ld4(mA, r0 + tt));
            postA = ld4(mA, r0 + tn);
            postB = ld4(mB, r0 + tn);
            e.path = path;
            e.s0_small = (s0 == -1.0f);
            e.s0 = e.s0_small ? 1.0f : s0;
        } else {
            float4 preA = ldA((int64_t)hot_i * N + i);
            postA = ldA((int64_t)(hot_i + 1) * N + i);
            postB = ldB((int64_t)(hot_i + 1) * N + i);
            double preC = 0.0;
            if (BOOK) {
                preC = mC[(int64_t)hot_i * N + i];
                postC = mC[(int64_t)(hot_i + 1) * N + i];
                asm volatile("" : "+v"(preC), "+v"(postC));
            }
            // pin every prologue load here: otherwise preA is sunk into the t != 0
            // branch (a second, dependent memory round trip), and a load still
            // pending at a branch merge makes the waitcnt pass drain every later
            // store with vmcnt(0) before the final state stores
            asm volatile("" : "+v"(preA.x), "+v"(preA.y), "+v"(preA.z), "+v"(preA.w), "+v"(postA.x),
                         "+v"(postB.x), "+v"(cash), "+v"(a.x), "+v"(a.y));
            HE_TIM(2);
            e.path = -1;
            e.s0_small = rst.S < 1e-6f;
            e.s0 = e.s0_small ? 1.0f : rst.S;
            pre = (t0 == 0) ? rst : as_mkt(preA);  // select of values, not addresses
            if (BOOK) pre.B = (t0 == 0) ? p.book_rst : preC;
        }
        e.t = t0;
        e.call = unpack_lo(pk);
        e.put = unpack_hi(pk);
        e.cash = cash;
    }
    // pv of the pre-step state; afterwards each step's pv (the reference carries
    // portfolio_value_t_minus_1 the same way, hedging_env_v2.py:268)
    double pv_last = live ? portfolio_value<BOOK>(p, e, pre) : 0.0;
    // policy rollouts: the current obs columns the policies read, and the episode sums
    float pol_o3 = 0.0f, pol_o4 = 0.0f, pol_cd = 0.0f, pol_pd = 0.0f;
    double acc[7] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    uint32_t acc_len = 0;
    if (POL && live) {
        float4 gpre;
        if (REPLAY) {
            const uint32_t tt = e.t > (uint32_t)p.T ? (uint32_t)p.T : e.t;
            gpre = tB[rrow(p, e.path, tt)];
        } else {
            if (e.t == 0) gpre = make_float4(p.rstv[4 + 7], 0.0f, p.rstv[4 + 9], 0.0f);
            else gpre = tg ? ldB((int64_t)slot0 * N + i) : gbm_greeks(pre.S);
        }
        const bool met = p.record_metrics != 0;
        pol_cd = met ? gpre.x : 0.0f;
        pol_pd = met ? gpre.z : 0.0f;
        pol_o3 = (p.maxh != 0) ? div_int_byf((float)e.call, p.maxh_f, p.inv_maxh_f) : 0.0f;
        pol_o4 = (p.maxh != 0) ? div_int_byf((float)e.put, p.maxh_f, p.inv_maxh_f) : 0.0f;
#pragma unroll
        for (int c = 0; c < 7; ++c) acc[c] = s.acc[(int64_t)c * N + i];
        acc_len = s.acc_len[i];
    }
    // multi-step rollouts: the episode summaries (he_episode_summaries), as lds_stepper
    constexpr bool SUMS = !SINGLE && !POL && !INFO;
    const bool sums = SUMS && io.sums;  // he_rollout only: he_step does not pay for them
    double sm0 = 0.0, sm1 = 0.0, sm2 = 0.0;
    uint32_t slen = 0;
    float last0 = 0.f, last1 = 0.f, last2 = 0.f, last3 = 0.f;
    if (sums && live) {
        sm0 = s.sum[i];
        sm1 = s.sum[N + i];
        sm2 = s.sum[2 * N + i];
        slen = s.sum_len[i];
        last0 = s.last[i];
        last1 = s.last[N + i];
        last2 = s.last[2 * N + i];
        last3 = s.last[3 * N + i];
    }
    bool reset_any = false;
    float* const orow = tile + (wave * kEpw + (lane < kEpw ? lane : 0)) * kObs;
    // step k of every env from market `post` (greeks + lag return `g`) with action ak:
    // state update, reward/done stores, the obs row into the wave's LDS tile, auto-reset
    auto step_part = [&](int k, const Mkt post, float4 g, float2 ak) {
        const int64_t koff = (int64_t)k * N;
        bool term = false;
        if (live) {
            // GBM: the lag return (and without tile_greeks the greeks) of the market
            // slot (see ld3A).  The step from t in {0, T} starts from the reset market;
            // at t == 0 pre is rst already (and spelling out both tests trips an
            // illegal VGPR-to-SGPR copy in the ROCm 7.2 backend)
            if constexpr (CT) {
                if (!tg) g = gbm_greeks(post.S);
                g.w = lag_return(post.S, (e.t >= (uint32_t)p.T) ? rst.S : pre.S);
            }
            if (POL) {
                ak = policy_action(p, io.pol.policy, e.call, e.put, pol_o3, pol_o4, pol_cd, pol_pd);
                if (io.pol.act_out) {
                    v2f av = {ak.x, ak.y};
                    ((GLOBAL v2f*)io.pol.act_out)[koff + i] = av;
                }
            }
            StepOut so;
            step_env<BOOK, FAST>(p, e, pre, post, ak.x, ak.y, pv_last, so);
            pv_last = so.pv;
            if (hook) {
                hook->rew = (float)so.reward;
                hook->rew64 = so.reward;
                hook->term = so.term;
            }
            if (POL) {  // the reference evaluation loops' sums, in step order
                acc[0] = acc[0] + so.reward;
                acc[1] = acc[1] + so.pnl;
                acc[2] = acc[2] + fabs(so.ps);
                acc[3] = acc[3] + so.tc;
                acc[4] = acc[4] + so.rpc;
                acc[5] = acc[5] + so.tcp;
                acc[6] = acc[6] + so.ps;
                acc_len += 1u;
                if (so.term) {
                    const unsigned long long r = atomicAdd(io.pol.count, 1ull);
                    if ((int64_t)r < io.pol.cap) {
                        he_episode_record rec;
                        rec.env_id = p.goff + i;
                        rec.length = (int32_t)acc_len;
                        rec.reserved = 0;
                        rec.reward_sum = acc[0];
                        rec.pnl_sum = acc[1];
                        rec.abs_pnl_sum = acc[2];
                        rec.cost_sum = acc[3];
                        rec.pnl_penalty_sum = acc[4];
                        rec.cost_penalty_sum = acc[5];
                        rec.per_share_pnl_sum = acc[6];
                        rec.reserved2 = 0.0;
                        io.pol.rec[r] = rec;
                    }
                    s.last[i] = (float)acc[0];
                    s.last[N + i] = (float)acc[1];
                    s.last[2 * N + i] = (float)acc[3];
                    s.last[3 * N + i] = (float)acc_len;
#pragma unroll
                    for (int c = 0; c < 7; ++c) acc[c] = 0.0;
                    acc_len = 0;
                }
            }
            if (SUMS) {
                const double a0 = sm0 + so.reward, a1 = sm1 + so.pnl, a2 = sm2 + so.tc;
                const uint32_t n1 = slen + 1u;
                float f0 = (float)a0, f1 = (float)a1, f2 = (float)a2, f3 = (float)n1;
                asm volatile("" : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3));
                last0 = so.term ? f0 : last0;
                last1 = so.term ? f1 : last1;
                last2 = so.term ? f2 : last2;
                last3 = so.term ? f3 : last3;
                sm0 = so.term ? 0.0 : a0;
                sm1 = so.term ? 0.0 : a1;
                sm2 = so.term ? 0.0 : a2;
                slen = so.term ? 0u : n1;
            }
            term = so.term;
            if (INFO) write_info(io.info, i, so, e, post, p.variant);
            float o[kObs];
            make_obs<FAST>(p, e, post, g, pre.S, pre.v, o);
#pragma unroll
            for (int c = 0; c < kObs; ++c) orow[c] = o[c];
            if (io.rew) ((GLOBAL float*)io.rew)[koff + i] = (float)so.reward;
            if (io.term) ((GLOBAL uint8_t*)io.term)[koff + i] = term ? 1 : 0;
            pre = post;
        }
        // wave-level done mask: waves without a terminating env skip the reset path
        if (p.autoreset && __ballot(term) != 0ull) {
            if (term) {
                if (io.tobs) {
#pragma unroll
                    for (int c = 0; c < kObs; ++c) io.tobs[i * kObs + c] = orow[c];
                }
                env_reset_common(p, e);
                if (REPLAY) {
                    replay_reset(p, s, i, e);
                    int64_t r = rrow(p, e.path, 0);
                    pre = as_mkt(tA[r]);
                    float o[kObs];
                    make_obs(p, e, pre, tB[r], pre.S, pre.v, o);
#pragma unroll
                    for (int c = 0; c < kObs; ++c) orow[c] = o[c];
                } else {
                    pre = rst;
#pragma unroll
                    for (int c = 0; c < kObs; ++c) orow[c] = p.rstv[4 + c];
                }
                reset_any = true;
            }
        }
        if (POL && live) {  // the obs row this step returns (post-reset for done envs)
            pol_o3 = orow[3];
            pol_o4 = orow[4];
            pol_cd = orow[7];
            pol_pd = orow[9];
        }
    };
    auto flush_part = [&](int k) {
        HE_TIM(3);
        if (io.obs) {
            // LDS-staged 16-B stores: measured 6.45 vs 7.14 us/step against per-lane
            // 4-B stores of the 52-B rows (MI355X, 65,536 envs, graph mode)
            flush_obs_wave(tile + wave * kEpw * kObs, io.obs + (int64_t)k * N * kObs, wrow0, wrows, lane);
        }
    };
    if constexpr (!REPLAY && !SINGLE) {
        // generate-mode rollout: the market and action inputs of step k+D are issued
        // before step k's stores.  vmcnt retires in issue order, so with D = 1 the
        // wait for step k+1's inputs also waits for step k-1's stores; at D = 4 those
        // stores were issued 4 steps earlier.  Every lane issues every load (clamped
        // index / step), so the wait counts are the same on every path.
        constexpr int D = kRolloutPrefetch;
        // dead lanes load a live lane's address of the same wave (no extra cache lines)
        const int64_t icl = wrow0 + (lane % kEpw);
        const int64_t ic = icl < N ? icl : N - 1;
        float2 ra[D];
        float4 rA[D], rB[D];
        double rC[D];
        ra[0] = a;
        rA[0] = postA;
        rB[0] = postB;
        rC[0] = postC;
        auto load = [&](int d, int kk) {
            kk = kk < k_steps ? kk : k_steps - 1;
            const int64_t r = (int64_t)(slot0 + kk + 1) * N + ic;
            if (!POL) ra[d] = ld2(gact, (int64_t)kk * N + ic);
            rA[d] = ldA(r);
            rB[d] = ldB(r);
            if (BOOK) rC[d] = mC[r];
        };
#pragma unroll
        for (int d = 1; d < D; ++d) load(d, d);
        for (int kb = 0; kb < k_steps; kb += D) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const int k = kb + d;
                if (k >= k_steps) break;
                Mkt post = as_mkt(rA[d]);
                if (BOOK) post.B = rC[d];
                const float4 g = rB[d];
                const float2 ak = ra[d];
                load(d, k + D);
                step_part(k, post, g, ak);
                flush_part(k);
            }
        }
    } else if (REPLAY && !SINGLE && p.T > kReplayPrefetch) {
        // replay rollout (train_ppo_v2.py:40's workload): the same D-deep ring, the rows of
        // step k+D issued before step k's stores.  Step kk's row is the env's path at its t
        // then (hedging_env_v2.py:223-231): from the state before step k, t_k + (kk - k) + 1
        // while no episode ends in between (t_k + (kk - k) < T); past an end the new path is
        // not drawn yet, so that slot is loaded from the old path and re-issued once the
        // reset has drawn it (every ring slot of a lane that just reset: its step k + m
        // reads row m of the new path) -- a wave-uniform branch once per episode.
        constexpr int D = kReplayPrefetch;
        const int32_t T = p.T;
        const int64_t icl = wrow0 + (lane % kEpw);
        const int64_t ic = icl < N ? icl : N - 1;
        float2 ra[D];
        float4 rA[D], rB[D];
        ra[0] = a;
        rA[0] = postA;
        rB[0] = postB;
        auto row_of = [&](int gap) {   // the post-step row of the step `gap` ahead of the current one
            const uint32_t tb = (live ? e.t : 0u) + (uint32_t)gap;
            const uint32_t tn = tb < (uint32_t)T ? tb + 1u : (uint32_t)T;
            return rrow(p, live ? (int64_t)e.path : 0, tn);
        };
        auto load = [&](int d, int kk, int gap) {
            kk = kk < k_steps ? kk : k_steps - 1;
            if (!POL) ra[d] = ld2(gact, (int64_t)kk * N + ic);
            const int64_t r = row_of(gap);
            rA[d] = ld4(mA, r);
            rB[d] = ld4(mB, r);
        };
#pragma unroll
        for (int d = 1; d < D; ++d) load(d, d, d);
        for (int kb = 0; kb < k_steps; kb += D) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const int k = kb + d;
                if (k >= k_steps) break;
                const Mkt post = as_mkt(rA[d]);
                const float4 g = rB[d];
                const float2 ak = ra[d];
                load(d, k + D, D);
                step_part(k, post, g, ak);
                // a lane that just reset (t back to 0 on a new path): its slots for steps
                // k + 1 .. k + D were issued from the old path
                if (__ballot(live && e.t == 0u) != 0ull) {
                    if (live && e.t == 0u) {
#pragma unroll
                        for (int m = 1; m <= D; ++m) {
                            const int sl = (d + m) % D;
                            const int64_t r = rrow(p, e.path, m);
                            rA[sl] = ld4(mA, r);
                            rB[sl] = ld4(mB, r);
                        }
                    }
                }
                flush_part(k);
            }
        }
    } else {
        for (int k = 0; k < k_steps; ++k) {
            Mkt post = as_mkt(postA);
            if (BOOK) post.B = postC;
            step_part(k, post, postB, a);
            if (REPLAY && live && k + 1 < k_steps) {
                const uint32_t tn = e.t + 1 > (uint32_t)p.T ? (uint32_t)p.T : e.t + 1;
                const int64_t r = rrow(p, e.path, tn);
                if (!POL) a = act[(int64_t)(k + 1) * N + i];
                postA = tA[r];
                postB = tB[r];
            }
            flush_part(k);
        }
    }
    if (live) {
        s.t[i] = e.t;
        s.pos[i] = pack_pos(e.call, e.put);
        s.cash[i] = e.cash;
        if (REPLAY && reset_any) {
            s.path[i] = e.path;
            s.s0[i] = e.s0_small ? -1.0f : e.s0;
        }
        if (POL) {
#pragma unroll
            for (int c = 0; c < 7; ++c) s.acc[(int64_t)c * N + i] = acc[c];
            s.acc_len[i] = acc_len;
        }
        if (sums) {
            s.sum[i] = sm0;
            s.sum[N + i] = sm1;
            s.sum[2 * N + i] = sm2;
            s.sum_len[i] = slen;
            s.last[i] = last0;
            s.last[N + i] = last1;
            s.last[2 * N + i] = last2;
            s.last[3 * N + i] = last3;
        }
        if (io.trunc) ((GLOBAL uint8_t*)io.trunc)[i] = 0;
    }
    if constexpr (SINGLE) {
        if (io.sig) raise_step_signal(io);
    }
    HE_TIM(4);
}

// Every step path: Params by value in the kernel arguments.
// GS (GBM only): the obs greeks are evaluated here instead of read from tileB
// (Params::tile_greeks == 0).
template <int MODE, bool INFO, bool SINGLE, bool BOOK, bool FAST, bool POL = false, bool GS = false>
__global__ __launch_bounds__(kBlock) void step_kernel(Params pk, State s, Io io, int k_steps, int slot0) {
    constexpr bool REPLAY = (MODE == HE_MODE_REPLAY);
    step_body<MODE, INFO, SINGLE, BOOK, FAST, POL, GS>(pk, pk.n, REPLAY ? pk.rec : pk.tileA,
                                                   REPLAY ? pk.recg : pk.tileB, pk.tileC, s, io, k_steps, slot0,
                                                       blockIdx.x);
}

// he_step without info: Params from a device-resident copy; the kernel arguments carry
// only the pointers the first loads need (132 B instead of ~850 B of kernarg segment).
struct StepIo {
    const float* act;
    float* obs;
    float* rew;
    uint8_t* term;
    uint8_t* trunc;
    float* tobs;
    uint32_t* sig;      // he_step_signal (Io::sig)
    uint32_t* sig_cnt;
    uint32_t sig_seq;
};
template <int MODE, bool BOOK, bool FAST, bool GS>
__global__ __launch_bounds__(kBlock) void step1_kernel(const Params* __restrict__ pc, int64_t n, const float4* tA,
                                                       const float4* tB, const double* tC, State s, StepIo sio,
                                                       int slot0) {
    Io io;
    io.act = sio.act;
    io.obs = sio.obs;
    io.rew = sio.rew;
    io.term = sio.term;
    io.trunc = sio.trunc;
    io.tobs = sio.tobs;
    io.info = he_info{};
    io.pol_on = false;
    io.sums = false;
    io.sig = sio.sig;
    io.sig_cnt = sio.sig_cnt;
    io.sig_seq = sio.sig_seq;
    step_body<MODE, false, true, BOOK, FAST, false, GS>(*pc, n, tA, tB, tC, s, io, 1, slot0, blockIdx.x);
}

// he_step with VecNormalize attached (he_vecnorm_attach): step1_kernel, then the first half
// of the VecNormalize step (vn_moments.h) over the rows this workgroup has just made --
// from its LDS obs staging tile and the rewards in registers, with no read back -- instead
// of a separate moments launch; the caller's he_vecnorm_apply is then the second half alone.
static_assert(kBlock == vn::kVnThreads && kEpb <= vn::kVnChunk, "one step workgroup = one moments partial");
template <int MODE, bool BOOK, bool FAST, bool GS>
__global__ __launch_bounds__(kBlock) void step1_vn_kernel(const Params* __restrict__ pc, int64_t n, const float4* tA,
                                                          const float4* tB, const double* tC, State s, StepIo sio,
                                                          int slot0, vn::MomentsArgs vm) {
    Io io;
    io.act = sio.act;
    io.obs = sio.obs;
    io.rew = sio.rew;
    io.term = sio.term;
    io.trunc = sio.trunc;
    io.tobs = sio.tobs;
    io.info = he_info{};
    io.pol_on = false;
    io.sums = false;
    io.sig = nullptr;  // more work follows the step in this launch
    // this thread's env (kEpw == 64: env = workgroup base + threadIdx.x): its running return
    // is loaded before the step, so the moments need no further memory round trip
    static_assert(kEpw == 64 && kEpb == kBlock, "one env per thread");
    const int64_t r = (int64_t)blockIdx.x * kEpb + threadIdx.x;
    const double ret_prev = (vm.upd_ret && r < n) ? vm.returns[r] : 0.0;
    const double col_shift = vn::load_col_shift(vm);
    VnHook hk{nullptr, 0.0f, 0.0, false};
    step_body<MODE, false, true, BOOK, FAST, false, GS>(*pc, n, tA, tB, tC, s, io, 1, slot0, blockIdx.x, &hk);
    __syncthreads();  // the workgroup's obs rows (LDS, the final ones incl. reset obs) visible to all its threads
    vn::moments_from_rows(vm, blockIdx.x, hk.tile, hk.rew, ret_prev, col_shift);
}

// he_step with VecNormalize attached for evaluation (he_vecnorm_attach_eval: the statistics
// frozen): step1_kernel, then the whole VecNormalize step over the workgroup's rows
// (vn::apply_frozen_rows) -- no moments, so nothing crosses workgroups and no second launch.
template <int MODE, bool BOOK, bool FAST, bool GS>
__global__ __launch_bounds__(kBlock) void step1_vne_kernel(const Params* __restrict__ pc, int64_t n, const float4* tA,
                                                           const float4* tB, const double* tC, State s, StepIo sio,
                                                           int slot0, vn::ApplyArgs va) {
    Io io;
    io.act = sio.act;
    io.obs = sio.obs;
    io.rew = sio.rew;
    io.term = sio.term;
    io.trunc = sio.trunc;
    io.tobs = sio.tobs;
    io.info = he_info{};
    io.pol_on = false;
    io.sums = false;
    io.sig = nullptr;
    static_assert(kEpw == 64 && kEpb == kBlock, "one env per thread");
    const int64_t r0 = (int64_t)blockIdx.x * kEpb;
    __shared__ vn::FrozenNorm fz;
    const vn::FrozenPre fp = vn::load_frozen(va, r0 + threadIdx.x, r0 + threadIdx.x < n);
    vn::prep_frozen(fz, va, fp);
    VnHook hk{nullptr, 0.0f, 0.0, false};
    step_body<MODE, false, true, BOOK, FAST, false, GS>(*pc, n, tA, tB, tC, s, io, 1, slot0, blockIdx.x, &hk);
    const int rows = (int)((n - r0) < kEpb ? n - r0 : kEpb);
    __syncthreads();  // the workgroup's obs rows (LDS, the final ones incl. reset obs) and fz visible to all
    vn::apply_frozen_rows(va, fz, r0, rows, hk.tile, fp, hk.rew, hk.rew64, hk.term, sio.tobs);
}

// The same moments after any other he_step launch (info requested, a fused market block).
__global__ __launch_bounds__(vn::kVnThreads) void vn_moments_after_step_kernel(vn::MomentsArgs vm) {
    vn::moments_body(vm, blockIdx.x);
}

// Rollout block with the next block's market in the same grid: workgroups
// [0, step_blocks) step block b from tile pk (as step_kernel), the rest generate block
// b+1 into tile pm (as market_kernel, workgroup bid - step_blocks).  One dispatch per
// block on the caller's stream: block b+1's steps are ordered after its market by the
// stream alone, with no cross-queue event between them (measured 25 us between the
// side-stream market's end and the next step dispatch at 65,536 envs).  The step
// workgroups come first in dispatch order and keep s_setprio 3.
// min waves per SIMD of step_market_kernel.  4 (VGPR cap 128: one step + three market
// workgroups per CU) measured +3.8% at 1,048,576 envs and +0% at 65,536, but spills
// ~100 B per lane to scratch; kept at the market kernel's 2 (167 VGPRs, 3 per CU)
constexpr int kFusedWaves = kMktWaves;
// Params of both tile buffers from the device copies (pc[buf] steps, pc[buf ^ 1] is the
// market's): a 0.2 KB kernarg segment instead of 2 x Params by value.
template <int MODE, bool BOOK, bool FAST, bool GS>
__global__ __launch_bounds__(kBlock, kFusedWaves) void step_market_kernel(const Params* __restrict__ pc, int32_t buf,
                                                                           State s, Io io, int k_steps, int slot0,
                                                                           Market cur, Market bak,
                                                                           int32_t step_blocks) {
    static_assert(kBlock == kMktEnvs * kMktLanes, "one workgroup shape for both roles");
    if ((int32_t)blockIdx.x < step_blocks) {
        const Params& pk = pc[buf];
        step_body<MODE, false, false, BOOK, FAST, false, GS>(pk, pk.n, pk.tileA, pk.tileB, pk.tileC, s, io, k_steps,
                                                              slot0, blockIdx.x);
    } else {
        market_body<MODE, BOOK>(pc[buf ^ 1], cur, bak, 0, (int64_t)blockIdx.x - step_blocks);
    }
}

// ------------------------------------------------------------------ LDS rollout
// he_rollout, GBM without a book: ONE launch per call, and the market never leaves the
// chip.  A workgroup owns kLdsEnvs = 64 envs and runs 2 + kLdsProd waves:
//   wave 0 (reward stepper): the f64 state chain of hedging_env_v2.py:181-262 -- trades,
//     costs, cash, portfolio value, P&L, reward -- one lane per env over all K steps,
//     and the reward / terminated stores; it owns the env state;
//   wave 1 (obs stepper): the positions alone (integer trade logic, :181-200) and the
//     13-float observation (:109-143), staged in LDS and stored as 16-B vectors;
//   waves 2.. (producers): the market of the NEXT kLdsM-step block -- Philox4x32-10
//     normals, the GBM price (rbergomi_sim.py:454-464), rolling-ATM marks
//     (option_calculator.py:11-27) and the obs greeks (hedging_env_v2.py:79-107) -- as
//     24-B records {S, C, P, delta_c, gamma, delta_p} into the other LDS buffer while
//     the steppers consume the current one.
// kLdsLanes lanes per env, lane `sub` making slots [sub H, sub H + H) of a block; the
// sequential f64 price chain passes from lane to lane through shuffles.  One workgroup
// barrier per block hands a buffer over.  The device functions and their operands are
// market_body's / step_kernel's, so the outputs are the tile kernels' bits (tests: LDS
// rollouts == tile rollouts == repeated he_step).  HBM traffic is the step I/O of
// hedging_env_v2.py:175-294 only: actions in, obs / reward / terminated out, and the
// per-env state + market position once per launch.
// SIMD-balanced wave roles (lds_role, below); HE_LDS_BALANCE=0 only in the placement
// diagnostics of tools/lds_hwid.py
#ifndef HE_LDS_BALANCE
#define HE_LDS_BALANCE 1
#endif


// Wave priorities (s_setprio).  The reward stepper above the obs stepper, GBM without a book
// (same-box A/B r03s9, config 2, two runs each: priority 0 312 / 300 us per launch, 1 319 /
// 313, 2 314 / 302, 3 305 / 296); with a book or Heston (producer-bound) at 0 (3: config 4
// +4 %, config 5 +3 %).  The obs wave is the GBM workgroup's critical chain: it wins issue
// over the producers.
constexpr int kPrioRewBook = 0, kPrioReplayRew = 0, kPrioObs = 2, kPrioProd = 1;
// GBM without a book (configs 2, 3): the four roles of a SIMD at four distinct priorities, the two
// producer roles one apart.  At equal priority the SIMD's issue arbitration falls back to age, and
// on 3 of a CU's 4 SIMDs the producer of the older workgroup won every tie: the CU's oldest
// workgroup finished ~10 % before the median and the youngest ~7 % after it, and a launch lasts as
// long as its slowest workgroup (tools/lds_timing.py, r05s6).  With no ties every workgroup wins one
// producer contest and loses one: the workgroups end within 17 us of each other instead of 53, and
// the launch takes 295.5 against 300.0 us (3 same-box pairs, r05s8_ab_prio_split.txt).
// (priority orders rew/obs/p0/p1 3/1/2/0, 2/3/1/0, 3/0/2/1, 1/2/3/0 measured +2.4 %, +0.4 %, +9 %,
// -0.2 %: r05s9_ab_prio_perm.txt)
constexpr int kPrioGbmRew = 3, kPrioGbmObs = 2, kPrioGbmProd0 = 1, kPrioGbmProd1 = 0;
// Producer lanes per env: 2 producer waves (4 waves per workgroup, 4 workgroups per CU at 128
// VGPRs); with a book or Heston same-box A/B against 4 (r02 g2): config 4 1.11e10 -> 1.21e10,
// config 5 1.19e10 -> 1.25e10 env-steps/s
constexpr int kLdsLanesGbm = 2, kLdsLanesBook = 2, kLdsMinWavesBook = 4;
constexpr int kLdsEnvs = 64;                         // envs per workgroup = one stepper wave
// slots per LDS market block (same-box A/B r02: M = 16 -12 %, M = 4 -3 %)
constexpr int kLdsM = 8;
constexpr int kLdsPrefetch = kLdsM % 6 == 0 ? 6 : (kLdsM % 4 == 0 ? 4 : kLdsM);  // steps of actions in flight
static_assert(kLdsM % kLdsPrefetch == 0, "the action ring index is the slot mod D");

// Workgroup geometry of one market configuration: `lanes` producer lanes per env in
// `lanes` producer waves (64 / lanes envs each), each lane making H consecutive slots.
// min waves per SIMD (GBM): 4 workgroups per CU need 4 (2 + prod) / 4 per SIMD if the
// hardware spreads every workgroup evenly; one more leaves room for an uneven placement.
// With a book the kernel is VALU-bound: 128 VGPRs (4 waves per SIMD) for the marks.
template <int MODE, bool BOOK>
struct LdsGeom {
    static constexpr bool HESTON = MODE == HE_MODE_HESTON;
    // Heston: two normals, a sqrt and a per-step Black-Scholes constant set per slot --
    // producer-bound like a book, so it takes the book's lane count
    static constexpr int lanes = (BOOK || HESTON) ? kLdsLanesBook : kLdsLanesGbm;
    static constexpr int prod = lanes;
    static constexpr int penvs = kLdsEnvs / lanes;
    static constexpr int threads = 64 * (2 + prod);  // + the reward and the obs stepper waves
    static constexpr int H = kLdsM / lanes;
    // the balanced placement (HE_LDS_BALANCE) puts exactly one wave of each of a CU's 4
    // workgroups on every SIMD: 4 waves per SIMD, 128 VGPRs (the lockstep producers hold
    // 122); the unbalanced build keeps a spare wave for an uneven placement
    static constexpr int minwaves = (BOOK || HESTON) ? kLdsMinWavesBook
                                                     : (HE_LDS_BALANCE ? 4 : (4 * (2 + prod) + 3) / 4 + 1);
    static_assert(H * lanes == kLdsM && penvs * lanes == kLdsEnvs, "producer lane layout");
};

// LDS: the market records, double-buffered by block, [slot][env]: {S, C} pairs and P
// (12 B per env-slot, conflict-free lane accesses), the obs wave's two row staging
// tiles, and with a book its f64 value per slot: 19.7 KB at M = 8 (GBM), so all 65,536
// envs of BASELINE configs[1] are resident at once; 27.9 KB with a book.
// Book tau-table rows held in LDS (8 KB): a book whose latest expiry is past it takes the
// tile kernels (lds_rollout_eligible).  The producers' per-option table reads are then LDS
// reads instead of L1/L2 gathers on their critical chain.
constexpr int kLdsBookRows = 256;
// The lean reward stepper's time-penalty terms theta (T - t) / 252 by episode step t, made once
// per launch (thp in LdsMarketT; without a book: headline 287.5 -> 283.7 us, 3 of 3 same-box
// pairs; with one config 4 lost 0.5 %, r05s17_ab_thp_table.txt): episodes of fewer than
// lds_thp_rows steps take the lean kernel without a book (lds_lean_config)
constexpr int lds_thp_rows() { return 512; }
template <int MODE, bool BOOK, bool LEAN = false>
struct LdsMarketT {
    static constexpr int NB = 2;                                       // market buffers
    static constexpr bool THP = LEAN && !BOOK;
    double thp[THP ? lds_thp_rows() : 1];
    float2 sc[NB][kLdsM][kLdsEnvs];
    float pp[NB][kLdsM][kLdsEnvs];
    float stage[2][kLdsEnvs * kObs];                                   // obs row staging, by step parity
    double bk[BOOK ? 2 : 1][BOOK ? kLdsM : 1][kLdsEnvs];                // book value of every slot
    float vv[MODE == HE_MODE_HESTON ? 2 : 1][MODE == HE_MODE_HESTON ? kLdsM : 1][kLdsEnvs];  // Heston: f32 v_t
    double btab[BOOK ? kLdsBookRows : 1][4];  // the book's tau table (p.book_tab), copied at launch start
    // the book's options, copied at launch start (config 4: 10.38 -> 8.98 ms per launch against
    // reading them through the scalar cache)
    BookOpt bopt[BOOK ? HE_BOOK_MAX : 1];
};
static_assert(kLdsM > 8 || sizeof(LdsMarketT<HE_MODE_GBM, false>) <= 40 * 1024, "4 workgroups per CU");
static_assert(kLdsM > 8 || sizeof(LdsMarketT<HE_MODE_GBM, false, true>) <= 40 * 1024 - 64, "4 workgroups per CU");
static_assert(kLdsM > 8 || sizeof(LdsMarketT<HE_MODE_HESTON, true>) <= 40 * 1024, "4 workgroups per CU");

#ifdef HE_LDS_TIMING
// Diagnostic builds only: per wave role (0 reward, 1 obs, 2-3 producers) and workgroup,
// {cycles from start to end, cycles spent in barriers (s_memtime), 100 MHz ticks from
// start to end (s_memrealtime)}, read by he_debug_lds_timing.
__device__ uint64_t g_lds_tim[4][4096][5];   // + the role's start and end on the 100 MHz clock
#define LDS_T0() uint64_t tim_t0 = __builtin_amdgcn_s_memtime(), tim_bar = 0, tim_r0 = __builtin_amdgcn_s_memrealtime()
#define LDS_BAR()                                                  \
    do {                                                           \
        const uint64_t tb_ = __builtin_amdgcn_s_memtime();         \
        __syncthreads();                                           \
        tim_bar += __builtin_amdgcn_s_memtime() - tb_;             \
    } while (0)
#define LDS_T1(role)                                                                     \
    do {                                                                                 \
        if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096) {                              \
            g_lds_tim[role][blockIdx.x][0] = __builtin_amdgcn_s_memtime() - tim_t0;      \
            g_lds_tim[role][blockIdx.x][1] = tim_bar;                                    \
            const uint64_t r1_ = __builtin_amdgcn_s_memrealtime();                       \
            g_lds_tim[role][blockIdx.x][2] = r1_ - tim_r0;                               \
            g_lds_tim[role][blockIdx.x][3] = tim_r0;                                     \
            g_lds_tim[role][blockIdx.x][4] = r1_;                                        \
        }                                                                                \
    } while (0)
#else
#define LDS_T0() do {} while (0)
#define LDS_BAR() __syncthreads()
#define LDS_T1(role) do {} while (0)
#endif

// Store one workgroup's 64 obs rows (the image, 832 floats) as 3 x 16 B + 4 B per lane:
// every lane active, no branch.  (Write-through sc1 stores: config 2 +-0, config 6 +1.5 %.)
__device__ __forceinline__ void flush_obs_full(const float* img, float* out, int64_t row0, int lane) {
    asm volatile("" ::: "memory");
    GLOBAL float* dst = (GLOBAL float*)out + row0 * kObs;
    GLOBAL v4f* d4 = (GLOBAL v4f*)dst;
    const v4f* s4 = reinterpret_cast<const v4f*>(img);
    d4[lane] = s4[lane];
    d4[lane + 64] = s4[lane + 64];
    d4[lane + 128] = s4[lane + 128];
    dst[768 + lane] = img[768 + lane];
    asm volatile("" ::: "memory");
}

// The stepper waves.  OBS = false: the reward wave; OBS = true: the obs wave.  Both make
// the same integer decisions from the same actions, so they agree on every position and
// done flag.  LEAN (the FAST configuration with every output present, lds_lean_config):
// the per-handle constants in registers and no branch in a step (selects; div_by_nb),
// so the unrolled steps of a block form one basic block the scheduler can overlap;
// otherwise the generic step_env / make_obs code.
//
// Memory-op discipline (what keeps the stores in flight): every lane is active -- a
// lane past the last env mirrors env N-1 (same inputs, so its stores write the same
// values to the same addresses) -- and a full block is straight-line code (unrolled
// slots, no branch around a load or store), so the waitcnt pass never merges paths with
// different outstanding memory ops.  (A copy of a pending load's register at a merge,
// e.g. the action ring at a loop back-edge behind a `break`, costs an s_waitcnt
// vmcnt(0): every store of the wave drained.)  A partial last block takes a generic loop.
// POL (he_rollout_policy, lean configurations): the baseline policy is evaluated by BOTH steppers
// from the obs row each has in hand -- the same function of the same operands, so the same action
// bits -- the obs stepper from the row it just made, the reward stepper from the positions it
// tracks and the obs greeks it re-evaluates from the slot's market; no action crosses the waves,
// and the LDS block pipeline is the stored-action rollout's.  The reward stepper keeps the
// evaluation loops' episode sums and records (step_body's POL), the obs stepper stores the actions.
template <int MODE, bool BOOK, bool LEAN, bool OBS, bool POL = false>
__device__ __forceinline__ void lds_stepper(const Params& p, State s, const Io& io, int k_steps, const Market& cur,
                                            LdsMarketT<MODE, BOOK, LEAN>& L, int64_t base) {
    constexpr int D = kLdsPrefetch;
    constexpr bool HESTON = MODE == HE_MODE_HESTON;
    const int lane = threadIdx.x & 63;
    const int64_t N = p.n;
    const int nfull = k_steps / kLdsM;          // full blocks
    const int tail = k_steps - nfull * kLdsM;   // steps of the partial last block
    const int64_t i0 = base + lane;
    const int64_t i = i0 < N ? i0 : N - 1;      // lanes past N mirror env N-1
    const int wrows = (int)((N - base) < kLdsEnvs ? (N - base) : kLdsEnvs);
    const Mkt rst{p.rstv[0], p.rstv[1], p.rstv[2], p.rstv[3], BOOK ? p.book_rst : 0.0};
    const GLOBAL v2f* gact = (const GLOBAL v2f*)io.act;
    GLOBAL float* const grew = (GLOBAL float*)io.rew;
    GLOBAL uint8_t* const gterm = (GLOBAL uint8_t*)io.term;
    if (!BOOK && !HESTON) {
        if (OBS) __builtin_amdgcn_s_setprio(kPrioGbmObs);
        else __builtin_amdgcn_s_setprio(kPrioGbmRew);
    } else {
        if (OBS) __builtin_amdgcn_s_setprio(kPrioObs);
        else __builtin_amdgcn_s_setprio(kPrioRewBook);
    }
    LDS_T0();
    Env e{};
    Mkt pre = rst;
    double pv_last = 0.0;
    {
        const uint32_t t0 = s.t[i];
        const uint32_t pk = s.pos[i];
        e.t = t0;
        e.call = unpack_lo(pk);
        e.put = unpack_hi(pk);
        e.path = -1;
        e.s0_small = rst.S < 1e-6f;
        e.s0 = e.s0_small ? 1.0f : rst.S;
        if (!OBS) {
            e.cash = s.cash[i];
            // the market the env stands at: the block-start record of market_body (f32 S)
            if (t0 != 0) {
                const double Sc = cur.S[i];
                const double Vc = HESTON ? cur.v[i] : p.var;
                // the book at the block start: market_body's slot 0 (same function, operands)
                const double Bc = BOOK ? book_value(p, Sc, Vc, (int32_t)t0, cur.M[i]) : 0.0;
                pre = Mkt{(float)Sc, HESTON ? (float)Vc : p.var_f, cur.C[i], cur.P[i], Bc};
            }
            pv_last = portfolio_value<BOOK>(p, e, pre);
        }
    }
    // the reward wave's episode summaries {return, sum pnl, sum cost, length} of the last
    // finished episode (he_episode_summaries) and the running sums behind them (s.sum)
    double sm0 = 0.0, sm1 = 0.0, sm2 = 0.0;
    uint32_t slen = 0;
    float last0 = 0.f, last1 = 0.f, last2 = 0.f, last3 = 0.f;
    if (!OBS) {
        sm0 = s.sum[i];
        sm1 = s.sum[N + i];
        sm2 = s.sum[2 * N + i];
        slen = s.sum_len[i];
        last0 = s.last[i];
        last1 = s.last[N + i];
        last2 = s.last[2 * N + i];
        last3 = s.last[3 * N + i];
    }
    auto account = [&](double reward, double pnl, double tc, bool term) {
        const double a0 = sm0 + reward, a1 = sm1 + pnl, a2 = sm2 + tc;
        const uint32_t n = slen + 1u;
        // the conversions made unconditionally (opaque): sunk under the selects they turn
        // them into branches, and the whole autoreset with them
        float f0 = (float)a0, f1 = (float)a1, f2 = (float)a2, f3 = (float)n;
        asm volatile("" : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3));
        last0 = term ? f0 : last0;
        last1 = term ? f1 : last1;
        last2 = term ? f2 : last2;
        last3 = term ? f3 : last3;
        sm0 = term ? 0.0 : a0;
        sm1 = term ? 0.0 : a1;
        sm2 = term ? 0.0 : a2;
        slen = term ? 0u : n;
    };
    float2 ra[D];
    if constexpr (!POL) {
#pragma unroll
        for (int d = 0; d < D; ++d) ra[d] = ld2(gact, (int64_t)(d < k_steps ? d : k_steps - 1) * N + i);
    } else {
#pragma unroll
        for (int d = 0; d < D; ++d) ra[d] = make_float2(0.0f, 0.0f);
    }
    // POL: the obs columns the policies read (3, 4, 7, 9) of the env's current obs row, as
    // step_body makes them at a launch start, and the episode sums of the evaluation loops
    const int pol = POL ? io.pol.policy : HE_POLICY_NO_HEDGE;
    const bool pol_greeks = POL && pol != HE_POLICY_NO_HEDGE;   // wave-uniform
    float po3 = 0.0f, po4 = 0.0f, pcd = 0.0f, ppd = 0.0f;
    double acc[7] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    uint32_t acc_len = 0;
    // (the lean configuration has max_contracts_held > 0 and record_metrics; the generic steppers
    // test them, as make_obs does)
    const bool pmh = LEAN || p.maxh != 0, prm = LEAN || p.record_metrics;
    if constexpr (POL) {
        po3 = pmh ? div_int_byf((float)e.call, p.maxh_f, p.inv_maxh_f) : 0.0f;
        po4 = pmh ? div_int_byf((float)e.put, p.maxh_f, p.inv_maxh_f) : 0.0f;
        if (e.t == 0) {
            pcd = p.rstv[4 + 7];
            ppd = p.rstv[4 + 9];
        } else if (pol_greeks && prm) {
            const float S0f = (float)cur.S[i];
            float4 g0;
            if constexpr (!LEAN) g0 = greeks_fast<!HESTON>(p, S0f, HESTON ? (float)cur.v[i] : p.var_f);
            else if constexpr (HESTON) g0 = greeks_fast<false>(p, S0f, (float)cur.v[i]);
            else g0 = greeks_lean(S0f, p.g_num_drift, p.g_inv_sst_f, p.g_sst_f);
            pcd = g0.x;
            ppd = g0.z;
        }
        if (!OBS) {
#pragma unroll
            for (int c = 0; c < 7; ++c) acc[c] = s.acc[(int64_t)c * N + i];
            acc_len = s.acc_len[i];
        }
    }
    // POL, the reward wave: step_body's sums in step order and the record of a finished episode
    auto pol_account = [&](double reward, double pnl, double ps, double tc, double rpc, double tcp, bool term) {
        acc[0] = acc[0] + reward;
        acc[1] = acc[1] + pnl;
        acc[2] = acc[2] + fabs(ps);
        acc[3] = acc[3] + tc;
        acc[4] = acc[4] + rpc;
        acc[5] = acc[5] + tcp;
        acc[6] = acc[6] + ps;
        acc_len += 1u;
        if (__ballot(term) != 0ull) {   // fixed-length episodes end together: uniform
            if (term) {
                if (i0 < N) {   // not the lanes mirroring env N - 1
                    const unsigned long long r = atomicAdd(io.pol.count, 1ull);
                    if ((int64_t)r < io.pol.cap) {
                        he_episode_record rec;
                        rec.env_id = p.goff + i;
                        rec.length = (int32_t)acc_len;
                        rec.reserved = 0;
                        rec.reward_sum = acc[0];
                        rec.pnl_sum = acc[1];
                        rec.abs_pnl_sum = acc[2];
                        rec.cost_sum = acc[3];
                        rec.pnl_penalty_sum = acc[4];
                        rec.cost_penalty_sum = acc[5];
                        rec.per_share_pnl_sum = acc[6];
                        rec.reserved2 = 0.0;
                        io.pol.rec[r] = rec;
                    }
                }
                last0 = (float)acc[0];
                last1 = (float)acc[1];
                last2 = (float)acc[3];
                last3 = (float)acc_len;
#pragma unroll
                for (int c = 0; c < 7; ++c) acc[c] = 0.0;
                acc_len = 0;
            }
        }
    };

    // ---- the block loop over a step function step(buf, sl, k, action, in_full_block)
    constexpr int NB = LdsMarketT<MODE, BOOK, LEAN>::NB;
    auto run_blk = [&](auto&& step) {
        LDS_BAR();  // block 0 produced
        for (int b = 0; b < nfull; ++b) {
#if defined(HE_LDS_DIAG) && HE_LDS_DIAG == 2
            LDS_BAR();  // diagnostic build: the steppers only keep the barrier count
            continue;
#endif
            const int buf = b % NB;
#pragma unroll
            for (int sl = 0; sl < kLdsM; ++sl) {
                const int k = b * kLdsM + sl;
                const float2 ak = ra[sl % D];
                if constexpr (!POL) {
                    const int kn = k + D;
                    ra[sl % D] = ld2(gact, (int64_t)(kn < k_steps ? kn : k_steps - 1) * N + i);
                }
                step(buf, sl, k, ak, std::true_type{});
            }
            LDS_BAR();  // buffer b % NB handed back, block b + 1 produced
        }
        if (tail) {
#if !(defined(HE_LDS_DIAG) && HE_LDS_DIAG == 2)
            const int buf = nfull % NB;
            for (int sl = 0; sl < tail; ++sl) {
                const int k = nfull * kLdsM + sl;
                step(buf, sl, k, POL ? make_float2(0.0f, 0.0f) : ld2(gact, (int64_t)k * N + i), std::false_type{});
            }
#endif
            LDS_BAR();
        }
    };

    if constexpr (LEAN) {
        // the FAST configuration's constants (fast_config): v2, loss != mse, generate mode
        const float mt_f = p.mt_f, maxh_f = p.maxh_f, inv_maxh_f = p.inv_maxh_f;
        const int32_t mt = p.mt, maxh = p.maxh, T = p.T;
        if (OBS) {
            const float s0s_f = p.s0s_f, inv_s0s_f = p.inv_s0s_f;
            const float T_f = p.T_f, inv_T_f = p.inv_T_f, var_f = p.var_f;
            // the per-step constants held in VGPRs (opaque: the scalar reloads they would
            // otherwise be rematerialized as share lgkmcnt with the LDS traffic)
            const float gnd = p.g_num_drift, gis = p.g_inv_sst_f, gsf = p.g_sst_f;
            float ro[kObs];
#pragma unroll
            for (int c = 0; c < kObs; ++c) ro[c] = p.rstv[4 + c];
            float preS = pre.S;
            if (e.t != 0) preS = (float)cur.S[i];
            // Heston: the slot's f32 variance v_t (obs column 5, the greeks' sigma) and the previous
            // step's (column 12's change)
            float preV = rst.v;
            if (HESTON && e.t != 0) preV = (float)cur.v[i];
            const double s0s_d = p.s0s_d, inv_s0s_d = p.inv_s0s_d;
            auto obs_step = [&](int buf, int sl, int k, float2 ak, auto full) {
                const float2 r0 = L.sc[buf][sl][lane];
                const float rP = L.pp[buf][sl][lane];
                const float vk = HESTON ? L.vv[HESTON ? buf : 0][HESTON ? sl : 0][lane] : var_f;
                // the obs greeks: greeks_fast of the market price, as market_kernel makes them
                // (a block's 8 evaluated in lockstep up front measured +-0: r03s24); Heston: at the
                // slot's variance, the generic steppers' greeks_fast<false>
                float4 g;
                if constexpr (HESTON) g = greeks_fast<false>(p, r0.x, vk);
                else g = greeks_lean(r0.x, gnd, gis, gsf);
                if constexpr (POL) {   // the policy on the obs row this env stands at (step_body's POL)
                    ak = policy_action(p, pol, e.call, e.put, po3, po4, pcd, ppd);
                    if (io.pol.act_out) {
                        v2f av = {ak.x, ak.y};
                        ((GLOBAL v2f*)io.pol.act_out)[(int64_t)k * N + i] = av;
                    }
                }
                // (i)-(ii) of step_env: the integer trade logic (:181-200)
                const int32_t nc = e.call + trade_round(ak.x * mt_f, mt);
                const int32_t nq = e.put + trade_round(ak.y * mt_f, mt);
                const int32_t cc = clamp_pos(nc, maxh);
                const int32_t qq = clamp_pos(nq, maxh);
                const uint32_t t1 = e.t + 1;
                const bool term = (int32_t)t1 >= T;
                // make_obs<true> (hedging_env_v2.py:109-143) on the post-step state, or the
                // reset obs on a terminal step (SB3 autoreset)
                float o[kObs];
                // the price columns over max(S0, 25).  S by an f32 Markstein step (div_f32_byf: S >=
                // 1e-8 and max(S0, 25) <= 1e20 (lds_lean_config), so S / max(S0, 25) is a normal
                // f32 number; 292.6 -> 287.8 us per launch for all three columns, r05s13_ab_obs_f32.txt).
                // C and P through f64 (div_f32_by): a deep out-of-the-money mark of a rolling ATM
                // option can be tiny -- |d| past ~13 at a small S or sigma, in GBM as in Heston --
                // where the f32 step's residual leaves the normal range
                if constexpr (HESTON) {
                    o[0] = div_f32_by(r0.x, s0s_d, inv_s0s_d);   // Heston: the same, S included
                } else {
                    o[0] = div_f32_byf(r0.x, s0s_f, inv_s0s_f);
                }
                o[1] = div_f32_by(r0.y, s0s_d, inv_s0s_d);
                o[2] = div_f32_by(rP, s0s_d, inv_s0s_d);
                o[3] = div_int_byf((float)cc, maxh_f, inv_maxh_f);
                o[4] = div_int_byf((float)qq, maxh_f, inv_maxh_f);
                o[5] = vk;
                o[6] = div_int_byf((float)(T - (int32_t)t1), T_f, inv_T_f);
                o[7] = g.x;
                o[8] = g.y;
                o[9] = g.z;
                o[10] = g.y;
                o[11] = lag_return_lean(r0.x, preS);
                o[12] = (preS == 0.0f) ? 0.0f : np_clipf(vk - (HESTON ? preV : var_f), -1.0f, 1.0f);
                // staged in LDS (two tiles, alternating by step: the next step's row writes
                // do not wait behind this step's read-back) and stored as whole 16-B lines
                float* const tile = L.stage[k & 1];
                // the reset row over it only on a step that ends an episode (a wave-uniform branch:
                // fixed-length episodes end together) instead of 13 selects every step (with the f32
                // quotients 287.8 -> 286.5 us, r05s13_ab_obs_f32.txt)
#pragma unroll
                for (int c = 0; c < kObs; ++c) tile[lane * kObs + c] = o[c];
                if (__ballot(term) != 0ull) {
                    if (term) {
#pragma unroll
                        for (int c = 0; c < kObs; ++c) tile[lane * kObs + c] = ro[c];
                    }
                }
                if (!POL || io.obs) {   // policy rollouts may return no obs (a kernel argument: uniform)
                    float* out = io.obs + (int64_t)k * N * kObs;
                    if constexpr (decltype(full)::value) flush_obs_full(tile, out, base, lane);
                    else flush_obs_wave(tile, out, base, wrows, lane);
                }
                if constexpr (POL) {   // the row this step returns (the reset row on a terminal step)
                    po3 = term ? ro[3] : o[3];
                    po4 = term ? ro[4] : o[4];
                    pcd = term ? ro[7] : o[7];
                    ppd = term ? ro[9] : o[9];
                }
                e.t = term ? 0u : t1;
                e.call = term ? 0 : cc;
                e.put = term ? 0 : qq;
                preS = term ? rst.S : r0.x;
                if (HESTON) preV = term ? rst.v : vk;
            };
            if (wrows == kLdsEnvs)
                run_blk([&](int buf, int sl, int k, float2 ak, auto) { obs_step(buf, sl, k, ak, std::true_type{}); });
            else
                run_blk([&](int buf, int sl, int k, float2 ak, auto) { obs_step(buf, sl, k, ak, std::false_type{}); });
        } else {
            const double tcpc = p.tcpc, slip_frac = p.slip_frac, lam = p.lam, w = p.w, theta = p.theta;
            const double shares_d = p.shares_d, inv_shares = p.inv_shares, den = p.den, inv_den = p.inv_den;
            const double inv_252 = p.inv_252, init_cash = p.initial_cash;
            const float shares_f = p.shares_f;
            // step_env's PV0 (:167-168): f32, of the reset market -- one constant here (+ the
            // reset market's book)
            double pv0 = (double)((shares_f * rst.S + 0.0f) + p.init_cash_f);
            if (BOOK) pv0 = pv0 + rst.B;
            // without a book: the time penalty by episode step, theta * (T - t1) / 252 (:257-259),
            // into this wave's table (T < lds_thp_rows: lds_lean_config) -- an LDS read per step
            // instead of an int conversion, an f64 quotient and a multiply; this wave's only
            if constexpr (LdsMarketT<MODE, BOOK, LEAN>::THP) {
                for (int t = lane; t <= T; t += 64)
                    L.thp[t] = theta * div_int_by((double)(T - t), 252.0, inv_252);
            }
            // the marks times 100 in f64, carried from step to step: (n C) 100 = n (C 100) exactly
            // (|n| < 2^16 contracts -- int16 positions, max_contracts_held <= 32767 -- times a 24-bit C
            // times 100 is at most 47 bits), so the slippage and option-value terms below are the
            // reference's products bit for bit with two conversions and two multiplies fewer a step
            double preC100 = (double)pre.C * 100.0, preP100 = (double)pre.P * 100.0;
            // the previous value an episode's first step differences against is PV0 (:167-168):
            // set where the episode starts (here, and by the autoreset below), not tested per step
            if (e.t == 0) pv_last = pv0;
            const double rstC100 = (double)rst.C * 100.0, rstP100 = (double)rst.P * 100.0;
            // POL: the reset row's policy columns, and the obs greeks' constants
            const float rs3 = p.rstv[4 + 3], rs4 = p.rstv[4 + 4], rs7 = p.rstv[4 + 7], rs9 = p.rstv[4 + 9];
            const float gnd = p.g_num_drift, gis = p.g_inv_sst_f, gsf = p.g_sst_f;
            run_blk([&](int buf, int sl, int k, float2 ak, auto) {
                const int64_t koff = (int64_t)k * N;
                const float2 sc = L.sc[buf][sl][lane];
                const float pP = L.pp[buf][sl][lane];
                const double C100 = (double)sc.y * 100.0, P100 = (double)pP * 100.0;
                const double pv_prev = pv_last;
                if constexpr (POL) ak = policy_action(p, pol, e.call, e.put, po3, po4, pcd, ppd);
                // (i)-(ii) trades (:181-200)
                const int32_t nc = e.call + trade_round(ak.x * mt_f, mt);
                const int32_t nq = e.put + trade_round(ak.y * mt_f, mt);
                const int32_t cc = clamp_pos(nc, maxh);
                const int32_t qq = clamp_pos(nq, maxh);
                const int32_t dc = cc - e.call, dp = qq - e.put;
                // (iii) commission + slippage on the pre-step marks (:203-213)
                const int32_t adc = dc < 0 ? -dc : dc, adp = dp < 0 ? -dp : dp;
                const double commission = (double)(adc + adp) * tcpc;
                const double slc = ((double)adc * preC100) * slip_frac;   // (((adc C) 100) slip: :205-209)
                const double slp = ((double)adp * preP100) * slip_frac;
                const double tc = commission + (slc + slp);
                const double cash = e.cash - tc;
                // (iv)-(vi) advance, mark-to-market (:216-238)
                const uint32_t t1 = e.t + 1;
                const bool term = (int32_t)t1 >= T;
                const double optv = (double)cc * C100 + (double)qq * P100;   // (cc C) 100 + (qq P) 100
                double pv = ((double)(shares_f * sc.x) + optv) + cash;
                if (BOOK) pv = pv + L.bk[buf][sl][lane];  // liability book (extension): after cash
                const double pnl = pv - pv_prev;
                const double ps = div_by_nb(pnl, shares_d, inv_shares);
                // (vii) reward (:243-262)
                const double term_v = div_by_nb(fabs(ps), den, inv_den);
                const double rpc = (-w) * term_v;
                const double tcp = lam * tc;
                const double thp = LdsMarketT<MODE, BOOK, LEAN>::THP
                                       ? L.thp[LdsMarketT<MODE, BOOK, LEAN>::THP ? t1 : 0]
                                       : theta * div_int_by((double)(T - (int32_t)t1), 252.0, inv_252);
                const double reward = (rpc - tcp) - thp;
                if (!POL || grew) grew[koff + i] = (float)reward;
                if (!POL || gterm) gterm[koff + i] = term ? 1 : 0;
                if constexpr (POL) {
                    pol_account(reward, pnl, ps, tc, rpc, tcp, term);
                    // the obs row this step returns, as the obs stepper makes it: the positions'
                    // columns and the greeks of the slot's market (greeks_lean / greeks_fast<false>)
                    float gx = 0.0f, gz = 0.0f;
                    if (pol_greeks) {
                        float4 g;
                        if constexpr (HESTON) g = greeks_fast<false>(p, sc.x, L.vv[HESTON ? buf : 0][HESTON ? sl : 0][lane]);
                        else g = greeks_lean(sc.x, gnd, gis, gsf);
                        gx = g.x;
                        gz = g.z;
                    }
                    po3 = term ? rs3 : div_int_byf((float)cc, maxh_f, p.inv_maxh_f);
                    po4 = term ? rs4 : div_int_byf((float)qq, maxh_f, p.inv_maxh_f);
                    pcd = term ? rs7 : gx;
                    ppd = term ? rs9 : gz;
                } else {
                    account(reward, pnl, tc, term);
                }
                pv_last = term ? pv0 : pv;
                // SB3 autoreset (selects)
                e.t = term ? 0u : t1;
                e.call = term ? 0 : cc;
                e.put = term ? 0 : qq;
                e.cash = term ? init_cash : cash;
                preC100 = term ? rstC100 : C100;
                preP100 = term ? rstP100 : P100;
            });
        }
    } else {
        // (the generic steps' Params fields pinned in SGPRs instead of the scalar-cache reloads:
        // config 5 +4 %, config 4 -1 %, r03s16)
        if (OBS && e.t != 0) pre = Mkt{(float)cur.S[i], HESTON ? (float)cur.v[i] : p.var_f, cur.C[i], cur.P[i], 0.0};
        // full: every lane an env of its own (wrows == kLdsEnvs), the obs rows stored by the
        // branch-free flush_obs_full (its rows == 64 test in flush_obs_wave held values live
        // across a branch in every step: config 5's obs stepper spilled there)
        auto step = [&](int buf, int sl, int k, float2 ak, auto full) {
            const int64_t koff = (int64_t)k * N;
            const float2 sc = L.sc[buf][sl][lane];
            const float vk = HESTON ? L.vv[HESTON ? buf : 0][HESTON ? sl : 0][lane] : p.var_f;
            const Mkt post{sc.x, vk, sc.y, L.pp[buf][sl][lane], BOOK ? L.bk[buf][sl][lane] : 0.0};
            if constexpr (POL) ak = policy_action(p, pol, e.call, e.put, po3, po4, pcd, ppd);
            if (OBS) {
                if (POL && io.pol.act_out) {
                    v2f av = {ak.x, ak.y};
                    ((GLOBAL v2f*)io.pol.act_out)[koff + i] = av;
                }
                // the obs greeks of market_body's greeks records (Heston: of the slot's v)
                float4 g = p.record_metrics ? greeks_fast<!HESTON>(p, post.S, post.v) : make_float4(0.f, 0.f, 0.f, 0.f);
                g.w = lag_return(post.S, pre.S);
                // (i)-(ii) of step_env: the integer trade logic (:181-200)
                const int32_t nc = e.call + trade_round(ak.x * p.mt_f, p.mt);
                const int32_t nq = e.put + trade_round(ak.y * p.mt_f, p.mt);
                e.call = clamp_pos(nc, p.maxh);
                e.put = clamp_pos(nq, p.maxh);
                e.t = e.t + 1;
                const bool term = (int32_t)e.t >= p.T;
                float o[kObs];
                make_obs<false>(p, e, post, g, pre.S, pre.v, o);
                float* const tile = L.stage[k & 1];
#pragma unroll
                for (int c = 0; c < kObs; ++c) tile[lane * kObs + c] = term ? p.rstv[4 + c] : o[c];  // SB3 autoreset obs
                if constexpr (POL) {   // the row this step returns
                    po3 = term ? p.rstv[4 + 3] : o[3];
                    po4 = term ? p.rstv[4 + 4] : o[4];
                    pcd = term ? p.rstv[4 + 7] : o[7];
                    ppd = term ? p.rstv[4 + 9] : o[9];
                }
                if (io.obs) {
                    if constexpr (decltype(full)::value) flush_obs_full(tile, io.obs + koff * kObs, base, lane);
                    else flush_obs_wave(tile, io.obs + koff * kObs, base, wrows, lane);
                }
                pre = term ? rst : post;
                if (term) env_reset_common(p, e);
            } else {
                StepOut so;
                step_env<BOOK, false>(p, e, pre, post, ak.x, ak.y, pv_last, so);
                pv_last = so.pv;
                if (grew) grew[koff + i] = (float)so.reward;
                if (gterm) gterm[koff + i] = so.term ? 1 : 0;
                if constexpr (POL) {
                    pol_account(so.reward, so.pnl, so.ps, so.tc, so.rpc, so.tcp, so.term);
                    // the row this step returns, as the obs stepper makes it (make_obs<false>'s columns
                    // of the post-trade positions and the slot's greeks, or the reset row)
                    float gx = 0.0f, gz = 0.0f;
                    if (pol_greeks && prm) {
                        const float4 g = greeks_fast<!HESTON>(p, post.S, post.v);
                        gx = g.x;
                        gz = g.z;
                    }
                    po3 = so.term ? p.rstv[4 + 3] : (pmh ? div_int_byf((float)e.call, p.maxh_f, p.inv_maxh_f) : 0.0f);
                    po4 = so.term ? p.rstv[4 + 4] : (pmh ? div_int_byf((float)e.put, p.maxh_f, p.inv_maxh_f) : 0.0f);
                    pcd = so.term ? p.rstv[4 + 7] : gx;
                    ppd = so.term ? p.rstv[4 + 9] : gz;
                } else {
                    account(so.reward, so.pnl, so.tc, so.term);
                }
                pre = so.term ? rst : post;
                if (so.term) env_reset_common(p, e);
            }
        };
        if (OBS && wrows == kLdsEnvs)
            run_blk([&](int buf, int sl, int k, float2 ak, auto) { step(buf, sl, k, ak, std::true_type{}); });
        else
            run_blk([&](int buf, int sl, int k, float2 ak, auto) { step(buf, sl, k, ak, std::false_type{}); });
    }
    LDS_T1(OBS ? 1 : 0);
    if (!OBS && i0 < N) {
        // a fresh (opaque) index: the compiler would otherwise keep every state address of
        // the prologue live across the block loop, in VGPR pairs, and spill them
        int64_t j = i;
        asm volatile("" : "+v"(j));
        s.t[j] = e.t;
        s.pos[j] = pack_pos(e.call, e.put);
        s.cash[j] = e.cash;
        if constexpr (POL) {   // step_body's POL state: the evaluation sums (s.sum untouched)
#pragma unroll
            for (int c = 0; c < 7; ++c) s.acc[(int64_t)c * N + j] = acc[c];
            s.acc_len[j] = acc_len;
        } else {
            s.sum[j] = sm0;
            s.sum[N + j] = sm1;
            s.sum[2 * N + j] = sm2;
            s.sum_len[j] = slen;
        }
        s.last[j] = last0;
        s.last[N + j] = last1;
        s.last[2 * N + j] = last2;
        s.last[3 * N + j] = last3;
    }
}

// s_setprio takes an immediate: kPrioProd + 1 when `up`, kPrioProd otherwise (a wave-uniform branch)
__device__ __forceinline__ void prod_prio_toggle(bool up) {
    if (up) __builtin_amdgcn_s_setprio(kPrioProd + 1);
    else __builtin_amdgcn_s_setprio(kPrioProd);
}

// Producer waves: block bp of 64 envs into LDS buffer bp & 1 while the steppers consume
// block bp - 1.  pw = producer wave index (kLdsPEnvs envs each).  Lanes past the last
// env mirror env N-1 like the steppers' (identical values, identical addresses).
template <int MODE, bool BOOK, bool LEAN>
__device__ __forceinline__ void lds_producer(const Params& p, int k_steps, const Market& cur,
                                             LdsMarketT<MODE, BOOK, LEAN>& W, int64_t base, int pw) {
    using G = LdsGeom<MODE, BOOK>;
    constexpr bool HESTON = G::HESTON;
    constexpr int kLdsLanes = G::lanes, kLdsPEnvs = G::penvs, kLdsH = G::H;
    const int lane = threadIdx.x & 63;
    const int sub = lane / kLdsPEnvs;
    const int le = pw * kLdsPEnvs + (lane % kLdsPEnvs);  // local env of this lane
    const int64_t N = p.n;
    const int nb = (k_steps + kLdsM - 1) / kLdsM;
    const uint32_t T = (uint32_t)p.T;
    const int64_t pi = (base + le) < N ? base + le : N - 1;
    if (!BOOK && !HESTON) {   // the producer roles one priority apart (kPrioGbmRew's note)
        if (pw == 0) __builtin_amdgcn_s_setprio(kPrioGbmProd0);
        else __builtin_amdgcn_s_setprio(kPrioGbmProd1);
    } else {
        __builtin_amdgcn_s_setprio(kPrioProd);
    }
    // the loop carries only the chain state (Sbs, Vbs, Mbs), a0, tpb and pi: the episode
    // counters are re-read after the loop and the Philox id is made per block, so nothing
    // else is live across the block loop (loop-invariant values spilled around it)
    uint64_t a0;                                     // env-step index of the launch's first step
    uint32_t tpb;                                    // episode step before slot 0 of block bp
    {
        const uint32_t ep0 = cur.ep[pi], t0 = cur.t[pi];
        const uint32_t off = t0 >= T ? T : t0;       // a0 = ep T + t (t = T: the next episode)
        a0 = (uint64_t)ep0 * T + off;
        tpb = off >= T ? 0u : off;
    }
    double Sbs = cur.S[pi];                          // f64 price before slot 0 of block bp
    double Vbs = HESTON ? cur.v[pi] : 0.0;           // Heston: f64 variance before it
    double Mbs = BOOK ? cur.M[pi] : 0.0;             // book: running max of S before it
    const int sl0 = sub * kLdsH;
    LDS_T0();
    for (int bp = 0; bp <= nb; ++bp) {
#if defined(HE_LDS_DIAG) && HE_LDS_DIAG == 1
        LDS_BAR();  // diagnostic build: the producers only keep the barrier count
        continue;
#endif
        if (bp < nb) {
            const int kb = bp * kLdsM;
            const int len = (k_steps - kb) < kLdsM ? (k_steps - kb) : kLdsM;
            // FULL: a whole kLdsM-slot block (every block of the launch but a ragged last
            // one): the per-slot `len` tests are compile-time true, so each stage's slots
            // are straight-line code -- independent chains the wave can interleave, and
            // one materialisation of each polynomial constant per stage instead of per slot
            auto block = [&](auto full) {
                constexpr bool FULL = decltype(full)::value;
                // LOCK: the lean GBM producers of a whole block evaluate their kLdsH slots in
                // lockstep (he_math.h *_n forms: the same operations per slot, so the same
                // bits, as kLdsH interleaved chains with shared constants)
                constexpr bool LOCK = FULL && LEAN && !HESTON;

            const int64_t gid = p.goff + pi;
            const uint64_t nf = a0 + (uint64_t)(kb + sl0);
            const uint32_t tpf = (tpb + (uint32_t)sl0) % T;
            double ex[kLdsH];   // own slots' growth factors S_j / S_{j-1} (before the clamp)
            double Vx[kLdsH];   // Heston: own slots' v after the step
            double Vin = Vbs;   // Heston: v before the lane's first slot
            if constexpr (LOCK) {
                // slot h's normal is the (nf + h - 2 m0)-th of the Box-Muller pairs of the
                // Philox blocks m0 = nf / 2, m0 + 1 (and m0 + 2 when nf is odd): cos, sin, ...
                const uint64_t m0 = nf >> 1;
                const bool odd = (nf & 1) != 0;
                double zs[kLdsH];
                if (__ballot(odd) == 0ull) {   // every lane even: blocks m0 .. m0 + kLdsH / 2 - 1
                    double zz[kLdsH];
                    philox_normals_n<kLdsH / 2>(p, gid, m0, zz);
#pragma unroll
                    for (int h = 0; h < kLdsH; ++h) zs[h] = zz[h];
                } else {
                    double zz[kLdsH + 2];
                    philox_normals_n<kLdsH / 2 + 1>(p, gid, m0, zz);
#pragma unroll
                    for (int h = 0; h < kLdsH; ++h) {
                        // both candidates pinned in registers: left alone, the select becomes
                        // zz[h + odd], a dynamically indexed array in scratch memory
                        double a = zz[h], b = zz[h + 1];
                        asm volatile("" : "+v"(a), "+v"(b));
                        zs[h] = odd ? b : a;
                    }
                }
                double arg[kLdsH];
#pragma unroll
                for (int h = 0; h < kLdsH; ++h) {
                    Vx[h] = 0.0;
                    const double dW = p.sqrt_dt * zs[h];
                    arg[h] = p.drift + p.sqrt_var * dW;   // rbergomi_sim.py:459-463
                }
                exp_k_n<kLdsH>(arg, ex);
            } else if constexpr (!HESTON) {
                // (1) the random part of every slot: Philox block m = n / 2 gives the
                // Box-Muller pair of steps 2m (cos) and 2m + 1 (sin)
                double zc = 0.0;
#pragma unroll
                for (int h = 0; h < kLdsH; ++h) {
                    ex[h] = 1.0;
                    Vx[h] = 0.0;
                    if (FULL || sl0 + h < len) {
                        const uint64_t n = nf + (uint64_t)h;
                        double z;
                        if (h == 0 || (n & 1) == 0) {
                            double z1, z2;
                            normals(p, gid, n >> 1, &z1, &z2);
                            z = (n & 1) ? z2 : z1;
                            zc = z2;
                        } else {
                            z = zc;
                        }
                        const double dW = p.sqrt_dt * z;
                        ex[h] = exp_k(p.drift + p.sqrt_var * dW);  // rbergomi_sim.py:459-463
                    }
                }
            } else {
                // (1) Heston (market_body's full-truncation Euler, rbergomi_sim.py:454-458):
                // Philox block n -> (z1, z2) per step; dw1 drives v, rho dw1 + sqrt(1 - rho^2)
                // dw2 the price
                // slot by slot (a rolled loop shifting each slot's pair in at the end, static
                // indices only): one Philox block and Box-Muller pair live at a time
                double w1[kLdsH], ws[kLdsH];
#pragma unroll
                for (int h = 0; h < kLdsH; ++h) w1[h] = ws[h] = 0.0;
#pragma unroll 1
                for (int h = 0; h < kLdsH; ++h) {
                    double a = 0.0, b = 0.0;
                    if (FULL || sl0 + h < len) {
                        double z1, z2;
                        normals(p, gid, nf + (uint64_t)h, &z1, &z2);
                        const double dw1 = p.sqrt_dt * z1, dw2 = p.sqrt_dt * z2;
                        a = dw1;
                        b = p.h_rho * dw1 + p.h_sqrt1mrho2 * dw2;
                    }
#pragma unroll
                    for (int q = 0; q + 1 < kLdsH; ++q) {
                        w1[q] = w1[q + 1];
                        ws[q] = ws[q + 1];
                    }
                    w1[kLdsH - 1] = a;
                    ws[kLdsH - 1] = b;
                }
                // (2a) the variance chain of the whole block in every lane (dw1 gathered from
                // the env's lanes): M sqrt, no exp; the lane keeps vp and sqrt(vp) of its slots
                double w1all[kLdsM];
#pragma unroll
                for (int r = 0; r < kLdsLanes; ++r)
#pragma unroll
                    for (int h = 0; h < kLdsH; ++h) w1all[r * kLdsH + h] = __shfl(w1[h], (lane % kLdsPEnvs) + r * kLdsPEnvs);
                double vpx[kLdsH], sqx[kLdsH];
#pragma unroll
                for (int h = 0; h < kLdsH; ++h) vpx[h] = sqx[h] = Vx[h] = 0.0;
                double v = Vbs;
                uint32_t tq = tpb;
#pragma unroll
                for (int j = 0; j < kLdsM; ++j) {
                    if (j == sl0) Vin = v;
                    double vp = 0.0, sq = 0.0;
                    if (FULL || j < len) {
                        if (tq == 0) v = p.var;  // autoreset: a new episode starts from v0
                        vp = v < 0.0 ? 0.0 : v;  // full truncation
                        sq = sqrt(vp);
                        v = (v + p.h_kappa * (p.h_theta - vp) * p.dt) + p.h_xi * sq * w1all[j];
                        tq = (tq + 1 == T) ? 0u : tq + 1;
                    }
#pragma unroll
                    for (int h = 0; h < kLdsH; ++h) {
                        vpx[h] = (j == sl0 + h) ? vp : vpx[h];
                        sqx[h] = (j == sl0 + h) ? sq : sqx[h];
                        Vx[h] = (j == sl0 + h) ? v : Vx[h];
                    }
                }
                Vbs = v;
                // (2b) the lane's own growth factors exp(drift + diff), market_body's operands
#pragma unroll
                for (int h = 0; h < kLdsH; ++h) {
                    const double drift = (p.mu - 0.5 * vpx[h]) * p.dt;
                    const double diff = sqx[h] * ws[h];
                    ex[h] = (FULL || sl0 + h < len) ? exp(drift + diff) : 1.0;
                }
            }
            // (2) the f64 price chain: the block's growth factors gathered from the env's
            // kLdsLanes lanes (independent shuffles, one latency), then every lane runs the
            // whole block's chain itself -- M products, no lane-to-lane hand-off -- keeping
            // its own slots (Sx) and the price before its first slot (Sin)
            double eall[kLdsM];
#pragma unroll
            for (int r = 0; r < kLdsLanes; ++r)
#pragma unroll
                for (int h = 0; h < kLdsH; ++h) eall[r * kLdsH + h] = __shfl(ex[h], (lane % kLdsPEnvs) + r * kLdsPEnvs);
            double Sx[kLdsH], Mx[kLdsH];
#pragma unroll
            for (int h = 0; h < kLdsH; ++h) Sx[h] = Sbs;
#pragma unroll
            for (int h = 0; h < kLdsH; ++h) Mx[h] = Mbs;
            double S = Sbs, Sin = Sbs, Mr = Mbs;
            {
                uint32_t tp = tpb;
#pragma unroll
                for (int j = 0; j < kLdsM; ++j) {
                    if (j == sl0) Sin = S;
                    if (FULL || j < len) {
                        if (tp == 0) {  // autoreset: a new episode starts from S0
                            S = p.s0;
                            if (BOOK) Mr = p.s0;
                        }
                        const double Sn = S * eall[j];
                        S = (Sn < 1e-8) ? 1e-8 : Sn;  // np.maximum(., 1e-8), NaN kept
                        if (BOOK) Mr = np_max(Mr, S);   // market_body's barrier monitor
                        tp = (tp + 1 == T) ? 0u : tp + 1;
                    }
#pragma unroll
                    for (int h = 0; h < kLdsH; ++h) Sx[h] = (j == sl0 + h) ? S : Sx[h];
                    if (BOOK) {
#pragma unroll
                        for (int h = 0; h < kLdsH; ++h) Mx[h] = (j == sl0 + h) ? Mr : Mx[h];
                    }
                }
            }
            Sbs = S;  // price after the block (every lane ran the whole chain)
            if (BOOK) Mbs = Mr;
            // (3) marks + obs greeks of every slot; the terminal step replays the marks of
            // the position before it (hedging_env_v2.py:229-231)
            uint32_t tp = tpf;
            const int wb = bp % LdsMarketT<MODE, BOOK, LEAN>::NB;
            double lkC[kLdsH], lkP[kLdsH];   // LOCK: the slots' marks, in lockstep
            if constexpr (LOCK) {
                double Sm[kLdsH], Km[kLdsH];
                uint32_t tq = tpf;
#pragma unroll
                for (int h = 0; h < kLdsH; ++h) {
                    const bool last = tq + 1 == T;
                    const double Sprev = (h == 0) ? Sin : Sx[h - 1];
                    Sm[h] = last ? ((tq == 0) ? p.s0 : Sprev) : Sx[h];
                    Km[h] = rint(Sm[h]);   // marks<GBM>: the rolling-ATM strike K = round(S)
                    tq = (tq + 1 == T) ? 0u : tq + 1;
                }
                bs_call_put_n<kLdsH>(Sm, Km, p.bs, lkC, lkP);
            }
            if constexpr (LOCK) {
#pragma unroll
                for (int h = 0; h < kLdsH; ++h) {
                    const int sl = sl0 + h;
                    W.sc[wb][sl][le] = make_float2((float)Sx[h], (float)lkC[h]);
                    W.pp[wb][sl][le] = (float)lkP[h];
                }
            } else {
                // marks<MODE> slot by slot: a rolled loop over registers rotated by one slot per
                // iteration (static indices only), so the Heston producers' per-slot Black-Scholes
                // constants and ndtr tails are one slot's live set, not kLdsH interleaved ones
                double rS[kLdsH], rV[kLdsH];
#pragma unroll
                for (int h = 0; h < kLdsH; ++h) {
                    rS[h] = Sx[h];
                    rV[h] = HESTON ? Vx[h] : p.var;
                }
                double Sprev = Sin, Vprev = Vin;
#pragma unroll 1
                for (int h = 0; h < kLdsH; ++h) {
                    if (FULL || sl0 + h < len) {
                        const bool last = tp + 1 == T;
                        const double Sm = last ? ((tp == 0) ? p.s0 : Sprev) : rS[0];
                        const double Vh = rV[0];
                        const double Vm = HESTON ? (last ? ((tp == 0) ? p.var : Vprev) : Vh) : p.var;
                        float C, P;
                        // the episode step of the marks: the slot's (tp + 1), or tp for the lagged ones
                        marks<MODE, !LEAN>(p, Sm, Vm, last ? tp : tp + 1u, &C, &P);
                        const int sl = sl0 + h;
                        W.sc[wb][sl][le] = make_float2((float)rS[0], C);
                        W.pp[wb][sl][le] = P;
                        if (HESTON) W.vv[HESTON ? wb : 0][HESTON ? sl : 0][le] = (float)Vh;
                        tp = (tp + 1 == T) ? 0u : tp + 1;
                    }
                    Sprev = rS[0];
                    Vprev = rV[0];
#pragma unroll
                    for (int q = 0; q + 1 < kLdsH; ++q) {
                        rS[q] = rS[q + 1];
                        rV[q] = rV[q + 1];
                    }
                }
            }
            if constexpr (BOOK) {
                // the book after the step into each slot (episode step tp + 1, the new S, not
                // lagged): market_body's tileC.  One slot at a time -- a rolled loop over
                // registers rotated by one slot per iteration (static indices only) -- so the
                // pricer's live set is one slot's, not kLdsH interleaved ones: unrolled, the
                // config 4 / 5 producers spilled 28 / 69 VGPRs (116 / 216 B of scratch per lane)
                double bS[kLdsH], bV[kLdsH], bM[kLdsH];
#pragma unroll
                for (int h = 0; h < kLdsH; ++h) {
                    bS[h] = Sx[h];
                    bV[h] = HESTON ? Vx[h] : p.var;
                    bM[h] = Mx[h];
                }
                uint32_t tb = tpf;
#pragma unroll 1
                for (int h = 0; h < kLdsH; ++h) {
                    // the two producer roles share each SIMD (one wave of each, from different
                    // workgroups): which one wins the issue ties changes slot by slot.  At one
                    // fixed priority the same role lost them all block long (role timing: prod0
                    // busy 6,981 / prod1 7,808 cycles per step, config 4): same box, config 4
                    // 7.25 -> 7.08 ms, config 5 1.71 -> 1.62 ms per launch (r04s5_ab_prod_prio.txt).
                    // Alternating 2:2 still left the second role the busier (config 4 5,533 / 6,144,
                    // config 5 4,955 / 6,244 cycles per step).  GBM: it is up on 3 slots of 4 --
                    // 5,696 / 5,828 and 5.71 -> 5.63 ms.  Heston keeps 2:2: 3:1 gave 5,137 / 6,072
                    // and +0.2 %, 4:0 6,498 / 4,451 and +0.6 % (r05s20_ab_prod_toggle.txt)
                    if (HESTON) prod_prio_toggle((h + pw) & 1);
                    else prod_prio_toggle(pw == 1 ? (h != 3) : (h == 3));
                    if (FULL || sl0 + h < len)
                        W.bk[wb][sl0 + h][le] = book_value<!HESTON>(p, bS[0], bV[0], (int32_t)(tb + 1), bM[0],
                                                                    &W.btab[0][0], &W.bopt[0]);
                    tb = (tb + 1 == T) ? 0u : tb + 1;
#pragma unroll
                    for (int q = 0; q + 1 < kLdsH; ++q) {
                        bS[q] = bS[q + 1];
                        bV[q] = bV[q + 1];
                        bM[q] = bM[q + 1];
                    }
                }
            }
            };
            if (len == kLdsM) block(std::true_type{});
            else block(std::false_type{});
            tpb = (uint32_t)(((uint64_t)tpb + kLdsM) % T);
        }
        LDS_BAR();  // block bp handed to the steppers
    }
    // the market position after the launch: every lane ran the whole price chain (Sbs, and
    // Heston's Vbs, the book's running max Mbs are the state after the last step); the last
    // slot's f32 marks are read back from its LDS record (written by this wave, and no wave
    // writes the buffers after the last barrier).  Kept out of the slot loop: a store branch
    // there held the launch-level values (env index, episode counters) live across the pricer.
    if (nb > 0 && sub == 0) {
        const int sll = (k_steps - 1) - (nb - 1) * kLdsM;
        const int wbl = (nb - 1) % LdsMarketT<MODE, BOOK, LEAN>::NB;
        // a fresh (opaque) index: the compiler would otherwise keep the prologue's state
        // addresses live across the block loop, in VGPR pairs, and spill them
        int64_t j = pi;
        asm volatile("" : "+v"(j));
        const uint32_t ep0 = cur.ep[j], t0 = cur.t[j];   // unchanged until these stores
        const uint32_t q = (t0 >= T ? T : t0) + (uint32_t)(k_steps - 1);
        cur.ep[j] = ep0 + q / T;
        cur.t[j] = q % T + 1u;
        cur.S[j] = Sbs;
        if (HESTON) cur.v[j] = Vbs;
        cur.C[j] = W.sc[wbl][sll][le].y;
        cur.P[j] = W.pp[wbl][sll][le];
        if (BOOK) cur.M[j] = Mbs;
    }
    LDS_T1(2 + (pw < 2 ? pw : 1));
}

// Role placement.  A workgroup's 4 waves land on the CU's 4 SIMDs (in the cyclic order
// 0 -> 2 -> 1 -> 3 from a varying start, MI355X_MICROARCH.md "LDS"), so with role = wave
// index the role a SIMD hosts depends on where each resident workgroup's placement
// started, and one SIMD can carry several obs steppers (the critical chain) while another
// has none.  HE_LDS_BALANCE: every workgroup takes a ticket from a per-CU counter (one
// atomic per workgroup) and its waves take role = (SIMD id + ticket) mod 4 -- a bijection
// over its 4 distinct SIMDs, and across the 4 workgroups resident on a CU (consecutive
// tickets) every SIMD hosts one wave of each role.  Wave-to-SIMD placement not
// one-per-SIMD (never seen) falls back to role = wave index.  Same-box A/B (r03s1, two
// runs each): configs 4 / 5 (producer-bound) 11.25 -> 10.54 ms and 2.49 -> 2.25 ms per
// launch; config 2 unchanged (its placement is already one role per SIMD on 230 of 256
// CUs, tools/lds_hwid.py).
#if HE_LDS_BALANCE || defined(HE_LDS_HWID)
__device__ uint32_t g_cu_ticket[4096];
#endif
#ifdef HE_LDS_HWID
// Diagnostic builds only: {HW_ID, XCC_ID, ticket, role} of every wave of the last launch
// (he_debug_lds_hwid)
__device__ uint32_t g_lds_hwid[16384][4][4];
#endif
__device__ __forceinline__ uint32_t hw_cu_key(uint32_t hw, uint32_t xcc) {
    // XCC 4 bits | SE_ID 3 | SH_ID 1 | CU_ID 4
    return ((xcc & 15u) << 8) | (((hw >> 13) & 7u) << 5) | (((hw >> 12) & 1u) << 4) | ((hw >> 8) & 15u);
}
template <int NWAVES>
__device__ __forceinline__ int lds_role(int wave) {
#if HE_LDS_BALANCE || defined(HE_LDS_HWID)
    if constexpr (NWAVES == 4) {
        __shared__ uint32_t sh_place[5];
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);     // HW_REG_HW_ID, 32 bits
        const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);   // HW_REG_XCC_ID
        const uint32_t simd = (hw >> 4) & 3u;
        if ((threadIdx.x & 63) == 0) sh_place[wave] = simd;
        if (threadIdx.x == 0) sh_place[4] = atomicAdd(&g_cu_ticket[hw_cu_key(hw, xcc & 15u)], 1u);
        __syncthreads();
        const uint32_t m = (1u << sh_place[0]) | (1u << sh_place[1]) | (1u << sh_place[2]) | (1u << sh_place[3]);
        int role = wave;
#if HE_LDS_BALANCE
        if (m == 15u) role = (int)((simd + sh_place[4]) & 3u);
#endif
#ifdef HE_LDS_HWID
        if ((threadIdx.x & 63) == 0 && blockIdx.x < 16384) {
            g_lds_hwid[blockIdx.x][wave][0] = hw;
            g_lds_hwid[blockIdx.x][wave][1] = xcc;
            g_lds_hwid[blockIdx.x][wave][2] = sh_place[4];
            g_lds_hwid[blockIdx.x][wave][3] = (uint32_t)role | (m << 8);
        }
#endif
        return __builtin_amdgcn_readfirstlane(role);
    }
#endif
    return wave;
}

// Wave roles are uniform (readfirstlane), so each role's loop is plain scalar control
// flow and all execute the same number of barriers; the roles' working sets never coexist.
// SGPRs capped at 96 (.sgpr_count 94): past 96 the hardware admits one wave per SIMD
// fewer than the occupancy API and the compiler report (MI355X_MICROARCH.md, Residency),
// and at 106 the 4 x 6 waves of 4 workgroups no longer fit a CU -- at 65,536 envs the
// launch ran in two rounds of workgroups (536 vs ~270 us).  The spills go to VGPR lanes.
constexpr int kLdsNumSgpr = 96;
template <int MODE, bool BOOK, bool LEAN, bool PERSIST = false, bool POL = false>
__global__ __launch_bounds__((LdsGeom<MODE, BOOK>::threads), (LdsGeom<MODE, BOOK>::minwaves))
    __attribute__((amdgpu_num_sgpr(kLdsNumSgpr))) void lds_rollout_kernel(const Params* __restrict__ pc, State s, Io io,
                                                                 int k_steps, Market cur) {
    __shared__ __attribute__((aligned(16))) LdsMarketT<MODE, BOOK, LEAN> lm;
    const Params& p = *pc;  // read through the scalar cache (a by-value copy spills)
    const int wave = lds_role<LdsGeom<MODE, BOOK>::threads / 64>(__builtin_amdgcn_readfirstlane(threadIdx.x >> 6));
    if constexpr (BOOK) {  // the tau table into LDS (rows <= kLdsBookRows: lds_rollout_eligible)
        const int nv = 4 * p.book_rows;
        for (int k = threadIdx.x; k < nv; k += LdsGeom<MODE, BOOK>::threads) (&lm.btab[0][0])[k] = p.book_tab[k];
        if ((int)threadIdx.x < p.book_n) lm.bopt[threadIdx.x] = p.book[threadIdx.x];
        __syncthreads();
    }
    if constexpr (!PERSIST) {   // one workgroup per 64-env tile
        const int64_t base = (int64_t)blockIdx.x * kLdsEnvs;
        if (wave == 0) lds_stepper<MODE, BOOK, LEAN, false, POL>(p, s, io, k_steps, cur, lm, base);
        else if (wave == 1) lds_stepper<MODE, BOOK, LEAN, true, POL>(p, s, io, k_steps, cur, lm, base);
        else lds_producer<MODE, BOOK, LEAN>(p, k_steps, cur, lm, base, wave - 2);
        return;
    }
    // PERSIST (launch_lds_rollout, more tiles than the device holds workgroups at once): a
    // workgroup runs tiles blockIdx.x, + gridDim.x, ..., the whole K-step rollout of each, so
    // the roles placed once (lds_role's per-CU balance) hold for every tile
    const int64_t tiles = (p.n + kLdsEnvs - 1) / kLdsEnvs;
    for (int64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
        // nothing hoisted out of the tile loop: each role's values stay inside its own code
        // (hoisted, the three roles' invariants all lived across the loop and spilled)
        asm volatile("" ::: "memory");
        const int64_t base = tile * kLdsEnvs;
        if (wave == 0) lds_stepper<MODE, BOOK, LEAN, false, POL>(p, s, io, k_steps, cur, lm, base);
        else if (wave == 1) lds_stepper<MODE, BOOK, LEAN, true, POL>(p, s, io, k_steps, cur, lm, base);
        else lds_producer<MODE, BOOK, LEAN>(p, k_steps, cur, lm, base, wave - 2);
        if (tile + gridDim.x < tiles) __syncthreads();   // every role done with lm before the next tile
    }
}

// ------------------------------------------------------------------ replay rollouts in LDS
// he_rollout in replay mode (train_ppo_v2.py:40's workload: the envs replay rows of a
// paths table through hedging_env_v2.py:223-231, bench config 6) on the LDS kernel's
// layout: a workgroup of 64 envs, a reward stepper and an obs stepper wave, and two LOADER
// waves in place of the producers.  The rows an env reads do not depend on its actions
// (episodes end at t = T whatever the agent does, and the next episode's row is the env's
// own PCG64 draw), so the loaders walk every env's (path, t) and PCG64 stream ahead of the
// steppers: for block b + 1 each issues its half of the M post-step rows {S, v, C, P} of
// every env (one lane per env; an env's rows of a block are contiguous in the table) a
// whole block before they go to LDS, evaluates their obs greeks there (the row's own
// greeks(), so the 16-B recg record is not read per step: 552 -> 425 us per launch, r03s10), and for an env
// whose episode ends in the block draws the new path (replay_reset's pcg64_integers) and
// loads its row 0 -- the reset obs and the next episode's starting market.  Needs T >= M
// (at most one episode end per env and block) and autoreset.
//
// The steppers' arithmetic is step_env / make_obs (generic configuration: any variant,
// loss, costs, record_metrics) with the episode's divisors held per env
// (replay_episode_consts), so the outputs are the tile kernels' bits
// (test_lds_replay_equals_tile_replay).
struct LdsReplay {
    float4 mk[2][kLdsM][kLdsEnvs];   // post-step row {S, v, C, P} of every slot
    float2 gd[2][kLdsM][kLdsEnvs];   // its {call_delta, put_delta}
    float gg[2][kLdsM][kLdsEnvs];    // its gamma
    float4 rk[2][kLdsEnvs];          // the new episode of an env ending in the block: row 0 {S0, v0, C0, P0}
    float4 rg[2][kLdsEnvs];          // and its greeks {call_delta, gamma, put_delta, -}
    float stage[2][kLdsEnvs * kObs]; // obs row staging, by step parity
};
static_assert(kLdsM > 8 || sizeof(LdsReplay) <= 40 * 1024 - 64, "4 workgroups per CU");

// Loader wave `part` (0, 1) stages the 32 envs [32 part, 32 part + 32) of the workgroup, two
// lanes per env: lane l holds env 32 part + (l & 31) and its slots [4 h, 4 h + 4) of every block,
// h = l >> 5.  Both lanes of an env walk its positions and PCG64 draws (the same values), the h = 0
// lane also loads the new-episode records and writes the state back.
//
// An env's 8 rows of a block are 128 B of the table, one whole line when the block starts on a
// line (rows t + 1 .. t + 8 with t = 0 mod 8).  With T = 4 mod 8 (the reference's 253-column
// tables) half the episodes run at t = 4 mod 8: every block's rows are the last 64 B of one line
// and the first 64 B of the next, whose other half is the next block's first 4 rows; read again a
// block later that line is fetched from memory a second time (config 6: reads 1.33x their bytes,
// r05tc1).  In that phase the h = 1 lane loads the whole second line -- its own 4 rows and the
// next block's first 4 -- and hands the latter to its h = 0 partner (lane - 32) for the next block.
__device__ __forceinline__ void lds_replay_loader(const Params& p, State s, int k_steps, LdsReplay& L,
                                                  int64_t base, int part) {
    constexpr int H = kLdsM / 2;
    static_assert(kLdsM == 8, "two lanes per env, 4 slots each: one 128-B line of rows per block");
    const int lane = threadIdx.x & 63;
    const int hh = lane >> 5;                 // the env's half of the block's slots
    const int le = part * 32 + (lane & 31);   // local env
    const int64_t N = p.n;
    const int64_t i0 = base + le;
    const int64_t i = i0 < N ? i0 : N - 1;    // lanes past N mirror env N-1
    const uint32_t T = (uint32_t)p.T;
    const int64_t W = p.rstride;              // a path's row stride (128-B lines, row 1 line-aligned)
    const GLOBAL v4f* rec = (const GLOBAL v4f*)p.rec;
    const GLOBAL v4f* recg = (const GLOBAL v4f*)p.recg;
    const int sl0 = hh * H;
    __builtin_amdgcn_s_setprio(kPrioProd);
    LDS_T0();
    int32_t path = s.path[i];
    uint32_t t = s.t[i];                      // episode step before the next slot (< T: autoreset)
    Pcg64 g;
    g.sh = s.pcg[i];
    g.sl = s.pcg[N + i];
    g.ih = s.pcg[2 * N + i];
    g.il = s.pcg[3 * N + i];
    g.has32 = s.pcgb[i];
    g.buf32 = s.pcgb[N + i];
    float s0enc = s.s0[i];
    const int nb = (k_steps + kLdsM - 1) / kLdsM;
    float4 A[H], B[H];
    float4 Y[H];            // h = 1 lanes: the second line's last 64 B, the next block's rows 0 .. 3
    bool hand = false;      // the issued block handed Y on (both lanes of the env agree)
    float4 R0 = make_float4(0.f, 0.f, 0.f, 0.f), G0 = R0;  // the new episode's row 0 (lanes ending in the block)
    int rsl = kLdsM;  // slot of the episode end in the issued block (kLdsM: none)
    // the loads of block bp from the position (path, t) before it; the position advanced past it
    auto issue = [&](int bp) {
        const int kb = bp * kLdsM;
        const int len = (k_steps - kb) < kLdsM ? (k_steps - kb) : kLdsM;
        // the previous block's hand-over: its Y, landed by now, to the h = 0 partner
        const bool take = hand;
        if (__ballot(take) != 0ull) {
#pragma unroll
            for (int h = 0; h < H; ++h) {
                Y[h].x = __shfl(Y[h].x, lane | 32);
                Y[h].y = __shfl(Y[h].y, lane | 32);
                Y[h].z = __shfl(Y[h].z, lane | 32);
                Y[h].w = __shfl(Y[h].w, lane | 32);
            }
        }
        // the step from t = T - 1 ends the episode (hedging_env_v2.py:217-219): slot T - 1 - t
        const uint32_t te = T - 1u - t;
        rsl = te < (uint32_t)len ? (int)te : kLdsM;
        int32_t np = path;
        if (rsl < kLdsM) np = (int32_t)pcg64_integers(g, (uint64_t)p.n_paths);  // replay_reset's draw
        const int64_t ro = (int64_t)path * W + p.roff + (int64_t)t + 1, rn = (int64_t)np * W + p.roff;
        // hand Y on from this block: no episode end in it, rows t + 1 .. t + 8 straddling two lines
        // by 64 B each, and the next block's slots 0 .. 3 still on this path (t + 8 <= T - 4)
        hand = rsl == kLdsM && (ro & 7) == 4 && t + 12u <= T;
        if (hh == 0 && take) {
#pragma unroll
            for (int h = 0; h < H; ++h) A[h] = Y[h];
        } else {
#pragma unroll
            for (int h = 0; h < H; ++h) {
                // slots up to the end read the old path's rows t + 1 + sl (row T holds the lagged
                // marks), the slots after it the new path's rows 1, 2, ...
                const int sl = sl0 + h;
                const int64_t r = (sl <= rsl) ? ro + sl : rn + (sl - rsl);
#if defined(HE_REPLAY_DIAG) && HE_REPLAY_DIAG == 1
                A[h] = make_float4(100.0f + (float)sl, 0.04f, 3.0f, 2.5f);  // diagnostic build: no table reads
#else
                A[h] = ld4(rec, r);
#endif
            }
        }
        if (hh == 1 && hand) {
#pragma unroll
            for (int h = 0; h < H; ++h) Y[h] = ld4(rec, ro + kLdsM + h);
        }
        if (hh == 0 && rsl < kLdsM) {   // lanes whose episode ends in the block (exec-masked:
            R0 = ld4(rec, rn);          // the others fetch nothing -- loaded for every env, these
            G0 = ld4(recg, rn);         // two 16-B records cost 2 lines per env and block)
        }
        if (rsl < kLdsM) {
            path = np;
            t = (uint32_t)(len - 1 - rsl);
        } else {
            t += (uint32_t)len;
        }
    };
    if (nb > 0) issue(0);
    for (int bp = 0; bp <= nb; ++bp) {
        if (bp < nb) {
            const int kb = bp * kLdsM;
            const int len = (k_steps - kb) < kLdsM ? (k_steps - kb) : kLdsM;
            const int wb = bp & 1;
#pragma unroll
            for (int h = 0; h < H; ++h) {
                const int sl = sl0 + h;
                if (sl < len) {
#if !(defined(HE_REPLAY_DIAG) && HE_REPLAY_DIAG == 1)
                    // table_greeks_kernel's record, here from the row itself
                    B[h] = p.record_metrics ? replay_greeks(p, A[h].x, A[h].y) : make_float4(0.f, 0.f, 0.f, 0.f);
#else
                    B[h] = make_float4(0.5f, 0.01f, -0.5f, 0.0f);
#endif
                    L.mk[wb][sl][le] = A[h];
                    L.gd[wb][sl][le] = make_float2(B[h].x, B[h].z);
                    L.gg[wb][sl][le] = B[h].y;
                }
            }
            if (hh == 0) {
                L.rk[wb][le] = R0;
                L.rg[wb][le] = G0;
                if (rsl < kLdsM) s0enc = (R0.x < 1e-6f) ? -1.0f : R0.x;  // replay_reset's S0 (-1: python 1.0)
            }
            if (bp + 1 < nb) issue(bp + 1);  // in flight while the steppers run block bp
        }
        LDS_BAR();  // block bp handed to the steppers
    }
    LDS_T1(2 + part);
    if (hh == 0 && i0 < N) {
        int64_t j = i;
        asm volatile("" : "+v"(j));
        s.path[j] = path;
        s.s0[j] = s0enc;
        s.pcg[j] = g.sh;
        s.pcg[N + j] = g.sl;
        s.pcgb[j] = g.has32;
        s.pcgb[N + j] = g.buf32;
    }
}

// The lane index within the wave, made where it is used: volatile, so the compiler can neither
// hoist it nor merge it with threadIdx.x -- a value kept live across the block loop costs a
// VGPR the replay steppers do not have (128 at 4 waves per SIMD).
__device__ __forceinline__ uint32_t fresh_lane() {
    uint32_t ln;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
    return ln;
}

// OBS = false: the reward wave (owns the env state); OBS = true: the obs wave.  FAST: the
// configuration of fast_replay_config (v2, loss != mse, shares_to_hedge != 0, record_metrics,
// max_contracts_held > 0) with its uniform branches compiled out.
// POL (he_rollout_policy in replay mode): the baseline policy evaluated by both steppers, as
// lds_stepper's POL -- here both read the rows' obs greeks from the loaders' LDS records.
template <bool OBS, bool FAST, bool POL = false>
__device__ __forceinline__ void lds_replay_stepper(const Params& p, State s, const Io& io, int k_steps,
                                                   LdsReplay& L, int64_t base) {
    constexpr int D = kLdsPrefetch;  // steps of actions in flight (8: +-0, r03s18)
    static_assert(kLdsM % D == 0, "the action ring index is the slot mod D");
    const int lane = threadIdx.x & 63;
    const int64_t N = p.n;
    const int nfull = k_steps / kLdsM;
    const int tail = k_steps - nfull * kLdsM;
    const int64_t i0 = base + lane;
    const int64_t i = i0 < N ? i0 : N - 1;
    const int wrows = (int)((N - base) < kLdsEnvs ? (N - base) : kLdsEnvs);
    const int32_t T = p.T;
    const GLOBAL v2f* gact = (const GLOBAL v2f*)io.act;
    GLOBAL float* const grew = (GLOBAL float*)io.rew;
    GLOBAL uint8_t* const gterm = (GLOBAL uint8_t*)io.term;
    __builtin_amdgcn_s_setprio(OBS ? kPrioObs : kPrioReplayRew);
    LDS_T0();
    Env e{};
    e.t = s.t[i];
    {
        const uint32_t pk = s.pos[i];
        e.call = unpack_lo(pk);
        e.put = unpack_hi(pk);
    }
    e.path = -1;
    const float s0enc = s.s0[i];
    e.s0_small = (s0enc == -1.0f);
    e.s0 = e.s0_small ? 1.0f : s0enc;
    replay_episode_consts<FAST>(p, e);
    // the row the env stands at (step_body's replay prologue)
    const uint32_t tt = e.t > (uint32_t)T ? (uint32_t)T : e.t;
    Mkt pre = as_mkt(ld4((const GLOBAL v4f*)p.rec, rrow(p, s.path[i], tt)));
    pre.B = 0.0;
    double pv_last = 0.0;
    double sm0 = 0.0, sm1 = 0.0, sm2 = 0.0;
    uint32_t slen = 0;
    float last0 = 0.f, last1 = 0.f, last2 = 0.f, last3 = 0.f;
    if (!OBS) {
        e.cash = s.cash[i];
        pv_last = portfolio_value<false>(p, e, pre);
        sm0 = s.sum[i];
        sm1 = s.sum[N + i];
        sm2 = s.sum[2 * N + i];
        slen = s.sum_len[i];
        last0 = s.last[i];
        last1 = s.last[N + i];
        last2 = s.last[2 * N + i];
        last3 = s.last[3 * N + i];
    }
    float2 ra[D];
#pragma unroll
    for (int d = 0; d < D; ++d)
        ra[d] = POL ? make_float2(0.0f, 0.0f) : ld2(gact, (int64_t)(d < k_steps ? d : k_steps - 1) * N + i);
    // POL: the policy columns (3, 4, 7, 9) of the env's current obs row (step_body's replay
    // prologue: the greeks of the row it stands at), and the evaluation loops' episode sums
    const int pol = POL ? io.pol.policy : HE_POLICY_NO_HEDGE;
    const bool pmh = FAST || p.maxh != 0, prm = FAST || p.record_metrics;
    float po3 = 0.0f, po4 = 0.0f, pcd = 0.0f, ppd = 0.0f;
    double acc[7] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    uint32_t acc_len = 0;
    if constexpr (POL) {
        po3 = pmh ? div_int_byf((float)e.call, p.maxh_f, p.inv_maxh_f) : 0.0f;
        po4 = pmh ? div_int_byf((float)e.put, p.maxh_f, p.inv_maxh_f) : 0.0f;
        const float4 g0 = ld4((const GLOBAL v4f*)p.recg, rrow(p, s.path[i], tt));
        pcd = prm ? g0.x : 0.0f;
        ppd = prm ? g0.z : 0.0f;
        if (!OBS) {
#pragma unroll
            for (int c = 0; c < 7; ++c) acc[c] = s.acc[(int64_t)c * N + i];
            acc_len = s.acc_len[i];
        }
    }
    // FAST: the per-handle constants of the step held in VGPRs (opaque).  Left to step_env's
    // Params reads, the SGPR-capped kernel re-loads them from the scalar cache inside every
    // step, and each such load's lgkmcnt(0) wait also drains the step's LDS reads.
    float c_mt_f = p.mt_f, c_shares_f = p.shares_f, c_init_cash_f = p.init_cash_f;
    float c_maxh_f = p.maxh_f, c_inv_maxh_f = p.inv_maxh_f, c_T_f = p.T_f, c_inv_T_f = p.inv_T_f;
    int32_t c_mt = p.mt, c_maxh = p.maxh;
    double c_tcpc = p.tcpc, c_slip = p.slip_frac, c_lam = p.lam, c_w = p.w, c_theta = p.theta;
    double c_shares_d = p.shares_d, c_inv_252 = p.inv_252, c_init_cash = p.initial_cash;
    if (FAST) {
        asm volatile("" : "+v"(c_mt_f), "+v"(c_mt), "+v"(c_maxh));
        if (OBS) {
            asm volatile("" : "+v"(c_maxh_f), "+v"(c_inv_maxh_f), "+v"(c_T_f), "+v"(c_inv_T_f));
        } else {
            asm volatile("" : "+v"(c_shares_f), "+v"(c_init_cash_f), "+v"(c_tcpc), "+v"(c_slip), "+v"(c_lam));
            asm volatile("" : "+v"(c_w), "+v"(c_theta), "+v"(c_shares_d), "+v"(c_inv_252), "+v"(c_init_cash));
        }
    }

    // the obs stepper's new episode for the envs ending at this step (a wave-uniform branch,
    // taken in a block where some lane's episode ends): env_reset_common + the new path's S0
    // and divisors, the market of row 0 and the reset obs (make_obs of row 0 at t = 0)
    auto new_episode_obs = [&](int buf, bool term, float* o) {
        if (__ballot(term) != 0ull) {
            const float4 r0 = L.rk[buf][lane];
            Env n = e;
            env_reset_common(p, n);
            n.s0_small = r0.x < 1e-6f;
            n.s0 = n.s0_small ? 1.0f : r0.x;
            replay_episode_consts<FAST>(p, n);
            const Mkt m0 = as_mkt(r0);
            const float4 g0 = L.rg[buf][lane];
            float ro[kObs];
            make_obs<FAST, true>(p, n, m0, g0, m0.S, m0.v, ro);
#pragma unroll
            for (int c = 0; c < kObs; ++c) o[c] = term ? ro[c] : o[c];
            e.t = term ? n.t : e.t;
            e.call = term ? n.call : e.call;
            e.put = term ? n.put : e.put;
            e.s0 = term ? n.s0 : e.s0;
            e.s0_small = term ? n.s0_small : e.s0_small;
            e.s0s_d = term ? n.s0s_d : e.s0s_d;
            e.inv_s0s_d = term ? n.inv_s0s_d : e.inv_s0s_d;
            e.s0s_f = term ? n.s0s_f : e.s0s_f;
            e.inv_s0s_f = term ? n.inv_s0s_f : e.inv_s0s_f;
            pre.S = term ? m0.S : pre.S;
            pre.v = term ? m0.v : pre.v;
        }
    };
    auto step = [&](int buf, int sl, int k, float2 ak, auto full) {
        const int64_t koff = (int64_t)k * N;
        Mkt post = as_mkt(L.mk[buf][sl][lane]);
        post.B = 0.0;
        if constexpr (POL) ak = policy_action(p, pol, e.call, e.put, po3, po4, pcd, ppd);
        if (OBS) {
            if (POL && io.pol.act_out) {
                v2f av = {ak.x, ak.y};
                ((GLOBAL v2f*)io.pol.act_out)[koff + i] = av;
            }
            const float2 gd = L.gd[buf][sl][lane];
            const float4 g = make_float4(gd.x, L.gg[buf][sl][lane], gd.y, lag_return(post.S, pre.S));
            // (i)-(ii) of step_env: the integer trade logic (:181-200)
            const int32_t nc = e.call + trade_round(ak.x * c_mt_f, c_mt);
            const int32_t nq = e.put + trade_round(ak.y * c_mt_f, c_mt);
            e.call = clamp_pos(nc, c_maxh);
            e.put = clamp_pos(nq, c_maxh);
            e.t = e.t + 1;
            const bool term = (int32_t)e.t >= T;
            float o[kObs];
            if (FAST) {  // make_obs<true, true> on the pinned constants (hedging_env_v2.py:109-143)
                // f32 Markstein steps (div_f32_byf): the FAST kernel runs only on an ordinary table
                // (he_env::table_ordinary: max(S0, 25) <= 2^24 and every price 0 or finite and of
                // magnitude >= 2^-100, so no quotient or residual leaves the normal range)
                o[0] = div_f32_byf(post.S, e.s0s_f, e.inv_s0s_f);
                o[1] = div_f32_byf(post.C, e.s0s_f, e.inv_s0s_f);
                o[2] = div_f32_byf(post.P, e.s0s_f, e.inv_s0s_f);
                o[3] = div_int_byf((float)e.call, c_maxh_f, c_inv_maxh_f);
                o[4] = div_int_byf((float)e.put, c_maxh_f, c_inv_maxh_f);
                o[5] = post.v;
                o[6] = div_int_byf((float)(T - (int32_t)e.t), c_T_f, c_inv_T_f);
                o[7] = g.x;
                o[8] = g.y;
                o[9] = g.z;
                o[10] = g.y;
                o[11] = g.w;  // e.t >= 1 after a step
                o[12] = (pre.S == 0.0f) ? 0.0f : np_clipf(post.v - pre.v, -1.0f, 1.0f);
            } else {
                make_obs<FAST, true>(p, e, post, g, pre.S, pre.v, o);
            }
            pre = post;
            new_episode_obs(buf, term, o);  // SB3 autoreset: the reset obs
            if constexpr (POL) {   // the row this step returns
                po3 = o[3];
                po4 = o[4];
                pcd = o[7];
                ppd = o[9];
            }
            float* const tile = L.stage[k & 1];
#pragma unroll
            for (int c = 0; c < kObs; ++c) tile[lane * kObs + c] = o[c];
            if (!POL || io.obs) {
                float* out = io.obs + koff * kObs;
                if constexpr (decltype(full)::value) flush_obs_full(tile, out, base, lane);
                else flush_obs_wave(tile, out, base, wrows, lane);
            }
        } else {
            StepOut so;
            if (FAST) {  // step_env<false, true, true> on the pinned constants (hedging_env_v2.py:175-262)
                const float pv0 = (c_shares_f * pre.S + 0.0f) + c_init_cash_f;  // f32 (:167-168)
                const double pv_prev = (e.t == 0) ? (double)pv0 : pv_last;
                const int32_t nc = e.call + trade_round(ak.x * c_mt_f, c_mt);
                const int32_t nq = e.put + trade_round(ak.y * c_mt_f, c_mt);
                const int32_t cc = clamp_pos(nc, c_maxh);
                const int32_t qq = clamp_pos(nq, c_maxh);
                const int32_t dc = cc - e.call, dp = qq - e.put;
                const int32_t adc = dc < 0 ? -dc : dc, adp = dp < 0 ? -dp : dp;
                const double commission = (double)(adc + adp) * c_tcpc;
                const double slc = (((double)adc * (double)pre.C) * 100.0) * c_slip;
                const double slp = (((double)adp * (double)pre.P) * 100.0) * c_slip;
                so.tc = commission + (slc + slp);
                e.cash = e.cash - so.tc;
                e.call = cc;
                e.put = qq;
                e.t = e.t + 1;
                so.term = (int32_t)e.t >= T;
                const double optv = ((double)cc * (double)post.C) * 100.0 + ((double)qq * (double)post.P) * 100.0;
                so.pv = ((double)(c_shares_f * post.S) + optv) + e.cash;
                so.pnl = so.pv - pv_prev;
#if defined(HE_REPLAY_DIAG) && HE_REPLAY_DIAG == 4  // diagnostic build: reciprocal multiplies, not divisions
                const double ps = so.pnl * c_inv_252;
                const double rpc = (-c_w) * (fabs(ps) * c_inv_252);
#else
                // the division core (div_f64_core): finite P&L on an ordinary table, shares_to_hedge
                // and the denominator normal (fast_replay_config); -0.2 %, r05s26_ab_replay_div_core.txt
                const double ps = div_f64_core(so.pnl, c_shares_d);
                const double rpc = (-c_w) * div_f64_core(fabs(ps), e.den);
#endif
                const double tcp = c_lam * so.tc;
                const double thp = c_theta * div_int_by((double)(T - (int32_t)e.t), 252.0, c_inv_252);
                so.reward = (rpc - tcp) - thp;
                so.ps = ps;   // (POL's sums; dead otherwise)
                so.rpc = rpc;
                so.tcp = tcp;
            } else {
                step_env<false, FAST, true>(p, e, pre, post, ak.x, ak.y, pv_last, so);
            }
            pv_last = so.pv;
#if !(defined(HE_REPLAY_DIAG) && HE_REPLAY_DIAG == 3)  // diagnostic build: no reward / done stores
            if (!POL || grew) grew[koff + i] = (float)so.reward;
            if (!POL || gterm) gterm[koff + i] = so.term ? 1 : 0;
#endif
            if constexpr (POL) {
                // step_body's POL sums, in step order, and the record of a finished episode
                acc[0] = acc[0] + so.reward;
                acc[1] = acc[1] + so.pnl;
                acc[2] = acc[2] + fabs(so.ps);
                acc[3] = acc[3] + so.tc;
                acc[4] = acc[4] + so.rpc;
                acc[5] = acc[5] + so.tcp;
                acc[6] = acc[6] + so.ps;
                acc_len += 1u;
                if (__ballot(so.term) != 0ull) {
                    if (so.term) {
                        if (i0 < N) {   // not the lanes mirroring env N - 1
                            const unsigned long long r = atomicAdd(io.pol.count, 1ull);
                            if ((int64_t)r < io.pol.cap) {
                                he_episode_record rec;
                                rec.env_id = p.goff + i;
                                rec.length = (int32_t)acc_len;
                                rec.reserved = 0;
                                rec.reward_sum = acc[0];
                                rec.pnl_sum = acc[1];
                                rec.abs_pnl_sum = acc[2];
                                rec.cost_sum = acc[3];
                                rec.pnl_penalty_sum = acc[4];
                                rec.cost_penalty_sum = acc[5];
                                rec.per_share_pnl_sum = acc[6];
                                rec.reserved2 = 0.0;
                                io.pol.rec[r] = rec;
                            }
                        }
                        last0 = (float)acc[0];
                        last1 = (float)acc[1];
                        last2 = (float)acc[3];
                        last3 = (float)acc_len;
#pragma unroll
                        for (int c = 0; c < 7; ++c) acc[c] = 0.0;
                        acc_len = 0;
                    }
                }
                // the policy columns of the row this step returns, as the obs stepper makes them:
                // the post-trade positions and the slot's greeks, or the new episode's row 0
                const float2 gd = L.gd[buf][sl][lane];
                const float4 rg = L.rg[buf][lane];
                const bool tm = so.term;
                po3 = pmh ? div_int_byf((float)(tm ? 0 : e.call), p.maxh_f, p.inv_maxh_f) : 0.0f;
                po4 = pmh ? div_int_byf((float)(tm ? 0 : e.put), p.maxh_f, p.inv_maxh_f) : 0.0f;
                pcd = prm ? (tm ? rg.x : gd.x) : 0.0f;
                ppd = prm ? (tm ? rg.z : gd.y) : 0.0f;
            }
            const double a0 = sm0 + so.reward, a1 = sm1 + so.pnl, a2 = sm2 + so.tc;
            const uint32_t n1 = slen + 1u;
            float f0 = (float)a0, f1 = (float)a1, f2 = (float)a2, f3 = (float)n1;
            asm volatile("" : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3));
            if constexpr (!POL) {
                last0 = so.term ? f0 : last0;
                last1 = so.term ? f1 : last1;
                last2 = so.term ? f2 : last2;
                last3 = so.term ? f3 : last3;
                sm0 = so.term ? 0.0 : a0;
                sm1 = so.term ? 0.0 : a1;
                sm2 = so.term ? 0.0 : a2;
                slen = so.term ? 0u : n1;
            }
            // SB3 autoreset, branch-free (the block's steps stay one basic block): the new
            // episode's row 0 is read every step, its denominator and the reset state selected
            const float4 r0 = L.rk[buf][lane];
            const bool small = r0.x < 1e-6f;
            const double den0 = replay_den<FAST>(p, small ? 1.0f : r0.x, small);
            const bool tm = so.term;
            e.t = tm ? 0u : e.t;
            e.call = tm ? 0 : e.call;
            e.put = tm ? 0 : e.put;
            e.cash = tm ? c_init_cash : e.cash;
            e.den = tm ? den0 : e.den;
            pre.S = tm ? r0.x : post.S;
            pre.v = tm ? r0.y : post.v;
            pre.C = tm ? r0.z : post.C;
            pre.P = tm ? r0.w : post.P;
        }
    };
    auto run = [&](auto full) {
        LDS_BAR();  // block 0 loaded
        for (int b = 0; b < nfull; ++b) {
#if defined(HE_REPLAY_DIAG) && HE_REPLAY_DIAG == 2
            LDS_BAR();  // diagnostic build: the steppers only keep the barrier count
            continue;
#endif
            const int buf = b & 1;
#pragma unroll
            for (int sl = 0; sl < kLdsM; ++sl) {
                const int k = b * kLdsM + sl;
#if defined(HE_REPLAY_DIAG) && HE_REPLAY_DIAG == 5  // diagnostic build: no action loads
                const float2 ak = make_float2(0.3f * (float)(sl - 4), -0.2f);
#else
                const float2 ak = ra[sl % D];
                if constexpr (!POL) {
                    const int kn = k + D;
                    ra[sl % D] = ld2(gact, (int64_t)(kn < k_steps ? kn : k_steps - 1) * N + i);
                }
#endif
                step(buf, sl, k, ak, full);
            }
            LDS_BAR();  // buffer b & 1 handed back, block b + 1 loaded
        }
        if (tail) {
            const int buf = nfull & 1;
            // the env index made afresh (mbcnt lane): i itself is then dead across the block
            // loop above, which kept it in scratch for these loads (the kernel's VGPR spill)
            const int64_t ia = base + (int64_t)fresh_lane();
            const int64_t it = ia < N ? ia : N - 1;
            for (int sl = 0; sl < tail; ++sl) {
                const int k = nfull * kLdsM + sl;
                step(buf, sl, k, POL ? make_float2(0.0f, 0.0f) : ld2(gact, (int64_t)k * N + it), std::false_type{});
            }
            LDS_BAR();
        }
    };
    if (wrows == kLdsEnvs) run(std::true_type{});
    else run(std::false_type{});
    LDS_T1(OBS ? 1 : 0);
    if (!OBS && i0 < N) {
        // the env index made afresh (the lane from mbcnt, not threadIdx): kept live across the
        // block loop for these stores, the prologue's i was this kernel's one VGPR spill
        int64_t j = base + (int64_t)fresh_lane();
        asm volatile("" : "+v"(j));
        s.t[j] = e.t;
        s.pos[j] = pack_pos(e.call, e.put);
        s.cash[j] = e.cash;
        if constexpr (POL) {   // step_body's POL state: the evaluation sums (s.sum untouched)
#pragma unroll
            for (int c = 0; c < 7; ++c) s.acc[(int64_t)c * N + j] = acc[c];
            s.acc_len[j] = acc_len;
        } else {
            s.sum[j] = sm0;
            s.sum[N + j] = sm1;
            s.sum[2 * N + j] = sm2;
            s.sum_len[j] = slen;
        }
        s.last[j] = last0;
        s.last[N + j] = last1;
        s.last[2 * N + j] = last2;
        s.last[3 * N + j] = last3;
    }
}

template <bool FAST, bool POL = false>
__global__ __launch_bounds__(256, 4) __attribute__((amdgpu_num_sgpr(kLdsNumSgpr))) void lds_replay_kernel(
    const Params* __restrict__ pc, State s, Io io, int k_steps) {
    __shared__ __attribute__((aligned(16))) LdsReplay lm;
    const Params& p = *pc;
    const int wave = lds_role<4>(__builtin_amdgcn_readfirstlane(threadIdx.x >> 6));
    const int64_t base = (int64_t)blockIdx.x * kLdsEnvs;
    if (wave == 0) lds_replay_stepper<false, FAST, POL>(p, s, io, k_steps, lm, base);
    else if (wave == 1) lds_replay_stepper<true, FAST, POL>(p, s, io, k_steps, lm, base);
    else lds_replay_loader(p, s, k_steps, lm, base, wave - 2);
}

// he_episode_summaries: the last finished episode of every env, [4][N] (the reward
// wave's coalesced per-field stores) re-laid out as [N][4] rows -- four coalesced 4-B
// loads and one 16-B store per env.  One launch, ~1 MB at 65,536 envs (four strided
// hipMemcpy2DAsync calls took ~26 us on the boundary, r04s1_rccl_boundary.json).
__global__ void summaries_kernel(const float* __restrict__ last, float4* __restrict__ out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = make_float4(last[i], last[n + i], last[2 * n + i], last[3 * n + i]);
}

// Test hooks (he_device_rng / he_device_math): the device build of the generate-mode
// RNG and math, element-wise, so tests can compare device words and values bit for bit
// with the host build, rocRAND and the oracle.
__global__ void device_rng_kernel(uint32_t k0, uint32_t k1, const uint64_t* gid, const uint64_t* n, int64_t count,
                                  uint32_t* words, double* normals) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= count) return;
    const u32x4 c = {(uint32_t)n[k], (uint32_t)(n[k] >> 32), (uint32_t)gid[k], (uint32_t)(gid[k] >> 32)};
    const u32x4 x = philox4x32_10(c, k0, k1);
    if (words) {
        words[4 * k] = x.x;
        words[4 * k + 1] = x.y;
        words[4 * k + 2] = x.z;
        words[4 * k + 3] = x.w;
    }
    if (normals) box_muller(u01(x.x, x.y), u01(x.z, x.w), normals + 2 * k, normals + 2 * k + 1);
}

// he_device_math / he_host_math: group g = elements [4g, 4g + 4) (ops 4 / 5: two (u1, u2)
// pairs), padded with `pad` past count.  Ops 1, 3, 5 are the lockstep forms the LDS
// producers run, ops 0, 2, 4 the scalar ones the tile kernels run: equal bit for bit.
HE_HD void math_group(int32_t op, const double* x, int64_t count, double* out, int64_t g, const BSConst& bs) {
    const double pad = (op == 4 || op == 5) ? 0.5 : ((op == 2 || op == 3) ? 500.0 : 0.0);
    double a[4], r[4], q[4];
    for (int h = 0; h < 4; ++h) a[h] = (4 * g + h < count) ? x[4 * g + h] : pad;
    switch (op) {
        case 0:
            for (int h = 0; h < 4; ++h) r[h] = exp_k(a[h]);
            break;
        case 1:
            exp_k_n<4>(a, r);
            break;
        case 2:   // the rolling-ATM call mark at S = a (marks<GBM>)
            for (int h = 0; h < 4; ++h) bs_call_put(a[h], rint(a[h]), bs, r + h, q + h);
            break;
        case 3: {
            double K[4];
            for (int h = 0; h < 4; ++h) K[h] = rint(a[h]);
            bs_call_put_n<4>(a, K, bs, r, q);
            break;
        }
        case 4:
            box_muller(a[0], a[1], r, r + 1);
            box_muller(a[2], a[3], r + 2, r + 3);
            break;
        default: {  // 5
            const double u1[2] = {a[0], a[2]}, u2[2] = {a[1], a[3]};
            double z1[2], z2[2];
            box_muller_n<2>(u1, u2, z1, z2);
            r[0] = z1[0], r[1] = z2[0], r[2] = z1[1], r[3] = z2[1];
        }
    }
    for (int h = 0; h < 4; ++h)
        if (4 * g + h < count) out[4 * g + h] = r[h];
}

__global__ void device_math_kernel(int32_t op, const double* x, int64_t count, double* out, BSConst bs) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (4 * g >= count) return;
    math_group(op, x, count, out, g, bs);
}

// the constant-sigma BS constants of the default GBM handle (fill_params' expressions)
static BSConst default_bs() {
    BSConst c;
    const double sig = sqrt(0.029028), T = 30.0 / 252.0, r = 0.04;
    c.intrinsic = 0;
    c.a = (r + 0.5 * pow(sig, 2.0)) * T;
    c.b = sig * sqrt(T);
    c.inv_b = 1.0 / c.b;
    c.disc = exp(-r * T);
    return c;
}

// Explicit reset of envs `ids` (NULL: all).  Generate: the market position of a
// reset env moves to the start of its next episode.  Replay: the episode row is the env's
// PCG64 draw, or eps[j] when given (he_reset_episodes: host-drawn indices, the env's own
// stream not advanced).
template <int MODE>
__global__ __launch_bounds__(kBlock) void reset_kernel(Params p, State s, Market cur, const int64_t* ids,
                                                       int64_t count, float* obs, he_info inf, const int64_t* eps) {
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= count) return;
    const int64_t i = ids ? ids[j] : j;
    if (i < 0 || i >= p.n) return;
    Env e;
    env_reset_common(p, e);
    float o[kObs];
    Mkt m;
    if (MODE == HE_MODE_REPLAY) {
        if (eps) {
            e.path = (int32_t)eps[j];   // validated on the host: 0 <= eps[j] < n_paths
            replay_start(p, e);
        } else {
            replay_reset(p, s, i, e);
        }
        int64_t r = rrow(p, e.path, 0);
        m = as_mkt(p.rec[r]);
        make_obs(p, e, m, p.recg[r], m.S, m.v, o);
        s.path[i] = e.path;
        s.s0[i] = e.s0_small ? -1.0f : e.s0;
    } else {
        cur.ep[i] = cur.ep[i] + 1u;  // 0xFFFFFFFF after seeding -> episode 0
        cur.t[i] = 0;
        cur.S[i] = p.s0;
        if (MODE == HE_MODE_HESTON) cur.v[i] = p.var;
        cur.C[i] = p.rstv[2];
        cur.P[i] = p.rstv[3];
        if (cur.M) cur.M[i] = p.s0;
        m = Mkt{p.rstv[0], p.rstv[1], p.rstv[2], p.rstv[3], 0.0};
        e.s0_small = m.S < 1e-6f;
        e.s0 = e.s0_small ? 1.0f : m.S;
        e.path = -1;
#pragma unroll
        for (int c = 0; c < kObs; ++c) o[c] = p.rstv[4 + c];
    }
    s.t[i] = 0;
    s.pos[i] = 0;
    s.cash[i] = e.cash;
#pragma unroll
    for (int c = 0; c < 7; ++c) s.acc[(int64_t)c * p.n + i] = 0.0;
    s.acc_len[i] = 0;
    for (int c = 0; c < 3; ++c) s.sum[(int64_t)c * p.n + i] = 0.0;
    s.sum_len[i] = 0;
    if (obs) {
#pragma unroll
        for (int c = 0; c < kObs; ++c) obs[i * kObs + c] = o[c];
    }
    if (inf.cash) inf.cash[i] = e.cash;
    if (inf.call_contracts) inf.call_contracts[i] = 0;
    if (inf.put_contracts) inf.put_contracts[i] = 0;
    if (inf.initial_S0_for_episode) inf.initial_S0_for_episode[i] = e.s0;
    if (inf.current_stock_price) inf.current_stock_price[i] = m.S;
    if (inf.current_volatility) inf.current_volatility[i] = m.v;
    if (inf.current_call_price) inf.current_call_price[i] = m.C;
    if (inf.current_put_price) inf.current_put_price[i] = m.P;
    if (inf.current_step) inf.current_step[i] = 0;
    if (inf.current_episode_idx) inf.current_episode_idx[i] = e.path;
}

// ------------------------------------------------------------------ host side
struct DeviceGuard {
    int prev = -1;
    bool ok = true;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// numpy.random.SeedSequence(seed).generate_state(4, uint64) -> PCG64 seeding
// (numpy/random/bit_generator.pyx, numpy/random/src/pcg64/pcg64.c).
void seed_sequence_pcg64(uint64_t seed, uint64_t out[4]) {
    const uint32_t INIT_A = 0x43b0d7e5u, MULT_A = 0x931e8875u, INIT_B = 0x8b51f9ddu,
                   MULT_B = 0x58f38dedu, MIX_L = 0xca01f9ddu, MIX_R = 0x4973f715u;
    std::vector<uint32_t> ent;
    if (seed == 0) ent.push_back(0);
    for (uint64_t v = seed; v; v >>= 32) ent.push_back((uint32_t)(v & 0xFFFFFFFFu));
    uint32_t hc = INIT_A;
    auto hashmix = [&](uint32_t value) {
        value ^= hc;
        hc *= MULT_A;
        value *= hc;
        value ^= value >> 16;
        return value;
    };
    auto mix = [&](uint32_t x, uint32_t y) {
        uint32_t r = MIX_L * x - MIX_R * y;
        r ^= r >> 16;
        return r;
    };
    uint32_t pool[4];
    for (int k = 0; k < 4; ++k) pool[k] = hashmix(k < (int)ent.size() ? ent[k] : 0u);
    for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b)
            if (a != b) pool[b] = mix(pool[b], hashmix(pool[a]));
    for (size_t a = 4; a < ent.size(); ++a)
        for (int b = 0; b < 4; ++b) pool[b] = mix(pool[b], hashmix(ent[a]));
    uint32_t words[8];
    uint32_t hb = INIT_B;
    for (int k = 0; k < 8; ++k) {
        uint32_t d = pool[k % 4];
        d ^= hb;
        hb *= MULT_B;
        d *= hb;
        d ^= d >> 16;
        words[k] = d;
    }
    uint64_t val[4];
    for (int k = 0; k < 4; ++k) val[k] = (uint64_t)words[2 * k] | ((uint64_t)words[2 * k + 1] << 32);
    // pcg64_set_seed(state, seed = val[0..1], inc = val[2..3]); srandom: state=0,
    // inc=(initseq<<1)|1, step, state += initstate, step.
    Pcg64 g;
    uint64_t init_hi = val[0], init_lo = val[1], seq_hi = val[2], seq_lo = val[3];
    g.ih = (seq_hi << 1) | (seq_lo >> 63);
    g.il = (seq_lo << 1) | 1ull;
    g.sh = 0;
    g.sl = 0;
    g.has32 = 0;
    g.buf32 = 0;
    pcg64_step(g);
    uint64_t nl = g.sl + init_lo;
    g.sh = g.sh + init_hi + (nl < g.sl ? 1ull : 0ull);
    g.sl = nl;
    pcg64_step(g);
    out[0] = g.sh;
    out[1] = g.sl;
    out[2] = g.ih;
    out[3] = g.il;
}

}  // namespace

struct he_env {
    he_config cfg;
    Params p;
    State s;
    Market cur;               // market position after the newest generated block
    Market bak[2];            // start position of the block held in tile buffer b
    std::string err;
    void* state_mem = nullptr;
    size_t state_bytes = 0;
    float4* rec = nullptr;
    float4* recg = nullptr;
    float4* tile = nullptr;   // 2 buffers x (tileA | tileB)
    float rstv[4 + kObs] = {};  // host copy of the reset market + obs (generate)
    float* rst = nullptr;     // reset market + obs (generate)
    Params* dparams = nullptr;  // device copies of tile_params(env, 0 / 1) for step1_kernel
    bool vn_on = false;          // he_vecnorm_attach: he_step also runs the VecNormalize moments
    bool vn_fused = false;       // ... and this he_step ran them in step1_vn_kernel (step1_vne_kernel)
    vn::MomentsArgs vn{};
    bool vne_on = false;         // he_vecnorm_attach_eval: he_step also runs the eval VecNormalize step
    vn::ApplyArgs vne{};
    he_vecnorm_params vne_p{};
    BookOpt* dbook = nullptr;   // liability book, device copy (generate modes)
    double* dbook_tab = nullptr;  // book tau table (book_option)
    int64_t* d_eps = nullptr;     // he_reset_episodes: the host-drawn episode rows, staged
    int64_t* h_eps = nullptr;     // ... through this pinned host buffer (an async DMA)
    hipEvent_t ev_eps = nullptr;  // recorded after the reset that read d_eps / h_eps: guards their reuse
    int32_t book_rows = 0;        // its rows: max expiry + 1
    unsigned long long* scratch_count = nullptr;  // he_rollout_policy without records
    double book_rst = 0.0;      // book value of the reset market (host copy)
    int64_t n_paths = 0;
    // every price of the loaded table 0 or finite and of magnitude >= 2^-100, every S0 <= 2^24
    // (he_load_paths): the FAST replay kernel's f32 obs quotients apply (fast_replay_config)
    bool table_ordinary = false;
    int32_t block_pos = 0;    // generate: next slot to consume; M = tile exhausted/invalid
    int32_t cur_buf = 0;      // tile buffer of the block being consumed
    int32_t next_state = 0;   // next block: 0 none, 1 generating on `xs` (ev_next), 2 ready
    bool fuse_market = true;  // rollouts: next block's market in the step grid (HE_FUSED_MARKET=0: side stream)
    bool lds_rollout = true;  // he_rollout (GBM, no book): lds_rollout_kernel (HE_LDS_ROLLOUT=0: tile kernels)
    // lds_rollout_kernel's grid: at most this many workgroups, each looping over 64-env tiles
    // (0: one workgroup per tile).  The device's resident count (CUs x workgroups per CU) unless
    // HE_LDS_PERSIST=0; HE_LDS_MAX_GRID=<n> caps it (tests: many tiles per workgroup).
    int64_t lds_grid = -1;    // -1: not computed yet
    int64_t lds_grid_cap = 0; // HE_LDS_MAX_GRID
    bool lds_persist = true;
    bool lds_policy = true;   // he_rollout_policy on lds_rollout_kernel<..., POL> (HE_LDS_POLICY=0: the tile kernels)
    int32_t prefetch_mode = 0; // 0 auto, 1 never, 2 always: market_kernel(b+1) on `xs` during block b
    hipStream_t xs = nullptr; // library side stream for market prefetch
    hipEvent_t ev_fork = nullptr, ev_next = nullptr;
    bool ready = false;       // a reset happened since create/seed
    void* ev_start = nullptr; // he_time_next_step events (hipEvent_t)
    void* ev_stop = nullptr;
    uint32_t* sig_flag = nullptr;  // he_step_signal: the armed flag (device address of host-mapped memory)
    uint32_t* d_sig_cnt = nullptr; // ... its workgroup counter (device word, 0 between steps)
    uint32_t sig_seq = 0;          // sequence number of the last armed he_step
    std::vector<std::pair<size_t, void*>> fields;  // (bytes, device ptr) for get/set_state
};

static he_status fail(he_env* env, he_status st, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (env) env->err = buf;
    return st;
}

#define HE_HIP(env, call)                                                                      \
    do {                                                                                       \
        hipError_t _e = (call);                                                                \
        if (_e != hipSuccess)                                                                  \
            return fail((env), HE_EHIP, "%s failed: %s", #call, hipGetErrorString(_e));        \
    } while (0)

static bool is_generate(const he_env* env) { return env->cfg.mode != HE_MODE_REPLAY; }

#ifdef HE_TIMING
static uint64_t* g_tim = nullptr;
#endif

static void fill_params(he_env* env) {
    const he_config& c = env->cfg;
    Params& p = env->p;
    memset(&p, 0, sizeof(p));
    p.n = c.n_envs;
    p.goff = c.global_env_offset;
    p.variant = c.variant;
    p.loss = c.loss_type;
    p.record_metrics = c.record_metrics ? 1 : 0;
    {   // HE_GREEKS_IN_STEP_MIN_ENVS in the environment overrides the threshold (tests, A/B)
        const char* ev = getenv("HE_GREEKS_IN_STEP_MIN_ENVS");
        const int64_t thr = (ev && *ev) ? (int64_t)atoll(ev) : kGreeksInStepMinEnvs;
        p.tile_greeks = (c.mode == HE_MODE_HESTON || c.n_envs < thr) ? 1 : 0;
    }
    p.autoreset = c.autoreset ? 1 : 0;
    p.mode = c.mode;
    p.mt = c.max_trade_per_step;
    p.maxh = c.max_contracts_held_per_type;
    p.mt_f = (float)c.max_trade_per_step;
    p.maxh_f = (float)c.max_contracts_held_per_type;
    p.init_cash_f = (float)c.initial_cash;
    p.tcpc = c.transaction_cost_per_contract;
    p.slip_frac = c.slippage_bps / 10000.0;
    p.lam = c.lambda_cost;
    p.w = c.pnl_penalty_weight;
    p.theta = c.theta_weight;
    p.initial_cash = c.initial_cash;
    p.shares_d = (double)c.shares_to_hedge;
    p.inv_shares = 1.0 / p.shares_d;
    p.shares_f = (float)c.shares_to_hedge;
    p.shares_zero = c.shares_to_hedge == 0;
    p.r_f = (float)c.risk_free_rate;
    p.tenor_f = (float)c.option_tenor_years;
    p.r_d = c.risk_free_rate;
    p.tenor_d = c.option_tenor_years;
    p.sqrt_tenor = sqrt(c.option_tenor_years);
    p.tenor_small = c.option_tenor_years <= 1e-6;
    p.key0 = (uint32_t)(c.seed & 0xFFFFFFFFu);
    p.key1 = (uint32_t)(c.seed >> 32);
    p.s0 = c.s0;
    p.var = c.variance;
    p.var_f = (float)c.variance;
    p.mu = c.mu;
    p.dt = c.dt;
    p.sqrt_dt = sqrt(c.dt);
    // rbergomi_sim.py:460-461: drift = (r - 0.5 v) dt; diff = sqrt(max(0, v)) * dW
    p.drift = (c.mu - 0.5 * c.variance) * c.dt;
    p.sqrt_var = sqrt(c.variance < 0.0 ? 0.0 : c.variance);
    // option_calculator.py:13-25 with python-float semantics (sigma**2 = libm pow)
    double sig = sqrt(c.variance < 0.0 ? 0.0 : c.variance);
    double T = c.option_tenor_years, r = c.risk_free_rate;
    p.bs.intrinsic = (T <= 0.0) || (sig <= 0.0);
    p.bs.a = (r + 0.5 * pow(sig, 2.0)) * T;
    p.bs.b = sig * sqrt(T);
    p.bs.inv_b = 1.0 / p.bs.b;
    p.bs.disc = exp(-r * T);
    p.mark = c.mark;
    p.fe_K = rint(c.s0);   // np.round(paths[:, 0]): every generated episode starts at s0
    // hedging_env_v2.py:84,95-99 for a constant f32 variance (numpy scalar powf)
    float vf = (float)c.variance;
    float vmax = (vf != vf) ? vf : (vf > 1e-8f ? vf : 1e-8f);
    p.g_sigma = sqrtf(vmax);
    p.g_num_drift = ((float)r + 0.5f * powf(p.g_sigma, 2.0f)) * (float)T;
    p.g_sst = (double)p.g_sigma * sqrt(T);
    p.g_inv_sst = 1.0 / p.g_sst;
    p.g_sst_f = (float)p.g_sst;
    p.g_inv_sst_f = (float)p.g_inv_sst;
    p.sqrt_tenor_f = (float)p.sqrt_tenor;
    p.h_kappa = c.heston_kappa;
    p.h_theta = c.heston_theta;
    p.h_xi = c.heston_xi;
    p.h_rho = c.heston_rho;
    double omr = 1.0 - c.heston_rho * c.heston_rho;
    p.h_sqrt1mrho2 = sqrt(omr < 0.0 ? 0.0 : omr);
    p.T = c.episode_length;
    p.T_f = (float)c.episode_length;
    p.inv_maxh_f = 1.0f / p.maxh_f;
    p.inv_T_f = 1.0f / p.T_f;
    p.inv_252 = 1.0 / 252.0;
    p.M = c.market_block;
    p.tileA = p.tileB = nullptr;  // set per launch (tile_params)
    memcpy(p.rstv, env->rstv, sizeof(p.rstv));
    if (is_generate(env)) {
        // every generate-mode episode starts at the same S0 = rstv[0] (f32), so the
        // reward denominator (hedging_env_v2.py:243-253) is one host constant
        float s0 = p.rstv[0];
        bool small = s0 < 1e-6f;
        float f = small ? 25.0f : (s0 > 25.0f || s0 != s0 ? s0 : 25.0f);
        if (c.loss_type == HE_LOSS_MSE) p.den = small ? (625.0 + 1e-9) : (double)(f * f + 1e-9f);
        else p.den = small ? (25.0 + 1e-9) : (double)(f + 1e-9f);
        p.inv_den = 1.0 / p.den;
        p.den_const = 1;
        p.s0s_const = 1;
        p.s0s_f = f;
        p.inv_s0s_f = 1.0f / f;
        p.s0s_d = (double)f;
        p.inv_s0s_d = 1.0 / (double)f;
    }
    p.rec = env->rec;
    p.recg = env->recg;
    p.book_n = is_generate(env) ? c.book_size : 0;
    // book_value's sigma terms at the handle's variance, the device's operations in the same
    // order (IEEE sqrt and division: the same bits) -- the GBM producers read them
    p.bk_sig = sqrt(p.var < 0.0 ? 0.0 : p.var);
    p.bk_isig = 1.0 / p.bk_sig;
    p.bk_s2 = p.bk_sig * p.bk_sig;
    p.bk_lam = (p.r_d + 0.5 * p.bk_s2) / p.bk_s2;
    p.book = env->dbook;
    p.book_tab = env->dbook_tab;
    p.book_rows = env->book_rows;
    p.book_rst = env->book_rst;
    p.tileC = nullptr;
#ifdef HE_TIMING
    if (!g_tim && hipMalloc(&g_tim, (size_t)5 * 8192 * 2 * 8) != hipSuccess) g_tim = nullptr;
    p.tim = g_tim;
#endif
    p.n_paths = env->n_paths;
    p.rstride = replay_stride(env->cfg.episode_length);
    p.roff = kRowOff;
}

template <int MODE>
static void launch_init_reset(he_env* env) {
    hipLaunchKernelGGL(init_reset_kernel<MODE>, dim3(1), dim3(64), 0, 0, env->p, env->rst);
}

static Params tile_params(const he_env* env, int b);

// Refresh the device copies of Params after fill_params.  Not stream-ordered, so the
// device is drained first (configuration calls only, never on the step path).
static he_status sync_dparams(he_env* env) {
    Params h[2] = {tile_params(env, 0), tile_params(env, 1)};
    HE_HIP(env, hipDeviceSynchronize());
    HE_HIP(env, hipMemcpy(env->dparams, h, sizeof(h), hipMemcpyHostToDevice));
    return HE_OK;
}

// (generate) reset market + reset obs, computed once on the device with the same
// device functions as the step path, then handed to every kernel by value.
static he_status upload_tables(he_env* env) {
    fill_params(env);
    if (is_generate(env)) {
        if (env->cfg.mode == HE_MODE_GBM) launch_init_reset<HE_MODE_GBM>(env);
        else launch_init_reset<HE_MODE_HESTON>(env);
        HE_HIP(env, hipGetLastError());
        HE_HIP(env, hipDeviceSynchronize());
        float rec[32];
        HE_HIP(env, hipMemcpy(rec, env->rst, sizeof(rec), hipMemcpyDeviceToHost));
        memcpy(env->rstv, rec, sizeof(env->rstv));
        if (env->cfg.book_size > 0) memcpy(&env->book_rst, rec + 20, sizeof(double));
        fill_params(env);
    }
    return sync_dparams(env);
}

// Params with the tile pointers of buffer b.
static Params tile_params(const he_env* env, int b) {
    Params p = env->p;
    if (!env->tile) return p;  // replay
    const size_t slots = (size_t)(env->cfg.market_block + 1) * (size_t)env->cfg.n_envs;
    p.tileA = env->tile + (size_t)b * 2 * slots;
    p.tileB = p.tileA + slots;
    if (env->cfg.book_size > 0) p.tileC = reinterpret_cast<double*>(env->tile + 4 * slots) + (size_t)b * slots;
    return p;
}

// A market_kernel launched beside step kernels (the side-stream prefetch) is held to
// 2 workgroups = 2 waves per SIMD by padding its LDS past a third of the CU's 160 KB:
// at 3 waves/SIMD it finishes sooner alone (74 vs 91 us per 64 steps at 65,536 envs)
// but takes issue slots from the latency-bound rollout wave (2.72 vs 2.27 us/step).
constexpr size_t kCuLds = 160 * 1024;
constexpr size_t kMktWgLds = kMktEnvs * (kMaxBlock + 1) * sizeof(double);  // one shS-sized array

template <int MODE, bool BOOK>
static void launch_market(he_env* env, int32_t advance_only, int buf, hipStream_t st, bool beside_steps) {
    int64_t blocks = (env->cfg.n_envs + kMktEnvs - 1) / kMktEnvs;
    const size_t stat = kMktWgLds * (1 + (MODE == HE_MODE_HESTON ? 1 : 0) + (BOOK ? 1 : 0));
    const size_t cap = kCuLds / 3 + 1024;  // > 1/3 of the CU: at most 2 workgroups
    const size_t pad = (beside_steps && stat < cap) ? cap - stat : 0;
    hipLaunchKernelGGL((market_kernel<MODE, BOOK>), dim3((unsigned)blocks), dim3(kMktEnvs * kMktLanes), pad, st,
                       tile_params(env, buf), env->cur, env->bak[buf], advance_only);
}

// generate the block that follows `cur` into tile buffer `buf` (advance_only = 0),
// or rewind `cur` to `advance_only` steps past the start of buffer `buf`'s block.
static he_status market(he_env* env, int32_t advance_only, int buf, hipStream_t st, bool beside_steps = false) {
    const bool book = env->cfg.book_size > 0;
    const bool b = beside_steps;
    if (env->cfg.mode == HE_MODE_GBM) {
        if (book) launch_market<HE_MODE_GBM, true>(env, advance_only, buf, st, b);
        else launch_market<HE_MODE_GBM, false>(env, advance_only, buf, st, b);
    } else {
        if (book) launch_market<HE_MODE_HESTON, true>(env, advance_only, buf, st, b);
        else launch_market<HE_MODE_HESTON, false>(env, advance_only, buf, st, b);
    }
    HE_HIP(env, hipGetLastError());
    return HE_OK;
}

// Make stream st wait for a pending prefetch on the side stream (join).
static he_status join_prefetch(he_env* env, hipStream_t st) {
    if (env->next_state == 1) {
        HE_HIP(env, hipStreamWaitEvent(st, env->ev_next, 0));
        env->next_state = 2;
    }
    return HE_OK;
}

// Bring `cur` to the position the envs are actually at (mid-block rewind) and
// drop every generated block.  Needed before partial resets and checkpoints.
static he_status materialize_market(he_env* env, hipStream_t st) {
    const int32_t M = env->cfg.market_block;
    he_status s = join_prefetch(env, st);
    if (s != HE_OK) return s;
    const bool generated_ahead = env->next_state != 0;
    if (env->block_pos < M || generated_ahead) {
        const int b = env->cur_buf;
        if (env->block_pos < M && env->block_pos > 0) {
            s = market(env, env->block_pos, b, st);
            if (s != HE_OK) return s;
        } else {
            // the current position is a block start: restore it from that block's bak
            const int bb = (env->block_pos >= M) ? (b ^ 1) : b;
            const Market& src = env->bak[bb];
            const int64_t N = env->cfg.n_envs;
            HE_HIP(env, hipMemcpyAsync(env->cur.ep, src.ep, N * 4, hipMemcpyDeviceToDevice, st));
            HE_HIP(env, hipMemcpyAsync(env->cur.t, src.t, N * 4, hipMemcpyDeviceToDevice, st));
            HE_HIP(env, hipMemcpyAsync(env->cur.S, src.S, N * 8, hipMemcpyDeviceToDevice, st));
            HE_HIP(env, hipMemcpyAsync(env->cur.C, src.C, N * 4, hipMemcpyDeviceToDevice, st));
            HE_HIP(env, hipMemcpyAsync(env->cur.P, src.P, N * 4, hipMemcpyDeviceToDevice, st));
            if (env->cur.v) HE_HIP(env, hipMemcpyAsync(env->cur.v, src.v, N * 8, hipMemcpyDeviceToDevice, st));
            if (env->cur.M) HE_HIP(env, hipMemcpyAsync(env->cur.M, src.M, N * 8, hipMemcpyDeviceToDevice, st));
        }
    }
    env->block_pos = M;
    env->next_state = 0;
    return HE_OK;
}

template <int MODE>
static void launch_reset(he_env* env, const int64_t* ids, int64_t count, float* obs, const he_info& inf,
                         hipStream_t st, const int64_t* eps = nullptr) {
    int64_t blocks = (count + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(reset_kernel<MODE>, dim3((unsigned)blocks), dim3(kBlock), 0, st, env->p, env->s,
                       env->cur, ids, count, obs, inf, eps);
}

template <int MODE, bool BOOK, bool FAST, bool GS>
static void launch_step_gs(he_env* env, const Params& p, const Io& io, bool info, int k, int slot0,
                           hipStream_t st) {
    int64_t blocks = (env->cfg.n_envs + kEpb - 1) / kEpb;
    if (io.pol_on) {  // policy rollouts (any k)
        void (*pk)(Params, State, Io, int, int) = step_kernel<MODE, false, false, BOOK, FAST, true, GS>;
        hipLaunchKernelGGL(pk, dim3((unsigned)blocks), dim3(kBlock), 0, st, p, env->s, io, k, slot0);
        return;
    }
    if (k == 1 && !info && !io.sums) {  // he_step (rollouts keep the episode summaries)
        constexpr bool REPLAY = (MODE == HE_MODE_REPLAY);
        const Params* pc = env->dparams + (REPLAY ? 0 : env->cur_buf);
        const float4* tA = REPLAY ? p.rec : p.tileA;
        const float4* tB = REPLAY ? p.recg : p.tileB;
        StepIo sio{io.act, io.obs, io.rew, io.term, io.trunc, io.tobs, io.sig, io.sig_cnt, io.sig_seq};
        if (env->vne_on && io.obs && io.rew && io.term && io.tobs) {  // + the eval VecNormalize step
            hipEvent_t a = (hipEvent_t)env->ev_start, b = (hipEvent_t)env->ev_stop;
            env->ev_start = env->ev_stop = nullptr;
            hipExtLaunchKernelGGL((step1_vne_kernel<MODE, BOOK, FAST, GS>), dim3((unsigned)blocks), dim3(kBlock), 0, st,
                                  a, b, 0, pc, p.n, tA, tB, (const double*)p.tileC, env->s, sio, slot0, env->vne);
            env->vn_fused = true;
            return;
        }
        if (env->vn_on) {  // + the VecNormalize moments in the same launch
            vn::MomentsArgs vm = env->vn;
            vm.obs = io.obs;
            vm.reward = io.rew;
            hipEvent_t a = (hipEvent_t)env->ev_start, b = (hipEvent_t)env->ev_stop;
            env->ev_start = env->ev_stop = nullptr;
            hipExtLaunchKernelGGL((step1_vn_kernel<MODE, BOOK, FAST, GS>), dim3((unsigned)blocks), dim3(kBlock), 0, st, a,
                                  b, 0, pc, p.n, tA, tB, (const double*)p.tileC, env->s, sio, slot0, vm);
            env->vn_fused = true;
            return;
        }
        if (env->ev_start) {
            hipEvent_t a = (hipEvent_t)env->ev_start, b = (hipEvent_t)env->ev_stop;
            env->ev_start = env->ev_stop = nullptr;
            hipExtLaunchKernelGGL((step1_kernel<MODE, BOOK, FAST, GS>), dim3((unsigned)blocks), dim3(kBlock), 0, st, a, b, 0,
                                  pc, p.n, tA, tB, (const double*)p.tileC, env->s, sio, slot0);
            return;
        }
        hipLaunchKernelGGL((step1_kernel<MODE, BOOK, FAST, GS>), dim3((unsigned)blocks), dim3(kBlock), 0, st, pc, p.n, tA, tB,
                           (const double*)p.tileC, env->s, sio, slot0);
        return;
    }
    void (*kern)(Params, State, Io, int, int);
    if (k == 1 && !io.sums)
        kern = info ? step_kernel<MODE, true, true, BOOK, false, false, GS>
                    : step_kernel<MODE, false, true, BOOK, FAST, false, GS>;
    else
        kern = info ? step_kernel<MODE, true, false, BOOK, false, false, GS>
                    : step_kernel<MODE, false, false, BOOK, FAST, false, GS>;
    if (env->ev_start) {  // one-shot: bracket exactly this dispatch (hipExtLaunchKernelGGL)
        hipEvent_t a = (hipEvent_t)env->ev_start, b = (hipEvent_t)env->ev_stop;
        env->ev_start = env->ev_stop = nullptr;
        hipExtLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kBlock), 0, st, a, b, 0, p, env->s, io, k, slot0);
        return;
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kBlock), 0, st, p, env->s, io, k, slot0);
}

template <int MODE, bool BOOK, bool FAST>
static void launch_step(he_env* env, const Params& p, const Io& io, bool info, int k, int slot0,
                        hipStream_t st) {
    if constexpr (MODE == HE_MODE_GBM) {
        if (!p.tile_greeks) {
            launch_step_gs<MODE, BOOK, FAST, true>(env, p, io, info, k, slot0, st);
            return;
        }
    }
    launch_step_gs<MODE, BOOK, FAST, false>(env, p, io, info, k, slot0, st);
}

template <int MODE, bool BOOK, bool FAST, bool GS>
static void launch_fused_gs(he_env* env, const Params& p, const Io& io, int k, int slot0, hipStream_t st) {
    const int64_t sblocks = (env->cfg.n_envs + kEpb - 1) / kEpb;
    const int64_t mblocks = (env->cfg.n_envs + kMktEnvs - 1) / kMktEnvs;
    const int nb = env->cur_buf ^ 1;
    const dim3 grid((unsigned)(sblocks + mblocks));
    size_t pad = 0;
    hipEvent_t a = nullptr, b = nullptr;
    if (env->ev_start) {  // one-shot: bracket exactly this dispatch (hipExtLaunchKernelGGL)
        a = (hipEvent_t)env->ev_start;
        b = (hipEvent_t)env->ev_stop;
        env->ev_start = env->ev_stop = nullptr;
    }
    (void)p;
    const Params* pc = env->dparams;
    const int32_t buf = env->cur_buf;
    if (a)
        hipExtLaunchKernelGGL((step_market_kernel<MODE, BOOK, FAST, GS>), grid, dim3(kBlock), pad, st, a, b, 0, pc, buf,
                              env->s, io, k, slot0, env->cur, env->bak[nb], (int32_t)sblocks);
    else
        hipLaunchKernelGGL((step_market_kernel<MODE, BOOK, FAST, GS>), grid, dim3(kBlock), pad, st, pc, buf, env->s, io,
                           k, slot0, env->cur, env->bak[nb], (int32_t)sblocks);
}

// step the current block (k steps from slot0) and generate the next block into the
// other tile buffer, one dispatch (step_market_kernel)
template <int MODE, bool BOOK, bool FAST>
static void launch_fused(he_env* env, const Params& p, const Io& io, int k, int slot0, hipStream_t st) {
    if constexpr (MODE == HE_MODE_GBM) {
        if (!p.tile_greeks) {
            launch_fused_gs<MODE, BOOK, FAST, true>(env, p, io, k, slot0, st);
            return;
        }
    }
    launch_fused_gs<MODE, BOOK, FAST, false>(env, p, io, k, slot0, st);
}

// Start the next block: make its market tile current (generated ahead on the side
// stream, or now on `st`), then prefetch the block after it on the side stream so
// that market_kernel(b+1) runs concurrently with the step kernels of block b.
static he_status advance_block(he_env* env, hipStream_t st, bool prefetch) {
    const int nb = env->cur_buf ^ 1;
    if (env->next_state == 0) {
        he_status s = market(env, 0, nb, st);
        if (s != HE_OK) return s;
    } else {
        he_status s = join_prefetch(env, st);
        if (s != HE_OK) return s;
    }
    env->cur_buf = nb;
    env->block_pos = 0;
    env->next_state = 0;
    if (prefetch) {
        // fork: the side stream starts after everything already enqueued on st
        HE_HIP(env, hipEventRecord(env->ev_fork, st));
        HE_HIP(env, hipStreamWaitEvent(env->xs, env->ev_fork, 0));
        he_status s = market(env, 0, nb ^ 1, env->xs, true);
        if (s != HE_OK) return s;
        HE_HIP(env, hipEventRecord(env->ev_next, env->xs));
        env->next_state = 1;
    }
    return HE_OK;
}

// The configuration the FAST step kernels are specialised for (generate modes).
static bool fast_config(const he_env* env) {
    const he_config& c = env->cfg;
    return c.mode != HE_MODE_REPLAY && c.variant == 2 && c.loss_type != HE_LOSS_MSE && c.shares_to_hedge != 0 &&
           c.record_metrics && c.max_contracts_held_per_type > 0 && c.episode_length > 0 &&
           env->p.s0s_const && env->p.den_const;
}

// The lean LDS steppers (branch-free, unguarded Markstein divisions, div_by_nb): the
// FAST configuration with every output buffer given, and prices and cash where every
// P&L is 0 or a normal number far from the f64 range ends (S0 and initial cash in
// [1e-30, 1e30]: a P&L is a difference of portfolio values, a multiple of their ulp).
static bool lds_lean_config(const he_env* env, const Io& io) {
    const he_config& c = env->cfg;
    const double s0 = c.s0, ic = fabs(c.initial_cash);
    const Params& p = env->p;
    // greeks_lean's constants (GBM); the Heston lean obs takes greeks_fast<false> at the slot's v
    const bool normal_greeks = c.mode == HE_MODE_HESTON || (!p.tenor_small && p.g_sigma > 1e-6f && p.g_sst >= 1e-9);
    // the lean kernels' producers make rolling-ATM marks only (marks<MODE, false>)
    // (S0 <= 1e20: S / max(S0, 25) >= 1e-8 / 1e20 stays a normal f32 for the f32 obs quotient)
    return fast_config(env) && io.obs && io.rew && io.term && s0 >= 1e-30 && s0 <= 1e20 && ic <= 1e30 &&
           normal_greeks && c.mark == HE_MARK_ROLLING_ATM && (c.book_size > 0 || p.T < lds_thp_rows());
}

// he_rollout through lds_rollout_kernel: GBM or Heston, with or without a book (HE_LDS_ROLLOUT=0
// falls back to the market-tile kernels).  The market position `cur` must be where the
// envs are (no block generated ahead, no mid-block position): materialize_market
// rewinds it, a no-op after an LDS rollout.  Afterwards `cur` is exact again and the
// tiles are invalid (the next he_step regenerates its block from `cur`).
static bool lds_rollout_eligible(const he_env* env) {
    return env->lds_rollout && (env->cfg.mode == HE_MODE_GBM || env->cfg.mode == HE_MODE_HESTON) &&
           (env->cfg.book_size == 0 || env->book_rows <= kLdsBookRows);
}

// he_rollout_policy through lds_rollout_kernel<..., POL>: every generate configuration the LDS
// rollout takes (the policy in both steppers, lean or generic), autoreset; the obs / reward /
// terminated buffers may be absent.
static bool lds_policy_eligible(const he_env* env) {
    return env->lds_policy && env->cfg.autoreset && lds_rollout_eligible(env);
}

static he_status launch_lds_rollout(he_env* env, const Io& io, int k_total, hipStream_t st) {
    he_status s = materialize_market(env, st);
    if (s != HE_OK) return s;
    const int64_t blocks = (env->cfg.n_envs + kLdsEnvs - 1) / kLdsEnvs;
    const Params* pc = env->dparams;  // buffer 0's copy: the tile pointers are not used
    const bool book = env->cfg.book_size > 0, pol = io.pol_on;
    bool lean = lds_lean_config(env, io);
    if (pol) {   // policy rollouts may return no obs / reward / done: the lean test on the rest
        Io o = io;
        o.obs = o.obs ? o.obs : reinterpret_cast<float*>(16);
        o.rew = o.rew ? o.rew : reinterpret_cast<float*>(16);
        o.term = o.term ? o.term : reinterpret_cast<uint8_t*>(16);
        lean = lds_lean_config(env, o);
    }
    void (*kern)(const Params*, State, Io, int, Market);
    void (*kern_p)(const Params*, State, Io, int, Market);   // the persistent-grid instance
    int threads;
#define HE_LDS_PICK(M, B, L)                                                  \
    do {                                                                      \
        if (pol) {                                                            \
            kern = lds_rollout_kernel<M, B, L, false, true>;                  \
            kern_p = lds_rollout_kernel<M, B, L, !(B), true>;                 \
        } else {                                                              \
            kern = lds_rollout_kernel<M, B, L, false>;                        \
            kern_p = lds_rollout_kernel<M, B, L, !(B)>;                       \
        }                                                                     \
        threads = LdsGeom<M, B>::threads;                                     \
    } while (0)
    if (env->cfg.mode == HE_MODE_HESTON) {
        if (lean) {
            if (book) HE_LDS_PICK(HE_MODE_HESTON, true, true);
            else HE_LDS_PICK(HE_MODE_HESTON, false, true);
        } else {
            if (book) HE_LDS_PICK(HE_MODE_HESTON, true, false);
            else HE_LDS_PICK(HE_MODE_HESTON, false, false);
        }
    } else if (book) {
        if (lean) HE_LDS_PICK(HE_MODE_GBM, true, true);
        else HE_LDS_PICK(HE_MODE_GBM, true, false);
    } else {
        if (lean) HE_LDS_PICK(HE_MODE_GBM, false, true);
        else HE_LDS_PICK(HE_MODE_GBM, false, false);
    }
#undef HE_LDS_PICK
    // the persistent grid: as many workgroups as the device holds at once (one round), each
    // looping over tiles -- past one round, workgroups that start as others finish take their
    // roles from a ticket that no longer lines up with the SIMDs they land on
    int64_t grid = blocks;
    if (env->lds_persist) {
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern_p, threads, 0) == hipSuccess &&
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, env->cfg.device) == hipSuccess &&
            per_cu > 0 && cus > 0 && grid > (int64_t)per_cu * cus)
            grid = (int64_t)per_cu * cus;
        (void)hipGetLastError();
    }
    if (env->lds_grid_cap > 0 && grid > env->lds_grid_cap) grid = env->lds_grid_cap;
    env->lds_grid = grid;
    // with a book the persistent instance spills (13 VGPRs) and measured slower (config 4
    // 5.64 vs 5.48 ms, config 5 1.49 vs 1.46 ms, profiles/r06bal_*): one workgroup per tile there
    if (grid < blocks && !book) kern = kern_p;
    else grid = blocks;
    if (env->ev_start) {  // one-shot: bracket exactly this dispatch
        hipEvent_t a = (hipEvent_t)env->ev_start, b = (hipEvent_t)env->ev_stop;
        env->ev_start = env->ev_stop = nullptr;
        hipExtLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(threads), 0, st, a, b, 0, pc, env->s, io, k_total,
                              env->cur);
    } else {
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(threads), 0, st, pc, env->s, io, k_total, env->cur);
    }
    HE_HIP(env, hipGetLastError());
    env->block_pos = env->cfg.market_block;
    env->next_state = 0;
    return HE_OK;
}

// he_rollout in replay mode through lds_replay_kernel (HE_LDS_ROLLOUT=0: step_kernel): every
// output buffer given, episodes of at least one LDS block (at most one episode end per env
// and block), autoreset (he_rollout's precondition).
static bool lds_replay_eligible(const he_env* env, const Io& io) {
    return env->lds_rollout && env->cfg.autoreset && env->p.T >= kLdsM && env->n_paths > 0 && io.obs && io.rew &&
           io.term;
}

// The configuration the FAST replay steppers are specialised for (step_env / make_obs with
// the uniform branches on these flags compiled out).
static bool fast_replay_config(const he_env* env) {
    const he_config& c = env->cfg;
    return c.mode == HE_MODE_REPLAY && c.variant == 2 && c.loss_type != HE_LOSS_MSE && c.shares_to_hedge != 0 &&
           c.record_metrics && c.max_contracts_held_per_type > 0 && env->p.T > 0 && env->table_ordinary &&
           fabs(env->p.shares_d) >= 0x1p-100 && fabs(env->p.shares_d) <= 0x1p100;
}

// he_rollout_policy in replay mode through lds_replay_kernel<..., POL> (the obs / reward /
// terminated buffers may be absent)
static bool lds_replay_policy_eligible(const he_env* env, const Io& io) {
    Io o = io;
    o.obs = o.obs ? o.obs : reinterpret_cast<float*>(16);   // (lds_replay_eligible's output test only)
    o.rew = o.rew ? o.rew : reinterpret_cast<float*>(16);
    o.term = o.term ? o.term : reinterpret_cast<uint8_t*>(16);
    return env->lds_policy && lds_replay_eligible(env, o);
}

static he_status launch_lds_replay(he_env* env, const Io& io, int k_total, hipStream_t st) {
    const int64_t blocks = (env->cfg.n_envs + kLdsEnvs - 1) / kLdsEnvs;
    const Params* pc = env->dparams;
    // policy rollouts on the generic steppers in every configuration (the FAST instance with the
    // policy's sums spilled 25 VGPRs)
    const bool fast = fast_replay_config(env);
    void (*kern)(const Params*, State, Io, int) =
        io.pol_on ? lds_replay_kernel<false, true> : (fast ? lds_replay_kernel<true> : lds_replay_kernel<false>);
    if (env->ev_start) {  // one-shot: bracket exactly this dispatch
        hipEvent_t a = (hipEvent_t)env->ev_start, b = (hipEvent_t)env->ev_stop;
        env->ev_start = env->ev_stop = nullptr;
        hipExtLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), 0, st, a, b, 0, pc, env->s, io, k_total);
    } else {
        hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), 0, st, pc, env->s, io, k_total);
    }
    HE_HIP(env, hipGetLastError());
    return HE_OK;
}

static he_status launch_steps(he_env* env, Io io, bool info, int k_total, void* stream, bool rollout = false) {
    const he_config& c = env->cfg;
    if (c.mode == HE_MODE_REPLAY && !env->rec) return fail(env, HE_ESTATE, "no paths loaded (he_load_paths)");
    if (!env->ready) return fail(env, HE_ESTATE, "he_reset must be called before stepping");
    DeviceGuard dg(c.device);
    hipStream_t st = (hipStream_t)stream;
    io.sums = rollout && !io.pol_on;
    if (c.mode == HE_MODE_REPLAY) {
        if (rollout && !info && !io.pol_on && lds_replay_eligible(env, io)) return launch_lds_replay(env, io, k_total, st);
        if (io.pol_on && lds_replay_policy_eligible(env, io)) return launch_lds_replay(env, io, k_total, st);
        launch_step<HE_MODE_REPLAY, false, false>(env, env->p, io, info, k_total, 0, st);
        HE_HIP(env, hipGetLastError());
        return HE_OK;
    }
    if (rollout && !info && !io.pol_on && lds_rollout_eligible(env)) return launch_lds_rollout(env, io, k_total, st);
    if (io.pol_on && lds_policy_eligible(env)) return launch_lds_rollout(env, io, k_total, st);
    const int32_t M = c.market_block;
    const int64_t N = c.n_envs;
    int done = 0;
    while (done < k_total) {
        bool fuse = false;
        if (env->block_pos >= M) {
            // auto policy (MI355X, graph-mode he_step, GBM): at 65,536 envs the
            // background market waves slow the latency-bound step_kernel more than
            // they save (6.94 vs 6.05 us/step); from 2^18 envs the step_kernel is
            // bandwidth-bound and overlap wins (+5% at 262k, +14% at 524k, +19% at 1M)
            bool want = env->prefetch_mode == 2 ||
                        (env->prefetch_mode == 0 && (k_total > 1 || c.n_envs >= kPrefetchMinEnvs));
            // rollouts: the next block's market rides in the step grid (stream-ordered,
            // no side-stream join).  Not with a liability book: its market is 3x the
            // step work and VALU-bound, the side stream's overlap measures the same
            // (configs 4/5: 1.25e10 / 1.12e10 env-steps/s either way)
            fuse = want && env->fuse_market && k_total > 1 && !info && !io.pol_on && c.book_size == 0;
            he_status s = advance_block(env, st, want && !fuse);
            if (s != HE_OK) return s;
        }
        int k = k_total - done;
        if (k > M - env->block_pos) k = M - env->block_pos;
        Io sub = io;
        if (io.act) sub.act = io.act + (int64_t)done * N * 2;
        if (io.pol.act_out) sub.pol.act_out = io.pol.act_out + (int64_t)done * N * 2;
        if (io.obs) sub.obs = io.obs + (int64_t)done * N * kObs;
        if (io.rew) sub.rew = io.rew + (int64_t)done * N;
        if (io.term) sub.term = io.term + (int64_t)done * N;
        Params p = tile_params(env, env->cur_buf);
        const bool book = c.book_size > 0;
        const bool fast = fast_config(env);
        if (fuse) {  // never with a book (see above)
            if (c.mode == HE_MODE_GBM) {
                if (fast) launch_fused<HE_MODE_GBM, false, true>(env, p, sub, k, env->block_pos, st);
                else launch_fused<HE_MODE_GBM, false, false>(env, p, sub, k, env->block_pos, st);
            } else {
                if (fast) launch_fused<HE_MODE_HESTON, false, true>(env, p, sub, k, env->block_pos, st);
                else launch_fused<HE_MODE_HESTON, false, false>(env, p, sub, k, env->block_pos, st);
            }
            env->next_state = 2;  // ordered on st before the next block's steps
        } else if (c.mode == HE_MODE_GBM) {
            if (book) {
                if (fast) launch_step<HE_MODE_GBM, true, true>(env, p, sub, info, k, env->block_pos, st);
                else launch_step<HE_MODE_GBM, true, false>(env, p, sub, info, k, env->block_pos, st);
            } else {
                if (fast) launch_step<HE_MODE_GBM, false, true>(env, p, sub, info, k, env->block_pos, st);
                else launch_step<HE_MODE_GBM, false, false>(env, p, sub, info, k, env->block_pos, st);
            }
        } else {
            if (book) {
                if (fast) launch_step<HE_MODE_HESTON, true, true>(env, p, sub, info, k, env->block_pos, st);
                else launch_step<HE_MODE_HESTON, true, false>(env, p, sub, info, k, env->block_pos, st);
            } else {
                if (fast) launch_step<HE_MODE_HESTON, false, true>(env, p, sub, info, k, env->block_pos, st);
                else launch_step<HE_MODE_HESTON, false, false>(env, p, sub, info, k, env->block_pos, st);
            }
        }
        HE_HIP(env, hipGetLastError());
        env->block_pos += k;
        done += k;
    }
    return HE_OK;
}

extern "C" {

const char* he_version(void) { return "libhedgeenv 0.2 (gfx950)"; }

const char* he_last_error(const he_env* env) {
    if (!env) return "null handle";
    return env->err.c_str();
}

he_status he_config_init(he_config* cfg, int32_t variant) {
    if (!cfg) return HE_EINVAL;
    if (variant != 1 && variant != 2) return HE_EINVAL;
    memset(cfg, 0, sizeof(*cfg));
    cfg->abi_version = HE_ABI_VERSION;
    cfg->variant = variant;
    cfg->mode = HE_MODE_GBM;
    cfg->loss_type = HE_LOSS_ABS;
    cfg->n_envs = 1;
    cfg->global_env_offset = 0;
    cfg->transaction_cost_per_contract = variant == 2 ? 0.65 : 0.05;
    cfg->lambda_cost = 1.0;
    cfg->pnl_penalty_weight = 0.01;
    cfg->theta_weight = 0.0;
    cfg->slippage_bps = 0.0;
    cfg->initial_cash = 0.0;
    cfg->shares_to_hedge = 10000;
    cfg->max_contracts_held_per_type = 200;
    cfg->max_trade_per_step = 15;
    cfg->record_metrics = 1;
    cfg->autoreset = 1;
    cfg->risk_free_rate = 0.04;
    cfg->option_tenor_years = 30.0 / 252.0;
    cfg->episode_length = 252;
    cfg->device = 0;
    cfg->seed = 42;
    cfg->s0 = 496.48001098632812;  // data/historical_prices.csv last close (f32-exact)
    cfg->variance = 0.029028;
    cfg->mu = 0.04;
    cfg->dt = 1.0 / 252.0;
    cfg->heston_kappa = 2.0;
    cfg->heston_theta = 0.029028;
    cfg->heston_xi = 0.3;
    cfg->heston_rho = -0.7;  // RHO_DEFAULT, rbergomi_sim.py:26
    cfg->market_block = 64;
    return HE_OK;
}

he_status he_create(const he_config* cfg, he_env** out) {
    if (!cfg || !out) return HE_EINVAL;
    *out = nullptr;
    he_env* env = new (std::nothrow) he_env();
    if (!env) return HE_ENOMEM;
    env->cfg = *cfg;
    he_config& c = env->cfg;
    *out = env;  // returned even on failure so the caller can read the message
    if (c.abi_version != HE_ABI_VERSION)
        return fail(env, HE_EINVAL, "abi_version %d != %d", c.abi_version, HE_ABI_VERSION);
    if (c.variant != 1 && c.variant != 2) return fail(env, HE_EINVAL, "variant must be 1 or 2");
    if (c.mode < 0 || c.mode > 2) return fail(env, HE_EINVAL, "bad mode %d", c.mode);
    if (c.loss_type < 0 || c.loss_type > 3) return fail(env, HE_EINVAL, "bad loss_type %d", c.loss_type);
    if (c.n_envs < 1 || c.n_envs > (int64_t)1 << 31) return fail(env, HE_EINVAL, "n_envs out of range");
    if (c.global_env_offset < 0) return fail(env, HE_EINVAL, "global_env_offset < 0");
    if (c.max_contracts_held_per_type < 0 || c.max_contracts_held_per_type > 32767)
        return fail(env, HE_EINVAL, "max_contracts_held_per_type must be in [0, 32767]");
    if (c.max_trade_per_step < 0 || c.max_trade_per_step > 32767)
        return fail(env, HE_EINVAL, "max_trade_per_step must be in [0, 32767]");
    if (c.mode != HE_MODE_REPLAY && (c.episode_length < 1 || c.episode_length > (1 << 30)))
        return fail(env, HE_EINVAL, "episode_length must be >= 1");
    if (c.book_size < 0 || c.book_size > HE_BOOK_MAX)
        return fail(env, HE_EINVAL, "book_size must be in [0, %d]", HE_BOOK_MAX);
    if (c.book_size > 0 && c.mode == HE_MODE_REPLAY)
        return fail(env, HE_EINVAL, "the liability book needs a generate mode (GBM / Heston)");
    if (c.mark != HE_MARK_ROLLING_ATM && c.mark != HE_MARK_FIXED_EUROPEAN)
        return fail(env, HE_EINVAL, "bad mark %d (he_mark)", c.mark);
    if (c.mark != HE_MARK_ROLLING_ATM && c.mode == HE_MODE_REPLAY)
        return fail(env, HE_EINVAL, "replay mode reads its marks from the table (mark must be HE_MARK_ROLLING_ATM)");
    for (int k = 0; k < c.book_size; ++k)
        if (c.book[k].type < HE_BOOK_CALL || c.book[k].type > HE_BOOK_UO_CALL)
            return fail(env, HE_EINVAL, "book[%d].type %d is not an he_book_type", k, c.book[k].type);
    if (c.market_block == 0) c.market_block = 64;
    if (c.market_block < 1 || c.market_block > kMaxBlock)
        return fail(env, HE_EINVAL, "market_block must be in [1, %d]", kMaxBlock);
    DeviceGuard dg(c.device);
    if (!dg.ok) return fail(env, HE_EHIP, "hipSetDevice(%d) failed", c.device);
    const int64_t N = c.n_envs;
    // one allocation, 256-B aligned SoA fields
    struct F {
        size_t bytes;
        void** dst;
        bool state;  // part of the checkpoint blob
    };
    std::vector<F> fs;
    fs.push_back({(size_t)N * 4, (void**)&env->s.t, true});
    fs.push_back({(size_t)N * 4, (void**)&env->s.pos, true});
    fs.push_back({(size_t)N * 8, (void**)&env->s.cash, true});
    fs.push_back({(size_t)N * 56, (void**)&env->s.acc, true});
    fs.push_back({(size_t)N * 4, (void**)&env->s.acc_len, true});
    fs.push_back({(size_t)N * 16, (void**)&env->s.last, true});
    fs.push_back({(size_t)N * 24, (void**)&env->s.sum, true});
    fs.push_back({(size_t)N * 4, (void**)&env->s.sum_len, true});
    if (c.mode == HE_MODE_REPLAY) {
        fs.push_back({(size_t)N * 4, (void**)&env->s.path, true});
        fs.push_back({(size_t)N * 4, (void**)&env->s.s0, true});
        fs.push_back({(size_t)N * 32, (void**)&env->s.pcg, true});
        fs.push_back({(size_t)N * 8, (void**)&env->s.pcgb, true});
    } else {
        Market* ms[3] = {&env->cur, &env->bak[0], &env->bak[1]};
        for (int k = 0; k < 3; ++k) {
            fs.push_back({(size_t)N * 4, (void**)&ms[k]->ep, k == 0});
            fs.push_back({(size_t)N * 4, (void**)&ms[k]->t, k == 0});
            fs.push_back({(size_t)N * 8, (void**)&ms[k]->S, k == 0});
            fs.push_back({(size_t)N * 4, (void**)&ms[k]->C, k == 0});
            fs.push_back({(size_t)N * 4, (void**)&ms[k]->P, k == 0});
            if (c.mode == HE_MODE_HESTON) fs.push_back({(size_t)N * 8, (void**)&ms[k]->v, k == 0});
            if (c.book_size > 0) fs.push_back({(size_t)N * 8, (void**)&ms[k]->M, k == 0});
        }
    }
    size_t total = 0;
    for (auto& f : fs) total += (f.bytes + 255) & ~(size_t)255;
    void* mem = nullptr;
    hipError_t e = hipMalloc(&mem, total);
    if (e != hipSuccess) return fail(env, HE_ENOMEM, "hipMalloc(%zu) failed: %s", total, hipGetErrorString(e));
    env->state_mem = mem;
    env->state_bytes = total;
    size_t off = 0;
    for (auto& f : fs) {
        *f.dst = (char*)mem + off;
        if (f.state) env->fields.push_back({f.bytes, *f.dst});
        off += (f.bytes + 255) & ~(size_t)255;
    }
    HE_HIP(env, hipMemset(mem, 0, total));
    {   // every mode: the LDS rollout kernels (HE_LDS_ROLLOUT=0) and policy rollouts on them
        // (HE_LDS_POLICY=0) can be switched off for A/B and parity runs against the tile kernels
        const char* el = getenv("HE_LDS_ROLLOUT");
        env->lds_rollout = !(el && el[0] == '0');
        const char* eo = getenv("HE_LDS_POLICY");
        env->lds_policy = !(eo && eo[0] == '0');
    }
    if (is_generate(env)) {
        // 2 buffers x ({S,v,C,P} | {greeks, lag}) float4 slots (+ 2 x f64 book slots)
        size_t tb = (size_t)4 * (size_t)(c.market_block + 1) * (size_t)N * sizeof(float4);
        if (c.book_size > 0) tb += (size_t)2 * (size_t)(c.market_block + 1) * (size_t)N * sizeof(double);
        e = hipMalloc(&env->tile, tb);
        if (e != hipSuccess) return fail(env, HE_ENOMEM, "hipMalloc(tile %zu) failed: %s", tb, hipGetErrorString(e));
        HE_HIP(env, hipMalloc(&env->rst, 32 * sizeof(float)));
        env->block_pos = c.market_block;
        env->prefetch_mode = c.market_prefetch;  // 0 auto, 1 never, 2 always
        {
            const char* ev = getenv("HE_FUSED_MARKET");
            env->fuse_market = !(ev && ev[0] == '0');
            const char* ep = getenv("HE_LDS_PERSIST");
            env->lds_persist = !(ep && ep[0] == '0');
            const char* eg = getenv("HE_LDS_MAX_GRID");
            env->lds_grid_cap = eg ? atoll(eg) : 0;
        }
        HE_HIP(env, hipStreamCreateWithFlags(&env->xs, hipStreamNonBlocking));
        HE_HIP(env, hipEventCreateWithFlags(&env->ev_fork, hipEventDisableTiming));
        HE_HIP(env, hipEventCreateWithFlags(&env->ev_next, hipEventDisableTiming));
    }
    HE_HIP(env, hipMalloc(&env->dparams, 2 * sizeof(Params)));
    if (c.book_size > 0) {
        BookOpt hb[HE_BOOK_MAX];
        for (int k = 0; k < c.book_size; ++k) {
            hb[k].type = c.book[k].type;
            hb[k].expiry = c.book[k].expiry;
            hb[k].K = c.book[k].strike;
            hb[k].H = c.book[k].barrier;
            hb[k].q100 = c.book[k].quantity * 100.0;
            hb[k].lnK = log(hb[k].K);
            hb[k].lnH = log(hb[k].H);
            hb[k].lnH2K = 2.0 * hb[k].lnH - hb[k].lnK;
            hb[k].invK = 1.0 / hb[k].K;
            hb[k].invH = 1.0 / hb[k].H;
        }
        HE_HIP(env, hipMalloc(&env->dbook, HE_BOOK_MAX * sizeof(BookOpt)));
        HE_HIP(env, hipMemcpy(env->dbook, hb, c.book_size * sizeof(BookOpt), hipMemcpyHostToDevice));
        int32_t max_exp = 1;
        for (int k = 0; k < c.book_size; ++k) max_exp = (c.book[k].expiry > max_exp) ? c.book[k].expiry : max_exp;
        HE_HIP(env, hipMalloc(&env->dbook_tab, (size_t)4 * (size_t)(max_exp + 1) * sizeof(double)));
        env->book_rows = max_exp + 1;
        hipLaunchKernelGGL(book_tab_kernel, dim3((unsigned)((max_exp + 256) / 256)), dim3(256), 0, 0, env->dbook_tab,
                           max_exp + 1, c.dt, c.risk_free_rate);
        HE_HIP(env, hipGetLastError());
        HE_HIP(env, hipDeviceSynchronize());
    }
    he_status st = upload_tables(env);
    if (st != HE_OK) return st;
    // default streams: env i seeded with (seed + global id) until he_seed is called
    if (c.mode == HE_MODE_REPLAY) {
        std::vector<uint64_t> seeds(N);
        for (int64_t i = 0; i < N; ++i) seeds[i] = c.seed + (uint64_t)(c.global_env_offset + i);
        return he_seed(env, nullptr, seeds.data(), N);
    }
    uint64_t sd = c.seed;
    return he_seed(env, nullptr, &sd, 1);
}

he_status he_destroy(he_env* env) {
    if (!env) return HE_OK;
    {
        DeviceGuard dg(env->cfg.device);
        if (env->state_mem) (void)hipFree(env->state_mem);
        if (env->rec) (void)hipFree(env->rec);
        if (env->recg) (void)hipFree(env->recg);
        if (env->tile) (void)hipFree(env->tile);
        if (env->rst) (void)hipFree(env->rst);
        if (env->dparams) (void)hipFree(env->dparams);
        if (env->dbook) (void)hipFree(env->dbook);
        if (env->dbook_tab) (void)hipFree(env->dbook_tab);
        if (env->ev_eps) (void)hipEventSynchronize(env->ev_eps);
        if (env->d_eps) (void)hipFree(env->d_eps);
        if (env->h_eps) (void)hipHostFree(env->h_eps);
        if (env->ev_eps) (void)hipEventDestroy(env->ev_eps);
        if (env->scratch_count) (void)hipFree(env->scratch_count);
        if (env->d_sig_cnt) (void)hipFree(env->d_sig_cnt);
        if (env->xs) {
            (void)hipStreamSynchronize(env->xs);
            (void)hipStreamDestroy(env->xs);
        }
        if (env->ev_fork) (void)hipEventDestroy(env->ev_fork);
        if (env->ev_next) (void)hipEventDestroy(env->ev_next);
    }
    delete env;
    return HE_OK;
}

he_status he_load_paths(he_env* env, const float* S, const float* v, const float* C, const float* P,
                        int64_t n_paths, int64_t n_cols) {
    if (!env) return HE_EINVAL;
    if (env->cfg.mode != HE_MODE_REPLAY) return fail(env, HE_ESTATE, "he_load_paths needs HE_MODE_REPLAY");
    if (!S || !v || !C || !P) return fail(env, HE_EINVAL, "null table pointer");
    if (n_paths < 1 || n_cols < 2) return fail(env, HE_ESHAPE, "Data shapes are inconsistent.");
    if (n_cols - 1 > (1 << 30)) return fail(env, HE_ESHAPE, "episode too long");
    DeviceGuard dg(env->cfg.device);
    const int64_t T = n_cols - 1;
    const int64_t W = replay_stride(T);   // padded row stride (see kRowOff); padding slots are zeros
    std::vector<float4> rec;
    try {
        rec.assign((size_t)(n_paths * W), make_float4(0.f, 0.f, 0.f, 0.f));
    } catch (...) {
        return fail(env, HE_ENOMEM, "host allocation of %lld records failed", (long long)(n_paths * W));
    }
    // an ordinary table (he_env::table_ordinary): prices 0 or finite and >= 2^-100 in magnitude,
    // S0 (row 0; < 1e-6 is replaced by 1) <= 2^24
    auto ordinary = [](float a) {   // 0, or finite and >= 2^-100 in magnitude
        return a == 0.0f || (fabsf(a) >= 7.8886090522101181e-31f && fabsf(a) <= 3.4028234663852886e38f);
    };
    bool ord = true;
    for (int64_t q = 0; q < n_paths; ++q) {
        for (int64_t t = 0; t <= T; ++t) {
            int64_t tc = t < T ? t : T - 1;  // terminal step keeps the last marks (:229-231)
            float4 r;
            r.x = S[q * n_cols + t];
            r.y = v[q * n_cols + t];
            r.z = C[q * T + tc];
            r.w = P[q * T + tc];
            rec[(size_t)(q * W + kRowOff + t)] = r;
            ord = ord && ordinary(r.x) && ordinary(r.z) && ordinary(r.w);
        }
        ord = ord && (S[q * n_cols] < 1e-6f || S[q * n_cols] <= 16777216.0f);
    }
    const size_t bytes = rec.size() * sizeof(float4);
    float4* d = nullptr;
    float4* dg2 = nullptr;
    hipError_t e = hipMalloc(&d, bytes);
    if (e != hipSuccess) return fail(env, HE_ENOMEM, "hipMalloc(paths) failed: %s", hipGetErrorString(e));
    e = hipMalloc(&dg2, bytes);
    if (e != hipSuccess) {
        (void)hipFree(d);
        return fail(env, HE_ENOMEM, "hipMalloc(path greeks) failed: %s", hipGetErrorString(e));
    }
    e = hipMemcpy(d, rec.data(), bytes, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(d);
        (void)hipFree(dg2);
        return fail(env, HE_EHIP, "hipMemcpy(paths) failed: %s", hipGetErrorString(e));
    }
    if (env->rec) (void)hipFree(env->rec);
    if (env->recg) (void)hipFree(env->recg);
    env->rec = d;
    env->recg = dg2;
    env->n_paths = n_paths;
    env->table_ordinary = ord;
    env->cfg.episode_length = (int32_t)T;
    env->ready = false;
    he_status st = upload_tables(env);
    if (st != HE_OK) return st;
    const int64_t count = (int64_t)rec.size();
    hipLaunchKernelGGL(table_greeks_kernel, dim3((unsigned)((count + kBlock - 1) / kBlock)), dim3(kBlock), 0, 0,
                       env->p, env->recg, count);
    HE_HIP(env, hipGetLastError());
    HE_HIP(env, hipDeviceSynchronize());
    return HE_OK;
}

he_status he_pcg64_seed_state(uint64_t seed, uint64_t state[4]) {
    if (!state) return HE_EINVAL;
    seed_sequence_pcg64(seed, state);
    return HE_OK;
}

he_status he_host_episode_draws(uint64_t seed, uint64_t n_paths, int64_t count, int64_t* out) {
    if (!out || count < 0 || n_paths < 1) return HE_EINVAL;
    uint64_t st[4];
    seed_sequence_pcg64(seed, st);
    Pcg64 g;
    g.sh = st[0];
    g.sl = st[1];
    g.ih = st[2];
    g.il = st[3];
    g.has32 = 0;
    g.buf32 = 0;
    for (int64_t k = 0; k < count; ++k) out[k] = pcg64_integers(g, n_paths);
    return HE_OK;
}

he_status he_host_philox(uint64_t seed, uint64_t env_id, uint64_t n, uint32_t out[4]) {
    if (!out) return HE_EINVAL;
    u32x4 c = {(uint32_t)n, (uint32_t)(n >> 32), (uint32_t)env_id, (uint32_t)(env_id >> 32)};
    u32x4 x = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    out[0] = x.x;
    out[1] = x.y;
    out[2] = x.z;
    out[3] = x.w;
    return HE_OK;
}

#ifdef HE_LDS_TIMING
he_status he_debug_lds_timing(void* host, size_t bytes) {
    const size_t cap = sizeof(g_lds_tim);
    if (bytes > cap) bytes = cap;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_lds_tim), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? HE_OK : HE_EHIP;
}
#endif

#ifdef HE_LDS_HWID
he_status he_debug_lds_hwid(void* host, size_t bytes) {
    const size_t cap = sizeof(g_lds_hwid);
    if (bytes > cap) bytes = cap;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_lds_hwid), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? HE_OK : HE_EHIP;
}
#endif

#ifdef HE_TIMING
he_status he_debug_timing(void* host, size_t bytes) {
    const size_t cap = (size_t)5 * 8192 * 2 * 8;
    if (bytes > cap) bytes = cap;
    return hipMemcpy(host, g_tim, bytes, hipMemcpyDeviceToHost) == hipSuccess ? HE_OK : HE_EHIP;
}
#endif

he_status he_device_rng(uint64_t seed, const uint64_t* env_ids, const uint64_t* step_index, int64_t count,
                        uint32_t* words, double* normals, void* stream) {
    if (count < 0 || (count > 0 && (!env_ids || !step_index))) return HE_EINVAL;
    if (count == 0) return HE_OK;
    hipLaunchKernelGGL(device_rng_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (uint32_t)seed, (uint32_t)(seed >> 32), env_ids, step_index, count, words, normals);
    return hipGetLastError() == hipSuccess ? HE_OK : HE_EHIP;
}

he_status he_device_math(int32_t op, const double* x, int64_t count, double* out, void* stream) {
    if (op < 0 || op > 5 || count < 0 || (count > 0 && (!x || !out))) return HE_EINVAL;
    if (count == 0) return HE_OK;
    const int64_t groups = (count + 3) / 4;
    hipLaunchKernelGGL(device_math_kernel, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       op, x, count, out, default_bs());
    return hipGetLastError() == hipSuccess ? HE_OK : HE_EHIP;
}

he_status he_host_math(int32_t op, const double* x, int64_t count, double* out) {
    if (op < 0 || op > 5 || count < 0 || (count > 0 && (!x || !out))) return HE_EINVAL;
    const BSConst bs = default_bs();
    for (int64_t g = 0; 4 * g < count; ++g) math_group(op, x, count, out, g, bs);
    return HE_OK;
}

he_status he_host_div_by(const double* a, int64_t count, double b, double* out) {
    if ((!a || !out) && count > 0) return HE_EINVAL;
    const double y = 1.0 / b;
    for (int64_t k = 0; k < count; ++k) out[k] = div_by(a[k], b, y);
    return HE_OK;
}

he_status he_host_box_muller(const double* u1, const double* u2, int64_t count, double* z1, double* z2) {
    if ((!u1 || !u2 || !z1 || !z2) && count > 0) return HE_EINVAL;
    for (int64_t k = 0; k < count; ++k) box_muller(u1[k], u2[k], z1 + k, z2 + k);
    return HE_OK;
}

he_status he_host_div_byf(const float* a, int64_t count, float b, float* out) {
    if ((!a || !out) && count > 0) return HE_EINVAL;
    const float y = 1.0f / b;
    for (int64_t k = 0; k < count; ++k) out[k] = div_byf(a[k], b, y);
    return HE_OK;
}

he_status he_seed(he_env* env, const int64_t* env_ids, const uint64_t* seeds, int64_t count) {
    if (!env) return HE_EINVAL;
    if (!seeds || count < 1) return fail(env, HE_EINVAL, "he_seed needs >= 1 seed");
    DeviceGuard dg(env->cfg.device);
    const int64_t N = env->cfg.n_envs;
    HE_HIP(env, hipDeviceSynchronize());
    if (env->cfg.mode == HE_MODE_REPLAY) {
        // read-modify-write the PCG64 arrays on the host (setup path, not per step)
        std::vector<uint64_t> pcg((size_t)(4 * N));
        std::vector<uint32_t> pcgb((size_t)(2 * N));
        HE_HIP(env, hipMemcpy(pcg.data(), env->s.pcg, pcg.size() * 8, hipMemcpyDeviceToHost));
        HE_HIP(env, hipMemcpy(pcgb.data(), env->s.pcgb, pcgb.size() * 4, hipMemcpyDeviceToHost));
        for (int64_t k = 0; k < count; ++k) {
            int64_t i = env_ids ? env_ids[k] : k;
            if (i < 0 || i >= N) return fail(env, HE_EINVAL, "env id %lld out of range", (long long)i);
            uint64_t st[4];
            seed_sequence_pcg64(seeds[k], st);
            for (int w = 0; w < 4; ++w) pcg[(size_t)(w * N + i)] = st[w];
            pcgb[(size_t)i] = 0;
            pcgb[(size_t)(N + i)] = 0;
        }
        HE_HIP(env, hipMemcpy(env->s.pcg, pcg.data(), pcg.size() * 8, hipMemcpyHostToDevice));
        HE_HIP(env, hipMemcpy(env->s.pcgb, pcgb.data(), pcgb.size() * 4, hipMemcpyHostToDevice));
    } else {
        // one Philox key per handle: per-env seeding has no generate-mode meaning
        if (env_ids || count != 1)
            return fail(env, HE_EINVAL, "generate modes take exactly one seed (the handle's Philox key), no env_ids");
        env->cfg.seed = seeds[0];
        fill_params(env);
        he_status s = sync_dparams(env);
        if (s != HE_OK) return s;
        // episode counters restart: the next reset starts episode 0 of every env
        HE_HIP(env, hipMemset(env->cur.ep, 0xFF, (size_t)N * 4));
        env->block_pos = env->cfg.market_block;
        env->ready = false;
    }
    return HE_OK;
}

he_status he_reset(he_env* env, const int64_t* env_ids, int64_t count, float* obs_out, const he_info* info,
                   void* stream) {
    if (!env) return HE_EINVAL;
    he_info inf;
    if (info) inf = *info;
    else memset(&inf, 0, sizeof(inf));
    const he_config& c = env->cfg;
    if (c.mode == HE_MODE_REPLAY && !env->rec) return fail(env, HE_ESTATE, "no paths loaded (he_load_paths)");
    if (!env_ids) count = c.n_envs;
    if (count < 0) return fail(env, HE_EINVAL, "count < 0");
    if (env_ids && !env->ready) return fail(env, HE_ESTATE, "the first reset must reset every env");
    if (count == 0) return HE_OK;
    DeviceGuard dg(c.device);
    hipStream_t st = (hipStream_t)stream;
    if (c.mode == HE_MODE_REPLAY) {
        launch_reset<HE_MODE_REPLAY>(env, env_ids, count, obs_out, inf, st);
    } else {
        // `cur` must be where the envs are (rewind): a partial reset keeps every other
        // env on its path, and a reset starts the episode after the env's current one
        // (cur.ep + 1), not after one a block generated ahead already reached
        he_status s = materialize_market(env, st);
        if (s != HE_OK) return s;
        env->block_pos = c.market_block;  // tiles regenerated on the next step
        env->next_state = 0;
        if (c.mode == HE_MODE_GBM) launch_reset<HE_MODE_GBM>(env, env_ids, count, obs_out, inf, st);
        else launch_reset<HE_MODE_HESTON>(env, env_ids, count, obs_out, inf, st);
    }
    HE_HIP(env, hipGetLastError());
    env->ready = true;
    return HE_OK;
}

he_status he_reset_episodes(he_env* env, const int64_t* env_ids, const int64_t* episode_idx, int64_t count,
                            float* obs_out, const he_info* info, void* stream) {
    if (!env) return HE_EINVAL;
    const he_config& c = env->cfg;
    if (c.mode != HE_MODE_REPLAY) return fail(env, HE_EINVAL, "he_reset_episodes: replay mode only");
    if (!env->rec) return fail(env, HE_ESTATE, "no paths loaded (he_load_paths)");
    if (!episode_idx) return fail(env, HE_EINVAL, "episode_idx is NULL");
    if (count < 0 || count > c.n_envs) return fail(env, HE_EINVAL, "count %lld not in [0, n_envs]", (long long)count);
    if (!env->ready && count != c.n_envs) return fail(env, HE_ESTATE, "the first reset must reset every env");
    for (int64_t j = 0; j < count; ++j)
        if (episode_idx[j] < 0 || episode_idx[j] >= env->p.n_paths)
            return fail(env, HE_EINVAL, "episode_idx[%lld] = %lld not in [0, %lld)", (long long)j,
                        (long long)episode_idx[j], (long long)env->p.n_paths);
    if (count == 0) return HE_OK;
    he_info inf;
    if (info) inf = *info;
    else memset(&inf, 0, sizeof(inf));
    DeviceGuard dg(c.device);
    hipStream_t st = (hipStream_t)stream;
    if (!env->d_eps || !env->h_eps || !env->ev_eps) {
        // the three staging objects are made together or not at all: a partial failure frees
        // what was made, so a later call retries from scratch instead of using a NULL buffer
        const size_t bytes = (size_t)c.n_envs * sizeof(int64_t);
        int64_t* d = nullptr;
        int64_t* h = nullptr;
        hipEvent_t ev = nullptr;
        hipError_t e = hipMalloc(&d, bytes);
        if (e == hipSuccess) e = hipHostMalloc((void**)&h, bytes, hipHostMallocDefault);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (e != hipSuccess) {
            if (ev) (void)hipEventDestroy(ev);
            if (h) (void)hipHostFree(h);
            if (d) (void)hipFree(d);
            (void)hipGetLastError();
            return fail(env, HE_EHIP, "he_reset_episodes: staging buffers: %s", hipGetErrorString(e));
        }
        if (env->ev_eps) (void)hipEventDestroy(env->ev_eps);
        if (env->h_eps) (void)hipHostFree(env->h_eps);
        if (env->d_eps) (void)hipFree(env->d_eps);
        env->d_eps = d;
        env->h_eps = h;
        env->ev_eps = ev;
    } else {
        // the previous call's copy and reset (on any stream) may still read the staging
        // buffers: wait for that reset alone, not for the caller's whole stream
        HE_HIP(env, hipEventSynchronize(env->ev_eps));
    }
    memcpy(env->h_eps, episode_idx, (size_t)count * sizeof(int64_t));
    HE_HIP(env, hipMemcpyAsync(env->d_eps, env->h_eps, (size_t)count * sizeof(int64_t), hipMemcpyHostToDevice, st));
    launch_reset<HE_MODE_REPLAY>(env, env_ids, count, obs_out, inf, st, env->d_eps);
    HE_HIP(env, hipGetLastError());
    HE_HIP(env, hipEventRecord(env->ev_eps, st));
    env->ready = true;
    return HE_OK;
}

he_status he_step(he_env* env, const float* actions, float* obs, float* reward, uint8_t* terminated,
                  uint8_t* truncated, float* terminal_obs, const he_info* info, void* stream) {
    if (!env) return HE_EINVAL;
    uint32_t* const sig = env->sig_flag;  // he_step_signal: one-shot, this step only (consumed on any return)
    env->sig_flag = nullptr;
    if (!actions) return fail(env, HE_EINVAL, "actions is NULL");
    Io io;
    memset(&io, 0, sizeof(io));
    io.act = actions;
    io.obs = obs;
    io.rew = reward;
    io.term = terminated;
    io.trunc = truncated;
    io.tobs = terminal_obs;
    bool want_info = false;
    if (info) {
        io.info = *info;
        const void* const* f = reinterpret_cast<const void* const*>(info);
        for (size_t k = 0; k < sizeof(he_info) / sizeof(void*); ++k) want_info |= f[k] != nullptr;
    }
    // he_vecnorm_attach arms THIS step only (one-shot): steps nobody armed -- the inner env
    // stepped directly, another wrapper's -- never touch a wrapper's returns or partials
    const bool vn = env->vn_on, vne = env->vne_on;
    if ((vn || vne) && (!obs || !reward)) {
        env->vn_on = env->vne_on = false;
        return fail(env, HE_EINVAL, "he_vecnorm_attach: he_step needs the obs and reward buffers");
    }
    if (vne && (!terminated || !terminal_obs)) {
        env->vne_on = false;
        return fail(env, HE_EINVAL, "he_vecnorm_attach_eval: he_step needs the terminated and terminal_obs buffers");
    }
    if (vne && want_info && env->vne.ep_ret && !io.info.reward_step) {
        // the info kernel runs, then the eval apply as its own launch: its Monitor sums add the
        // f64 reward, which only info->reward_step carries out of the step
        env->vne_on = false;
        return fail(env, HE_EINVAL, "he_vecnorm_attach_eval with Monitor sums: an he_step that requests info "
                                    "must request info->reward_step too");
    }
    if (sig) {
        if (vn || vne) {
            env->vn_on = env->vne_on = false;
            return fail(env, HE_EINVAL, "he_step_signal: the signal covers a step with no VecNormalize attached");
        }
        io.sig = sig;
        io.sig_cnt = env->d_sig_cnt;
        io.sig_seq = env->sig_seq + 1u == 0u ? 1u : env->sig_seq + 1u;
    }
    env->vn_fused = false;
    he_status s = launch_steps(env, io, want_info, 1, stream);
    if (sig && s == HE_OK) env->sig_seq = io.sig_seq;
    env->vn_on = env->vne_on = false;
    if (s == HE_OK && vne && !env->vn_fused) {
        // another step kernel ran (info requested): the eval VecNormalize step as its own
        // launch.  he_vecnorm_step with training = 0 launches the apply kernel alone, which reads
        // only the frozen statistics (never the scratch partials), for any n.
        // Monitor's sums take the f64 reward, which that kernel wrote to info->reward_step
        const vn::ApplyArgs& a = env->vne;
        he_status sv = he_vecnorm_step(&env->vne_p, env->cfg.n_envs, obs, reward, terminated, terminal_obs,
                                       a.returns, const_cast<double*>(a.stats), const_cast<double*>(a.stats),
                                       a.obs_out, a.rew_out, a.tobs_out, a.ep_ret, a.ep_len, a.ep_ret_done,
                                       a.ep_len_done, io.info.reward_step, stream);
        return sv == HE_OK ? sv : fail(env, sv, "he_step: the eval VecNormalize launch failed (status %d)", (int)sv);
    }
    if (s != HE_OK || !vn || env->vn_fused) return s;
    // VecNormalize attached, and this step took another kernel: the moments after it
    vn::MomentsArgs vm = env->vn;
    vm.obs = obs;
    vm.reward = reward;
    const int64_t blocks = (env->cfg.n_envs + kEpb - 1) / kEpb;
    hipLaunchKernelGGL(vn_moments_after_step_kernel, dim3((unsigned)blocks), dim3(vn::kVnThreads), 0,
                       (hipStream_t)stream, vm);
    HE_HIP(env, hipGetLastError());
    return HE_OK;
}

he_status he_vecnorm_attach(he_env* env, const he_vecnorm_params* p, double* returns, double* stats, void* scratch) {
    if (!env) return HE_EINVAL;
    if (!p) {  // detach
        env->vn_on = false;
        return HE_OK;
    }
    if (p->obs_dim != kObs || !isfinite(p->gamma)) return fail(env, HE_EINVAL, "bad he_vecnorm_params");
    if (!returns || !stats || !scratch) return fail(env, HE_EINVAL, "returns / stats / scratch are NULL");
    if (kEpb != vn::kVnChunk)  // he_vecnorm_apply merges one partial per 256 rows
        return fail(env, HE_EINVAL, "he_vecnorm_attach needs 256 envs per step workgroup (HE_STEP_EPW=64)");
    if (env->cfg.n_envs > (int64_t)vn::kVnMaxBlocks * kEpb)
        return fail(env, HE_EINVAL, "he_vecnorm_attach covers up to %d envs (use he_vecnorm_step)",
                    vn::kVnMaxBlocks * kEpb);
    vn::MomentsArgs m = {};
    m.n = env->cfg.n_envs;
    m.rows_per_block = kEpb;
    m.upd_obs = p->training && p->norm_obs;
    m.upd_ret = p->training != 0;
    m.shift_mean = 1;
    m.gamma = p->gamma;
    m.returns = returns;
    m.stats = stats;
    m.part = (double*)scratch;
    env->vn = m;
    env->vn_on = m.upd_obs || m.upd_ret;
    return HE_OK;
}

he_status he_vecnorm_attach_eval(he_env* env, const he_vecnorm_params* p, const he_vecnorm_out* out) {
    if (!env) return HE_EINVAL;
    if (!p) {  // disarm
        env->vne_on = false;
        return HE_OK;
    }
    if (p->obs_dim != kObs || p->training || !(p->clip_obs >= 0.0) || !(p->clip_reward >= 0.0) || !(p->epsilon >= 0.0))
        return fail(env, HE_EINVAL, "bad he_vecnorm_params (the eval arm takes training = 0)");
    if (!out || !out->stats || !out->returns || !out->obs_out || !out->reward_out)
        return fail(env, HE_EINVAL, "he_vecnorm_out: stats / returns / obs_out / reward_out are NULL");
    if ((out->ep_return != nullptr) != (out->ep_length != nullptr) ||
        (out->ep_return && (!out->ep_return_done || !out->ep_length_done)))
        return fail(env, HE_EINVAL, "he_vecnorm_out: the Monitor buffers come together");
    if (kEpb != vn::kVnChunk)
        return fail(env, HE_EINVAL, "he_vecnorm_attach_eval needs 256 envs per step workgroup");
    vn::ApplyArgs a = {};
    a.norm_obs = p->norm_obs != 0;
    a.norm_reward = p->norm_reward != 0;
    a.clip_obs = p->clip_obs;
    a.clip_rew = p->clip_reward;
    a.eps = p->epsilon;
    a.stats = out->stats;
    a.returns = out->returns;
    a.obs_out = out->obs_out;
    a.rew_out = out->reward_out;
    a.tobs_out = out->terminal_obs_out;
    a.ep_ret = out->ep_return;
    a.ep_len = out->ep_length;
    a.ep_ret_done = out->ep_return_done;
    a.ep_len_done = out->ep_length_done;
    env->vne = a;
    env->vne_p = *p;
    env->vne_on = true;
    env->vn_on = false;
    return HE_OK;
}

he_status he_rollout(he_env* env, int32_t k_steps, const float* actions, float* obs, float* reward,
                     uint8_t* terminated, void* stream) {
    if (!env) return HE_EINVAL;
    if (!actions) return fail(env, HE_EINVAL, "actions is NULL");
    if (k_steps < 1) return fail(env, HE_EINVAL, "k_steps must be >= 1");
    if (!env->cfg.autoreset) return fail(env, HE_ESTATE, "he_rollout needs autoreset=1");
    Io io;
    memset(&io, 0, sizeof(io));
    io.act = actions;
    io.obs = obs;
    io.rew = reward;
    io.term = terminated;
    return launch_steps(env, io, false, k_steps, stream, true);
}

he_status he_rollout_policy(he_env* env, int32_t k_steps, int32_t policy, float* actions_out, float* obs,
                            float* reward, uint8_t* terminated, he_episode_record* records, int64_t record_capacity,
                            unsigned long long* record_count, void* stream) {
    if (!env) return HE_EINVAL;
    if (k_steps < 1) return fail(env, HE_EINVAL, "k_steps must be >= 1");
    if (policy < HE_POLICY_NO_HEDGE || policy > HE_POLICY_DELTA_THRESHOLD)
        return fail(env, HE_EINVAL, "policy %d is not an he_policy", policy);
    if (!env->cfg.autoreset) return fail(env, HE_ESTATE, "he_rollout_policy needs autoreset=1");
    if (record_capacity < 0 || (record_capacity > 0 && (!records || !record_count)))
        return fail(env, HE_EINVAL, "records / record_count must be device pointers when record_capacity > 0");
    Io io;
    memset(&io, 0, sizeof(io));
    io.obs = obs;
    io.rew = reward;
    io.term = terminated;
    io.pol_on = true;
    io.pol.policy = policy;
    io.pol.act_out = actions_out;
    io.pol.rec = records;
    io.pol.cap = record_capacity;
    io.pol.count = record_count;
    if (record_capacity == 0) {  // no records: the atomic still needs a valid counter
        if (!env->scratch_count) HE_HIP(env, hipMalloc(&env->scratch_count, sizeof(unsigned long long)));
        io.pol.count = env->scratch_count;
    }
    return launch_steps(env, io, false, k_steps, stream);
}

he_status he_episode_summaries(he_env* env, float* out, void* stream) {
    if (!env || !out) return HE_EINVAL;
    DeviceGuard dg(env->cfg.device);
    const int64_t N = env->cfg.n_envs;
    if ((reinterpret_cast<uintptr_t>(out) & 15u) != 0) return fail(env, HE_EINVAL, "out must be 16-byte aligned");
    hipLaunchKernelGGL(summaries_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       env->s.last, reinterpret_cast<float4*>(out), N);
    HE_HIP(env, hipGetLastError());
    return HE_OK;
}

he_status he_sync_market(he_env* env, void* stream) {
    if (!env) return HE_EINVAL;
    if (!is_generate(env)) return HE_OK;
    DeviceGuard dg(env->cfg.device);
    return join_prefetch(env, (hipStream_t)stream);
}

he_status he_time_next_step(he_env* env, void* start_event, void* stop_event) {
    if (!env) return HE_EINVAL;
    if ((start_event == nullptr) != (stop_event == nullptr))
        return fail(env, HE_EINVAL, "pass both events or neither");
    env->ev_start = start_event;
    env->ev_stop = stop_event;
    return HE_OK;
}

he_status he_host_alloc(size_t bytes, void** host_ptr, void** device_ptr) {
    if (!host_ptr || !device_ptr || bytes == 0) return HE_EINVAL;
    *host_ptr = *device_ptr = nullptr;
    void* h = nullptr;
    if (hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
        (void)hipGetLastError();
        return HE_ENOMEM;
    }
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipHostFree(h);
        return HE_EHIP;
    }
    memset(h, 0, bytes);
    *host_ptr = h;
    *device_ptr = d;
    return HE_OK;
}

he_status he_host_free(void* host_ptr) {
    if (!host_ptr) return HE_OK;
    return hipHostFree(host_ptr) == hipSuccess ? HE_OK : HE_EHIP;
}

he_status he_stream_wait(void* stream) {
    return hipStreamSynchronize((hipStream_t)stream) == hipSuccess ? HE_OK : HE_EHIP;
}

he_status he_step_signal(he_env* env, uint32_t* flag) {
    if (!env) return HE_EINVAL;
    if (flag && (reinterpret_cast<uintptr_t>(flag) & 3u) != 0) return fail(env, HE_EINVAL, "flag must be 4-byte aligned");
    if (flag && !env->d_sig_cnt) {
        DeviceGuard dg(env->cfg.device);
        uint32_t* c = nullptr;
        HE_HIP(env, hipMalloc(&c, 256));
        if (hipMemset(c, 0, 256) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
            (void)hipGetLastError();
            (void)hipFree(c);
            return fail(env, HE_EHIP, "he_step_signal: counter allocation failed");
        }
        env->d_sig_cnt = c;
    }
    env->sig_flag = flag;
    return HE_OK;
}

uint32_t he_signal_seq(const he_env* env) { return env ? env->sig_seq : 0u; }

he_status he_signal_wait(he_env* env, const uint32_t* flag_host, void* stream) {
    if (!env || !flag_host) return HE_EINVAL;
    if (env->sig_seq == 0u) return fail(env, HE_ESTATE, "he_signal_wait: no he_step has been signalled");
    const uint32_t want = env->sig_seq;
    // spin on the host's view of the flag: a small-N step lands in ~5-10 us.  Past kSpin the
    // runtime's blocking wait takes over (a step queued behind long work burns no core), and
    // the flag must then hold the step's number: the kernel raises it before it ends.
    constexpr double kSpinUs = 200.0;
    if (__atomic_load_n(flag_host, __ATOMIC_ACQUIRE) == want) return HE_OK;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t it = 1;; ++it) {
        if (__atomic_load_n(flag_host, __ATOMIC_ACQUIRE) == want) return HE_OK;
        __builtin_ia32_pause();
        if ((it & 255u) == 0u &&
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() > kSpinUs)
            break;
    }
    DeviceGuard dg(env->cfg.device);
    HE_HIP(env, hipStreamSynchronize((hipStream_t)stream));
    if (__atomic_load_n(flag_host, __ATOMIC_ACQUIRE) == want) return HE_OK;
    return fail(env, HE_ESTATE, "he_signal_wait: the stream is idle and the flag holds %u, not step %u",
                (unsigned)__atomic_load_n(flag_host, __ATOMIC_ACQUIRE), (unsigned)want);
}

int64_t he_num_envs(const he_env* env) { return env ? env->cfg.n_envs : -1; }
int32_t he_episode_length(const he_env* env) { return env ? env->cfg.episode_length : -1; }
int64_t he_num_episodes(const he_env* env) { return env ? env->n_paths : -1; }

he_status he_get_config(const he_env* env, he_config* out) {
    if (!env || !out) return HE_EINVAL;
    *out = env->cfg;
    return HE_OK;
}

// Checkpoint blob: an 8-byte header {ready flag, format << 8}, then every state field.
// Format 3 added the version byte to the header; the field list is the one round-2 blobs
// (format 0: a bare ready flag) already carried, so those restore too (same size).  A
// change to the field list takes a new format number.
constexpr uint64_t kStateFormat = 3;
constexpr uint64_t kStateFormatLegacy = 0;

size_t he_state_size(const he_env* env) {
    if (!env) return 0;
    size_t n = 8;  // header: ready flag | format << 8
    for (auto& f : env->fields) n += f.first;
    return n;
}

he_status he_get_state(he_env* env, void* host_buf, size_t size) {
    if (!env || !host_buf) return HE_EINVAL;
    if (size != he_state_size(env)) return fail(env, HE_EINVAL, "state buffer size %zu != %zu", size, he_state_size(env));
    DeviceGuard dg(env->cfg.device);
    HE_HIP(env, hipDeviceSynchronize());
    if (is_generate(env)) {
        he_status s = materialize_market(env, 0);
        if (s != HE_OK) return s;
        HE_HIP(env, hipDeviceSynchronize());
    }
    char* dst = (char*)host_buf;
    uint64_t hdr = (env->ready ? 1u : 0u) | (kStateFormat << 8);
    memcpy(dst, &hdr, 8);
    dst += 8;
    for (auto& f : env->fields) {
        HE_HIP(env, hipMemcpy(dst, f.second, f.first, hipMemcpyDeviceToHost));
        dst += f.first;
    }
    return HE_OK;
}

he_status he_set_state(he_env* env, const void* host_buf, size_t size) {
    if (!env || !host_buf) return HE_EINVAL;
    if (size >= 8) {
        uint64_t h0;
        memcpy(&h0, host_buf, 8);
        if ((h0 >> 8) != kStateFormat && (h0 >> 8) != kStateFormatLegacy)
            return fail(env, HE_EINVAL, "checkpoint format %llu != %llu: saved by another libhedgeenv version",
                        (unsigned long long)(h0 >> 8), (unsigned long long)kStateFormat);
    }
    if (size != he_state_size(env)) return fail(env, HE_EINVAL, "state buffer size %zu != %zu", size, he_state_size(env));
    DeviceGuard dg(env->cfg.device);
    HE_HIP(env, hipDeviceSynchronize());
    const char* src = (const char*)host_buf;
    uint64_t hdr;
    memcpy(&hdr, src, 8);
    src += 8;
    for (auto& f : env->fields) {
        HE_HIP(env, hipMemcpy(f.second, src, f.first, hipMemcpyHostToDevice));
        src += f.first;
    }
    env->ready = (hdr & 0xFF) != 0;
    // the restored `cur` is the envs' position: drop every block generated from the old
    // trajectory (a fused rollout leaves next_state 2, a side-stream prefetch 1)
    env->block_pos = env->cfg.market_block;
    env->next_state = 0;
    return HE_OK;
}

}  // extern "C"
