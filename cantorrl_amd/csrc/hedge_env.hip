// hedge_env.hip -- libhedgeenv: the batched hedging environment for MI355X.
//
// One thread owns one env.  Per-env state is struct-of-arrays in HBM (every
// field access is a coalesced 4/8-byte-per-lane stream); the 13-float obs rows
// are staged through LDS so the [N][13] output leaves the CU as contiguous
// 16-byte-per-lane stores.  Done-masking uses a wave ballot so that waves with
// no terminating env skip the reset path entirely.
//
// Reference semantics restated here (file:line in /root/reference):
//   step            src/env/hedging_env_v2.py:175-294  (v1 src/env/hedging_env.py:171-270)
//   observation     src/env/hedging_env_v2.py:109-143
//   greeks          src/env/hedging_env_v2.py:79-107
//   reset           src/env/hedging_env_v2.py:145-173
//   BS marks        quantconnect/option_calculator.py:11-27
//   price advance   src/sim/rbergomi_sim.py:454-464
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <new>
#include <string>
#include <vector>

#include "../../include/hedge_env.h"
#include "he_math.h"

using namespace he;

namespace {

constexpr int kBlock = 256;
constexpr int kObs = HE_OBS_DIM;

// ------------------------------------------------------------------ parameters
struct Params {
    int64_t n;
    int64_t goff;
    int32_t T;
    int32_t variant, loss, record_metrics, autoreset, mode;
    int32_t mt, maxh;
    float mt_f;
    float init_cash_f;
    double tcpc, slip_frac, lam, w, theta, initial_cash;
    double shares_d;
    float shares_f;
    int32_t shares_zero;
    // observation / greeks constants (hedging_env_v2.py:57-58)
    float r_f, tenor_f;
    double r_d, tenor_d, sqrt_tenor;
    int32_t tenor_small;  // tenor <= 1e-6
    // generate-mode market
    uint32_t key0, key1;
    double s0;
    double var;           // GBM variance (Heston v0)
    float var_f;
    double sqrt_var, drift, sqrt_dt, mu, dt;
    BSConst bs;           // constant-sigma BS constants (GBM)
    float g_sigma, g_num_drift;  // constant-variance greeks: sigma, (r+0.5 sigma**2)*T (f32)
    double g_sst;                // sigma*sqrt(T) (f64)
    double h_kappa, h_theta, h_xi, h_rho, h_sqrt1mrho2;
    // replay
    const float4* rec;    // [n_paths][T+1] {S, v, C, P}, C/P at T = C/P at T-1
    int64_t n_paths;
};

struct State {
    uint32_t* t;
    uint32_t* pos;     // (uint16)call | (uint16)put << 16
    double* cash;
    int32_t* path;     // replay episode row
    float* s0;         // replay initial_S0_for_episode; -1 encodes the python 1.0 substitution
    uint64_t* pcg;     // replay [4][N]: state_hi, state_lo, inc_hi, inc_lo
    uint32_t* pcgb;    // replay [2][N]: has_uint32, uinteger
    double* S;         // generate f64 price
    float* C;
    float* P;
    uint32_t* ep;      // generate episode counter
    double* var;       // Heston variance
};

struct Io {
    const float* act;  // [K][N][2]
    float* obs;        // [K][N][13]
    float* rew;        // [K][N]
    uint8_t* term;     // [K][N]
    uint8_t* trunc;    // [N]
    float* tobs;       // [N][13]
    he_info info;
};

struct Env {
    uint32_t t;
    int32_t call, put;
    double cash;
    float S, v, C, P;   // current f32 market view (what the reference env holds)
    double S64, var64;  // generate-mode f64 state
    uint32_t ep;
    int32_t path;
    float s0;           // initial_S0_for_episode as f32 (1.0 when substituted)
    bool s0_small;
};

__device__ __forceinline__ int32_t unpack_lo(uint32_t p) { return (int32_t)(int16_t)(p & 0xFFFFu); }
__device__ __forceinline__ int32_t unpack_hi(uint32_t p) { return (int32_t)(int16_t)(p >> 16); }
__device__ __forceinline__ uint32_t pack_pos(int32_t c, int32_t q) {
    return ((uint32_t)(uint16_t)(int16_t)c) | (((uint32_t)(uint16_t)(int16_t)q) << 16);
}

// ------------------------------------------------------------------ greeks / obs
// hedging_env_v2.py:79-107.  S, v: the f32 current price / variance.
template <bool CONST_VAR>
__device__ __forceinline__ void greeks(const Params& p, float S, float v, double* cd, double* gam,
                                       double* pd) {
    float K = rintf(S);  // np.round: half-even
    if (S <= 1e-6f) {    // weak python 1e-6 compares as float32(1e-6)
        *cd = (K == 0.0f) ? 0.5 : ((K > 0.0f) ? 0.0 : 1.0);
        *pd = (K == 0.0f) ? -0.5 : ((K < 0.0f) ? 0.0 : -1.0);
        *gam = 0.0;
        return;
    }
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
        *cd = (S > K) ? 1.0 : ((S == K) ? 0.5 : 0.0);
        *pd = (S < K) ? -1.0 : ((S == K) ? -0.5 : 0.0);
        *gam = 0.0;
        return;
    }
    float Kc = np_maxf(K, 1e-6f);
    float num = logf(S / Kc) + num_drift;
    double d1;
    if (sst < 1e-9) {
        float s = (num > 0.0f) ? 1.0f : ((num < 0.0f) ? -1.0f : num);  // np.sign
        d1 = (double)(s * 10.0f);
    } else {
        d1 = (double)num / sst;
    }
    double n1 = ndtr(d1);
    *cd = n1;
    *pd = n1 - 1.0;
    double gd = (double)S * sst;
    *gam = (fabs(gd) < 1e-9) ? 0.0 : norm_pdf(d1) / gd;
}

// hedging_env_v2.py:109-143
template <bool CONST_VAR>
__device__ __forceinline__ void make_obs(const Params& p, const Env& e, float Sp, float vp, float* o) {
    float s0s = np_maxf(e.s0, 25.0f);
    o[0] = e.S / s0s;
    o[1] = e.C / s0s;
    o[2] = e.P / s0s;
    if (p.maxh != 0) {
        o[3] = (float)((double)e.call / (double)p.maxh);
        o[4] = (float)((double)e.put / (double)p.maxh);
    } else {
        o[3] = 0.0f;
        o[4] = 0.0f;
    }
    o[5] = e.v;
    o[6] = (p.T != 0) ? (float)((double)(p.T - (int32_t)e.t) / (double)p.T) : 0.0f;
    if (p.record_metrics) {
        double cd, g, pd;
        greeks<CONST_VAR>(p, e.S, e.v, &cd, &g, &pd);
        o[7] = (float)cd;
        o[8] = (float)g;
        o[9] = (float)pd;
        o[10] = (float)g;
    } else {
        o[7] = o[8] = o[9] = o[10] = 0.0f;
    }
    float ls = 0.0f, lv = 0.0f;
    if (!(e.t == 0 || Sp == 0.0f)) {
        ls = (e.S - Sp) / Sp;
        lv = e.v - vp;
    }
    o[11] = np_clipf(ls, -1.0f, 1.0f);
    o[12] = np_clipf(lv, -1.0f, 1.0f);
}

// f64 Black-Scholes marks at K = round(S) (rolling ATM, rbergomi_sim.py:418,437-446).
template <int MODE>
__device__ __forceinline__ void marks(const Params& p, double S64, double var64, float* C, float* P) {
    double K = rint(S64);
    double c, q;
    if (MODE == HE_MODE_HESTON) {
        BSConst h;
        double sig = sqrt(var64 < 0.0 ? 0.0 : var64);
        h.intrinsic = (p.tenor_d <= 0.0) || (sig <= 0.0);
        h.a = (p.r_d + 0.5 * (sig * sig)) * p.tenor_d;
        h.b = sig * p.sqrt_tenor;
        h.disc = p.bs.disc;
        bs_call_put(S64, K, h, &c, &q);
    } else {
        bs_call_put(S64, K, p.bs, &c, &q);
    }
    *C = (float)c;
    *P = (float)q;
}

// ------------------------------------------------------------------ load / store
template <int MODE>
__device__ __forceinline__ void load_env(const Params& p, const State& s, int64_t i, Env& e) {
    e.t = s.t[i];
    uint32_t pk = s.pos[i];
    e.call = unpack_lo(pk);
    e.put = unpack_hi(pk);
    e.cash = s.cash[i];
    if (MODE == HE_MODE_REPLAY) {
        e.path = s.path[i];
        float s0 = s.s0[i];
        e.s0_small = (s0 == -1.0f);
        e.s0 = e.s0_small ? 1.0f : s0;
        uint32_t tt = e.t > (uint32_t)p.T ? (uint32_t)p.T : e.t;
        float4 r = p.rec[(int64_t)e.path * (p.T + 1) + tt];
        e.S = r.x;
        e.v = r.y;
        e.C = r.z;
        e.P = r.w;
    } else {
        e.S64 = s.S[i];
        e.S = (float)e.S64;
        e.C = s.C[i];
        e.P = s.P[i];
        e.ep = s.ep[i];
        float s0f = (float)p.s0;
        e.s0_small = s0f < 1e-6f;
        e.s0 = e.s0_small ? 1.0f : s0f;
        if (MODE == HE_MODE_HESTON) {
            e.var64 = s.var[i];
            e.v = (float)e.var64;
        } else {
            e.var64 = p.var;
            e.v = p.var_f;
        }
    }
}

template <int MODE>
__device__ __forceinline__ void store_env(const State& s, int64_t i, const Env& e, bool reset) {
    s.t[i] = e.t;
    s.pos[i] = pack_pos(e.call, e.put);
    s.cash[i] = e.cash;
    if (MODE == HE_MODE_REPLAY) {
        if (reset) {
            s.path[i] = e.path;
            s.s0[i] = e.s0_small ? -1.0f : e.s0;
        }
    } else {
        s.S[i] = e.S64;
        s.C[i] = e.C;
        s.P[i] = e.P;
        if (reset) s.ep[i] = e.ep;
        if (MODE == HE_MODE_HESTON) s.var[i] = e.var64;
    }
}

// hedging_env_v2.py:145-173.  Replay: draw the episode row from the env's PCG64
// stream (gymnasium np_random.integers(num_episodes)); generate: next episode.
template <int MODE>
__device__ __forceinline__ void reset_env(const Params& p, const State& s, int64_t i, Env& e) {
    if (MODE == HE_MODE_REPLAY) {
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
        float4 r = p.rec[(int64_t)e.path * (p.T + 1)];
        e.S = r.x;
        e.v = r.y;
        e.C = r.z;
        e.P = r.w;
        e.s0_small = e.S < 1e-6f;
        e.s0 = e.s0_small ? 1.0f : e.S;
    } else {
        e.ep = e.ep + 1u;  // 0xFFFFFFFF after seeding -> episode 0
        e.S64 = p.s0;
        e.S = (float)e.S64;
        if (MODE == HE_MODE_HESTON) {
            e.var64 = p.var;
            e.v = (float)e.var64;
        }
        marks<MODE>(p, e.S64, e.var64, &e.C, &e.P);
    }
    e.t = 0;
    e.call = 0;
    e.put = 0;
    e.cash = p.initial_cash;
}

// ------------------------------------------------------------------ one step
struct StepOut {
    double reward;
    bool term;
    float Sp, vp;  // S_t_minus_1, v_t_minus_1 after the step
    // info
    double pnl, ps, tc, commission, slippage, rpc, tcp, thp, pv;
    float fc, fp;
    int32_t rqc, rqp, dc, dp;
};

// hedging_env_v2.py:175-262 (v1: hedging_env.py:171-245)
template <int MODE>
__device__ __forceinline__ void step_env(const Params& p, Env& e, float a0, float a1, int64_t gid,
                                         StepOut& o) {
    // portfolio_value_t_minus_1 is a pure function of the pre-step state
    double pv_prev;
    if (e.t == 0) {
        float pv0 = (p.shares_f * e.S + 0.0f) + p.init_cash_f;  // f32 (:167-168)
        pv_prev = (double)pv0;
    } else {
        double optv = ((double)e.call * (double)e.C) * 100.0 + ((double)e.put * (double)e.P) * 100.0;
        pv_prev = ((double)(p.shares_f * e.S) + optv) + e.cash;
    }
    // (i)-(ii) integer trade logic (:181-200)
    float fc = a0 * p.mt_f;
    float fp = a1 * p.mt_f;
    int32_t rqc = trade_round(fc, p.mt);
    int32_t rqp = trade_round(fp, p.mt);
    int32_t nc = e.call + rqc, np_ = e.put + rqp;
    nc = nc < -p.maxh ? -p.maxh : (nc > p.maxh ? p.maxh : nc);
    np_ = np_ < -p.maxh ? -p.maxh : (np_ > p.maxh ? p.maxh : np_);
    int32_t dc = nc - e.call, dp = np_ - e.put;
    e.call = nc;
    e.put = np_;
    // (iii) commission + slippage on pre-advance marks (:203-213)
    int32_t adc = dc < 0 ? -dc : dc, adp = dp < 0 ? -dp : dp;
    double commission = (double)(adc + adp) * p.tcpc;
    double slippage = 0.0, tc;
    if (p.variant == 2) {
        double sc = (((double)adc * (double)e.C) * 100.0) * p.slip_frac;
        double sp = (((double)adp * (double)e.P) * 100.0) * p.slip_frac;
        slippage = sc + sp;
        tc = commission + slippage;
    } else {
        tc = commission;
    }
    e.cash = e.cash - tc;
    // (iv)-(v) advance (:216-231)
    o.Sp = e.S;
    o.vp = e.v;
    uint32_t t_old = e.t;
    e.t = e.t + 1;
    bool term = (int32_t)e.t >= p.T;
    if (MODE == HE_MODE_REPLAY) {
        uint32_t tt = e.t > (uint32_t)p.T ? (uint32_t)p.T : e.t;
        float4 r = p.rec[(int64_t)e.path * (p.T + 1) + tt];  // C/P at T hold row T-1
        e.S = r.x;
        e.v = r.y;
        e.C = r.z;
        e.P = r.w;
    } else {
        uint64_t n = (uint64_t)e.ep * (uint64_t)p.T + (uint64_t)t_old;
        u32x4 ctr = {(uint32_t)n, (uint32_t)(n >> 32), (uint32_t)gid, (uint32_t)((uint64_t)gid >> 32)};
        u32x4 x = philox4x32_10(ctr, p.key0, p.key1);
        double u1 = u01(x.x, x.y), u2 = u01(x.z, x.w);
        double rad = sqrt(-2.0 * log(u1));
        double ang = 6.283185307179586 * u2;
        double Snew;
        if (MODE == HE_MODE_HESTON) {
            double sn, cs;
            sincos(ang, &sn, &cs);
            double z1 = rad * cs, z2 = rad * sn;
            double vp = e.var64 < 0.0 ? 0.0 : e.var64;  // full truncation
            double dw1 = p.sqrt_dt * z1, dw2 = p.sqrt_dt * z2;
            double dW = p.h_rho * dw1 + p.h_sqrt1mrho2 * dw2;  // rbergomi_sim.py:457
            double drift = (p.mu - 0.5 * vp) * p.dt;
            double diff = sqrt(vp) * dW;
            Snew = e.S64 * exp(drift + diff);
            e.var64 = e.var64 + p.h_kappa * (p.h_theta - vp) * p.dt + p.h_xi * sqrt(vp) * dw1;
        } else {
            double z0 = rad * cos(ang);
            double dW = p.sqrt_dt * z0;
            double diff = p.sqrt_var * dW;
            Snew = e.S64 * exp(p.drift + diff);
        }
        e.S64 = (Snew < 1e-8) ? 1e-8 : Snew;  // np.maximum(., 1e-8), NaN kept
        e.S = (float)e.S64;
        if (MODE == HE_MODE_HESTON) e.v = (float)e.var64;
        if (!term) marks<MODE>(p, e.S64, e.var64, &e.C, &e.P);
    }
    // (vi) mark-to-market (:233-238)
    double optv = ((double)e.call * (double)e.C) * 100.0 + ((double)e.put * (double)e.P) * 100.0;
    double pv = ((double)(p.shares_f * e.S) + optv) + e.cash;
    double pnl = pv - pv_prev;
    double ps = p.shares_zero ? pnl : pnl / p.shares_d;
    // (vii) reward (:243-262)
    double term_v;
    if (p.loss == HE_LOSS_MSE) {
        float f = np_maxf(e.s0, 25.0f);
        double den = e.s0_small ? (625.0 + 1e-9) : (double)(f * f + 1e-9f);
        term_v = (ps * ps) / den;
    } else {
        float f = np_maxf(e.s0, 25.0f);
        double den = e.s0_small ? (25.0 + 1e-9) : (double)(f + 1e-9f);
        term_v = fabs(ps) / den;
    }
    double rpc = (-p.w) * term_v;
    double tcp = p.lam * tc;
    double thp = 0.0, reward;
    if (p.variant == 2) {
        thp = p.theta * ((double)(p.T - (int32_t)e.t) / 252.0);
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

__device__ __forceinline__ void write_info(const he_info& inf, int64_t i, const StepOut& o,
                                           const Env& e, int variant) {
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
    if (inf.current_stock_price) inf.current_stock_price[i] = e.S;
    if (inf.current_volatility) inf.current_volatility[i] = e.v;
    if (inf.current_call_price) inf.current_call_price[i] = e.C;
    if (inf.current_put_price) inf.current_put_price[i] = e.P;
    if (inf.current_step) inf.current_step[i] = (int32_t)e.t;
}

// Write a [rows][13] tile staged in LDS to out (row-major [N][13]) with 16-B stores.
__device__ __forceinline__ void flush_obs_tile(const float* tile, float* out, int64_t row0, int rows) {
    float* dst = out + row0 * kObs;
    const int nf = rows * kObs;
    const int nv = nf >> 2;  // row0*13*4 is 16-B aligned because row0 % 4 == 0
    float4* d4 = reinterpret_cast<float4*>(dst);
    const float4* s4 = reinterpret_cast<const float4*>(tile);
    for (int k = threadIdx.x; k < nv; k += kBlock) d4[k] = s4[k];
    for (int k = (nv << 2) + threadIdx.x; k < nf; k += kBlock) dst[k] = tile[k];
}

// ------------------------------------------------------------------ kernels
// K fused steps; K == 1 is the Gym step.  INFO: write he_info fields.
template <int MODE, bool INFO>
__global__ __launch_bounds__(kBlock) void step_kernel(Params p, State s, Io io, int k_steps) {
    __shared__ __attribute__((aligned(16))) float tile[kBlock * kObs];
    const int64_t row0 = (int64_t)blockIdx.x * kBlock;
    const int64_t i = row0 + threadIdx.x;
    const bool live = i < p.n;
    const int rows = (int)((p.n - row0) < kBlock ? (p.n - row0) : kBlock);
    constexpr bool CONST_VAR = (MODE == HE_MODE_GBM);
    Env e;
    if (live) load_env<MODE>(p, s, i, e);
    bool reset_any = false;
    for (int k = 0; k < k_steps; ++k) {
        const int64_t koff = (int64_t)k * p.n;
        float o[kObs];
        bool term = false;
        if (live) {
            float2 a = reinterpret_cast<const float2*>(io.act)[koff + i];
            StepOut so;
            step_env<MODE>(p, e, a.x, a.y, p.goff + i, so);
            term = so.term;
            if (INFO) write_info(io.info, i, so, e, p.variant);
            make_obs<CONST_VAR>(p, e, so.Sp, so.vp, o);
            if (io.rew) io.rew[koff + i] = (float)so.reward;
            if (io.term) io.term[koff + i] = term ? 1 : 0;
        }
        // wave-level done mask: waves without a terminating env skip the reset path
        if (p.autoreset && __ballot(term) != 0ull) {
            if (term) {
                if (io.tobs) {
#pragma unroll
                    for (int c = 0; c < kObs; ++c) io.tobs[i * kObs + c] = o[c];
                }
                reset_env<MODE>(p, s, i, e);
                make_obs<CONST_VAR>(p, e, e.S, e.v, o);
                reset_any = true;
            }
        }
        if (io.obs) {
#pragma unroll
            for (int c = 0; c < kObs; ++c) tile[threadIdx.x * kObs + c] = o[c];
            __syncthreads();
            flush_obs_tile(tile, io.obs + koff * kObs, row0, rows);
            __syncthreads();
        }
    }
    if (live) {
        store_env<MODE>(s, i, e, reset_any);
        if (io.trunc) io.trunc[i] = 0;
    }
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void reset_kernel(Params p, State s, const int64_t* ids,
                                                       int64_t count, float* obs) {
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= count) return;
    const int64_t i = ids ? ids[j] : j;
    if (i < 0 || i >= p.n) return;
    Env e;
    load_env<MODE>(p, s, i, e);
    reset_env<MODE>(p, s, i, e);
    store_env<MODE>(s, i, e, true);
    if (obs) {
        float o[kObs];
        make_obs<MODE == HE_MODE_GBM>(p, e, e.S, e.v, o);
#pragma unroll
        for (int c = 0; c < kObs; ++c) obs[i * kObs + c] = o[c];
    }
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
    std::string err;
    void* state_mem = nullptr;
    size_t state_bytes = 0;
    float4* rec = nullptr;
    int64_t n_paths = 0;
    bool seeded = false;
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

static void fill_params(he_env* env) {
    const he_config& c = env->cfg;
    Params& p = env->p;
    memset(&p, 0, sizeof(p));
    p.n = c.n_envs;
    p.goff = c.global_env_offset;
    p.variant = c.variant;
    p.loss = c.loss_type;
    p.record_metrics = c.record_metrics ? 1 : 0;
    p.autoreset = c.autoreset ? 1 : 0;
    p.mode = c.mode;
    p.mt = c.max_trade_per_step;
    p.maxh = c.max_contracts_held_per_type;
    p.mt_f = (float)c.max_trade_per_step;
    p.init_cash_f = (float)c.initial_cash;
    p.tcpc = c.transaction_cost_per_contract;
    p.slip_frac = c.slippage_bps / 10000.0;
    p.lam = c.lambda_cost;
    p.w = c.pnl_penalty_weight;
    p.theta = c.theta_weight;
    p.initial_cash = c.initial_cash;
    p.shares_d = (double)c.shares_to_hedge;
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
    p.bs.disc = exp(-r * T);
    // hedging_env_v2.py:84,95-99 for a constant f32 variance (numpy scalar powf)
    float vf = (float)c.variance;
    float vmax = (vf != vf) ? vf : (vf > 1e-8f ? vf : 1e-8f);
    p.g_sigma = sqrtf(vmax);
    p.g_num_drift = ((float)r + 0.5f * powf(p.g_sigma, 2.0f)) * (float)T;
    p.g_sst = (double)p.g_sigma * sqrt(T);
    p.h_kappa = c.heston_kappa;
    p.h_theta = c.heston_theta;
    p.h_xi = c.heston_xi;
    p.h_rho = c.heston_rho;
    double omr = 1.0 - c.heston_rho * c.heston_rho;
    p.h_sqrt1mrho2 = sqrt(omr < 0.0 ? 0.0 : omr);
    p.T = c.episode_length;
    p.rec = env->rec;
    p.n_paths = env->n_paths;
}

template <int MODE>
static void launch_reset(he_env* env, const int64_t* ids, int64_t count, float* obs, hipStream_t st) {
    int64_t blocks = (count + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(reset_kernel<MODE>, dim3((unsigned)blocks), dim3(kBlock), 0, st, env->p, env->s,
                       ids, count, obs);
}

template <int MODE>
static void launch_step(he_env* env, const Io& io, bool info, int k, hipStream_t st) {
    int64_t blocks = (env->cfg.n_envs + kBlock - 1) / kBlock;
    if (info)
        hipLaunchKernelGGL((step_kernel<MODE, true>), dim3((unsigned)blocks), dim3(kBlock), 0, st, env->p,
                           env->s, io, k);
    else
        hipLaunchKernelGGL((step_kernel<MODE, false>), dim3((unsigned)blocks), dim3(kBlock), 0, st, env->p,
                           env->s, io, k);
}

static he_status launch_any(he_env* env, const Io& io, bool info, int k, void* stream) {
    const he_config& c = env->cfg;
    if (c.mode == HE_MODE_REPLAY && !env->rec) return fail(env, HE_ESTATE, "no paths loaded (he_load_paths)");
    DeviceGuard dg(c.device);
    hipStream_t st = (hipStream_t)stream;
    if (c.mode == HE_MODE_REPLAY) launch_step<HE_MODE_REPLAY>(env, io, info, k, st);
    else if (c.mode == HE_MODE_GBM) launch_step<HE_MODE_GBM>(env, io, info, k, st);
    else launch_step<HE_MODE_HESTON>(env, io, info, k, st);
    HE_HIP(env, hipGetLastError());
    return HE_OK;
}

extern "C" {

const char* he_version(void) { return "libhedgeenv 0.1 (gfx950)"; }

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
    return HE_OK;
}

he_status he_create(const he_config* cfg, he_env** out) {
    if (!cfg || !out) return HE_EINVAL;
    *out = nullptr;
    he_env* env = new (std::nothrow) he_env();
    if (!env) return HE_ENOMEM;
    env->cfg = *cfg;
    const he_config& c = env->cfg;
    he_status st = HE_OK;
    if (c.abi_version != HE_ABI_VERSION) st = fail(env, HE_EINVAL, "abi_version %d != %d", c.abi_version, HE_ABI_VERSION);
    else if (c.variant != 1 && c.variant != 2) st = fail(env, HE_EINVAL, "variant must be 1 or 2");
    else if (c.mode < 0 || c.mode > 2) st = fail(env, HE_EINVAL, "bad mode %d", c.mode);
    else if (c.loss_type < 0 || c.loss_type > 3) st = fail(env, HE_EINVAL, "bad loss_type %d", c.loss_type);
    else if (c.n_envs < 1 || c.n_envs > (int64_t)1 << 31) st = fail(env, HE_EINVAL, "n_envs out of range");
    else if (c.global_env_offset < 0) st = fail(env, HE_EINVAL, "global_env_offset < 0");
    else if (c.max_contracts_held_per_type < 0 || c.max_contracts_held_per_type > 32767)
        st = fail(env, HE_EINVAL, "max_contracts_held_per_type must be in [0, 32767]");
    else if (c.max_trade_per_step < 0 || c.max_trade_per_step > 32767)
        st = fail(env, HE_EINVAL, "max_trade_per_step must be in [0, 32767]");
    else if (c.mode != HE_MODE_REPLAY && (c.episode_length < 1 || c.episode_length > (1 << 30)))
        st = fail(env, HE_EINVAL, "episode_length must be >= 1");
    if (st != HE_OK) {
        *out = env;  // keep the handle so the caller can read the message
        return st;
    }
    DeviceGuard dg(c.device);
    if (!dg.ok) {
        *out = env;
        return fail(env, HE_EHIP, "hipSetDevice(%d) failed", c.device);
    }
    const int64_t N = c.n_envs;
    // carve one allocation: 256-B aligned SoA fields
    struct F { size_t bytes; void** dst; };
    std::vector<F> fs;
    fs.push_back({(size_t)N * 4, (void**)&env->s.t});
    fs.push_back({(size_t)N * 4, (void**)&env->s.pos});
    fs.push_back({(size_t)N * 8, (void**)&env->s.cash});
    if (c.mode == HE_MODE_REPLAY) {
        fs.push_back({(size_t)N * 4, (void**)&env->s.path});
        fs.push_back({(size_t)N * 4, (void**)&env->s.s0});
        fs.push_back({(size_t)N * 32, (void**)&env->s.pcg});
        fs.push_back({(size_t)N * 8, (void**)&env->s.pcgb});
    } else {
        fs.push_back({(size_t)N * 8, (void**)&env->s.S});
        fs.push_back({(size_t)N * 4, (void**)&env->s.C});
        fs.push_back({(size_t)N * 4, (void**)&env->s.P});
        fs.push_back({(size_t)N * 4, (void**)&env->s.ep});
        if (c.mode == HE_MODE_HESTON) fs.push_back({(size_t)N * 8, (void**)&env->s.var});
    }
    size_t total = 0;
    for (auto& f : fs) total += (f.bytes + 255) & ~(size_t)255;
    void* mem = nullptr;
    hipError_t e = hipMalloc(&mem, total);
    if (e != hipSuccess) {
        *out = env;
        return fail(env, HE_ENOMEM, "hipMalloc(%zu) failed: %s", total, hipGetErrorString(e));
    }
    env->state_mem = mem;
    env->state_bytes = total;
    size_t off = 0;
    for (auto& f : fs) {
        *f.dst = (char*)mem + off;
        env->fields.push_back({f.bytes, *f.dst});
        off += (f.bytes + 255) & ~(size_t)255;
    }
    e = hipMemset(mem, 0, total);
    if (e != hipSuccess) {
        *out = env;
        return fail(env, HE_EHIP, "hipMemset failed: %s", hipGetErrorString(e));
    }
    fill_params(env);
    *out = env;
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
    std::vector<float4> rec;
    try {
        rec.resize((size_t)(n_paths * n_cols));
    } catch (...) {
        return fail(env, HE_ENOMEM, "host allocation of %lld records failed", (long long)(n_paths * n_cols));
    }
    for (int64_t q = 0; q < n_paths; ++q) {
        for (int64_t t = 0; t <= T; ++t) {
            int64_t tc = t < T ? t : T - 1;  // terminal step keeps the last marks (:229-231)
            float4 r;
            r.x = S[q * n_cols + t];
            r.y = v[q * n_cols + t];
            r.z = C[q * T + tc];
            r.w = P[q * T + tc];
            rec[(size_t)(q * n_cols + t)] = r;
        }
    }
    float4* d = nullptr;
    hipError_t e = hipMalloc(&d, rec.size() * sizeof(float4));
    if (e != hipSuccess) return fail(env, HE_ENOMEM, "hipMalloc(paths) failed: %s", hipGetErrorString(e));
    e = hipMemcpy(d, rec.data(), rec.size() * sizeof(float4), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(d);
        return fail(env, HE_EHIP, "hipMemcpy(paths) failed: %s", hipGetErrorString(e));
    }
    if (env->rec) (void)hipFree(env->rec);
    env->rec = d;
    env->n_paths = n_paths;
    env->cfg.episode_length = (int32_t)T;
    fill_params(env);
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

he_status he_seed(he_env* env, const int64_t* env_ids, const uint64_t* seeds, int64_t count) {
    if (!env) return HE_EINVAL;
    if (!seeds || count < 1) return fail(env, HE_EINVAL, "he_seed needs >= 1 seed");
    DeviceGuard dg(env->cfg.device);
    const int64_t N = env->cfg.n_envs;
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
        env->cfg.seed = seeds[0];
        fill_params(env);
        // episode counters restart: 0xFFFFFFFF so that the next reset starts episode 0
        HE_HIP(env, hipMemset(env->s.ep, 0xFF, (size_t)N * 4));
    }
    env->seeded = true;
    return HE_OK;
}

he_status he_reset(he_env* env, const int64_t* env_ids, int64_t count, float* obs_out, void* stream) {
    if (!env) return HE_EINVAL;
    const he_config& c = env->cfg;
    if (c.mode == HE_MODE_REPLAY && !env->rec) return fail(env, HE_ESTATE, "no paths loaded (he_load_paths)");
    if (!env_ids) count = c.n_envs;
    if (count < 0) return fail(env, HE_EINVAL, "count < 0");
    if (count == 0) return HE_OK;
    DeviceGuard dg(c.device);
    hipStream_t st = (hipStream_t)stream;
    if (c.mode == HE_MODE_REPLAY) launch_reset<HE_MODE_REPLAY>(env, env_ids, count, obs_out, st);
    else if (c.mode == HE_MODE_GBM) launch_reset<HE_MODE_GBM>(env, env_ids, count, obs_out, st);
    else launch_reset<HE_MODE_HESTON>(env, env_ids, count, obs_out, st);
    HE_HIP(env, hipGetLastError());
    return HE_OK;
}

he_status he_step(he_env* env, const float* actions, float* obs, float* reward, uint8_t* terminated,
                  uint8_t* truncated, float* terminal_obs, const he_info* info, void* stream) {
    if (!env) return HE_EINVAL;
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
    return launch_any(env, io, want_info, 1, stream);
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
    return launch_any(env, io, false, k_steps, stream);
}

int64_t he_num_envs(const he_env* env) { return env ? env->cfg.n_envs : -1; }
int32_t he_episode_length(const he_env* env) { return env ? env->cfg.episode_length : -1; }
int64_t he_num_episodes(const he_env* env) { return env ? env->n_paths : -1; }

he_status he_get_config(const he_env* env, he_config* out) {
    if (!env || !out) return HE_EINVAL;
    *out = env->cfg;
    return HE_OK;
}

size_t he_state_size(const he_env* env) {
    if (!env) return 0;
    size_t n = 0;
    for (auto& f : env->fields) n += f.first;
    return n;
}

he_status he_get_state(he_env* env, void* host_buf, size_t size) {
    if (!env || !host_buf) return HE_EINVAL;
    if (size != he_state_size(env)) return fail(env, HE_EINVAL, "state buffer size %zu != %zu", size, he_state_size(env));
    DeviceGuard dg(env->cfg.device);
    HE_HIP(env, hipDeviceSynchronize());
    char* dst = (char*)host_buf;
    for (auto& f : env->fields) {
        HE_HIP(env, hipMemcpy(dst, f.second, f.first, hipMemcpyDeviceToHost));
        dst += f.first;
    }
    return HE_OK;
}

he_status he_set_state(he_env* env, const void* host_buf, size_t size) {
    if (!env || !host_buf) return HE_EINVAL;
    if (size != he_state_size(env)) return fail(env, HE_EINVAL, "state buffer size %zu != %zu", size, he_state_size(env));
    DeviceGuard dg(env->cfg.device);
    HE_HIP(env, hipDeviceSynchronize());
    const char* src = (const char*)host_buf;
    for (auto& f : env->fields) {
        HE_HIP(env, hipMemcpy(f.second, src, f.first, hipMemcpyHostToDevice));
        src += f.first;
    }
    return HE_OK;
}

}  // extern "C"
