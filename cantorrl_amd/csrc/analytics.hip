// analytics.hip -- offline path analytics of the reference as one-pass HIP scans (part
// of libhedgeenv; C ABI in include/hedge_env.h).
//
//   he_fixed_european_marks  src/sim/option_price_assignment.py:10-52
//       (calculate_annualized_vol_matrix + black_scholes_vectorized over every column)
//   he_bs_delta_hedge        src/tools/bs_delta.py:11-55 (bs_delta_hedge)
//
// Both take the expanding-window realized volatility std(log returns[:t], ddof=1) *
// sqrt(252) at every column t.  The reference recomputes it from scratch per column,
// O(T^2) per path; here one thread per path carries a running (Welford) mean / M2 of
// the log returns, O(T).  The arithmetic per column follows the reference's operation
// order in f64 (ndtr as scipy's cephes, he_math.h).  Rows are read and written in
// order by their own thread: each 128-B line serves 16 consecutive columns from L2.

#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include "../../include/hedge_env.h"
#include "he_math.h"

namespace {

constexpr int kAnThreads = 256;

// python max(x, 0.0): the first argument unless the second is larger (NaN stays)
__device__ __forceinline__ double py_max0(double x) { return (0.0 > x) ? 0.0 : x; }

struct Welford {
    double mean = 0.0, m2 = 0.0;
    __device__ __forceinline__ void add(double x, double k) {   // k = count after adding x
        const double d = x - mean;
        mean += d / k;
        m2 += d * (x - mean);
    }
};

__global__ void __launch_bounds__(kAnThreads) euro_marks_kernel(const double* __restrict__ P, int64_t n, int T1,
                                                                 double r, double* __restrict__ vols,
                                                                 double* __restrict__ calls,
                                                                 double* __restrict__ puts) {
    const int64_t i = (int64_t)blockIdx.x * kAnThreads + threadIdx.x;
    if (i >= n) return;
    const double* row = P + i * T1;
    const double S0 = row[0];
    const double K = rint(S0);                 // np.round(paths[:, 0]) (:36)
    const double sqrt252 = sqrt(252.0);        // math.sqrt(252) (:30)
    Welford w;
    double Sprev = S0;
    for (int t = 0; t < T1; ++t) {
        const double S = row[t];
        double sig = 0.0;                      // vols[:, 0] stays 0 (:25)
        if (t >= 1) {
            w.add(log(S / Sprev), (double)t);  // np.log(slice[:, 1:] / slice[:, :-1]) (:28)
            // np.std(ddof=1): sqrt(M2 / (t - 1)); one return gives 0 / 0 = NaN (:29)
            sig = (t >= 2) ? sqrt(w.m2 / (double)(t - 1)) * sqrt252 : NAN;
        }
        Sprev = S;
        if (vols) vols[i * T1 + t] = sig;
        const double T = fmax(1.0 - (double)t / 252.0, 0.0);    // np.clip(1 - t/252, 0, None) (:38)
        double c, p;
        he::bs_vectorized(S, K, T, r, sig, &c, &p);               // black_scholes_vectorized (:10-21)
        calls[i * T1 + t] = c;
        puts[i * T1 + t] = p;
    }
}

__global__ void __launch_bounds__(kAnThreads) bs_hedge_kernel(const double* __restrict__ P, int64_t n, int T1,
                                                               double r, double dt, double* __restrict__ pnl) {
    const int64_t i = (int64_t)blockIdx.x * kAnThreads + threadIdx.x;
    if (i >= n) return;
    const double* row = P + i * T1;
    const double K = row[0];                                   // :42
    const double Ttot = (double)T1 * dt;                       // :38
    const double sqrt252 = sqrt(252.0);
    Welford w;
    double cash = 0.0, prev = 0.0, Sprev = K;
    for (int t = 0; t < T1; ++t) {
        const double S = row[t];
        // calculate_annualized_vol(prices[:t+1]) (:26-34): 0 for < 2 prices or < 2 returns
        double sig = 0.0;
        if (t >= 1) {
            w.add(log(S / Sprev), (double)t);
            if (t >= 2) sig = sqrt(w.m2 / (double)(t - 1)) * sqrt252;
        }
        Sprev = S;
        const double Tr = py_max0(Ttot - (double)t * dt);      // max(T_total - t * DT, 0.0) (:47)
        const bool flat = (sig < 1e-8) || (Tr <= 0.0);
        double d1 = 0.0, sqT = 0.0;
        if (!flat) {
            sqT = sqrt(Tr);
            d1 = (log(S / K) + (r + 0.5 * (sig * sig)) * Tr) / (sig * sqT);
        }
        const double delta = flat ? ((S > K) ? 1.0 : 0.0) : he::ndtr(d1);   // black_scholes_delta (:20-24)
        const double dd = delta - prev;
        cash -= dd * S;
        prev = delta;
        double call;                                             // black_scholes_price (:11-18)
        if (flat) call = py_max0(S - K * exp(-r * Tr));
        else call = S * he::ndtr(d1) - K * exp(-r * Tr) * he::ndtr(d1 - sig * sqT);
        pnl[i * T1 + t] = cash + prev * S - call;
    }
}

}  // namespace

extern "C" {

he_status he_fixed_european_marks(const double* paths, int64_t n_paths, int32_t n_cols, double r, double* vols,
                                  double* calls, double* puts, void* stream) {
    if (n_paths < 0 || n_cols < 1) return HE_EINVAL;
    if (n_paths == 0) return HE_OK;
    if (!paths || !calls || !puts) return HE_EINVAL;
    hipLaunchKernelGGL(euro_marks_kernel, dim3((unsigned)((n_paths + kAnThreads - 1) / kAnThreads)),
                       dim3(kAnThreads), 0, (hipStream_t)stream, paths, n_paths, (int)n_cols, r, vols, calls, puts);
    return hipGetLastError() == hipSuccess ? HE_OK : HE_EHIP;
}

he_status he_bs_delta_hedge(const double* paths, int64_t n_paths, int32_t n_cols, double r, double dt, double* pnl,
                            void* stream) {
    if (n_paths < 0 || n_cols < 1 || !(dt > 0.0)) return HE_EINVAL;
    if (n_paths == 0) return HE_OK;
    if (!paths || !pnl) return HE_EINVAL;
    hipLaunchKernelGGL(bs_hedge_kernel, dim3((unsigned)((n_paths + kAnThreads - 1) / kAnThreads)), dim3(kAnThreads),
                       0, (hipStream_t)stream, paths, n_paths, (int)n_cols, r, dt, pnl);
    return hipGetLastError() == hipSuccess ? HE_OK : HE_EHIP;
}

}  // extern "C"
