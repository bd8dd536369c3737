/* rbergomi.h -- C ABI of librbergomi, the MI355X rough-Bergomi path and option-mark
 * generator (offline data for the env's replay mode).
 *
 * Replaces, in the reference (/root/reference/src/sim/rbergomi_sim.py):
 *   rb_estimate_base_params   estimate_base_params                  :174-195
 *   rb_estimate_parts         estimate_xi / estimate_H / estimate_eta / estimate_rho
 *                                                                   :63-171
 *   rb_sample_params          per-path perturbations                :379-383
 *   rb_simulate_paths         rbergomi_lambda / rbergomi_phi / fractional_gaussian /
 *                             forward_variance + the price advance  :224-258, :385-400,
 *                                                                   :454-464
 *   rb_price_options          price_rbergomi_option_gpu             :261-306
 *   rb_price_atm_marks        the per-day rolling-ATM pricing loop  :404-451
 *   rb_generate               generate_paths_and_options            :309-499
 * The NPZ wire format (:528) is written by cantorrl_amd/rbergomi.py.
 *
 * Normals.  The reference draws complex Z ~ N(0,1) + i N(0,1) per path and takes
 * W = ifft(Z) sqrt(M); its price increments are (Re W, Im W) and its fractional
 * process is Re ifft(phi Z) = (lam (*) Re W) / sqrt(M), a circular convolution with
 * lam_k = t_k^(2H) / 2.  W is itself i.i.d. N(0,1) + i N(0,1) (ifft * sqrt(M) is
 * unitary), so the kernels draw W directly from Philox4x32-10 and convolve -- no
 * FFT.  Every device entry also accepts W (or the unit normals) as an input, which
 * is how the tests feed the reference's own draws through it.
 *
 * Philox counter of a draw: (block, domain << 24 | sub, lo(gid), hi(gid)), key =
 * (lo(seed), hi(seed)); gid = path_offset + path (or option) index, so a shard
 * of paths generated on any GPU equals the same rows of a one-GPU run.
 *   domain 1  parameter perturbations, blocks 0..2 (z0..z5, z5 unused)
 *   domain 2  main-path W_j, block j
 *   domain 3  option MC, block = mc_path * M_opt + b (f64 normals) or
 *             mc_path * M_opt / 2 + b (f32 normals); sub = day * 2 + type
 *
 * Conventions: every pointer passed to a device entry is device memory; calls are
 * stream-ordered and asynchronous (no host sync inside); arrays are row-major f64.
 * Errors are status codes, with a message from rb_last_error() (thread-local).
 */
#ifndef CANTORRL_RBERGOMI_H
#define CANTORRL_RBERGOMI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RB_ABI_VERSION 1

typedef enum rb_status {
    RB_OK = 0,
    RB_EINVAL = 1,   /* bad argument / config */
    RB_EHIP = 3,     /* HIP runtime error */
} rb_status;

typedef enum rb_option_type { RB_CALL = 0, RB_PUT = 1 } rb_option_type;

/* Normals of the MC option pricer: f64 Box-Muller on 53-bit uniforms (the
 * reference's precision) or f32 Box-Muller on 32-bit uniforms (4 normals per
 * Philox block; tails truncated at 6.66 sigma). */
typedef enum rb_normals { RB_NORMALS_F64 = 0, RB_NORMALS_F32 = 1 } rb_normals;

typedef struct rb_base_params {
    double S0, xi, H, eta, rho;
} rb_base_params;

typedef struct rb_config {
    int32_t abi_version;      /* RB_ABI_VERSION */
    int32_t n_steps;          /* N_STEPS (:15), 1..1023 */
    int64_t n_paths;          /* paths of this call (a shard of the whole set) */
    int64_t path_offset;      /* global id of path 0 */
    uint64_t seed;            /* SEED (:17) */
    double r;                 /* R (:13) */
    double dt;                /* DT (:14) */
    double option_tenor;      /* T_OPTION_TENOR (:19); int(tenor / dt) + 1 <= 64 */
    int32_t n_mc;             /* N_PATHS_OPTION_MC (:20) */
    int32_t normals;          /* rb_normals, MC pricer only */
    double perturb_std[5];    /* PERTURB_{S0,XI,H,ETA,RHO}_STD (:29-33) */
    double min_xi_factor;     /* MIN_XI_FACTOR (:35) */
    double min_eta_factor;    /* MIN_ETA_FACTOR (:36) */
    double clip_h_min, clip_h_max;       /* :37-38 */
    double clip_rho_min, clip_rho_max;   /* :39-40 */
    int32_t reserved_i[4];
    double reserved[4];
} rb_config;

const char* rb_version(void);
const char* rb_last_error(void);

/* Defaults of rbergomi_sim.py:13-40 (n_paths = N_PATHS = 100000). */
int32_t rb_config_init(rb_config* cfg, int32_t abi_version);

/* Host.  estimate_base_params(prices, dt) (:174-195), with every fallback. */
int32_t rb_estimate_base_params(const double* prices, int64_t n, double dt, rb_base_params* out);

/* Host.  From the log returns of prices: out = {estimate_xi(r, dt) (:63-65),
 * estimate_H(r) (:82-133), estimate_eta(r) (:135-153), estimate_rho(r) (:155-171)}
 * before the defaults of :190-193 (NaN where the reference would return NaN). */
int32_t rb_estimate_parts(const double* prices, int64_t n, double dt, double out[4]);

/* params [5][n_paths] = rows S0, xi, H, eta, rho (:379-383).  unit_normals
 * [5][n_paths] (N(0,1); row k is scaled by perturb_std[k]) or NULL for Philox. */
int32_t rb_sample_params(const rb_config* cfg, const rb_base_params* base, const double* unit_normals,
                         double* params, void* stream);

/* paths, vol [n_paths][n_steps + 1] from params [5][n_paths] and W
 * [n_paths][M][2] (M = next_pow2(n_steps + 1); (Re, Im) pairs) or NULL for Philox. */
int32_t rb_simulate_paths(const rb_config* cfg, const double* params, const double* W, double* paths,
                          double* vol, void* stream);

/* price[i] = price_rbergomi_option_gpu of option i (type rb_option_type) with
 * cfg->option_tenor, cfg->n_mc MC paths; W [n_options][n_mc][M_opt][2] or NULL
 * (Philox, gid = path_offset + i, sub = type). */
int32_t rb_price_options(const rb_config* cfg, int64_t n_options, int32_t type, const double* S0,
                         const double* K, const double* xi, const double* H, const double* eta,
                         const double* rho, const double* W, double* price, void* stream);

/* call, put [n_paths][n_steps]: day d (0-based) = the option struck at
 * K = rint(paths[p][d]) with xi = vol[p][d] and the path's H, eta, rho (:404-451). */
int32_t rb_price_atm_marks(const rb_config* cfg, const double* params, const double* paths,
                           const double* vol, double* call, double* put, void* stream);

/* rb_sample_params -> rb_simulate_paths -> rb_price_atm_marks (Philox throughout).
 * params [5][n_paths] is caller-owned scratch and an output. */
int32_t rb_generate(const rb_config* cfg, const rb_base_params* base, double* params, double* paths,
                    double* vol, double* call, double* put, void* stream);

/* Host helper for tests: n Philox f64 normals of (seed, domain, sub, gid) blocks
 * [block0, block0 + n/2), as the device draws them. */
int32_t rb_host_normals(uint64_t seed, int32_t domain, uint32_t sub, uint64_t gid, uint32_t block0,
                        int64_t n, double* out);

/* Test hook: the MC pricer's f64 Box-Muller pair (mc_kernel's normals) on n caller-given
 * uniform pairs in (0, 1), device pointers, stream-ordered. */
int32_t rb_device_mc_box_muller(const double* u1, const double* u2, int64_t n, double* z1, double* z2,
                                void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CANTORRL_RBERGOMI_H */
