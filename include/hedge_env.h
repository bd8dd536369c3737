/*
 * hedge_env.h -- C ABI of libhedgeenv: a batched, device-resident dynamic-hedging
 * environment for MI355X (gfx950).  Drop-in replacement for the per-env
 * `HedgingEnv` of bcosm/CantorRL (src/env/hedging_env_v2.py, v1 hedging_env.py)
 * run N-at-a-time inside HIP kernels.
 *
 * Conventions
 *   - Plain C types only.  Every entry point returns an he_status; the message of
 *     the last failure on a handle is he_last_error(handle).  No C++ exception
 *     crosses this boundary.
 *   - The CALLER owns every I/O buffer passed to he_reset/he_step/he_rollout;
 *     those are DEVICE pointers on the handle's device (e.g. torch data_ptr()).
 *     The LIBRARY owns the per-env state (SoA, HBM-resident) and RNG streams.
 *   - `stream` is an opaque hipStream_t (NULL = the legacy default stream).
 *     he_reset/he_step/he_rollout only enqueue work: no host synchronisation,
 *     no allocation, so they can be captured into a hipGraph.
 *   - One handle must be driven from one host thread at a time.  Distinct
 *     handles (also on distinct devices) are independent.
 *
 * Reference interface each entry point replaces (file:line in /root/reference):
 *   he_config_init  <- HedgingEnv.__init__ keyword defaults   hedging_env_v2.py:10-22 (v1 hedging_env.py:10-20)
 *   he_create       <- HedgingEnv.__init__                    hedging_env_v2.py:10-77
 *   he_load_paths   <- np.load(...).astype(float32) + shape check  hedging_env_v2.py:36-51
 *   he_seed         <- reset(seed=...) re-seeding: gymnasium seeding.np_random
 *                      (Generator(PCG64(SeedSequence(seed))))  hedging_env_v2.py:146-148
 *   he_reset        <- HedgingEnv.reset                       hedging_env_v2.py:145-173
 *   he_step         <- HedgingEnv.step (+ SB3 VecEnv auto-reset, train_ppo_v2.py:127-141)
 *                                                             hedging_env_v2.py:175-294
 *   he_rollout      <- SB3 collect_rollouts' inner loop over VecEnv.step for n_steps
 *                      (train_ppo_v2.py:48,222-230) with actions supplied up front
 *   he_rollout_policy <- evaluate_baseline_policy(policy_no_hedge / policy_delta_every_step)
 *                      (src/agents/baselines.py:32-103) and run_benchmark_strategy(
 *                      delta_hedging_action_selector) (src/benchmark/delta_and_nothing.py:33-163):
 *                      the policy evaluated on the device from each step's obs, fused
 *                      into the rollout kernel (the LDS kernels' steppers, or the tile
 *                      step kernel), with per-episode sums recorded on device
 *   he_get_state / he_set_state  <- env pickling by SubprocVecEnv / checkpoints (no
 *                      reference equivalent; state is otherwise lost across processes)
 */
#ifndef HEDGE_ENV_H
#define HEDGE_ENV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HE_ABI_VERSION 4   /* 4: he_vecnorm_step/apply take Monitor's f64 rewards */
#define HE_BOOK_MAX 8
#define HE_OBS_DIM 13
#define HE_ACT_DIM 2

typedef enum he_status {
    HE_OK = 0,
    HE_EINVAL = 1,   /* bad argument / config value            */
    HE_ESHAPE = 2,   /* inconsistent table shapes (ValueError)  */
    HE_EHIP = 3,     /* HIP runtime failure                     */
    HE_ENOMEM = 4,   /* device allocation failed                */
    HE_ESTATE = 5    /* call not valid in the current state     */
} he_status;

typedef enum he_mode {
    HE_MODE_REPLAY = 0,  /* replay NPZ paths (reference semantics)           */
    HE_MODE_GBM = 1,     /* generate: GBM + Philox, BS rolling-ATM marks       */
    HE_MODE_HESTON = 2   /* generate: Heston full-truncation Euler (extension) */
} he_mode;

/* How generate modes mark the two hedge instruments C, P at env step t (replay reads
 * them from the table).  Both keep the env's terminal-step lag (hedging_env_v2.py:229-231). */
typedef enum he_mark {
    HE_MARK_ROLLING_ATM = 0,    /* 30-day call/put struck at K = round(S_t), re-struck every step:
                                   the reference generator's marks (rbergomi_sim.py:418,437-446),
                                   option_calculator.py:11-27 form                               */
    HE_MARK_FIXED_EUROPEAN = 1  /* one call/put per episode struck at K = round(S_0), expiring
                                   one year after the episode start: T = max(1 - t/252, 0),
                                   black_scholes_vectorized (option_price_assignment.py:10-21,
                                   33-49) at the market's volatility (GBM: sqrt(variance);
                                   Heston: sqrt(max(v_t, 0)))                                   */
} he_mark;

typedef enum he_loss {
    HE_LOSS_MSE = 0,
    HE_LOSS_ABS = 1,
    HE_LOSS_CVAR = 2,    /* identical to ABS inside the env (hedging_env_v2.py:250-253) */
    HE_LOSS_OTHER = 3    /* any other string: |x| branch (:252-253)                    */
} he_loss;

/* Liability book (extension, generate modes; BASELINE.json configs[3]/[4]): options
 * every env carries besides the hedged shares.  The book is marked at every step
 * from the env's own market (S_t, v_t, t) and enters the portfolio value
 * (hedging_env_v2.py:233-236): PV = shares*S + options + cash + sum_k q_k*100*V_k. */
typedef enum he_book_type {
    HE_BOOK_CALL = 0,      /* European call, Black-Scholes (option_calculator.py:11-27 form) */
    HE_BOOK_PUT = 1,       /* European put                                                  */
    HE_BOOK_UO_CALL = 2    /* up-and-out call: worthless once S_t >= barrier at a step date;
                              alive: closed-form continuous-barrier price (Hull, q = 0)     */
} he_book_type;

typedef struct he_book_option {
    int32_t type;          /* he_book_type                                                  */
    int32_t expiry;        /* in env steps from the episode start: tau = (expiry - t) * dt  */
    double strike;         /* K                                                             */
    double barrier;        /* H (HE_BOOK_UO_CALL)                                           */
    double quantity;       /* contracts (x100 shares); negative = short, i.e. a liability   */
} he_book_option;

typedef struct he_config {
    int32_t abi_version;        /* = HE_ABI_VERSION                                  */
    int32_t variant;            /* 1: hedging_env.py, 2: hedging_env_v2.py          */
    int32_t mode;               /* he_mode                                           */
    int32_t loss_type;          /* he_loss                                           */
    int64_t n_envs;             /* envs on this handle (>=1)                         */
    int64_t global_env_offset;  /* global id of env 0 (multi-GPU sharding)           */
    /* HedgingEnv ctor keywords (hedging_env_v2.py:10-22) */
    double transaction_cost_per_contract;
    double lambda_cost;
    double pnl_penalty_weight;
    double theta_weight;        /* v2 only                                           */
    double slippage_bps;        /* v2 only                                           */
    double initial_cash;
    int64_t shares_to_hedge;
    int32_t max_contracts_held_per_type;   /* 0..32767                               */
    int32_t max_trade_per_step;            /* 0..32767                               */
    int32_t record_metrics;                /* 0: greeks are zeros (:80-81)           */
    int32_t autoreset;                     /* 1: SB3 VecEnv auto-reset inside step   */
    /* env constants (hedging_env_v2.py:56-58) */
    double risk_free_rate;      /* 0.04                                              */
    double option_tenor_years;  /* 30/252                                            */
    /* generate modes (price advance rbergomi_sim.py:454-464) */
    int32_t episode_length;     /* T (replay: taken from the table)                  */
    int32_t device;             /* HIP device ordinal                                */
    uint64_t seed;              /* Philox key                                        */
    double s0;                  /* initial price                                     */
    double variance;            /* GBM: constant variance v; Heston: v0              */
    double mu;                  /* drift rate of the advance (R = 0.04)              */
    double dt;                  /* 1/252                                             */
    double heston_kappa;
    double heston_theta;
    double heston_xi;
    double heston_rho;
    int32_t market_block;       /* generate modes: steps of market data generated per
                                   market_kernel launch (1..64, default 64)          */
    int32_t market_prefetch;    /* market of block b+1 generated ahead: 0 auto (fused
                                   rollouts, or he_step from 131,072 envs), 1 never,
                                   2 always.  he_rollout without a book generates it in
                                   the step grid on `stream` (step_market_kernel), the
                                   other paths on the side stream                    */
    int32_t book_size;          /* generate modes: options in the liability book (0..8) */
    int32_t mark;               /* generate modes: he_mark (replay: must be ROLLING_ATM) */
    he_book_option book[HE_BOOK_MAX];
    double reserved[7];
} he_config;

/* Optional per-step info outputs (device pointers, each may be NULL).  Field names
 * follow the reference info dict (hedging_env_v2.py:268-293). */
typedef struct he_info {
    double* step_pnl_total;
    double* per_share_step_pnl;
    double* raw_pnl_deviation_abs;
    double* transaction_costs_total;
    double* commission_cost;
    double* slippage_cost;
    double* reward_pnl_component;
    double* transaction_cost_penalty;
    double* theta_penalty;
    double* reward_step;            /* the f64 reward before the f32 cast */
    double* portfolio_value;
    double* cash;
    int32_t* call_contracts;
    int32_t* put_contracts;
    float* scaled_float_call;
    float* scaled_float_put;
    int32_t* requested_calls_rounded_clipped;
    int32_t* requested_puts_rounded_clipped;
    int32_t* actual_calls_traded;
    int32_t* actual_puts_traded;
    float* initial_S0_for_episode;
    /* market view after the step (pre-reset), for callers that read env
     * attributes (src/benchmark/delta_and_nothing.py:71-79) */
    float* current_stock_price;
    float* current_volatility;
    float* current_call_price;
    float* current_put_price;
    int32_t* current_step;
    int32_t* current_episode_idx;   /* replay: path row of the episode; generate: -1 */
} he_info;

typedef struct he_env he_env;

/* Fill *cfg with the reference ctor defaults of `variant` (1 or 2), GBM market
 * defaults (S0=496.48, v=0.029028, mu=0.04, dt=1/252, T=252, seed=42), n_envs=1. */
he_status he_config_init(he_config* cfg, int32_t variant);

he_status he_create(const he_config* cfg, he_env** out);
he_status he_destroy(he_env* env);
const char* he_last_error(const he_env* env);   /* never NULL */
const char* he_version(void);

/* Replay tables, HOST pointers, row-major f32 (the reference casts to f32 on load):
 * S, v: [n_paths][n_cols]; C, P: [n_paths][n_cols-1]; n_cols = episode_length+1. */
he_status he_load_paths(he_env* env, const float* S, const float* v, const float* C,
                        const float* P, int64_t n_paths, int64_t n_cols);

/* Seed per-env episode streams.  Replay: env_ids[i] gets
 * Generator(PCG64(SeedSequence(seeds[i]))) (host pointers; env_ids NULL = envs
 * 0..count-1).  Generate modes: seeds[0] becomes the Philox key of the whole
 * handle and every episode counter restarts. */
he_status he_seed(he_env* env, const int64_t* env_ids, const uint64_t* seeds, int64_t count);

/* Reset envs (env_ids: DEVICE int64 list, NULL = all) and write their obs rows
 * into obs_out[N][13] (device; rows of other envs untouched; may be NULL).  If
 * info is not NULL its position fields (cash, call/put contracts, current_*,
 * initial_S0_for_episode, current_episode_idx) receive the post-reset values. */
he_status he_reset(he_env* env, const int64_t* env_ids, int64_t count, float* obs_out,
                   const he_info* info, void* stream);

/* Replay mode: reset envs to given episode rows -- SURVEY 8(b)'s he_reset(episode_idx):
 * hedging_env_v2.py:145-173 with current_episode_idx taken from the caller instead of the
 * env's np_random.integers(num_episodes), so host-drawn PCG64 indices reproduce the
 * reference's episode choice (the env's own PCG64 stream is not advanced).  episode_idx:
 * HOST int64[count], each in [0, n_paths) (HE_EINVAL otherwise, checked before anything
 * runs); env_ids: DEVICE int64 list as he_reset (NULL = envs 0..count-1).  Synchronises
 * `stream` before staging the indices (a reset-path call, not a step-path one). */
he_status he_reset_episodes(he_env* env, const int64_t* env_ids, const int64_t* episode_idx, int64_t count,
                            float* obs_out, const he_info* info, void* stream);

/* One step of every env.  actions [N][2] f32 in, obs [N][13] f32 out (the reset
 * obs for envs that terminated when autoreset=1), reward [N] f32 (f64 reward cast
 * as SB3 stores it), terminated/truncated [N] u8.  terminal_obs [N][13] receives
 * the pre-reset obs of terminated envs only (NULL = skip).  info may be NULL. */
he_status he_step(he_env* env, const float* actions, float* obs, float* reward,
                  uint8_t* terminated, uint8_t* truncated, float* terminal_obs,
                  const he_info* info, void* stream);

/* k_steps fused steps (autoreset semantics), one launch: actions [K][N][2] in;
 * obs [K][N][13], reward [K][N], terminated [K][N] out (obs/reward/terminated may
 * be NULL to skip).  Per-env state stays in registers across the K steps. */
he_status he_rollout(he_env* env, int32_t k_steps, const float* actions, float* obs,
                     float* reward, uint8_t* terminated, void* stream);

/* Baseline policies evaluated inside the fused step kernel (no action input). */
typedef enum he_policy {
    HE_POLICY_NO_HEDGE = 0,          /* baselines.py:74-75 / delta_and_nothing.py:117-119: [0, 0]      */
    HE_POLICY_DELTA_EVERY_STEP = 1,  /* baselines.py:77-103: trade calls (else puts) to offset the
                                        portfolio delta from obs[3,4,7,9]; f32 as the reference       */
    HE_POLICY_DELTA_THRESHOLD = 2    /* delta_and_nothing.py:122-163: calls for positive, puts for
                                        negative delta needed, skipped under half a call's delta      */
} he_policy;

/* One finished episode of a policy rollout: sums over its steps, in step order, of the
 * f64 reward and info fields the reference evaluation loops accumulate
 * (baselines.py:47-54, delta_and_nothing.py:80-86). */
typedef struct he_episode_record {
    int64_t env_id;          /* global env id                                          */
    int32_t length;          /* steps                                                   */
    int32_t reserved;
    double reward_sum;       /* sum reward                                              */
    double pnl_sum;          /* sum info["step_pnl_total"]                              */
    double abs_pnl_sum;      /* sum info["raw_pnl_deviation_abs"] (|per-share P&L|)     */
    double cost_sum;         /* sum info["transaction_costs_total"]                     */
    double pnl_penalty_sum;  /* sum info["reward_pnl_component"]                        */
    double cost_penalty_sum; /* sum info["transaction_cost_penalty"]                    */
    double per_share_pnl_sum;/* sum info["per_share_step_pnl"] (train_ppo_v2.py:484)    */
    double reserved2;
} he_episode_record;

/* k_steps fused steps with actions from `policy` (he_policy) computed on the device from
 * each env's current obs; autoreset semantics as he_rollout.  actions_out [K][N][2],
 * obs/reward/terminated as he_rollout (each may be NULL).  Every episode that ends
 * appends one he_episode_record at records[atomicAdd(record_count, 1)] while that
 * index is < record_capacity (DEVICE pointers; the caller zeroes *record_count).
 * Episode sums run from the last he_reset of the env and are kept by this entry point
 * and by the generate-mode he_rollout (he_step does not update them). */
he_status he_rollout_policy(he_env* env, int32_t k_steps, int32_t policy, float* actions_out, float* obs,
                            float* reward, uint8_t* terminated, he_episode_record* records,
                            int64_t record_capacity, unsigned long long* record_count, void* stream);

/* Per-env episode summaries, the payload ranks all-gather at rollout boundaries (SURVEY
 * 8(e); Monitor's episode return / length, train_ppo_v2.py:119, and the evaluation sums
 * of :481-514): out[N][4] f32 (DEVICE pointer) = {return, sum of step P&L, sum of
 * transaction costs, length} of each env's most recently finished episode (zeros before
 * the first).  Maintained by he_rollout in generate modes (the LDS path) and by
 * he_rollout_policy; the running sums restart at he_reset.  Stream-ordered; out must be
 * 16-byte aligned (one float4 row per env; HE_EINVAL otherwise). */
he_status he_episode_summaries(he_env* env, float* out, void* stream);

/* Generate modes run market_kernel for block b+1 on a library-owned side stream
 * while the step kernels of block b run on `stream` (he_step, tile-path policy rollouts, books;
 * he_rollout otherwise generates it inside its own grid on `stream`, which needs no
 * join).  he_sync_market makes `stream` wait for a side-stream prefetch: call it
 * before ending a hipGraph capture that contains he_step/he_rollout calls.  No-op in
 * replay mode and when nothing is pending. */
he_status he_sync_market(he_env* env, void* stream);

/* Measurement: the next step_kernel dispatch (he_step / he_rollout) records
 * start_event / stop_event (opaque hipEvent_t) around exactly that dispatch
 * (hipExtLaunchKernelGGL), so hipEventElapsedTime gives the kernel's own duration
 * without the launch gaps.  One-shot; NULL, NULL cancels. */
he_status he_time_next_step(he_env* env, void* start_event, void* stop_event);

/* Host-mapped I/O for small env counts (no reference equivalent: the reference's env is a
 * host object, src/env/hedging_env_v2.py:175-294, stepped from baselines.py:45-51 and through
 * SubprocVecEnv pipes, train_ppo_v2.py:127-141).  he_host_alloc returns `bytes` of zeroed
 * pinned host memory (hipHostMalloc mapped + coherent) and the address a kernel uses for it:
 * he_step's actions / obs / reward / flags / terminal_obs / info pointers may point into it, so a
 * step is one launch and one he_stream_wait, with no DMA in either direction -- the host path of
 * N_ENVS = 2 (train_ppo_v2.py:45) and of the single env.  Free with he_host_free after the last
 * step that used it has completed.  he_stream_wait(stream) = hipStreamSynchronize. */
he_status he_host_alloc(size_t bytes, void** host_ptr, void** device_ptr);
he_status he_host_free(void* host_ptr);
he_status he_stream_wait(void* stream);

/* Step completion signal for the host-mapped path (the same host loops as he_host_alloc).
 * he_step_signal(env, flag) arms the handle's NEXT he_step (one-shot; NULL cancels): `flag` is the
 * DEVICE address of a 4-byte word of he_host_alloc'd memory.  The armed he_step's kernel stores the
 * step's sequence number (he_signal_seq: 1, 2, ... per handle) into the word after every output of
 * the step, with system-scope release ordering, so once the CPU reads that number the step's
 * host-mapped outputs are in place.  he_signal_wait(env, flag_host, stream) waits for the last
 * signalled step by reading the word through its HOST address: a short spin, then (a step queued behind
 * long work) hipStreamSynchronize(stream) and a final check (HE_ESTATE if the flag still differs).
 * It replaces he_stream_wait when that step is the last work on the stream the caller waits for;
 * he_step with VecNormalize attached refuses the signal (HE_EINVAL).  A handle's first
 * he_step_signal allocates the device word that counts the step's workgroups (a device
 * synchronize, once); later calls only arm.  The kernel's end is still
 * reported to the runtime as usual, so later stream-ordered work and events are unaffected. */
he_status he_step_signal(he_env* env, uint32_t* flag);
uint32_t he_signal_seq(const he_env* env);
he_status he_signal_wait(he_env* env, const uint32_t* flag_host, void* stream);

/* Introspection. */
int64_t he_num_envs(const he_env* env);
int32_t he_episode_length(const he_env* env);
int64_t he_num_episodes(const he_env* env);     /* replay table rows; 0 otherwise */
he_status he_get_config(const he_env* env, he_config* out);

/* Checkpointing: opaque blob of the whole per-env state (+ RNG streams). */
size_t he_state_size(const he_env* env);
he_status he_get_state(he_env* env, void* host_buf, size_t size);
he_status he_set_state(he_env* env, const void* host_buf, size_t size);

/* Host reference of the seeding used by he_seed (exported for tests):
 * state[0..3] = {state_hi, state_lo, inc_hi, inc_lo} of PCG64(SeedSequence(seed)). */
he_status he_pcg64_seed_state(uint64_t seed, uint64_t state[4]);

/* Host builds of the device RNG code (same source, he_math.h), for CPU tests:
 * count episode indices Generator(PCG64(SeedSequence(seed))).integers(n_paths),
 * and the 4 Philox4x32-10 words of (seed, global env id, env-step index n). */
he_status he_host_episode_draws(uint64_t seed, uint64_t n_paths, int64_t count, int64_t* out);
he_status he_host_philox(uint64_t seed, uint64_t env_id, uint64_t n, uint32_t out[4]);
/* out[k] = a[k] / b through the reciprocal-multiply division the step kernel uses
 * for its constant divisors (must equal IEEE a[k] / b bit for bit). */
he_status he_host_div_by(const double* a, int64_t count, double b, double* out);
/* The generate-mode Box-Muller pair (he_math.h box_muller) on host arrays, for tests. */
he_status he_host_box_muller(const double* u1, const double* u2, int64_t count, double* z1, double* z2);
/* f32 twin for the obs quotients by per-handle constants (must equal IEEE a[k] / b). */
he_status he_host_div_byf(const float* a, int64_t count, float b, float* out);
/* Device builds of the same RNG for tests (DEVICE pointers, stream-ordered): the 4 Philox
 * words of (seed, env_ids[k], step_index[k]) into words[4k..4k+3] (= rocRAND
 * rocrand_init(seed, env_ids[k], 4 step_index[k]) + rocrand4) and the Box-Muller pair the
 * generate modes draw from them into normals[2k..2k+1]; either output may be NULL. */
he_status he_device_rng(uint64_t seed, const uint64_t* env_ids, const uint64_t* step_index, int64_t count,
                        uint32_t* words, double* normals, void* stream);
/* Generate-mode math on the device (DEVICE pointers) and on the host (HOST pointers), for
 * bit-identity and accuracy tests: op 0 the price-advance exp (he_math.h exp_k), op 2 the
 * rolling-ATM call mark of the default GBM handle at S = x (bs_call_put, K = round(S)),
 * op 4 Box-Muller on (u1, u2) pairs of x; ops 1, 3, 5 the same through the lockstep forms
 * the LDS producers run (exp_k_n, bs_call_put_n, box_muller_n; groups of 4 elements). */
he_status he_device_math(int32_t op, const double* x, int64_t count, double* out, void* stream);
he_status he_host_math(int32_t op, const double* x, int64_t count, double* out);

/* ---- VecNormalize and Monitor on the device ---------------------------------------
 * SB3 2.6.0 VecNormalize (+ RunningMeanStd) as wrapped around the env at
 * train_ppo_v2.py:204,305,450, and Monitor's per-episode return / length (:119),
 * restated from SB3's published algorithm (SB3 is not in this image: parity with
 * it is unpinned; oracle/vecnorm_oracle.py restates it in NumPy).
 *
 * stats: device f64 [2 D + 4] = obs_mean[D], obs_var[D], obs_count, ret_mean, ret_var,
 * ret_count (RunningMeanStd(shape=(D,)) and RunningMeanStd(shape=())).  The batch
 * moments are one-pass f64 sums of shifted values per block, merged in block order
 * (deterministic). */
typedef struct he_vecnorm_params {
    int32_t obs_dim;        /* D; 13 (HE_OBS_DIM) is the one supported */
    int32_t training;       /* update obs_rms / ret_rms / returns */
    int32_t norm_obs;
    int32_t norm_reward;
    double gamma;           /* discount of the running return */
    double clip_obs;        /* 10.0 */
    double clip_reward;     /* 10.0 */
    double epsilon;         /* 1e-8 */
    int32_t reserved[4];
} he_vecnorm_params;

/* Sizes of the device buffers the caller owns. */
int64_t he_vecnorm_stats_len(int32_t obs_dim);                 /* doubles: 2 D + 4 */
int64_t he_vecnorm_scratch_bytes(int64_t n, int32_t obs_dim);

/* RunningMeanStd init: means 0, variances 1, counts 1e-4. */
he_status he_vecnorm_init(double* stats, int32_t obs_dim, void* stream);

/* VecNormalize.step_wait on one batch of n envs (obs [n][D], reward [n] f32, done [n]):
 * obs_rms.update(obs) (training && norm_obs); returns = returns * gamma + reward and
 * ret_rms.update(returns) (training); obs_out = clip((obs - mean) / sqrt(var + eps));
 * reward_out = clip(reward / sqrt(ret_var + eps)) (norm_reward, else a copy);
 * terminal_obs_out[i] normalized for done rows (when both pointers are given);
 * returns[done] = 0.  Monitor (ep_return / ep_length non-NULL): ep_reward [n] f64 -- the
 * env's own f64 step rewards (he_info::reward_step), which SB3's Monitor sums because it wraps
 * each env inside the VecEnv (train_ppo_v2.py:119; hedging_env_v2.py:262,294), not the f32
 * VecEnv buffer -- are summed per env in step order, and a done row copies its episode's
 * sum / length to ep_return_done / ep_length_done and restarts from 0 (ep_reward is then
 * required: HE_EINVAL without it). */
he_status he_vecnorm_step(const he_vecnorm_params* p, int64_t n, const float* obs, const float* reward,
                          const uint8_t* done, const float* terminal_obs, double* returns, double* stats,
                          void* scratch, float* obs_out, float* reward_out, float* terminal_obs_out,
                          double* ep_return, int32_t* ep_length, double* ep_return_done,
                          int32_t* ep_length_done, const double* ep_reward, void* stream);

/* The same step split in two, for n <= 65,536 (one moments partial per he_step
 * workgroup): he_vecnorm_attach(env, p, returns, stats, scratch) arms the NEXT he_step on
 * `env` (one-shot, consumed by that call whatever its status) to also run the first half
 * -- the batch moments of the obs and reward it writes, and returns = returns * gamma +
 * reward -- in its own launch (no effect unless p->training; p = NULL disarms);
 * he_vecnorm_apply, with the arguments of he_vecnorm_step and the same buffers, is then
 * the second half alone: the statistics update and the normalization.  Replaces
 * he_vecnorm_step's moments launch.  Arm right before each he_step whose output the
 * apply consumes: steps nobody armed (the inner env stepped directly, another wrapper's
 * step) leave the buffers alone, and the handle holds no pointer past the armed step. */
he_status he_vecnorm_attach(he_env* env, const he_vecnorm_params* p, double* returns, double* stats, void* scratch);
he_status he_vecnorm_apply(const he_vecnorm_params* p, int64_t n, const float* obs, const float* reward,
                           const uint8_t* done, const float* terminal_obs, double* returns, double* stats,
                           void* scratch, float* obs_out, float* reward_out, float* terminal_obs_out,
                           double* ep_return, int32_t* ep_length, double* ep_return_done,
                           int32_t* ep_length_done, const double* ep_reward, void* stream);

/* Evaluation (VecNormalize(training=False), train_ppo_v2.py:450-453): with the statistics
 * frozen nothing of the step crosses envs, so the NEXT he_step on `env` (one-shot, consumed
 * by that call whatever its status; p = NULL disarms) can do the whole of he_vecnorm_step's
 * work itself -- obs_out, reward_out, terminal_obs_out of done rows, returns[done] = 0, the
 * Monitor sums -- in its own launch: the caller then calls no he_vecnorm_* function for that
 * step.  he_step must get the obs, reward, terminated and terminal_obs buffers; a step that
 * takes another kernel (info requested) runs he_vecnorm_apply itself after it, with
 * info->reward_step as the Monitor sums' f64 rewards (required then when the Monitor buffers
 * are given; the fused launch adds the f64 reward from its registers).  p->training must be 0;
 * out's buffers are he_vecnorm_step's (scratch unused). */
typedef struct he_vecnorm_out {
    const double* stats;
    double* returns;
    float* obs_out;
    float* reward_out;
    float* terminal_obs_out;    /* may be NULL */
    double* ep_return;          /* Monitor sums: all four NULL, or all four given */
    int32_t* ep_length;
    double* ep_return_done;
    int32_t* ep_length_done;
} he_vecnorm_out;
he_status he_vecnorm_attach_eval(he_env* env, const he_vecnorm_params* p, const he_vecnorm_out* out);

/* VecNormalize.reset: returns = 0; obs_rms.update(obs) (training && norm_obs);
 * obs_out normalized (norm_obs, else a copy). */
he_status he_vecnorm_reset(const he_vecnorm_params* p, int64_t n, const float* obs, double* returns,
                           double* stats, void* scratch, float* obs_out, void* stream);

/* ---- Offline analytics over price paths -------------------------------------------
 * paths: device f64 [n_paths][n_cols] (row-major, the NPZ / .npy layout).
 * One thread per path scans the columns once: the expanding-window realized
 * volatility is a running (Welford) mean / M2 of the log returns, so the reference's
 * O(n_cols^2) per path becomes O(n_cols). */

/* src/sim/option_price_assignment.py:10-52: vols[:, t] = std(log returns of
 * paths[:, :t+1], ddof=1) * sqrt(252) (0 at t = 0, NaN at t = 1 as NumPy gives), and
 * the fixed-strike European Black-Scholes marks with K = rint(paths[:, 0]),
 * T = max(1 - t/252, 0), rate r.  vols may be NULL. */
he_status he_fixed_european_marks(const double* paths, int64_t n_paths, int32_t n_cols, double r, double* vols,
                                  double* calls, double* puts, void* stream);

/* src/tools/bs_delta.py:36-55: a daily Black-Scholes delta hedge of a call struck at
 * paths[:, 0] expiring at n_cols * dt, with the realized volatility of the path so far;
 * pnl[:, t] = cash + delta * S - call after the rebalance at t. */
he_status he_bs_delta_hedge(const double* paths, int64_t n_paths, int32_t n_cols, double r, double dt, double* pnl,
                            void* stream);

/* Failure detection (the reference's src/agents/test_inf.py checks rewards
 * for infinities by hand): *count += number of non-finite values among n f32 values
 * of a (obs rows, rewards, ...), one wave-level reduction and one atomic per wave.
 * Stream-ordered; read *count when convenient. */
he_status he_count_nonfinite(const float* a, int64_t n, unsigned long long* count, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HEDGE_ENV_H */
