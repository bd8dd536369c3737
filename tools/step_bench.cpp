// A/B harness for libhedgeenv builds: graph-mode he_step throughput at a fixed env
// count, one line per library given on the command line (built with different
// -D flags by tools/step_ab.sh).  Same protocol as bench.py's graph mode: one
// eager market block, he_sync_market, then graphs of 64 he_step launches.
//
//   step_bench N lib1.so [lib2.so ...]
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "../include/hedge_env.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

struct Api {
    decltype(&he_config_init) config_init;
    decltype(&he_create) create;
    decltype(&he_destroy) destroy;
    decltype(&he_reset) reset;
    decltype(&he_step) step;
    decltype(&he_rollout) rollout;
    decltype(&he_sync_market) sync_market;
    decltype(&he_last_error) last_error;
    void* handle;
};

static Api load(const char* path) {
    void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) { fprintf(stderr, "dlopen %s: %s\n", path, dlerror()); exit(1); }
    Api a;
    a.handle = h;
    a.config_init = (decltype(a.config_init))dlsym(h, "he_config_init");
    a.create = (decltype(a.create))dlsym(h, "he_create");
    a.destroy = (decltype(a.destroy))dlsym(h, "he_destroy");
    a.reset = (decltype(a.reset))dlsym(h, "he_reset");
    a.step = (decltype(a.step))dlsym(h, "he_step");
    a.rollout = (decltype(a.rollout))dlsym(h, "he_rollout");
    a.sync_market = (decltype(a.sync_market))dlsym(h, "he_sync_market");
    a.last_error = (decltype(a.last_error))dlsym(h, "he_last_error");
    return a;
}

int main(int argc, char** argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    if (argc < 3) { fprintf(stderr, "usage: step_bench N lib.so...\n"); return 2; }
    const int64_t N = atoll(argv[1]);
    // STEP_BENCH_ROLLOUT=K: he_rollout of K fused steps per launch instead of he_step
    const int RK = getenv("STEP_BENCH_ROLLOUT") ? atoi(getenv("STEP_BENCH_ROLLOUT")) : 0;
    const int64_t KK = RK > 0 ? RK : 1;
    float *act, *obs, *rew;
    uint8_t *term, *trunc;
    CK(hipMalloc(&act, KK * N * 8));
    CK(hipMalloc(&obs, KK * N * 52));
    CK(hipMalloc(&rew, KK * N * 4));
    CK(hipMalloc(&term, KK * N));
    CK(hipMalloc(&trunc, N));
    std::vector<float> ha(KK * N * 2);
    for (int64_t i = 0; i < KK * N * 2; ++i) ha[i] = (float)((i * 2654435761u) % 2001) / 1000.0f - 1.0f;
    CK(hipMemcpy(act, ha.data(), KK * N * 8, hipMemcpyHostToDevice));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int li = 2; li < argc; ++li) {
        Api api = load(argv[li]);
        he_config c;
        api.config_init(&c, 2);
        c.n_envs = N;
        c.mode = HE_MODE_GBM;
        c.market_prefetch = getenv("STEP_BENCH_PREFETCH") ? 2 : ((RK > 0 && !getenv("STEP_BENCH_NOPF")) ? 0 : 1);  // always / (auto) / never
        he_env* env;
        if (api.create(&c, &env) != HE_OK) { fprintf(stderr, "create: %s\n", api.last_error(env)); return 1; }
        if (api.reset(env, nullptr, 0, obs, nullptr, st) != HE_OK) return 1;
        float* o = getenv("STEP_BENCH_NO_OBS") ? nullptr : obs;
        auto one = [&]() {
            if (RK > 0) return api.rollout(env, RK, act, o, rew, term, st);
            return api.step(env, act, o, rew, term, trunc, nullptr, nullptr, st);
        };
        const int per_graph = RK > 0 ? (64 / RK > 0 ? 64 / RK : 1) : 64;
        for (int k = 0; k < per_graph; ++k)
            if (one() != HE_OK) { fprintf(stderr, "step: %s\n", api.last_error(env)); return 1; }
        api.sync_market(env, st);
        CK(hipStreamSynchronize(st));
        hipGraph_t g[4];
        hipGraphExec_t ge[4];
        for (int gi = 0; gi < 4; ++gi) {
            CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
            for (int k = 0; k < per_graph; ++k) one();
            api.sync_market(env, st);
            CK(hipStreamEndCapture(st, &g[gi]));
            CK(hipGraphInstantiate(&ge[gi], g[gi], nullptr, nullptr, 0));
        }
        const int warm = getenv("STEP_BENCH_REPS") ? 1 : 8;
        for (int r = 0; r < warm; ++r) CK(hipGraphLaunch(ge[r & 3], st));
        CK(hipStreamSynchronize(st));
        const int reps = getenv("STEP_BENCH_REPS") ? atoi(getenv("STEP_BENCH_REPS")) : 160;
        CK(hipEventRecord(a, st));
        for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge[r & 3], st));
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        double us = ms * 1000.0 / (reps * (double)per_graph * KK);
        printf("%-24s%s%s%s N=%lld  %.3f us/step  %.4e env-steps/s\n", argv[li], o ? "" : " (no obs)", c.market_prefetch == 2 ? " (prefetch)" : "", RK > 0 ? " (rollout)" : "", (long long)N, us, N / us * 1e6);
        typedef he_status (*tim_fn)(void*, size_t);
        tim_fn tim = (tim_fn)dlsym(api.handle, "he_debug_timing");
        if (tim) {
            // per-wave timestamps of the last step_kernel: {realtime 100 MHz, shader clock}
            const int W = 8192, P = 5;  // [5][8192][2]
            std::vector<uint64_t> t((size_t)5 * W * 2);
            tim(t.data(), t.size() * 8);
            const int nw = (int)((N + 63) / 64);
            auto at = [&](int k, int w, int c) { return t[((size_t)k * W + w) * 2 + c]; };
            uint64_t rt0 = ~0ull, rt0max = 0, rtend = 0;
            double dc[P] = {0};
            for (int w = 0; w < nw; ++w) {
                rt0 = std::min(rt0, at(0, w, 0));
                rt0max = std::max(rt0max, at(0, w, 0));
                rtend = std::max(rtend, at(4, w, 0));
                for (int k = 1; k < P; ++k) dc[k] += (double)(at(k, w, 1) - at(k - 1, w, 1));
            }
            printf("   waves %d: start spread %.2f us, first start -> last end %.2f us\n", nw, (rt0max - rt0) * 0.01,
                   (rtend - rt0) * 0.01);
            printf("   mean shader cycles: entry->scalar %.0f, ->vector %.0f, ->compute %.0f, ->end %.0f\n",
                   dc[1] / nw, dc[2] / nw, dc[3] / nw, dc[4] / nw);
            // histogram of wave start offsets (realtime ticks of 10 ns)
            int hist[12] = {0};
            for (int w = 0; w < nw; ++w) { int b = (int)((at(0, w, 0) - rt0) / 25); hist[b > 11 ? 11 : b]++; }
            printf("   start histogram (0.25 us bins):");
            for (int b = 0; b < 12; ++b) printf(" %d", hist[b]);
            printf("\n");
        }
        for (int gi = 0; gi < 4; ++gi) { hipGraphExecDestroy(ge[gi]); hipGraphDestroy(g[gi]); }
        api.destroy(env);
    }
    return 0;
}
