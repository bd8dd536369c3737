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

#include <vector>

#include "../include/hedge_env.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

struct Api {
    decltype(&he_config_init) config_init;
    decltype(&he_create) create;
    decltype(&he_destroy) destroy;
    decltype(&he_reset) reset;
    decltype(&he_step) step;
    decltype(&he_sync_market) sync_market;
    decltype(&he_last_error) last_error;
};

static Api load(const char* path) {
    void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) { fprintf(stderr, "dlopen %s: %s\n", path, dlerror()); exit(1); }
    Api a;
    a.config_init = (decltype(a.config_init))dlsym(h, "he_config_init");
    a.create = (decltype(a.create))dlsym(h, "he_create");
    a.destroy = (decltype(a.destroy))dlsym(h, "he_destroy");
    a.reset = (decltype(a.reset))dlsym(h, "he_reset");
    a.step = (decltype(a.step))dlsym(h, "he_step");
    a.sync_market = (decltype(a.sync_market))dlsym(h, "he_sync_market");
    a.last_error = (decltype(a.last_error))dlsym(h, "he_last_error");
    return a;
}

int main(int argc, char** argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    if (argc < 3) { fprintf(stderr, "usage: step_bench N lib.so...\n"); return 2; }
    const int64_t N = atoll(argv[1]);
    float *act, *obs, *rew;
    uint8_t *term, *trunc;
    CK(hipMalloc(&act, N * 8));
    CK(hipMalloc(&obs, N * 52));
    CK(hipMalloc(&rew, N * 4));
    CK(hipMalloc(&term, N));
    CK(hipMalloc(&trunc, N));
    std::vector<float> ha(N * 2);
    for (int64_t i = 0; i < N * 2; ++i) ha[i] = (float)((i * 2654435761u) % 2001) / 1000.0f - 1.0f;
    CK(hipMemcpy(act, ha.data(), N * 8, hipMemcpyHostToDevice));
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
        c.reserved_i = getenv("STEP_BENCH_PREFETCH") ? 2 : 1;  // always / never
        he_env* env;
        if (api.create(&c, &env) != HE_OK) { fprintf(stderr, "create: %s\n", api.last_error(env)); return 1; }
        if (api.reset(env, nullptr, 0, obs, nullptr, st) != HE_OK) return 1;
        float* o = getenv("STEP_BENCH_NO_OBS") ? nullptr : obs;
        for (int k = 0; k < 64; ++k)
            if (api.step(env, act, o, rew, term, trunc, nullptr, nullptr, st) != HE_OK) return 1;
        api.sync_market(env, st);
        CK(hipStreamSynchronize(st));
        hipGraph_t g[4];
        hipGraphExec_t ge[4];
        for (int gi = 0; gi < 4; ++gi) {
            CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
            for (int k = 0; k < 64; ++k) api.step(env, act, o, rew, term, trunc, nullptr, nullptr, st);
            api.sync_market(env, st);
            CK(hipStreamEndCapture(st, &g[gi]));
            CK(hipGraphInstantiate(&ge[gi], g[gi], nullptr, nullptr, 0));
        }
        for (int r = 0; r < 8; ++r) CK(hipGraphLaunch(ge[r & 3], st));
        CK(hipStreamSynchronize(st));
        const int reps = 160;
        CK(hipEventRecord(a, st));
        for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge[r & 3], st));
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        double us = ms * 1000.0 / (reps * 64.0);
        printf("%-24s%s%s N=%lld  %.3f us/step  %.4e env-steps/s\n", argv[li], o ? "" : " (no obs)", c.reserved_i == 2 ? " (prefetch)" : "", (long long)N, us, N / us * 1e6);
        for (int gi = 0; gi < 4; ++gi) { hipGraphExecDestroy(ge[gi]); hipGraphDestroy(g[gi]); }
        api.destroy(env);
    }
    return 0;
}
