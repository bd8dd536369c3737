// Floor of a one-thread-per-env step at 65,536 envs on MI355X: an empty kernel and
// copy kernels that move the step_kernel's bytes (72 B read, 74 B written per env)
// with the same grid (256 x 256).  Timed with hipExtLaunchKernelGGL events.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include <vector>
#include <algorithm>

__global__ __launch_bounds__(256) void k_empty(int n) {}

// 72 B in, 74 B out per env, same field shapes as step_kernel<GBM>
__global__ __launch_bounds__(256) void k_copy(int n, const uint32_t* t, const uint32_t* pos, const double* cash,
                                            const float2* act, const float4* preA, const float4* postA,
                                            const float4* postB, uint32_t* t_o, uint32_t* pos_o, double* cash_o,
                                            float* obs, float* rew, uint8_t* term, uint8_t* trunc) {
    __shared__ __attribute__((aligned(16))) float tile[256 * 13];
    int i = blockIdx.x * 256 + threadIdx.x;
    uint32_t a = t[i], b = pos[i];
    double c = cash[i];
    float2 ac = act[i];
    float4 p0 = preA[i], p1 = postA[i], p2 = postB[i];
    float o[13] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w, p2.x, p2.y, p2.z, ac.x, ac.y};
    for (int k = 0; k < 13; ++k) tile[threadIdx.x * 13 + k] = o[k] + (float)a;
    t_o[i] = a + 1;
    pos_o[i] = b ^ 1u;
    cash_o[i] = c + 1.0;
    rew[i] = p1.x - p0.x;
    term[i] = (uint8_t)(a & 1);
    trunc[i] = 0;
    __syncthreads();
    float4* d4 = reinterpret_cast<float4*>(obs + (size_t)blockIdx.x * 256 * 13);
    const float4* s4 = reinterpret_cast<const float4*>(tile);
    for (int k = threadIdx.x; k < 832; k += 256) d4[k] = s4[k];
}

// same as k_copy with a step_kernel-sized (~800 B) kernarg segment
struct BigArgs {
    const uint32_t* t; const uint32_t* pos; const double* cash; const float2* act;
    const float4* preA; const float4* postA; const float4* postB;
    uint32_t* t_o; uint32_t* pos_o; double* cash_o; float* obs; float* rew; uint8_t* term; uint8_t* trunc;
    double pad[86];
};
__global__ __launch_bounds__(256) void k_copy_big(int n, BigArgs g) {
    __shared__ __attribute__((aligned(16))) float tile[256 * 13];
    int i = blockIdx.x * 256 + threadIdx.x;
    uint32_t a = g.t[i], b = g.pos[i];
    double c = g.cash[i] + g.pad[85];
    float2 ac = g.act[i];
    float4 p0 = g.preA[i], p1 = g.postA[i], p2 = g.postB[i];
    float o[13] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w, p2.x, p2.y, p2.z, ac.x, ac.y};
    for (int k = 0; k < 13; ++k) tile[threadIdx.x * 13 + k] = o[k] + (float)a;
    g.t_o[i] = a + 1;
    g.pos_o[i] = b ^ 1u;
    g.cash_o[i] = c + 1.0;
    g.rew[i] = p1.x - p0.x;
    g.term[i] = (uint8_t)(a & 1);
    g.trunc[i] = 0;
    __syncthreads();
    float4* d4 = reinterpret_cast<float4*>(g.obs + (size_t)blockIdx.x * 256 * 13);
    const float4* s4 = reinterpret_cast<const float4*>(tile);
    for (int k = threadIdx.x; k < 832; k += 256) d4[k] = s4[k];
}

// kernarg fetch cost: the same trivial kernel touching 1 or 12 distinct 64-B lines
// of an 800-B kernarg segment (one scalar round trip either way)
__global__ __launch_bounds__(256) void k_args1(int n, BigArgs g) {
    int i = blockIdx.x * 256 + threadIdx.x;
    g.rew[i] = (float)g.pad[0];
}
__global__ __launch_bounds__(256) void k_args12(int n, BigArgs g) {
    int i = blockIdx.x * 256 + threadIdx.x;
    double a0 = g.pad[0], a1 = g.pad[8], a2 = g.pad[16], a3 = g.pad[24], a4 = g.pad[32], a5 = g.pad[40],
           a6 = g.pad[48], a7 = g.pad[56], a8 = g.pad[64], a9 = g.pad[72], a10 = g.pad[80], a11 = g.pad[85];
    asm volatile("" : "+s"(a0), "+s"(a1), "+s"(a2), "+s"(a3), "+s"(a4), "+s"(a5), "+s"(a6), "+s"(a7), "+s"(a8),
                 "+s"(a9), "+s"(a10), "+s"(a11));
    g.rew[i] = (float)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + a8 + a9 + a10 + a11);
}

// pure streaming: 146 B per env as float4 loads/stores (ideal coalescing)
__global__ __launch_bounds__(256) void k_stream(int nv, const float4* src, float4* dst) {
    int i = blockIdx.x * 256 + threadIdx.x;
    for (int k = i; k < nv; k += gridDim.x * 256) dst[k] = src[k];
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const int N = 65536;
    std::vector<void*> bufs;
    auto alloc = [&](size_t b) { void* p; hipMalloc(&p, b); hipMemset(p, 0, b); bufs.push_back(p); return p; };
    uint32_t* t = (uint32_t*)alloc(N * 4); uint32_t* pos = (uint32_t*)alloc(N * 4); double* cash = (double*)alloc(N * 8);
    float2* act = (float2*)alloc(N * 8); float4* preA = (float4*)alloc(N * 16); float4* postA = (float4*)alloc(N * 16);
    float4* postB = (float4*)alloc(N * 16);
    uint32_t* t_o = (uint32_t*)alloc(N * 4); uint32_t* pos_o = (uint32_t*)alloc(N * 4); double* cash_o = (double*)alloc(N * 8);
    float* obs = (float*)alloc(N * 52); float* rew = (float*)alloc(N * 4); uint8_t* term = (uint8_t*)alloc(N);
    uint8_t* trunc = (uint8_t*)alloc(N);
    const int nv = N * 146 / 16 / 2;
    float4* s1 = (float4*)alloc((size_t)nv * 16); float4* s2 = (float4*)alloc((size_t)nv * 16);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    auto timeit = [&](const char* name, auto launch) {
        std::vector<float> v;
        for (int r = 0; r < 300; ++r) {
            launch(a, b);
            hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            if (r >= 20) v.push_back(ms * 1000.f);
        }
        std::sort(v.begin(), v.end());
        printf("%-28s median %.3f us  p10 %.3f  p90 %.3f\n", name, v[v.size() / 2], v[v.size() / 10], v[v.size() * 9 / 10]);
    };
    timeit("empty 256x256", [&](hipEvent_t e0, hipEvent_t e1) {
        hipExtLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, 0, e0, e1, 0, N); });
    timeit("copy step-shaped 146B/env", [&](hipEvent_t e0, hipEvent_t e1) {
        hipExtLaunchKernelGGL(k_copy, dim3(256), dim3(256), 0, 0, e0, e1, 0, N, t, pos, cash, act, preA, postA, postB,
                              t_o, pos_o, cash_o, obs, rew, term, trunc); });
    timeit("stream float4 9.57MB", [&](hipEvent_t e0, hipEvent_t e1) {
        hipExtLaunchKernelGGL(k_stream, dim3(1024), dim3(256), 0, 0, e0, e1, 0, nv, s1, s2); });
    // back-to-back throughput of the copy kernel (launch gaps included)
    hipEventRecord(a, 0);
    for (int r = 0; r < 1000; ++r)
        hipLaunchKernelGGL(k_copy, dim3(256), dim3(256), 0, 0, N, t, pos, cash, act, preA, postA, postB, t_o, pos_o,
                           cash_o, obs, rew, term, trunc);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("copy back-to-back: %.3f us/launch\n", ms);
    // graph mode: 64 back-to-back launches per graph, 50 replays
    BigArgs g{t, pos, cash, act, preA, postA, postB, t_o, pos_o, cash_o, obs, rew, term, trunc, {}};
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    auto graph_time = [&](const char* name, auto launch) {
        hipGraph_t gr; hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int r = 0; r < 64; ++r) launch();
        CK(hipStreamEndCapture(st, &gr));
        CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
        for (int r = 0; r < 5; ++r) hipGraphLaunch(ge, st);
        hipStreamSynchronize(st);
        hipEventRecord(a, st);
        for (int r = 0; r < 50; ++r) hipGraphLaunch(ge, st);
        hipEventRecord(b, st);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        printf("graph x64 %-22s %.3f us/launch\n", name, ms * 1000.f / (50 * 64));
        hipGraphExecDestroy(ge); hipGraphDestroy(gr);
    };
    graph_time("empty", [&] { hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, st, N); });
    graph_time("copy", [&] {
        hipLaunchKernelGGL(k_copy, dim3(256), dim3(256), 0, st, N, t, pos, cash, act, preA, postA, postB, t_o,
                           pos_o, cash_o, obs, rew, term, trunc); });
    graph_time("kernarg 1 line", [&] { hipLaunchKernelGGL(k_args1, dim3(256), dim3(256), 0, st, N, g); });
    graph_time("kernarg 12 lines", [&] { hipLaunchKernelGGL(k_args12, dim3(256), dim3(256), 0, st, N, g); });
    graph_time("copy big kernarg", [&] { hipLaunchKernelGGL(k_copy_big, dim3(256), dim3(256), 0, st, N, g); });
    hipEventRecord(a, st);
    for (int r = 0; r < 1000; ++r) hipLaunchKernelGGL(k_copy_big, dim3(256), dim3(256), 0, st, N, g);
    hipEventRecord(b, st);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("copy big kernarg back-to-back: %.3f us/launch\n", ms);
    for (void* p : bufs) hipFree(p);
    return 0;
}
