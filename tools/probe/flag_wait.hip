// Small-N host step latency probe (MI355X): what a one-workgroup step costs from the host's
// launch to the host seeing its outputs, by completion mechanism.
//   (a) hipStreamSynchronize after the launch (the current he_stream_wait)
//   (b) hipEventRecord + hipEventSynchronize
//   (c) the kernel stores a sequence number into host-coherent memory after its outputs
//       (system-scope release); the host spins on it
// The kernel reads 2 actions from mapped memory and writes 16 floats back, as the N=2 step.
//   hipcc --offload-arch=gfx950 -O2 -o tools/probe/flag_wait tools/probe/flag_wait.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void step_like(const float* act, float* out, unsigned* flag, unsigned seq) {
    const int i = threadIdx.x;
    float a = act[i & 3];
    float v = a;
    for (int k = 0; k < 64; ++k) v = fmaf(v, 1.0001f, 0.5f);
    if (i < 16) out[i] = v;
    if (flag) {
        __syncthreads();
        if (i == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

struct Act8 { float a[8]; };
__global__ void step_like_kernarg(Act8 act, float* out, unsigned* flag, unsigned seq) {
    const int i = threadIdx.x;
    float a = act.a[i & 3];
    float v = a;
    for (int k = 0; k < 64; ++k) v = fmaf(v, 1.0001f, 0.5f);
    if (i < 16) out[i] = v;
    __syncthreads();
    if (i == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void report(const char* name, std::vector<double>& t) {
    std::sort(t.begin(), t.end());
    double s = 0;
    for (double x : t) s += x;
    printf("%-44s median %7.2f us  p10 %7.2f  p90 %7.2f  mean %7.2f\n", name, t[t.size() / 2], t[t.size() / 10],
           t[t.size() * 9 / 10], s / t.size());
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 3000;
    if (argc > 2 && atoi(argv[2]) == 1) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
    CK(hipSetDevice(0));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    void* h = nullptr;
    CK(hipHostMalloc(&h, 4096, hipHostMallocMapped | hipHostMallocCoherent));
    void* d = nullptr;
    CK(hipHostGetDevicePointer(&d, h, 0));
    float* hact = (float*)h;
    volatile unsigned* hflag = (volatile unsigned*)((char*)h + 1024);
    const float* dact = (const float*)d;
    float* dout = (float*)((char*)d + 256);
    unsigned* dflag = (unsigned*)((char*)d + 1024);
    *hflag = 0;
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    std::vector<double> t(n);
    for (int w = 0; w < 200; ++w) {
        hipLaunchKernelGGL(step_like, dim3(1), dim3(64), 0, st, dact, dout, nullptr, 0u);
        CK(hipStreamSynchronize(st));
    }
    for (int i = 0; i < n; ++i) {
        double a = now_us();
        hact[0] = (float)i;
        hipLaunchKernelGGL(step_like, dim3(1), dim3(64), 0, st, dact, dout, nullptr, 0u);
        CK(hipStreamSynchronize(st));
        t[i] = now_us() - a;
    }
    report("launch + hipStreamSynchronize", t);
    for (int i = 0; i < n; ++i) {
        double a = now_us();
        hipLaunchKernelGGL(step_like, dim3(1), dim3(64), 0, st, dact, dout, nullptr, 0u);
        CK(hipEventRecord(ev, st));
        CK(hipEventSynchronize(ev));
        t[i] = now_us() - a;
    }
    report("launch + event record + synchronize", t);
    for (int i = 0; i < n; ++i) {
        double a = now_us();
        hipLaunchKernelGGL(step_like, dim3(1), dim3(64), 0, st, dact, dout, nullptr, 0u);
        t[i] = now_us() - a;
    }
    CK(hipStreamSynchronize(st));
    report("launch only", t);
    unsigned seq = 1;
    long timeouts = 0;
    for (int i = 0; i < n; ++i) {
        double a = now_us();
        ++seq;
        hipLaunchKernelGGL(step_like, dim3(1), dim3(64), 0, st, dact, dout, dflag, seq);
        double lim = a + 1e6;
        while (*hflag != seq) {
            if (now_us() > lim) { ++timeouts; break; }
        }
        t[i] = now_us() - a;
    }
    report("launch + host spin on a kernel-written flag", t);
    CK(hipStreamSynchronize(st));
    // the flag seen, then a stream synchronize (what the runtime still owes)
    for (int i = 0; i < n; ++i) {
        ++seq;
        hipLaunchKernelGGL(step_like, dim3(1), dim3(64), 0, st, dact, dout, dflag, seq);
        double lim = now_us() + 1e6;
        while (*hflag != seq) {
            if (now_us() > lim) { ++timeouts; break; }
        }
        double a = now_us();
        CK(hipStreamSynchronize(st));
        t[i] = now_us() - a;
    }
    report("hipStreamSynchronize after the flag", t);
    // back-to-back: flag-waited steps with no stream synchronize in between (the runtime's queue grows
    // only by retired packets)
    for (int i = 0; i < n; ++i) {
        double a = now_us();
        ++seq;
        hipLaunchKernelGGL(step_like, dim3(1), dim3(64), 0, st, dact, dout, dflag, seq);
        double lim = a + 1e6;
        while (*hflag != seq) {
            if (now_us() > lim) { ++timeouts; break; }
        }
        t[i] = now_us() - a;
    }
    report("flag-waited steps, second run", t);
    for (int i = 0; i < n; ++i) {
        double a = now_us();
        ++seq;
        Act8 av;
        for (int j = 0; j < 8; ++j) av.a[j] = hact[j];
        hipLaunchKernelGGL(step_like_kernarg, dim3(1), dim3(64), 0, st, av, dout, dflag, seq);
        double lim = a + 1e6;
        while (*hflag != seq) {
            if (now_us() > lim) { ++timeouts; break; }
        }
        t[i] = now_us() - a;
    }
    report("actions in kernargs, flag-waited", t);
    for (int i = 0; i < n; ++i) {
        double a = now_us();
        ++seq;
        hipLaunchKernelGGL(step_like, dim3(4), dim3(256), 0, st, dact, dout, dflag, seq);
        double lim = a + 1e6;
        while (*hflag != seq) {
            if (now_us() > lim) { ++timeouts; break; }
        }
        t[i] = now_us() - a;
    }
    report("4 x 256 threads, flag-waited (no counter)", t);
    CK(hipStreamSynchronize(st));
    printf("timeouts %ld\n", timeouts);
    CK(hipEventDestroy(ev));
    CK(hipHostFree(h));
    CK(hipStreamDestroy(st));
    return timeouts ? 2 : 0;
}
