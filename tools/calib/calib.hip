// Read-traffic calibration kernels for the TCC request counters (tools/traffic_calib.py):
// known byte counts in the access shapes the step kernels use.  Each kernel reads `rows`
// 128-B lines of a table whose row stride is `stride` float4s and writes one float per
// workgroup (negligible next to the reads).
#include <hip/hip_runtime.h>
#include <cstdint>

// every lane one 16-B piece, a wave 1 KiB of consecutive bytes (the wide coalesced read)
__global__ void __launch_bounds__(256) calib_stream(const float4* __restrict__ src, int64_t n16, float* out) {
    float acc = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
        const float4 v = src[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.678f) out[blockIdx.x] = acc;   // keeps the loads; never true on the zero table
}

// lds_replay_loader's shape: a workgroup of 2 waves covers 64 rows; wave `part` lane l reads the
// 4 consecutive float4s [part * 4, part * 4 + 4) of row blockIdx * 64 + l -- a 64-B half line per
// lane, the two halves of each line from the two waves
__global__ void __launch_bounds__(128) calib_halfline(const float4* __restrict__ src, int64_t rows, int64_t stride,
                                                      float* out) {
    const int lane = threadIdx.x & 63, part = threadIdx.x >> 6;
    const int64_t r = (int64_t)blockIdx.x * 64 + lane;
    float acc = 0.f;
    if (r < rows) {
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const float4 v = src[r * stride + part * 4 + h];
            acc += v.x + v.y + v.z + v.w;
        }
    }
    if (acc == 12345.678f) out[blockIdx.x] = acc;
}

// one wave per 64 rows, every lane its whole 128-B line (8 float4s)
__global__ void __launch_bounds__(64) calib_fullline(const float4* __restrict__ src, int64_t rows, int64_t stride,
                                                     float* out) {
    const int64_t r = (int64_t)blockIdx.x * 64 + threadIdx.x;
    float acc = 0.f;
    if (r < rows) {
#pragma unroll
        for (int h = 0; h < 8; ++h) {
            const float4 v = src[r * stride + h];
            acc += v.x + v.y + v.z + v.w;
        }
    }
    if (acc == 12345.678f) out[blockIdx.x] = acc;
}

extern "C" int calib_run(int which, const void* src, int64_t rows, int64_t stride, void* out, hipStream_t s) {
    const float4* t = (const float4*)src;
    float* o = (float*)out;
    if (which == 0) calib_stream<<<4096, 256, 0, s>>>(t, rows * 8, o);
    else if (which == 1) calib_halfline<<<(unsigned)((rows + 63) / 64), 128, 0, s>>>(t, rows, stride, o);
    else calib_fullline<<<(unsigned)((rows + 63) / 64), 64, 0, s>>>(t, rows, stride, o);
    return (int)hipGetLastError();
}
