// floor.hip -- floors for the Gym-API step kernel (he_step, one launch per env-step):
// what a launch of step1_kernel's grid costs when it does nothing, and when it only moves
// he_step's bytes.  Built by tools/floor/run.py (hipcc -shared), timed there in hipGraphs
// of 64 launches (the bench's graph mode) and under rocprofv3.
//   floor_empty   grid (N / 256) x 256, no memory access
//   floor_copy    the same grid; per env: reads 56 B (state 16, action 8, 2 market records
//                 12 + 12 + greeks 8) and writes 74 B (state 16, obs 52 as one row, reward
//                 4, flags 2) -- he_step's 134 B at 65,536 envs, dependent store after load
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void floor_empty(int64_t n, float* sink) {
    if ((int64_t)blockIdx.x * 256 + threadIdx.x == n + 1) sink[0] = 0.0f;  // never true
}

__global__ __launch_bounds__(256) void floor_copy(int64_t n, const float4* __restrict__ in, float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    // 3.5 x 16 B in: coalesced float4 rows of a [n][4] SoA-ish layout
    const float4 a = in[i], b = in[n + i], c = in[2 * n + i];
    const float2 d = reinterpret_cast<const float2*>(in + 3 * n)[i];
    const float s = a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w + c.x + c.y + c.z + c.w + d.x + d.y;
    float* o = out + i * 13;                 // 52-B rows, as the obs output
#pragma unroll
    for (int k = 0; k < 13; ++k) o[k] = s + (float)k;
    float* t = out + n * 13;                 // reward, state (16 B as 4 floats), flags
    t[i] = s;
    reinterpret_cast<float4*>(t + n)[i] = make_float4(s, s, s, s);
    reinterpret_cast<uint16_t*>(t + 5 * n)[i] = (uint16_t)s;
}

extern "C" int floor_launch(int which, int64_t n, const void* in, void* out, void* stream) {
    const unsigned blocks = (unsigned)((n + 255) / 256);
    if (which == 0)
        hipLaunchKernelGGL(floor_empty, dim3(blocks), dim3(256), 0, (hipStream_t)stream, n, (float*)out);
    else
        hipLaunchKernelGGL(floor_copy, dim3(blocks), dim3(256), 0, (hipStream_t)stream, n, (const float4*)in,
                           (float*)out);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
