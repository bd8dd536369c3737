// v_rcp_f64 accuracy over the Mills reciprocal's range d in [3.5, 43] (mills(): 1/d by
// rcp + Newton steps): relative error of the raw instruction and after one and two Newton
// steps, against the correctly rounded 1/d of the host.  hipcc --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

__global__ void k(const double* d, double* r0, double* r1, double* r2, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = d[i];
    double y = __builtin_amdgcn_rcp(x);
    r0[i] = y;
    y = fma(fma(-x, y, 1.0), y, y);
    r1[i] = y;
    y = fma(fma(-x, y, 1.0), y, y);
    r2[i] = y;
}

int main() {
    const int n = 1 << 24;
    std::vector<double> d(n), a(n), b(n), c(n);
    for (int i = 0; i < n; ++i) d[i] = 3.5 + (43.0 - 3.5) * (i + 0.37) / n;
    double *dd, *da, *db, *dc;
    hipMalloc(&dd, n * 8); hipMalloc(&da, n * 8); hipMalloc(&db, n * 8); hipMalloc(&dc, n * 8);
    hipMemcpy(dd, d.data(), n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dd, da, db, dc, n);
    hipMemcpy(a.data(), da, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(b.data(), db, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(c.data(), dc, n * 8, hipMemcpyDeviceToHost);
    double e0 = 0, e1 = 0, e2 = 0;
    long n1 = 0, n2 = 0;
    for (int i = 0; i < n; ++i) {
        const double q = 1.0 / d[i];
        e0 = fmax(e0, fabs(a[i] / q - 1));
        e1 = fmax(e1, fabs(b[i] / q - 1));
        e2 = fmax(e2, fabs(c[i] / q - 1));
        n1 += b[i] != q;
        n2 += c[i] != q;
    }
    printf("v_rcp_f64 on [3.5, 43], %d points: max rel err raw %.3e, 1 Newton %.3e (%ld not RN), 2 Newton %.3e (%ld not RN)\n",
           n, e0, e1, n1, e2, n2);
    return 0;
}
