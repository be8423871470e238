// Streaming read / copy ceilings of HBM on the box (dwordx4 per lane,
// grid-stride, many waves): the practical peak the roofline fractions are
// read against.  Dev tool: hipcc --offload-arch=gfx950 -O3 bw_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void k_read(const double4 *__restrict__ a, size_t n, double *out) {
    double s = 0.0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const double4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.678) out[0] = s;  // keeps the loads live
}

__global__ __launch_bounds__(256) void k_copy(const double4 *__restrict__ a, double4 *__restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) b[i] = a[i];
}

int main() {
    const size_t bytes = 8ull << 30, n = bytes / sizeof(double4);
    double4 *a, *b;
    double *o;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess || hipMalloc(&o, 8) != hipSuccess)
        return 1;
    (void)hipMemset(a, 0, bytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int grid : {1024, 2048, 4096, 8192, 16384}) {
        float best_r = 1e9f, best_c = 1e9f;
        for (int r = 0; r < 4; ++r) {
            float ms;
            hipEventRecord(e0);
            hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, a, n, o);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms, e0, e1);
            if (r && ms < best_r) best_r = ms;
            hipEventRecord(e0);
            hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, a, b, n);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms, e0, e1);
            if (r && ms < best_c) best_c = ms;
        }
        printf("{\"grid\": %d, \"read_gbs\": %.0f, \"copy_gbs\": %.0f}\n", grid, bytes / (best_r * 1e-3) / 1e9,
               2.0 * bytes / (best_c * 1e-3) / 1e9);
    }
    return 0;
}
