// Latency / issue micro-benchmark of the fp64 primitives the combine and the
// augmented segment stage are built from (gfx950).  One wave per block (or 4
// for the barrier rows); prints core-clock cycles per operation (s_memtime).
// Dev tool only: hipcc --offload-arch=gfx950 -O3 lat_bench.hip -o lat_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

typedef double d4 __attribute__((ext_vector_type(4)));
#define REP 256

__device__ __forceinline__ d4 mfma(double a, double b, d4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }

// 0: dependent MFMA chain (accumulator dependency)
// 1: 4 independent MFMA chains interleaved (issue rate)
// 2: dependent f64 FMA chain
// 3: dependent v_rsq_f64 chain
// 4: MFMA -> readlane of its result -> next MFMA operand (round trip)
// 5: LDS write -> read round trip (dependent, one wave)
// 6: s_barrier, 4 waves, nothing else
// 7: LDS exchange + barrier, 4 waves (write 2 KB tile, barrier, read 2 tiles)
// 8: independent f64 FMAs (issue rate)
// 9: v_rcp_f64 dependent chain
__global__ __launch_bounds__(256) void k_lat(int which, double seed, double *out, long long *cyc) {
    __shared__ double lds[4 * 512 + 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    double x = seed + lane * 1e-3;
    d4 a0 = {x, x, x, x}, a1 = a0, a2 = a0, a3 = a0;
    double s = x;
    for (int i = threadIdx.x; i < 4 * 512 + 64; i += blockDim.x) lds[i] = 1.0 + i * 1e-6;
    __syncthreads();
    long long t0 = clock64();
    switch (which) {
        case 0:
            for (int i = 0; i < REP; ++i) a0 = mfma(x, s, a0);
            break;
        case 1:
            for (int i = 0; i < REP; ++i) {
                a0 = mfma(x, s, a0); a1 = mfma(x, s, a1); a2 = mfma(x, s, a2); a3 = mfma(x, s, a3);
            }
            break;
        case 2:
            for (int i = 0; i < REP; ++i) s = __builtin_fma(s, 0.999, 1e-3);
            break;
        case 3:
            for (int i = 0; i < REP; ++i) s = __builtin_amdgcn_rsq(s) + 0.5;
            break;
        case 4:
            for (int i = 0; i < REP; ++i) {
                a0 = mfma(x, s, a0);
                const int lo = __builtin_amdgcn_readlane(__double2loint(a0[1]), 5);
                const int hi = __builtin_amdgcn_readlane(__double2hiint(a0[1]), 5);
                s = __hiloint2double(hi, lo) * 1e-3;
            }
            break;
        case 5:
            for (int i = 0; i < REP; ++i) {
                lds[wv * 512 + lane] = s;
                __builtin_amdgcn_wave_barrier();
                s = lds[wv * 512 + ((lane + 1) & 63)] * 0.5 + 0.25;
            }
            break;
        case 6:
            for (int i = 0; i < REP; ++i) { __builtin_amdgcn_s_barrier(); s = s * 0.5 + 0.25; }
            break;
        case 7:
            for (int i = 0; i < REP; ++i) {
                double2 *p = reinterpret_cast<double2 *>(lds + wv * 512);
                p[lane] = double2{s, s};
                p[64 + lane] = double2{s, s};
                __syncthreads();
                const double2 *q = reinterpret_cast<const double2 *>(lds + ((wv + 1) & 3) * 512);
                const double2 *q2 = reinterpret_cast<const double2 *>(lds + ((wv + 2) & 3) * 512);
                double2 v0 = q[lane], v1 = q[64 + lane], v2 = q2[lane], v3 = q2[64 + lane];
                s = (v0.x + v1.y + v2.x + v3.y) * 0.25;
                __syncthreads();
            }
            break;
        case 8:
            {
                double s1 = s + 1, s2 = s + 2, s3 = s + 3, s4 = s + 4, s5 = s + 5, s6 = s + 6, s7 = s + 7;
                for (int i = 0; i < REP; ++i) {
                    s = __builtin_fma(s, 0.999, 1e-3); s1 = __builtin_fma(s1, 0.999, 1e-3);
                    s2 = __builtin_fma(s2, 0.999, 1e-3); s3 = __builtin_fma(s3, 0.999, 1e-3);
                    s4 = __builtin_fma(s4, 0.999, 1e-3); s5 = __builtin_fma(s5, 0.999, 1e-3);
                    s6 = __builtin_fma(s6, 0.999, 1e-3); s7 = __builtin_fma(s7, 0.999, 1e-3);
                }
                s += s1 + s2 + s3 + s4 + s5 + s6 + s7;
            }
            break;
        case 9:
            for (int i = 0; i < REP; ++i) s = __builtin_amdgcn_rcp(s) + 0.5;
            break;
    }
    long long t1 = clock64();
    out[blockIdx.x * 256 + threadIdx.x] = s + a0[0] + a1[1] + a2[2] + a3[3];
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    const char *names[] = {"mfma_f64 dependent", "mfma_f64 4 independent (per mfma)", "fma_f64 dependent",
                           "rsq_f64 dependent (+add)", "mfma->readlane->mfma", "lds write->read (+fma)",
                           "s_barrier 4 waves (+fma)", "lds 2-tile exchange + 2 barriers", "fma_f64 8 independent (per fma)",
                           "rcp_f64 dependent (+add)"};
    const int per[] = {1, 4, 1, 1, 1, 1, 1, 1, 8, 1};
    double *out; long long *cyc;
    hipMalloc(&out, 64 * 256 * sizeof(double));
    hipMalloc(&cyc, 64 * sizeof(long long));
    for (int w = 0; w < 10; ++w) {
        const int threads = (w == 6 || w == 7) ? 256 : 64;
        std::vector<long long> h(8);
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(k_lat, dim3(8), dim3(threads), 0, 0, w, 1.0, out, cyc);
            hipDeviceSynchronize();
        }
        hipMemcpy(h.data(), cyc, 8 * sizeof(long long), hipMemcpyDeviceToHost);
        std::sort(h.begin(), h.end());
        printf("%-40s %8.1f cycles\n", names[w], (double)h[4] / REP / per[w]);
    }
    return 0;
}
