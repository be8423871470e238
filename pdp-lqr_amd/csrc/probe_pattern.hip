// Bench-only probe (libpdplqr_probe.so, not part of the C ABI in pdplqr.h):
// the HBM access pattern of the serial solver's streamed kernels with no
// arithmetic on the chain.  One wave per problem walks N stage records of
// three arrays (problem-major [b][N][rec], as the boundary and workspace lay
// them out), four stages of loads in flight, and writes one small record per
// stage.  Its time is the ceiling the backward / rollout kernels' data flow
// allows on the box: bench.py reports each kernel's time against it
// (scripts/ubench/stream_layout.hip sweeps layouts, depths and store kinds:
// none of them moves this ceiling, profiles/r02/stream_*.log).
#include <hip/hip_runtime.h>

namespace {

constexpr int kDepth = 4;

__global__ __launch_bounds__(256) void k_probe_pattern(const double2 *__restrict__ a0, int r0,
                                                       const double2 *__restrict__ a1, int r1,
                                                       const double2 *__restrict__ a2, int r2,
                                                       double2 *__restrict__ w, int rw, int P, int N,
                                                       double *__restrict__ sink) {
    const int p = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
    if (p >= P) return;
    const size_t base = (size_t)p * N;
    double2 buf[kDepth][6];
    // record j of stage k of array a with r chunks per stage; lanes past the
    // record re-read its last chunk (clamped: no exec-masked loads)
    auto load = [&](int d, int k) {
        k = k < N - 1 ? k : N - 1;
        const size_t s = base + k;
        buf[d][0] = a0[s * r0 + min(l, r0 - 1)];
        buf[d][1] = a0[s * r0 + min(l + 64, r0 - 1)];
        buf[d][2] = a1[s * r1 + min(l, r1 - 1)];
        buf[d][3] = a1[s * r1 + min(l + 64, r1 - 1)];
        buf[d][4] = a2[s * r2 + min(l, r2 - 1)];
        buf[d][5] = a2[s * r2 + min(l + 64, r2 - 1)];
    };
#pragma unroll
    for (int d = 0; d < kDepth; ++d) load(d, d);
    double acc = 0.0;
    for (int k = 0; k < N; k += kDepth) {
#pragma unroll
        for (int d = 0; d < kDepth; ++d) {
#pragma unroll
            for (int i = 0; i < 6; ++i) acc += buf[d][i].x * buf[d][i].y;
            if (l < rw && k + d < N) w[(base + k + d) * rw + l] = make_double2(acc, (double)k);
            load(d, k + kDepth + d);
        }
    }
    if (acc == 1234.5) sink[0] = acc;  // keeps the loads live
}

// Streaming copy with 16-byte loads / stores (the guide's float4 copy, 6.29
// TB/s measured): every thread keeps four loads in flight, grid-stride over
// the buffer.  The achievable-HBM reference the roofline lines quote beside the
// 8 TB/s spec (torch's copy_ runs the runtime's blit kernel instead).
__global__ __launch_bounds__(256) void k_probe_copy(const double2 *__restrict__ a, double2 *__restrict__ b,
                                                    size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const double2 v0 = a[i], v1 = a[i + stride], v2 = a[i + 2 * stride], v3 = a[i + 3 * stride];
        b[i] = v0;
        b[i + stride] = v1;
        b[i + 2 * stride] = v2;
        b[i + 3 * stride] = v3;
    }
    for (; i < n; i += stride) b[i] = a[i];
}

// Variants of the same copy (bench.py reports the best; scripts/copy_sweep.py):
//   mode 1: one 16-byte element per thread, a grid that covers the buffer once;
//   mode 2: four consecutive 16-byte elements per thread (64 B), grid covers once;
//   mode 3: mode 2 with non-temporal loads and stores (streamed once, no reuse).
template <int MODE>
__global__ __launch_bounds__(256) void k_probe_copy_v(const double2 *__restrict__ a, double2 *__restrict__ b,
                                                      size_t n) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if constexpr (MODE == 1) {
        if (t < n) b[t] = a[t];
    } else {
        const size_t i = 4 * t;
        if (i + 3 < n) {
            double2 v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if constexpr (MODE == 3) {
                    v[k].x = __builtin_nontemporal_load(&a[i + k].x);
                    v[k].y = __builtin_nontemporal_load(&a[i + k].y);
                } else {
                    v[k] = a[i + k];
                }
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if constexpr (MODE == 3) {
                    __builtin_nontemporal_store(v[k].x, &b[i + k].x);
                    __builtin_nontemporal_store(v[k].y, &b[i + k].y);
                } else {
                    b[i + k] = v[k];
                }
            }
        } else {
            for (size_t j = i; j < n; ++j) b[j] = a[j];
        }
    }
}

}  // namespace

// The copy variants above (mode 1..3; mode 0 = pdplqr_probe_copy's grid-stride
// form with `blocks` blocks).  Returns 0 or a hipError_t.
extern "C" int pdplqr_probe_copy_mode(const void *src, void *dst, size_t nbytes, int mode, int blocks, void *stream) {
    if (nbytes % 16) return (int)hipErrorInvalidValue;
    const size_t n = nbytes / 16;
    const hipStream_t st = (hipStream_t)stream;
    const double2 *a = (const double2 *)src;
    double2 *b = (double2 *)dst;
    if (mode == 0) {
        if (blocks < 1) return (int)hipErrorInvalidValue;
        hipLaunchKernelGGL(k_probe_copy, dim3(blocks), dim3(256), 0, st, a, b, n);
    } else if (mode == 1) {
        hipLaunchKernelGGL(k_probe_copy_v<1>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a, b, n);
    } else if (mode == 2 || mode == 3) {
        const size_t th = (n + 3) / 4;
        if (mode == 2) hipLaunchKernelGGL(k_probe_copy_v<2>, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, st, a, b, n);
        else hipLaunchKernelGGL(k_probe_copy_v<3>, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, st, a, b, n);
    } else {
        return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

// 16-byte streaming copy of nbytes (a multiple of 16); returns 0 or a hipError_t.
extern "C" int pdplqr_probe_copy(const void *src, void *dst, size_t nbytes, int blocks, void *stream) {
    if (nbytes % 16 || blocks < 1) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(k_probe_copy, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const double2 *)src,
                       (double2 *)dst, nbytes / 16);
    return (int)hipGetLastError();
}

// Chunks are 16 bytes; r0, r1, r2 in [1, 128], rw in [0, 64].  Returns 0 or a
// hipError_t.  Buffers hold P * N records of their size.
extern "C" int pdplqr_probe_pattern(const void *a0, int r0, const void *a1, int r1, const void *a2, int r2, void *w,
                                    int rw, int P, int N, void *sink, void *stream) {
    if (r0 < 1 || r0 > 128 || r1 < 1 || r1 > 128 || r2 < 1 || r2 > 128 || rw < 0 || rw > 64 || P < 1 || N < 1)
        return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(k_probe_pattern, dim3((P + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                       (const double2 *)a0, r0, (const double2 *)a1, r1, (const double2 *)a2, r2, (double2 *)w, rw, P,
                       N, (double *)sink);
    return (int)hipGetLastError();
}
