// debug_hooks.hip -- test-only entry points (not part of include/pdplqr.h):
// device kernels exercised directly by the GPU unit tests
// (tests/test_gpu_combine.py).  Nothing in the solver path calls them.
#include "combine_mw.hpp"
#include "combine_qd.hpp"
#include "combine_qd1.hpp"
#include "combine_tiles.hpp"
#include "parallel.hpp"

// out = a (x) b on the device (one wave), elements in host memory; LU: the
// LU form of the combine (CondensedSystemSolverType::LU).
template <int T, bool LU>
__global__ __launch_bounds__(64) void k_debug_combine(const double *a, const double *b, double *out, int n, int *ok) {
    __shared__ pdplqr::CombSmem<T> sm;
    const bool good = pdplqr::tcombine<T, LU>(out, a, b, n, true, true, sm, threadIdx.x);
    if (threadIdx.x == 0) *ok = good ? 1 : 0;
}

extern "C" int pdplqr_debug_combine_form(int n, const double *a, const double *b, double *out, int lu) {
    using namespace pdplqr;
    const int T = n <= 16 ? 1 : (n <= 32 ? 2 : (n <= 64 ? 4 : 0));  // 4: the LDS kernels (kernels_wide.hip)
    if (!T) return PDPLQR_ERR_UNSUPPORTED;
    const size_t es = (size_t)(3 * n * n + 2 * n) * sizeof(double);
    double *d = nullptr;
    int *dok = nullptr, okh = 0;
    PDPLQR_HIP_TRY(hipMalloc(&d, 3 * es));
    PDPLQR_HIP_TRY(hipMalloc(&dok, sizeof(int)));
    PDPLQR_HIP_TRY(hipMemcpy(d, a, es, hipMemcpyHostToDevice));
    PDPLQR_HIP_TRY(hipMemcpy((char *)d + es, b, es, hipMemcpyHostToDevice));
    const double *da = d, *db = (const double *)((char *)d + es);
    double *dout = (double *)((char *)d + 2 * es);
    if (T == 4) {
        const int rc = launch_debug_combine_wide(da, db, dout, n, dok, lu != 0);
        if (rc) return rc;
    } else if (T == 1 && lu) hipLaunchKernelGGL((k_debug_combine<1, true>), dim3(1), dim3(64), 0, 0, da, db, dout, n, dok);
    else if (T == 1) hipLaunchKernelGGL((k_debug_combine<1, false>), dim3(1), dim3(64), 0, 0, da, db, dout, n, dok);
    else if (lu) hipLaunchKernelGGL((k_debug_combine<2, true>), dim3(1), dim3(64), 0, 0, da, db, dout, n, dok);
    else hipLaunchKernelGGL((k_debug_combine<2, false>), dim3(1), dim3(64), 0, 0, da, db, dout, n, dok);
    PDPLQR_HIP_TRY(hipDeviceSynchronize());
    PDPLQR_HIP_TRY(hipMemcpy(out, dout, es, hipMemcpyDeviceToHost));
    PDPLQR_HIP_TRY(hipMemcpy(&okh, dok, sizeof(int), hipMemcpyDeviceToHost));
    (void)hipFree(d);
    (void)hipFree(dok);
    return okh ? PDPLQR_OK : PDPLQR_ERR_NUMERIC;
}

// the 4-wave combine of the horizon scan (combine_mw.hpp); fcf = 0: only P, p
template <int T>
__global__ __launch_bounds__(256) void k_debug_combine_mw(const double *a, const double *b, double *out, int n, int fcf,
                                                          int *ok) {
    extern __shared__ __attribute__((aligned(16))) double mwbuf[];
    const pdplqr::MwSmem sm = pdplqr::mw_smem(mwbuf, n);
    const int nn = n * n, es = 3 * nn + 2 * n;
    // operands staged into LDS as the scan kernel does (mw_combine writes S
    // over the right operand's P block)
    const int own = (int)((pdplqr::mw_smem_bytes(n) + 15) / 16 * 2), slot = (es + 1) & ~1;
    double *la = mwbuf + own, *lb = la + slot;
    for (int q = threadIdx.x; q < es; q += blockDim.x) {
        la[q] = a[q];
        lb[q] = b[q];
    }
    __syncthreads();
    const bool good = pdplqr::mw_combine<T>(out, out + nn, out + 2 * nn, out + 2 * nn + n, out + 3 * nn + n,
                                            pdplqr::elem_in(la, n), pdplqr::elem_in(lb, n), n, fcf != 0, sm);
    if (threadIdx.x == 0) *ok = good ? 1 : 0;
}

extern "C" int pdplqr_debug_combine_mw(int n, const double *a, const double *b, double *out, int fcf) {
    using namespace pdplqr;
    const int T = n <= 16 ? 1 : (n <= 32 ? 2 : 0);
    if (!T) return PDPLQR_ERR_UNSUPPORTED;
    const size_t es = (size_t)(3 * n * n + 2 * n) * sizeof(double);
    double *d = nullptr;
    int *dok = nullptr, okh = 0;
    PDPLQR_HIP_TRY(hipMalloc(&d, 3 * es));
    PDPLQR_HIP_TRY(hipMalloc(&dok, sizeof(int)));
    PDPLQR_HIP_TRY(hipMemcpy(d, a, es, hipMemcpyHostToDevice));
    PDPLQR_HIP_TRY(hipMemcpy((char *)d + es, b, es, hipMemcpyHostToDevice));
    PDPLQR_HIP_TRY(hipMemcpy((char *)d + 2 * es, out, es, hipMemcpyHostToDevice));  // untouched blocks kept
    const double *da = d, *db = (const double *)((char *)d + es);
    double *dout = (double *)((char *)d + 2 * es);
    const size_t sm = (size_t)((mw_smem_bytes(n) + 15) / 16 * 2 + 2 * ((3 * n * n + 2 * n + 1) & ~1)) * sizeof(double);
    if (T == 1) hipLaunchKernelGGL(k_debug_combine_mw<1>, dim3(1), dim3(256), sm, 0, da, db, dout, n, fcf, dok);
    else hipLaunchKernelGGL(k_debug_combine_mw<2>, dim3(1), dim3(256), sm, 0, da, db, dout, n, fcf, dok);
    PDPLQR_HIP_TRY(hipDeviceSynchronize());
    PDPLQR_HIP_TRY(hipMemcpy(out, dout, es, hipMemcpyDeviceToHost));
    PDPLQR_HIP_TRY(hipMemcpy(&okh, dok, sizeof(int), hipMemcpyDeviceToHost));
    (void)hipFree(d);
    (void)hipFree(dok);
    return okh ? PDPLQR_OK : PDPLQR_ERR_NUMERIC;
}

// the n = 24 blocked-LDL^T combine of the horizon kernels (combine_qd.hpp)
__global__ __launch_bounds__(256) void k_debug_combine_qd(const double *a, const double *b, double *out, int fcf,
                                                          int *ok) {
    extern __shared__ __attribute__((aligned(16))) double qbuf[];
    constexpr int n = pdplqr::QD_N, nn = n * n, es = 3 * nn + 2 * n, slot = (es + 1) & ~1;
    double *la = qbuf + pdplqr::qd_smem_doubles() + 2, *lb = la + slot;  // 16-byte aligned
    for (int q = threadIdx.x; q < es; q += blockDim.x) {
        la[q] = a[q];
        lb[q] = b[q];
    }
    __syncthreads();
    const bool good = pdplqr::qd_combine(out, out + nn, out + 2 * nn, out + 2 * nn + n, out + 3 * nn + n,
                                         pdplqr::elem_in(la, n), pdplqr::elem_in(lb, n), fcf != 0, qbuf);
    if (threadIdx.x == 0) *ok = good ? 1 : 0;
}

extern "C" int pdplqr_debug_combine_qd(const double *a, const double *b, double *out, int fcf) {
    using namespace pdplqr;
    constexpr int n = QD_N;
    const size_t es = (size_t)(3 * n * n + 2 * n) * sizeof(double);
    double *d = nullptr;
    int *dok = nullptr, okh = 0;
    PDPLQR_HIP_TRY(hipMalloc(&d, 3 * es));
    PDPLQR_HIP_TRY(hipMalloc(&dok, sizeof(int)));
    PDPLQR_HIP_TRY(hipMemcpy(d, a, es, hipMemcpyHostToDevice));
    PDPLQR_HIP_TRY(hipMemcpy((char *)d + es, b, es, hipMemcpyHostToDevice));
    PDPLQR_HIP_TRY(hipMemcpy((char *)d + 2 * es, out, es, hipMemcpyHostToDevice));  // untouched blocks kept
    const double *da = d, *db = (const double *)((char *)d + es);
    double *dout = (double *)((char *)d + 2 * es);
    const size_t sm = (size_t)(qd_smem_doubles() + 2 + 2 * ((3 * n * n + 2 * n + 1) & ~1)) * sizeof(double);
    hipLaunchKernelGGL(k_debug_combine_qd, dim3(1), dim3(256), sm, 0, da, db, dout, fcf, dok);
    PDPLQR_HIP_TRY(hipDeviceSynchronize());
    PDPLQR_HIP_TRY(hipMemcpy(out, dout, es, hipMemcpyDeviceToHost));
    PDPLQR_HIP_TRY(hipMemcpy(&okh, dok, sizeof(int), hipMemcpyDeviceToHost));
    (void)hipFree(d);
    (void)hipFree(dok);
    return okh ? PDPLQR_OK : PDPLQR_ERR_NUMERIC;
}

extern "C" int pdplqr_debug_combine(int n, const double *a, const double *b, double *out) {
    return pdplqr_debug_combine_form(n, a, b, out, 0);
}


// Raw v_rsq_f64 (no Newton refinement) over an array: the accuracy that
// decides how many Newton steps rsqrt_f64 needs.
__global__ void k_debug_rsq(const double *x, double *y, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = __builtin_amdgcn_rsq(x[i]);
}

extern "C" int pdplqr_debug_rsq(int n, const double *x, double *y) {
    double *d = nullptr;
    PDPLQR_HIP_TRY(hipMalloc(&d, 2 * (size_t)n * sizeof(double)));
    PDPLQR_HIP_TRY(hipMemcpy(d, x, (size_t)n * sizeof(double), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_debug_rsq, dim3((n + 255) / 256), dim3(256), 0, 0, d, d + n, n);
    PDPLQR_HIP_TRY(hipDeviceSynchronize());
    PDPLQR_HIP_TRY(hipMemcpy(y, d + n, (size_t)n * sizeof(double), hipMemcpyDeviceToHost));
    (void)hipFree(d);
    return PDPLQR_OK;
}

// rsqrt_f64 (device_common.hpp) over an array: the refined reciprocal square root.
__global__ void k_debug_rsqrt(const double *x, double *y, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = pdplqr::rsqrt_f64(x[i]);
}

extern "C" int pdplqr_debug_rsqrt(int n, const double *x, double *y) {
    double *d = nullptr;
    PDPLQR_HIP_TRY(hipMalloc(&d, 2 * (size_t)n * sizeof(double)));
    PDPLQR_HIP_TRY(hipMemcpy(d, x, (size_t)n * sizeof(double), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_debug_rsqrt, dim3((n + 255) / 256), dim3(256), 0, 0, d, d + n, n);
    PDPLQR_HIP_TRY(hipDeviceSynchronize());
    PDPLQR_HIP_TRY(hipMemcpy(y, d + n, (size_t)n * sizeof(double), hipMemcpyDeviceToHost));
    (void)hipFree(d);
    return PDPLQR_OK;
}

// Host-side plan of the rank-fold trees (parallel.hpp rank_tree_op, the
// indexing k_rank_tree_mw runs): out[6] = {suf, carry, fcf, a, b, dst} of
// block q at `level` for rank r of R; returns the block count of that level
// (tests/test_rank_tree_plan.py simulates the trees on CPU with it).
extern "C" int pdplqr_debug_rank_tree(int R, int r, int level, int q, int *out) {
    const int per = pdplqr::rank_tree_blocks(r, level) + pdplqr::rank_tree_blocks(R - 1 - r, level);
    if (q >= 0 && q < per && out) {
        const pdplqr::RankTreeOp op = pdplqr::rank_tree_op(R, r, level, q);
        out[0] = op.suf;
        out[1] = op.carry;
        out[2] = op.fcf;
        out[3] = op.a;
        out[4] = op.b;
        out[5] = op.dst;
    }
    return per;
}

// Test hook (CPU, no device): the suffix-scan round plan of scan_round_operands
// (the block -> (i, j) indexing k_seg_scan / k_seg_scan_mw run): out[2] = {i, j}
// of block q in the round of distance `dist`, form sk; returns the block count
// of the round and -1 in out[0] when block q has nothing to do
// (tests/test_rank_tree_plan.py simulates the Sklansky rounds with it).
extern "C" int pdplqr_debug_scan_round(int S, int dist, int sk, int q, int *out) {
    const int per = pdplqr::scan_round_blocks(S, dist, sk);
    if (q >= 0 && q < per && out) {
        int i = -1, j = -1;
        if (!pdplqr::scan_round_operands(S, dist, sk, q, i, j)) i = -1;
        out[0] = i;
        out[1] = j;
    }
    return per;
}

// Test hook: the one-wave n <= 12 junction-LDL^T combine (combine_qd1.hpp) of
// two elements [F | C | f | P | p] (column-major blocks); returns
// PDPLQR_ERR_NUMERIC when a pivot has the wrong sign.
template <int NN>
__global__ __launch_bounds__(64) void k_debug_combine_qd1(const double *a, const double *b, double *out, int fcf,
                                                         int *ok) {
    __shared__ __attribute__((aligned(16))) double qs[pdplqr::Qd1<NN>::smem];
    constexpr int n = NN, nn = n * n, es = 3 * nn + 2 * n;
    __shared__ __attribute__((aligned(16))) double la[es + 1], lb[es + 1];
    for (int q = threadIdx.x; q < es; q += 64) {
        la[q] = a[q];
        lb[q] = b[q];
    }
    pdplqr::wave_sync();
    const bool good = pdplqr::qd1_combine<NN>(out, out + nn, out + 2 * nn, out + 2 * nn + n, out + 3 * nn + n,
                                              pdplqr::elem_in(la, n), pdplqr::elem_in(lb, n), fcf != 0, qs,
                                              threadIdx.x);
    if (threadIdx.x == 0) *ok = good ? 1 : 0;
}

extern "C" int pdplqr_debug_combine_qd1(int n, const double *a, const double *b, double *out, int fcf) {
    using namespace pdplqr;
    if (n != 4 && n != 8 && n != 12) return PDPLQR_ERR_INVALID;
    const size_t es = (size_t)(3 * n * n + 2 * n) * sizeof(double);
    double *d = nullptr;
    int *dok = nullptr, okh = 0;
    PDPLQR_HIP_TRY(hipMalloc(&d, 3 * es));
    PDPLQR_HIP_TRY(hipMalloc(&dok, sizeof(int)));
    PDPLQR_HIP_TRY(hipMemcpy(d, a, es, hipMemcpyHostToDevice));
    PDPLQR_HIP_TRY(hipMemcpy((char *)d + es, b, es, hipMemcpyHostToDevice));
    PDPLQR_HIP_TRY(hipMemcpy((char *)d + 2 * es, out, es, hipMemcpyHostToDevice));  // untouched blocks kept
    const double *da = d, *db = (const double *)((char *)d + es);
    double *dout = (double *)((char *)d + 2 * es);
    if (n == 4) hipLaunchKernelGGL(k_debug_combine_qd1<4>, dim3(1), dim3(64), 0, 0, da, db, dout, fcf, dok);
    else if (n == 8) hipLaunchKernelGGL(k_debug_combine_qd1<8>, dim3(1), dim3(64), 0, 0, da, db, dout, fcf, dok);
    else hipLaunchKernelGGL(k_debug_combine_qd1<12>, dim3(1), dim3(64), 0, 0, da, db, dout, fcf, dok);
    PDPLQR_HIP_TRY(hipDeviceSynchronize());
    PDPLQR_HIP_TRY(hipMemcpy(out, dout, es, hipMemcpyDeviceToHost));
    PDPLQR_HIP_TRY(hipMemcpy(&okh, dok, sizeof(int), hipMemcpyDeviceToHost));
    (void)hipFree(d);
    (void)hipFree(dok);
    return okh ? PDPLQR_OK : PDPLQR_ERR_NUMERIC;
}

// Test hook (CPU, no device): the boundary-map composition radix map_radix
// picks for n-state maps over J = S + 1 entries (tests/test_rank_tree_plan.py).
extern "C" int pdplqr_debug_map_radix(int n, int J) { return pdplqr::map_radix(n, J); }
