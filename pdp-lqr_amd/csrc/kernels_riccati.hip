// kernels_riccati.hip -- batched serial square-root Riccati on MI355X (gfx950).
//
// Restates LQRSolver (reference include/clqr/lqr/lqr_solver.hpp:41-77) and
// LQRKernel (lqr_kernel.hpp:80-212) for `batch` independent problems:
//   * k_update_problem_data: lqr_solver.hpp:41-56 (memory-bound elementwise)
//   * k_penalty:             the rho D^T D / D^T rho g preamble of every kernel
//                            step (lqr_kernel.hpp:82-88,106-112); independent
//                            across stages, so it runs as one parallel pass
//   * k_riccati_bwd<T>:      terminal_step_with_factorization + the backward
//                            recursion of step_with_factorization (:80-147)
//   * k_riccati_bwd_nofact:  the *_without_factorization recursion (:94-101,150-178)
//   * k_riccati_fwd:         forward_step (:181-212) as u = K x + d, x+ = c + A x + B u
//
// Backward mapping: ONE wavefront per problem.  Stage matrices live in the
// f64 MFMA C/D layout (v_mfma_f64_16x16x4_f64: lane l = 16 g + c holds rows
// g, g+4, g+8, g+12 of column c of a 16x16 tile, one register per row group).
// With P = 16 T the padded stage size (u at 0..m-1, x at m..s-1, identity on
// the padding), each stage is
//     W = Lxx_next^T E          (MFMA, A operand = L_next read from LDS)
//     M = H~ + W^T W            (MFMA, both operands = W's registers, no data movement)
//     L = chol(M)               (right-looking, column broadcast through LDS)
// i.e. M = H~ + V V^T with V = E^T Lxx_next exactly as lqr_kernel.hpp:121-126.
#include "internal.hpp"

namespace pdplqr {

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ d4 mfma_f64(double a, double b, d4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// packed lower (column-major) index of (i, j), i >= j, dimension d
__device__ __forceinline__ int pidx(int i, int j, int d) { return j * d - ((j * (j - 1)) >> 1) + (i - j); }

__device__ __forceinline__ double shfl_xor_f64(double v, int mask) { return __shfl_xor(v, mask, 64); }

// ---------------------------------------------------------------------------
// update_problem_data (lqr_solver.hpp:41-56)
// ---------------------------------------------------------------------------
__global__ void k_update_problem_data(Shape sh, const double *__restrict__ H, const double *__restrict__ hv,
                                      const double *__restrict__ ws, const double *__restrict__ ys,
                                      const double *__restrict__ zs, const double *__restrict__ irho,
                                      double sigma, double *__restrict__ Hw, double *__restrict__ hw,
                                      double *__restrict__ gw, const short2 *__restrict__ tab_s,
                                      const short2 *__restrict__ tab_n) {
    const long long totH = sh.perHw * sh.batch, toth = sh.perh * sh.batch, totg = (long long)sh.ny * sh.batch;
    const long long total = totH + toth + totg;
    const long long stepg = (long long)gridDim.x * blockDim.x;
    const int s = sh.s;
    for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stepg) {
        if (t < totH) {
            const long long b = t / sh.perHw;
            const long long r = t - b * sh.perHw;
            const double *Hb = H + b * sh.perH;
            int i, j;
            double v;
            if (r < (long long)sh.N * sh.ps) {
                const int k = (int)(r / sh.ps), q = (int)(r - (long long)k * sh.ps);
                const short2 ij = tab_s[q];
                i = ij.x; j = ij.y;
                v = Hb[(long long)k * s * s + i + j * s];
            } else {
                const int q = (int)(r - (long long)sh.N * sh.ps);
                const short2 ij = tab_n[q];
                i = ij.x; j = ij.y;
                v = Hb[(long long)sh.N * s * s + i + j * sh.n];
            }
            Hw[t] = (i == j) ? v + sigma : v;
        } else if (t < totH + toth) {
            const long long u = t - totH;
            hw[u] = hv[u] - sigma * ws[u];
        } else {
            const long long u = t - totH - toth;
            gw[u] = zs[u] - irho[u] * ys[u];
        }
    }
}

int launch_update_problem_data(const Shape &sh, const double *H, const double *hv, const double *ws,
                               const double *ys, const double *zs, const double *irho, double sigma, double *Hw,
                               double *hw, double *gw, const short2 *tab_s, const short2 *tab_n,
                               hipStream_t st) {
    const long long total = (sh.perHw + sh.perh + sh.ny) * (long long)sh.batch;
    const int threads = 256;
    long long blocks = (total + threads - 1) / threads;
    if (blocks > 8192) blocks = 8192;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_update_problem_data, dim3((unsigned)blocks), dim3(threads), 0, st, sh, H, hv, ws, ys, zs,
                       irho, sigma, Hw, hw, gw, tab_s, tab_n);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

// ---------------------------------------------------------------------------
// rho penalty: H~ += D^T diag(rho) D ; h~ -= D^T (rho o g)   (lqr_kernel.hpp:82-88)
// ---------------------------------------------------------------------------
__global__ void k_penalty(Shape sh, const double *__restrict__ D, const double *__restrict__ rho,
                          const double *__restrict__ gw, double *__restrict__ Hw, double *__restrict__ hw,
                          const int32_t *__restrict__ d_off, const int32_t *__restrict__ y_off,
                          const short2 *__restrict__ tab_s, const short2 *__restrict__ tab_n, int with_H) {
    // one thread per (b, k, packed entry) for H, then per (b, k, i) for h
    const long long totH = with_H ? sh.perHw * sh.batch : 0;
    const long long toth = sh.perh * sh.batch;
    const long long stepg = (long long)gridDim.x * blockDim.x;
    const int s = sh.s, n = sh.n, N = sh.N;
    for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < totH + toth; t += stepg) {
        if (t < totH) {
            const long long b = t / sh.perHw;
            const long long r = t - b * sh.perHw;
            int k, i, j;
            if (r < (long long)N * sh.ps) {
                k = (int)(r / sh.ps);
                const short2 ij = tab_s[(int)(r - (long long)k * sh.ps)];
                i = ij.x; j = ij.y;
            } else {
                k = N;
                const short2 ij = tab_n[(int)(r - (long long)N * sh.ps)];
                i = ij.x; j = ij.y;
            }
            const int nc = y_off[k + 1] - y_off[k];
            if (nc == 0) continue;
            const double *Dk = D + b * sh.ndD + d_off[k];
            const double *rk = rho + b * sh.ny + y_off[k];
            double a = 0.0;
            for (int q = 0; q < nc; ++q) a += Dk[q + i * nc] * (rk[q] * Dk[q + j * nc]);
            Hw[t] += a;
        } else {
            const long long u = t - totH;
            const long long b = u / sh.perh;
            const int r = (int)(u - b * sh.perh);
            const int k = r < N * s ? r / s : N;
            const int i = r < N * s ? r - k * s : r - N * s;
            const int nc = y_off[k + 1] - y_off[k];
            if (nc == 0) continue;
            const double *Dk = D + b * sh.ndD + d_off[k];
            const double *rk = rho + b * sh.ny + y_off[k];
            const double *gk = gw + b * sh.ny + y_off[k];
            double a = 0.0;
            for (int q = 0; q < nc; ++q) a += Dk[q + i * nc] * (rk[q] * gk[q]);
            hw[u] -= a;
        }
    }
    (void)n;
}

int launch_penalty(const Shape &sh, const double *D, const double *rho, const double *gw, double *Hw,
                   double *hw, const int32_t *d_off, const int32_t *y_off, const short2 *tab_s,
                   const short2 *tab_n, int with_H, int max_nc, hipStream_t st) {
    if (max_nc <= 0) return PDPLQR_OK;
    const long long total = ((with_H ? sh.perHw : 0) + sh.perh) * (long long)sh.batch;
    const int threads = 256;
    long long blocks = (total + threads - 1) / threads;
    if (blocks > 8192) blocks = 8192;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_penalty, dim3((unsigned)blocks), dim3(threads), 0, st, sh, D, rho, gw, Hw, hw, d_off,
                       y_off, tab_s, tab_n, with_H);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

// ---------------------------------------------------------------------------
// Backward with factorization: one wavefront per problem, f64 MFMA tiles.
// ---------------------------------------------------------------------------
// Loads the padded stage matrix H~ into C/D-layout tiles.  Indices in
// [lo, hi) map to the stored packed block (dimension dim, offset off);
// everything else is the identity padding.
template <int T>
__device__ __forceinline__ void load_M(d4 (&M)[T][T], const double *__restrict__ Hp, int dim, int off, int lo, int hi,
                                       int g, int c) {
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int b = 0; b < T; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * a + 4 * r + g, j = 16 * b + c;
                double v;
                if (i >= lo && i < hi && j >= lo && j < hi) {
                    const int ii = i - off, jj = j - off;
                    v = (ii >= jj) ? Hp[pidx(ii, jj, dim)] : Hp[pidx(jj, ii, dim)];
                } else {
                    v = (i == j) ? 1.0 : 0.0;
                }
                M[a][b][r] = v;
            }
}

// Wave-scope ordering of LDS traffic between lanes of ONE wavefront: LDS
// instructions of a wave retire in issue order, so a compiler-level barrier is
// all that is needed (no s_barrier; the workgroup is a single wave).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ double readlane_f64(double v, int lane) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}

// 1/sqrt(x): hardware estimate + two Newton steps (full fp64 accuracy).
__device__ __forceinline__ double rsqrt_f64(double x) {
    double r = __builtin_amdgcn_rsq(x);
    double e = __builtin_fma(-x * r, r, 1.0);
    r = __builtin_fma(0.5 * r, e, r);
    e = __builtin_fma(-x * r, r, 1.0);
    return __builtin_fma(0.5 * r, e, r);
}

// Stage-k inputs of one lane, loaded one stage ahead (register prefetch).
template <int T>
struct StageIn {
    double E[4 * T][T];  // MFMA B operand: E[4 cc + g][16 b + c]
    d4 H[T][T];          // MFMA C input: H~[16 a + 4 r + g][16 b + c] (padded)
    double c[4 * T];     // c[4 cc + g]
    double h[T];         // h~[16 b + c]
};

template <int T>
__device__ __forceinline__ void load_stage(StageIn<T> &in, const double *__restrict__ Ek, const double *__restrict__ ck,
                                           const double *__restrict__ Hk, const double *__restrict__ hk, int n,
                                           int s, int g, int c) {
#pragma unroll
    for (int cc = 0; cc < 4 * T; ++cc) {
        const int t = 4 * cc + g;
#pragma unroll
        for (int b = 0; b < T; ++b) {
            const int j = 16 * b + c;
            in.E[cc][b] = (t < n && j < s) ? Ek[t + j * n] : 0.0;
        }
        in.c[cc] = (t < n) ? ck[t] : 0.0;
    }
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int b = 0; b < T; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * a + 4 * r + g, j = 16 * b + c;
                double v;
                if (i < s && j < s)
                    v = (i >= j) ? Hk[pidx(i, j, s)] : Hk[pidx(j, i, s)];
                else
                    v = (i == j) ? 1.0 : 0.0;
                in.H[a][b][r] = v;
            }
#pragma unroll
    for (int b = 0; b < T; ++b) {
        const int j = 16 * b + c;
        in.h[b] = (j < s) ? hk[j] : 0.0;
    }
}

// Right-looking Cholesky of the symmetric padded matrix in C/D layout, pivots
// jbeg..jend-1.  Column j is broadcast through LDS from row j (the row group
// that owns row j holds M[j][*] = M[*][j]; M stays exactly symmetric because
// every update is applied to both triangles with the same products).  The
// owners write zeros for columns <= j, so every lane can update
// M -= raw_i raw_k / M[j][j] without masking; the pivot column itself is left
// unscaled and finalised by finalize_L (L[i][j] = M[i][j] / sqrt(M[j][j])).
// With `aug`, the first `m` pivots also eliminate the linear column lpr (the
// lp_k of lqr_kernel.hpp:142-146): lpr_i -= l_ij lu'_j with lu'_j = lp_j / L_jj,
// which is exactly lu <- Luu^{-1} lu followed by p -= Lxu lu.  All lanes of the
// wave run in lock step and LDS ops of one wave retire in order, so no barrier
// is needed between the owners' writes and the readers.
template <int T>
__device__ __forceinline__ int chol_tiles(d4 (&M)[T][T], double (&myinv)[T], double (&lpr)[T][4], double *cb,
                                          double *luq, int jbeg, int jend, int m, bool aug, int g, int c) {
    int fail = -1;
    const bool lane0 = (g == 0) && (c == 0);
#pragma unroll
    for (int j = 0; j < 16 * T; ++j) {
        if (j >= jbeg && j < jend) {
            const int tr = j >> 4, rr = (j >> 2) & 3, gj = j & 3, bj = j >> 4, cj = j & 15;
            if (g == gj) {
#pragma unroll
                for (int b = 0; b < T; ++b) {
                    const int jc = 16 * b + c;
                    cb[jc] = (jc > j) ? M[tr][b][rr] : 0.0;
                }
            }
            wave_sync();
            const double djj = readlane_f64(M[tr][bj][rr], (gj << 4) + cj);
            if (!(djj > 0.0) && fail < 0) fail = j;
            const double inv = rsqrt_f64(djj);
            const double inv2 = inv * inv;
            if (c == cj) myinv[bj] = inv;
            double lc[T];
#pragma unroll
            for (int b = 0; b < T; ++b) lc[b] = cb[16 * b + c] * inv2;
            const bool augj = aug && j < m;
            const double lpj = augj ? readlane_f64(lpr[tr][rr], gj << 4) : 0.0;
            const double qj = lpj * inv2;
#pragma unroll
            for (int a = 0; a < T; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const double li = cb[16 * a + 4 * r + g];
#pragma unroll
                    for (int b = 0; b < T; ++b) M[a][b][r] = __builtin_fma(-li, lc[b], M[a][b][r]);
                    // q = lp_j / M[j][j]; lpr_i -= raw_i * q  (raw_i = 0 for i <= j)
                    if (augj) lpr[a][r] = __builtin_fma(-li, qj, lpr[a][r]);
                }
            if (augj && lane0) luq[j] = lpj * inv;
            wave_sync();
        }
    }
    return fail;
}

// L[i][jc] = M[i][jc] / sqrt(M[jc][jc]) below the diagonal, 0 above, for the
// factored columns jc < jend; identity padding elsewhere is left as is.
template <int T>
__device__ __forceinline__ void finalize_L(d4 (&M)[T][T], const double (&myinv)[T], int jbeg, int jend, int g,
                                           int c) {
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int b = 0; b < T; ++b) {
            const int jc = 16 * b + c;
            if (jc >= jbeg && jc < jend) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * a + 4 * r + g;
                    M[a][b][r] = (i >= jc) ? M[a][b][r] * myinv[b] : 0.0;
                }
            }
        }
}

template <int T>
struct BwdSmem {
    static constexpr int P = 16 * T;
    static constexpr int LD = P + 1;  // odd leading dimension: conflict-free column reads
    double L[P * LD];                 // L_{k+1} then L_k (padded, column-major, lower, zero upper)
    double col[P];                    // Cholesky column broadcast
    double pbt[P];                    // Pb_tmp = Lxx_next^T c
    double pv[P];                     // p_{k+1}, then p_k
    double lp[P];                     // lp_k (column -> row redistribution)
    double luq[P];                    // lu'_k = Luu^{-1} lu
};

template <int T>
__device__ __forceinline__ void store_L_lds(const d4 (&M)[T][T], double *L, int g, int c) {
    constexpr int LD = 16 * T + 1;
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int b = 0; b < T; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) L[(16 * a + 4 * r + g) + (16 * b + c) * LD] = M[a][b][r];
}

// Per-stage rollout record FR_k = [L(:, 0:m) (s x m, column-major) | lu'_k (m)]:
// exactly what LQRKernel::forward_step reads (Luu, Lxu, lu; lqr_kernel.hpp:190-198).
#ifndef PDPLQR_BWD_WAVES
#define PDPLQR_BWD_WAVES 4  // waves per SIMD for T = 1: 16 problems per CU fit in one residency round
#endif
template <int T>
__global__ __launch_bounds__(64, (T == 1 ? PDPLQR_BWD_WAVES : 1)) void k_riccati_bwd(RiccatiArgs A) {
    constexpr int P = 16 * T, LD = P + 1;
    __shared__ BwdSmem<T> sm;
    const int lane = threadIdx.x, g = lane >> 4, c = lane & 15;
    const long long b = blockIdx.x;
    const Shape &sh = A.sh;
    const int n = sh.n, m = sh.m, N = sh.N, s = sh.s;
    const int nch = (n + 3) >> 2;
    const long long frs = (long long)s * m + m;
    const double *Eb = A.E + b * sh.perE;
    const double *cb = A.c + b * sh.perc;
    const double *Hb = A.Hw + b * sh.perHw;
    const double *hb = A.hw + b * sh.perh;
    double *FRb = A.KD + b * sh.perKD;
    double *Lcb = A.Lc ? A.Lc + b * sh.perHw : nullptr;
    double *lpb = A.lpc ? A.lpc + b * sh.perh : nullptr;
    int fail_stage = -1;

    // ---- terminal: L_N = chol(H~_N), lp_N = h~_N  (lqr_kernel.hpp:80-91) ----
    {
        d4 M[T][T];
        load_M<T>(M, Hb + (long long)N * sh.ps, n, m, m, s, g, c);
        double myinv[T], lpr[T][4];
#pragma unroll
        for (int q = 0; q < T; ++q) myinv[q] = 1.0;
        const int f = chol_tiles<T>(M, myinv, lpr, sm.col, sm.luq, m, s, m, false, g, c);
        finalize_L<T>(M, myinv, m, s, g, c);
        if (f >= 0) fail_stage = N;
        store_L_lds<T>(M, sm.L, g, c);
        if (lane < n) {
            const double v = hb[(long long)N * s + lane];
            sm.pv[lane] = v;
            if (lpb) lpb[(long long)N * s + lane] = v;
        }
        if (Lcb)
#pragma unroll
            for (int a = 0; a < T; ++a)
#pragma unroll
                for (int bt = 0; bt < T; ++bt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int i = 16 * a + 4 * r + g, j = 16 * bt + c;
                        if (j >= m && i >= j && i < s)
                            Lcb[(long long)N * sh.ps + pidx(i - m, j - m, n)] = M[a][bt][r];
                    }
        wave_sync();
    }

    StageIn<T> cur;
    load_stage<T>(cur, Eb + (long long)(N - 1) * n * s, cb + (long long)(N - 1) * n, Hb + (long long)(N - 1) * sh.ps,
                  hb + (long long)(N - 1) * s, n, s, g, c);
    for (int k = N - 1; k >= 0; --k) {
        StageIn<T> nxt;
        if (k > 0)
            load_stage<T>(nxt, Eb + (long long)(k - 1) * n * s, cb + (long long)(k - 1) * n,
                          Hb + (long long)(k - 1) * sh.ps, hb + (long long)(k - 1) * s, n, s, g, c);
        // ---- A operand: Lxx_next^T, read from LDS (L_{k+1}) ----
        double av[4 * T][T];
#pragma unroll
        for (int cc = 0; cc < 4 * T; ++cc) {
            const int t = 4 * cc + g;
#pragma unroll
            for (int a = 0; a < T; ++a) {
                const int tp = 16 * a + c;
                av[cc][a] = (cc < nch && t < n && tp < n) ? sm.L[(m + t) + (m + tp) * LD] : 0.0;
            }
        }
        // ---- W = Lxx_next^T E  (= V^T, V = E^T Lxx_next, lqr_kernel.hpp:121) ----
        d4 W[T][T];
#pragma unroll
        for (int a = 0; a < T; ++a)
#pragma unroll
            for (int bt = 0; bt < T; ++bt) W[a][bt] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int cc = 0; cc < 4 * T; ++cc)
            if (cc < nch)
#pragma unroll
                for (int a = 0; a < T; ++a)
#pragma unroll
                    for (int bt = 0; bt < T; ++bt) W[a][bt] = mfma_f64(av[cc][a], cur.E[cc][bt], W[a][bt]);
        // ---- Pb_tmp = Lxx_next^T c (lqr_kernel.hpp:138), reduced over row groups ----
#pragma unroll
        for (int a = 0; a < T; ++a) {
            double part = 0.0;
#pragma unroll
            for (int cc = 0; cc < 4 * T; ++cc)
                if (cc < nch) part = __builtin_fma(av[cc][a], cur.c[cc], part);
            part += shfl_xor_f64(part, 16);
            part += shfl_xor_f64(part, 32);
            if (g == 0) sm.pbt[16 * a + c] = part;
        }
        // ---- M = H~ + W^T W  (= H~ + V V^T, lqr_kernel.hpp:123-124) ----
        d4 M[T][T];
#pragma unroll
        for (int a = 0; a < T; ++a)
#pragma unroll
            for (int bt = 0; bt < T; ++bt) M[a][bt] = cur.H[a][bt];
#pragma unroll
        for (int kc = 0; kc < 4 * T; ++kc)
            if (kc < nch) {
                const int ka = kc >> 2, r = kc & 3;
#pragma unroll
                for (int a = 0; a < T; ++a)
#pragma unroll
                    for (int bt = 0; bt < T; ++bt) M[a][bt] = mfma_f64(W[ka][a][r], W[ka][bt][r], M[a][bt]);
            }
        // ---- lp = h~ + E^T (Lxx_next Pb_tmp + p_next) = h~ + W^T Pb_tmp + E^T p_next
        //      (lqr_kernel.hpp:139-143; E^T Lxx_next = W^T) ----
        wave_sync();
        double lpr[T][4];
        {
            double part[T];
#pragma unroll
            for (int bt = 0; bt < T; ++bt) part[bt] = 0.0;
#pragma unroll
            for (int kc = 0; kc < 4 * T; ++kc)
                if (kc < nch) {
                    const int t = 4 * kc + g;
                    const double pb = (t < n) ? sm.pbt[t] : 0.0;
                    const double pn = (t < n) ? sm.pv[t] : 0.0;
#pragma unroll
                    for (int bt = 0; bt < T; ++bt) {
                        part[bt] = __builtin_fma(W[kc >> 2][bt][kc & 3], pb, part[bt]);
                        part[bt] = __builtin_fma(cur.E[kc][bt], pn, part[bt]);
                    }
                }
#pragma unroll
            for (int bt = 0; bt < T; ++bt) {
                part[bt] += shfl_xor_f64(part[bt], 16);
                part[bt] += shfl_xor_f64(part[bt], 32);
                if (g == 0) sm.lp[16 * bt + c] = cur.h[bt] + part[bt];
            }
            wave_sync();
#pragma unroll
            for (int a = 0; a < T; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * a + 4 * r + g;
                    lpr[a][r] = (i < s) ? sm.lp[i] : 0.0;
                }
        }
        // ---- L = chol(M) (lqr_kernel.hpp:126) with lu <- Luu^{-1} lu, p -= Lxu lu (:145-146) ----
        double myinv[T];
#pragma unroll
        for (int q = 0; q < T; ++q) myinv[q] = 1.0;
        const int f = chol_tiles<T>(M, myinv, lpr, sm.col, sm.luq, 0, s, m, true, g, c);
        if (f >= 0 && fail_stage < 0) fail_stage = k;
        finalize_L<T>(M, myinv, 0, s, g, c);
        store_L_lds<T>(M, sm.L, g, c);
        // p_k -> LDS (next stage's p_next) and the factor cache
        if (c == 0) {
#pragma unroll
            for (int a = 0; a < T; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * a + 4 * r + g;
                    if (i >= m && i < s) {
                        sm.pv[i - m] = lpr[a][r];
                        if (lpb) lpb[(long long)k * s + i] = lpr[a][r];
                    }
                }
        }
        // rollout record: L(:, 0:m) and lu'
        double *FRk = FRb + (long long)k * frs;
#pragma unroll
        for (int a = 0; a < T; ++a)
#pragma unroll
            for (int bt = 0; bt < T; ++bt) {
                const int jc = 16 * bt + c;
                if (jc < m)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int i = 16 * a + 4 * r + g;
                        if (i < s) FRk[jc * s + i] = M[a][bt][r];
                    }
            }
        wave_sync();
        if (lane < m) {
            const double q = sm.luq[lane];
            FRk[(long long)s * m + lane] = q;
            if (lpb) lpb[(long long)k * s + lane] = q;
        }
        if (Lcb)
#pragma unroll
            for (int a = 0; a < T; ++a)
#pragma unroll
                for (int bt = 0; bt < T; ++bt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int i = 16 * a + 4 * r + g, j = 16 * bt + c;
                        if (i >= j && i < s) Lcb[(long long)k * sh.ps + pidx(i, j, s)] = M[a][bt][r];
                    }
        if (k > 0) cur = nxt;
    }
    if (lane == 0) A.status[b] = fail_stage < 0 ? 0 : fail_stage + 1;
}

int launch_riccati_backward(const RiccatiArgs &a, hipStream_t st) {
    if (a.sh.s <= 16) {
        hipLaunchKernelGGL(k_riccati_bwd<1>, dim3(a.sh.batch), dim3(64), 0, st, a);
    } else if (a.sh.s <= 32) {
        hipLaunchKernelGGL(k_riccati_bwd<2>, dim3(a.sh.batch), dim3(64), 0, st, a);
    } else {
        set_error("backward: n + m > 32 is not supported by this build");
        return PDPLQR_ERR_UNSUPPORTED;
    }
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

// ---------------------------------------------------------------------------
// Backward without factorization (lqr_kernel.hpp:94-101,150-178): only the
// linear terms, reusing the cached factors L_k (keep_factors).  One wavefront
// per problem; writes lp_k to the cache and lu'_k into the rollout record.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_riccati_bwd_nofact(RiccatiArgs A) {
    constexpr int P = 32;
    __shared__ double Lk[P * P];  // this stage's L (packed -> dense, column-major, ld = s)
    __shared__ double Ln[P * P];  // next stage's Lxx (ld = n)
    __shared__ double cvec[P], va[P], vb[P], lp[P], pn[P];
    const int lane = threadIdx.x;
    const long long b = blockIdx.x;
    const Shape &sh = A.sh;
    const int n = sh.n, m = sh.m, N = sh.N, s = sh.s;
    const long long frs = (long long)s * m + m;
    const double *Eb = A.E + b * sh.perE;
    const double *cb = A.c + b * sh.perc;
    const double *hb = A.hw + b * sh.perh;
    double *FRb = A.KD + b * sh.perKD;
    const double *Lcb = A.Lc + b * sh.perHw;
    double *lpb = A.lpc + b * sh.perh;
    // terminal (lqr_kernel.hpp:94-101): lp_N = h~_N ; Lxx_N from the cache
    if (lane < n) {
        const double v = hb[(long long)N * s + lane];
        pn[lane] = v;
        lpb[(long long)N * s + lane] = v;
    }
    for (int q = lane; q < sh.pn; q += 64) {
        const short2 ij = A.tab_n[q];
        const double v = Lcb[(long long)N * sh.ps + q];
        Ln[ij.x + ij.y * n] = v;
        if (ij.x != ij.y) Ln[ij.y + ij.x * n] = 0.0;
    }
    __syncthreads();
    for (int k = N - 1; k >= 0; --k) {
        const double *Ek = Eb + (long long)k * n * s;
        for (int q = lane; q < sh.ps; q += 64) {
            const short2 ij = A.tab_s[q];
            const double v = Lcb[(long long)k * sh.ps + q];
            Lk[ij.x + ij.y * s] = v;
            if (ij.x != ij.y) Lk[ij.y + ij.x * s] = 0.0;
        }
        if (lane < n) cvec[lane] = cb[(long long)k * n + lane];
        __syncthreads();
        if (lane < n) {  // Pb_tmp = Lxx_next^T c
            double a = 0.0;
            for (int t = lane; t < n; ++t) a += Ln[t + lane * n] * cvec[t];
            va[lane] = a;
        }
        __syncthreads();
        if (lane < n) {  // Pb = Lxx_next Pb_tmp + p_next
            double a = 0.0;
            for (int t = 0; t <= lane; ++t) a += Ln[lane + t * n] * va[t];
            vb[lane] = a + pn[lane];
        }
        __syncthreads();
        if (lane < s) {  // lp = h~ + E^T Pb
            double a = 0.0;
            for (int t = 0; t < n; ++t) a += Ek[t + lane * n] * vb[t];
            lp[lane] = hb[(long long)k * s + lane] + a;
        }
        __syncthreads();
        if (lane == 0) {  // lu <- Luu^{-1} lu
            for (int i = 0; i < m; ++i) {
                double v = lp[i];
                for (int j = 0; j < i; ++j) v -= Lk[i + j * s] * lp[j];
                lp[i] = v / Lk[i + i * s];
            }
        }
        __syncthreads();
        if (lane < n) {  // p -= Lxu lu
            double a = 0.0;
            for (int i = 0; i < m; ++i) a += Lk[(m + lane) + i * s] * lp[i];
            const double pnew = lp[m + lane] - a;
            lp[m + lane] = pnew;
            pn[lane] = pnew;
        }
        __syncthreads();
        if (lane < m) FRb[(long long)k * frs + (long long)s * m + lane] = lp[lane];
        if (lane < s) lpb[(long long)k * s + lane] = lp[lane];
        // the next iteration's Lxx_next is this stage's bottom-right block
        for (int q = lane; q < n * n; q += 64) {
            const int i = q % n, j = q / n;
            Ln[i + j * n] = Lk[(m + i) + (m + j) * s];
        }
        __syncthreads();
    }
}

int launch_riccati_backward_nofact(const RiccatiArgs &a, hipStream_t st) {
    if (a.sh.s > 32) {
        set_error("backward_without_factorization: n + m > 32 is not supported by this build");
        return PDPLQR_ERR_UNSUPPORTED;
    }
    hipLaunchKernelGGL(k_riccati_bwd_nofact, dim3(a.sh.batch), dim3(64), 0, st, a);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

// ---------------------------------------------------------------------------
// Forward rollout, LQRKernel::forward_step (lqr_kernel.hpp:181-212):
//     u = -Luu^{-T} (lu' + Lxu^T x) ;  x+ = c + A x + B u
// from the rollout record FR_k = [L(:, 0:m) | lu'_k].  One wavefront per
// problem; lane (g, cl) owns rows t = cl + 16 q (q < R) and the columns
// j = 4 jj + g of E, partial sums are reduced over the 4 row groups.  The
// next stage's data is prefetched into registers while this stage computes,
// so the recursion's latency hides under the HBM stream.
// ---------------------------------------------------------------------------
template <int R, int MM>
struct FwdIn {
    static constexpr int NJ = 4 * R;  // columns per lane: s <= 16 R
    double E[R][NJ];                  // E[cl + 16 q][4 jj + g]
    double c[R];                      // c[cl + 16 q]
    double lxu[NJ];                   // Lxu[4 qq + g][cl]  (lanes cl < m)
    double luu[MM];                   // Luu[i][cl], i < m  (lanes cl < m)
    double lu;                        // lu'[cl]
};

template <int R, int MM>
__device__ __forceinline__ void fwd_load(FwdIn<R, MM> &in, const double *__restrict__ Ek, const double *__restrict__ ck,
                                         const double *__restrict__ Fk, int n, int m, int s, int g, int cl) {
    constexpr int NJ = 4 * R;
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int t = cl + 16 * q;
#pragma unroll
        for (int jj = 0; jj < NJ; ++jj) {
            const int j = 4 * jj + g;
            in.E[q][jj] = (t < n && j < s) ? Ek[t + j * n] : 0.0;
        }
        in.c[q] = (t < n) ? ck[t] : 0.0;
    }
    const bool own = cl < m;
#pragma unroll
    for (int qq = 0; qq < NJ; ++qq) {
        const int t = 4 * qq + g;
        in.lxu[qq] = (own && t < n) ? Fk[cl * s + m + t] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < MM; ++i) in.luu[i] = (own && i < m) ? Fk[cl * s + i] : 0.0;
    in.lu = own ? Fk[s * m + cl] : 0.0;
}

template <int R, int MM>
__global__ __launch_bounds__(64) void k_riccati_fwd(Shape sh, const double *__restrict__ E,
                                                    const double *__restrict__ c, const double *__restrict__ FR,
                                                    const double *__restrict__ x0, double *__restrict__ ws) {
    constexpr int NJ = 4 * R;
    __shared__ double sw[64];  // w_k = [u; x]
    const int lane = threadIdx.x, g = lane >> 4, cl = lane & 15;
    const long long b = blockIdx.x;
    const int n = sh.n, m = sh.m, N = sh.N, s = sh.s;
    const long long frs = (long long)s * m + m;
    const double *Eb = E + b * sh.perE;
    const double *cb = c + b * sh.perc;
    const double *Fb = FR + b * sh.perKD;
    double *wb = ws + b * sh.perh;
    if (lane < n) {
        const double v = x0[b * n + lane];
        sw[m + lane] = v;
        wb[m + lane] = v;  // ws[0].tail(n) = x0 (lqr_solver.hpp:73)
    }
    wave_sync();
    FwdIn<R, MM> cur, nxt;
    fwd_load<R, MM>(cur, Eb, cb, Fb, n, m, s, g, cl);
    for (int k = 0; k < N; ++k) {
        if (k + 1 < N)
            fwd_load<R, MM>(nxt, Eb + (long long)(k + 1) * n * s, cb + (long long)(k + 1) * n,
                            Fb + (long long)(k + 1) * frs, n, m, s, g, cl);
        // v = lu' + Lxu^T x (lanes cl < m), x-part of E w
        double xv[NJ];
#pragma unroll
        for (int qq = 0; qq < NJ; ++qq) {
            const int t = 4 * qq + g;
            xv[qq] = (t < n) ? sw[m + t] : 0.0;
        }
        double v = 0.0;
#pragma unroll
        for (int qq = 0; qq < NJ; ++qq) v = __builtin_fma(cur.lxu[qq], xv[qq], v);
        v += shfl_xor_f64(v, 16);
        v += shfl_xor_f64(v, 32);
        v += cur.lu;
        double ax[R];
#pragma unroll
        for (int q = 0; q < R; ++q) {
            double a = 0.0;
#pragma unroll
            for (int jj = 0; jj < NJ; ++jj) {
                const int j = 4 * jj + g;
                if (j >= m && j < s) a = __builtin_fma(cur.E[q][jj], sw[j], a);
            }
            ax[q] = a;
        }
        // u = -Luu^{-T} v: back substitution, u_i broadcast from lane i
        double acc = 0.0, myu = 0.0;
#pragma unroll
        for (int i = MM - 1; i >= 0; --i) {
            if (i < m) {
                const double cand = -(v + acc) / cur.luu[i];  // valid on lane cl == i (luu[i] = Luu[i][i])
                const double ui = readlane_f64(cand, i);
                if (cl == i) myu = ui;
                acc = __builtin_fma(cur.luu[i], ui, acc);  // lanes cl < i: Luu[i][cl] u_i
                if (lane == 0) sw[i] = ui;
            }
        }
        wave_sync();
        // x+ = c + A x + B u  (lqr_kernel.hpp:201-203), reduced over row groups
        double xn[R];
#pragma unroll
        for (int q = 0; q < R; ++q) {
            double a = ax[q];
#pragma unroll
            for (int jj = 0; jj < NJ; ++jj) {
                const int j = 4 * jj + g;
                if (j < m) a = __builtin_fma(cur.E[q][jj], sw[j], a);
            }
            a += shfl_xor_f64(a, 16);
            a += shfl_xor_f64(a, 32);
            xn[q] = a + cur.c[q];
        }
        wave_sync();
        if (g == 0 && cl < m) wb[(long long)k * s + cl] = myu;
        if (g == 0) {
#pragma unroll
            for (int q = 0; q < R; ++q) {
                const int t = cl + 16 * q;
                if (t < n) {
                    sw[m + t] = xn[q];
                    wb[(long long)(k + 1) * s + ((k + 1 < N) ? m : 0) + t] = xn[q];
                }
            }
        }
        wave_sync();
        if (k + 1 < N) cur = nxt;
    }
}

int launch_riccati_forward(const Shape &sh, const double *E, const double *c, const double *FR, const double *x0,
                           double *ws, hipStream_t st) {
    const dim3 grid(sh.batch), blk(64);
    if (sh.s > 32) {
        set_error("forward: n + m > 32 is not supported by this build");
        return PDPLQR_ERR_UNSUPPORTED;
    }
    const int R = sh.s <= 16 ? 1 : 2;
    if (R == 1) {
        if (sh.m <= 4) hipLaunchKernelGGL((k_riccati_fwd<1, 4>), grid, blk, 0, st, sh, E, c, FR, x0, ws);
        else if (sh.m <= 8) hipLaunchKernelGGL((k_riccati_fwd<1, 8>), grid, blk, 0, st, sh, E, c, FR, x0, ws);
        else hipLaunchKernelGGL((k_riccati_fwd<1, 16>), grid, blk, 0, st, sh, E, c, FR, x0, ws);
    } else {
        if (sh.m <= 8) hipLaunchKernelGGL((k_riccati_fwd<2, 8>), grid, blk, 0, st, sh, E, c, FR, x0, ws);
        else if (sh.m <= 16) hipLaunchKernelGGL((k_riccati_fwd<2, 16>), grid, blk, 0, st, sh, E, c, FR, x0, ws);
        else hipLaunchKernelGGL((k_riccati_fwd<2, 32>), grid, blk, 0, st, sh, E, c, FR, x0, ws);
    }
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

}  // namespace pdplqr
