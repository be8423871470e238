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
#include "device_common.hpp"
#include "parallel.hpp"

#include <stdint.h>
#include <stdlib.h>

namespace pdplqr {

// ---------------------------------------------------------------------------
// update_problem_data (lqr_solver.hpp:41-56)
// ---------------------------------------------------------------------------
__global__ void k_update_problem_data(Shape sh, const double *__restrict__ H, const double *__restrict__ hv,
                                      const double *__restrict__ ws, const double *__restrict__ ys,
                                      const double *__restrict__ zs, const double *__restrict__ irho,
                                      double sigma, double *__restrict__ Hw, double *__restrict__ hw,
                                      double *__restrict__ gw, const short2 *__restrict__ tab_s,
                                      const short2 *__restrict__ tab_n, int skipH) {
    // skipH: H~ is already in Hw for this sigma (pdplqr_handle::hw_cached)
    const long long totH = skipH ? 0 : sh.perHw * sh.batch, toth = sh.perh * sh.batch,
                    totg = (long long)sh.ny * sh.batch;
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
                if (q >= sh.pn) {  // 16-byte alignment pad of the problem
                    Hw[t] = 0.0;
                    continue;
                }
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
                               hipStream_t st, bool skipH) {
    const long long total = ((skipH ? 0 : sh.perHw) + sh.perh + sh.ny) * (long long)sh.batch;
    const int threads = 256;
    long long blocks = (total + threads - 1) / threads;
    if (blocks > 8192) blocks = 8192;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_update_problem_data, dim3((unsigned)blocks), dim3(threads), 0, st, sh, H, hv, ws, ys, zs,
                       irho, sigma, Hw, hw, gw, tab_s, tab_n, (int)skipH);
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
                const int q = (int)(r - (long long)N * sh.ps);
                if (q >= sh.pn) continue;  // alignment pad
                const short2 ij = tab_n[q];
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
// Per-stage rollout record FR_k = [L(:, 0:m) (s x m, column-major) | lu'_k (m)]:
// exactly what LQRKernel::forward_step reads (Luu, Lxu, lu; lqr_kernel.hpp:190-198).
#ifndef PDPLQR_BWD_WAVES
#define PDPLQR_BWD_WAVES 4  // waves per SIMD for T = 1: 16 problems per CU fit in one residency round
#endif
template <int T>
__global__ __launch_bounds__(64, (T == 1 ? PDPLQR_BWD_WAVES : 1)) void k_riccati_bwd(RiccatiArgs A) {
    __shared__ BwdSmem<T> sm;
    const int lane = wave_lane(), g = lane >> 4, c = lane & 15;
    const long long b = blockIdx.x;
    const Shape &sh = A.sh;
    const int n = sh.n, m = sh.m, N = sh.N, s = sh.s;
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
        double lpr[T][4];
        const bool okN = chol_tiles<T>(M, lpr, sm.col, sm.inv, sm.luq, m, s, m, false, g, c);
        finalize_L<T>(M, sm.inv, m, s, g, c);
        if (!okN) fail_stage = N;
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
        d4 M[T][T];
        double lpr[T][4];
        const bool okk = riccati_stage<T>(sm, cur, M, lpr, n, m, s, g, c);
        if (!okk && fail_stage < 0) fail_stage = k;
        // p_k -> factor cache
        if (lpb && c == 0) {
#pragma unroll
            for (int a = 0; a < T; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * a + 4 * r + g;
                    if (i >= m && i < s) lpb[(long long)k * s + i] = lpr[a][r];
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

// ---------------------------------------------------------------------------
// Shape-specialised backward (n = NN, m = MM known at compile time) with the
// stage inputs streamed by LDS-DMA (global_load_lds_dwordx4, no VGPRs): the
// record of stage k-1 -- E (n s), c (n), h~ (s), packed H~ (s(s+1)/2) -- lands
// in the other half of a double buffer while stage k computes.  Requires every
// section to be a whole number of 16-byte chunks (even double counts).
// ---------------------------------------------------------------------------
template <int NN, int MM>
struct FastShape {
    static constexpr int n = NN, m = MM, s = NN + MM;
    static constexpr int ps = s * (s + 1) / 2;
    static constexpr int OE = 0, OC = n * s, OH = OC + n, OP = OH + s, Q = OP + ps;
    static constexpr int CH = Q / 2, NI = (CH + 63) / 64;
    static constexpr bool ok = (n * s) % 2 == 0 && n % 2 == 0 && s % 2 == 0 && ps % 2 == 0;
};

template <int T, int NN, int MM, bool KEEP>
__global__ __launch_bounds__(64, (T == 1 ? PDPLQR_BWD_WAVES : 1)) void k_riccati_bwd_fast(RiccatiArgs A) {
    using SH = FastShape<NN, MM>;
    constexpr int n = SH::n, m = SH::m, s = SH::s, ps = SH::ps, NI = SH::NI, CH = SH::CH;
    static_assert(SH::ok, "fast path needs 16-byte stage sections");
    __shared__ BwdSmem<T> sm;
    __shared__ __attribute__((aligned(16))) double stg[2][NI * 128];
    const int lane = wave_lane(), g = lane >> 4, c = lane & 15;
    const long long b = blockIdx.x;
    const Shape &sh = A.sh;
    const int N = sh.N;
    const double *Eb = A.E + b * sh.perE;
    const double *cb = A.c + b * sh.perc;
    const double *Hb = A.Hw + b * sh.perHw;
    const double *hb = A.hw + b * sh.perh;
    double *FRb = A.KD + b * sh.perKD;
    double *Lcb = KEEP ? A.Lc + b * sh.perHw : nullptr;
    double *lpb = KEEP ? A.lpc + b * sh.perh : nullptr;
    int fail_stage = -1;

    // per-lane DMA source offsets (section, offset) for each of the NI chunks
    auto dma = [&](int k, int slot) {
#pragma unroll
        for (int q = 0; q < NI; ++q) {
            int ch = q * 64 + lane;
            ch = ch < CH ? ch : CH - 1;  // surplus lanes re-load the last chunk into an unused slot
            const int d = 2 * ch;
            const double *src = d < SH::OC   ? Eb + (long long)k * n * s + d
                                : d < SH::OH ? cb + (long long)k * n + (d - SH::OC)
                                : d < SH::OP ? hb + (long long)k * s + (d - SH::OH)
                                             : Hb + (long long)k * ps + (d - SH::OP);
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                             (__attribute__((address_space(3))) void *)(&stg[slot][q * 128]), 16, 0,
                                             0);
        }
    };

    // ---- terminal (lqr_kernel.hpp:80-91) ----
    {
        d4 M[T][T];
        load_M<T>(M, Hb + (long long)N * ps, n, m, m, s, g, c);
        double lpr[T][4];
        const bool okN = chol_tiles<T>(M, lpr, sm.col, sm.inv, sm.luq, m, s, m, false, g, c);
        finalize_L<T>(M, sm.inv, m, s, g, c);
        if (!okN) fail_stage = N;
        store_L_lds<T>(M, sm.L, g, c);
        if (lane < n) {
            const double v = hb[(long long)N * s + lane];
            sm.pv[lane] = v;
            if (KEEP) lpb[(long long)N * s + lane] = v;
        }
        if (KEEP)
#pragma unroll
            for (int a = 0; a < T; ++a)
#pragma unroll
                for (int bt = 0; bt < T; ++bt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int i = 16 * a + 4 * r + g, j = 16 * bt + c;
                        if (j >= m && i >= j && i < s)
                            Lcb[(long long)N * ps + pidx(i - m, j - m, n)] = M[a][bt][r];
                    }
        wave_sync();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    dma(N - 1, (N - 1) & 1);
    for (int k = N - 1; k >= 0; --k) {
        if (k > 0) {
            dma(k - 1, (k - 1) & 1);
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");  // stage k's record has landed
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const double *R = stg[k & 1];
        StageIn<T> cur;
#pragma unroll
        for (int cc = 0; cc < 4 * T; ++cc) {
            const int t = 4 * cc + g;
#pragma unroll
            for (int bt = 0; bt < T; ++bt) {
                const int j = 16 * bt + c;
                cur.E[cc][bt] = (t < n && j < s) ? R[SH::OE + j * n + t] : 0.0;
            }
            cur.c[cc] = (t < n) ? R[SH::OC + t] : 0.0;
        }
#pragma unroll
        for (int bt = 0; bt < T; ++bt) {
            const int j = 16 * bt + c;
            cur.h[bt] = (j < s) ? R[SH::OH + j] : 0.0;
        }
#pragma unroll
        for (int a = 0; a < T; ++a)
#pragma unroll
            for (int bt = 0; bt < T; ++bt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * a + 4 * r + g, j = 16 * bt + c;
                    cur.H[a][bt][r] = (i < s && j < s) ? R[SH::OP + (i >= j ? pidx(i, j, s) : pidx(j, i, s))]
                                                       : (i == j ? 1.0 : 0.0);
                }
        d4 M[T][T];
        double lpr[T][4];
        const bool okk = riccati_stage<T>(sm, cur, M, lpr, n, m, s, g, c);
        if (!okk && fail_stage < 0) fail_stage = k;
        // rollout record FR_k = [L(:, 0:m) | lu']
        double *FRk = FRb + (long long)k * (s * m + m);
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
        if (lane < m) FRk[s * m + lane] = sm.luq[lane];
        if (KEEP) {
            if (lane < m) lpb[(long long)k * s + lane] = sm.luq[lane];
            if (lane < n) lpb[(long long)k * s + m + lane] = sm.pv[lane];
#pragma unroll
            for (int a = 0; a < T; ++a)
#pragma unroll
                for (int bt = 0; bt < T; ++bt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int i = 16 * a + 4 * r + g, j = 16 * bt + c;
                        if (i >= j && i < s) Lcb[(long long)k * ps + pidx(i, j, s)] = M[a][bt][r];
                    }
        }
    }
    if (lane == 0) A.status[b] = fail_stage < 0 ? 0 : fail_stage + 1;
}

template <int T, int NN, int MM>
static void launch_fast(const RiccatiArgs &a, hipStream_t st) {
    if (a.Lc) hipLaunchKernelGGL((k_riccati_bwd_fast<T, NN, MM, true>), dim3(a.sh.batch), dim3(64), 0, st, a);
    else hipLaunchKernelGGL((k_riccati_bwd_fast<T, NN, MM, false>), dim3(a.sh.batch), dim3(64), 0, st, a);
}

// ---------------------------------------------------------------------------
// Value-form backward on 3 x 3 register tiles (32 < s <= 48, n % 4 == 0,
// m % 4 == 0, m <= 16; keep_factors = 0): the 12/4 kernels_schur.hip scheme
// at T = 3.  The stage matrix M_k = H~_k + E^T P_{k+1} E and lp = h~ + E^T
// (P_{k+1} c + p_{k+1}) (lqr_kernel.hpp:121-143 with P = Lxx Lxx^T) are formed
// from P_{k+1} itself (LDS, symmetrised on read), and only the m u-pivots are
// eliminated (chol_tiles over [0, m), lp carried): the trailing block left is
// P_k, the carried lp rows are p_k (lqr_kernel.hpp:145-146).  16 pivots a
// stage instead of the full factor's 40 at 24/16, and no L round trip.  The
// stage records arrive by LDS-DMA as in k_riccati_bwd_fast; the rollout
// record is the same [L(:, 0:m) | lu'].  Status as the value-form 12/4 path:
// a u-pivot that is not positive, or a P_k diagonal that is psd_bad.
// PDPLQR_NO_VF3=1: the full-factor k_riccati_bwd_fast<3> (A/B).
// ---------------------------------------------------------------------------
template <int NN, int MM>
__global__ __launch_bounds__(64, 1) void k_riccati_bwd_vf3(RiccatiArgs A) {
    constexpr int T = 3;
    using SH = FastShape<NN, MM>;
    constexpr int n = SH::n, m = SH::m, s = SH::s, ps = SH::ps, NI = SH::NI, CH = SH::CH;
    constexpr int PL = n + 1;          // leading dimension of P in LDS
    constexpr int NC = n / 4;          // K chunks over the state index
    constexpr int TG = (n + 15) / 16;  // row tiles of G = P E
    static_assert(SH::ok && s > 32 && s <= 16 * T && n % 4 == 0 && m % 4 == 0 && m <= 16, "value-form T = 3 shape");
    // pivot broadcast, 1/sqrt(pivot), lu', lp redistribution: BwdSmem without
    // its factor block (37.5 KB a block in all: 4 blocks, one per SIMD, per CU)
    struct VfSmem {
        alignas(16) double col[4 * 16 * T];
        double inv[16 * T], luq[16 * T], lp[16 * T];
    };
    __shared__ VfSmem sm;
    __shared__ double Ps[n * PL];
    __shared__ double pvs[n];
    __shared__ __attribute__((aligned(16))) double stg[2][NI * 128];
    const int lane = wave_lane(), g = lane >> 4, c = lane & 15;
    const long long b = blockIdx.x;
    const Shape &sh = A.sh;
    const int N = sh.N;
    const double *Eb = A.E + b * sh.perE;
    const double *cb = A.c + b * sh.perc;
    const double *Hb = A.Hw + b * sh.perHw;
    const double *hb = A.hw + b * sh.perh;
    double *FRb = A.KD + b * sh.perKD;
    int fail_stage = -1;

    auto dma = [&](int k, int slot) {
#pragma unroll
        for (int q = 0; q < NI; ++q) {
            int ch = q * 64 + lane;
            ch = ch < CH ? ch : CH - 1;
            const int d = 2 * ch;
            const double *src = d < SH::OC   ? Eb + (long long)k * n * s + d
                                : d < SH::OH ? cb + (long long)k * n + (d - SH::OC)
                                : d < SH::OP ? hb + (long long)k * s + (d - SH::OH)
                                             : Hb + (long long)k * ps + (d - SH::OP);
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                             (__attribute__((address_space(3))) void *)(&stg[slot][q * 128]), 16, 0,
                                             0);
        }
    };

    // ---- terminal (lqr_kernel.hpp:80-91): P_N = H~_N (packed, order n), p_N = h~_N ----
    {
        const double *HN = Hb + (long long)N * ps;
        bool bad = false;
        for (int q = lane; q < n * n; q += 64) {
            const int i = q % n, j = q / n;
            const double v = HN[i >= j ? pidx(i, j, n) : pidx(j, i, n)];
            Ps[i + j * PL] = v;
            if (i == j && psd_bad(v)) bad = true;
        }
        if (lane < n) pvs[lane] = hb[(long long)N * s + lane];
        if (__any(bad)) fail_stage = N;
        wave_sync();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    dma(N - 1, (N - 1) & 1);
    for (int k = N - 1; k >= 0; --k) {
        if (k > 0) {
            dma(k - 1, (k - 1) & 1);
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");  // stage k's record has landed
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        wave_sync();
        const double *R = stg[k & 1];
        // E[t][j] (t = 4 cc + g, j = 16 bt + c): the B operand of G = P E and,
        // by symmetry of the layouts, the A operand of E^T G
        double Ev[NC][T], cv[NC], pv[NC], ap[NC][TG];
#pragma unroll
        for (int cc = 0; cc < NC; ++cc) {
            const int t = 4 * cc + g;
#pragma unroll
            for (int bt = 0; bt < T; ++bt) {
                const int j = 16 * bt + c;
                Ev[cc][bt] = (j < s) ? R[SH::OE + j * n + t] : 0.0;
            }
            cv[cc] = R[SH::OC + t];
            pv[cc] = pvs[t];
#pragma unroll
            for (int a = 0; a < TG; ++a) {  // P[16 a + c][t], symmetrised
                const int i = 16 * a + c;
                const int ic = i < n ? i : 0;
                ap[cc][a] = (i < n) ? 0.5 * (Ps[ic + t * PL] + Ps[t + ic * PL]) : 0.0;
            }
        }
        d4 M[T][T];
#pragma unroll
        for (int a = 0; a < T; ++a)
#pragma unroll
            for (int bt = 0; bt < T; ++bt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * a + 4 * r + g, j = 16 * bt + c;
                    M[a][bt][r] = (i < s && j < s) ? R[SH::OP + (i >= j ? pidx(i, j, s) : pidx(j, i, s))]
                                                   : (i == j ? 1.0 : 0.0);
                }
        double hv[T];
#pragma unroll
        for (int bt = 0; bt < T; ++bt) hv[bt] = (16 * bt + c < s) ? R[SH::OH + 16 * bt + c] : 0.0;
        // ---- G = P E (rows: state index, TG tiles) ----
        d4 G[TG][T];
#pragma unroll
        for (int a = 0; a < TG; ++a)
#pragma unroll
            for (int bt = 0; bt < T; ++bt) G[a][bt] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int cc = 0; cc < NC; ++cc)
#pragma unroll
            for (int a = 0; a < TG; ++a)
#pragma unroll
                for (int bt = 0; bt < T; ++bt) G[a][bt] = mfma_f64(ap[cc][a], Ev[cc][bt], G[a][bt]);
        // ---- M = H~ + E^T G ----
#pragma unroll
        for (int cc = 0; cc < NC; ++cc)
#pragma unroll
            for (int a = 0; a < T; ++a)
#pragma unroll
                for (int bt = 0; bt < T; ++bt) M[a][bt] = mfma_f64(Ev[cc][a], G[cc >> 2][bt][cc & 3], M[a][bt]);
        // ---- lp = h~ + G^T c + E^T p_{k+1} (column j = 16 bt + c), to rows ----
        double lpr[T][4];
        {
#pragma unroll
            for (int bt = 0; bt < T; ++bt) {
                double part = 0.0;
#pragma unroll
                for (int cc = 0; cc < NC; ++cc) {
                    part = __builtin_fma(G[cc >> 2][bt][cc & 3], cv[cc], part);
                    part = __builtin_fma(Ev[cc][bt], pv[cc], part);
                }
                part += shfl_xor_f64(part, 16);
                part += shfl_xor_f64(part, 32);
                if (g == 0) sm.lp[16 * bt + c] = hv[bt] + part;
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
        // ---- the m u-pivots (lp carried): trailing block = P_k, lp rows x = p_k ----
        const bool okk = chol_tiles<T>(M, lpr, sm.col, sm.inv, sm.luq, 0, m, m, true, g, c);
        bool bad = false;
#pragma unroll
        for (int a = 0; a < T; ++a)
#pragma unroll
            for (int bt = 0; bt < T; ++bt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * a + 4 * r + g, j = 16 * bt + c;
                    if (i >= m && i < s && j >= m && j < s) {
                        Ps[(i - m) + (j - m) * PL] = M[a][bt][r];
                        if (i == j && psd_bad(M[a][bt][r])) bad = true;
                    }
                }
        if (c == 0)
#pragma unroll
            for (int a = 0; a < T; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * a + 4 * r + g;
                    if (i >= m && i < s) pvs[i - m] = lpr[a][r];
                }
        if ((!okk || __any(bad)) && fail_stage < 0) fail_stage = k;
        // ---- rollout record FR_k = [L(:, 0:m) | lu'], L(i, j) = M[i][j] / sqrt(M[j][j]) ----
        double *FRk = FRb + (long long)k * (s * m + m);
        if (c < m) {
            const double iv = sm.inv[c];
#pragma unroll
            for (int a = 0; a < T; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * a + 4 * r + g;
                    if (i < s) FRk[c * s + i] = (i >= c) ? M[a][0][r] * iv : 0.0;
                }
        }
        if (lane < m) FRk[s * m + lane] = sm.luq[lane];
        wave_sync();
    }
    if (lane == 0) A.status[b] = fail_stage < 0 ? 0 : fail_stage + 1;
}

// The wide shapes the 3 x 3 register-tile kernels are instantiated for: every
// (n, m) with n % 4 = m % 4 = 0, m <= 16 and 32 < n + m <= 48 (the value-form
// backward k_riccati_bwd_vf3 and the DMA rollout k_rollout_dma3; other wide
// shapes keep the block-wide kernels of kernels_big.hip / kernels_wide.hip).
template <int NN, int MM>
struct Wide3 {
    static constexpr int n = NN, m = MM;
};
template <typename F>
static bool wide3_dispatch(int n, int m, F &&f) {
    bool hit = false;
    auto one = [&](auto shape) {
        if (!hit && n == decltype(shape)::n && m == decltype(shape)::m) {
            f(shape);
            hit = true;
        }
    };
    one(Wide3<32, 4>{}), one(Wide3<28, 8>{}), one(Wide3<24, 12>{}), one(Wide3<20, 16>{});
    one(Wide3<36, 4>{}), one(Wide3<32, 8>{}), one(Wide3<28, 12>{}), one(Wide3<24, 16>{});
    one(Wide3<40, 4>{}), one(Wide3<36, 8>{}), one(Wide3<32, 12>{}), one(Wide3<28, 16>{});
    one(Wide3<44, 4>{}), one(Wide3<40, 8>{}), one(Wide3<36, 12>{}), one(Wide3<32, 16>{});
    return hit;
}

// 16-byte alignment of every per-problem / per-stage block (fast path).
static bool fast_aligned(const RiccatiArgs &a) {
    const Shape &sh = a.sh;
    auto al = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    return al(a.E) && al(a.c) && al(a.Hw) && al(a.hw) && sh.perE % 2 == 0 && sh.perc % 2 == 0 &&
           sh.perHw % 2 == 0 && sh.perh % 2 == 0;
}

int launch_riccati_backward(const RiccatiArgs &a, hipStream_t st) {
    {
        const int rc = launch_riccati_backward_schur(a, st);  // keep_factors = 0, n + m <= 16
        if (rc != PDPLQR_ERR_UNSUPPORTED) return rc;
    }
    const bool fast_ok = fast_aligned(a);
    if (fast_ok && a.sh.n == 12 && a.sh.m == 4) {
        launch_fast<1, 12, 4>(a, st);
    } else if (fast_ok && a.sh.n == 24 && a.sh.m == 8) {
        launch_fast<2, 24, 8>(a, st);
    } else if (fast_ok && wide3_dispatch(a.sh.n, a.sh.m, [&](auto shape) {
                   using W = decltype(shape);
                   if (a.Lc)  // the factor cache: the full factor
                       hipLaunchKernelGGL((k_riccati_bwd_fast<3, W::n, W::m, true>), dim3(a.sh.batch), dim3(64), 0, st, a);
                   else hipLaunchKernelGGL((k_riccati_bwd_vf3<W::n, W::m>), dim3(a.sh.batch), dim3(64), 0, st, a);
               })) {
        // 32 < s <= 48 on 3 x 3 register tiles (one wave per problem) instead of
        // the block-wide LDS kernels of kernels_big.hip / kernels_wide.hip
    } else if (a.sh.s <= 16) {
        hipLaunchKernelGGL(k_riccati_bwd<1>, dim3(a.sh.batch), dim3(64), 0, st, a);
    } else if (a.sh.s <= 32) {
        hipLaunchKernelGGL(k_riccati_bwd<2>, dim3(a.sh.batch), dim3(64), 0, st, a);
    } else if (big_shape(a.sh)) {
        return launch_riccati_backward_big(a, st);
    } else if (xl_shape(a.sh)) {
        return launch_riccati_backward_xl(a, st);
    } else {
        set_error("backward: n + m > 256 is not supported by this build");
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
template <int P>  // P >= n + m: 32, or 64 for the shapes of kernels_big.hip
__global__ __launch_bounds__(64) void k_riccati_bwd_nofact(RiccatiArgs A) {
    __shared__ double Lk[P * P];  // this stage's L (packed -> dense, column-major, ld = s)
    __shared__ double Ln[P * P];  // next stage's Lxx (ld = n)
    __shared__ double cvec[P], va[P], vb[P], lp[P], pn[P];
    const int lane = wave_lane();
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
    // compile-time shapes: the streamed vector recursion (kernels_nofact.hip)
    {
        const int rc = launch_nofact_dma(a, st);
        if (rc != PDPLQR_ERR_UNSUPPORTED) return rc;
    }
    if (a.sh.s > 64) {
        if (xl_shape(a.sh)) return launch_riccati_backward_nofact_xl(a, st);
        set_error("backward_without_factorization: n + m > 256 is not supported by this build");
        return PDPLQR_ERR_UNSUPPORTED;
    }
    if (a.sh.s <= 32) hipLaunchKernelGGL(k_riccati_bwd_nofact<32>, dim3(a.sh.batch), dim3(64), 0, st, a);
    else hipLaunchKernelGGL(k_riccati_bwd_nofact<64>, dim3(a.sh.batch), dim3(64), 0, st, a);
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

template <int R, int MM, bool SEG>
__global__ __launch_bounds__(64) void k_riccati_fwd(Shape sh, const double *__restrict__ E,
                                                    const double *__restrict__ c, const double *__restrict__ FR,
                                                    const double *__restrict__ x0, double *__restrict__ ws, SegFwd sf) {
    constexpr int NJ = 4 * R;
    __shared__ double sw[64];  // w_k = [u; x]
    __shared__ double suh[64]; // u_hat of this segment
    const int lane = wave_lane(), g = lane >> 4, cl = lane & 15;
    const int n = sh.n, m = sh.m, s = sh.s;
    long long b;
    int N0, N1;
    bool last;
    if (SEG) {
        b = blockIdx.x / sf.S;
        const int seg = blockIdx.x % sf.S;
        N0 = sf.seg_start[seg];
        N1 = N0 + sf.seg_len[seg];
        last = (seg == sf.S - 1) && sf.last_is_terminal;
        const double *xh = sf.xhat + (b * (sf.S + 1) + seg) * n;
        if (lane < n) {
            sw[m + lane] = xh[lane];
            suh[lane] = last ? 0.0 : sf.lam[(b * (sf.S + 1) + seg + 1) * n + lane];
        }
        if (!last && seg == sf.S - 1 && lane < n)  // shard slice end: x after the slice
            ws[b * sh.perh + (long long)N1 * s + lane] = sf.xhat[(b * (sf.S + 1) + sf.S) * n + lane];
    } else {
        b = blockIdx.x;
        N0 = 0;
        N1 = sh.N;
        last = true;
        if (lane < n) sw[m + lane] = x0[b * n + lane];
    }
    const int N = sh.N;
    const long long frs = (long long)s * m + m;
    const double *Eb = E + b * sh.perE;
    const double *cb = c + b * sh.perc;
    const double *Fb = FR + b * sh.perKD;
    const double *Gb = SEG ? sf.G + b * (long long)N * m * n : nullptr;
    double *wb = ws + b * sh.perh;
    if (lane < n) wb[(long long)N0 * s + m + lane] = sw[m + lane];  // ws[N0].tail(n) = x_hat (lqr_solver_parallel.hpp:224)
    wave_sync();
    // G u_hat term per stage: lanes (g, cl < m) own G[cl][4 qq + g]
    double uh[NJ];
#pragma unroll
    for (int qq = 0; qq < NJ; ++qq) {
        const int t = 4 * qq + g;
        uh[qq] = (SEG && !last && t < n) ? suh[t] : 0.0;
    }
    FwdIn<R, MM> cur, nxt;
    double gq[NJ], gqn[NJ];
    fwd_load<R, MM>(cur, Eb + (long long)N0 * n * s, cb + (long long)N0 * n, Fb + (long long)N0 * frs, n, m, s, g, cl);
#pragma unroll
    for (int qq = 0; qq < NJ; ++qq) {
        const int t = 4 * qq + g;
        gq[qq] = (SEG && !last && cl < m && t < n) ? Gb[(long long)N0 * m * n + cl + t * m] : 0.0;
    }
    for (int k = N0; k < N1; ++k) {
        if (k + 1 < N1) {
            fwd_load<R, MM>(nxt, Eb + (long long)(k + 1) * n * s, cb + (long long)(k + 1) * n,
                            Fb + (long long)(k + 1) * frs, n, m, s, g, cl);
#pragma unroll
            for (int qq = 0; qq < NJ; ++qq) {
                const int t = 4 * qq + g;
                gqn[qq] = (SEG && !last && cl < m && t < n) ? Gb[(long long)(k + 1) * m * n + cl + t * m] : 0.0;
            }
        }
        // v = lu' + Lxu^T x - G u_hat  (lqr_kernel_parallel.hpp:195-197 / lqr_kernel.hpp:197)
        double v = 0.0;
#pragma unroll
        for (int qq = 0; qq < NJ; ++qq) {
            const int t = 4 * qq + g;
            const double xt = (t < n) ? sw[m + t] : 0.0;
            v = __builtin_fma(cur.lxu[qq], xt, v);
            if (SEG) v = __builtin_fma(-gq[qq], uh[qq], v);
        }
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
        // u = -Luu^{-T} v: back substitution, u_i broadcast from lane i.  The
        // reciprocals of the diagonal do not depend on the chain (rcp, hoisted).
        double rdg[MM];
#pragma unroll
        for (int i = 0; i < MM; ++i) rdg[i] = rcp_f64(cur.luu[i]);  // used on lane cl == i only
        double acc = 0.0, myu = 0.0;
#pragma unroll
        for (int i = MM - 1; i >= 0; --i) {
            if (i < m) {
                const double cand = -(v + acc) * rdg[i];  // valid on lane cl == i (luu[i] = Luu[i][i])
                const double ui = readlane_f64(cand, i);
                if (cl == i) myu = ui;
                acc = __builtin_fma(cur.luu[i], ui, acc);  // lanes cl < i: Luu[i][cl] u_i
                if (lane == 0) sw[i] = ui;
            }
        }
        wave_sync();
        const bool upd = last || (k < N1 - 1);  // update_x_next (lqr_solver_parallel.hpp:231)
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
        if (g == 0 && upd) {
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
        if (k + 1 < N1) {
            cur = nxt;
#pragma unroll
            for (int qq = 0; qq < NJ; ++qq) gq[qq] = gqn[qq];
        }
    }
}

// ---------------------------------------------------------------------------
// Segment rollout with the stage records streamed through an LDS-DMA ring
// (compile-time 16 < s <= 32 shapes, one wave per segment).  The generic
// kernel above prefetches one stage ahead in registers, which at one wave per
// SIMD leaves the HBM latency exposed (half of its wave cycles wait on
// memory).  Here D - 1 stages are in flight: E_k, c_k, the rollout record and
// G_k land in slot k % D by global_load_lds_dwordx4; the per-stage arithmetic
// is the generic kernel's, reading the slot.  vm ops per iteration: NI DMA +
// 1 u store + R x stores, so "stage k has landed" is a fixed vmcnt.
// ---------------------------------------------------------------------------
template <int NN, int MM>
struct SegRec {
    static constexpr int n = NN, m = MM, s = NN + MM, FRS = s * m + m;
    static constexpr int OE = 0, OC = n * s, OF = OC + n, OG = OF + FRS, REC = OG + m * n;
    static constexpr int CH = REC / 2, NI = (CH + 63) / 64, TAIL = CH - (NI - 1) * 64;
    static constexpr bool ok = (n * s) % 2 == 0 && n % 2 == 0 && FRS % 2 == 0 && (m * n) % 2 == 0 && s <= 32;
};

template <int NN, int MM, int D>
__global__ __launch_bounds__(64) void k_seg_fwd_dma(Shape sh, const double *__restrict__ E,
                                                    const double *__restrict__ c, const double *__restrict__ FR,
                                                    double *__restrict__ ws, SegFwd sf) {
    using SR = SegRec<NN, MM>;
    static_assert(SR::ok, "segment rollout record layout");
    constexpr int R = NN + MM <= 16 ? 1 : 2, NJ = 4 * R, n = NN, m = MM, s = NN + MM, NI = SR::NI;
    constexpr int VM = (1 + R) + (D - 2) * (NI + 1 + R) + NI;  // vm ops younger than stage k's DMA
    static_assert(VM <= 63, "vmcnt range");
    __shared__ __attribute__((aligned(16))) double ring[D][SR::REC];
    __shared__ double sw[64];   // w_k = [u; x]
    __shared__ double suh[64];  // u_hat of this segment
    const int lane = wave_lane(), g = lane >> 4, cl = lane & 15;
    const long long b = blockIdx.x / sf.S;
    const int seg = blockIdx.x % sf.S;
    const int N0 = sf.seg_start[seg], N1 = N0 + sf.seg_len[seg];
    const bool last = (seg == sf.S - 1) && sf.last_is_terminal;
    const int N = sh.N;
    const double *Eb = E + b * sh.perE;
    const double *cb = c + b * sh.perc;
    const double *Fb = FR + b * sh.perKD;
    const double *Gb = sf.G + b * (long long)N * m * n;
    double *wb = ws + b * sh.perh;
    {
        const double *xh = sf.xhat + (b * (sf.S + 1) + seg) * n;
        if (lane < n) {
            sw[m + lane] = xh[lane];
            suh[lane] = last ? 0.0 : sf.lam[(b * (sf.S + 1) + seg + 1) * n + lane];
        }
        if (!last && seg == sf.S - 1 && lane < n)  // shard slice end: x after the slice
            wb[(long long)N1 * s + lane] = sf.xhat[(b * (sf.S + 1) + sf.S) * n + lane];
    }
    auto dma = [&](int k, int slot) {
#pragma unroll
        for (int q = 0; q < NI; ++q) {
            if (q < NI - 1 || lane < SR::TAIL) {
                const int d = 2 * (q * 64 + lane);
                const double *src = d < SR::OC   ? Eb + (long long)k * (n * s) + d
                                    : d < SR::OF ? cb + (long long)k * n + (d - SR::OC)
                                    : d < SR::OG ? Fb + (long long)k * SR::FRS + (d - SR::OF)
                                                 : Gb + (long long)k * (m * n) + (d - SR::OG);
                dma16(src, &ring[slot][q * 128]);
            }
        }
    };
#pragma unroll
    for (int j = 0; j < D - 1; ++j) dma(N0 + j < N1 ? N0 + j : N1 - 1, j);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane < n) wb[(long long)N0 * s + m + lane] = sw[m + lane];  // ws[N0].tail(n) = x_hat
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
    double uh[NJ];
#pragma unroll
    for (int qq = 0; qq < NJ; ++qq) {
        const int t = 4 * qq + g;
        uh[qq] = (!last && t < n) ? suh[t] : 0.0;
    }
    for (int k = N0; k < N1; ++k) {
        const int kr = k - N0, kp = k + D - 1;
        dma(kp < N1 ? kp : N1 - 1, (kr + D - 1) % D);  // past the end: re-load into a consumed slot
        if (kr < D - 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM) : "memory");
        wave_sync();
        const double *Rk = ring[kr % D];
        FwdIn<R, MM> cur;
        fwd_load<R, MM>(cur, Rk + SR::OE, Rk + SR::OC, Rk + SR::OF, n, m, s, g, cl);
        double gq[NJ];
#pragma unroll
        for (int qq = 0; qq < NJ; ++qq) {
            const int t = 4 * qq + g;
            gq[qq] = (!last && cl < m && t < n) ? Rk[SR::OG + cl + t * m] : 0.0;
        }
        double v = 0.0;
#pragma unroll
        for (int qq = 0; qq < NJ; ++qq) {
            const int t = 4 * qq + g;
            const double xt = (t < n) ? sw[m + t] : 0.0;
            v = __builtin_fma(cur.lxu[qq], xt, v);
            v = __builtin_fma(-gq[qq], uh[qq], v);
        }
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
        double rdg[MM];
#pragma unroll
        for (int i = 0; i < MM; ++i) rdg[i] = rcp_f64(cur.luu[i]);
        double acc = 0.0, myu = 0.0;
#pragma unroll
        for (int i = MM - 1; i >= 0; --i) {
            const double cand = -(v + acc) * rdg[i];  // valid on lane cl == i
            const double ui = readlane_f64(cand, i);
            if (cl == i) myu = ui;
            acc = __builtin_fma(cur.luu[i], ui, acc);
            if (lane == 0) sw[i] = ui;
        }
        wave_sync();
        const bool upd = last || (k < N1 - 1);  // update_x_next (lqr_solver_parallel.hpp:231)
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
        if (g == 0 && cl < m) gstore(wb + (long long)k * s + cl, myu);
        if (g == 0 && upd) {
#pragma unroll
            for (int q = 0; q < R; ++q) {
                const int t = cl + 16 * q;
                if (t < n) {
                    sw[m + t] = xn[q];
                    gstore(wb + (long long)(k + 1) * s + ((k + 1 < N) ? m : 0) + t, xn[q]);
                }
            }
        }
        wave_sync();
    }
}

// ---------------------------------------------------------------------------
// The serial rollout for 32 < s <= 48 (R = 3 row tiles) with the stage
// records streamed through an LDS-DMA ring, as k_seg_fwd_dma does for the
// segments: E_k, c_k and the rollout record land in slot k % D by
// global_load_lds_dwordx4, D - 1 stages ahead.  The register-prefetch
// k_riccati_fwd<3> keeps only one stage in flight at one wave per SIMD.
// vm ops per iteration: NI DMA + 1 u store + RX x stores (RX = ceil(n / 16)
// row tiles that hold state rows), so "stage k has landed" is a fixed vmcnt.
// ---------------------------------------------------------------------------
template <int NN, int MM>
struct SerRec3 {
    static constexpr int n = NN, m = MM, s = NN + MM, FRS = s * m + m;
    static constexpr int OE = 0, OC = n * s, OF = OC + n, REC = OF + FRS;
    static constexpr int CH = REC / 2, NI = (CH + 63) / 64, TAIL = CH - (NI - 1) * 64;
    static constexpr bool ok = (n * s) % 2 == 0 && n % 2 == 0 && FRS % 2 == 0 && s > 32 && s <= 48 && m <= 16;
};

template <int NN, int MM, int D>
__global__ __launch_bounds__(64) void k_rollout_dma3(Shape sh, const double *__restrict__ E,
                                                     const double *__restrict__ c, const double *__restrict__ FR,
                                                     const double *__restrict__ x0, double *__restrict__ ws) {
    using SR = SerRec3<NN, MM>;
    static_assert(SR::ok, "serial rollout record layout");
    constexpr int R = 3, NJ = 4 * R, n = NN, m = MM, s = NN + MM, NI = SR::NI, RX = (NN + 15) / 16;
    constexpr int VM = (1 + RX) + (D - 2) * (NI + 1 + RX) + NI;  // vm ops younger than stage k's DMA
    static_assert(VM <= 63 && D >= 2, "vmcnt range");
    __shared__ __attribute__((aligned(16))) double ring[D][SR::REC];
    __shared__ double sw[64];  // w_k = [u; x]
    const int lane = wave_lane(), g = lane >> 4, cl = lane & 15;
    const long long b = blockIdx.x;
    const int N = sh.N;
    const double *Eb = E + b * sh.perE;
    const double *cb = c + b * sh.perc;
    const double *Fb = FR + b * sh.perKD;
    double *wb = ws + b * sh.perh;
    if (lane < n) sw[m + lane] = x0[b * n + lane];
    auto dma = [&](int k, int slot) {
#pragma unroll
        for (int q = 0; q < NI; ++q) {
            if (q < NI - 1 || lane < SR::TAIL) {
                const int d = 2 * (q * 64 + lane);
                const double *src = d < SR::OC   ? Eb + (long long)k * (n * s) + d
                                    : d < SR::OF ? cb + (long long)k * n + (d - SR::OC)
                                                 : Fb + (long long)k * SR::FRS + (d - SR::OF);
                dma16(src, &ring[slot][q * 128]);
            }
        }
    };
#pragma unroll
    for (int j = 0; j < D - 1; ++j) dma(j < N ? j : N - 1, j);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
    if (lane < n) wb[m + lane] = sw[m + lane];  // ws[0].tail(n) = x0
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
    for (int k = 0; k < N; ++k) {
        const int kp = k + D - 1;
        dma(kp < N ? kp : N - 1, kp % D);  // past the end: re-load into a consumed slot
        if (k < D - 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM) : "memory");
        wave_sync();
        const double *Rk = ring[k % D];
        FwdIn<R, MM> cur;
        fwd_load<R, MM>(cur, Rk + SR::OE, Rk + SR::OC, Rk + SR::OF, n, m, s, g, cl);
        // v = lu' + Lxu^T x  (lqr_kernel.hpp:197)
        double v = 0.0;
#pragma unroll
        for (int qq = 0; qq < NJ; ++qq) {
            const int t = 4 * qq + g;
            const double xt = (t < n) ? sw[m + t] : 0.0;
            v = __builtin_fma(cur.lxu[qq], xt, v);
        }
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
        double rdg[MM];
#pragma unroll
        for (int i = 0; i < MM; ++i) rdg[i] = rcp_f64(cur.luu[i]);
        double acc = 0.0, myu = 0.0;
#pragma unroll
        for (int i = MM - 1; i >= 0; --i) {
            const double cand = -(v + acc) * rdg[i];  // valid on lane cl == i
            const double ui = readlane_f64(cand, i);
            if (cl == i) myu = ui;
            acc = __builtin_fma(cur.luu[i], ui, acc);
            if (lane == 0) sw[i] = ui;
        }
        wave_sync();
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
        if (g == 0 && cl < m) gstore(wb + (long long)k * s + cl, myu);
        if (g == 0) {
#pragma unroll
            for (int q = 0; q < RX; ++q) {
                const int t = cl + 16 * q;
                if (t < n) {
                    sw[m + t] = xn[q];
                    gstore(wb + (long long)(k + 1) * s + ((k + 1 < N) ? m : 0) + t, xn[q]);
                }
            }
        }
        wave_sync();
    }
}

static bool ser3_aligned(const Shape &sh, const double *E, const double *c, const double *FR) {
    auto al = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    return al(E) && al(c) && al(FR) && sh.perE % 2 == 0 && sh.perc % 2 == 0 && sh.perKD % 2 == 0;
}

static bool segfwd_aligned(const Shape &sh, const double *E, const double *c, const double *FR, const SegFwd &sf) {
    auto al = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    return al(E) && al(c) && al(FR) && al(sf.G) && sh.perE % 2 == 0 && sh.perc % 2 == 0 && sh.perKD % 2 == 0 &&
           ((long long)sh.N * sh.m * sh.n) % 2 == 0;
}

template <bool SEG>
static int launch_fwd(const Shape &sh, const double *E, const double *c, const double *FR, const double *x0,
                      double *ws, const SegFwd &sf, hipStream_t st) {
    const dim3 grid((unsigned)(SEG ? sh.batch * sf.S : sh.batch)), blk(64);
    if (!SEG && ser3_aligned(sh, E, c, FR) && wide3_dispatch(sh.n, sh.m, [&](auto shape) {
            using W = decltype(shape);
            hipLaunchKernelGGL((k_rollout_dma3<W::n, W::m, 3>), grid, blk, 0, st, sh, E, c, FR, x0, ws);
        })) {
        PDPLQR_HIP_TRY(hipGetLastError());
        return PDPLQR_OK;
    }
    if (!SEG && sh.s > 32 && sh.s <= 48 && sh.m <= 16) {
        // 32 < s <= 48: the register rollout on 3 row tiles (one wave per problem)
        hipLaunchKernelGGL((k_riccati_fwd<3, 16, false>), grid, blk, 0, st, sh, E, c, FR, x0, ws, sf);
        PDPLQR_HIP_TRY(hipGetLastError());
        return PDPLQR_OK;
    }
    if (sh.s > 32) {
        if (!SEG && big_shape(sh)) return launch_riccati_forward_big(sh, E, c, FR, x0, ws, st);
        if (!SEG && xl_shape(sh)) return launch_riccati_forward_xl(sh, E, c, FR, x0, ws, st);
        if (SEG && big_shape(sh)) return launch_riccati_forward_seg_big(sh, E, c, FR, sf, ws, st);
        set_error(SEG ? "segment forward: n + m > 32 is not supported by this build"
                      : "forward: n + m > 64 is not supported by this build");
        return PDPLQR_ERR_UNSUPPORTED;
    }
    const int R = sh.s <= 16 ? 1 : 2;
    if (R == 1) {
        if (sh.m <= 4) hipLaunchKernelGGL((k_riccati_fwd<1, 4, SEG>), grid, blk, 0, st, sh, E, c, FR, x0, ws, sf);
        else if (sh.m <= 8) hipLaunchKernelGGL((k_riccati_fwd<1, 8, SEG>), grid, blk, 0, st, sh, E, c, FR, x0, ws, sf);
        else hipLaunchKernelGGL((k_riccati_fwd<1, 16, SEG>), grid, blk, 0, st, sh, E, c, FR, x0, ws, sf);
    } else {
        if (sh.m <= 8) hipLaunchKernelGGL((k_riccati_fwd<2, 8, SEG>), grid, blk, 0, st, sh, E, c, FR, x0, ws, sf);
        else if (sh.m <= 16) hipLaunchKernelGGL((k_riccati_fwd<2, 16, SEG>), grid, blk, 0, st, sh, E, c, FR, x0, ws, sf);
        else hipLaunchKernelGGL((k_riccati_fwd<2, 32, SEG>), grid, blk, 0, st, sh, E, c, FR, x0, ws, sf);
    }
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

int launch_riccati_forward(const Shape &sh, const double *E, const double *c, const double *FR, const double *x0,
                           double *ws, hipStream_t st) {
    const int rc = launch_rollout_dma(sh, E, c, FR, x0, ws, st);  // kernels_rollout.hip
    if (rc != PDPLQR_ERR_UNSUPPORTED) return rc;
    SegFwd none{};
    return launch_fwd<false>(sh, E, c, FR, x0, ws, none, st);
}

int launch_riccati_forward_seg(const Shape &sh, const double *E, const double *c, const double *FR, const SegFwd &sf,
                               double *ws, hipStream_t st) {
    if (xl_shape(sh)) return launch_riccati_forward_seg_xl(sh, E, c, FR, sf, ws, st);
    if (sh.n == 24 && sh.m == 8 && segfwd_aligned(sh, E, c, FR, sf)) {
        hipLaunchKernelGGL((k_seg_fwd_dma<24, 8, 3>), dim3((unsigned)(sh.batch * sf.S)), dim3(64), 0, st, sh, E, c,
                           FR, ws, sf);
        PDPLQR_HIP_TRY(hipGetLastError());
        return PDPLQR_OK;
    }
    // 12/4 (C2's one-problem solve: segments of a few stages): a 5-deep ring
    // puts a whole short segment's records in flight at once -- one memory
    // latency per segment instead of one per stage (k_riccati_fwd prefetches
    // one stage ahead)
    if (sh.n == 12 && sh.m == 4 && segfwd_aligned(sh, E, c, FR, sf)) {
        hipLaunchKernelGGL((k_seg_fwd_dma<12, 4, 5>), dim3((unsigned)(sh.batch * sf.S)), dim3(64), 0, st, sh, E, c,
                           FR, ws, sf);
        PDPLQR_HIP_TRY(hipGetLastError());
        return PDPLQR_OK;
    }
    return launch_fwd<true>(sh, E, c, FR, nullptr, ws, sf, st);
}

}  // namespace pdplqr
