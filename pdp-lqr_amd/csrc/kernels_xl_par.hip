// kernels_xl_par.hip -- the PARALLEL solver (LQRParallelSolver) past the LDS
// kernels: stage sizes 64 < n + m <= 256 and state sizes 64 < n <= 255.  The
// same algorithm and outputs as kernels_wide.hip (and the tiled kernels), with
// every matrix in a global-memory workspace slot (xl_la.hpp routines; L2
// resident) and the blocks of a launch striding over the items (segments,
// scan entries, boundaries), so that the workspace is xl_grid slots however
// many items a round has.  Restates:
//   * k_seg_bwd_xl: ParallelLQRKernel::step_with_factorization
//     (lqr_kernel_parallel.hpp:88-136) over a segment in the augmented value
//     form of k_seg_bwd_wide: per stage PE = P E~, YE = F E~, M = H~ + E~^T PE,
//     the m u-pivots of [[M, YE^T], [YE, -C]] with the aug column
//     [h~ + E~^T (P c + p); F c + f], leaving P_k, F_k, C_k, p_k, f_k;
//   * k_seg_bwd_nofact_xl: reduction_without_factorization
//     (lqr_solver_parallel.hpp:190-211, lqr_kernel_parallel.hpp:139-168) on
//     the value-function cache, f as the closed-loop rollout from x = 0
//     (k_seg_bwd_nofact's reading);
//   * xl_combine: the element combine (condensed_system.hpp:203-290 Cholesky
//     form, :82-137 LU form) in wide_combine's formulas;
//   * k_seg_scan_xl / k_seg_maps_xl / k_map_scan_xl / k_rank_maps_xl: one
//     suffix-scan round, the boundary maps, one radix-4 composition round and
//     the horizon-shard rank maps, as their _wide counterparts;
//   * k_fwd_seg_xl: the segment rollout with the G_k u_hat coupling
//     (lqr_kernel_parallel.hpp:195-198), k_riccati_fwd_big<true>'s steps.
#include "combine_tiles.hpp"  // ElemIn, elem_in
#include "parallel.hpp"
#include "xl_la.hpp"

#include <algorithm>
#include <string>

namespace pdplqr {

// LDS scratch of the element kernels
struct XlSm {
    double v[8][XL_S];
    double prow[2 * XL_S];
    double mul[XL_S], sinv[XL_S];
    double rv[4];
    int piv[XL_S], ra[4];
};

// Y = P_b (I + C_a P_b)^{-1}, Z = I - C_a Y with C_a in B[0] (wide_core's two
// forms); B[0..4]: n x n workspace buffers.  Returns the indices of Y, Z and a
// free buffer.
__device__ bool xl_core(double *const *B, const double *Pb, int n, bool lu, XlSm &sm, int &iy, int &iz, int &ifr) {
    double *B0 = B[0], *B1 = B[1], *B2 = B[2], *B3 = B[3];
    bool ok;
    if (!lu) {
        blk_copy(B1, n, mv_n(Pb, n), n, n);
        ok = xl_chol(B1, n, n, sm.sinv);                                            // R
        xl_mm(B2, n, B0, n, false, B1, n, false, n, n, n, nullptr, 0);              // C_a R
        xl_mm(B3, n, B1, n, true, B2, n, false, n, n, n, nullptr, 0, 1.0, 1.0);     // I + R^T C_a R
        blk_copy(B2, n, mv_t(B1, n), n, n);                                         // R^T
        ok = xl_chol(B3, n, n, sm.sinv) && ok;                                      // Q
        blk_trsm_l(B3, n, n, B2, n, n, nullptr);                                    // U = Q^{-1} R^T
        xl_mm(B1, n, B2, n, true, B2, n, false, n, n, n, nullptr, 0);               // Y = U^T U
        xl_mm(B3, n, B0, n, false, B1, n, false, n, n, n, nullptr, 0, -1.0, 1.0);   // Z = I - C_a Y
        iy = 1;
        iz = 3;
        ifr = 2;
    } else {
        xl_mm(B1, n, Pb, n, false, B0, n, false, n, n, n, nullptr, 0, 1.0, 1.0);    // I + P_b C_a
        blk_copy(B2, n, mv_n(Pb, n), n, n);                                         // P_b
        ok = xl_gauss_jordan(B1, n, sm.piv, sm.prow, sm.mul, 2 * n, sm.rv, sm.ra);  // [A | P_b] -> A^{-1} P_b
        for (int q = threadIdx.x; q < n * n; q += 256) {
            const int i = q % n, j = q / n;
            B3[q] = 0.5 * (B2[sm.piv[i] + j * n] + B2[sm.piv[j] + i * n]);
        }
        xl_mm(B1, n, B0, n, false, B3, n, false, n, n, n, nullptr, 0, -1.0, 1.0);   // Z = I - C_a Y
        iy = 3;
        iz = 1;
        ifr = 2;
    }
    return ok;
}

// out = a (x) b (wide_combine): fcf forms F, C, f; pp forms P, p.  Outputs
// must not alias the inputs.  W: 5 n^2 doubles of workspace.
__device__ bool xl_combine(double *oF, double *oC, double *of, double *oP, double *op, ElemIn ea, ElemIn eb, int n,
                           bool fcf, bool pp, bool lu, double *W, XlSm &sm) {
    const long long nn = (long long)n * n;
    double *const B[5] = {W, W + nn, W + 2 * nn, W + 3 * nn, W + 4 * nn};
    double *B0 = B[0], *B4 = B[4];
    double *pb = sm.v[0], *fa = sm.v[1], *v1 = sm.v[2], *v3 = sm.v[3], *t4 = sm.v[4], *t5 = sm.v[5];
    blk_copy(B0, n, mv_n(ea.C, n), n, n);  // C_a
    blk_vcopy(pb, eb.p, n);
    blk_vcopy(fa, ea.f, n);
    if (fcf) blk_mv(v1, mv_n(B0, n), pb, n, n, -1.0, fa);      // f_a - C_a p_b
    if (pp) blk_mv(v3, mv_n(eb.P, n), fa, n, n, 1.0, pb);      // p_b + P_b f_a
    int iy, iz, ifr;
    const bool ok = xl_core(B, eb.P, n, lu, sm, iy, iz, ifr);
    double *Y = B[iy], *Z = B[iz], *Fr = B[ifr];
    if (pp) {
        blk_copy(Fr, n, mv_n(ea.F, n), n, n);                                    // F_a
        xl_mm(B4, n, Y, n, false, Fr, n, false, n, n, n, nullptr, 0);            // Y F_a
        xl_mm(Y, n, Fr, n, true, B4, n, false, n, n, n, ea.P, n);                // P_a + F_a^T Y F_a
        blk_store_sym(oP, n, Y, n, n);
        blk_mv(t4, mv_t(Z, n), v3, n, n, 1.0, nullptr);                          // Z^T v3
        blk_mv(op, mv_t(Fr, n), t4, n, n, 1.0, ea.p);                            // p_a + F_a^T Z^T v3
    }
    if (fcf) {
        if (!pp) blk_copy(Fr, n, mv_n(ea.F, n), n, n);
        xl_mm(Y, n, Z, n, false, Fr, n, false, n, n, n, nullptr, 0);             // Z F_a (Y is free)
        blk_copy(Fr, n, mv_n(eb.F, n), n, n);                                    // F_b
        xl_mm(oF, n, Fr, n, false, Y, n, false, n, n, n, nullptr, 0);            // F_b Z F_a
        xl_mm(Y, n, Z, n, false, B0, n, false, n, n, n, nullptr, 0);             // Z C_a
        xl_mm(B4, n, Y, n, false, Fr, n, true, n, n, n, nullptr, 0);             // Z C_a F_b^T
        blk_mv(t5, mv_n(Z, n), v1, n, n, 1.0, nullptr);                          // Z v1
        xl_mm(Z, n, Fr, n, false, B4, n, false, n, n, n, eb.C, n);               // F_b Z C_a F_b^T + C_b
        blk_store_sym(oC, n, Z, n, n);
        blk_mv(of, mv_n(Fr, n), t5, n, n, 1.0, eb.f);                            // F_b Z v1 + f_b
    }
    return ok;
}

__device__ __forceinline__ double *xl_slot(double *xlw, const Shape &sh) {
    return xlw + (long long)blockIdx.x * xl_par_slot_doubles(sh);
}

// ---------------------------------------------------------------------------
// one Hillis-Steele round of the suffix scan (k_seg_scan_wide)
// ---------------------------------------------------------------------------
template <bool LU>
__global__ __launch_bounds__(256) void k_seg_scan_xl(ScanArgs A, int batch, long long slot) {
    __shared__ XlSm sm;
    const int n = A.n, S = A.S, d = A.dist;
    const long long es = 3LL * n * n + 2 * n, nn = (long long)n * n;
    double *W = A.xlw + (long long)blockIdx.x * slot;
    for (long long it = blockIdx.x; it < (long long)batch * S; it += gridDim.x) {
        const long long b = it / S;
        const int i = (int)(it % S);
        const long long is = A.istride ? A.istride : es;
        const double *in = A.in + b * (A.bstride ? A.bstride : (long long)S * es);
        double *o = A.out + b * (long long)S * es + (long long)i * es;
        if (i + d >= S) {  // block-uniform
            const double *src = in + (long long)i * is;
            for (long long q = threadIdx.x; q < es; q += 256) o[q] = src[q];
            __syncthreads();
            continue;
        }
        const bool fcf = !(A.terminal && i + 2 * d - 1 >= S - 1);
        const bool ok = xl_combine(o, o + nn, o + 2 * nn, o + 2 * nn + n, o + 3 * nn + n,
                                   elem_in(in + (long long)i * is, n), elem_in(in + (long long)(i + d) * is, n), n,
                                   fcf, true, LU, W, sm);
        if (!fcf)
            for (long long q = threadIdx.x; q < 2 * nn + n; q += 256) o[q] = 0.0;  // [F | C | f]
        if (!ok && threadIdx.x == 0) atomicOr(A.flag + b, 1);
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// boundary maps (k_seg_maps_wide): x_j = Phi_j x_{j-1} + phi_j, solved as
// (I + C P_j) [Phi | phi] = [F | f - C p_j]
// ---------------------------------------------------------------------------
template <bool LU>
__global__ __launch_bounds__(256) void k_seg_maps_xl(MapArgs A, int batch, long long slot) {
    __shared__ XlSm sm;
    const int tid = threadIdx.x;
    const int n = A.n, S = A.S, J = S + 1;
    const long long nn = (long long)n * n, es = 3 * nn + 2 * n, mw = nn + n;
    double *W = A.xlw + (long long)blockIdx.x * slot;
    double *const B0 = W, *const B1 = W + nn, *const B2 = W + 2 * nn, *const B3 = W + 3 * nn;
    for (long long it = blockIdx.x; it < (long long)batch * J; it += gridDim.x) {
        const long long b = it / J;
        const int j = (int)(it % J);
        const double *right = A.right ? A.right + b * (A.rstride ? A.rstride : es) : nullptr;
        double *vo = A.vfun + (b * J + j) * mw;
        double *mo = A.maps + (b * J + j) * mw;
        bool ok = true;
        const double *vP = nullptr, *vp = nullptr;
        if (j < S && right) {  // V_j = suf_j (x) right: (P, p) only
            ok = xl_combine(nullptr, nullptr, nullptr, vo, vo + nn, elem_in(A.suf + (b * S + j) * es, n),
                            elem_in(right, n), n, false, true, LU, W, sm);
            vP = vo;
            vp = vo + nn;
        } else {
            const double *src = j < S ? A.suf + (b * S + j) * es : right;
            if (src) {
                vP = src + 2 * nn + n;
                vp = src + 3 * nn + n;
            }
            for (long long q = tid; q < mw; q += 256) vo[q] = src ? (q < nn ? vP[q] : vp[q - nn]) : 0.0;
        }
        __syncthreads();
        const double *src = j > 0 ? A.elem + (b * S + j - 1) * es : A.left ? A.left + b * es : nullptr;
        double *phi = sm.v[5], *x = sm.v[6];
        const double *Phi = nullptr;  // the j = 0 map's matrix (workspace or the element's F) or null
        if (src && vP) {
            const ElemIn e = elem_in(src, n);
            double *pv = sm.v[0], *v = sm.v[2];
            blk_copy(B0, n, mv_n(e.C, n), n, n);
            blk_vcopy(pv, vp, n);
            blk_mv(v, mv_n(B0, n), pv, n, n, -1.0, e.f);  // f - C p_j
            if (!LU) {
                blk_copy(B1, n, mv_n(vP, n), n, n);
                ok = xl_chol(B1, n, n, sm.sinv) && ok;                                        // R
                xl_mm(B2, n, B0, n, false, B1, n, false, n, n, n, nullptr, 0);                // C R
                xl_mm(B3, n, B1, n, true, B2, n, false, n, n, n, nullptr, 0, 1.0, 1.0);       // I + R^T C R
                ok = xl_chol(B3, n, n, sm.sinv) && ok;                                        // Q
                xl_mm(B2, n, B1, n, true, e.F, n, false, n, n, n, nullptr, 0);                // R^T F
                blk_mv(phi, mv_t(B1, n), v, n, n, 1.0, nullptr);                              // R^T v
                blk_trsm_l(B3, n, n, B2, n, n, phi);   // Q^{-1}
                blk_trsm_lt(B3, n, n, B2, n, n, phi);  // Q^{-T}
                blk_trsm_lt(B1, n, n, B2, n, n, phi);  // R^{-T}
                if (j > 0) {
                    for (long long q = tid; q < nn; q += 256) mo[q] = B2[q];
                    for (int q = tid; q < n; q += 256) mo[nn + q] = phi[q];
                } else Phi = B2;
            } else {
                // W = [I + C P_j | F | v] in B1 | B2 | B3 (n x (2n + 1), ld n)
                xl_mm(B1, n, B0, n, false, vP, n, false, n, n, n, nullptr, 0, 1.0, 1.0);
                blk_copy(B2, n, mv_n(e.F, n), n, n);
                blk_vcopy(B3, v, n);
                ok = xl_gauss_jordan(B1, n, sm.piv, sm.prow, sm.mul, 2 * n + 1, sm.rv, sm.ra) && ok;
                for (long long q = tid; q < nn + n; q += 256) {  // row piv[i] of the right part: row i
                    const int i = (int)(q % n), jj = (int)(q / n);
                    const double xv = B2[sm.piv[i] + (long long)jj * n];
                    if (jj < n) {
                        if (j > 0) mo[q] = xv;
                        else B0[q] = xv;  // Phi of boundary 0 (C is no longer needed)
                    } else {
                        phi[i] = xv;
                        if (j > 0) mo[nn + i] = xv;
                    }
                }
                __syncthreads();
                if (j == 0) Phi = B0;
            }
        } else if (src) {
            const ElemIn e = elem_in(src, n);
            blk_vcopy(phi, e.f, n);
            if (j > 0)
                for (long long q = tid; q < mw; q += 256) mo[q] = q < nn ? e.F[q] : e.f[q - nn];
            else Phi = e.F;
        }
        if (!ok && tid == 0) atomicOr(A.flag + b, 2);
        if (j == 0) {  // x_0 = Phi x0 + phi (x0 itself without a global prefix), lambda_0 = P_0 x_0 + p_0
            double *x0 = sm.v[7];
            blk_vcopy(x0, A.x0 + b * (long long)n, n);
            if (Phi) blk_mv(x, mv_n(Phi, n), x0, n, n, 1.0, phi);
            else blk_vcopy(x, x0, n);
            for (int q = tid; q < n; q += 256) {
                mo[nn + q] = x[q];
                A.xhat[b * (long long)J * n + q] = x[q];
            }
            if (vP) blk_mv(A.lam + b * (long long)J * n, mv_n(vP, n), x, n, n, 1.0, vp);
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// one radix-4 round of the prefix composition of the boundary maps (k_map_scan_wide)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_map_scan_xl(MapScanArgs A, int batch, long long slot) {
    __shared__ double pacc[XL_S], po[XL_S];
    const int tid = threadIdx.x;
    const int n = A.n, J = A.S + 1, d = A.dist;
    const long long nn = (long long)n * n, mw = nn + n;
    double *W = A.xlw + (long long)blockIdx.x * slot;
    for (long long it = blockIdx.x; it < (long long)batch * J; it += gridDim.x) {
        const long long b = it / J;
        const int j = (int)(it % J);
        const double *in = A.in + b * J * mw;
        double *out = A.out + b * J * mw;
        if (j < d) {  // anchored earlier: keep x_j for this round's partners
            for (int q = tid; q < n; q += 256) out[(long long)j * mw + nn + q] = in[(long long)j * mw + nn + q];
            __syncthreads();
            continue;
        }
        double *Pacc = W, *T = W + nn;
        blk_copy(Pacc, n, mv_n(in + (long long)j * mw, n), n, n);
        blk_vcopy(pacc, in + (long long)j * mw + nn, n);
        bool done = false;
        for (int k = 1; k <= 3 && !done; ++k) {
            const int ia = j - k * d;  // >= 0: the previous partner was not anchored (>= d)
            const double *ea = in + (long long)ia * mw;
            blk_mv(po, mv_n(Pacc, n), ea + nn, n, n, 1.0, pacc);  // Phi_acc phi_a + phi_acc
            if (ia < d) {  // anchored partner: po = x_j
                for (int q = tid; q < n; q += 256) {
                    out[(long long)j * mw + nn + q] = po[q];
                    A.xhat[(b * J + j) * (long long)n + q] = po[q];
                }
                const double *v = A.vfun + (b * J + j) * mw;
                blk_mv(A.lam + (b * J + j) * (long long)n, mv_n(v, n), po, n, n, 1.0, v + nn);
                done = true;
                break;
            }
            xl_mm(T, n, Pacc, n, false, ea, n, false, n, n, n, nullptr, 0);  // Phi_acc Phi_a
            double *const t = Pacc;
            Pacc = T;
            T = t;
            blk_vcopy(pacc, po, n);
        }
        if (!done)
            for (long long q = tid; q < mw; q += 256) out[(long long)j * mw + q] = q < nn ? Pacc[q] : pacc[q - nn];
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// horizon shards: the boundary map of rank element e_j under V_{j+1}
// (k_rank_maps_wide), then their application to x0 in turn
// ---------------------------------------------------------------------------
template <bool LU>
__global__ __launch_bounds__(256) void k_rank_maps_xl(const double *elems_all, const double *suf, int R, int r, int n,
                                                     int batch, double *maps, int *flag, double *xlw, long long slot) {
    __shared__ XlSm sm;
    const long long nn = (long long)n * n, es = 3 * nn + 2 * n, mw = nn + n;
    double *W = xlw + (long long)blockIdx.x * slot;
    for (long long it = blockIdx.x; it < (long long)batch * r; it += gridDim.x) {
        const long long b = it / r;
        const int j = (int)(it % r);
        const ElemIn e = elem_in(elems_all + ((long long)j * batch + b) * es, n);  // rank-major all-gather
        const double *v = suf + (b * R + j + 1) * es;                               // V_{j+1}
        double *const B[5] = {W, W + nn, W + 2 * nn, W + 3 * nn, W + 4 * nn};
        double *pv = sm.v[0], *v2 = sm.v[2];
        double *mo = maps + (b * r + j) * mw;
        blk_copy(B[0], n, mv_n(e.C, n), n, n);
        blk_vcopy(pv, v + 3 * nn + n, n);
        blk_mv(v2, mv_n(B[0], n), pv, n, n, -1.0, e.f);  // f - C p
        int iy, iz, ifr;
        const bool ok = xl_core(B, v + 2 * nn + n, n, LU, sm, iy, iz, ifr);
        blk_mv(mo + nn, mv_n(B[iz], n), v2, n, n, 1.0, nullptr);                            // Z (f - C p)
        xl_mm(mo, n, B[iz], n, false, e.F, n, false, n, n, n, nullptr, 0);                   // Z F
        if (!ok && threadIdx.x == 0) atomicOr(flag + b, 4);
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_rank_chain_xl(const double *maps, const double *x0, int r, int n,
                                                      double *out_pre_all) {
    __shared__ double xa[XL_S], xb[XL_S];
    const int tid = threadIdx.x;
    const long long nn = (long long)n * n, es = 3 * nn + 2 * n, mw = nn + n;
    const long long b = blockIdx.x;
    if (tid < n) xa[tid] = x0[b * n + tid];
    __syncthreads();
    double *x = xa, *y = xb;
    for (int j = 0; j < r; ++j) {  // x <- Phi_j x + phi_j
        const double *mo = maps + (b * r + j) * mw;
        if (tid < n) {
            double a = mo[nn + tid];
            for (int t = 0; t < n; ++t) a = __builtin_fma(mo[tid + (long long)t * n], x[t], a);
            y[tid] = a;
        }
        __syncthreads();
        double *t = x;
        x = y;
        y = t;
    }
    double *out = out_pre_all + b * es;
    for (long long q = tid; q < es; q += 256) out[q] = (q >= 2 * nn && q < 2 * nn + n) ? x[q - 2 * nn] : 0.0;
}

// ---------------------------------------------------------------------------
// segment backward (k_seg_bwd_wide) for n + m > 64.  Workspace slot: Pm, Fm,
// Cm (n x n), XA = P E~, XB = F E~ (n x s), Mb (s x s).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_seg_bwd_xl(SegArgs A) {
    __shared__ double pv[XL_S], fv[XL_S], cv[XL_S], pc[XL_S], fy[XL_S], lp[XL_S], sinv[XL_S];
    __shared__ int s_bad;
    const int tid = threadIdx.x;
    const Shape &sh = A.sh;
    const int n = sh.n, m = sh.m, s = n + m, S = A.S, ps = sh.ps;
    const long long nn = (long long)n * n, frs = (long long)s * m + m;
    double *const Pm = xl_slot(A.xlw, sh), *const Fm = Pm + nn, *const Cm = Fm + nn, *const XA = Cm + nn,
                  *const XB = XA + (long long)n * s, *const Mb = XB + (long long)n * s;
    for (long long it = blockIdx.x; it < (long long)sh.batch * S; it += gridDim.x) {
        const long long bi = it / S;
        const int seg = (int)(it % S);
        if (A.flag && seg == 0 && tid == 0) A.flag[bi] = 0;
        const int N0 = A.seg_start[seg], N1 = N0 + A.seg_len[seg];
        const bool last = (seg == S - 1) && A.last_is_terminal;
        const double *Eb = A.E + bi * sh.perE;
        const double *cb = A.c + bi * sh.perc;
        const double *Hb = A.Hw + bi * sh.perHw;
        const double *hb = A.hw + bi * sh.perh;
        double *FRb = A.FR + bi * sh.perKD;
        double *Gb = A.G ? A.G + bi * (long long)sh.N * m * n : nullptr;
        double *Lcb = A.Lc ? A.Lc + bi * sh.perHw : nullptr;
        double *lpb = A.lpc ? A.lpc + bi * sh.perh : nullptr;
        int fail_stage = -1;
        // ---- segment terminal: the real one (P = H~_N, p = h~_N, F = 0) or the
        //      dummy (P = 0, p = 0, F = I, C = 0, f = 0) ----
        {
            const double *HN = Hb + (long long)sh.N * ps;
            if (tid == 0) s_bad = 0;
            __syncthreads();
            for (long long q = tid; q < nn; q += 256) {
                const int i = (int)(q % n), j = (int)(q / n);
                const double v = last ? HN[i >= j ? pidx(i, j, n) : pidx(j, i, n)] : 0.0;
                Pm[q] = v;
                Fm[q] = (!last && i == j) ? 1.0 : 0.0;
                Cm[q] = 0.0;
                if (last && i == j && psd_bad(v)) s_bad = 1;
            }
            for (int q = tid; q < n; q += 256) {
                pv[q] = last ? hb[(long long)sh.N * s + q] : 0.0;
                fv[q] = 0.0;
            }
            if (last) {
                const int pn = n * (n + 1) / 2;
                if (Lcb)
                    for (int t = tid; t < pn; t += 256) Lcb[(long long)sh.N * ps + t] = HN[t];
                if (lpb)
                    for (int t = tid; t < n; t += 256) lpb[(long long)sh.N * s + t] = hb[(long long)sh.N * s + t];
            }
            __syncthreads();
            if (s_bad) fail_stage = sh.N;
        }
        const bool yon = !last;  // the y block (F, C, f) is identically zero on the last segment
        for (int k = N1 - 1; k >= N0; --k) {
            const double *Ek = Eb + (long long)k * n * s;
            blk_vcopy(cv, cb + (long long)k * n, n);
            blk_mv(pc, mv_n(Pm, n), cv, n, n, 1.0, pv);  // P c + p
            if (tid == 0) s_bad = 0;  // every thread has read the previous stage's flag (blk_mv's barriers)
            if (yon) blk_mv(fy, mv_n(Fm, n), cv, n, n, 1.0, fv);  // F c + f
            xl_mm(XA, n, Pm, n, false, Ek, n, false, n, s, n, nullptr, 0);  // P E~
            if (yon) xl_mm(XB, n, Fm, n, false, Ek, n, false, n, s, n, nullptr, 0);  // F E~
            blk_mv(lp, mv_t(Ek, n), pc, s, n, 1.0, hb + (long long)k * s);  // h~ + E~^T (P c + p)
            for (long long q = tid; q < (long long)s * s; q += 256) {  // M = H~ + E~^T P E~
                const int i = (int)(q % s), j = (int)(q / s);
                Mb[q] = Hb[(long long)k * ps + (i >= j ? pidx(i, j, s) : pidx(j, i, s))];
            }
            xl_mm(Mb, s, Ek, n, true, XA, n, false, s, s, n, Mb, s);
            // ---- eliminate the u pivots of [[M, YE^T], [YE, -C]] (one barrier per pivot) ----
            double *FRk = FRb + (long long)k * frs;
            double *Gk = Gb ? Gb + (long long)k * m * n : nullptr;
            bool ok = true;
            for (int j = 0; j < m; ++j) {
                __syncthreads();
                const double d = Mb[j + (long long)j * s];
                ok = ok && d > 0.0;
                const double inv2 = 1.0 / d, invs = rsqrt_f64(d);
                const double lpj = lp[j];
                // column j is final: rollout record, coupling gain
                for (int i = tid; i < s; i += 256)
                    FRk[(long long)j * s + i] = i >= j ? Mb[i + (long long)j * s] * invs : 0.0;
                if (yon && Gk)
                    for (int r = tid; r < n; r += 256) Gk[j + r * m] = -XB[r + (long long)j * n] * invs;
                if (tid == 0) {
                    FRk[(long long)s * m + j] = lpj * invs;
                    sinv[j] = invs;
                }
                const int rr = s - j - 1;
                for (long long q = tid; q < (long long)rr * rr; q += 256) {
                    const int i = j + 1 + (int)(q % rr), l = j + 1 + (int)(q / rr);
                    if (l > i) continue;
                    Mb[i + (long long)l * s] = __builtin_fma(-Mb[i + (long long)j * s] * inv2, Mb[l + (long long)j * s],
                                                             Mb[i + (long long)l * s]);
                }
                for (int i = j + 1 + tid; i < s; i += 256) lp[i] = __builtin_fma(-Mb[i + (long long)j * s] * inv2, lpj, lp[i]);
                if (yon) {
                    for (long long q = tid; q < (long long)n * rr; q += 256) {
                        const int r = (int)(q % n), l = j + 1 + (int)(q / n);
                        XB[r + (long long)l * n] = __builtin_fma(-XB[r + (long long)j * n] * inv2,
                                                                 Mb[l + (long long)j * s], XB[r + (long long)l * n]);
                    }
                    for (long long q = tid; q < nn; q += 256) {
                        const int r = (int)(q % n), c = (int)(q / n);
                        if (c > r) continue;
                        Cm[q] = __builtin_fma(XB[r + (long long)j * n] * inv2, XB[c + (long long)j * n], Cm[q]);
                    }
                    for (int r = tid; r < n; r += 256) fy[r] = __builtin_fma(-XB[r + (long long)j * n] * inv2, lpj, fy[r]);
                }
            }
            __syncthreads();
            // ---- P_k (lower block, symmetric by construction), p_k, f_k, F_k ----
            for (long long q = tid; q < nn; q += 256) {
                const int i = (int)(q % n), j = (int)(q / n);
                const int hi = i > j ? i : j, lo = i > j ? j : i;
                const double v = Mb[(m + hi) + (long long)(m + lo) * s];
                Pm[q] = v;
                if (i == j && psd_bad(v)) s_bad = 1;
                if (Lcb && i >= j) Lcb[(long long)k * ps + pidx(i, j, n)] = v;
                if (yon) Fm[q] = XB[q + (long long)m * n];  // the y block's x columns
            }
            for (int q = tid; q < s; q += 256) {
                const double v = q < m ? lp[q] * sinv[q] : lp[q];  // [lu'; p_k]
                if (lpb) lpb[(long long)k * s + q] = v;
                if (q >= m) pv[q - m] = v;
            }
            if (yon)
                for (int q = tid; q < n; q += 256) fv[q] = fy[q];
            __syncthreads();
            if ((!ok || s_bad) && fail_stage < 0) fail_stage = k;
        }
        // ---- export the element (update_segment_data, lqr_solver_parallel.hpp:182-187) ----
        double *eo = A.elem + (bi * S + seg) * (3 * nn + 2 * n);
        double *eF = eo, *eC = eo + nn, *ef = eo + 2 * nn, *eP = ef + n, *ep = eP + nn;
        for (long long q = tid; q < nn; q += 256) {
            const int i = (int)(q % n), j = (int)(q / n);
            eP[q] = Pm[q];
            eF[q] = last ? 0.0 : Fm[q];
            eC[q] = last ? 0.0 : Cm[i >= j ? i + (long long)j * n : j + (long long)i * n];
        }
        for (int q = tid; q < n; q += 256) {
            ep[q] = pv[q];
            ef[q] = last ? 0.0 : fv[q];
        }
        if (tid == 0) A.seg_status[bi * S + seg] = fail_stage < 0 ? 0 : fail_stage + 1;
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// segment backward without factorization (k_seg_bwd_nofact) for n + m > 64:
// P_{k+1} from the value-function cache into the workspace slot (n x n)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_seg_bwd_nofact_xl(SegArgs A) {
    __shared__ double cvec[XL_S], va[XL_S], vb[XL_S], lp[XL_S], pn[XL_S], xs[XL_S], scr[XL_S];
    const int tid = threadIdx.x;
    const Shape &sh = A.sh;
    const int n = sh.n, m = sh.m, s = sh.s, S = A.S;
    const long long nn = (long long)n * n, frs = (long long)s * m + m;
    double *const Pn = xl_slot(A.xlw, sh);
    for (long long it = blockIdx.x; it < (long long)sh.batch * S; it += gridDim.x) {
        const long long b = it / S;
        const int seg = (int)(it % S);
        if (A.flag && seg == 0 && tid == 0) A.flag[b] = 0;
        const int N0 = A.seg_start[seg], N1 = N0 + A.seg_len[seg];
        const bool last = (seg == S - 1) && A.last_is_terminal;
        const double *Eb = A.E + b * sh.perE;
        const double *cb = A.c + b * sh.perc;
        const double *hb = A.hw + b * sh.perh;
        double *FRb = A.FR + b * sh.perKD;
        const double *Lcb = A.Lc + b * sh.perHw;
        double *lpb = A.lpc ? A.lpc + b * sh.perh : nullptr;
        auto load_P = [&](int k) {  // packed lower n x n at stage offset k ps -> dense
            __syncthreads();
            for (long long q = tid; q < nn; q += 256) {
                const int i = (int)(q % n), j = (int)(q / n);
                Pn[q] = Lcb[(long long)k * sh.ps + (i >= j ? pidx(i, j, n) : pidx(j, i, n))];
            }
            __syncthreads();
        };
        // segment terminal: the real one (lqr_kernel.hpp:94-101) or the dummy P = 0, p = 0
        for (int q = tid; q < n; q += 256) {
            pn[q] = last ? hb[(long long)sh.N * s + q] : 0.0;
            if (last && lpb) lpb[(long long)sh.N * s + q] = pn[q];
        }
        if (last) load_P(sh.N);
        else {
            for (long long q = tid; q < nn; q += 256) Pn[q] = 0.0;
            __syncthreads();
        }
        for (int k = N1 - 1; k >= N0; --k) {
            const double *Ek = Eb + (long long)k * n * s;
            const double *FRk = FRb + (long long)k * frs;  // L(i, j) = FRk[j s + i], j < m
            blk_vcopy(cvec, cb + (long long)k * n, n);
            blk_mv(vb, mv_n(Pn, n), cvec, n, n, 1.0, pn);                     // P_{k+1} c + p_{k+1}
            blk_mv(lp, mv_t(Ek, n), vb, s, n, 1.0, hb + (long long)k * s);   // h~ + E^T (P c + p)
            xl_solve_u(lp, FRk, s, m, s, scr);  // lu <- Luu^{-1} lu, p = lp_x - Lxu lu
            for (int q = tid; q < n; q += 256) pn[q] = lp[m + q];
            for (int q = tid; q < m; q += 256) FRb[(long long)k * frs + (long long)s * m + q] = lp[q];
            if (lpb)
                for (int q = tid; q < s; q += 256) lpb[(long long)k * s + q] = lp[q];
            load_P(k);
        }
        double *eo = A.elem + (b * S + seg) * (3 * nn + 2 * n);
        double *ep = eo + 3 * nn + n, *ef = eo + 2 * nn;
        for (int q = tid; q < n; q += 256) ep[q] = pn[q];
        if (last) {
            for (int q = tid; q < n; q += 256) ef[q] = 0.0;
            __syncthreads();
            continue;
        }
        // f: closed-loop rollout of the segment from x = 0 (u = -Luu^{-T}(lu' + Lxu^T x))
        for (int q = tid; q < n; q += 256) xs[q] = 0.0;
        __syncthreads();
        for (int k = N0; k < N1; ++k) {
            const double *Ek = Eb + (long long)k * n * s;
            const double *Fk = FRb + (long long)k * frs;
            for (int j = tid; j < m; j += 256) {
                double a = Fk[(long long)s * m + j];
                for (int i = 0; i < n; ++i) a = __builtin_fma(Fk[(long long)j * s + m + i], xs[i], a);
                va[j] = -a;
            }
            for (int j = m - 1; j >= 0; --j) {  // u = Luu^{-T} v
                __syncthreads();
                const double uj = va[j] / Fk[(long long)j * s + j];
                __syncthreads();
                for (int i = tid; i < j; i += 256) va[i] = __builtin_fma(-Fk[(long long)i * s + j], uj, va[i]);
                if (tid == 0) va[j] = uj;
            }
            __syncthreads();
            double xn = 0.0;
            if (tid < n) {
                xn = cb[(long long)k * n + tid];
                for (int j = 0; j < m; ++j) xn = __builtin_fma(Ek[tid + (long long)j * n], va[j], xn);
                for (int t = 0; t < n; ++t) xn = __builtin_fma(Ek[tid + (long long)(m + t) * n], xs[t], xn);
            }
            __syncthreads();
            if (tid < n) xs[tid] = xn;
            __syncthreads();
        }
        for (int q = tid; q < n; q += 256) ef[q] = xs[q];
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// segment rollout (k_riccati_fwd_big<true>) for n + m > 64: one block per segment
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_fwd_seg_xl(Shape sh, const double *__restrict__ E,
                                                   const double *__restrict__ c, const double *__restrict__ FR,
                                                   double *__restrict__ ws, SegFwd sf) {
    __shared__ double w[XL_S], uh[XL_S], v[XL_S];
    const int tid = threadIdx.x;
    const long long b = blockIdx.x / sf.S;
    const int seg = blockIdx.x % sf.S;
    const int n = sh.n, m = sh.m, N = sh.N, s = sh.s;
    const int K0 = sf.seg_start[seg], K1 = K0 + sf.seg_len[seg];
    const bool last = seg == sf.S - 1 && sf.last_is_terminal;
    const long long frs = (long long)s * m + m;
    const double *Eb = E + b * sh.perE;
    const double *cb = c + b * sh.perc;
    const double *Fb = FR + b * sh.perKD;
    const double *Gb = sf.G + b * (long long)N * m * n;
    double *wb = ws + b * sh.perh;
    const double *xh = sf.xhat + b * (sf.S + 1) * (long long)n;
    for (int q = tid; q < n; q += 256) {
        const double x = xh[(long long)seg * n + q];
        w[m + q] = x;
        uh[q] = last ? 0.0 : sf.lam[(b * (sf.S + 1) + seg + 1) * n + q];
        wb[(long long)K0 * s + m + q] = x;  // ws[N0].tail(n) = x_hat
        if (!last && seg == sf.S - 1) wb[(long long)K1 * s + q] = xh[(long long)sf.S * n + q];
    }
    __syncthreads();
    for (int k = K0; k < K1; ++k) {
        const double *Fk = Fb + (long long)k * frs;
        // v_j = -(lu'_j + sum_i Lxu(i, j) x_i - sum_t G(j, t) u_hat_t)
        for (int j = tid; j < m; j += 256) {
            double a = Fk[(long long)s * m + j];
            for (int i = 0; i < n; ++i) a = __builtin_fma(Fk[(long long)j * s + m + i], w[m + i], a);
            if (!last) {
                const double *Gk = Gb + (long long)k * m * n;
                for (int t = 0; t < n; ++t) a = __builtin_fma(-Gk[j + (long long)t * m], uh[t], a);
            }
            v[j] = -a;
        }
        for (int j = m - 1; j >= 0; --j) {  // u = Luu^{-T} v
            __syncthreads();
            const double uj = v[j] / Fk[(long long)j * s + j];
            __syncthreads();
            for (int i = tid; i < j; i += 256) v[i] = __builtin_fma(-Fk[(long long)i * s + j], uj, v[i]);
            if (tid == 0) v[j] = uj;
        }
        __syncthreads();
        for (int j = tid; j < m; j += 256) {
            w[j] = v[j];
            wb[(long long)k * s + j] = v[j];
        }
        __syncthreads();
        const bool upd = last || (k < K1 - 1);  // update_x_next
        double xn = 0.0;  // x+ = c + E [u; x], one state row per thread
        if (tid < n) {
            const double *Ek = Eb + (long long)k * n * s;
            xn = cb[(long long)k * n + tid];
            for (int j = 0; j < s; ++j) xn = __builtin_fma(Ek[tid + (long long)j * n], w[j], xn);
        }
        __syncthreads();
        if (tid < n && upd) {
            w[m + tid] = xn;
            wb[(long long)(k + 1) * s + ((k + 1 < N) ? m : 0) + tid] = xn;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
int xl_par_slots(int device) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
    return 2 * cus;  // two blocks a CU: one's pivot barriers under the other's products
}

static unsigned xl_grid_of(long long items, int xl_grid) {
    return (unsigned)std::max<long long>(1, std::min<long long>(items, xl_grid));
}

static int xl_missing(const char *what) {
    set_error(std::string(what) + ": no XL workspace (n + m > 64 / n > 64)");
    return PDPLQR_ERR_UNSUPPORTED;
}

int launch_seg_backward_xl(const SegArgs &a, hipStream_t st) {
    if (!a.xlw || a.xl_grid <= 0) return xl_missing("segment backward");
    hipLaunchKernelGGL(k_seg_bwd_xl, dim3(xl_grid_of((long long)a.sh.batch * a.S, a.xl_grid)), dim3(256), 0, st, a);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

int launch_seg_backward_nofact_xl(const SegArgs &a, hipStream_t st) {
    if (!a.xlw || a.xl_grid <= 0) return xl_missing("segment backward_without_factorization");
    if (!a.Lc) {
        set_error("PARALLEL backward_without_factorization needs keep_factors = 1");
        return PDPLQR_ERR_UNSUPPORTED;
    }
    hipLaunchKernelGGL(k_seg_bwd_nofact_xl, dim3(xl_grid_of((long long)a.sh.batch * a.S, a.xl_grid)), dim3(256), 0, st,
                       a);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

static long long elem_slot(int n) { return 5LL * n * n; }

int launch_seg_scan_xl(const ScanArgs &a, int batch, hipStream_t st) {
    if (!a.xlw || a.xl_grid <= 0) return xl_missing("suffix scan");
    if (a.sk) return PDPLQR_ERR_UNSUPPORTED;  // Hillis-Steele rounds only (operands read from HBM)
    const dim3 g(xl_grid_of((long long)batch * a.S, a.xl_grid));
    if (a.lu) hipLaunchKernelGGL(k_seg_scan_xl<true>, g, dim3(256), 0, st, a, batch, elem_slot(a.n));
    else hipLaunchKernelGGL(k_seg_scan_xl<false>, g, dim3(256), 0, st, a, batch, elem_slot(a.n));
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

int launch_seg_maps_xl(const MapArgs &a, int batch, hipStream_t st) {
    if (!a.xlw || a.xl_grid <= 0) return xl_missing("boundary maps");
    const dim3 g(xl_grid_of((long long)batch * (a.S + 1), a.xl_grid));
    if (a.lu) hipLaunchKernelGGL(k_seg_maps_xl<true>, g, dim3(256), 0, st, a, batch, elem_slot(a.n));
    else hipLaunchKernelGGL(k_seg_maps_xl<false>, g, dim3(256), 0, st, a, batch, elem_slot(a.n));
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

int launch_map_scan_xl(const MapScanArgs &a, int batch, hipStream_t st) {
    if (!a.xlw || a.xl_grid <= 0) return xl_missing("map composition");
    static_assert(PDPLQR_MAP_RADIX == 4, "k_map_scan_xl composes radix-4 rounds");
    hipLaunchKernelGGL(k_map_scan_xl, dim3(xl_grid_of((long long)batch * (a.S + 1), a.xl_grid)), dim3(256), 0, st, a,
                       batch, elem_slot(a.n));
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

int launch_rank_fold_maps_xl(const double *elems, const double *suf, const double *x0, int R, int r, int n, int batch,
                             double *maps, double *out_pre, int *flag, bool lu, double *xlw, int xl_grid,
                             hipStream_t st) {
    if (!xlw || xl_grid <= 0) return xl_missing("rank maps");
    const dim3 g(xl_grid_of((long long)batch * r, xl_grid));
    if (lu)
        hipLaunchKernelGGL(k_rank_maps_xl<true>, g, dim3(256), 0, st, elems, suf, R, r, n, batch, maps, flag, xlw,
                           elem_slot(n));
    else
        hipLaunchKernelGGL(k_rank_maps_xl<false>, g, dim3(256), 0, st, elems, suf, R, r, n, batch, maps, flag, xlw,
                           elem_slot(n));
    hipLaunchKernelGGL(k_rank_chain_xl, dim3((unsigned)batch), dim3(256), 0, st, maps, x0, r, n, out_pre);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

int launch_riccati_forward_seg_xl(const Shape &sh, const double *E, const double *c, const double *FR,
                                  const SegFwd &sf, double *ws, hipStream_t st) {
    hipLaunchKernelGGL(k_fwd_seg_xl, dim3((unsigned)(sh.batch * sf.S)), dim3(256), 0, st, sh, E, c, FR, ws, sf);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

}  // namespace pdplqr
