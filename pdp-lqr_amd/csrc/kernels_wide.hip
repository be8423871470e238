// kernels_wide.hip -- the PARALLEL solver for the wide shapes 32 < n + m <= 64
// (and state sizes 32 < n <= 63), one 256-thread block per segment / element
// with the matrices in LDS (blk_la.hpp).
//
// Same algorithm and outputs as the tiled kernels (kernels_segment.hip,
// kernels_parallel.hip), restating the same reference code:
//   * k_seg_bwd_wide: ParallelLQRKernel::step_with_factorization
//     (lqr_kernel_parallel.hpp:88-136) over a segment in the augmented value
//     form of kernels_segment.hip: per stage
//         PE = P E~,  YE = F E~,  M = H~ + E~^T PE,
//         eliminate the m u-pivots of [[M, YE^T], [YE, -C]] with the aug
//         column [h~ + E~^T (P c + p); F c + f]
//     which leaves P_k, F_k, C_k, p_k, f_k (no x pivots, no n^3 recursion).
//     Records: FR_k = [L(:, 0:m) | lu'], G_k, the factor cache P_k / lp_k.
//   * wide_combine: the element combine (condensed_system.hpp
//     :203-290 Cholesky form, :82-137 LU form) in the formulas of
//     combine_tiles.hpp (Y = P_b (I + C_a P_b)^{-1}, Z = I - C_a Y).
//   * k_seg_scan_wide / k_seg_maps_wide / k_map_scan_wide: one scan round,
//     the boundary maps and one radix-4 composition round, as k_seg_scan,
//     k_seg_maps, k_map_scanR.
// Every blk_* call is a block-wide step bracketed by barriers (blk_la.hpp).
#include "blk_la.hpp"
#include "combine_tiles.hpp"  // ElemIn, elem_in
#include "parallel.hpp"

namespace pdplqr {

namespace {
constexpr int VL = 64;  // vector slot length (doubles)
}

// ---------------------------------------------------------------------------
// element kernels: LDS = 4 n x n matrices (B0..B3, B1 | B2 contiguous for the
// Gauss-Jordan [A | R]), 8 vectors, pivot scratch
// ---------------------------------------------------------------------------
struct WideSmem {
    double *B[4];
    double *v[8];
    double *prow, *mul, *sinv;
    int *piv;
};

static size_t wide_elem_smem_bytes(int n) {
    return (size_t)(4 * n * n + 8 * VL + 2 * VL + VL + VL) * sizeof(double) + VL * sizeof(int);
}

__device__ __forceinline__ WideSmem wide_smem(double *base, int n) {
    WideSmem s;
    for (int q = 0; q < 4; ++q) s.B[q] = base + q * n * n;
    double *v = base + 4 * n * n;
    for (int q = 0; q < 8; ++q) s.v[q] = v + q * VL;
    s.prow = v + 8 * VL;
    s.mul = s.prow + 2 * VL;
    s.sinv = s.mul + VL;
    s.piv = reinterpret_cast<int *>(s.sinv + VL);
    return s;
}

// Y = P_b (I + C_a P_b)^{-1}, Z = I - C_a Y with C_a in B0 (LDS) and P_b a
// global n x n block.  Returns the buffers holding Y, Z and the free one.
// Cholesky form: R = chol(P_b), S = I + R^T C_a R = Q Q^T, U = Q^{-1} R^T
// (R^T carried through the elimination of S), Y = U^T U.  LU form:
// Gauss-Jordan with partial pivoting on [I + P_b C_a | P_b], Y symmetrised.
__device__ __noinline__ bool wide_core(const WideSmem &sm, const double *Pb, int n, bool lu, double **Y, double **Z,
                                       double **Fr) {
    double *B0 = sm.B[0], *B1 = sm.B[1], *B2 = sm.B[2], *B3 = sm.B[3];
    bool ok;
    if (!lu) {
        blk_copy(B1, n, mv_n(Pb, n), n, n);
        ok = blk_chol(B1, n, n, n, sm.sinv);                                         // R
        blk_mm(B2, n, mv_n(B0, n), mv_n(B1, n), n, n, n, 1.0, 0.0, mv_none(), false);  // C_a R
        blk_mm(B3, n, mv_t(B1, n), mv_n(B2, n), n, n, n, 1.0, 1.0, mv_none(), true);   // I + R^T C_a R
        blk_copy(B2, n, mv_t(B1, n), n, n);                                          // R^T
        ok = blk_chol(B3, n, n, n, sm.sinv, B2, n, n) && ok;                         // U = Q^{-1} R^T
        blk_mm(B1, n, mv_t(B2, n), mv_n(B2, n), n, n, n, 1.0, 0.0, mv_none(), true);   // Y = U^T U
        blk_mm(B3, n, mv_n(B0, n), mv_n(B1, n), n, n, n, -1.0, 1.0, mv_none(), false);  // Z = I - C_a Y
        *Y = B1;
        *Z = B3;
        *Fr = B2;
    } else {
        blk_mm(B1, n, mv_n(Pb, n), mv_n(B0, n), n, n, n, 1.0, 1.0, mv_none(), false);  // I + P_b C_a
        blk_copy(B2, n, mv_n(Pb, n), n, n);                                           // P_b
        ok = blk_gauss_jordan(B1, n, sm.piv, sm.prow, sm.mul, 2 * n);
        for (int q = threadIdx.x; q < n * n; q += BLK_THREADS) {
            const int i = q % n, j = q / n;
            B3[q] = 0.5 * (B2[sm.piv[i] + j * n] + B2[sm.piv[j] + i * n]);
        }
        blk_mm(B1, n, mv_n(B0, n), mv_n(B3, n), n, n, n, -1.0, 1.0, mv_none(), false);  // Z = I - C_a Y
        *Y = B3;
        *Z = B1;
        *Fr = B2;
    }
    return ok;
}

// out = a (x) b, the output blocks addressed separately (see tcombine_parts);
// fcf: form F, C, f; pp: form P, p.  Outputs must not alias the inputs.
__device__ __noinline__ bool wide_combine(double *oF, double *oC, double *of, double *oP, double *op, ElemIn ea,
                                          ElemIn eb, int n, bool fcf, bool pp, bool lu, const WideSmem &sm) {
    double *B0 = sm.B[0];
    double *pb = sm.v[0], *fa = sm.v[1], *v1 = sm.v[2], *v3 = sm.v[3], *t4 = sm.v[4], *t5 = sm.v[5];
    blk_copy(B0, n, mv_n(ea.C, n), n, n);  // C_a
    blk_vcopy(pb, eb.p, n);
    blk_vcopy(fa, ea.f, n);
    if (fcf) blk_mv(v1, mv_n(B0, n), pb, n, n, -1.0, fa);  // f_a - C_a p_b
    if (pp) blk_mv(v3, mv_n(eb.P, n), fa, n, n, 1.0, pb);  // p_b + P_b f_a
    double *Y, *Z, *Fr;
    const bool ok = wide_core(sm, eb.P, n, lu, &Y, &Z, &Fr);
    if (pp) {
        blk_copy(Fr, n, mv_n(ea.F, n), n, n);                                                 // F_a
        blk_mm(Y, n, mv_n(Y, n), mv_n(Fr, n), n, n, n, 1.0, 0.0, mv_none(), false);             // Y F_a
        blk_mm(Y, n, mv_t(Fr, n), mv_n(Y, n), n, n, n, 1.0, 0.0, mv_n(ea.P, n), false);         // P_a + F_a^T Y F_a
        blk_store_sym(oP, n, Y, n, n);
        blk_mv(t4, mv_t(Z, n), v3, n, n, 1.0, nullptr);                                        // Z^T v3
        blk_mv(op, mv_t(Fr, n), t4, n, n, 1.0, ea.p);                                          // p_a + F_a^T Z^T v3
    }
    if (fcf) {
        if (!pp) blk_copy(Fr, n, mv_n(ea.F, n), n, n);
        blk_mm(Y, n, mv_n(Z, n), mv_n(Fr, n), n, n, n, 1.0, 0.0, mv_none(), false);   // Z F_a (Y is free)
        blk_copy(Fr, n, mv_n(eb.F, n), n, n);                                         // F_b
        blk_mm(oF, n, mv_n(Fr, n), mv_n(Y, n), n, n, n, 1.0, 0.0, mv_none(), false);  // F_b Z F_a
        blk_mm(Y, n, mv_n(Z, n), mv_n(B0, n), n, n, n, 1.0, 0.0, mv_none(), false);   // Z C_a
        blk_mm(Y, n, mv_n(Y, n), mv_t(Fr, n), n, n, n, 1.0, 0.0, mv_none(), false);   // Z C_a F_b^T
        blk_mv(t5, mv_n(Z, n), v1, n, n, 1.0, nullptr);                              // Z v1
        blk_mm(Z, n, mv_n(Fr, n), mv_n(Y, n), n, n, n, 1.0, 0.0, mv_n(eb.C, n), false);  // F_b Z C_a F_b^T + C_b
        blk_store_sym(oC, n, Z, n, n);
        blk_mv(of, mv_n(Fr, n), t5, n, n, 1.0, eb.f);  // F_b Z v1 + f_b
    }
    return ok;
}

// ---------------------------------------------------------------------------
// one Hillis-Steele round of the suffix scan (k_seg_scan)
// ---------------------------------------------------------------------------
template <bool LU>
__global__ __launch_bounds__(256) void k_seg_scan_wide(ScanArgs A) {
    extern __shared__ __attribute__((aligned(16))) double wbuf[];
    const int n = A.n, S = A.S, d = A.dist;
    const int es = 3 * n * n + 2 * n, nn = n * n;
    const long long b = blockIdx.x / S;
    const int i = blockIdx.x % S;
    const long long is = A.istride ? A.istride : es;
    const double *in = A.in + b * (A.bstride ? A.bstride : (long long)S * es);
    double *out = A.out + b * (long long)S * es;
    double *o = out + (long long)i * es;
    if (i + d >= S) {  // block-uniform
        const double *src = in + (long long)i * is;
        for (int q = threadIdx.x; q < es; q += BLK_THREADS) o[q] = src[q];
        return;
    }
    const bool fcf = !(A.terminal && i + 2 * d - 1 >= S - 1);
    const WideSmem sm = wide_smem(wbuf, n);
    const bool ok = wide_combine(o, o + nn, o + 2 * nn, o + 2 * nn + n, o + 3 * nn + n,
                                 elem_in(in + (long long)i * is, n), elem_in(in + (long long)(i + d) * is, n), n, fcf,
                                 true, LU, sm);
    if (!fcf)
        for (int q = threadIdx.x; q < 2 * nn + n; q += BLK_THREADS) o[q] = 0.0;  // [F | C | f]
    if (!ok && threadIdx.x == 0) atomicOr(A.flag + b, 1);
}

// ---------------------------------------------------------------------------
// boundary maps (k_seg_maps): x_j = Phi_j x_{j-1} + phi_j, Phi = Z F,
// phi = Z (f - C p_j), Z = (I + C P_j)^{-1}
// ---------------------------------------------------------------------------
template <bool LU>
__global__ __launch_bounds__(256) void k_seg_maps_wide(MapArgs A) {
    extern __shared__ __attribute__((aligned(16))) double wbuf[];
    const int tid = threadIdx.x;
    const int n = A.n, S = A.S, J = S + 1, nn = n * n;
    const int es = 3 * nn + 2 * n, mw = nn + n;
    const long long b = blockIdx.x / J;
    const int j = blockIdx.x % J;
    const WideSmem sm = wide_smem(wbuf, n);
    const double *right = A.right ? A.right + b * (A.rstride ? A.rstride : (long long)es) : nullptr;
    double *vo = A.vfun + (b * J + j) * (long long)mw;
    double *mo = A.maps + (b * J + j) * (long long)mw;
    bool ok = true;
    const double *vP = nullptr, *vp = nullptr;
    if (j < S && right) {  // V_j = suf_j (x) right: (P, p) only
        ok = wide_combine(nullptr, nullptr, nullptr, vo, vo + nn, elem_in(A.suf + (b * S + j) * (long long)es, n),
                          elem_in(right, n), n, false, true, LU, sm);
        __threadfence_block();
        __syncthreads();
        vP = vo;
        vp = vo + nn;
    } else {
        const double *src = j < S ? A.suf + (b * S + j) * (long long)es : right;
        if (src) {
            vP = src + 2 * nn + n;
            vp = src + 3 * nn + n;
        }
        for (int q = tid; q < mw; q += BLK_THREADS) vo[q] = src ? (q < nn ? vP[q] : vp[q - nn]) : 0.0;
    }
    const double *src = j > 0 ? A.elem + (b * S + j - 1) * (long long)es : A.left ? A.left + b * (long long)es
                                                                                 : nullptr;
    double *phi = sm.v[5], *x = sm.v[6];
    double *Phi = nullptr;  // LDS n x n (j = 0 with a value function) or null
    const double *PhiG = nullptr;  // the map's matrix in global memory (no value function)
    if (src && vP) {
        // Phi = Z F, phi = Z (f - C p_j) with Z = (I + C P_j)^{-1} as a SOLVE of
        // (I + C P_j) [Phi | phi] = [F | f - C p_j] -- not I - C Y times the
        // right-hand side: when C P_j is large (|CP| ~ 1e4 at 50/10 with
        // penalties) Z is small and I - C Y cancels, costing ~4 digits per map
        // (boundary states 1e-10 off instead of 1e-12, tests/test_gpu_wide.py).
        //   CHOLESKY: R = chol(P_j), S = I + R^T C R = Q Q^T,
        //             [Phi | phi] = R^{-T} Q^{-T} Q^{-1} R^T [F | v]
        //   LU:       Gauss-Jordan with partial pivoting on [I + C P_j | F | v]
        //             (the reference LU form factors I + C P with PartialPivLU)
        const ElemIn e = elem_in(src, n);
        double *B0 = sm.B[0], *B1 = sm.B[1], *B2 = sm.B[2], *B3 = sm.B[3];
        double *pv = sm.v[0], *v = sm.v[2];
        blk_copy(B0, n, mv_n(e.C, n), n, n);
        blk_vcopy(pv, vp, n);
        blk_mv(v, mv_n(B0, n), pv, n, n, -1.0, e.f);  // f - C p_j
        Phi = j > 0 ? nullptr : B2;
        if (!LU) {
            blk_copy(B1, n, mv_n(vP, n), n, n);
            ok = blk_chol(B1, n, n, n, sm.sinv) && ok;                                       // R
            blk_mm(B2, n, mv_n(B0, n), mv_n(B1, n), n, n, n, 1.0, 0.0, mv_none(), false);   // C R
            blk_mm(B3, n, mv_t(B1, n), mv_n(B2, n), n, n, n, 1.0, 1.0, mv_none(), true);    // I + R^T C R
            ok = blk_chol(B3, n, n, n, sm.sinv) && ok;                                       // Q
            blk_mm(B2, n, mv_t(B1, n), mv_n(e.F, n), n, n, n, 1.0, 0.0, mv_none(), false);  // R^T F
            blk_mv(phi, mv_t(B1, n), v, n, n, 1.0, nullptr);                                // R^T v
            blk_trsm_l(B3, n, n, B2, n, n, phi);   // Q^{-1}
            blk_trsm_lt(B3, n, n, B2, n, n, phi);  // Q^{-T}
            blk_trsm_lt(B1, n, n, B2, n, n, phi);  // R^{-T}
            if (j > 0) {
                for (int q = tid; q < nn; q += BLK_THREADS) mo[q] = B2[q];
                for (int q = tid; q < n; q += BLK_THREADS) mo[nn + q] = phi[q];
            }
        } else {
            // W = [I + C P_j | F | v] in B1 | B2 | B3 (n x (2n + 1), ld n)
            blk_mm(B1, n, mv_n(B0, n), mv_n(vP, n), n, n, n, 1.0, 1.0, mv_none(), false);
            blk_copy(B2, n, mv_n(e.F, n), n, n);
            blk_vcopy(B3, v, n);
            ok = blk_gauss_jordan(B1, n, sm.piv, sm.prow, sm.mul, 2 * n + 1) && ok;
            // row piv[i] of the right part is row i of the solution
            for (int q = tid; q < nn + n; q += BLK_THREADS) {
                const int i = q % n, jj = q / n;  // jj = n: the vector column
                const double x = B2[sm.piv[i] + jj * n];
                if (jj < n) {
                    if (j > 0) mo[q] = x;
                    else B0[q] = x;  // Phi of boundary 0 (C is no longer needed)
                } else {
                    phi[i] = x;
                    if (j > 0) mo[nn + i] = x;
                }
            }
            __syncthreads();
            if (j == 0) Phi = B0;
        }
    } else if (src) {
        const ElemIn e = elem_in(src, n);
        blk_vcopy(phi, e.f, n);
        if (j > 0)
            for (int q = tid; q < mw; q += BLK_THREADS) mo[q] = q < nn ? e.F[q] : e.f[q - nn];
        else PhiG = e.F;
    }
    if (!ok && tid == 0) atomicOr(A.flag + b, 2);
    if (j > 0) return;
    // j = 0: x_0 = Phi x0 + phi (x0 itself without a global prefix), lambda_0 = P_0 x_0 + p_0
    double *x0 = sm.v[7];
    blk_vcopy(x0, A.x0 + b * (long long)n, n);
    if (Phi) blk_mv(x, mv_n(Phi, n), x0, n, n, 1.0, phi);
    else if (PhiG) blk_mv(x, mv_n(PhiG, n), x0, n, n, 1.0, phi);
    else blk_vcopy(x, x0, n);
    for (int q = tid; q < n; q += BLK_THREADS) {
        mo[nn + q] = x[q];
        A.xhat[b * (long long)J * n + q] = x[q];
    }
    if (vP) blk_mv(A.lam + b * (long long)J * n, mv_n(vP, n), x, n, n, 1.0, vp);
}

// ---------------------------------------------------------------------------
// one radix-4 round of the prefix composition of the boundary maps (k_map_scanR at radix 4)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_map_scan_wide(MapScanArgs A) {
    extern __shared__ __attribute__((aligned(16))) double wbuf[];
    const int tid = threadIdx.x;
    const int n = A.n, J = A.S + 1, d = A.dist, nn = n * n, mw = nn + n;
    const long long b = blockIdx.x / J;
    const int j = blockIdx.x % J;
    const double *in = A.in + b * (long long)J * mw;
    double *out = A.out + b * (long long)J * mw;
    if (j < d) {  // anchored earlier: keep x_j for this round's partners
        for (int q = tid; q < n; q += BLK_THREADS) out[(long long)j * mw + nn + q] = in[(long long)j * mw + nn + q];
        return;
    }
    double *Pacc = wbuf, *pacc = wbuf + nn, *po = pacc + VL;
    blk_copy(Pacc, n, mv_n(in + (long long)j * mw, n), n, n);
    blk_vcopy(pacc, in + (long long)j * mw + nn, n);
#pragma unroll 1
    for (int k = 1; k <= 3; ++k) {
        const int ia = j - k * d;  // >= 0: the previous partner was not anchored (>= d)
        const double *ea = in + (long long)ia * mw;
        blk_mv(po, mv_n(Pacc, n), ea + nn, n, n, 1.0, pacc);  // Phi_acc phi_a + phi_acc
        if (ia < d) {  // anchored partner: po = x_j
            for (int q = tid; q < n; q += BLK_THREADS) {
                out[(long long)j * mw + nn + q] = po[q];
                A.xhat[(b * J + j) * (long long)n + q] = po[q];
            }
            const double *v = A.vfun + (b * J + j) * (long long)mw;
            blk_mv(A.lam + (b * J + j) * (long long)n, mv_n(v, n), po, n, n, 1.0, v + nn);
            return;
        }
        blk_mm(Pacc, n, mv_n(Pacc, n), mv_n(ea, n), n, n, n, 1.0, 0.0, mv_none(), false);  // Phi_acc Phi_a
        blk_vcopy(pacc, po, n);
    }
    for (int q = tid; q < mw; q += BLK_THREADS) out[(long long)j * mw + q] = q < nn ? Pacc[q] : pacc[q - nn];
}

// ---------------------------------------------------------------------------
// horizon shards, log-depth prefix (k_rank_maps / k_rank_chain): the boundary
// map of rank element e_j under V_{j+1} (suffix entry j + 1 of the rank scan),
// then their application to x0 in turn
// ---------------------------------------------------------------------------
template <bool LU>
__global__ __launch_bounds__(256) void k_rank_maps_wide(const double *elems_all, const double *suf, int R, int r,
                                                        int n, int batch, double *maps, int *flag) {
    extern __shared__ __attribute__((aligned(16))) double wbuf[];
    const int nn = n * n, es = 3 * nn + 2 * n, mw = nn + n;
    const long long b = blockIdx.x / r;
    const int j = blockIdx.x % r;
    const ElemIn e = elem_in(elems_all + ((long long)j * batch + b) * es, n);  // rank-major all-gather
    const double *v = suf + (b * R + j + 1) * (long long)es;                  // V_{j+1}
    const WideSmem sm = wide_smem(wbuf, n);
    double *B0 = sm.B[0], *pv = sm.v[0], *v2 = sm.v[2];
    double *mo = maps + (b * r + j) * (long long)mw;
    blk_copy(B0, n, mv_n(e.C, n), n, n);
    blk_vcopy(pv, v + 3 * nn + n, n);
    blk_mv(v2, mv_n(B0, n), pv, n, n, -1.0, e.f);  // f - C p
    double *Y, *Z, *Fr;
    const bool ok = wide_core(sm, v + 2 * nn + n, n, LU, &Y, &Z, &Fr);
    blk_mv(mo + nn, mv_n(Z, n), v2, n, n, 1.0, nullptr);                               // Z (f - C p)
    blk_mm(mo, n, mv_n(Z, n), mv_n(e.F, n), n, n, n, 1.0, 0.0, mv_none(), false);  // Z F
    if (!ok && threadIdx.x == 0) atomicOr(flag + b, 4);
}

__global__ __launch_bounds__(64) void k_rank_chain_wide(const double *maps, const double *x0, int r, int n,
                                                        double *out_pre_all) {
    __shared__ double xa[64], xb[64];
    const int lane = threadIdx.x;
    const int nn = n * n, es = 3 * nn + 2 * n, mw = nn + n;
    const long long b = blockIdx.x;
    if (lane < n) xa[lane] = x0[b * n + lane];
    wave_sync();
    double *x = xa, *y = xb;
    for (int j = 0; j < r; ++j) {  // x <- Phi_j x + phi_j
        const double *mo = maps + (b * r + j) * (long long)mw;
        if (lane < n) {
            double a = mo[nn + lane];
            for (int t = 0; t < n; ++t) a = __builtin_fma(mo[lane + t * n], x[t], a);
            y[lane] = a;
        }
        wave_sync();
        double *t = x;
        x = y;
        y = t;
    }
    double *out = out_pre_all + b * es;
    for (int q = lane; q < es; q += 64) out[q] = (q >= 2 * nn && q < 2 * nn + n) ? x[q - 2 * nn] : 0.0;
}

int launch_rank_fold_maps_wide(const double *elems, const double *suf, const double *x0, int R, int r, int n,
                               int batch, double *maps, double *out_pre, int *flag, bool lu, hipStream_t st) {
    const size_t sm = wide_elem_smem_bytes(n);
    const void *k = lu ? reinterpret_cast<const void *>(&k_rank_maps_wide<true>)
                       : reinterpret_cast<const void *>(&k_rank_maps_wide<false>);
    if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm) != hipSuccess) {
        set_error("rank maps (n > 32): LDS request too large");
        return PDPLQR_ERR_UNSUPPORTED;
    }
    void *args[] = {const_cast<double **>(&elems), const_cast<double **>(&suf), &R, &r, &n, &batch, &maps, &flag};
    PDPLQR_HIP_TRY(hipLaunchKernel(k, dim3((unsigned)(batch * r)), dim3(256), args, sm, st));
    hipLaunchKernelGGL(k_rank_chain_wide, dim3((unsigned)batch), dim3(64), 0, st, maps, x0, r, n, out_pre);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

// ---------------------------------------------------------------------------
// segment backward (k_seg_bwd_aug) for n + m > 32
// LDS: XA (n x s: P, then P E~), XB (n x s: F at column offset 0 or m, then
// F E~), Mb (s x s: E~, then the stage matrix), Cm (n x n), vectors.
// ---------------------------------------------------------------------------
// serial (the value-form serial backward, SegArgs::serial): no y block (XB,
// Cm), so more blocks fit a CU (50/10: 115 -> 71 KB, two blocks a CU)
static size_t wide_seg_smem_bytes(int n, int s, bool serial = false) {
    return (size_t)((serial ? 1 : 2) * n * s + s * s + (serial ? 0 : n * n) + s * (s + 1) / 2 + 8 * VL) *
           sizeof(double);
}

// Stage inputs of stage k in flight in registers (issued before the pivot
// loop of stage k + 1, written to LDS after it): E~ (<= 16 per thread), packed
// H~ (<= 9), c, h~.
struct WideIn {
    double E[16], H[9], c, h;
};

__device__ __forceinline__ void wide_in_load(WideIn &in, const double *Ek, const double *Hk, const double *ck,
                                             const double *hk, int n, int s, int ps) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int i = tid + q * BLK_THREADS, ic = i < n * s ? i : n * s - 1;  // unconditional load (clamped, then a select):
        const double v = Ek[ic];                                          // a guarded load is an exec-mask region with its own wait
        in.E[q] = i < n * s ? v : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 9; ++q) {
        const int i = tid + q * BLK_THREADS, ic = i < ps ? i : ps - 1;
        const double v = Hk[ic];
        in.H[q] = i < ps ? v : 0.0;
    }
    const double cvl = ck[tid < n ? tid : n - 1], hvl = hk[tid < s ? tid : s - 1];
    in.c = tid < n ? cvl : 0.0;
    in.h = tid < s ? hvl : 0.0;
}

__device__ __forceinline__ void wide_in_store(const WideIn &in, double *Es, double *Hs, double *cv, double *hv, int n,
                                              int s, int ps) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int i = tid + q * BLK_THREADS;
        if (i < n * s) Es[i] = in.E[q];
    }
#pragma unroll
    for (int q = 0; q < 9; ++q) {
        const int i = tid + q * BLK_THREADS;
        if (i < ps) Hs[i] = in.H[q];
    }
    if (tid < n) cv[tid] = in.c;
    if (tid < s) hv[tid] = in.h;
}

#if PDPLQR_SEGW_PROFILE
__device__ unsigned long long g_segw[16];
#define SEGW_T(ph)                                                              \
    {                                                                           \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();             \
        segw_acc[ph] += t_ - segw_prev;                                         \
        segw_prev = t_;                                                         \
    }
extern "C" int pdplqr_debug_segw(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_segw), sizeof(g_segw)) == hipSuccess ? 0 : -2;
}
#else
#define SEGW_T(ph)
#endif

__global__ __launch_bounds__(256) void k_seg_bwd_wide(SegArgs A) {
    extern __shared__ __attribute__((aligned(16))) double wbuf[];
    const int tid = threadIdx.x;
    const Shape &sh = A.sh;
    const int n = sh.n, m = sh.m, s = n + m, S = A.S;
    const long long bi = blockIdx.x / S;
    const int seg = blockIdx.x % S;
    if (A.flag && !A.serial && seg == 0 && tid == 0) A.flag[bi] = 0;
    const int N0 = A.serial ? 0 : A.seg_start[seg], N1 = A.serial ? sh.N : N0 + A.seg_len[seg];
    const bool last = A.serial || ((seg == S - 1) && A.last_is_terminal);
    const long long frs = (long long)s * m + m;
    const int ps = sh.ps;
    const double *Eb = A.E + bi * sh.perE;
    const double *cb = A.c + bi * sh.perc;
    const double *Hb = A.Hw + bi * sh.perHw;
    const double *hb = A.hw + bi * sh.perh;
    double *FRb = A.FR + bi * sh.perKD;
    double *Gb = A.G ? A.G + bi * (long long)sh.N * m * n : nullptr;
    double *Lcb = A.Lc ? A.Lc + bi * sh.perHw : nullptr;
    double *lpb = A.lpc ? A.lpc + bi * sh.perh : nullptr;
    const bool ser = A.serial != 0;  // no y block (wide_seg_smem_bytes)
    double *XA = wbuf, *XB = ser ? nullptr : XA + n * s;
    double *Mb = ser ? XA + n * s : XB + n * s;
    double *Cm = ser ? nullptr : Mb + s * s;
    double *Hs = ser ? Mb + s * s : Cm + n * n, *vec = Hs + s * (s + 1) / 2;
    double *pv = vec, *fv = vec + VL, *cv = vec + 2 * VL, *hv = vec + 3 * VL, *pc = vec + 4 * VL,
           *fy = vec + 5 * VL, *lp = vec + 6 * VL, *sinv = vec + 7 * VL;
    __shared__ int s_bad;
    int fail_stage = -1;
#if PDPLQR_SEGW_PROFILE
    unsigned long long segw_prev = __builtin_amdgcn_s_memtime(), segw_acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#endif
    WideIn nxt;
    if (N1 > N0)  // stage N1 - 1's inputs, in flight during the terminal
        wide_in_load(nxt, Eb + (long long)(N1 - 1) * n * s, Hb + (long long)(N1 - 1) * ps, cb + (long long)(N1 - 1) * n,
                     hb + (long long)(N1 - 1) * s, n, s, ps);
    // ---- segment terminal: the real one (P = H~_N, p = h~_N, F = 0) or the
    //      dummy (P = 0, p = 0, F = I, C = 0, f = 0) ----
    {
        const double *HN = Hb + (long long)sh.N * ps;
        if (tid == 0) s_bad = 0;
        __syncthreads();
        for (int q = tid; q < n * n; q += BLK_THREADS) {
            const int i = q % n, j = q / n;
            XA[q] = last ? HN[i >= j ? pidx(i, j, n) : pidx(j, i, n)] : 0.0;
            if (!ser) {
                XB[q] = (!last && i == j) ? 1.0 : 0.0;
                Cm[q] = 0.0;
            }
            if (last && i == j && psd_bad(XA[q])) s_bad = 1;
        }
        for (int q = tid; q < n; q += BLK_THREADS) {
            pv[q] = last ? hb[(long long)sh.N * s + q] : 0.0;
            fv[q] = 0.0;
        }
        if (last) {
            const int pn = n * (n + 1) / 2;
            if (Lcb)
                for (int t = tid; t < pn; t += BLK_THREADS) Lcb[(long long)sh.N * ps + t] = HN[t];
            if (lpb)
                for (int t = tid; t < n; t += BLK_THREADS) lpb[(long long)sh.N * s + t] = hb[(long long)sh.N * s + t];
        }
        if (N1 > N0) wide_in_store(nxt, Mb, Hs, cv, hv, n, s, ps);
        __syncthreads();
        if (s_bad) fail_stage = sh.N;
    }
    const double *Fp = XB;  // F (n x n, ld n) inside XB
    const bool yon = !last;  // the y block (F, C, f) is identically zero on the last segment
    for (int k = N1 - 1; k >= N0; --k) {
        // Mb = E~_k, Hs = H~_k (packed), cv = c_k, hv = h~_k (written at the end of stage k + 1)
        SEGW_T(8);
        blk_mv(pc, mv_n(XA, n), cv, n, n, 1.0, pv);  // P c + p
        if (tid == 0) s_bad = 0;  // every thread has read the previous stage's flag (blk_mv's barrier)
        if (yon) blk_mv(fy, mv_n(Fp, n), cv, n, n, 1.0, fv);  // F c + f
        SEGW_T(0);
        blk_mm(XA, n, mv_n(XA, n), mv_n(Mb, n), n, s, n, 1.0, 0.0, mv_none(), false);  // P E~
        if (yon) blk_mm(XB, n, mv_n(Fp, n), mv_n(Mb, n), n, s, n, 1.0, 0.0, mv_none(), false);  // F E~
        SEGW_T(1);
        blk_mv(lp, mv_t(Mb, n), pc, s, n, 1.0, hv);  // h~ + E~^T (P c + p)
        SEGW_T(2);
        blk_mm(Mb, s, mv_t(Mb, n), mv_n(XA, n), s, s, n, 1.0, 0.0, mv_pk(Hs, s), true);
        // stage k - 1's inputs in flight during the pivots
        SEGW_T(3);
        if (k > N0)
            wide_in_load(nxt, Eb + (long long)(k - 1) * n * s, Hb + (long long)(k - 1) * ps, cb + (long long)(k - 1) * n,
                         hb + (long long)(k - 1) * s, n, s, ps);
        // ---- eliminate the u pivots of [[M, YE^T], [YE, -C]] (one barrier per pivot) ----
        double *FRk = FRb + (long long)k * frs;
        double *Gk = Gb + (long long)k * m * n;
        const int ri = tid & 63, cg = tid >> 6;  // row, column group (s, n <= 64)
        bool ok = true;
        SEGW_T(4);
        double *luq = fy;  // lu' (no y block: fy is free)
        for (int j = 0; j < m;) {
            if (!yon && j + 1 < m) {
                // two pivots per barrier (lds_axpy2_strided: the same fmas as two steps)
                const double d0 = Mb[j + j * s], a1j = Mb[(j + 1) + j * s];
                const double inv0 = 1.0 / d0, invs0 = rsqrt_f64(d0);
                const double d1 = __builtin_fma(-(a1j * inv0), a1j, Mb[(j + 1) + (j + 1) * s]);
                ok = ok && d0 > 0.0 && d1 > 0.0;
                const double inv1 = 1.0 / d1, invs1 = rsqrt_f64(d1);
                const double lpj = lp[j], lp1 = __builtin_fma(-(a1j * inv0), lpj, lp[j + 1]);
                if (tid < s) {
                    const double c0 = Mb[tid + j * s];
                    FRk[(long long)j * s + tid] = tid >= j ? c0 * invs0 : 0.0;
                    const double a1 = __builtin_fma(-(c0 * inv0), a1j, Mb[tid + (j + 1) * s]);
                    FRk[(long long)(j + 1) * s + tid] = tid >= j + 1 ? a1 * invs1 : 0.0;
                }
                if (tid == 255) {
                    FRk[(long long)s * m + j] = lpj * invs0;
                    FRk[(long long)s * m + j + 1] = lp1 * invs1;
                    sinv[j] = invs0;
                    sinv[j + 1] = invs1;
                    luq[j] = lpj * invs0;
                    luq[j + 1] = lp1 * invs1;
                }
                if (ri >= j + 2 && ri < s) {
                    const double f0 = Mb[ri + j * s] * inv0;
                    const double f1 = __builtin_fma(-f0, a1j, Mb[ri + (j + 1) * s]) * inv1;
                    lds_axpy2_strided(Mb + ri, s, Mb + j * s, Mb + (j + 1) * s, f0, f1, inv0, a1j, j + 2 + cg, ri, 4);
                    if (cg == 0) lp[ri] = __builtin_fma(-f1, lp1, __builtin_fma(-f0, lpj, lp[ri]));
                }
                __syncthreads();
                j += 2;
                continue;
            }
            const double d = Mb[j + j * s];
            ok = ok && d > 0.0;
            const double inv2 = 1.0 / d, invs = rsqrt_f64(d);
            const double lpj = lp[j];
            // column j is final: rollout record, coupling gain
            if (tid < s) FRk[(long long)j * s + tid] = tid >= j ? Mb[tid + j * s] * invs : 0.0;
            if (yon && tid >= 128 && tid < 128 + n) Gk[j + (tid - 128) * m] = -XB[(tid - 128) + j * n] * invs;
            if (tid == 255) {
                FRk[(long long)s * m + j] = lpj * invs;
                sinv[j] = invs;
                if (!yon) luq[j] = lpj * invs;
            }
            // row ri, columns l = cg (mod 4): M's trailing rows, then the y block's
            if (ri > j && ri < s) {
                const double lij = Mb[ri + j * s] * inv2;
                lds_axpy_strided(Mb + ri, s, Mb + j * s, lij, j + 1 + cg, ri, 4);
                if (cg == 0) lp[ri] = __builtin_fma(-lij, lpj, lp[ri]);
            }
            if (yon && ri < n) {
                const double yrj = XB[ri + j * n] * inv2;
                lds_axpy_strided(XB + ri, n, Mb + j * s, yrj, j + 1 + cg, s - 1, 4);
                lds_axpy_strided(Cm + ri, n, XB + j * n, -yrj, cg, ri, 4);
                if (cg == 0) fy[ri] = __builtin_fma(-yrj, lpj, fy[ri]);
            }
            __syncthreads();
            ++j;
        }
        SEGW_T(5);
        // ---- P_k (lower block, symmetric by construction), p_k, f_k; F_k stays in XB at column m ----
        for (int q = tid; q < n * n; q += BLK_THREADS) {
            const int i = q % n, j = q / n;
            const int hi = i > j ? i : j, lo = i > j ? j : i;
            const double v = Mb[(m + hi) + (m + lo) * s];
            XA[q] = v;
            if (i == j && psd_bad(v)) s_bad = 1;
            if (Lcb && i >= j) Lcb[(long long)k * ps + pidx(i, j, n)] = v;
        }
        for (int q = tid; q < s; q += BLK_THREADS) {
            const double v = q < m ? (yon ? lp[q] * sinv[q] : luq[q]) : lp[q];  // [lu'; p_k]
            if (lpb) lpb[(long long)k * s + q] = v;
            if (q >= m) pv[q - m] = v;
        }
        if (yon)
            for (int q = tid; q < n; q += BLK_THREADS) fv[q] = fy[q];
        if (yon) Fp = XB + m * n;
        SEGW_T(6);
        if (k > N0) {
            __syncthreads();  // every read of M is done
            wide_in_store(nxt, Mb, Hs, cv, hv, n, s, ps);
        }
        __syncthreads();
        SEGW_T(7);
        if ((!ok || s_bad) && fail_stage < 0) fail_stage = k;
    }
#if PDPLQR_SEGW_PROFILE
    if (blockIdx.x == 0 && tid == 0)
        for (int q = 0; q < 9; ++q) g_segw[q] = segw_acc[q];
#endif
    if (A.serial) {
        if (tid == 0) A.seg_status[bi] = fail_stage < 0 ? 0 : fail_stage + 1;
        return;
    }
    // ---- export the element (update_segment_data, lqr_solver_parallel.hpp:182-187) ----
    double *eo = A.elem + (bi * S + seg) * (long long)(3 * n * n + 2 * n);
    double *eF = eo, *eC = eo + n * n, *ef = eo + 2 * n * n, *eP = ef + n, *ep = eP + n * n;
    for (int q = tid; q < n * n; q += BLK_THREADS) {
        const int i = q % n, j = q / n;
        eP[q] = XA[q];
        eF[q] = last ? 0.0 : Fp[q];
        eC[q] = last ? 0.0 : Cm[i >= j ? i + j * n : j + i * n];
    }
    for (int q = tid; q < n; q += BLK_THREADS) {
        ep[q] = pv[q];
        ef[q] = last ? 0.0 : fv[q];
    }
    if (tid == 0) A.seg_status[bi * S + seg] = fail_stage < 0 ? 0 : fail_stage + 1;
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static bool wide_attr_set(const void *k, size_t bytes) {
    return hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) == hipSuccess;
}

bool wide_state(int n) { return n > 32 && n <= 64; }
bool wide_stage(const Shape &sh) { return sh.s > 32 && sh.s <= 64; }

size_t wide_seg_smem(const Shape &sh) { return wide_seg_smem_bytes(sh.n, sh.s); }
size_t wide_elem_smem(int n) { return wide_elem_smem_bytes(n); }

int wide_seg_backward_slots(const Shape &sh, int device) {
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
    const size_t sm = wide_seg_smem_bytes(sh.n, sh.s);
    wide_attr_set(reinterpret_cast<const void *>(&k_seg_bwd_wide), sm);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_seg_bwd_wide, 256, sm) != hipSuccess || per <= 0) per = 1;
    return cus * per;
}

int wide_scan_slots(int n, int device) {
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
    const size_t sm = wide_elem_smem_bytes(n);
    wide_attr_set(reinterpret_cast<const void *>(&k_seg_scan_wide<false>), sm);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_seg_scan_wide<false>, 256, sm) != hipSuccess || per <= 0)
        per = 1;
    return cus * per;
}

// the serial backward in value form (keep_factors = 0: no L_k cache to fill):
// the m u-pivots per stage instead of the full s-pivot factorisation of
// k_riccati_bwd_big; the same rollout record [L(:, 0:m) | lu'].
int launch_riccati_backward_value_wide(const RiccatiArgs &r, hipStream_t st) {
    SegArgs a{};
    a.sh = r.sh;
    a.S = 1;
    a.last_is_terminal = 1;
    a.E = r.E;
    a.c = r.c;
    a.Hw = r.Hw;
    a.hw = r.hw;
    a.FR = r.KD;
    a.G = nullptr;
    a.Lc = nullptr;
    a.lpc = r.lpc;
    a.elem = nullptr;
    a.seg_status = r.status;
    a.serial = 1;
    const size_t sm = wide_seg_smem_bytes(a.sh.n, a.sh.s, true);
    if (!wide_attr_set(reinterpret_cast<const void *>(&k_seg_bwd_wide), sm)) {
        set_error("backward (n + m > 32): LDS request too large");
        return PDPLQR_ERR_UNSUPPORTED;
    }
    hipLaunchKernelGGL(k_seg_bwd_wide, dim3((unsigned)a.sh.batch), dim3(256), sm, st, a);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

int launch_seg_backward_wide(const SegArgs &a, hipStream_t st) {
    const size_t sm = wide_seg_smem_bytes(a.sh.n, a.sh.s);
    if (!wide_attr_set(reinterpret_cast<const void *>(&k_seg_bwd_wide), sm)) {
        set_error("segment backward (n + m > 32): LDS request too large");
        return PDPLQR_ERR_UNSUPPORTED;
    }
    hipLaunchKernelGGL(k_seg_bwd_wide, dim3((unsigned)(a.sh.batch * a.S)), dim3(256), sm, st, a);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

int launch_seg_scan_wide(const ScanArgs &a, int batch, hipStream_t st) {
    const size_t sm = wide_elem_smem_bytes(a.n);
    const void *k = a.lu ? reinterpret_cast<const void *>(&k_seg_scan_wide<true>)
                         : reinterpret_cast<const void *>(&k_seg_scan_wide<false>);
    if (!wide_attr_set(k, sm)) {
        set_error("suffix scan (n > 32): LDS request too large");
        return PDPLQR_ERR_UNSUPPORTED;
    }
    void *args[] = {const_cast<ScanArgs *>(&a)};
    PDPLQR_HIP_TRY(hipLaunchKernel(k, dim3((unsigned)(batch * a.S)), dim3(256), args, sm, st));
    return PDPLQR_OK;
}

int launch_seg_maps_wide(const MapArgs &a, int batch, hipStream_t st) {
    const size_t sm = wide_elem_smem_bytes(a.n);
    const void *k = a.lu ? reinterpret_cast<const void *>(&k_seg_maps_wide<true>)
                         : reinterpret_cast<const void *>(&k_seg_maps_wide<false>);
    if (!wide_attr_set(k, sm)) {
        set_error("boundary maps (n > 32): LDS request too large");
        return PDPLQR_ERR_UNSUPPORTED;
    }
    void *args[] = {const_cast<MapArgs *>(&a)};
    PDPLQR_HIP_TRY(hipLaunchKernel(k, dim3((unsigned)(batch * (a.S + 1))), dim3(256), args, sm, st));
    return PDPLQR_OK;
}

int launch_map_scan_wide(const MapScanArgs &a, int batch, hipStream_t st) {
    const size_t sm = (size_t)(a.n * a.n + 2 * VL) * sizeof(double);
    hipLaunchKernelGGL(k_map_scan_wide, dim3((unsigned)(batch * (a.S + 1))), dim3(256), sm, st, a);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

// test hook (debug_hooks.hip pdplqr_debug_combine_form): out = a (x) b on one block
template <bool LU>
__global__ __launch_bounds__(256) void k_debug_combine_wide(const double *a, const double *b, double *out, int n,
                                                            int *ok) {
    extern __shared__ __attribute__((aligned(16))) double wbuf[];
    const int nn = n * n;
    const bool good = wide_combine(out, out + nn, out + 2 * nn, out + 2 * nn + n, out + 3 * nn + n, elem_in(a, n),
                                   elem_in(b, n), n, true, true, LU, wide_smem(wbuf, n));
    if (threadIdx.x == 0) *ok = good ? 1 : 0;
}

int launch_debug_combine_wide(const double *a, const double *b, double *out, int n, int *ok, bool lu) {
    const size_t sm = wide_elem_smem_bytes(n);
    const void *k = lu ? reinterpret_cast<const void *>(&k_debug_combine_wide<true>)
                       : reinterpret_cast<const void *>(&k_debug_combine_wide<false>);
    if (!wide_attr_set(k, sm)) return PDPLQR_ERR_UNSUPPORTED;
    void *args[] = {const_cast<double **>(&a), const_cast<double **>(&b), &out, &n, &ok};
    PDPLQR_HIP_TRY(hipLaunchKernel(k, dim3(1), dim3(256), args, sm, 0));
    return PDPLQR_OK;
}

}  // namespace pdplqr
