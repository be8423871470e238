// combine_tiles.hpp -- the segment-element combine on MFMA tiles (one wave).
//
// Elements e = (F, C, f, P, p) (condensed_system.hpp) are n x n
// blocks, n <= 16 T.  Every matrix lives in registers in the
// v_mfma_f64_16x16x4_f64 C/D layout, T x T tiles (lane (g, c) holds rows
// 16 a + 4 r + g of column 16 b + c), padded with the identity / zeros.  The
// one product primitive is C = X^T Y: its MFMA A operand (X^T)[16 a + c][k] is
// X's own register X[k][16 a + c] and its B operand is Y's register, so no
// data moves between products.  Every product of the combine is arranged in
// that form (transposed inputs are loaded transposed from memory; Z^T is
// formed directly as I - Y C_a; C_a, P_b and Y are symmetric).
//
//     R = chol(P_b), Q = chol(I + R^T C_a R), U = Q^{-1} R^T,
//     Y = U^T U = P_b (I + C_a P_b)^{-1},  Z = I - C_a Y = (I + C_a P_b)^{-1}
//     F = F_b Z F_a,  C = F_b Z C_a F_b^T + C_b,  f = F_b Z (f_a - C_a p_b) + f_b,
//     P = P_a + F_a^T Y F_a,  p = p_a + F_a^T Z^T (p_b + P_b f_a).
// Both factorisations run on registers only (elim_regs: DPP / permlane
// broadcasts); U is carried through the second one as extra columns; the
// matrix-vector products are single-column MFMAs on the same operands.
#pragma once

#include "device_common.hpp"

namespace pdplqr {

template <int T>
struct WM {
    d4 t[T][T];
};

// Phase timestamps of the combines (debug builds with -DPDPLQR_COMB_PROFILE:
// lane 0 of every block records wall_clock64() at each mark into slot
// blockIdx % 1024, 32 marks per block; read back with pdplqr_debug_comb_times).
#if defined(PDPLQR_COMB_PROFILE) && defined(PDPLQR_COMB_PROFILE_TU)  // kernels_parallel.hip only
extern __device__ unsigned long long g_comb_t[1024 * 32];
#define COMB_MARK(k)                                                                     \
    do {                                                                                 \
        if (threadIdx.x == 0) g_comb_t[(blockIdx.x % 1024) * 32 + (k)] = wall_clock64(); \
    } while (0)
#else
#define COMB_MARK(k) \
    do {             \
    } while (0)
#endif

template <int T>
struct CombSmem {
    static constexpr int P = 16 * T, PL = P + 1;
    union {
        struct {
            alignas(16) double A[P * (P + 2)];  // Q^T (row stride P + 2), then Z (vector products)
            double B[P * PL];  // R -> U in place, then output staging (symmetrisation)
        };
        alignas(16) double W[2 * P * P];  // [I + P_b C_a | P_b] of the LU form (comb_core_lu)
    };
    alignas(16) double cb[P];  // pivot-row broadcast of chol_tiles; pivot rows of the LU form
    double sinv[P], luq[P];
};

// M <- n x n block at p (column-major, leading dimension ld, or its transpose);
// outside the block: `pad` on the diagonal, 0 elsewhere
// K-chunk-outer products (PDPLQR_TN_CHUNK_OUTER=1; =0 one chain per output
// tile, every MFMA in its own basic block) and branch-free tile loads
// (PDPLQR_BF_LOAD=1: clamped address + select).  Same-box A/B on the 24 x 24
// combine (profiles/r03/comb_ab.log): chunk-outer 1824 -> 1676 ticks, the
// branch-free loads 1728 -> 1824 (they also read the all-padding registers a
// guard skips as a whole), so they stay off here.

template <int T>
__device__ __forceinline__ void wm_load(WM<T> &M, const double *p, int ld, int n, bool trans, double pad, int g,
                                        int c) {
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int b = 0; b < T; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                // branch-free: an unconditional read at a clamped address and a
                // select (a guarded read compiles to an exec-mask region with its
                // own wait per element)
                const int i = 16 * a + 4 * r + g, j = 16 * b + c;
                double v = (i == j) ? pad : 0.0;
                if (i < n && j < n) v = trans ? p[j + i * ld] : p[i + j * ld];
                M.t[a][b][r] = v;
            }
}

template <int T>
__device__ __forceinline__ void wm_store(const WM<T> &M, double *p, int ld, int n, int g, int c) {
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int b = 0; b < T; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * a + 4 * r + g, j = 16 * b + c;
                if (i < n && j < n) p[i + j * ld] = M.t[a][b][r];
            }
}

// p <- M^T (n x n block, column-major, leading dimension n)
template <int T>
__device__ __forceinline__ void wm_store_t(const WM<T> &M, double *p, int n, int g, int c) {
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int b = 0; b < T; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * a + 4 * r + g, j = 16 * b + c;
                if (i < n && j < n) p[j + i * n] = M.t[a][b][r];
            }
}

// C = sgn X^T Y + diag I (+ add); only the K chunks that hold rows < n
template <int T>
__device__ __forceinline__ void wm_tn(WM<T> &C, const WM<T> &X, const WM<T> &Y, int n, double sgn, double diag,
                                      const WM<T> *add, int g, int c) {
    // K chunk outermost: the T x T output tiles are independent accumulation
    // chains, issued back to back inside one chunk (one uniform branch per
    // chunk for a runtime n; a chain per tile would put every MFMA in its own
    // basic block and wait for the previous one's result)
    d4 acc[T][T];
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int b = 0; b < T; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * a + 4 * r + g, j = 16 * b + c;
                acc[a][b][r] = (add ? add->t[a][b][r] : 0.0) + (i == j ? diag : 0.0);
            }
    if constexpr (T == 1) {
        // one output tile: its K chunks would be ONE dependent chain (~186
        // cycles a link); on separate accumulators they issue back to back
        const d4 z = {0.0, 0.0, 0.0, 0.0};
        d4 p1 = z, p2 = z, p3 = z;
        acc[0][0] = mfma_f64(sgn * X.t[0][0][0], Y.t[0][0][0], acc[0][0]);
        if (4 < n) p1 = mfma_f64(sgn * X.t[0][0][1], Y.t[0][0][1], z);
        if (8 < n) p2 = mfma_f64(sgn * X.t[0][0][2], Y.t[0][0][2], z);
        if (12 < n) p3 = mfma_f64(sgn * X.t[0][0][3], Y.t[0][0][3], z);
        acc[0][0] = (acc[0][0] + p1) + (p2 + p3);
    } else {
#pragma unroll
        for (int kt = 0; kt < T; ++kt)
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
                if (16 * kt + 4 * kk < n) {
#pragma unroll
                    for (int a = 0; a < T; ++a)
#pragma unroll
                        for (int b = 0; b < T; ++b)
                            acc[a][b] = mfma_f64(sgn * X.t[kt][a][kk], Y.t[kt][b][kk], acc[a][b]);
                }
    }
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int b = 0; b < T; ++b) C.t[a][b] = acc[a][b];
}

// ---------------------------------------------------------------------------
// Register-only elimination (no LDS, no branches per pivot).  For pivot j the
// lanes need the pivot column at their own rows and the pivot row at their own
// columns.  In the C/D layout column j of tile (a, j/16) sits in lane
// (g, j & 15) of every row group: DPP row_newbcast copies it to the 16 lanes of
// the row (v_mov_b64_dpp, one instruction per double).  Row j sits in row group
// j & 3: v_permlane16_swap / v_permlane32_swap on two copies of a register
// leave the even- and odd-group (lower- and upper-half) values side by side,
// and the compile-time group index picks the pivot's (4 VALU per double).
// ---------------------------------------------------------------------------
template <int S>
__device__ __forceinline__ double dpp_newbcast(double v) {
    long long b = __builtin_bit_cast(long long, v);
    b = __builtin_amdgcn_update_dpp((long long)0, b, 0x150 + S, 0xF, 0xF, false);
    return __builtin_bit_cast(double, b);
}

// lane (g, c) <- lane (g, src) of v (src folds to a constant after unrolling)
__device__ __forceinline__ double bcast_lane16(double v, int src) {
    switch (src) {
        case 0: return dpp_newbcast<0>(v);
        case 1: return dpp_newbcast<1>(v);
        case 2: return dpp_newbcast<2>(v);
        case 3: return dpp_newbcast<3>(v);
        case 4: return dpp_newbcast<4>(v);
        case 5: return dpp_newbcast<5>(v);
        case 6: return dpp_newbcast<6>(v);
        case 7: return dpp_newbcast<7>(v);
        case 8: return dpp_newbcast<8>(v);
        case 9: return dpp_newbcast<9>(v);
        case 10: return dpp_newbcast<10>(v);
        case 11: return dpp_newbcast<11>(v);
        case 12: return dpp_newbcast<12>(v);
        case 13: return dpp_newbcast<13>(v);
        case 14: return dpp_newbcast<14>(v);
        default: return dpp_newbcast<15>(v);
    }
}

// lane (g, c) <- lane (gj, c) of v.  v_permlane16_swap(x, y) with x = y = v
// returns (x', y') = (value of the even group, value of the odd group) of each
// 32-lane half; v_permlane32_swap likewise returns (lower half, upper half).
__device__ __forceinline__ double bcast_group(double v, int gj) {
    int lo = __double2loint(v), hi = __double2hiint(v);
    const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    lo = (gj & 1) ? a[1] : a[0];
    hi = (gj & 1) ? b[1] : b[0];
    const auto a2 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto b2 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    lo = (gj & 2) ? a2[1] : a2[0];
    hi = (gj & 2) ? b2[1] : b2[0];
    return __hiloint2double(hi, lo);
}

// Right-looking elimination of the pivots 0..n-1 of the symmetric padded
// matrix M (left unscaled: M's lower part ends as d_j L[:, j], L unit lower,
// d_j the pivots), optionally carrying TB column tiles B through the same row
// operations (B <- L^{-1} B).  colinv[b] = 1/sqrt(d) of column 16 b + c,
// rowinv[a][r] = 1/sqrt(d) of row 16 a + 4 r + g (AUG only).  Upper-triangle
// entries of M are left as garbage.  False if a pivot is not positive.
template <int T, bool AUG, int NN, int TB>
__device__ __forceinline__ bool elim_regs_n(WM<T> &M, d4 (&B)[T][TB], int n_rt, double (&colinv)[T],
                                            double (&rowinv)[T][4], int g, int c) {
    constexpr int P = 16 * T;
    const int n = NN > 0 ? NN : n_rt;
    bool ok = true;
#pragma unroll
    for (int b = 0; b < T; ++b) colinv[b] = 1.0;
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) rowinv[a][r] = 1.0;
    // one uniform branch per BLK pivots: the BLK bodies are straight-line
    // code, so a pivot's broadcasts and reciprocal overlap the previous
    // updates.  Pivots past n inside the last block act on the identity
    // padding (d = 1, zero row and column): exact no-ops.  Measured
    // (scripts/ubench/elim_bench.hip): 16 x 16 with [B | I] 431 -> 317
    // cycles per pivot, 24 of 32 with B 476 -> 392.
    constexpr int BLK = T == 1 ? 16 : 8;
#pragma unroll
    for (int jb = 0; jb < P; jb += BLK) {
        if (jb >= n) break;
#pragma unroll
        for (int jj = 0; jj < BLK; ++jj) {
            const int j = jb + jj;
            const int tj = j >> 4, cj = j & 15, gj = j & 3, rj = (j >> 2) & 3;
            const double djj = readlane_f64(M.t[tj][tj][rj], (gj << 4) + cj);
            ok = ok && (djj > 0.0);
            // 1/d on the critical path (v_rcp_f64 + one third-order step);
            // 1/sqrt(d) only feeds the final scaling
            const double inv2 = rcp_f64(djj), inv = rsqrt_f64(djj);
            colinv[tj] = (c == cj) ? inv : colinv[tj];
            if (AUG) rowinv[tj][rj] = (g == gj) ? inv : rowinv[tj][rj];
            double lc[T], lb[TB], li[T][4];
#pragma unroll
            for (int b = tj; b < T; ++b) {
                const double v = bcast_group(M.t[tj][b][rj], gj);
                lc[b] = (16 * b + c > j) ? v * inv2 : 0.0;
            }
            if (AUG)
#pragma unroll
                for (int b = 0; b < TB; ++b) lb[b] = bcast_group(B[tj][b][rj], gj) * inv2;
#pragma unroll
            for (int a = tj; a < T; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const double v = bcast_lane16(M.t[a][tj][r], cj);
                    // rows <= j keep their values (finished rows of B)
                    li[a][r] = (AUG && a == tj && 16 * a + 4 * r + g <= j) ? 0.0 : v;
                }
#pragma unroll
            for (int a = tj; a < T; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
#pragma unroll
                    for (int b = tj; b < T; ++b) M.t[a][b][r] = __builtin_fma(-li[a][r], lc[b], M.t[a][b][r]);
                    if (AUG)
#pragma unroll
                        for (int b = 0; b < TB; ++b) B[a][b][r] = __builtin_fma(-li[a][r], lb[b], B[a][b][r]);
                }
        }
    }
    return ok;
}

// The 4 x 4 block step of the blocked Cholesky applies T = L4^{-1} (lower,
// wave-uniform) to a tile's rows j0..j0+3, which every lane (g, c) holds as
// register j0/4 = X[j0 + g][c].  That register IS the B operand of
// v_mfma_f64_16x16x4_f64 (B[k][n] = lane (k, n)), so with A[m][k] = T[m][k]
// in rows m < 4 (zeros below) one MFMA leaves (T X_rows)[g][c] in register 0
// of lane (g, c): the layout of the panel.  t4_operand builds that A operand
// once per block (lane (g, c) supplies A[c][g]); each tile then costs one
// MFMA instead of four row-group broadcasts, ten FMAs and a select chain.
// PDPLQR_T4_MFMA=0 keeps the broadcast form (A/B diagnostics).
// Blocked-Cholesky trailing update on the upper tiles only, the next block's
// diagonal tile first (PDPLQR_CHOL_UPPER=0: every tile pair, row order; A/B)

// The lane picks are products with 0/1 weights (loop-invariant per lane), not
// selects: a select chain over values used nowhere else was turned into
// divergent branches that sank the 4 x 4 block arithmetic into them.
__device__ __forceinline__ double t4_operand(const double (&Ti)[4][4], int g, int c) {
    double a = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        double r = 0.0;  // T[i][g], zero above the diagonal
#pragma unroll
        for (int k = 0; k <= i; ++k) r = __builtin_fma(Ti[i][k], (g == k) ? 1.0 : 0.0, r);
        a = __builtin_fma(r, (c == i) ? 1.0 : 0.0, a);
    }
    return a;
}

__device__ __forceinline__ double t4_apply(double ta, double xrow) {
    const d4 z = mfma_f64(ta, xrow, d4{0.0, 0.0, 0.0, 0.0});
    return z[0];
}

// Blocked Cholesky of a full symmetric 16 x 16 tile M = C C^T (both
// triangles held, as MFMA products leave them), carrying TB column tiles:
// B <- C^{-1} B (final, no row scaling left).  Four pivots per block:
//   - the 4 x 4 diagonal block reaches every lane by readlane; its Cholesky
//     factor and inverse T4 are formed wave-uniformly;
//   - the panel V (lane (g, c) = C[c][j0 + g]) comes from the block's own ROW
//     (register blk of the row groups, the symmetric image of the column) by
//     four row-group broadcasts, masked to the trailing rows c >= j0 + 4;
//   - the trailing updates are ONE MFMA per tile: M -= V V^T and
//     B -= V (T4 B_block), whose B operand is the block's register itself.
// Against one pivot at a time (elim_regs) the dependent chain per pivot shrinks
// to a quarter of the broadcasts and rank-1 updates.  False if a pivot is not
// positive.  M is left stale (only B is an output).
template <int TB>
__device__ __forceinline__ bool chol_blk4_aug(d4 &M, d4 (&B)[TB], int g, int c) {
    bool ok = true;
#pragma unroll
    for (int blk = 0; blk < 4; ++blk) {
        const int j0 = 4 * blk;
        double a[4][4], L[4][4], T[4][4], inv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int k = 0; k <= i; ++k) a[i][k] = readlane_f64(M[blk], 16 * i + j0 + k);  // M[j0+i][j0+k]
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // right-looking Cholesky (uniform values)
            ok = ok && (a[j][j] > 0.0);
            inv[j] = rsqrt_f64(a[j][j]);
            L[j][j] = a[j][j] * inv[j];
#pragma unroll
            for (int i = j + 1; i < 4; ++i) L[i][j] = a[i][j] * inv[j];
#pragma unroll
            for (int i = j + 1; i < 4; ++i)
#pragma unroll
                for (int k = j + 1; k <= i; ++k) a[i][k] = __builtin_fma(-L[i][j], L[k][j], a[i][k]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // T = L^{-1} (lower)
            T[i][i] = inv[i];
#pragma unroll
            for (int j = 0; j < i; ++j) {
                double v = 0.0;
#pragma unroll
                for (int k = j; k < i; ++k) v = __builtin_fma(L[i][k], T[k][j], v);
                T[i][j] = -v * inv[i];
            }
        }
        const double top = t4_operand(T, g, c);
        const double v = t4_apply(top, M[blk]);
        const double vt = (c >= j0 + 4) ? v : 0.0;  // panel, trailing rows only
#pragma unroll
        for (int tb = 0; tb < TB; ++tb) B[tb][blk] = t4_apply(top, B[tb][blk]);  // T4 B_block
        if (blk < 3) M = mfma_f64(-vt, vt, M);
#pragma unroll
        for (int tb = 0; tb < TB; ++tb) B[tb] = mfma_f64(-vt, B[tb][blk], B[tb]);
    }
    return ok;
}

// chol_blk4_aug generalised to T x T tiles and a runtime order n (identity
// padding past n; blocks past ceil(n / 4) are skipped as exact no-ops).
// AUG: carries TB column tiles, B <- C^{-1} B (final); M is left stale.
// !AUG: M <- C^T, the transposed factor (upper triangle, zeros below,
// identity padding kept): each block's ROW of C^T is exactly its panel V.
// KEEP (default !AUG): M <- C^T as well -- with AUG, the factor and the
// carried solve C^{-1} B in one pass.
template <int T, bool AUG, int TB, bool KEEP = !AUG>
__device__ __forceinline__ bool chol_blk4(WM<T> &M, d4 (&B)[T][TB], int n, int g, int c) {
    bool ok = true;
    const int nb = (n + 3) >> 2;
#pragma unroll
    for (int blk = 0; blk < 4 * T; ++blk) {
        if (blk >= nb) break;  // wave-uniform
        const int tj = blk >> 2, rj = blk & 3, cj = 4 * rj, j0 = 4 * blk;
        double a[4][4], L[4][4], Ti[4][4], inv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int k = 0; k <= i; ++k) a[i][k] = readlane_f64(M.t[tj][tj][rj], 16 * i + cj + k);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            ok = ok && (a[j][j] > 0.0);
            inv[j] = rsqrt_f64(a[j][j]);
            L[j][j] = a[j][j] * inv[j];
#pragma unroll
            for (int i = j + 1; i < 4; ++i) L[i][j] = a[i][j] * inv[j];
#pragma unroll
            for (int i = j + 1; i < 4; ++i)
#pragma unroll
                for (int k = j + 1; k <= i; ++k) a[i][k] = __builtin_fma(-L[i][j], L[k][j], a[i][k]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            Ti[i][i] = inv[i];
#pragma unroll
            for (int j = 0; j < i; ++j) {
                double v = 0.0;
#pragma unroll
                for (int k = j; k < i; ++k) v = __builtin_fma(L[i][k], Ti[k][j], v);
                Ti[i][j] = -v * inv[i];
            }
        }
        double vt[T];
        const double top = t4_operand(Ti, g, c);
#pragma unroll
        for (int ta = 0; ta < T; ++ta) {
            vt[ta] = 0.0;
            if (ta < tj) continue;
            const double v = t4_apply(top, M.t[tj][ta][rj]);  // (T M_rows)[g][16 ta + c]
            const int col = 16 * ta + c;
            vt[ta] = (col >= j0 + 4) ? v : 0.0;  // trailing rows of the panel
            if (KEEP) M.t[tj][ta][rj] = (col >= j0) ? v : 0.0;  // row block of C^T, final
        }
        if (AUG) {
#pragma unroll
            for (int tb = 0; tb < TB; ++tb) {  // block rows of B: T4 B_block (register rj of tile row tj)
                B[tj][tb][rj] = t4_apply(top, B[tj][tb][rj]);
            }
        }
        // Trailing update, upper tiles only (the panels read M's row blocks
        // M.t[tj][ta], ta >= tj, and the diagonal tiles; a lower tile is never
        // read again).  The next block's diagonal tile goes first: its
        // readlanes wait on that one product.
        const int ntj = (blk + 1) >> 2;
        if (ntj < T) M.t[ntj][ntj] = mfma_f64(-vt[ntj], vt[ntj], M.t[ntj][ntj]);
#pragma unroll
        for (int ta = 0; ta < T; ++ta)
#pragma unroll
            for (int tb = 0; tb < T; ++tb)
                if (ta >= tj && tb >= ta && !(ta == ntj && tb == ntj))
                    M.t[ta][tb] = mfma_f64(-vt[ta], vt[tb], M.t[ta][tb]);
        if (AUG)
#pragma unroll
            for (int ta = 0; ta < T; ++ta)
#pragma unroll
                for (int tb = 0; tb < TB; ++tb)
                    if (ta >= tj) B[ta][tb] = mfma_f64(-vt[ta], B[tj][tb][rj], B[ta][tb]);
    }
    if (KEEP)
#pragma unroll
        for (int ta = 0; ta < T; ++ta)
#pragma unroll
            for (int tb = 0; tb < T; ++tb)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (16 * ta + 4 * r + g > 16 * tb + c) M.t[ta][tb][r] = 0.0;
    return ok;
}

// The pivot count stays a runtime bound: compile-time counts for several n
// (straight-line copies, 170 KB for the scan kernel) measured 5x slower --
// instruction fetch from L2 once the kernel outgrows the instruction cache.
template <int T, bool AUG, int TB = T>
__device__ __forceinline__ bool elim_regs(WM<T> &M, d4 (&B)[T][TB], int n, double (&colinv)[T],
                                          double (&rowinv)[T][4], int g, int c) {
    return elim_regs_n<T, AUG, 0, TB>(M, B, n, colinv, rowinv, g, c);
}

// M <- chol(M) (lower, zeros above, identity padding kept) on registers only
template <int T>
__device__ __forceinline__ bool wm_chol_regs(WM<T> &M, int n, int g, int c) {
    double colinv[T], rowinv[T][4];
    const bool ok = elim_regs<T, false>(M, M.t, n, colinv, rowinv, g, c);
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int b = 0; b < T; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * a + 4 * r + g, jc = 16 * b + c;
                if (jc < n) M.t[a][b][r] = (i >= jc) ? M.t[a][b][r] * colinv[b] : 0.0;
            }
    return ok;
}

// Y = P_b (I + C_a P_b)^{-1}, Z = I - C_a Y, Zt = Z^T.  False if P_b or the
// SPD core is not positive definite.
//     R = chol(P_b), S = I + R^T C_a R = Q Q^T, U = Q^{-1} R^T, Y = U^T U
// U comes out of the elimination of S carrying R^T as extra columns (row i
// scaled by 1/sqrt(d_i) at the end), so no triangular solve is needed.

template <int T>
__device__ __forceinline__ bool comb_core(WM<T> &Y, WM<T> &Z, WM<T> &Zt, const WM<T> &Ca, const double *Pb, int n,
                                          CombSmem<T> &sm, int lane) {
    constexpr int PL = 16 * T + 1;
    const int g = lane >> 4, c = lane & 15;
    WM<T> R, S, U;
    COMB_MARK(1);
    // blocked factors (chol_blk4): R^T comes out directly, R through LDS
    wm_load(U, Pb, n, n, false, 1.0, g, c);
    bool ok = chol_blk4<T, false, T>(U, U.t, n, g, c);  // U = R^T
    wm_store(U, sm.B, PL, n, g, c);
    wave_sync();
    wm_load(R, sm.B, PL, n, true, 1.0, g, c);
    COMB_MARK(2);
    {
        WM<T> T1;
        wm_tn(T1, Ca, R, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);  // C_a R
        wm_tn(S, R, T1, n, 1.0, 1.0, (const WM<T> *)nullptr, g, c);   // I + R^T C_a R
    }
    COMB_MARK(3);
    ok = chol_blk4<T, true, T>(S, U.t, n, g, c) && ok;  // U = Q^{-1} R^T
    COMB_MARK(4);
    COMB_MARK(5);
    wm_tn(Y, U, U, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);  // Y = U^T U
    wm_tn(Z, Ca, Y, n, -1.0, 1.0, (const WM<T> *)nullptr, g, c);  // Z = I - C_a Y
    wm_tn(Zt, Y, Ca, n, -1.0, 1.0, (const WM<T> *)nullptr, g, c);  // Z^T = I - Y C_a
    wave_sync();
    COMB_MARK(6);
    return ok;
}

// LU form of the same core (CondensedSystemLUSolver, condensed_system.hpp:
// 32-147, which factors I + C P with PartialPivLU): no definiteness needed --
// for PSD C_a, P_b every eigenvalue of I + P_b C_a is >= 1, so a semidefinite
// value function (zero state cost) combines where the Cholesky form fails.
//     Y = (I + P_b C_a)^{-1} P_b  (= P_b (I + C_a P_b)^{-1}, symmetric)
// by Gauss-Jordan elimination with partial (row) pivoting on [I + P_b C_a | P_b]
// in LDS: the same pivot rows as PartialPivLU (largest |a| among the rows not
// yet used, lowest row on ties), kept in place instead of swapped.  Lanes own
// rows (lane % 16 T) and interleaved column sets (lane / 16 T); the pivot row
// reaches every lane as a broadcast LDS read.  Y is symmetrised on the way
// back to registers; Z, Z^T follow as in the Cholesky form.  False if a pivot
// is zero or not finite.
template <int T>
__device__ __forceinline__ bool comb_core_lu(WM<T> &Y, WM<T> &Z, WM<T> &Zt, const WM<T> &Ca, const double *Pb, int n,
                                             CombSmem<T> &sm, int lane) {
    constexpr int P = 16 * T, LP = 64 / P;
    const int g = lane >> 4, c = lane & 15;
    double *W = sm.W;  // [A | P_b] column-major, leading dimension n
    int *piv_row = reinterpret_cast<int *>(sm.cb);  // piv_row[k]: the row that pivoted column k
    {
        WM<T> Pm, Am;
        wm_load(Pm, Pb, n, n, false, 0.0, g, c);
        wm_tn(Am, Pm, Ca, n, 1.0, 1.0, (const WM<T> *)nullptr, g, c);  // I + P_b C_a (P_b symmetric)
        wave_sync();
        wm_store(Am, W, n, n, g, c);
        wm_store(Pm, W + n * n, n, n, g, c);
        wave_sync();
    }
    const bool row = lane % P < n;
    const int i = row ? lane % P : 0, q = lane / P;  // rows >= n read row 0 and write nothing
    bool used = false, ok = true;
    for (int k = 0; k < n; ++k) {
        // pivot: max |a_ik| over the unused rows (lowest row on ties)
        double v = (row && q == 0 && !used) ? fabs(W[i + k * n]) : -1.0;
        int arg = lane % P;
#pragma unroll
        for (int mk = 1; mk < 64; mk <<= 1) {
            const double ov = shfl_xor_f64(v, mk);
            const int oa = __shfl_xor(arg, mk, 64);
            if (ov > v || (ov == v && oa < arg)) {
                v = ov;
                arg = oa;
            }
        }
        const int p = __builtin_amdgcn_readfirstlane(arg);
        const double piv = W[p + k * n];
        ok = ok && piv != 0.0 && fabs(piv) <= 1.7976931348623157e308;
        const double inv = 1.0 / piv;
        const bool me = row && i == p;
        used = used || me;
        if (lane == 0) piv_row[k] = p;
        const double mi = W[i + k * n] * inv;  // this row's multiplier
        wave_sync();
        for (int j = q; j < 2 * n; j += LP) {
            const double rp = W[p + j * n];  // pivot row: broadcast read
            const double own = W[i + j * n];
            const double nv = me ? rp * inv : __builtin_fma(-mi, rp, own);
            if (row) W[i + j * n] = nv;
        }
        wave_sync();
    }
    // row piv_row[k] now holds row k of Y = [A | P_b]'s solved right-hand side
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int b = 0; b < T; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int ii = 16 * a + 4 * r + g, jj = 16 * b + c;
                double y = 0.0;
                if (ii < n && jj < n)
                    y = 0.5 * (W[piv_row[ii] + (n + jj) * n] + W[piv_row[jj] + (n + ii) * n]);
                Y.t[a][b][r] = y;
            }
    wave_sync();
    wm_tn(Z, Ca, Y, n, -1.0, 1.0, (const WM<T> *)nullptr, g, c);   // Z = I - C_a Y
    wm_tn(Zt, Y, Ca, n, -1.0, 1.0, (const WM<T> *)nullptr, g, c);  // Z^T = I - Y C_a
    return ok;
}

// the core of either condensed form (CondensedSystemSolverType)
template <int T, bool LU>
__device__ __forceinline__ bool comb_core_t(WM<T> &Y, WM<T> &Z, WM<T> &Zt, const WM<T> &Ca, const double *Pb, int n,
                                            CombSmem<T> &sm, int lane) {
    if constexpr (LU) return comb_core_lu<T>(Y, Z, Zt, Ca, Pb, n, sm, lane);
    else return comb_core<T>(Y, Z, Zt, Ca, Pb, n, sm, lane);
}

// n-vectors in the B-operand / C-layout column 0 of the tiles: lane (g, 0)
// holds x[16 kt + 4 r + g] in t[kt][r]; other lanes hold 0.
template <int T>
struct WV {
    d4 t[T];
};

template <int T>
__device__ __forceinline__ void wv_load(WV<T> &x, const double *p, int n, int g, int c) {
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 16 * a + 4 * r + g;
            x.t[a][r] = (c == 0 && i < n) ? p[i] : 0.0;
        }
}

template <int T>
__device__ __forceinline__ void wv_store(const WV<T> &x, double *p, int n, int g, int c) {
    if (c == 0)
#pragma unroll
        for (int a = 0; a < T; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * a + 4 * r + g;
                if (i < n) p[i] = x.t[a][r];
            }
}

// y = sgn X^T x (+ add): the single-column form of wm_tn
template <int T>
__device__ __forceinline__ void wv_tn(WV<T> &y, const WM<T> &X, const WV<T> &x, int n, double sgn,
                                      const WV<T> *add) {
    d4 acc[T];  // chunk outermost (see wm_tn)
#pragma unroll
    for (int a = 0; a < T; ++a) acc[a] = add ? add->t[a] : d4{0.0, 0.0, 0.0, 0.0};
    if constexpr (T <= 2) {
        // T output tiles only: even and odd K chunks on separate accumulators
        // (two chains of half the length, summed at the end)
        d4 odd[T];
#pragma unroll
        for (int a = 0; a < T; ++a) odd[a] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kt = 0; kt < T; ++kt)
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
                if (16 * kt + 4 * kk < n) {
#pragma unroll
                    for (int a = 0; a < T; ++a) {
                        if (kk & 1) odd[a] = mfma_f64(sgn * X.t[kt][a][kk], x.t[kt][kk], odd[a]);
                        else acc[a] = mfma_f64(sgn * X.t[kt][a][kk], x.t[kt][kk], acc[a]);
                    }
                }
#pragma unroll
        for (int a = 0; a < T; ++a) acc[a] += odd[a];
    } else {
#pragma unroll
        for (int kt = 0; kt < T; ++kt)
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
                if (16 * kt + 4 * kk < n) {
#pragma unroll
                    for (int a = 0; a < T; ++a) acc[a] = mfma_f64(sgn * X.t[kt][a][kk], x.t[kt][kk], acc[a]);
                }
    }
#pragma unroll
    for (int a = 0; a < T; ++a) y.t[a] = acc[a];
}

// symmetric store: out = (M + M^T) / 2 (n x n, ld n) through the LDS staging buffer
template <int T>
__device__ __forceinline__ void wm_store_sym(const WM<T> &M, double *out, int n, CombSmem<T> &sm, int lane) {
    constexpr int PL = 16 * T + 1;
    wm_store(M, sm.B, PL, n, lane >> 4, lane & 15);
    wave_sync();
    for (int q = lane; q < n * n; q += 64) {
        const int i = q % n, j = q / n;
        out[q] = 0.5 * (sm.B[i + j * PL] + sm.B[j + i * PL]);
    }
    wave_sync();
}

// Input element blocks, each column-major n x n (or n-vectors), anywhere in
// global memory or LDS.
struct ElemIn {
    const double *F, *C, *f, *P, *p;
};

// [F | C | f | P | p] contiguous (the element layout of the scans)
__device__ __forceinline__ ElemIn elem_in(const double *e, int n) {
    const int nn = n * n;
    return ElemIn{e, e + nn, e + 2 * nn, e + 2 * nn + n, e + 3 * nn + n};
}

// out = a (x) b  (a earlier, b later).  The output blocks are addressed
// separately (oF, oC, of are not touched when need_FCf is false, oP, op not
// when need_Pp is false).  P_a and C_b are read once, as addends of the last
// products: they are loaded up front so a global-memory source costs no
// exposed latency.
//
// Aliasing contract (the in-place Sklansky rounds of k_seg_scan rely on it,
// tests/test_gpu_parallel.py::test_sklansky_scan_matches_hillis_steele):
// an output block may alias an input block only when
//   * that input is P_a, which is loaded into registers (Pa) before the first
//     store, and the first store (oP) depends on Pa; or
//   * that input lives in a buffer the caller staged elsewhere (LDS) first.
// Every other input block is read from its source after the first store, so
// it must not overlap any output.  An edit that moves a store ahead of a read,
// or reads P_a from memory again, breaks the in-place rounds.
template <int T, bool LU = false>
__device__ __forceinline__ bool tcombine_parts(double *oF, double *oC, double *of, double *oP, double *op,
                                               const ElemIn &ea, const ElemIn &eb, int n, bool need_FCf,
                                               bool need_Pp, CombSmem<T> &sm, int lane) {
    const int g = lane >> 4, c = lane & 15;
    const double *aF = ea.F, *aC = ea.C, *af = ea.f, *ap = ea.p;
    const double *bF = eb.F, *bf = eb.f, *bP = eb.P, *bp = eb.p;
    WM<T> Pa, Cb;
    if (need_Pp) wm_load(Pa, ea.P, n, n, false, 0.0, g, c);
    if (need_FCf) wm_load(Cb, eb.C, n, n, false, 0.0, g, c);
    WM<T> Ca, Y, Z, Zt;
    COMB_MARK(0);
    wm_load(Ca, aC, n, n, false, 0.0, g, c);
    const bool ok = comb_core_t<T, LU>(Y, Z, Zt, Ca, bP, n, sm, lane);
    WM<T> Fa;
    wm_load(Fa, aF, n, n, false, 0.0, g, c);
    if (need_Pp) {  // P = P_a + F_a^T (Y F_a)
        WM<T> W, Pn;
        wm_tn(W, Y, Fa, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);
        wm_tn(Pn, Fa, W, n, 1.0, 0.0, &Pa, g, c);
        wm_store_sym(Pn, oP, n, sm, lane);
    }
    COMB_MARK(7);
    if (need_FCf) {
        WM<T> Fbt, W, Fn;
        wm_load(Fbt, bF, n, n, true, 0.0, g, c);                     // F_b^T
        wm_tn(W, Zt, Fa, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);   // Z F_a
        wm_tn(Fn, Fbt, W, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);  // F_b Z F_a
        wm_store(Fn, oF, n, n, g, c);
        WM<T> W2t, W3, Cn;
        wm_tn(W2t, Ca, Zt, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);   // C_a Z^T = (Z C_a)^T
        wm_tn(W3, W2t, Fbt, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);  // Z C_a F_b^T
        wm_tn(Cn, Fbt, W3, n, 1.0, 0.0, &Cb, g, c);                     // F_b Z C_a F_b^T + C_b
        wm_store_sym(Cn, oC, n, sm, lane);
    }
    COMB_MARK(8);
    // vectors on the same tiles (single-column MFMAs; x in column 0)
    if (need_FCf) {
        WV<T> pb, fa, v1, v2, fb, fo;
        wv_load(pb, bp, n, g, c);
        wv_load(fa, af, n, g, c);
        wv_tn(v1, Ca, pb, n, -1.0, &fa);        // v1 = f_a - C_a p_b  (C_a symmetric)
        wv_tn(v2, Zt, v1, n, 1.0, (const WV<T> *)nullptr);  // Z v1
        WM<T> Fbt;
        wm_load(Fbt, bF, n, n, true, 0.0, g, c);
        wv_load(fb, bf, n, g, c);
        wv_tn(fo, Fbt, v2, n, 1.0, &fb);        // f = F_b Z v1 + f_b
        wv_store(fo, of, n, g, c);
    }
    if (need_Pp) {
        WM<T> Pb;
        WV<T> fa, pb, v3, v4, pa, po;
        wm_load(Pb, bP, n, n, false, 0.0, g, c);
        wv_load(fa, af, n, g, c);
        wv_load(pb, bp, n, g, c);
        wv_tn(v3, Pb, fa, n, 1.0, &pb);         // v3 = p_b + P_b f_a  (P_b symmetric)
        wv_tn(v4, Z, v3, n, 1.0, (const WV<T> *)nullptr);   // Z^T v3
        wv_load(pa, ap, n, g, c);
        wv_tn(po, Fa, v4, n, 1.0, &pa);         // p = p_a + F_a^T Z^T v3
        wv_store(po, op, n, g, c);
    }
    wave_sync();
    COMB_MARK(9);
    return ok;
}

template <int T, bool LU = false>
__device__ __forceinline__ bool tcombine(double *out, const double *ea, const double *eb, int n, bool need_FCf,
                                         bool need_Pp, CombSmem<T> &sm, int lane) {
    const int nn = n * n;
    return tcombine_parts<T, LU>(out, out + nn, out + 2 * nn, out + 2 * nn + n, out + 3 * nn + n, elem_in(ea, n),
                             elem_in(eb, n), n, need_FCf, need_Pp, sm, lane);
}

// ---------------------------------------------------------------------------
// Closed-loop boundary map of an element under a value function (one wave):
//     [Phi | phi] = (I + C P)^{-1} [F | f - C p]
// as a SOLVE, not as (I - C Y) times the right-hand side: when C P is large
// (|C P| ~ 1e4) Z = (I + C P)^{-1} is small and I - C Y cancels, which costs
// digits in every boundary state (tests/test_gpu_wide.py, 50/10 with
// penalties: 1e-10 off instead of 1e-12).  The reference never forms Z either:
// its Cholesky form goes through P^{-1} and (C + P^{-1})^{-1}
// (condensed_system.hpp:252-289), its LU form solves with PartialPivLU of
// I + C P (:117-137).
//   CHOLESKY: R = chol(P), S = I + R^T C R = Q Q^T,
//             [Phi | phi] = R^{-T} Q^{-T} Q^{-1} R^T [F | v] = V^T Q^{-1} R^T [F | v],
//             V = Q^{-1} R^{-1}: chol(P) carries the identity (R^{-1}), chol(S)
//             carries [R^T F | R^T v | R^{-1}], one product V^T [X1 | x3] after it
//             (round 2 ran three triangular solves in LDS, one lane per column:
//             a dependent LDS read per FMA);
//   LU:       Gauss-Jordan with partial pivoting on [I + C P | F | v]
//             (comb_core_lu's pivot rule).
// The result lands in LDS: Phi at out (n x n, ld n), phi at out + n n.
// Scratch: tmap_smem_doubles(n) doubles (16-byte aligned) at `scr`.
// ---------------------------------------------------------------------------
__host__ __device__ inline int tmap_smem_doubles(int n) {
    const int P = n <= 16 ? 16 : 32, PL = P + 1;
    const int chol = 2 * P * PL + (n + 1) * n;     // R^T, Q^T, [B | b] (ld n)
    const int lu = n * (2 * n + 1) + (2 * n + 1) + n;  // W, pivot row, pivot rows (int)
    return ((chol > lu ? chol : lu) + 1) & ~1;
}

template <int T, bool LU>
__device__ __forceinline__ bool tmap_solve(const double *F, const double *C, const double *f, const double *Pj,
                                           const double *pj, int n, double *scr, double *out, int lane) {
    constexpr int P = 16 * T, PL = P + 1;
    const int g = lane >> 4, c = lane & 15;
    bool ok = true;
    WM<T> Cs, Pm;
    WV<T> pv, fv, v;
    wm_load(Cs, C, n, n, false, 0.0, g, c);
    wv_load(pv, pj, n, g, c);
    wv_load(fv, f, n, g, c);
    wv_tn(v, Cs, pv, n, -1.0, &fv);  // v = f - C p  (C symmetric)
    if constexpr (!LU) {
        // R = chol(P) carrying the identity (U = R^T and R^{-1} in one pass),
        // S = I + R^T C R = Q Q^T carrying [R^T F | R^T v | R^{-1}]:
        // [X1 | x3 | V] = Q^{-1} [...], and [Phi | phi] = V^T [X1 | x3]
        // (= R^{-T} Q^{-T} Q^{-1} R^T [F | v]; no triangular solve left)
        double *Rt = scr;
        WM<T> U, R;
        d4 BB[T][2 * T + 1];
#pragma unroll
        for (int a = 0; a < T; ++a)
#pragma unroll
            for (int bt = 0; bt < T; ++bt)
#pragma unroll
                for (int r = 0; r < 4; ++r) BB[a][T + 1 + bt][r] = (16 * a + 4 * r + g == 16 * bt + c) ? 1.0 : 0.0;
        {
            d4 Ri[T][T];
#pragma unroll
            for (int a = 0; a < T; ++a)
#pragma unroll
                for (int bt = 0; bt < T; ++bt) Ri[a][bt] = BB[a][T + 1 + bt];
            wm_load(U, Pj, n, n, false, 1.0, g, c);
            ok = chol_blk4<T, true, T, true>(U, Ri, n, g, c);  // U = R^T (upper), Ri = R^{-1}
#pragma unroll
            for (int a = 0; a < T; ++a)
#pragma unroll
                for (int bt = 0; bt < T; ++bt) BB[a][T + 1 + bt] = Ri[a][bt];
        }
        wm_store(U, Rt, PL, n, g, c);
        wave_sync();
        wm_load(R, Rt, PL, n, true, 1.0, g, c);  // R
        WM<T> S;
        {
            WM<T> T1;
            wm_tn(T1, Cs, R, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);  // C R
            wm_tn(S, R, T1, n, 1.0, 1.0, (const WM<T> *)nullptr, g, c);   // I + R^T C R
        }
        {
            WM<T> Fs, X;
            WV<T> y;
            wm_load(Fs, F, n, n, false, 0.0, g, c);
            wm_tn(X, R, Fs, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);  // R^T F
            wv_tn(y, R, v, n, 1.0, (const WV<T> *)nullptr);              // R^T v
#pragma unroll
            for (int a = 0; a < T; ++a) {
#pragma unroll
                for (int bt = 0; bt < T; ++bt) BB[a][bt] = X.t[a][bt];
                BB[a][T] = y.t[a];
            }
        }
        ok = chol_blk4<T, true, 2 * T + 1>(S, BB, n, g, c) && ok;
        WM<T> X1, V, Phi;
        WV<T> x3, ph;
#pragma unroll
        for (int a = 0; a < T; ++a) {
#pragma unroll
            for (int bt = 0; bt < T; ++bt) {
                X1.t[a][bt] = BB[a][bt];
                V.t[a][bt] = BB[a][T + 1 + bt];
            }
            x3.t[a] = BB[a][T];
        }
        wm_tn(Phi, V, X1, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);  // V^T X1
        wv_tn(ph, V, x3, n, 1.0, (const WV<T> *)nullptr);             // V^T x3
        wave_sync();  // every lane's reads of Rt done before out (may alias scr) is written
        wm_store(Phi, out, n, n, g, c);
        wv_store(ph, out + n * n, n, g, c);
        wave_sync();
    } else {
        const int ncol = 2 * n + 1;
        double *W = scr, *prow = scr + n * ncol;
        int *piv = reinterpret_cast<int *>(prow + ncol);
        {
            WM<T> A, Fs;
            wm_load(Pm, Pj, n, n, false, 0.0, g, c);
            wm_tn(A, Cs, Pm, n, 1.0, 1.0, (const WM<T> *)nullptr, g, c);  // I + C P  (C symmetric)
            wm_store(A, W, n, n, g, c);
            wm_load(Fs, F, n, n, false, 0.0, g, c);
            wm_store(Fs, W + n * n, n, n, g, c);
            wv_store(v, W + 2 * n * n, n, g, c);
        }
        wave_sync();
        const bool row = lane < n;
        const int i = row ? lane : 0;
        bool used = false;
        for (int k = 0; k < n; ++k) {
            double a = (row && !used) ? fabs(W[i + k * n]) : -1.0;
            int arg = lane;
#pragma unroll
            for (int mk = 1; mk < 64; mk <<= 1) {
                const double oa = shfl_xor_f64(a, mk);
                const int ob = __shfl_xor(arg, mk, 64);
                if (oa > a || (oa == a && ob < arg)) {
                    a = oa;
                    arg = ob;
                }
            }
            const int p = __builtin_amdgcn_readfirstlane(arg);
            const double pvv = W[p + k * n];
            ok = ok && pvv != 0.0 && fabs(pvv) <= 1.7976931348623157e308;
            const double inv = 1.0 / pvv;
            const bool me = row && i == p;
            used = used || me;
            if (lane == 0) piv[k] = p;
            for (int j = lane; j < ncol; j += 64) prow[j] = W[p + j * n];
            const double mi = W[i + k * n] * inv;
            wave_sync();
            if (row)
                for (int j = 0; j < ncol; ++j) W[i + j * n] = me ? prow[j] * inv : __builtin_fma(-mi, prow[j], W[i + j * n]);
            wave_sync();
        }
        // row piv[i] of the right part is row i of the solution
        for (int q = lane; q < n * n + n; q += 64) {
            const int ii = q % n, jj = q / n;
            out[q] = W[piv[ii] + (n + jj) * n];
        }
    }
    wave_sync();
    return ok;
}

}  // namespace pdplqr
