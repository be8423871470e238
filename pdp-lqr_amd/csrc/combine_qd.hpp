// combine_qd.hpp -- the segment-element combine (SURVEY.md 0.1,
// condensed_system.hpp:203-290) at n = 24 on a 256-thread block as ONE
// blocked LDL^T elimination, instead of the two 24-pivot Cholesky
// factorisations and the products between them of combine_mw.hpp.
//
// An element e = (F, C, f, P, p) of stages [s, e) is the saddle function
//     Phi_e(x, lam) = 1/2 x^T P x + p^T x + lam^T (F x + f) - 1/2 lam^T C lam
// of the state x at its start and the costate lam at its end: x_end =
// F x + f - C lam (lqr_kernel_parallel.hpp:97-135).  Combining a ([s, m)) with
// b ([m, e)) takes the extremum over the junction state x_m and costate lam_m:
//     Phi_ab(x_s, lam_e) = ext Phi_a(x_s, lam_m) + Phi_b(x_m, lam_e) - lam_m^T x_m,
// i.e. the Schur complement of the junction block J = [[P_b, -I], [-I, -C_a]]
// (rows / columns x_m, lam_m) in the symmetric matrix over
//     [x_m, lam_m | x_s, lam_e | 1]:   (lam_m, x_s) = F_a,  (x_m, lam_e) = F_b^T,
//     (x_s, x_s) = P_a,  (lam_e, lam_e) = -C_b,  column 1: p_b, f_a, p_a, f_b.
// The complement is [[P, F^T, p], [F, -C, f]]: the combined element (the same
// as Z = (I + C_a P_b)^{-1}, F = F_b Z F_a, ... of condensed_system.hpp).
//
// J is quasi-definite when P_b is definite and C_a semidefinite.  Eliminated in
// the order x_0, lam_0, x_1, lam_1, ... every leading block is nonsingular,
// with pivots d > 0 on x and d < 0 on lam (the status: anything else is
// flagged, as chol(P_b) failing is in the Cholesky form); this order keeps full
// accuracy for ill-conditioned P_b (numpy restatement on 24/8 elements: 3e-15
// against 1e-8 for x-first elimination -- chol(P_b), then -C_a - P_b^{-1} --
// at cond(P_b) = 1e8; the two-Cholesky form 1e-13).
//
// Schedule: 48 pivots in 6 blocks of 8.  The 96 x 96 matrix (+ the linear
// column) lives in 16 x 16 MFMA tiles, lower triangle only (21 tiles).  Wave 0
// owns the three diagonal tiles (every pivot block lives in one of them); waves
// 1..3 own the others.  Per block t of pivots J:
//   1. wave 0 takes block t - 1's update of the diagonal tile holding J first,
//      publishes its rows J, factors the 8 x 8 pivot block LDL^T (wave-uniform)
//      and publishes L, 1/d; meanwhile the owners of the tiles below it take
//      that update and publish the pivot COLUMNS J (= rows J by symmetry), then
//      the updates of the tiles whose pivots come later;     -> barrier A
//   2. every thread forms V = L^{-1} M[J, col], W = D^{-1} V for one column
//      (97 columns over the four waves);                   -> barrier B
//   3. the linear column row by row; the tiles take M[I, K] -= V[:, I]^T W[:, K]
//      as two MFMAs (A operand V of the tile's rows, B operand W of its
//      columns, read from LDS), the tiles of the next pivots first (step 1).
// Two barriers a block, no products outside the elimination.  Each wave's code
// is specialised at compile time (tile list, step), so the MFMAs of a step
// issue back to back without branches.
#pragma once

#include "combine_tiles.hpp"

namespace pdplqr {

constexpr int QD_N = 24;                  // state dimension of this combine
constexpr int QD_NJ = 2 * QD_N;           // junction pivots (x_m, lam_m interleaved)
constexpr int QD_NT = 4 * QD_N;           // matrix rows: junction, then x_s, lam_e
constexpr int QD_AUG = QD_NT;             // the linear column
constexpr int QD_NCOL = QD_NT + 1;
constexpr int QD_PRS = 10;                // pivot rows: [column][8] at stride 10 (16-byte rows)
constexpr int QD_VWS = 18;                // [column][V 0..7 | W 0..7] at stride 18 (odd bank step)
constexpr int QD_STEPS = QD_NJ / 8;
// The right-of-panel update of block t is issued after barrier A_{t+1}, so
// its MFMAs run under block t + 1's factor (VALU) instead of ahead of the
// barrier: C4 rank 0.364 -> 0.356 ms pipelined (profiles/r06/qd_defer_ab/).
// PDPLQR_QD_DEFER=0: the old order (A/B switch)
#ifndef PDPLQR_QD_DEFER
#define PDPLQR_QD_DEFER 1
#endif
#define QD_DEFER PDPLQR_QD_DEFER

__host__ __device__ constexpr int qd_smem_doubles() { return QD_NCOL * QD_PRS + QD_NCOL * QD_VWS + 36 + 2; }

// Phase stamps (diagnostic builds with -DPDPLQR_COMB_PROFILE, kernels_parallel.hip):
// shader-clock sums over the 6 blocks of one combine, by thread 0 (a junction
// wave) into slots 23..26 and thread 128 (an outer wave) into 27..30.
#if defined(PDPLQR_COMB_PROFILE) && defined(PDPLQR_COMB_PROFILE_TU)
#define QD_PROF 1
struct QdProf {
    unsigned long long acc[4] = {0, 0, 0, 0}, t = __builtin_amdgcn_s_memtime();
    __device__ void mark(int k) {
        const unsigned long long u = __builtin_amdgcn_s_memtime();
        acc[k] += u - t;
        t = u;
    }
    __device__ void save(int slot0) {
        for (int k = 0; k < 4; ++k) g_comb_t[(blockIdx.x % 1024) * 32 + slot0 + k] = acc[k];
    }
};
#define QD_MARK(k) prof.mark(k)
#else
#define QD_PROF 0
#define QD_MARK(k) \
    do {           \
    } while (0)
#endif

// Tile lists (compile time).  Wave 0: the diagonal tiles.  Waves 1..3: the
// others, balanced for the tiles holding the next block's pivots (K = 0 at
// block 0, 1 at blocks 1-2, 2 at blocks 3-4): 2/2/1, 1/2/1, 1/1/1.
template <int W>
struct QdTiles;
template <>
struct QdTiles<0> {
    static constexpr int n = 3;
    static constexpr int I[6] = {0, 1, 2, 0, 0, 0}, K[6] = {0, 1, 2, 0, 0, 0};
};
template <>
struct QdTiles<1> {
    static constexpr int n = 6;
    static constexpr int I[6] = {1, 2, 2, 3, 3, 4}, K[6] = {0, 0, 1, 2, 3, 3};
};
template <>
struct QdTiles<2> {
    static constexpr int n = 6;
    static constexpr int I[6] = {3, 4, 3, 4, 4, 4}, K[6] = {0, 0, 1, 1, 2, 4};
};
template <>
struct QdTiles<3> {
    static constexpr int n = 6;
    static constexpr int I[6] = {5, 5, 5, 5, 5, 5}, K[6] = {0, 1, 2, 3, 4, 5};
};

// Tile (I, K) of the matrix before the elimination, branch-free: every
// candidate is read at a clamped address and selected (a row group of 4 never
// straddles the x_s / lam_e boundary at 24, so the row class is known at
// compile time; the column class of tile column 4 is a lane select).
template <int I, int K, int R>
__device__ __forceinline__ double qd_elem(const ElemIn &ea, const ElemIn &eb, bool fcf, int g, int c) {
    // one load at a lane-selected address and v = load * f + k (a select of
    // loaded values compiles to divergent branches around the loads)
    constexpr int n = QD_N;
    if constexpr (I <= 2 && K <= 2) {  // junction x junction: P_b / -C_a / -I coupling
        const int a = 8 * I + 2 * R + (g >> 1), b = 8 * K + (c >> 1), q = a + b * n;
        const int si = g & 1, sj = c & 1;  // 16 I + 4 R is even
        const double *p = (si & sj) ? ea.C + q : eb.P + q;
        const double f = si == sj ? (si ? -1.0 : 1.0) : 0.0, k = (si != sj && a == b) ? -1.0 : 0.0;
        return __builtin_fma(*p, f, k);
    } else if constexpr (K <= 2) {  // outer rows x junction columns: F_a, F_b^T
        constexpr int rb = 16 * (I - 3) + 4 * R;  // outer row of g = 0
        const int a = 8 * K + (c >> 1), s = c & 1;
        if constexpr (rb < n) {  // x_s rows: (lam_m a, x_s) = F_a[a][row]
            return ea.F[a + (rb + g) * n] * (s ? 1.0 : 0.0);
        } else {  // lam_e rows: (x_m a, lam_e v) = F_b[v][a]
            return eb.F[(rb - n + g) + a * n] * ((s == 0 && fcf) ? 1.0 : 0.0);
        }
    } else {  // outer x outer: P_a, -C_b
        constexpr int rb = 16 * (I - 3) + 4 * R;
        const int w = 16 * (K - 3) + c, wx = w < n, wc = wx ? w : w - n;
        if constexpr (rb < n) {
            return ea.P[(rb + g) + wc * n] * (wx ? 1.0 : 0.0);
        } else {
            return eb.C[(rb - n + g) + wc * n] * ((!wx && fcf) ? -1.0 : 0.0);
        }
    }
}

template <int I, int K>
__device__ __forceinline__ d4 qd_tile(const ElemIn &ea, const ElemIn &eb, bool fcf, int g, int c) {
    return d4{qd_elem<I, K, 0>(ea, eb, fcf, g, c), qd_elem<I, K, 1>(ea, eb, fcf, g, c),
              qd_elem<I, K, 2>(ea, eb, fcf, g, c), qd_elem<I, K, 3>(ea, eb, fcf, g, c)};
}

// Row i < 96 of the linear column (branch-free): p_b, f_a on the junction
// rows x_m, lam_m; p_a, f_b on the outer rows x_s, lam_e.
__device__ __forceinline__ double qd_lin_bf(const ElemIn &ea, const ElemIn &eb, bool fcf, int i) {
    constexpr int n = QD_N, NJ = QD_NJ;
    const int u = i - NJ;
    const int idx = i < NJ ? (i >> 1) : (u < n ? u : u - n);
    const double *p = i < NJ ? ((i & 1) ? ea.f : eb.p) : (u < n ? ea.p : eb.f);
    return p[idx] * ((i < NJ || u < n || fcf) ? 1.0 : 0.0);
}

template <int W>
__device__ __forceinline__ void qd_assemble(d4 (&Q)[6], const ElemIn &ea, const ElemIn &eb, bool fcf, int g, int c) {
    using TL = QdTiles<W>;
#define QD_ASM(s) \
    if constexpr ((s) < TL::n) Q[s] = qd_tile<TL::I[s], TL::K[s]>(ea, eb, fcf, g, c);
    QD_ASM(0) QD_ASM(1) QD_ASM(2) QD_ASM(3) QD_ASM(4) QD_ASM(5)
#undef QD_ASM
}

// MFMA operands of the tiles with LO <= K <= HI from the V / W of the current
// block: [A0, A1, B0, B1] = V of its rows and W of its columns at the pivots
// g and 4 + g (K chunks 0 and 1).
template <int W, int LO, int HI>
__device__ __forceinline__ void qd_operands(double (&op)[6][4], const double *vw, int g, int c) {
    using TL = QdTiles<W>;
#pragma unroll
    for (int s = 0; s < TL::n; ++s) {
        if (TL::K[s] < LO || TL::K[s] > HI) continue;
        const double *va = vw + (16 * TL::I[s] + c) * QD_VWS, *vb = vw + (16 * TL::K[s] + c) * QD_VWS + 8;
        op[s][0] = va[g];
        op[s][1] = va[4 + g];
        op[s][2] = vb[g];
        op[s][3] = vb[4 + g];
    }
}

// The rank-8 update of the tiles with LO <= K <= HI: every first K chunk,
// then every second (independent MFMAs back to back).  SPLIT: the second
// chunk on its own accumulator (one product deep; the critical tiles).
template <int W, int LO, int HI, bool SPLIT>
__device__ __forceinline__ void qd_update(d4 (&Q)[6], const double (&op)[6][4]) {
    using TL = QdTiles<W>;
    d4 Z[6];
#pragma unroll
    for (int s = 0; s < TL::n; ++s)
        if (TL::K[s] >= LO && TL::K[s] <= HI) Q[s] = mfma_f64(-op[s][0], op[s][2], Q[s]);
#pragma unroll
    for (int s = 0; s < TL::n; ++s)
        if (TL::K[s] >= LO && TL::K[s] <= HI) {
            if (SPLIT) Z[s] = mfma_f64(-op[s][1], op[s][3], d4{0.0, 0.0, 0.0, 0.0});
            else Q[s] = mfma_f64(-op[s][1], op[s][3], Q[s]);
        }
    if (SPLIT)
#pragma unroll
        for (int s = 0; s < TL::n; ++s)
            if (TL::K[s] >= LO && TL::K[s] <= HI) Q[s] += Z[s];
}

// Publish block T's pivot rows M[8 T .. 8 T + 7, :] from the tiles of column
// tile T / 2 (the diagonal tile: rows J at its 16 columns; below it: the
// columns J at its 16 rows, by symmetry).
template <int W, int T>
__device__ __forceinline__ void qd_publish(const d4 (&Q)[6], double *pr, int g, int c) {
    using TL = QdTiles<W>;
    constexpr int pt = T >> 1, h = T & 1;
#pragma unroll
    for (int s = 0; s < TL::n; ++s) {
        if (TL::K[s] != pt) continue;
        if (TL::I[s] == pt) {
#pragma unroll
            for (int rr = 0; rr < 2; ++rr) pr[(16 * pt + c) * QD_PRS + 4 * rr + g] = Q[s][2 * h + rr];
        } else if ((c >> 3) == h) {
#pragma unroll
            for (int r = 0; r < 4; ++r) pr[(16 * TL::I[s] + 4 * r + g) * QD_PRS + (c & 7)] = Q[s][r];
        }
    }
}

// Block T: LDL^T of the pivot block in pr (wave-uniform values, every wave
// after barrier A): L (strict lower) and 1/d in registers.  False if a pivot
// has the wrong sign.  (Round 6: wave 0 factored before barrier A and broadcast
// L, 1/d through LDS; every wave factoring for itself drops the store, the 22
// LDS reads per thread and wave 0's factor from ahead of the barrier.)
template <int T>
__device__ __forceinline__ bool qd_factor_regs(const double *pr, double (&L)[8][8], double (&inv)[8]) {
    constexpr int J0 = 8 * T;
    double a[8][8];
#pragma unroll
    for (int l = 0; l < 8; ++l)
#pragma unroll
        for (int l2 = 0; l2 <= l; ++l2) a[l][l2] = pr[(J0 + l2) * QD_PRS + l];
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const double d = a[j][j];
        ok = ok && ((j & 1) == 0 ? d > 0.0 : d < 0.0);  // J0 even: j even is an x pivot
        inv[j] = rcp_f64(d);
#pragma unroll
        for (int i = j + 1; i < 8; ++i) L[i][j] = a[i][j] * inv[j];
#pragma unroll
        for (int i = j + 1; i < 8; ++i)
#pragma unroll
            for (int k = j + 1; k <= i; ++k) a[i][k] = __builtin_fma(-L[i][j], a[k][j], a[i][k]);
    }
    return ok;
}

// Every wave: the column / linear-column row of this thread (25 per wave).
__device__ __forceinline__ int qd_col(int tid) { return 25 * (tid >> 6) + (tid & 63); }

// One combine's block loop on wave W.
template <int W>
__device__ __forceinline__ bool qd_wave(d4 (&Q)[6], double &lin, double *pr, double *vw, double *lb, int g, int c,
                                        int tid) {
    constexpr int PRS = QD_PRS, VWS = QD_VWS, AUG = QD_AUG, NCOL = QD_NCOL, NT = QD_NT;
    const int lane = tid & 63;
    const int col = qd_col(tid);
    const bool own = (tid & 63) < 25 && col < NCOL;  // this thread's column (and row of the linear column)
    double op[6][4], V[8];
    bool ok = true;
#if QD_PROF
    QdProf prof;
#endif
    // block 0's pivot rows, from the assembled tiles
    qd_publish<W, 0>(Q, pr, g, c);
    (void)lb;
    (void)lane;
#pragma unroll
    for (int t = 0; t < QD_STEPS; ++t) {
        const int J0 = 8 * t;
        if (own && col >= J0 && col < J0 + 8) pr[AUG * PRS + (col - J0)] = lin;  // linear column, rows J
        QD_MARK(0);
        __syncthreads();  // A_t
        QD_MARK(1);
#if QD_DEFER
        // block t - 1's update of the tiles right of block t's panel (operands
        // read before A_t): issued here so the matrix pipe runs it under the
        // factor's VALU chain instead of ahead of the barrier
#define QD_REST(TT, PN) \
    if (t == (TT) + 1) qd_update<W, PN + 1, 5, false>(Q, op);
        QD_REST(0, 0) QD_REST(1, 1) QD_REST(2, 1) QD_REST(3, 2) QD_REST(4, 2)
#undef QD_REST
#endif
        // ---- the pivot block's LDL^T (every wave), V, W of this thread's column ----
        {
            const bool act = own && col >= J0 + 8;
            const int cc = act ? col : J0 + 8;  // clamped (branch-free reads)
            typedef double d2 __attribute__((ext_vector_type(2)));
            double x[8], L[8][8], inv[8];
#pragma unroll
            for (int l = 0; l < 4; ++l) {
                const d2 v = reinterpret_cast<const d2 *>(pr + cc * PRS)[l];
                x[2 * l] = v.x;
                x[2 * l + 1] = v.y;
            }
            bool okt = true;
#define QD_FAC(TT) \
    if (t == (TT)) okt = qd_factor_regs<TT>(pr, L, inv);
            QD_FAC(0) QD_FAC(1) QD_FAC(2) QD_FAC(3) QD_FAC(4) QD_FAC(5)
#undef QD_FAC
            ok = ok && okt;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                double v = x[j];
#pragma unroll
                for (int k = 0; k < j; ++k) v = __builtin_fma(-L[j][k], V[k], v);
                V[j] = v;
            }
            if (act) {
                double *o = vw + col * VWS;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    o[j] = V[j];
                    o[8 + j] = V[j] * inv[j];
                }
            }
        }
        QD_MARK(2);
        __syncthreads();  // B_t
        QD_MARK(3);
        if (own && col >= J0 + 8 && col < NT) {  // linear column, row col: -= V[:, col]^T W[:, AUG]
            const double *w = vw + AUG * VWS + 8;
#pragma unroll
            for (int j = 0; j < 8; ++j) lin = __builtin_fma(-V[j], w[j], lin);
        }
        // ---- block t's update: the tiles of block t + 1's pivots first ----
        if (t == QD_STEPS - 1) {
            qd_operands<W, 3, 5>(op, vw, g, c);
            qd_update<W, 3, 5, false>(Q, op);
            break;
        }
        constexpr int dummy = 0;
        (void)dummy;
        const int pn = (t + 1) >> 1;  // column tile of block t + 1's pivots
#define QD_STEP(TT, PN)                                            \
    if (t == (TT)) {                                               \
        qd_operands<W, PN, PN>(op, vw, g, c);                      \
        qd_update<W, PN, PN, true>(Q, op);                         \
        qd_operands<W, PN + 1, 5>(op, vw, g, c);                   \
        qd_publish<W, (TT) + 1>(Q, pr, g, c);                      \
        if (!QD_DEFER) qd_update<W, PN + 1, 5, false>(Q, op);      \
    }
        QD_STEP(0, 0)
        QD_STEP(1, 1)
        QD_STEP(2, 1)
        QD_STEP(3, 2)
        QD_STEP(4, 2)
#undef QD_STEP
        (void)pn;
    }
#if QD_PROF
    if (tid == 0) prof.save(27);
    if (tid == 64) prof.save(23);
#endif
    return ok;
}

// out = a (x) b for n = 24 on a 256-thread block; qs: qd_smem_doubles() of LDS
// (16-byte aligned).  The operands are read before any output is written and
// only through ea / eb, so outputs may alias the global copies of operands
// the caller staged into LDS.  fcf = false: only P, p are written.  Returns the
// block-uniform status (every x pivot positive, every lam pivot negative).
__device__ __forceinline__ bool qd_combine(double *oF, double *oC, double *of, double *oP, double *op,
                                           const ElemIn &ea, const ElemIn &eb, bool fcf, double *qs) {
    constexpr int n = QD_N, NT = QD_NT, NCOL = QD_NCOL, PRS = QD_PRS, VWS = QD_VWS;
    constexpr int XS = QD_NJ, LE = QD_NJ + n;
    const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, c = lane & 15;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches on the role
    double *pr = qs, *vw = qs + NCOL * PRS, *lb = vw + NCOL * VWS;
    int *okw = reinterpret_cast<int *>(lb + 36);
    COMB_MARK(0);
    d4 Q[6];
    const int col = qd_col(tid);
    double lin = qd_lin_bf(ea, eb, fcf, (lane < 25 && col < NT) ? col : 0);  // row col of the linear column
    if (wv == 0) qd_assemble<0>(Q, ea, eb, fcf, g, c);
    else if (wv == 1) qd_assemble<1>(Q, ea, eb, fcf, g, c);
    else if (wv == 2) qd_assemble<2>(Q, ea, eb, fcf, g, c);
    else qd_assemble<3>(Q, ea, eb, fcf, g, c);
    COMB_MARK(1);
    bool ok = true;
    if (wv == 0) ok = qd_wave<0>(Q, lin, pr, vw, lb, g, c, tid);
    else if (wv == 1) qd_wave<1>(Q, lin, pr, vw, lb, g, c, tid);
    else if (wv == 2) qd_wave<2>(Q, lin, pr, vw, lb, g, c, tid);
    else qd_wave<3>(Q, lin, pr, vw, lb, g, c, tid);
    COMB_MARK(7);
    // ---- outputs: x_s = rows / columns 48 .. 71, lam_e = 72 .. 95 ----
    auto out_tile = [&](const d4 &T, int I, int K) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 16 * I + 4 * r + g, j = 16 * K + c;
            const double v = T[r];
            if (i < LE && j < LE) {
                if (i >= j) {
                    oP[(i - XS) + (j - XS) * n] = v;
                    oP[(j - XS) + (i - XS) * n] = v;
                }
            } else if (fcf) {
                if (j < LE) {
                    oF[(i - LE) + (j - XS) * n] = v;
                } else if (i >= j) {
                    oC[(i - LE) + (j - LE) * n] = -v;
                    oC[(j - LE) + (i - LE) * n] = -v;
                }
            }
        }
    };
    if (wv == 1) {
        out_tile(Q[4], 3, 3);
        out_tile(Q[5], 4, 3);
    } else if (wv == 2) {
        out_tile(Q[5], 4, 4);
    } else if (wv == 3 && fcf) {
        out_tile(Q[3], 5, 3);
        out_tile(Q[4], 5, 4);
        out_tile(Q[5], 5, 5);
    }
    if (lane < 25) {
        if (col >= XS && col < LE) op[col - XS] = lin;
        if (fcf && col >= LE && col < NT) of[col - LE] = lin;
    }
    if (tid == 0) okw[0] = 1;
    __syncthreads();
    if (!ok) okw[0] = 0;  // wave 0 carries the pivot checks
    __syncthreads();
    COMB_MARK(8);
    return okw[0] != 0;
}

#undef QD_MARK
#undef QD_PROF

}  // namespace pdplqr
