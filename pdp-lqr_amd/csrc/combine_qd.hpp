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
// column) lives in 16 x 16 MFMA tiles, lower triangle only (21 tiles).  Per
// block of pivots J (two barriers, no products outside the elimination):
//   1. the owners publish the pivot rows M[J, :] to LDS (by symmetry the
//      pivot COLUMNS of the tiles below the diagonal);            -> barrier A
//   2. waves 2, 3 (one thread per column) factor the 8 x 8 pivot block LDL^T
//      (wave-uniform) and form V = L^{-1} M[J, col], W = D^{-1} V;  -> barrier B
//   3. every active tile takes the rank-8 update M[I, K] -= V[:, I]^T W[:, K]
//      as two MFMAs (A operand V of the tile's rows, B operand W of its
//      columns, both read from LDS); the linear column row by row.
// Roles: waves 0, 1 own the 15 tiles of the junction columns (and the linear
// column, one row a thread); waves 2, 3 own the 6 tiles of the outer block and
// do step 2.  The critical path of a block is  B -> the tiles holding the next
// pivots (K = their tile) -> publish -> A -> LDL^T, V, W -> B;  every other
// update of the block (the outer tiles, junction tiles whose pivots come
// later) has its operands read before A and its MFMAs issued after it, beside
// step 2 of the next block.  Each wave's code is specialised at compile time
// (tile list, step), so the MFMAs of a step issue back to back without
// branches.
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

__host__ __device__ constexpr int qd_smem_doubles() { return QD_NCOL * QD_PRS + QD_NCOL * QD_VWS + 2; }

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

// Tile lists of waves 1..3 (compile time; wave 0 owns no tile).  The tiles
// whose column holds the next block's pivots (K = 0 at block 0, 1 at blocks
// 1-2, 2 at blocks 3-4) are the critical ones: 2/2/2, 2/2/1, 1/2/1 a wave;
// 7 tiles each in all.
template <int W>
struct QdTiles;
template <>
struct QdTiles<1> {
    static constexpr int n = 7;
    static constexpr int I[7] = {0, 1, 1, 2, 2, 3, 4}, K[7] = {0, 0, 1, 1, 2, 3, 3};
};
template <>
struct QdTiles<2> {
    static constexpr int n = 7;
    static constexpr int I[7] = {2, 3, 3, 4, 3, 4, 4}, K[7] = {0, 0, 1, 1, 2, 2, 4};
};
template <>
struct QdTiles<3> {
    static constexpr int n = 7;
    static constexpr int I[7] = {4, 5, 5, 5, 5, 5, 5}, K[7] = {0, 0, 1, 2, 3, 4, 5};
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
__device__ __forceinline__ void qd_assemble(d4 (&Q)[7], const ElemIn &ea, const ElemIn &eb, bool fcf, int g, int c) {
    using TL = QdTiles<W>;
#define QD_ASM(s) Q[s] = qd_tile<TL::I[s], TL::K[s]>(ea, eb, fcf, g, c);
    QD_ASM(0) QD_ASM(1) QD_ASM(2) QD_ASM(3) QD_ASM(4) QD_ASM(5) QD_ASM(6)
#undef QD_ASM
}

// MFMA operands of the tiles with LO <= K <= HI from the V / W of the current
// block: [A0, A1, B0, B1] = V of its rows and W of its columns at the pivots
// g and 4 + g (K chunks 0 and 1).
template <int W, int LO, int HI>
__device__ __forceinline__ void qd_operands(double (&op)[7][4], const double *vw, int g, int c) {
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
__device__ __forceinline__ void qd_update(d4 (&Q)[7], const double (&op)[7][4]) {
    using TL = QdTiles<W>;
    d4 Z[7];
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

// Waves 1..3: the tiles.  After barrier B of block t: the tiles holding block
// t + 1's pivots take block t's update and publish (critical); the other
// active tiles read their operands and take the update after barrier A of
// block t + 1, beside wave 0's factorisation.
template <int W>
__device__ __forceinline__ void qd_tile_wave(d4 (&Q)[7], double *pr, const double *vw, int g, int c) {
    using TL = QdTiles<W>;
    constexpr int PRS = QD_PRS;
    double op[7][4];
#if QD_PROF
    QdProf prof;
#endif
#pragma unroll
    for (int t = 0; t < QD_STEPS; ++t) {
        const int pt = t >> 1, h = t & 1;
        // ---- publish block t's pivot rows M[8 t .. 8 t + 7, :] ----
#pragma unroll
        for (int s = 0; s < TL::n; ++s) {
            if (TL::K[s] != pt) continue;
            if (TL::I[s] == pt) {  // the diagonal tile: rows J at its 16 columns
#pragma unroll
                for (int rr = 0; rr < 2; ++rr) pr[(16 * pt + c) * PRS + 4 * rr + g] = Q[s][2 * h + rr];
            } else if ((c >> 3) == h) {  // below it: columns J at its 16 rows (symmetry)
#pragma unroll
                for (int r = 0; r < 4; ++r) pr[(16 * TL::I[s] + 4 * r + g) * PRS + (c & 7)] = Q[s][r];
            }
        }
        QD_MARK(0);
        __syncthreads();  // A_t
        QD_MARK(3);
        // block t - 1's updates of the tiles whose pivots come later
        if (t == 1) qd_update<W, 1, 5, false>(Q, op);
        if (t == 2 || t == 3) qd_update<W, 2, 5, false>(Q, op);
        if (t == 4 || t == 5) qd_update<W, 3, 5, false>(Q, op);
        __syncthreads();  // B_t
        QD_MARK(1);
        // block t's update: the tiles of block t + 1's pivots now, the rest read
        if (t == 0) {
            qd_operands<W, 0, 0>(op, vw, g, c);
            qd_update<W, 0, 0, true>(Q, op);
            qd_operands<W, 1, 5>(op, vw, g, c);
        } else if (t == 1 || t == 2) {
            qd_operands<W, 1, 1>(op, vw, g, c);
            qd_update<W, 1, 1, true>(Q, op);
            qd_operands<W, 2, 5>(op, vw, g, c);
        } else if (t == 3 || t == 4) {
            qd_operands<W, 2, 2>(op, vw, g, c);
            qd_update<W, 2, 2, true>(Q, op);
            qd_operands<W, 3, 5>(op, vw, g, c);
        } else {
            qd_operands<W, 3, 5>(op, vw, g, c);
        }
        QD_MARK(2);
    }
    qd_update<W, 3, 5, false>(Q, op);  // block 5
#if QD_PROF
    if (threadIdx.x == 64) prof.save(23);
#endif
}

// Wave 0: per block, the LDL^T of the 8 x 8 pivot block (wave-uniform) and
// V = L^{-1} M[J, col], W = D^{-1} V of every column (columns lane, lane + 64),
// and the linear column (rows lane, lane + 64).
__device__ __forceinline__ bool qd_factor_wave(double (&lin)[2], double *pr, double *vw, int lane) {
    constexpr int PRS = QD_PRS, VWS = QD_VWS, NCOL = QD_NCOL, NT = QD_NT, AUG = QD_AUG;
    bool ok = true;
#if QD_PROF
    QdProf prof;
#endif
#pragma unroll 1
    for (int t = 0; t < QD_STEPS; ++t) {
        const int J0 = 8 * t;
        // publish the linear column's rows J (rows lane and lane + 64)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int row = lane + 64 * u;
            if (row >= J0 && row < J0 + 8) pr[AUG * PRS + (row - J0)] = lin[u];
        }
        __syncthreads();  // A_t
        QD_MARK(0);
        double a[8][8], x[2][8];
#pragma unroll
        for (int l = 0; l < 8; ++l)
#pragma unroll
            for (int l2 = 0; l2 <= l; ++l2) a[l][l2] = pr[(J0 + l2) * PRS + l];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int col = lane + 64 * u, cc = (col >= J0 + 8 && col < NCOL) ? col : J0 + 8;  // clamped
#pragma unroll
            for (int l = 0; l < 8; ++l) x[u][l] = pr[cc * PRS + l];
        }
        // right-looking LDL^T of the pivot block carrying the two columns: after
        // pivot j, x[j] = V[j] = (L^{-1} x)[j] (the fmas of a forward
        // substitution with L, in its order)
        double inv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const double d = a[j][j];
            ok = ok && ((j & 1) == 0 ? d > 0.0 : d < 0.0);  // J0 even: j even is an x pivot
            inv[j] = rcp_f64(d);
            double Lj[8];
#pragma unroll
            for (int i = j + 1; i < 8; ++i) Lj[i] = a[i][j] * inv[j];
#pragma unroll
            for (int i = j + 1; i < 8; ++i) {
#pragma unroll
                for (int k = j + 1; k <= i; ++k) a[i][k] = __builtin_fma(-Lj[i], a[k][j], a[i][k]);
#pragma unroll
                for (int u = 0; u < 2; ++u) x[u][i] = __builtin_fma(-Lj[i], x[u][j], x[u][i]);
            }
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int col = lane + 64 * u;
            if (col >= J0 + 8 && col < NCOL) {
                double *o = vw + col * VWS;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    o[j] = x[u][j];
                    o[8 + j] = x[u][j] * inv[j];
                }
            }
        }
        wave_sync();  // W of the linear column (lane 32's second column) to every lane
        const double *w = vw + AUG * VWS + 8;
#pragma unroll
        for (int u = 0; u < 2; ++u) {  // linear column, row lane + 64 u: -= V[:, row]^T W[:, AUG]
            const int row = lane + 64 * u;
            if (row >= J0 + 8 && row < NT)
#pragma unroll
                for (int j = 0; j < 8; ++j) lin[u] = __builtin_fma(-x[u][j], w[j], lin[u]);
        }
        QD_MARK(1);
        __syncthreads();  // B_t
        QD_MARK(2);
    }
#if QD_PROF
    if (threadIdx.x == 0) prof.save(27);
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
    double *pr = qs, *vw = qs + NCOL * PRS;
    int *okw = reinterpret_cast<int *>(vw + NCOL * VWS);
    COMB_MARK(0);
    d4 Q[7];
    double lin[2] = {0.0, 0.0};
    bool ok = true;
    if (wv == 0) {
        lin[0] = qd_lin_bf(ea, eb, fcf, lane);
        lin[1] = qd_lin_bf(ea, eb, fcf, lane < 32 ? lane + 64 : 0);
    } else if (wv == 1) {
        qd_assemble<1>(Q, ea, eb, fcf, g, c);
    } else if (wv == 2) {
        qd_assemble<2>(Q, ea, eb, fcf, g, c);
    } else {
        qd_assemble<3>(Q, ea, eb, fcf, g, c);
    }
    COMB_MARK(1);
    if (wv == 0) ok = qd_factor_wave(lin, pr, vw, lane);
    else if (wv == 1) qd_tile_wave<1>(Q, pr, vw, g, c);
    else if (wv == 2) qd_tile_wave<2>(Q, pr, vw, g, c);
    else qd_tile_wave<3>(Q, pr, vw, g, c);
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
    if (wv == 0) {
        if (lane >= XS) op[lane - XS] = lin[0];                       // rows 48 .. 63
        if (lane < LE - 64) op[lane + 64 - XS] = lin[1];              // rows 64 .. 71
        if (fcf && lane >= LE - 64 && lane < NT - 64) of[lane + 64 - LE] = lin[1];  // rows 72 .. 95
    } else if (wv == 1) {
        out_tile(Q[5], 3, 3);
        out_tile(Q[6], 4, 3);
    } else if (wv == 2) {
        out_tile(Q[6], 4, 4);
    } else if (fcf) {
        out_tile(Q[4], 5, 3);
        out_tile(Q[5], 5, 4);
        out_tile(Q[6], 5, 5);
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
