// combine_qd1.hpp -- the segment-element combine (SURVEY.md 0.1,
// condensed_system.hpp:203-290) for n <= 12 (n % 4 == 0) on ONE wavefront, as
// one blocked LDL^T elimination of the quasi-definite junction block: the
// single-wave form of combine_qd.hpp (which explains the algebra).  The
// element e = (F, C, f, P, p) combine a (x) b is the Schur complement of the
// junction J = [[P_b, -I], [-I, -C_a]] (rows / columns x_m, lam_m interleaved)
// in the symmetric matrix over [x_m, lam_m | x_s, lam_e | 1]; the outer block
// left after the 2n junction pivots is [[P, F^T, p], [F, -C, f]].
//
// One wave holds the whole 4n x 4n matrix as 16 x 16 MFMA tiles (lower
// triangle, TN (TN + 1) / 2 tiles, TN = 4n / 16) and its linear column (lane =
// row).  Per block of 8 pivots:
//   1. the pivot rows go to LDS (the diagonal tile's rows, the pivot columns of
//      the tiles below it by symmetry, the linear column's 8 entries);
//   2. every lane factors the 8 x 8 pivot block LDL^T (wave-uniform values, no
//      broadcast of the factor: the one-wave form needs no third LDS trip);
//   3. lane = column: V = L^{-1} M[J, col], W = D^{-1} V to LDS;
//   4. the linear column row by row, then M[I, K] -= V[:, I]^T W[:, K] on the
//      trailing tiles as two MFMAs each (K chunks of 4 pivots).
// Against the Cholesky form (tcombine_parts: chol(P_b), then chol(I + R^T C_a R)
// and the products between): 2n pivots in 2n / 8 blocks and no products
// outside the elimination.  Pivot signs are the status: every x pivot > 0 and
// every lam pivot < 0 (P_b definite, C_a semidefinite), as chol(P_b) failing
// is in the Cholesky form.
#pragma once

#include "combine_tiles.hpp"

namespace pdplqr {

template <int NN>
struct Qd1 {
    static constexpr int n = NN, NJ = 2 * NN, NT = 4 * NN, AUG = NT, NCOL = NT + 1;
    static constexpr int TN = NT / 16;  // tile rows
    static constexpr int STEPS = NJ / 8;
    static constexpr int PRS = 10;  // pivot rows: [column][8] at stride 10 (16-byte rows)
    static constexpr int VWS = 18;  // [column][V 0..7 | W 0..7] at stride 18
    static constexpr int smem = NCOL * PRS + NCOL * VWS;  // doubles of LDS per wave
    static_assert(NN % 4 == 0 && NT % 16 == 0 && NCOL <= 64, "one-wave junction combine: n % 4 == 0, n <= 12");
};

__host__ __device__ constexpr int qd1_tile(int I, int K) { return I * (I + 1) / 2 + K; }

// Entry (16 I + 4 R + g, 16 K + c) of the matrix before the elimination.  One
// load at a lane-selected address scaled by a lane-selected factor (a select
// among loaded values compiles to divergent branches around the loads).
template <int NN, int I, int K, int R>
__device__ __forceinline__ double qd1_elem(const ElemIn &ea, const ElemIn &eb, bool fcf, int g, int c) {
    constexpr int n = NN, NJ = 2 * NN, XE = NJ + NN;
    constexpr int rb = 16 * I + 4 * R;  // row of g = 0 (a row group never straddles NJ or XE: n % 4 == 0)
    const int i = rb + g, j = 16 * K + c;
    const double *p;
    double f, k = 0.0;
    if constexpr (rb < NJ) {  // junction row: x_m (i even) / lam_m (odd) a
        const int a = i >> 1, si = i & 1;
        if (j < NJ) {
            const int bb = j >> 1, sj = j & 1;
            p = (si & sj) ? ea.C + (a + bb * n) : eb.P + (a + bb * n);
            f = si == sj ? (si ? -1.0 : 1.0) : 0.0;
            k = (si != sj && a == bb) ? -1.0 : 0.0;
        } else if (j < XE) {  // (lam_m a, x_s v) = F_a[a][v]
            p = ea.F + (a + (j - NJ) * n);
            f = si ? 1.0 : 0.0;
        } else {  // (x_m a, lam_e v) = F_b[v][a]
            p = eb.F + ((j - XE) + a * n);
            f = (si == 0 && fcf) ? 1.0 : 0.0;
        }
    } else if constexpr (rb < XE) {  // x_s row u
        const int u = i - NJ;
        if (j < NJ) {  // (x_s u, lam_m bb) = F_a[bb][u]
            p = ea.F + ((j >> 1) + u * n);
            f = (j & 1) ? 1.0 : 0.0;
        } else if (j < XE) {  // P_a
            p = ea.P + (u + (j - NJ) * n);
            f = 1.0;
        } else {
            p = ea.P;
            f = 0.0;
        }
    } else {  // lam_e row u
        const int u = i - XE;
        if (j < NJ) {  // (lam_e u, x_m bb) = F_b[u][bb]
            p = eb.F + (u + (j >> 1) * n);
            f = ((j & 1) == 0 && fcf) ? 1.0 : 0.0;
        } else if (j < XE) {
            p = eb.F;
            f = 0.0;
        } else {  // -C_b
            p = eb.C + (u + (j - XE) * n);
            f = fcf ? -1.0 : 0.0;
        }
    }
    return __builtin_fma(*p, f, k);
}

template <int NN, int I, int K>
__device__ __forceinline__ d4 qd1_tile_in(const ElemIn &ea, const ElemIn &eb, bool fcf, int g, int c) {
    return d4{qd1_elem<NN, I, K, 0>(ea, eb, fcf, g, c), qd1_elem<NN, I, K, 1>(ea, eb, fcf, g, c),
              qd1_elem<NN, I, K, 2>(ea, eb, fcf, g, c), qd1_elem<NN, I, K, 3>(ea, eb, fcf, g, c)};
}

// out = a (x) b for n = NN on one wave; sm: Qd1<NN>::smem doubles of this
// wave's LDS (16-byte aligned).  Operands are read before any output is
// written and only through ea / eb.  fcf = false: only P, p are written.
// Returns the wave-uniform status.
template <int NN>
__device__ __forceinline__ bool qd1_combine(double *oF, double *oC, double *of, double *oP, double *op,
                                            const ElemIn &ea, const ElemIn &eb, bool fcf, double *sm, int lane) {
    using Q1 = Qd1<NN>;
    constexpr int n = NN, NJ = Q1::NJ, XE = NJ + NN, NT = Q1::NT, AUG = Q1::AUG, NCOL = Q1::NCOL;
    constexpr int TN = Q1::TN, PRS = Q1::PRS, VWS = Q1::VWS;
    constexpr int NTL = TN * (TN + 1) / 2;
    typedef double d2 __attribute__((ext_vector_type(2)));
    const int g = lane >> 4, c = lane & 15;
    double *pr = sm, *vw = sm + NCOL * PRS;
    d4 Q[NTL];
    // ---- assembly (every operand load issued before the first use) ----
#define QD1_T(I, K) \
    if constexpr ((I) < TN && (K) <= (I)) Q[qd1_tile(I, K)] = qd1_tile_in<NN, I, K>(ea, eb, fcf, g, c);
    QD1_T(0, 0) QD1_T(1, 0) QD1_T(1, 1) QD1_T(2, 0) QD1_T(2, 1) QD1_T(2, 2)
#undef QD1_T
    double lin;
    {
        const int i = lane < NT ? lane : 0, u = i - NJ;
        const double *p = i < NJ ? ((i & 1) ? ea.f + (i >> 1) : eb.p + (i >> 1)) : (u < n ? ea.p + u : eb.f + (u - n));
        lin = *p * ((lane < NT && (i < NJ || u < n || fcf)) ? 1.0 : 0.0);
    }
    bool ok = true;
#pragma unroll
    for (int t = 0; t < Q1::STEPS; ++t) {
        const int J0 = 8 * t, IT = J0 >> 4, h = (J0 >> 3) & 1;
        // ---- 1. pivot rows J0 .. J0 + 7 ----
#pragma unroll
        for (int I = 0; I < TN; ++I) {
            if (I < IT) continue;
            const d4 &T = Q[qd1_tile(I, IT)];
            if (I == IT) {
#pragma unroll
                for (int rr = 0; rr < 2; ++rr) pr[(16 * IT + c) * PRS + 4 * rr + g] = T[2 * h + rr];
            } else if ((c >> 3) == h) {
#pragma unroll
                for (int r = 0; r < 4; ++r) pr[(16 * I + 4 * r + g) * PRS + (c & 7)] = T[r];
            }
        }
        if (lane >= J0 && lane < J0 + 8) pr[AUG * PRS + (lane - J0)] = lin;
        wave_sync();
        // ---- 2. LDL^T of the pivot block (every lane, uniform values) ----
        double L[8][8], inv[8];
        {
            double a[8][8];
#pragma unroll
            for (int l = 0; l < 8; ++l)
#pragma unroll
                for (int l2 = 0; l2 <= l; ++l2) a[l][l2] = pr[(J0 + l2) * PRS + l];
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
        }
        // ---- 3. V, W of column `lane` (clamped reads: branch-free) ----
        double V[8];
        {
            const bool act = lane >= J0 + 8 && lane < NCOL;
            const int cc = act ? lane : J0 + 8;
            double x[8];
#pragma unroll
            for (int l = 0; l < 4; ++l) {
                const d2 v = reinterpret_cast<const d2 *>(pr + cc * PRS)[l];
                x[2 * l] = v.x;
                x[2 * l + 1] = v.y;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                double v = x[j];
#pragma unroll
                for (int k = 0; k < j; ++k) v = __builtin_fma(-L[j][k], V[k], v);
                V[j] = v;
            }
            if (act) {
                d2 *o = reinterpret_cast<d2 *>(vw + lane * VWS);
#pragma unroll
                for (int l = 0; l < 4; ++l) o[l] = d2{V[2 * l], V[2 * l + 1]};
#pragma unroll
                for (int l = 0; l < 4; ++l) o[4 + l] = d2{V[2 * l] * inv[2 * l], V[2 * l + 1] * inv[2 * l + 1]};
            }
        }
        wave_sync();
        // ---- 4. the linear column, then the trailing tiles ----
        if (lane >= J0 + 8 && lane < NT) {
            const double *w = vw + AUG * VWS + 8;
#pragma unroll
            for (int j = 0; j < 8; ++j) lin = __builtin_fma(-V[j], w[j], lin);
        }
        const int KT = (J0 + 8) >> 4;  // first tile column with a live (not yet eliminated) column
        double op4[NTL][4];
#pragma unroll
        for (int I = 0; I < TN; ++I)
#pragma unroll
            for (int K = 0; K <= I; ++K) {
                if (K < KT) continue;
                const double *va = vw + (16 * I + c) * VWS, *vb = vw + (16 * K + c) * VWS + 8;
                double *o = op4[qd1_tile(I, K)];
                o[0] = va[g];
                o[1] = va[4 + g];
                o[2] = vb[g];
                o[3] = vb[4 + g];
            }
        // the tiles of column KT first (they hold the next block's pivot rows, which
        // the next publish waits for), then the rest; within each group every
        // first K chunk before every second (independent MFMAs back to back)
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
            for (int I = 0; I < TN; ++I)
#pragma unroll
                for (int K = 0; K <= I; ++K) {
                    if (K < KT || (pass == 0) != (K == KT)) continue;
                    const double *o = op4[qd1_tile(I, K)];
                    Q[qd1_tile(I, K)] = mfma_f64(-o[0], o[2], Q[qd1_tile(I, K)]);
                }
#pragma unroll
            for (int I = 0; I < TN; ++I)
#pragma unroll
                for (int K = 0; K <= I; ++K) {
                    if (K < KT || (pass == 0) != (K == KT)) continue;
                    const double *o = op4[qd1_tile(I, K)];
                    Q[qd1_tile(I, K)] = mfma_f64(-o[1], o[3], Q[qd1_tile(I, K)]);
                }
        }
        wave_sync();  // this block's LDS reads retire before the next block's writes
    }
    // ---- outputs: x_s = rows / columns NJ .. XE - 1, lam_e = XE .. NT - 1 ----
#pragma unroll
    for (int I = 0; I < TN; ++I)
#pragma unroll
        for (int K = 0; K <= I; ++K) {
            if (16 * I + 15 < NJ || 16 * K + 15 < NJ) continue;
            const d4 &T = Q[qd1_tile(I, K)];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * I + 4 * r + g, j = 16 * K + c;
                const double v = T[r];
                if (i < NJ || j < NJ || i < j) continue;
                if (i < XE) {  // j <= i < XE: P
                    oP[(i - NJ) + (j - NJ) * n] = v;
                    oP[(j - NJ) + (i - NJ) * n] = v;
                } else if (fcf) {
                    if (j < XE) {
                        oF[(i - XE) + (j - NJ) * n] = v;
                    } else {
                        oC[(i - XE) + (j - XE) * n] = -v;
                        oC[(j - XE) + (i - XE) * n] = -v;
                    }
                }
            }
        }
    if (lane >= NJ && lane < XE) op[lane - NJ] = lin;
    if (fcf && lane >= XE && lane < NT) of[lane - XE] = lin;
    return ok;
}

}  // namespace pdplqr
