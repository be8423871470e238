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
// Cholesky factors come from chol_tiles (device_common.hpp); the triangular
// solve for U and the matrix-vector products go through LDS.
#pragma once

#include "device_common.hpp"

namespace pdplqr {

template <int T>
struct WM {
    d4 t[T][T];
};

template <int T>
struct CombSmem {
    static constexpr int P = 16 * T, PL = P + 1;
    double A[P * PL];  // Q, then Z (vector products)
    double B[P * PL];  // R -> U in place, then output staging (symmetrisation)
    alignas(16) double cb[P];
    double sinv[P], luq[P];
    double v1[P], v2[P], v3[P], v4[P];
};

// M <- n x n block at p (column-major, leading dimension ld, or its transpose);
// outside the block: `pad` on the diagonal, 0 elsewhere
template <int T>
__device__ __forceinline__ void wm_load(WM<T> &M, const double *p, int ld, int n, bool trans, double pad, int g,
                                        int c) {
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int b = 0; b < T; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
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

// C = sgn X^T Y + diag I (+ add); only the K chunks that hold rows < n
template <int T>
__device__ __forceinline__ void wm_tn(WM<T> &C, const WM<T> &X, const WM<T> &Y, int n, double sgn, double diag,
                                      const WM<T> *add, int g, int c) {
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int b = 0; b < T; ++b) {
            d4 acc;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * a + 4 * r + g, j = 16 * b + c;
                acc[r] = (add ? add->t[a][b][r] : 0.0) + (i == j ? diag : 0.0);
            }
#pragma unroll
            for (int kt = 0; kt < T; ++kt)
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
                    if (16 * kt + 4 * kk < n) acc = mfma_f64(sgn * X.t[kt][a][kk], Y.t[kt][b][kk], acc);
            C.t[a][b] = acc;
        }
}

template <int T>
__device__ __forceinline__ bool wm_chol(WM<T> &M, int n, CombSmem<T> &sm, int g, int c) {
    double lpr[T][4];
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) lpr[a][r] = 0.0;
    const bool ok = chol_tiles<T>(M.t, lpr, sm.cb, sm.sinv, sm.luq, 0, n, 0, false, g, c);
    finalize_L<T>(M.t, sm.sinv, 0, n, g, c);
    wave_sync();
    return ok;
}

// Y = P_b (I + C_a P_b)^{-1}, Z = I - C_a Y, Zt = Z^T.  False if P_b or the
// SPD core is not positive definite.
template <int T>
__device__ __forceinline__ bool comb_core(WM<T> &Y, WM<T> &Z, WM<T> &Zt, const WM<T> &Ca, const double *Pb, int n,
                                          CombSmem<T> &sm, int lane) {
    constexpr int P = 16 * T, PL = P + 1;
    const int g = lane >> 4, c = lane & 15;
    WM<T> R, S;
    wm_load(R, Pb, n, n, false, 1.0, g, c);
    bool ok = wm_chol(R, n, sm, g, c);
    {
        WM<T> T1;
        wm_tn(T1, Ca, R, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);  // C_a R
        wm_tn(S, R, T1, n, 1.0, 1.0, (const WM<T> *)nullptr, g, c);   // I + R^T C_a R
    }
    ok = wm_chol(S, n, sm, g, c) && ok;  // Q
    wm_store(S, sm.A, PL, P, g, c);
    wm_store(R, sm.B, PL, P, g, c);
    wave_sync();
    // U = Q^{-1} R^T, column j on lane j, in place over R: lane j reads only
    // R[j][i] with i <= j (the lower triangle; R^T[i][j] = 0 for i > j) and
    // writes U[i][j] = B[i + j PL], an entry no other lane reads later.
    if (lane < n) {
        const int j = lane;
        for (int i = 0; i < n; ++i) {
            double v = (i <= j) ? sm.B[j + i * PL] : 0.0;
            for (int k = 0; k < i; ++k) v -= sm.A[i + k * PL] * sm.B[k + j * PL];
            sm.B[i + j * PL] = v * sm.sinv[i];  // sinv[i] = 1 / Q[i][i]
        }
    }
    wave_sync();
    WM<T> U;
    wm_load(U, sm.B, PL, n, false, 1.0, g, c);
    wm_tn(Y, U, U, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);  // Y = U^T U
    wm_tn(Z, Ca, Y, n, -1.0, 1.0, (const WM<T> *)nullptr, g, c);  // Z = I - C_a Y
    wm_tn(Zt, Y, Ca, n, -1.0, 1.0, (const WM<T> *)nullptr, g, c);  // Z^T = I - Y C_a
    wave_sync();
    return ok;
}

// y = add + op(M) x  (n-vectors, M column-major ld), lanes over rows
__device__ __forceinline__ void lds_mv(double *y, const double *M, int ld, bool trans, const double *x,
                                       const double *add, double sgn, int n, int lane) {
    if (lane < n) {
        double acc = 0.0;
        for (int k = 0; k < n; ++k) acc = __builtin_fma(trans ? M[k + lane * ld] : M[lane + k * ld], x[k], acc);
        y[lane] = (add ? add[lane] : 0.0) + sgn * acc;
    }
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

// out = a (x) b  (a earlier, b later).  Element memory (global or LDS):
// [F | C | f | P | p], column-major n x n blocks.  out must not alias a or b.
template <int T>
__device__ __forceinline__ bool tcombine(double *out, const double *ea, const double *eb, int n, bool need_FCf,
                                         bool need_Pp, CombSmem<T> &sm, int lane) {
    constexpr int PL = 16 * T + 1;
    const int g = lane >> 4, c = lane & 15;
    const int nn = n * n;
    const double *aF = ea, *aC = ea + nn, *af = ea + 2 * nn, *aP = ea + 2 * nn + n, *ap = ea + 3 * nn + n;
    const double *bF = eb, *bC = eb + nn, *bf = eb + 2 * nn, *bP = eb + 2 * nn + n, *bp = eb + 3 * nn + n;
    double *oF = out, *oC = out + nn, *of = out + 2 * nn, *oP = out + 2 * nn + n, *op = out + 3 * nn + n;
    WM<T> Ca, Y, Z, Zt;
    wm_load(Ca, aC, n, n, false, 0.0, g, c);
    const bool ok = comb_core(Y, Z, Zt, Ca, bP, n, sm, lane);
    WM<T> Fa;
    wm_load(Fa, aF, n, n, false, 0.0, g, c);
    if (need_Pp) {  // P = P_a + F_a^T (Y F_a)
        WM<T> W, Pn, Pa;
        wm_tn(W, Y, Fa, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);
        wm_load(Pa, aP, n, n, false, 0.0, g, c);
        wm_tn(Pn, Fa, W, n, 1.0, 0.0, &Pa, g, c);
        wm_store_sym(Pn, oP, n, sm, lane);
    }
    if (need_FCf) {
        WM<T> Fbt, W, Fn;
        wm_load(Fbt, bF, n, n, true, 0.0, g, c);                     // F_b^T
        wm_tn(W, Zt, Fa, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);   // Z F_a
        wm_tn(Fn, Fbt, W, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);  // F_b Z F_a
        wm_store(Fn, oF, n, n, g, c);
        WM<T> W2t, W3, Cn, Cb;
        wm_tn(W2t, Ca, Zt, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);   // C_a Z^T = (Z C_a)^T
        wm_tn(W3, W2t, Fbt, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);  // Z C_a F_b^T
        wm_load(Cb, bC, n, n, false, 0.0, g, c);
        wm_tn(Cn, Fbt, W3, n, 1.0, 0.0, &Cb, g, c);                     // F_b Z C_a F_b^T + C_b
        wm_store_sym(Cn, oC, n, sm, lane);
    }
    // vectors, with Z in LDS
    wm_store(Z, sm.A, PL, n, g, c);
    wave_sync();
    if (need_FCf) {
        lds_mv(sm.v1, aC, n, false, bp, af, -1.0, n, lane);   // v1 = f_a - C_a p_b
        wave_sync();
        lds_mv(sm.v2, sm.A, PL, false, sm.v1, nullptr, 1.0, n, lane);  // Z v1
        wave_sync();
        lds_mv(of, bF, n, false, sm.v2, bf, 1.0, n, lane);    // f = F_b Z v1 + f_b
    }
    if (need_Pp) {
        lds_mv(sm.v3, bP, n, false, af, bp, 1.0, n, lane);     // v3 = p_b + P_b f_a
        wave_sync();
        lds_mv(sm.v4, sm.A, PL, true, sm.v3, nullptr, 1.0, n, lane);  // Z^T v3
        wave_sync();
        lds_mv(op, aF, n, true, sm.v4, ap, 1.0, n, lane);      // p = p_a + F_a^T Z^T v3
    }
    wave_sync();
    return ok;
}

}  // namespace pdplqr
