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
// solve for U runs with the column in registers (Q staged in LDS); the
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
// blockIdx % 1024; read back with pdplqr_debug_comb_times).
#if defined(PDPLQR_COMB_PROFILE) && defined(PDPLQR_COMB_PROFILE_TU)  // kernels_parallel.hip only
extern __device__ unsigned long long g_comb_t[1024 * 16];
#define COMB_MARK(k)                                                                     \
    do {                                                                                 \
        if (threadIdx.x == 0) g_comb_t[(blockIdx.x % 1024) * 16 + (k)] = wall_clock64(); \
    } while (0)
#else
#define COMB_MARK(k) \
    do {             \
    } while (0)
#endif

template <int T>
struct CombSmem {
    static constexpr int P = 16 * T, PL = P + 1;
    alignas(16) double A[P * (P + 2)];  // Q^T (row stride P + 2), then Z (vector products)
    double B[P * PL];  // R -> U in place, then output staging (symmetrisation)
    alignas(16) double cb[P];  // pivot-row broadcast of chol_tiles
    double sinv[P], luq[P];
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
    finalize_L<T>(M.t, sm.sinv, 0, n, g, c);  // sinv[i] = 1 / L[i][i]
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
    COMB_MARK(1);
    wm_load(R, Pb, n, n, false, 1.0, g, c);
    bool ok = wm_chol(R, n, sm, g, c);
    COMB_MARK(2);
    {
        WM<T> T1;
        wm_tn(T1, Ca, R, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);  // C_a R
        wm_tn(S, R, T1, n, 1.0, 1.0, (const WM<T> *)nullptr, g, c);   // I + R^T C_a R
    }
    COMB_MARK(3);
    ok = wm_chol(S, n, sm, g, c) && ok;  // Q
    COMB_MARK(4);
    // U = Q^{-1} R^T by forward substitution, column j on lane j with the
    // column in registers (loops unrolled over the padded size P).  Q is
    // staged transposed (row i of Q contiguous: 128-bit broadcast reads),
    // R as is (lane j reads its row j = column j of R^T).
    constexpr int PQ = P + 2;  // even row stride keeps the 16-byte alignment
    double *Qt = sm.A, *Rs = sm.B;
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int b = 0; b < T; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * a + 4 * r + g, j = 16 * b + c;
                Qt[j + i * PQ] = S.t[a][b][r];  // Qt[k + i PQ] = Q[i][k]
                Rs[i + j * PL] = R.t[a][b][r];
            }
    wave_sync();
    double u[P];
    const int j = lane < P ? lane : P - 1;
#pragma unroll
    for (int i = 0; i < P; ++i) {
        if (i < n) {
            double v0 = (i <= j) ? Rs[j + i * PL] : 0.0, v1 = 0.0;
            const double2 *qrow = reinterpret_cast<const double2 *>(Qt + i * PQ);
#pragma unroll
            for (int k2 = 0; k2 < (i + 1) / 2; ++k2) {
                const double2 q = qrow[k2];
                v0 = __builtin_fma(-q.x, u[2 * k2], v0);
                if (2 * k2 + 1 < i) v1 = __builtin_fma(-q.y, u[2 * k2 + 1], v1);
            }
            u[i] = (v0 + v1) * sm.sinv[i];  // sinv[i] = 1 / Q[i][i]
        } else {
            u[i] = (i == j) ? 1.0 : 0.0;  // identity padding
        }
    }
    wave_sync();  // all reads of Qt / Rs done
    // U (column j on lane j) -> C/D layout through LDS
    if (lane < P)
#pragma unroll
        for (int i = 0; i < P; ++i) Rs[i + lane * PL] = u[i];
    wave_sync();
    COMB_MARK(5);
    WM<T> U;
    wm_load(U, Rs, PL, P, false, 1.0, g, c);
    wm_tn(Y, U, U, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);  // Y = U^T U
    wm_tn(Z, Ca, Y, n, -1.0, 1.0, (const WM<T> *)nullptr, g, c);  // Z = I - C_a Y
    wm_tn(Zt, Y, Ca, n, -1.0, 1.0, (const WM<T> *)nullptr, g, c);  // Z^T = I - Y C_a
    wave_sync();
    COMB_MARK(6);
    return ok;
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
#pragma unroll
    for (int a = 0; a < T; ++a) {
        d4 acc = add ? add->t[a] : d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kt = 0; kt < T; ++kt)
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
                if (16 * kt + 4 * kk < n) acc = mfma_f64(sgn * X.t[kt][a][kk], x.t[kt][kk], acc);
        y.t[a] = acc;
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
// when need_Pp is false) and must not alias the inputs.  P_a and C_b are read
// once, as addends of the last products: they are loaded up front so a
// global-memory source costs no exposed latency.
template <int T>
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
    const bool ok = comb_core(Y, Z, Zt, Ca, bP, n, sm, lane);
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

template <int T>
__device__ __forceinline__ bool tcombine(double *out, const double *ea, const double *eb, int n, bool need_FCf,
                                         bool need_Pp, CombSmem<T> &sm, int lane) {
    const int nn = n * n;
    return tcombine_parts<T>(out, out + nn, out + 2 * nn, out + 2 * nn + n, out + 3 * nn + n, elem_in(ea, n),
                             elem_in(eb, n), n, need_FCf, need_Pp, sm, lane);
}

}  // namespace pdplqr
