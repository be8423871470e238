// combine_mw.hpp -- the segment-element combine (SURVEY.md 0.1,
// condensed_system.hpp:203-290, Cholesky form) spread over a 4-wave workgroup.
//
// The one-wave combine (combine_tiles.hpp tcombine_parts) is a chain of two
// 24-pivot factorisations and ~12 products of 2 x 2 f64 tiles on ONE SIMD; a
// dependent v_mfma_f64_16x16x4 costs ~186 cycles and 24 independent ones of a
// product ~1,700 (scripts/ubench/lat_bench.hip), so most of its 16 us is MFMA
// issue of products that do not depend on each other.  Here the algebra is
// re-arranged so that everything except the two factorisations is at most one
// product deep after them, and the products run on four waves:
//
//     R = chol(P_b),   S = I + R^T C_a R = Q Q^T
//     X1 = Q^{-1} R^T F_a,   W = Q^{-1} R^T C_a F_b^T,         (carried through chol(S))
//     x3 = Q^{-1} R^T (f_a - C_a p_b),   x4 = Q^{-1} R^T C_a (p_b + P_b f_a)
// and with Y = P_b (I + C_a P_b)^{-1} = R S^{-1} R^T:
//     F = F_b F_a - W^T X1                  (= F_b Z F_a,  Z = I - C_a Y)
//     C = F_b C_a F_b^T + C_b - W^T W        (= F_b Z C_a F_b^T + C_b)
//     P = P_a + X1^T X1                      (= P_a + F_a^T Y F_a)
//     f = F_b v1 + f_b - W^T x3              (v1 = f_a - C_a p_b)
//     p = p_a + F_a^T u - X1^T x4            (u = p_b + P_b f_a)
// Phases (barriers between them), waves w0..w3:
//   A  w0: R = chol(P_b) (U = R^T to LDS);  w1: K2 = F_b F_a, C_a u, v1;
//      w2: K0 = C_a F_b^T;  w3: K0 (own copy), F_b v1 + f_b, p_a + F_a^T u
//      (inputs only)
//   B  w0: S;  w1: R^T F_a;  w2: R^T K0 (R read from LDS) -> LDS;
//      w3: R^T C_a u, R^T v1, K1 = F_b K0 + C_b
//   C  every wave: chol(S) carrying ONE column tile of the right-hand sides
//   D  w0: P;  w1: F;  w2: C;  w3: f, p                                    -> HBM
// When the right operand holds the real terminal (F = C = f = 0 there and in
// the result) only P and p are formed.  The result equals the one-wave
// combine's to rounding (same algebra, different association).
#pragma once

#include "combine_tiles.hpp"

namespace pdplqr {

// LDS of one combine, in a dynamic buffer sized by mw_smem_bytes(n): five
// n x n blocks at leading dimension ld = n + 1 (odd for even n: column reads
// hit distinct banks) and four n-vectors.  At n = 24: 24.6 KB, 6 blocks per CU.
// Phase B: R^T C_a u and R^T v1 on wave 3 (idle there otherwise) instead of
// after R^T F_a on wave 1, the slowest wave of the phase (comb_ab.log: the
// block waited 2.5 us for it).  0: on wave 1 (A/B).

struct MwSmem {
    int ld;
    double *S;   // w0: R transpose scratch, then S; phase D: w0's staging
    double *B1;  // w1: R scratch, then R^T F_a; after chol: X1
    double *B2;  // w2: R scratch, then R^T C_a F_b^T; after chol: W
    double *K1;  // w3: F_b C_a F_b^T + C_b; phase D: w2's staging
    double *K2;  // w3: F_b F_a
    double *bv;  // [R^T v1 | R^T C_a u] (columns of ld n); after chol: [x3 | x4]
    double *fv, *pv;  // F_b v1 + f_b, p_a + F_a^T u
    int *ok;
};

__host__ __device__ inline size_t mw_smem_bytes(int n) {
    return (size_t)(5 * n * (n + 1) + 4 * n) * sizeof(double) + 16;
}

__device__ __forceinline__ MwSmem mw_smem(double *base, int n) {
    MwSmem m;
    m.ld = n + 1;
    const int blk = n * (n + 1);
    m.S = base;
    m.B1 = base + blk;
    m.B2 = base + 2 * blk;
    m.K1 = base + 3 * blk;
    m.K2 = base + 4 * blk;
    m.bv = base + 5 * blk;
    m.fv = m.bv + 2 * n;
    m.pv = m.fv + n;
    m.ok = reinterpret_cast<int *>(m.pv + n);
    return m;
}

// column tile j (T row tiles) of an n x n column-major block in LDS (ld PL)
template <int T>
__device__ __forceinline__ void mw_col_load(d4 (&B)[T][1], const double *p, int PL, int j, int n, int g, int c) {
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 16 * a + 4 * r + g, jj = 16 * j + c;
            B[a][0][r] = (i < n && jj < n) ? p[i + jj * PL] : 0.0;
        }
}

template <int T>
__device__ __forceinline__ void mw_col_store(const d4 (&B)[T][1], double *p, int PL, int j, int n, int g, int c) {
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 16 * a + 4 * r + g, jj = 16 * j + c;
            if (i < n && jj < n) p[i + jj * PL] = B[a][0][r];
        }
}

// two vectors as columns 0, 1 of one column tile (ld n): [v | w] in LDS
template <int T>
__device__ __forceinline__ void mw_vec2_load(d4 (&B)[T][1], const double *p, int n, int g, int c) {
    const int P = n;
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 16 * a + 4 * r + g;
            B[a][0][r] = (i < n && c < 2) ? p[i + c * P] : 0.0;
        }
}

template <int T>
__device__ __forceinline__ void mw_vec2_store(const d4 (&B)[T][1], double *p, int n, int g, int c) {
    const int P = n;
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 16 * a + 4 * r + g;
            if (i < n && c < 2) p[i + c * P] = B[a][0][r];
        }
}

// R = chol(P_b) in C layout (lower; identity padding) through the wave's own
// LDS region `scr` (chol_blk4 leaves R^T).  False if P_b is not definite.
template <int T>
__device__ __forceinline__ bool mw_chol_R(WM<T> &R, const double *Pb, double *scr, int PL, int n, int g, int c) {
    WM<T> U;
    wm_load(U, Pb, n, n, false, 1.0, g, c);
    COMB_MARK(19);  // P_b loaded
    const bool ok = chol_blk4<T, false, T>(U, U.t, n, g, c);  // U = R^T
    COMB_MARK(20);  // factored
    wm_store(U, scr, PL, n, g, c);
    wave_sync();
    wm_load(R, scr, PL, n, true, 1.0, g, c);
    wave_sync();
    return ok;
}

// symmetric store out = (M + M^T) / 2 (n x n, ld n) through `stg` (ld PL)
template <int T>
__device__ __forceinline__ void mw_store_sym(const WM<T> &M, double *out, double *stg, int PL, int n, int lane) {
    wm_store(M, stg, PL, n, lane >> 4, lane & 15);
    wave_sync();
    for (int q = lane; q < n * n; q += 64) {
        const int i = q % n, j = q / n;
        out[q] = 0.5 * (stg[i + j * PL] + stg[j + i * PL]);
    }
}

// out = a (x) b on a 256-thread block (4 waves).  fcf = false: the right
// operand holds the real terminal; only P, p are written (F, C, f untouched).
// Returns (block-uniform) whether both factorisations were definite.
template <int T>
__device__ __forceinline__ bool mw_combine(double *oF, double *oC, double *of, double *oP, double *op,
                                           const ElemIn &ea, const ElemIn &eb, int n, bool fcf, const MwSmem &sm) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
    const int PL = sm.ld;
    bool ok = true;
    COMB_MARK(0);
    // ---------------- phase A ----------------
    // (matrices are loaded right before their last use: at most four 2 x 2
    // tile matrices live per wave)
    // R is factored ONCE (wave 0) and shared through LDS: waves 1 and 2 form
    // the products that do not need R meanwhile (a redundant factorisation per
    // wave costs issue slots the co-resident blocks of a scan round need).
    // Wave 0's factor U = R^T lands in sm.S; S then goes to the staged P_b
    // slot (P_b is dead after phase A), so the R reads and S cannot race.
    WM<T> R, K0w3;  // K0w3: wave 3's C_a F_b^T, phase A -> B
    double *Sd = const_cast<double *>(eb.P);  // S, leading dimension n
    if (wv == 0) {
        ok = mw_chol_R<T>(R, eb.P, sm.S, sm.ld, n, g, c);
    } else if (wv == 1) {
        WV<T> fa, pb, u, cu;
        wv_load(fa, ea.f, n, g, c);
        wv_load(pb, eb.p, n, g, c);
        {
            WM<T> Pb;
            wm_load(Pb, eb.P, n, n, false, 0.0, g, c);
            wv_tn(u, Pb, fa, n, 1.0, &pb);  // u = p_b + P_b f_a
        }
        WM<T> Ca;
        wm_load(Ca, ea.C, n, n, false, 0.0, g, c);
        wv_tn(cu, Ca, u, n, 1.0, (const WV<T> *)nullptr);  // C_a u
        wv_store(cu, sm.bv + n, n, g, c);
        if (fcf) {
            WV<T> v1;
            wv_tn(v1, Ca, pb, n, -1.0, &fa);  // v1 = f_a - C_a p_b
            wv_store(v1, sm.bv, n, g, c);
            WM<T> Fa, Fbt, B;
            wm_load(Fa, ea.F, n, n, false, 0.0, g, c);
            wm_load(Fbt, eb.F, n, n, true, 0.0, g, c);
            wm_tn(B, Fbt, Fa, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);  // F_b F_a
            wm_store(B, sm.K2, PL, n, g, c);
        }
    } else if (wv == 2) {
        if (fcf) {
            WM<T> Ca, Fbt, K0;
            wm_load(Ca, ea.C, n, n, false, 0.0, g, c);
            wm_load(Fbt, eb.F, n, n, true, 0.0, g, c);
            wm_tn(K0, Ca, Fbt, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);  // C_a F_b^T
            wm_store(K0, sm.B2, PL, n, g, c);
        }
    } else {
        WV<T> fa, pb, u;
        wv_load(fa, ea.f, n, g, c);
        wv_load(pb, eb.p, n, g, c);
        {
            WM<T> Pb;
            wm_load(Pb, eb.P, n, n, false, 0.0, g, c);
            wv_tn(u, Pb, fa, n, 1.0, &pb);  // u = p_b + P_b f_a
        }
        {
            WM<T> Fa;
            WV<T> pa, t;
            wv_load(pa, ea.p, n, g, c);
            wm_load(Fa, ea.F, n, n, false, 0.0, g, c);
            wv_tn(t, Fa, u, n, 1.0, &pa);  // p_a + F_a^T u
            wv_store(t, sm.pv, n, g, c);
        }
        if (fcf) {
            WM<T> Ca, Fbt;
            WV<T> v1, fb, fo;
            wm_load(Ca, ea.C, n, n, false, 0.0, g, c);
            wv_tn(v1, Ca, pb, n, -1.0, &fa);  // v1 = f_a - C_a p_b
            wm_load(Fbt, eb.F, n, n, true, 0.0, g, c);
            wv_load(fb, eb.f, n, g, c);
            wv_tn(fo, Fbt, v1, n, 1.0, &fb);  // F_b v1 + f_b
            wv_store(fo, sm.fv, n, g, c);
            wm_tn(K0w3, Ca, Fbt, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);  // C_a F_b^T
            // F_b K0 + C_b follows in phase B: here it would outlast wave 0's
            // factorisation and hold the phase-A barrier (comb_phases: full
            // combines waited ~1.4 us for this wave)
        }
    }
    COMB_MARK(1);  // wave 0: R formed
    __syncthreads();  // U = R^T in sm.S; P_b's slot free
    // ---------------- phase B ----------------
    if (wv == 0) {
        WM<T> Ca, T1, S;
        wm_load(Ca, ea.C, n, n, false, 0.0, g, c);
        wm_tn(T1, Ca, R, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);  // C_a R
        wm_tn(S, R, T1, n, 1.0, 1.0, (const WM<T> *)nullptr, g, c);   // I + R^T C_a R
        wm_store(S, Sd, n, n, g, c);
        if (lane == 0) sm.ok[0] = ok;
    } else if (wv == 1) {
        wm_load(R, sm.S, PL, n, true, 1.0, g, c);
        {
            WM<T> Fa, B;
            wm_load(Fa, ea.F, n, n, false, 0.0, g, c);
            wm_tn(B, R, Fa, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);  // R^T F_a
            wm_store(B, sm.B1, PL, n, g, c);
        }
    } else if (wv == 3) {  // the two vector products on the wave phase B leaves idle
        wm_load(R, sm.S, PL, n, true, 1.0, g, c);
        WV<T> cu, v1, y;
        wv_load(cu, sm.bv + n, n, g, c);
        if (fcf) wv_load(v1, sm.bv, n, g, c);
        wv_tn(y, R, cu, n, 1.0, (const WV<T> *)nullptr);  // R^T C_a u
        wv_store(y, sm.bv + n, n, g, c);
        if (fcf) {
            wv_tn(y, R, v1, n, 1.0, (const WV<T> *)nullptr);  // R^T v1
            wv_store(y, sm.bv, n, g, c);
            WM<T> Fbt, Cb, K;
            wm_load(Fbt, eb.F, n, n, true, 0.0, g, c);
            wm_load(Cb, eb.C, n, n, false, 0.0, g, c);
            wm_tn(K, Fbt, K0w3, n, 1.0, 0.0, &Cb, g, c);  // F_b C_a F_b^T + C_b (read in phase D)
            wm_store(K, sm.K1, PL, n, g, c);
        }
    } else if (wv == 2 && fcf) {
        WM<T> K0, B;
        wm_load(R, sm.S, PL, n, true, 1.0, g, c);
        wm_load(K0, sm.B2, PL, n, false, 0.0, g, c);
        wm_tn(B, R, K0, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);  // R^T C_a F_b^T
        wm_store(B, sm.B2, PL, n, g, c);
    }
    COMB_MARK(2);  // wave 0: S stored
    __syncthreads();
    COMB_MARK(3);  // every wave through phase B
    // ---------------- phase C: chol(S) carrying one column tile per wave ----------------
    // T = 2: w0 / w1 the two tiles of X1, w2 / w3 those of W (w3 also [x3 | x4]);
    // T = 1: w0 [x3 | x4], w1 X1, w2 W.  Without F, C, f: X1 and x4 only.
    ok = ok && sm.ok[0];
    {
        WM<T> S;
        wm_load(S, Sd, n, n, false, 1.0, g, c);
        d4 B[T][1], V[T][1];
        int kind = -1, tile = 0;  // 0: X1, 1: W, 2: vectors (block-uniform)
        if (T == 2) {
            kind = wv < 2 ? 0 : (fcf ? 1 : (wv == 2 ? 2 : -1));
            tile = wv & 1;
        } else {
            kind = wv == 0 ? 2 : (wv == 1 ? 0 : (wv == 2 && fcf ? 1 : -1));
        }
        const bool vec3 = T == 2 && wv == 3 && fcf;  // w3 carries the vectors beside its W tile
        if (kind == 0) mw_col_load<T>(B, sm.B1, PL, tile, n, g, c);
        else if (kind == 1) mw_col_load<T>(B, sm.B2, PL, tile, n, g, c);
        else if (kind == 2) mw_vec2_load<T>(B, sm.bv, n, g, c);
        if (vec3) mw_vec2_load<T>(V, sm.bv, n, g, c);
        bool okS = true;
        if (vec3) {
            d4 BV[T][2];
#pragma unroll
            for (int a = 0; a < T; ++a) {
                BV[a][0] = B[a][0];
                BV[a][1] = V[a][0];
            }
            okS = chol_blk4<T, true, 2>(S, BV, n, g, c);
#pragma unroll
            for (int a = 0; a < T; ++a) {
                B[a][0] = BV[a][0];
                V[a][0] = BV[a][1];
            }
        } else if (kind >= 0) {
            okS = chol_blk4<T, true, 1>(S, B, n, g, c);
        }
        COMB_MARK(4);  // wave 0: chol(S) done
        __syncthreads();  // every wave has read its right-hand sides
        if (kind == 0) mw_col_store<T>(B, sm.B1, PL, tile, n, g, c);
        else if (kind == 1) mw_col_store<T>(B, sm.B2, PL, tile, n, g, c);
        else if (kind == 2) mw_vec2_store<T>(B, sm.bv, n, g, c);
        if (vec3) mw_vec2_store<T>(V, sm.bv, n, g, c);
        if (wv == (T == 2 ? 0 : 1) && lane == 0) sm.ok[1] = okS;
    }
    __syncthreads();
    COMB_MARK(5);  // phase C complete
    ok = ok && sm.ok[1];
    // ---------------- phase D ----------------
    if (wv == 0) {  // P = P_a + X1^T X1
        WM<T> X1, Pa, Pn;
        wm_load(X1, sm.B1, PL, n, false, 0.0, g, c);
        wm_load(Pa, ea.P, n, n, false, 0.0, g, c);
        wm_tn(Pn, X1, X1, n, 1.0, 0.0, &Pa, g, c);
        mw_store_sym<T>(Pn, oP, sm.S, PL, n, lane);
    } else if (wv == 1 && fcf) {  // F = F_b F_a - W^T X1
        WM<T> X1, Wm, K2, Fn;
        wm_load(X1, sm.B1, PL, n, false, 0.0, g, c);
        wm_load(Wm, sm.B2, PL, n, false, 0.0, g, c);
        wm_load(K2, sm.K2, PL, n, false, 0.0, g, c);
        wm_tn(Fn, Wm, X1, n, -1.0, 0.0, &K2, g, c);
        wm_store(Fn, oF, n, n, g, c);
    } else if (wv == 2 && fcf) {  // C = F_b C_a F_b^T + C_b - W^T W
        WM<T> Wm, K1, Cn;
        wm_load(Wm, sm.B2, PL, n, false, 0.0, g, c);
        wm_load(K1, sm.K1, PL, n, false, 0.0, g, c);
        wave_sync();  // K1 is in registers before the staging reuses its region
        wm_tn(Cn, Wm, Wm, n, -1.0, 0.0, &K1, g, c);
        mw_store_sym<T>(Cn, oC, sm.K1, PL, n, lane);
    } else if (wv == 3) {  // f = F_b v1 + f_b - W^T x3,  p = p_a + F_a^T u - X1^T x4
        WM<T> X1;
        WV<T> x3, x4, pa, po;
        wm_load(X1, sm.B1, PL, n, false, 0.0, g, c);
        wv_load(x4, sm.bv + n, n, g, c);
        wv_load(pa, sm.pv, n, g, c);
        wv_tn(po, X1, x4, n, -1.0, &pa);
        wv_store(po, op, n, g, c);
        if (fcf) {
            WM<T> Wm;
            WV<T> fb, fo;
            wm_load(Wm, sm.B2, PL, n, false, 0.0, g, c);
            wv_load(x3, sm.bv, n, g, c);
            wv_load(fb, sm.fv, n, g, c);
            wv_tn(fo, Wm, x3, n, -1.0, &fb);
            wv_store(fo, of, n, g, c);
        }
    }
    COMB_MARK(6);  // wave 0: P stored
#ifdef PDPLQR_COMB_PROFILE
    __syncthreads();
#endif
    COMB_MARK(7);  // every wave through phase D
    COMB_MARK(8);
    COMB_MARK(9);
    return ok;
}

}  // namespace pdplqr
