// blk_la.hpp -- dense linear algebra of one 256-thread block (4 wavefronts) on
// matrices of order <= 64 held in LDS, for the wide shapes 32 < n + m <= 64
// (kernels_wide.hip).  The tiled kernels keep a whole stage matrix in the MFMA
// registers of one wave; past 32 rows that no longer fits, so here the
// matrices live in LDS and every product is split over the four waves by
// 16 x 16 output tile (at most 16 tiles: four v_mfma_f64_16x16x4_f64
// accumulators per wave), its operands read straight from LDS (or global
// memory) in the MFMA A/B layouts.  Factorisations are right-looking, one
// pivot per block barrier, a row per thread (or per thread pair).
//
// Conventions: column-major, element (i, j) of a view at p[i + j ld]
// (transposed views: p[j + i ld]; packed symmetric views: the lower-packed
// layout of the model's H, pidx()).  Every blk_* call starts and ends on a
// block barrier, so consecutive calls may read what the previous one wrote
// and a product may overwrite its own operands (the tiles are accumulated in
// registers and stored after a barrier).
#pragma once

#include "device_common.hpp"

namespace pdplqr {

constexpr int BLK_THREADS = 256;

// read view of a matrix: dense (optionally transposed) or packed symmetric
struct Mv {
    const double *p;
    int ld;
    int kind;  // 0 dense, 1 transposed, 2 packed symmetric (ld = order)
    __device__ __forceinline__ double at(int i, int j) const {
        if (kind == 0) return p[i + j * ld];
        if (kind == 1) return p[j + i * ld];
        return p[i >= j ? pidx(i, j, ld) : pidx(j, i, ld)];
    }
};

__device__ __forceinline__ Mv mv_n(const double *p, int ld) { return Mv{p, ld, 0}; }
__device__ __forceinline__ Mv mv_t(const double *p, int ld) { return Mv{p, ld, 1}; }
__device__ __forceinline__ Mv mv_pk(const double *p, int order) { return Mv{p, order, 2}; }
__device__ __forceinline__ Mv mv_none() { return Mv{nullptr, 0, 0}; }

// C (M x N, ldc) = alpha A B + diag I + add, A: M x K, B: K x N (views).
// lower: only tiles on or below the diagonal are formed (C symmetric by
// construction) and mirrored on store.  C may alias A, B (not add when
// lower).  M, N <= 64.
// element offset of a view: strides for dense / transposed, the packed lower
// index of (max, min) for packed symmetric views (PK)
template <bool PK>
__device__ __forceinline__ int mv_off(int i, int j, int si, int sj, int ld) {
    if constexpr (PK) return i >= j ? pidx(i, j, ld) : pidx(j, i, ld);
    else return i * si + j * sj;
}

// The product loop, specialised on whether A / B are packed views: the view
// kind is hoisted out of the loop (a runtime switch per element cost a scalar
// branch per load) and the loads are branch-free (clamped indices and a
// select: a guarded load compiles to an exec-mask region with its own wait).
// LDS pointer of a generic one known to address LDS (ds_read instead of the
// flat path, which takes the vector-memory pipeline and both wait counters)
typedef const __attribute__((address_space(3))) double *lds_cptr;
__device__ __forceinline__ bool in_lds(const void *p) {
    return __builtin_amdgcn_is_shared((const __attribute__((address_space(0))) void *)p);
}

template <bool PA, bool PB, bool SH>
__device__ __forceinline__ void blk_mm_loop(d4 (&acc)[4], const int (&ti)[4], const int (&tj)[4], const bool (&on)[4],
                                            const Mv &A, const Mv &B, int M, int N, int K, int g, int c) {
    const int sai = A.kind == 1 ? A.ld : 1, saj = A.kind == 1 ? 1 : A.ld;
    const int sbi = B.kind == 1 ? B.ld : 1, sbj = B.kind == 1 ? 1 : B.ld;
    for (int k0 = 0; k0 < K; k0 += 4) {
        const int k = k0 + g;
        const int kc = k < K ? k : K - 1;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            if (!on[t]) continue;  // wave-uniform
            const int i = 16 * ti[t] + c, j = 16 * tj[t] + c;
            const int ic = i < M ? i : M - 1, jc = j < N ? j : N - 1;
            double av, bv;
            if constexpr (SH) {
                av = ((lds_cptr)A.p)[mv_off<PA>(ic, kc, sai, saj, A.ld)];
                bv = ((lds_cptr)B.p)[mv_off<PB>(kc, jc, sbi, sbj, B.ld)];
            } else {
                av = A.p[mv_off<PA>(ic, kc, sai, saj, A.ld)];
                bv = B.p[mv_off<PB>(kc, jc, sbi, sbj, B.ld)];
            }
            const double a = (k < K && i < M) ? av : 0.0;
            const double b = (k < K && j < N) ? bv : 0.0;
            acc[t] = mfma_f64(a, b, acc[t]);
        }
    }
}

__device__ __noinline__ void blk_mm(double *C, int ldc, Mv A, Mv B, int M, int N, int K, double alpha, double diag,
                                    Mv add, bool lower) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
    const int TM = (M + 15) >> 4, TN = (N + 15) >> 4;
    d4 acc[4];
    int ti[4], tj[4];
    bool on[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int q = wv + 4 * t;
        ti[t] = q % TM;
        tj[t] = q / TM;
        on[t] = q < TM * TN && (!lower || ti[t] >= tj[t]);
        acc[t] = d4{0.0, 0.0, 0.0, 0.0};
    }
    __syncthreads();  // the operands are complete
    const bool sh = in_lds(A.p) && in_lds(B.p);  // wave-uniform
    if (sh) {
        if (A.kind != 2 && B.kind != 2) blk_mm_loop<false, false, true>(acc, ti, tj, on, A, B, M, N, K, g, c);
        else if (A.kind == 2 && B.kind != 2) blk_mm_loop<true, false, true>(acc, ti, tj, on, A, B, M, N, K, g, c);
        else if (A.kind != 2) blk_mm_loop<false, true, true>(acc, ti, tj, on, A, B, M, N, K, g, c);
        else blk_mm_loop<true, true, true>(acc, ti, tj, on, A, B, M, N, K, g, c);
    } else {
        if (A.kind != 2 && B.kind != 2) blk_mm_loop<false, false, false>(acc, ti, tj, on, A, B, M, N, K, g, c);
        else if (A.kind == 2 && B.kind != 2) blk_mm_loop<true, false, false>(acc, ti, tj, on, A, B, M, N, K, g, c);
        else if (A.kind != 2) blk_mm_loop<false, true, false>(acc, ti, tj, on, A, B, M, N, K, g, c);
        else blk_mm_loop<true, true, false>(acc, ti, tj, on, A, B, M, N, K, g, c);
    }
    __syncthreads();  // every read of the operands is done: C may overwrite them
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        if (!on[t]) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 16 * ti[t] + 4 * r + g, j = 16 * tj[t] + c;
            if (i < M && j < N) {
                double v = alpha * acc[t][r] + (i == j ? diag : 0.0);
                if (add.p) v += add.at(i, j);
                C[i + j * ldc] = v;
                if (lower && ti[t] > tj[t]) C[j + i * ldc] = v;
            }
        }
    }
    __syncthreads();
}

// y (M) = alpha A x + add (vectors in LDS or global; y must not alias x).
// M <= 64: the rows on the lanes and K split over the four waves (k = w mod 4),
// the partial sums added through LDS -- a quarter of the dependent chain of one
// row per thread
__device__ __noinline__ void blk_mv(double *y, Mv A, const double *x, int M, int K, double alpha, const double *add) {
    __shared__ double part[4][64];
    const int tid = threadIdx.x;
    __syncthreads();
    if (M <= 64) {
        const int i = tid & 63, w = tid >> 6;
        double a = 0.0;
        if (A.kind != 2 && in_lds(A.p) && in_lds(x)) {  // LDS operands
            const int si = A.kind == 1 ? A.ld : 1, sk = A.kind == 1 ? 1 : A.ld;
            const lds_cptr ap = (lds_cptr)A.p, xp = (lds_cptr)x;
            if (i < M)
                for (int k = w; k < K; k += 4) a = __builtin_fma(ap[i * si + k * sk], xp[k], a);
        } else if (i < M)
            for (int k = w; k < K; k += 4) a = __builtin_fma(A.at(i, k), x[k], a);
        part[w][i] = a;
        __syncthreads();
        if (tid < M) y[tid] = alpha * ((part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid])) + (add ? add[tid] : 0.0);
    } else if (tid < M) {
        double a = 0.0;
        for (int k = 0; k < K; ++k) a = __builtin_fma(A.at(tid, k), x[k], a);
        y[tid] = alpha * a + (add ? add[tid] : 0.0);
    }
    __syncthreads();
}

// dst (M x N, ldd) <- view (copy / transpose / unpack)
__device__ __noinline__ void blk_copy(double *dst, int ldd, Mv src, int M, int N) {
    __syncthreads();
    for (int q = threadIdx.x; q < M * N; q += BLK_THREADS) {
        const int i = q % M, j = q / M;
        dst[i + j * ldd] = src.at(i, j);
    }
    __syncthreads();
}

__device__ __noinline__ void blk_vcopy(double *dst, const double *src, int n) {
    __syncthreads();
    for (int q = threadIdx.x; q < n; q += BLK_THREADS) dst[q] = src ? src[q] : 0.0;
    __syncthreads();
}

// dst (n x n, global or LDS) = (S + S^T) / 2 of the n x n block S (ld lds)
__device__ __noinline__ void blk_store_sym(double *dst, int ldd, const double *S, int lds, int n) {
    __syncthreads();
    for (int q = threadIdx.x; q < n * n; q += BLK_THREADS) {
        const int i = q % n, j = q / n;
        dst[i + j * ldd] = 0.5 * (S[i + j * lds] + S[j + i * lds]);
    }
    __syncthreads();
}

// Right-looking Cholesky of the lower triangle of M (n x n, ld, n <= 64),
// optionally carrying nb right-hand-side columns B (n x nb, ldb): on return
// M's lower triangle is L (zeros above) and B = L^{-1} B.  Pivot semantics of
// chol_tiles (device_common.hpp): a pivot j < m must be positive (else the
// result is flagged, false); a pivot j >= m that is not positive stops the
// factorisation (sinv = 1 from there, the trailing block restored to its
// input values, Eigen's LLT), flagged only when psd_bad.  m = n: every pivot
// must be positive.  sinv: n doubles of LDS scratch.
__device__ __noinline__ bool blk_chol(double *M, int ld, int n, int m, double *sinv, double *B = nullptr, int ldb = 0,
                                      int nb = 0) {
    const int tid = threadIdx.x, ri = tid & 63, cg = tid >> 6;
    bool ok = true, live = true;
    int jdead = n;
    for (int j = 0; j < n; ++j) {
        __syncthreads();
        const double d = M[j + j * ld];
        ok = ok && (j < m ? d > 0.0 : !psd_bad(d));
        if (live && !(j < m || d > 0.0)) jdead = j;
        live = live && (j < m || d > 0.0);
        const double inv2 = live ? 1.0 / d : 0.0;
        if (tid == 0) sinv[j] = live ? rsqrt_f64(d) : 1.0;
        const int i = ri;
        if (live && i > j && i < n) {  // live: block-uniform
            const double lij = M[i + j * ld] * inv2;
            lds_axpy_strided(M + i, ld, M + j * ld, lij, j + 1 + cg, i, 4);  // loads before stores, four at a time
            if (nb > 0) lds_axpy_strided(B + i, ldb, B + j, lij, cg, nb - 1, 4, ldb);
        }
    }
    __syncthreads();
    if (jdead < n) {  // block-uniform, rare: undo the live pivots' updates of the dead block
        for (int p = jdead - 1; p >= 0; --p) {
            const double inv2 = 1.0 / M[p + p * ld];
            const int i = ri;
            if (i >= jdead && i < n) {
                const double lip = M[i + p * ld] * inv2;
                for (int l = jdead + cg; l <= i; l += 4) M[i + l * ld] = __builtin_fma(lip, M[l + p * ld], M[i + l * ld]);
            }
            __syncthreads();
        }
    }
    for (int q = tid; q < n * n; q += BLK_THREADS) {
        const int i = q % n, j = q / n;
        M[i + j * ld] = i >= j ? M[i + j * ld] * sinv[j] : 0.0;
    }
    for (int q = tid; q < n * nb; q += BLK_THREADS) {
        const int i = q % n, l = q / n;
        B[i + l * ldb] *= sinv[i];
    }
    __syncthreads();
    return ok;
}

// Triangular solves with the lower factor L (n x n, ld) of blk_chol, in place
// on nb right-hand-side columns B (ld ldb) and optionally one more column v:
//   blk_trsm_l:  L X = B      blk_trsm_lt:  L^T X = B
// One barrier per row: the row of step i is final before step i and only
// read in it (the other rows are updated with L(k, i) / L(i, i) times it, the
// division by L(i, i) applied to every row at the end).
__device__ __noinline__ void blk_trsm_l(const double *L, int ld, int n, double *B, int ldb, int nb, double *v) {
    const int tid = threadIdx.x, nc = nb + (v ? 1 : 0);
    for (int i = 0; i < n; ++i) {
        __syncthreads();
        const int rows = n - 1 - i;
        const double inv = 1.0 / L[i + i * ld];
        for (int q = tid; q < rows * nc; q += BLK_THREADS) {
            const int k = i + 1 + q % rows, col = q / rows;
            const double lk = L[k + i * ld] * inv;
            if (col < nb) B[k + col * ldb] = __builtin_fma(-lk, B[i + col * ldb], B[k + col * ldb]);
            else v[k] = __builtin_fma(-lk, v[i], v[k]);
        }
    }
    __syncthreads();
    for (int q = tid; q < n * nc; q += BLK_THREADS) {
        const int k = q % n, col = q / n;
        const double inv = 1.0 / L[k + k * ld];
        if (col < nb) B[k + col * ldb] *= inv;
        else v[k] *= inv;
    }
    __syncthreads();
}

__device__ __noinline__ void blk_trsm_lt(const double *L, int ld, int n, double *B, int ldb, int nb, double *v) {
    const int tid = threadIdx.x, nc = nb + (v ? 1 : 0);
    for (int i = n - 1; i >= 0; --i) {
        __syncthreads();
        const int rows = i;  // k = 0 .. i - 1
        if (rows == 0) continue;
        const double inv = 1.0 / L[i + i * ld];
        for (int q = tid; q < rows * nc; q += BLK_THREADS) {
            const int k = q % rows, col = q / rows;
            const double lk = L[i + k * ld] * inv;  // L^T(k, i)
            if (col < nb) B[k + col * ldb] = __builtin_fma(-lk, B[i + col * ldb], B[k + col * ldb]);
            else v[k] = __builtin_fma(-lk, v[i], v[k]);
        }
    }
    __syncthreads();
    for (int q = tid; q < n * nc; q += BLK_THREADS) {
        const int k = q % n, col = q / n;
        const double inv = 1.0 / L[k + k * ld];
        if (col < nb) B[k + col * ldb] *= inv;
        else v[k] *= inv;
    }
    __syncthreads();
}

// Gauss-Jordan elimination with partial (row) pivoting of W = [A | R]
// (n x ncol, ld n; the LU form of the combine): the same pivot rows as
// PartialPivLU (largest |a| among the rows not yet used, lowest row on ties),
// kept in place.  On return row piv[k] of the right part holds row k of
// A^{-1} R.  prow: ncol doubles, mul: n doubles, piv: n ints of LDS scratch.
// False if a pivot is zero or not finite.
__device__ __noinline__ bool blk_gauss_jordan(double *W, int n, int *piv, double *prow, double *mul, int ncol) {
    const int tid = threadIdx.x, lane = tid & 63;
    bool used = false, ok = true;  // used: wave 0, lane = row
    for (int k = 0; k < n; ++k) {
        __syncthreads();
        if (tid < 64) {
            double v = (lane < n && !used) ? fabs(W[lane + k * n]) : -1.0;
            int arg = lane;
#pragma unroll
            for (int mk = 1; mk < 64; mk <<= 1) {
                const double ov = shfl_xor_f64(v, mk);
                const int oa = __shfl_xor(arg, mk, 64);
                if (ov > v || (ov == v && oa < arg)) {
                    v = ov;
                    arg = oa;
                }
            }
            used = used || (lane == arg);
            if (lane == 0) piv[k] = arg;
        }
        __syncthreads();
        const int p = piv[k];
        const double pv = W[p + k * n];
        ok = ok && pv != 0.0 && fabs(pv) <= 1.7976931348623157e308;
        const double inv = 1.0 / pv;
        for (int j = tid; j < ncol; j += BLK_THREADS) prow[j] = W[p + j * n];
        for (int i = tid; i < n; i += BLK_THREADS) mul[i] = W[i + k * n] * inv;
        __syncthreads();
        for (int q = tid; q < ncol * n; q += BLK_THREADS) {
            const int i = q % n, j = q / n;
            W[q] = (i == p) ? prow[j] * inv : __builtin_fma(-mul[i], prow[j], W[q]);
        }
    }
    __syncthreads();
    return ok;
}

}  // namespace pdplqr
