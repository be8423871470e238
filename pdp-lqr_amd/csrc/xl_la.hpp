// xl_la.hpp -- block-wide (256-thread) linear algebra on global-memory
// matrices of order up to 256 (the size-generic kernels_xl*.hip paths): the
// products by blk_mm on 64 x 64 output blocks, one barrier per pivot for the
// factorisations and triangular solves.  Every routine is bracketed by
// barriers, as blk_la.hpp's.
#pragma once
#include "blk_la.hpp"

namespace pdplqr {

constexpr int XL_S = 256;  // largest n + m of the XL paths

// C (M x N, ld ldc) = alpha A B + diag I + add over 64 x 64 output blocks
// (blk_mm per block; C must not alias A or B, add may be C itself).
// lower_blocks: only the blocks on or below the block diagonal (a symmetric
// update of which only the lower triangle is read)
__device__ __noinline__ void xl_mm(double *C, int ldc, const double *A, int lda, bool at, const double *B, int ldb,
                                   bool bt, int M, int N, int K, const double *add, int ldadd, double alpha = 1.0,
                                   double diag = 0.0, bool lower_blocks = false) {
    for (int j0 = 0; j0 < N; j0 += 64)
        for (int i0 = lower_blocks ? j0 : 0; i0 < M; i0 += 64) {
            const Mv av = at ? mv_t(A + (long long)i0 * lda, lda) : mv_n(A + i0, lda);
            const Mv bv = bt ? mv_t(B + j0, ldb) : mv_n(B + (long long)j0 * ldb, ldb);
            const Mv dv = add ? mv_n(add + i0 + (long long)j0 * ldadd, ldadd) : mv_none();
            blk_mm(C + i0 + (long long)j0 * ldc, ldc, av, bv, min(64, M - i0), min(64, N - j0), K, alpha,
                   i0 == j0 ? diag : 0.0, dv, false);
        }
}

// dst <- src (lower triangle of an n x n block, ld)
__device__ __noinline__ void xl_copy_lower(double *dst, const double *src, int ld, int n) {
    __syncthreads();
    for (int q = threadIdx.x; q < n * n; q += 256) {
        const int i = q % n, j = q / n;
        if (i >= j) dst[i + (long long)j * ld] = src[i + (long long)j * ld];
    }
    __syncthreads();
}

constexpr int XL_PW = 16;  // panel width of xl_llt

// Eigen's block size of llt_inplace<Lower>::blocked (Eigen/src/Cholesky/LLT.h)
// for order n; 0 below 32 (the unblocked form).  The oracle's llt_block_size.
__device__ __forceinline__ int xl_eigen_bs(int n) {
    if (n < 32) return 0;
    const int bs = (n / 8 / 16) * 16;
    return bs < 8 ? 8 : (bs > 128 ? 128 : bs);
}

// In-place blocked right-looking Cholesky of the lower triangle of A (n x n,
// ld) with Eigen's LLT stop: pivot j < m must be positive (else flagged and the
// factorisation goes on, as the tiled kernels do), a pivot j >= m that is not
// positive stops it, flagged only when psd_bad.  What the stop leaves is
// Eigen's: LLT::compute factors blocks of xl_eigen_bs(n) columns (the diagonal
// block A11 left-looking, then A21 <- A21 A11^{-T}, A22 -= A21 A21^T), so when
// pivot j in the block starting at k0 is not positive, the columns before k0
// hold L, A11's columns k0 .. j - 1 their factor (rows inside A11), and every
// other entry of the columns >= k0 the Schur complement of the columns < k0:
// recomputed from A0 (the input) as A0 - L(:, :k0) L(:, :k0)^T, with A11's
// factored columns kept (the oracle's llt_lower; below order 32 -- unblocked,
// k0 = j -- the input values from column j on).  Per panel of XL_PW columns: the panel (every row below
// its top) is factored in LDS, one barrier per pivot (the update with the raw
// pivot column a_ij a_lj / d_j, the columns scaled when written back), then
// the trailing lower triangle takes the panel's rank-XL_PW update on MFMA
// (xl_mm, lower blocks).  Entries above the diagonal may be overwritten.
// sinv: n doubles of LDS scratch.  Returns the block-uniform status.
__device__ __noinline__ bool xl_llt(double *A, int ld, int n, int m, const double *A0, double *sinv) {
    __shared__ double pan[XL_S * XL_PW];
    const int tid = threadIdx.x;
    bool ok = true;
    int jdead = n;
    for (int j0 = 0; j0 < n; j0 += XL_PW) {
        const int w = min(XL_PW, n - j0), rows = n - j0;
        __syncthreads();
        for (int q = tid; q < rows * w; q += 256) {
            const int i = q % rows, l = q / rows;
            if (i >= l) pan[i + l * XL_S] = A[(j0 + i) + (long long)(j0 + l) * ld];
        }
        int wl = w;  // live columns of the panel
        for (int jj = 0; jj < w; ++jj) {
            __syncthreads();
            const int j = j0 + jj;
            const double d = pan[jj + jj * XL_S];
            ok = ok && (j < m ? d > 0.0 : !psd_bad(d));
            if (!(j < m || d > 0.0)) {  // block-uniform
                jdead = j;
                wl = jj;
                break;
            }
            const double inv = 1.0 / d;
            if (tid == 0) sinv[j] = rsqrt_f64(d);
            const int r = rows - jj - 1, c = w - jj - 1;  // rows below the pivot, panel columns right of it
            for (int q = tid; q < r * c; q += 256) {
                const int i = jj + 1 + q % r, l = jj + 1 + q / r;
                if (l > i) continue;
                pan[i + l * XL_S] = __builtin_fma(-pan[i + jj * XL_S] * inv, pan[l + jj * XL_S], pan[i + l * XL_S]);
            }
        }
        __syncthreads();
        for (int q = tid; q < rows * wl; q += 256) {
            const int i = q % rows, l = q / rows;
            if (i >= l) A[(j0 + i) + (long long)(j0 + l) * ld] = pan[i + l * XL_S] * sinv[j0 + l];
        }
        if (jdead < n) break;  // block-uniform
        const int t = j0 + w;
        if (t < n) {  // trailing update A(t:, t:) -= L(t:, j0:t) L(t:, j0:t)^T
            double *Lp = A + t + (long long)j0 * ld, *Ct = A + t + (long long)t * ld;
            xl_mm(Ct, ld, Lp, ld, false, Lp, ld, true, n - t, n - t, w, Ct, ld, -1.0, 0.0, true);
        }
    }
    __syncthreads();
    if (jdead < n) {  // Eigen's stop (block-uniform, rare)
        const int bs = xl_eigen_bs(n);
        const int k0 = bs ? (jdead / bs) * bs : jdead, b = bs ? min(bs, n - k0) : 0;
        // A11's factored columns k0 .. jdead - 1 (rows k0 .. k0 + b - 1) aside
        for (int q = tid; q < b * b; q += 256) {
            const int i = q % b, l = q / b;
            if (k0 + l < jdead && i >= l) pan[i + l * XL_S] = A[(k0 + i) + (long long)(k0 + l) * ld];
        }
        __syncthreads();
        if (k0 > 0) {  // A(k0:, k0:) = A0(k0:, k0:) - L(k0:, :k0) L(k0:, :k0)^T (lower blocks)
            const double *Lp = A + k0;
            xl_mm(A + k0 + (long long)k0 * ld, ld, Lp, ld, false, Lp, ld, true, n - k0, n - k0, k0,
                  A0 + k0 + (long long)k0 * ld, ld, -1.0, 0.0, true);
        } else {
            xl_copy_lower(A, A0, ld, n);
        }
        __syncthreads();
        for (int q = tid; q < b * b; q += 256) {
            const int i = q % b, l = q / b;
            if (k0 + l < jdead && i >= l) A[(k0 + i) + (long long)(k0 + l) * ld] = pan[i + l * XL_S];
        }
        __syncthreads();
    }
    return ok;
}


// B (n x nb, ld ldb) <- L^{-1} B, L lower (ld): one barrier per pivot, the
// row updates spread over the block with the unscaled pivot row, the rows
// scaled at the end
__device__ __noinline__ void xl_fsub(const double *L, int ld, int n, double *B, int ldb, int nb) {
    const int tid = threadIdx.x;
    for (int j = 0; j < n; ++j) {
        __syncthreads();
        const double inv = 1.0 / L[j + (long long)j * ld];
        const int r = n - j - 1;
        for (int q = tid; q < r * nb; q += 256) {
            const int i = j + 1 + q % r, c = q / r;
            B[i + (long long)c * ldb] =
                __builtin_fma(-L[i + (long long)j * ld], B[j + (long long)c * ldb] * inv, B[i + (long long)c * ldb]);
        }
    }
    __syncthreads();
    for (int q = tid; q < n * nb; q += 256) {
        const int i = q % n, c = q / n;
        B[i + (long long)c * ldb] /= L[i + (long long)i * ld];
    }
    __syncthreads();
}

// B <- L^{-T} B (back substitution on L^T), the same scheme
__device__ __noinline__ void xl_bsub_t(const double *L, int ld, int n, double *B, int ldb, int nb) {
    const int tid = threadIdx.x;
    for (int j = n - 1; j >= 0; --j) {
        __syncthreads();
        const double inv = 1.0 / L[j + (long long)j * ld];
        for (int q = tid; q < j * nb; q += 256) {
            const int i = q % j, c = q / j;
            B[i + (long long)c * ldb] =
                __builtin_fma(-L[j + (long long)i * ld], B[j + (long long)c * ldb] * inv, B[i + (long long)c * ldb]);
        }
    }
    __syncthreads();
    for (int q = tid; q < n * nb; q += 256) {
        const int i = q % n, c = q / n;
        B[i + (long long)c * ldb] /= L[i + (long long)i * ld];
    }
    __syncthreads();
}

__device__ __noinline__ double xl_block_sum(double f, double *s_red) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) f += __shfl_xor(f, o, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = f;
    __syncthreads();
    return (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
}

// lu <- Luu^{-1} lu (rows < m of lp) and p = lp_x - Lxu lu (lp's x rows), L
// (s x s, ld): column-oriented forward substitution, one barrier per pivot --
// step j subtracts L(i, j) lu_j from every row below j (lp[j] itself is final
// before step j and divided by L(j, j) at the end), the same operation order
// per row as a row-by-row substitution.  pn: unused (kept for the callers).
__device__ __noinline__ void xl_solve_u(double *lp, const double *L, int ld, int m, int s, double *pn) {
    const int tid = threadIdx.x;
    (void)pn;
    for (int j = 0; j < m; ++j) {
        __syncthreads();
        const double xj = lp[j] / L[j + (long long)j * ld];
        for (int i = j + 1 + tid; i < s; i += 256) lp[i] = __builtin_fma(-L[i + (long long)j * ld], xj, lp[i]);
    }
    __syncthreads();
    for (int j = tid; j < m; j += 256) lp[j] /= L[j + (long long)j * ld];
    __syncthreads();
}

// In-place Cholesky with every pivot required positive (m = n; flagged
// otherwise) and zeros above the diagonal, blk_chol's output form for orders
// past 64
__device__ __noinline__ bool xl_chol(double *A, int ld, int n, double *sinv) {
    const bool ok = xl_llt(A, ld, n, n, A, sinv);
    for (int q = threadIdx.x; q < n * n; q += 256) {
        const int i = q % n, j = q / n;
        if (i < j) A[i + (long long)j * ld] = 0.0;
    }
    __syncthreads();
    return ok;
}

// blk_gauss_jordan for n <= 256: W = [A | R] (n x ncol, ld n) with partial
// (row) pivoting, the same pivot choice (largest |a| among the unused rows,
// lowest row on ties; thread i owns row i in the search), kept in place: row
// piv[k] of the right part holds row k of A^{-1} R on return.  prow: ncol,
// mul: n doubles, piv: n ints, red: 8 doubles + 8 ints of LDS scratch.
__device__ __noinline__ bool xl_gauss_jordan(double *W, int n, int *piv, double *prow, double *mul, int ncol,
                                             double *rv, int *ra) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    bool used = false, ok = true;  // thread tid: row tid
    for (int k = 0; k < n; ++k) {
        __syncthreads();
        double v = (tid < n && !used) ? fabs(W[tid + (long long)k * n]) : -1.0;
        int arg = tid;
#pragma unroll
        for (int mk = 1; mk < 64; mk <<= 1) {
            const double ov = shfl_xor_f64(v, mk);
            const int oa = __shfl_xor(arg, mk, 64);
            if (ov > v || (ov == v && oa < arg)) {
                v = ov;
                arg = oa;
            }
        }
        if (lane == 0) {
            rv[wv] = v;
            ra[wv] = arg;
        }
        __syncthreads();
        double bv = rv[0];
        int ba = ra[0];
        for (int w = 1; w < 4; ++w)
            if (rv[w] > bv || (rv[w] == bv && ra[w] < ba)) {
                bv = rv[w];
                ba = ra[w];
            }
        used = used || (tid == ba);
        if (tid == 0) piv[k] = ba;
        const int p = ba;
        const double pv = W[p + (long long)k * n];
        ok = ok && pv != 0.0 && fabs(pv) <= 1.7976931348623157e308;
        const double inv = 1.0 / pv;
        for (int j = tid; j < ncol; j += 256) prow[j] = W[p + (long long)j * n];
        for (int i = tid; i < n; i += 256) mul[i] = W[i + (long long)k * n] * inv;
        __syncthreads();
        for (int q = tid; q < ncol * n; q += 256) {
            const int i = q % n, j = q / n;
            W[q] = (i == p) ? prow[j] * inv : __builtin_fma(-mul[i], prow[j], W[q]);
        }
    }
    __syncthreads();
    return ok;
}

}  // namespace pdplqr
