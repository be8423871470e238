// kkt.hip -- QDLDLSolver on MI355X: the KKT system of kkt.hpp solved by a
// block LDL^T in QDLDL's elimination order.
//
// The reference (qdldl_solver.hpp:36-151, kkt.hpp:45-331) assembles the KKT
// matrix in the natural order [u0, x1,u1, ..., xN | y0, lambda1,y1, ...,
// lambdaN,yN] and factors it with QDLDL's up-looking LDL^T.  In that order
// every primal pivot comes first, so the factorisation is
//     K = [H  C^T; C  -Reg],   H = blockdiag(H_k + sigma I),
//     S = -Reg - C H^{-1} C^T  (the condensed dual system),
// and S is block tridiagonal over the dual groups [y0], [lambda_k; y_k]
// (group k couples to k +- 1 through the shared primal block z_k).  Only the
// y diagonal (-inv_rho, update_rho_vecs kkt.hpp:105-122) changes between
// factorisations, so the work splits into
//   k_kkt_stage  (once per model, parallel over (problem, stage)):
//                L_k = chol(H_k + sigma I), V_k = L_k^{-1} C_kk^T,
//                U_k = L_k^{-1} C_{k+1,k}^T and the dual blocks V^T V, U^T U, U^T V
//   k_kkt_factor (backward, serial over groups, one wave per problem):
//                block Cholesky of -S = Reg + C H^{-1} C^T
//   k_kkt_rhs    (update_problem_data, form_rhs kkt.hpp:224-300)
//   k_kkt_x0     (forward: update_rhs_initial_stage kkt.hpp:207-222, accumulating +=)
//   k_kkt_solve1/2/3 (forward, QDLDL_solve): w = L^{-1} r_p, dual condense,
//                block forward/back substitution on -S, z = L^{-T}(w - V lam - U lam+).
// Stage-0 state constraints are ignored by the KKT (kkt.hpp:218-221): C_00 has
// only the u columns of D_0 and x0 enters only through S0 x0 and A0 x0.
#include "combine_tiles.hpp"
#include "device_common.hpp"
#include "admm.hpp"
#include "solvers.hpp"

#include <algorithm>
#include <vector>

namespace pdplqr {

struct KKTArgs {
    Shape sh;
    int P;          // padded block size (16 or 32), leading dimension of every block
    int dim;        // KKT dimension per problem
    double sigma;   // frozen primal regularisation (kkt_sigma)
    double rho_dyn; // frozen dynamics regularisation
    const double *E, *c, *H, *h, *D;
    const int32_t *d_off, *y_off, *ncs;
    const int32_t *prim_off, *prim_dim, *dual_off, *gdim;
    double *blk;    // [b][N+1][6][P*P]: L, V, U, VtV, UtU, UtV
    double *fac;    // [b][N+1][3][P*P]: Lkk, L_{k+1,k} (P = 16: its transpose), Lkk^{-1} (P = 16)
    double *rhs;    // [b][dim]
    double *wv;     // [b][N+1][4][P]: w, t, t1, lam
    double *ppk;    // P = 16: H^{-1} (packed) and G^T per stage [b][N+1][2][256] (PPK)
    int32_t *status;
    int32_t *pstat;  // per problem: a primal block H_k + sigma I was not positive definite
};

// ---------------------------------------------------------------------------
// wave-level helpers on column-major blocks in LDS (leading dimension ld)
// ---------------------------------------------------------------------------
// C (r x c) (+)= alpha op(A) op(B), inner dimension kd
__device__ __forceinline__ void kgemm(double *C, int ldc, const double *A, int lda, bool tA, const double *B, int ldb,
                                      bool tB, int r, int c, int kd, double alpha, bool acc, int lane) {
    for (int idx = lane; idx < r * c; idx += 64) {
        const int i = idx % r, j = idx / r;
        double s = 0.0;
        for (int k = 0; k < kd; ++k) {
            const double a = tA ? A[k + i * lda] : A[i + k * lda];
            const double b = tB ? B[j + k * ldb] : B[k + j * ldb];
            s = __builtin_fma(a, b, s);
        }
        C[i + j * ldc] = (acc ? C[i + j * ldc] : 0.0) + alpha * s;
    }
}

// in-place lower Cholesky of the n x n block (upper part zeroed)
__device__ __forceinline__ bool kchol(double *A, int ld, int n, int lane) {
    bool ok = true;
    for (int j = 0; j < n; ++j) {
        const double d = A[j + j * ld];
        ok = ok && (d > 0.0);
        const double r = sqrt(d), ir = 1.0 / r;
        wave_sync();
        for (int i = j + 1 + lane; i < n; i += 64) A[i + j * ld] *= ir;
        if (lane == 0) A[j + j * ld] = r;
        wave_sync();
        const int t = n - j - 1;
        for (int q = lane; q < t * t; q += 64) {
            const int i = j + 1 + q % t, k = j + 1 + q / t;
            if (i >= k) A[i + k * ld] -= A[i + j * ld] * A[k + j * ld];
        }
        wave_sync();
    }
    for (int idx = lane; idx < n * n; idx += 64) {
        const int i = idx % n, j = idx / n;
        if (i < j) A[i + j * ld] = 0.0;
    }
    wave_sync();
    return ok;
}

// B (n x c) <- L^{-1} B, lanes over columns
__device__ __forceinline__ void ktrsm(const double *L, int ldl, double *B, int ldb, int n, int c, int lane) {
    for (int j = lane; j < c; j += 64)
        for (int i = 0; i < n; ++i) {
            double v = B[i + j * ldb];
            for (int k = 0; k < i; ++k) v -= L[i + k * ldl] * B[k + j * ldb];
            B[i + j * ldb] = v / L[i + i * ldl];
        }
}

// x (n) <- L^{-1} x or L^{-T} x, column-oriented with the lanes over rows
__device__ __forceinline__ void ktrsv(const double *L, int ldl, double *x, int n, bool trans, int lane) {
    if (!trans) {
        for (int j = 0; j < n; ++j) {
            const double xj = x[j] / L[j + j * ldl];
            wave_sync();
            if (lane == 0) x[j] = xj;
            for (int i = j + 1 + lane; i < n; i += 64) x[i] -= L[i + j * ldl] * xj;
            wave_sync();
        }
    } else {
        for (int j = n - 1; j >= 0; --j) {
            const double xj = x[j] / L[j + j * ldl];
            wave_sync();
            if (lane == 0) x[j] = xj;
            for (int i = lane; i < j; i += 64) x[i] -= L[j + i * ldl] * xj;  // (L^T)[i][j] = L[j][i]
            wave_sync();
        }
    }
}

__device__ __forceinline__ void kcopy_out(double *dst, const double *src, int n, int lane) {
    for (int q = lane; q < n; q += 64) dst[q] = src[q];
}

// reference column of KKT-ordered primal index a of stage k ((x, u) order
// for 0 < k < N; u for k = 0; x for k = N)
__device__ __forceinline__ int kref(int k, int N, int n, int m, int a) {
    if (k == 0 || k == N) return a;
    return a < n ? m + a : a - n;
}

// ---------------------------------------------------------------------------
// k_kkt_stage: primal factor and dual blocks of stage k (once per model)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_kkt_stage(KKTArgs A) {
    extern __shared__ double lds[];
    const int P = A.P, PP = P * P;
    double *L = lds, *V = lds + PP, *U = lds + 2 * PP, *T = lds + 3 * PP;
    const Shape &sh = A.sh;
    const int n = sh.n, m = sh.m, s = sh.s, N = sh.N, lane = wave_lane();
    const long long b = blockIdx.x / (N + 1);
    const int k = blockIdx.x % (N + 1);
    const int p = A.prim_dim[k], g = A.gdim[k], g1 = k < N ? A.gdim[k + 1] : 0;
    const int nck = A.ncs[k];
    const double *Hk = A.H + b * sh.perH + (long long)k * s * s;  // terminal: n x n at N s^2
    const int ldH = k < N ? s : n;
    const double *Ek = A.E + b * sh.perE + (long long)k * n * s;
    const double *Dk = A.D + b * sh.ndD + A.d_off[k];
    for (int q = lane; q < 4 * PP; q += 64) lds[q] = 0.0;
    wave_sync();
    for (int idx = lane; idx < p * p; idx += 64) {
        const int a = idx % p, c = idx / p;
        const double v = Hk[kref(k, N, n, m, a) + kref(k, N, n, m, c) * ldH];
        L[a + c * P] = (a == c) ? v + A.sigma : v;
    }
    // V <- C_kk^T (p x g), U <- C_{k+1,k}^T (p x g1)
    for (int idx = lane; idx < p * g; idx += 64) {
        const int a = idx % p, r = idx / p;
        double v;
        if (k == 0) v = Dk[r + a * nck];  // y0 rows: D0 u-columns
        else if (r < n) v = (a == r) ? -1.0 : 0.0;  // lambda_k rows: -x_k
        else v = Dk[(r - n) + kref(k, N, n, m, a) * nck];
        V[a + r * P] = v;
    }
    for (int idx = lane; idx < p * g1; idx += 64) {
        const int a = idx % p, r = idx / p;
        U[a + r * P] = (r < n) ? Ek[r + kref(k, N, n, m, a) * n] : 0.0;  // lambda_{k+1} rows: E_k
    }
    wave_sync();
    const bool ok = kchol(L, P, p, lane);
    ktrsm(L, P, V, P, p, g, lane);
    ktrsm(L, P, U, P, p, g1, lane);
    wave_sync();
    double *out = A.blk + (b * (N + 1) + k) * 6LL * PP;
    kcopy_out(out, L, PP, lane);
    kcopy_out(out + PP, V, PP, lane);
    kcopy_out(out + 2 * PP, U, PP, lane);
    kgemm(T, P, V, P, true, V, P, false, g, g, p, 1.0, false, lane);  // V^T V
    wave_sync();
    kcopy_out(out + 3 * PP, T, PP, lane);
    wave_sync();
    kgemm(T, P, U, P, true, U, P, false, g1, g1, p, 1.0, false, lane);  // U^T U
    wave_sync();
    kcopy_out(out + 4 * PP, T, PP, lane);
    wave_sync();
    for (int q = lane; q < PP; q += 64) T[q] = 0.0;
    wave_sync();
    kgemm(T, P, U, P, true, V, P, false, g1, g, p, 1.0, false, lane);  // U^T V
    wave_sync();
    kcopy_out(out + 5 * PP, T, PP, lane);
    if (!ok && lane == 0) A.pstat[b] = 1;  // primal block not positive definite
}

// ---------------------------------------------------------------------------
// k_kkt_factor: block Cholesky of -S (backward; QDLDL_factor's dual part)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_kkt_factor(KKTArgs A, const double *__restrict__ inv_rho) {
    extern __shared__ double lds[];
    const int P = A.P, PP = P * P;
    double *M = lds, *Lp = lds + PP, *X = lds + 2 * PP;
    const Shape &sh = A.sh;
    const int n = sh.n, N = sh.N, lane = wave_lane();
    const long long b = blockIdx.x;
    const double *ir = inv_rho + b * sh.ny;
    int fail = 0;
    for (int q = lane; q < 3 * PP; q += 64) lds[q] = 0.0;
    wave_sync();
    int gp = 0;
    for (int k = 0; k <= N; ++k) {
        const int g = A.gdim[k];
        const double *bk = A.blk + (b * (N + 1) + k) * 6LL * PP;
        const double *bp = A.blk + (b * (N + 1) + k - 1) * 6LL * PP;
        for (int idx = lane; idx < PP; idx += 64) {
            const int i = idx % P, j = idx / P;
            double v = 0.0;
            if (i < g && j < g) {
                v = bk[3 * PP + idx];
                if (k > 0) v += bp[4 * PP + idx];
                if (i == j) v += (k == 0) ? ir[A.y_off[0] + i] : (i < n ? A.rho_dyn : ir[A.y_off[k] + i - n]);
            }
            M[idx] = v;
        }
        wave_sync();
        if (k > 0) kgemm(M, P, Lp, P, false, Lp, P, true, g, g, gp, -1.0, true, lane);  // -= L_{k,k-1} L_{k,k-1}^T
        wave_sync();
        const bool ok = kchol(M, P, g, lane);
        if (!ok && !fail) fail = k + 1;
        double *fk = A.fac + (b * (N + 1) + k) * 3LL * PP;
        kcopy_out(fk, M, PP, lane);
        if (k < N) {
            const int g1 = A.gdim[k + 1];
            // L_{k+1,k} = (U^T V)_k Lkk^{-T}:  X = Lkk^{-1} (U^T V)^T  (g x g1), then transpose
            for (int idx = lane; idx < PP; idx += 64) {
                const int i = idx % P, j = idx / P;
                X[idx] = (i < g && j < g1) ? bk[5 * PP + j + i * P] : 0.0;
            }
            wave_sync();
            ktrsm(M, P, X, P, g, g1, lane);
            wave_sync();
            for (int idx = lane; idx < PP; idx += 64) {
                const int i = idx % P, j = idx / P;
                Lp[idx] = (i < g1 && j < g) ? X[j + i * P] : 0.0;
            }
            wave_sync();
            kcopy_out(fk + PP, Lp, PP, lane);
            wave_sync();
        }
        gp = g;
    }
    // status: first failing dual group + 1, or N + 2 when a primal block failed
    if (lane == 0) A.status[b] = fail ? fail : (A.pstat[b] ? N + 2 : 0);
}

// ---------------------------------------------------------------------------
// P = 16 (every primal and dual block fits one 16 x 16 MFMA tile, e.g. 12/4
// with nc <= 4): the same block Cholesky on registers.  X_k = L_{k,k-1}^T
// stays in C/D-layout registers from group to group:
//     M = D_k - X_k^T X_k                        (one MFMA product)
//     eliminate M's g pivots carrying [B^T | I]  (elim_regs, no LDS)
//     X_{k+1} = Lkk^{-1} (U^T V)_k^T, Lkk^{-1}
// Tiles in HBM use the tile-native order tn(i, j): lane (i & 3) 16 + j holds
// rows i = 4 r + (i & 3), r = i >> 2, as 4 contiguous doubles -- one 32-byte
// load per lane, 2 KB per tile, fully coalesced.
// ---------------------------------------------------------------------------
__device__ __forceinline__ d4 tn_load(const double *tile, int lane) {
    return *reinterpret_cast<const d4 *>(tile + 4 * lane);
}

__device__ __forceinline__ void tn_store(double *tile, int lane, const d4 &v) {
    *(__attribute__((address_space(1))) d4 *)(tile + 4 * lane) = v;
}

// Triangular tiles (L^{-1} lower, L^{-T} upper: exact zeros on the other side,
// the elimination that forms them only combines earlier rows) are stored
// packed in tile-native order: lane (g, c) keeps its nonzero rows r0..r1 (a
// contiguous range) at off.., lanes in order -- 136 doubles, so a solve reads
// 1,088 B per triangular tile instead of 2 KB.  With F(d) = sum_{j<d}
// (floor(j/4) + 1): lower (4r + g >= c) r0 = ceil((c - g)/4)+, off = sum_{g'<g}
// (64 - F(15 - g')) + 4c - F(c - g - 1)+; upper (4r + g <= c) r1 = floor((c - g)/4),
// off = sum_{g'<g} F(16 - g') + F(c - g)+.  Tile slots stay 256 doubles apart.
struct TriLane {
    int off, r0, r1;
};

__device__ __forceinline__ int tri_f(int d) {
    const int q = d >> 2, t = d & 3;
    return 2 * q * (q + 1) + t * (q + 1);
}

__device__ __forceinline__ TriLane tri_lane(int g, int c, bool upper) {
    TriLane t;
    int base = 0;
#pragma unroll
    for (int gg = 0; gg < 3; ++gg)
        if (gg < g) base += upper ? tri_f(16 - gg) : 64 - tri_f(15 - gg);
    if (!upper) {
        t.r0 = c > g ? (c - g + 3) >> 2 : 0;
        t.r1 = 3;
        t.off = base + 4 * c - tri_f(c > g ? c - g - 1 : 0);
    } else {
        t.r0 = 0;
        t.r1 = c >= g ? (c - g) >> 2 : -1;
        t.off = base + tri_f(c > g ? c - g : 0);
    }
    return t;
}

// branch-free: rows outside r0..r1 read a valid slot and are masked to 0.
// The raw / mask split lets a prefetching loop keep the raw values in its
// buffer and mask at the point of use (masking at the load makes the compiler
// wait for the load right there).
__device__ __forceinline__ d4 tri_load_raw(const double *tile, const TriLane &t) {
    d4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = tile[(r >= t.r0 && r <= t.r1) ? t.off + r - t.r0 : 0];
    return v;
}

__device__ __forceinline__ d4 tri_mask(const d4 &raw, const TriLane &t) {
    d4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = (r >= t.r0 && r <= t.r1) ? raw[r] : 0.0;
    return v;
}

__device__ __forceinline__ d4 tri_load(const double *tile, const TriLane &t) {
    return tri_mask(tri_load_raw(tile, t), t);
}

__device__ __forceinline__ void tri_store(double *tile, const TriLane &t, const d4 &v) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
        if (r >= t.r0 && r <= t.r1) tile[t.off + r - t.r0] = v[r];
}

// Symmetric tiles (H_k^{-1} = L^{-T} L^{-1}: an MFMA product X^T X sums the same
// products in the same order for (i, j) and (j, i), so it is exactly symmetric)
// are stored as their packed lower triangle; lane (g, c) reads row 4r + g of
// column c from its own lower slot or from the mirror (c, 4r + g), which lives
// in lane (c & 3, 4r + g), row c >> 2.  Indices per lane, once.
struct SymLane {
    int idx[4];
};

__device__ __forceinline__ SymLane sym_lane(int g, int c) {
    SymLane sl;
    const TriLane own = tri_lane(g, c, false);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = 4 * r + g;
        const TriLane mir = tri_lane(c & 3, i, false);
        sl.idx[r] = i >= c ? own.off + r - own.r0 : mir.off + (c >> 2) - mir.r0;
    }
    return sl;
}

__device__ __forceinline__ d4 sym_load(const double *tile, const SymLane &sl) {
    d4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = tile[sl.idx[r]];
    return v;
}

// P = 16 primal data of the parallel solve phases, ppk [b][N+1][2][256]:
//   slot 0: H_k^{-1} (symmetric, packed lower), slot 1: G_k^T, the coupling
//   columns of stage k's primal block -- column c < n: C_{k+1,k}^T (lambda_{k+1}:
//   E_k in KKT order), column n + j: the y_k column j of C_kk^T (D_k).  The
//   lambda_k columns of C_kk^T are -I on x_k and are applied implicitly.
// Then with z' = H^{-1} r_p:  t_k = C_kk z' = [-z'_x ; (G z')_y],
// t1_k = C_{k+1,k} z' = (G z')_lambda, and the back substitution is
// z = z' - H^{-1} (C_kk^T lam_k + C_{k+1,k}^T lam_{k+1}) = z' - H^{-1} (G^T q - [lam_k,x ; 0])
// with q = [lam_{k+1,lambda} ; lam_{k,y}].  3 KB of tiles per stage and phase
// instead of 4.5 (L^{-1} / L^{-T}, V, U).  Needs n + nc_0 <= 16 (kkt_init).
constexpr long long PPK = 512;  // doubles per stage

__device__ __forceinline__ d4 kkt_g_tile(const KKTArgs &A, long long b, int k, int g, int c) {
    const Shape &sh = A.sh;
    const int n = sh.n, m = sh.m, s = sh.s, N = sh.N;
    const int p = A.prim_dim[k], g1 = k < N ? A.gdim[k + 1] : 0, nck = A.ncs[k];
    const double *Ek = A.E + b * sh.perE + (long long)(k < N ? k : 0) * n * s;
    const double *Dk = A.D + b * sh.ndD + A.d_off[k];
    d4 G;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = 4 * r + g;  // primal index in KKT order
        double v = 0.0;
        if (i < p) {
            if (c < n) {
                if (c < g1) v = Ek[c + kref(k, N, n, m, i) * n];  // lambda_{k+1} rows: E_k
            } else if (c - n < nck) {
                v = k == 0 ? Dk[(c - n) + i * nck] : Dk[(c - n) + kref(k, N, n, m, i) * nck];  // y_k rows
            }
        }
        G[r] = v;
    }
    return G;
}

// C/D-layout transpose of a 16 x 16 tile through LDS (t: 16 x 17 doubles)
__device__ __forceinline__ d4 tile_transpose(const d4 &v, double *t, int g, int c) {
#pragma unroll
    for (int r = 0; r < 4; ++r) t[(4 * r + g) + 17 * c] = v[r];
    wave_sync();
    d4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = t[c + 17 * (4 * r + g)];
    wave_sync();
    return o;
}

// once per model, after k_kkt_stage: D_k = (V^T V)_k + (U^T U)_{k-1} + rho_dyn
// on the lambda diagonal (identity padding) and (U^T V)_k^T of every group in
// tile-native order: dpk [b][N+1][2][256]
__global__ __launch_bounds__(64) void k_kkt_pack16(KKTArgs A, double *__restrict__ dpk) {
    const Shape &sh = A.sh;
    const int N = sh.N, lane = wave_lane(), g = lane >> 4, c = lane & 15;
    const long long b = blockIdx.x / (N + 1);
    const int k = blockIdx.x % (N + 1);
    const int gk = A.gdim[k], g1 = k < N ? A.gdim[k + 1] : 0;
    const double *bk = A.blk + (b * (N + 1) + k) * 6LL * 256;
    const double *bp = bk - 6 * 256;
    d4 D, Bt;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = 4 * r + g;
        double v = (i == c) ? 1.0 : 0.0;
        if (i < gk && c < gk) {
            v = bk[3 * 256 + i + 16 * c] + (k > 0 ? bp[4 * 256 + i + 16 * c] : 0.0);
            if (i == c && k > 0 && i < sh.n) v += A.rho_dyn;  // lambda rows: -rho_dyn I (frozen)
        }
        D[r] = v;
        Bt[r] = (i < gk && c < g1) ? bk[5 * 256 + c + 16 * i] : 0.0;
    }
    double *o = dpk + (b * (N + 1) + k) * 512LL;
    tn_store(o, lane, D);
    tn_store(o + 256, lane, Bt);
    // primal data of the parallel solve phases (ppk, see PPK): H^{-1} and G^T.
    // L^{-1} by re-eliminating L L^T carrying I (identity padding past p).
    const int p = A.prim_dim[k];
    WM<1> Lt, M;
    wm_load<1>(Lt, bk, 16, p, true, 0.0, g, c);
    wm_tn<1>(M, Lt, Lt, p, 1.0, 0.0, (const WM<1> *)nullptr, g, c);  // L L^T
#pragma unroll
    for (int r = 0; r < 4; ++r)
        if (4 * r + g == c && c >= p) M.t[0][0][r] = 1.0;
    d4 Bi[1][1];
#pragma unroll
    for (int r = 0; r < 4; ++r) Bi[0][0][r] = (4 * r + g == c) ? 1.0 : 0.0;
    double colinv[1], rowinv[1][4];
    elim_regs<1, true, 1>(M, Bi, 16, colinv, rowinv, g, c);
    WM<1> Li, Hi;
#pragma unroll
    for (int r = 0; r < 4; ++r) Li.t[0][0][r] = Bi[0][0][r] * rowinv[0][r];  // L^{-1}
    wm_tn<1>(Hi, Li, Li, 16, 1.0, 0.0, (const WM<1> *)nullptr, g, c);      // H^{-1} = L^{-T} L^{-1}
    double *q = A.ppk + (b * (N + 1) + k) * PPK;
    tri_store(q, tri_lane(g, c, false), Hi.t[0][0]);  // symmetric: packed lower
    tn_store(q + 256, lane, kkt_g_tile(A, b, k, g, c));
}

// P = 16: the per-stage work of k_kkt_stage + the primal half of k_kkt_pack16
// on MFMA register tiles (one wave per (problem, stage), no LDS matrices):
//   L = chol(H_k + sigma I) with [C_kk^T | C_{k+1,k}^T | I] carried through the
//   blocked elimination (chol_blk4_aug): V = L^{-1} C_kk^T, U = L^{-1} C_{k+1,k}^T,
//   L^{-1} come out directly; V^T V, U^T U, U^T V are one MFMA product each.
// Writes the primal data ppk (H^{-1} = L^{-T} L^{-1}, G^T; see PPK) and the three
// dual blocks (tile-native, into blk's first three tiles) for k_kkt_pack16d,
// which adds the neighbour's U^T U.  The generic LDS kernel took 15.4 ms + 3.4 ms
// of packing per model at C5 (N = 512, batch 1024).
__global__ __launch_bounds__(64) void k_kkt_stage16(KKTArgs A) {
    const Shape &sh = A.sh;
    const int n = sh.n, m = sh.m, s = sh.s, N = sh.N, lane = wave_lane(), g = lane >> 4, c = lane & 15;
    const long long b = blockIdx.x / (N + 1);
    const int k = blockIdx.x % (N + 1);
    const int p = A.prim_dim[k], gk = A.gdim[k], g1 = k < N ? A.gdim[k + 1] : 0;
    const int nck = A.ncs[k];
    const double *Hk = A.H + b * sh.perH + (long long)k * s * s;
    const int ldH = k < N ? s : n;
    const double *Ek = A.E + b * sh.perE + (long long)(k < N ? k : 0) * n * s;
    const double *Dk = A.D + b * sh.ndD + A.d_off[k];
    d4 M, B[3];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = 4 * r + g;  // row (primal index in KKT order), column c
        double h = (i == c) ? 1.0 : 0.0, v = 0.0, u = 0.0;
        if (i < p && c < p) {
            h = Hk[kref(k, N, n, m, i) + kref(k, N, n, m, c) * ldH];
            if (i == c) h += A.sigma;
        }
        if (i < p && c < gk) {  // C_kk^T
            if (k == 0) v = Dk[c + i * nck];                       // y0 rows: D0 u-columns
            else if (c < n) v = (i == c) ? -1.0 : 0.0;             // lambda_k rows: -x_k
            else v = Dk[(c - n) + kref(k, N, n, m, i) * nck];      // y_k rows
        }
        if (i < p && c < g1 && c < n) u = Ek[c + kref(k, N, n, m, i) * n];  // lambda_{k+1} rows: E_k
        M[r] = h;
        B[0][r] = v;
        B[1][r] = u;
        B[2][r] = (i == c) ? 1.0 : 0.0;
    }
    const bool ok = chol_blk4_aug<3>(M, B, g, c);  // B <- L^{-1} B
    WM<1> V, U, VtV, UtU, UtV;
    V.t[0][0] = B[0];
    U.t[0][0] = B[1];
    wm_tn<1>(VtV, V, V, 16, 1.0, 0.0, (const WM<1> *)nullptr, g, c);
    wm_tn<1>(UtU, U, U, 16, 1.0, 0.0, (const WM<1> *)nullptr, g, c);
    wm_tn<1>(UtV, U, V, 16, 1.0, 0.0, (const WM<1> *)nullptr, g, c);
    WM<1> Li, Hi;
    Li.t[0][0] = B[2];
    wm_tn<1>(Hi, Li, Li, 16, 1.0, 0.0, (const WM<1> *)nullptr, g, c);  // H^{-1} = L^{-T} L^{-1}
    double *q = A.ppk + (b * (N + 1) + k) * PPK;
    tri_store(q, tri_lane(g, c, false), Hi.t[0][0]);  // symmetric: packed lower
    tn_store(q + 256, lane, kkt_g_tile(A, b, k, g, c));
    double *o = A.blk + (b * (N + 1) + k) * 6LL * 256;
    tn_store(o, lane, VtV.t[0][0]);
    tn_store(o + 256, lane, UtU.t[0][0]);
    tn_store(o + 512, lane, UtV.t[0][0]);
    if (!ok && lane == 0) A.pstat[b] = 1;  // primal block not positive definite
}

// P = 16, after k_kkt_stage16: D_k = (V^T V)_k + (U^T U)_{k-1} + rho_dyn on the
// lambda diagonal (identity padding) and (U^T V)_k^T, tile-native into dpk --
// k_kkt_pack16's dual half on the tile-native blocks
__global__ __launch_bounds__(64) void k_kkt_pack16d(KKTArgs A, double *__restrict__ dpk) {
    __shared__ double tt[16 * 17];
    const Shape &sh = A.sh;
    const int N = sh.N, lane = wave_lane(), g = lane >> 4, c = lane & 15;
    const long long b = blockIdx.x / (N + 1);
    const int k = blockIdx.x % (N + 1);
    const int gk = A.gdim[k];
    const double *o = A.blk + (b * (N + 1) + k) * 6LL * 256;
    d4 D = tn_load(o, lane);
    if (k > 0) {
        const d4 P = tn_load(o - 6 * 256 + 256, lane);  // (U^T U)_{k-1}
#pragma unroll
        for (int r = 0; r < 4; ++r) D[r] += P[r];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = 4 * r + g;
        if (i == c && k > 0 && i < sh.n) D[r] += A.rho_dyn;  // lambda rows: -rho_dyn I (frozen)
        if (!(i < gk && c < gk)) D[r] = (i == c) ? 1.0 : 0.0;
    }
    double *out = dpk + (b * (N + 1) + k) * 512LL;
    tn_store(out, lane, D);
    tn_store(out + 256, lane, tile_transpose(tn_load(o + 512, lane), tt, g, c));  // (U^T V)^T
}

// forward phase 1, P = 16 (parallel over stages): z' = H^{-1} r_p and, by one
// more single-column MFMA product, G z' -> t_k = C_kk z', t1_k = C_{k+1,k} z'
// (see PPK).  wv [b][N+1][64]: z' | t | t1 | lam.
__global__ __launch_bounds__(64) void k_kkt_solve1_16(KKTArgs A) {
    __shared__ double sz[16], so[16];
    const Shape &sh = A.sh;
    const int n = sh.n, N = sh.N, lane = wave_lane(), g = lane >> 4, c = lane & 15;
    const long long b = blockIdx.x / (N + 1);
    const int k = blockIdx.x % (N + 1);
    const int p = A.prim_dim[k];
    const double *q = A.ppk + (b * (N + 1) + k) * PPK;
    WM<1> Hi, Gt;
    Hi.t[0][0] = sym_load(q, sym_lane(g, c));
    Gt.t[0][0] = tn_load(q + 256, lane);
    const double *rp = A.rhs + b * A.dim + A.prim_off[k];
    WV<1> r, z, o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int i = 4 * j + g;
        r.t[0][j] = (c == 0 && i < p) ? rp[i] : 0.0;
    }
    wv_tn<1>(z, Hi, r, 16, 1.0, (const WV<1> *)nullptr);  // H^{-1} r (symmetric)
    wv_tn<1>(o, Gt, z, 16, 1.0, (const WV<1> *)nullptr);  // G z'
    wv_store<1>(z, sz, 16, g, c);
    wv_store<1>(o, so, 16, g, c);
    wave_sync();
    double *w = A.wv + (b * (N + 1) + k) * 64LL;
    if (lane < 16) {
        const int nck = A.ncs[k];
        double t;
        if (k == 0) t = lane < nck ? so[n + (lane < 16 - n ? lane : 0)] : 0.0;  // group 0 = y_0
        else t = lane < n ? -sz[lane] : so[lane];                             // [lambda_k ; y_k]
        w[lane] = sz[lane];
        w[16 + lane] = t;
        w[32 + lane] = lane < n ? so[lane] : 0.0;  // lambda_{k+1} part only
    }
}

// forward phase 3, P = 16 (parallel): z_k = z' - H^{-1} (G^T q - [lam_k,x ; 0]),
// q = [lam_{k+1} (lambda part) ; lam_k (y part)] (see PPK), unpacked into ws
__global__ __launch_bounds__(64) void k_kkt_solve3_16(KKTArgs A, const double *__restrict__ x0,
                                                      double *__restrict__ ws) {
    __shared__ double zs[16], qs[16];
    __shared__ double tt[16 * 17];
    const Shape &sh = A.sh;
    const int n = sh.n, m = sh.m, s = sh.s, N = sh.N, lane = wave_lane(), g = lane >> 4, c = lane & 15;
    const long long b = blockIdx.x / (N + 1);
    const int k = blockIdx.x % (N + 1);
    const double *q = A.ppk + (b * (N + 1) + k) * PPK;
    WM<1> Hi, G;
    Hi.t[0][0] = sym_load(q, sym_lane(g, c));
    G.t[0][0] = tile_transpose(tn_load(q + 256, lane), tt, g, c);
    const double *wk = A.wv + (b * (N + 1) + k) * 64LL;
    if (lane < 16) {
        const int nck = A.ncs[k];
        double v = 0.0;
        if (lane < n) v = k < N ? wk[64 + 48 + lane] : 0.0;  // lam_{k+1}, lambda part
        else if (lane - n < nck) v = wk[48 + (k == 0 ? lane - n : lane)];  // lam_k, y part
        qs[lane] = v;
    }
    wave_sync();
    WV<1> zp, lk, qv, sv, z;
    wv_load<1>(zp, wk, 16, g, c);
    wv_load<1>(lk, wk + 48, k == 0 ? 0 : n, g, c);  // lam_k, lambda part (x_k rows of -I)
    wv_load<1>(qv, qs, 16, g, c);
    wv_tn<1>(sv, G, qv, 16, 1.0, (const WV<1> *)nullptr);  // G^T q
#pragma unroll
    for (int r = 0; r < 4; ++r) sv.t[0][r] -= lk.t[0][r];
    wv_tn<1>(z, Hi, sv, 16, -1.0, &zp);  // z' - H^{-1} s
    wv_store<1>(z, zs, 16, g, c);
    wave_sync();
    double *wb = ws + b * sh.perh;
    if (k == 0) {  // ws[0] = [u0; x0] (qdldl_solver.hpp:133-134)
        if (lane < m) wb[lane] = zs[lane];
        else if (lane < s) wb[lane] = x0[b * n + lane - m];
    } else if (k < N) {
        if (lane < n) wb[(long long)k * s + m + lane] = zs[lane];
        else if (lane < s) wb[(long long)k * s + lane - n] = zs[lane];
    } else {
        if (lane < n) wb[(long long)N * s + lane] = zs[lane];
    }
}

// per backward: the y diagonal 1/rho of every group, dreg [b][N+1][16] (zero
// on lambda rows and padding), so the serial factor reads no index arrays
__global__ void k_kkt_dreg16(KKTArgs A, const double *__restrict__ inv_rho, double *__restrict__ dreg) {
    const Shape &sh = A.sh;
    const long long total = (long long)sh.batch * (sh.N + 1) * 16;
    for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (long long)gridDim.x * blockDim.x) {
        const int i = (int)(t & 15);
        const long long bk = t >> 4;
        const int k = (int)(bk % (sh.N + 1));
        const long long b = bk / (sh.N + 1);
        const int nl = k == 0 ? 0 : sh.n, gk = A.gdim[k];
        double v = 0.0;
        if (i >= nl && i < gk) v = inv_rho[b * sh.ny + A.y_off[k] + i - nl];
        dreg[t] = v;
    }
}

// per forward, after solve1: the dual right-hand side of the forward
// substitution, bvec [b][N+1][16] = -(r_d - t_k - t1_{k-1}) (zero padding)
__global__ void k_kkt_bvec16(KKTArgs A, double *__restrict__ bvec) {
    const Shape &sh = A.sh;
    const long long total = (long long)sh.batch * (sh.N + 1) * 16;
    for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (long long)gridDim.x * blockDim.x) {
        const int i = (int)(t & 15);
        const long long bk = t >> 4;
        const int k = (int)(bk % (sh.N + 1));
        const long long b = bk / (sh.N + 1);
        double v = 0.0;
        if (i < A.gdim[k]) {
            const double *w = A.wv + bk * 64;
            const double t1 = k > 0 ? w[-64 + 32 + i] : 0.0;
            v = -(A.rhs[b * A.dim + A.dual_off[k] + i] - w[16 + i] - t1);
        }
        bvec[t] = v;
    }
}

// Every group is eliminated over all 16 pivots: the padding is the identity
// (exact no-op pivots) and X's padding is zero, so the loop reads no group
// dimensions -- only two tiles and the y diagonal, loaded two groups ahead.
// PDPLQR_KKT_BLK4: the per-group factorisation as 4-pivot blocks with MFMA
// trailing updates (chol_blk4_aug) instead of 16 single pivots (elim_regs).



// ---------------------------------------------------------------------------
// P = 16, two waves per problem: the TWISTED block factorisation of -S.
// The serial chain above walks all N + 1 dual groups with one wave per problem
// (one wave per SIMD at C5's batch 1024: latency-bound).  Here wave 0
// eliminates groups 0 .. p-1 top-down (the natural-order chain) and wave 1
// eliminates groups N .. p+1 bottom-up (the same recursion on the reversed
// system, whose coupling block is Bt_{k-1}^T):
//     M'_k = D_k - Z_k^T Z_k,  L'_kk = chol(M'_k),  Z_{k-1} = L'_kk^{-1} Bt_{k-1}^T
// and the middle group p = N / 2 takes both sides' Schur complements:
//     M_p = D_p - X_p^T X_p - Z_p^T Z_p.
// The factor is a different (twisted) elimination order of the same SPD
// matrix, so the solution agrees with QDLDL's natural order to rounding.  Each
// wave's chain is half as long and two waves share a SIMD.  Storage: group
// k < p as before (X_{k+1}, Lkk^{-1}); group k > p: Z_{k-1} at +256,
// L'_kk^{-1} at +512; group p: L_pp^{-1} at +512.
// ---------------------------------------------------------------------------

__device__ __forceinline__ d4 tile_identity(int g, int c) {
    d4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = (4 * r + g == c) ? 1.0 : 0.0;
    return v;
}

// Inputs of step i of a sweep are loaded two steps ahead into one of two
// buffers used alternately (a 2x-unrolled loop: no register rotation, which
// made the compiler wait for the freshly issued loads at every back edge).
struct SolveIn {
    d4 X, L;
    WV<1> v;
};

struct FacIn {
    d4 D, B;
    double dr[4];
};

// Branch-free store of a column-0 vector (lane (g, 0) holds entries 4r + g):
// every lane of a row group stores the same value to the same address.  A
// lane-predicated store is an exec-masked branch, and the compiler's wait-count
// merge after it drains every load in flight -- the sweeps' prefetch.
__device__ __forceinline__ void wv_store_rows(const WV<1> &v, double *p, int g) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const double x = bcast_lane16(v.t[0][r], 0);
        p[4 * r + g] = x;
    }
}

// A scheduling barrier after each load group keeps the loads where they are
// written (the machine scheduler would otherwise sink them towards their use,
// shortening the prefetch distance).
__device__ __forceinline__ void sweep_fence() {
    __builtin_amdgcn_sched_barrier(0);
}

template <class In, class LD, class ST>
__device__ __forceinline__ void sweep2(int cnt, LD &&ld, ST &&step) {
    if (cnt <= 0) return;
    In a, b;
    ld(a, 0);
    ld(b, min(1, cnt - 1));
    int i = 0;
    for (; i + 1 < cnt; i += 2) {
        step(a, i);
        sweep_fence();
        ld(a, min(i + 2, cnt - 1));  // past the end: re-loads the last step (harmless)
        sweep_fence();
        step(b, i + 1);
        sweep_fence();
        ld(b, min(i + 3, cnt - 1));
        sweep_fence();
    }
    if (i < cnt) step(a, i);
}

__global__ __launch_bounds__(128) void k_kkt_factor16_tw(KKTArgs A, const double *__restrict__ dpk,
                                                        const double *__restrict__ dreg) {
    __shared__ double tt[16 * 17];            // wave 1's transposes
    __shared__ __attribute__((aligned(32))) double zmid[256];  // Z_p, C/D layout per lane
    __shared__ int wfail[2];
    const Shape &sh = A.sh;
    const int N = sh.N, p = N / 2;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
    const TriLane tl = tri_lane(g, c, false);  // packed L^{-1} tiles
    __builtin_assume(lane >= 0 && lane < 64);
    const long long b = blockIdx.x;
    const double *tiles = dpk + b * (N + 1) * 512LL;
    const double *dg = dreg + b * (N + 1) * 16LL;
    double *fb = A.fac + b * (N + 1) * 3LL * 256;
    int fail = 0;  // 1 + the lowest failing group
    WM<1> X;       // wave 0: X_k = L_{k,k-1}^T; wave 1: Z_k
    X.t[0][0] = d4{0.0, 0.0, 0.0, 0.0};
    auto load_D = [&](int k) {
        d4 D = tn_load(tiles + k * 512LL, lane);
#pragma unroll
        for (int r = 0; r < 4; ++r) D[r] += (4 * r + g == c) ? dg[k * 16 + 4 * r + g] : 0.0;
        return D;
    };
    // group k's inputs: D_k (tile-native) with the y diagonal dreg_k, and the
    // coupling tile Bt_{kb} (kb = k top-down, k - 1 bottom-up)
    auto fload = [&](FacIn &in, int k, int kb) {
        in.D = tn_load(tiles + k * 512LL, lane);
        in.B = tn_load(tiles + kb * 512LL + 256, lane);
#pragma unroll
        for (int r = 0; r < 4; ++r) in.dr[r] = dg[k * 16 + 4 * r + g];
    };
    auto fstep = [&](const FacIn &in, int k, bool first, bool bottom) {
        WM<1> M, D;
        d4 B[2];
        D.t[0][0] = in.D;
#pragma unroll
        for (int r = 0; r < 4; ++r) D.t[0][0][r] += (4 * r + g == c) ? in.dr[r] : 0.0;
        B[0] = bottom ? tile_transpose(in.B, tt, g, c) : in.B;  // Bt_{k-1}^T bottom-up
        if (!first) wm_tn<1>(M, X, X, 16, -1.0, 0.0, &D, g, c);  // D_k - X_k^T X_k (Z_k^T Z_k)
        else M = D;
        B[1] = tile_identity(g, c);
        const bool ok = chol_blk4_aug<2>(M.t[0][0], B, g, c);
        if (!ok && (bottom || !fail)) fail = k + 1;  // bottom-up: the last one is the lowest
        X.t[0][0] = B[0];
        double *fk = fb + k * 768LL;
        // X_{k+1} (top) / Z_{k-1} (bottom).  X = Lkk^{-1} (U^T V)_k^T keeps the
        // zero columns c >= n of (U^T V)^T (U's y columns): those lanes store nothing
        // block LDL^T form for the solve (k_kkt_solve2_16_tw): T = Lkk^{-T} X
        // (= M^{-1} Bt_k top-down, M'^{-1} Bt_{k-1}^T bottom-up; the top chain's
        // keeps the zero columns c >= n), and Lkk^{-1} (packed): the solve forms
        // M^{-1} z = Lkk^{-T} Lkk^{-1} z itself (one product less in this chain)
        WM<1> Li, Xc, Tm;
        Li.t[0][0] = B[1];
        Xc.t[0][0] = B[0];
        wm_tn<1>(Tm, Li, Xc, 16, 1.0, 0.0, (const WM<1> *)nullptr, g, c);
        if (bottom || c < sh.n) tn_store(fk + 256, lane, Tm.t[0][0]);
        tri_store(fk + 512, tl, B[1]);  // Lkk^{-1} / L'_kk^{-1}, packed
    };
    if (wv == 0) {
        sweep2<FacIn>(p, [&](FacIn &in, int i) { fload(in, i, i); },
                      [&](const FacIn &in, int i) { fstep(in, i, i == 0, false); });
    } else {
        sweep2<FacIn>(N - p, [&](FacIn &in, int i) { fload(in, N - i, N - i - 1); },
                      [&](const FacIn &in, int i) { fstep(in, N - i, i == 0, true); });
        *reinterpret_cast<d4 *>(zmid + 4 * lane) = X.t[0][0];  // Z_p
    }
    if (lane == 0) wfail[wv] = fail;
    __syncthreads();
    if (wv == 0) {
        WM<1> Z, M, M1, D;
        Z.t[0][0] = *reinterpret_cast<const d4 *>(zmid + 4 * lane);
        D.t[0][0] = load_D(p);
        if (p > 0) {
            wm_tn<1>(M1, X, X, 16, -1.0, 0.0, &D, g, c);
            wm_tn<1>(M, Z, Z, 16, -1.0, 0.0, &M1, g, c);  // D_p - X_p^T X_p - Z_p^T Z_p
        } else {
            wm_tn<1>(M, Z, Z, 16, -1.0, 0.0, &D, g, c);
        }
        d4 B[2];
        B[0] = d4{0.0, 0.0, 0.0, 0.0};
        B[1] = tile_identity(g, c);
        const bool ok = chol_blk4_aug<2>(M.t[0][0], B, g, c);
        tri_store(fb + p * 768LL + 512, tl, B[1]);  // L_pp^{-1}, packed
        int f = fail;
        if (!ok && (!f || p + 1 < f)) f = p + 1;
        if (wfail[1] && (!f || wfail[1] < f)) f = wfail[1];
        if (lane == 0) A.status[b] = f ? f : (A.pstat[b] ? N + 2 : 0);
    }
}

// forward phase 2 on the twisted factor: L y = bvec from both ends toward the
// middle group, its 16 x 16 solve, then L^T lam = y outward (two waves)
__global__ __launch_bounds__(128) void k_kkt_solve2_16_tw(KKTArgs A, const double *__restrict__ bvec) {
    __shared__ double tt[2][16 * 17];
    __shared__ double vmid[16], lmid[16];
    const Shape &sh = A.sh;
    const int N = sh.N, p = N / 2;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
    const TriLane tl = tri_lane(g, c, false);  // packed Lkk^{-1} tiles
    __builtin_assume(lane >= 0 && lane < 64);
    const long long b = blockIdx.x;
    double *wvb = A.wv + b * (N + 1) * 4LL * 16;
    const double *fb = A.fac + b * (N + 1) * 3LL * 256;
    const double *bv = bvec + b * (N + 1) * 16LL;
    double *T = tt[wv];
    auto vin_raw = [&](const double *src) {  // a 16-vector, row 4 r + g in every lane (branch-free)
        WV<1> v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v.t[0][r] = src[4 * r + g];
        return v;
    };
    auto vmask = [&](const WV<1> &raw) {  // column 0 keeps it
        WV<1> v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v.t[0][r] = (c == 0) ? raw.t[0][r] : 0.0;
        return v;
    };
    auto vin = [&](const double *src) { return vmask(vin_raw(src)); };
    // raw loads into the prefetch buffer; the masks are applied in the step.
    // Wave 0 reads T tiles with zero, unstored columns c >= n, wave 1 full T'
    // tiles; lanes c >= n of wave 0 re-read lane (g, n - 1)'s slot, a cache
    // line fetched anyway (branch-free: a masked load would drain the prefetch
    // at the merge).  The forward sweep needs no M^{-1}.
    const bool xcol = wv == 1 || c < sh.n;
    const int xl = xcol ? lane : (lane & 48) + sh.n - 1;
    auto xmask = [&](const d4 &x) { return xcol ? x : d4{0.0, 0.0, 0.0, 0.0}; };
    auto fload = [&](SolveIn &in, long long toff, const double *vsrc) {
        in.X = tn_load(fb + toff, xl);
        in.v = vin_raw(vsrc);
    };
    auto bload = [&](SolveIn &in, int k) {
        in.X = tn_load(fb + k * 768LL + 256, xl);
        in.L = tri_load_raw(fb + k * 768LL + 512, tl);
        in.v = vin_raw(wvb + (long long)k * 64 + 48);
    };
    WV<1> z;
    z.t[0] = d4{0.0, 0.0, 0.0, 0.0};
    // forward step: z_k = bvec_k - T^T z_prev, T = T_{k-1} (top) or T'_{k+1} (bottom)
    auto fstep = [&](const SolveIn &in, int k, bool first) {
        WV<1> v = vmask(in.v);
        if (!first) {
            WM<1> Tk;
            Tk.t[0][0] = xmask(in.X);
            wv_tn<1>(v, Tk, z, 16, -1.0, &v);
        }
        z = v;
        wv_store_rows(z, wvb + (long long)k * 64 + 48, g);
    };
    // ---- forward substitution from both ends ----
    if (wv == 0) {  // steps k = 0 .. p-1: T_{k-1} stored by group k - 1
        sweep2<SolveIn>(p, [&](SolveIn &in, int i) { fload(in, max(i - 1, 0) * 768LL + 256, bv + i * 16); },
               [&](const SolveIn &in, int i) { fstep(in, i, i == 0); });
    } else {  // steps k = N .. p+1: T'_{k+1} stored by group k + 1
        sweep2<SolveIn>(N - p,
               [&](SolveIn &in, int i) {
                   const int k = N - i;
                   fload(in, min(k + 1, N) * 768LL + 256, bv + k * 16);
               },
               [&](const SolveIn &in, int i) { fstep(in, N - i, i == 0); });
        wv_store<1>(z, vmid, 16, g, c);  // z'_{p+1}
    }
    __syncthreads();
    // ---- the middle group: z_p = bvec_p - T_{p-1}^T z_{p-1} - T'_{p+1}^T z'_{p+1}, lam_p = M_p^{-1} z_p ----
    if (wv == 0) {
        WV<1> v = vin(bv + p * 16);
        if (p > 0) {
            WM<1> Tp;
            Tp.t[0][0] = d4{0.0, 0.0, 0.0, 0.0};
            if (c < sh.n) Tp.t[0][0] = tn_load(fb + (p - 1) * 768LL + 256, lane);
            wv_tn<1>(v, Tp, z, 16, -1.0, &v);
        }
        WM<1> Tq;
        Tq.t[0][0] = tn_load(fb + (p + 1) * 768LL + 256, lane);
        const WV<1> zb = vin(vmid);
        wv_tn<1>(v, Tq, zb, 16, -1.0, &v);
        WM<1> Linv, LinvT;
        Linv.t[0][0] = tri_load(fb + p * 768LL + 512, tl);
        LinvT.t[0][0] = tile_transpose(Linv.t[0][0], T, g, c);
        WV<1> yp, lam;
        wv_tn<1>(yp, LinvT, v, 16, 1.0, (const WV<1> *)nullptr);
        wv_tn<1>(lam, Linv, yp, 16, 1.0, (const WV<1> *)nullptr);  // M_p^{-1} z_p
        wv_store<1>(lam, wvb + (long long)p * 64 + 48, 16, g, c);
        wv_store<1>(lam, lmid, 16, g, c);
    }
    __syncthreads();
    // ---- back substitution outward; z_k was written by this wave (same rows) ----
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    WV<1> lam = vin(lmid);
    // step k: lam_k = M_k^{-1} z_k - T lam_prev, T = T_k (top) or T'_k (bottom),
    // both stored by group k; M^{-1} z_k = Lkk^{-T} Lkk^{-1} z_k does not wait for lam_prev
    auto bstep = [&](const SolveIn &in, int k) {
        WM<1> TT, Linv, LinvT;
        Linv.t[0][0] = tri_mask(in.L, tl);
        LinvT.t[0][0] = tile_transpose(Linv.t[0][0], T, g, c);
        WV<1> y, w;
        wv_tn<1>(y, LinvT, vmask(in.v), 16, 1.0, (const WV<1> *)nullptr);  // Lkk^{-1} z_k
        wv_tn<1>(w, Linv, y, 16, 1.0, (const WV<1> *)nullptr);             // M_k^{-1} z_k
        TT.t[0][0] = tile_transpose(xmask(in.X), T, g, c);
        wv_tn<1>(lam, TT, lam, 16, -1.0, &w);
        wv_store_rows(lam, wvb + (long long)k * 64 + 48, g);
    };
    if (wv == 0)
        sweep2<SolveIn>(p, [&](SolveIn &in, int i) { bload(in, p - 1 - i); },
               [&](const SolveIn &in, int i) { bstep(in, p - 1 - i); });
    else
        sweep2<SolveIn>(N - p, [&](SolveIn &in, int i) { bload(in, p + 1 + i); },
               [&](const SolveIn &in, int i) { bstep(in, p + 1 + i); });
}

// ---------------------------------------------------------------------------
// k_kkt_rhs: form_rhs (kkt.hpp:224-300) -- one thread per (problem, KKT row)
// row descriptors: kind 0 = primal (stage, KKT index), 1 = y (stage, q),
// 2 = lambda_{k+1} (k, i)
// ---------------------------------------------------------------------------
__global__ void k_kkt_rhs(KKTArgs A, const int4 *__restrict__ rows, const double *__restrict__ ws,
                          const double *__restrict__ ys, const double *__restrict__ zs,
                          const double *__restrict__ irho, double sigma) {
    const Shape &sh = A.sh;
    const long long total = (long long)A.dim * sh.batch;
    for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (long long)gridDim.x * blockDim.x) {
        const long long b = t / A.dim;
        const int r = (int)(t - b * A.dim);
        const int4 d = rows[r];
        double v;
        if (d.x == 0) {
            const long long o = b * sh.perh + (long long)d.y * sh.s + kref(d.y, sh.N, sh.n, sh.m, d.z);
            v = -A.h[o] + sigma * ws[o];
        } else if (d.x == 1) {
            const long long o = b * sh.ny + A.y_off[d.y] + d.z;
            v = zs[o] - irho[o] * ys[o];
        } else {
            v = -A.c[b * sh.perc + (long long)d.y * sh.n + d.z];
        }
        A.rhs[b * A.dim + r] = v;
    }
}

// update_rhs_initial_stage (kkt.hpp:207-222): rhs_u0 += -S0 x0, rhs_lambda1 += -A0 x0
__global__ __launch_bounds__(64) void k_kkt_x0(KKTArgs A, const double *__restrict__ x0) {
    const Shape &sh = A.sh;
    const int n = sh.n, m = sh.m, s = sh.s, lane = wave_lane();
    const long long b = blockIdx.x;
    const double *H0 = A.H + b * sh.perH, *E0 = A.E + b * sh.perE, *x = x0 + b * n;
    double *r = A.rhs + b * A.dim;
    if (lane < m) {
        double a = 0.0;
        for (int j = 0; j < n; ++j) a += H0[lane + (m + j) * s] * x[j];
        r[lane] += -a;
    } else if (lane >= 32 && lane - 32 < n) {
        const int i = lane - 32;
        double a = 0.0;
        for (int j = 0; j < n; ++j) a += E0[i + (m + j) * n] * x[j];
        r[A.dual_off[1] + i] += -a;
    }
}

// forward phase 1 (parallel over stages): w = L^{-1} r_p, t = V^T w, t1 = U^T w
__global__ __launch_bounds__(64) void k_kkt_solve1(KKTArgs A) {
    extern __shared__ double lds[];
    const int P = A.P, PP = P * P;
    double *L = lds, *w = lds + PP;
    const Shape &sh = A.sh;
    const int N = sh.N, lane = wave_lane();
    const long long b = blockIdx.x / (N + 1);
    const int k = blockIdx.x % (N + 1);
    const int p = A.prim_dim[k], g = A.gdim[k], g1 = k < N ? A.gdim[k + 1] : 0;
    const double *bk = A.blk + (b * (N + 1) + k) * 6LL * PP;
    for (int q = lane; q < PP; q += 64) L[q] = bk[q];
    const double *r = A.rhs + b * A.dim + A.prim_off[k];
    for (int q = lane; q < P; q += 64) w[q] = q < p ? r[q] : 0.0;
    wave_sync();
    ktrsv(L, P, w, p, false, lane);
    double *o = A.wv + (b * (N + 1) + k) * 4LL * P;
    for (int j = lane; j < P; j += 64) {
        double t = 0.0, t1 = 0.0;
        for (int a = 0; a < p; ++a) {
            t = __builtin_fma(bk[PP + a + j * P], w[a], t);        // V^T w
            t1 = __builtin_fma(bk[2 * PP + a + j * P], w[a], t1);  // U^T w
        }
        o[j] = w[j];
        o[P + j] = j < g ? t : 0.0;
        o[2 * P + j] = j < g1 ? t1 : 0.0;
    }
}

// forward phase 2 (serial over groups): (-S) lam = -(r_d - C H^{-1} r_p)
__global__ __launch_bounds__(64) void k_kkt_solve2(KKTArgs A) {
    extern __shared__ double lds[];
    const int P = A.P, PP = P * P;
    double *Lk = lds, *Lo = lds + PP, *v = lds + 2 * PP, *yp = v + P;
    const Shape &sh = A.sh;
    const int N = sh.N, lane = wave_lane();
    const long long b = blockIdx.x;
    const double *rd = A.rhs + b * A.dim;
    double *wvb = A.wv + b * (N + 1) * 4LL * P;
    const double *fb = A.fac + b * (N + 1) * 3LL * PP;
    for (int q = lane; q < P; q += 64) yp[q] = 0.0;
    wave_sync();
    for (int k = 0; k <= N; ++k) {  // L y = b
        const int g = A.gdim[k];
        for (int q = lane; q < PP; q += 64) {
            Lk[q] = fb[(long long)k * 3 * PP + q];
            Lo[q] = k > 0 ? fb[(long long)(k - 1) * 3 * PP + PP + q] : 0.0;  // L_{k,k-1}
        }
        wave_sync();
        for (int i = lane; i < P; i += 64) {
            double bi = 0.0;
            if (i < g) {
                const double t1 = k > 0 ? wvb[(long long)(k - 1) * 4 * P + 2 * P + i] : 0.0;
                bi = -(rd[A.dual_off[k] + i] - wvb[(long long)k * 4 * P + P + i] - t1);
                if (k > 0)
                    for (int j = 0; j < P; ++j) bi -= Lo[i + j * P] * yp[j];
            }
            v[i] = bi;
        }
        wave_sync();
        ktrsv(Lk, P, v, g, false, lane);
        for (int i = lane; i < P; i += 64) {
            wvb[(long long)k * 4 * P + 3 * P + i] = v[i];
            yp[i] = v[i];
        }
        wave_sync();
    }
    for (int q = lane; q < P; q += 64) yp[q] = 0.0;
    wave_sync();
    for (int k = N; k >= 0; --k) {  // L^T lam = y
        const int g = A.gdim[k];
        for (int q = lane; q < PP; q += 64) {
            Lk[q] = fb[(long long)k * 3 * PP + q];
            Lo[q] = k < N ? fb[(long long)k * 3 * PP + PP + q] : 0.0;  // L_{k+1,k}
        }
        wave_sync();
        for (int i = lane; i < P; i += 64) {
            double vi = 0.0;
            if (i < g) {
                vi = wvb[(long long)k * 4 * P + 3 * P + i];
                if (k < N)
                    for (int j = 0; j < P; ++j) vi -= Lo[j + i * P] * yp[j];  // (L_{k+1,k}^T lam_{k+1})_i
            }
            v[i] = vi;
        }
        wave_sync();
        ktrsv(Lk, P, v, g, true, lane);
        for (int i = lane; i < P; i += 64) {
            wvb[(long long)k * 4 * P + 3 * P + i] = v[i];
            yp[i] = v[i];
        }
        wave_sync();
    }
}

// forward phase 3 (parallel): z_k = L^{-T}(w - V lam_k - U lam_{k+1}), unpacked into ws
__global__ __launch_bounds__(64) void k_kkt_solve3(KKTArgs A, const double *__restrict__ x0, double *__restrict__ ws) {
    extern __shared__ double lds[];
    const int P = A.P, PP = P * P;
    double *L = lds, *z = lds + PP;
    const Shape &sh = A.sh;
    const int n = sh.n, m = sh.m, s = sh.s, N = sh.N, lane = wave_lane();
    const long long b = blockIdx.x / (N + 1);
    const int k = blockIdx.x % (N + 1);
    const int p = A.prim_dim[k], g = A.gdim[k], g1 = k < N ? A.gdim[k + 1] : 0;
    const double *bk = A.blk + (b * (N + 1) + k) * 6LL * PP;
    const double *wk = A.wv + (b * (N + 1) + k) * 4LL * P;
    const double *wn = wk + 4LL * P;  // stage k+1 (lam_{k+1})
    for (int q = lane; q < PP; q += 64) L[q] = bk[q];
    for (int a = lane; a < P; a += 64) {
        double v = 0.0;
        if (a < p) {
            v = wk[a];
            for (int j = 0; j < g; ++j) v -= bk[PP + a + j * P] * wk[3 * P + j];
            for (int j = 0; j < g1; ++j) v -= bk[2 * PP + a + j * P] * wn[3 * P + j];
        }
        z[a] = v;
    }
    wave_sync();
    ktrsv(L, P, z, p, true, lane);
    double *wb = ws + b * sh.perh;
    if (k == 0) {  // ws[0] = [u0; x0] (qdldl_solver.hpp:133-134)
        if (lane < m) wb[lane] = z[lane];
        else if (lane < s) wb[lane] = x0[b * n + lane - m];
    } else if (k < N) {
        if (lane < n) wb[(long long)k * s + m + lane] = z[lane];
        else if (lane < s) wb[(long long)k * s + lane - n] = z[lane];
    } else {
        if (lane < n) wb[(long long)N * s + lane] = z[lane];
    }
}

// ---------------------------------------------------------------------------
// host state
// ---------------------------------------------------------------------------
struct KKTState {
    int P = 16, dim = 0;
    std::vector<int32_t> prim_off, prim_dim, dual_off, gdim;
    int32_t *d_prim_off = nullptr, *d_prim_dim = nullptr, *d_dual_off = nullptr, *d_gdim = nullptr, *d_ncs = nullptr;
    int4 *rows = nullptr;
    int32_t *pstat = nullptr;
    double *blk = nullptr, *fac = nullptr, *rhs = nullptr, *wv = nullptr;
    double *dpk = nullptr;   // P = 16: D_k and (U^T V)_k^T tiles, tile-native [b][N+1][2][256]
    double *dreg = nullptr;  // P = 16: y diagonal per group [b][N+1][16]
    double *bvec = nullptr;  // P = 16: forward-substitution right-hand sides [b][N+1][16]
    double *ppk = nullptr;   // P = 16: H^{-1} (packed) and G^T per stage [b][N+1][2][256]
    bool formed = false;
    // Riccati-ordered elimination (kkt_riccati.hip): the uniform row count nc,
    // or -1 where the block LDL^T kernels below run
    int ric = -1;
    double *rec = nullptr;    // rollout records [b][N][FS]
    double *x0acc = nullptr;  // sum of the x0s since update_problem_data [b][n]
    double *Ef = nullptr, *Df = nullptr;  // frozen E, D once set_model re-runs (else the model's)
    double *ncache = nullptr;  // factor cache of the linear-only pass (ADMM), allocated on first use
    double *xlw = nullptr;     // KKT_RIC_XL: per-problem workspace (kernels_xl.hip)
};

template <typename X>
static int kalloc(pdplqr_handle h, X **p, size_t count) {
    *p = nullptr;
    void *q = nullptr;
    hipError_t e = hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(X));
    if (e != hipSuccess) {
        set_error(std::string("hipMalloc: ") + hipGetErrorString(e));
        return PDPLQR_ERR_ALLOC;
    }
    h->allocs.push_back(q);
    *p = reinterpret_cast<X *>(q);
    return PDPLQR_OK;
}

static KKTArgs kkt_args(pdplqr_handle h) {
    KKTState *ks = h->kkt;
    KKTArgs a;
    a.sh = h->sh;
    a.P = ks->P;
    a.dim = ks->dim;
    a.sigma = h->cfg.kkt_sigma;
    a.rho_dyn = h->cfg.rho_dyn;
    a.E = h->E;
    a.c = h->c;
    a.H = h->H;
    a.h = h->h;
    a.D = h->D;
    a.d_off = h->d_off;
    a.y_off = h->y_off;
    a.ncs = ks->d_ncs;
    a.prim_off = ks->d_prim_off;
    a.prim_dim = ks->d_prim_dim;
    a.dual_off = ks->d_dual_off;
    a.gdim = ks->d_gdim;
    a.blk = ks->blk;
    a.fac = ks->fac;
    a.rhs = ks->rhs;
    a.wv = ks->wv;
    a.ppk = ks->ppk;
    a.status = h->status;
    a.pstat = ks->pstat;
    return a;
}

int kkt_init(pdplqr_handle h) {
    const Shape &sh = h->sh;
    const int n = sh.n, m = sh.m, s = sh.s, N = sh.N;
    KKTState *ks = new (std::nothrow) KKTState();
    if (!ks) return PDPLQR_ERR_ALLOC;
    h->kkt = ks;
    ks->prim_off.resize(N + 1);
    ks->prim_dim.resize(N + 1);
    ks->dual_off.resize(N + 1);
    ks->gdim.resize(N + 1);
    int po = 0, dmax = s;
    for (int k = 0; k <= N; ++k) {
        ks->prim_off[k] = po;
        ks->prim_dim[k] = k == 0 ? m : (k < N ? s : n);
        po += ks->prim_dim[k];
    }
    int dof = po;  // = N s
    for (int k = 0; k <= N; ++k) {
        ks->dual_off[k] = dof;
        ks->gdim[k] = (k == 0 ? 0 : n) + h->ncs[k];
        dof += ks->gdim[k];
        dmax = std::max(dmax, ks->gdim[k]);
    }
    ks->dim = dof;
    const long long B = sh.batch;
    int rc;
    ks->ric = kkt_ric_nc(sh, h->ncs, dmax <= 32);
    if (ks->ric >= 0) {  // Riccati-ordered path: no tile buffers
        if ((rc = kalloc(h, &ks->rec, B * kkt_ric_rec_doubles(sh, ks->ric))) || (rc = kalloc(h, &ks->x0acc, B * n)) ||
            (ks->ric == KKT_RIC_XL && (rc = kalloc(h, &ks->xlw, B * kkt_xl_ws_doubles(sh)))))
            return rc;
        PDPLQR_HIP_TRY(hipMemset(ks->x0acc, 0, B * n * sizeof(double)));
        return PDPLQR_OK;
    }
    if (dmax > 32) {
        set_error(sh.s > 64 ? "KKT solver: n + m > 256, or more than 256 constraint rows on a stage"
                            : "KKT solver: more than 64 constraint rows on a stage with n + m > 32");
        return PDPLQR_ERR_UNSUPPORTED;
    }
    // P = 16 also needs stage 0's y columns beside the lambda_1 columns of G_0 (PPK)
    ks->P = dmax <= 16 && n + h->ncs[0] <= 16 ? 16 : 32;
    const long long PP = (long long)ks->P * ks->P;
    // row descriptors (kind, stage, index)
    std::vector<int4> rows(ks->dim);
    for (int k = 0; k <= N; ++k) {
        for (int a = 0; a < ks->prim_dim[k]; ++a) rows[ks->prim_off[k] + a] = make_int4(0, k, a, 0);
        const int base = ks->dual_off[k];
        if (k == 0) {
            for (int q = 0; q < h->ncs[0]; ++q) rows[base + q] = make_int4(1, 0, q, 0);
        } else {
            for (int i = 0; i < n; ++i) rows[base + i] = make_int4(2, k - 1, i, 0);
            for (int q = 0; q < h->ncs[k]; ++q) rows[base + n + q] = make_int4(1, k, q, 0);
        }
    }
    if ((rc = kalloc(h, &ks->d_prim_off, N + 1)) || (rc = kalloc(h, &ks->d_prim_dim, N + 1)) ||
        (rc = kalloc(h, &ks->d_dual_off, N + 1)) || (rc = kalloc(h, &ks->d_gdim, N + 1)) ||
        (rc = kalloc(h, &ks->d_ncs, N + 1)) || (rc = kalloc(h, &ks->rows, ks->dim)) || (rc = kalloc(h, &ks->pstat, B)) ||
        (rc = kalloc(h, &ks->blk, B * (N + 1) * 6 * PP)) || (rc = kalloc(h, &ks->fac, B * (N + 1) * 3 * PP)) ||
        (rc = kalloc(h, &ks->rhs, B * ks->dim)) ||
        (ks->P == 16 && ((rc = kalloc(h, &ks->dpk, B * (N + 1) * 512)) || (rc = kalloc(h, &ks->dreg, B * (N + 1) * 16)) ||
                         (rc = kalloc(h, &ks->bvec, B * (N + 1) * 16)) ||
                         (rc = kalloc(h, &ks->ppk, B * (N + 1) * PPK)))) || (rc = kalloc(h, &ks->wv, B * (N + 1) * 4 * ks->P)))
        return rc;
    PDPLQR_HIP_TRY(hipMemcpy(ks->d_prim_off, ks->prim_off.data(), (N + 1) * sizeof(int32_t), hipMemcpyHostToDevice));
    PDPLQR_HIP_TRY(hipMemcpy(ks->d_prim_dim, ks->prim_dim.data(), (N + 1) * sizeof(int32_t), hipMemcpyHostToDevice));
    PDPLQR_HIP_TRY(hipMemcpy(ks->d_dual_off, ks->dual_off.data(), (N + 1) * sizeof(int32_t), hipMemcpyHostToDevice));
    PDPLQR_HIP_TRY(hipMemcpy(ks->d_gdim, ks->gdim.data(), (N + 1) * sizeof(int32_t), hipMemcpyHostToDevice));
    PDPLQR_HIP_TRY(hipMemcpy(ks->d_ncs, h->ncs.data(), (N + 1) * sizeof(int32_t), hipMemcpyHostToDevice));
    PDPLQR_HIP_TRY(hipMemcpy(ks->rows, rows.data(), rows.size() * sizeof(int4), hipMemcpyHostToDevice));
    PDPLQR_HIP_TRY(hipMemset(ks->wv, 0, B * (N + 1) * 4 * ks->P * sizeof(double)));
    PDPLQR_HIP_TRY(hipMemset(ks->pstat, 0, B * sizeof(int32_t)));
    return PDPLQR_OK;
}

void kkt_release(pdplqr_handle h) {
    delete h->kkt;
    h->kkt = nullptr;
}

// The reference forms the KKT matrix once, in the QDLDLSolver constructor
// (qdldl_solver.hpp:36-45): the first model upload plays that role here.
int kkt_on_model(pdplqr_handle h) {
    KKTState *ks = h->kkt;
    if (ks->formed) return PDPLQR_OK;
    const Shape &sh = h->sh;
    if (ks->ric >= 0) {  // H + sigma_f I, packed: the matrix part that is formed once
        Shape hs = sh;
        hs.perh = 0;  // only the H~ part of the update kernel
        hs.ny = 0;
        const int rc = launch_update_problem_data(hs, h->H, h->h, nullptr, nullptr, nullptr, nullptr, h->cfg.kkt_sigma,
                                                  h->Hw, h->hw, h->gw, h->tab_s, h->tab_n, h->stream, false);
        if (rc) return rc;
        ks->formed = true;
        return PDPLQR_OK;
    }
    KKTArgs a = kkt_args(h);
    const size_t smem = 4 * (size_t)ks->P * ks->P * sizeof(double);
    const dim3 stages((unsigned)(sh.batch * (sh.N + 1))), wave(64);
    if (ks->P == 16) {
        hipLaunchKernelGGL(k_kkt_stage16, stages, wave, 0, h->stream, a);
        hipLaunchKernelGGL(k_kkt_pack16d, stages, wave, 0, h->stream, a, ks->dpk);
    } else {
        hipLaunchKernelGGL(k_kkt_stage, stages, wave, smem, h->stream, a);
        if (ks->P == 16) hipLaunchKernelGGL(k_kkt_pack16, stages, wave, 0, h->stream, a, ks->dpk);
    }
    PDPLQR_HIP_TRY(hipGetLastError());
    ks->formed = true;
    return PDPLQR_OK;
}

// A later set_model keeps the matrix frozen (qdldl_solver.hpp:36-45 forms it in
// the constructor only): the Riccati path snapshots E and D once, before the
// first overwrite (H + sigma_f I already lives in Hw).  The right-hand side
// keeps reading the current model (form_rhs re-reads model_, kkt.hpp:224-300).
// Deviation: the x0 terms of update_rhs_initial_stage use the CURRENT S0, A0 in
// the reference, the frozen ones here.
int kkt_before_model(pdplqr_handle h) {
    KKTState *ks = h->kkt;
    if (!ks || ks->ric < 0 || !ks->formed || ks->Ef) return PDPLQR_OK;
    const Shape &sh = h->sh;
    int rc;
    if ((rc = kalloc(h, &ks->Ef, sh.batch * sh.perE)) ||
        (sh.ndD > 0 && (rc = kalloc(h, &ks->Df, sh.batch * (long long)sh.ndD))))
        return rc;
    PDPLQR_HIP_TRY(hipMemcpyAsync(ks->Ef, h->E, sh.batch * sh.perE * sizeof(double), hipMemcpyDeviceToDevice, h->stream));
    if (sh.ndD > 0)
        PDPLQR_HIP_TRY(hipMemcpyAsync(ks->Df, h->D, sh.batch * (long long)sh.ndD * sizeof(double),
                                      hipMemcpyDeviceToDevice, h->stream));
    return PDPLQR_OK;
}

int kkt_update(pdplqr_handle h, const double *ws, const double *ys, const double *zs, const double *irho,
               double sigma) {
    KKTState *ks = h->kkt;
    const Shape &sh = h->sh;
    if (ks->ric >= 0) {  // h - sigma w, z - inv_rho o y; the x0 sum restarts
        const int rc = launch_update_problem_data(sh, h->H, h->h, ws, ys, zs, irho, sigma, h->Hw, h->hw, h->gw,
                                                  h->tab_s, h->tab_n, h->stream, true);
        if (rc) return rc;
        PDPLQR_HIP_TRY(hipMemsetAsync(ks->x0acc, 0, sh.batch * sh.n * sizeof(double), h->stream));
        return PDPLQR_OK;
    }
    KKTArgs a = kkt_args(h);
    const long long total = (long long)ks->dim * sh.batch;
    const unsigned grid = (unsigned)std::min<long long>((total + 255) / 256, 65536);
    hipLaunchKernelGGL(k_kkt_rhs, dim3(grid), dim3(256), 0, h->stream, a, ks->rows, ws, ys, zs, irho, sigma);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

int kkt_backward(pdplqr_handle h, const double *inv_rho) {
    KKTState *ks = h->kkt;
    const Shape &sh = h->sh;
    if (ks->ric >= 0) {
        const int rc = launch_kkt_ric_backward(sh, ks->ric, ks->Ef ? ks->Ef : h->E, h->c, ks->Df ? ks->Df : h->D, h->Hw,
                                               h->hw, h->gw, inv_rho, h->d_off, h->y_off, h->ncs[sh.N], h->cfg.rho_dyn,
                                               ks->rec, h->status, h->stream, ks->xlw);
        if (rc != PDPLQR_ERR_UNSUPPORTED) return rc;
        set_error("KKT backward: unaligned buffers for the Riccati-ordered path");
        return rc;
    }
    KKTArgs a = kkt_args(h);
    const size_t smem = 3 * (size_t)ks->P * ks->P * sizeof(double);
    if (ks->P == 16) {
        const long long total = (long long)sh.batch * (sh.N + 1) * 16;
        const unsigned grid = (unsigned)std::min<long long>((total + 255) / 256, 65536);
        hipLaunchKernelGGL(k_kkt_dreg16, dim3(grid), dim3(256), 0, h->stream, a, inv_rho, ks->dreg);
        hipLaunchKernelGGL(k_kkt_factor16_tw, dim3((unsigned)sh.batch), dim3(128), 0, h->stream, a, ks->dpk, ks->dreg);
    }
    else hipLaunchKernelGGL(k_kkt_factor, dim3((unsigned)sh.batch), dim3(64), smem, h->stream, a, inv_rho);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

bool kkt_linear_supported(pdplqr_handle h) {
    KKTState *ks = h->kkt;
    return ks && (ks->ric == 0 || ks->ric == 4) && !getenv("PDPLQR_KKT_NO_LINEAR");
}

// The factorisation with the linear pass's cache (ADMM iteration 1, and after
// a rho change: the KKT matrix depends on rho through the y diagonal)
int kkt_backward_cached(pdplqr_handle h, const double *inv_rho) {
    KKTState *ks = h->kkt;
    const Shape &sh = h->sh;
    int rc;
    if (!ks->ncache && (rc = kalloc(h, &ks->ncache, sh.batch * kkt_ric_cache_doubles(sh, ks->ric)))) return rc;
    h->rec_gain = false;  // the cache-writing backward leaves the P~ record (pdplqr_handle_s::rec_gain)
    rc = launch_kkt_ric_backward(sh, ks->ric, ks->Ef ? ks->Ef : h->E, h->c, ks->Df ? ks->Df : h->D, h->Hw, h->hw,
                                 h->gw, inv_rho, h->d_off, h->y_off, h->ncs[sh.N], h->cfg.rho_dyn, ks->rec, h->status,
                                 h->stream, ks->ncache);
    if (rc == PDPLQR_ERR_UNSUPPORTED) set_error("KKT backward: unaligned buffers for the Riccati-ordered path");
    return rc;
}

int kkt_rhs_restart(pdplqr_handle h) {
    KKTState *ks = h->kkt;
    PDPLQR_HIP_TRY(hipMemsetAsync(ks->x0acc, 0, h->sh.batch * h->sh.n * sizeof(double), h->stream));
    return PDPLQR_OK;
}

// Same rho, new right-hand side (h~, g of the last update_problem_data)
int kkt_backward_linear(pdplqr_handle h, const double *inv_rho) {
    KKTState *ks = h->kkt;
    const Shape &sh = h->sh;
    return launch_kkt_ric_nofact(sh, ks->ric, ks->Df ? ks->Df : h->D, h->hw, h->gw, inv_rho, h->d_off, h->y_off,
                                 h->ncs[sh.N], h->cfg.rho_dyn, ks->ncache, ks->rec, h->stream);
}

int kkt_forward(pdplqr_handle h, const double *x0, double *ws) {
    KKTState *ks = h->kkt;
    const Shape &sh = h->sh;
    if (ks->ric >= 0)
        return launch_kkt_ric_forward(sh, ks->Ef ? ks->Ef : h->E, h->c, ks->rec, x0, ks->x0acc, ws, h->cfg.rho_dyn,
                                      h->stream, ks->ric, h->rec_gain);
    KKTArgs a = kkt_args(h);
    const size_t P = ks->P, PP = P * P;
    const dim3 stages((unsigned)(sh.batch * (sh.N + 1))), probs((unsigned)sh.batch), wave(64);
    hipLaunchKernelGGL(k_kkt_x0, probs, wave, 0, h->stream, a, x0);
    if (P == 16) hipLaunchKernelGGL(k_kkt_solve1_16, stages, wave, 0, h->stream, a);
    else hipLaunchKernelGGL(k_kkt_solve1, stages, wave, (PP + P) * sizeof(double), h->stream, a);
    if (P == 16) {
        const long long total = (long long)sh.batch * (sh.N + 1) * 16;
        const unsigned grid = (unsigned)std::min<long long>((total + 255) / 256, 65536);
        hipLaunchKernelGGL(k_kkt_bvec16, dim3(grid), dim3(256), 0, h->stream, a, ks->bvec);
        hipLaunchKernelGGL(k_kkt_solve2_16_tw, probs, dim3(128), 0, h->stream, a, (const double *)ks->bvec);
    }
    else hipLaunchKernelGGL(k_kkt_solve2, probs, wave, (2 * PP + 2 * P) * sizeof(double), h->stream, a);
    if (P == 16) hipLaunchKernelGGL(k_kkt_solve3_16, stages, wave, 0, h->stream, a, x0, ws);
    else hipLaunchKernelGGL(k_kkt_solve3, stages, wave, (PP + P) * sizeof(double), h->stream, a, x0, ws);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

int kkt_forward_admm(pdplqr_handle h, const double *x0, const AdmmArgs &q, bool fuse, bool check) {
    KKTState *ks = h->kkt;
    if (!ks || ks->ric != 4 || h->rec_gain) return PDPLQR_ERR_UNSUPPORTED;
    return launch_kkt_ric_forward_admm(h->sh, ks->Ef ? ks->Ef : h->E, h->c, ks->rec, x0, ks->x0acc, h->cfg.rho_dyn,
                                       q, fuse, check, h->stream);
}

int kkt_dim(pdplqr_handle h) { return h->kkt ? h->kkt->dim : 0; }

bool kkt_ric_active(pdplqr_handle h) { return h->kkt && h->kkt->ric >= 0; }

// a plain backward of this handle's KKT path leaves the E^ record
bool kkt_plain_rec_ehat(pdplqr_handle h) { return h->kkt && h->kkt->ric >= 0 && kkt_ric_rec_ehat(h->kkt->ric); }

}  // namespace pdplqr
