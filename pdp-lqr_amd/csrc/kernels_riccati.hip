// kernels_riccati.hip -- batched serial square-root Riccati on MI355X (gfx950).
//
// Restates LQRSolver (reference include/clqr/lqr/lqr_solver.hpp:41-77) and
// LQRKernel (lqr_kernel.hpp:80-212) for `batch` independent problems:
//   * k_update_problem_data: lqr_solver.hpp:41-56 (memory-bound elementwise)
//   * k_penalty:             the rho D^T D / D^T rho g preamble of every kernel
//                            step (lqr_kernel.hpp:82-88,106-112); independent
//                            across stages, so it runs as one parallel pass
//   * k_riccati_bwd<T>:      terminal_step_with_factorization + the backward
//                            recursion of step_with_factorization (:80-147)
//   * k_riccati_bwd_nofact:  the *_without_factorization recursion (:94-101,150-178)
//   * k_riccati_fwd:         forward_step (:181-212) as u = K x + d, x+ = c + A x + B u
//
// Backward mapping: ONE wavefront per problem.  Stage matrices live in the
// f64 MFMA C/D layout (v_mfma_f64_16x16x4_f64: lane l = 16 g + c holds rows
// g, g+4, g+8, g+12 of column c of a 16x16 tile, one register per row group).
// With P = 16 T the padded stage size (u at 0..m-1, x at m..s-1, identity on
// the padding), each stage is
//     W = Lxx_next^T E          (MFMA, A operand = L_next read from LDS)
//     M = H~ + W^T W            (MFMA, both operands = W's registers, no data movement)
//     L = chol(M)               (right-looking, column broadcast through LDS)
// i.e. M = H~ + V V^T with V = E^T Lxx_next exactly as lqr_kernel.hpp:121-126.
#include "internal.hpp"

namespace pdplqr {

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ d4 mfma_f64(double a, double b, d4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// packed lower (column-major) index of (i, j), i >= j, dimension d
__device__ __forceinline__ int pidx(int i, int j, int d) { return j * d - ((j * (j - 1)) >> 1) + (i - j); }

__device__ __forceinline__ double shfl_xor_f64(double v, int mask) { return __shfl_xor(v, mask, 64); }

// ---------------------------------------------------------------------------
// update_problem_data (lqr_solver.hpp:41-56)
// ---------------------------------------------------------------------------
__global__ void k_update_problem_data(Shape sh, const double *__restrict__ H, const double *__restrict__ hv,
                                      const double *__restrict__ ws, const double *__restrict__ ys,
                                      const double *__restrict__ zs, const double *__restrict__ irho,
                                      double sigma, double *__restrict__ Hw, double *__restrict__ hw,
                                      double *__restrict__ gw, const short2 *__restrict__ tab_s,
                                      const short2 *__restrict__ tab_n) {
    const long long totH = sh.perHw * sh.batch, toth = sh.perh * sh.batch, totg = (long long)sh.ny * sh.batch;
    const long long total = totH + toth + totg;
    const long long stepg = (long long)gridDim.x * blockDim.x;
    const int s = sh.s;
    for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stepg) {
        if (t < totH) {
            const long long b = t / sh.perHw;
            const long long r = t - b * sh.perHw;
            const double *Hb = H + b * sh.perH;
            int i, j;
            double v;
            if (r < (long long)sh.N * sh.ps) {
                const int k = (int)(r / sh.ps), q = (int)(r - (long long)k * sh.ps);
                const short2 ij = tab_s[q];
                i = ij.x; j = ij.y;
                v = Hb[(long long)k * s * s + i + j * s];
            } else {
                const int q = (int)(r - (long long)sh.N * sh.ps);
                const short2 ij = tab_n[q];
                i = ij.x; j = ij.y;
                v = Hb[(long long)sh.N * s * s + i + j * sh.n];
            }
            Hw[t] = (i == j) ? v + sigma : v;
        } else if (t < totH + toth) {
            const long long u = t - totH;
            hw[u] = hv[u] - sigma * ws[u];
        } else {
            const long long u = t - totH - toth;
            gw[u] = zs[u] - irho[u] * ys[u];
        }
    }
}

int launch_update_problem_data(const Shape &sh, const double *H, const double *hv, const double *ws,
                               const double *ys, const double *zs, const double *irho, double sigma, double *Hw,
                               double *hw, double *gw, const short2 *tab_s, const short2 *tab_n,
                               hipStream_t st) {
    const long long total = (sh.perHw + sh.perh + sh.ny) * (long long)sh.batch;
    const int threads = 256;
    long long blocks = (total + threads - 1) / threads;
    if (blocks > 8192) blocks = 8192;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_update_problem_data, dim3((unsigned)blocks), dim3(threads), 0, st, sh, H, hv, ws, ys, zs,
                       irho, sigma, Hw, hw, gw, tab_s, tab_n);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

// ---------------------------------------------------------------------------
// rho penalty: H~ += D^T diag(rho) D ; h~ -= D^T (rho o g)   (lqr_kernel.hpp:82-88)
// ---------------------------------------------------------------------------
__global__ void k_penalty(Shape sh, const double *__restrict__ D, const double *__restrict__ rho,
                          const double *__restrict__ gw, double *__restrict__ Hw, double *__restrict__ hw,
                          const int32_t *__restrict__ d_off, const int32_t *__restrict__ y_off,
                          const short2 *__restrict__ tab_s, const short2 *__restrict__ tab_n, int with_H) {
    // one thread per (b, k, packed entry) for H, then per (b, k, i) for h
    const long long totH = with_H ? sh.perHw * sh.batch : 0;
    const long long toth = sh.perh * sh.batch;
    const long long stepg = (long long)gridDim.x * blockDim.x;
    const int s = sh.s, n = sh.n, N = sh.N;
    for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < totH + toth; t += stepg) {
        if (t < totH) {
            const long long b = t / sh.perHw;
            const long long r = t - b * sh.perHw;
            int k, i, j;
            if (r < (long long)N * sh.ps) {
                k = (int)(r / sh.ps);
                const short2 ij = tab_s[(int)(r - (long long)k * sh.ps)];
                i = ij.x; j = ij.y;
            } else {
                k = N;
                const short2 ij = tab_n[(int)(r - (long long)N * sh.ps)];
                i = ij.x; j = ij.y;
            }
            const int nc = y_off[k + 1] - y_off[k];
            if (nc == 0) continue;
            const double *Dk = D + b * sh.ndD + d_off[k];
            const double *rk = rho + b * sh.ny + y_off[k];
            double a = 0.0;
            for (int q = 0; q < nc; ++q) a += Dk[q + i * nc] * (rk[q] * Dk[q + j * nc]);
            Hw[t] += a;
        } else {
            const long long u = t - totH;
            const long long b = u / sh.perh;
            const int r = (int)(u - b * sh.perh);
            const int k = r < N * s ? r / s : N;
            const int i = r < N * s ? r - k * s : r - N * s;
            const int nc = y_off[k + 1] - y_off[k];
            if (nc == 0) continue;
            const double *Dk = D + b * sh.ndD + d_off[k];
            const double *rk = rho + b * sh.ny + y_off[k];
            const double *gk = gw + b * sh.ny + y_off[k];
            double a = 0.0;
            for (int q = 0; q < nc; ++q) a += Dk[q + i * nc] * (rk[q] * gk[q]);
            hw[u] -= a;
        }
    }
    (void)n;
}

int launch_penalty(const Shape &sh, const double *D, const double *rho, const double *gw, double *Hw,
                   double *hw, const int32_t *d_off, const int32_t *y_off, const short2 *tab_s,
                   const short2 *tab_n, int with_H, int max_nc, hipStream_t st) {
    if (max_nc <= 0) return PDPLQR_OK;
    const long long total = ((with_H ? sh.perHw : 0) + sh.perh) * (long long)sh.batch;
    const int threads = 256;
    long long blocks = (total + threads - 1) / threads;
    if (blocks > 8192) blocks = 8192;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_penalty, dim3((unsigned)blocks), dim3(threads), 0, st, sh, D, rho, gw, Hw, hw, d_off,
                       y_off, tab_s, tab_n, with_H);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

// ---------------------------------------------------------------------------
// Backward with factorization: one wavefront per problem, f64 MFMA tiles.
// ---------------------------------------------------------------------------
template <int T>
struct BwdSmem {
    static constexpr int P = 16 * T;
    static constexpr int LD = P + 1;  // odd leading dimension: conflict-free column reads
    double L[2][P * LD];              // L_{k+1} / L_k, padded, column-major, lower (zero upper)
    double col[2][P];                 // Cholesky column broadcast (double-buffered by step parity)
    double cvec[P], hvec[P];          // c_k, h~_k
    double va[P], vb[P];              // Pb_tmp, Pb
    double lp[P];                     // lp_k
    double pv[2][P];                  // p_{k+1} / p_k
    double ks[(P + 1) * P];           // K / d back-substitution scratch (lane-private rows)
};

// Loads the padded stage matrix H~ into C/D-layout tiles.  Indices in
// [lo, hi) map to the stored packed block (dimension dim, offset off);
// everything else is the identity padding.
template <int T>
__device__ __forceinline__ void load_M(d4 (&M)[T][T], const double *__restrict__ Hp, int dim, int off, int lo, int hi,
                                       int g, int c) {
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int b = 0; b < T; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * a + 4 * r + g, j = 16 * b + c;
                double v;
                if (i >= lo && i < hi && j >= lo && j < hi) {
                    const int ii = i - off, jj = j - off;
                    v = (ii >= jj) ? Hp[pidx(ii, jj, dim)] : Hp[pidx(jj, ii, dim)];
                } else {
                    v = (i == j) ? 1.0 : 0.0;
                }
                M[a][b][r] = v;
            }
}

// Right-looking Cholesky of the symmetric padded matrix held in C/D layout.
// Column j is broadcast through LDS from row j (symmetry: the row-group that
// owns row j holds M[j][*] = M[*][j]).  Columns >= `jend` are left untouched
// (identity padding).  Returns the first failing column or -1.
template <int T>
__device__ __forceinline__ int chol_tiles(d4 (&M)[T][T], double (*col)[16 * T], int jbeg, int jend, int g, int c) {
    int fail = -1;
#pragma unroll
    for (int j = 0; j < 16 * T; ++j) {
        if (j >= jbeg && j < jend) {
            const int tr = j >> 4, rr = (j >> 2) & 3, gj = j & 3;
            double *cb = col[j & 1];
            if (g == gj) {
#pragma unroll
                for (int b = 0; b < T; ++b) cb[16 * b + c] = M[tr][b][rr];
            }
            __syncthreads();
            const double djj = cb[j];
            if (!(djj > 0.0) && fail < 0) fail = j;
            const double d = sqrt(djj);
            const double inv = 1.0 / d;
            double lc[T], lr[T][4];
#pragma unroll
            for (int b = 0; b < T; ++b) {
                const int jc = 16 * b + c;
                const double v = cb[jc] * inv;
                lc[b] = jc > j ? v : (jc == j ? d : 0.0);
            }
#pragma unroll
            for (int a = 0; a < T; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * a + 4 * r + g;
                    const double v = cb[i] * inv;
                    lr[a][r] = i > j ? v : (i == j ? d : 0.0);
                }
#pragma unroll
            for (int a = 0; a < T; ++a)
#pragma unroll
                for (int b = 0; b < T; ++b) {
                    const int jc = 16 * b + c;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const double upd = M[a][b][r] - lr[a][r] * lc[b];
                        M[a][b][r] = (jc == j) ? lr[a][r] : (jc > j ? upd : M[a][b][r]);
                    }
                }
        }
    }
    return fail;
}

template <int T>
__device__ __forceinline__ void store_L_lds(const d4 (&M)[T][T], double *L, int g, int c) {
    constexpr int LD = 16 * T + 1;
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int b = 0; b < T; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) L[(16 * a + 4 * r + g) + (16 * b + c) * LD] = M[a][b][r];
}

template <int T>
__global__ __launch_bounds__(64) void k_riccati_bwd(RiccatiArgs A) {
    constexpr int P = 16 * T, LD = P + 1;
    __shared__ BwdSmem<T> sm;
    const int lane = threadIdx.x, g = lane >> 4, c = lane & 15;
    const long long b = blockIdx.x;
    const Shape &sh = A.sh;
    const int n = sh.n, m = sh.m, N = sh.N, s = sh.s;
    const int nch = (n + 3) >> 2;
    const double *Eb = A.E + b * sh.perE;
    const double *cb = A.c + b * sh.perc;
    const double *Hb = A.Hw + b * sh.perHw;
    const double *hb = A.hw + b * sh.perh;
    double *KDb = A.KD + b * sh.perKD;
    double *Lcb = A.Lc ? A.Lc + b * sh.perHw : nullptr;
    double *lpb = A.lpc ? A.lpc + b * sh.perh : nullptr;
    int fail_stage = -1;

    // ---- terminal: L_N = chol(H~_N), lp_N = h~_N  (lqr_kernel.hpp:80-91) ----
    int cur = 0;
    {
        d4 M[T][T];
        load_M<T>(M, Hb + (long long)N * sh.ps, n, m, m, s, g, c);
        const int f = chol_tiles<T>(M, sm.col, m, s, g, c);
        if (f >= 0) fail_stage = N;
        store_L_lds<T>(M, sm.L[cur], g, c);
        if (lane < n) {
            const double v = hb[(long long)N * s + lane];
            sm.pv[cur][lane] = v;
            if (lpb) lpb[(long long)N * s + lane] = v;
        }
        __syncthreads();
        if (Lcb)
            for (int q = lane; q < sh.pn; q += 64) {
                const short2 ij = A.tab_n[q];
                Lcb[(long long)N * sh.ps + q] = sm.L[cur][(m + ij.x) + (m + ij.y) * LD];
            }
    }

    for (int k = N - 1; k >= 0; --k) {
        const int nx = cur;
        cur ^= 1;
        const double *Ek = Eb + (long long)k * n * s;
        // ---- loads: E as the MFMA B operand, H~ as the C input, c and h~ via LDS ----
        double Eop[4 * T][T];
#pragma unroll
        for (int cc = 0; cc < 4 * T; ++cc)
#pragma unroll
            for (int bt = 0; bt < T; ++bt) {
                const int t = 4 * cc + g, j = 16 * bt + c;
                Eop[cc][bt] = (cc < nch && t < n && j < s) ? Ek[t + j * n] : 0.0;
            }
        d4 M[T][T];
        load_M<T>(M, Hb + (long long)k * sh.ps, s, 0, 0, s, g, c);
        if (lane < n) sm.cvec[lane] = cb[(long long)k * n + lane];
        if (lane < s) sm.hvec[lane] = hb[(long long)k * s + lane];
        __syncthreads();

        const double *Ln = sm.L[nx];
        // ---- Pb_tmp = Lxx_next^T c ; Pb = Lxx_next Pb_tmp + p_next (lqr_kernel.hpp:138-140) ----
        if (lane < n) {
            double a = 0.0;
            for (int t = lane; t < n; ++t) a += Ln[(m + t) + (m + lane) * LD] * sm.cvec[t];
            sm.va[lane] = a;
        }
        __syncthreads();
        if (lane < n) {
            double a = 0.0;
            for (int t = 0; t <= lane; ++t) a += Ln[(m + lane) + (m + t) * LD] * sm.va[t];
            sm.vb[lane] = a + sm.pv[nx][lane];
        }
        // ---- W = Lxx_next^T E ; M = H~ + W^T W  (lqr_kernel.hpp:121-124) ----
        d4 W[T][T];
#pragma unroll
        for (int a = 0; a < T; ++a)
#pragma unroll
            for (int bt = 0; bt < T; ++bt) W[a][bt] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int cc = 0; cc < 4 * T; ++cc) {
            if (cc < nch) {
                const int t = 4 * cc + g;
#pragma unroll
                for (int a = 0; a < T; ++a) {
                    const int tp = 16 * a + c;
                    const double av = (t < n && tp < n) ? Ln[(m + t) + (m + tp) * LD] : 0.0;
#pragma unroll
                    for (int bt = 0; bt < T; ++bt) W[a][bt] = mfma_f64(av, Eop[cc][bt], W[a][bt]);
                }
            }
        }
#pragma unroll
        for (int kc = 0; kc < 4 * T; ++kc) {
            if (kc < nch) {
                const int ka = kc >> 2, r = kc & 3;
#pragma unroll
                for (int a = 0; a < T; ++a)
#pragma unroll
                    for (int bt = 0; bt < T; ++bt) M[a][bt] = mfma_f64(W[ka][a][r], W[ka][bt][r], M[a][bt]);
            }
        }
        __syncthreads();
        // ---- lp = h~ + E^T Pb (lqr_kernel.hpp:142-143), reduced over the 4 row groups ----
        {
            double part[T];
#pragma unroll
            for (int bt = 0; bt < T; ++bt) part[bt] = 0.0;
#pragma unroll
            for (int cc = 0; cc < 4 * T; ++cc) {
                const int t = 4 * cc + g;
                if (cc < nch && t < n) {
                    const double pb = sm.vb[t];
#pragma unroll
                    for (int bt = 0; bt < T; ++bt) part[bt] += Eop[cc][bt] * pb;
                }
            }
#pragma unroll
            for (int bt = 0; bt < T; ++bt) {
                part[bt] += shfl_xor_f64(part[bt], 16);
                part[bt] += shfl_xor_f64(part[bt], 32);
                const int j = 16 * bt + c;
                if (g == 0 && j < s) sm.lp[j] = sm.hvec[j] + part[bt];
            }
        }
        // ---- L = chol(M) (lqr_kernel.hpp:126) ----
        const int f = chol_tiles<T>(M, sm.col, 0, s, g, c);
        if (f >= 0 && fail_stage < 0) fail_stage = k;
        double *Lk = sm.L[cur];
        store_L_lds<T>(M, Lk, g, c);
        __syncthreads();
        // ---- lu <- Luu^{-1} lu (:145) ----
        if (lane == 0) {
            for (int i = 0; i < m; ++i) {
                double v = sm.lp[i];
                for (int j = 0; j < i; ++j) v -= Lk[i + j * LD] * sm.lp[j];
                sm.lp[i] = v / Lk[i + i * LD];
            }
        }
        __syncthreads();
        // ---- p -= Lxu lu (:146) ----
        if (lane < n) {
            double a = 0.0;
            for (int i = 0; i < m; ++i) a += Lk[(m + lane) + i * LD] * sm.lp[i];
            const double pnew = sm.lp[m + lane] - a;
            sm.pv[cur][lane] = pnew;
            sm.lp[m + lane] = pnew;
        }
        // ---- rollout gains: K = -Luu^{-T} Lxu^T, d = -Luu^{-T} lu (lqr_kernel.hpp:197-198) ----
        if (lane <= n) {
            double *ks = sm.ks + lane * P;
            for (int i = m - 1; i >= 0; --i) {
                double v = (lane < n) ? -Lk[(m + lane) + i * LD] : -sm.lp[i];
                for (int j = i + 1; j < m; ++j) v -= Lk[j + i * LD] * ks[j];
                v /= Lk[i + i * LD];
                ks[i] = v;
                KDb[(long long)k * (m * n + m) + (lane < n ? i + lane * m : m * n + i)] = v;
            }
        }
        __syncthreads();
        if (Lcb) {
            for (int q = lane; q < sh.ps; q += 64) {
                const short2 ij = A.tab_s[q];
                Lcb[(long long)k * sh.ps + q] = Lk[ij.x + ij.y * LD];
            }
            if (lane < s) lpb[(long long)k * s + lane] = sm.lp[lane];
        }
    }
    if (lane == 0) A.status[b] = fail_stage < 0 ? 0 : fail_stage + 1;
}

int launch_riccati_backward(const RiccatiArgs &a, hipStream_t st) {
    if (a.sh.s <= 16) {
        hipLaunchKernelGGL(k_riccati_bwd<1>, dim3(a.sh.batch), dim3(64), 0, st, a);
    } else if (a.sh.s <= 32) {
        hipLaunchKernelGGL(k_riccati_bwd<2>, dim3(a.sh.batch), dim3(64), 0, st, a);
    } else {
        set_error("backward: n + m > 32 is not supported by this build");
        return PDPLQR_ERR_UNSUPPORTED;
    }
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

// ---------------------------------------------------------------------------
// Backward without factorization (lqr_kernel.hpp:94-101,150-178): only the
// linear terms, reusing the cached factors L_k.  One wavefront per problem.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_riccati_bwd_nofact(RiccatiArgs A) {
    constexpr int P = 32;
    __shared__ double Lk[P * P];  // this stage's L (packed -> dense, column-major, ld = s)
    __shared__ double Ln[P * P];  // next stage's Lxx (ld = n)
    __shared__ double cvec[P], va[P], vb[P], lp[P], pn[P];
    const int lane = threadIdx.x;
    const long long b = blockIdx.x;
    const Shape &sh = A.sh;
    const int n = sh.n, m = sh.m, N = sh.N, s = sh.s;
    const double *Eb = A.E + b * sh.perE;
    const double *cb = A.c + b * sh.perc;
    const double *hb = A.hw + b * sh.perh;
    double *KDb = A.KD + b * sh.perKD;
    const double *Lcb = A.Lc + b * sh.perHw;
    double *lpb = A.lpc + b * sh.perh;
    // terminal (lqr_kernel.hpp:94-101): lp_N = h~_N ; Lxx_N from the cache
    if (lane < n) {
        const double v = hb[(long long)N * s + lane];
        pn[lane] = v;
        lpb[(long long)N * s + lane] = v;
    }
    for (int q = lane; q < sh.pn; q += 64) {
        const short2 ij = A.tab_n[q];
        const double v = Lcb[(long long)N * sh.ps + q];
        Ln[ij.x + ij.y * n] = v;
        Ln[ij.y + ij.x * n] = (ij.x == ij.y) ? v : 0.0;
    }
    __syncthreads();
    for (int k = N - 1; k >= 0; --k) {
        const double *Ek = Eb + (long long)k * n * s;
        for (int q = lane; q < sh.ps; q += 64) {
            const short2 ij = A.tab_s[q];
            const double v = Lcb[(long long)k * sh.ps + q];
            Lk[ij.x + ij.y * s] = v;
            if (ij.x != ij.y) Lk[ij.y + ij.x * s] = 0.0;
        }
        if (lane < n) cvec[lane] = cb[(long long)k * n + lane];
        __syncthreads();
        if (lane < n) {  // Pb_tmp = Lxx_next^T c
            double a = 0.0;
            for (int t = lane; t < n; ++t) a += Ln[t + lane * n] * cvec[t];
            va[lane] = a;
        }
        __syncthreads();
        if (lane < n) {  // Pb = Lxx_next Pb_tmp + p_next
            double a = 0.0;
            for (int t = 0; t <= lane; ++t) a += Ln[lane + t * n] * va[t];
            vb[lane] = a + pn[lane];
        }
        __syncthreads();
        if (lane < s) {  // lp = h~ + E^T Pb
            double a = 0.0;
            for (int t = 0; t < n; ++t) a += Ek[t + lane * n] * vb[t];
            lp[lane] = hb[(long long)k * s + lane] + a;
        }
        __syncthreads();
        if (lane == 0) {
            for (int i = 0; i < m; ++i) {
                double v = lp[i];
                for (int j = 0; j < i; ++j) v -= Lk[i + j * s] * lp[j];
                lp[i] = v / Lk[i + i * s];
            }
        }
        __syncthreads();
        if (lane < n) {
            double a = 0.0;
            for (int i = 0; i < m; ++i) a += Lk[(m + lane) + i * s] * lp[i];
            const double pnew = lp[m + lane] - a;
            lp[m + lane] = pnew;
            pn[lane] = pnew;
        }
        __syncthreads();
        if (lane == 0) {  // d = -Luu^{-T} lu ; K is unchanged
            double dv[P];
            for (int i = m - 1; i >= 0; --i) {
                double v = -lp[i];
                for (int j = i + 1; j < m; ++j) v -= Lk[j + i * s] * dv[j];
                v /= Lk[i + i * s];
                dv[i] = v;
                KDb[(long long)k * (m * n + m) + m * n + i] = v;
            }
        }
        if (lane < s) lpb[(long long)k * s + lane] = lp[lane];
        // the next iteration's Lxx_next is this stage's bottom-right block
        __syncthreads();
        for (int q = lane; q < n * n; q += 64) {
            const int i = q % n, j = q / n;
            Ln[i + j * n] = Lk[(m + i) + (m + j) * s];
        }
        __syncthreads();
    }
}

int launch_riccati_backward_nofact(const RiccatiArgs &a, hipStream_t st) {
    if (a.sh.s > 32) {
        set_error("backward_without_factorization: n + m > 32 is not supported by this build");
        return PDPLQR_ERR_UNSUPPORTED;
    }
    hipLaunchKernelGGL(k_riccati_bwd_nofact, dim3(a.sh.batch), dim3(64), 0, st, a);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

// ---------------------------------------------------------------------------
// Forward rollout (lqr_kernel.hpp:181-212): u = K x + d ; x+ = c + A x + B u.
// One wavefront per problem.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_riccati_fwd(Shape sh, const double *__restrict__ E,
                                                    const double *__restrict__ c, const double *__restrict__ KD,
                                                    const double *__restrict__ x0, double *__restrict__ ws) {
    __shared__ double xs[64], us[64];
    const int lane = threadIdx.x;
    const long long b = blockIdx.x;
    const int n = sh.n, m = sh.m, N = sh.N, s = sh.s;
    const double *Eb = E + b * sh.perE;
    const double *cb = c + b * sh.perc;
    const double *KDb = KD + b * sh.perKD;
    double *wb = ws + b * sh.perh;
    if (lane < n) {
        const double v = x0[b * n + lane];
        xs[lane] = v;
        wb[m + lane] = v;  // ws[0].tail(n) = x0 (lqr_solver.hpp:73)
    }
    __syncthreads();
    for (int k = 0; k < N; ++k) {
        const double *Kk = KDb + (long long)k * (m * n + m);
        const double *Ek = Eb + (long long)k * n * s;
        if (lane < m) {
            double u = Kk[m * n + lane];
            for (int t = 0; t < n; ++t) u += Kk[lane + t * m] * xs[t];
            us[lane] = u;
            wb[(long long)k * s + lane] = u;
        }
        __syncthreads();
        double xn = 0.0;
        if (lane < n) {
            double a = cb[(long long)k * n + lane];
            for (int t = 0; t < n; ++t) a += Ek[lane + (m + t) * n] * xs[t];
            for (int j = 0; j < m; ++j) a += Ek[lane + j * n] * us[j];
            xn = a;
        }
        __syncthreads();
        if (lane < n) {
            xs[lane] = xn;
            wb[(long long)(k + 1) * s + ((k + 1 < N) ? m : 0) + lane] = xn;
        }
        __syncthreads();
    }
}

int launch_riccati_forward(const Shape &sh, const double *E, const double *c, const double *KD, const double *x0,
                           double *ws, hipStream_t st) {
    if (sh.n > 64 || sh.m > 64) {
        set_error("forward: n or m > 64 unsupported");
        return PDPLQR_ERR_UNSUPPORTED;
    }
    hipLaunchKernelGGL(k_riccati_fwd, dim3(sh.batch), dim3(64), 0, st, sh, E, c, KD, x0, ws);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

}  // namespace pdplqr
