// kernels_xl.hip -- the serial solver (LQRSolver) for stage sizes
// 64 < n + m <= 256: one 256-thread block per problem, the stage matrices in
// a per-problem global-memory workspace (L2-resident; too large for LDS),
// products by the block-wide MFMA routine of blk_la.hpp on 64 x 64 output
// blocks.  A generality path: the reference is dynamic-size
// (lqr_kernel.hpp:104-147 on Eigen::MatrixXd), and these kernels restate it
// literally, in its own factor form:
//   * k_riccati_bwd_xl: terminal_step_with_factorization (lqr_kernel.hpp:80-91)
//     and step_with_factorization (:104-147) --
//         V = E~^T Lxx_{k+1},  M = H~ + V V^T,  L = llt(M)
//         lp = h~ + E~^T (Lxx (Lxx^T c) + p_{k+1}),  lu <- Luu^{-1} lu,
//         p_k = lp_x - Lxu lu
//     with Eigen's LLT stop as LLT::compute leaves it for these orders (>= 65:
//     the blocked form, xl_la.hpp xl_llt -- the later columns at the Schur
//     complement of the finished blocks) and the same status as every backward.
//     Records FR_k = [L(:, 0:m) | lu'], the factor cache (packed L_k, lp_k)
//     when it exists;
//   * k_riccati_bwd_nofact_xl: step_without_factorization (:150-178) on the
//     cached factors;
//   * k_riccati_fwd_xl: forward_step (:181-212).
// Workspace per problem (RiccatiArgs::xl_ws, xl_ws_doubles): V (s x n), two
// s x s factor buffers (this stage's, the next stage's) and the factorisation's
// input, leading dimension s.
#include "parallel.hpp"
#include "xl_la.hpp"

namespace pdplqr {

bool xl_shape(const Shape &sh) { return sh.s > 64 && sh.s <= XL_S; }

// lp (s) = h~ + E~^T (Lxx (Lxx^T c) + p): t, pb: n doubles of LDS
__device__ void xl_linear(double *lp, const double *hk, const double *Ek, const double *ck, const double *Lxx, int ldl,
                          const double *p, int n, int s, double *t, double *pb) {
    const int tid = threadIdx.x;
    __syncthreads();
    for (int j = tid; j < n; j += 256) {  // t = Lxx^T c
        double a = 0.0;
        for (int i = j; i < n; ++i) a = __builtin_fma(Lxx[i + (long long)j * ldl], ck[i], a);
        t[j] = a;
    }
    __syncthreads();
    for (int i = tid; i < n; i += 256) {  // pb = Lxx t + p
        double a = p[i];
        for (int j = 0; j <= i; ++j) a = __builtin_fma(Lxx[i + (long long)j * ldl], t[j], a);
        pb[i] = a;
    }
    __syncthreads();
    for (int j = tid; j < s; j += 256) {  // lp = h~ + E~^T pb
        double a = hk[j];
        for (int i = 0; i < n; ++i) a = __builtin_fma(Ek[i + (long long)j * n], pb[i], a);
        lp[j] = a;
    }
    __syncthreads();
}

__global__ __launch_bounds__(256) void k_riccati_bwd_xl(RiccatiArgs A) {
    __shared__ double sinv[XL_S], lp[XL_S], pv[XL_S], t[XL_S], pb[XL_S];
    const int tid = threadIdx.x;
    const Shape &sh = A.sh;
    const int n = sh.n, m = sh.m, s = sh.s, N = sh.N, ps = sh.ps;
    const long long b = blockIdx.x;
    const double *Eb = A.E + b * sh.perE;
    const double *cb = A.c + b * sh.perc;
    const double *Hb = A.Hw + b * sh.perHw;
    const double *hb = A.hw + b * sh.perh;
    double *FRb = A.KD + b * sh.perKD;
    double *Lcb = A.Lc ? A.Lc + b * sh.perHw : nullptr;
    double *lpb = A.lpc ? A.lpc + b * sh.perh : nullptr;
    double *W = A.xl_ws + b * xl_ws_doubles(sh);
    double *const V = W, *const L0 = W + (long long)s * n, *const L1 = L0 + (long long)s * s;
    double *const M0 = L1 + (long long)s * s;  // the factorisation's input (Eigen's stop)
    auto Lb = [&](int k) { return (k & 1) ? L1 : L0; };
    const long long frs = (long long)s * m + m;
    int fail_stage = -1;
    // ---- terminal: L_N = llt(H~_N) (order n, stored at (m, m) of the factor buffer), p_N = h~_N ----
    double *Ln = Lb(N);
    double *LxxN = Ln + m + (long long)m * s;
    const double *HN = Hb + (long long)N * ps;
    for (int q = tid; q < n * n; q += 256) {
        const int i = q % n, j = q / n;
        LxxN[i + (long long)j * s] = i >= j ? HN[pidx(i, j, n)] : 0.0;
    }
    xl_copy_lower(M0, LxxN, s, n);
    if (!xl_llt(LxxN, s, n, 0, M0, sinv)) fail_stage = N;
    for (int q = tid; q < n * n; q += 256) {  // V reads Lxx as a full matrix: zeros above the diagonal
        const int i = q % n, j = q / n;
        if (i < j) LxxN[i + (long long)j * s] = 0.0;
    }
    for (int q = tid; q < n; q += 256) {
        pv[q] = hb[(long long)N * s + q];
        if (lpb) lpb[(long long)N * s + q] = pv[q];
    }
    if (Lcb)
        for (int q = tid; q < n * n; q += 256) {
            const int i = q % n, j = q / n;
            if (i >= j) Lcb[(long long)N * ps + pidx(i, j, n)] = LxxN[i + (long long)j * s];
        }
    for (int k = N - 1; k >= 0; --k) {
        const double *Ek = Eb + (long long)k * n * s;
        double *Lk = Lb(k);
        const double *Lxx = Lb(k + 1) + m + (long long)m * s;  // Lxx_{k+1}, ld s
        // V = E~^T Lxx_{k+1} (s x n): only its lower triangle is meaningful, the
        // upper part of the factor buffer is zero
        xl_mm(V, s, Ek, n, true, Lxx, s, false, s, n, n, nullptr, 0);
        // M = H~ + V V^T into Lk (H~ unpacked first, then added in place)
        __syncthreads();
        for (int q = tid; q < s * s; q += 256) {
            const int i = q % s, j = q / s;
            Lk[i + (long long)j * s] = Hb[(long long)k * ps + (i >= j ? pidx(i, j, s) : pidx(j, i, s))];
        }
        xl_mm(Lk, s, V, s, false, V, s, true, s, s, n, Lk, s);
        xl_linear(lp, hb + (long long)k * s, Ek, cb + (long long)k * n, Lxx, s, pv, n, s, t, pb);
        xl_copy_lower(M0, Lk, s, s);
        const bool ok = xl_llt(Lk, s, s, m, M0, sinv);
        if (!ok && fail_stage < 0) fail_stage = k;
        xl_solve_u(lp, Lk, s, m, s, pb);
        for (int q = tid; q < n; q += 256) pv[q] = lp[m + q];
        // records: FR_k = [L(:, 0:m) | lu'] (zeros above the diagonal), caches
        double *FRk = FRb + (long long)k * frs;
        for (int q = tid; q < s * m; q += 256) {
            const int i = q % s, j = q / s;
            FRk[(long long)j * s + i] = i >= j ? Lk[i + (long long)j * s] : 0.0;
        }
        for (int q = tid; q < m; q += 256) FRk[(long long)s * m + q] = lp[q];
        if (lpb)
            for (int q = tid; q < s; q += 256) lpb[(long long)k * s + q] = lp[q];
        if (Lcb)
            for (int q = tid; q < s * s; q += 256) {
                const int i = q % s, j = q / s;
                if (i >= j) Lcb[(long long)k * ps + pidx(i, j, s)] = Lk[i + (long long)j * s];
            }
        // the next stage reads Lxx of this buffer: its upper part must be zero
        for (int q = tid; q < s * s; q += 256) {
            const int i = q % s, j = q / s;
            if (i < j) Lk[i + (long long)j * s] = 0.0;
        }
        __syncthreads();
    }
    if (tid == 0) A.status[b] = fail_stage < 0 ? 0 : fail_stage + 1;
}

__global__ __launch_bounds__(256) void k_riccati_bwd_nofact_xl(RiccatiArgs A) {
    __shared__ double lp[XL_S], pv[XL_S], t[XL_S], pb[XL_S];
    const int tid = threadIdx.x;
    const Shape &sh = A.sh;
    const int n = sh.n, m = sh.m, s = sh.s, N = sh.N, ps = sh.ps;
    const long long b = blockIdx.x;
    const double *Eb = A.E + b * sh.perE;
    const double *cb = A.c + b * sh.perc;
    const double *hb = A.hw + b * sh.perh;
    double *FRb = A.KD + b * sh.perKD;
    const double *Lcb = A.Lc + b * sh.perHw;
    double *lpb = A.lpc + b * sh.perh;
    double *W = A.xl_ws + b * xl_ws_doubles(sh);
    double *const L0 = W + (long long)s * n, *const L1 = L0 + (long long)s * s;
    auto Lb = [&](int k) { return (k & 1) ? L1 : L0; };
    const long long frs = (long long)s * m + m;
    // the cached factors unpacked into the workspace (ld s; Lxx of the
    // terminal at (m, m)); the same products as the factorising backward
    auto unpack = [&](double *L, int k) {
        __syncthreads();
        if (k == N) {
            for (int q = tid; q < n * n; q += 256) {
                const int i = q % n, j = q / n;
                L[(m + i) + (long long)(m + j) * s] = i >= j ? Lcb[(long long)N * ps + pidx(i, j, n)] : 0.0;
            }
        } else {
            for (int q = tid; q < s * s; q += 256) {
                const int i = q % s, j = q / s;
                L[i + (long long)j * s] = i >= j ? Lcb[(long long)k * ps + pidx(i, j, s)] : 0.0;
            }
        }
        __syncthreads();
    };
    for (int q = tid; q < n; q += 256) {  // lp_N = h~_N (lqr_kernel.hpp:94-101)
        pv[q] = hb[(long long)N * s + q];
        lpb[(long long)N * s + q] = pv[q];
    }
    unpack(Lb(N), N);
    for (int k = N - 1; k >= 0; --k) {
        double *Lk = Lb(k);
        unpack(Lk, k);
        const double *Lxx = Lb(k + 1) + m + (long long)m * s;
        xl_linear(lp, hb + (long long)k * s, Eb + (long long)k * n * s, cb + (long long)k * n, Lxx, s, pv, n, s, t, pb);
        xl_solve_u(lp, Lk, s, m, s, pb);
        for (int q = tid; q < n; q += 256) pv[q] = lp[m + q];
        for (int q = tid; q < m; q += 256) FRb[(long long)k * frs + (long long)s * m + q] = lp[q];
        for (int q = tid; q < s; q += 256) lpb[(long long)k * s + q] = lp[q];
        __syncthreads();
    }
}

// forward_step (lqr_kernel.hpp:181-212): u = -Luu^{-T} (lu' + Lxu^T x),
// x+ = c + E~ [u; x]; ws[k s .. k s + s) = [u_k; x_k], ws[N s ..) = x_N
__global__ __launch_bounds__(256) void k_riccati_fwd_xl(Shape sh, const double *__restrict__ E,
                                                      const double *__restrict__ c, const double *__restrict__ FR,
                                                      const double *__restrict__ x0, double *__restrict__ ws) {
    __shared__ double w[XL_S], v[XL_S];
    const int tid = threadIdx.x;
    const int n = sh.n, m = sh.m, N = sh.N, s = sh.s;
    const long long b = blockIdx.x;
    const long long frs = (long long)s * m + m;
    const double *Eb = E + b * sh.perE;
    const double *cb = c + b * sh.perc;
    const double *Fb = FR + b * sh.perKD;
    double *wb = ws + b * sh.perh;
    for (int q = tid; q < n; q += 256) {
        w[m + q] = x0[b * n + q];
        wb[(long long)(N > 0 ? m : 0) + q] = w[m + q];
    }
    __syncthreads();
    for (int k = 0; k < N; ++k) {
        const double *Fk = Fb + (long long)k * frs;
        for (int j = tid; j < m; j += 256) {  // v = -(lu' + Lxu^T x)
            double a = Fk[(long long)s * m + j];
            for (int i = 0; i < n; ++i) a = __builtin_fma(Fk[(long long)j * s + m + i], w[m + i], a);
            v[j] = -a;
        }
        for (int j = m - 1; j >= 0; --j) {  // u = Luu^{-T} v (back substitution)
            __syncthreads();
            const double uj = v[j] / Fk[(long long)j * s + j];
            __syncthreads();
            for (int i = tid; i < j; i += 256) v[i] = __builtin_fma(-Fk[(long long)i * s + j], uj, v[i]);
            if (tid == 0) v[j] = uj;
        }
        __syncthreads();
        for (int j = tid; j < m; j += 256) {
            w[j] = v[j];
            wb[(long long)k * s + j] = v[j];
        }
        __syncthreads();
        const double *Ek = Eb + (long long)k * n * s;
        double xn = 0.0;  // n < 256: one state row per thread
        if (tid < n) {
            xn = cb[(long long)k * n + tid];
            for (int j = 0; j < s; ++j) xn = __builtin_fma(Ek[tid + (long long)j * n], w[j], xn);
        }
        __syncthreads();
        if (tid < n) {
            w[m + tid] = xn;
            wb[(long long)(k + 1) * s + ((k + 1 < N) ? m : 0) + tid] = xn;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// QDLDLSolver's KKT system (kkt.hpp:124-300) at 64 < n + m <= 256: the reverse
// stage-order elimination of kkt_riccati.hip (see its header for why it gives
// the reference's solution) with k_kkt_ric_bwd_wide's steps on the global
// workspace.  Per stage, from the value function (P, p) of stage k + 1:
//     P~ = (I + rho_dyn P)^{-1} P   the Neumann series while e = rho_dyn ||P||_F
//                                   <= PDPLQR_KKT_NEUMANN_MAX, else the Cholesky
//                                   of S = I + rho_dyn P with P carried through
//                                   both triangular solves,
//     G = P~ E~,  M = H~ + E~^T G + D^T rho D,
//     lp = h~ + G^T (c - rho_dyn p) + E~^T p - D^T rho g   (stage 0: D's u columns),
// then the m u-pivots of M leave P_k, p_k.  Record per stage (the wide layout,
// kkt_ric_rec_doubles): [L(:, 0:m) | lu' | p_{k+1} | P~_{k+1} (n x n)].
// Workspace per problem (kkt_xl_ws_doubles): XA (n x s: P, then G), Pt, T0
// (n x n), Mb (s x s; the series' second term buffer before M is formed).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_kkt_ric_bwd_xl(Shape sh, const double *__restrict__ E,
                                                       const double *__restrict__ c, const double *__restrict__ D,
                                                       const double *__restrict__ Hw, const double *__restrict__ hw,
                                                       const double *__restrict__ gw, const double *__restrict__ irho,
                                                       const int32_t *__restrict__ d_off,
                                                       const int32_t *__restrict__ y_off, double rd, double *rec,
                                                       int32_t *status, double *xws) {
    __shared__ double pv[XL_S], lp[XL_S], t1[XL_S], rq[XL_S], gq[XL_S], sinv[XL_S], s_red[4];
    __shared__ int s_bad;
    const int tid = threadIdx.x;
    const long long b = blockIdx.x;
    const int n = sh.n, m = sh.m, s = sh.s, N = sh.N, ps = sh.ps;
    const long long FS = (long long)s * m + m + n + (long long)n * n;
    const double *Eb = E + b * sh.perE;
    const double *cb = c + b * sh.perc;
    const double *Hb = Hw + b * sh.perHw;
    const double *hb = hw + b * sh.perh;
    const double *Db = D ? D + b * (long long)sh.ndD : nullptr;
    const double *gb = gw + b * (long long)sh.ny;
    const double *ib = irho ? irho + b * (long long)sh.ny : nullptr;
    double *RB = rec + b * N * FS;
    double *const XA = xws + b * kkt_xl_ws_doubles(sh);
    double *const Pt = XA + (long long)n * s, *const T0 = Pt + (long long)n * n, *const Mb = T0 + (long long)n * n;
    int fail_stage = -1;
    // ---- terminal: P_N = H~_N + D_N^T rho D_N, p_N = h~_N - D_N^T rho g_N ----
    {
        const int ncN = y_off[N + 1] - y_off[N];
        const double *DN = Db ? Db + d_off[N] : nullptr;
        if (tid == 0) s_bad = 0;
        for (int q = tid; q < ncN; q += 256) {
            rq[q] = 1.0 / ib[y_off[N] + q];
            gq[q] = gb[y_off[N] + q];
        }
        __syncthreads();
        const double *HN = Hb + (long long)N * ps;
        for (int q = tid; q < n * n; q += 256) {
            const int i = q % n, j = q / n;
            double v = HN[i >= j ? pidx(i, j, n) : pidx(j, i, n)];
            for (int r = 0; r < ncN; ++r) v = __builtin_fma(DN[r + i * ncN] * rq[r], DN[r + j * ncN], v);
            XA[q] = v;
            if (i == j && psd_bad(v)) s_bad = 1;
        }
        for (int i = tid; i < n; i += 256) {
            double v = hb[(long long)N * s + i];
            for (int r = 0; r < ncN; ++r) v = __builtin_fma(-DN[r + i * ncN] * rq[r], gq[r], v);
            pv[i] = v;
        }
        __syncthreads();
        if (s_bad) fail_stage = N;
    }
    for (int k = N - 1; k >= 0; --k) {
        double *Rk = RB + (long long)k * FS;
        const int nck = y_off[k + 1] - y_off[k];
        const double *Dk = Db ? Db + d_off[k] : nullptr;
        const double *Ek = Eb + (long long)k * n * s;
        // ---- P~ ----
        double f = 0.0;
        for (int q = tid; q < n * n; q += 256) f = __builtin_fma(XA[q], XA[q], f);
        const double e = rd * sqrt(xl_block_sum(f, s_red));  // block-uniform
        bool pt_ok = true;
        if (e > PDPLQR_KKT_NEUMANN_MAX) {
            for (int q = tid; q < n * n; q += 256) {
                const int i = q % n, j = q / n;
                Pt[q] = XA[q];
                T0[q] = __builtin_fma(rd, XA[q], i == j ? 1.0 : 0.0);
            }
            pt_ok = xl_llt(T0, n, n, n, T0, sinv);  // every pivot must be positive (m = n)
            xl_fsub(T0, n, n, Pt, n, n);
            xl_bsub_t(T0, n, n, Pt, n, n);
            for (int q = tid; q < n * n; q += 256) {  // symmetrise (pairs i > j)
                const int i = q % n, j = q / n;
                if (i > j) {
                    const double v = 0.5 * (Pt[i + j * n] + Pt[j + i * n]);
                    Pt[i + j * n] = v;
                    Pt[j + i * n] = v;
                }
            }
            __syncthreads();
        } else {
            for (int q = tid; q < n * n; q += 256) {
                Pt[q] = XA[q];
                T0[q] = XA[q];
            }
            double *cur = T0, *nxt = Mb;
            double ej = e;
            for (int j = 0; j < 8 && ej > 1e-16; ++j) {  // block-uniform
                xl_mm(nxt, n, XA, n, false, cur, n, false, n, n, n, nullptr, 0, -rd);
                for (int q = tid; q < n * n; q += 256) Pt[q] += nxt[q];
                double *const t = cur;
                cur = nxt;
                nxt = t;
                ej *= e;
            }
            __syncthreads();
        }
        // ---- record: p_{k+1}, P~_{k+1}; stage inputs ----
        for (int q = tid; q < n; q += 256) {
            Rk[s * m + m + q] = pv[q];
            t1[q] = __builtin_fma(-rd, pv[q], cb[(long long)k * n + q]);  // c - rho_dyn p
        }
        for (int q = tid; q < n * n; q += 256) Rk[s * m + m + n + q] = Pt[q];
        for (int q = tid; q < nck; q += 256) {
            rq[q] = 1.0 / ib[y_off[k] + q];
            gq[q] = gb[y_off[k] + q];
        }
        xl_mm(XA, n, Pt, n, false, Ek, n, false, n, s, n, nullptr, 0);  // G = P~ E~
        // lp = h~ + G^T (c - rho_dyn p) + E~^T p - D^T rho g;  M = H~ unpacked
        for (int j = tid; j < s; j += 256) {
            double a = hb[(long long)k * s + j];
            for (int i = 0; i < n; ++i) {
                a = __builtin_fma(XA[i + (long long)j * n], t1[i], a);
                a = __builtin_fma(Ek[i + (long long)j * n], pv[i], a);
            }
            if (k > 0 || j < m)
                for (int r = 0; r < nck; ++r) a = __builtin_fma(-Dk[r + j * nck] * rq[r], gq[r], a);
            lp[j] = a;
        }
        for (int q = tid; q < s * s; q += 256) {
            const int i = q % s, j = q / s;
            Mb[q] = Hb[(long long)k * ps + (i >= j ? pidx(i, j, s) : pidx(j, i, s))];
        }
        xl_mm(Mb, s, Ek, n, true, XA, n, false, s, s, n, Mb, s);  // M = H~ + E~^T G
        if (nck > 0) {  // + D^T rho D (lower; stage 0: the u columns only)
            for (int q = tid; q < s * s; q += 256) {
                const int i = q % s, j = q / s;
                if (i < j || (k == 0 && i >= m)) continue;
                double v = Mb[q];
                for (int r = 0; r < nck; ++r) v = __builtin_fma(Dk[r + i * nck] * rq[r], Dk[r + j * nck], v);
                Mb[q] = v;
            }
        }
        // ---- the m u-pivots (one barrier per pivot), L-form record ----
        bool ok = true;
        if (tid == 0) s_bad = 0;
        for (int j = 0; j < m; ++j) {
            __syncthreads();
            const double d = Mb[j + (long long)j * s];
            ok = ok && d > 0.0;
            const double inv = 1.0 / d, invs = rsqrt_f64(d);
            const double lpj = lp[j];
            for (int i = tid; i < s; i += 256) Rk[(long long)j * s + i] = i >= j ? Mb[i + (long long)j * s] * invs : 0.0;
            if (tid == 0) Rk[(long long)s * m + j] = lpj * invs;
            const int r = s - j - 1;
            for (int q = tid; q < r * r; q += 256) {
                const int i = j + 1 + q % r, l = j + 1 + q / r;
                if (l > i) continue;
                Mb[i + (long long)l * s] =
                    __builtin_fma(-Mb[i + (long long)j * s] * inv, Mb[l + (long long)j * s], Mb[i + (long long)l * s]);
            }
            for (int i = j + 1 + tid; i < s; i += 256) lp[i] = __builtin_fma(-Mb[i + (long long)j * s] * inv, lpj, lp[i]);
        }
        __syncthreads();
        // ---- P_k, p_k ----
        for (int q = tid; q < n * n; q += 256) {
            const int i = q % n, j = q / n;
            const int hi = i > j ? i : j, lo = i > j ? j : i;
            const double v = Mb[(m + hi) + (long long)(m + lo) * s];
            XA[q] = v;
            if (i == j && psd_bad(v)) s_bad = 1;
        }
        for (int q = tid; q < n; q += 256) pv[q] = lp[m + q];
        __syncthreads();
        if ((!ok || !pt_ok || s_bad) && fail_stage < 0) fail_stage = k;
    }
    if (tid == 0) status[b] = fail_stage < 0 ? 0 : fail_stage + 1;
}

// forward: the L-form rollout plus the lambda correction
// x+ = v - rho_dyn (P~ (v - rho_dyn p) + p), v = A x + B u + c (k_kkt_ric_fwd_wide
// on a 256-thread block); the solve uses the sum of the x0s since
// update_problem_data, ws[0]'s x part is the call's x0 (kkt.hpp:207-222)
__global__ __launch_bounds__(256) void k_kkt_ric_fwd_xl(Shape sh, const double *__restrict__ E,
                                                       const double *__restrict__ c, const double *__restrict__ RB,
                                                       const double *__restrict__ x0, double *__restrict__ x0acc,
                                                       double *__restrict__ ws, double rd) {
    __shared__ double w[XL_S], v[XL_S], sz[XL_S], sx0[XL_S];
    const int tid = threadIdx.x;
    const long long b = blockIdx.x;
    const int n = sh.n, m = sh.m, N = sh.N, s = sh.s;
    const long long FS = (long long)s * m + m + n + (long long)n * n;
    const double *Eb = E + b * sh.perE;
    const double *cb = c + b * sh.perc;
    const double *Rb = RB + b * N * FS;
    double *wb = ws + b * sh.perh;
    for (int q = tid; q < n; q += 256) {
        const double x = x0[b * n + q];
        const double xa = x0acc[b * n + q] + x;
        x0acc[b * n + q] = xa;
        w[m + q] = xa;
        sx0[q] = x;
    }
    __syncthreads();
    for (int k = 0; k < N; ++k) {
        const double *Fk = Rb + (long long)k * FS;
        for (int j = tid; j < m; j += 256) {  // v = -(lu' + Lxu^T x)
            double a = Fk[(long long)s * m + j];
            for (int i = 0; i < n; ++i) a = __builtin_fma(Fk[(long long)j * s + m + i], w[m + i], a);
            v[j] = -a;
        }
        for (int j = m - 1; j >= 0; --j) {  // u = Luu^{-T} v
            __syncthreads();
            const double uj = v[j] / Fk[(long long)j * s + j];
            __syncthreads();
            for (int i = tid; i < j; i += 256) v[i] = __builtin_fma(-Fk[(long long)i * s + j], uj, v[i]);
            if (tid == 0) v[j] = uj;
        }
        __syncthreads();
        for (int j = tid; j < m; j += 256) w[j] = v[j];
        __syncthreads();
        for (int q = tid; q < s; q += 256) wb[(long long)k * s + q] = q < m ? w[q] : (k == 0 ? sx0[q - m] : w[q]);
        const double *pk = Fk + (long long)s * m + m, *Ptk = pk + n;
        const double *Ek = Eb + (long long)k * n * s;
        double a = 0.0;  // n < 256: one state row per thread
        if (tid < n) {
            a = cb[(long long)k * n + tid];
            for (int j = 0; j < s; ++j) a = __builtin_fma(Ek[tid + (long long)j * n], w[j], a);
            sz[tid] = __builtin_fma(-rd, pk[tid], a);  // v - rho_dyn p
        }
        __syncthreads();
        if (tid < n) {
            double y = 0.0;
            for (int t = 0; t < n; ++t) y = __builtin_fma(Ptk[tid + (long long)t * n], sz[t], y);
            a = __builtin_fma(-rd, y + pk[tid], a);
        }
        __syncthreads();
        if (tid < n) w[m + tid] = a;
        __syncthreads();
    }
    for (int q = tid; q < n; q += 256) wb[(long long)N * s + q] = w[m + q];
}

int launch_riccati_backward_xl(const RiccatiArgs &a, hipStream_t st) {
    if (!xl_shape(a.sh) || !a.xl_ws) return PDPLQR_ERR_UNSUPPORTED;
    hipLaunchKernelGGL(k_riccati_bwd_xl, dim3((unsigned)a.sh.batch), dim3(256), 0, st, a);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

int launch_riccati_backward_nofact_xl(const RiccatiArgs &a, hipStream_t st) {
    if (!xl_shape(a.sh) || !a.xl_ws || !a.Lc || !a.lpc) return PDPLQR_ERR_UNSUPPORTED;
    hipLaunchKernelGGL(k_riccati_bwd_nofact_xl, dim3((unsigned)a.sh.batch), dim3(256), 0, st, a);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

int launch_riccati_forward_xl(const Shape &sh, const double *E, const double *c, const double *FR, const double *x0,
                              double *ws, hipStream_t st) {
    if (!xl_shape(sh)) return PDPLQR_ERR_UNSUPPORTED;
    hipLaunchKernelGGL(k_riccati_fwd_xl, dim3((unsigned)sh.batch), dim3(256), 0, st, sh, E, c, FR, x0, ws);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

int launch_kkt_xl_backward(const Shape &sh, const double *E, const double *c, const double *D, const double *Hw,
                           const double *hw, const double *gw, const double *irho, const int32_t *d_off,
                           const int32_t *y_off, double rho_dyn, double *rec, int32_t *status, double *xws,
                           hipStream_t st) {
    if (!xl_shape(sh) || !xws) return PDPLQR_ERR_UNSUPPORTED;
    hipLaunchKernelGGL(k_kkt_ric_bwd_xl, dim3((unsigned)sh.batch), dim3(256), 0, st, sh, E, c,
                       sh.ndD > 0 ? D : nullptr, Hw, hw, gw, sh.ny > 0 ? irho : nullptr, d_off, y_off, rho_dyn, rec,
                       status, xws);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

int launch_kkt_xl_forward(const Shape &sh, const double *E, const double *c, const double *rec, const double *x0,
                          double *x0acc, double *ws, double rho_dyn, hipStream_t st) {
    if (!xl_shape(sh)) return PDPLQR_ERR_UNSUPPORTED;
    hipLaunchKernelGGL(k_kkt_ric_fwd_xl, dim3((unsigned)sh.batch), dim3(256), 0, st, sh, E, c, rec, x0, x0acc, ws,
                       rho_dyn);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

}  // namespace pdplqr
