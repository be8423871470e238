// kernels_parallel.hip -- LQRParallelSolver on MI355X: horizon segments,
// associative segment combine, segment rollout.
//
// Restates reference lqr_solver_parallel.hpp:64-238, lqr_kernel_parallel.hpp:52-218
// and condensed_system.hpp:8-299:
//   * k_seg_bwd<T>: one wavefront per (problem, segment) runs the segment's
//     Riccati recursion from a zero terminal (the real terminal for the last
//     segment, lqr_kernel_parallel.hpp:52-67) and accumulates the segment
//     element (F, C, f) plus G_k (step_with_factorization, :88-136).  It exports
//     e = (F, C, f, P = Lxx Lxx^T, p) as update_segment_data does
//     (lqr_solver_parallel.hpp:182-187, condensed_system.hpp:64-74).
//   * k_seg_scan: one Hillis-Steele round of the prefix and suffix scans of the
//     elements under the associative operator
//         Z = (I + C_a P_b)^{-1}, F = F_b Z F_a, C = F_b Z C_a F_b^T + C_b,
//         f = F_b Z (f_a - C_a p_b) + f_b, P = P_a + F_a^T P_b Z F_a,
//         p = p_a + F_a^T Z^T (p_b + P_b f_a).
//     The reference folds the same operator serially on the master thread
//     (condensed_system.hpp:82-137 LU form, :203-290 Cholesky form); here
//     P_b Z = Y = R (I + R^T C_a R)^{-1} R^T with R = chol(P_b), an SPD solve,
//     evaluated on MFMA tiles (combine_tiles.hpp).
//   * k_seg_boundary: x_hat_i = (I + C_pre P_suf)^{-1}(F_pre x0 + f_pre - C_pre p_suf)
//     and u_hat_i = p_suf(i+1) + P_suf(i+1) x_hat_{i+1} (condensed forward).
//   * the rollout reuses k_riccati_fwd with the G_k u_hat coupling
//     (lqr_kernel_parallel.hpp:195-198).
#define PDPLQR_COMB_PROFILE_TU 1  // the combine phase marks live in this translation unit
#include "combine_tiles.hpp"
#include "device_common.hpp"
#include "parallel.hpp"

namespace pdplqr {

#ifdef PDPLQR_COMB_PROFILE
__device__ unsigned long long g_comb_t[1024 * 16];
#endif

// Element views: [F | C | f | P | p] packed contiguously (3 n^2 + 2 n doubles)
struct Elem {
    double *F, *C, *f, *P, *p;
};

__device__ __forceinline__ Elem elem_view(double *base, int n) {
    Elem e;
    e.F = base;
    e.C = base + n * n;
    e.f = base + 2 * n * n;
    e.P = base + 2 * n * n + n;
    e.p = base + 3 * n * n + n;
    return e;
}

__device__ __forceinline__ void elem_copy(double *dst, const double *src, int n, int lane) {
    const int sz = 3 * n * n + 2 * n;
    for (int q = lane; q < sz; q += 64) dst[q] = src[q];
}

// ---------------------------------------------------------------------------
// Segment backward: the reference's reduction_per_thread (lqr_solver_parallel.hpp:164-188)
// ---------------------------------------------------------------------------
// Element-recursion scratch of one segment wave, carved from dynamic LDS and
// sized by the actual n, m (fixed 16T x 16T arrays would cap T = 2 at one wave
// per CU).
struct SegView {
    double *F, *C, *Ft, *Ct, *Acl;  // n x n (ld n)
    double *Es, *FB, *K, *G;        // E (n x s), F_next B (n x m), K, G (m x n)
    double *f, *ft, *cv, *dv;       // n, n, n, m
};

__host__ __device__ inline size_t seg_smem_doubles(int n, int m) {
    const int s = n + m;
    return 5 * (size_t)n * n + (size_t)n * s + 3 * (size_t)n * m + 3 * (size_t)n + m;
}

__device__ __forceinline__ SegView seg_view(double *dyn, int n, int m) {
    const int s = n + m, nn = n * n;
    SegView v;
    v.F = dyn;
    v.C = v.F + nn;
    v.Ft = v.C + nn;
    v.Ct = v.Ft + nn;
    v.Acl = v.Ct + nn;
    v.Es = v.Acl + nn;
    v.FB = v.Es + n * s;
    v.K = v.FB + n * m;
    v.G = v.K + m * n;
    v.f = v.G + m * n;
    v.ft = v.f + n;
    v.cv = v.ft + n;
    v.dv = v.cv + n;
    return v;
}

template <int T>
__global__ __launch_bounds__(64) void k_seg_bwd(SegArgs A) {
    constexpr int LD = 16 * T + 1;
    __shared__ BwdSmem<T> sm;
    extern __shared__ double seg_dyn[];
    const int lane = threadIdx.x, g = lane >> 4, c = lane & 15;
    const Shape &sh = A.sh;
    const int n = sh.n, m = sh.m, s = sh.s, S = A.S;
    const SegView ss = seg_view(seg_dyn, n, m);
    const long long b = blockIdx.x / S;
    const int seg = blockIdx.x % S;
    const int N0 = A.seg_start[seg], N1 = N0 + A.seg_len[seg];
    const bool last = (seg == S - 1) && A.last_is_terminal;
    const long long frs = (long long)s * m + m;
    const double *Eb = A.E + b * sh.perE;
    const double *cb = A.c + b * sh.perc;
    const double *Hb = A.Hw + b * sh.perHw;
    const double *hb = A.hw + b * sh.perh;
    double *FRb = A.FR + b * sh.perKD;
    double *Gb = A.G + b * (long long)sh.N * m * n;
    double *Lcb = A.Lc ? A.Lc + b * sh.perHw : nullptr;
    double *lpb = A.lpc ? A.lpc + b * sh.perh : nullptr;
    int fail_stage = -1;

    // ---- segment terminal (lqr_kernel_parallel.hpp:52-67) ----
    if (last) {
        d4 M[T][T];
        load_M<T>(M, Hb + (long long)sh.N * sh.ps, n, m, m, s, g, c);
        double lpr[T][4];
        const bool okN = chol_tiles<T>(M, lpr, sm.col, sm.inv, sm.luq, m, s, m, false, g, c);
        finalize_L<T>(M, sm.inv, m, s, g, c);
        if (!okN) fail_stage = sh.N;
        store_L_lds<T>(M, sm.L, g, c);
        if (lane < n) {
            const double v = hb[(long long)sh.N * s + lane];
            sm.pv[lane] = v;
            if (lpb) lpb[(long long)sh.N * s + lane] = v;
        }
        if (Lcb)
#pragma unroll
            for (int a = 0; a < T; ++a)
#pragma unroll
                for (int bt = 0; bt < T; ++bt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int i = 16 * a + 4 * r + g, j = 16 * bt + c;
                        if (j >= m && i >= j && i < s)
                            Lcb[(long long)sh.N * sh.ps + pidx(i - m, j - m, n)] = M[a][bt][r];
                    }
    } else {  // dummy: L = 0, lp = 0, F = I, C = 0, f = 0
        for (int q = lane; q < (16 * T) * LD; q += 64) sm.L[q] = 0.0;
        for (int q = lane; q < 16 * T; q += 64) sm.pv[q] = 0.0;
        for (int q = lane; q < n * n; q += 64) {
            ss.F[q] = (q % n == q / n) ? 1.0 : 0.0;
            ss.C[q] = 0.0;
        }
        for (int q = lane; q < n; q += 64) ss.f[q] = 0.0;
    }
    wave_sync();

    for (int k = N1 - 1; k >= N0; --k) {
        StageIn<T> cur;
        load_stage<T>(cur, Eb + (long long)k * n * s, cb + (long long)k * n, Hb + (long long)k * sh.ps,
                      hb + (long long)k * s, n, s, g, c);
        d4 M[T][T];
        double lpr[T][4];
        const bool okk = riccati_stage<T>(sm, cur, M, lpr, n, m, s, g, c);
        if (!okk && fail_stage < 0) fail_stage = k;
        double *FRk = FRb + (long long)k * frs;
#pragma unroll
        for (int a = 0; a < T; ++a)
#pragma unroll
            for (int bt = 0; bt < T; ++bt) {
                const int jc = 16 * bt + c;
                if (jc < m)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int i = 16 * a + 4 * r + g;
                        if (i < s) FRk[jc * s + i] = M[a][bt][r];
                    }
            }
        if (lane < m) FRk[(long long)s * m + lane] = sm.luq[lane];
        if (lpb) {
            if (lane < m) lpb[(long long)k * s + lane] = sm.luq[lane];
            if (lane < n) lpb[(long long)k * s + m + lane] = sm.pv[lane];
        }
        if (Lcb)
#pragma unroll
            for (int a = 0; a < T; ++a)
#pragma unroll
                for (int bt = 0; bt < T; ++bt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int i = 16 * a + 4 * r + g, j = 16 * bt + c;
                        if (i >= j && i < s) Lcb[(long long)k * sh.ps + pidx(i, j, s)] = M[a][bt][r];
                    }
        if (last) continue;
        // ---- segment element recursion (lqr_kernel_parallel.hpp:97-135) ----
        const double *Ek = Eb + (long long)k * n * s;
        const double *L = sm.L;  // L_k, padded, ld LD
        for (int q = lane; q < n * s; q += 64) ss.Es[q] = Ek[q];
        if (lane < n) ss.cv[lane] = cb[(long long)k * n + lane];
        wave_sync();
        // K = -Luu^{-T} Lxu^T (:105,107) and d = -Luu^{-T} lu (:106,108)
        if (lane <= n) {
            for (int i = m - 1; i >= 0; --i) {
                double v = (lane < n) ? -L[(m + lane) + i * LD] : -sm.luq[i];
                for (int j = i + 1; j < m; ++j)
                    v -= L[j + i * LD] * ((lane < n) ? ss.K[j + lane * m] : ss.dv[j]);
                v /= L[i + i * LD];
                if (lane < n) ss.K[i + lane * m] = v;
                else ss.dv[i] = v;
            }
        }
        // FB = F_next B (n x m): B^T F_next^T of :126 transposed
        for (int q = lane; q < n * m; q += 64) {
            const int t = q % n, i = q / n;
            double acc = 0.0;
            for (int r = 0; r < n; ++r) acc = __builtin_fma(ss.F[t + r * n], ss.Es[r + i * n], acc);
            ss.FB[t + i * n] = acc;
        }
        wave_sync();
        // G = -Luu^{-1} B^T F_next^T (:127-128): column t of G from row t of FB
        if (lane < n) {
            for (int i = 0; i < m; ++i) {
                double v = -ss.FB[lane + i * n];
                for (int j = 0; j < i; ++j) v -= L[i + j * LD] * ss.G[j + lane * m];
                v /= L[i + i * LD];
                ss.G[i + lane * m] = v;
                Gb[(long long)k * m * n + i + lane * m] = v;
            }
        }
        // Acl = A + B K (:129) ; ft = c + B d (:132)
        for (int q = lane; q < n * n; q += 64) {
            const int t = q % n, j = q / n;
            double acc = ss.Es[t + (m + j) * n];
            for (int i = 0; i < m; ++i) acc = __builtin_fma(ss.Es[t + i * n], ss.K[i + j * m], acc);
            ss.Acl[q] = acc;
        }
        if (lane < n) {
            double acc = ss.cv[lane];
            for (int i = 0; i < m; ++i) acc = __builtin_fma(ss.Es[lane + i * n], ss.dv[i], acc);
            ss.ft[lane] = acc;
        }
        wave_sync();
        // F = F_next Acl (:130); f = F_next ft + f_next (:133); C = C_next + G^T G (:134)
        for (int q = lane; q < n * n; q += 64) {
            const int t = q % n, j = q / n;
            double acc = 0.0;
            for (int r = 0; r < n; ++r) acc = __builtin_fma(ss.F[t + r * n], ss.Acl[r + j * n], acc);
            ss.Ft[q] = acc;
            double cc = 0.0;
            for (int i = 0; i < m; ++i) cc = __builtin_fma(ss.G[i + t * m], ss.G[i + j * m], cc);
            ss.Ct[q] = ss.C[q] + cc;
        }
        double fnew = 0.0;
        if (lane < n) {
            double acc = 0.0;
            for (int r = 0; r < n; ++r) acc = __builtin_fma(ss.F[lane + r * n], ss.ft[r], acc);
            fnew = acc + ss.f[lane];
        }
        wave_sync();
        for (int q = lane; q < n * n; q += 64) {
            ss.F[q] = ss.Ft[q];
            ss.C[q] = ss.Ct[q];
        }
        if (lane < n) ss.f[lane] = fnew;
        wave_sync();
    }
    // ---- export the element (update_segment_data, lqr_solver_parallel.hpp:182-187) ----
    double *eo = A.elem + (b * S + seg) * (long long)(3 * n * n + 2 * n);
    Elem e = elem_view(eo, n);
    for (int q = lane; q < n * n; q += 64) {
        const int i = q % n, j = q / n;
        double acc = 0.0;
        for (int t = 0; t < n; ++t) acc = __builtin_fma(sm.L[(m + i) + (m + t) * LD], sm.L[(m + j) + (m + t) * LD], acc);
        e.P[q] = acc;  // P = Lxx Lxx^T (condensed_system.hpp:69,188)
        e.F[q] = last ? 0.0 : ss.F[q];
        e.C[q] = last ? 0.0 : ss.C[q];
    }
    if (lane < n) {
        e.f[lane] = last ? 0.0 : ss.f[lane];
        e.p[lane] = sm.pv[lane];
    }
    if (lane == 0) A.seg_status[b * S + seg] = fail_stage < 0 ? 0 : fail_stage + 1;
}

// ---------------------------------------------------------------------------
// Segment backward without factorization: reduction_without_factorization
// (lqr_solver_parallel.hpp:190-211) with ParallelLQRKernel::
// step_without_factorization (lqr_kernel_parallel.hpp:139-168).  The cached
// factors L_k of the last factorising backward are reused; only the linear
// terms change: lp_k, lu'_k (into the rollout record) and the element vectors
// p, f.  f = F_{k+1}(c + B d) + f_{k+1} (:160-165) is evaluated as what it
// is -- the end state of the segment's closed-loop rollout from x = 0 under
// the new feed-forward d = -Luu^{-T} lu' -- so no per-stage F_k is stored.
// F, C, P of the element are unchanged (update_segment_data(p, f, id),
// condensed_system.hpp:76-80).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_seg_bwd_nofact(SegArgs A) {
    constexpr int P = 32;
    __shared__ double Lk[P * P];  // this stage's L (dense, ld s)
    __shared__ double Ln[P * P];  // next stage's Lxx (ld n)
    __shared__ double cvec[P], va[P], vb[P], lp[P], pn[P], xs[P], us[P];
    const int lane = threadIdx.x;
    const Shape &sh = A.sh;
    const int n = sh.n, m = sh.m, s = sh.s, S = A.S;
    const long long b = blockIdx.x / S;
    const int seg = blockIdx.x % S;
    const int N0 = A.seg_start[seg], N1 = N0 + A.seg_len[seg];
    const bool last = (seg == S - 1) && A.last_is_terminal;
    const long long frs = (long long)s * m + m;
    const double *Eb = A.E + b * sh.perE;
    const double *cb = A.c + b * sh.perc;
    const double *hb = A.hw + b * sh.perh;
    double *FRb = A.FR + b * sh.perKD;
    const double *Lcb = A.Lc + b * sh.perHw;
    double *lpb = A.lpc ? A.lpc + b * sh.perh : nullptr;
    // segment terminal: the real one (lqr_kernel.hpp:94-101) or the dummy L = 0, lp = 0
    if (lane < n) pn[lane] = last ? hb[(long long)sh.N * s + lane] : 0.0;
    if (last && lpb && lane < n) lpb[(long long)sh.N * s + lane] = pn[lane];
    for (int q = lane; q < n * n; q += 64) {
        const int i = q % n, j = q / n;
        Ln[q] = (last && i >= j) ? Lcb[(long long)sh.N * sh.ps + pidx(i, j, n)] : 0.0;
    }
    wave_sync();
    for (int k = N1 - 1; k >= N0; --k) {
        const double *Ek = Eb + (long long)k * n * s;
        for (int q = lane; q < s * s; q += 64) {
            const int i = q % s, j = q / s;
            Lk[q] = (i >= j) ? Lcb[(long long)k * sh.ps + pidx(i, j, s)] : 0.0;
        }
        if (lane < n) cvec[lane] = cb[(long long)k * n + lane];
        wave_sync();
        if (lane < n) {  // Pb_tmp = Lxx_next^T c
            double a = 0.0;
            for (int t = lane; t < n; ++t) a += Ln[t + lane * n] * cvec[t];
            va[lane] = a;
        }
        wave_sync();
        if (lane < n) {  // Pb = Lxx_next Pb_tmp + p_next
            double a = 0.0;
            for (int t = 0; t <= lane; ++t) a += Ln[lane + t * n] * va[t];
            vb[lane] = a + pn[lane];
        }
        wave_sync();
        if (lane < s) {  // lp = h~ + E^T Pb
            double a = 0.0;
            for (int t = 0; t < n; ++t) a += Ek[t + lane * n] * vb[t];
            lp[lane] = hb[(long long)k * s + lane] + a;
        }
        wave_sync();
        if (lane == 0) {  // lu <- Luu^{-1} lu
            for (int i = 0; i < m; ++i) {
                double v = lp[i];
                for (int j = 0; j < i; ++j) v -= Lk[i + j * s] * lp[j];
                lp[i] = v / Lk[i + i * s];
            }
        }
        wave_sync();
        if (lane < n) {  // p -= Lxu lu
            double a = 0.0;
            for (int i = 0; i < m; ++i) a += Lk[(m + lane) + i * s] * lp[i];
            const double pnew = lp[m + lane] - a;
            lp[m + lane] = pnew;
            pn[lane] = pnew;
        }
        wave_sync();
        if (lane < m) FRb[(long long)k * frs + (long long)s * m + lane] = lp[lane];
        if (lpb && lane < s) lpb[(long long)k * s + lane] = lp[lane];
        for (int q = lane; q < n * n; q += 64) {
            const int i = q % n, j = q / n;
            Ln[q] = Lk[(m + i) + (m + j) * s];
        }
        wave_sync();
    }
    double *eo = A.elem + (b * S + seg) * (long long)(3 * n * n + 2 * n);
    Elem e = elem_view(eo, n);
    if (lane < n) e.p[lane] = pn[lane];
    if (last) {
        if (lane < n) e.f[lane] = 0.0;
        return;
    }
    // f: closed-loop rollout of the segment from x = 0 (u = -Luu^{-T}(lu' + Lxu^T x))
    if (lane < n) xs[lane] = 0.0;
    wave_sync();
    for (int k = N0; k < N1; ++k) {
        const double *Ek = Eb + (long long)k * n * s;
        const double *FRk = FRb + (long long)k * frs;  // [L(:, 0:m) | lu']
        if (lane < m) {
            double v = FRk[(long long)s * m + lane];
            for (int t = 0; t < n; ++t) v += FRk[lane * s + m + t] * xs[t];
            va[lane] = v;
        }
        wave_sync();
        if (lane == 0)
            for (int i = m - 1; i >= 0; --i) {
                double v = va[i];
                for (int j = i + 1; j < m; ++j) v += FRk[i * s + j] * us[j];  // Luu[j][i] u_j
                us[i] = -v / FRk[i * s + i];
            }
        wave_sync();
        double xn = 0.0;
        if (lane < n) {
            xn = cb[(long long)k * n + lane];
            for (int j = 0; j < m; ++j) xn += Ek[lane + j * n] * us[j];
            for (int t = 0; t < n; ++t) xn += Ek[lane + (m + t) * n] * xs[t];
        }
        wave_sync();
        if (lane < n) xs[lane] = xn;
        wave_sync();
    }
    if (lane < n) e.f[lane] = xs[lane];
}

int launch_seg_backward_nofact(const SegArgs &a, hipStream_t st) {
    if (a.sh.s > 32 || !a.Lc) {
        set_error("PARALLEL backward_without_factorization needs keep_factors = 1 and n + m <= 32");
        return PDPLQR_ERR_UNSUPPORTED;
    }
    hipLaunchKernelGGL(k_seg_bwd_nofact, dim3((unsigned)(a.sh.batch * a.S)), dim3(64), 0, st, a);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

// ---------------------------------------------------------------------------
// One Hillis-Steele round: inclusive prefix (dir 0) or suffix (dir 1) scan.
// ---------------------------------------------------------------------------
// Both operand elements are prefetched into LDS with one LDS-DMA burst (a
// single HBM/L2 latency) before the combine reads them.
// (es = 3 n^2 + 2 n is odd for odd n: the last double goes by a plain copy;
// the caller waits on vmcnt and then wave_sync()s.)
template <int T>
__device__ __forceinline__ void elem_prefetch(double *dst, const double *src, int es, int lane) {
    const int chunks = es / 2;
    for (int q = 0; q * 64 < chunks; ++q) {
        const int ch = q * 64 + lane;
        if (ch < chunks) dma16(src + 2 * ch, dst + 2 * q * 64);
    }
    if ((es & 1) && lane == 0) dst[es - 1] = src[es - 1];
}

template <int T>
__global__ __launch_bounds__(64) void k_seg_scan(ScanArgs A) {
    __shared__ CombSmem<T> sm;
    extern __shared__ __attribute__((aligned(16))) double ebuf[];  // 2 elements (launcher: elems_smem(n, 2))
    const int lane = threadIdx.x;
    const int n = A.n, S = A.S, d = A.dist;
    const int es = 3 * n * n + 2 * n;
    const long long b = blockIdx.x / (2 * S);
    const int rem = blockIdx.x % (2 * S);
    const int dir = rem / S, i = rem % S;
    const double *in = (dir == 0 ? A.pre_in : A.suf_in) + b * (long long)S * es;
    double *out = (dir == 0 ? A.pre_out : A.suf_out) + b * (long long)S * es;
    int ia, ib;
    if (dir == 0) {  // pre_i = pre_{i-d} (x) pre_i
        if (i - d < 0) {
            elem_copy(out + (long long)i * es, in + (long long)i * es, n, lane);
            return;
        }
        ia = i - d; ib = i;
    } else {  // suf_i = suf_i (x) suf_{i+d}
        if (i + d >= S) {
            elem_copy(out + (long long)i * es, in + (long long)i * es, n, lane);
            return;
        }
        ia = i; ib = i + d;
    }
    // Both directions need full elements: the next round's combine reads the
    // right operand's P, p (Z = (I + C_a P_b)^{-1}).  A suffix ending at the
    // real terminal has F = C = f = 0.
    const int esp = (es + 1) & ~1;  // 16-byte aligned second buffer
    elem_prefetch<T>(ebuf, in + (long long)ia * es, es, lane);
    elem_prefetch<T>(ebuf + esp, in + (long long)ib * es, es, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
    const bool ok = tcombine<T>(out + (long long)i * es, ebuf, ebuf + esp, n, true, true, sm, lane);
    if (!ok && lane == 0) atomicOr(A.flag, 1);
}

// ---------------------------------------------------------------------------
// Boundary states: x_hat_i from the exclusive prefix (optionally left-folded
// with a global prefix) and the suffix (optionally right-folded with a global
// suffix); u_hat_i in a second pass.
// ---------------------------------------------------------------------------
template <int T>
__global__ __launch_bounds__(64) void k_seg_xhat(BoundaryArgs A) {
    extern __shared__ __attribute__((aligned(16))) double dyn[];
    __shared__ CombSmem<T> sm;
    const int lane = threadIdx.x;
    const int n = A.n, S = A.S;
    const int es = 3 * n * n + 2 * n;
    const long long b = blockIdx.x / (S + 1);
    const int i = blockIdx.x % (S + 1);  // i == S: state after the last segment (shard mode)
    double *pre = dyn, *suf = dyn + es, *tmp = dyn + 2 * es;  // tmp + es: combine output
    const double *preb = A.pre + b * (long long)S * es;
    const double *sufb = A.suf + b * (long long)S * es;
    // prefix before segment i: global_left (x) pre_{i-1}
    if (i == 0) {
        if (A.left) elem_copy(pre, A.left + b * (long long)es, n, lane);
        else {
            Elem e = elem_view(pre, n);
            for (int q = lane; q < n * n; q += 64) {
                e.F[q] = (q % n == q / n) ? 1.0 : 0.0;
                e.C[q] = 0.0;
                e.P[q] = 0.0;
            }
            for (int q = lane; q < n; q += 64) { e.f[q] = 0.0; e.p[q] = 0.0; }
        }
        wave_sync();
    } else {
        if (A.left) {
            elem_copy(tmp, A.left + b * (long long)es, n, lane);
            elem_copy(suf, preb + (long long)(i - 1) * es, n, lane);  // scratch
            wave_sync();
            tcombine<T>(pre, tmp, suf, n, true, false, sm, lane);
        } else {
            elem_copy(pre, preb + (long long)(i - 1) * es, n, lane);
            wave_sync();
        }
    }
    // suffix from segment i: suf_i (x) global_right ; for i == S only global_right
    bool have_suf = true;
    if (i < S) {
        if (A.right) {
            elem_copy(tmp, sufb + (long long)i * es, n, lane);
            elem_copy(suf, A.right + b * (long long)es, n, lane);
            wave_sync();
            double *o = tmp + es;  // scratch beyond tmp: pre | suf | tmp | tmp2 fit in 4 es (see launcher)
            tcombine<T>(o, tmp, suf, n, false, true, sm, lane);
            elem_copy(suf, o, n, lane);
            wave_sync();
        } else {
            elem_copy(suf, sufb + (long long)i * es, n, lane);
            wave_sync();
        }
    } else {
        if (A.right) {
            elem_copy(suf, A.right + b * (long long)es, n, lane);
            wave_sync();
        } else {
            have_suf = false;
        }
    }
    Elem P = elem_view(pre, n), Sf = elem_view(suf, n);
    double *x0 = tmp;  // reuse
    if (lane < n) x0[lane] = A.x0[b * n + lane];
    wave_sync();
    // rhs = F_pre x0 + f_pre - C_pre p_suf
    double *rhs = tmp + es;  // scratch (the fold output is consumed)
    for (int r = lane; r < n; r += 64) {
        double acc = P.f[r];
        for (int k = 0; k < n; ++k) acc = __builtin_fma(P.F[r + k * n], x0[k], acc);
        if (have_suf)
            for (int k = 0; k < n; ++k) acc = __builtin_fma(-P.C[r + k * n], Sf.p[k], acc);
        rhs[r] = acc;
    }
    wave_sync();
    double *xh = A.xhat + (b * (long long)(S + 1) + i) * n;
    if (have_suf) {
        // x = (I + C_pre P_suf)^{-1} rhs = Z rhs with Z from comb_core(C_pre, P_suf)
        constexpr int PL = 16 * T + 1;
        WM<T> Ca, Y, Z, Zt;
        wm_load(Ca, P.C, n, n, false, 0.0, lane >> 4, lane & 15);
        const bool ok = comb_core(Y, Z, Zt, Ca, Sf.P, n, sm, lane);
        if (!ok && lane == 0) atomicOr(A.flag, 2);
        wm_store(Z, sm.A, PL, n, lane >> 4, lane & 15);
        wave_sync();
        lds_mv(sm.v2, sm.A, PL, false, rhs, nullptr, 1.0, n, lane);
        wave_sync();
        if (lane < n) xh[lane] = sm.v2[lane];
        // costate at the start of segment i: lambda = P_suf x + p_suf (stored for u_hat_{i-1})
        double *lam = A.lam + (b * (long long)(S + 1) + i) * n;
        wave_sync();
        for (int r = lane; r < n; r += 64) {
            double acc = Sf.p[r];
            for (int k = 0; k < n; ++k) acc = __builtin_fma(Sf.P[r + k * n], sm.v2[k], acc);
            lam[r] = acc;
        }
    } else {
        if (lane < n) xh[lane] = rhs[lane];
    }
}

// Resident segment waves the device can hold for this shape: CUs x the
// segment backward's occupancy.  Refining the horizon beyond that adds scan
// rounds without adding parallelism.
int seg_backward_slots(const Shape &sh, int device) {
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
    const size_t smem = seg_smem_doubles(sh.n, sh.m) * sizeof(double);
    hipError_t e = sh.s <= 16 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_seg_bwd<1>, 64, smem)
                              : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_seg_bwd<2>, 64, smem);
    if (e != hipSuccess || per <= 0) per = 1;
    return cus * per;
}

// Resident scan waves (one combine each) the device holds for this shape.
int seg_scan_slots(const Shape &sh, int device) {
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
    const size_t smem = 2 * (size_t)((3 * sh.n * sh.n + 2 * sh.n + 1) & ~1) * sizeof(double);
    hipError_t e = sh.n <= 16 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_seg_scan<1>, 64, smem)
                              : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_seg_scan<2>, 64, smem);
    if (e != hipSuccess || per <= 0) per = 1;
    return cus * per;
}

int launch_seg_backward(const SegArgs &a, hipStream_t st) {
    const dim3 grid((unsigned)(a.sh.batch * a.S)), blk(64);
    const size_t smem = seg_smem_doubles(a.sh.n, a.sh.m) * sizeof(double);
    if (a.sh.s <= 16) hipLaunchKernelGGL(k_seg_bwd<1>, grid, blk, smem, st, a);
    else if (a.sh.s <= 32) hipLaunchKernelGGL(k_seg_bwd<2>, grid, blk, smem, st, a);
    else {
        set_error("parallel solver: n + m > 32 is not supported by this build");
        return PDPLQR_ERR_UNSUPPORTED;
    }
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

static size_t elems_smem(int n, int elems) { return (size_t)elems * (3 * n * n + 2 * n) * sizeof(double); }

static int tile_order(int n) { return n <= 16 ? 1 : (n <= 32 ? 2 : 0); }

int launch_seg_scan(const ScanArgs &a, int batch, hipStream_t st) {
    const dim3 grid((unsigned)(batch * 2 * a.S)), blk(64);
    const int T = tile_order(a.n);
    const size_t smem = 2 * (size_t)((3 * a.n * a.n + 2 * a.n + 1) & ~1) * sizeof(double);
    if (T == 1) hipLaunchKernelGGL(k_seg_scan<1>, grid, blk, smem, st, a);
    else if (T == 2) hipLaunchKernelGGL(k_seg_scan<2>, grid, blk, smem, st, a);
    else return PDPLQR_ERR_UNSUPPORTED;
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

int launch_seg_xhat(const BoundaryArgs &a, int batch, hipStream_t st) {
    const dim3 grid((unsigned)(batch * (a.S + 1))), blk(64);
    const int T = tile_order(a.n);
    if (T == 1) hipLaunchKernelGGL(k_seg_xhat<1>, grid, blk, elems_smem(a.n, 4), st, a);
    else if (T == 2) hipLaunchKernelGGL(k_seg_xhat<2>, grid, blk, elems_smem(a.n, 4), st, a);
    else return PDPLQR_ERR_UNSUPPORTED;
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

// Combine a short list of elements on one wave (the per-rank fold of the
// horizon-sharded solve): out_pre = e_0 (x) ... (x) e_{r-1} (identity if r = 0),
// out_suf = e_{r+1} (x) ... (x) e_{R-1} (P = p = 0 marker when r = R-1).
template <int T>
__global__ __launch_bounds__(64) void k_fold_shards(const double *elems_all, int R, int r, int n, int batch,
                                                    double *out_pre_all, double *out_suf_all, int *has_suf, int *flag) {
    extern __shared__ __attribute__((aligned(16))) double dyn[];
    __shared__ CombSmem<T> sm;
    const int lane = threadIdx.x;
    const int es = 3 * n * n + 2 * n;
    const long long b = blockIdx.x;
    // element j of problem b: elems_all[(j * batch + b) * es]; outputs [b][es]
    const double *elems = elems_all + b * es;
    const long long stride = (long long)batch * es;
    double *out_pre = out_pre_all + b * es, *out_suf = out_suf_all + b * es;
    double *acc = dyn, *nx = dyn + es, *o = dyn + 2 * es;
    // prefix
    {
        Elem e = elem_view(acc, n);
        for (int q = lane; q < n * n; q += 64) {
            e.F[q] = (q % n == q / n) ? 1.0 : 0.0;
            e.C[q] = 0.0;
            e.P[q] = 0.0;
        }
        for (int q = lane; q < n; q += 64) { e.f[q] = 0.0; e.p[q] = 0.0; }
        wave_sync();
        for (int j = 0; j < r; ++j) {
            elem_copy(nx, elems + (long long)j * stride, n, lane);
            wave_sync();
            if (j == 0) {
                elem_copy(acc, nx, n, lane);
            } else {
                if (!tcombine<T>(o, acc, nx, n, true, false, sm, lane) && lane == 0) atomicOr(flag, 4);
                elem_copy(acc, o, n, lane);
            }
            wave_sync();
        }
        elem_copy(out_pre, acc, n, lane);
    }
    // suffix (right fold from the end: e_{R-1}, then e_j (x) acc)
    if (r + 1 >= R) {
        if (lane == 0 && b == 0) *has_suf = 0;
        return;
    }
    elem_copy(acc, elems + (long long)(R - 1) * stride, n, lane);
    wave_sync();
    for (int j = R - 2; j > r; --j) {
        elem_copy(nx, elems + (long long)j * stride, n, lane);
        wave_sync();
        if (!tcombine<T>(o, nx, acc, n, true, true, sm, lane) && lane == 0) atomicOr(flag, 8);
        elem_copy(acc, o, n, lane);
        wave_sync();
    }
    elem_copy(out_suf, acc, n, lane);
    if (lane == 0 && b == 0) *has_suf = 1;
}

int launch_fold_shards(const double *elems, int R, int r, int n, int batch, double *out_pre, double *out_suf,
                       int *has_suf, int *flag, hipStream_t st) {
    const int T = tile_order(n);
    if (T == 1)
        hipLaunchKernelGGL(k_fold_shards<1>, dim3(batch), dim3(64), elems_smem(n, 3), st, elems, R, r, n, batch,
                           out_pre, out_suf, has_suf, flag);
    else if (T == 2)
        hipLaunchKernelGGL(k_fold_shards<2>, dim3(batch), dim3(64), elems_smem(n, 3), st, elems, R, r, n, batch,
                           out_pre, out_suf, has_suf, flag);
    else
        return PDPLQR_ERR_UNSUPPORTED;
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

// Local total element of a shard = suffix scan entry 0 (already computed):
// copied out by the caller.

}  // namespace pdplqr

#ifdef PDPLQR_COMB_PROFILE
extern "C" int pdplqr_debug_comb_times(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(pdplqr::g_comb_t), sizeof(unsigned long long) * 1024 * 16) == hipSuccess ? 0 : -2;
}
#endif
