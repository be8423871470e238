// kernels_big.hip -- the serial solver for stage sizes 32 < n + m <= 64.
//
// The tiled kernels hold a stage matrix in at most 2 x 2 MFMA tiles of one
// wavefront (n + m <= 32).  Past that, a problem takes a 256-thread block whose
// stage matrices live in LDS (3 x 64 x 65 doubles, about 100 KB):
//   * k_riccati_bwd_big (keep_factors = 1; without a factor cache the value
//     form of kernels_wide.hip runs): terminal_step_with_factorization + step_with_factorization
//     (reference include/clqr/lqr/lqr_kernel.hpp:80-91, 104-147):
//         V = E^T Lxx_next,  M = H~ + V V^T,  L = chol(M),
//         Pb = Lxx_next (Lxx_next^T c) + p_next,  lp = h~ + E^T Pb,
//         lu <- Luu^{-1} lu,  p -= Lxu lu
//     with the same pivot semantics as chol_tiles (device_common.hpp): a
//     control pivot must be positive, a state pivot <= 0 stops the
//     factorisation (later columns stay unscaled), flagged only when clearly
//     negative or not finite.  Outputs as the tiled kernels: the rollout record
//     FR_k = [L(:, 0:m) | lu'], optionally the packed L_k and lp_k.
//   * k_riccati_fwd_big: forward_step (lqr_kernel.hpp:181-205), one wave per
//     problem: u = -Luu^{-T}(lu' + Lxu^T x), x+ = c + A x + B u.
// V and M are MFMA products split over the 4 waves (blk_la.hpp); the next
// stage's E~, H~, c, h~ are loaded into registers during the Cholesky and
// stored to LDS after it.
#include "blk_la.hpp"
#include "device_common.hpp"
#include "parallel.hpp"

#include <stdint.h>
#include <stdlib.h>

namespace pdplqr {

namespace {
constexpr int BS = 64;       // largest stage size
constexpr int BLD = BS + 1;  // odd leading dimension of the LDS matrices
constexpr int BT = 256;      // threads per problem
}  // namespace

// Right-looking Cholesky of M[j0:j1, j0:j1] (lower triangle, ld BLD) by the
// whole block.  The pivot column is left unscaled while the trailing matrix is
// updated with raw_i raw_l / d_jj and finalised afterwards (sinv[j] = 1 /
// sqrt(d_jj), 1 once the factorisation has stopped), as chol_tiles /
// finalize_L.  Returns true if every pivot passed (block-uniform).
__device__ __forceinline__ bool chol_big(double *M, double *sinv, int j0, int j1, int m) {
    const int tid = threadIdx.x, ri = tid & 63, cg = tid >> 6;
    bool ok = true, live = true;
    int jdead = j1;
    for (int j = j0; j < j1; ++j) {
        __syncthreads();
        const double d = M[j + j * BLD];
        ok = ok && (j < m ? d > 0.0 : !psd_bad(d));
        if (live && !(j < m || d > 0.0)) jdead = j;
        live = live && (j < m || d > 0.0);
        const double inv = live ? rsqrt_f64(d) : 0.0;
        const double inv2 = inv * inv;
        if (tid == 0) sinv[j] = live ? inv : 1.0;
        const int i = ri;
        if (i > j && i < j1) {
            const double lij = M[i + j * BLD] * inv2;
            lds_axpy_strided(M + i, BLD, M + j * BLD, lij, j + 1 + cg, i, 4);  // loads before stores, four at a time
        }
    }
    __syncthreads();
    // Eigen's left-looking stop (device_common.hpp chol_restore_tail): columns
    // >= jdead back to their original values -- undo the live pivots' updates
    // of that block, in reverse order, with the same products
    if (jdead < j1) {  // block-uniform, rare
        for (int p = jdead - 1; p >= j0; --p) {
            const double inv2 = sinv[p] * sinv[p];
            const int i = ri;
            if (i >= jdead && i < j1) {
                const double lip = M[i + p * BLD] * inv2;
                for (int l = jdead + cg; l <= i; l += 4) M[i + l * BLD] = __builtin_fma(lip, M[l + p * BLD], M[i + l * BLD]);
            }
            __syncthreads();
        }
    }
    for (int q = tid; q < (j1 - j0) * (j1 - j0); q += BT) {
        const int i = j0 + q % (j1 - j0), j = j0 + q / (j1 - j0);
        M[i + j * BLD] = i >= j ? M[i + j * BLD] * sinv[j] : 0.0;
    }
    __syncthreads();
    return ok;
}

// Stage inputs of stage k - 1 in flight in registers during stage k's
// Cholesky (kernels_wide.hip's scheme): E~ (<= 16 doubles per thread), packed
// H~ (<= 9), c, h~.
struct BigIn {
    double E[16], H[9], c, h;
};

__device__ __forceinline__ void big_in_load(BigIn &in, const double *Ek, const double *Hk, const double *ck,
                                            const double *hk, int n, int s, int ps) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int i = tid + q * BT, ic = i < n * s ? i : n * s - 1;  // unconditional load (clamped, then a select):
        const double v = Ek[ic];                                          // a guarded load is an exec-mask region with its own wait
        in.E[q] = i < n * s ? v : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 9; ++q) {
        const int i = tid + q * BT, ic = i < ps ? i : ps - 1;
        const double v = Hk[ic];
        in.H[q] = i < ps ? v : 0.0;
    }
    const double cvl = ck[tid < n ? tid : n - 1], hvl = hk[tid < s ? tid : s - 1];
    in.c = tid < n ? cvl : 0.0;
    in.h = tid < s ? hvl : 0.0;
}

// E~ into Es (ld BLD), H~ packed into Hs, c, h~
__device__ __forceinline__ void big_in_store(const BigIn &in, double *Es, double *Hs, double *cv, double *hv, int n,
                                             int s, int ps) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int i = tid + q * BT;
        if (i < n * s) Es[(i % n) + (i / n) * BLD] = in.E[q];
    }
#pragma unroll
    for (int q = 0; q < 9; ++q) {
        const int i = tid + q * BT;
        if (i < ps) Hs[i] = in.H[q];
    }
    if (tid < n) cv[tid] = in.c;
    if (tid < s) hv[tid] = in.h;
}

__global__ __launch_bounds__(BT) void k_riccati_bwd_big(RiccatiArgs A) {
    __shared__ double M[BS * BLD];   // L_{k+1} at the start of stage k, then H~_k + V V^T -> L_k
    __shared__ double V[BS * BLD];   // V = E_k^T Lxx_{k+1}  (s x n)
    __shared__ double Es[BS * BLD];  // E_k (n x s)
    __shared__ double Hs[BS * (BS + 1) / 2];  // H~_k, packed lower
    __shared__ double cv[BS], hv[BS], pbt[BS], pb[BS], pn[BS], lp[BS], sinv[BS];
    const int tid = threadIdx.x;
    const long long b = blockIdx.x;
    const Shape &sh = A.sh;
    const int n = sh.n, m = sh.m, N = sh.N, s = sh.s, ps = sh.ps;
    const long long frs = (long long)s * m + m;
    const double *Eb = A.E + b * sh.perE;
    const double *cb = A.c + b * sh.perc;
    const double *Hb = A.Hw + b * sh.perHw;
    const double *hb = A.hw + b * sh.perh;
    double *FRb = A.KD + b * sh.perKD;
    double *Lcb = A.Lc ? A.Lc + b * sh.perHw : nullptr;
    double *lpb = A.lpc ? A.lpc + b * sh.perh : nullptr;
    auto Lxx = [&](int i, int t) -> double { return M[(m + i) + (m + t) * BLD]; };
    int fail_stage = -1;
    BigIn nxt;
    if (N > 0)
        big_in_load(nxt, Eb + (long long)(N - 1) * n * s, Hb + (long long)(N - 1) * ps, cb + (long long)(N - 1) * n,
                    hb + (long long)(N - 1) * s, n, s, ps);

    // ---- terminal (lqr_kernel.hpp:80-91): L_N = chol(H~_N) at offset m, lp_N = h~_N ----
    for (int q = tid; q < n * n; q += BT) {
        const int i = q % n, j = q / n;
        if (i >= j) M[(m + i) + (m + j) * BLD] = Hb[(long long)N * sh.ps + pidx(i, j, n)];
    }
    if (tid < n) {
        const double v = hb[(long long)N * s + tid];
        pn[tid] = v;
        if (lpb) lpb[(long long)N * s + tid] = v;
    }
    if (!chol_big(M, sinv, m, s, m)) fail_stage = N;
    if (Lcb)
        for (int q = tid; q < sh.pn; q += BT) {
            const short2 ij = A.tab_n[q];
            Lcb[(long long)N * sh.ps + q] = Lxx(ij.x, ij.y);
        }
    if (N > 0) big_in_store(nxt, Es, Hs, cv, hv, n, s, ps);
    __syncthreads();

    for (int k = N - 1; k >= 0; --k) {
        // Es = E_k, Hs = H~_k, cv = c_k, hv = h~_k (stored at the end of stage k + 1)
        // V = E^T Lxx (s x n; Lxx lower, zeros above: chol_big's finalisation)
        blk_mm(V, BLD, mv_t(Es, BLD), mv_n(M + m + m * BLD, BLD), s, n, n, 1.0, 0.0, mv_none(), false);
        if (tid < n) {  // Pb_tmp = Lxx^T c
            double a = 0.0;
            for (int i = tid; i < n; ++i) a = __builtin_fma(Lxx(i, tid), cv[i], a);
            pbt[tid] = a;
        }
        __syncthreads();
        if (tid < n) {  // Pb = Lxx Pb_tmp + p_next
            double a = 0.0;
            for (int t = 0; t <= tid; ++t) a = __builtin_fma(Lxx(tid, t), pbt[t], a);
            pb[tid] = a + pn[tid];
        }
        __syncthreads();
        if (tid < s) {  // lp = h~ + E^T Pb
            double a = hv[tid];
            for (int i = 0; i < n; ++i) a = __builtin_fma(Es[i + tid * BLD], pb[i], a);
            lp[tid] = a;
        }
        // M = H~ + V V^T (lower; M no longer holds L_{k+1})
        blk_mm(M, BLD, mv_n(V, BLD), mv_t(V, BLD), s, s, n, 1.0, 0.0, mv_pk(Hs, s), true);
        if (k > 0)  // stage k - 1's inputs in flight during the factorisation
            big_in_load(nxt, Eb + (long long)(k - 1) * n * s, Hb + (long long)(k - 1) * ps,
                        cb + (long long)(k - 1) * n, hb + (long long)(k - 1) * s, n, s, ps);
        if (!chol_big(M, sinv, 0, s, m) && fail_stage < 0) fail_stage = k;
        // lu <- Luu^{-1} lu ; p -= Lxu lu  (wave 0, lane i holds lp_i)
        if (tid < 64) {
            double x = tid < s ? lp[tid] : 0.0;
            for (int j = 0; j < m; ++j) {
                const double uj = readlane_f64(x, j) / M[j + j * BLD];
                if (tid == j) x = uj;
                else if (tid > j && tid < s) x = __builtin_fma(-M[tid + j * BLD], uj, x);
            }
            if (tid < s) {
                lp[tid] = x;
                if (tid >= m) pn[tid - m] = x;
                if (lpb) lpb[(long long)k * s + tid] = x;
                if (tid < m) FRb[(long long)k * frs + (long long)s * m + tid] = x;
            }
        }
        double *FRk = FRb + (long long)k * frs;
        for (int q = tid; q < s * m; q += BT) FRk[q] = M[(q % s) + (q / s) * BLD];
        if (Lcb)
            for (int q = tid; q < sh.ps; q += BT) {
                const short2 ij = A.tab_s[q];
                Lcb[(long long)k * sh.ps + q] = M[ij.x + ij.y * BLD];
            }
        if (k > 0) big_in_store(nxt, Es, Hs, cv, hv, n, s, ps);  // Es, Hs, cv, hv are free since M was formed
        __syncthreads();
    }
    if (tid == 0) A.status[b] = fail_stage < 0 ? 0 : fail_stage + 1;
}

// forward_step (lqr_kernel.hpp:181-205) for s <= 64: one wave per problem
// (SEG: per (problem, segment) of the parallel solver, with the coupling
// u_hat = lambda of the next boundary through G_k, lqr_kernel_parallel.hpp:
// 195-198, and update_x_next, lqr_solver_parallel.hpp:231, as k_seg_fwd_dma).
// ws[k s .. k s + s) = [u_k; x_k], ws[N s .. N s + n) = x_N.
template <bool SEG>
__global__ __launch_bounds__(64) void k_riccati_fwd_big(Shape sh, const double *__restrict__ E,
                                                       const double *__restrict__ c, const double *__restrict__ FR,
                                                       const double *__restrict__ x0, double *__restrict__ ws,
                                                       SegFwd sf) {
    __shared__ double w[BS], uh[BS];
    const int lane = wave_lane();
    const long long b = SEG ? blockIdx.x / sf.S : blockIdx.x;
    const int seg = SEG ? blockIdx.x % sf.S : 0;
    const int n = sh.n, m = sh.m, N = sh.N, s = sh.s;
    const int K0 = SEG ? sf.seg_start[seg] : 0, K1 = SEG ? K0 + sf.seg_len[seg] : N;
    const bool last = !SEG || (seg == sf.S - 1 && sf.last_is_terminal);
    const long long frs = (long long)s * m + m;
    const double *Eb = E + b * sh.perE;
    const double *cb = c + b * sh.perc;
    const double *Fb = FR + b * sh.perKD;
    const double *Gb = SEG ? sf.G + b * (long long)N * m * n : nullptr;
    double *wb = ws + b * sh.perh;
    if (lane < n) {
        if (SEG) {
            const double *xh = sf.xhat + b * (sf.S + 1) * (long long)n;
            const double v = xh[(long long)seg * n + lane];
            w[m + lane] = v;
            uh[lane] = last ? 0.0 : sf.lam[(b * (sf.S + 1) + seg + 1) * n + lane];
            wb[(long long)K0 * s + m + lane] = v;  // ws[N0].tail(n) = x_hat
            if (!last && seg == sf.S - 1) wb[(long long)K1 * s + lane] = xh[(long long)sf.S * n + lane];
        } else {
            const double v = x0[b * n + lane];
            w[m + lane] = v;
            wb[(long long)(N > 0 ? m : 0) + lane] = v;
        }
    }
    wave_sync();
    for (int k = K0; k < K1; ++k) {
        const double *Fk = Fb + (long long)k * frs;
        // v_j = -lu'_j - sum_i Lxu(i, j) x_i (+ sum_t G(j, t) u_hat_t)  (lane j < m)
        double v = 0.0;
        if (lane < m) {
            double a = Fk[(long long)s * m + lane];
            for (int i = 0; i < n; ++i) a = __builtin_fma(Fk[(long long)lane * s + m + i], w[m + i], a);
            if (SEG && !last) {
                const double *Gk = Gb + (long long)k * m * n;
                for (int t = 0; t < n; ++t) a = __builtin_fma(-Gk[lane + t * m], uh[t], a);
            }
            v = -a;
        }
        // u = Luu^{-T} v (back substitution, column j of Luu^T = row j of Luu)
        for (int j = m - 1; j >= 0; --j) {
            const double uj = readlane_f64(v, j) / Fk[(long long)j * s + j];
            if (lane == j) v = uj;
            else if (lane < j) v = __builtin_fma(-Fk[(long long)lane * s + j], uj, v);
        }
        if (lane < m) {
            w[lane] = v;
            wb[(long long)k * s + lane] = v;
        }
        wave_sync();
        const bool upd = last || (k < K1 - 1);  // update_x_next
        // x+ = c + E [u; x]
        double xn = 0.0;
        if (lane < n) {
            const double *Ek = Eb + (long long)k * n * s;
            double a = cb[(long long)k * n + lane];
            for (int j = 0; j < s; ++j) a = __builtin_fma(Ek[lane + (long long)j * n], w[j], a);
            xn = a;
        }
        wave_sync();
        if (lane < n && upd) {
            w[m + lane] = xn;
            wb[(long long)(k + 1) * s + ((k + 1 < N) ? m : 0) + lane] = xn;
        }
        wave_sync();
    }
}

bool big_shape(const Shape &sh) { return sh.s > 32 && sh.s <= BS; }

int launch_riccati_backward_value_wide(const RiccatiArgs &r, hipStream_t st);  // kernels_wide.hip

int launch_riccati_backward_big(const RiccatiArgs &a, hipStream_t st) {
    // keep_factors = 0: the value form (m pivots a stage, MFMA products)
    if (!a.Lc) return launch_riccati_backward_value_wide(a, st);
    hipLaunchKernelGGL(k_riccati_bwd_big, dim3(a.sh.batch), dim3(BT), 0, st, a);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

int launch_riccati_forward_big(const Shape &sh, const double *E, const double *c, const double *FR, const double *x0,
                               double *ws, hipStream_t st) {
    hipLaunchKernelGGL(k_riccati_fwd_big<false>, dim3(sh.batch), dim3(64), 0, st, sh, E, c, FR, x0, ws, SegFwd{});
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

int launch_riccati_forward_seg_big(const Shape &sh, const double *E, const double *c, const double *FR,
                                   const SegFwd &sf, double *ws, hipStream_t st) {
    hipLaunchKernelGGL(k_riccati_fwd_big<true>, dim3((unsigned)(sh.batch * sf.S)), dim3(64), 0, st, sh, E, c, FR,
                       nullptr, ws, sf);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

}  // namespace pdplqr
