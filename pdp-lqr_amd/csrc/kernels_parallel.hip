// kernels_parallel.hip -- LQRParallelSolver on MI355X: horizon segments,
// associative segment combine, segment rollout.
//
// Restates reference lqr_solver_parallel.hpp:64-238, lqr_kernel_parallel.hpp:52-218
// and condensed_system.hpp:8-299:
//   * the segment backward (element e = (F, C, f, P, p) of every segment) is
//     k_seg_bwd_aug in kernels_segment.hip; k_seg_bwd_nofact below is its
//     linear-terms-only counterpart.
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
// Segment backward without factorization: reduction_without_factorization
// (lqr_solver_parallel.hpp:190-211) with ParallelLQRKernel::
// step_without_factorization (lqr_kernel_parallel.hpp:139-168).  The factor
// cache of the last factorising backward is reused (P_k = Lxx Lxx^T per stage,
// written by k_seg_bwd_aug, plus L(:, 0:m) in the rollout record); only the
// linear terms change: lp_k, lu'_k (into the rollout record) and the element vectors
// p, f.  f = F_{k+1}(c + B d) + f_{k+1} (:160-165) is evaluated as what it
// is -- the end state of the segment's closed-loop rollout from x = 0 under
// the new feed-forward d = -Luu^{-T} lu' -- so no per-stage F_k is stored.
// F, C, P of the element are unchanged (update_segment_data(p, f, id),
// condensed_system.hpp:76-80).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_seg_bwd_nofact(SegArgs A) {
    constexpr int P = 32;
    __shared__ double Pn[P * P];  // P_{k+1} (dense, ld n) from the factor cache
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
    auto load_P = [&](int k) {  // packed lower n x n at stage offset k ps -> dense
        for (int q = lane; q < n * n; q += 64) {
            const int i = q % n, j = q / n;
            Pn[q] = Lcb[(long long)k * sh.ps + (i >= j ? pidx(i, j, n) : pidx(j, i, n))];
        }
    };
    // segment terminal: the real one (lqr_kernel.hpp:94-101) or the dummy P = 0, p = 0
    if (lane < n) pn[lane] = last ? hb[(long long)sh.N * s + lane] : 0.0;
    if (last && lpb && lane < n) lpb[(long long)sh.N * s + lane] = pn[lane];
    if (last) load_P(sh.N);
    else
        for (int q = lane; q < n * n; q += 64) Pn[q] = 0.0;
    wave_sync();
    for (int k = N1 - 1; k >= N0; --k) {
        const double *Ek = Eb + (long long)k * n * s;
        const double *FRk = FRb + (long long)k * frs;  // L(i, j) = FRk[j s + i], j < m
        if (lane < n) cvec[lane] = cb[(long long)k * n + lane];
        wave_sync();
        if (lane < n) {  // Pb = P_{k+1} c + p_{k+1}
            double a = 0.0;
            for (int t = 0; t < n; ++t) a = __builtin_fma(Pn[lane + t * n], cvec[t], a);
            vb[lane] = a + pn[lane];
        }
        wave_sync();
        if (lane < s) {  // lp = h~ + E^T Pb (lqr_kernel.hpp:138-143)
            double a = 0.0;
            for (int t = 0; t < n; ++t) a = __builtin_fma(Ek[t + lane * n], vb[t], a);
            lp[lane] = hb[(long long)k * s + lane] + a;
        }
        wave_sync();
        if (lane == 0) {  // lu <- Luu^{-1} lu
            for (int i = 0; i < m; ++i) {
                double v = lp[i];
                for (int j = 0; j < i; ++j) v -= FRk[j * s + i] * lp[j];
                lp[i] = v / FRk[i * s + i];
            }
        }
        wave_sync();
        if (lane < n) {  // p -= Lxu lu
            double a = 0.0;
            for (int i = 0; i < m; ++i) a = __builtin_fma(FRk[i * s + m + lane], lp[i], a);
            const double pnew = lp[m + lane] - a;
            lp[m + lane] = pnew;
            pn[lane] = pnew;
        }
        wave_sync();
        if (lane < m) FRb[(long long)k * frs + (long long)s * m + lane] = lp[lane];
        if (lpb && lane < s) lpb[(long long)k * s + lane] = lp[lane];
        load_P(k);
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
