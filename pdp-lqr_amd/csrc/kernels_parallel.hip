// kernels_parallel.hip -- LQRParallelSolver on MI355X: horizon segments,
// associative segment combine, segment rollout.
//
// Restates reference lqr_solver_parallel.hpp:64-238, lqr_kernel_parallel.hpp:52-218
// and condensed_system.hpp:8-299:
//   * the segment backward (element e = (F, C, f, P, p) of every segment) is
//     k_seg_bwd_aug in kernels_segment.hip; k_seg_bwd_nofact below is its
//     linear-terms-only counterpart.
//   * k_seg_scan: one Hillis-Steele round of the suffix scan of the elements
//     under the associative operator
//         Z = (I + C_a P_b)^{-1}, F = F_b Z F_a, C = F_b Z C_a F_b^T + C_b,
//         f = F_b Z (f_a - C_a p_b) + f_b, P = P_a + F_a^T P_b Z F_a,
//         p = p_a + F_a^T Z^T (p_b + P_b f_a).
//     The reference folds the same operator serially on the master thread
//     (condensed_system.hpp:82-137 LU form, :203-290 Cholesky form); here
//     P_b Z = Y = R (I + R^T C_a R)^{-1} R^T with R = chol(P_b), an SPD solve,
//     evaluated on MFMA tiles (combine_tiles.hpp).  Suffix entry i is the value
//     function (P, p) at the start of segment i.
//   * k_seg_maps: the closed-loop boundary map of every segment under those
//     value functions, x_{i+1} = Z_i (F_i x_i + f_i - C_i p_{i+1}),
//     Z_i = (I + C_i P_{i+1})^{-1}; k_map_scan composes the maps (prefix scan
//     of affine maps: one matrix product per combine, no factorisation) into
//     the boundary states x_hat_i and costates lambda_i = P_i x_hat_i + p_i
//     (the condensed forward).
//   * the rollout reuses k_riccati_fwd with the G_k u_hat coupling
//     (lqr_kernel_parallel.hpp:195-198), u_hat from lambda_{i+1}.
#define PDPLQR_COMB_PROFILE_TU 1  // the combine phase marks live in this translation unit
#include "combine_mw.hpp"
#include "combine_qd.hpp"
#include "combine_qd1.hpp"
#include "combine_tiles.hpp"
#include "device_common.hpp"
#include "parallel.hpp"

namespace pdplqr {

#ifdef PDPLQR_COMB_PROFILE
__device__ unsigned long long g_comb_t[1024 * 32];
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
template <int P>  // P >= n + m: 32, or 64 for the wide shapes
__global__ __launch_bounds__(64) void k_seg_bwd_nofact(SegArgs A) {
    __shared__ double Pn[P * P];  // P_{k+1} (dense, ld n) from the factor cache
    __shared__ double cvec[P], va[P], vb[P], lp[P], pn[P], xs[P], us[P];
    const int lane = wave_lane();
    const Shape &sh = A.sh;
    const int n = sh.n, m = sh.m, s = sh.s, S = A.S;
    const long long b = blockIdx.x / S;
    const int seg = blockIdx.x % S;
    if (A.flag && seg == 0 && lane == 0) A.flag[b] = 0;
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
    if (xl_shape(a.sh)) return launch_seg_backward_nofact_xl(a, st);
    if (a.sh.s > 64 || !a.Lc) {
        set_error("PARALLEL backward_without_factorization needs keep_factors = 1");
        return PDPLQR_ERR_UNSUPPORTED;
    }
    if (a.sh.s <= 32) hipLaunchKernelGGL(k_seg_bwd_nofact<32>, dim3((unsigned)(a.sh.batch * a.S)), dim3(64), 0, st, a);
    else hipLaunchKernelGGL(k_seg_bwd_nofact<64>, dim3((unsigned)(a.sh.batch * a.S)), dim3(64), 0, st, a);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

// ---------------------------------------------------------------------------
// One Hillis-Steele round: inclusive prefix (dir 0) or suffix (dir 1) scan.
// ---------------------------------------------------------------------------
// LDS[dst, dst + len) <- src[0, len) (doubles) with one LDS-DMA burst (a single
// HBM/L2 latency) when src and dst are 16-byte aligned, by a plain copy
// otherwise.  The caller waits on vmcnt(0) and then wave_sync()s.
__device__ __forceinline__ void stage_range(double *dst, const double *src, int len, int lane) {
    if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0) {
        const int chunks = len >> 1;
        for (int q = 0; q * 64 < chunks; ++q) {
            const int ch = q * 64 + lane;
            if (ch < chunks) dma16(src + 2 * ch, dst + 2 * q * 64);
        }
        if ((len & 1) && lane == 0) dst[len - 1] = src[len - 1];
    } else {
        for (int q = lane; q < len; q += 64) dst[q] = src[q];
    }
}

// LDS images of the two combine operands without the blocks read only once as
// addends (P_a, C_b: loaded from global memory by tcombine_parts), 2 n^2 + 2 n
// doubles each: a = [F | C | f | p], b = [F | f | P | p].  At 24/8 the scan
// kernel then needs 19.2 KB of element LDS instead of 28.4 KB, and 4 blocks
// fit a CU (the register file holds 4 waves of it anyway).
__device__ __forceinline__ int op_stage_len(int n) { return (2 * n * n + 2 * n + 1) & ~1; }

__device__ __forceinline__ ElemIn stage_left(double *dst, const double *e, int n, int lane) {
    const int nn = n * n;
    stage_range(dst, e, 2 * nn + n, lane);                  // F | C | f
    stage_range(dst + 2 * nn + n, e + 3 * nn + n, n, lane);  // p
    return ElemIn{dst, dst + nn, dst + 2 * nn, e + 2 * nn + n, dst + 2 * nn + n};
}

__device__ __forceinline__ ElemIn stage_right(double *dst, const double *e, int n, int lane) {
    const int nn = n * n;
    stage_range(dst, e, nn, lane);                        // F
    stage_range(dst + nn, e + 2 * nn, nn + 2 * n, lane);  // f | P | p
    return ElemIn{dst, e + nn, dst + nn, dst + nn + n, dst + 2 * nn + n};
}

static size_t op_stage_bytes(int n) { return 2 * (size_t)((2 * n * n + 2 * n + 1) & ~1) * sizeof(double); }

// Block-wide (256 threads) LDS[dst, dst + len) <- src[0, len): one LDS-DMA burst
// per wave (global_load_lds_dwordx4, 1 KB per instruction) when both are
// 16-byte aligned, a plain copy otherwise.  The caller waits on vmcnt(0) and
// then __syncthreads().  The 4-wave combines stage BOTH operands up front this
// way: every later read is an LDS read, so the combine pays one memory latency
// instead of one per dependent global load of its phases.
__device__ __forceinline__ void stage_range_blk(double *dst, const double *src, int len) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0) {
        const int chunks = len >> 1;
        for (int q = wv; q * 64 < chunks; q += 4) {
            const int ch = q * 64 + lane;
            if (ch < chunks) dma16(src + 2 * ch, dst + 2 * q * 64);
        }
        if ((len & 1) && threadIdx.x == 0) dst[len - 1] = src[len - 1];
    } else {
        for (int q = threadIdx.x; q < len; q += 256) dst[q] = src[q];
    }
}

// doubles of the 4-wave combine's own LDS, rounded up to a 16-byte boundary
__host__ __device__ inline int mw_smem_doubles(int n) { return (int)((mw_smem_bytes(n) + 15) / 16 * 2); }
__host__ __device__ inline int elem_slot(int n) { return (3 * n * n + 2 * n + 1) & ~1; }

// The 4-wave combine of the n = 24 kernels: the blocked LDL^T of the junction
// block (combine_qd.hpp) unless built with -DPDPLQR_QD_COMBINE=0 (the
// two-Cholesky mw_combine, A/B).  Both read their operands only through ea /
// eb (staged in LDS by every caller) and use the combine's own LDS `buf`.
#ifndef PDPLQR_QD_COMBINE
#define PDPLQR_QD_COMBINE 1
#endif
static_assert(qd_smem_doubles() <= (5 * QD_N * (QD_N + 1) + 4 * QD_N) + 2, "qd scratch fits the mw region (mw_smem_bytes)");
template <int T, int NC>
__device__ __forceinline__ bool mw_combine_nc(double *oF, double *oC, double *of, double *oP, double *op,
                                              const ElemIn &ea, const ElemIn &eb, int n, bool fcf, double *buf) {
    if constexpr (NC == QD_N && PDPLQR_QD_COMBINE) {
        return qd_combine(oF, oC, of, oP, op, ea, eb, fcf, buf);
    } else {
        return mw_combine<T>(oF, oC, of, oP, op, ea, eb, n, fcf, mw_smem(buf, n));
    }
}

template <int T, bool LU, int NC = 0>
__global__ __launch_bounds__(64) void k_seg_scan(ScanArgs A) {
    __shared__ CombSmem<T> sm;
    extern __shared__ __attribute__((aligned(16))) double ebuf[];  // 2 operand images (op_stage_bytes)
    const int lane = wave_lane();
    const int n = NC ? NC : A.n, S = A.S, d = A.dist;
    const int es = 3 * n * n + 2 * n;
    const int per = scan_round_blocks(S, d, A.sk);
    const long long b = blockIdx.x / per;
    int i, j;
    if (!scan_round_operands(S, d, A.sk, blockIdx.x % per, i, j)) return;
    const long long is = A.istride ? A.istride : es;
    const double *in = A.in + b * (A.bstride ? A.bstride : (long long)S * es);
    double *out = A.out + b * (long long)S * es;
    if (j < 0) {  // suf_i already reaches the end of its block / the last segment
        if (in != out) elem_copy(out + (long long)i * es, in + (long long)i * is, n, lane);
        return;
    }
    // The right operand covers segments [j, min(j + d - 1, S - 1)].  When
    // that range holds the real terminal its F = C = f = 0, and so are the
    // result's: only the value function (P, p) is combined.  In place (sk = 2)
    // is safe: every operand block but P_a is staged in LDS first, and P_a is
    // read into registers that the symmetrised P store depends on.
    const bool fcf = !(A.terminal && j + d - 1 >= S - 1);
    const ElemIn ea = stage_left(ebuf, in + (long long)i * is, n, lane);
    const ElemIn eb = stage_right(ebuf + op_stage_len(n), in + (long long)j * is, n, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
    double *o = out + (long long)i * es;
    const int nn = n * n;
    const bool ok = tcombine_parts<T, LU>(o, o + nn, o + 2 * nn, o + 2 * nn + n, o + 3 * nn + n, ea, eb, n, fcf,
                                          true, sm, lane);
    if (!fcf)
        for (int q = lane; q < 2 * n * n + n; q += 64) o[q] = 0.0;  // [F | C | f]
    if (!ok && lane == 0) atomicOr(A.flag + b, 1);  // per problem
}

// Two Hillis-Steele rounds (distances d and 2 d) in one launch, two waves per
// block: wave 0 forms a_i = e_i + e_{i+d}, wave 1 a_{i+2d} = e_{i+2d} + e_{i+3d}
// (the a_{i+2d} of block i + 2d, formed again: idle CUs are cheap here), both
// into the block's private scratch slots; after the block barrier wave 0
// forms a_i + a_{i+2d}.  The result equals two radix-2 rounds exactly (the
// same combines in the same order); a pair of rounds costs two combine
// latencies but one dispatch, operand fetch and write-back less.  Each
// combine's right operand covers [first, min(first + span - 1, S - 1)]; when
// that range holds the real terminal, F = C = f = 0 (see k_seg_scan).
// The n = 12 CHOLESKY combines of the two-round scan run the one-wave blocked
// LDL^T of the junction block (combine_qd1.hpp) unless built with
// -DPDPLQR_QD1_COMBINE=0 (the Cholesky form tcombine_parts, A/B).
#ifndef PDPLQR_QD1_COMBINE
#define PDPLQR_QD1_COMBINE 1
#endif
template <int NC, bool LU>
constexpr bool use_qd1() { return PDPLQR_QD1_COMBINE && !LU && NC == 12; }

template <int T, bool LU, int NC = 0>
__device__ __forceinline__ void seg_scan4_block(const ScanArgs &A, long long blk, CombSmem<T> (&smv)[2], double *ebuf,
                                                double *qd1s = nullptr) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n = NC ? NC : A.n, S = A.S, d = A.dist;
    const int es = 3 * n * n + 2 * n, nn = n * n, ol = op_stage_len(n);
    const long long b = blk / S;
    const int i = (int)(blk % S);
    const long long is = A.istride ? A.istride : es;
    const double *in = A.in + b * (A.bstride ? A.bstride : (long long)S * es);
    double *out = A.out + b * (long long)S * es;
    double *scr = A.scratch + (b * S + i) * 2LL * es;
    constexpr bool QD1 = use_qd1<NC, LU>();
    // per wave: two operand images (QD1: the whole elements, so the assembly
    // reads LDS only -- one memory latency per combine)
    double *eb = ebuf + wv * 2 * (QD1 ? elem_slot(n) : ol);
    CombSmem<T> &sm = smv[wv];
    auto combine = [&](double *o, const double *left, const double *right, bool fcf) {
        bool ok;
        if constexpr (QD1) {
            stage_range(eb, left, es, lane);
            stage_range(eb + elem_slot(n), right, es, lane);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            wave_sync();
            ok = qd1_combine<12>(o, o + nn, o + 2 * nn, o + 2 * nn + n, o + 3 * nn + n, elem_in(eb, n),
                                 elem_in(eb + elem_slot(n), n), fcf, qd1s + wv * Qd1<12>::smem, lane);
        } else {
            const ElemIn ea = stage_left(eb, left, n, lane);
            const ElemIn er = stage_right(eb + ol, right, n, lane);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            wave_sync();
            ok = tcombine_parts<T, LU>(o, o + nn, o + 2 * nn, o + 2 * nn + n, o + 3 * nn + n, ea, er, n, fcf, true, sm,
                                       lane);
        }
        if (!fcf)
            for (int q = lane; q < 2 * nn + n; q += 64) o[q] = 0.0;  // [F | C | f]
        return ok;
    };
    auto fcf_of = [&](int last) { return !(A.terminal && last >= S - 1); };  // right operand's last segment
    if (i + d >= S) {  // suf_i already reaches the last segment (block-uniform)
        if (wv == 0) elem_copy(out + (long long)i * es, in + (long long)i * is, n, lane);
        return;
    }
    const bool two = i + 2 * d < S;  // block-uniform
    bool ok = true;
    if (wv == 0) {
        ok = combine(two ? scr : out + (long long)i * es, in + (long long)i * is, in + (long long)(i + d) * is,
                     fcf_of(i + 2 * d - 1));
    } else if (two) {
        if (i + 3 * d >= S) elem_copy(scr + es, in + (long long)(i + 2 * d) * is, n, lane);
        else
            ok = combine(scr + es, in + (long long)(i + 2 * d) * is, in + (long long)(i + 3 * d) * is,
                         fcf_of(i + 4 * d - 1));
    }
    if (two) {
        __syncthreads();  // the scratch slots are written and visible to the block
        if (wv == 0) ok = combine(out + (long long)i * es, scr, scr + es, fcf_of(i + 4 * d - 1)) && ok;
    }
    if (!ok && lane == 0) atomicOr(A.flag + b, 1);  // per problem
}

template <int T, bool LU, int NC = 0>
__global__ __launch_bounds__(128) void k_seg_scan4(ScanArgs A) {
    __shared__ CombSmem<T> smv[2];
    __shared__ __attribute__((aligned(16))) double qd1s[use_qd1<NC, LU>() ? 2 * Qd1<12>::smem : 2];
    extern __shared__ __attribute__((aligned(16))) double ebuf[];  // per wave: 2 operand images
    seg_scan4_block<T, LU, NC>(A, blockIdx.x, smv, ebuf, qd1s);
}


// One Hillis-Steele round with the 4-wave combine (combine_mw.hpp; CHOLESKY
// form): the same operands, output and terminal rule as k_seg_scan.
// the combine of block `blk` of one round (the body of k_seg_scan_mw, shared
// with the all-rounds kernel below)
template <int T, int NC = 0>
__device__ __forceinline__ void mw_scan_block(const ScanArgs &A, long long blk, double *mwbuf) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n = NC ? NC : A.n, S = A.S, d = A.dist;
    const int es = 3 * n * n + 2 * n, nn = n * n;
    const int per = scan_round_blocks(S, d, A.sk);
    const long long b = blk / per;
    int i, j;
    if (!scan_round_operands(S, d, A.sk, (int)(blk % per), i, j)) return;  // block-uniform
    const long long is = A.istride ? A.istride : es;
    const double *in = A.in + b * (A.bstride ? A.bstride : (long long)S * es);
    double *out = A.out + b * (long long)S * es;
    if (j < 0) {  // block-uniform
        if (wv == 0 && in != out) elem_copy(out + (long long)i * es, in + (long long)i * is, n, lane);
        return;
    }
    // both operands are staged in LDS before any store: in place (sk = 2) is safe
    const bool fcf = !(A.terminal && j + d - 1 >= S - 1);
    COMB_MARK(16);  // kernel entry
#ifdef PDPLQR_COMB_PROFILE
    if (threadIdx.x == 0) {
        g_comb_t[(blockIdx.x % 1024) * 32 + 21] = d;  // the round
        g_comb_t[(blockIdx.x % 1024) * 32 + 22] = fcf;
    }
#endif
    double *ea = mwbuf + mw_smem_doubles(n), *eb = ea + elem_slot(n);
    stage_range_blk(ea, in + (long long)i * is, es);
    stage_range_blk(eb, in + (long long)j * is, es);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    COMB_MARK(17);  // operands staged
    double *o = out + (long long)i * es;
    const bool ok = mw_combine_nc<T, NC>(o, o + nn, o + 2 * nn, o + 2 * nn + n, o + 3 * nn + n, elem_in(ea, n),
                                         elem_in(eb, n), n, fcf, mwbuf);
#ifdef PDPLQR_COMB_PROFILE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    COMB_MARK(18);  // wave 0's stores complete
#endif
    if (!fcf && wv == 1)
        for (int q = lane; q < 2 * nn + n; q += 64) o[q] = 0.0;  // [F | C | f]
    if (!ok && threadIdx.x == 0) atomicOr(A.flag + b, 1);
}

template <int T, int NC = 0>
__global__ __launch_bounds__(256, 2) void k_seg_scan_mw(ScanArgs A) {
    extern __shared__ __attribute__((aligned(16))) double mwbuf[];
    mw_scan_block<T, NC>(A, blockIdx.x, mwbuf);
}


// ---------------------------------------------------------------------------
// Boundary maps.  With the value function V_j = (P_j, p_j) at boundary j (the
// suffix-scan entry j, right-folded with the global suffix of later shards),
// the state at boundary j follows from the state at boundary j - 1 through
// the element (F, C, f) of segment j - 1:
//     x_j = Phi_j x_{j-1} + phi_j,  Z = (I + C P_j)^{-1},
//     Phi_j = Z F,  phi_j = Z (f - C p_j)
// -- the condensed forward of condensed_system.hpp:117-137 (LU form) and
// :262-290 (Cholesky form), which walks this recursion serially.  Block j = 0
// maps x0 through the global prefix of earlier shards (or the identity) and
// writes x_0 directly.  maps: [b][S+1][Phi | phi], vfun: [b][S+1][P | p].
// ---------------------------------------------------------------------------
template <int T, bool LU, int NC = 0>
__global__ __launch_bounds__(64) void k_seg_maps(MapArgs A) {
    extern __shared__ __attribute__((aligned(16))) double dyn[];  // 2 operand images when A.right
    __shared__ CombSmem<T> sm;
    const int lane = wave_lane(), g = lane >> 4, c = lane & 15;
    const int n = NC ? NC : A.n, S = A.S, J = S + 1, nn = n * n;
    const int es = 3 * nn + 2 * n, mw = nn + n;
    const long long b = blockIdx.x / J;
    const int j = blockIdx.x % J;
    const double *right = A.right ? A.right + b * (A.rstride ? A.rstride : (long long)es) : nullptr;
    double *vo = A.vfun + (b * J + j) * (long long)mw;
    double *mo = A.maps + (b * J + j) * (long long)mw;
    bool ok = true;
    // V_j: [P | p] at vP, vp (global), or absent (j == S on the last shard)
    const double *vP = nullptr, *vp = nullptr;
    if (j < S && right) {
        const ElemIn ea = stage_left(dyn, A.suf + (b * S + j) * (long long)es, n, lane);
        const ElemIn eb = stage_right(dyn + op_stage_len(n), right, n, lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        wave_sync();
        ok = tcombine_parts<T, LU>(nullptr, nullptr, nullptr, vo, vo + nn, ea, eb, n, false, true, sm, lane);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // vo is re-read by other lanes below
        vP = vo;
        vp = vo + nn;
    } else {
        const double *src = j < S ? A.suf + (b * S + j) * (long long)es : right;
        if (src) {
            vP = src + 2 * nn + n;
            vp = src + 3 * nn + n;
            for (int q = lane; q < mw; q += 64) vo[q] = q < nn ? vP[q] : vp[q - nn];
        } else {
            for (int q = lane; q < mw; q += 64) vo[q] = 0.0;
        }
    }
    // source element: segment j - 1, the global prefix (j = 0, later shards), or the identity
    const double *src = j > 0 ? A.elem + (b * S + j - 1) * (long long)es : A.left ? A.left + b * (long long)es
                                                                                 : nullptr;
    WM<T> Phi, PhiT;
    WV<T> phi;
    if (src) {
        if (vP) {  // [Phi | phi] = (I + C P_j)^{-1} [F | f - C p_j] (tmap_solve: a solve, no I - C Y)
            double *mscr = dyn + (A.right ? 2 * op_stage_len(n) : 0), *mout = mscr + tmap_smem_doubles(n);
            ok = tmap_solve<T, LU>(src, src + nn, src + 2 * nn, vP, vp, n, mscr, mout, lane) && ok;
            wv_load(phi, mout + nn, n, g, c);
            if (j > 0) wm_load(Phi, mout, n, n, false, 0.0, g, c);
            else wm_load(PhiT, mout, n, n, true, 0.0, g, c);
        } else {
            wv_load(phi, src + 2 * nn, n, g, c);
            if (j > 0) wm_load(Phi, src, n, n, false, 0.0, g, c);
            else wm_load(PhiT, src, n, n, true, 0.0, g, c);
        }
    }
    if (!ok && lane == 0) atomicOr(A.flag + b, 2);
    if (j > 0) {
        wm_store(Phi, mo, n, n, g, c);
        wv_store(phi, mo + nn, n, g, c);
        return;
    }
    // j = 0: x_0 = Phi x0 + phi (x0 itself without a global prefix), lambda_0 = P_0 x_0 + p_0
    WV<T> x0v, x;
    wv_load(x0v, A.x0 + b * (long long)n, n, g, c);
    if (src) wv_tn(x, PhiT, x0v, n, 1.0, &phi);
    else x = x0v;
    wv_store(x, mo + nn, n, g, c);
    wv_store(x, A.xhat + b * (long long)J * n, n, g, c);
    if (vP) {
        WM<T> Pv;
        WV<T> pv, lam;
        wm_load(Pv, vP, n, n, false, 0.0, g, c);
        wv_load(pv, vp, n, g, c);
        wv_tn(lam, Pv, x, n, 1.0, &pv);  // P symmetric
        wv_store(lam, A.lam + b * (long long)J * n, n, g, c);
    }
}

// The boundary map of element e under the value function (vP, vp) on a
// 4-wave block (CHOLESKY form, every operand in LDS):
//     R = chol(P), S = I + R^T C R = Q Q^T,  X1 = Q^{-1} R^T F,
//     V = Q^{-1} R^{-1},  x3 = Q^{-1} R^T (f - C p)
//     Phi = V^T X1,  phi = V^T x3
// -- the solve of (I + C P) [Phi | phi] = [F | f - C p] (no I - C Y
// cancellation, see tmap_solve in combine_tiles.hpp).  Wave 0 returns Phi (or
// Phi^T when trans) and phi; every wave returns the block-uniform status.
template <int T>
__device__ __forceinline__ bool mw_map(const ElemIn &e, const double *vP, const double *vp, int n, const MwSmem &sm,
                                       bool trans, WM<T> &Phi, WV<T> &phi) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
    const int PL = sm.ld;
    bool ok = true;
    WM<T> R;
    // ---- phase A: R = chol(P_j) (w0, w1); R^{-1} (w2: the same factorisation
    //      carrying the identity) ----
    if (wv < 2) {
        ok = mw_chol_R<T>(R, vP, sm.S + wv * (n * PL), PL, n, g, c) && ok;
    } else if (wv == 2) {
        WM<T> Pm, Ri;
#pragma unroll
        for (int a = 0; a < T; ++a)
#pragma unroll
            for (int bt = 0; bt < T; ++bt)
#pragma unroll
                for (int r = 0; r < 4; ++r) Ri.t[a][bt][r] = (16 * a + 4 * r + g == 16 * bt + c) ? 1.0 : 0.0;
        wm_load(Pm, vP, n, n, false, 1.0, g, c);
        ok = chol_blk4<T, true, T>(Pm, Ri.t, n, g, c) && ok;  // Ri = R^{-1}
        wm_store(Ri, sm.B2, PL, n, g, c);
    }
    // ---- phase B ----
    if (wv == 0) {
        WM<T> Cs, T1, Sm;
        wm_load(Cs, e.C, n, n, false, 0.0, g, c);
        wm_tn(T1, Cs, R, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);  // C R
        wm_tn(Sm, R, T1, n, 1.0, 1.0, (const WM<T> *)nullptr, g, c);  // I + R^T C R
        wm_store(Sm, sm.S, PL, n, g, c);
        if (lane == 0) sm.ok[0] = ok;
    } else if (wv == 1) {
        WM<T> Fs, B;
        wm_load(Fs, e.F, n, n, false, 0.0, g, c);
        wm_tn(B, R, Fs, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);  // R^T F
        wm_store(B, sm.B1, PL, n, g, c);
        WM<T> Cs;
        WV<T> pv, fs, v, y;
        wm_load(Cs, e.C, n, n, false, 0.0, g, c);
        wv_load(pv, vp, n, g, c);
        wv_load(fs, e.f, n, g, c);
        wv_tn(v, Cs, pv, n, -1.0, &fs);                  // v = f - C p_j
        wv_tn(y, R, v, n, 1.0, (const WV<T> *)nullptr);  // R^T v
        wv_store(y, sm.bv, n, g, c);
    }
    if (wv == 2 && lane == 0) sm.ok[2] = ok;
    __syncthreads();
    ok = ok && sm.ok[0] && sm.ok[2];
    // ---- phase C: chol(S) carrying one column tile per wave: X1 = Q^{-1} R^T F,
    //      V = Q^{-1} R^{-1}, x3 = Q^{-1} R^T v ----
    {
        WM<T> Sm;
        wm_load(Sm, sm.S, PL, n, false, 1.0, g, c);
        d4 B[T][1], V[T][1];
        int kind, tile = 0;  // 0: X1, 1: V, 2: x3
        if (T == 2) {
            kind = wv < 2 ? 0 : 1;
            tile = wv & 1;
        } else {
            kind = wv == 0 ? 2 : (wv == 1 ? 0 : (wv == 2 ? 1 : -1));
        }
        const bool vec3 = T == 2 && wv == 3;
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
            okS = chol_blk4<T, true, 2>(Sm, BV, n, g, c);
#pragma unroll
            for (int a = 0; a < T; ++a) {
                B[a][0] = BV[a][0];
                V[a][0] = BV[a][1];
            }
        } else if (kind >= 0) {
            okS = chol_blk4<T, true, 1>(Sm, B, n, g, c);
        }
        __syncthreads();
        if (kind == 0) mw_col_store<T>(B, sm.B1, PL, tile, n, g, c);
        else if (kind == 1) mw_col_store<T>(B, sm.B2, PL, tile, n, g, c);
        else if (kind == 2) mw_vec2_store<T>(B, sm.bv, n, g, c);
        if (vec3) mw_vec2_store<T>(V, sm.bv, n, g, c);
        if (wv == 0 && lane == 0) sm.ok[1] = okS;
    }
    __syncthreads();
    ok = ok && sm.ok[1];
    // ---- phase D: [Phi | phi] = R^{-T} Q^{-T} [X1 | x3] = V^T [X1 | x3]: the
    //      solve of (I + C P_j) [Phi | phi] = [F | v] (no I - C Y cancellation,
    //      see tmap_solve in combine_tiles.hpp) ----
    if (wv == 0) {
        WM<T> Vm, X1;
        WV<T> x3;
        wm_load(Vm, sm.B2, PL, n, false, 0.0, g, c);
        wm_load(X1, sm.B1, PL, n, false, 0.0, g, c);
        wv_load(x3, sm.bv, n, g, c);
        wv_tn(phi, Vm, x3, n, 1.0, (const WV<T> *)nullptr);
        if (!trans) wm_tn(Phi, Vm, X1, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);  // V^T X1
        else wm_tn(Phi, X1, Vm, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);        // Phi^T = X1^T V
    }
    return ok;
}

// k_seg_maps on a 4-wave block (CHOLESKY form, combine_mw.hpp): the same
// outputs.  V_j = suf_j (x) right is the P-only 4-wave combine; the map is
// mw_map's solve, with the products after the factorisations one deep and
// split over the waves by output tile.
template <int T, int NC = 0>
__global__ __launch_bounds__(256, 2) void k_seg_maps_mw(MapArgs A) {
    extern __shared__ __attribute__((aligned(16))) double mwbuf[];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
    const int n = NC ? NC : A.n, S = A.S, J = S + 1, nn = n * n;
    const int es = 3 * nn + 2 * n, mw = nn + n;
    const long long b = blockIdx.x / J;
    const int j = blockIdx.x % J;
    const MwSmem sm = mw_smem(mwbuf, n);
    const double *right = A.right ? A.right + b * (A.rstride ? A.rstride : (long long)es) : nullptr;
    double *vo = A.vfun + (b * J + j) * (long long)mw;
    double *mo = A.maps + (b * J + j) * (long long)mw;
    bool ok = true;
    const double *vP = nullptr, *vp = nullptr;
    // every global operand staged into LDS up front (one memory latency):
    // slot 0 the source element; slots 1, 2 suf_j and right when V_j is a
    // combine, else slot 1 the [P | p] of V_j (suf_j's or right's)
    double *es0 = mwbuf + mw_smem_doubles(n), *es1 = es0 + elem_slot(n), *es2 = es1 + elem_slot(n);
    const double *src_g = j > 0 ? A.elem + (b * S + j - 1) * (long long)es : A.left ? A.left + b * (long long)es
                                                                                   : nullptr;
    const bool vcomb = j < S && right;
    const double *vsrc = j < S ? A.suf + (b * S + j) * (long long)es : right;  // element holding V_j (or null)
    if (src_g) stage_range_blk(es0, src_g, es);
    if (vcomb) {
        stage_range_blk(es1, vsrc, es);
        stage_range_blk(es2, right, es);
    } else if (vsrc) {
        stage_range_blk(es1, vsrc + 2 * nn + n, mw);  // [P | p]
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (vcomb && NC == QD_N && PDPLQR_QD_COMBINE) {  // block-uniform
        // the junction elimination reads its operands only while assembling, long
        // before its (barrier-ordered) output stores: [P | p] goes straight into
        // es1 (V_j for the map below, no global round trip) and then to vfun
        ok = qd_combine(nullptr, nullptr, nullptr, es1, es1 + nn, elem_in(es1, n), elem_in(es2, n), false, mwbuf);
        for (int q = threadIdx.x; q < mw; q += 256) vo[q] = es1[q];
    } else if (vcomb) {
        ok = mw_combine_nc<T, NC>(nullptr, nullptr, nullptr, vo, vo + nn, elem_in(es1, n), elem_in(es2, n), n, false,
                                  mwbuf);
        __syncthreads();  // vo (written by waves 0 and 3) is complete; es1 is free
        for (int q = threadIdx.x; q < mw; q += 256) es1[q] = vo[q];
        __syncthreads();
    } else if (wv == 0) {
        for (int q = lane; q < mw; q += 64) vo[q] = vsrc ? es1[q] : 0.0;
    }
    if (vsrc) {
        vP = es1;
        vp = es1 + nn;
    }
    const double *src = src_g ? es0 : nullptr;
    WV<T> phi, x;
    bool have_x = false;  // j = 0: x_0 formed (wave 0)
    if (src && vP && NC == QD_N && PDPLQR_QD_COMBINE) {
        // n = 24: the map as ONE junction elimination (combine_qd.hpp).  The
        // element b_V = (I, 0, 0, P_j, p_j) -- no stages, value function V_j --
        // composed after e: its junction is (I + C P_j) x_j = F x + f - C p_j,
        // so (e (x) b_V).F = Phi_j and .f = phi_j.
        const int es = 3 * nn + 2 * n;
        for (int q = threadIdx.x; q < es; q += 256)
            es2[q] = q < nn ? ((q % (n + 1)) == 0 ? 1.0 : 0.0) : q < 2 * nn + n ? 0.0 : es1[q - (2 * nn + n)];
        __syncthreads();
        ok = qd_combine(es1, es1 + nn, es1 + 2 * nn, es1 + 2 * nn + n, es1 + 3 * nn + n, elem_in(src, n),
                        elem_in(es2, n), true, mwbuf) && ok;  // ends with a block barrier: es1 complete
        if (j > 0) {
            for (int q = threadIdx.x; q < mw; q += 256) mo[q] = q < nn ? es1[q] : es1[2 * nn + (q - nn)];
        } else if (wv == 0) {
            WM<T> PhiT;
            WV<T> x0v;
            wm_load(PhiT, es1, n, n, true, 0.0, g, c);
            wv_load(phi, es1 + 2 * nn, n, g, c);
            wv_load(x0v, A.x0 + b * (long long)n, n, g, c);
            wv_tn(x, PhiT, x0v, n, 1.0, &phi);
            have_x = true;
        }
        if (wv == 0) {  // x_0's lambda below reads P_0 from es2 (es1 now holds the map)
            vP = es2 + 2 * nn + n;
            vp = es2 + 3 * nn + n;
        }
    } else if (src && vP) {
        WM<T> Phi;
        ok = mw_map<T>(elem_in(src, n), vP, vp, n, sm, j == 0, Phi, phi) && ok;
        if (wv == 0) {
            if (j > 0) {
                wm_store(Phi, mo, n, n, g, c);
                wv_store(phi, mo + nn, n, g, c);
            } else {
                WV<T> x0v;
                wv_load(x0v, A.x0 + b * (long long)n, n, g, c);
                wv_tn(x, Phi, x0v, n, 1.0, &phi);
                have_x = true;
            }
        }
    } else if (wv == 0 && src) {  // no value function after this boundary: the map is the element's (F, f)
        const ElemIn e = elem_in(src, n);
        wv_load(phi, e.f, n, g, c);
        if (j > 0) {
            WM<T> Fs;
            wm_load(Fs, e.F, n, n, false, 0.0, g, c);
            wm_store(Fs, mo, n, n, g, c);
            wv_store(phi, mo + nn, n, g, c);
        } else {
            WM<T> PhiT;
            WV<T> x0v;
            wm_load(PhiT, src, n, n, true, 0.0, g, c);
            wv_load(x0v, A.x0 + b * (long long)n, n, g, c);
            wv_tn(x, PhiT, x0v, n, 1.0, &phi);
            have_x = true;
        }
    } else if (wv == 0 && j == 0) {  // x_0 itself
        wv_load(x, A.x0 + b * (long long)n, n, g, c);
        have_x = true;
    }
    if (!ok && threadIdx.x == 0) atomicOr(A.flag + b, 2);
    if (j > 0 || wv != 0 || !have_x) return;
    // j = 0: x_0 = Phi x0 + phi, lambda_0 = P_0 x_0 + p_0
    wv_store(x, mo + nn, n, g, c);
    wv_store(x, A.xhat + b * (long long)J * n, n, g, c);
    if (vP) {
        WM<T> Pv;
        WV<T> pv, lam;
        wm_load(Pv, vP, n, n, false, 0.0, g, c);
        wv_load(pv, vp, n, g, c);
        wv_tn(lam, Pv, x, n, 1.0, &pv);
        wv_store(lam, A.lam + b * (long long)J * n, n, g, c);
    }
}

// ---------------------------------------------------------------------------
// One Hillis-Steele round of the prefix composition of the boundary maps:
// m_j <- m_j o m_{j-d}.  Map 0 is the constant x_0, so after the round with
// distance d the entries j < 2 d are anchored at x0: their phi is x_j (written
// to xhat with lambda_j = P_j x_j + p_j) and their Phi is never read again.
// ---------------------------------------------------------------------------
template <int T>
__global__ __launch_bounds__(64) void k_map_scan(MapScanArgs A) {
    const int lane = wave_lane(), g = lane >> 4, c = lane & 15;
    const int n = A.n, J = A.S + 1, d = A.dist, nn = n * n, mw = nn + n;
    const long long b = blockIdx.x / J;
    const int j = blockIdx.x % J;
    const double *in = A.in + b * (long long)J * mw;
    double *out = A.out + b * (long long)J * mw;
    if (j < d) {  // anchored earlier: keep x_j for the next round's left operands
        for (int q = lane; q < n; q += 64) out[(long long)j * mw + nn + q] = in[(long long)j * mw + nn + q];
        return;
    }
    const int ia = j - d;
    const double *ej = in + (long long)j * mw, *ea = in + (long long)ia * mw;
    WM<T> PjT;
    WV<T> pa, pj, po;
    wm_load(PjT, ej, n, n, true, 0.0, g, c);
    wv_load(pa, ea + nn, n, g, c);
    wv_load(pj, ej + nn, n, g, c);
    wv_tn(po, PjT, pa, n, 1.0, &pj);  // Phi_j phi_a + phi_j
    wv_store(po, out + (long long)j * mw + nn, n, g, c);
    if (ia >= d) {  // not anchored yet: compose the matrices
        WM<T> Pa, Po;
        wm_load(Pa, ea, n, n, false, 0.0, g, c);
        wm_tn(Po, PjT, Pa, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);
        wm_store(Po, out + (long long)j * mw, n, n, g, c);
        return;
    }
    wv_store(po, A.xhat + (b * J + j) * (long long)n, n, g, c);
    const double *v = A.vfun + (b * J + j) * (long long)mw;
    WM<T> Pv;
    WV<T> pv, lam;
    wm_load(Pv, v, n, n, false, 0.0, g, c);
    wv_load(pv, v + nn, n, g, c);
    wv_tn(lam, Pv, po, n, 1.0, &pv);
    wv_store(lam, A.lam + (b * J + j) * (long long)n, n, g, c);
}

// Radix-R form of the same composition: one round of distance d composes m_j
// with m_{j-d}, m_{j-2d}, ..., m_{j-(R-1)d} in turn, stopping at the first
// anchored partner (index < d), so after the round the entries j < R d are
// anchored: ceil(log_R (S + 1)) launches instead of ceil(log2 (S + 1)), each at
// most R - 1 products in sequence.  The radix is chosen per solve (map_radix:
// the fewest rounds, then the smallest R for them) up to the compile-time RM
// the partner registers are sized for.  The running map is kept transposed
// (Phi^T), the form the matrix-vector product reads.
template <int T, int NC = 0, int RM = 4>
__device__ __forceinline__ void map_scan_block(const MapScanArgs &A, long long blk) {
    const int lane = wave_lane(), g = lane >> 4, c = lane & 15;
    const int n = NC ? NC : A.n, J = A.S + 1, d = A.dist, nn = n * n, mw = nn + n;
    const int R = A.radix;  // <= RM (launch_map_scan)
    const long long b = blk / J;
    const int j = (int)(blk % J);
    const double *in = A.in + b * (long long)J * mw;
    double *out = A.out + b * (long long)J * mw;
    if (j < d) {  // anchored earlier: keep x_j for this round's partners
        for (int q = lane; q < n; q += 64) out[(long long)j * mw + nn + q] = in[(long long)j * mw + nn + q];
        return;
    }
    // partners j - d, ..., j - K d; the K-th is anchored (index < d) when j / d <= R - 1.
    // Every operand is loaded up front (none depends on the running map), so
    // the round pays one memory latency, not one per partner.
    const int K = j / d < R - 1 ? j / d : R - 1;
    const bool anch = j / d <= R - 1;
    WM<T> PaccT, Pa[RM - 1];
    WV<T> pacc, pa[RM - 1];
    wm_load(PaccT, in + (long long)j * mw, n, n, true, 0.0, g, c);
    wv_load(pacc, in + (long long)j * mw + nn, n, g, c);
#pragma unroll
    for (int k = 0; k < RM - 1; ++k) {
        const double *ea = in + (long long)(j - (k + 1) * d) * mw;
        if (k < K) wv_load(pa[k], ea + nn, n, g, c);
        if (k < K - (anch ? 1 : 0)) wm_load(Pa[k], ea, n, n, false, 0.0, g, c);
    }
    WM<T> Pv;
    WV<T> pv;
    const double *v = A.vfun + (b * J + j) * (long long)mw;
    if (anch) {
        wm_load(Pv, v, n, n, false, 0.0, g, c);
        wv_load(pv, v + nn, n, g, c);
    }
    // (guards, no break / return inside: the loop must unroll, or the partner
    // arrays go to scratch)
    const int KM = anch ? K - 1 : K;  // matrix products before the anchored partner's vector one
#pragma unroll
    for (int k = 0; k < RM - 1; ++k) {
        if (k < KM) {
            WV<T> po;
            wv_tn(po, PaccT, pa[k], n, 1.0, &pacc);  // Phi_acc phi_a + phi_acc
            WM<T> Pn;
            wm_tn(Pn, Pa[k], PaccT, n, 1.0, 0.0, (const WM<T> *)nullptr, g, c);  // Phi_a^T Phi_acc^T = (Phi_acc Phi_a)^T
            PaccT = Pn;
            pacc = po;
        }
    }
    if (anch) {  // anchored partner K - 1: x_j = Phi_acc x_a + phi_acc
        WV<T> po, xa;
#pragma unroll
        for (int k = 0; k < RM - 1; ++k)
            if (k == K - 1) xa = pa[k];
        wv_tn(po, PaccT, xa, n, 1.0, &pacc);
        wv_store(po, out + (long long)j * mw + nn, n, g, c);
        wv_store(po, A.xhat + (b * J + j) * (long long)n, n, g, c);
        WV<T> lam;
        wv_tn(lam, Pv, po, n, 1.0, &pv);
        wv_store(lam, A.lam + (b * J + j) * (long long)n, n, g, c);
        return;
    }
    wm_store_t(PaccT, out + (long long)j * mw, n, g, c);  // Phi_acc (natural) from its transpose
    wv_store(pacc, out + (long long)j * mw + nn, n, g, c);
}

template <int T, int NC = 0, int RM = 4>
__global__ __launch_bounds__(64) void k_map_scanR(MapScanArgs A) {
    map_scan_block<T, NC, RM>(A, blockIdx.x);
}

// Largest radix of the one-wave composition kernels: the partners' registers
// (RM - 1 maps of WM<T>) and R - 1 products in sequence per round.  12 x 12
// maps (T = 1): 2 rounds of radix 17 take 7.0 + 7.4 us against 4 radix-4
// rounds of 4.7 us (C2, gpurun r6e).  24 x 24 (T = 2): a product in the chain
// costs ~1.5 us, so radix 8 (3 rounds of 11.4-14.1 us, the C4 rank, r6f) loses
// to radix 4 (5 rounds of ~6.9 us).
static inline int map_radix_max(int n) { return n <= 16 ? 17 : 4; }

int map_radix(int n, int J) {
    if (PDPLQR_MAP_RADIX != 4) return PDPLQR_MAP_RADIX;
    if (xl_state(n) || wide_state(n)) return 4;  // (k_map_scan_wide / _xl: radix-4 rounds)
    const int RM = map_radix_max(n);
    auto rounds = [&](int R) {
        int r = 0;
        for (long long d = 1; d < J; d *= R) ++r;
        return r;
    };
    const int best = rounds(RM);
    int R = 2;
    while (rounds(R) > best) ++R;
    return R;
}

static int tile_order(int n);

// dynamic LDS of the 4-wave kernels: the combine's own + staged operand elements
static size_t mw_scan_bytes(int n) { return (size_t)(mw_smem_doubles(n) + 2 * elem_slot(n)) * sizeof(double); }
static size_t mw_maps_bytes(int n) { return (size_t)(mw_smem_doubles(n) + 3 * elem_slot(n)) * sizeof(double); }

// n = 24 (the C4 horizon shape) runs kernel instances with n a compile-time
// constant: every bounds guard of the tile loads / stores folds away (the
// runtime-n scan kernel is ~14 k instructions, past the instruction cache a
// 4-wave block with four different phase paths cycles through).
static inline bool ct_n24(int n) { return n == 24; }
// n = 12 (the C2 / headline state size) likewise for the n <= 16 kernels
static inline bool ct_n12(int n) { return n == 12; }

// the 4-wave combine runs the CHOLESKY rounds at T = 2 (PDPLQR_SCAN_1WAVE: the
// one-wave k_seg_scan; PDPLQR_SCAN_MW=1 also at T = 1, A/B)
// (n <= 16 keeps the one-wave combines: the 4-wave ones in Sklansky rounds
// measured C2 0.113 against 0.103 ms with the two-round k_seg_scan4, r5q)
bool seg_scan_mw(int n, bool lu, int mw) {
    if (!mw || lu) return false;
    return tile_order(n) == 2;
}

// Resident scan combines the device holds for this shape.
int seg_scan_slots(const Shape &sh, int device) {
    if (xl_state(sh.n)) return xl_par_slots(device);
    if (wide_state(sh.n)) return wide_scan_slots(sh.n, device);
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
    const size_t smem = op_stage_bytes(sh.n);
    hipError_t e;
    if (seg_scan_mw(sh.n, false, sh.mw))
        e = sh.n <= 16 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_seg_scan_mw<1>, 256, mw_scan_bytes(sh.n))
                       : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_seg_scan_mw<2>, 256, mw_scan_bytes(sh.n));
    else
        e = sh.n <= 16 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_seg_scan<1, false>, 64, smem)
                       : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_seg_scan<2, false>, 64, smem);
    if (e != hipSuccess || per <= 0) per = 1;
    return cus * per;
}

static size_t elems_smem(int n, int elems) { return (size_t)elems * (3 * n * n + 2 * n) * sizeof(double); }

static int tile_order(int n) { return n <= 16 ? 1 : (n <= 32 ? 2 : 0); }

// T = 1 only: at T = 2 two waves' combine LDS (~75 KB a block) halves the
// resident blocks, and C4's scans need every slot.
bool seg_scan4_supported(int n) { return tile_order(n) == 1; }

int launch_seg_scan4(const ScanArgs &a, int batch, hipStream_t st) {
    const dim3 grid((unsigned)(batch * a.S)), blk(128);
    const size_t smem = 2 * op_stage_bytes(a.n);
    if (!seg_scan4_supported(a.n) || !a.scratch) return PDPLQR_ERR_UNSUPPORTED;
    const size_t smem_qd1 = 2 * 2 * (size_t)elem_slot(a.n) * sizeof(double);  // whole operand elements (QD1)
    if (a.lu) hipLaunchKernelGGL((k_seg_scan4<1, true>), grid, blk, smem, st, a);
    else if (ct_n12(a.n)) hipLaunchKernelGGL((k_seg_scan4<1, false, 12>), grid, blk, (use_qd1<12, false>() ? smem_qd1 : smem),
                                             st, a);
    else hipLaunchKernelGGL((k_seg_scan4<1, false>), grid, blk, smem, st, a);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

int launch_seg_scan(const ScanArgs &a, int batch, hipStream_t st) {
    if (xl_state(a.n)) return launch_seg_scan_xl(a, batch, st);
    if (wide_state(a.n)) {
        if (a.sk) return PDPLQR_ERR_UNSUPPORTED;  // the wide combine reads its operands from HBM
        return launch_seg_scan_wide(a, batch, st);
    }
    const dim3 grid((unsigned)(batch * scan_round_blocks(a.S, a.dist, a.sk))), blk(64);
    const int T = tile_order(a.n);
    const size_t smem = op_stage_bytes(a.n);
    if (seg_scan_mw(a.n, a.lu, a.mw)) {
        const size_t sm = mw_scan_bytes(a.n);
        if (T == 1) hipLaunchKernelGGL(k_seg_scan_mw<1>, grid, dim3(256), sm, st, a);
        else if (ct_n24(a.n)) hipLaunchKernelGGL((k_seg_scan_mw<2, 24>), grid, dim3(256), sm, st, a);
        else hipLaunchKernelGGL(k_seg_scan_mw<2>, grid, dim3(256), sm, st, a);
        PDPLQR_HIP_TRY(hipGetLastError());
        return PDPLQR_OK;
    }
    if (T == 1 && a.lu) hipLaunchKernelGGL((k_seg_scan<1, true>), grid, blk, smem, st, a);
    else if (T == 1) hipLaunchKernelGGL((k_seg_scan<1, false>), grid, blk, smem, st, a);
    else if (T == 2 && a.lu) hipLaunchKernelGGL((k_seg_scan<2, true>), grid, blk, smem, st, a);
    else if (T == 2 && ct_n24(a.n)) hipLaunchKernelGGL((k_seg_scan<2, false, 24>), grid, blk, smem, st, a);
    else if (T == 2) hipLaunchKernelGGL((k_seg_scan<2, false>), grid, blk, smem, st, a);
    else return PDPLQR_ERR_UNSUPPORTED;
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

int launch_seg_maps(const MapArgs &a, int batch, hipStream_t st) {
    if (xl_state(a.n)) return launch_seg_maps_xl(a, batch, st);
    if (wide_state(a.n)) return launch_seg_maps_wide(a, batch, st);
    const dim3 grid((unsigned)(batch * (a.S + 1))), blk(64);
    const int T = tile_order(a.n);
    if (seg_scan_mw(a.n, a.lu, a.mw)) {
        const size_t sm = mw_maps_bytes(a.n);
        if (T == 1) hipLaunchKernelGGL(k_seg_maps_mw<1>, grid, dim3(256), sm, st, a);
        else if (ct_n24(a.n)) hipLaunchKernelGGL((k_seg_maps_mw<2, 24>), grid, dim3(256), sm, st, a);
        else hipLaunchKernelGGL(k_seg_maps_mw<2>, grid, dim3(256), sm, st, a);
        PDPLQR_HIP_TRY(hipGetLastError());
        return PDPLQR_OK;
    }
    const size_t smem = (a.right ? op_stage_bytes(a.n) : 0) + (size_t)(tmap_smem_doubles(a.n) + a.n * a.n + a.n) * sizeof(double);
    if (T == 1 && a.lu) hipLaunchKernelGGL((k_seg_maps<1, true>), grid, blk, smem, st, a);
    else if (T == 1 && ct_n12(a.n)) hipLaunchKernelGGL((k_seg_maps<1, false, 12>), grid, blk, smem, st, a);
    else if (T == 1) hipLaunchKernelGGL((k_seg_maps<1, false>), grid, blk, smem, st, a);
    else if (T == 2 && a.lu) hipLaunchKernelGGL((k_seg_maps<2, true>), grid, blk, smem, st, a);
    else if (T == 2 && ct_n24(a.n)) hipLaunchKernelGGL((k_seg_maps<2, false, 24>), grid, blk, smem, st, a);
    else if (T == 2) hipLaunchKernelGGL((k_seg_maps<2, false>), grid, blk, smem, st, a);
    else return PDPLQR_ERR_UNSUPPORTED;
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

int launch_map_scan(const MapScanArgs &a, int batch, hipStream_t st) {
    if (xl_state(a.n)) return launch_map_scan_xl(a, batch, st);
    if (wide_state(a.n)) {
        static_assert(PDPLQR_MAP_RADIX == 4, "k_map_scan_wide composes radix-4 rounds");
        return launch_map_scan_wide(a, batch, st);
    }
    const dim3 grid((unsigned)(batch * (a.S + 1))), blk(64);
    const int T = tile_order(a.n);
    if (PDPLQR_MAP_RADIX == 4) {
        if (a.radix < 2 || a.radix > map_radix_max(a.n)) return PDPLQR_ERR_INVALID;
        if (T == 1 && ct_n12(a.n)) hipLaunchKernelGGL((k_map_scanR<1, 12, 17>), grid, blk, 0, st, a);
        else if (T == 1) hipLaunchKernelGGL((k_map_scanR<1, 0, 17>), grid, blk, 0, st, a);
        else if (T == 2 && ct_n24(a.n)) hipLaunchKernelGGL((k_map_scanR<2, 24, 4>), grid, blk, 0, st, a);
        else if (T == 2) hipLaunchKernelGGL((k_map_scanR<2, 0, 4>), grid, blk, 0, st, a);
        else return PDPLQR_ERR_UNSUPPORTED;
    } else if (T == 1) hipLaunchKernelGGL(k_map_scan<1>, grid, blk, 0, st, a);
    else if (T == 2) hipLaunchKernelGGL(k_map_scan<2>, grid, blk, 0, st, a);
    else return PDPLQR_ERR_UNSUPPORTED;
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

// Fold the all-gathered rank elements (horizon-sharded solve).  Block b
// (< batch) folds the prefix out_pre = e_0 (x) ... (x) e_{r-1} of problem b
// (identity if r = 0); block batch + b folds the suffix out_suf =
// e_{r+1} (x) ... (x) e_{R-1}.  The two chains run concurrently, and each
// combine forms only what its consumer reads: k_seg_maps maps x0 through the
// prefix's (F, C, f) and right-folds the suffix's value function (P, p) into
// the boundary value functions, and a right fold e_j (x) acc reads acc's
// (P, p) only.  So the prefix chain skips the P path and the suffix chain the
// F, C path; the unformed blocks are written as zeros.
template <int T, bool LU>
__global__ __launch_bounds__(64) void k_fold_shards(const double *elems_all, int R, int r, int n, int batch,
                                                    double *out_pre_all, double *out_suf_all, int *has_suf, int *flag) {
    extern __shared__ __attribute__((aligned(16))) double dyn[];
    __shared__ CombSmem<T> sm;
    const int lane = wave_lane();
    const int es = 3 * n * n + 2 * n, nfcf = 2 * n * n + n;
    const bool suffix = blockIdx.x >= (unsigned)batch;
    const long long b = suffix ? blockIdx.x - batch : blockIdx.x;
    // element j of problem b: elems_all[(j * batch + b) * es]; outputs [b][es]
    const double *elems = elems_all + b * es;
    const long long stride = (long long)batch * es;
    double *acc = dyn, *nx = dyn + es, *o = dyn + 2 * es;
    if (!suffix) {
        double *out = out_pre_all + b * es;
        if (r == 0) {
            for (int q = lane; q < es; q += 64) out[q] = (q < n * n && q % n == q / n) ? 1.0 : 0.0;
            return;
        }
        elem_copy(acc, elems, n, lane);
        wave_sync();
        for (int j = 1; j < r; ++j) {
            elem_copy(nx, elems + (long long)j * stride, n, lane);
            wave_sync();
            if (!tcombine<T, LU>(o, acc, nx, n, true, false, sm, lane) && lane == 0) atomicOr(flag + b, 4);
            wave_sync();
            double *t = acc;
            acc = o;
            o = t;
        }
        for (int q = lane; q < es; q += 64) out[q] = q < nfcf ? acc[q] : 0.0;
        return;
    }
    double *out = out_suf_all + b * es;
    if (r + 1 >= R) {
        if (lane == 0 && b == 0) *has_suf = 0;
        return;
    }
    elem_copy(acc, elems + (long long)(R - 1) * stride, n, lane);
    wave_sync();
    for (int j = R - 2; j > r; --j) {
        elem_copy(nx, elems + (long long)j * stride, n, lane);
        wave_sync();
        if (!tcombine<T, LU>(o, nx, acc, n, false, true, sm, lane) && lane == 0) atomicOr(flag + b, 8);
        wave_sync();
        double *t = acc;
        acc = o;
        o = t;
    }
    for (int q = lane; q < es; q += 64) out[q] = q < nfcf ? 0.0 : acc[q];
    if (lane == 0 && b == 0) *has_suf = 1;
}

// Log-depth alternative of the prefix chain (pdplqr_shard_forward picks it
// when it is shorter): with the rank suffix scan done (suf [b][R][es], entry
// j = e_j (x) ... (x) e_{R-1}), the state at the start of rank j + 1's slice
// follows from the state at the start of rank j's through the boundary map
// of e_j under V_{j+1} = (P, p) of suffix entry j + 1 -- the same map as
// k_seg_maps, Phi = Z F, phi = Z (f - C p), Z = (I + C P)^{-1}.  The r maps
// of ranks j < r are formed in parallel (k_rank_maps); one wave applies them
// to x0 in turn (k_rank_chain, matrix-vector products only) and writes the
// prefix element (F = C = 0, f = x at the slice start), which k_seg_maps
// maps to exactly that state.
template <int T, bool LU>
__global__ __launch_bounds__(64) void k_rank_maps(const double *elems_all, const double *suf, int R, int r, int n,
                                                  int batch, double *maps, int *flag) {
    extern __shared__ __attribute__((aligned(16))) double dyn[];  // tmap_solve scratch
    const int lane = wave_lane();
    const int nn = n * n, es = 3 * nn + 2 * n, mw = nn + n;
    const long long b = blockIdx.x / r;
    const int j = blockIdx.x % r;
    const double *src = elems_all + ((long long)j * batch + b) * es;  // e_j, rank-major all-gather
    const double *v = suf + (b * R + j + 1) * (long long)es;           // V_{j+1}
    double *mo = maps + (b * r + j) * (long long)mw;
    double *mout = dyn + tmap_smem_doubles(n);
    // [Phi | phi] = (I + C P)^{-1} [F | f - C p]
    const bool ok = tmap_solve<T, LU>(src, src + nn, src + 2 * nn, v + 2 * nn + n, v + 3 * nn + n, n, dyn, mout, lane);
    for (int q = lane; q < mw; q += 64) mo[q] = mout[q];
    if (!ok && lane == 0) atomicOr(flag + b, 4);
}

// k_rank_maps on a 4-wave block (CHOLESKY form): the map of e_j under
// V_{j+1} by mw_map, both operands staged into LDS first.  A one-wave
// tmap_solve chains three triangular solves after the factorisations
// (43 us per launch at n = 24); mw_map spreads them over the waves.
template <int T, int NC = 0>
__global__ __launch_bounds__(256) void k_rank_maps_mw(const double *elems_all, const double *suf, int R, int r, int n_,
                                                      int batch, double *maps, int *flag) {
    extern __shared__ __attribute__((aligned(16))) double mwbuf[];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
    const int n = NC ? NC : n_;
    const int nn = n * n, es = 3 * nn + 2 * n, mw = nn + n;
    const long long b = blockIdx.x / r;
    const int j = blockIdx.x % r;
    const MwSmem sm = mw_smem(mwbuf, n);
    double *es0 = mwbuf + mw_smem_doubles(n), *es1 = es0 + elem_slot(n);
    stage_range_blk(es0, elems_all + ((long long)j * batch + b) * es, es);           // e_j (rank-major all-gather)
    stage_range_blk(es1, suf + (b * R + j + 1) * (long long)es + 2 * nn + n, mw);  // [P | p] of V_{j+1}
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    WM<T> Phi;
    WV<T> phi;
    const bool ok = mw_map<T>(elem_in(es0, n), es1, es1 + nn, n, sm, false, Phi, phi);
    double *mo = maps + (b * r + j) * (long long)mw;
    if (wv == 0) {
        wm_store(Phi, mo, n, n, g, c);
        wv_store(phi, mo + nn, n, g, c);
    }
    if (!ok && threadIdx.x == 0) atomicOr(flag + b, 4);
}

template <int T>
__global__ __launch_bounds__(64) void k_rank_chain(const double *maps, const double *x0, int r, int n,
                                                   double *out_pre_all) {
    const int lane = wave_lane(), g = lane >> 4, c = lane & 15;
    const int nn = n * n, es = 3 * nn + 2 * n, mw = nn + n;
    const long long b = blockIdx.x;
    WV<T> x;
    wv_load(x, x0 + b * n, n, g, c);
    WM<T> PhiT;
    WV<T> phi;
    wm_load(PhiT, maps + b * r * (long long)mw, n, n, true, 0.0, g, c);
    wv_load(phi, maps + b * r * (long long)mw + nn, n, g, c);
    for (int j = 0; j < r; ++j) {
        WV<T> y;
        wv_tn(y, PhiT, x, n, 1.0, &phi);  // x <- Phi_j x + phi_j
        x = y;
        if (j + 1 < r) {  // the next map's loads do not depend on x
            const double *mo = maps + (b * r + j + 1) * (long long)mw;
            wm_load(PhiT, mo, n, n, true, 0.0, g, c);
            wv_load(phi, mo + nn, n, g, c);
        }
    }
    double *out = out_pre_all + b * es;
    for (int q = lane; q < es; q += 64)
        if (q < 2 * nn || q >= 2 * nn + n) out[q] = 0.0;
    wv_store(x, out + 2 * nn, n, g, c);
}

int launch_rank_fold_maps(const double *elems, const double *suf, const double *x0, int R, int r, int n, int batch,
                          double *maps, double *out_pre, int *flag, bool lu, hipStream_t st, double *xlw,
                          int xl_grid) {
    if (r <= 0) return PDPLQR_OK;
    if (xl_state(n))
        return launch_rank_fold_maps_xl(elems, suf, x0, R, r, n, batch, maps, out_pre, flag, lu, xlw, xl_grid, st);
    if (wide_state(n)) return launch_rank_fold_maps_wide(elems, suf, x0, R, r, n, batch, maps, out_pre, flag, lu, st);
    const int T = tile_order(n);
    const dim3 gm(batch * r), blk(64);
    const size_t rsm = (size_t)(tmap_smem_doubles(n) + n * n + n) * sizeof(double);
    if (T == 1) {
        if (lu) hipLaunchKernelGGL((k_rank_maps<1, true>), gm, blk, rsm, st, elems, suf, R, r, n, batch, maps, flag);
        else hipLaunchKernelGGL((k_rank_maps<1, false>), gm, blk, rsm, st, elems, suf, R, r, n, batch, maps, flag);
        hipLaunchKernelGGL(k_rank_chain<1>, dim3(batch), dim3(64), 0, st, maps, x0, r, n, out_pre);
    } else if (T == 2) {
        if (lu) hipLaunchKernelGGL((k_rank_maps<2, true>), gm, blk, rsm, st, elems, suf, R, r, n, batch, maps, flag);
        else if (seg_scan_mw(n, false) && ct_n24(n))
            hipLaunchKernelGGL((k_rank_maps_mw<2, 24>), gm, dim3(256),
                               (size_t)(mw_smem_doubles(n) + elem_slot(n) + ((n * n + n + 1) & ~1)) * sizeof(double),
                               st, elems, suf, R, r, n, batch, maps, flag);
        else if (seg_scan_mw(n, false))
            hipLaunchKernelGGL(k_rank_maps_mw<2>, gm, dim3(256),
                               (size_t)(mw_smem_doubles(n) + elem_slot(n) + ((n * n + n + 1) & ~1)) * sizeof(double),
                               st, elems, suf, R, r, n, batch, maps, flag);
        else hipLaunchKernelGGL((k_rank_maps<2, false>), gm, blk, rsm, st, elems, suf, R, r, n, batch, maps, flag);
        hipLaunchKernelGGL(k_rank_chain<2>, dim3(batch), dim3(64), 0, st, maps, x0, r, n, out_pre);
    } else {
        return PDPLQR_ERR_UNSUPPORTED;
    }
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

// One level of the rank-fold trees (RankTreeArgs) on 4-wave blocks: block
// (b, q) combines one pair of the prefix list (q < its block count) or of the
// suffix list with mw_combine, both operands staged in LDS first (the scan
// round's body).  A suffix pair whose right operand is the list's last partial
// holds the real terminal: P, p only, [F | C | f] zeroed (k_seg_maps reads
// only the suffix's value function, the prefix's (F, C, f)).  Depth
// max(ceil(log2 r), ceil(log2(R - 1 - r))) combines, against ceil(log2 R)
// scan rounds plus the boundary-map round and the map chain of the scan form.
template <int T, int NC = 0>
__global__ __launch_bounds__(256, 2) void k_rank_tree_mw(RankTreeArgs A) {
    extern __shared__ __attribute__((aligned(16))) double mwbuf[];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n = NC ? NC : A.n, nn = n * n, es = 3 * nn + 2 * n;
    const int per = rank_tree_blocks(A.r, A.level) + rank_tree_blocks(A.R - 1 - A.r, A.level);
    const long long b = blockIdx.x / per;
    const RankTreeOp op = rank_tree_op(A.R, A.r, A.level, (int)(blockIdx.x % per));  // block-uniform
    auto src = [&](int i) {
        return A.level == 0 ? A.gathered + (long long)i * A.gstride + b * es : A.in + (b * A.R + i) * (long long)es;
    };
    const double *ia = src(op.a);
    double *o = op.dst < 0 ? (op.suf ? A.right : A.left) + b * es : A.out + (b * A.R + op.dst) * (long long)es;
    if (op.carry) {  // odd last partial: carried to the next level
        if (wv == 0) elem_copy(o, ia, n, lane);
        return;
    }
    const double *ib = src(op.b);
    const bool fcf = op.fcf, suf = op.suf;
    double *ea = mwbuf + mw_smem_doubles(n), *eb = ea + elem_slot(n);
    stage_range_blk(ea, ia, es);
    stage_range_blk(eb, ib, es);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const bool ok = mw_combine_nc<T, NC>(o, o + nn, o + 2 * nn, o + 2 * nn + n, o + 3 * nn + n, elem_in(ea, n),
                                         elem_in(eb, n), n, fcf, mwbuf);
    if (!fcf && wv == 1)
        for (int p = lane; p < 2 * nn + n; p += 64) o[p] = 0.0;  // [F | C | f]
    if (!ok && threadIdx.x == 0) atomicOr(A.flag + b, suf ? 8 : 4);
}

int launch_rank_tree(const RankTreeArgs &a, int batch, hipStream_t st) {
    const int per = rank_tree_blocks(a.r, a.level) + rank_tree_blocks(a.R - 1 - a.r, a.level);
    if (per == 0) return PDPLQR_OK;
    if (!seg_scan_mw(a.n, false) || wide_state(a.n)) return PDPLQR_ERR_UNSUPPORTED;
    const dim3 grid((unsigned)(batch * per));
    const size_t sm = mw_scan_bytes(a.n);
    if (ct_n24(a.n)) hipLaunchKernelGGL((k_rank_tree_mw<2, 24>), grid, dim3(256), sm, st, a);
    else hipLaunchKernelGGL(k_rank_tree_mw<2>, grid, dim3(256), sm, st, a);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

int launch_fold_shards(const double *elems, int R, int r, int n, int batch, double *out_pre, double *out_suf,
                       int *has_suf, int *flag, bool lu, hipStream_t st) {
    const int T = tile_order(n);
    const dim3 gr(2 * batch), blk(64);
    const size_t sm = elems_smem(n, 3);
    if (T == 1 && lu)
        hipLaunchKernelGGL((k_fold_shards<1, true>), gr, blk, sm, st, elems, R, r, n, batch, out_pre, out_suf, has_suf,
                           flag);
    else if (T == 1)
        hipLaunchKernelGGL((k_fold_shards<1, false>), gr, blk, sm, st, elems, R, r, n, batch, out_pre, out_suf,
                           has_suf, flag);
    else if (T == 2 && lu)
        hipLaunchKernelGGL((k_fold_shards<2, true>), gr, blk, sm, st, elems, R, r, n, batch, out_pre, out_suf, has_suf,
                           flag);
    else if (T == 2)
        hipLaunchKernelGGL((k_fold_shards<2, false>), gr, blk, sm, st, elems, R, r, n, batch, out_pre, out_suf,
                           has_suf, flag);
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
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(pdplqr::g_comb_t), sizeof(unsigned long long) * 1024 * 32) == hipSuccess ? 0 : -2;
}
#endif
