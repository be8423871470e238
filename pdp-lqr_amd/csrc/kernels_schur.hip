// kernels_schur.hip -- value-matrix form of the batched backward Riccati
// (keep_factors = 0, n + m <= 16).
//
// The reference's step_with_factorization (lqr_kernel.hpp:104-147) factors the
// whole stage matrix M_k = H~_k + E^T Lxx_{k+1} Lxx_{k+1}^T E and carries the
// square-root factor Lxx_k to the next stage.  What leaves a stage is
//   * the u-columns of the factor, L(:, 0:m) = [Luu; Lxu], and lu' = Luu^{-1} lu
//     (the rollout record consumed by forward_step, :181-212), and
//   * the value function P_k = Lxx Lxx^T, p_k = lp_x - Lxu lu'.
// P_k is exactly the trailing block left after eliminating only the m
// u-pivots of M_k (Mxx - Lxu Lxu^T), so this kernel never factors the x block:
// it keeps P_{k+1} as the trailing block of the previous stage's tile, in
// MFMA C layout registers, and forms
//     G   = P_{k+1} E~            (MFMA; A operand = P's own registers by symmetry)
//     M_k = H~_k + E~^T G         (MFMA; B operand = G's registers, no data movement)
//     lp  = h~_k + G^T c~ + E~^T p~_{k+1}   (= h~ + E^T (P c + p), :138-143)
// where E~ is E embedded at the x rows m..s-1 of the 16-wide tile.  Then m
// right-looking pivots (chol_tiles, augmented with lp) leave P_k, p_k in place.
// Per stage this is 4 pivots instead of 16 and no L round trip through LDS.
//
// The factor cache (keep_factors = 1, needed by backward_without_factorization
// and get_value_function) still takes the full-factor kernels.
#include "device_common.hpp"

#include <stdint.h>
#include <stdlib.h>

namespace pdplqr {

// Stage-k inputs of one lane.
struct SchurIn {
    double E[4];   // E~[4 kk + g][c]   (x row t = 4 kk + g - m, column c)
    double ct[4];  // c~[4 kk + g]
    d4 H;          // H~[4 r + g][c]    (identity on the padding)
    double h;      // h~[c]
};

// Loads stage inputs from a stage record: E (n x s, column-major), c (n),
// packed lower H~ (s), h~ (s).  Works on global memory and on the LDS copy.
__device__ __forceinline__ void schur_load(SchurIn &in, const double *__restrict__ Ek, const double *__restrict__ ck,
                                           const double *__restrict__ Hk, const double *__restrict__ hk, int n,
                                           int m, int s, int g, int c) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
        const int t = 4 * kk + g - m;
        const bool xr = t >= 0 && t < n;
        in.E[kk] = (xr && c < s) ? Ek[t + c * n] : 0.0;
        in.ct[kk] = xr ? ck[t] : 0.0;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = 4 * r + g;
        in.H[r] = (i < s && c < s) ? Hk[i >= c ? pidx(i, c, s) : pidx(c, i, s)] : (i == c ? 1.0 : 0.0);
    }
    in.h = (c < s) ? hk[c] : 0.0;
}

struct SchurSmem {
    alignas(16) double col[16];  // pivot-row broadcast (colpos order)
    alignas(16) double lpt[16];  // lp_k, column -> row redistribution (colpos order)
    double inv[16];              // 1 / sqrt(pivot), u columns
    double luq[16];              // lu' = Luu^{-1} lu
    union {
        double tp[16 * 17];           // transpose of P_k (odd leading dimension: conflict-free)
        alignas(16) double rec[128];  // rollout record staging (one coalesced store per stage)
    };
};

// One stage.  Pm: in = tile whose trailing (x) block is P_{k+1}; out = M_k
// after the m u-pivots (trailing block P_k, u columns unscaled L).  prow:
// p~ in row layout (prow[r] = p[4 r + g - m] on x rows).
__device__ __forceinline__ bool schur_stage(d4 &Pm, double (&prow)[4], const SchurIn &in, SchurSmem &sm, int m,
                                            int s, int g, int c) {
    const int k0 = m >> 2, k1 = (s - 1) >> 2;  // K chunks that hold x rows
    d4 G = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
        if (kk >= k0 && kk <= k1) G = mfma_f64(Pm[kk], in.E[kk], G);
    d4 Mn = in.H;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
        if (kk >= k0 && kk <= k1) Mn = mfma_f64(in.E[kk], G[kk], Mn);
    double part = 0.0;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
        if (kk >= k0 && kk <= k1) {
            part = __builtin_fma(G[kk], in.ct[kk], part);
            part = __builtin_fma(in.E[kk], prow[kk], part);
        }
    part = sum_groups(part);
    if (g == 0) sm.lpt[colpos<1>(c)] = in.h + part;
    wave_sync();
    double lpr[1][4];
    {
        const double2 *q = reinterpret_cast<const double2 *>(sm.lpt + 4 * g);
        const double2 a = q[0], b = q[1];
        lpr[0][0] = a.x;
        lpr[0][1] = a.y;
        lpr[0][2] = b.x;
        lpr[0][3] = b.y;
    }
    d4 Mt[1][1];
    Mt[0][0] = Mn;
    bool ok = chol_tiles<1>(Mt, lpr, sm.col, sm.inv, sm.luq, 0, m, m, true, g, c);
    Pm = Mt[0][0];
#pragma unroll
    for (int r = 0; r < 4; ++r) prow[r] = lpr[0][r];
    // P_k <- (P_k + P_k^T) / 2.  The square-root recursion is symmetric by
    // construction; here the rounding-level antisymmetric part of M_k would
    // otherwise be carried as A^T e A from stage to stage and grow with the
    // open-loop dynamics (the next stage reads P's registers as P^T).
#pragma unroll
    for (int r = 0; r < 4; ++r) sm.tp[(4 * r + g) * 17 + c] = Pm[r];
    wave_sync();
#pragma unroll
    for (int r = 0; r < 4; ++r) Pm[r] = 0.5 * (Pm[r] + sm.tp[c * 17 + 4 * r + g]);
    // P_k = Lxx Lxx^T has a positive diagonal whenever M_k is positive definite
    bool bad = false;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = 4 * r + g;
        if (i == c && i >= m && i < s && !(Pm[r] > 0.0)) bad = true;
    }
    return ok && !__any(bad);
}

// Rollout record FR_k = [L(:, 0:m) | lu'] (same format as the full-factor path).
__device__ __forceinline__ void schur_store_record(double *FRk, const d4 &Pm, const SchurSmem &sm, int m, int s,
                                                   int g, int c) {
    if (c < m) {
        const double iv = sm.inv[c];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 4 * r + g;
            if (i < s) gstore(FRk + c * s + i, (i >= c) ? Pm[r] * iv : 0.0);
        }
    }
    const int lane = 16 * g + c;
    if (lane < m) gstore(FRk + s * m + lane, sm.luq[lane]);
}

// Same record, staged in LDS and written with one dwordx4 store instruction
// (lanes < FS/2): coalesced, and a fixed vm-op count for the DMA accounting.
template <int M, int S>
__device__ __forceinline__ void schur_store_record_staged(double *FRk, const d4 &Pm, SchurSmem &sm, int g, int c) {
    constexpr int FS = S * M + M;
    static_assert(FS % 2 == 0 && FS <= 128, "record staging");
    const int lane = 16 * g + c;
    if (c < M) {
        const double iv = sm.inv[c];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 4 * r + g;
            if (i < S) sm.rec[c * S + i] = (i >= c) ? Pm[r] * iv : 0.0;
        }
    }
    if (lane < M) sm.rec[S * M + lane] = sm.luq[lane];
    wave_sync();
    if (lane < FS / 2) gstore2(FRk + 2 * lane, reinterpret_cast<const d2v *>(sm.rec)[lane]);
}

// Stage-record layout of the LDS-DMA variant (compile-time shapes).
template <int NN, int MM>
struct SchurShape {
    static constexpr int n = NN, m = MM, s = NN + MM;
    static constexpr int ps = s * (s + 1) / 2;
    static constexpr int OE = 0, OC = n * s, OH = OC + n, OP = OH + s, Q = OP + ps;
    static constexpr int CH = Q / 2, NI = (CH + 63) / 64;
    static constexpr bool ok = (n * s) % 2 == 0 && n % 2 == 0 && s % 2 == 0 && ps % 2 == 0 && s <= 16;
};

#ifndef PDPLQR_SCHUR_WAVES
#define PDPLQR_SCHUR_WAVES 4
#endif

// NN = MM = 0: runtime shape, register prefetch of the next stage.
// NN, MM > 0 : compile-time shape, stage records streamed by LDS-DMA
//              (global_load_lds_dwordx4) into a double buffer.
template <int NN, int MM>
__global__ __launch_bounds__(64, (NN > 0 ? PDPLQR_SCHUR_WAVES : 3)) void k_riccati_bwd_schur(RiccatiArgs A) {
    constexpr bool CT = NN > 0;
    using SH = SchurShape<(CT ? NN : 2), (CT ? MM : 2)>;
    constexpr int NI = CT ? SH::NI : 1;
    __shared__ SchurSmem sm;
    __shared__ __attribute__((aligned(16))) double stg[CT ? 2 : 1][CT ? NI * 128 : 2];
    const int lane = threadIdx.x, g = lane >> 4, c = lane & 15;
    const long long b = blockIdx.x;
    const Shape &sh = A.sh;
    const int n = CT ? NN : sh.n, m = CT ? MM : sh.m, s = n + m;
    const int ps = CT ? SH::ps : sh.ps;
    const int N = sh.N;
    const double *Eb = A.E + b * sh.perE;
    const double *cb = A.c + b * sh.perc;
    const double *Hb = A.Hw + b * sh.perHw;
    const double *hb = A.hw + b * sh.perh;
    double *FRb = A.KD + b * sh.perKD;
    const int frs = s * m + m;
    int fail_stage = -1;

    auto dma = [&](int k, int slot) {
#pragma unroll
        for (int q = 0; q < NI; ++q) {
            int ch = q * 64 + lane;
            ch = ch < SH::CH ? ch : SH::CH - 1;  // surplus lanes re-load the last chunk
            const int d = 2 * ch;
            const double *src = d < SH::OC   ? Eb + (long long)k * SH::n * SH::s + d
                                : d < SH::OH ? cb + (long long)k * SH::n + (d - SH::OC)
                                : d < SH::OP ? hb + (long long)k * SH::s + (d - SH::OH)
                                             : Hb + (long long)k * SH::ps + (d - SH::OP);
            dma16(src, &stg[slot][q * 128]);
        }
    };

    // ---- terminal (lqr_kernel.hpp:80-91): P_N = H~_N, p_N = h~_N ----
    d4 Pm;
    double prow[4];
    {
        d4 Mt[1][1];
        load_M<1>(Mt, Hb + (long long)N * ps, n, m, m, s, g, c);
        Pm = Mt[0][0];
        bool bad = false;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 4 * r + g;
            const bool xr = i >= m && i < s;
            prow[r] = xr ? hb[(long long)N * s + (i - m)] : 0.0;
            if (i == c && xr && !(Pm[r] > 0.0)) bad = true;
        }
        if (__any(bad)) fail_stage = N;
    }

    if constexpr (CT) {
        // vm ops per iteration: NI DMA (stage k-1) + 1 record store, so after
        // issuing DMA(k-1) "DMA(k) has landed" is vmcnt(NI + 1); the first
        // iteration has no store behind DMA(N-1) yet.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // terminal loads
        dma(N - 1, (N - 1) & 1);
        for (int k = N - 1; k >= 0; --k) {
            if (k > 0) {
                dma(k - 1, (k - 1) & 1);
                if (k == N - 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");
                else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI + 1) : "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            const double *R = stg[k & 1];
            SchurIn in;
            schur_load(in, R + SH::OE, R + SH::OC, R + SH::OP, R + SH::OH, n, m, s, g, c);
            const bool ok = schur_stage(Pm, prow, in, sm, m, s, g, c);
            if (!ok && fail_stage < 0) fail_stage = k;
            schur_store_record_staged<SH::m, SH::s>(FRb + (long long)k * frs, Pm, sm, g, c);
            wave_sync();  // the record's LDS reads retire before the next DMA overwrites the slot
        }
    } else {
        SchurIn nxt;
        schur_load(nxt, Eb + (long long)(N - 1) * n * s, cb + (long long)(N - 1) * n, Hb + (long long)(N - 1) * ps,
                   hb + (long long)(N - 1) * s, n, m, s, g, c);
        for (int k = N - 1; k >= 0; --k) {
            const SchurIn in = nxt;
            if (k > 0)
                schur_load(nxt, Eb + (long long)(k - 1) * n * s, cb + (long long)(k - 1) * n,
                           Hb + (long long)(k - 1) * ps, hb + (long long)(k - 1) * s, n, m, s, g, c);
            const bool ok = schur_stage(Pm, prow, in, sm, m, s, g, c);
            if (!ok && fail_stage < 0) fail_stage = k;
            schur_store_record(FRb + (long long)k * frs, Pm, sm, m, s, g, c);
        }
    }
    if (lane == 0) A.status[b] = fail_stage < 0 ? 0 : fail_stage + 1;
}

static bool schur_aligned(const RiccatiArgs &a) {
    const Shape &sh = a.sh;
    auto al = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    return al(a.E) && al(a.c) && al(a.Hw) && al(a.hw) && sh.perE % 2 == 0 && sh.perc % 2 == 0 &&
           sh.perHw % 2 == 0 && sh.perh % 2 == 0;
}

// Returns PDPLQR_ERR_UNSUPPORTED when the shape / options need the full-factor kernels.
int launch_riccati_backward_schur(const RiccatiArgs &a, hipStream_t st) {
    const Shape &sh = a.sh;
    if (a.Lc || sh.s > 16 || getenv("PDPLQR_NO_SCHUR")) return PDPLQR_ERR_UNSUPPORTED;
    if (sh.n == 12 && sh.m == 4 && schur_aligned(a) && !getenv("PDPLQR_NO_DMA"))
        hipLaunchKernelGGL((k_riccati_bwd_schur<12, 4>), dim3(sh.batch), dim3(64), 0, st, a);
    else
        hipLaunchKernelGGL((k_riccati_bwd_schur<0, 0>), dim3(sh.batch), dim3(64), 0, st, a);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

}  // namespace pdplqr
