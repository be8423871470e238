// kernels_nofact.hip -- backward_without_factorization for compile-time shapes
// (LQRKernel::step_without_factorization, lqr_kernel.hpp:150-178; the terminal
// step :94-101), streamed like the rollout (kernels_rollout.hip).
//
// With the factors L_k cached (keep_factors = 1), a stage only moves vectors:
//     Pb   = Lxx_{k+1} (Lxx_{k+1}^T c_k) + p_{k+1}      (:171-173)
//     lp   = h~_k + E_k^T Pb                           (:175-176)
//     lu' = Luu_k^{-1} lu ;  p_k = lp_x - Lxu_k lu'    (:177-178)
// The only serial dependence is p_{k+1} -> p_k.  Everything that does not
// touch p is taken off the chain one stage ahead:
//     w_k = Lxx_{k+1} (Lxx_{k+1}^T c_k),   q_k = h~_k + E_k^T w_k
// (formed while stage k+1 is processed), leaving the chain
//     lp = q_k + E_k^T p_{k+1}  (one permlane-reduced dot per lane column),
//     four readlane steps of the forward substitution (lanes c >= m collect
//     Lxu lu' on the way), p_k = lp_x - Lxu lu'.
// One wavefront per problem keeps the stage records [E_k | c_k | h~_k | packed
// L_k] (356 doubles at 12/4) in a D-deep LDS-DMA ring; every iteration issues
// exactly NI DMA instructions and 2 stores, so "stage k - 1 has landed" is one
// fixed vmcnt.  Output: lu' into the rollout record FR_k (its L part is
// unchanged) and lp_k = [lu'; p_k] into the factor cache, as the generic kernel.
#include "device_common.hpp"

#include <stdint.h>
#include <stdlib.h>

namespace pdplqr {

template <int NN, int MM>
struct NofactShape {
    static constexpr int n = NN, m = MM, s = NN + MM, ps = s * (s + 1) / 2;
    static constexpr int OE = 0, OC = n * s, OH = OC + n, OL = OH + s, REC = OL + ps;  // doubles per stage
    static constexpr int CH = REC / 2, NI = (CH + 63) / 64, TAIL = CH - (NI - 1) * 64;
    static constexpr bool ok = (n * s) % 2 == 0 && n % 2 == 0 && s % 2 == 0 && ps % 2 == 0 && s <= 16 &&
                               n <= 12 && m <= 4;
};

#ifndef PDPLQR_NOFACT_DEPTH
#define PDPLQR_NOFACT_DEPTH 4
#endif

template <int NN, int MM, int D>
__global__ __launch_bounds__(64) void k_nofact_dma(RiccatiArgs A) {
    using SH = NofactShape<NN, MM>;
    constexpr int n = SH::n, m = SH::m, s = SH::s, NI = SH::NI;
    static_assert(SH::ok, "nofact DMA layout");
    static_assert(D >= 3, "stage k - 1 must be resident while stage k is processed");
    __shared__ __attribute__((aligned(16))) double ring[D][SH::REC];
    __shared__ double sp[16], st[16], sw[16];
    const int lane = wave_lane(), g = lane >> 4, cl = lane & 15;
    const Shape &sh = A.sh;
    const long long b = blockIdx.x;
    const int N = sh.N;
    const double *Eb = A.E + b * sh.perE;
    const double *cb = A.c + b * sh.perc;
    const double *hb = A.hw + b * sh.perh;
    const double *Lb = A.Lc + b * sh.perHw;
    double *FRb = A.KD + b * sh.perKD;
    double *lpb = A.lpc + b * sh.perh;
    constexpr int frs = s * m + m;

    auto dma = [&](int k, int slot) {
#pragma unroll
        for (int q = 0; q < NI; ++q) {
            if (q < NI - 1 || lane < SH::TAIL) {
                const int d = 2 * (q * 64 + lane);
                const double *src = d < SH::OC   ? Eb + (long long)k * (n * s) + d
                                    : d < SH::OH ? cb + (long long)k * n + (d - SH::OC)
                                    : d < SH::OL ? hb + (long long)k * s + (d - SH::OH)
                                                 : Lb + (long long)k * SH::ps + (d - SH::OL);
                dma16(src, &ring[slot][q * 128]);
            }
        }
    };
    // w = Lxx (Lxx^T c) and q = h + E^T w for the stage record R (E, c, h) and
    // the packed factor Lp (dimension dim, x block at offset off); q on lane
    // column cl (all groups)
    auto offchain = [&](const double *R, const double *Lp, int dim, int off) -> double {
        const int j = cl < n ? cl : n - 1;
        double a = 0.0;
#pragma unroll
        for (int qq = 0; qq < (n + 3) / 4; ++qq) {  // t_j = sum_{i >= j} Lxx[i][j] c_i
            const int i = 4 * qq + g;
            const int ic = i < n ? i : n - 1;
            const double l = Lp[pidx(off + (ic >= j ? ic : j), off + j, dim)];
            a = __builtin_fma((i < n && i >= j) ? l : 0.0, R[SH::OC + ic], a);
        }
        a = sum_groups(a);
        if (g == 0 && cl < n) st[cl] = a;
        wave_sync();
        double w = 0.0;  // w_i = sum_{j <= i} Lxx[i][j] t_j   (i = cl)
#pragma unroll
        for (int qq = 0; qq < (n + 3) / 4; ++qq) {
            const int jj = 4 * qq + g;
            const int jc = jj < n ? jj : n - 1;
            const double l = Lp[pidx(off + (j >= jc ? j : jc), off + jc, dim)];
            w = __builtin_fma((jj < n && jj <= j) ? l : 0.0, st[jc], w);
        }
        w = sum_groups(w);
        if (g == 0 && cl < n) sw[cl] = w;
        wave_sync();
        double qv = 0.0;  // q_c = h_c + sum_i E[i][c] w_i   (c = cl)
#pragma unroll
        for (int qq = 0; qq < (n + 3) / 4; ++qq) {
            const int i = 4 * qq + g;
            const int ic = i < n ? i : n - 1;
            qv = __builtin_fma(i < n ? R[SH::OE + ic + cl * n] : 0.0, sw[ic], qv);
        }
        return sum_groups(qv) + R[SH::OH + cl];
    };

    // ---- terminal (lqr_kernel.hpp:94-101): lp_N = h~_N ----
    if (lane < n) {
        const double v = hb[(long long)N * s + lane];
        sp[lane] = v;
        lpb[(long long)N * s + lane] = v;
    }
#pragma unroll
    for (int j = 0; j < D - 1; ++j) {
        const int k = N - 1 - j;
        dma(k >= 0 ? k : 0, ((k % D) + D) % D);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
    double q = offchain(ring[(N - 1) % D], Lb + (long long)N * SH::ps, n, 0);  // q_{N-1} with Lxx_N

    for (int k = N - 1; k >= 0; --k) {
        const int kp = k - (D - 1);
        dma(kp >= 0 ? kp : 0, ((kp % D) + D) % D);  // slot of stage k + 1 (consumed)
        // stage k - 1 (issued D - 2 iterations ago) has landed once at most
        // 5 (D - 2) younger vm ops (NI = 3 DMA + 2 stores per iteration) remain
        if (k >= N - (D - 2)) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NI + 2) * (D - 2)) : "memory");
        wave_sync();
        const double *R = ring[k % D];
        const double *Lk = R + SH::OL;
        // off-chain reads of this stage's factor
        const int cm = cl < m ? cl : m - 1;
        const double rdiag = 1.0 / Lk[pidx(cm, cm, s)];
        double lcol[MM];
#pragma unroll
        for (int j = 0; j < MM; ++j) lcol[j] = (cl > j) ? Lk[pidx(cl > j ? cl : j, j, s)] : 0.0;  // L[cl][j], cl > j
        // ---- chain: lp = q + E^T p_{k+1} ----
        double a = 0.0;
#pragma unroll
        for (int qq = 0; qq < (n + 3) / 4; ++qq) {
            const int i = 4 * qq + g;
            const int ic = i < n ? i : n - 1;
            a = __builtin_fma(i < n ? R[SH::OE + ic + cl * n] : 0.0, sp[ic], a);
        }
        const double lp = sum_groups(a) + q;
        // lu' = Luu^{-1} lu (forward substitution, lanes cl < m); lanes cl >= m
        // accumulate (Lxu lu')[cl - m]
        double acc = 0.0, myu = 0.0;
#pragma unroll
        for (int j = 0; j < MM; ++j) {
            const double uj = readlane_f64((lp - acc) * rdiag, j);  // valid on lane cl == j
            if (cl == j) myu = uj;
            acc = __builtin_fma(lcol[j], uj, acc);
        }
        const double pk = lp - acc;  // lanes cl >= m: p_k[cl - m]
        wave_sync();                 // every read of sp (p_{k+1}) precedes its overwrite
        if (g == 0 && cl >= m) sp[cl - m] = pk;
        // exactly two stores per iteration (vmcnt accounting above)
        if (lane < m) gstore(FRb + (long long)k * frs + s * m + lane, myu);
        if (lane < s) gstore(lpb + (long long)k * s + lane, lane < m ? myu : pk);
        // ---- off the chain: q_{k-1} from L_k and stage k - 1's record ----
        if (k > 0) q = offchain(ring[(k - 1) % D], Lk, s, m);
        wave_sync();
    }
}

static bool nofact_aligned(const RiccatiArgs &a) {
    const Shape &sh = a.sh;
    auto al = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    return al(a.E) && al(a.c) && al(a.hw) && al(a.Lc) && al(a.KD) && sh.perE % 2 == 0 && sh.perc % 2 == 0 &&
           sh.perh % 2 == 0 && sh.perHw % 2 == 0;
}

// PDPLQR_ERR_UNSUPPORTED: shape / alignment not covered (the generic kernel runs)
int launch_nofact_dma(const RiccatiArgs &a, hipStream_t st) {
    const Shape &sh = a.sh;
    if (!a.Lc || !a.lpc || getenv("PDPLQR_NO_DMA") || !nofact_aligned(a)) return PDPLQR_ERR_UNSUPPORTED;
    if (sh.n == 12 && sh.m == 4)
        hipLaunchKernelGGL((k_nofact_dma<12, 4, PDPLQR_NOFACT_DEPTH>), dim3(sh.batch), dim3(64), 0, st, a);
    else
        return PDPLQR_ERR_UNSUPPORTED;
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

}  // namespace pdplqr
