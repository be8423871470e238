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
#include "admm.hpp"
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

// The off-chain part of a stage, shared by both streamed kernels:
//     w = Lxx (Lxx^T c),  q = h~ + E^T w
// for the stage record R (E column-major at oe, c at oc) and the packed factor
// Lp (dimension dim, x block at offset off); h~ of lane column cl is ht, q
// returns on lane column cl (all groups).  st, sw: 16-double LDS scratch.
// ge: the bank-spread row slice of the E reads (see k_nofact_dma).
template <int NN>
__device__ __forceinline__ double nofact_q(const double *R, int oe, int oc, const double *Lp, int dim, int off,
                                           double ht, double *st, double *sw, int g, int ge, int cl) {
    constexpr int n = NN;
    const int j = cl < n ? cl : n - 1;
    double a = 0.0;
#pragma unroll
    for (int qq = 0; qq < (n + 3) / 4; ++qq) {  // t_j = sum_{i >= j} Lxx[i][j] c_i
        const int i = 4 * qq + g;
        const int ic = i < n ? i : n - 1;
        const double l = Lp[pidx(off + (ic >= j ? ic : j), off + j, dim)];
        a = __builtin_fma((i < n && i >= j) ? l : 0.0, R[oc + ic], a);
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
        const int i = 4 * qq + ge;
        const int ic = i < n ? i : n - 1;
        qv = __builtin_fma(i < n ? R[oe + ic + cl * n] : 0.0, sw[ic], qv);
    }
    return sum_groups(qv) + ht;
}

// Ring depth 3 (8.9 KB of LDS): 16 blocks per CU, so batch 4096 is one
// residency round; depth 4 (11.8 KB) fit 13 and left a second, mostly idle
// round: backward_without_factorization 2.83 -> 2.64 ms at the headline
// config (profiles/r03/nofact_depth_ab.log).
#ifndef PDPLQR_NOFACT_DEPTH
#define PDPLQR_NOFACT_DEPTH 3
#endif
// The fused ADMM pass (k_nofact_admm_dma, 15.6 KB at depth 4) runs C5's batch
// of 1024 at 4 blocks per CU, where LDS does not bound the residency: it keeps
// depth 4.
#ifndef PDPLQR_NOFACT_ADMM_DEPTH
#define PDPLQR_NOFACT_ADMM_DEPTH 4
#endif

template <int NN, int MM, int D, bool X1 = false>
__global__ __launch_bounds__(64) void k_nofact_dma(RiccatiArgs A) {
    simd_exclusive<X1>();
    using SH = NofactShape<NN, MM>;
    constexpr int n = SH::n, m = SH::m, s = SH::s, NI = SH::NI;
    static_assert(SH::ok, "nofact DMA layout");
    static_assert(D >= 3, "stage k - 1 must be resident while stage k is processed");
    __shared__ __attribute__((aligned(16))) double ring[D][SH::REC];
    __shared__ double sp[16], st[16], sw[16];
    const int lane = wave_lane(), g = lane >> 4, cl = lane & 15;
    // E[i][c] reads (column-major, stride n = 12): lane (g, c) takes rows i = 4 q + ge.
    // With ge = g the two row groups of a 32-lane half put columns c and c + 8 on
    // the same ds_read_b64 bank (12 * 8 = 0 mod 32); swapping the row slice of the
    // upper 8 columns spreads them over all 32 banks.  sum_groups still adds the
    // same four partials in the same order (its butterfly is symmetric): the
    // results are bit-identical.
    const int ge = g ^ ((cl >> 3) << 1);
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
    auto offchain = [&](const double *R, const double *Lp, int dim, int off) -> double {
        return nofact_q<NN>(R, SH::OE, SH::OC, Lp, dim, off, R[SH::OH + cl], st, sw, g, ge, cl);
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
            const int i = 4 * qq + ge;  // bank-spread row slice (see ge)
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

// ---------------------------------------------------------------------------
// ADMM iterations >= 2 (admm.hip): the z / y / w step of iteration it and the
// backward_without_factorization of iteration it + 1 in ONE streamed pass.
// The backward needs h~_k = h_k - sigma w_k^{it+1} - D_k^T (rho o g_k^{it+1}),
// and everything that forms it -- w~_k (the rollout's output), w_k, D_k, z_k,
// y_k, the bounds and rho of stage k -- is per stage.  So the stage record
// grows by those (120 doubles at 12/4 with nc = 4: 476 doubles, 4 DMA
// instructions) and the update of stage k - 1 runs while stage k is
// processed, off the p-chain, right before its h~ enters q_{k-1}.  Lanes
// (g, c): row g of D_k (nc = 4 rows), column c (s = 16); D w~ is a butterfly
// over c, D^T (rho o g) a permlane sum over g.  The stand-alone update pass
// (k_admm_update) and its w~ / w / h~ round trip through HBM disappear.
// Requirements: nc_k = NC for k < N, nc_N = 0 (else admm.hip runs the
// unfused path).  CHECK: the termination test of iteration it over the whole
// problem (one wave = one problem: a wave-wide max, then admm_decide).
// ---------------------------------------------------------------------------
template <int NN, int MM, int NC>
struct NofactAdmmShape {
    static constexpr int n = NN, m = MM, s = NN + MM, ps = s * (s + 1) / 2;
    static constexpr int OE = 0, OC = n * s, OH = OC + n, OL = OH + s, OWT = OL + ps, OW = OWT + s, OD = OW + s,
                         OZ = OD + NC * s, OY = OZ + NC, OLB = OY + NC, OUB = OLB + NC, ORHO = OUB + NC,
                         OIR = ORHO + NC, REC = OIR + NC;
    static constexpr int CH = REC / 2, NI = (CH + 63) / 64, TAIL = CH - (NI - 1) * 64;
    static constexpr bool ok = s == 16 && NC == 4 && n % 2 == 0 && (n * s) % 2 == 0 && ps % 2 == 0;
};

template <int NN, int MM, int NC, int D, bool CHECK, bool X1 = false>
__global__ __launch_bounds__(64) void k_nofact_admm_dma(RiccatiArgs A, AdmmArgs Q) {
    simd_exclusive<X1>();
    using SH = NofactAdmmShape<NN, MM, NC>;
    constexpr int n = SH::n, m = SH::m, s = SH::s, NI = SH::NI;
    static_assert(SH::ok, "fused nofact / ADMM layout");
    __shared__ __attribute__((aligned(16))) double ring[D][SH::REC];
    __shared__ double sp[16], st[16], sw[16];
    const int lane = wave_lane(), g = lane >> 4, cl = lane & 15;
    // E[i][c] reads (column-major, stride n = 12): lane (g, c) takes rows i = 4 q + ge.
    // With ge = g the two row groups of a 32-lane half put columns c and c + 8 on
    // the same ds_read_b64 bank (12 * 8 = 0 mod 32); swapping the row slice of the
    // upper 8 columns spreads them over all 32 banks.  sum_groups still adds the
    // same four partials in the same order (its butterfly is symmetric): the
    // results are bit-identical.
    const int ge = g ^ ((cl >> 3) << 1);
    const Shape &sh = A.sh;
    const long long b = blockIdx.x;
    if (Q.done[b]) return;  // frozen problem: no update, no backward (wave-uniform)
    const int N = sh.N;
    const double al = Q.alpha, bl = 1.0 - Q.alpha;
    const double *hb = Q.hv + b * sh.perh;  // the MODEL's h
    const double *Lb = A.Lc + b * sh.perHw;
    double *FRb = A.KD + b * sh.perKD;
    double *lpb = A.lpc + b * sh.perh;
    double *wb = Q.w + b * sh.perh, *hwb = Q.hw + b * sh.perh;
    double *zb = Q.z + b * sh.ny, *yb = Q.y + b * sh.ny, *gb = Q.gw + b * sh.ny;
    constexpr int frs = s * m + m;
    // per-lane source of each DMA chunk: base at stage 0 + stage stride
    const double *gbase[NI];
    int gstride[NI];
#pragma unroll
    for (int q = 0; q < NI; ++q) {
        int ch = q * 64 + lane;
        ch = ch < SH::CH ? ch : SH::CH - 1;
        const int d = 2 * ch;
        const long long pb = b * sh.perh, yb0 = b * sh.ny;
        if (d < SH::OC) { gbase[q] = A.E + b * sh.perE + d; gstride[q] = n * s; }
        else if (d < SH::OH) { gbase[q] = A.c + b * sh.perc + (d - SH::OC); gstride[q] = n; }
        else if (d < SH::OL) { gbase[q] = Q.hv + pb + (d - SH::OH); gstride[q] = s; }
        else if (d < SH::OWT) { gbase[q] = Lb + (d - SH::OL); gstride[q] = SH::ps; }
        else if (d < SH::OW) { gbase[q] = Q.wt + pb + (d - SH::OWT); gstride[q] = s; }
        else if (d < SH::OD) { gbase[q] = Q.w + pb + (d - SH::OW); gstride[q] = s; }
        else if (d < SH::OZ) { gbase[q] = Q.D + b * sh.ndD + (d - SH::OD); gstride[q] = NC * s; }
        else if (d < SH::OY) { gbase[q] = Q.z + yb0 + (d - SH::OZ); gstride[q] = NC; }
        else if (d < SH::OLB) { gbase[q] = Q.y + yb0 + (d - SH::OY); gstride[q] = NC; }
        else if (d < SH::OUB) { gbase[q] = Q.lb + yb0 + (d - SH::OLB); gstride[q] = NC; }
        else if (d < SH::ORHO) { gbase[q] = Q.ub + yb0 + (d - SH::OUB); gstride[q] = NC; }
        else if (d < SH::OIR) { gbase[q] = Q.rho + yb0 + (d - SH::ORHO); gstride[q] = NC; }
        else { gbase[q] = Q.irho + yb0 + (d - SH::OIR); gstride[q] = NC; }
    }
    auto dma = [&](int k, int slot) {
#pragma unroll
        for (int q = 0; q < NI; ++q)
            if (q < NI - 1 || lane < SH::TAIL) dma16(gbase[q] + (long long)k * gstride[q], &ring[slot][q * 128]);
    };
    double rp = 0.0, dwm = 0.0, zm = 0.0, rd = 0.0, dty = 0.0, act = 0.0;
    // The ADMM step of stage kk from its ring record; returns h~_kk[cl].
    // Exactly 5 stores (z, y, g: lanes c == 0; w, h~: row group 0).
    auto upd = [&](const double *R, int kk) -> double {
        const double wt = R[SH::OWT + cl], wo = R[SH::OW + cl];
        const double wn = al * wt + bl * wo;
        const double d = R[SH::OD + g + cl * NC];  // D_kk[g][cl]
        const double v = sum_row16(d * wt), vw = sum_row16(d * wo);
        const double zr = R[SH::OZ + g], yr = R[SH::OY + g], rr = R[SH::ORHO + g], ir = R[SH::OIR + g];
        const double vrel = al * v + bl * zr;
        const double zn = fmin(fmax(vrel + ir * yr, R[SH::OLB + g]), R[SH::OUB + g]);
        const double yn = yr + rr * (vrel - zn);
        const double gn = zn - ir * yn;
        const long long yo = (long long)kk * NC + g;
        if (cl == 0) gstore(zb + yo, zn);
        if (cl == 0) gstore(yb + yo, yn);
        if (cl == 0) gstore(gb + yo, gn);
        const double ag = sum_groups(d * (rr * gn));  // (D^T (rho o g))[cl]
        const double hj = (R[SH::OH + cl] - Q.sigma * wn) - ag;
        if (g == 0) gstore(wb + (long long)kk * s + cl, wn);
        if (g == 0) gstore(hwb + (long long)kk * s + cl, hj);
        if (CHECK) {
            const double dwn = al * v + bl * vw;
            rp = fmax(rp, fabs(dwn - zn));
            dwm = fmax(dwm, fabs(dwn));
            zm = fmax(zm, fabs(zn));
            if (zn <= R[SH::OLB + g] || zn >= R[SH::OUB + g]) act = 1.0;
            rd = fmax(rd, fabs(sum_groups(d * (rr * (zn - zr)))));
            dty = fmax(dty, fabs(sum_groups(d * yn)));
        }
        return hj;
    };
    // P c and q = h~ + E^T (P c) for record R with factor Lp (as k_nofact_dma)
    auto offchain = [&](const double *R, const double *Lp, int dim, int off, double ht) -> double {
        return nofact_q<NN>(R, SH::OE, SH::OC, Lp, dim, off, ht, st, sw, g, ge, cl);
    };

    // ---- terminal (nc_N = 0): w_N relaxed, h~_N = h_N - sigma w_N; lp_N = h~_N ----
    if (lane < n) {
        const long long o = (long long)N * s + lane;
        const double wn = al * Q.wt[b * sh.perh + o] + bl * wb[o];
        const double hN = hb[o] - Q.sigma * wn;
        wb[o] = wn;
        hwb[o] = hN;
        sp[lane] = hN;
        lpb[o] = hN;
    }
#pragma unroll
    for (int j = 0; j < D - 1; ++j) {
        const int k = N - 1 - j;
        dma(k >= 0 ? k : 0, ((k % D) + D) % D);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
    double q;
    {
        const double *R = ring[(N - 1) % D];
        const double ht = upd(R, N - 1);
        q = offchain(R, Lb + (long long)N * SH::ps, n, 0, ht);  // q_{N-1} with Lxx_N
    }
    constexpr int VM = NI + 7;  // vm ops per iteration: NI DMA + 2 backward stores + 5 update stores
    for (int k = N - 1; k >= 0; --k) {
        const int kp = k - (D - 1);
        dma(kp >= 0 ? kp : 0, ((kp % D) + D) % D);
        if (k >= N - (D - 2)) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM * (D - 2)) : "memory");
        wave_sync();
        const double *R = ring[k % D];
        const double *Lk = R + SH::OL;
        const int cm = cl < m ? cl : m - 1;
        const double rdiag = 1.0 / Lk[pidx(cm, cm, s)];
        double lcol[MM];
#pragma unroll
        for (int j = 0; j < MM; ++j) lcol[j] = (cl > j) ? Lk[pidx(cl > j ? cl : j, j, s)] : 0.0;
        double a = 0.0;
#pragma unroll
        for (int qq = 0; qq < (n + 3) / 4; ++qq) {
            const int i = 4 * qq + ge;  // bank-spread row slice (see ge)
            const int ic = i < n ? i : n - 1;
            a = __builtin_fma(i < n ? R[SH::OE + ic + cl * n] : 0.0, sp[ic], a);
        }
        const double lp = sum_groups(a) + q;
        double acc = 0.0, myu = 0.0;
#pragma unroll
        for (int j = 0; j < MM; ++j) {
            const double uj = readlane_f64((lp - acc) * rdiag, j);
            if (cl == j) myu = uj;
            acc = __builtin_fma(lcol[j], uj, acc);
        }
        const double pk = lp - acc;
        wave_sync();
        if (g == 0 && cl >= m) sp[cl - m] = pk;
        if (lane < m) gstore(FRb + (long long)k * frs + s * m + lane, myu);
        if (lane < s) gstore(lpb + (long long)k * s + lane, lane < m ? myu : pk);
        if (k > 0) {
            const double *Rn = ring[(k - 1) % D];
            const double ht = upd(Rn, k - 1);
            q = offchain(Rn, Lk, s, m, ht);
        }
        wave_sync();
    }
    if (CHECK) {
#pragma unroll
        for (int msk = 32; msk >= 1; msk >>= 1) {
            rp = fmax(rp, __shfl_xor(rp, msk, 64));
            dwm = fmax(dwm, __shfl_xor(dwm, msk, 64));
            zm = fmax(zm, __shfl_xor(zm, msk, 64));
            rd = fmax(rd, __shfl_xor(rd, msk, 64));
            dty = fmax(dty, __shfl_xor(dty, msk, 64));
                act = fmax(act, __shfl_xor(act, msk, 64));
        }
        if (lane == 0) admm_decide(Q, (int)b, rp, dwm, zm, rd, dty, act);
    }
}

int launch_nofact_admm(const RiccatiArgs &a, const AdmmArgs &q, bool check, hipStream_t st) {
    const Shape &sh = a.sh;
    if (getenv("PDPLQR_NO_ADMM_FUSE") || !a.Lc || !a.lpc || sh.n != 12 || sh.m != 4 || sh.ny != 4 * sh.N)
        return PDPLQR_ERR_UNSUPPORTED;
    auto al = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    if (!al(a.E) || !al(a.c) || !al(a.Lc) || !al(q.hv) || !al(q.wt) || !al(q.w) || !al(q.D) || !al(q.z) ||
        !al(q.y) || !al(q.lb) || !al(q.ub) || !al(q.rho) || !al(q.irho) || sh.perE % 2 || sh.perc % 2 ||
        sh.perh % 2 || sh.perHw % 2 || sh.ndD % 2 || sh.ny % 2)
        return PDPLQR_ERR_UNSUPPORTED;
    with_x1(sh.x1, [&](auto x1) {
        constexpr bool X = decltype(x1)::value;
        if (check)
            hipLaunchKernelGGL((k_nofact_admm_dma<12, 4, 4, PDPLQR_NOFACT_ADMM_DEPTH, true, X>), dim3(sh.batch),
                               dim3(64), 0, st, a, q);
        else
            hipLaunchKernelGGL((k_nofact_admm_dma<12, 4, 4, PDPLQR_NOFACT_ADMM_DEPTH, false, X>), dim3(sh.batch),
                               dim3(64), 0, st, a, q);
    });
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
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
    if (!a.Lc || !a.lpc || !nofact_aligned(a)) return PDPLQR_ERR_UNSUPPORTED;
    if (sh.n == 12 && sh.m == 4)
        with_x1(sh.x1, [&](auto x1) {
            hipLaunchKernelGGL((k_nofact_dma<12, 4, PDPLQR_NOFACT_DEPTH, decltype(x1)::value>), dim3(sh.batch),
                               dim3(64), 0, st, a);
        });
    else
        return PDPLQR_ERR_UNSUPPORTED;
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

}  // namespace pdplqr
