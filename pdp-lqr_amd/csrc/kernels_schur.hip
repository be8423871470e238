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
#include "schur_stage.hpp"

#include <stdint.h>
#include <stdlib.h>

namespace pdplqr {


// Stage-record layout of the LDS-DMA variant (compile-time shapes).
// HBM record = E (n x s, column-major), c, h~, packed H~ (offsets OE..OP).
// The LDS copy stores E's columns at stride LDE: the read of E~ row
// 4 kk + g - m, column c by a 32-lane half is LDE c + g (+ const); LDE = n = 12
// puts c and c + 8 on one bank (2-way on all four reads), LDE = 2 x odd = 14
// hits 32 distinct banks.  A 16-byte chunk (2 rows of one column, n even)
// moves as a unit, so the copy stays one ds_write_b128 per chunk with a fixed
// per-lane destination (LO* = LDS offsets).
// NC > 0 (fused rho penalty): D (NC x s), rho (NC), g (NC) follow H~.
template <int NN, int MM, int NC = 0>
struct SchurShape {
    static constexpr int n = NN, m = MM, s = NN + MM;
    static constexpr int ps = s * (s + 1) / 2;
    static constexpr int OE = 0, OC = n * s, OH = OC + n, OP = OH + s, OD = OP + ps, OR = OD + NC * s, OG = OR + NC,
                         Q = OG + NC;
    static constexpr int CH = Q / 2, NI = (CH + 63) / 64;
    static constexpr int LDE = n;
    static constexpr int LSH = (LDE - n) * s;  // shift of everything after E in the LDS copy
    static constexpr int LOC = OC + LSH, LOH = OH + LSH, LOP = OP + LSH, LOD = OD + LSH, LOR = OR + LSH,
                         LOG = OG + LSH;
    static constexpr int SLOT = NI * 128 + LSH;  // every lane's chunk of the last load lands inside
    static constexpr bool ok = (n * s) % 2 == 0 && n % 2 == 0 && s % 2 == 0 && ps % 2 == 0 && s <= 16 && NC % 2 == 0;
};

// Symmetrise P every PDPLQR_SYM_EVERY stages (1, 2 or 4) on the compile-time
// shape path; the runtime-shape path symmetrises every stage.
#ifndef PDPLQR_SYM_EVERY
#define PDPLQR_SYM_EVERY 4
#endif
using SymOn = std::integral_constant<bool, true>;
using SymOff = std::integral_constant<bool, false>;


#ifndef PDPLQR_SCHUR_WAVES
#define PDPLQR_SCHUR_WAVES 4
#endif
// waves per SIMD of the fused-penalty instance (NC > 0): its fourth staging
// chunk and the write-back addresses do not fit 128 VGPRs (at 4 waves the
// compiler spilled inside the stage loop, and every scratch reload drains the
// staging loads); C5 runs one wave per SIMD (batch 1024) anyway
#ifndef PDPLQR_PEN_WAVES
#define PDPLQR_PEN_WAVES 2
#endif
// the fused-penalty instance has the registers (2 waves per SIMD) for G and M
// on three independent MFMA accumulators each (schur_stage SPLIT = 1); C5 runs
// it at one wave per SIMD, where the stage chain is what bounds it

// NN = MM = 0: runtime shape, register prefetch of the next stage.
// NN, MM > 0 : compile-time shape, stage records streamed by LDS-DMA
//              (global_load_lds_dwordx4) into a double buffer.
// NC > 0: the rho penalty of every stage (lqr_kernel.hpp:82-88,106-112) fused
// into the stream: the stage record carries D_k (NC rows), rho_k, g_k; the
// penalised H~_k + D^T rho D and h~_k - D^T rho g feed the stage and are written
// back in place (the reference's data.H += / data.h -= semantics, so a second
// backward without update_problem_data penalises again, as there).
template <int NN, int MM, bool GAIN = false, int NC = 0, bool X1 = false>
__global__ __launch_bounds__(64, (X1 ? 1 : NN > 0 ? (NC > 0 ? PDPLQR_PEN_WAVES : PDPLQR_SCHUR_WAVES) : 3)) void k_riccati_bwd_schur(
    RiccatiArgs A) {
    PDPLQR_PROBE_BEGIN
    simd_exclusive<X1>();
    static_assert(!GAIN || (NN == 12 && MM == 4), "gain-form record: 12/4 block path");
    static_assert(NN == 0 || GAIN, "the compile-time shape writes the gain-form record");
    static_assert(NC == 0 || (GAIN && NC == 4), "fused penalty: 12/4 gain-form path, 4 rows per stage");
    constexpr bool CT = NN > 0;
    using SH = SchurShape<(CT ? NN : 2), (CT ? MM : 2), NC>;
    constexpr int NI = CT ? SH::NI : 1;
    __shared__ SchurSmem sm;
    __shared__ __attribute__((aligned(16))) double stg[CT ? 2 : 1][CT ? SH::SLOT : 2];
    const int lane = wave_lane(), g = lane >> 4, c = lane & 15;
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
    const int frs = GAIN ? n * m + m : s * m + m;  // doubles per stage of the record
    int fail_stage = -1;
    const double *Db = NC > 0 ? A.D + b * (long long)sh.ndD : nullptr;
    const double *rb = NC > 0 ? A.rho + b * (long long)sh.ny : nullptr;
    const double *gb = NC > 0 ? A.gw + b * (long long)sh.ny : nullptr;

    // ---- terminal (lqr_kernel.hpp:80-91): P_N = H~_N, p_N = h~_N ----
    d4 Pm;
    double prow[4];
    {
        d4 Mt[1][1];
        load_M<1>(Mt, Hb + (long long)N * ps, n, m, m, s, g, c);
        Pm = Mt[0][0];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 4 * r + g;
            prow[r] = (i >= m && i < s) ? hb[(long long)N * s + (i - m)] : 0.0;
        }
        if constexpr (NC > 0) {
            const int ncN = A.nc_last;
            if (ncN > 0) {  // rare: plain loops (D_N is ncN x n), written back in place as the stages
                const double *DN = Db + A.d_off[N], *rN = rb + A.y_off[N], *gN = gb + A.y_off[N];
                for (int q = 0; q < ncN; ++q) {
                    const double rq = rN[q], gq = gN[q];
                    const double dc = c >= m ? DN[q + (c - m) * ncN] : 0.0;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int i = 4 * r + g;
                        const double di = i >= m ? DN[q + (i - m) * ncN] : 0.0;
                        Pm[r] = __builtin_fma(di, rq * dc, Pm[r]);
                        prow[r] = __builtin_fma(-di, rq * gq, prow[r]);
                    }
                }
                double *HN = A.Hw + b * sh.perHw + (long long)N * ps;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 4 * r + g;
                    if (i >= m && c >= m && i >= c) HN[pidx(i - m, c - m, n)] = Pm[r];
                    if (c == 0 && i >= m) A.hw[b * sh.perh + (long long)N * s + (i - m)] = prow[r];
                }
            }
        }
        bool bad = false;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 4 * r + g;
            if (i == c && i >= m && i < s && psd_bad(Pm[r])) bad = true;  // P_N = H~_N semidefinite is valid
        }
        if (__any(bad)) fail_stage = N;
    }

    if constexpr (CT) {
        // Stage records go HBM -> registers -> LDS: register sets RA / RB hold
        // the records of the next two stages in flight (2 x NI x 16 B per lane),
        // so each load has two stage steps to land; stage k - 1 is written to
        // its LDS slot right after stage k is processed.  (The former one-ahead
        // LDS-DMA ring had one step, ~3.5 us, which left the HBM latency
        // exposed at 4 waves per SIMD.)
        d2v RA[NI], RB[NI];
        // per-lane stage-0 address and stage stride of each 16-byte chunk,
        // fixed for the whole horizon: the loop only forms base + k stride
        // (selecting the source array per stage made divergent branches)
        const double *gbase[NI];
        int gstride[NI];
#pragma unroll
        for (int q = 0; q < NI; ++q) {
            int ch = q * 64 + lane;
            ch = ch < SH::CH ? ch : SH::CH - 1;
            const int d = 2 * ch;
            gbase[q] = d < SH::OC   ? Eb + d
                       : d < SH::OH ? cb + (d - SH::OC)
                       : d < SH::OP ? hb + (d - SH::OH)
                       : d < SH::OD ? Hb + (d - SH::OP)
                       : d < SH::OR ? Db + (d - SH::OD)
                       : d < SH::OG ? rb + (d - SH::OR)
                                    : gb + (d - SH::OG);
            gstride[q] = d < SH::OC   ? SH::n * SH::s
                         : d < SH::OH ? SH::n
                         : d < SH::OP ? SH::s
                         : d < SH::OD ? SH::ps
                         : d < SH::OR ? NC * SH::s
                                      : NC;
        }
        auto gload = [&](d2v(&R)[NI], int k) {
#pragma unroll
            for (int q = 0; q < NI; ++q) {
                const double *src = gbase[q] + (long long)k * gstride[q];
                // issued through asm: the compiler's waitcnt pass would otherwise
                // wait for every outstanding load at the first use (its loop
                // model merges the guarded loads); the waits are explicit below
                asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(R[q]) : "v"(src) : "memory");
            }
        };
        // R's loads have landed once at most `after` younger vm ops are
        // outstanding.  One immediate per call site: a branchy wait made the
        // compiler copy R (still in flight) into other registers.
        // store instructions per stage (all unconditional): the record (1),
        // plus with NC > 0 the in-place write-back of h~ (1) and of the packed H~ (4)
        constexpr int ST = 1 + (NC > 0 ? 5 : 0);
        static_assert(NI == 3 || NI == 4, "register staging");
        auto vwait5 = [&](d2v(&R)[NI]) {  // steady state
            if constexpr (NI == 3)
                asm volatile("s_waitcnt vmcnt(%3)" : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]) : "n"(NI + 2 * ST) : "memory");
            else
                asm volatile("s_waitcnt vmcnt(%4)" : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]), "+v"(R[3]) : "n"(NI + 2 * ST)
                             : "memory");
        };
        auto vwait4 = [&](d2v(&R)[NI]) {  // first step
            if constexpr (NI == 3)
                asm volatile("s_waitcnt vmcnt(%3)" : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]) : "n"(NI + ST) : "memory");
            else
                asm volatile("s_waitcnt vmcnt(%4)" : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]), "+v"(R[3]) : "n"(NI + ST)
                             : "memory");
        };
        auto vwait0 = [&](d2v(&R)[NI]) {
            if constexpr (NI == 3) asm volatile("s_waitcnt vmcnt(0)" : "+v"(R[0]), "+v"(R[1]), "+v"(R[2])::"memory");
            else asm volatile("s_waitcnt vmcnt(0)" : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]), "+v"(R[3])::"memory");
        };
        auto lput = [&](const d2v(&R)[NI], int slot) {
#pragma unroll
            for (int q = 0; q < NI; ++q) {
                // chunk ch (doubles 2 ch, 2 ch + 1) of the HBM record to its LDS
                // place: E's column ch / (n/2) moves by (LDE - n) per column,
                // everything after E by LSH (recomputed per stage from the lane
                // id: held across the loop it spilled)
                // (lanes past the record's last chunk write copies of it
                // past the record's end, inside the slot)
                const int ch = q * 64 + lane;
                constexpr int EC = SH::OC / 2;  // chunks of E
                const int dst = (q * 64 >= EC)       ? 2 * ch + SH::LSH
                                : (q * 64 + 63 < EC) ? 2 * ch + (SH::LDE - SH::n) * (ch / (SH::n / 2))
                                                     : 2 * ch + (SH::LDE - SH::n) * min(ch / (SH::n / 2), SH::s);
                __builtin_assume((dst & 1) == 0);  // 16-byte chunks: keeps one ds_write_b128
                *reinterpret_cast<d2v *>(&stg[slot][dst]) = R[q];
            }
        };
        // Every step issues exactly 3 loads (stage k - 3, clamped to stage 0 at
        // the end: re-loads that are never written to LDS) and 1 record store
        // (2 with PDPLQR_REC_DIRECT), so "X's loads have landed" is always
        // vmcnt(5) (7) -- the other set's 3 loads and two steps' stores are
        // younger; the first step follows the prologue (3 loads + one step's
        // stores: vmcnt(4) (5)).
        // Stage k: its record is read from LDS slot k & 1, its rollout record
        // stored (1 or 2 vm ops).
        auto process = [&](int k, auto sym, bool sym_rt) {
            const double *R = stg[k & 1];
            SchurIn in;
            schur_load(in, R + SH::OE, R + SH::LOC, R + SH::LOP, R + SH::LOH, n, m, s, g, c, SH::LDE);
            if constexpr (NC > 0) {
                // H~ += D^T diag(rho) D as (a^T)(sgn a) with a = sqrt|rho| D (lane (g, c): row g,
                // column c): entry (i, j) and (j, i) multiply the same two factors in the same
                // order, so the penalised tile stays bitwise symmetric and the duplicate
                // write-back stores below (each entry from both of its lanes) carry equal bits
                const double dgc = R[SH::LOD + g + c * NC], rq = R[SH::LOR + g], gq = R[SH::LOG + g];
                const double a = sqrt(fabs(rq)) * dgc;
                const d4 H0 = in.H;
                const double h0 = in.h;
                in.H = mfma_f64(a, rq < 0.0 ? -a : a, in.H);
                in.h -= sum_groups(dgc * (rq * gq));  // h~ -= D^T (rho o g)
                double *Hk = A.Hw + b * sh.perHw + (long long)k * SH::ps;
                // only entries whose bits the penalty changed are written back
                // (a box on u changes the u block alone); lane 0 always stores,
                // so every store instruction has a live lane and the fixed
                // vm-op counts of the waits hold
                auto changed = [&](double x, double y) {
                    return lane == 0 || __double_as_longlong(x) != __double_as_longlong(y);
                };
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 4 * r + g;
                    if (changed(in.H[r], H0[r])) gstore(Hk + (i >= c ? pidx(i, c, SH::s) : pidx(c, i, SH::s)), in.H[r]);
                }
                if (changed(in.h, h0)) gstore(A.hw + b * sh.perh + (long long)k * SH::s + c, in.h);
            }
            double w, luq[4];
            GainOut go;
            // the fused-penalty instance (2 waves per SIMD launch bounds) has
            // the registers for G and M on three accumulators each (SPLIT = 1)
            const bool ok = schur_stage<SH::m, decltype(sym)::value, GAIN, GAIN, (NC > 0 ? 1 : 0)>(
                Pm, prow, in, sm, m, s, g, c, w, luq, sym_rt, &go);
            fail_stage = (!ok && fail_stage < 0) ? k : fail_stage;
            schur_store_record_gain<SH::m, SH::s>(FRb + (long long)k * frs, go, g, c);
            wave_sync();  // stage k's LDS reads retire before slot reuse
        };
        auto step = [&](int k, d2v(&X)[NI], bool first, auto sym, bool sym_rt) {  // X: stage k - 1 on entry, k - 3 on exit
            process(k, sym, sym_rt);
            if (first) vwait4(X);
            else vwait5(X);
            if (k >= 1) lput(X, (k - 1) & 1);
            gload(X, k >= 3 ? k - 3 : 0);
            wave_sync();
        };
        // No load may still be in flight where control flow joins: the
        // compiler is free to copy an asm output there (it cannot know the
        // value is still arriving) and to reuse the source registers, which
        // the landing load then overwrites.  (It did exactly that at the loop
        // exit: the set loaded by the last pair's head was moved into other
        // registers and its old registers became the final stage's MFMA
        // accumulators -- stage 0 of a random ~2 % of the problems came out
        // wrong or NaN, depending on when the load landed.)  So the last pair
        // drains the counter with an operand-less wait, and the final stage
        // reads only LDS.
        auto drain = [&]() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };
        gload(RA, N - 1);
        vwait0(RA);
        lput(RA, (N - 1) & 1);
        gload(RA, N >= 2 ? N - 2 : 0);
        gload(RB, N >= 3 ? N - 3 : 0);
        wave_sync();
        // pairs (k, k - 1): the pair head symmetrises (every pair head for
        // PDPLQR_SYM_EVERY = 2, every other one for 4), the second stage only
        // when PDPLQR_SYM_EVERY = 1
        step(N - 1, RA, true, SymOn{}, true);
        if (N < 3) drain();
        int k = N - 2;
        for (; k >= 1; k -= 2) {
            step(k, RB, false, SymOn{}, PDPLQR_SYM_EVERY < 4 || ((N - 2 - k) & 2) == 0);
            step(k - 1, RA, false, std::integral_constant<bool, (PDPLQR_SYM_EVERY <= 1)>{}, true);
            if (k < 3) drain();  // wave-uniform: the last pair
        }
        if (k == 0) process(0, SymOn{}, true);  // its record went to LDS slot 0 in step 1
    } else {
        SchurIn nxt;
        schur_load(nxt, Eb + (long long)(N - 1) * n * s, cb + (long long)(N - 1) * n, Hb + (long long)(N - 1) * ps,
                   hb + (long long)(N - 1) * s, n, m, s, g, c, n);
        for (int k = N - 1; k >= 0; --k) {
            const SchurIn in = nxt;
            if (k > 0)
                schur_load(nxt, Eb + (long long)(k - 1) * n * s, cb + (long long)(k - 1) * n,
                           Hb + (long long)(k - 1) * ps, hb + (long long)(k - 1) * s, n, m, s, g, c, n);
            double w, luq[4];
            const bool ok = schur_stage<0>(Pm, prow, in, sm, m, s, g, c, w, luq);
            if (!ok && fail_stage < 0) fail_stage = k;
            schur_store_record(FRb + (long long)k * frs, Pm, sm, m, s, g, c);
        }
    }
    if (lane == 0) A.status[b] = fail_stage < 0 ? 0 : fail_stage + 1;
    PDPLQR_PROBE_END(lane, b)
}

PDPLQR_PROBE_DEFINE(schur)

static bool schur_aligned(const RiccatiArgs &a) {
    const Shape &sh = a.sh;
    auto al = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    return al(a.E) && al(a.c) && al(a.Hw) && al(a.hw) && sh.perE % 2 == 0 && sh.perc % 2 == 0 &&
           sh.perHw % 2 == 0 && sh.perh % 2 == 0;
}

static bool schur_ct(const RiccatiArgs &a) {  // the compile-time 12/4 kernel applies
    const Shape &sh = a.sh;
    return !a.Lc && sh.n == 12 && sh.m == 4 && schur_aligned(a);
}

// The backward for these arguments leaves the gain-form record [K~ | k~]
// (the forward must then run launch_rollout_dma(..., gain = true)).
bool schur_gain_record(const RiccatiArgs &a) { return schur_ct(a); }

// The fused-penalty backward applies: the 12/4 gain-form kernel, nc = 4 rows on
// every stage k < N (the C5 layout), nc_N <= 4, 16-byte aligned per-problem
// blocks of D, rho and g.
int launch_riccati_backward_pen(const RiccatiArgs &a, int nc, hipStream_t st) {
    const Shape &sh = a.sh;
    auto al = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    if (nc != 4 || a.nc_last > 4 || !schur_gain_record(a) || !a.D || !a.rho ||
        !a.gw || !al(a.D) || !al(a.rho) || !al(a.gw) || sh.ny % 2 || sh.ndD % 2)
        return PDPLQR_ERR_UNSUPPORTED;
    with_x1(sh.x1, [&](auto x1) {
        hipLaunchKernelGGL((k_riccati_bwd_schur<12, 4, true, 4, decltype(x1)::value>), dim3(sh.batch), dim3(64), 0, st,
                           a);
    });
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

// Returns PDPLQR_ERR_UNSUPPORTED when the shape / options need the full-factor kernels.
int launch_riccati_backward_schur(const RiccatiArgs &a, hipStream_t st) {
    const Shape &sh = a.sh;
    if (a.Lc || sh.s > 16) return PDPLQR_ERR_UNSUPPORTED;
    if (schur_gain_record(a))
        with_x1(sh.x1, [&](auto x1) {
            hipLaunchKernelGGL((k_riccati_bwd_schur<12, 4, true, 0, decltype(x1)::value>), dim3(sh.batch), dim3(64), 0,
                               st, a);
        });
    else
        hipLaunchKernelGGL((k_riccati_bwd_schur<0, 0>), dim3(sh.batch), dim3(64), 0, st, a);
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

}  // namespace pdplqr
