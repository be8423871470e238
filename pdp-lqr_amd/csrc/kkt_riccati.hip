// kkt_riccati.hip -- QDLDLSolver's KKT system (kkt.hpp:124-300) eliminated in
// REVERSE stage order: a Riccati-ordered block LDL^T of the same matrix, with
// its frozen regularisation carried exactly.
//
// The reference assembles (kkt.hpp:124-205, qdldl_solver.hpp:36-45)
//     [ H_k + sigma_f I   C^T        ]   sigma_f = kkt_sigma (1e-6, frozen),
//     [ C                -Reg        ]   Reg = rho_dyn I on every lambda_k,
//                                              diag(inv_rho) on every y_k
// and factors it with QDLDL in natural order (primal pivots first).  The
// solution of a nonsingular quasi-definite system does not depend on the
// elimination order, so eliminating it stage by stage from the END gives the
// same (w, y, lambda) to rounding, and each step is a value-function update:
//   * y_k (row D_k w_k - inv_rho y_k = g_k, g = z - inv_rho o y_in):
//       y_k = rho (D_k w_k - g_k)  ->  H~ += D^T rho D,  h~ -= D^T rho g
//     (rho = 1 / inv_rho of backward(), g from update_problem_data: exactly the
//      Riccati solvers' penalty, lqr_kernel.hpp:106-112; stage 0 keeps only the
//      u columns of D_0, as the KKT drops D_x0 x0, kkt.hpp:218-221);
//   * lambda_{k+1} (row E_k w_k + c_k - x_{k+1} - rho_dyn lambda_{k+1} = 0):
//       eliminating lambda and x_{k+1} against the value function V_{k+1} =
//       (P, p) leaves the Moreau envelope of V_{k+1} at v = E_k w_k + c_k,
//         P~ = (P^{-1} + rho_dyn I)^{-1} = P (I + rho_dyn P)^{-1},
//         p~ = (I + rho_dyn P)^{-1} p,
//       and the minimiser x_{k+1} = v - rho_dyn (P~ v + p~)  (the costate
//       lambda_{k+1} = P~ v + p~);
//   * (u_k, x_k): the value-form stage of kernels_schur.hip on
//       M_k = H~_k + E~^T P~ E~ (+ D^T rho D),  lp = h~ + E^T (P~ c + p~).
// P~ is formed by the Neumann series P~ = sum_j (-rho_dyn P)^j P (one MFMA
// product per term) while e = rho_dyn ||P||_F is small enough for eight terms
// to reach rounding (e <= 0.015: rho_dyn = 1e-6 and ||P|| up to 1.5e4), and
// EXACTLY otherwise: Gauss-Jordan inversion of the SPD S = I + rho_dyn P and
// P~ = P S^{-1} (ptilde_exact; the wide kernel: Cholesky of S and two
// triangular solves).  A non-SPD S is flagged in the status, as a bad pivot.
// p~ never appears alone: lp = h~ + G^T (c - rho_dyn p) + E~^T p with
// G = P~ E~, and the forward uses x+ = v - rho_dyn (P~ (v - rho_dyn p) + p).
//
// Per stage this reads E, c, h~, packed H~ = H + sigma_f I, D, inv_rho, g
// (428 doubles at 12/4 with 4 rows) once and writes the rollout record
// [K~ | k~ | p_{k+1} | P~_{k+1} (fp64, packed lower)] -- against the
// natural-order path's once-per-model H^{-1} / G tiles and its three solve
// phases over explicit fp64 tiles (kkt.hip).  P~ stays fp64: rho_dyn P~ has
// norm rho_dyn lambda / (1 + rho_dyn lambda), up to 1 when rho_dyn ||P|| is large,
// so a rounded P~ would move x by its own relative rounding.
//
// update_rhs_initial_stage ACCUMULATES -S0 x0 and -A0 x0 into the right-hand
// side on every forward (kkt.hpp:207-222): the solve then uses the sum of every
// x0 passed since the last update_problem_data (x0acc here), while ws[0]'s x
// part is the x0 of the call (qdldl_solver.hpp:129-131).
#include "admm.hpp"
#include "blk_la.hpp"
#include "schur_stage.hpp"
#include "solvers.hpp"

#include <stdint.h>
#include <stdlib.h>

namespace pdplqr {

struct KKTRicArgs {
    Shape sh;
    const double *E, *c, *D;  // model
    const double *Hw, *hw;    // H + sigma_f I (packed), h - sigma w
    const double *gw;         // z - inv_rho o y (update_problem_data)
    const double *irho;       // backward's inv_rho
    const int32_t *d_off, *y_off;
    double *rec;              // [b][N][KKT_FS] rollout records
    double *cache = nullptr;  // linear-pass factor cache [b][N][KKT_CF] (ADMM), or null
    int32_t *status;
    double rho_dyn;
    int nc_last;              // constraint rows of the terminal stage
};

// Record per stage (PDPLQR_KKT_EHAT = 1, default):
//     K~ (m x n row-major) | k~ (m) | E^ = (I - rho_dyn P~_{k+1}) E~ | c^
// with c^ = (I - rho_dyn P~_{k+1})(c - rho_dyn p_{k+1}): the lambda
// correction x+ = v - rho_dyn (P~ (v - rho_dyn p) + p), v = A x + B u + c, is
// x+ = (I - rho_dyn P~)(v - rho_dyn p) = E^ [u; x] + c^, so the forward is a
// plain gain-form rollout on E^, c^ (one group sum and no LDS round trip less
// per stage, and E, c are not read again).  E^ is stored in the backward's C
// layout: element 64 (r - 1) + 16 g + c = E^[x row 4 (r - 1) + g][tile column c].
// 256 doubles = two 16-byte DMA instructions per lane.
// The ADMM runs (a backward that writes the linear pass's cache, then the
// linear pass) keep the P~ record K~ | k~ | p_{k+1} (n) | P~_{k+1} (fp64;
// packed lower, pidx(i, j, n)) and the forward applies the correction itself:
// rewriting c^ in the linear pass costs that pass more (one wave per SIMD:
// every instruction is on its time) than the forward saves (profiles/r04).
// Both forms share the 256-double stage stride; the handle records which one
// the last backward left (KKTState::rec_ehat).
template <int NN, int MM>
struct KRecShape {
    static constexpr int n = NN, m = MM, s = NN + MM;
    static constexpr int OK = 0, OKQ = n * m;
    static constexpr int OEH = OKQ + m, OCH = OEH + 3 * 64;  // E^ record
    static constexpr int OPV = OKQ + m, OPT = OPV + n;        // P~ record
    static constexpr int FS_EH = OCH + n, FS_PT = OPT + n * (n + 1) / 2;
    static constexpr int FS = FS_EH > FS_PT ? FS_EH : FS_PT;  // stage stride
    static_assert(NN == 12 && MM == 4, "E^ record: 12/4");
};

// c^ store of the EHAT record: lanes (g, c >= 4) hold c^[c - 4] (column
// layout) and store it (the four row groups write equal values); lanes c < 4
// are masked off.  One store instruction with live lanes every stage, so the
// callers' fixed vm-op counts hold; the loads in flight are asm-issued, so the
// exec-mask region cannot make the compiler drain them.  (A cross-lane copy
// for lanes c < 4 cost an LDS round trip a stage in the linear ADMM pass.)
__device__ __forceinline__ void kkt_store_chat(double *Rk_och, double v, int c) {
    if (c >= 4) gstore(Rk_och + (c - 4), v);
}

// Factor cache of the linear-only pass (k_kkt_ric_nofact; written by the
// backward when KKTRicArgs::cache is set), per stage three lane-interleaved
// pair slots (lane L's two doubles at 2 L: one 16-byte load per lane, 1 KB
// contiguous per instruction) and the packed Luu^{-1}:
//   KC_EE  (e0, e1)  E^ = E~ - rho_dyn G, x rows 4 + g and 8 + g (G = P~ E~)
//   KC_EW  (e2, w)   x row 12 + g of E^;  w = Lxu (lane (g, c): L(c, g))
//   KC_QR  (q, rD)   q = G^T c~ (column c);  rho D (lane (g, c): rho_g D[g][c],
//                    stage 0 without the x columns)
//   KC_T   T = Luu^{-1} packed lower, t = i (i + 1) / 2 + j (10 doubles, read
//          wave-uniform by five 16-byte loads)
// so that lp = h~ + q + E^^T p - (rho D)^T g, lu' = T lu, k~ = T^T lu',
// p_k = lp_x - Lxu lu': the right-hand-side dependent part of the backward.
// Ten load instructions a stage let the pass keep five stages in flight
// within the 63 outstanding vector-memory operations a wave may have.
// (ADMM runs keep the P~ record: the pass rewrites k~ and p_{k+1}.)
constexpr int KC_EE = 0, KC_EW = 128, KC_QR = 256, KC_T = 384;
constexpr int KKT_CF = 400;

// Stage record streamed by the backward: E | c | h~ | packed H~ | D | inv_rho | g
template <int NN, int MM, int NC>
struct KBwdShape {
    static constexpr int n = NN, m = MM, s = NN + MM, nc = NC;
    static constexpr int ps = s * (s + 1) / 2;
    static constexpr int OE = 0, OC = n * s, OH = OC + n, OP = OH + s, OD = OP + ps, OI = OD + nc * s,
                         OG = OI + nc, Q = OG + nc;
    static constexpr int CH = Q / 2, NI = (CH + 63) / 64, SLOT = NI * 128;
    static_assert(Q % 2 == 0 && OC % 2 == 0 && OH % 2 == 0 && OP % 2 == 0 && OD % 2 == 0 && OI % 2 == 0, "chunks");
};

// sum of a value over the whole wave (every lane gets it)
__device__ __forceinline__ double wave_sum(double v) { return sum_groups(sum_row16(v)); }

// PDPLQR_KKT_NEUMANN_MAX (device_common.hpp): the Neumann / exact P~ switch

// Exact P~ = (I + rho_dyn P)^{-1} P of the x block (tile indices 4..15) of a
// 16 x 16 C/D-layout tile: in-place Gauss-Jordan inversion of S = I + rho_dyn P
// (12 pivots, no pivoting: S is SPD with eigenvalues >= 1 whenever P is PSD,
// so every pivot is >= 1), then one product P S^{-1}.  Rows / columns < 4 of the
// result are not meaningful (the callers read the x block only).  False if a
// pivot is not positive (P not PSD enough for S to be SPD).
// (inlined: a call inside the stage loop would save / restore registers whose
// staging loads are still in flight, the hazard tests/test_kernel_static.py guards)
__device__ __forceinline__ bool ptilde_exact(const d4 &P, double rd, int g, int c, d4 &Pt) {
    d4 S;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = 4 * r + g;
        S[r] = (i >= 4 && c >= 4) ? rd * P[r] : 0.0;
        if (i == c) S[r] += 1.0;
    }
    bool ok = true;
#pragma unroll
    for (int j = 4; j < 16; ++j) {
        const int rj = j >> 2, gj = j & 3;
        double colj[4];  // S[4 r + g][j] of the lane's rows (u rows: 0)
        colj[0] = 0.0;
#pragma unroll
        for (int r = 1; r < 4; ++r) colj[r] = __shfl(S[r], 16 * g + j, 64);
        const double rowj = __shfl(S[rj], 16 * gj + c, 64);  // S[j][c]
        const double piv = readlane_f64(S[rj], 16 * gj + j);
        ok = ok && piv > 0.0;
        const double ip = rcp_f64(piv);
#pragma unroll
        for (int r = 1; r < 4; ++r) {
            const int i = 4 * r + g;
            const double a = colj[r] * ip;
            S[r] = (i == j) ? ((c == j) ? ip : rowj * ip) : ((c == j) ? -a : __builtin_fma(-a, rowj, S[r]));
        }
    }
    const d4 z = {0.0, 0.0, 0.0, 0.0};
    Pt = mfma_f64_x3(P[1], S[1], P[2], S[2], P[3], S[3], z);  // P^T S^{-1} = P S^{-1}
    return ok;
}

// P~ of the x block for the 12/4 kernels: the Neumann series while it has
// converged to rounding (e <= PDPLQR_KKT_NEUMANN_MAX, wave-uniform), the exact
// inversion above otherwise.  False: S = I + rho_dyn P was not SPD.
__device__ __forceinline__ bool ptilde_12(const d4 &Pm, double rd, int g, int c, d4 &Pt) {
    // the powers by a product tree instead of a chain of J products:
    // P^2 | P^3 = P^2 P, P^4 = P^2 P^2 | P^5..P^8 = P^4 P^{1..4} | P^9 = P^8 P,
    // so J = 3 (rho_dyn ||P|| ~ 1e-4) is two dependent products, not three
    // (every power of the symmetric P is symmetric: its registers serve as the
    // A operand, read as the transpose, like P's own).  P^2, P^3, P^4 are
    // issued before the norm that picks J is known: the norm's cross-lane sum
    // and square root then run beside the products instead of ahead of them
    // on the stage chain (a smaller J leaves them unused).
    const d4 z = {0.0, 0.0, 0.0, 0.0};
    auto mul = [&](const d4 &X, const d4 &Y) { return mfma_f64_x3(X[1], Y[1], X[2], Y[2], X[3], Y[3], z); };
    const d4 Q2 = mul(Pm, Pm);
    const d4 Q3 = mul(Q2, Pm);
    const d4 Q4 = mul(Q2, Q2);
    double f = 0.0;
#pragma unroll
    for (int r = 1; r < 4; ++r) f = (c >= 4) ? __builtin_fma(Pm[r], Pm[r], f) : f;
    const double e = rd * sqrt(wave_sum(f));
    if (__builtin_amdgcn_readfirstlane((int)(e > PDPLQR_KKT_NEUMANN_MAX))) return ptilde_exact(Pm, rd, g, c, Pt);
    // J terms (-rho_dyn)^j P^{j+1}, j = 1..J, while e^j > 1e-16 (wave-uniform)
    int J = 0;
    for (double ej = e; J < 8 && ej > 1e-16; ej *= e) ++J;
    auto acc = [&](const d4 &Q, double f) {
#pragma unroll
        for (int r = 0; r < 4; ++r) Pt[r] = __builtin_fma(f, Q[r], Pt[r]);
    };
    const double r1 = -rd, r2 = rd * rd, r3 = -r2 * rd, r4 = r2 * r2;
    Pt = Pm;
    if (J >= 1) {
        if (J >= 2) {
            if (J >= 4) {
                const d4 Q5 = mul(Q4, Pm);
                d4 Q6 = z, Q7 = z, Q8 = z, Q9 = z;
                if (J >= 5) Q6 = mul(Q4, Q2);
                if (J >= 6) Q7 = mul(Q4, Q3);
                if (J >= 7) Q8 = mul(Q4, Q4);
                if (J >= 8) Q9 = mul(Q8, Pm);
                // smallest terms first
                if (J >= 8) acc(Q9, r4 * r4);
                if (J >= 7) acc(Q8, r4 * r3);
                if (J >= 6) acc(Q7, r4 * r2);
                if (J >= 5) acc(Q6, r4 * r1);
                acc(Q5, r4);
            }
            if (J >= 3) acc(Q4, r3);
            acc(Q3, r2);
        }
        acc(Q2, r1);
    }
    return true;
}

template <int NC, bool X1 = false>
__global__ __launch_bounds__(64, 1) void k_kkt_ric_bwd(KKTRicArgs A) {
    PDPLQR_PROBE_BEGIN
    simd_exclusive<X1>();
    constexpr int NN = 12, MM = 4;
    using SH = KBwdShape<NN, MM, NC>;
    using RS = KRecShape<NN, MM>;
    constexpr int NI = SH::NI, n = NN, m = MM, s = NN + MM;
    // record store instructions per stage, all issued every stage (the counts
    // below are exact without the ADMM cache; its extra stores only make the
    // waits stricter): [K~ | k~] + E^ (3) + c^, or [K~ | k~] + p_{k+1} + P~ (3)
    // (the packed P~ stores are lane-masked but every instruction has live lanes)
    constexpr int ST = 5;
    __shared__ SchurSmem sm;
    __shared__ __attribute__((aligned(16))) double stg[2][SH::SLOT];
    const int lane = wave_lane(), g = lane >> 4, c = lane & 15;
    const long long b = blockIdx.x;
    const Shape &sh = A.sh;
    const int N = sh.N;
    const double *Eb = A.E + b * sh.perE;
    const double *cb = A.c + b * sh.perc;
    const double *Hb = A.Hw + b * sh.perHw;
    const double *hb = A.hw + b * sh.perh;
    const double *Db = A.D + b * (long long)sh.ndD;
    const double *gb = A.gw + b * (long long)sh.ny;
    const double *ib = A.irho + b * (long long)sh.ny;
    double *RB = A.rec + b * (long long)N * RS::FS;
    const double rd = A.rho_dyn;
    double *const cache = A.cache;  // (a member read inside the stage lambda would put A in scratch)
    // the E^ record for a plain solve, the P~ record when the ADMM cache is written
    const bool ehat = cache == nullptr;
    int fail_stage = -1;

    // ---- terminal: P_N = H~_N + D_N^T rho D_N, p_N = h~_N - D_N^T rho g_N ----
    d4 Pm;
    double prow[4];
    {
        d4 Mt[1][1];
        load_M<1>(Mt, Hb + (long long)N * sh.ps, n, m, m, s, g, c);
        Pm = Mt[0][0];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 4 * r + g;
            prow[r] = i >= m ? hb[(long long)N * s + (i - m)] : 0.0;
        }
        const int ncN = A.nc_last;
        if (ncN > 0) {  // rare: plain loops (nc_N <= 4, D_N is nc_N x n)
            const double *DN = Db + A.d_off[N];
            const double *gN = gb + A.y_off[N], *iN = ib + A.y_off[N];
            for (int q = 0; q < ncN; ++q) {
                const double rq = 1.0 / iN[q], gq = gN[q];
                const double dc = c >= m ? DN[q + (c - m) * ncN] : 0.0;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 4 * r + g;
                    const double di = i >= m ? DN[q + (i - m) * ncN] : 0.0;
                    Pm[r] = __builtin_fma(di * rq, dc, Pm[r]);
                    prow[r] = __builtin_fma(-di * rq, gq, prow[r]);
                }
            }
        }
        bool bad = false;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 4 * r + g;
            if (i == c && i >= m && psd_bad(Pm[r])) bad = true;
        }
        if (__any(bad)) fail_stage = N;
    }

    // ---- stage records: HBM -> registers (two sets in flight) -> LDS, as the
    // 12/4 value-form backward (kernels_schur.hip) ----
    d2v RA[NI], RB2[NI];
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
                   : d < SH::OI ? Db + (d - SH::OD)
                   : d < SH::OG ? ib + (d - SH::OI)
                                : gb + (d - SH::OG);
        gstride[q] = d < SH::OC ? n * s : d < SH::OH ? n : d < SH::OP ? s : d < SH::OD ? sh.ps : d < SH::OI ? NC * s : NC;
    }
    auto gload = [&](d2v(&R)[NI], int k) {
#pragma unroll
        for (int q = 0; q < NI; ++q) {
            const double *src = gbase[q] + (long long)k * gstride[q];
            asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(R[q]) : "v"(src) : "memory");
        }
    };
    // "set X has landed": the younger vm ops are the other set's NI loads and
    // two steps' ST stores (steady state), one step's stores (first step)
    auto vwait_steady = [&](d2v(&R)[NI]) {
        if constexpr (NI == 4)
            asm volatile("s_waitcnt vmcnt(%4)" : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]), "+v"(R[3]) : "n"(NI + 2 * ST) : "memory");
        else asm volatile("s_waitcnt vmcnt(%3)" : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]) : "n"(NI + 2 * ST) : "memory");
    };
    auto vwait_first = [&](d2v(&R)[NI]) {
        if constexpr (NI == 4)
            asm volatile("s_waitcnt vmcnt(%4)" : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]), "+v"(R[3]) : "n"(NI + ST) : "memory");
        else asm volatile("s_waitcnt vmcnt(%3)" : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]) : "n"(NI + ST) : "memory");
    };
    auto vwait0 = [&](d2v(&R)[NI]) {
        if constexpr (NI == 4)
            asm volatile("s_waitcnt vmcnt(0)" : "+v"(R[0]), "+v"(R[1]), "+v"(R[2]), "+v"(R[3])::"memory");
        else asm volatile("s_waitcnt vmcnt(0)" : "+v"(R[0]), "+v"(R[1]), "+v"(R[2])::"memory");
    };
    auto lput = [&](const d2v(&R)[NI], int slot) {
#pragma unroll
        for (int q = 0; q < NI; ++q) *reinterpret_cast<d2v *>(&stg[slot][2 * (q * 64 + lane)]) = R[q];
    };

    auto process = [&](int k, bool sym) __attribute__((always_inline)) {
        const double *R = stg[k & 1];
        double *Rk = RB + (long long)k * RS::FS;
        SchurIn in;
        schur_load(in, R + SH::OE, R + SH::OC, R + SH::OP, R + SH::OH, n, m, s, g, c, n);
        // ---- the lambda_{k+1} elimination: P~ = (I + rho_dyn P)^{-1} P ----
        d4 Pt;
        const bool pt_ok = ptilde_12(Pm, rd, g, c, Pt);
        // ---- record part 1: p_{k+1} (lanes (g, c = 1..3): p[4 c + g - m]) and P~_{k+1} ----
        if (!ehat) {  // (wave-uniform)
            // every lane stores (duplicates carry the same value): one store
            // instruction per part, no exec-mask branch
            const int cp = c < 1 ? 1 : (c > 3 ? 3 : c);
            // (a select chain on cp became a dynamically indexed private array)
            const double pv = __builtin_fma(prow[1], (double)(cp == 1), __builtin_fma(prow[2], (double)(cp == 2),
                                                                                       prow[3] * (double)(cp == 3)));
            gstore(Rk + RS::OPV + (4 * cp + g - m), pv);
            // P~ (fp64, packed lower of the x block): lane (g, c >= m) holds
            // x rows g, 4 + g, 8 + g of x column c - m
            if (c >= m) {
#pragma unroll
                for (int r = 1; r < 4; ++r) {
                    const int i = 4 * (r - 1) + g, j = c - m;
                    if (i >= j) gstore(Rk + RS::OPT + pidx(i, j, n), Pt[r]);
                }
            }
        }
        // ---- G = P~ E~, M = H~ + E~^T G + D^T rho D ----
        // (one wave per SIMD at C5: the stage is chain-bound, and the split
        // accumulators of mfma_f64_x3 take two MFMA latencies off each product)
        const d4 z4 = {0.0, 0.0, 0.0, 0.0};
        const d4 G = mfma_f64_x3(Pt[1], in.E[1], Pt[2], in.E[2], Pt[3], in.E[3], z4);
        d4 Mn = mfma_f64_x3(in.E[1], G[1], in.E[2], G[2], in.E[3], G[3], in.H);
        double part = 0.0, rhoD = 0.0;
        if constexpr (NC > 0) {
            // lane (g, c): D[g][c] (rows g < NC); stage 0 keeps only the u columns
            const bool dv = g < NC && (k > 0 || c < m);
            const double dgc = dv ? R[SH::OD + (g < NC ? g : 0) + c * NC] : 0.0;
            const double rq = (g < NC) ? rcp_f64(R[SH::OI + (g < NC ? g : 0)]) : 0.0;
            const double gq = (g < NC) ? R[SH::OG + (g < NC ? g : 0)] : 0.0;
            rhoD = rq * dgc;
            Mn += mfma_f64(dgc, rhoD, z4);         // D^T diag(rho) D (off the G -> M chain)
            part = -dgc * rq * gq;                 // -(D^T rho g)[c]
        }
        double *Ck = cache ? cache + ((long long)b * N + k) * KKT_CF : nullptr;
        double qcol = 0.0, e2c = 0.0;
        if (ehat) {
            // ---- record part 1: E^ = E~ - rho_dyn P~ E~ (= E~ - rho_dyn G), c^ ----
            double cv = 0.0;
#pragma unroll
            for (int r = 1; r < 4; ++r) {
                gstore(Rk + RS::OEH + 64 * (r - 1) + lane, __builtin_fma(-rd, G[r], in.E[r]));
                const double mh = __builtin_fma(-rd, Pt[r], (4 * r + g == c) ? 1.0 : 0.0);  // M^ = I - rho_dyn P~
                cv = __builtin_fma(mh, __builtin_fma(-rd, prow[r], in.ct[r]), cv);      // M^ (c - rho_dyn p)
            }
            kkt_store_chat(Rk + RS::OCH, sum_groups(cv), c);
        }
        if (Ck) {  // wave-uniform: the linear pass's copy of this stage's factor
            double ev[3];
#pragma unroll
            for (int kk = 1; kk < 4; ++kk) {
                ev[kk - 1] = __builtin_fma(-rd, G[kk], in.E[kk]);
                qcol = __builtin_fma(G[kk], in.ct[kk], qcol);
            }
            qcol = sum_groups(qcol);
            gstore2(Ck + KC_EE + 2 * lane, d2v{ev[0], ev[1]});
            gstore2(Ck + KC_QR + 2 * lane, d2v{qcol, rhoD});
            e2c = ev[2];
        }
#pragma unroll
        for (int kk = 1; kk < 4; ++kk) {
            part = __builtin_fma(G[kk], __builtin_fma(-rd, prow[kk], in.ct[kk]), part);  // G^T (c - rho_dyn p)
            part = __builtin_fma(in.E[kk], prow[kk], part);                             // E~^T p
        }
        part = sum_groups(part);
        sm.lpt[colpos<1>(c)] = in.h + part;
        wave_sync();
        double lpr[4];
        {
            const double2 *q = reinterpret_cast<const double2 *>(sm.lpt + 4 * g);
            const double2 a = q[0], bb = q[1];
            lpr[0] = a.x;
            lpr[1] = a.y;
            lpr[2] = bb.x;
            lpr[3] = bb.y;
        }
        double w, luq[4];
        GainOut go;
        // (LPW: lu rides in W's column 0 -- the cache's w slot is read on the
        // x columns only, and go.T still carries Luu^{-1} for it)
        bool ok = schur_block_pivots<MM, true, true>(Mn, lpr, w, luq, g, c, &go, sm.col, sm.lu4);
        Pm = Mn;
#pragma unroll
        for (int r = 0; r < 4; ++r) prow[r] = lpr[r];
        if (sym) {
#pragma unroll
            for (int r = 0; r < 4; ++r) sm.tp[(4 * r + g) * PDPLQR_TP_LD + c] = Pm[r];
            wave_sync();
#pragma unroll
            for (int r = 0; r < 4; ++r) Pm[r] = 0.5 * (Pm[r] + sm.tp[c * PDPLQR_TP_LD + 4 * r + g]);
        }
        bool bad = false;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 4 * r + g;
            if (i == c && i >= m && psd_bad(Pm[r])) bad = true;
        }
        ok = (int)ok & (int)!__any(bad) & (int)pt_ok;
        fail_stage = (!ok && fail_stage < 0) ? k : fail_stage;
        schur_store_record_gain<MM, s>(Rk, go, g, c);  // [K~ | k~]
        if (Ck) {
            double tv = 0.0;
#pragma unroll
            for (int i = 0; i < MM; ++i)
#pragma unroll
                for (int j = 0; j <= i; ++j) tv = (lane == i * (i + 1) / 2 + j) ? go.T[i][j] : tv;
            gstore2(Ck + KC_EW + 2 * lane, d2v{e2c, w});
            if (lane < MM * (MM + 1) / 2) gstore(Ck + KC_T + lane, tv);
        }
        wave_sync();  // stage k's LDS reads retire before slot reuse
    };
    auto step = [&](int k, d2v(&X)[NI], bool first, bool sym) {
        process(k, sym);
        if (first) vwait_first(X);
        else vwait_steady(X);
        if (k >= 1) lput(X, (k - 1) & 1);
        gload(X, k >= 3 ? k - 3 : 0);
        wave_sync();
    };
    auto drain = [&]() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };
    gload(RA, N - 1);
    vwait0(RA);
    lput(RA, (N - 1) & 1);
    gload(RA, N >= 2 ? N - 2 : 0);
    gload(RB2, N >= 3 ? N - 3 : 0);
    wave_sync();
    step(N - 1, RA, true, true);
    if (N < 3) drain();
    int k = N - 2;
    for (; k >= 1; k -= 2) {
        step(k, RB2, false, ((N - 2 - k) & 2) == 0);
        step(k - 1, RA, false, false);
        if (k < 3) drain();
    }
    if (k == 0) process(0, true);
    if (lane == 0) A.status[b] = fail_stage < 0 ? 0 : fail_stage + 1;
    PDPLQR_PROBE_END(lane, b)
}

PDPLQR_PROBE_DEFINE(kkt)

// ---------------------------------------------------------------------------
// The right-hand-side part of the backward on a cached factor (the KKT
// matrix, i.e. rho, unchanged; h~ and g new): QDLDLSolver::solve after a
// factorisation (qdldl_solver.hpp:88-151) in the Riccati order.  Per stage
// (KKT_CF cache, written by k_kkt_ric_bwd):
//     lp = h~ + q + E^^T p_{k+1} - (rho D)^T g,   lu' = T lu,   k~ = T^T lu',
//     p_k = lp_x - Lxu lu'
// and the rollout record's k~ and p_{k+1} are rewritten (K~, P~ stay).  One
// wave per problem (one per SIMD at C5, so the pass is bound by the memory
// latency its lookahead covers): the cache of PDPLQR_KKT_NF_DEPTH stages is in
// flight into registers at a time.
// ---------------------------------------------------------------------------
// global_load_dwordx2 with an immediate byte offset (signed 13 bits), asm-issued
// like the other staging loads (the waits are explicit)
template <int OFF>
__device__ __forceinline__ void gl_at(double &x, const double *p) {
    static_assert(OFF >= -4096 && OFF < 4096, "global offset range");
    asm volatile("global_load_dwordx2 %0, %1, off offset:%2" : "=v"(x) : "v"(p), "n"(OFF) : "memory");
}

template <int OFF>
__device__ __forceinline__ void gl4_at(d2v &x, const double *p) {
    static_assert(OFF >= -4096 && OFF < 4096, "global offset range");
    asm volatile("global_load_dwordx4 %0, %1, off offset:%2" : "=v"(x) : "v"(p), "n"(OFF) : "memory");
}

// f(integral_constant<int, I>) for I = B .. E - 1 (compile-time set indices)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

#ifndef PDPLQR_KKT_NF_DEPTH
#define PDPLQR_KKT_NF_DEPTH 5
#endif

template <int NC, bool X1 = false>
__global__ __launch_bounds__(64) void k_kkt_ric_nofact(KKTRicArgs A) {
    simd_exclusive<X1>();
    constexpr int n = 12, m = 4, s = 16;
    using RS = KRecShape<n, m>;
    __shared__ double pc[16];
    const int lane = wave_lane(), g = lane >> 4, c = lane & 15;
    const long long b = blockIdx.x;
    const Shape &sh = A.sh;
    const int N = sh.N;
    const double *hb = A.hw + b * sh.perh;
    const double *gb = NC > 0 ? A.gw + b * (long long)sh.ny : nullptr;
    const double *Cb = A.cache + b * (long long)N * KKT_CF;
    double *RB = A.rec + b * (long long)N * RS::FS;
    // terminal: p_N = h~_N - D_N^T rho g_N (x rows)
    double prow[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = 4 * r + g;
        prow[r] = i >= m ? hb[(long long)N * s + (i - m)] : 0.0;
    }
    const int ncN = A.nc_last;
    if (ncN > 0) {
        const double *DN = A.D + b * (long long)sh.ndD + A.d_off[N];
        const double *gN = A.gw + b * (long long)sh.ny + A.y_off[N];
        const double *iN = A.irho + b * (long long)sh.ny + A.y_off[N];
        for (int q = 0; q < ncN; ++q) {
            const double rq = 1.0 / iN[q], gq = gN[q];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 4 * r + g;
                const double di = i >= m ? DN[q + (i - m) * ncN] : 0.0;
                prow[r] = __builtin_fma(-di * rq, gq, prow[r]);
            }
        }
    }
    double sel[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) sel[j] = (g == j) ? 1.0 : 0.0;
    // One register set per stage in flight: the cache pair slots (three
    // 16-byte loads), Luu^{-1} (five, wave-uniform), h~ and g.  The sets are
    // loaded by asm and waited for by an explicit vmcnt with the set's
    // registers as operands (compiler-placed waits drained every set at the top
    // of the loop).  DEPTH sets, the loop unrolled by DEPTH so no set is copied.
    constexpr int DEPTH = PDPLQR_KKT_NF_DEPTH, LV = 10, STS = 2;  // loads per set, stores per stage
    // "set j landed" with exactly the vm ops issued after its loads still in
    // flight: the other sets' loads, and the stores and reloads of the stages
    // in between -- (DEPTH - 1) LV + STS j in the first trip, (DEPTH - 1)(LV + STS)
    // from then on (a looser count would wait for younger loads too and cut
    // the lookahead)
    static_assert((DEPTH - 1) * (LV + STS) + LV <= 63, "vmcnt range");
    struct Set {
        d2v ee, ew, qr, t[5];
        double h, gv;
    };
    auto gl = [](double &x, const double *p) {
        asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(x) : "v"(p) : "memory");
    };
    auto load = [&](Set &X, int k) {
        const double *Ck = Cb + (long long)k * KKT_CF;
        const double *B1 = Ck + 2 * lane;  // lane-interleaved pair slots
        const double *B3 = Ck + KC_T;      // T (wave-uniform)
        gl4_at<8 * KC_EE>(X.ee, B1);
        gl4_at<8 * KC_EW>(X.ew, B1);
        gl4_at<8 * KC_QR>(X.qr, B1);
        gl4_at<0>(X.t[0], B3);
        gl4_at<16>(X.t[1], B3);
        gl4_at<32>(X.t[2], B3);
        gl4_at<48>(X.t[3], B3);
        gl4_at<64>(X.t[4], B3);
        gl(X.h, hb + (long long)k * s + c);
        gl(X.gv, NC > 0 ? gb + (long long)k * NC + (g < NC ? g : 0) : hb);
    };
    auto wait = [&](Set &X, auto cnt) {
        asm volatile("s_waitcnt vmcnt(%10)"
                         : "+v"(X.ee), "+v"(X.ew), "+v"(X.qr), "+v"(X.t[0]), "+v"(X.t[1]), "+v"(X.t[2]), "+v"(X.t[3]),
                           "+v"(X.t[4]), "+v"(X.h), "+v"(X.gv)
                         : "n"(decltype(cnt)::value)
                         : "memory");
    };
    // (registers of a set touched after a wait: the compiler must not reuse
    // them under loads still in flight)
    auto touch = [&](Set &X) {
        asm volatile("" : "+v"(X.ee), "+v"(X.ew), "+v"(X.qr), "+v"(X.t[0]), "+v"(X.t[1]), "+v"(X.t[2]), "+v"(X.t[3]),
                     "+v"(X.t[4]), "+v"(X.h), "+v"(X.gv));
    };
    auto stage = [&](Set &X, int k, auto cnt) {
        wait(X, cnt);
        const double e[3] = {X.ee.x, X.ee.y, X.ew.x};
        const double xw = X.ew.y, xq = X.qr.x;
        const double xrd = NC > 0 ? X.qr.y : 0.0, xgv = NC > 0 ? X.gv : 0.0;
        double T[10];
#pragma unroll
        for (int t = 0; t < 10; ++t) T[t] = (t & 1) ? X.t[t >> 1].y : X.t[t >> 1].x;
        double *Rk = RB + (long long)k * RS::FS;
        {  // record (the P~ form of ADMM runs): p_{k+1} (lanes (g, c = 1..3): p[4 c + g - m]), as the backward writes it
            const int cp = c < 1 ? 1 : (c > 3 ? 3 : c);
            const double pv = __builtin_fma(prow[1], (double)(cp == 1), __builtin_fma(prow[2], (double)(cp == 2),
                                                                                       prow[3] * (double)(cp == 3)));
            gstore(Rk + RS::OPV + (4 * cp + g - m), pv);
        }
        double part = 0.0;
#pragma unroll
        for (int r = 0; r < 3; ++r) part = __builtin_fma(e[r], prow[r + 1], part);
        if (NC > 0) part = __builtin_fma(-xrd, xgv, part);
        const double lp = X.h + xq + sum_groups(part);  // lp[c], every group
        double lu[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) lu[j] = readlane_f64(lp, j);
        // T[i][j] at t = i (i + 1) / 2 + j
        double luq[4], kq[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            double v = 0.0;
#pragma unroll
            for (int j = 0; j <= i; ++j) v = __builtin_fma(T[i * (i + 1) / 2 + j], lu[j], v);
            luq[i] = v;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            double v = 0.0;
#pragma unroll
            for (int l = i; l < 4; ++l) v = __builtin_fma(T[l * (l + 1) / 2 + i], luq[l], v);
            kq[i] = v;
        }
        const double kv = lane == 0 ? kq[0] : lane == 1 ? kq[1] : lane == 2 ? kq[2] : kq[3];
        if (lane < m) gstore(Rk + RS::OKQ + lane, kv);
        double lq = 0.0;
#pragma unroll
        for (int j = 0; j < 4; ++j) lq = __builtin_fma(sel[j], luq[j], lq);
        const double pcol = lp - sum_groups(xw * lq);  // p_k[c - m] on c >= m
        if (g == 0) pc[c] = pcol;
        wave_sync();
#pragma unroll
        for (int r = 1; r < 4; ++r) prow[r] = pc[4 * r + g];
        wave_sync();
    };
    // (loads unconditional, at clamped stages: a load inside a branch made the
    // wait-count pass drain every set in flight at the top of the loop)
    Set X[DEPTH];
    static_for<0, DEPTH>([&](auto J) {
        constexpr int j = decltype(J)::value;
        load(X[j], N - 1 - j >= 0 ? N - 1 - j : 0);
    });
    int k = N - 1;
    if (k >= DEPTH - 1) {  // first trip: fewer younger ops than in the steady state
        static_for<0, DEPTH>([&](auto J) {
            constexpr int j = decltype(J)::value;
            stage(X[j], k - j, std::integral_constant<int, (DEPTH - 1) * LV + STS * j>{});
            load(X[j], k - j - DEPTH >= 0 ? k - j - DEPTH : 0);
        });
        k -= DEPTH;
    }
    for (; k >= DEPTH - 1; k -= DEPTH) {
        static_for<0, DEPTH>([&](auto J) {
            constexpr int j = decltype(J)::value;
            stage(X[j], k - j, std::integral_constant<int, (DEPTH - 1) * (LV + STS)>{});
            load(X[j], k - j - DEPTH >= 0 ? k - j - DEPTH : 0);
        });
    }
    // the last k + 1 < DEPTH stages: every set landed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    static_for<0, DEPTH>([&](auto J) { touch(X[decltype(J)::value]); });
    static_for<0, DEPTH - 1>([&](auto J) {
        constexpr int j = decltype(J)::value;
        if (k - j >= 0) stage(X[j], k - j, std::integral_constant<int, (DEPTH - 1) * LV>{});
    });
}

// ---------------------------------------------------------------------------
// forward: the gain-form rollout of kernels_rollout.hip plus the lambda
// correction x+ = v - rho_dyn (P~ (v - rho_dyn p) + p), v = A x + B u + c.
//
// UPD (ADMM iterations on the C5 row layout, admm.hip): the z / y / w step of
// the iteration runs in the same pass, stage by stage right after w~_k leaves
// the chain -- w~ never goes to HBM and the separate update pass
// (k_admm_update) disappears.  The ring record grows by the stage's w, D, z,
// y, bounds, rho, 1 / rho and the model's h (120 doubles); the operations are
// k_admm_update's (KKT form: h~ = h - sigma w, rho enters through g), the
// stage's row sums by the same DPP butterfly; FUSE: also the next
// update_problem_data's h~ and g; CHECK: the termination test (wave-wide
// maxima, then admm_decide).  Rows: exactly Q.uni = 4 per stage k < N, none
// at the terminal.
// ---------------------------------------------------------------------------
// ring depth of the ADMM (UPD) rollout: stages in flight
#ifndef PDPLQR_KKT_UPD_RING
#define PDPLQR_KKT_UPD_RING 4
#endif
template <int D, bool UPD = false, bool FUSE = false, bool CHECK = false, bool EH = false, bool X1 = false>
__global__ __launch_bounds__(64) void k_kkt_ric_fwd(Shape sh, const double *__restrict__ E,
                                                    const double *__restrict__ c, const double *__restrict__ FR,
                                                    const double *__restrict__ x0, double *__restrict__ x0acc,
                                                    double *__restrict__ ws, double rho_dyn, AdmmArgs Q) {
    simd_exclusive<X1>();
    constexpr int n = 12, m = 4, s = 16, NC = 4;
    using RS = KRecShape<n, m>;
    constexpr int FS = RS::FS;  // stage stride of the record in HBM
    // ring record: [E | c |] F (the rollout record, FRL doubles) [| ADMM rows];
    // EH (the E^ record of a plain solve): E and c are not read (E^, c^ carry
    // them); otherwise the P~ record and the correction applied here
    static_assert(!EH || !UPD, "ADMM runs keep the P~ record");
    constexpr int FRL = EH ? RS::FS_EH : RS::FS_PT;
    constexpr int OE = 0, OC = EH ? 0 : n * s, OF = EH ? 0 : OC + n, OW = OF + FRL, OD = OW + s, OZ = OD + NC * s,
                  OY = OZ + NC, OLB = OY + NC, OUB = OLB + NC, ORH = OUB + NC, OIR = ORH + NC, OH = OIR + NC;
    constexpr int REC = UPD ? OH + s : OW, CH = REC / 2, NI = (CH + 63) / 64;
    constexpr int TAIL = CH - (NI - 1) * 64;
    constexpr int NQ = 3;
    static_assert(REC % 2 == 0 && OW % 2 == 0 && (NI >= 2 && NI <= 5), "record layout");
    // vm ops per stage: NI DMA + the stores (plain: the w~ store; UPD: z, y, w
    // [+ g, h~ with FUSE], each an instruction with live lanes)
    constexpr int ST = UPD ? (FUSE ? 5 : 3) : 1;
    __shared__ __attribute__((aligned(16))) double ring[D][REC];
    __shared__ double sx[16], sz[16], sx0[16];
    const int lane = wave_lane(), g = lane >> 4, cl = lane & 15;
    const long long b = blockIdx.x;
    if (UPD && Q.done[b]) return;  // frozen problem: no solve, no update (wave-uniform)
    const int N = sh.N;
    const double *Eb = E + b * sh.perE;
    const double *cb = c + b * sh.perc;
    const double *Fb = FR + b * (long long)N * FS;
    double *wb = ws + b * sh.perh;
    const double al = UPD ? Q.alpha : 0.0, bl = 1.0 - al;
    const long long pb = b * sh.perh, yb0 = b * (long long)sh.ny;

    auto dma = [&](int k, int slot) {
#pragma unroll
        for (int q = 0; q < NI; ++q) {
            if (q < NI - 1 || lane < TAIL) {
                const int d = 2 * (q * 64 + lane);
                const double *src = d < OC   ? Eb + (long long)k * (n * s) + d
                                    : d < OF ? cb + (long long)k * n + (d - OC)
                                    : d < OW ? Fb + (long long)k * FS + (d - OF)
                                    : d < OD ? Q.w + pb + (long long)k * s + (d - OW)
                                    : d < OZ ? Q.D + b * sh.ndD + (long long)k * NC * s + (d - OD)
                                    : d < OY ? Q.z + yb0 + (long long)k * NC + (d - OZ)
                                    : d < OLB ? Q.y + yb0 + (long long)k * NC + (d - OY)
                                    : d < OUB ? Q.lb + yb0 + (long long)k * NC + (d - OLB)
                                    : d < ORH ? Q.ub + yb0 + (long long)k * NC + (d - OUB)
                                    : d < OIR ? Q.rho + yb0 + (long long)k * NC + (d - ORH)
                                    : d < OH ? Q.irho + yb0 + (long long)k * NC + (d - OIR)
                                             : Q.hv + pb + (long long)k * s + (d - OH);
                dma16(src, &ring[slot][q * 128]);
            }
        }
    };
    double rp = 0.0, dwm = 0.0, zm = 0.0, rd = 0.0, dty = 0.0, act = 0.0;
    // the ADMM step of stage k from its ring record and this lane's w~_k[cl]
    auto upd = [&](const double *R, int k, double wt) {
        const double wo = R[OW + cl];
        const double wn = al * wt + bl * wo;
        const double d = R[OD + g + cl * NC];  // D_k[g][cl]
        const double v = sum_row16(d * wt), vw = sum_row16(d * wo);
        const double zr = R[OZ + g], yr = R[OY + g], rr = R[ORH + g], ir = R[OIR + g];
        const double vrel = al * v + bl * zr;
        const double zn = fmin(fmax(vrel + ir * yr, R[OLB + g]), R[OUB + g]);
        const double yn = yr + rr * (vrel - zn);
        const long long yo = yb0 + (long long)k * NC + g;
        if (cl == 0) gstore(Q.z + yo, zn);
        if (cl == 0) gstore(Q.y + yo, yn);
        if (FUSE && cl == 0) gstore(Q.gw + yo, zn - ir * yn);
        if (g == 0) gstore(Q.w + pb + (long long)k * s + cl, wn);
        if (FUSE && g == 0) gstore(Q.hw + pb + (long long)k * s + cl, R[OH + cl] - Q.sigma * wn);
        if (CHECK) {
            const double dwn = al * v + bl * vw;  // D w^{k+1}
            rp = fmax(rp, fabs(dwn - zn));
            dwm = fmax(dwm, fabs(dwn));
            zm = fmax(zm, fabs(zn));
            if (zn <= R[OLB + g] || zn >= R[OUB + g]) act = 1.0;
            // D^T rho (z+ - z) and D^T y+ of column cl, summed over the rows in
            // k_admm_update's order (row 0 first, one fma per row): the row
            // values come from their groups by readlane, D[r][cl] from the ring
            const double tz = rr * (zn - zr);
            double ad = 0.0, ay = 0.0;
#pragma unroll
            for (int r = 0; r < NC; ++r) {
                const double dr = R[OD + r + cl * NC];
                ad = __builtin_fma(dr, readlane_f64(tz, 16 * r), ad);
                ay = __builtin_fma(dr, readlane_f64(yn, 16 * r), ay);
            }
            rd = fmax(rd, fabs(ad));
            dty = fmax(dty, fabs(ay));
        }
    };

    // update_rhs_initial_stage accumulates: the solve sees the sum of the x0s
    double x0own = 0.0;
    if (lane < n) {
        x0own = x0[b * n + lane];
        const double xa = x0acc[b * n + lane] + x0own;
        x0acc[b * n + lane] = xa;
        sx[lane] = xa;
        sx0[lane] = x0own;
    }
#pragma unroll
    for (int j = 0; j < D - 1; ++j) dma(j < N ? j : N - 1, j);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();

    for (int k = 0; k < N; ++k) {
        const int kp = k + D - 1;
        dma(kp < N ? kp : N - 1, kp % D);
        if (k < D - 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NI + ST) * (D - 1)) : "memory");
        const double *R = ring[k % D];
        const double *F = R + OF;
        const int cm = cl < m ? cl : m - 1, cn = cl < n ? cl : n - 1;
        const double g0 = (g == 0) ? 1.0 : 0.0;
        double kx[NQ], ex[NQ], eu[m], xt[NQ];
        double pt[NQ];
        // (EH) E^ row cn: element 64 (cn >> 2) + 16 (cn & 3) + tile column
        const int eh = RS::OEH + 64 * (cn >> 2) + 16 * (cn & 3);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int t = 4 * q + g;
            kx[q] = F[RS::OK + cm * n + t];
            if constexpr (EH) {
                ex[q] = F[eh + m + t];
                pt[q] = 0.0;
            } else {
                ex[q] = R[OE + (m + t) * n + cn];
                pt[q] = F[RS::OPT + (t >= cn ? pidx(t, cn, n) : pidx(cn, t, n))];  // P~[4 q + g][cl]
            }
        }
#pragma unroll
        for (int i = 0; i < m; ++i) eu[i] = g0 * (EH ? F[eh + i] : R[OE + i * n + cn]);
        const double kq = F[RS::OKQ + cm];
        const double cc = EH ? F[RS::OCH + cn] : R[OC + cn];
        const double pv = EH ? 0.0 : F[RS::OPV + cn];
        // ---- chain ----
        const int lx = UPD ? (cl >= m ? cl - m : 0) : ((lane >= m && lane < s) ? lane - m : 0);
        const double xk = k == 0 ? sx0[lx] : sx[lx];  // ws[0]'s x part is the call's x0
#pragma unroll
        for (int q = 0; q < NQ; ++q) xt[q] = sx[4 * q + g];
        double v = 0.0, a = 0.0;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            v = __builtin_fma(kx[q], xt[q], v);
            a = __builtin_fma(ex[q], xt[q], a);
        }
        v = sum_groups(v) + kq;
        double myu = 0.0;
#pragma unroll
        for (int i = 0; i < m; ++i) {
            const double ui = readlane_f64(-v, i);  // u = -(k~ + K~ x)
            if (cl == i) myu = ui;
            a = __builtin_fma(eu[i], ui, a);
        }
        a = sum_groups(a) + cc;  // v = A x + B u + c (every group); EH: x+ = E^ [u; x] + c^
        if constexpr (UPD) upd(R, k, (cl < m) ? myu : xk);  // every group holds w~_k[cl]
        else if (lane < s) gstore(wb + (long long)k * s + lane, (lane < m) ? myu : xk);
        double xn = a;
        if constexpr (!EH) {
            // ---- lambda correction: x+ = v - rho_dyn (P~ (v - rho_dyn p) + p) ----
            if (g == 0 && cl < n) sz[cl] = __builtin_fma(-rho_dyn, pv, a);
            wave_sync();
            double y = 0.0;
#pragma unroll
            for (int q = 0; q < NQ; ++q) y = __builtin_fma(pt[q], sz[4 * q + g], y);
            y = sum_groups(y);
            xn = __builtin_fma(-rho_dyn, y + pv, a);
        }
        wave_sync();  // all reads of x_k done before it is overwritten
        if (g == 0 && cl < n) sx[cl] = xn;
        wave_sync();
    }
    if constexpr (UPD) {
        // terminal (no rows): w_N relaxed, h~_N = h_N - sigma w_N
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane < n) {
            const long long o = pb + (long long)N * s + lane;
            const double wn = al * sx[lane] + bl * Q.w[o];
            Q.w[o] = wn;
            if (FUSE) Q.hw[o] = Q.hv[o] - Q.sigma * wn;
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
        return;
    }
    if (lane < n) wb[(long long)N * s + lane] = sx[lane];
}


// ---------------------------------------------------------------------------
// Wide shapes (n + m <= 64, any per-stage constraint counts): the same
// elimination on one 256-thread block per problem with the matrices in LDS
// (blk_la.hpp).  Per stage k (value function (P, p) of stage k + 1):
//     P~ = (I + rho_dyn P)^{-1} P   (Neumann series / exact, as the 12/4 kernel),
//     G = P~ E~,  M = H~ + E~^T G + D^T rho D,
//     lp = h~ + G^T (c - rho_dyn p) + E~^T p - D^T rho g   (stage 0: D's u columns),
// then the m u-pivots of M (L-form record, as the serial solver's FR_k) leave
// P_k, p_k.  Record per stage: [L(:, 0:m) | lu' | p_{k+1} | P~_{k+1}] (fp64).
// LDS: XA (n x s: P, then G), XB (n x s: the Neumann term or chol(S)), Mb (s x s: E~,
// then M), Pt (n x n: P~), vectors.
// ---------------------------------------------------------------------------
namespace {
constexpr int KW_VL = 64;
}

__device__ __forceinline__ int kw_fs(int n, int m) { return (n + m) * m + m + n + n * n; }

static size_t kw_smem_bytes(int n, int s) { return (size_t)(2 * n * s + s * s + n * n + 8 * KW_VL) * sizeof(double); }

__global__ __launch_bounds__(256) void k_kkt_ric_bwd_wide(KKTRicArgs A) {
    extern __shared__ __attribute__((aligned(16))) double wbuf[];
    __shared__ int s_bad;
    __shared__ double s_red[4];
    const int tid = threadIdx.x;
    const long long b = blockIdx.x;
    const Shape &sh = A.sh;
    const int n = sh.n, m = sh.m, s = sh.s, N = sh.N, FS = kw_fs(n, m);
    const double *Eb = A.E + b * sh.perE;
    const double *cb = A.c + b * sh.perc;
    const double *Hb = A.Hw + b * sh.perHw;
    const double *hb = A.hw + b * sh.perh;
    const double *Db = A.D ? A.D + b * (long long)sh.ndD : nullptr;
    const double *gb = A.gw + b * (long long)sh.ny;
    const double *ib = A.irho ? A.irho + b * (long long)sh.ny : nullptr;
    double *RB = A.rec + b * (long long)N * FS;
    const double rd = A.rho_dyn;
    double *XA = wbuf, *XB = XA + n * s, *Mb = XB + n * s, *Pt = Mb + s * s, *vec = Pt + n * n;
    double *pv = vec, *cv = vec + KW_VL, *lp = vec + 2 * KW_VL, *t1 = vec + 3 * KW_VL, *rq = vec + 4 * KW_VL,
           *gq = vec + 5 * KW_VL;
    int fail_stage = -1;
    // ---- terminal: P_N = H~_N + D_N^T rho D_N, p_N = h~_N - D_N^T rho g_N ----
    {
        const int ncN = A.y_off[N + 1] - A.y_off[N];
        const double *DN = Db ? Db + A.d_off[N] : nullptr;
        const double *gN = gb + A.y_off[N], *iN = ib ? ib + A.y_off[N] : nullptr;
        if (tid == 0) s_bad = 0;
        for (int q = tid; q < ncN; q += BLK_THREADS) {
            rq[q] = 1.0 / iN[q];
            gq[q] = gN[q];
        }
        __syncthreads();
        const double *HN = Hb + (long long)N * sh.ps;
        for (int q = tid; q < n * n; q += BLK_THREADS) {
            const int i = q % n, j = q / n;
            double v = HN[i >= j ? pidx(i, j, n) : pidx(j, i, n)];
            for (int r = 0; r < ncN; ++r) v = __builtin_fma(DN[r + i * ncN] * rq[r], DN[r + j * ncN], v);
            XA[q] = v;
            if (i == j && psd_bad(v)) s_bad = 1;
        }
        for (int i = tid; i < n; i += BLK_THREADS) {
            double v = hb[(long long)N * s + i];
            for (int r = 0; r < ncN; ++r) v = __builtin_fma(-DN[r + i * ncN] * rq[r], gq[r], v);
            pv[i] = v;
        }
        __syncthreads();
        if (s_bad) fail_stage = N;
    }
    for (int k = N - 1; k >= 0; --k) {
        double *Rk = RB + (long long)k * FS;
        const int nck = A.y_off[k + 1] - A.y_off[k];
        const double *Dk = Db ? Db + A.d_off[k] : nullptr;
        // ---- P~ = (I + rho_dyn P)^{-1} P: the Neumann series while e = rho_dyn ||P||_F
        // <= PDPLQR_KKT_NEUMANN_MAX (terms while e^(j+1) > 1e-16), exact otherwise ----
        double f = 0.0;
        for (int q = tid; q < n * n; q += BLK_THREADS) f = __builtin_fma(XA[q], XA[q], f);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) f += __shfl_xor(f, o, 64);
        if ((tid & 63) == 0) s_red[tid >> 6] = f;
        __syncthreads();
        const double e = rd * sqrt((s_red[0] + s_red[1]) + (s_red[2] + s_red[3]));  // block-uniform
        bool pt_ok = true;
        if (e > PDPLQR_KKT_NEUMANN_MAX) {
            // S = I + rho_dyn P (XB), Cholesky carrying P (Pt): Pt = L^{-1} P, then L^T X = Pt
            for (int q = tid; q < n * n; q += BLK_THREADS) {
                const int i = q % n, j = q / n;
                Pt[q] = XA[q];
                XB[q] = __builtin_fma(rd, XA[q], i == j ? 1.0 : 0.0);
            }
            pt_ok = blk_chol(XB, n, n, n, t1, Pt, n, n);
            blk_trsm_lt(XB, n, n, Pt, n, n, nullptr);
            for (int q = tid; q < n * n; q += BLK_THREADS) {  // symmetrise (pairs i > j)
                const int i = q % n, j = q / n;
                if (i > j) {
                    const double v = 0.5 * (Pt[i + j * n] + Pt[j + i * n]);
                    Pt[i + j * n] = v;
                    Pt[j + i * n] = v;
                }
            }
            __syncthreads();
        } else {
            blk_copy(Pt, n, mv_n(XA, n), n, n);
            blk_copy(XB, n, mv_n(XA, n), n, n);
            double ej = e;
            for (int j = 0; j < 8 && ej > 1e-16; ++j) {  // block-uniform
                blk_mm(XB, n, mv_n(XA, n), mv_n(XB, n), n, n, n, -rd, 0.0, mv_none(), false);
                for (int q = tid; q < n * n; q += BLK_THREADS) Pt[q] += XB[q];
                ej *= e;
            }
        }
        // ---- record: p_{k+1}, P~_{k+1}; stage inputs ----
        for (int q = tid; q < n; q += BLK_THREADS) Rk[s * m + m + q] = pv[q];
        for (int q = tid; q < n * n; q += BLK_THREADS) Rk[s * m + m + n + q] = Pt[q];
        for (int q = tid; q < n; q += BLK_THREADS) {
            cv[q] = cb[(long long)k * n + q];
            t1[q] = __builtin_fma(-rd, pv[q], cb[(long long)k * n + q]);  // c - rho_dyn p
        }
        for (int q = tid; q < nck; q += BLK_THREADS) {
            rq[q] = 1.0 / ib[A.y_off[k] + q];
            gq[q] = gb[A.y_off[k] + q];
        }
        blk_copy(Mb, n, mv_n(Eb + (long long)k * n * s, n), n, s);  // E~
        blk_mm(XA, n, mv_n(Pt, n), mv_n(Mb, n), n, s, n, 1.0, 0.0, mv_none(), false);  // G = P~ E~
        // lp = h~ + G^T (c - rho_dyn p) + E~^T p - D^T rho g
        if (tid < s) {
            const int j = tid;
            double a = hb[(long long)k * s + j];
            for (int i = 0; i < n; ++i) {
                a = __builtin_fma(XA[i + j * n], t1[i], a);
                a = __builtin_fma(Mb[i + j * n], pv[i], a);
            }
            if (k > 0 || j < m)
                for (int r = 0; r < nck; ++r) a = __builtin_fma(-Dk[r + j * nck] * rq[r], gq[r], a);
            lp[j] = a;
        }
        // M = H~ + E~^T G (in place over E~), then + D^T rho D
        blk_mm(Mb, s, mv_t(Mb, n), mv_n(XA, n), s, s, n, 1.0, 0.0, mv_pk(Hb + (long long)k * sh.ps, s), true);
        if (nck > 0) {
            for (int q = tid; q < s * s; q += BLK_THREADS) {
                const int i = q % s, j = q / s;
                if (i < j || (k == 0 && i >= m)) continue;  // lower; stage 0: u columns only
                double v = Mb[q];
                for (int r = 0; r < nck; ++r) v = __builtin_fma(Dk[r + i * nck] * rq[r], Dk[r + j * nck], v);
                Mb[q] = v;
            }
            __syncthreads();
        }
        // ---- the m u-pivots (one barrier per pivot), L-form record ----
        bool ok = true;
        if (tid == 0) s_bad = 0;
        const int i = tid & 63, cg = tid >> 6;  // row, column group (s <= 64; k_seg_bwd_wide's scheme)
        for (int j = 0; j < m;) {
            if (j + 1 < m) {  // two pivots per barrier (lds_axpy2_strided: the two steps' fmas, in order)
                const double d0 = Mb[j + j * s], a1j = Mb[(j + 1) + j * s];
                const double inv0 = 1.0 / d0, invs0 = rsqrt_f64(d0);
                const double d1 = __builtin_fma(-(a1j * inv0), a1j, Mb[(j + 1) + (j + 1) * s]);
                ok = ok && d0 > 0.0 && d1 > 0.0;
                const double inv1 = 1.0 / d1, invs1 = rsqrt_f64(d1);
                const double lpj = lp[j], lp1 = __builtin_fma(-(a1j * inv0), lpj, lp[j + 1]);
                if (tid < s) {
                    const double c0 = Mb[tid + j * s];
                    Rk[j * s + tid] = tid >= j ? c0 * invs0 : 0.0;
                    const double a1 = __builtin_fma(-(c0 * inv0), a1j, Mb[tid + (j + 1) * s]);
                    Rk[(j + 1) * s + tid] = tid >= j + 1 ? a1 * invs1 : 0.0;
                }
                if (tid == 255) {
                    Rk[s * m + j] = lpj * invs0;
                    Rk[s * m + j + 1] = lp1 * invs1;
                }
                if (i >= j + 2 && i < s) {
                    const double f0 = Mb[i + j * s] * inv0;
                    const double f1 = __builtin_fma(-f0, a1j, Mb[i + (j + 1) * s]) * inv1;
                    lds_axpy2_strided(Mb + i, s, Mb + j * s, Mb + (j + 1) * s, f0, f1, inv0, a1j, j + 2 + cg, i, 4);
                    if (cg == 0) lp[i] = __builtin_fma(-f1, lp1, __builtin_fma(-f0, lpj, lp[i]));
                }
                __syncthreads();
                j += 2;
                continue;
            }
            const double d = Mb[j + j * s];
            ok = ok && d > 0.0;
            const double inv2 = 1.0 / d, invs = rsqrt_f64(d);
            const double lpj = lp[j];
            if (tid < s) Rk[j * s + tid] = tid >= j ? Mb[tid + j * s] * invs : 0.0;
            if (tid == 255) Rk[s * m + j] = lpj * invs;
            if (i > j && i < s) {
                const double lij = Mb[i + j * s] * inv2;
                lds_axpy_strided(Mb + i, s, Mb + j * s, lij, j + 1 + cg, i, 4);
                if (cg == 0) lp[i] = __builtin_fma(-lij, lpj, lp[i]);
            }
            __syncthreads();
            ++j;
        }
        // ---- P_k, p_k ----
        for (int q = tid; q < n * n; q += BLK_THREADS) {
            const int i = q % n, j = q / n;
            const int hi = i > j ? i : j, lo = i > j ? j : i;
            const double v = Mb[(m + hi) + (m + lo) * s];
            XA[q] = v;
            if (i == j && psd_bad(v)) s_bad = 1;
        }
        for (int q = tid; q < n; q += BLK_THREADS) pv[q] = lp[m + q];
        __syncthreads();
        if ((!ok || !pt_ok || s_bad) && fail_stage < 0) fail_stage = k;
    }
    if (tid == 0) A.status[b] = fail_stage < 0 ? 0 : fail_stage + 1;
}

// forward: the L-form rollout (k_riccati_fwd_big) plus the lambda correction
// x+ = v - rho_dyn (P~ (v - rho_dyn p) + p), v = A x + B u + c; one wave per problem
__global__ __launch_bounds__(64) void k_kkt_ric_fwd_wide(Shape sh, const double *__restrict__ E,
                                                        const double *__restrict__ c, const double *__restrict__ RB,
                                                        const double *__restrict__ x0, double *__restrict__ x0acc,
                                                        double *__restrict__ ws, double rho_dyn) {
    __shared__ double w[64], sz[64], sx0[64];
    const int lane = wave_lane();
    const long long b = blockIdx.x;
    const int n = sh.n, m = sh.m, N = sh.N, s = sh.s, FS = kw_fs(n, m);
    const double *Eb = E + b * sh.perE;
    const double *cb = c + b * sh.perc;
    const double *Rb = RB + b * (long long)N * FS;
    double *wb = ws + b * sh.perh;
    if (lane < n) {  // update_rhs_initial_stage accumulates: the solve sees the sum of the x0s
        const double x = x0[b * n + lane];
        const double xa = x0acc[b * n + lane] + x;
        x0acc[b * n + lane] = xa;
        w[m + lane] = xa;
        sx0[lane] = x;
    }
    wave_sync();
    for (int k = 0; k < N; ++k) {
        const double *Fk = Rb + (long long)k * FS;
        double v = 0.0;
        if (lane < m) {
            double a = Fk[(long long)s * m + lane];
            for (int i = 0; i < n; ++i) a = __builtin_fma(Fk[(long long)lane * s + m + i], w[m + i], a);
            v = -a;
        }
        for (int j = m - 1; j >= 0; --j) {
            const double uj = readlane_f64(v, j) / Fk[(long long)j * s + j];
            if (lane == j) v = uj;
            else if (lane < j) v = __builtin_fma(-Fk[(long long)lane * s + j], uj, v);
        }
        if (lane < m) w[lane] = v;
        wave_sync();
        if (lane < s) wb[(long long)k * s + lane] = lane < m ? v : (k == 0 ? sx0[lane - m] : w[lane]);
        const double *pk = Fk + s * m + m, *Ptk = pk + n;
        double a = 0.0;
        if (lane < n) {
            const double *Ek = Eb + (long long)k * n * s;
            a = cb[(long long)k * n + lane];
            for (int j = 0; j < s; ++j) a = __builtin_fma(Ek[lane + (long long)j * n], w[j], a);
            sz[lane] = __builtin_fma(-rho_dyn, pk[lane], a);  // v - rho_dyn p
        }
        wave_sync();
        if (lane < n) {
            double y = 0.0;
            for (int t = 0; t < n; ++t) y = __builtin_fma(Ptk[lane + t * n], sz[t], y);
            a = __builtin_fma(-rho_dyn, y + pk[lane], a);
        }
        wave_sync();
        if (lane < n) w[m + lane] = a;
        wave_sync();
    }
    if (lane < n) wb[(long long)N * s + lane] = w[m + lane];
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static bool kric_al(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// The Riccati-ordered KKT path applies: 12/4, the same row count nc in {0, 4}
// on every stage k < N (nc_N <= 4), 16-byte aligned per-problem blocks; the
// LDS kernels where the block LDL^T tiles do not fit (n + m or n + nc_k > 32,
// ldl_fits false) up to n + m <= 64, any ncs.
int kkt_ric_nc(const Shape &sh, const std::vector<int32_t> &ncs, bool ldl_fits) {
    if (xl_shape(sh)) {
        for (int k = 0; k <= sh.N; ++k)
            if (ncs[k] > 256) return -1;  // the per-stage rho / g slots of k_kkt_ric_bwd_xl
        return KKT_RIC_XL;
    }
    if (!ldl_fits && sh.s <= 64) {
        for (int k = 0; k <= sh.N; ++k)
            if (ncs[k] > 64) return -1;  // the per-stage rho / g slots of k_kkt_ric_bwd_wide
        return KKT_RIC_WIDE;
    }
    if (sh.n != 12 || sh.m != 4 || getenv("PDPLQR_KKT_LDL")) return -1;
    const int nc = ncs[0];
    if (nc != 0 && nc != 4) return -1;
    for (int k = 0; k < sh.N; ++k)
        if (ncs[k] != nc) return -1;
    if (ncs[sh.N] > 4) return -1;
    if (sh.perE % 2 || sh.perc % 2 || sh.perHw % 2 || sh.perh % 2 || (nc && (sh.ny % 2 || sh.ndD % 2))) return -1;
    return nc;
}

size_t kkt_ric_rec_doubles(const Shape &sh, int ric) {
    if (ric == KKT_RIC_WIDE || ric == KKT_RIC_XL) return (size_t)sh.N * ((size_t)sh.s * sh.m + sh.m + sh.n + (size_t)sh.n * sh.n);
    return (size_t)sh.N * KRecShape<12, 4>::FS;
}

int launch_kkt_ric_backward(const Shape &sh, int nc, const double *E, const double *c, const double *D,
                            const double *Hw, const double *hw, const double *gw, const double *irho,
                            const int32_t *d_off, const int32_t *y_off, int nc_last, double rho_dyn, double *rec,
                            int32_t *status, hipStream_t st, double *cache) {
    if (nc == KKT_RIC_XL)
        return launch_kkt_xl_backward(sh, E, c, D, Hw, hw, gw, irho, d_off, y_off, rho_dyn, rec, status, cache, st);
    if (nc == KKT_RIC_WIDE) {
        KKTRicArgs a;
        a.sh = sh;
        a.E = E;
        a.c = c;
        a.D = sh.ndD > 0 ? D : nullptr;
        a.Hw = Hw;
        a.hw = hw;
        a.gw = gw;
        a.irho = sh.ny > 0 ? irho : nullptr;
        a.d_off = d_off;
        a.y_off = y_off;
        a.rec = rec;
        a.status = status;
        a.rho_dyn = rho_dyn;
        a.nc_last = nc_last;
        const size_t sm = kw_smem_bytes(sh.n, sh.s);
        if (hipFuncSetAttribute(reinterpret_cast<const void *>(&k_kkt_ric_bwd_wide),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm) != hipSuccess) {
            set_error("KKT backward (wide): LDS request too large");
            return PDPLQR_ERR_HIP;
        }
        hipLaunchKernelGGL(k_kkt_ric_bwd_wide, dim3((unsigned)sh.batch), dim3(256), sm, st, a);
        PDPLQR_HIP_TRY(hipGetLastError());
        return PDPLQR_OK;
    }
    if (!kric_al(E) || !kric_al(c) || !kric_al(Hw) || !kric_al(hw) || (nc && (!kric_al(D) || !kric_al(gw) || !kric_al(irho))))
        return PDPLQR_ERR_UNSUPPORTED;
    KKTRicArgs a;
    a.sh = sh;
    a.E = E;
    a.c = c;
    a.D = D;
    a.Hw = Hw;
    a.hw = hw;
    a.gw = gw;
    a.irho = irho;
    a.d_off = d_off;
    a.y_off = y_off;
    a.rec = rec;
    a.status = status;
    a.rho_dyn = rho_dyn;
    a.nc_last = nc_last;
    a.cache = cache;
    with_x1(sh.x1, [&](auto x1) {
        constexpr bool X = decltype(x1)::value;
        if (nc == 4) hipLaunchKernelGGL((k_kkt_ric_bwd<4, X>), dim3((unsigned)sh.batch), dim3(64), 0, st, a);
        else hipLaunchKernelGGL((k_kkt_ric_bwd<0, X>), dim3((unsigned)sh.batch), dim3(64), 0, st, a);
    });
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

bool kkt_ric_rec_ehat(int ric) { return ric == 0 || ric == 4; }

size_t kkt_ric_cache_doubles(const Shape &sh, int ric) {
    return ric == 0 || ric == 4 ? (size_t)sh.N * KKT_CF : 0;
}

int launch_kkt_ric_nofact(const Shape &sh, int nc, const double *D, const double *hw, const double *gw,
                          const double *irho, const int32_t *d_off, const int32_t *y_off, int nc_last, double rho_dyn,
                          const double *cache, double *rec, hipStream_t st) {
    if (nc != 0 && nc != 4) return PDPLQR_ERR_UNSUPPORTED;
    KKTRicArgs a;
    a.sh = sh;
    a.E = a.c = a.Hw = nullptr;
    a.D = D;
    a.hw = hw;
    a.gw = gw;
    a.irho = irho;
    a.d_off = d_off;
    a.y_off = y_off;
    a.rec = rec;
    a.cache = const_cast<double *>(cache);
    a.status = nullptr;
    a.rho_dyn = rho_dyn;  // (the E^ record's c^ = M^ c - rho_dyn M^ p)
    a.nc_last = nc_last;
    with_x1(sh.x1, [&](auto x1) {
        constexpr bool X = decltype(x1)::value;
        if (nc == 4) hipLaunchKernelGGL((k_kkt_ric_nofact<4, X>), dim3((unsigned)sh.batch), dim3(64), 0, st, a);
        else hipLaunchKernelGGL((k_kkt_ric_nofact<0, X>), dim3((unsigned)sh.batch), dim3(64), 0, st, a);
    });
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

int launch_kkt_ric_forward(const Shape &sh, const double *E, const double *c, const double *rec, const double *x0,
                           double *x0acc, double *ws, double rho_dyn, hipStream_t st, int ric, bool ehat) {
    if (ric == KKT_RIC_XL) return launch_kkt_xl_forward(sh, E, c, rec, x0, x0acc, ws, rho_dyn, st);
    if (ric == KKT_RIC_WIDE) {
        hipLaunchKernelGGL(k_kkt_ric_fwd_wide, dim3((unsigned)sh.batch), dim3(64), 0, st, sh, E, c, rec, x0, x0acc,
                           ws, rho_dyn);
        PDPLQR_HIP_TRY(hipGetLastError());
        return PDPLQR_OK;
    }
    with_x1(sh.x1, [&](auto x1) {
        constexpr bool X = decltype(x1)::value;
        if (ehat)
            hipLaunchKernelGGL((k_kkt_ric_fwd<4, false, false, false, true, X>),
                               dim3((unsigned)sh.batch), dim3(64), 0, st, sh, E, c, rec, x0, x0acc, ws, rho_dyn,
                               AdmmArgs{});
        else
            hipLaunchKernelGGL((k_kkt_ric_fwd<4, false, false, false, false, X>), dim3((unsigned)sh.batch), dim3(64),
                               0, st, sh, E, c, rec, x0, x0acc, ws, rho_dyn, AdmmArgs{});
    });
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

// The KKT rollout with the ADMM update of the iteration in the same pass
// (admm.hip; C5 layout: 12/4, 4 rows on every stage k < N, none at N).
int launch_kkt_ric_forward_admm(const Shape &sh, const double *E, const double *c, const double *rec,
                                const double *x0, double *x0acc, double rho_dyn, const AdmmArgs &q, bool fuse,
                                bool check, hipStream_t st) {
    auto al = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    if (getenv("PDPLQR_NO_ADMM_FUSE") || sh.n != 12 || sh.m != 4 || q.uni != 4 || !q.no_penalty ||
        sh.ny != 4 * sh.N || !al(E) || !al(c) || !al(rec) || !al(q.w) || !al(q.D) || !al(q.z) || !al(q.y) ||
        !al(q.lb) || !al(q.ub) || !al(q.rho) || !al(q.irho) || !al(q.hv) || sh.perE % 2 || sh.perc % 2 ||
        sh.perh % 2 || sh.ndD % 2 || sh.ny % 2)
        return PDPLQR_ERR_UNSUPPORTED;
    const dim3 grid((unsigned)sh.batch), blk(64);
    with_x1(sh.x1, [&](auto x1) {
        constexpr bool X = decltype(x1)::value;
        constexpr int RG = PDPLQR_KKT_UPD_RING;
        double *const nows = nullptr;
        if (fuse && check)
            hipLaunchKernelGGL((k_kkt_ric_fwd<RG, true, true, true, false, X>), grid, blk, 0, st, sh, E, c, rec, x0,
                               x0acc, nows, rho_dyn, q);
        else if (fuse)
            hipLaunchKernelGGL((k_kkt_ric_fwd<RG, true, true, false, false, X>), grid, blk, 0, st, sh, E, c, rec, x0,
                               x0acc, nows, rho_dyn, q);
        else if (check)
            hipLaunchKernelGGL((k_kkt_ric_fwd<RG, true, false, true, false, X>), grid, blk, 0, st, sh, E, c, rec, x0,
                               x0acc, nows, rho_dyn, q);
        else
            hipLaunchKernelGGL((k_kkt_ric_fwd<RG, true, false, false, false, X>), grid, blk, 0, st, sh, E, c, rec, x0,
                               x0acc, nows, rho_dyn, q);
    });
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

}  // namespace pdplqr
