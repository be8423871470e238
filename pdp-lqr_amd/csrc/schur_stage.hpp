// schur_stage.hpp -- one value-form Riccati stage on a 16-wide MFMA tile (one
// wavefront per problem), shared by the batched backward (kernels_schur.hip)
// and the Riccati-ordered KKT solve (kkt_riccati.hip).  See kernels_schur.hip
// for the derivation (lqr_kernel.hpp:104-147 in value-matrix form).
#pragma once
#include <type_traits>

#include "combine_tiles.hpp"
#include "device_common.hpp"

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
// Branch-free: addresses are clamped into the record and the values masked
// (a guarded LDS read compiles to an exec-mask region per element).
// `lde` is E's column stride (n in HBM; padded in the LDS copy, see SchurShape).
__device__ __forceinline__ void schur_load(SchurIn &in, const double *__restrict__ Ek, const double *__restrict__ ck,
                                           const double *__restrict__ Hk, const double *__restrict__ hk, int n,
                                           int m, int s, int g, int c, int lde) {
    const int cc = c < s ? c : s - 1;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
        const int t = 4 * kk + g - m;
        const bool xr = t >= 0 && t < n;
        const int tc = t < 0 ? 0 : (t < n ? t : n - 1);
        const double e = Ek[tc + cc * lde], cv = ck[tc];
        in.E[kk] = (xr && c < s) ? e : 0.0;
        in.ct[kk] = xr ? cv : 0.0;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = 4 * r + g;
        const int ic = i < s ? i : s - 1;
        const double v = Hk[ic >= cc ? pidx(ic, cc, s) : pidx(cc, ic, s)];
        in.H[r] = (i < s && c < s) ? v : (i == c ? 1.0 : 0.0);
    }
    const double hv = hk[cc];
    in.h = (c < s) ? hv : 0.0;
}

// P's transpose in LDS at leading dimension 17.  (A bank-conflict-free layout
// -- stride 18, E at stride 14 -- cut SQ_LDS_BANK_CONFLICT 149 -> 130 M cycles
// per launch but not the time, 3.13 -> 3.14 ms: the conflicts sit on the LDS
// pipe beside the VALU / MFMA chain; docs/DESIGN_HISTORY.md, round 2.)
#define PDPLQR_TP_LD 17

struct SchurSmem {
    alignas(16) double col[64];  // pivot-row broadcast, one slot per row group (colpos order)
    alignas(16) double lpt[16];  // lp_k, column -> row redistribution (colpos order)
    double inv[16];              // 1 / sqrt(pivot), u columns
    double luq[16];              // lu' = Luu^{-1} lu
    alignas(16) double lu4[4];   // (unused slot; keeps the record staging 16-byte aligned)
    union {
        double tp[16 * PDPLQR_TP_LD];  // transpose of P_k (leading dimension: see PDPLQR_TP_LD)
        alignas(16) double rec[128];  // rollout record staging (one coalesced store per stage)
    };
};


// PDPLQR_SCHUR_SUBST: W, lu' and the gain record by forward / back
// substitution with Luu (no explicit T = Luu^{-1}, 16 fewer uniform VALU a
// stage); PDPLQR_SCHUR_DPP: per-row-group picks and the column-0 merge as
// masked DPP moves (row_mask / bank_mask) instead of v_cndmask pairs (m = 4)
// (default on: same-box A/B r4f, headline backward 3.22 -> 2.96 ms with LPW,
// C5 KKT 1.297 -> 1.260 ms, C5 Riccati 0.913 -> 0.872 ms)

// G = P E~ and M = H~ + E~^T G as independent per-chunk MFMAs summed by VALU
// (compile-time m = 4) instead of one accumulation chain (A/B: schur_stage)

// Compile-time m <= 4: the m u-pivots as ONE block step.  Every u row sits in
// register 0 (row j = row group j), so
//   * Muu (m x m) and lu come to every lane by v_readlane; Luu = chol(Muu),
//     T = Luu^{-1} and lu' = T lu are computed wave-uniformly (no broadcast
//     chain per pivot);
//   * lane (g, c) forms W[c][g] = sum_l M[c][l] T[g][l] = L(c, g) -- the u
//     columns of the factor (Lxu below, Luu on the u rows) -- from column c of
//     the u rows (register 0 of groups l, gathered by permlane swaps);
//   * that one value per lane is both MFMA operands of P_k = Mxx - W W^T and
//     the A operand of lp_x -= W lu' (one 16x16x4 MFMA each).
// The u block of the tile is left as Muu - Luu Luu^T (~0); only the x block
// and the x rows of lp are read by the next stage.
// PDPLQR_SCHUR_T4 = 1 forms W with one MFMA (t4_apply, as the blocked
// Cholesky does): 32 fewer VALU and 18 fewer cross-lane ops per loop trip, but
// the MFMA sits on the stage chain; same-box A/B (scripts/gpu_r2k.sh) 3.11 ->
// 3.13 ms per backward, so it stays off.

// Gain-form rollout record (GAIN, 12/4 value-form path): the forward needs
// u = -Luu^{-T}(lu' + Lxu^T x) = -(k~ + K~ x) with K~ = T^T Lxu^T (m x n) and
// k~ = T^T lu' (T = Luu^{-1}): 52 instead of 68 doubles per stage, and the
// forward loses its back substitution.  Off the P chain: every lane already
// holds its whole row W[c][0..m) of the u columns.
struct GainOut {
    double kt;  // lane (g, c): K~[g][c - m] on x rows c >= m
    double kq;  // k~[g] (every lane of group g)
    double T[4][4];  // Luu^{-1} (wave-uniform; read by the KKT factor cache only)
};

// PDPLQR_SCHUR_LDSU = 1: the u rows reach the lanes through LDS instead of
// v_readlane / permlane broadcasts -- one ds_write and 12 ds_read_b128 (LDS
// pipe) for 14 f64 readlanes and 4 row-group broadcasts (44 VALU).

// LPW (the batched backward's gain path; PDPLQR_SCHUR_LPW): lu rides in W.
// Column 0 of the u rows is replaced by lu before the u-row columns are
// gathered, so lane (g, 0) forms W_0 = Luu^{-1} lu = lu' and its gain column
// Luu^{-T} lu' = k~: the MFMA's B operand is w on every lane (its column 0 is
// lu', as LP_IN_P wants), k~ needs no uniform pass and no lane pick, and lu is
// never read to the scalar side.  Row 0 of the product (u row) is dead.
template <int MM, bool GAIN = false, bool LPW = false>
__device__ __forceinline__ bool schur_block_pivots(d4 &M, double (&lpr)[4], double &w, double (&luq)[4], int g,
                                                   int c, GainOut *go = nullptr, double *ldsu = nullptr,
                                                   double *ldsl = nullptr) {
    static_assert(MM >= 1 && MM <= 4, "u block");
    static_assert(!LPW || (GAIN && MM == 4), "lu in W: 12/4 gain path");
    double a[4][4], lu[4], L[4][4], T[4][4], inv[4];
    bool ok = true;
    {
#pragma unroll
        for (int i = 0; i < MM; ++i) {
            lu[i] = readlane_f64(lpr[0], 16 * i);
#pragma unroll
            for (int j = 0; j <= i; ++j) a[i][j] = readlane_f64(M[0], 16 * i + j);  // M[i][j]: group i, lane j
        }
    }
#pragma unroll
    for (int j = 0; j < MM; ++j) {  // right-looking Cholesky of Muu (uniform values)
        ok = ok && (a[j][j] > 0.0);
        inv[j] = rsqrt_f64(a[j][j]);
        L[j][j] = a[j][j] * inv[j];
#pragma unroll
        for (int i = j + 1; i < MM; ++i) L[i][j] = a[i][j] * inv[j];
#pragma unroll
        for (int i = j + 1; i < MM; ++i)
#pragma unroll
            for (int k = j + 1; k <= i; ++k) a[i][k] = __builtin_fma(-L[i][j], L[k][j], a[i][k]);
    }
#pragma unroll
    for (int i = 0; i < MM; ++i) {  // T = Luu^{-1} (lower), row by row
        T[i][i] = inv[i];
#pragma unroll
        for (int j = 0; j < i; ++j) {
            double v = 0.0;
#pragma unroll
            for (int k = j; k < i; ++k) v = __builtin_fma(L[i][k], T[k][j], v);
            T[i][j] = -v * inv[i];
        }
    }
#pragma unroll
    for (int i = 0; i < MM; ++i) {  // lu' = Luu^{-1} lu (forward substitution)
        double v = lu[i];
#pragma unroll
        for (int j = 0; j < i; ++j) v = __builtin_fma(-L[i][j], luq[j], v);
        luq[i] = v * inv[i];
    }
    // column c of the u rows: m_l = M[l][c] (group l, register 0)
    if constexpr (LPW) M[0] = (c == 0) ? lpr[0] : M[0];  // the readlanes above took Muu first
    double ml[4];
#pragma unroll
        for (int l = 0; l < MM; ++l) ml[l] = bcast_group(M[0], l);
    w = 0.0;
    double Wc[4];  // W[c][j], j < m: this lane's row of the u columns
#pragma unroll
    for (int j = 0; j < MM; ++j) {  // W_c = Luu^{-1} m_c (forward substitution, no T)
        double v = ml[j];
#pragma unroll
        for (int l = 0; l < j; ++l) v = __builtin_fma(-L[j][l], Wc[l], v);
        Wc[j] = v * inv[j];
    }
#pragma unroll
    for (int j = 0; j < MM; ++j) w = (g == j) ? Wc[j] : w;  // W[c][g]; groups g >= m keep 0
    if constexpr (GAIN) {  // K~[i][c] = sum_{l >= i} T[l][i] W[c][l], k~[i] = sum_{l >= i} T[l][i] lu'[l]
        double ka[4] = {0.0, 0.0, 0.0, 0.0}, kb[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int i = MM - 1; i >= 0; --i) {  // Luu^{-T} W_c, Luu^{-T} lu' (back substitution)
            double a = Wc[i], q = luq[i];
#pragma unroll
            for (int l = i + 1; l < MM; ++l) {
                a = __builtin_fma(-L[l][i], ka[l], a);
                q = __builtin_fma(-L[l][i], kb[l], q);
            }
            ka[i] = a * inv[i];
            kb[i] = q * inv[i];
        }
        double kt = 0.0, kq = 0.0;
        if constexpr (LPW) {
            // lane (g, 0) holds k~[g]; lanes (g, 1..3) take it (DPP quad_perm
            // [0,0,0,0] on bank 0 of every row) so the record store's four
            // k~ writers carry equal values
            kt = pick_group(ka);
            const int lo = __builtin_amdgcn_update_dpp(__double2loint(kt), __double2loint(kt), 0x00, 0xF, 0x1, false);
            const int hi = __builtin_amdgcn_update_dpp(__double2hiint(kt), __double2hiint(kt), 0x00, 0xF, 0x1, false);
            kt = __hiloint2double(hi, lo);
            kq = kt;
        } else {
#pragma unroll
            for (int i = 0; i < MM; ++i) {
                kt = (g == i) ? ka[i] : kt;
                kq = (g == i) ? kb[i] : kq;
            }
        }
        go->kt = kt;
        go->kq = kq;
#pragma unroll
        for (int i = 0; i < MM; ++i)
#pragma unroll
            for (int j = 0; j <= i; ++j) go->T[i][j] = T[i][j];
    }
    // lp -= W lu' rides in the same MFMA: column 0 of M (u column 0: dead
    // after this stage -- the next stage reads P's x rows through the x
    // K-chunks only, and G's u rows are never used) carries lp in, the B
    // operand's column 0 carries lu', so D[:, 0] = lp - W lu'; then the
    // column-0 result to every lane of its row (DPP row_newbcast:0)
    if constexpr (LPW) {
#pragma unroll
        for (int r = 1; r < 4; ++r) M[r] = (c == 0) ? lpr[r] : M[r];
        M = mfma_f64(-w, w, M);  // M - W W^T; column 0: lp - W lu' (lane (g, 0): w = lu'[g])
    } else {
        const double lq = (g < MM) ? luq[g < MM ? g : 0] : 0.0;
#pragma unroll
        for (int r = 0; r < 4; ++r) M[r] = (c == 0) ? lpr[r] : M[r];
        M = mfma_f64(-w, (c == 0) ? lq : w, M);  // M - W W^T; column 0: lp - W lu'
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) lpr[r] = bcast_lane16(M[r], 0);
    return ok;
}

// One stage.  Pm: in = tile whose trailing (x) block is P_{k+1}; out = M_k
// after the m u-pivots (trailing block P_k, u columns unscaled L).  prow:
// p~ in row layout (prow[r] = p[4 r + g - m] on x rows).
template <int MM, bool SYM = true, bool GAIN = false, bool LPW = false, int SPLIT = 0>
__device__ __forceinline__ bool schur_stage(d4 &Pm, double (&prow)[4], const SchurIn &in, SchurSmem &sm, int m,
                                            int s, int g, int c, double &w, double (&luq)[4], bool sym_rt = true,
                                            GainOut *go = nullptr) {
    const int k0 = m >> 2, k1 = (s - 1) >> 2;  // K chunks that hold x rows
    d4 G = {0.0, 0.0, 0.0, 0.0};
    d4 Mn = in.H;
    if constexpr (SPLIT && MM == 4) {
        // the three x chunks (kk = 1..3 at m = 4, s = 16) on independent
        // accumulators, summed by VALU: a dependent f64 MFMA waits ~186 cycles
        // for its predecessor, three independent ones issue back to back
        // (scripts/ubench/lat_bench.hip), so each product leaves the stage
        // chain ~250 cycles earlier for 8 v_add_f64 (the headline instance, at
        // 4 waves per SIMD within 128 VGPRs, keeps the single chain: SPLIT = 0)
        const d4 z = {0.0, 0.0, 0.0, 0.0};
        const d4 g1 = mfma_f64(Pm[1], in.E[1], z), g2 = mfma_f64(Pm[2], in.E[2], z),
                 g3 = mfma_f64(Pm[3], in.E[3], z);
        G = (g1 + g2) + g3;
        const d4 m1 = mfma_f64(in.E[1], G[1], in.H), m2 = mfma_f64(in.E[2], G[2], z),
                 m3 = mfma_f64(in.E[3], G[3], z);
        Mn = (m1 + m2) + m3;
    } else {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
            if (kk >= k0 && kk <= k1) G = mfma_f64(Pm[kk], in.E[kk], G);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
            if (kk >= k0 && kk <= k1) Mn = mfma_f64(in.E[kk], G[kk], Mn);
    }
    double part = 0.0;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
        if (kk >= k0 && kk <= k1) {
            part = __builtin_fma(G[kk], in.ct[kk], part);
            part = __builtin_fma(in.E[kk], prow[kk], part);
        }
    part = sum_groups(part);
    sm.lpt[colpos<1>(c)] = in.h + part;  // every group holds the same sum
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
    bool ok;
    if constexpr (MM > 0) {
        ok = schur_block_pivots<MM, GAIN, LPW>(Mn, lpr[0], w, luq, g, c, go, sm.col, sm.lu4);
        Pm = Mn;
    } else {
        d4 Mt[1][1];
        Mt[0][0] = Mn;
        ok = chol_tiles<1>(Mt, lpr, sm.col, sm.inv, sm.luq, 0, m, m, true, g, c);
        Pm = Mt[0][0];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) prow[r] = lpr[0][r];
    // P_k <- (P_k + P_k^T) / 2.  The square-root recursion is symmetric by
    // construction; here the rounding-level antisymmetric part of M_k would
    // otherwise be carried as A^T e A from stage to stage and grow with the
    // open-loop dynamics (the next stage reads P's registers as P^T).  It
    // grows by ~||A||^2 per stage, so resetting it every few stages (SYM on a
    // subset of the stages, PDPLQR_SYM_EVERY) keeps it at rounding level while
    // the LDS round trip leaves the other stages' chains.
    if (SYM && sym_rt) {  // wave-uniform
#pragma unroll
        for (int r = 0; r < 4; ++r) sm.tp[(4 * r + g) * PDPLQR_TP_LD + c] = Pm[r];
        wave_sync();
#pragma unroll
        for (int r = 0; r < 4; ++r) Pm[r] = 0.5 * (Pm[r] + sm.tp[c * PDPLQR_TP_LD + 4 * r + g]);
    }
    // P_k = Lxx Lxx^T: semidefinite (psd_bad: non-finite or clearly negative diagonal)
    bool bad = false;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = 4 * r + g;
        if (i == c && i >= m && i < s && psd_bad(Pm[r])) bad = true;
    }
    return (int)ok & (int)!__any(bad);  // no short-circuit: no branch
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

// Gain-form record [K~ (m x n, row-major) | k~] in ONE store: lane (g, c >= M)
// writes K~[g][c - M], lanes (g, c < M) write k~[g] (three of them a duplicate
// of the same value to the same address).
template <int M, int S>
__device__ __forceinline__ void schur_store_record_gain(double *FRk, const GainOut &go, int g, int c) {
    static_assert(M == 4 && S == 16, "one K~ row per row group");
    constexpr int NX = S - M;
    gstore(FRk + (c >= M ? g * NX + (c - M) : M * NX + g), c >= M ? go.kt : go.kq);
}


}  // namespace pdplqr
