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

// LDS layouts chosen by the bank rule of ds_read_b64 (32-lane halves, bank =
// double index mod 32; MI355X_MICROARCH.md section LDS): PDPLQR_LDS_PAD = 1
//   * P's transpose with leading dimension 18 (2 x odd): the read c * 18 + 4 r + g
//     of a half (g in {0,1} or {2,3}, c = 0..15) hits 32 distinct banks
//     (stride 17 puts (c = 15, g = 1) on (c = 0, g = 0): 2-way);
//   * E's columns in the staged record at stride 14 instead of 12 (below);
//   * lp_k written by row group 0 only.
// Measured (profiles/r02, same box, interleaved): SQ_LDS_BANK_CONFLICT
// 149 -> 130 M cycles per launch, backward 3.13 -> 3.14 ms (no gain: the
// conflicts sit on the LDS pipe beside the VALU / MFMA chain), so it is off.
#ifndef PDPLQR_LDS_PAD
#define PDPLQR_LDS_PAD 0
#endif
#define PDPLQR_TP_LD (PDPLQR_LDS_PAD ? 18 : 17)

struct SchurSmem {
    alignas(16) double col[64];  // pivot-row broadcast, one slot per row group (colpos order)
    alignas(16) double lpt[16];  // lp_k, column -> row redistribution (colpos order)
    double inv[16];              // 1 / sqrt(pivot), u columns
    double luq[16];              // lu' = Luu^{-1} lu
    alignas(16) double lu4[4];   // lu of the u rows (PDPLQR_SCHUR_LDSU)
    union {
        double tp[16 * PDPLQR_TP_LD];  // transpose of P_k (leading dimension: see PDPLQR_TP_LD)
        alignas(16) double rec[128];  // rollout record staging (one coalesced store per stage)
    };
};

#ifndef PDPLQR_LP_IN_P
#define PDPLQR_LP_IN_P 1
#endif

// PDPLQR_SCHUR_SUBST: W, lu' and the gain record by forward / back
// substitution with Luu (no explicit T = Luu^{-1}, 16 fewer uniform VALU a
// stage); PDPLQR_SCHUR_DPP: per-row-group picks and the column-0 merge as
// masked DPP moves (row_mask / bank_mask) instead of v_cndmask pairs (m = 4)
// (default on: same-box A/B r4f, headline backward 3.22 -> 2.96 ms with LPW,
// C5 KKT 1.297 -> 1.260 ms, C5 Riccati 0.913 -> 0.872 ms)
#ifndef PDPLQR_SCHUR_SUBST
#define PDPLQR_SCHUR_SUBST 1
#endif
#ifndef PDPLQR_SCHUR_DPP
#define PDPLQR_SCHUR_DPP 0
#endif
#ifndef PDPLQR_SCHUR_LPW
#define PDPLQR_SCHUR_LPW 1
#endif

// G = P E~ and M = H~ + E~^T G as independent per-chunk MFMAs summed by VALU
// (compile-time m = 4) instead of one accumulation chain (A/B: schur_stage)
#ifndef PDPLQR_SCHUR_SPLIT
#define PDPLQR_SCHUR_SPLIT 0
#endif

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
#ifndef PDPLQR_SCHUR_T4
#define PDPLQR_SCHUR_T4 0
#endif

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
#ifndef PDPLQR_SCHUR_LDSU
#define PDPLQR_SCHUR_LDSU 0
#endif

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
    static_assert(!GAIN || !PDPLQR_SCHUR_T4, "gain record needs the VALU W");
    static_assert(!LPW || (GAIN && MM == 4 && PDPLQR_LP_IN_P && !PDPLQR_SCHUR_LDSU), "lu in W: 12/4 gain path");
    double a[4][4], lu[4], L[4][4], T[4][4], inv[4];
    bool ok = true;
#if PDPLQR_SCHUR_LDSU
    double ml[4];  // column c of the u rows: m_l = M[l][c]
    if constexpr (MM == 4) {
        // lane (g, c) holds M[g][c] (register 0): stored at [c][g]; lu[g] by lanes (g, 0)
        ldsu[4 * c + g] = M[0];
        if (c == 0) ldsl[g] = lpr[0];
        wave_sync();
        const double2 *q = reinterpret_cast<const double2 *>(ldsu);
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // column j of Muu (uniform address: broadcast reads)
            const double2 v0 = q[2 * j], v1 = q[2 * j + 1];
            a[0][j] = v0.x;
            a[1][j] = v0.y;
            a[2][j] = v1.x;
            a[3][j] = v1.y;
        }
        const double2 l0 = reinterpret_cast<const double2 *>(ldsl)[0], l1 = reinterpret_cast<const double2 *>(ldsl)[1];
        lu[0] = l0.x;
        lu[1] = l0.y;
        lu[2] = l1.x;
        lu[3] = l1.y;
        const double2 c0 = q[2 * c], c1 = q[2 * c + 1];
        ml[0] = c0.x;
        ml[1] = c0.y;
        ml[2] = c1.x;
        ml[3] = c1.y;
    } else
#endif
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
#if PDPLQR_SCHUR_SUBST
#pragma unroll
    for (int i = 0; i < MM; ++i) {  // lu' = Luu^{-1} lu (forward substitution)
        double v = lu[i];
#pragma unroll
        for (int j = 0; j < i; ++j) v = __builtin_fma(-L[i][j], luq[j], v);
        luq[i] = v * inv[i];
    }
#else
#pragma unroll
    for (int i = 0; i < MM; ++i) {  // lu' = T lu
        double v = 0.0;
#pragma unroll
        for (int j = 0; j <= i; ++j) v = __builtin_fma(T[i][j], lu[j], v);
        luq[i] = v;
    }
#endif
#if PDPLQR_SCHUR_T4
    // W = T times the u rows (register 0 of every lane: the B operand) as one
    // MFMA (combine_tiles.hpp t4_apply); T zero-padded past m
    double Tz[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) Tz[i][j] = (i < MM) ? T[i < MM ? i : 0][j < MM ? j : 0] : 0.0;
    w = t4_apply(t4_operand(Tz, g, c), M[0]);
#else
    // column c of the u rows: m_l = M[l][c] (group l, register 0)
    if constexpr (LPW) M[0] = (c == 0) ? lpr[0] : M[0];  // the readlanes above took Muu first
#if PDPLQR_SCHUR_LDSU
    if constexpr (MM != 4)
#else
    double ml[4];
#endif
#pragma unroll
        for (int l = 0; l < MM; ++l) ml[l] = bcast_group(M[0], l);
    w = 0.0;
    double Wc[4];  // W[c][j], j < m: this lane's row of the u columns
#if PDPLQR_SCHUR_SUBST
#pragma unroll
    for (int j = 0; j < MM; ++j) {  // W_c = Luu^{-1} m_c (forward substitution, no T)
        double v = ml[j];
#pragma unroll
        for (int l = 0; l < j; ++l) v = __builtin_fma(-L[j][l], Wc[l], v);
        Wc[j] = v * inv[j];
    }
#else
#pragma unroll
    for (int j = 0; j < MM; ++j) {
        double v = 0.0;
#pragma unroll
        for (int l = 0; l <= j; ++l) v = __builtin_fma(T[j][l], ml[l], v);
        Wc[j] = v;
    }
#endif
    if constexpr (PDPLQR_SCHUR_DPP && MM == 4) {
        w = pick_group(Wc);  // W[c][g]
    } else {
#pragma unroll
        for (int j = 0; j < MM; ++j) w = (g == j) ? Wc[j] : w;  // W[c][g]; groups g >= m keep 0
    }
    if constexpr (GAIN) {  // K~[i][c] = sum_{l >= i} T[l][i] W[c][l], k~[i] = sum_{l >= i} T[l][i] lu'[l]
        double ka[4] = {0.0, 0.0, 0.0, 0.0}, kb[4] = {0.0, 0.0, 0.0, 0.0};
#if PDPLQR_SCHUR_SUBST
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
#else
#pragma unroll
        for (int i = 0; i < MM; ++i) {
#pragma unroll
            for (int l = i; l < MM; ++l) {
                ka[i] = __builtin_fma(T[l][i], Wc[l], ka[i]);
                kb[i] = __builtin_fma(T[l][i], luq[l], kb[i]);
            }
        }
#endif
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
        } else if constexpr (PDPLQR_SCHUR_DPP && MM == 4) {
            kt = pick_group(ka);
            kq = pick_group(kb);
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
#endif
#if PDPLQR_LP_IN_P
    // lp -= W lu' rides in the same MFMA: column 0 of M (u column 0: dead
    // after this stage -- the next stage reads P's x rows through the x
    // K-chunks only, and G's u rows are never used) carries lp in, the B
    // operand's column 0 carries lu', so D[:, 0] = lp - W lu'; then the
    // column-0 result to every lane of its row (DPP row_newbcast:0)
    if constexpr (LPW) {
#pragma unroll
        for (int r = 1; r < 4; ++r) M[r] = (c == 0) ? lpr[r] : M[r];
        M = mfma_f64(-w, w, M);  // M - W W^T; column 0: lp - W lu' (lane (g, 0): w = lu'[g])
    } else if constexpr (PDPLQR_SCHUR_DPP && MM == 4) {
        // masked DPP moves instead of lane selects: lanes c < 4 (DPP bank 0 of
        // every row) take lp and lu' -- columns 1..3 are dead u columns as
        // well (they feed only G's u rows next stage), so they may carry the
        // same lp - W lu' as column 0
        const double lq = pick_group(luq);
#pragma unroll
        for (int r = 0; r < 4; ++r) M[r] = dpp_keep<0xF, 0x1>(M[r], lpr[r]);
        M = mfma_f64(-w, dpp_keep<0xF, 0x1>(w, lq), M);  // M - W W^T; columns 0..3: lp - W lu'
    } else {
        const double lq = (g < MM) ? luq[g < MM ? g : 0] : 0.0;
#pragma unroll
        for (int r = 0; r < 4; ++r) M[r] = (c == 0) ? lpr[r] : M[r];
        M = mfma_f64(-w, (c == 0) ? lq : w, M);  // M - W W^T; column 0: lp - W lu'
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) lpr[r] = bcast_lane16(M[r], 0);
#else
    M = mfma_f64(-w, w, M);  // M - W W^T
    // lp -= W lu': one MFMA with lu' as column 0 of the B operand, then the
    // column-0 result to every lane of its row (DPP row_newbcast:0)
    const double lb = (c == 0 && g < MM) ? luq[g < MM ? g : 0] : 0.0;
    const d4 y = mfma_f64(w, lb, d4{0.0, 0.0, 0.0, 0.0});
#pragma unroll
    for (int r = 0; r < 4; ++r) lpr[r] -= bcast_lane16(y[r], 0);
#endif
    return ok;
}

// One stage.  Pm: in = tile whose trailing (x) block is P_{k+1}; out = M_k
// after the m u-pivots (trailing block P_k, u columns unscaled L).  prow:
// p~ in row layout (prow[r] = p[4 r + g - m] on x rows).
template <int MM, bool SYM = true, bool GAIN = false, bool LPW = false, int SPLIT = PDPLQR_SCHUR_SPLIT>
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
        // chain ~250 cycles earlier for 8 v_add_f64
        // (PDPLQR_SCHUR_SPLIT = 2: two accumulators, chunks 1 | 2, 3 -- fewer
        // live registers than three)
        const d4 z = {0.0, 0.0, 0.0, 0.0};
        if constexpr (SPLIT == 2) {
            const d4 g2 = mfma_f64(Pm[2], in.E[2], z), g1 = mfma_f64(Pm[1], in.E[1], z);
            G = g1 + mfma_f64(Pm[3], in.E[3], g2);
            const d4 m2 = mfma_f64(in.E[2], G[2], z), m1 = mfma_f64(in.E[1], G[1], in.H);
            Mn = m1 + mfma_f64(in.E[3], G[3], m2);
        } else {
            const d4 g1 = mfma_f64(Pm[1], in.E[1], z), g2 = mfma_f64(Pm[2], in.E[2], z),
                     g3 = mfma_f64(Pm[3], in.E[3], z);
            G = (g1 + g2) + g3;
            const d4 m1 = mfma_f64(in.E[1], G[1], in.H), m2 = mfma_f64(in.E[2], G[2], z),
                     m3 = mfma_f64(in.E[3], G[3], z);
            Mn = (m1 + m2) + m3;
        }
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
    if (!PDPLQR_LDS_PAD || g == 0) sm.lpt[colpos<1>(c)] = in.h + part;  // every group holds the same sum
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

// Same record, staged in LDS and written with one dwordx4 store instruction
// (lanes < FS/2): coalesced, and a fixed vm-op count for the DMA accounting.
template <int M, int S>
__device__ __forceinline__ void schur_store_record_staged(double *FRk, double w, const double (&luq)[4], SchurSmem &sm,
                                                          int g, int c) {
    constexpr int FS = S * M + M;
    static_assert(FS % 2 == 0 && FS <= 128, "record staging");
    const int lane = 16 * g + c;
    if (g < M) sm.rec[g * S + c] = (c >= g) ? w : 0.0;  // L(c, g), column g of the record
    if (lane < M) sm.rec[S * M + lane] = luq[lane < M ? lane : 0];
    wave_sync();
    if (lane < FS / 2) gstore2(FRk + 2 * lane, reinterpret_cast<const d2v *>(sm.rec)[lane]);
}

// The same record stored straight from the registers (PDPLQR_REC_DIRECT): for
// m = 4, s = 16 column g of L is lane (g, c)'s own slot FR[16 g + c], so the
// 64 lanes write the L part with ONE contiguous store and lanes 0..3 the lu'
// part with a second; no LDS round trip.  Two stores per stage.
template <int M, int S>
__device__ __forceinline__ void schur_store_record_direct(double *FRk, double w, const double (&luq)[4], int g,
                                                          int c) {
    static_assert(M == 4 && S == 16, "one record column per row group");
    const int lane = 16 * g + c;
    gstore(FRk + lane, (c >= g) ? w : 0.0);
    if (lane < M) gstore(FRk + S * M + lane, luq[lane < M ? lane : 0]);
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

// Record from the tile (chol_tiles path): u columns of M scaled by 1/sqrt(d)
// (sm.inv), lu' from sm.luq; staged in LDS, one coalesced store.
template <int M, int S>
__device__ __forceinline__ void schur_store_record_tile(double *FRk, const d4 &Pm, SchurSmem &sm, int g, int c) {
    constexpr int FS = S * M + M;
    const int lane = 16 * g + c;
    const int cm = c < M ? c : M - 1;
    const double iv = sm.inv[cm];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = 4 * r + g;
        if (c < M && i < S) sm.rec[c * S + i] = (i >= c) ? Pm[r] * iv : 0.0;
    }
    if (lane < M) sm.rec[S * M + lane] = sm.luq[lane];
    wave_sync();
    if (lane < FS / 2) gstore2(FRk + 2 * lane, reinterpret_cast<const d2v *>(sm.rec)[lane]);
}


}  // namespace pdplqr
