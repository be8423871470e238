// kernels_segment.hip -- segment backward of the parallel solver in augmented
// value form (reference: ParallelLQRKernel::step_with_factorization,
// lqr_kernel_parallel.hpp:88-136, driven by reduction_per_thread,
// lqr_solver_parallel.hpp:164-188).
//
// Per stage k the reference factors the full stage matrix
// M_k = H~_k + E^T Lxx Lxx^T E (s pivots), then forms K, d, G_k = -Luu^{-1} B^T F^T,
// Acl = A + B K and the element recursion
//     F_k = F_{k+1} Acl,  f_k = F_{k+1}(c + B d) + f_{k+1},  C_k = C_{k+1} + G_k^T G_k.
// All of that is ONE value-form Riccati stage of an augmented problem with
// state [x; y] (y+ = y, no cost on y): with the value matrix
//     Q_{k+1} = [[P, F^T], [F, -C]]  (2n x 2n),  q_{k+1} = [p; f]
// the stage matrix over [u; x; y] is
//     [[ H~ + E~^T P E~ , (F E~)^T ],
//      [ F E~           ,  -C      ]]
// with aug column [h~ + E~^T (P c + p); F c + f], and eliminating only the m
// u-pivots leaves exactly Q_k = [[P_k, F_k^T], [F_k, -C_k]], q_k = [p_k; f_k]
// (F_k = F A - Z Lxu^T with Z = F B Luu^{-T} = -G_k^T, -C_k = -C - Z Z^T).  So
// per stage: 3 MFMA products (P E~, E~^T(P E~), E~^T F^T) and m pivots of a
// (2n + m)-wide tile matrix, against s pivots plus a scalar n^3 recursion in
// the direct form.  G_k comes out of the eliminated u rows of the y columns.
//
// The value matrix lives in MFMA C-layout registers, padded to 16 T with
// T = ceil((2n + m) / 16) (<= 4 since n + m <= 32).  Index map of the padded
// dimension: u = 0..m-1, x = m..s-1, y = s..s+n-1.  Only the upper-right y
// block (F^T) is read; the lower-left one is never updated.
//
// The factor cache of a PARALLEL handle (Lc) holds P_k = Lxx Lxx^T, packed
// lower n x n at stage offset k ps: it is all backward_without_factorization
// needs besides the rollout record (k_seg_bwd_nofact).
#include "device_common.hpp"
#include <stdlib.h>
#include "parallel.hpp"

namespace pdplqr {

template <int T>
struct AugSmem {
    static constexpr int P = 16 * T;
    alignas(16) double col[P];  // pivot-row broadcast (colpos<T> order)
    alignas(16) double lpt[P];  // aug column, column -> row layout (colpos<T> order)
    double inv[32];             // 1 / sqrt(u pivot)
    double luq[32];             // lu' = Luu^{-1} lu
    double tp[32 * 33];         // transpose of the [u; x] block (P symmetrisation)
};

// Stage-k inputs of one lane.  s <= 32: the [u; x] block spans at most two
// tiles and the x rows at most 8 K chunks of 4.
struct AugIn {
    double E[8][2];  // E~[4 kk + g][16 b + c]  (x row 4 kk + g - m)
    d4 H[2][2];      // H~[16 a + 4 r + g][16 b + c], zero outside s x s
    double ct[8];    // c~[4 kk + g]
    double h[2];     // h~[16 b + c]
};

__device__ __forceinline__ void aug_load(AugIn &in, const double *__restrict__ Ek, const double *__restrict__ ck,
                                         const double *__restrict__ Hk, const double *__restrict__ hk, int n, int m,
                                         int g, int c) {
    const int s = n + m, k0 = m >> 2, k1 = (s - 1) >> 2;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
        const int t = 4 * kk + g - m;
        const bool xr = kk >= k0 && kk <= k1 && t >= 0 && t < n;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const int j = 16 * b + c;
            in.E[kk][b] = (xr && j < s) ? Ek[t + j * n] : 0.0;
        }
        in.ct[kk] = xr ? ck[t] : 0.0;
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * a + 4 * r + g, j = 16 * b + c;
                in.H[a][b][r] = (i < s && j < s) ? Hk[i >= j ? pidx(i, j, s) : pidx(j, i, s)] : 0.0;
            }
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const int j = 16 * b + c;
        in.h[b] = (j < s) ? hk[j] : 0.0;
    }
}

// Right-looking elimination of the u pivots 0..m-1 of the augmented stage
// matrix (same broadcast scheme as chol_tiles: row j through LDS, pivot
// column left unscaled, 1/sqrt(pivot) in sm.inv), with the aug column lpr.
// Tiles entirely below the [u; x] rows and left of the y columns (the
// lower-left F block) are never read and are skipped.
template <int T>
__device__ __forceinline__ bool aug_elim(d4 (&M)[T][T], double (&lpr)[T][4], AugSmem<T> &sm, int m, int s, int g,
                                         int c) {
    constexpr int TP = T < 2 ? T : 2;  // tiles that can hold u pivots (m < 32)
    bool ok = true;
    const bool lane0 = (g == 0) && (c == 0);
    const double2 *rows = reinterpret_cast<const double2 *>(sm.col + g * 4 * T);
#pragma unroll
    for (int tr = 0; tr < TP; ++tr)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
#pragma unroll 1
            for (int gj = 0; gj < 4; ++gj) {
                const int j = 16 * tr + 4 * rr + gj;
                if (j >= m) break;
                if (g == gj) {
#pragma unroll
                    for (int b = 0; b < T; ++b) {
                        const int jc = 16 * b + c;
                        sm.col[colpos<T>(jc)] = (jc > j) ? M[tr][b][rr] : 0.0;
                    }
                }
                wave_sync();
                const double djj = readlane_f64(M[tr][tr][rr], (gj << 4) + (j & 15));
                ok = ok && (djj > 0.0);
                const double inv = rsqrt_f64(djj);
                const double inv2 = inv * inv;
                if (lane0) sm.inv[j] = inv;
                double lc[T];
#pragma unroll
                for (int b = 0; b < T; ++b) lc[b] = sm.col[colpos<T>(16 * b + c)] * inv2;
                const double lpj = readlane_f64(lpr[tr][rr], gj << 4);
                const double qj = lpj * inv2;
                double li[T][4];
#pragma unroll
                for (int q = 0; q < 2 * T; ++q) {
                    const double2 v = rows[q];
                    li[q >> 1][(q & 1) * 2] = v.x;
                    li[q >> 1][(q & 1) * 2 + 1] = v.y;
                }
#pragma unroll
                for (int a = 0; a < T; ++a)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
#pragma unroll
                        for (int b = 0; b < T; ++b)
                            if (!(16 * a >= s && 16 * (b + 1) <= s))
                                M[a][b][r] = __builtin_fma(-li[a][r], lc[b], M[a][b][r]);
                        lpr[a][r] = __builtin_fma(-li[a][r], qj, lpr[a][r]);
                    }
                if (lane0) sm.luq[j] = lpj * inv;
                wave_sync();
            }
        }
    return ok;
}

// One wavefront per (problem, segment).  NN, MM > 0: compile-time shape.
template <int T, int NN, int MM>
__global__ __launch_bounds__(64) void k_seg_bwd_aug(SegArgs A) {
    constexpr bool CT = NN > 0;
    __shared__ AugSmem<T> sm;
    const int lane = wave_lane(), g = lane >> 4, c = lane & 15;
    const Shape &sh = A.sh;
    const int n = CT ? NN : sh.n, m = CT ? MM : sh.m, s = n + m, S = A.S;
    const int k0 = m >> 2, k1 = (s - 1) >> 2;  // K chunks holding x rows
    const long long bi = blockIdx.x / S;
    const int seg = blockIdx.x % S;
    if (A.flag && seg == 0 && lane == 0) A.flag[bi] = 0;
    const int N0 = A.seg_start[seg], N1 = N0 + A.seg_len[seg];
    const bool last = (seg == S - 1) && A.last_is_terminal;
    const long long frs = (long long)s * m + m;
    const int ps = sh.ps;
    const double *Eb = A.E + bi * sh.perE;
    const double *cb = A.c + bi * sh.perc;
    const double *Hb = A.Hw + bi * sh.perHw;
    const double *hb = A.hw + bi * sh.perh;
    double *FRb = A.FR + bi * sh.perKD;
    double *Gb = A.G + bi * (long long)sh.N * m * n;
    double *Lcb = A.Lc ? A.Lc + bi * sh.perHw : nullptr;
    double *lpb = A.lpc ? A.lpc + bi * sh.perh : nullptr;
    int fail_stage = -1;

    // ---- segment terminal (lqr_kernel_parallel.hpp:52-67): the real one
    // (P = H~_N, p = h~_N, no element) or the dummy P = 0, p = 0, F = I, C = 0, f = 0
    d4 Q[T][T];
    double q[T][4];
    {
        const double *HN = Hb + (long long)sh.N * ps;
        bool bad = false;
#pragma unroll
        for (int a = 0; a < T; ++a)
#pragma unroll
            for (int bt = 0; bt < T; ++bt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * a + 4 * r + g, j = 16 * bt + c;
                    const bool xi = i >= m && i < s, xj = j >= m && j < s;
                    double v = 0.0;
                    if (last) {
                        if (xi && xj) v = HN[i >= j ? pidx(i - m, j - m, n) : pidx(j - m, i - m, n)];
                        if (xi && i == j && psd_bad(v)) bad = true;
                    } else if ((xi && j == i - m + s) || (xj && i == j - m + s)) {
                        v = 1.0;
                    }
                    Q[a][bt][r] = v;
                }
#pragma unroll
        for (int a = 0; a < T; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * a + 4 * r + g;
                q[a][r] = (last && i >= m && i < s) ? hb[(long long)sh.N * s + (i - m)] : 0.0;
            }
        if (last) {
            if (__any(bad)) fail_stage = sh.N;
            const int pn = n * (n + 1) / 2;
            if (Lcb)
                for (int t = lane; t < pn; t += 64) Lcb[(long long)sh.N * ps + t] = HN[t];
            if (lpb && lane < n) lpb[(long long)sh.N * s + lane] = hb[(long long)sh.N * s + lane];
        }
    }

    AugIn nxt;
    aug_load(nxt, Eb + (long long)(N1 - 1) * n * s, cb + (long long)(N1 - 1) * n, Hb + (long long)(N1 - 1) * ps,
             hb + (long long)(N1 - 1) * s, n, m, g, c);
    for (int k = N1 - 1; k >= N0; --k) {
        const AugIn in = nxt;
        if (k > N0)
            aug_load(nxt, Eb + (long long)(k - 1) * n * s, cb + (long long)(k - 1) * n, Hb + (long long)(k - 1) * ps,
                     hb + (long long)(k - 1) * s, n, m, g, c);
        // ---- G = P E~ (rows of the [u; x] tiles; only the x rows are used) ----
        d4 G[2][2];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int bt = 0; bt < 2; ++bt) {
                G[a][bt] = d4{0.0, 0.0, 0.0, 0.0};
                // one [u; x] tile (s <= 16, C2's 12/4): odd K chunks on a second
                // accumulator -- the tile's chain is the only one in flight
                constexpr bool SPL = CT && NN + MM <= 16;
                d4 Go = d4{0.0, 0.0, 0.0, 0.0};
                if (a < T && bt < T && 16 * a < s && 16 * bt < s) {
#pragma unroll
                    for (int kk = 0; kk < 8; ++kk)
                        if ((kk >> 2) < T && kk >= k0 && kk <= k1) {
                            const double av = Q[(kk >> 2) < T ? (kk >> 2) : 0][a < T ? a : 0][kk & 3];
                            if (SPL && (kk & 1)) Go = mfma_f64(av, in.E[kk][bt], Go);
                            else G[a][bt] = mfma_f64(av, in.E[kk][bt], G[a][bt]);
                        }
                    if (SPL) G[a][bt] += Go;
                }
            }
        // ---- aug column in column layout (reads the old y columns = F^T):
        //      [u; x]: h~ + G^T c~ + E~^T p~ ; y: F c (+ f below, row layout) ----
#pragma unroll
        for (int bt = 0; bt < T; ++bt) {
            const int j = 16 * bt + c;
            const bool cux = j < s;
            double part = 0.0;
#pragma unroll
            for (int kk = 0; kk < 8; ++kk)
                if ((kk >> 2) < T && kk >= k0 && kk <= k1) {
                    const double qv = Q[(kk >> 2) < T ? (kk >> 2) : 0][bt][kk & 3];
                    const double bop = (bt < 2 && cux) ? G[kk >> 2][bt < 2 ? bt : 0][kk & 3] : qv;
                    part = __builtin_fma(bop, in.ct[kk], part);
                    if (bt < 2) part = __builtin_fma(in.E[kk][bt < 2 ? bt : 0], q[kk >> 2][kk & 3], part);
                }
            part = sum_groups(part);
            if (bt < 2 && cux) part += in.h[bt < 2 ? bt : 0];
            if (g == 0) sm.lpt[colpos<T>(j)] = part;
        }
        // ---- stage matrix rows [u; x]: [H~ + E~^T G | E~^T F^T]; y rows keep Q ----
#pragma unroll
        for (int bt = 0; bt < T; ++bt) {
            const bool cux = 16 * bt + c < s;
            d4 acc[2];
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                if (a < T && 16 * a < s) {
                    const d4 h0 = (bt < 2) ? in.H[a][bt < 2 ? bt : 0] : d4{0.0, 0.0, 0.0, 0.0};
                    acc[a] = cux ? h0 : d4{0.0, 0.0, 0.0, 0.0};
                    constexpr bool SPL = CT && NN + MM <= 16;
                    d4 ao = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
                    for (int kk = 0; kk < 8; ++kk)
                        if ((kk >> 2) < T && kk >= k0 && kk <= k1) {
                            const double qv = Q[(kk >> 2) < T ? (kk >> 2) : 0][bt][kk & 3];
                            const double bop = (bt < 2 && cux) ? G[kk >> 2][bt < 2 ? bt : 0][kk & 3] : qv;
                            if (SPL && (kk & 1)) ao = mfma_f64(in.E[kk][a], bop, ao);
                            else acc[a] = mfma_f64(in.E[kk][a], bop, acc[a]);
                        }
                    if (SPL) acc[a] += ao;
                }
            }
#pragma unroll
            for (int a = 0; a < 2; ++a)
                if (a < T && 16 * a < s)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (16 * a + 4 * r + g < s) Q[a < T ? a : 0][bt][r] = acc[a][r];
        }
        wave_sync();
        double lpr[T][4];
        {
            const double2 *rw = reinterpret_cast<const double2 *>(sm.lpt + g * 4 * T);
#pragma unroll
            for (int qq = 0; qq < 2 * T; ++qq) {
                const double2 v = rw[qq];
                lpr[qq >> 1][(qq & 1) * 2] = v.x;
                lpr[qq >> 1][(qq & 1) * 2 + 1] = v.y;
            }
#pragma unroll
            for (int a = 0; a < T; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (16 * a + 4 * r + g >= s) lpr[a][r] += q[a][r];  // + f
        }
        // ---- eliminate the u pivots: leaves Q_k, q_k ----
        bool ok = aug_elim<T>(Q, lpr, sm, m, s, g, c);
#pragma unroll
        for (int a = 0; a < T; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) q[a][r] = lpr[a][r];
        // ---- P_k <- (P_k + P_k^T) / 2 (see kernels_schur.hip) and diag check ----
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int bt = 0; bt < 2; ++bt)
                if (a < T && bt < T)
#pragma unroll
                    for (int r = 0; r < 4; ++r) sm.tp[(16 * a + 4 * r + g) * 33 + 16 * bt + c] = Q[a < T ? a : 0][bt < T ? bt : 0][r];
        wave_sync();
        bool bad = false;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int bt = 0; bt < 2; ++bt)
                if (a < T && bt < T)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int i = 16 * a + 4 * r + g, j = 16 * bt + c;
                        if (i >= m && j >= m && i < s && j < s) {
                            const double v = 0.5 * (Q[a < T ? a : 0][bt < T ? bt : 0][r] + sm.tp[j * 33 + i]);
                            Q[a < T ? a : 0][bt < T ? bt : 0][r] = v;
                            if (i == j && psd_bad(v)) bad = true;
                        }
                    }
        ok = ok && !__any(bad);
        if (!ok && fail_stage < 0) fail_stage = k;
        // ---- rollout record FR_k = [L(:, 0:m) | lu'] ----
        double *FRk = FRb + (long long)k * frs;
#pragma unroll
        for (int bt = 0; bt < 2; ++bt)
            if (bt < T) {
                const int j = 16 * bt + c;
                if (j < m) {
                    const double iv = sm.inv[j];
#pragma unroll
                    for (int a = 0; a < 2; ++a)
                        if (a < T)
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                const int i = 16 * a + 4 * r + g;
                                if (i < s) FRk[j * s + i] = (i >= j) ? Q[a < T ? a : 0][bt][r] * iv : 0.0;
                            }
                }
            }
        if (lane < m) FRk[(long long)s * m + lane] = sm.luq[lane];
        // ---- G_k = -Z^T = -L(y, u)^T (eliminated u rows of the y columns) ----
        if (!last) {
            double *Gk = Gb + (long long)k * m * n;
#pragma unroll
            for (int a = 0; a < 2; ++a)
                if (a < T)
#pragma unroll
                    for (int bt = 0; bt < T; ++bt)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int i = 16 * a + 4 * r + g, j = 16 * bt + c;
                            if (i < m && j >= s && j < s + n) Gk[i + (j - s) * m] = -Q[a < T ? a : 0][bt][r] * sm.inv[i];
                        }
        }
        // ---- factor cache: P_k (packed lower), lp_k = [lu'; p_k] ----
        if (Lcb) {
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int bt = 0; bt < 2; ++bt)
                    if (a < T && bt < T)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int i = 16 * a + 4 * r + g, j = 16 * bt + c;
                            if (j >= m && i >= j && i < s)
                                Lcb[(long long)k * ps + pidx(i - m, j - m, n)] = Q[a < T ? a : 0][bt < T ? bt : 0][r];
                        }
        }
        if (lpb) {
            if (lane < m) lpb[(long long)k * s + lane] = sm.luq[lane];
            if (c == 0)
#pragma unroll
                for (int a = 0; a < 2; ++a)
                    if (a < T)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int i = 16 * a + 4 * r + g;
                            if (i >= m && i < s) lpb[(long long)k * s + i] = q[a < T ? a : 0][r];
                        }
        }
    }
    // ---- export the element (update_segment_data, lqr_solver_parallel.hpp:182-187) ----
    double *eo = A.elem + (bi * S + seg) * (long long)(3 * n * n + 2 * n);
    double *eF = eo, *eC = eo + n * n, *ef = eo + 2 * n * n, *eP = ef + n, *ep = eP + n * n;
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int bt = 0; bt < T; ++bt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * a + 4 * r + g, j = 16 * bt + c;
                const double v = Q[a][bt][r];
                const bool xi = i >= m && i < s, xj = j >= m && j < s;
                const bool yi = i >= s && i < s + n, yj = j >= s && j < s + n;
                if (xi && xj) eP[(i - m) + (j - m) * n] = v;                 // P = Lxx Lxx^T
                if (xi && yj) eF[(j - s) + (i - m) * n] = last ? 0.0 : v;   // F (stored as F^T)
                if (yi && yj) eC[(i - s) + (j - s) * n] = last ? 0.0 : -v;  // C
            }
    if (c == 0)
#pragma unroll
        for (int a = 0; a < T; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * a + 4 * r + g;
                if (i >= m && i < s) ep[i - m] = q[a][r];
                if (i >= s && i < s + n) ef[i - s] = last ? 0.0 : q[a][r];
            }
    if (lane == 0) A.seg_status[bi * S + seg] = fail_stage < 0 ? 0 : fail_stage + 1;
}

// ---------------------------------------------------------------------------
// The same segment backward on a 4-wave workgroup (horizon shards at 24/8:
// one problem, a few hundred segments -- the stage chain of ONE wave is the
// latency the whole C4 slice waits on).  Wave w owns column tile w of the
// padded stage matrix (columns 16 w .. 16 w + 15, all 64 rows); column D =
// s + n carries the aug vector (rows [u; x]: lp, rows y: F c + f), so the
// elimination updates it with the matrix.  Per stage:
//   * waves whose columns include [u; x]: G = P E~ (rows x; P symmetrised
//     from the published x block), then rows [u; x] = H~ + E~^T G;
//   * y (and aug) columns: rows [u; x] = E~^T Q[x, col] from the wave's own
//     registers, rows y unchanged (-C, f);  the rows y of the [u; x] columns
//     (F E~) are never formed: the elimination takes the pivot COLUMNS from the
//     pivot rows by symmetry, so nothing reads them;
//   * lp (column -> row via LDS) and F c complete the aug column;
//   * the m u-pivots in blocks of 4: every wave publishes its part of the 4
//     pivot rows, Muu^{-1} is formed wave-uniformly, and each row tile takes one
//     rank-4 MFMA update  M -= M[:, J] (Muu^{-1} M[J, :])  (A operand = pivot
//     rows by symmetry, B operand = X of the lane's own column).
// Records as k_seg_bwd_aug: FR_k = [L(:, 0:m) | lu'] with L(:, J) = M[:, J]
// Luu^{-T}, G_k = -L(y, u)^T, the factor cache P_k / lp_k, the element.
// Conditions: s <= 32 (the x columns sit in tiles 0, 1), D = s + n < 64,
// m % 4 == 0, m <= 16.
// ---------------------------------------------------------------------------
#ifdef PDPLQR_COMB_PROFILE
__device__ unsigned long long g_aug_t[1024 * 16];
// slots 0-7 the stage phases, 8-13 three marks per pivot block, 14 / 15 the
// shader clock (clock64) at marks 0 / 7
#define AUG_MARK(q)                                                                              \
    do {                                                                                         \
        if (tid == 0 && k == N1 - 2) {                                                           \
            g_aug_t[(blockIdx.x % 1024) * 16 + (q)] = wall_clock64();                            \
            if ((q) == 0 || (q) == 7) g_aug_t[(blockIdx.x % 1024) * 16 + 14 + ((q) == 7)] = clock64(); \
        }                                                                                        \
    } while (0)
#else
#define AUG_MARK(q) \
    do {            \
    } while (0)
#endif

template <int NN, int MM>
// PDPLQR_AUG_MW_OCC: resident blocks per CU the register allocation targets
// (2: 215 VGPRs, no spill; 3: 168 VGPRs with 19 spill ops per stage -- the
// N = 8192 slice 0.49 -> 0.62 ms, forced 4-wave N = 65536 1.32 -> 1.54 ms)
#ifndef PDPLQR_AUG_PIV8
#define PDPLQR_AUG_PIV8 0
#endif
#ifndef PDPLQR_AUG_MW_OCC
#define PDPLQR_AUG_MW_OCC 2
#endif
__global__ __launch_bounds__(256, PDPLQR_AUG_MW_OCC) void k_seg_bwd_aug_mw(SegArgs A) {
    constexpr int n = NN, m = MM, s = NN + MM, D = s + NN, AUG = D;
    constexpr int ps = s * (s + 1) / 2, PN = n * (n + 1) / 2;
    constexpr int XLD = n + 1;                       // leading dimension of the published P block
    constexpr int IN = n * s + ps + n + s;           // stage input doubles: E~ | H~ packed | c | h~
    constexpr int INQ = (IN + 255) / 256;            // per thread
    constexpr int K0 = m / 4, K1 = s / 4;            // K chunks of the x rows
    static_assert(s <= 32 && D < 64 && m % 4 == 0 && m <= 16 && n % 4 == 0, "4-wave aug shape");
    // u-pivots per elimination block: 8 when m allows (one publish / barrier /
    // factor round for m = 8 instead of two), else 4 (PDPLQR_AUG_PIV8=0: 4 always)
    constexpr int PIVB = (PDPLQR_AUG_PIV8 && m % 8 == 0) ? 8 : 4;
    __shared__ double Xq[n * XLD];                   // P_{k+1} (x rows, x cols)
    __shared__ double In[IN];                        // E~ (n x s) | H~ packed | c | h~ of this stage
    __shared__ double Pr[2][PIVB * 64];              // pivot rows of block 0 / 1 at every column
    __shared__ double augr[64];                      // per row of the aug column: h~ + G^T c ([u; x]), F c (y), 0
    __shared__ int s_bad;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, g = lane >> 4, c = lane & 15;
    const int col = 16 * wv + c;
    const bool cux = col < s, cy = col >= s && col < D, caug = col == AUG;
    const Shape &sh = A.sh;
    const int S = A.S;
    const long long bi = blockIdx.x / S;
    const int seg = blockIdx.x % S;
    if (A.flag && seg == 0 && tid == 0) A.flag[bi] = 0;
    const int N0 = A.seg_start[seg], N1 = N0 + A.seg_len[seg];
    const bool last = (seg == S - 1) && A.last_is_terminal;
    const long long frs = (long long)s * m + m;
    const double *Eb = A.E + bi * sh.perE;
    const double *cb = A.c + bi * sh.perc;
    const double *Hb = A.Hw + bi * sh.perHw;
    const double *hb = A.hw + bi * sh.perh;
    double *FRb = A.FR + bi * sh.perKD;
    double *Gb = A.G + bi * (long long)sh.N * m * n;
    double *Lcb = A.Lc ? A.Lc + bi * sh.perHw : nullptr;
    double *lpb = A.lpc ? A.lpc + bi * sh.perh : nullptr;
    const double *Es = In, *Hs = In + n * s, *cs = Hs + ps, *hs = cs + n;
    int fail_stage = -1;
    // stage inputs: HBM -> registers (issued a stage ahead) -> LDS
    double pre[INQ];
    // branch-free: every thread issues INQ loads at clamped addresses (a guarded
    // load compiles to an exec-mask region with its own wait)
    auto in_load = [&](int k) {
        const long long oE = (long long)k * n * s, oH = (long long)k * sh.ps, oc = (long long)k * n,
                        oh = (long long)k * s;
#pragma unroll
        for (int q = 0; q < INQ; ++q) {
            const int i = min(tid + 256 * q, IN - 1);
            const long long off = i < n * s ? oE + i
                                  : i < n * s + ps ? oH + (i - n * s)
                                  : i < n * s + ps + n ? oc + (i - n * s - ps)
                                                       : oh + (i - n * s - ps - n);
            const double *base = i < n * s ? Eb : i < n * s + ps ? Hb : i < n * s + ps + n ? cb : hb;
            pre[q] = __builtin_nontemporal_load(base + off);
        }
    };
    auto in_store = [&]() {
#pragma unroll
        for (int q = 0; q < INQ; ++q) {
            const int i = tid + 256 * q;
            if (i < IN) In[i] = pre[q];
        }
    };
    if (N1 > N0) in_load(N1 - 1);
    // ---- segment terminal: Q over [x; y; aug] ----
    d4 Q[4];
    {
        const double *HN = Hb + (long long)sh.N * sh.ps;
        bool bad = false;
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * a + 4 * r + g;
                const bool xi = i >= m && i < s, yi = i >= s && i < D;
                const bool xj = col >= m && col < s;
                double v = 0.0;
                if (last) {
                    if (xi && xj) v = HN[i >= col ? pidx(i - m, col - m, n) : pidx(col - m, i - m, n)];
                    if (xi && caug) v = hb[(long long)sh.N * s + (i - m)];
                    if (xi && i == col && psd_bad(v)) bad = true;
                } else if (xi && cy && col - s == i - m) {
                    v = 1.0;  // F^T = I (rows x of the y columns)
                }
                (void)yi;
                Q[a][r] = v;
            }
        if (tid == 0) s_bad = 0;
        if (tid >= D && tid < 64) augr[tid] = 0.0;  // padding rows (never written again)
        __syncthreads();
        if (bad) s_bad = 1;
        if (last) {
            if (Lcb)
                for (int t = tid; t < PN; t += 256) Lcb[(long long)sh.N * sh.ps + t] = HN[t];
            if (lpb)
                for (int t = tid; t < n; t += 256) lpb[(long long)sh.N * s + t] = hb[(long long)sh.N * s + t];
        }
        in_store();
        __syncthreads();
        if (s_bad) fail_stage = sh.N;
    }
    for (int k = N1 - 1; k >= N0; --k) {
        AUG_MARK(0);
        // ---- publish P_{k+1} (rows x of the x columns); next stage's inputs in flight ----
        if (col >= m && col < s)
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * a + 4 * r + g;
                    if (i >= m && i < s) Xq[(i - m) + (col - m) * XLD] = Q[a][r];
                }
        if (k > N0) in_load(k - 1);
        __syncthreads();  // B1
        AUG_MARK(1);
        if (tid == 0) s_bad = 0;  // every thread read the previous stage's flag before B1
        // ---- G = P E~ (rows x, [u; x] columns: waves 0, 1) ----
        // Every operand is read from LDS before the first product, so the two
        // accumulation chains run back to back (a wait on each product's LDS
        // reads put the LDS latency on the chain: 1.2 us per stage, r3g).
        constexpr int NK = K1 - K0;
        // (branch-free: clamped LDS addresses, values masked by a 0 / 1 factor)
        const double fux = cux ? 1.0 : 0.0;
        const int colc = cux ? col : 0;
        double bvE[NK];  // E~[kx - m][col] (B operand of G)
#pragma unroll
        for (int q = 0; q < NK; ++q) bvE[q] = fux * Es[(4 * (K0 + q) + g - m) + colc * n];
        // the aug pieces' operands (c rows of this lane group, h~[col]), read here so
        // their LDS latency hides under the products instead of chaining before B2
        double cxv[NK];
#pragma unroll
        for (int q = 0; q < NK; ++q) cxv[q] = cs[4 * (K0 + q) + g - m];
        const double hcol = hs[colc];
        d4 G[2] = {d4{0.0, 0.0, 0.0, 0.0}, d4{0.0, 0.0, 0.0, 0.0}};
        if (wv < 2) {
            double avP[2][NK];  // P_sym[16 a + c][kx]
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                const int i = 16 * a + c;
                const bool xi = i >= m && i < s;
                const int ii = xi ? i - m : 0;
                const double hx = xi ? 0.5 : 0.0;
#pragma unroll
                for (int q = 0; q < NK; ++q) {
                    const int kx = 4 * (K0 + q) + g;
                    avP[a][q] = hx * (Xq[ii + (kx - m) * XLD] + Xq[(kx - m) + ii * XLD]);
                }
            }
            // even / odd K chunks on separate accumulators: four chains of
            // NK / 2 instead of two of NK (a dependent f64 MFMA waits ~186 cycles)
            d4 Go[2] = {d4{0.0, 0.0, 0.0, 0.0}, d4{0.0, 0.0, 0.0, 0.0}};
#pragma unroll
            for (int q = 0; q < NK; ++q)
#pragma unroll
                for (int a = 0; a < 2; ++a) {
                    if (q & 1) Go[a] = mfma_f64(avP[a][q], bvE[q], Go[a]);
                    else G[a] = mfma_f64(avP[a][q], bvE[q], G[a]);
                }
#pragma unroll
            for (int a = 0; a < 2; ++a) G[a] += Go[a];
        }
        AUG_MARK(2);
        // ---- rows [u; x]: H~ + E~^T G ([u; x] columns), E~^T Q[x, col] (y / aug columns) ----
        d4 Mu[2];
        {
            double avE[2][NK];  // E~^T[16 a + c][kx] = E~[kx - m][16 a + c]
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                const int i = 16 * a + c;
                const double fi = i < s ? 1.0 : 0.0;
                const int ic = i < s ? i : 0;
#pragma unroll
                for (int q = 0; q < NK; ++q) {
                    const int kx = 4 * (K0 + q) + g;
                    avE[a][q] = fi * Es[(kx - m) + ic * n];
                }
            }
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * a + 4 * r + g;
                    const bool on = cux && i < s;
                    const int ic = on ? i : 0, jc = on ? col : 0;
                    Mu[a][r] = (on ? 1.0 : 0.0) * Hs[ic >= jc ? pidx(ic, jc, s) : pidx(jc, ic, s)];
                }
            d4 Mo[2] = {d4{0.0, 0.0, 0.0, 0.0}, d4{0.0, 0.0, 0.0, 0.0}};
#pragma unroll
            for (int q = 0; q < NK; ++q) {
                const int kk = K0 + q;
                const double bv = cux ? G[kk >> 2][kk & 3] : Q[kk >> 2][kk & 3];
#pragma unroll
                for (int a = 0; a < 2; ++a) {
                    if (q & 1) Mo[a] = mfma_f64(avE[a][q], bv, Mo[a]);
                    else Mu[a] = mfma_f64(avE[a][q], bv, Mu[a]);
                }
            }
#pragma unroll
            for (int a = 0; a < 2; ++a) Mu[a] += Mo[a];
        }
        // ---- aug pieces: augr[col] = h~ + G^T c ([u; x] columns), F c (y columns) ----
        {
            double part = 0.0;
#pragma unroll
            for (int kk = K0; kk < K1; ++kk)
                part = __builtin_fma(cux ? G[kk >> 2][kk & 3] : Q[kk >> 2][kk & 3], cxv[kk - K0], part);
            part = sum_groups(part);
            if (g == 0) {
                if (cux || cy) augr[col] = (cux ? hcol : 0.0) + part;
            }
        }
#pragma unroll
        for (int a = 0; a < 2; ++a) Q[a] = Mu[a];
        AUG_MARK(3);
        __syncthreads();  // B2
        AUG_MARK(4);
        if (caug) {  // aug column: rows [u; x] += h~ + G^T c (E~^T p is already in), rows y += F c
            // every read issued before the first add (the default schedule waited on each pair)
            double av[4][4];
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r) av[a][r] = augr[16 * a + 4 * r + g];
            __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);  // the DS reads
            __builtin_amdgcn_sched_group_barrier(0x002, 16, 0); // then the adds
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r) Q[a][r] += av[a][r];
        }
        // ---- the m u-pivots, 4 per block ----
        double *FRk = FRb + (long long)k * frs;
        double *Gk = Gb + (long long)k * m * n;
        bool ok = true;
        if constexpr (PIVB == 8) {
#pragma unroll
        for (int blk = 0; blk < m / 8; ++blk) {
            const int j0 = 8 * blk;
            double *P8 = Pr[blk & 1];
            P8[g * 64 + col] = Q[0][2 * blk];            // row j0 + g at this column
            P8[(4 + g) * 64 + col] = Q[0][2 * blk + 1];  // row j0 + 4 + g
            __syncthreads();
            AUG_MARK(8 + 3 * blk);
            // every LDS read of the block up front, then the arithmetic
            double L[8][8], pr[8], avv[4][2], mi[8], lu[8];
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j <= i; ++j) L[i][j] = P8[i * 64 + j0 + j];
#pragma unroll
            for (int l = 0; l < 8; ++l) pr[l] = P8[l * 64 + col];
#pragma unroll
            for (int a = 0; a < 4; ++a)  // M[16 a + c][j0 + 4 h + g] by symmetry (aug / padding: not rows)
#pragma unroll
                for (int h = 0; h < 2; ++h) avv[a][h] = (16 * a + c < D ? 1.0 : 0.0) * P8[(4 * h + g) * 64 + 16 * a + c];
            // Cholesky of the 8 x 8 pivot block in place (wave-uniform); the
            // diagonal keeps 1 / L_jj
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                ok = ok && (L[j][j] > 0.0);
                const double iv = rsqrt_f64(L[j][j]);
                L[j][j] = iv;
#pragma unroll
                for (int i = j + 1; i < 8; ++i) L[i][j] *= iv;
#pragma unroll
                for (int i = j + 1; i < 8; ++i)
#pragma unroll
                    for (int kq = j + 1; kq <= i; ++kq) L[i][kq] = __builtin_fma(-L[i][j], L[kq][j], L[i][kq]);
            }
            // forward substitution L^{-1} v (in place)
            auto fsub = [&](double (&v)[8]) {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    double t = v[i];
#pragma unroll
                    for (int l = 0; l < i; ++l) t = __builtin_fma(-L[i][l], v[l], t);
                    v[i] = t * L[i][i];
                }
            };
            // X[J][col] = Muu^{-1} M[J, col] = L^{-T} (L^{-1} pr)
            fsub(pr);
#pragma unroll
            for (int i = 7; i >= 0; --i) {
                double t = pr[i];
#pragma unroll
                for (int l = i + 1; l < 8; ++l) t = __builtin_fma(-L[l][i], pr[l], t);
                pr[i] = t * L[i][i];
            }
            double xg0 = 0.0, xg1 = 0.0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                xg0 = (g == i) ? pr[i] : xg0;
                xg1 = (g == i) ? pr[4 + i] : xg1;
            }
            // rank-8 update of every row tile (two K = 4 MFMAs)
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                if (wv < 2 && a >= 2) continue;  // rows y of the [u; x] columns are never read
                Q[a] = mfma_f64(-avv[a][0], xg0, Q[a]);
                Q[a] = mfma_f64(-avv[a][1], xg1, Q[a]);
            }
            AUG_MARK(9 + 3 * blk);
            // records: L(i, J) = M[i][J] L_JJ^{-T}  (row i: forward substitution);
            // their operands are read after the update is issued (registers)
            const int ir = (wv == 0) ? lane : s + lane;
            const bool rec = (wv == 0 && ir < s) || (wv == 1 && !last && lane < n);
            const int irc = ir < 64 ? ir : 0;
#pragma unroll
            for (int l = 0; l < 8; ++l) mi[l] = P8[l * 64 + irc];
#pragma unroll
            for (int l = 0; l < 8; ++l) lu[l] = P8[l * 64 + AUG];
            if (rec) {
                fsub(mi);
#pragma unroll
                for (int l = 0; l < 8; ++l) {
                    if (wv == 0) gstore(FRk + (long long)(j0 + l) * s + ir, ir >= j0 + l ? mi[l] : 0.0);
                    else gstore(Gk + (j0 + l) + lane * m, -mi[l]);
                }
            }
            if (tid == 2 * 64) {  // lu' = L^{-1} lu, lu = M[J][aug]
                fsub(lu);
#pragma unroll
                for (int l = 0; l < 8; ++l) {
                    gstore(FRk + (long long)s * m + j0 + l, lu[l]);
                    if (lpb) gstore(lpb + (long long)k * s + j0 + l, lu[l]);
                }
            }
            AUG_MARK(10 + 3 * blk);
        }
        } else {
#pragma unroll
        for (int blk = 0; blk < m / 4; ++blk) {
            const int j0 = 4 * blk;
            double *P4 = Pr[blk & 1];
            P4[g * 64 + col] = Q[0][blk];  // row j0 + g at this column
            __syncthreads();
            AUG_MARK(8 + 3 * blk);
            // every LDS read of the block up front (one wait), then the arithmetic
            double a4[4][4], L[4][4], T4[4][4], inv[4], pr[4], avv[4], mi[4], lu[4];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j <= i; ++j) a4[i][j] = P4[i * 64 + j0 + j];
#pragma unroll
            for (int l = 0; l < 4; ++l) pr[l] = P4[l * 64 + col];
#pragma unroll
            for (int a = 0; a < 4; ++a)  // M[16 a + c][j0 + g] = M[j0 + g][16 a + c] (symmetry;
                avv[a] = (16 * a + c < D ? 1.0 : 0.0) * P4[g * 64 + 16 * a + c];  // aug / padding: not rows)
#pragma unroll
            for (int a = 2; a < 4; ++a)  // keep the row-tile 2, 3 reads here, with the others (the
                asm volatile("" ::"v"(avv[a]));  // compiler sank them into the wave-2/3 branch: one LDS wait each)
            // records: wave 0 the FR rows i < s, wave 1 the coupling rows s + lane
            const int ir = (wv == 0) ? lane : s + lane;
            const bool rec = (wv == 0 && ir < s) || (wv == 1 && !last && lane < n);
            const int irc = ir < 64 ? ir : 0;
#pragma unroll
            for (int l = 0; l < 4; ++l) mi[l] = P4[l * 64 + irc];
#pragma unroll
            for (int l = 0; l < 4; ++l) lu[l] = P4[l * 64 + AUG];
            __builtin_amdgcn_sched_barrier(0);  // every LDS read above issues before the factor
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                ok = ok && (a4[j][j] > 0.0);
                inv[j] = rsqrt_f64(a4[j][j]);
                L[j][j] = a4[j][j] * inv[j];
#pragma unroll
                for (int i = j + 1; i < 4; ++i) L[i][j] = a4[i][j] * inv[j];
#pragma unroll
                for (int i = j + 1; i < 4; ++i)
#pragma unroll
                    for (int kq = j + 1; kq <= i; ++kq) a4[i][kq] = __builtin_fma(-L[i][j], L[kq][j], a4[i][kq]);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {  // T4 = Luu^{-1}
                T4[i][i] = inv[i];
#pragma unroll
                for (int j = 0; j < i; ++j) {
                    double v = 0.0;
#pragma unroll
                    for (int kq = j; kq < i; ++kq) v = __builtin_fma(L[i][kq], T4[kq][j], v);
                    T4[i][j] = -v * inv[i];
                }
            }
            // X[g][col] = (Muu^{-1} M[J, col])[g] = (T4^T (T4 pr))[g]
            double y4[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                double v = 0.0;
#pragma unroll
                for (int l = 0; l <= i; ++l) v = __builtin_fma(T4[i][l], pr[l], v);
                y4[i] = v;
            }
            double xg = 0.0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                double v = 0.0;
#pragma unroll
                for (int l = i; l < 4; ++l) v = __builtin_fma(T4[l][i], y4[l], v);
                xg = (g == i) ? v : xg;
            }
            // rank-4 update of every row tile: M[16 a + c'][col] -= M[16 a + c'][J] X[J][col]
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                if (wv < 2 && a >= 2) continue;  // rows y of the [u; x] columns are never read
                Q[a] = mfma_f64(-avv[a], xg, Q[a]);
            }
            AUG_MARK(9 + 3 * blk);
            // records: L(i, j0 + l) = sum_l' M[i][j0 + l'] T4[l][l']
            if (rec) {
#pragma unroll
                for (int l = 0; l < 4; ++l) {
                    double v = 0.0;
#pragma unroll
                    for (int l2 = 0; l2 <= l; ++l2) v = __builtin_fma(mi[l2], T4[l][l2], v);
                    if (wv == 0) gstore(FRk + (long long)(j0 + l) * s + ir, ir >= j0 + l ? v : 0.0);
                    else gstore(Gk + (j0 + l) + lane * m, -v);
                }
            }
            if (tid == 2 * 64) {  // lu' = T4 lu, lu = M[J][aug]
#pragma unroll
                for (int l = 0; l < 4; ++l) {
                    double v = 0.0;
#pragma unroll
                    for (int l2 = 0; l2 <= l; ++l2) v = __builtin_fma(T4[l][l2], lu[l2], v);
                    gstore(FRk + (long long)s * m + j0 + l, v);
                    if (lpb) gstore(lpb + (long long)k * s + j0 + l, v);
                }
            }
            AUG_MARK(10 + 3 * blk);
        }
        }
        AUG_MARK(5);
        // ---- P_k diagonal check, factor cache (P_k packed lower, p_k) ----
        {
            bool bad = false;
            if (col >= m && col < s)
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int i = 16 * a + 4 * r + g;
                        if (i == col && psd_bad(Q[a][r])) bad = true;
                        if (Lcb && i >= col && i < s) gstore(Lcb + (long long)k * sh.ps + pidx(i - m, col - m, n), Q[a][r]);
                    }
            if (caug && lpb)
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int i = 16 * a + 4 * r + g;
                        if (i >= m && i < s) gstore(lpb + (long long)k * s + i, Q[a][r]);
                    }
            if (bad) s_bad = 1;
        }
        AUG_MARK(6);
        if (k > N0) in_store();  // this stage's inputs were last read before B2
        __syncthreads();  // B_end: inputs, flags
        AUG_MARK(7);
        if ((!ok || s_bad) && fail_stage < 0) fail_stage = k;
    }
    // ---- export the element ----
    double *eo = A.elem + (bi * S + seg) * (long long)(3 * n * n + 2 * n);
    double *eF = eo, *eC = eo + n * n, *ef = eo + 2 * n * n, *eP = ef + n, *ep = eP + n * n;
    if (col >= m && col < s)  // P (publish, then symmetrise)
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * a + 4 * r + g;
                if (i >= m && i < s) Xq[(i - m) + (col - m) * XLD] = Q[a][r];
            }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 16 * a + 4 * r + g;
            const bool xi = i >= m && i < s, yi = i >= s && i < D;
            if (xi && cy) eF[(col - s) + (i - m) * n] = last ? 0.0 : Q[a][r];  // F = (F^T)^T
            if (yi && cy) eC[(i - s) + (col - s) * n] = last ? 0.0 : -Q[a][r];
            if (xi && caug) ep[i - m] = Q[a][r];
            if (yi && caug) ef[i - s] = last ? 0.0 : Q[a][r];
        }
    __syncthreads();
    for (int q = tid; q < n * n; q += 256) {
        const int i = q % n, j = q / n;
        eP[q] = 0.5 * (Xq[i + j * XLD] + Xq[j + i * XLD]);
    }
    if (tid == 0) A.seg_status[bi * S + seg] = fail_stage < 0 ? 0 : fail_stage + 1;
}

// Kernel for this shape: tile order T = ceil((2 n + m) / 16), compile-time
// specialisations for the benchmark shapes.
static const void *aug_kernel(const Shape &sh) {
    const int D = sh.s + sh.n;
    if (sh.s > 32 || sh.N < 1) return nullptr;
    if (sh.n == 24 && sh.m == 8) return reinterpret_cast<const void *>(&k_seg_bwd_aug<4, 24, 8>);
    if (sh.n == 12 && sh.m == 4) return reinterpret_cast<const void *>(&k_seg_bwd_aug<2, 12, 4>);
    if (D <= 16) return reinterpret_cast<const void *>(&k_seg_bwd_aug<1, 0, 0>);
    if (D <= 32) return reinterpret_cast<const void *>(&k_seg_bwd_aug<2, 0, 0>);
    if (D <= 48) return reinterpret_cast<const void *>(&k_seg_bwd_aug<3, 0, 0>);
    return reinterpret_cast<const void *>(&k_seg_bwd_aug<4, 0, 0>);
}

// the 4-wave stage for 24/8 (PDPLQR_AUG_1WAVE: the one-wave k_seg_bwd_aug, A/B)
static bool aug_mw(const Shape &sh) { return sh.mw && sh.n == 24 && sh.m == 8; }

int seg_backward_slots(const Shape &sh, int device) {
    if (xl_shape(sh)) return xl_par_slots(device);
    if (wide_stage(sh)) return wide_seg_backward_slots(sh, device);
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
    if (aug_mw(sh)) {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_seg_bwd_aug_mw<24, 8>, 256, 0) != hipSuccess || per <= 0)
            per = 1;
        return cus * per;
    }
    const void *k = aug_kernel(sh);
    if (!k || hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, 64, 0) != hipSuccess || per <= 0) per = 1;
    return cus * per;
}

int launch_seg_backward(const SegArgs &a, hipStream_t st) {
    if (xl_shape(a.sh)) return launch_seg_backward_xl(a, st);
    if (wide_stage(a.sh)) return launch_seg_backward_wide(a, st);
    if (aug_mw(a.sh) && a.sh.N >= 1) {
        hipLaunchKernelGGL((k_seg_bwd_aug_mw<24, 8>), dim3((unsigned)(a.sh.batch * a.S)), dim3(256), 0, st, a);
        PDPLQR_HIP_TRY(hipGetLastError());
        return PDPLQR_OK;
    }
    const void *k = aug_kernel(a.sh);
    if (!k) {
        set_error("parallel solver: n + m > 32 is not supported by this build");
        return PDPLQR_ERR_UNSUPPORTED;
    }
    void *args[] = {const_cast<SegArgs *>(&a)};
    PDPLQR_HIP_TRY(hipLaunchKernel(k, dim3((unsigned)(a.sh.batch * a.S)), dim3(64), args, 0, st));
    return PDPLQR_OK;
}

}  // namespace pdplqr

#ifdef PDPLQR_COMB_PROFILE
extern "C" int pdplqr_debug_aug_times(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(pdplqr::g_aug_t), sizeof(unsigned long long) * 1024 * 16) == hipSuccess ? 0 : -2;
}
#endif
