// parallel.hpp -- argument blocks of the parallel (segmented) solver kernels.
#pragma once
#include "internal.hpp"

namespace pdplqr {

struct SegArgs {
    Shape sh;
    int S;                    // device segments per problem
    const int32_t *seg_start;  // [S]
    const int32_t *seg_len;    // [S]
    int last_is_terminal;      // 1: the last segment ends at the real terminal node N
    const double *E, *c, *Hw, *hw;
    double *FR, *G;            // rollout records [b][N][s m + m], coupling gains [b][N][m n]
    double *Lc, *lpc;          // factor cache (nullable)
    double *elem;              // [b][S][3 n^2 + 2 n]
    int32_t *seg_status;       // [b][S]
    int serial = 0;            // k_seg_bwd_wide as the serial value-form backward: one segment [0, N),
                               // no element, status per problem (seg_start / seg_len unused)
    int *flag = nullptr;       // [b] the scans' / maps' failure flag: zeroed by segment 0's block
                               // (the later kernels of the solve set it; no memset launch)
    double *xlw = nullptr;     // n + m > 64 (kernels_xl_par.hip): xl_grid workspace slots of
    int xl_grid = 0;           // xl_par_slot_doubles each, the blocks striding over the items
};

struct ScanArgs {
    int n, S, dist;
    int terminal;              // the last element ends at the real terminal (F = C = f = 0)
    const double *in;          // suffix scan ping-pong [b][S][es]
    long long istride = 0, bstride = 0;  // element / problem strides of `in` (0: [b][S][es])
    double *out;
    int *flag;                 // [b]: a combine was not positive definite
    int lu = 0;                // LU form of the combine (CondensedSystemSolverType::LU)
    double *scratch = nullptr; // radix-4 rounds: two private element slots per block [b][S][2][es]
    int mw = 1;                // the 4-wave combine may run (Shape::mw)
    // Round form.  0: Hillis-Steele (every entry i < S - dist combines with
    // i + dist; in -> out ping-pong).  Sklansky (the same ceil(log2 S) rounds,
    // half the combines per round): 1 = the first round (dist 1; in -> out,
    // entries without a partner copied), 2 = a later round, in place (in == out):
    // entry i in the lower half of its 2 dist block combines with the first
    // entry j of the upper half, which already holds [j, j + dist - 1].
    int sk = 0;
    double *xlw = nullptr;     // n > 64: workspace slots (SegArgs::xlw)
    int xl_grid = 0;
};

// Blocks per problem of one scan round.
__host__ __device__ inline int scan_round_blocks(int S, int dist, int sk) {
    return sk == 2 ? dist * ((S - dist + 2 * dist - 1) / (2 * dist)) : S;
}

// Operands of block q of a round: the result goes to entry i, the right
// operand is entry j (j < 0: entry i is copied / kept, no combine); false when
// the block has nothing to do.  The right operand covers [j, min(j + dist - 1,
// S - 1)] in every form.
__host__ __device__ inline bool scan_round_operands(int S, int dist, int sk, int q, int &i, int &j) {
    if (sk == 2) {
        const int blk = q / dist, pos = q % dist;
        i = blk * 2 * dist + pos;
        j = blk * 2 * dist + dist;
        return j < S;
    }
    if (sk == 1) {
        // the S / 2 combines (2 k, 2 k + 1) take the first blocks, the copies of
        // the unpaired entries the rest: the dispatcher hands consecutive blocks
        // to different CUs, so the combines -- the round's critical path -- get
        // a CU each before any copy block lands next to one
        const int nc = S >> 1;
        if (q < nc) {
            i = 2 * q;
            j = i + 1;
        } else {
            const int k = q - nc;
            i = 2 * k + 1 < S ? 2 * k + 1 : S - 1;  // odd entries, then the last one of an odd S
            j = -1;
        }
        return true;
    }
    i = q;
    j = i + dist < S ? i + dist : -1;
    return true;
}

struct MapArgs {
    int n, S;
    const double *elem;        // segment elements [b][S][es]
    const double *suf;         // inclusive suffix scan [b][S][es]
    const double *left;        // optional global prefix element [b][es] (horizon shards)
    const double *right;       // optional global suffix element [b][es]
    long long rstride = 0;     // problem stride of `right` (0: es)
    const double *x0;          // [b][n]
    double *maps;              // [b][S+1][n^2 + n]  boundary maps (Phi | phi)
    double *vfun;              // [b][S+1][n^2 + n]  value functions at the boundaries (P | p)
    double *xhat, *lam;        // [b][S+1][n]
    int *flag;
    int lu = 0;                // LU form of the combine
    int mw = 1;                // the 4-wave kernels may run (Shape::mw)
    double *xlw = nullptr;     // n > 64: workspace slots (SegArgs::xlw)
    int xl_grid = 0;
};

struct MapScanArgs {
    int n, S, dist;
    int radix = 4;             // this solve's composition radix (map_radix; 4 for the wide / XL kernels)
    const double *in;          // [b][S+1][n^2 + n]
    double *out;
    const double *vfun;
    double *xhat, *lam;
    double *xlw = nullptr;     // n > 64: workspace slots (SegArgs::xlw)
    int xl_grid = 0;
};

// Rank fold of a horizon shard as two pairwise reduction trees over the
// all-gathered rank elements (k_rank_tree_mw): the prefix list e_0 .. e_{r-1}
// and the suffix list e_{r+1} .. e_{R-1} of rank r, one launch per level.
// At level l a list of m partials pairs entries (2k, 2k + 1); an odd last
// entry is carried.  Partials of level l > 0 live in `in` [b][R][es] at slot
// k (prefix) or R / 2 + k (suffix); a list's last level writes `left` /
// `right` [b][es].
struct RankTreeArgs {
    int n, R, r, level;
    const double *gathered;    // [R][b][es] (rank-major all-gather)
    long long gstride;         // rank stride of `gathered` (b * es)
    const double *in;          // level l > 0: the partials of level l - 1
    double *out;               // partials of this level
    double *left, *right;      // [b][es] prefix (F, C, f) / suffix (P, p) results
    int *flag;
};

__host__ __device__ inline int rank_tree_len(int m0, int level) {
    int m = m0;
    for (int l = 0; l < level; ++l) m = (m + 1) >> 1;
    return m;
}
// blocks per problem of a list at `level` (0 when the list is done or empty)
__host__ __device__ inline int rank_tree_blocks(int m0, int level) {
    const int m = rank_tree_len(m0, level);
    return m > 1 ? (m + 1) >> 1 : 0;
}

// What block q (of one problem) does at `level`: combine operands a (earlier)
// and b (later) of the prefix (suf = false) or suffix list -- at level 0 rank
// indices into the all-gather, later the partial slots of `in` -- or carry a
// alone (carry); the result goes to partial slot dst, or to left / right when
// dst < 0.  fcf = false: b holds the real terminal (the suffix list's last
// partial), only P, p are formed.
struct RankTreeOp {
    bool suf, carry, fcf;
    int a, b, dst;
};
__host__ __device__ inline RankTreeOp rank_tree_op(int R, int r, int level, int q) {
    const int mp0 = r, ms0 = R - 1 - r;
    const int bp = rank_tree_blocks(mp0, level);
    RankTreeOp op;
    op.suf = q >= bp;
    const int k = op.suf ? q - bp : q, m0 = op.suf ? ms0 : mp0;
    const int m = rank_tree_len(m0, level);
    const int base = level == 0 ? (op.suf ? r + 1 : 0) : (op.suf ? R / 2 : 0);
    op.a = base + 2 * k;
    op.carry = 2 * k + 1 >= m;
    op.b = op.carry ? -1 : op.a + 1;
    op.fcf = !(op.suf && 2 * k + 1 == m - 1);
    op.dst = rank_tree_len(m0, level + 1) == 1 ? -1 : (op.suf ? R / 2 : 0) + k;
    return op;
}

struct SegFwd {
    int S;
    const int32_t *seg_start, *seg_len;
    int last_is_terminal;
    const double *G;           // [b][N][m n]
    const double *xhat, *lam;  // [b][S+1][n]
};

int launch_seg_backward(const SegArgs &a, hipStream_t st);
int seg_backward_slots(const Shape &sh, int device);
int seg_scan_slots(const Shape &sh, int device);
int launch_seg_backward_nofact(const SegArgs &a, hipStream_t st);
int launch_seg_scan(const ScanArgs &a, int batch, hipStream_t st);
// one launch = the two Hillis-Steele rounds at distances dist and 2 dist (two
// waves per block); false when this shape keeps the radix-2 rounds
bool seg_scan4_supported(int n);
bool seg_scan_mw(int n, bool lu, int mw = 1);  // the 4-wave combine runs the scan rounds
int launch_seg_scan4(const ScanArgs &a, int batch, hipStream_t st);
int launch_seg_maps(const MapArgs &a, int batch, hipStream_t st);
// Composition radix of the boundary-map prefix scan (2 or 4).
#ifndef PDPLQR_MAP_RADIX
#define PDPLQR_MAP_RADIX 4
#endif
int launch_map_scan(const MapScanArgs &a, int batch, hipStream_t st);
// radix of the boundary-map composition for n-state maps over J = S + 1 entries
int map_radix(int n, int J);
int launch_fold_shards(const double *elems, int R, int r, int n, int batch, double *out_pre, double *out_suf,
                       int *has_suf, int *flag, bool lu, hipStream_t st);
int launch_rank_fold_maps(const double *elems, const double *suf, const double *x0, int R, int r, int n, int batch,
                          double *maps, double *out_pre, int *flag, bool lu, hipStream_t st, double *xlw = nullptr,
                          int xl_grid = 0);
int launch_rank_tree(const RankTreeArgs &a, int batch, hipStream_t st);
// wide shapes (kernels_wide.hip): 32 < n + m <= 64 stage kernels, 32 < n element kernels
bool wide_state(int n);
bool wide_stage(const Shape &sh);
int wide_seg_backward_slots(const Shape &sh, int device);
int wide_scan_slots(int n, int device);
int launch_seg_backward_wide(const SegArgs &a, hipStream_t st);
int launch_seg_scan_wide(const ScanArgs &a, int batch, hipStream_t st);
int launch_seg_maps_wide(const MapArgs &a, int batch, hipStream_t st);
int launch_map_scan_wide(const MapScanArgs &a, int batch, hipStream_t st);
int launch_debug_combine_wide(const double *a, const double *b, double *out, int n, int *ok, bool lu);
int launch_rank_fold_maps_wide(const double *elems, const double *suf, const double *x0, int R, int r, int n,
                               int batch, double *maps, double *out_pre, int *flag, bool lu, hipStream_t st);
int launch_riccati_forward_seg_big(const Shape &sh, const double *E, const double *c, const double *FR,
                                   const SegFwd &sf, double *ws, hipStream_t st);
int launch_riccati_forward_seg(const Shape &sh, const double *E, const double *c, const double *FR, const SegFwd &sf,
                               double *ws, hipStream_t st);
// n + m > 64 stage kernels, n > 64 element kernels (kernels_xl_par.hip): global
// workspace slots, each block striding over the items
__host__ __device__ inline bool xl_state(int n) { return n > 64; }
// doubles of one workspace slot: the stage kernels' P, F, C (n x n), P E~, F E~
// (n x s), M (s x s); the element kernels' five n x n buffers
__host__ __device__ inline long long xl_par_slot_doubles(const Shape &sh) {
    const long long n = sh.n, s = sh.s;
    long long d = 0;
    if (sh.s > 64) d = 3 * n * n + 2 * n * s + s * s;
    if (sh.n > 64) d = d > 5 * n * n ? d : 5 * n * n;
    return d;
}
int xl_par_slots(int device);  // workspace slots (blocks) of the XL parallel kernels
int launch_seg_backward_xl(const SegArgs &a, hipStream_t st);
int launch_seg_backward_nofact_xl(const SegArgs &a, hipStream_t st);
int launch_seg_scan_xl(const ScanArgs &a, int batch, hipStream_t st);
int launch_seg_maps_xl(const MapArgs &a, int batch, hipStream_t st);
int launch_map_scan_xl(const MapScanArgs &a, int batch, hipStream_t st);
int launch_rank_fold_maps_xl(const double *elems, const double *suf, const double *x0, int R, int r, int n, int batch,
                             double *maps, double *out_pre, int *flag, bool lu, double *xlw, int xl_grid,
                             hipStream_t st);
int launch_riccati_forward_seg_xl(const Shape &sh, const double *E, const double *c, const double *FR,
                                  const SegFwd &sf, double *ws, hipStream_t st);

}  // namespace pdplqr
