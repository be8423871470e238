// solvers.hip -- dispatch of the protocol calls to the three solver kinds.
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "admm.hpp"
#include "parallel.hpp"
#include "solvers.hpp"

namespace pdplqr {

static int unsupported(const char *what) {
    set_error(std::string(what) + ": not implemented in this build");
    return PDPLQR_ERR_UNSUPPORTED;
}

// ---------------------------------------------------------------------------
// PARALLEL solver state (LQRParallelSolver, lqr_solver_parallel.hpp:19-238)
// ---------------------------------------------------------------------------
struct ParallelState {
    std::vector<int32_t> ref_start, ref_len;  // the reference's segmentation (:64-88)
    std::vector<int32_t> seg_start_h, seg_len_h;  // device segments (each reference segment refined)
    int S = 0;
    int32_t *seg_start = nullptr, *seg_len = nullptr, *seg_status = nullptr;
    double *G = nullptr, *elem = nullptr, *bufA = nullptr, *bufB = nullptr, *xhat = nullptr, *lam = nullptr;
    double *scan4 = nullptr;  // radix-4 scan scratch [b][S][2][es] (T = 1 shapes)
    double *mapA = nullptr, *mapB = nullptr, *vfun = nullptr;  // boundary maps (ping-pong), value functions
    const double *suf_final = nullptr;
    int *flag = nullptr;
    int xl_grid = 0;  // n + m > 64 or n > 64: workspace slots in h->xl_ws (kernels_xl_par.hip)
    // horizon shards
    double *left = nullptr, *right = nullptr, *gathered = nullptr;
    int gathered_cap = 0;
    double *rscan[2] = {nullptr, nullptr}, *rmaps = nullptr;  // rank suffix scan, rank maps
    int rcap = 0;
    int *has_suf = nullptr;
};

template <typename X>
static int palloc(pdplqr_handle h, X **p, size_t count) {
    *p = nullptr;
    if (count == 0) count = 1;
    void *q = nullptr;
    hipError_t e = hipMalloc(&q, count * sizeof(X));
    if (e != hipSuccess) {
        set_error(std::string("hipMalloc: ") + hipGetErrorString(e));
        return PDPLQR_ERR_ALLOC;
    }
    h->allocs.push_back(q);
    *p = reinterpret_cast<X *>(q);
    return PDPLQR_OK;
}

// Reference segmentation (lqr_solver_parallel.hpp:70-81): Nseg_i = int(N/(scale+ns-1))
// for i < ns-1, scale = 1.55 under load balancing; the last takes the remainder.
static bool ref_segmentation(int N, int ns, bool lb, std::vector<int32_t> &st, std::vector<int32_t> &len) {
    const double alpha = 1.55, scale = lb ? alpha : 1.0;
    st.assign(ns, 0);
    len.assign(ns, 0);
    for (int i = 0; i < ns; ++i) {
        st[i] = (i == 0) ? 0 : st[i - 1] + len[i - 1];
        len[i] = (i < ns - 1) ? (int)((double)N / (scale + ns - 1)) : N - st[i];
        if (len[i] < 1) return false;
    }
    return true;
}

static RiccatiArgs riccati_args(pdplqr_handle h) {
    RiccatiArgs a;
    a.sh = h->sh;
    a.E = h->E;
    a.c = h->c;
    a.Hw = h->Hw;
    a.hw = h->hw;
    a.KD = h->KD;
    a.Lc = h->Lc;
    a.lpc = h->lpc;
    a.status = h->status;
    a.tab_s = h->tab_s;
    a.tab_n = h->tab_n;
    a.xl_ws = h->xl_ws;
    return a;
}

static bool scan_sklansky(const Shape &sh);

static int parallel_init(pdplqr_handle h) {
    h->sh.mw = 1;
    const Shape &sh = h->sh;
    if (sh.s > 256) return unsupported("PARALLEL solver with n + m > 256");
    ParallelState *ps = new ParallelState();
    h->par = ps;
    const int ns = h->cfg.num_segments;
    if (h->cfg.condensed_type == PDPLQR_CONDENSED_CHOLESKY && ns < 2) {
        // condensed_system.hpp:230-236 reads workspace_[1] out of bounds for ns = 1
        set_error("CHOLESKY condensed system needs num_segments >= 2 (the reference reads out of bounds)");
        return PDPLQR_ERR_INVALID;
    }
    if (!ref_segmentation(sh.N, ns, h->cfg.load_balancing != 0, ps->ref_start, ps->ref_len)) {
        set_error("segmentation yields an empty segment (N < num_segments + 0.55, lqr_solver_parallel.hpp:77-78)");
        return PDPLQR_ERR_INVALID;
    }
    // device refinement: split every reference segment into pieces of <= Lsub
    // stages.  The number of device segments S per problem trades the serial
    // segment backward (N/S stages per wave, batch S waves over the resident
    // slots) against the suffix scan (log2 S rounds of batch S combines), the
    // boundary maps (one combine-sized round) and their composition (log2 S
    // rounds of one matrix product each):
    //     t(S) = a ceil(N/S) ceil(batch S / slots_bwd) + b (ceil(log2 S) + 1) ceil(batch S / slots_scan)
    //            + c ceil(log2 (S + 1))
    // with a, b, c the per-stage (backward + rollout), per-combine and
    // per-composition latencies of one wave (profiles/r01 c4_v12: a ~10 us,
    // b ~45 us, c ~5.5 us at 24/8; a ~10 us, b ~15 us for s <= 16).
    int Lsub = h->cfg.segment_len;
    const bool auto_len = Lsub <= 0;
    for (int family = 0; family < 2 && auto_len; ++family) {
        // family 0: the 4-wave kernels where they apply (Shape::mw); family 1
        // (only when family 0 ended with long segments): the one-wave kernels.
        // The 4-wave combine and stage need 256 threads and ~53 KB of LDS per
        // segment, so their resident slots run out first: at 24/8 the slice of
        // an 8-rank split (N = 8192) runs 0.48 ms on them against 0.59 one-wave,
        // but a whole N = 65536 horizon is cut into 505 segments of 130 stages
        // and runs 1.29 ms against 1.15 with the one-wave kernels' 1009 segments
        // of 65 (scripts/c4_variants.py, profiles/r03/c4_family.log).
        if (family == 1) {
            int longest = 0;
            for (int i = 0; i < ns; ++i)
                longest = std::max(longest, (ps->ref_len[i] + ((ps->ref_len[i] + Lsub - 1) / Lsub) - 1) /
                                                ((ps->ref_len[i] + Lsub - 1) / Lsub));
            if (longest <= 64) break;
            h->sh.mw = 0;
        }
        const double a = 10.0, b = sh.s <= 16 ? 15.0 : 45.0, cm = sh.s <= 16 ? 4.0 : 5.5;
        const long long sb = seg_backward_slots(sh, h->cfg.device), ss = seg_scan_slots(sh, h->cfg.device);
        const long long B = sh.batch;
        // device segments and the longest one for a sub-segment length L (every
        // reference segment is cut separately, so S can exceed N / L by up to ns)
        auto pieces = [&](int L, int &longest) {
            long long S = 0;
            longest = 0;
            for (int i = 0; i < ns; ++i) {
                const int p = (ps->ref_len[i] + L - 1) / L;
                S += p;
                longest = std::max(longest, (ps->ref_len[i] + p - 1) / p);
            }
            return S;
        };
        const bool sk = scan_sklansky(h->sh);  // (Sklansky rounds: S / 2 combines each)
        auto cost = [&](long long S, long long per) {
            const long long sc = sk ? (S + 1) / 2 : S;
            const long long rb = (B * S + sb - 1) / sb, rs = (B * sc + ss - 1) / ss;
            int lg = 0, lg1 = 0;
            while ((1LL << lg) < S) ++lg;
            while ((1LL << lg1) < S + 1) ++lg1;
            return a * per * rb + b * (lg + 1) * rs + cm * lg1;
        };
        int maxlen = 1;
        for (int i = 0; i < ns; ++i) maxlen = std::max(maxlen, (int)ps->ref_len[i]);
        int lg0;
        const long long S0 = pieces(maxlen, lg0);
        double bc = cost(S0, lg0);
        Lsub = maxlen;
        std::vector<long long> cand;
        for (long long S = 2; S <= sh.N; S <<= 1) cand.push_back(S);
        if (sb / B >= 1 && sb / B <= sh.N) cand.push_back(sb / B);
        for (long long St : cand) {
            // smallest L whose cut fits St segments: a target at the slot count
            // must not spill a few segments into a second residency round
            int lo = 1, hi = maxlen, dummy;
            while (lo < hi) {
                const int mid = (lo + hi) / 2;
                if (pieces(mid, dummy) <= St) hi = mid;
                else lo = mid + 1;
            }
            int longest;
            const long long S = pieces(lo, longest);
            if (longest < 4 && S > (long long)ns) continue;  // keep >= 4 stages per segment
            const double cS = cost(S, longest);
            if (cS < bc) {
                bc = cS;
                Lsub = lo;
            }
        }
    }
    for (int i = 0; i < ns; ++i) {
        const int pieces = (ps->ref_len[i] + Lsub - 1) / Lsub;
        const int base = ps->ref_len[i] / pieces, extra = ps->ref_len[i] % pieces;
        int st = ps->ref_start[i];
        for (int q = 0; q < pieces; ++q) {
            const int len = base + (q < extra ? 1 : 0);
            ps->seg_start_h.push_back(st);
            ps->seg_len_h.push_back(len);
            st += len;
        }
    }
    ps->S = (int)ps->seg_start_h.size();
    const long long B = sh.batch, S = ps->S, es = 3LL * sh.n * sh.n + 2LL * sh.n;
    int rc;
    if ((rc = palloc(h, &ps->seg_start, S)) || (rc = palloc(h, &ps->seg_len, S)) ||
        (rc = palloc(h, &ps->seg_status, B * S)) || (rc = palloc(h, &ps->G, B * sh.N * sh.m * sh.n)) ||
        (rc = palloc(h, &ps->elem, B * S * es)) || (rc = palloc(h, &ps->bufA, B * S * es)) ||
        (rc = palloc(h, &ps->bufB, B * S * es)) || (rc = palloc(h, &ps->xhat, B * (S + 1) * sh.n)) ||
        (seg_scan4_supported(sh.n) && (rc = palloc(h, &ps->scan4, B * S * 2 * es))) ||
        (rc = palloc(h, &ps->lam, B * (S + 1) * sh.n)) || (rc = palloc(h, &ps->flag, B)) ||
        (rc = palloc(h, &ps->mapA, B * (S + 1) * (sh.n * sh.n + sh.n))) ||
        (rc = palloc(h, &ps->mapB, B * (S + 1) * (sh.n * sh.n + sh.n))) ||
        (rc = palloc(h, &ps->vfun, B * (S + 1) * (sh.n * sh.n + sh.n))) ||
        (rc = palloc(h, &ps->left, B * es)) || (rc = palloc(h, &ps->right, B * es)) ||
        (rc = palloc(h, &ps->has_suf, 1)))
        return rc;
    if (xl_shape(sh) || xl_state(sh.n)) {  // the XL kernels' workspace slots
        ps->xl_grid = xl_par_slots(h->cfg.device);
        if ((rc = palloc(h, &h->xl_ws, (long long)ps->xl_grid * xl_par_slot_doubles(sh)))) return rc;
    }
    PDPLQR_HIP_TRY(hipMemcpy(ps->seg_start, ps->seg_start_h.data(), S * sizeof(int32_t), hipMemcpyHostToDevice));
    PDPLQR_HIP_TRY(hipMemcpy(ps->seg_len, ps->seg_len_h.data(), S * sizeof(int32_t), hipMemcpyHostToDevice));
    PDPLQR_HIP_TRY(hipMemset(ps->flag, 0, B * sizeof(int)));
    PDPLQR_HIP_TRY(hipMemset(ps->seg_status, 0, B * S * sizeof(int32_t)));
    return PDPLQR_OK;
}

// segment backward + suffix scan; `last_is_terminal` = 0 for a non-final
// horizon shard.
static int parallel_scans(pdplqr_handle h, int last_is_terminal);

// The suffix scan runs Sklansky rounds (half the combines of a Hillis-Steele
// round, same depth) on the shapes whose combine kernels stage their operands
// before storing (n <= 32) and that do not take the two-round k_seg_scan4
// launches (n <= 16: radix-4 Hillis-Steele).
static bool scan_sklansky(const Shape &sh) { return sh.n <= 32 && !seg_scan4_supported(sh.n); }
void graph_release(pdplqr_handle h);

static int parallel_backward(pdplqr_handle h, int last_is_terminal, bool fact = true) {
    ParallelState *ps = h->par;
    const Shape &sh = h->sh;
    SegArgs a;
    a.sh = sh;
    a.S = ps->S;
    a.seg_start = ps->seg_start;
    a.seg_len = ps->seg_len;
    a.last_is_terminal = last_is_terminal;
    a.E = h->E;
    a.c = h->c;
    a.Hw = h->Hw;
    a.hw = h->hw;
    a.FR = h->KD;
    a.G = ps->G;
    a.Lc = h->Lc;
    a.lpc = h->lpc;
    a.elem = ps->elem;
    a.seg_status = ps->seg_status;
    a.flag = ps->flag;  // reset by the segment backward itself
    a.xlw = h->xl_ws;
    a.xl_grid = ps->xl_grid;
    int rc = fact ? launch_seg_backward(a, h->stream) : launch_seg_backward_nofact(a, h->stream);
    if (rc) return rc;
    return parallel_scans(h, last_is_terminal);
}

// inclusive suffix scan of the segment elements (ceil(log2 S) rounds): entry i
// is the value function at the start of segment i
static int parallel_scans(pdplqr_handle h, int last_is_terminal) {
    ParallelState *ps = h->par;
    const Shape &sh = h->sh;
    const double *sin = ps->elem;
    double *bufs[2] = {ps->bufA, ps->bufB};
    int round = 0;
    const bool r4 = ps->scan4 != nullptr;  // two rounds per launch (k_seg_scan4)
    if (scan_sklansky(sh) && ps->S > 1) {
        // Sklansky rounds: the first into bufA, the later ones in place there
        for (int d = 1; d < ps->S; d <<= 1) {
            ScanArgs s;
            s.n = sh.n;
            s.S = ps->S;
            s.dist = d;
            s.terminal = last_is_terminal;
            s.in = d == 1 ? sin : ps->bufA;
            s.out = ps->bufA;
            s.flag = ps->flag;
            s.lu = h->cfg.condensed_type == PDPLQR_CONDENSED_LU;
            s.mw = sh.mw;
            s.sk = d == 1 ? 1 : 2;
            s.xlw = h->xl_ws;
            s.xl_grid = ps->xl_grid;
            int rc = launch_seg_scan(s, sh.batch, h->stream);
            if (rc) return rc;
        }
        ps->suf_final = ps->bufA;
        return PDPLQR_OK;
    }
    for (int d = 1; d < ps->S; d <<= (r4 ? 2 : 1), ++round) {
        ScanArgs s;
        s.n = sh.n;
        s.S = ps->S;
        s.dist = d;
        s.terminal = last_is_terminal;
        s.in = sin;
        s.out = bufs[round & 1];
        s.flag = ps->flag;
        s.lu = h->cfg.condensed_type == PDPLQR_CONDENSED_LU;
        s.scratch = ps->scan4;
        s.mw = sh.mw;
        s.xlw = h->xl_ws;
        s.xl_grid = ps->xl_grid;
        int rc = r4 ? launch_seg_scan4(s, sh.batch, h->stream) : launch_seg_scan(s, sh.batch, h->stream);
        if (rc) return rc;
        sin = s.out;
    }
    ps->suf_final = sin;
    return PDPLQR_OK;
}

// condensed forward: boundary maps under the suffix value functions, their
// prefix composition (ceil(log2 (S + 1)) rounds), then the segment rollouts
static int parallel_forward(pdplqr_handle h, const double *x0, double *ws, const double *left, const double *right,
                            int last_is_terminal, long long rstride = 0) {
    ParallelState *ps = h->par;
    const Shape &sh = h->sh;
    MapArgs ma;
    ma.n = sh.n;
    ma.S = ps->S;
    ma.elem = ps->elem;
    ma.suf = ps->suf_final;
    ma.left = left;
    ma.right = right;
    ma.rstride = rstride;
    ma.x0 = x0;
    ma.maps = ps->mapA;
    ma.vfun = ps->vfun;
    ma.xhat = ps->xhat;
    ma.lam = ps->lam;
    ma.flag = ps->flag;
    ma.lu = h->cfg.condensed_type == PDPLQR_CONDENSED_LU;
    ma.mw = sh.mw;
    ma.xlw = h->xl_ws;
    ma.xl_grid = ps->xl_grid;
    int rc = launch_seg_maps(ma, sh.batch, h->stream);
    if (rc) return rc;
    double *mb[2] = {ps->mapA, ps->mapB};
    int round = 0;
    const int radix = map_radix(sh.n, ps->S + 1);
    for (int d = 1; d < ps->S + 1; d *= radix, ++round) {
        MapScanArgs ms;
        ms.n = sh.n;
        ms.S = ps->S;
        ms.dist = d;
        ms.radix = radix;
        ms.in = mb[round & 1];
        ms.out = mb[(round + 1) & 1];
        ms.vfun = ps->vfun;
        ms.xhat = ps->xhat;
        ms.lam = ps->lam;
        ms.xlw = h->xl_ws;
        ms.xl_grid = ps->xl_grid;
        if ((rc = launch_map_scan(ms, sh.batch, h->stream))) return rc;
    }
    SegFwd sf;
    sf.S = ps->S;
    sf.seg_start = ps->seg_start;
    sf.seg_len = ps->seg_len;
    sf.last_is_terminal = last_is_terminal;
    sf.G = ps->G;
    sf.xhat = ps->xhat;
    sf.lam = ps->lam;
    return launch_riccati_forward_seg(sh, h->E, h->c, h->KD, sf, ws, h->stream);
}

// ---------------------------------------------------------------------------
int solver_init(pdplqr_handle h) {
    switch (h->cfg.solver) {
        case PDPLQR_SOLVER_SERIAL:
            if (h->sh.s > 256) return unsupported("SERIAL solver with n + m > 256");
            if (xl_shape(h->sh)) return palloc(h, &h->xl_ws, (size_t)h->sh.batch * xl_ws_doubles(h->sh));
            return PDPLQR_OK;
        case PDPLQR_SOLVER_PARALLEL:
            return parallel_init(h);
        default:
            return kkt_init(h);
    }
}

void solver_release(pdplqr_handle h) {
    graph_release(h);
    admm_release(h);
    delete h->par;
    h->par = nullptr;
    kkt_release(h);
}

int solver_on_model(pdplqr_handle h) {
    return h->cfg.solver == PDPLQR_SOLVER_KKT ? kkt_on_model(h) : PDPLQR_OK;
}

int solver_update(pdplqr_handle h, const double *ws, const double *ys, const double *zs, const double *irho,
                  double sigma) {
    if (h->cfg.solver == PDPLQR_SOLVER_KKT) return kkt_update(h, ws, ys, zs, irho, sigma);
    const bool cacheable = h->max_nc <= 0;
    const bool skipH = cacheable && h->hw_cached && h->hw_sigma == sigma;
    const int rc = launch_update_problem_data(h->sh, h->H, h->h, ws, ys, zs, irho, sigma, h->Hw, h->hw, h->gw,
                                              h->tab_s, h->tab_n, h->stream, skipH);
    h->hw_cached = rc == PDPLQR_OK && cacheable;
    h->hw_sigma = sigma;
    return rc;
}

// ---------------------------------------------------------------------------
// HIP graphs.  A protocol call issues a fixed sequence of launches whose
// arguments depend only on the handle and on the call's device pointers (the
// parallel solver: ~20 short kernels, launch-rate bound from the host).  The
// sequence is captured once per (pointer set, stream) and replayed with one
// hipGraphLaunch.  Host-side state the sequence sets is set outside the
// captured part.  Opt-in (PDPLQR_GRAPH=1): measured on MI355X the replay is
// not faster -- C2 (N = 1024 single problem, ~20 kernels) 0.169 ms issued
// directly vs 0.176 ms replayed; the GPU-side dispatch gap, not the host
// launch rate, separates the kernels.  A stream that cannot capture (the
// legacy null stream) falls back to direct issue.
// ---------------------------------------------------------------------------
void graph_release(pdplqr_handle h) {
    for (auto &g : h->graphs) {
        if (g.exec) (void)hipGraphExecDestroy(g.exec);
        g = pdplqr_handle_s::Graph{};
    }
}

template <class Issue>
static int run_graphed(pdplqr_handle h, int slot, const void *k1, const void *k2, Issue &&issue) {
    static const bool off = getenv("PDPLQR_GRAPH") == nullptr;
    if (off || !h->stream) return issue();
    auto &g = h->graphs[slot];
    if (g.exec && g.k1 == k1 && g.k2 == k2 && g.stream == h->stream) {
        PDPLQR_HIP_TRY(hipGraphLaunch(g.exec, h->stream));
        return PDPLQR_OK;
    }
    if (g.exec) {
        (void)hipGraphExecDestroy(g.exec);
        g = pdplqr_handle_s::Graph{};
    }
    if (hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal) != hipSuccess) {
        (void)hipGetLastError();
        return issue();
    }
    const int rc = issue();
    hipGraph_t graph = nullptr;
    const hipError_t e = hipStreamEndCapture(h->stream, &graph);
    if (rc || e != hipSuccess || !graph) {
        if (graph) (void)hipGraphDestroy(graph);
        (void)hipGetLastError();
        return rc ? rc : issue();  // capture failed: run the sequence directly
    }
    hipGraphExec_t exec = nullptr;
    const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (ei != hipSuccess) {
        (void)hipGetLastError();
        return issue();
    }
    g.exec = exec;
    g.k1 = k1;
    g.k2 = k2;
    g.stream = h->stream;
    PDPLQR_HIP_TRY(hipGraphLaunch(g.exec, h->stream));
    return PDPLQR_OK;
}

// the constraint row count shared by every stage k < N, or 0
static int uniform_nc(pdplqr_handle h) {
    const int N = h->sh.N;
    if (N < 1) return 0;
    const int nc = h->ncs[0];
    for (int k = 1; k < N; ++k)
        if (h->ncs[k] != nc) return 0;
    return nc;
}

int solver_backward(pdplqr_handle h, const double *rho) {
    if (h->cfg.solver == PDPLQR_SOLVER_PARALLEL) h->shard_last = 1;
    // the record form is host state: set outside the (replayable) launch sequence
    h->rec_gain = (h->cfg.solver == PDPLQR_SOLVER_SERIAL && schur_gain_record(riccati_args(h))) ||
                  (h->cfg.solver == PDPLQR_SOLVER_KKT && kkt_plain_rec_ehat(h));
    // the record form selects the backward kernel: it is part of the graph key
    // (a replay of the other form's capture would leave the record in the
    // layout the forward does not read)
    return run_graphed(h, 0, rho, reinterpret_cast<const void *>((intptr_t)(h->rec_gain ? 2 : 1)), [&]() -> int {
        if (h->cfg.solver == PDPLQR_SOLVER_KKT) return kkt_backward(h, rho);  // rho = inv_rho (qdldl_solver.hpp:88)
        if (h->cfg.solver == PDPLQR_SOLVER_SERIAL && h->max_nc > 0) {
            // the penalty inside the streamed backward (one pass, H~ / h~ penalised in place)
            const int nc = uniform_nc(h);
            if (nc > 0 && h->rec_gain) {
                RiccatiArgs a = riccati_args(h);
                a.D = h->D;
                a.rho = rho;
                a.gw = h->gw;
                a.d_off = h->d_off;
                a.y_off = h->y_off;
                a.nc_last = h->ncs[h->sh.N];
                const int rc = launch_riccati_backward_pen(a, nc, h->stream);
                if (rc != PDPLQR_ERR_UNSUPPORTED) return rc;
            }
        }
        int rc = launch_penalty(h->sh, h->D, rho, h->gw, h->Hw, h->hw, h->d_off, h->y_off, h->tab_s, h->tab_n, 1,
                                h->max_nc, h->stream);
        if (rc) return rc;
        if (h->cfg.solver == PDPLQR_SOLVER_PARALLEL) return parallel_backward(h, 1);
        return launch_riccati_backward(riccati_args(h), h->stream);
    });
}

int solver_backward_nofact(pdplqr_handle h, const double *rho) {
    const int last = h->shard_last;
    h->rec_gain = false;  // the nofact kernels write lu' into the L-form record
    return run_graphed(h, 1, rho, reinterpret_cast<const void *>((intptr_t)(last + 1)), [&]() -> int {
        int rc = launch_penalty(h->sh, h->D, rho, h->gw, h->Hw, h->hw, h->d_off, h->y_off, h->tab_s, h->tab_n, 0,
                                h->max_nc, h->stream);
        if (rc) return rc;
        // LQRParallelSolver::backward_without_factorization (lqr_solver_parallel.hpp:148-154)
        if (h->cfg.solver == PDPLQR_SOLVER_PARALLEL) return parallel_backward(h, last, false);
        return launch_riccati_backward_nofact(riccati_args(h), h->stream);
    });
}

int solver_backward_prepared(pdplqr_handle h) {
    const bool fact = h->Lc == nullptr || h->lpc == nullptr;
    if (h->cfg.solver == PDPLQR_SOLVER_PARALLEL) return parallel_backward(h, 1, fact);
    const RiccatiArgs a = riccati_args(h);
    h->rec_gain = fact && schur_gain_record(a);
    return fact ? launch_riccati_backward(a, h->stream) : launch_riccati_backward_nofact(a, h->stream);
}

// ADMM: the update of iteration it fused into the backward of it + 1
// (serial solver with cached factors; ERR_UNSUPPORTED otherwise)
int solver_nofact_admm(pdplqr_handle h, const AdmmArgs &a, bool check) {
    if (h->cfg.solver != PDPLQR_SOLVER_SERIAL) return PDPLQR_ERR_UNSUPPORTED;
    for (int k = 0; k < h->sh.N; ++k)
        if (h->ncs[k] != 4) return PDPLQR_ERR_UNSUPPORTED;
    if (h->ncs[h->sh.N] != 0) return PDPLQR_ERR_UNSUPPORTED;
    h->rec_gain = false;
    return launch_nofact_admm(riccati_args(h), a, check, h->stream);
}

int solver_forward(pdplqr_handle h, const double *x0, double *ws) {
    // a forward sequence captured for the other record form is stale
    auto &g = h->graphs[2];
    if (g.exec && h->graph_rec_gain != h->rec_gain) {
        (void)hipGraphExecDestroy(g.exec);
        g = pdplqr_handle_s::Graph{};
    }
    h->graph_rec_gain = h->rec_gain;
    return run_graphed(h, 2, x0, ws, [&]() -> int {
        if (h->cfg.solver == PDPLQR_SOLVER_KKT) return kkt_forward(h, x0, ws);
        if (h->cfg.solver == PDPLQR_SOLVER_PARALLEL) return parallel_forward(h, x0, ws, nullptr, nullptr, 1);
        if (h->rec_gain) {
            const int rc = launch_rollout_dma(h->sh, h->E, h->c, h->KD, x0, ws, h->stream, true);
            if (rc == PDPLQR_ERR_UNSUPPORTED) set_error("forward: the model changed layout since backward");
            return rc;
        }
        return launch_riccati_forward(h->sh, h->E, h->c, h->KD, x0, ws, h->stream);
    });
}

int solver_clear(pdplqr_handle) { return PDPLQR_OK; }

int solver_status(pdplqr_handle h, int32_t *flags) {
    const Shape &sh = h->sh;
    if (h->cfg.solver != PDPLQR_SOLVER_PARALLEL) {
        PDPLQR_HIP_TRY(hipMemcpy(flags, h->status, (size_t)sh.batch * sizeof(int32_t), hipMemcpyDeviceToHost));
        return PDPLQR_OK;
    }
    ParallelState *ps = h->par;
    std::vector<int32_t> st((size_t)sh.batch * ps->S), flag(sh.batch);
    PDPLQR_HIP_TRY(hipMemcpy(st.data(), ps->seg_status, st.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
    PDPLQR_HIP_TRY(hipMemcpy(flag.data(), ps->flag, flag.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
    for (int b = 0; b < sh.batch; ++b) {
        int v = 0;
        for (int i = 0; i < ps->S; ++i) v = std::max(v, (int)st[(size_t)b * ps->S + i]);
        // a failed condensed (segment) combine is reported as N + 2, the
        // analogue of the condensed backward returning false (condensed_system.hpp:217-226)
        flags[b] = v ? v : (flag[b] ? sh.N + 2 : 0);
    }
    return PDPLQR_OK;
}

}  // namespace pdplqr

using namespace pdplqr;

extern "C" {

int pdplqr_get_segments(pdplqr_handle h, int32_t *idx_start, int32_t *Nseg) {
    if (!h || !idx_start || !Nseg) return PDPLQR_ERR_INVALID;
    if (h->md) {  // the reference segmentation of the whole horizon (host arithmetic)
        std::vector<int32_t> st, len;
        if (!ref_segmentation(h->sh.N, h->cfg.num_segments, h->cfg.load_balancing != 0, st, len)) {
            set_error("segmentation yields an empty segment");
            return PDPLQR_ERR_INVALID;
        }
        for (size_t i = 0; i < st.size(); ++i) {
            idx_start[i] = st[i];
            Nseg[i] = len[i];
        }
        return PDPLQR_OK;
    }
    if (h->cfg.solver != PDPLQR_SOLVER_PARALLEL || !h->par) {
        set_error("get_segments needs a PARALLEL handle");
        return PDPLQR_ERR_INVALID;
    }
    for (size_t i = 0; i < h->par->ref_start.size(); ++i) {
        idx_start[i] = h->par->ref_start[i];
        Nseg[i] = h->par->ref_len[i];
    }
    return PDPLQR_OK;
}

int pdplqr_shard_element_size(pdplqr_handle h) {
    if (!h) return PDPLQR_ERR_INVALID;
    return 3 * h->sh.n * h->sh.n + 2 * h->sh.n;
}

// Horizon shards: this handle holds one slice of the
// horizon.  Backward = segment recursion + local scans; the slice element is the
// suffix-scan entry 0 (e_0 (x) ... (x) e_{S-1}).  Elements: [batch][3n^2+2n].
static int shard_backward_common(pdplqr_handle h, const double *rho, int is_last_shard, double *elem_out, int mem,
                                 bool fact) {
    if (!h || !elem_out) return PDPLQR_ERR_INVALID;
    if (h->cfg.solver != PDPLQR_SOLVER_PARALLEL || !h->par) {
        set_error("shard_backward needs a PARALLEL handle");
        return PDPLQR_ERR_INVALID;
    }
    if (!h->updated) {
        set_error("shard_backward before update_problem_data");
        return PDPLQR_ERR_STATE;
    }
    if (!fact && (!h->factored || !h->Lc)) {
        set_error("shard_backward_without_factorization needs keep_factors = 1 and a preceding shard_backward");
        return PDPLQR_ERR_STATE;
    }
    if (!fact && (is_last_shard ? 1 : 0) != h->shard_last) {
        set_error("shard_backward_without_factorization: is_last_shard differs from the factorising call's");
        return PDPLQR_ERR_INVALID;
    }
    PDPLQR_HIP_TRY(hipSetDevice(h->cfg.device));
    const Shape &sh = h->sh;
    const double *drho = h->st_rho;
    if (sh.ny > 0) {
        if (!rho) return PDPLQR_ERR_INVALID;
        if (mem == PDPLQR_MEM_DEVICE) drho = rho;
        else PDPLQR_HIP_TRY(hipMemcpyAsync(h->st_rho, rho, (size_t)sh.batch * sh.ny * sizeof(double),
                                           hipMemcpyHostToDevice, h->stream));
    }
    // backward: H~ += D^T rho D and h~ -= D^T rho g; without factorization only
    // the linear term (lqr_kernel.hpp:106-112, 150-158)
    int rc = launch_penalty(sh, h->D, drho, h->gw, h->Hw, h->hw, h->d_off, h->y_off, h->tab_s, h->tab_n, fact ? 1 : 0,
                            h->max_nc, h->stream);
    if (rc) return rc;
    if ((rc = parallel_backward(h, is_last_shard ? 1 : 0, fact))) return rc;
    h->shard_last = is_last_shard ? 1 : 0;
    ParallelState *ps = h->par;
    const long long es = 3LL * sh.n * sh.n + 2LL * sh.n;
    // suffix entry 0 of every problem: suf_final[b][0] (rows of es at pitch S es)
    PDPLQR_HIP_TRY(hipMemcpy2DAsync(elem_out, (size_t)es * sizeof(double), ps->suf_final,
                                    (size_t)ps->S * es * sizeof(double), (size_t)es * sizeof(double),
                                    (size_t)sh.batch,
                                    mem == PDPLQR_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                                    h->stream));
    if (mem != PDPLQR_MEM_DEVICE) PDPLQR_HIP_TRY(hipStreamSynchronize(h->stream));
    if (fact) h->factored = true;
    return PDPLQR_OK;
}

int pdplqr_shard_backward(pdplqr_handle h, const double *rho, int is_last_shard, double *elem_out, int mem) {
    return shard_backward_common(h, rho, is_last_shard, elem_out, mem, true);
}

// LQRParallelSolver::backward_without_factorization (lqr_solver_parallel.hpp:
// 148-154,190-211) on one slice: the segment factorizations and the condensed
// (F, C, P) are reused; the element's f, p are new (F, C, P bit-identical to
// the factorising call's), so a rank exchange needs only f, p (2n doubles).
int pdplqr_shard_backward_without_factorization(pdplqr_handle h, const double *rho, int is_last_shard,
                                                double *elem_out, int mem) {
    return shard_backward_common(h, rho, is_last_shard, elem_out, mem, false);
}

// elems_all: [num_shards][batch][3n^2+2n] (rank-major, the all-gather output).
int pdplqr_shard_forward(pdplqr_handle h, const double *x0, const double *elems_all, int32_t num_shards,
                         int32_t shard_id, double *ws, int mem) {
    if (!h || !x0 || !elems_all || !ws) return PDPLQR_ERR_INVALID;
    if (h->cfg.solver != PDPLQR_SOLVER_PARALLEL || !h->par) {
        set_error("shard_forward needs a PARALLEL handle");
        return PDPLQR_ERR_INVALID;
    }
    if (num_shards < 1 || shard_id < 0 || shard_id >= num_shards) {
        set_error("shard_forward: bad shard index");
        return PDPLQR_ERR_INVALID;
    }
    if (!h->factored) {
        set_error("shard_forward before shard_backward");
        return PDPLQR_ERR_STATE;
    }
    PDPLQR_HIP_TRY(hipSetDevice(h->cfg.device));
    const Shape &sh = h->sh;
    ParallelState *ps = h->par;
    const long long es = 3LL * sh.n * sh.n + 2LL * sh.n;
    const double *dx0 = x0, *delems = elems_all;
    if (mem != PDPLQR_MEM_DEVICE) {
        if (!ps->gathered) {
            int rc = palloc(h, &ps->gathered, (long long)num_shards * sh.batch * es);
            if (rc) return rc;
            ps->gathered_cap = num_shards;
        } else if (ps->gathered_cap < num_shards) {
            set_error("shard_forward: number of shards grew between calls");
            return PDPLQR_ERR_INVALID;
        }
        PDPLQR_HIP_TRY(hipMemcpyAsync(ps->gathered, elems_all, (size_t)num_shards * sh.batch * es * sizeof(double),
                                      hipMemcpyHostToDevice, h->stream));
        PDPLQR_HIP_TRY(hipMemcpyAsync(h->st_x0, x0, (size_t)sh.batch * sh.n * sizeof(double), hipMemcpyHostToDevice,
                                      h->stream));
        delems = ps->gathered;
        dx0 = h->st_x0;
    }
    // Fold of the gathered rank elements.  Chain (k_fold_shards): the longer of
    // the prefix / suffix chains, max(r - 1, R - r - 2) sequential combines.
    // Scan: the rank suffix scan (ceil(log2 R) rounds of k_seg_scan, every
    // suffix entry) plus, for r > 0, the rank boundary maps (one combine-sized
    // round) and their matrix-vector chain.  Tree (4-wave combines, CHOLESKY
    // form): the prefix and suffix lists reduced pairwise, max(ceil(log2 r),
    // ceil(log2(R - 1 - r))) levels and nothing after them (k_seg_maps maps x0
    // through the prefix as in the chain form).  The shortest one runs;
    // PDPLQR_SHARD_FOLD=chain|scan|tree forces one (diagnostics and tests).
    const int R = num_shards, r = shard_id;
    const bool lu = h->cfg.condensed_type == PDPLQR_CONDENSED_LU;
    int lgR = 0;
    while ((1 << lgR) < R) ++lgR;
    bool use_scan = lgR + (r > 0 ? 1 : 0) < std::max(r - 1, R - r - 2);
    // with the 4-wave scan rounds (seg_scan_mw) a round costs about half a
    // one-wave chain combine: the log-depth forms win for every rank
    bool use_tree = R > 1 && seg_scan_mw(sh.n, lu) && !wide_state(sh.n);
    if (const char *f = getenv("PDPLQR_SHARD_FOLD")) {
        use_tree = use_tree && f[0] == 't';
        use_scan = R > 1 && f[0] == 's';
    }
    if (sh.n > 32) use_scan = R > 1;  // the n > 32 element kernels fold by the scan form only
    int rc;
    const double *left = nullptr, *right = nullptr;
    long long rstride = 0;
    if (use_tree) {
        if (ps->rcap < R) {
            if ((rc = palloc(h, &ps->rscan[0], (long long)sh.batch * R * es)) ||
                (rc = palloc(h, &ps->rscan[1], (long long)sh.batch * R * es)) ||
                (rc = palloc(h, &ps->rmaps, (long long)sh.batch * R * (sh.n * sh.n + sh.n))))
                return rc;
            ps->rcap = R;
        }
        const long long gstride = (long long)sh.batch * es;
        RankTreeArgs ta;
        ta.n = sh.n;
        ta.R = R;
        ta.r = r;
        ta.gathered = delems;
        ta.gstride = gstride;
        ta.left = ps->left;
        ta.right = ps->right;
        ta.flag = ps->flag;
        for (ta.level = 0; rank_tree_blocks(r, ta.level) + rank_tree_blocks(R - 1 - r, ta.level) > 0; ++ta.level) {
            ta.in = ps->rscan[(ta.level + 1) & 1];
            ta.out = ps->rscan[ta.level & 1];
            if ((rc = launch_rank_tree(ta, sh.batch, h->stream))) return rc;
        }
        // a one-element list is the gathered element itself
        if (r == 1) left = delems;
        else if (r > 1) left = ps->left;
        if (r == R - 2) right = delems + (long long)(R - 1) * gstride;
        else if (r < R - 2) right = ps->right;
    } else if (use_scan) {
        if (ps->rcap < R) {
            if ((rc = palloc(h, &ps->rscan[0], (long long)sh.batch * R * es)) ||
                (rc = palloc(h, &ps->rscan[1], (long long)sh.batch * R * es)) ||
                (rc = palloc(h, &ps->rmaps, (long long)sh.batch * R * (sh.n * sh.n + sh.n))))
                return rc;
            ps->rcap = R;
        }
        const double *sin = delems;
        int round = 0;
        for (int d = 1; d < R; d <<= 1, ++round) {
            ScanArgs sa;
            sa.n = sh.n;
            sa.S = R;
            sa.dist = d;
            sa.terminal = 1;  // the last rank's element ends at the real terminal
            sa.in = sin;
            if (round == 0) {  // rank-major all-gather layout [R][batch][es]
                sa.istride = (long long)sh.batch * es;
                sa.bstride = es;
            }
            sa.out = ps->rscan[round & 1];
            sa.flag = ps->flag;
            sa.lu = lu;
            sa.xlw = h->xl_ws;
            sa.xl_grid = ps->xl_grid;
            if ((rc = launch_seg_scan(sa, sh.batch, h->stream))) return rc;
            sin = sa.out;
        }
        if (r + 1 < R) {
            right = sin + (long long)(r + 1) * es;
            rstride = (long long)R * es;
        }
        if (r > 0) {
            if ((rc = launch_rank_fold_maps(delems, sin, dx0, R, r, sh.n, sh.batch, ps->rmaps, ps->left, ps->flag,
                                            h->cfg.condensed_type == PDPLQR_CONDENSED_LU, h->stream, h->xl_ws,
                                            ps->xl_grid)))
                return rc;
            left = ps->left;
        }
    } else if (R > 1) {
        rc = launch_fold_shards(delems, num_shards, shard_id, sh.n, sh.batch, ps->left, ps->right, ps->has_suf,
                                ps->flag, h->cfg.condensed_type == PDPLQR_CONDENSED_LU, h->stream);
        if (rc) return rc;
        left = shard_id > 0 ? ps->left : nullptr;
        right = shard_id + 1 < num_shards ? ps->right : nullptr;
    }
    double *dws = mem == PDPLQR_MEM_DEVICE ? ws : h->st_ws;
    if ((rc = parallel_forward(h, dx0, dws, left, right, h->shard_last, rstride))) return rc;
    if (mem != PDPLQR_MEM_DEVICE) {
        PDPLQR_HIP_TRY(hipMemcpyAsync(ws, dws, (size_t)sh.batch * sh.perh * sizeof(double), hipMemcpyDeviceToHost,
                                      h->stream));
        PDPLQR_HIP_TRY(hipStreamSynchronize(h->stream));
    }
    return PDPLQR_OK;
}

}  // extern "C"

// Internal diagnostics (not part of include/pdplqr.h): copy a PARALLEL
// handle's segment buffers to host.  which: 0 elem, 1 boundary value functions [b][S+1][n^2+n], 2 suffix
// scan, 3 xhat [b][S+1][n], 4 lam, 5 device segment starts/lengths (int32 pairs).
extern "C" int pdplqr_debug_parallel(pdplqr_handle h, int which, void *out, long long bytes) {
    if (!h || !h->par) return PDPLQR_ERR_INVALID;
    ParallelState *ps = h->par;
    PDPLQR_HIP_TRY(hipStreamSynchronize(h->stream));
    const void *src = nullptr;
    switch (which) {
        case 0: src = ps->elem; break;
        case 1: src = ps->vfun; break;
        case 2: src = ps->suf_final; break;
        case 3: src = ps->xhat; break;
        case 4: src = ps->lam; break;
        case 5: {
            int32_t *o = reinterpret_cast<int32_t *>(out);
            for (int i = 0; i < ps->S && (long long)(2 * i + 1) * 4 < bytes; ++i) {
                o[2 * i] = ps->seg_start_h[i];
                o[2 * i + 1] = ps->seg_len_h[i];
            }
            return ps->S;
        }
        default: return PDPLQR_ERR_INVALID;
    }
    PDPLQR_HIP_TRY(hipMemcpy(out, src, (size_t)bytes, hipMemcpyDeviceToHost));
    return ps->S;
}
