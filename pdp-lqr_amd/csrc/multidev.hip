// multidev.hip -- one process drives several GPUs: the horizon of a PARALLEL
// handle split into contiguous slices, one per device (pdplqr_config.devices,
// SURVEY.md 8(b)).  The multi-GPU form of LQRParallelSolver
// (lqr_solver_parallel.hpp:22-25,142-146,213-238) for a C / C++ caller that has
// no torch.distributed: each slice is a PARALLEL shard handle on its device
// (segment backward + local suffix scan -> the slice element, solvers.hip
// pdplqr_shard_backward); the R elements (3n^2 + 2n doubles per problem) are
// all-gathered over RCCL (ncclAllGather on ncclCommInitAll communicators, one
// group call across the devices' streams); each shard then folds the gathered
// elements and rolls out its slice (pdplqr_shard_forward).
//
// The driver only slices and assembles: the per-slice numerics are the shard
// API's, which tests/test_gpu_horizon.py checks against the serial oracle.
// Devices may repeat (a same-device rehearsal): the exchange then goes through
// device copies instead of RCCL (which needs distinct devices); so does
// PDPLQR_MD_P2P=1.  RCCL is loaded with dlopen on first use, so the library
// carries no link-time RCCL dependency.
#include <dlfcn.h>
#include <stdlib.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

#include "internal.hpp"
#include "solvers.hpp"

namespace pdplqr {

// ---------------------------------------------------------------------------
// the slicing plan (host only; also exported for tests)
// ---------------------------------------------------------------------------
// Slice r = [N0, N1): the first N % R slices one stage longer (pdplqr/horizon.py
// split_horizon).  Row / D offsets follow from ncs; only the last slice keeps
// the terminal's rows (the others end at the dummy zero terminal,
// lqr_kernel_parallel.hpp:60-66).
void md_plan(int N, int R, const std::vector<int32_t> &ncs, int n, int m, std::vector<MdSlice> &out) {
    const int s = n + m;
    std::vector<long long> yo(N + 2, 0), dof(N + 2, 0);
    for (int k = 0; k <= N; ++k) {
        yo[k + 1] = yo[k] + ncs[k];
        dof[k + 1] = dof[k] + (long long)ncs[k] * (k < N ? s : n);
    }
    out.assign(R, MdSlice{});
    const int base = N / R, extra = N % R;
    int st = 0;
    for (int r = 0; r < R; ++r) {
        MdSlice &p = out[r];
        p.N0 = st;
        p.N1 = st + base + (r < extra ? 1 : 0);
        st = p.N1;
        p.last = r == R - 1;
        p.y0 = yo[p.N0];
        p.ny_st = yo[p.N1] - yo[p.N0];
        p.nc_term = p.last ? ncs[N] : 0;
        p.d0 = dof[p.N0];
        p.nd_st = dof[p.N1] - dof[p.N0];
        p.ncs.assign(ncs.begin() + p.N0, ncs.begin() + p.N1);
        p.ncs.push_back(p.nc_term);
    }
}

// ---------------------------------------------------------------------------
// RCCL, resolved at run time
// ---------------------------------------------------------------------------
namespace {
typedef void *ncclComm_t;
typedef int (*fn_init_all)(ncclComm_t *, int, const int *);
typedef int (*fn_all_gather)(const void *, void *, size_t, int, ncclComm_t, hipStream_t);
typedef int (*fn_group)();
typedef int (*fn_destroy)(ncclComm_t);
typedef const char *(*fn_err)(int);
constexpr int NCCL_FLOAT64 = 8;  // ncclDouble (rccl.h ncclDataType_t)

struct Rccl {
    void *so = nullptr;
    fn_init_all init_all = nullptr;
    fn_all_gather all_gather = nullptr;
    fn_group group_start = nullptr, group_end = nullptr;
    fn_destroy destroy = nullptr;
    fn_err err = nullptr;
    // once per process (handles may be created on several threads)
    bool load() {
        static std::once_flag once;
        std::call_once(once, [this] { resolve(); });
        return ok;
    }
    bool ok = false;
    void resolve() {
        so = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!so) so = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!so) return;
        init_all = (fn_init_all)dlsym(so, "ncclCommInitAll");
        all_gather = (fn_all_gather)dlsym(so, "ncclAllGather");
        group_start = (fn_group)dlsym(so, "ncclGroupStart");
        group_end = (fn_group)dlsym(so, "ncclGroupEnd");
        destroy = (fn_destroy)dlsym(so, "ncclCommDestroy");
        err = (fn_err)dlsym(so, "ncclGetErrorString");
        ok = init_all && all_gather && group_start && group_end && destroy;
    }
};
Rccl g_rccl;

std::string nccl_msg(int r) { return g_rccl.err ? g_rccl.err(r) : std::to_string(r); }
}  // namespace

struct MultiDev {
    int R = 0;
    std::vector<int> dev;
    std::vector<MdSlice> plan;
    std::vector<pdplqr_handle> sh;
    std::vector<hipStream_t> st;
    std::vector<hipEvent_t> ev;   // elem / fp ready on its shard's stream (device-copy exchange)
    std::vector<hipEvent_t> xev;  // shard r's exchange copies done (they read every other shard's buffers)
    std::vector<hipEvent_t> tail;  // shard r's queued work (the caller stream's join)
    // the caller's stream on devices[0] (pdplqr_set_stream): device inputs are
    // ordered after it by an event, and it waits for the slices' work at the end
    // of every call; NULL: the devices are drained before device inputs are read
    hipStream_t caller = nullptr;
    hipEvent_t cev = nullptr;     // recorded on `caller`, waited on by every slice stream
    bool xpending = false;        // a device-copy exchange was issued since the last backward
    // per shard, on its device: model staging (set_model), vectors, elements,
    // the (f, p) parts of the element and their gather (backward_without_factorization)
    std::vector<double *> ws, ys, zs, ir, rho, x0, elem, gathered, wout, fp, gathered_fp;
    // on the first device: the full D and row / D offsets (admm_solve's update pass)
    double *Dfull = nullptr;
    int32_t *d_off = nullptr, *y_off = nullptr;
    std::vector<ncclComm_t> comm;
    bool rccl = false;
    std::vector<std::vector<void *>> allocs;
};

static int md_alloc(MultiDev *md, int r, double **p, long long count) {
    void *q = nullptr;
    PDPLQR_HIP_TRY(hipSetDevice(md->dev[r]));
    const hipError_t e = hipMalloc(&q, (size_t)std::max(1LL, count) * sizeof(double));
    if (e != hipSuccess) {
        set_error(std::string("multi-device hipMalloc: ") + hipGetErrorString(e));
        return PDPLQR_ERR_ALLOC;
    }
    md->allocs[r].push_back(q);
    *p = reinterpret_cast<double *>(q);
    return PDPLQR_OK;
}

static hipMemcpyKind md_kind(int mem, bool to_device) {
    if (mem == PDPLQR_MEM_DEVICE) return hipMemcpyDefault;  // unified addressing: peer or local
    return to_device ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost;
}

// rows of `width` doubles, one per problem: dst (pitch dp) <- src (pitch sp)
static int md_copy2d(double *dst, long long dp, const double *src, long long sp, long long width, int rows,
                     hipMemcpyKind kind, hipStream_t s) {
    if (width <= 0) return PDPLQR_OK;
    PDPLQR_HIP_TRY(hipMemcpy2DAsync(dst, (size_t)dp * sizeof(double), src, (size_t)sp * sizeof(double),
                                    (size_t)width * sizeof(double), (size_t)rows, kind, s));
    return PDPLQR_OK;
}

// Device-memory inputs may still be in production on a stream of the caller
// (torch's current stream, say) while the driver's copies run on the slices'
// own non-blocking streams.  With a caller stream set (pdplqr_set_stream) every
// slice stream waits for an event recorded on it -- no host synchronisation;
// without one every device is drained first.
static int md_inputs_ready(MultiDev *md, int mem) {
    if (mem != PDPLQR_MEM_DEVICE) return PDPLQR_OK;
    if (md->caller) {
        PDPLQR_HIP_TRY(hipSetDevice(md->dev[0]));
        PDPLQR_HIP_TRY(hipEventRecord(md->cev, md->caller));
        for (int r = 0; r < md->R; ++r) {
            PDPLQR_HIP_TRY(hipSetDevice(md->dev[r]));
            PDPLQR_HIP_TRY(hipStreamWaitEvent(md->st[r], md->cev, 0));
        }
        return PDPLQR_OK;
    }
    for (int r = 0; r < md->R; ++r) {
        if (std::find(md->dev.begin(), md->dev.begin() + r, md->dev[r]) != md->dev.begin() + r) continue;
        PDPLQR_HIP_TRY(hipSetDevice(md->dev[r]));
        PDPLQR_HIP_TRY(hipDeviceSynchronize());
    }
    return PDPLQR_OK;
}

// The caller stream waits (events) for everything the slices queued so far:
// outputs are read, inputs freed or overwritten there.  No-op without one.
static int md_join_caller(MultiDev *md) {
    if (!md->caller) return PDPLQR_OK;
    for (int r = 0; r < md->R; ++r) {
        PDPLQR_HIP_TRY(hipSetDevice(md->dev[r]));
        PDPLQR_HIP_TRY(hipEventRecord(md->tail[r], md->st[r]));
    }
    PDPLQR_HIP_TRY(hipSetDevice(md->dev[0]));
    for (int r = 0; r < md->R; ++r) PDPLQR_HIP_TRY(hipStreamWaitEvent(md->caller, md->tail[r], 0));
    return PDPLQR_OK;
}

static int md_sync(MultiDev *md) {
    for (int r = 0; r < md->R; ++r) {
        PDPLQR_HIP_TRY(hipSetDevice(md->dev[r]));
        PDPLQR_HIP_TRY(hipStreamSynchronize(md->st[r]));
    }
    return PDPLQR_OK;
}

void md_release(pdplqr_handle h) {
    MultiDev *md = h->md;
    if (!md) return;
    for (int r = 0; r < md->R; ++r) {
        (void)hipSetDevice(md->dev[r]);
        if (r < (int)md->st.size() && md->st[r]) (void)hipStreamSynchronize(md->st[r]);
    }
    if (md->rccl)
        for (ncclComm_t c : md->comm)
            if (c) (void)g_rccl.destroy(c);
    if (md->cev) {
        (void)hipSetDevice(md->dev[0]);
        (void)hipEventDestroy(md->cev);
    }
    for (int r = 0; r < md->R; ++r) {
        (void)hipSetDevice(md->dev[r]);
        if (r < (int)md->ev.size() && md->ev[r]) (void)hipEventDestroy(md->ev[r]);
        if (r < (int)md->xev.size() && md->xev[r]) (void)hipEventDestroy(md->xev[r]);
        if (r < (int)md->tail.size() && md->tail[r]) (void)hipEventDestroy(md->tail[r]);
        if (r < (int)md->sh.size() && md->sh[r]) (void)pdplqr_destroy(md->sh[r]);
        for (void *p : md->allocs[r]) (void)hipFree(p);
    }
    delete md;
    h->md = nullptr;
}

int md_create(pdplqr_handle h, const pdplqr_config &C) {
    const int R = C.num_devices;
    if (C.solver != PDPLQR_SOLVER_PARALLEL) {
        set_error("num_devices needs the PARALLEL solver (the horizon is split across the devices)");
        return PDPLQR_ERR_INVALID;
    }
    if (C.N < R) {
        set_error("num_devices > N: every device needs at least one stage");
        return PDPLQR_ERR_INVALID;
    }
    int ndev = 0;
    PDPLQR_HIP_TRY(hipGetDeviceCount(&ndev));
    std::vector<int> devs;
    for (int r = 0; r < R; ++r) {
        const int d = C.devices ? C.devices[r] : r;
        if (d < 0 || d >= ndev) {
            set_error("devices[" + std::to_string(r) + "] = " + std::to_string(d) + " is not a visible HIP device");
            return PDPLQR_ERR_INVALID;
        }
        devs.push_back(d);
    }
    MultiDev *md = new MultiDev();
    h->md = md;
    md->R = R;
    md->dev = devs;
    md->allocs.resize(R);
    md_plan(C.N, R, h->ncs, C.nx, C.nu, md->plan);
    const long long B = C.batch, es = 3LL * C.nx * C.nx + 2LL * C.nx;
    const int n = C.nx, s = C.nx + C.nu;
    md->sh.assign(R, nullptr);
    md->st.assign(R, nullptr);
    md->ev.assign(R, nullptr);
    md->xev.assign(R, nullptr);
    md->tail.assign(R, nullptr);
    md->fp.assign(R, nullptr);
    md->gathered_fp.assign(R, nullptr);
    md->ws.assign(R, nullptr);
    md->ys.assign(R, nullptr);
    md->zs.assign(R, nullptr);
    md->ir.assign(R, nullptr);
    md->rho.assign(R, nullptr);
    md->x0.assign(R, nullptr);
    md->elem.assign(R, nullptr);
    md->gathered.assign(R, nullptr);
    md->wout.assign(R, nullptr);
    int rc;
    for (int r = 0; r < R; ++r) {
        const MdSlice &p = md->plan[r];
        const int Nl = p.N1 - p.N0;
        pdplqr_config sc = C;
        sc.N = Nl;
        sc.device = md->dev[r];
        sc.num_devices = 0;
        sc.devices = nullptr;
        sc.ncs = p.ncs.data();
        sc.keep_factors = 1;
        // the slice's device segmentation is automatic (segment_len); its
        // reference segment count only has to satisfy CHOLESKY's ns >= 2
        // (condensed_system.hpp:230): a slice of < 3 stages is one segment in
        // the LU form (the same answer), as pdplqr/horizon.py HorizonShard
        const bool chol = C.condensed_type == PDPLQR_CONDENSED_CHOLESKY && Nl >= 3;
        sc.num_segments = chol ? 2 : 1;
        if (!chol) sc.condensed_type = PDPLQR_CONDENSED_LU;
        if ((rc = pdplqr_create(&sc, &md->sh[r]))) return rc;
        md->st[r] = reinterpret_cast<hipStream_t>(pdplqr_get_stream(md->sh[r]));
        const long long perh = (long long)Nl * s + n, ny = p.ny_st + p.nc_term;
        if ((rc = md_alloc(md, r, &md->ws[r], B * perh)) || (rc = md_alloc(md, r, &md->wout[r], B * perh)) ||
            (rc = md_alloc(md, r, &md->ys[r], B * ny)) || (rc = md_alloc(md, r, &md->zs[r], B * ny)) ||
            (rc = md_alloc(md, r, &md->ir[r], B * ny)) || (rc = md_alloc(md, r, &md->rho[r], B * ny)) ||
            (rc = md_alloc(md, r, &md->x0[r], B * n)) || (rc = md_alloc(md, r, &md->elem[r], B * es)) ||
            (rc = md_alloc(md, r, &md->gathered[r], (long long)R * B * es)) ||
            (rc = md_alloc(md, r, &md->fp[r], B * 2 * n)) ||
            (rc = md_alloc(md, r, &md->gathered_fp[r], (long long)R * B * 2 * n)))
            return rc;
        PDPLQR_HIP_TRY(hipSetDevice(md->dev[r]));
        PDPLQR_HIP_TRY(hipEventCreateWithFlags(&md->ev[r], hipEventDisableTiming));
        PDPLQR_HIP_TRY(hipEventCreateWithFlags(&md->xev[r], hipEventDisableTiming));
        PDPLQR_HIP_TRY(hipEventCreateWithFlags(&md->tail[r], hipEventDisableTiming));
    }
    PDPLQR_HIP_TRY(hipSetDevice(md->dev[0]));
    PDPLQR_HIP_TRY(hipEventCreateWithFlags(&md->cev, hipEventDisableTiming));
    // admm_solve's update pass runs on the first device over the whole horizon
    {
        double *p = nullptr;
        if ((rc = md_alloc(md, 0, &md->Dfull, B * h->sh.ndD))) return rc;
        if ((rc = md_alloc(md, 0, &p, (C.N + 2 + 1) / 2 * 2))) return rc;  // (int32 offsets in double-sized slots)
        md->d_off = reinterpret_cast<int32_t *>(p);
        if ((rc = md_alloc(md, 0, &p, (C.N + 2 + 1) / 2 * 2))) return rc;
        md->y_off = reinterpret_cast<int32_t *>(p);
        PDPLQR_HIP_TRY(hipSetDevice(md->dev[0]));
        PDPLQR_HIP_TRY(hipMemcpy(md->d_off, h->d_off_h.data(), (C.N + 2) * sizeof(int32_t), hipMemcpyHostToDevice));
        PDPLQR_HIP_TRY(hipMemcpy(md->y_off, h->y_off_h.data(), (C.N + 2) * sizeof(int32_t), hipMemcpyHostToDevice));
    }
    // peer access between distinct devices (the 2D slice copies, the device-copy exchange)
    for (int a = 0; a < R; ++a)
        for (int b = 0; b < R; ++b) {
            if (md->dev[a] == md->dev[b]) continue;
            int can = 0;
            PDPLQR_HIP_TRY(hipDeviceCanAccessPeer(&can, md->dev[a], md->dev[b]));
            if (!can) continue;
            PDPLQR_HIP_TRY(hipSetDevice(md->dev[a]));
            const hipError_t e = hipDeviceEnablePeerAccess(md->dev[b], 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
                set_error(std::string("hipDeviceEnablePeerAccess: ") + hipGetErrorString(e));
                return PDPLQR_ERR_HIP;
            }
            (void)hipGetLastError();
        }
    std::vector<int> sorted = md->dev;
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::unique(sorted.begin(), sorted.end()) == sorted.end();
    if (distinct && !getenv("PDPLQR_MD_P2P")) {
        if (!g_rccl.load()) {
            set_error("num_devices > 1: librccl.so.1 not found (set PDPLQR_MD_P2P=1 for device copies)");
            return PDPLQR_ERR_UNSUPPORTED;
        }
        md->comm.assign(R, nullptr);
        const int e = g_rccl.init_all(md->comm.data(), R, md->dev.data());
        if (e != 0) {
            set_error("ncclCommInitAll: " + nccl_msg(e));
            return PDPLQR_ERR_HIP;
        }
        md->rccl = true;
    }
    return PDPLQR_OK;
}

int md_set_model(pdplqr_handle h, int mask, const double *E, const double *c, const double *H, const double *hv,
                 const double *D, int mem) {
    MultiDev *md = h->md;
    const Shape &g = h->sh;
    const int n = g.n, s = g.s, N = g.N, Bi = g.batch;
    const hipMemcpyKind kind = md_kind(mem, true);
    int rc;
    if ((rc = md_inputs_ready(md, mem))) return rc;
    for (int r = 0; r < md->R; ++r) {
        const MdSlice &p = md->plan[r];
        const int Nl = p.N1 - p.N0;
        const long long perE = (long long)Nl * n * s, perc = (long long)Nl * n;
        const long long perH = (long long)Nl * s * s + (long long)n * n, perh = (long long)Nl * s + n;
        const long long ndD = p.nd_st + (long long)p.nc_term * n;
        hipStream_t S = md->st[r];
        PDPLQR_HIP_TRY(hipSetDevice(md->dev[r]));
        // staging on the shard's device, released once the shard holds its copy
        double *sE = nullptr, *sc = nullptr, *sH = nullptr, *sh = nullptr, *sD = nullptr;
        std::vector<void *> tmp;
        auto talloc = [&](double **q, long long cnt) -> int {
            void *v = nullptr;
            const hipError_t e = hipMalloc(&v, (size_t)std::max(1LL, cnt * Bi) * sizeof(double));
            if (e != hipSuccess) {
                set_error(std::string("multi-device set_model staging: ") + hipGetErrorString(e));
                return PDPLQR_ERR_ALLOC;
            }
            tmp.push_back(v);
            *q = reinterpret_cast<double *>(v);
            return PDPLQR_OK;
        };
        rc = PDPLQR_OK;
        if (!rc && (mask & PDPLQR_MODEL_E) && !(rc = talloc(&sE, perE)))
            rc = md_copy2d(sE, perE, E + (long long)p.N0 * n * s, g.perE, perE, Bi, kind, S);
        if (!rc && (mask & PDPLQR_MODEL_C) && !(rc = talloc(&sc, perc)))
            rc = md_copy2d(sc, perc, c + (long long)p.N0 * n, g.perc, perc, Bi, kind, S);
        if (!rc && (mask & PDPLQR_MODEL_H) && !(rc = talloc(&sH, perH))) {
            rc = md_copy2d(sH, perH, H + (long long)p.N0 * s * s, g.perH, (long long)Nl * s * s, Bi, kind, S);
            if (!rc && p.last)
                rc = md_copy2d(sH + (long long)Nl * s * s, perH, H + (long long)N * s * s, g.perH, (long long)n * n, Bi,
                               kind, S);
            else if (!rc)
                PDPLQR_HIP_TRY(hipMemset2DAsync(sH + (long long)Nl * s * s, perH * sizeof(double), 0,
                                                (size_t)n * n * sizeof(double), Bi, S));
        }
        if (!rc && (mask & PDPLQR_MODEL_HV) && !(rc = talloc(&sh, perh))) {
            rc = md_copy2d(sh, perh, hv + (long long)p.N0 * s, g.perh, (long long)Nl * s, Bi, kind, S);
            if (!rc && p.last)
                rc = md_copy2d(sh + (long long)Nl * s, perh, hv + (long long)N * s, g.perh, n, Bi, kind, S);
            else if (!rc)
                PDPLQR_HIP_TRY(hipMemset2DAsync(sh + (long long)Nl * s, perh * sizeof(double), 0, n * sizeof(double),
                                                Bi, S));
        }
        if (!rc && (mask & PDPLQR_MODEL_D) && ndD > 0 && !(rc = talloc(&sD, ndD))) {
            rc = md_copy2d(sD, ndD, D + p.d0, g.ndD, p.nd_st, Bi, kind, S);
            if (!rc && p.nc_term > 0)
                rc = md_copy2d(sD + p.nd_st, ndD, D + h->d_off_h[N], g.ndD, (long long)p.nc_term * n, Bi, kind, S);
        }
        if (!rc)
            rc = pdplqr_set_model_arrays(md->sh[r], mask, sE ? sE : nullptr, sc, sH, sh, sD ? sD : nullptr,
                                         PDPLQR_MEM_DEVICE);
        (void)hipStreamSynchronize(S);
        for (void *v : tmp) (void)hipFree(v);
        if (rc) return rc;
    }
    if ((mask & PDPLQR_MODEL_D) && g.ndD > 0) {  // the full D for admm_solve's update pass (first device)
        PDPLQR_HIP_TRY(hipSetDevice(md->dev[0]));
        PDPLQR_HIP_TRY(hipMemcpyAsync(md->Dfull, D, (size_t)Bi * g.ndD * sizeof(double), kind, md->st[0]));
        PDPLQR_HIP_TRY(hipStreamSynchronize(md->st[0]));
    }
    if (mem != PDPLQR_MEM_DEVICE) {  // host bytes this upload moved (pdplqr_get_model_upload_bytes)
        long long bytes = 0;
        if (mask & PDPLQR_MODEL_E) bytes += (long long)Bi * g.perE;
        if (mask & PDPLQR_MODEL_C) bytes += (long long)Bi * g.perc;
        if (mask & PDPLQR_MODEL_H) bytes += (long long)Bi * g.perH;
        if (mask & PDPLQR_MODEL_HV) bytes += (long long)Bi * g.perh;
        if (mask & PDPLQR_MODEL_D) bytes += (long long)Bi * g.ndD;
        h->model_upload_bytes += bytes * (long long)sizeof(double);
    }
    h->model_set = true;
    if (mask & (PDPLQR_MODEL_H | PDPLQR_MODEL_HV)) h->updated = false;
    return md_join_caller(md);
}

// per-stage vectors of the slice: the stage rows [a0, a1) and, for the last
// slice, the terminal rows [t0, t1) (offsets in the full per-problem vector)
static int md_vec(const double *src, long long pitch, double *dst, long long dpitch, long long a0, long long a1,
                  long long t0, long long t1, int rows, hipMemcpyKind kind, hipStream_t S) {
    int rc = md_copy2d(dst, dpitch, src + a0, pitch, a1 - a0, rows, kind, S);
    if (!rc && t1 > t0) rc = md_copy2d(dst + (a1 - a0), dpitch, src + t0, pitch, t1 - t0, rows, kind, S);
    return rc;
}

int md_update(pdplqr_handle h, const double *ws, const double *ys, const double *zs, const double *irho, double sigma,
              int mem) {
    MultiDev *md = h->md;
    const Shape &g = h->sh;
    const int n = g.n, m = g.m, s = g.s, N = g.N, Bi = g.batch;
    const hipMemcpyKind kind = md_kind(mem, true);
    int rc;
    if ((rc = md_inputs_ready(md, mem))) return rc;
    for (int r = 0; r < md->R; ++r) {
        const MdSlice &p = md->plan[r];
        const int Nl = p.N1 - p.N0;
        const long long perh = (long long)Nl * s + n, ny = p.ny_st + p.nc_term;
        PDPLQR_HIP_TRY(hipSetDevice(md->dev[r]));
        hipStream_t S = md->st[r];
        // w of the slice's stages, then its end state: x_N (last) or x_{N1} (the
        // next slice's first state; only sigma w touches it and the dummy
        // terminal of a non-final slice ignores it)
        const long long t0 = p.last ? (long long)N * s : (long long)p.N1 * s + m;
        if ((rc = md_vec(ws, g.perh, md->ws[r], perh, (long long)p.N0 * s, (long long)p.N1 * s, t0, t0 + n, Bi, kind,
                         S)))
            return rc;
        if (ny > 0) {
            const long long y0 = p.y0, y1 = p.y0 + p.ny_st, z0 = h->y_off_h[N], z1 = z0 + p.nc_term;
            if ((rc = md_vec(ys, g.ny, md->ys[r], ny, y0, y1, z0, z1, Bi, kind, S)) ||
                (rc = md_vec(zs, g.ny, md->zs[r], ny, y0, y1, z0, z1, Bi, kind, S)) ||
                (rc = md_vec(irho, g.ny, md->ir[r], ny, y0, y1, z0, z1, Bi, kind, S)))
                return rc;
        }
        if ((rc = pdplqr_update_problem_data(md->sh[r], md->ws[r], ny ? md->ys[r] : nullptr, ny ? md->zs[r] : nullptr,
                                             ny ? md->ir[r] : nullptr, sigma, PDPLQR_MEM_DEVICE)))
            return rc;
    }
    if (mem != PDPLQR_MEM_DEVICE && (rc = md_sync(md))) return rc;  // host inputs may be reused on return
    h->updated = true;
    return md_join_caller(md);
}

// backward (fact) or backward_without_factorization: the slice backwards, then
// the exchange -- the whole slice elements (3n^2 + 2n doubles per problem) after
// a factorising backward, only their (f, p) (2n) without factorization
// (reduction_without_factorization's update_segment_data(p, f, id),
// lqr_solver_parallel.hpp:207-210): F, C, P of the last gather stay valid.
int md_backward(pdplqr_handle h, const double *rho, int mem, bool fact) {
    MultiDev *md = h->md;
    const Shape &g = h->sh;
    const int N = g.N, Bi = g.batch, n = g.n;
    const long long es = 3LL * n * n + 2LL * n;
    const long long cnt = (long long)Bi * (fact ? es : 2LL * n);
    const hipMemcpyKind kind = md_kind(mem, true);
    int rc;
    if ((rc = md_inputs_ready(md, mem))) return rc;
    // the last device-copy exchange read every slice's element / (f, p) buffer
    // on the reading slice's stream: no slice rewrites its buffer before all of
    // those copies are done
    if (md->xpending) {
        for (int q = 0; q < md->R; ++q) {
            PDPLQR_HIP_TRY(hipSetDevice(md->dev[q]));
            for (int r = 0; r < md->R; ++r) PDPLQR_HIP_TRY(hipStreamWaitEvent(md->st[q], md->xev[r], 0));
        }
        md->xpending = false;
    }
    for (int r = 0; r < md->R; ++r) {
        const MdSlice &p = md->plan[r];
        const long long ny = p.ny_st + p.nc_term;
        PDPLQR_HIP_TRY(hipSetDevice(md->dev[r]));
        if (ny > 0) {
            if (!rho) {
                set_error("backward: constraints declared but rho is null");
                return PDPLQR_ERR_INVALID;
            }
            const long long z0 = h->y_off_h[N];
            if ((rc = md_vec(rho, g.ny, md->rho[r], ny, p.y0, p.y0 + p.ny_st, z0, z0 + p.nc_term, Bi, kind,
                             md->st[r])))
                return rc;
        }
        const double *rr = ny ? md->rho[r] : nullptr;
        if (fact) rc = pdplqr_shard_backward(md->sh[r], rr, p.last ? 1 : 0, md->elem[r], PDPLQR_MEM_DEVICE);
        else
            rc = pdplqr_shard_backward_without_factorization(md->sh[r], rr, p.last ? 1 : 0, md->elem[r],
                                                             PDPLQR_MEM_DEVICE);
        if (rc) return rc;
        if (!fact) {  // pack [f | p] per problem (element offsets 2n^2 and 3n^2 + n)
            if ((rc = md_copy2d(md->fp[r], 2 * n, md->elem[r] + 2LL * n * n, es, n, Bi, hipMemcpyDeviceToDevice,
                                md->st[r])) ||
                (rc = md_copy2d(md->fp[r] + n, 2 * n, md->elem[r] + 3LL * n * n + n, es, n, Bi,
                                hipMemcpyDeviceToDevice, md->st[r])))
                return rc;
        }
        PDPLQR_HIP_TRY(hipEventRecord(md->ev[r], md->st[r]));
    }
    const std::vector<double *> &src = fact ? md->elem : md->fp;
    const std::vector<double *> &dst = fact ? md->gathered : md->gathered_fp;
    // the exchange: every slice receives [R][batch][width] (rank-major)
    if (md->rccl) {
        int e = g_rccl.group_start();
        hipError_t he = hipSuccess;
        for (int r = 0; r < md->R && e == 0 && he == hipSuccess; ++r) {
            he = hipSetDevice(md->dev[r]);
            if (he == hipSuccess)
                e = g_rccl.all_gather(src[r], dst[r], (size_t)cnt, NCCL_FLOAT64, md->comm[r], md->st[r]);
        }
        const int e2 = g_rccl.group_end();  // always closes the group, also after an error inside it
        if (he != hipSuccess) {
            set_error(std::string("hipSetDevice: ") + hipGetErrorString(he));
            return PDPLQR_ERR_HIP;
        }
        if (e || e2) {
            set_error("ncclAllGather: " + nccl_msg(e ? e : e2));
            return PDPLQR_ERR_HIP;
        }
    } else {
        for (int r = 0; r < md->R; ++r) {
            PDPLQR_HIP_TRY(hipSetDevice(md->dev[r]));
            for (int q = 0; q < md->R; ++q) {
                PDPLQR_HIP_TRY(hipStreamWaitEvent(md->st[r], md->ev[q], 0));
                PDPLQR_HIP_TRY(hipMemcpyAsync(dst[r] + q * cnt, src[q], (size_t)cnt * sizeof(double),
                                              hipMemcpyDefault, md->st[r]));
            }
            PDPLQR_HIP_TRY(hipEventRecord(md->xev[r], md->st[r]));
        }
        md->xpending = true;
    }
    if (!fact) {  // scatter the gathered (f, p) into the element slots of the last full gather
        for (int r = 0; r < md->R; ++r) {
            PDPLQR_HIP_TRY(hipSetDevice(md->dev[r]));
            for (int q = 0; q < md->R; ++q) {
                double *eq = md->gathered[r] + (long long)q * Bi * es;
                const double *fq = md->gathered_fp[r] + (long long)q * Bi * 2 * n;
                if ((rc = md_copy2d(eq + 2LL * n * n, es, fq, 2 * n, n, Bi, hipMemcpyDeviceToDevice, md->st[r])) ||
                    (rc = md_copy2d(eq + 3LL * n * n + n, es, fq + n, 2 * n, n, Bi, hipMemcpyDeviceToDevice,
                                    md->st[r])))
                    return rc;
            }
        }
    }
    if (mem != PDPLQR_MEM_DEVICE && (rc = md_sync(md))) return rc;
    if (fact) h->factored = true;
    return md_join_caller(md);
}

int md_forward(pdplqr_handle h, const double *x0, double *ws, int mem) {
    MultiDev *md = h->md;
    const Shape &g = h->sh;
    const int n = g.n, s = g.s, N = g.N, Bi = g.batch;
    int rc;
    if ((rc = md_inputs_ready(md, mem))) return rc;
    for (int r = 0; r < md->R; ++r) {
        PDPLQR_HIP_TRY(hipSetDevice(md->dev[r]));
        if ((rc = md_copy2d(md->x0[r], n, x0, n, n, Bi, md_kind(mem, true), md->st[r]))) return rc;
        if ((rc = pdplqr_shard_forward(md->sh[r], md->x0[r], md->gathered[r], md->R, r, md->wout[r],
                                       PDPLQR_MEM_DEVICE)))
            return rc;
    }
    // assemble ws: each slice's stages, then the last slice's x_N
    for (int r = 0; r < md->R; ++r) {
        const MdSlice &p = md->plan[r];
        const int Nl = p.N1 - p.N0;
        const long long perh = (long long)Nl * s + n;
        PDPLQR_HIP_TRY(hipSetDevice(md->dev[r]));
        const hipMemcpyKind kind = md_kind(mem, false);
        if ((rc = md_copy2d(ws + (long long)p.N0 * s, g.perh, md->wout[r], perh, (long long)Nl * s, Bi, kind,
                            md->st[r])))
            return rc;
        if (p.last && (rc = md_copy2d(ws + (long long)N * s, g.perh, md->wout[r] + (long long)Nl * s, perh, n, Bi, kind,
                                      md->st[r])))
            return rc;
    }
    // device outputs with a caller stream: ordered on it (events); otherwise
    // ws is complete when the call returns
    if (md->caller && mem == PDPLQR_MEM_DEVICE) return md_join_caller(md);
    return md_sync(md);
}

int md_status(pdplqr_handle h, int32_t *flags) {
    MultiDev *md = h->md;
    const int Bi = h->sh.batch, N = h->sh.N;
    std::vector<int32_t> f(Bi);
    for (int b = 0; b < Bi; ++b) flags[b] = 0;
    for (int r = 0; r < md->R; ++r) {
        const MdSlice &p = md->plan[r];
        const int Nl = p.N1 - p.N0;
        const int rc = pdplqr_get_status(md->sh[r], f.data());
        if (rc) return rc;
        for (int b = 0; b < Bi; ++b) {
            if (!f[b]) continue;
            // a stage index of the slice (1-based) -> of the horizon; a failed
            // condensed combine (Nl + 2) -> N + 2
            const int v = f[b] >= Nl + 2 ? N + 2 : p.N0 + f[b];
            flags[b] = std::max(flags[b], v);
        }
    }
    return PDPLQR_OK;
}

int md_synchronize(pdplqr_handle h) { return md_sync(h->md); }

int md_clear(pdplqr_handle h) {
    MultiDev *md = h->md;
    for (int r = 0; r < md->R; ++r) {
        const int rc = pdplqr_clear_workspace(md->sh[r]);
        if (rc) return rc;
    }
    return PDPLQR_OK;
}

void *md_stream(pdplqr_handle h) {
    MultiDev *md = h->md;
    if (md->caller) return reinterpret_cast<void *>(md->caller);
    return md->R > 0 ? reinterpret_cast<void *>(md->st[0]) : nullptr;
}

// pdplqr_set_stream on a split handle: the caller's stream, on devices[0]
// (NULL: back to draining the devices before device inputs are read).  What
// the slices queued before the switch is joined to the new stream.
int md_set_stream(pdplqr_handle h, void *stream) {
    MultiDev *md = h->md;
    hipStream_t next = reinterpret_cast<hipStream_t>(stream);
    if (next) {
        int d = -1;
        PDPLQR_HIP_TRY(hipStreamGetDevice(next, &d));
        if (d != md->dev[0]) {
            set_error("set_stream: a num_devices > 1 handle takes a stream of its first device (devices[0])");
            return PDPLQR_ERR_INVALID;
        }
    }
    md->caller = next;
    return md_join_caller(md);
}

int md_primary_device(pdplqr_handle h) { return h->md->dev[0]; }

void md_admm_view(pdplqr_handle h, const double **D, const int32_t **d_off, const int32_t **y_off) {
    *D = h->md->Dfull;
    *d_off = h->md->d_off;
    *y_off = h->md->y_off;
}

}  // namespace pdplqr

using namespace pdplqr;

// Host-only: the slicing plan of a num_devices split (tests; no GPU call).
// out: R rows of 8 int64 -- N0, N1, last, y0, ny_stages, nc_terminal, d0, nd_stages.
extern "C" int pdplqr_multidev_plan(int32_t N, int32_t R, const int32_t *ncs, int32_t nx, int32_t nu, int64_t *out) {
    if (N < 1 || R < 1 || R > N || nx < 1 || nu < 1 || !out) return PDPLQR_ERR_INVALID;
    std::vector<int32_t> v(N + 1, 0);
    if (ncs)
        for (int k = 0; k <= N; ++k) v[k] = ncs[k];
    std::vector<MdSlice> plan;
    md_plan(N, R, v, nx, nu, plan);
    for (int r = 0; r < R; ++r) {
        const MdSlice &p = plan[r];
        int64_t *o = out + 8 * r;
        o[0] = p.N0;
        o[1] = p.N1;
        o[2] = p.last;
        o[3] = p.y0;
        o[4] = p.ny_st;
        o[5] = p.nc_term;
        o[6] = p.d0;
        o[7] = p.nd_st;
    }
    return PDPLQR_OK;
}
