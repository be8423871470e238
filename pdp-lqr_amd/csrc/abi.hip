// abi.hip -- the C ABI of libpdplqr (include/pdplqr.h): handle lifecycle,
// host<->device staging and the update_problem_data -> backward -> forward
// protocol of the reference solvers.  No CPU fallback exists: every compute
// entry point runs on the HIP device or returns an error.
#include <string.h>

#include <algorithm>
#include <new>
#include <string>
#include <vector>

#include "internal.hpp"
#include "solvers.hpp"

namespace pdplqr {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }

int device_simds(int device) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
    return 4 * cus;  // CDNA: four SIMDs per CU
}

bool one_wave_per_simd(int device, long long waves) {
    return waves <= device_simds(device) && !getenv("PDPLQR_NO_X1");
}

static int invalid(const std::string &msg) {
    set_error(msg);
    return PDPLQR_ERR_INVALID;
}

template <typename X>
static int dalloc(pdplqr_handle h, X **p, size_t count) {
    *p = nullptr;
    if (count == 0) count = 1;
    void *q = nullptr;
    hipError_t e = hipMalloc(&q, count * sizeof(X));
    if (e != hipSuccess) {
        set_error(std::string("hipMalloc(") + std::to_string(count * sizeof(X)) + " B): " + hipGetErrorString(e));
        return PDPLQR_ERR_ALLOC;
    }
    h->allocs.push_back(q);
    *p = reinterpret_cast<X *>(q);
    return PDPLQR_OK;
}

// Copies `count` doubles from host or device memory into device buffer `dst`
// (or returns the device pointer itself when no copy is needed).
static int stage_in(pdplqr_handle h, const double *src, double *dst, long long count, int mem, const double **out) {
    if (count <= 0) {
        *out = dst;
        return PDPLQR_OK;
    }
    if (!src) return invalid("null input pointer");
    if (mem == PDPLQR_MEM_DEVICE) {
        *out = src;
        return PDPLQR_OK;
    }
    PDPLQR_HIP_TRY(hipMemcpyAsync(dst, src, (size_t)count * sizeof(double), hipMemcpyHostToDevice, h->stream));
    h->host_staged = true;
    *out = dst;
    return PDPLQR_OK;
}

}  // namespace pdplqr

using namespace pdplqr;

extern "C" {

void pdplqr_config_init(pdplqr_config *cfg) {
    if (!cfg) return;
    memset(cfg, 0, sizeof(*cfg));
    cfg->batch = 1;
    cfg->solver = PDPLQR_SOLVER_SERIAL;
    cfg->num_segments = 1;
    cfg->load_balancing = 1;
    cfg->condensed_type = PDPLQR_CONDENSED_CHOLESKY;
    cfg->keep_factors = 1;
    cfg->rho_dyn = 1e-6;
    cfg->kkt_sigma = 1e-6;
}

const char *pdplqr_last_error(void) { return g_last_error.c_str(); }

int pdplqr_device_count(int32_t *count) {
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) {
        set_error(std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
        if (count) *count = 0;
        return PDPLQR_ERR_HIP;
    }
    if (count) *count = c;
    return PDPLQR_OK;
}

static void free_all(pdplqr_handle h) {
    for (void *p : h->allocs) (void)hipFree(p);
    h->allocs.clear();
    if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
    h->own_stream = nullptr;
}

int pdplqr_create(const pdplqr_config *cfg, pdplqr_handle *out) {
    if (!cfg || !out) return invalid("null argument");
    *out = nullptr;
    const pdplqr_config &C = *cfg;
    if (C.N < 1) return invalid("Horizon must be at least 1.");  // lqr_model.hpp:75-77
    if (C.nx < 1 || C.nu < 1) return invalid("nx and nu must be >= 1");
    if (C.batch < 1) return invalid("batch must be >= 1");
    if (C.solver < PDPLQR_SOLVER_SERIAL || C.solver > PDPLQR_SOLVER_KKT) return invalid("unknown solver kind");
    if (C.solver == PDPLQR_SOLVER_PARALLEL) {
        if (C.condensed_type != PDPLQR_CONDENSED_LU && C.condensed_type != PDPLQR_CONDENSED_CHOLESKY)
            return invalid("Unsupported CondensedSystemSolverType");  // lqr_solver_parallel.hpp:99
        if (C.num_segments < 1) return invalid("num_segments must be >= 1");
    }
    pdplqr_handle h = new (std::nothrow) pdplqr_handle_s();
    if (!h) return invalid("out of host memory");
    h->cfg = C;
    h->cfg.ncs = nullptr;
    Shape &sh = h->sh;
    sh.n = C.nx;
    sh.m = C.nu;
    sh.N = C.N;
    sh.batch = C.batch;
    sh.s = sh.n + sh.m;
    sh.ps = sh.s * (sh.s + 1) / 2;
    sh.pn = sh.n * (sh.n + 1) / 2;
    h->ncs.assign(C.N + 1, 0);
    if (C.ncs)
        for (int k = 0; k <= C.N; ++k) h->ncs[k] = C.ncs[k];
    h->d_off_h.assign(C.N + 2, 0);
    h->y_off_h.assign(C.N + 2, 0);
    h->max_nc = 0;
    for (int k = 0; k <= C.N; ++k) {
        if (h->ncs[k] < 0) {
            delete h;
            return invalid("negative constraint count");
        }
        const int dim = k < C.N ? sh.s : sh.n;
        h->d_off_h[k + 1] = h->d_off_h[k] + h->ncs[k] * dim;
        h->y_off_h[k + 1] = h->y_off_h[k] + h->ncs[k];
        h->max_nc = std::max(h->max_nc, (int)h->ncs[k]);
    }
    sh.ny = h->y_off_h[C.N + 1];
    sh.ndD = h->d_off_h[C.N + 1];
    sh.perE = (long long)sh.N * sh.n * sh.s;
    sh.perc = (long long)sh.N * sh.n;
    sh.perH = (long long)sh.N * sh.s * sh.s + (long long)sh.n * sh.n;
    sh.perh = (long long)sh.N * sh.s + sh.n;
    sh.perHw = ((long long)sh.N * sh.ps + sh.pn + 1) / 2 * 2;  // 16-byte aligned per problem
    sh.perKD = (long long)sh.N * (sh.s * sh.m + sh.m);  // rollout record [L(:,0:m) | lu']

    if (C.num_devices > 1 || (C.num_devices == 1 && C.devices)) {  // the horizon split over devices (multidev.hip)
        if (C.num_devices > 1024) {
            delete h;
            return invalid("num_devices out of range");
        }
        h->cfg.devices = nullptr;
        const int mrc = md_create(h, C);
        if (mrc) {
            md_release(h);
            delete h;
            return mrc;
        }
        *out = h;
        return PDPLQR_OK;
    }
    int rc = PDPLQR_OK;
    hipError_t e = hipSetDevice(C.device);
    if (e != hipSuccess) {
        set_error(std::string("hipSetDevice: ") + hipGetErrorString(e));
        delete h;
        return PDPLQR_ERR_HIP;
    }
    e = hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        set_error(std::string("hipStreamCreate: ") + hipGetErrorString(e));
        delete h;
        return PDPLQR_ERR_HIP;
    }
    h->stream = h->own_stream;
    sh.x1 = one_wave_per_simd(C.device, sh.batch);
    const long long B = sh.batch;
#define ALLOC(ptr, cnt)                                  \
    do {                                                 \
        if ((rc = dalloc(h, &(ptr), (size_t)(cnt))) != 0) \
            goto fail;                                   \
    } while (0)
    ALLOC(h->E, B * sh.perE);
    ALLOC(h->c, B * sh.perc);
    ALLOC(h->H, B * sh.perH);
    ALLOC(h->h, B * sh.perh);
    ALLOC(h->D, B * sh.ndD);
    ALLOC(h->Hw, B * sh.perHw);
    ALLOC(h->hw, B * sh.perh);
    ALLOC(h->gw, B * sh.ny);
    ALLOC(h->KD, B * sh.perKD);
    if (C.keep_factors) {
        ALLOC(h->Lc, B * sh.perHw);
        ALLOC(h->lpc, B * sh.perh);
    }
    ALLOC(h->status, B);
    ALLOC(h->d_off, C.N + 2);
    ALLOC(h->y_off, C.N + 2);
    ALLOC(h->tab_s, sh.ps);
    ALLOC(h->tab_n, sh.pn);
    ALLOC(h->st_ws, B * sh.perh);
    ALLOC(h->st_y, B * sh.ny);
    ALLOC(h->st_z, B * sh.ny);
    ALLOC(h->st_ir, B * sh.ny);
    ALLOC(h->st_rho, B * sh.ny);
    ALLOC(h->st_x0, B * sh.n);
#undef ALLOC
    {
        std::vector<short2> ts(sh.ps), tn(sh.pn);
        int q = 0;
        for (int j = 0; j < sh.s; ++j)
            for (int i = j; i < sh.s; ++i) ts[q++] = make_short2((short)i, (short)j);
        q = 0;
        for (int j = 0; j < sh.n; ++j)
            for (int i = j; i < sh.n; ++i) tn[q++] = make_short2((short)i, (short)j);
        e = hipMemcpy(h->tab_s, ts.data(), ts.size() * sizeof(short2), hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(h->tab_n, tn.data(), tn.size() * sizeof(short2), hipMemcpyHostToDevice);
        if (e == hipSuccess)
            e = hipMemcpy(h->d_off, h->d_off_h.data(), h->d_off_h.size() * sizeof(int32_t), hipMemcpyHostToDevice);
        if (e == hipSuccess)
            e = hipMemcpy(h->y_off, h->y_off_h.data(), h->y_off_h.size() * sizeof(int32_t), hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemset(h->status, 0, B * sizeof(int32_t));
        if (e == hipSuccess) e = hipMemset(h->D, 0, std::max<long long>(1, B * sh.ndD) * sizeof(double));
        if (e != hipSuccess) {
            set_error(std::string("create: ") + hipGetErrorString(e));
            rc = PDPLQR_ERR_HIP;
            goto fail;
        }
    }
    rc = solver_init(h);
    if (rc != PDPLQR_OK) goto fail;
    // the null-stream fills of create and solver_init are complete before any
    // (non-blocking) handle stream runs
    if (!h->md && hipStreamSynchronize(nullptr) != hipSuccess) {
        set_error("create: synchronize after the workspace fills failed");
        rc = PDPLQR_ERR_HIP;
        goto fail;
    }
    *out = h;
    return PDPLQR_OK;
fail:
    solver_release(h);
    free_all(h);
    delete h;
    return rc;
}

int pdplqr_destroy(pdplqr_handle h) {
    if (!h) return PDPLQR_OK;
    if (h->md) {
        const int d0 = md_primary_device(h);
        md_release(h);
        (void)hipSetDevice(d0);  // admm_solve's vectors (allocated on the first device)
        admm_release(h);
        for (void *p : h->allocs) (void)hipFree(p);
        delete h;
        return PDPLQR_OK;
    }
    (void)hipSetDevice(h->cfg.device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    solver_release(h);
    free_all(h);
    delete h;
    return PDPLQR_OK;
}

int pdplqr_set_stream(pdplqr_handle h, void *stream) {
    if (!h) return invalid("null handle");
    if (h->md) return md_set_stream(h, stream);
    hipStream_t next = stream ? reinterpret_cast<hipStream_t>(stream) : h->own_stream;
    if (next != h->stream) {
        // work already queued on the old stream (set_model's repack, a solve)
        // precedes everything queued on the new one: without this a model
        // uploaded before the switch can still be in flight when the first
        // kernel on the new stream reads it
        PDPLQR_HIP_TRY(hipSetDevice(h->cfg.device));
        hipEvent_t ev;
        PDPLQR_HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        hipError_t e = hipEventRecord(ev, h->stream);
        if (e == hipSuccess) e = hipStreamWaitEvent(next, ev, 0);
        (void)hipEventDestroy(ev);
        PDPLQR_HIP_TRY(e);
    }
    h->stream = next;
    return PDPLQR_OK;
}

void *pdplqr_get_stream(pdplqr_handle h) {
    if (h && h->md) return md_stream(h);  // the caller stream, else the first slice's device stream
    return h ? reinterpret_cast<void *>(h->stream) : nullptr;
}

int pdplqr_synchronize(pdplqr_handle h) {
    if (!h) return invalid("null handle");
    if (h->md) return md_synchronize(h);
    PDPLQR_HIP_TRY(hipSetDevice(h->cfg.device));
    PDPLQR_HIP_TRY(hipStreamSynchronize(h->stream));
    return PDPLQR_OK;
}

int pdplqr_set_model_arrays(pdplqr_handle h, int mask, const double *E, const double *c, const double *H,
                            const double *hv, const double *D, int mem) {
    if (!h) return invalid("null handle");
    if (mask & ~PDPLQR_MODEL_ALL) return invalid("set_model_arrays: unknown mask bits");
    if (!h->model_set && mask != PDPLQR_MODEL_ALL) return invalid("set_model_arrays: the first upload needs every array");
    if (((mask & PDPLQR_MODEL_E) && !E) || ((mask & PDPLQR_MODEL_C) && !c) || ((mask & PDPLQR_MODEL_H) && !H) ||
        ((mask & PDPLQR_MODEL_HV) && !hv))
        return invalid("set_model: null E/c/H/h");
    if ((mask & PDPLQR_MODEL_D) && h->sh.ndD > 0 && !D) return invalid("set_model: constraints declared but D is null");
    if (h->md) return md_set_model(h, mask, E, c, H, hv, D, mem);
    PDPLQR_HIP_TRY(hipSetDevice(h->cfg.device));
    const Shape &sh = h->sh;
    const long long B = sh.batch;
    const hipMemcpyKind kind = mem == PDPLQR_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    if (h->cfg.solver == PDPLQR_SOLVER_KKT && (mask & (PDPLQR_MODEL_E | PDPLQR_MODEL_D))) {
        const int rc = kkt_before_model(h);  // the frozen KKT matrix keeps the constructor's E, D
        if (rc) return rc;
    }
    long long bytes = 0;
    auto put = [&](double *dst, const double *src, long long count) -> int {
        PDPLQR_HIP_TRY(hipMemcpyAsync(dst, src, count * sizeof(double), kind, h->stream));
        bytes += count * (long long)sizeof(double);
        return PDPLQR_OK;
    };
    int rc;
    if ((mask & PDPLQR_MODEL_E) && (rc = put(h->E, E, B * sh.perE))) return rc;
    if ((mask & PDPLQR_MODEL_C) && (rc = put(h->c, c, B * sh.perc))) return rc;
    if ((mask & PDPLQR_MODEL_H) && (rc = put(h->H, H, B * sh.perH))) return rc;
    if ((mask & PDPLQR_MODEL_HV) && (rc = put(h->h, hv, B * sh.perh))) return rc;
    if ((mask & PDPLQR_MODEL_D) && sh.ndD > 0 && (rc = put(h->D, D, B * sh.ndD))) return rc;
    if (mem != PDPLQR_MEM_DEVICE) {
        PDPLQR_HIP_TRY(hipStreamSynchronize(h->stream));
        h->model_upload_bytes += bytes;
    }
    const bool first = !h->model_set;
    h->model_set = true;
    if ((mask & (PDPLQR_MODEL_H | PDPLQR_MODEL_HV)) && h->cfg.solver != PDPLQR_SOLVER_KKT) {
        h->hw_cached = false;  // H~ is re-formed from the new model
        h->updated = false;
    }
    // KKT: the matrix (H + sigma_f I) is frozen at the first upload and the
    // right-hand side was formed by update_problem_data (form_rhs,
    // kkt.hpp:224-300), so a later H / h upload leaves the protocol state as
    // it is: backward without a new update_problem_data stays valid, as in the
    // reference's QDLDLSolver.
    // The factor cache survives a model upload: the reference re-reads model_
    // lazily and never invalidates its workspace factors (lqr_solver.hpp:25,65-70).
    return first || h->cfg.solver == PDPLQR_SOLVER_KKT ? solver_on_model(h) : PDPLQR_OK;
}

int pdplqr_set_model(pdplqr_handle h, const double *E, const double *c, const double *H, const double *hv,
                     const double *D, int mem) {
    if (!h) return invalid("null handle");
    if (!E || !c || !H || !hv) return invalid("set_model: null E/c/H/h");
    return pdplqr_set_model_arrays(h, PDPLQR_MODEL_ALL, E, c, H, hv, D, mem);
}

int pdplqr_get_model_upload_bytes(pdplqr_handle h, int64_t *bytes) {
    if (!h || !bytes) return invalid("null handle or output");
    *bytes = h->model_upload_bytes;
    return PDPLQR_OK;
}

int pdplqr_update_problem_data(pdplqr_handle h, const double *ws, const double *ys, const double *zs,
                               const double *inv_rho, double sigma, int mem) {
    if (!h) return invalid("null handle");
    if (!h->model_set) {
        set_error("update_problem_data before set_model");
        return PDPLQR_ERR_STATE;
    }
    if (h->md) return md_update(h, ws, ys, zs, inv_rho, sigma, mem);
    PDPLQR_HIP_TRY(hipSetDevice(h->cfg.device));
    const Shape &sh = h->sh;
    const long long B = sh.batch;
    const double *dws, *dy = h->st_y, *dz = h->st_z, *dir = h->st_ir;
    int rc;
    if ((rc = stage_in(h, ws, h->st_ws, B * sh.perh, mem, &dws))) return rc;
    if (sh.ny > 0) {
        if ((rc = stage_in(h, ys, h->st_y, B * sh.ny, mem, &dy))) return rc;
        if ((rc = stage_in(h, zs, h->st_z, B * sh.ny, mem, &dz))) return rc;
        if ((rc = stage_in(h, inv_rho, h->st_ir, B * sh.ny, mem, &dir))) return rc;
    }
    rc = solver_update(h, dws, dy, dz, dir, sigma);
    if (rc) return rc;
    if (h->host_staged) PDPLQR_HIP_TRY(hipStreamSynchronize(h->stream));
    h->host_staged = false;
    h->updated = true;
    return PDPLQR_OK;
}

static int backward_common(pdplqr_handle h, const double *rho, int mem, bool fact) {
    if (!h) return invalid("null handle");
    if (!h->updated) {
        set_error("backward before update_problem_data");
        return PDPLQR_ERR_STATE;
    }
    if (!fact && !h->factored) {
        set_error("backward_without_factorization needs a preceding backward");
        return PDPLQR_ERR_STATE;
    }
    if (h->md) return md_backward(h, rho, mem, fact);
    PDPLQR_HIP_TRY(hipSetDevice(h->cfg.device));
    h->host_staged = false;
    const Shape &sh = h->sh;
    const double *drho = h->st_rho;
    int rc;
    if (sh.ny > 0 && (rc = stage_in(h, rho, h->st_rho, (long long)sh.batch * sh.ny, mem, &drho))) return rc;
    rc = fact ? solver_backward(h, drho) : solver_backward_nofact(h, drho);
    if (rc) return rc;
    if (h->host_staged) PDPLQR_HIP_TRY(hipStreamSynchronize(h->stream));
    h->host_staged = false;
    if (fact) h->factored = true;
    return PDPLQR_OK;
}

int pdplqr_backward(pdplqr_handle h, const double *rho, int mem) { return backward_common(h, rho, mem, true); }

int pdplqr_backward_without_factorization(pdplqr_handle h, const double *rho, int mem) {
    if (h && h->cfg.solver == PDPLQR_SOLVER_KKT) {
        set_error("QDLDLSolver has no backward_without_factorization");
        return PDPLQR_ERR_UNSUPPORTED;
    }
    if (h && !h->cfg.keep_factors) {
        set_error("backward_without_factorization requires keep_factors = 1");
        return PDPLQR_ERR_STATE;
    }
    return backward_common(h, rho, mem, false);
}

int pdplqr_forward(pdplqr_handle h, const double *x0, double *ws, int mem) {
    if (!h) return invalid("null handle");
    if (!h->factored) {
        set_error("forward before backward");
        return PDPLQR_ERR_STATE;
    }
    if (!x0 || !ws) return invalid("forward: null x0/ws");
    if (h->md) return md_forward(h, x0, ws, mem);
    PDPLQR_HIP_TRY(hipSetDevice(h->cfg.device));
    const Shape &sh = h->sh;
    const double *dx0;
    int rc;
    if ((rc = stage_in(h, x0, h->st_x0, (long long)sh.batch * sh.n, mem, &dx0))) return rc;
    double *dws = mem == PDPLQR_MEM_DEVICE ? ws : h->st_ws;
    rc = solver_forward(h, dx0, dws);
    if (rc) return rc;
    h->host_staged = false;
    if (mem != PDPLQR_MEM_DEVICE) {
        PDPLQR_HIP_TRY(hipMemcpyAsync(ws, dws, (size_t)sh.batch * sh.perh * sizeof(double), hipMemcpyDeviceToHost,
                                      h->stream));
        PDPLQR_HIP_TRY(hipStreamSynchronize(h->stream));
    }
    return PDPLQR_OK;
}

int pdplqr_clear_workspace(pdplqr_handle h) {
    if (!h) return invalid("null handle");
    if (h->md) return md_clear(h);
    PDPLQR_HIP_TRY(hipSetDevice(h->cfg.device));
    const Shape &sh = h->sh;
    const long long B = sh.batch;
    PDPLQR_HIP_TRY(hipMemsetAsync(h->Hw, 0, B * sh.perHw * sizeof(double), h->stream));
    h->hw_cached = false;
    PDPLQR_HIP_TRY(hipMemsetAsync(h->hw, 0, B * sh.perh * sizeof(double), h->stream));
    if (sh.ny) PDPLQR_HIP_TRY(hipMemsetAsync(h->gw, 0, B * sh.ny * sizeof(double), h->stream));
    PDPLQR_HIP_TRY(hipMemsetAsync(h->KD, 0, B * sh.perKD * sizeof(double), h->stream));
    if (h->Lc) PDPLQR_HIP_TRY(hipMemsetAsync(h->Lc, 0, B * sh.perHw * sizeof(double), h->stream));
    if (h->lpc) PDPLQR_HIP_TRY(hipMemsetAsync(h->lpc, 0, B * sh.perh * sizeof(double), h->stream));
    int rc = solver_clear(h);
    if (rc) return rc;
    PDPLQR_HIP_TRY(hipStreamSynchronize(h->stream));
    return PDPLQR_OK;
}

int pdplqr_get_value_function(pdplqr_handle h, int32_t b, int32_t k, double *P, double *p) {
    if (!h) return invalid("null handle");
    if (h->cfg.solver != PDPLQR_SOLVER_SERIAL || !h->cfg.keep_factors)
        return invalid("get_value_function needs a SERIAL handle with keep_factors = 1");
    const Shape &sh = h->sh;
    if (b < 0 || b >= sh.batch || k < 0 || k > sh.N) return invalid("get_value_function: index out of range");
    if (!h->factored) {
        set_error("get_value_function before backward");
        return PDPLQR_ERR_STATE;
    }
    PDPLQR_HIP_TRY(hipSetDevice(h->cfg.device));
    const int dim = k < sh.N ? sh.s : sh.n, off = dim - sh.n;
    const int pk = k < sh.N ? sh.ps : sh.pn;
    std::vector<double> Lp(pk), lp(dim);
    PDPLQR_HIP_TRY(hipStreamSynchronize(h->stream));
    PDPLQR_HIP_TRY(hipMemcpy(Lp.data(), h->Lc + (long long)b * sh.perHw + (long long)k * sh.ps, pk * sizeof(double),
                             hipMemcpyDeviceToHost));
    PDPLQR_HIP_TRY(hipMemcpy(lp.data(), h->lpc + (long long)b * sh.perh + (long long)k * sh.s, dim * sizeof(double),
                             hipMemcpyDeviceToHost));
    auto Lat = [&](int i, int j) -> double {  // packed lower, column-major
        if (i < j) return 0.0;
        return Lp[j * dim - (j * (j - 1)) / 2 + (i - j)];
    };
    const int n = sh.n;
    if (P)
        for (int j = 0; j < n; ++j)
            for (int i = 0; i < n; ++i) {
                double a = 0.0;
                for (int t = 0; t < n; ++t) a += Lat(off + i, off + t) * Lat(off + j, off + t);
                P[i + j * n] = a;
            }
    if (p)
        for (int i = 0; i < n; ++i) p[i] = lp[off + i];
    return PDPLQR_OK;
}

int pdplqr_get_status(pdplqr_handle h, int32_t *flags) {
    if (!h || !flags) return invalid("null argument");
    if (h->md) return md_status(h, flags);
    PDPLQR_HIP_TRY(hipSetDevice(h->cfg.device));
    PDPLQR_HIP_TRY(hipStreamSynchronize(h->stream));
    return solver_status(h, flags);
}

}  // extern "C"
