// admm.hip -- the ADMM outer loop for conic LQ around the three solvers
// (DESIGN.md section 5 "ADMM outer loop").
//
// The reference's protocol is the x-update of an OSQP-style ADMM (SURVEY
// section 0.1): update_problem_data(ws, ys, zs, inv_rho, sigma) forms
// H~ = H + sigma I, h~ = h - sigma w_bar, g = z - inv_rho o y
// (lqr_solver.hpp:41-56) and backward(rho) adds D^T rho D and -D^T rho g
// (lqr_kernel.hpp:106-112).  It stores the bounds e_lb <= D w <= e_ub
// (lqr_model.hpp:21-24) but never reads them: the outer loop is absent
// (README.md:8).  It is restated here from OSQP's published iteration
// (Stellato et al., "OSQP: an operator splitting solver for quadratic
// programs", Math. Prog. Comp. 12 (2020), Algorithm 1), with the dynamics as
// the hard equality constraints of the x-update (solved exactly by the LQ
// solve) and D w in [e_lb, e_ub] as the ADMM-split constraint:
//     w~      = LQ solve with (w^k, y^k, z^k)                  (the protocol)
//     v       = D w~,       v_rel = alpha v + (1 - alpha) z^k
//     w^{k+1} = alpha w~ + (1 - alpha) w^k
//     z^{k+1} = clamp(v_rel + inv_rho o y^k, e_lb, e_ub)
//     y^{k+1} = y^k + rho o (v_rel - z^{k+1})
// Termination (every check_every iterations and at max_iter), per problem:
//     r_prim = |D w^{k+1} - z^{k+1}|_inf <= eps_abs + eps_rel max(|D w^{k+1}|_inf, |z^{k+1}|_inf)
//     r_dual = |D^T rho o (z^{k+1} - z^k)|_inf <= eps_abs + eps_rel |D^T y^{k+1}|_inf
// (the ADMM dual residual of Boyd et al. 2011, section 3.3: the dynamics
// multipliers of the LQ solve are not formed).  A converged problem is frozen:
// its w, y, z stop changing while the rest of the batch iterates.
//
// With rho fixed the stage matrices never change after the first backward, so
// iterations >= 2 need only vectors:
//   * k_admm_update (one thread per stage, one 64-stage wave per problem slice)
//     does the z/y/w step AND the next update_problem_data + penalty linear
//     term in the same pass: h~ = h - sigma w^{k+1} - D^T (rho o g^{k+1}),
//     g^{k+1} = z^{k+1} - inv_rho o y^{k+1} -- in the same operation order as
//     k_update_problem_data followed by k_penalty, so the fused and the
//     protocol-level iterations agree bit for bit;
//   * the backward is backward_without_factorization (keep_factors = 1) or
//     the factorizing kernel on the unchanged H~ (keep_factors = 0);
//   * the KKT solver re-forms its right-hand side (form_rhs) and re-solves
//     with the factor of the first iteration (the KKT matrix depends on rho
//     only, qdldl_solver.hpp:88-109).
#include <algorithm>

#include "solvers.hpp"

namespace pdplqr {

struct AdmmState {
    double *wt = nullptr;  // LQ solution of the current iteration (forward output)
    double *w = nullptr, *y = nullptr, *z = nullptr;
    double *lb = nullptr, *ub = nullptr, *rho = nullptr, *irho = nullptr;
    double *dzr = nullptr;  // rho o (z^{k+1} - z^k), scratch of the residual pass
    double *x0 = nullptr;
    double *prim = nullptr, *dual = nullptr;  // [b] residuals at the last check
    unsigned long long *acc = nullptr;         // [b][5] running maxima (bit patterns of non-negative doubles)
    int32_t *done = nullptr, *iters = nullptr, *conv = nullptr, *active = nullptr;
    int32_t *active_h = nullptr;  // pinned
};

struct AdmmArgs {
    Shape sh;
    const double *D, *hv, *wt, *lb, *ub, *rho, *irho;
    double *w, *y, *z, *dzr, *hw, *gw;
    const int32_t *d_off, *y_off, *done;
    unsigned long long *acc;
    double alpha, sigma;
};

enum { ACC_PRIM = 0, ACC_DW = 1, ACC_Z = 2, ACC_DUAL = 3, ACC_DTY = 4, ACC_N = 5 };

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = fmax(v, __shfl_xor(v, m, 64));
    return v;
}

// grid (ceil((N + 1) / 256), batch), 256 threads: thread = stage k of problem b
template <bool FUSE, bool CHECK>
__global__ void __launch_bounds__(256) k_admm_update(AdmmArgs a) {
    const Shape &sh = a.sh;
    const int b = blockIdx.y;
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const bool act = k <= sh.N && a.done[b] == 0;
    double rp = 0.0, dwm = 0.0, zm = 0.0, rd = 0.0, dty = 0.0;
    if (act) {
        const int dim = k < sh.N ? sh.s : sh.n;
        const long long wo = (long long)b * sh.perh + (long long)k * sh.s;
        const int yo0 = a.y_off[k], nc = a.y_off[k + 1] - yo0;
        const long long yo = (long long)b * sh.ny + yo0;
        const double *Dk = a.D + (long long)b * sh.ndD + a.d_off[k];
        const double *wt = a.wt + wo;
        double *w = a.w + wo;
        const double al = a.alpha, bl = 1.0 - a.alpha;
        for (int r = 0; r < nc; ++r) {
            double v = 0.0, vw = 0.0;
            for (int j = 0; j < dim; ++j) {
                const double d = Dk[r + j * nc];
                v += d * wt[j];
                vw += d * w[j];
            }
            const double zr = a.z[yo + r], yr = a.y[yo + r], rr = a.rho[yo + r], ir = a.irho[yo + r];
            const double vrel = al * v + bl * zr;
            const double zn = fmin(fmax(vrel + ir * yr, a.lb[yo + r]), a.ub[yo + r]);
            const double yn = yr + rr * (vrel - zn);
            a.z[yo + r] = zn;
            a.y[yo + r] = yn;
            if (FUSE) a.gw[yo + r] = zn - ir * yn;
            if (CHECK) {
                a.dzr[yo + r] = rr * (zn - zr);
                const double dwn = al * v + bl * vw;  // D w^{k+1}
                rp = fmax(rp, fabs(dwn - zn));
                dwm = fmax(dwm, fabs(dwn));
                zm = fmax(zm, fabs(zn));
            }
        }
        const double *hk = a.hv + wo;
        double *hwk = a.hw + wo;
        const double *gk = a.gw + yo;
        for (int j = 0; j < dim; ++j) {
            const double wn = al * wt[j] + bl * w[j];
            w[j] = wn;
            if (FUSE || CHECK) {
                double ag = 0.0, ad = 0.0, ay = 0.0;
                for (int r = 0; r < nc; ++r) {
                    const double d = Dk[r + j * nc];
                    if (FUSE) ag += d * (a.rho[yo + r] * gk[r]);
                    if (CHECK) {
                        ad += d * a.dzr[yo + r];
                        ay += d * a.y[yo + r];
                    }
                }
                if (FUSE) {
                    // k_update_problem_data then k_penalty: (h - sigma w) - sum
                    double hj = hk[j] - a.sigma * wn;
                    if (nc > 0) hj -= ag;
                    hwk[j] = hj;
                }
                if (CHECK) {
                    rd = fmax(rd, fabs(ad));
                    dty = fmax(dty, fabs(ay));
                }
            }
        }
    }
    if (CHECK) {
        // one problem per block: wave maxima, then one atomic per wave
        rp = wave_max(rp);
        dwm = wave_max(dwm);
        zm = wave_max(zm);
        rd = wave_max(rd);
        dty = wave_max(dty);
        if ((threadIdx.x & 63) == 0 && a.done[b] == 0) {
            unsigned long long *ac = a.acc + (long long)b * ACC_N;
            atomicMax(ac + ACC_PRIM, (unsigned long long)__double_as_longlong(rp));
            atomicMax(ac + ACC_DW, (unsigned long long)__double_as_longlong(dwm));
            atomicMax(ac + ACC_Z, (unsigned long long)__double_as_longlong(zm));
            atomicMax(ac + ACC_DUAL, (unsigned long long)__double_as_longlong(rd));
            atomicMax(ac + ACC_DTY, (unsigned long long)__double_as_longlong(dty));
        }
    }
}

// per problem: termination test of iteration `it`, then reset the maxima
__global__ void k_admm_check(int batch, int it, double eps_abs, double eps_rel, unsigned long long *acc,
                             int32_t *done, int32_t *iters, int32_t *conv, double *prim, double *dual,
                             int32_t *active) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch || done[b]) return;
    unsigned long long *ac = acc + (long long)b * ACC_N;
    const double rp = __longlong_as_double((long long)ac[ACC_PRIM]), dw = __longlong_as_double((long long)ac[ACC_DW]),
                 zm = __longlong_as_double((long long)ac[ACC_Z]), rd = __longlong_as_double((long long)ac[ACC_DUAL]),
                 dty = __longlong_as_double((long long)ac[ACC_DTY]);
#pragma unroll
    for (int q = 0; q < ACC_N; ++q) ac[q] = 0ull;
    iters[b] = it;
    prim[b] = rp;
    dual[b] = rd;
    const bool ok = rp <= eps_abs + eps_rel * fmax(dw, zm) && rd <= eps_abs + eps_rel * dty;
    if (ok) {
        done[b] = 1;
        conv[b] = 1;
    } else {
        atomicAdd(active, 1);
    }
}

__global__ void k_admm_init(long long ny_total, const double *__restrict__ rho, double *__restrict__ irho) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < ny_total) irho[t] = 1.0 / rho[t];
}

template <typename X>
static int aalloc(pdplqr_handle h, X **p, size_t count) {
    *p = nullptr;
    void *q = nullptr;
    hipError_t e = hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(X));
    if (e != hipSuccess) {
        set_error(std::string("hipMalloc: ") + hipGetErrorString(e));
        return PDPLQR_ERR_ALLOC;
    }
    h->allocs.push_back(q);
    *p = reinterpret_cast<X *>(q);
    return PDPLQR_OK;
}

static int admm_alloc(pdplqr_handle h) {
    if (h->admm) return PDPLQR_OK;
    AdmmState *s = new AdmmState();
    h->admm = s;
    const Shape &sh = h->sh;
    const long long B = sh.batch, W = B * sh.perh, Y = B * sh.ny;
    int rc;
    if ((rc = aalloc(h, &s->wt, W)) || (rc = aalloc(h, &s->w, W)) || (rc = aalloc(h, &s->y, Y)) ||
        (rc = aalloc(h, &s->z, Y)) || (rc = aalloc(h, &s->lb, Y)) || (rc = aalloc(h, &s->ub, Y)) ||
        (rc = aalloc(h, &s->rho, Y)) || (rc = aalloc(h, &s->irho, Y)) || (rc = aalloc(h, &s->dzr, Y)) ||
        (rc = aalloc(h, &s->x0, B * sh.n)) || (rc = aalloc(h, &s->prim, B)) || (rc = aalloc(h, &s->dual, B)) ||
        (rc = aalloc(h, &s->acc, B * ACC_N)) || (rc = aalloc(h, &s->done, B)) || (rc = aalloc(h, &s->iters, B)) ||
        (rc = aalloc(h, &s->conv, B)) || (rc = aalloc(h, &s->active, 1)))
        return rc;
    PDPLQR_HIP_TRY(hipHostMalloc((void **)&s->active_h, sizeof(int32_t), hipHostMallocDefault));
    return PDPLQR_OK;
}

void admm_release(pdplqr_handle h) {
    if (!h->admm) return;
    if (h->admm->active_h) (void)hipHostFree(h->admm->active_h);
    delete h->admm;
    h->admm = nullptr;
}

}  // namespace pdplqr

using namespace pdplqr;

extern "C" {

void pdplqr_admm_settings_init(pdplqr_admm_settings *s) {
    if (!s) return;
    s->sigma = 1e-6;  // lqr_example.cpp:170
    s->alpha = 1.6;   // OSQP default relaxation
    s->max_iter = 4000;
    s->check_every = 25;
    s->eps_abs = 1e-3;
    s->eps_rel = 1e-3;
}

int pdplqr_admm_solve(pdplqr_handle h, const pdplqr_admm_settings *st, const double *x0, const double *lb,
                      const double *ub, const double *rho, double *ws, double *ys, double *zs, int mem) {
    if (!h || !st) return PDPLQR_ERR_INVALID;
    if (!h->model_set) {
        set_error("admm_solve before set_model");
        return PDPLQR_ERR_STATE;
    }
    if (!x0 || !ws) {
        set_error("admm_solve: null x0/ws");
        return PDPLQR_ERR_INVALID;
    }
    const Shape &sh = h->sh;
    if (sh.ny > 0 && (!lb || !ub || !rho || !ys || !zs)) {
        set_error("admm_solve: constraints declared but lb/ub/rho/ys/zs is null");
        return PDPLQR_ERR_INVALID;
    }
    if (st->max_iter < 1 || st->check_every < 1 || !(st->alpha > 0.0 && st->alpha < 2.0) || !(st->sigma >= 0.0) ||
        !(st->eps_abs >= 0.0) || !(st->eps_rel >= 0.0)) {
        set_error("admm_solve: bad settings (max_iter >= 1, check_every >= 1, 0 < alpha < 2, sigma, eps >= 0)");
        return PDPLQR_ERR_INVALID;
    }
    PDPLQR_HIP_TRY(hipSetDevice(h->cfg.device));
    int rc = admm_alloc(h);
    if (rc) return rc;
    AdmmState *s = h->admm;
    hipStream_t S = h->stream;
    const long long B = sh.batch, W = B * sh.perh, Y = B * sh.ny;
    const hipMemcpyKind kin = mem == PDPLQR_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    PDPLQR_HIP_TRY(hipMemcpyAsync(s->w, ws, W * sizeof(double), kin, S));
    PDPLQR_HIP_TRY(hipMemcpyAsync(s->x0, x0, B * sh.n * sizeof(double), kin, S));
    if (Y > 0) {
        PDPLQR_HIP_TRY(hipMemcpyAsync(s->y, ys, Y * sizeof(double), kin, S));
        PDPLQR_HIP_TRY(hipMemcpyAsync(s->z, zs, Y * sizeof(double), kin, S));
        PDPLQR_HIP_TRY(hipMemcpyAsync(s->lb, lb, Y * sizeof(double), kin, S));
        PDPLQR_HIP_TRY(hipMemcpyAsync(s->ub, ub, Y * sizeof(double), kin, S));
        PDPLQR_HIP_TRY(hipMemcpyAsync(s->rho, rho, Y * sizeof(double), kin, S));
        hipLaunchKernelGGL(k_admm_init, dim3((unsigned)((Y + 255) / 256)), dim3(256), 0, S, Y, s->rho, s->irho);
        PDPLQR_HIP_TRY(hipGetLastError());
    }
    PDPLQR_HIP_TRY(hipMemsetAsync(s->acc, 0, B * ACC_N * sizeof(unsigned long long), S));
    PDPLQR_HIP_TRY(hipMemsetAsync(s->done, 0, B * sizeof(int32_t), S));
    PDPLQR_HIP_TRY(hipMemsetAsync(s->conv, 0, B * sizeof(int32_t), S));
    PDPLQR_HIP_TRY(hipMemsetAsync(s->iters, 0, B * sizeof(int32_t), S));
    PDPLQR_HIP_TRY(hipMemsetAsync(s->prim, 0, B * sizeof(double), S));
    PDPLQR_HIP_TRY(hipMemsetAsync(s->dual, 0, B * sizeof(double), S));

    const bool kkt = h->cfg.solver == PDPLQR_SOLVER_KKT;
    AdmmArgs a;
    a.sh = sh;
    a.D = h->D;
    a.hv = h->h;
    a.wt = s->wt;
    a.lb = s->lb;
    a.ub = s->ub;
    a.rho = s->rho;
    a.irho = s->irho;
    a.w = s->w;
    a.y = s->y;
    a.z = s->z;
    a.dzr = s->dzr;
    a.hw = h->hw;
    a.gw = h->gw;
    a.d_off = h->d_off;
    a.y_off = h->y_off;
    a.done = s->done;
    a.acc = s->acc;
    a.alpha = st->alpha;
    a.sigma = st->sigma;
    const dim3 ugrid((unsigned)((sh.N + 1 + 255) / 256), (unsigned)B), ublk(256);
    const double *irho_or_null = Y > 0 ? s->irho : nullptr;
    int it = 1;
    for (;; ++it) {
        // x-update: the reference protocol (iteration 1), then vectors only
        if (it == 1 || kkt) {
            if ((rc = solver_update(h, s->w, s->y, s->z, irho_or_null, st->sigma))) return rc;
            h->updated = true;
        }
        if (it == 1) {
            if ((rc = solver_backward(h, kkt ? s->irho : s->rho))) return rc;
            h->factored = true;
        } else if (!kkt) {
            if ((rc = solver_backward_prepared(h))) return rc;
        }
        if ((rc = solver_forward(h, s->x0, s->wt))) return rc;
        if (Y == 0) {  // nothing to split: one LQ solve is the answer
            PDPLQR_HIP_TRY(hipMemcpyAsync(s->w, s->wt, W * sizeof(double), hipMemcpyDeviceToDevice, S));
            std::vector<int32_t> one(B, 1);
            PDPLQR_HIP_TRY(hipMemcpyAsync(s->iters, one.data(), B * sizeof(int32_t), hipMemcpyHostToDevice, S));
            PDPLQR_HIP_TRY(hipMemcpyAsync(s->conv, one.data(), B * sizeof(int32_t), hipMemcpyHostToDevice, S));
            PDPLQR_HIP_TRY(hipStreamSynchronize(S));
            break;
        }
        const bool last = it >= st->max_iter;
        const bool check = last || it % st->check_every == 0;
        const bool fuse = !kkt && !last;
        if (fuse && check) hipLaunchKernelGGL((k_admm_update<true, true>), ugrid, ublk, 0, S, a);
        else if (fuse) hipLaunchKernelGGL((k_admm_update<true, false>), ugrid, ublk, 0, S, a);
        else if (check) hipLaunchKernelGGL((k_admm_update<false, true>), ugrid, ublk, 0, S, a);
        else hipLaunchKernelGGL((k_admm_update<false, false>), ugrid, ublk, 0, S, a);
        PDPLQR_HIP_TRY(hipGetLastError());
        if (check) {
            PDPLQR_HIP_TRY(hipMemsetAsync(s->active, 0, sizeof(int32_t), S));
            hipLaunchKernelGGL(k_admm_check, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, S, (int)B, it,
                               st->eps_abs, st->eps_rel, s->acc, s->done, s->iters, s->conv, s->prim, s->dual,
                               s->active);
            PDPLQR_HIP_TRY(hipGetLastError());
            PDPLQR_HIP_TRY(hipMemcpyAsync(s->active_h, s->active, sizeof(int32_t), hipMemcpyDeviceToHost, S));
            PDPLQR_HIP_TRY(hipStreamSynchronize(S));
            if (*s->active_h == 0) break;
        }
        if (last) break;
    }
    // fused iterations leave h~/g of the NEXT x-update in the workspace; the
    // protocol state is "updated and factored" either way
    const hipMemcpyKind kout = mem == PDPLQR_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    PDPLQR_HIP_TRY(hipMemcpyAsync(ws, s->w, W * sizeof(double), kout, S));
    if (Y > 0) {
        PDPLQR_HIP_TRY(hipMemcpyAsync(ys, s->y, Y * sizeof(double), kout, S));
        PDPLQR_HIP_TRY(hipMemcpyAsync(zs, s->z, Y * sizeof(double), kout, S));
    }
    if (mem != PDPLQR_MEM_DEVICE) PDPLQR_HIP_TRY(hipStreamSynchronize(S));
    h->hw_cached = false;
    h->admm_iters = it;
    return PDPLQR_OK;
}

int pdplqr_admm_info(pdplqr_handle h, int32_t *iters, int32_t *converged, double *prim_res, double *dual_res) {
    if (!h) return PDPLQR_ERR_INVALID;
    if (!h->admm) {
        set_error("admm_info before admm_solve");
        return PDPLQR_ERR_STATE;
    }
    PDPLQR_HIP_TRY(hipSetDevice(h->cfg.device));
    PDPLQR_HIP_TRY(hipStreamSynchronize(h->stream));
    AdmmState *s = h->admm;
    const size_t B = (size_t)h->sh.batch;
    if (iters) PDPLQR_HIP_TRY(hipMemcpy(iters, s->iters, B * sizeof(int32_t), hipMemcpyDeviceToHost));
    if (converged) PDPLQR_HIP_TRY(hipMemcpy(converged, s->conv, B * sizeof(int32_t), hipMemcpyDeviceToHost));
    if (prim_res) PDPLQR_HIP_TRY(hipMemcpy(prim_res, s->prim, B * sizeof(double), hipMemcpyDeviceToHost));
    if (dual_res) PDPLQR_HIP_TRY(hipMemcpy(dual_res, s->dual, B * sizeof(double), hipMemcpyDeviceToHost));
    return h->admm_iters;
}

}  // extern "C"
