// solvers.hip -- dispatch of the protocol calls to the three solver kinds.
#include "solvers.hpp"

namespace pdplqr {

static int unsupported(const char *what) {
    set_error(std::string(what) + ": not implemented in this build");
    return PDPLQR_ERR_UNSUPPORTED;
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
    return a;
}

int solver_init(pdplqr_handle h) {
    if (h->cfg.solver == PDPLQR_SOLVER_SERIAL) {
        if (h->sh.s > 32) return unsupported("SERIAL solver with n + m > 32");
        return PDPLQR_OK;
    }
    return unsupported(h->cfg.solver == PDPLQR_SOLVER_PARALLEL ? "PARALLEL solver" : "KKT solver");
}

void solver_release(pdplqr_handle) {}

int solver_on_model(pdplqr_handle) { return PDPLQR_OK; }

int solver_update(pdplqr_handle h, const double *ws, const double *ys, const double *zs, const double *irho,
                  double sigma) {
    return launch_update_problem_data(h->sh, h->H, h->h, ws, ys, zs, irho, sigma, h->Hw, h->hw, h->gw, h->tab_s,
                                      h->tab_n, h->stream);
}

int solver_backward(pdplqr_handle h, const double *rho) {
    int rc = launch_penalty(h->sh, h->D, rho, h->gw, h->Hw, h->hw, h->d_off, h->y_off, h->tab_s, h->tab_n, 1,
                            h->max_nc, h->stream);
    if (rc) return rc;
    return launch_riccati_backward(riccati_args(h), h->stream);
}

int solver_backward_nofact(pdplqr_handle h, const double *rho) {
    int rc = launch_penalty(h->sh, h->D, rho, h->gw, h->Hw, h->hw, h->d_off, h->y_off, h->tab_s, h->tab_n, 0,
                            h->max_nc, h->stream);
    if (rc) return rc;
    return launch_riccati_backward_nofact(riccati_args(h), h->stream);
}

int solver_forward(pdplqr_handle h, const double *x0, double *ws) {
    return launch_riccati_forward(h->sh, h->E, h->c, h->KD, x0, ws, h->stream);
}

int solver_clear(pdplqr_handle) { return PDPLQR_OK; }

}  // namespace pdplqr

using namespace pdplqr;

extern "C" {

int pdplqr_get_segments(pdplqr_handle h, int32_t *, int32_t *) {
    if (!h) return PDPLQR_ERR_INVALID;
    return unsupported("get_segments");
}

int pdplqr_shard_element_size(pdplqr_handle h) {
    if (!h) return PDPLQR_ERR_INVALID;
    return 3 * h->sh.n * h->sh.n + 2 * h->sh.n;
}

int pdplqr_shard_backward(pdplqr_handle h, const double *, int, double *, int) {
    if (!h) return PDPLQR_ERR_INVALID;
    return unsupported("shard_backward");
}

int pdplqr_shard_forward(pdplqr_handle h, const double *, const double *, int32_t, int32_t, double *, int) {
    if (!h) return PDPLQR_ERR_INVALID;
    return unsupported("shard_forward");
}

}  // extern "C"
