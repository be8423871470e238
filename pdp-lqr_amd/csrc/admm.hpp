// admm.hpp -- the ADMM outer loop's device arguments and termination /
// adaptive-rho decision, shared by the stand-alone update kernel (admm.hip)
// and the update fused into the streamed backward (kernels_nofact.hip).
#pragma once
#include "internal.hpp"

namespace pdplqr {

struct AdmmArgs {
    Shape sh;
    const double *D, *hv, *wt, *lb, *ub, *rho, *irho;
    double *w, *y, *z, *hw, *gw;
    const int32_t *d_off, *y_off;
    int32_t *done, *iters, *conv, *active;
    double *prim, *dual, *rscale;
    double alpha, sigma, eps_abs, eps_rel, rho_tol;
    int max_nc, it, adaptive;
    int no_penalty = 0;  // fused next-update h~ without the penalty term (KKT: rho enters through g)
    int uni = 0;         // > 0: every stage k < N has exactly uni rows, the terminal none (offsets by arithmetic)
};

// Termination test of iteration a.it for problem b from the five maxima
// (r_prim, |Dw|, |z|, r_dual, |D^T y|), then OSQP's rho estimate when the
// test fails (admm.hip header).  One thread per problem.
// act > 0: some row's z sits at one of its bounds (an active constraint).
__device__ __forceinline__ void admm_decide(const AdmmArgs &a, int b, double rp, double dwm, double zm, double rd,
                                            double dty, double act) {
    a.iters[b] = a.it;
    a.prim[b] = rp;
    a.dual[b] = rd;
    double f = 1.0;
    if (rp <= a.eps_abs + a.eps_rel * fmax(dwm, zm) && rd <= a.eps_abs + a.eps_rel * dty) {
        a.done[b] = 1;
        a.conv[b] = 1;
    } else {
        atomicAdd(a.active, 1);
        // no rescale while no row is active (y is rounding noise there and the
        // dual normalisation undefined -- the estimate would collapse to ~1e-14
        // and pin rho at its lower clamp) or |D^T y| vanishes (OSQP's 1e-30 guard)
        if (a.adaptive && act > 0.0 && dty > 1e-30) {
            // OSQP's compute_rho_estimate: the ratio of the normalised
            // residuals, with its division guard 1e-30
            const double pn = rp / (fmax(dwm, zm) + 1e-30), dn = rd / (dty + 1e-30);
            const double e = sqrt(pn / (dn + 1e-30));
            if (e > a.rho_tol || e < 1.0 / a.rho_tol) {
                f = e;
                atomicOr(a.active + 1, 1);
            }
        }
    }
    a.rscale[b] = f;
}

// Fused ADMM update + backward_without_factorization (kernels_nofact.hip):
// PDPLQR_ERR_UNSUPPORTED when the shape / constraint layout is not covered.
int launch_nofact_admm(const RiccatiArgs &r, const AdmmArgs &a, bool check, hipStream_t st);

// KKT (Riccati-ordered, C5 row layout): the rollout with the ADMM update of the
// iteration in the same pass (kkt_riccati.hip); ERR_UNSUPPORTED otherwise
int launch_kkt_ric_forward_admm(const Shape &sh, const double *E, const double *c, const double *rec,
                                const double *x0, double *x0acc, double rho_dyn, const AdmmArgs &q, bool fuse,
                                bool check, hipStream_t st);
int kkt_forward_admm(pdplqr_handle h, const double *x0, const AdmmArgs &q, bool fuse, bool check);

}  // namespace pdplqr
