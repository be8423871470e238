// solvers.hpp -- per-solver-kind implementation hooks behind the C ABI.
#pragma once
#include "internal.hpp"

namespace pdplqr {
int solver_init(pdplqr_handle h);      // allocate solver-specific state
void solver_release(pdplqr_handle h);  // free it (device buffers are in h->allocs)
int solver_on_model(pdplqr_handle h);  // after set_model (KKT: assemble + analyse)
int solver_update(pdplqr_handle h, const double *ws, const double *ys, const double *zs, const double *irho,
                  double sigma);
int solver_backward(pdplqr_handle h, const double *rho);
int solver_backward_nofact(pdplqr_handle h, const double *rho);
// Riccati solvers: backward on a workspace whose rho penalty is already folded
// in (H~ from the last factorizing backward, h~ formed by k_admm_update):
// backward_without_factorization when the factors are kept, else the
// factorizing kernels on the unchanged H~
int solver_backward_prepared(pdplqr_handle h);
void admm_release(pdplqr_handle h);  // admm.hip
struct AdmmArgs;
int solver_nofact_admm(pdplqr_handle h, const AdmmArgs &a, bool check);
int solver_forward(pdplqr_handle h, const double *x0, double *ws);
int solver_clear(pdplqr_handle h);
int solver_status(pdplqr_handle h, int32_t *flags);  // per-problem status (host)

// KKT solver (kkt.hip)
int kkt_init(pdplqr_handle h);
void kkt_release(pdplqr_handle h);
int kkt_on_model(pdplqr_handle h);
int kkt_update(pdplqr_handle h, const double *ws, const double *ys, const double *zs, const double *irho,
               double sigma);
int kkt_backward(pdplqr_handle h, const double *inv_rho);
// ADMM: the backward also writes the factor cache (false: no cached path for this shape);
// kkt_backward_cached / kkt_backward_linear run the factor and the rhs-only pass
bool kkt_linear_supported(pdplqr_handle h);
int kkt_backward_cached(pdplqr_handle h, const double *inv_rho);
int kkt_backward_linear(pdplqr_handle h, const double *inv_rho);
int kkt_rhs_restart(pdplqr_handle h);  // x0 sum of the rhs restarts (ADMM: h~, g formed by the update pass)
int kkt_forward(pdplqr_handle h, const double *x0, double *ws);
int kkt_dim(pdplqr_handle h);
int kkt_before_model(pdplqr_handle h);  // set_model on a formed KKT handle: keep the frozen matrix
bool kkt_ric_active(pdplqr_handle h);  // the Riccati-ordered path serves this handle
bool kkt_plain_rec_ehat(pdplqr_handle h);  // a plain KKT backward leaves the E^ record (kept in rec_gain)
// Riccati-ordered KKT path (kkt_riccati.hip): nc of the uniform 12/4 row
// layout, KKT_RIC_WIDE for the LDS kernels (any ncs, n + m <= 64),
// KKT_RIC_XL for the global-workspace kernels (kernels_xl.hip: 64 < n + m <= 256,
// per-stage rows <= 256), or -1
constexpr int KKT_RIC_WIDE = 1000;
constexpr int KKT_RIC_XL = 1001;
int launch_kkt_xl_backward(const Shape &sh, const double *E, const double *c, const double *D, const double *Hw,
                           const double *hw, const double *gw, const double *irho, const int32_t *d_off,
                           const int32_t *y_off, double rho_dyn, double *rec, int32_t *status, double *xws,
                           hipStream_t st);
int launch_kkt_xl_forward(const Shape &sh, const double *E, const double *c, const double *rec, const double *x0,
                          double *x0acc, double *ws, double rho_dyn, hipStream_t st);
int kkt_ric_nc(const Shape &sh, const std::vector<int32_t> &ncs, bool ldl_fits);
size_t kkt_ric_rec_doubles(const Shape &sh, int ric);  // rollout record doubles per problem
int launch_kkt_ric_backward(const Shape &sh, int nc, const double *E, const double *c, const double *D,
                            const double *Hw, const double *hw, const double *gw, const double *irho,
                            const int32_t *d_off, const int32_t *y_off, int nc_last, double rho_dyn, double *rec,
                            int32_t *status, hipStream_t st, double *cache = nullptr);
// (KKT_RIC_XL: `cache` is the per-problem workspace, kkt_xl_ws_doubles)
// linear-only pass on the factor cache the backward wrote (ric 0 / 4 only)
size_t kkt_ric_cache_doubles(const Shape &sh, int ric);  // per problem; 0 where unsupported
bool kkt_ric_rec_ehat(int ric);  // a plain backward of this path leaves the E^ record
int launch_kkt_ric_nofact(const Shape &sh, int nc, const double *D, const double *hw, const double *gw,
                          const double *irho, const int32_t *d_off, const int32_t *y_off, int nc_last, double rho_dyn,
                          const double *cache, double *rec, hipStream_t st);
int launch_kkt_ric_forward(const Shape &sh, const double *E, const double *c, const double *rec, const double *x0,
                           double *x0acc, double *ws, double rho_dyn, hipStream_t st, int ric, bool ehat);
// num_devices > 1 (multidev.hip): the horizon split over the devices of one process
int md_create(pdplqr_handle h, const pdplqr_config &C);
void md_release(pdplqr_handle h);
int md_set_model(pdplqr_handle h, int mask, const double *E, const double *c, const double *H, const double *hv,
                 const double *D, int mem);
int md_update(pdplqr_handle h, const double *ws, const double *ys, const double *zs, const double *irho, double sigma,
              int mem);
int md_backward(pdplqr_handle h, const double *rho, int mem, bool fact = true);
int md_forward(pdplqr_handle h, const double *x0, double *ws, int mem);
int md_status(pdplqr_handle h, int32_t *flags);
int md_synchronize(pdplqr_handle h);
int md_clear(pdplqr_handle h);
void *md_stream(pdplqr_handle h);
int md_set_stream(pdplqr_handle h, void *stream);
int md_primary_device(pdplqr_handle h);  // the device admm_solve's vectors live on
void md_admm_view(pdplqr_handle h, const double **D, const int32_t **d_off, const int32_t **y_off);
}  // namespace pdplqr
