/*
 * pdplqr.h -- C ABI of the MI355X-native PDP-LQR solver (libpdplqr.so).
 *
 * This is the drop-in boundary for the reference's solver protocol
 *     update_problem_data -> backward -> forward
 * of Luyao787/PDP-LQR (header-only C++/Eigen/OpenMP).  Every entry point below
 * names the reference interface it replaces (file:line, relative to the
 * reference root).  The C++ facade headers under include/clqr/ (same class
 * names as the reference) and the Python host mirror (pdp-lqr_amd/pdplqr) are
 * the only callers.  No torch or HIP types cross this boundary: plain
 * pointers, sizes and int status codes (0 = ok, < 0 = error; no exceptions).
 *
 * Data layout at the boundary ("reference layout"): every per-stage block is
 * Eigen column-major, blocks are stage-major, problems are batch-major.  With
 * n = nx, m = nu, s = n + m, nc_k = constraint rows of stage k:
 *   E   [batch][N][n*s]            E_k = [B A]          (lqr_model.hpp:14)
 *   c   [batch][N][n]                                   (lqr_model.hpp:15)
 *   H   [batch][N*s*s + n*n]       H_k = [R S; S^T Q], then Q_N (lqr_model.hpp:18,33)
 *   h   [batch][N*s + n]           h_k = [r; q], then q_N
 *   D   [batch][sum_k nc_k*dim_k]  D_k = [Du Dx] (dim_k = s, or n at k = N)
 *   ws  [batch][N*s + n]           w_k = [u_k; x_k], then x_N
 *   ys, zs, rho, inv_rho [batch][sum_k nc_k]
 *   x0  [batch][n]
 * Pointers are host or device memory as the `mem` argument says; host buffers
 * are borrowed for the call only (copied to device before the call returns
 * or, for outputs, after the stream has drained).  One HIP stream per handle;
 * a handle is not thread-safe.
 */
#ifndef PDPLQR_H
#define PDPLQR_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PDPLQR_VERSION_MAJOR 0
#define PDPLQR_VERSION_MINOR 1

/* status codes */
#define PDPLQR_OK 0
#define PDPLQR_ERR_INVALID (-1)     /* bad argument / configuration            */
#define PDPLQR_ERR_HIP (-2)         /* HIP runtime error (message in last_error) */
#define PDPLQR_ERR_ALLOC (-3)       /* device allocation failed                 */
#define PDPLQR_ERR_STATE (-4)       /* protocol order violated                  */
#define PDPLQR_ERR_UNSUPPORTED (-5) /* shape/solver not supported by this build */
#define PDPLQR_ERR_NUMERIC (-6)     /* factorization failure (QDLDL path)       */

/* memory location of pointer arguments */
#define PDPLQR_MEM_HOST 0
#define PDPLQR_MEM_DEVICE 1

/* solver kinds: the three reference solvers */
#define PDPLQR_SOLVER_SERIAL 0   /* LQRSolver          (lqr_solver.hpp:9-77)            */
#define PDPLQR_SOLVER_PARALLEL 1 /* LQRParallelSolver  (lqr_solver_parallel.hpp:19-238) */
#define PDPLQR_SOLVER_KKT 2      /* QDLDLSolver        (qdldl_solver.hpp:14-151)        */

/* CondensedSystemSolverType (lqr_solver_parallel.hpp:14-17) */
#define PDPLQR_CONDENSED_LU 0
#define PDPLQR_CONDENSED_CHOLESKY 1

typedef struct pdplqr_handle_s *pdplqr_handle;

/* Construction arguments.  Replaces the solver constructors
 *   LQRSolver(const LQRModel&)                                  lqr_solver.hpp:11,31-39
 *   LQRParallelSolver(model, num_segments, load_balancing, type) lqr_solver_parallel.hpp:22-25,64-113
 *   QDLDLSolver(const LQRModel&)                                qdldl_solver.hpp:17,36-45
 * plus the LQRModel dimensions (lqr_model.hpp:74-80).  `batch` independent
 * problems of identical shape are solved together (new: the reference has no
 * batch API).  `ncs` (N+1 entries, shared by the batch) may be NULL (all 0). */
typedef struct {
    int32_t nx, nu, N;
    int32_t batch;
    int32_t solver;          /* PDPLQR_SOLVER_*                                   */
    int32_t num_segments;    /* PARALLEL: reference segment count (>= 1)          */
    int32_t load_balancing;  /* PARALLEL: alpha = 1.55 segmentation (:70)         */
    int32_t condensed_type;  /* PARALLEL: PDPLQR_CONDENSED_*                      */
    int32_t device;          /* HIP device ordinal                                 */
    int32_t keep_factors;    /* keep L_k, lp_k per stage (needed by
                                backward_without_factorization and the value
                                function getter); 0 = keep only the rollout
                                gains K_k, d_k                                     */
    const int32_t *ncs;      /* N+1 constraint counts or NULL                      */
    double rho_dyn;          /* KKT: lambda regularization, reference 1e-6 (:38)   */
    double kkt_sigma;        /* KKT: sigma frozen into the matrix, reference 1e-6 (:39) */
    int32_t segment_len;     /* PARALLEL: device sub-segment length (0 = auto).  Every
                                reference segment is refined into pieces of at most this
                                many stages; results are identical up to rounding. */
    int32_t num_devices;     /* PARALLEL: > 1 splits the horizon into num_devices
                                contiguous slices, one per GPU, driven by this one
                                handle (replaces the OpenMP team of
                                LQRParallelSolver, lqr_solver_parallel.hpp:22-25,102-113):
                                slice backward on every device, one RCCL all-gather of
                                the slice elements (3 nx^2 + 2 nx doubles per problem),
                                slice forward.  0 or 1: one device (`device`).
                                backward_without_factorization all-gathers only the
                                slices' (f, p) (2 nx doubles per problem,
                                lqr_solver_parallel.hpp:207-210); admm_solve runs its
                                vectors on the first device around the slices' protocol
                                calls.  With num_devices > 1 the shard_* calls are
                                unsupported, `device` is ignored, and set_stream takes
                                the caller's stream on devices[0] (see below).  num_devices = 1 with a non-NULL
                                `devices` runs the same split with one slice (RCCL
                                communicator of one rank). */
    const int32_t *devices;  /* num_devices HIP ordinals, or NULL = 0 .. num_devices - 1.
                                A device may repeat (same-device rehearsal: the exchange
                                then uses device copies, as with PDPLQR_MD_P2P=1). */
} pdplqr_config;

/* Fill `cfg` with the reference defaults (keep_factors = 1, load_balancing = 1,
 * CHOLESKY, rho_dyn = kkt_sigma = 1e-6).
 * Shape limits of this build (the reference is size-generic, lqr_kernel.hpp:104-147):
 * nx + nu <= 256 for every solver: up to 32 on MFMA tiles in one wavefront,
 * 33..64 on register tiles or LDS-resident stage matrices, one 256-thread
 * block per problem / segment / element (kernels_big.hip, kernels_wide.hip);
 * KKT rows per stage <= 64 past the block LDL^T tiles; 65..256 on
 * global-memory stage and element matrices (kernels_xl.hip, kernels_xl_par.hip:
 * every protocol call, pdplqr_admm_solve and the horizon-shard calls; KKT rows
 * per stage <= 256 there).  pdplqr_create returns
 * PDPLQR_ERR_UNSUPPORTED past them. */
void pdplqr_config_init(pdplqr_config *cfg);

int pdplqr_create(const pdplqr_config *cfg, pdplqr_handle *out);
int pdplqr_destroy(pdplqr_handle h);

/* Thread-local message of the last failing call ("" if none). */
const char *pdplqr_last_error(void);

/* Stream control (hipStream_t passed as void*). NULL = the handle's own stream.
   Switching makes the new stream wait (an event, no host sync) for what the
   handle queued on the old one, e.g. set_model's upload: the event is recorded
   on the OLD stream, so that stream must still be alive when the handle
   switches away from it (switch before destroying a stream the handle uses).
   num_devices > 1: the stream is the caller's, on devices[0] (else
   PDPLQR_ERR_INVALID); the slices keep their own streams, wait (an event) for
   the caller's stream before reading device inputs, and the caller's stream
   waits for the slices' work at the end of every call, forward's device
   outputs included -- no host synchronisation.  NULL (the default): device
   inputs are read after a drain of every slice device, and forward returns
   with ws complete. */
int pdplqr_set_stream(pdplqr_handle h, void *hip_stream);
void *pdplqr_get_stream(pdplqr_handle h);
int pdplqr_synchronize(pdplqr_handle h);

/* Problem data, reference layout.  Replaces filling LQRModel::nodes[k].{E,c,H,h,D_con}
 * (lqr_model.hpp:8-64,85-88) and the solver's `const LQRModel& model_` read
 * (lqr_solver.hpp:25).  D may be NULL when all nc_k = 0.  For the KKT solver the
 * matrix is frozen here, as QDLDLSolver freezes it at construction (qdldl_solver.hpp:40-42). */
int pdplqr_set_model(pdplqr_handle h, const double *E, const double *c, const double *H, const double *hv,
                     const double *D, int mem);

/* The same upload restricted to the arrays in `mask` (PDPLQR_MODEL_*; the other
 * pointers are ignored and may be NULL).  The reference reads its model lazily
 * -- H, h when update_problem_data copies them (lqr_solver.hpp:41-56), E, c,
 * D_con when backward / forward run (lqr_kernel.hpp:118-119,186-188) -- so the
 * C++ facade re-uploads exactly the arrays a call reads, and only those that
 * changed.  An upload of E, c or D alone keeps the protocol state (a backward
 * may follow the update directly); H or h needs a new update_problem_data. */
#define PDPLQR_MODEL_E 1
#define PDPLQR_MODEL_C 2
#define PDPLQR_MODEL_H 4
#define PDPLQR_MODEL_HV 8
#define PDPLQR_MODEL_D 16
#define PDPLQR_MODEL_ALL 31
int pdplqr_set_model_arrays(pdplqr_handle h, int mask, const double *E, const double *c, const double *H,
                            const double *hv, const double *D, int mem);

/* Model bytes copied host -> device by set_model / set_model_arrays since the
 * handle was created (device-memory uploads are not counted). */
int pdplqr_get_model_upload_bytes(pdplqr_handle h, int64_t *bytes);

/* LQRSolver::update_problem_data(ws, ys, zs, inv_rho_vecs, sigma)      lqr_solver.hpp:41-56
 * LQRParallelSolver::update_problem_data                               lqr_solver_parallel.hpp:115-140
 * QDLDLSolver::update_problem_data -> KKTSystem::form_rhs              qdldl_solver.hpp:80-86, kkt.hpp:224-300
 * ys/zs/inv_rho may be NULL when all nc_k = 0. */
int pdplqr_update_problem_data(pdplqr_handle h, const double *ws, const double *ys, const double *zs,
                               const double *inv_rho, double sigma, int mem);

/* LQRSolver::backward(rho_vecs)                                         lqr_solver.hpp:58-63
 * LQRParallelSolver::backward(rho_vecs)                                 lqr_solver_parallel.hpp:142-146
 * QDLDLSolver::backward(inv_rho_vecs) -- NOTE the KKT solver takes the  qdldl_solver.hpp:88-109
 * INVERSE rho vectors, as the reference's does. */
int pdplqr_backward(pdplqr_handle h, const double *rho, int mem);

/* LQRSolver::backward_without_factorization                            lqr_solver.hpp:65-70
 * LQRParallelSolver::backward_without_factorization                    lqr_solver_parallel.hpp:148-154
 * Requires keep_factors = 1 and a preceding pdplqr_backward. */
int pdplqr_backward_without_factorization(pdplqr_handle h, const double *rho, int mem);

/* LQRSolver::forward(x0, ws)                                            lqr_solver.hpp:72-77
 * LQRParallelSolver::forward(x0, ws)                                    lqr_solver_parallel.hpp:213-238
 * QDLDLSolver::forward(x0, ws)                                          qdldl_solver.hpp:111-151
 * Writes every ws entry (ws[0].x = x0 included).  Host `ws` is written after
 * the stream drains; device `ws` is written asynchronously on the stream. */
int pdplqr_forward(pdplqr_handle h, const double *x0, double *ws, int mem);

/* LQRSolver::clear_workspace (lqr_solver.hpp:12-14) */
int pdplqr_clear_workspace(pdplqr_handle h);

/* Value function of problem b at stage k: P = Lxx Lxx^T (n x n, column-major)
 * and p = lp.tail(n), from the serial workspace (lqr_solver.hpp:24-26 keeps it
 * protected; the condensed systems form P the same way, condensed_system.hpp:69,188).
 * SERIAL solver with keep_factors = 1 only.  Host outputs. */
int pdplqr_get_value_function(pdplqr_handle h, int32_t b, int32_t k, double *P, double *p);

/* Per-problem factorization status after backward: 0 = ok, otherwise 1 + the
 * first stage whose Cholesky met a non-positive pivot (the reference ignores
 * Eigen's LLT info, lqr_kernel.hpp:89,126).  `flags` has `batch` entries, host. */
int pdplqr_get_status(pdplqr_handle h, int32_t *flags);

/* Segmentation actually used by a PARALLEL handle (lqr_solver_parallel.hpp:64-88):
 * idx_start/Nseg each hold num_segments entries, host. */
int pdplqr_get_segments(pdplqr_handle h, int32_t *idx_start, int32_t *Nseg);

/* ---------------------------------------------------------------------- */
/* Horizon sharding across GPUs (new; the reference is one process).       */
/* A PARALLEL handle built with pdplqr_config.N = the LOCAL slice length   */
/* solves its slice; ranks exchange one segment element each (RCCL over    */
/* xGMI, done by the caller) between the two phases:                        */
/*   pdplqr_shard_backward   -> element (F, C, f, P, p) in `elem_out`       */
/*   all-gather of elements across ranks                                    */
/*   pdplqr_shard_forward    <- every rank's element, this rank's index     */
/* Element layout (doubles): F[n*n] C[n*n] f[n] P[n*n] p[n] (3n^2+2n).      */
/* ---------------------------------------------------------------------- */
int pdplqr_shard_element_size(pdplqr_handle h);
int pdplqr_shard_backward(pdplqr_handle h, const double *rho, int is_last_shard, double *elem_out, int mem);
/* LQRParallelSolver::backward_without_factorization (lqr_solver_parallel.hpp:148-154,190-211)
 * on the slice: keep_factors = 1 and a preceding pdplqr_shard_backward with the same
 * is_last_shard.  Writes the whole element; only its f and p differ from the
 * factorising call's (F, C, P bit-identical), so ranks need to exchange only
 * f, p (2n doubles per problem) and keep the rest of the last all-gather. */
int pdplqr_shard_backward_without_factorization(pdplqr_handle h, const double *rho, int is_last_shard,
                                                double *elem_out, int mem);
int pdplqr_shard_forward(pdplqr_handle h, const double *x0, const double *elems_all, int32_t num_shards,
                         int32_t shard_id, double *ws, int mem);

/* The slicing of a num_devices = R split (pdplqr_config.num_devices), host
 * arithmetic only (no device call): per slice r, 8 int64 at out[8 r]:
 * N0, N1 (stages [N0, N1)), last (holds the real terminal), y0 / ny_stages (its
 * stages' constraint rows in the full y vector), nc_terminal (its terminal's
 * rows: nc_N for the last slice, 0 otherwise), d0 / nd_stages (its stages'
 * entries in the full D array).  ncs: N+1 entries or NULL. */
int pdplqr_multidev_plan(int32_t N, int32_t R, const int32_t *ncs, int32_t nx, int32_t nu, int64_t *out);

/* ---------------------------------------------------------------------- */
/* ADMM outer loop for conic LQ (new).  The         */
/* reference stores e_lb <= D_con w <= e_ub (lqr_model.hpp:21-24) and       */
/* solves the ADMM x-update (update_problem_data / backward / forward,      */
/* lqr_solver.hpp:41-77), but the outer loop is absent (README.md:8).       */
/* This runs it on the device for the whole batch: OSQP's iteration        */
/* (Stellato et al. 2020, Algorithm 1) with the dynamics solved exactly by  */
/* the handle's solver, projection onto [lb, ub], sigma fixed, rho fixed or */
/* adapted by OSQP's rule (settings.adaptive_rho), and                     */
/* the ADMM residuals of admm.hip's header.  Works with all three solver    */
/* kinds; iterations >= 2 reuse the first iteration's factorization         */
/* (backward_without_factorization with keep_factors = 1).                  */
/* ---------------------------------------------------------------------- */
typedef struct {
    double sigma;        /* proximal weight (lqr_example.cpp:170: 1e-6)            */
    double alpha;        /* over-relaxation, 0 < alpha < 2 (OSQP default 1.6)      */
    int32_t max_iter;    /* iteration cap                                          */
    int32_t check_every; /* termination test period (one 4-byte D2H read each)     */
    double eps_abs, eps_rel; /* tolerances (OSQP defaults 1e-3); 0 = run max_iter  */
    int32_t adaptive_rho;    /* 1: OSQP's rho update at each termination test (a  */
                             /* per-problem scale of rho, then one refactorization) */
    double adaptive_rho_tolerance; /* rescale when the estimate leaves [1/tol, tol] (5) */
} pdplqr_admm_settings;

void pdplqr_admm_settings_init(pdplqr_admm_settings *s);

/* x0 [batch][n]; lb, ub, rho [batch][ny] (e_lb, e_ub, rho_vecs of          */
/* lqr_example.cpp:12-50,169); ws [batch][N*s+n], ys, zs [batch][ny]: warm   */
/* start in, solution out (w^k, y^k, z^k of the last iteration).  After the */
/* call the handle is "updated and factored" (forward may follow).          */
int pdplqr_admm_solve(pdplqr_handle h, const pdplqr_admm_settings *s, const double *x0, const double *lb,
                      const double *ub, const double *rho, double *ws, double *ys, double *zs, int mem);

/* Per-problem outcome of the last admm_solve (host arrays of `batch`        */
/* entries, each may be NULL): iterations run, 1 if the termination test     */
/* passed, primal / dual residual at the last test; `rho` (batch * ny, may be */
/* NULL) the final rho vectors.  Returns the number of iterations of the     */
/* batch (>= 1) or an error code.                                             */
int pdplqr_admm_info(pdplqr_handle h, int32_t *iters, int32_t *converged, double *prim_res, double *dual_res,
                     double *rho);

/* Device info helpers (for hosts that do not link HIP). */
int pdplqr_device_count(int32_t *count);

#ifdef __cplusplus
}
#endif

#endif /* PDPLQR_H */
