/*
 * pdplqr_oracle.c -- CPU restatement of the reference PDP-LQR algorithms.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * product path in pdp-lqr_amd/csrc.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product path never calls it.
 *
 * PARITY STATUS: "parity unpinned" with respect to reference *outputs*.
 *   The reference (Luyao787/PDP-LQR @ 2025-11-21) is header-only C++ on top of
 *   Eigen3 and QDLDL, neither of which exists in this image, and it ships no
 *   tests, fixtures or golden vectors.  This
 *   restatement is therefore pinned against (a) an independent dense-KKT
 *   solve (the unique optimum, tests/golden/make_golden.py) and (b) the
 *   quadrotor example known-answer values.
 *
 * Plain C99, Eigen-free, column-major like Eigen's default.  Every routine
 * cites the reference file:line it restates (paths relative to the reference
 * root).  Sizes: n = nx, m = nu, s = n + m.  Stage variables are w = [u; x].
 *
 * Flat data conventions (shared with the Python wrapper oracle/oracle.py):
 *   E  : N blocks of n x s           (E_k = [B A], lqr_model.hpp:14)
 *   c  : N blocks of n
 *   H  : N blocks of s x s, then the terminal n x n   (lqr_model.hpp:18,33)
 *   h  : N blocks of s, then the terminal n
 *   D  : ragged, stage k block is nc_k x dim_k        (lqr_model.hpp:23)
 *   ws : ragged like h (k < N: s entries, k = N: n entries)
 *   ys, zs, rho, inv_rho : ragged, stage k has nc_k entries
 */
#define _GNU_SOURCE /* sched_setaffinity: the reference's thread pinning (lqr_solver_parallel.hpp:102-112) */
#include <math.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>

#define IX(i, j, ld) ((size_t)(j) * (size_t)(ld) + (size_t)(i))

/* ------------------------------------------------------------------------ */
/* Model                                                                    */
/* ------------------------------------------------------------------------ */
typedef struct {
    int n, m, N;
    int *nc;      /* N+1 */
    int *d_off;   /* N+2, offsets into D */
    int *y_off;   /* N+2, offsets into ys/zs/rho */
    double *E, *c, *H, *h, *D;
} orc_model;

static int stage_dim(const orc_model *md, int k) { return k < md->N ? md->n + md->m : md->n; }
static size_t H_off(const orc_model *md, int k) { int s = md->n + md->m; return (size_t)k * s * s; }
static size_t h_off(const orc_model *md, int k) { int s = md->n + md->m; return (size_t)k * s; }

static void *xcalloc(size_t n, size_t sz) { return calloc(n ? n : 1, sz); }

static orc_model *model_create(int n, int m, int N, const int *nc, const double *E, const double *c,
                               const double *H, const double *h, const double *D) {
    orc_model *md = (orc_model *)xcalloc(1, sizeof(orc_model));
    int s = n + m, k;
    md->n = n; md->m = m; md->N = N;
    md->nc = (int *)xcalloc(N + 1, sizeof(int));
    md->d_off = (int *)xcalloc(N + 2, sizeof(int));
    md->y_off = (int *)xcalloc(N + 2, sizeof(int));
    for (k = 0; k <= N; ++k) {
        md->nc[k] = nc ? nc[k] : 0;
        md->d_off[k + 1] = md->d_off[k] + md->nc[k] * (k < N ? s : n);
        md->y_off[k + 1] = md->y_off[k] + md->nc[k];
    }
    md->E = (double *)xcalloc((size_t)N * n * s, sizeof(double));
    md->c = (double *)xcalloc((size_t)N * n, sizeof(double));
    md->H = (double *)xcalloc((size_t)N * s * s + (size_t)n * n, sizeof(double));
    md->h = (double *)xcalloc((size_t)N * s + n, sizeof(double));
    md->D = (double *)xcalloc((size_t)md->d_off[N + 1], sizeof(double));
    memcpy(md->E, E, sizeof(double) * (size_t)N * n * s);
    memcpy(md->c, c, sizeof(double) * (size_t)N * n);
    memcpy(md->H, H, sizeof(double) * ((size_t)N * s * s + (size_t)n * n));
    memcpy(md->h, h, sizeof(double) * ((size_t)N * s + n));
    if (md->d_off[N + 1] > 0 && D) memcpy(md->D, D, sizeof(double) * (size_t)md->d_off[N + 1]);
    return md;
}

static void model_destroy(orc_model *md) {
    if (!md) return;
    free(md->nc); free(md->d_off); free(md->y_off);
    free(md->E); free(md->c); free(md->H); free(md->h); free(md->D);
    free(md);
}

/* ------------------------------------------------------------------------ */
/* Dense helpers (Eigen semantics)                                          */
/* ------------------------------------------------------------------------ */

/* Largest stage size of the restatement. */
#define ORC_SMAX 256

/* Eigen llt_inplace<Lower>::unblocked (Eigen/src/Cholesky/LLT.h) on the
 * diagonal block [off, off + sz) of the column-major L (ld): left-looking --
 * column k takes the products of the block's earlier columns only; on a pivot
 * <= 0 it returns k (relative to off) with column k and the later columns of
 * the block untouched.  Returns -1 on success. */
static int llt_unblocked(double *L, int ld, int off, int sz) {
    int i, k, p;
    for (k = 0; k < sz; ++k) {
        double x = L[IX(off + k, off + k, ld)];
        for (p = 0; p < k; ++p) x -= L[IX(off + k, off + p, ld)] * L[IX(off + k, off + p, ld)];
        if (x <= 0.0) return k;
        x = sqrt(x);
        L[IX(off + k, off + k, ld)] = x;
        for (i = k + 1; i < sz; ++i) {
            double a = L[IX(off + i, off + k, ld)];
            for (p = 0; p < k; ++p) a -= L[IX(off + i, off + p, ld)] * L[IX(off + k, off + p, ld)];
            L[IX(off + i, off + k, ld)] = a / x;
        }
    }
    return -1;
}

/* Eigen's block size of llt_inplace<Lower>::blocked for a matrix of order
 * dim (0: dim < 32, the unblocked form runs). */
static int llt_block_size(int dim) {
    int bs;
    if (dim < 32) return 0;
    bs = dim / 8;
    bs = (bs / 16) * 16;
    if (bs < 8) bs = 8;
    if (bs > 128) bs = 128;
    return bs;
}

/* `L = M.llt().matrixL()` (lqr_kernel.hpp:89,126; condensed_system.hpp:188-247):
 * Eigen's LLT::compute runs llt_inplace<Lower>::blocked -- the unblocked form
 * below order 32, else blocks of llt_block_size(dim) columns: the diagonal
 * block A11 unblocked, then A21 <- A21 A11^{-T}, then A22 -= A21 A21^T.  A
 * pivot <= 0 inside A11 ends it: the columns of the finished blocks hold L, A11
 * its columns up to the pivot (rows inside A11), and every other entry of the
 * later columns (A21 of the block included) the Schur complement of the
 * finished blocks.  The reference ignores the failure and uses that lower
 * triangle.  Writes L (ld = dim) with a zero upper triangle;
 * returns -1 on success or the failing column. */
static int llt_lower(const double *M, double *L, int dim) {
    int i, j, k, p, fail = -1;
    const int bs = llt_block_size(dim);
    for (j = 0; j < dim; ++j)
        for (i = 0; i < dim; ++i) L[IX(i, j, dim)] = M[IX(i, j, dim)];
    if (!bs) {
        fail = llt_unblocked(L, dim, 0, dim);
    } else {
        for (k = 0; k < dim; k += bs) {
            const int b = bs < dim - k ? bs : dim - k, rs = dim - k - b;
            const int ret = llt_unblocked(L, dim, k, b);
            if (ret >= 0) {
                fail = k + ret;
                break;
            }
            /* A21 <- A21 A11^{-T}: row by row, forward substitution with A11 */
            for (i = k + b; i < dim; ++i)
                for (j = 0; j < b; ++j) {
                    double a = L[IX(i, k + j, dim)];
                    for (p = 0; p < j; ++p) a -= L[IX(i, k + p, dim)] * L[IX(k + j, k + p, dim)];
                    L[IX(i, k + j, dim)] = a / L[IX(k + j, k + j, dim)];
                }
            /* A22 -= A21 A21^T (lower triangle) */
            (void)rs;
            for (j = k + b; j < dim; ++j)
                for (i = j; i < dim; ++i) {
                    double a = L[IX(i, j, dim)];
                    for (p = 0; p < b; ++p) a -= L[IX(i, k + p, dim)] * L[IX(j, k + p, dim)];
                    L[IX(i, j, dim)] = a;
                }
        }
    }
    for (j = 0; j < dim; ++j)
        for (i = 0; i < j; ++i) L[IX(i, j, dim)] = 0.0;
    return fail;
}

/* Solve L y = b in place, L lower (leading dim ld), size r. */
static void trsv_lower(const double *L, int ld, int r, double *b) {
    int i, j;
    for (i = 0; i < r; ++i) {
        double a = b[i];
        for (j = 0; j < i; ++j) a -= L[IX(i, j, ld)] * b[j];
        b[i] = a / L[IX(i, i, ld)];
    }
}

/* Solve L^T y = b in place (upper back substitution). */
static void trsv_lower_t(const double *L, int ld, int r, double *b) {
    int i, j;
    for (i = r - 1; i >= 0; --i) {
        double a = b[i];
        for (j = i + 1; j < r; ++j) a -= L[IX(j, i, ld)] * b[j];
        b[i] = a / L[IX(i, i, ld)];
    }
}

/* ------------------------------------------------------------------------ */
/* Per-stage workspace: LQRKernelData + ParallelLQRKernelData                */
/* (lqr_kernel.hpp:8-75, lqr_kernel_parallel.hpp:9-47)                       */
/* ------------------------------------------------------------------------ */
typedef struct {
    int dim, nc, terminal;
    double *H, *h, *g, *L, *lp;
    double *G, *F, *C, *f, *K, *d; /* parallel extras */
} orc_stage;

static void stage_init(orc_stage *st, int n, int m, int nc, int terminal) {
    int s = n + m;
    st->terminal = terminal;
    st->dim = terminal ? n : s;
    st->nc = nc;
    st->H = (double *)xcalloc((size_t)st->dim * st->dim, sizeof(double));
    st->h = (double *)xcalloc(st->dim, sizeof(double));
    st->g = (double *)xcalloc(nc, sizeof(double));
    st->L = (double *)xcalloc((size_t)st->dim * st->dim, sizeof(double));
    st->lp = (double *)xcalloc(st->dim, sizeof(double));
    st->G = (double *)xcalloc((size_t)m * n, sizeof(double));
    st->F = (double *)xcalloc((size_t)n * n, sizeof(double));
    st->C = (double *)xcalloc((size_t)n * n, sizeof(double));
    st->f = (double *)xcalloc(n, sizeof(double));
    st->K = (double *)xcalloc((size_t)m * n, sizeof(double));
    st->d = (double *)xcalloc(m, sizeof(double));
}

static void stage_zero(orc_stage *st, int n, int m) {
    memset(st->H, 0, sizeof(double) * st->dim * st->dim);
    memset(st->h, 0, sizeof(double) * st->dim);
    if (st->nc) memset(st->g, 0, sizeof(double) * st->nc);
    memset(st->L, 0, sizeof(double) * st->dim * st->dim);
    memset(st->lp, 0, sizeof(double) * st->dim);
    memset(st->G, 0, sizeof(double) * m * n);
    memset(st->F, 0, sizeof(double) * n * n);
    memset(st->C, 0, sizeof(double) * n * n);
    memset(st->f, 0, sizeof(double) * n);
    memset(st->K, 0, sizeof(double) * m * n);
    memset(st->d, 0, sizeof(double) * m);
}

static void stage_free(orc_stage *st) {
    free(st->H); free(st->h); free(st->g); free(st->L); free(st->lp);
    free(st->G); free(st->F); free(st->C); free(st->f); free(st->K); free(st->d);
}

/* update_problem_data for one stage (lqr_solver.hpp:41-56) */
static void stage_update(const orc_model *md, int k, orc_stage *st, const double *ws, const double *ys,
                         const double *zs, const double *inv_rho, double sigma) {
    int dim = stage_dim(md, k), i, j;
    const double *Hm = md->H + H_off(md, k);
    const double *hm = md->h + h_off(md, k);
    const double *w = ws + h_off(md, k);
    for (j = 0; j < dim; ++j)
        for (i = 0; i < dim; ++i) st->H[IX(i, j, dim)] = Hm[IX(i, j, dim)];
    for (i = 0; i < dim; ++i) st->H[IX(i, i, dim)] += sigma;
    for (i = 0; i < dim; ++i) st->h[i] = hm[i] - sigma * w[i];
    if (md->nc[k] > 0) {
        int o = md->y_off[k];
        for (i = 0; i < md->nc[k]; ++i) st->g[i] = zs[o + i] - inv_rho[o + i] * ys[o + i];
    }
}

/* The rho-penalty preamble shared by the kernels (lqr_kernel.hpp:82-88,106-112):
 * H += D^T diag(rho) D ; h -= D^T (rho o g).  with_H = 0 skips the H part
 * (the *_without_factorization variants, lqr_kernel.hpp:96-99,152-155). */
static void stage_penalty(const orc_model *md, int k, orc_stage *st, const double *rho, int with_H) {
    int nc = md->nc[k], dim = stage_dim(md, k), i, j, r;
    const double *D = md->D + md->d_off[k];
    const double *rv = rho + md->y_off[k];
    if (nc <= 0) return;
    if (with_H)
        for (j = 0; j < dim; ++j)
            for (i = 0; i < dim; ++i) {
                double a = 0.0;
                for (r = 0; r < nc; ++r) a += D[IX(r, i, nc)] * (rv[r] * D[IX(r, j, nc)]);
                st->H[IX(i, j, dim)] += a;
            }
    for (i = 0; i < dim; ++i) {
        double a = 0.0;
        for (r = 0; r < nc; ++r) a += D[IX(r, i, nc)] * (rv[r] * st->g[r]);
        st->h[i] -= a;
    }
}

/* LQRKernel::terminal_step_with_factorization (lqr_kernel.hpp:80-91) */
static void k_terminal_fact(const orc_model *md, orc_stage *st, const double *rho) {
    stage_penalty(md, md->N, st, rho, 1);
    llt_lower(st->H, st->L, st->dim);
    memcpy(st->lp, st->h, sizeof(double) * st->dim);
}

/* LQRKernel::terminal_step_without_factorization (lqr_kernel.hpp:94-101) */
static void k_terminal_nofact(const orc_model *md, orc_stage *st, const double *rho) {
    stage_penalty(md, md->N, st, rho, 0);
    memcpy(st->lp, st->h, sizeof(double) * st->dim);
}

/* Shared tail of step_with/without_factorization (lqr_kernel.hpp:128-146 and
 * 159-177): Pb = Lxx_next (Lxx_next^T c) + p_next ; lp = h + E^T Pb ;
 * lu <- Luu^{-1} lu ; p -= Lxu lu. */
static void k_linear_tail(const orc_model *md, int k, const orc_stage *nx_, orc_stage *st) {
    int n = md->n, m = md->m, s = n + m, i, j;
    int nd = nx_->dim, xo = nd - n; /* bottomRightCorner(n, n) of next L */
    const double *E = md->E + (size_t)k * n * s;
    const double *c = md->c + (size_t)k * n;
    double Pb_tmp[ORC_SMAX], Pb[ORC_SMAX];
    for (j = 0; j < n; ++j) { /* Pb_tmp = Lxx^T c */
        double a = 0.0;
        for (i = 0; i < n; ++i) a += nx_->L[IX(xo + i, xo + j, nd)] * c[i];
        Pb_tmp[j] = a;
    }
    for (i = 0; i < n; ++i) { /* Pb = Lxx Pb_tmp + p_next */
        double a = 0.0;
        for (j = 0; j < n; ++j) a += nx_->L[IX(xo + i, xo + j, nd)] * Pb_tmp[j];
        Pb[i] = a + nx_->lp[xo + i];
    }
    for (j = 0; j < s; ++j) { /* lp = h + E^T Pb */
        double a = 0.0;
        for (i = 0; i < n; ++i) a += E[IX(i, j, n)] * Pb[i];
        st->lp[j] = st->h[j] + a;
    }
    trsv_lower(st->L, s, m, st->lp); /* lu <- Luu^{-1} lu */
    for (i = 0; i < n; ++i) {        /* p -= Lxu lu */
        double a = 0.0;
        for (j = 0; j < m; ++j) a += st->L[IX(m + i, j, s)] * st->lp[j];
        st->lp[m + i] -= a;
    }
}

/* LQRKernel::step_with_factorization (lqr_kernel.hpp:104-147) */
static void k_step_fact(const orc_model *md, int k, const double *rho, const orc_stage *nx_, orc_stage *st) {
    int n = md->n, m = md->m, s = n + m, i, j, t;
    int nd = nx_->dim, xo = nd - n;
    const double *E = md->E + (size_t)k * n * s;
    double *V = (double *)xcalloc((size_t)s * s, sizeof(double)), *M = (double *)xcalloc((size_t)s * s, sizeof(double));
    stage_penalty(md, k, st, rho, 1);
    for (j = 0; j < n; ++j) /* V = E^T Lxx_next  (s x n) */
        for (i = 0; i < s; ++i) {
            double a = 0.0;
            for (t = 0; t < n; ++t) a += E[IX(t, i, n)] * nx_->L[IX(xo + t, xo + j, nd)];
            V[IX(i, j, s)] = a;
        }
    for (j = 0; j < s; ++j) /* M = H + V V^T */
        for (i = 0; i < s; ++i) {
            double a = 0.0;
            for (t = 0; t < n; ++t) a += V[IX(i, t, s)] * V[IX(j, t, s)];
            M[IX(i, j, s)] = st->H[IX(i, j, s)] + a;
        }
    llt_lower(M, st->L, s);
    free(V);
    free(M);
    k_linear_tail(md, k, nx_, st);
    (void)m;
}

/* LQRKernel::step_without_factorization (lqr_kernel.hpp:150-178) */
static void k_step_nofact(const orc_model *md, int k, const double *rho, const orc_stage *nx_, orc_stage *st) {
    stage_penalty(md, k, st, rho, 0);
    k_linear_tail(md, k, nx_, st);
}

/* LQRKernel::forward_step (lqr_kernel.hpp:181-212):
 * u = -Luu^{-T}(lu + Lxu^T x) ; x_next = c + A x + B u. */
static void k_forward(const orc_model *md, int k, const orc_stage *st, double *w, double *w_next,
                      const double *uhat_G /* nullable: G*uhat term of the parallel kernel */,
                      int update_x_next) {
    int n = md->n, m = md->m, s = n + m, i, j;
    const double *E = md->E + (size_t)k * n * s;
    const double *c = md->c + (size_t)k * n;
    double *x = w + m, *u = w;
    int xdim_next = (k + 1 < md->N) ? s : n;
    double *x_next = w_next + (xdim_next - n);
    double xn[ORC_SMAX];
    for (i = 0; i < m; ++i) {
        double a = -st->lp[i];
        for (j = 0; j < n; ++j) a -= st->L[IX(m + j, i, s)] * x[j];
        if (uhat_G) a += uhat_G[i];
        u[i] = a;
    }
    trsv_lower_t(st->L, s, m, u);
    if (!update_x_next) return;
    for (i = 0; i < n; ++i) {
        double a = c[i];
        for (j = 0; j < n; ++j) a += E[IX(i, m + j, n)] * x[j];
        for (j = 0; j < m; ++j) a += E[IX(i, j, n)] * u[j];
        xn[i] = a;
    }
    memcpy(x_next, xn, sizeof(double) * n);
}

/* ------------------------------------------------------------------------ */
/* LQRSolver (lqr_solver.hpp:9-77)                                          */
/* ------------------------------------------------------------------------ */
typedef struct {
    orc_model *md;
    orc_stage *ws; /* N+1 */
} orc_serial;

void *orc_serial_create(int n, int m, int N, const int *nc, const double *E, const double *c, const double *H,
                        const double *h, const double *D) {
    orc_serial *o;
    int k;
    if (N < 1 || n < 1 || m < 1 || n + m > ORC_SMAX) return NULL; /* lqr_model.hpp:75-77; s <= 256 here */
    o = (orc_serial *)xcalloc(1, sizeof(orc_serial));
    o->md = model_create(n, m, N, nc, E, c, H, h, D);
    o->ws = (orc_stage *)xcalloc(N + 1, sizeof(orc_stage));
    for (k = 0; k <= N; ++k) stage_init(&o->ws[k], n, m, o->md->nc[k], k == N); /* :31-39 */
    return o;
}

void orc_serial_destroy(void *p) {
    orc_serial *o = (orc_serial *)p;
    int k;
    if (!o) return;
    for (k = 0; k <= o->md->N; ++k) stage_free(&o->ws[k]);
    free(o->ws);
    model_destroy(o->md);
    free(o);
}

void orc_serial_clear_workspace(void *p) { /* :12-14 */
    orc_serial *o = (orc_serial *)p;
    int k;
    for (k = 0; k <= o->md->N; ++k) stage_zero(&o->ws[k], o->md->n, o->md->m);
}

void orc_serial_update_problem_data(void *p, const double *ws, const double *ys, const double *zs,
                                    const double *inv_rho, double sigma) { /* :41-56 */
    orc_serial *o = (orc_serial *)p;
    int k;
    for (k = 0; k <= o->md->N; ++k) stage_update(o->md, k, &o->ws[k], ws, ys, zs, inv_rho, sigma);
}

void orc_serial_backward(void *p, const double *rho) { /* :58-63 */
    orc_serial *o = (orc_serial *)p;
    int k, N = o->md->N;
    k_terminal_fact(o->md, &o->ws[N], rho);
    for (k = N - 1; k >= 0; --k) k_step_fact(o->md, k, rho, &o->ws[k + 1], &o->ws[k]);
}

void orc_serial_backward_without_factorization(void *p, const double *rho) { /* :65-70 */
    orc_serial *o = (orc_serial *)p;
    int k, N = o->md->N;
    k_terminal_nofact(o->md, &o->ws[N], rho);
    for (k = N - 1; k >= 0; --k) k_step_nofact(o->md, k, rho, &o->ws[k + 1], &o->ws[k]);
}

void orc_serial_forward(void *p, const double *x0, double *ws) { /* :72-77 */
    orc_serial *o = (orc_serial *)p;
    int k, N = o->md->N, n = o->md->n, m = o->md->m, s = n + m;
    memcpy(ws + m, x0, sizeof(double) * n); /* ws[0].tail(n) = x0 */
    for (k = 0; k < N; ++k) k_forward(o->md, k, &o->ws[k], ws + (size_t)k * s, ws + (size_t)(k + 1) * s, NULL, 1);
}

/* Workspace accessors (the reference's workspace_ is protected, :24-26):
 * L_k (dim x dim) and lp_k (dim). */
void orc_serial_get_stage(void *p, int k, double *L, double *lp) {
    orc_serial *o = (orc_serial *)p;
    orc_stage *st = &o->ws[k];
    if (L) memcpy(L, st->L, sizeof(double) * st->dim * st->dim);
    if (lp) memcpy(lp, st->lp, sizeof(double) * st->dim);
}

/* ------------------------------------------------------------------------ */
/* ParallelLQRKernel (lqr_kernel_parallel.hpp:49-219)                       */
/* ------------------------------------------------------------------------ */

/* terminal_step_* (lqr_kernel_parallel.hpp:52-85): the last segment uses the
 * real terminal; any other segment a dummy zero value function, F = I. */
static void pk_terminal(const orc_model *md, orc_stage *st, const double *rho, int last, int fact) {
    int n = md->n, i;
    if (last) {
        if (fact) k_terminal_fact(md, st, rho);
        else k_terminal_nofact(md, st, rho);
        return;
    }
    memset(st->L, 0, sizeof(double) * st->dim * st->dim);
    memset(st->lp, 0, sizeof(double) * st->dim);
    memset(st->C, 0, sizeof(double) * n * n);
    memset(st->f, 0, sizeof(double) * n);
    memset(st->F, 0, sizeof(double) * n * n);
    for (i = 0; i < n; ++i) st->F[IX(i, i, n)] = 1.0;
}

/* step_with_factorization (lqr_kernel_parallel.hpp:88-136) and
 * step_without_factorization (:139-168). */
static void pk_step(const orc_model *md, int k, const double *rho, const orc_stage *nx_, orc_stage *st, int last,
                    int fact) {
    int n = md->n, m = md->m, s = n + m, i, j, t;
    const double *E = md->E + (size_t)k * n * s;
    const double *c = md->c + (size_t)k * n;
    double *tmp, ftmp[ORC_SMAX];
    if (fact) k_step_fact(md, k, rho, nx_, st);
    else k_step_nofact(md, k, rho, nx_, st);
    if (last) return;
    /* d = -Luu^{-T} lu (:106,108 / :154-155) */
    for (i = 0; i < m; ++i) st->d[i] = -st->lp[i];
    trsv_lower_t(st->L, s, m, st->d);
    /* f = F_next (c + B d) + f_next (:132-133 / :165-166) */
    for (i = 0; i < n; ++i) {
        double a = c[i];
        for (j = 0; j < m; ++j) a += E[IX(i, j, n)] * st->d[j];
        ftmp[i] = a;
    }
    for (i = 0; i < n; ++i) {
        double a = 0.0;
        for (j = 0; j < n; ++j) a += nx_->F[IX(i, j, n)] * ftmp[j];
        st->f[i] = a + nx_->f[i];
    }
    if (!fact) return;
    tmp = (double *)xcalloc((size_t)n * n, sizeof(double));
    /* K = -Luu^{-T} Lxu^T (:105,107) ; K is m x n */
    for (j = 0; j < n; ++j) {
        double col[ORC_SMAX];
        for (i = 0; i < m; ++i) col[i] = -st->L[IX(m + j, i, s)];
        trsv_lower_t(st->L, s, m, col);
        for (i = 0; i < m; ++i) st->K[IX(i, j, m)] = col[i];
    }
    /* G = -Luu^{-1} B^T F_next^T (:126-128) ; G is m x n */
    for (j = 0; j < n; ++j) {
        double col[ORC_SMAX];
        for (i = 0; i < m; ++i) {
            double a = 0.0;
            for (t = 0; t < n; ++t) a += E[IX(t, i, n)] * nx_->F[IX(j, t, n)];
            col[i] = -a;
        }
        trsv_lower(st->L, s, m, col);
        for (i = 0; i < m; ++i) st->G[IX(i, j, m)] = col[i];
    }
    /* F = F_next (A + B K) (:129-130) */
    for (j = 0; j < n; ++j)
        for (i = 0; i < n; ++i) {
            double a = E[IX(i, m + j, n)];
            for (t = 0; t < m; ++t) a += E[IX(i, t, n)] * st->K[IX(t, j, m)];
            tmp[IX(i, j, n)] = a;
        }
    for (j = 0; j < n; ++j)
        for (i = 0; i < n; ++i) {
            double a = 0.0;
            for (t = 0; t < n; ++t) a += nx_->F[IX(i, t, n)] * tmp[IX(t, j, n)];
            st->F[IX(i, j, n)] = a;
        }
    /* C = C_next + G^T G (:134) */
    for (j = 0; j < n; ++j)
        for (i = 0; i < n; ++i) {
            double a = 0.0;
            for (t = 0; t < m; ++t) a += st->G[IX(t, i, m)] * st->G[IX(t, j, m)];
            st->C[IX(i, j, n)] = nx_->C[IX(i, j, n)] + a;
        }
    free(tmp);
}

/* ------------------------------------------------------------------------ */
/* Condensed segment systems (condensed_system.hpp)                          */
/* ------------------------------------------------------------------------ */

/* LU with partial pivoting of an r x r matrix (Eigen::PartialPivLU semantics:
 * P A = L U, row pivoting on max |a|). */
static void lu_factor(double *A, int *piv, int r) {
    int i, j, k;
    for (k = 0; k < r; ++k) {
        int p = k;
        double best = fabs(A[IX(k, k, r)]);
        for (i = k + 1; i < r; ++i)
            if (fabs(A[IX(i, k, r)]) > best) { best = fabs(A[IX(i, k, r)]); p = i; }
        piv[k] = p;
        if (p != k)
            for (j = 0; j < r; ++j) { double t = A[IX(k, j, r)]; A[IX(k, j, r)] = A[IX(p, j, r)]; A[IX(p, j, r)] = t; }
        if (A[IX(k, k, r)] != 0.0)
            for (i = k + 1; i < r; ++i) A[IX(i, k, r)] /= A[IX(k, k, r)];
        for (j = k + 1; j < r; ++j)
            for (i = k + 1; i < r; ++i) A[IX(i, j, r)] -= A[IX(i, k, r)] * A[IX(k, j, r)];
    }
}

static void lu_solve(const double *LU, const int *piv, int r, double *b) {
    int i, j;
    for (i = 0; i < r; ++i)
        if (piv[i] != i) { double t = b[i]; b[i] = b[piv[i]]; b[piv[i]] = t; }
    for (i = 0; i < r; ++i)
        for (j = 0; j < i; ++j) b[i] -= LU[IX(i, j, r)] * b[j];
    for (i = r - 1; i >= 0; --i) {
        for (j = i + 1; j < r; ++j) b[i] -= LU[IX(i, j, r)] * b[j];
        b[i] /= LU[IX(i, i, r)];
    }
}

/* LLT solve in place: (L L^T) x = b. */
static void llt_solve(const double *L, int r, double *b) {
    trsv_lower(L, r, r, b);
    trsv_lower_t(L, r, r, b);
}

typedef struct {
    double *A, *C, *P, *At, *Pinv, *c, *p, *xhat, *uhat;
    double *PC, *PA, *D, *LU, *Lp, *Lc; /* factor storage */
    int *piv;
} orc_cseg;

typedef struct {
    int n, ns, type; /* type 0 = LU, 1 = CHOLESKY */
    orc_cseg *seg;
} orc_condensed;

static orc_condensed *cond_create(int n, int ns, int type) {
    orc_condensed *cs = (orc_condensed *)xcalloc(1, sizeof(orc_condensed));
    int i, j;
    cs->n = n; cs->ns = ns; cs->type = type;
    cs->seg = (orc_cseg *)xcalloc(ns, sizeof(orc_cseg));
    for (i = 0; i < ns; ++i) {
        orc_cseg *g = &cs->seg[i];
        g->A = (double *)xcalloc(n * n, sizeof(double));
        g->C = (double *)xcalloc(n * n, sizeof(double));
        g->P = (double *)xcalloc(n * n, sizeof(double));
        g->At = (double *)xcalloc(n * n, sizeof(double));
        g->Pinv = (double *)xcalloc(n * n, sizeof(double));
        g->PC = (double *)xcalloc(n * n, sizeof(double));
        g->PA = (double *)xcalloc(n * n, sizeof(double));
        g->D = (double *)xcalloc(n * n, sizeof(double));
        g->LU = (double *)xcalloc(n * n, sizeof(double));
        g->Lp = (double *)xcalloc(n * n, sizeof(double));
        g->Lc = (double *)xcalloc(n * n, sizeof(double));
        g->c = (double *)xcalloc(n, sizeof(double));
        g->p = (double *)xcalloc(n, sizeof(double));
        g->xhat = (double *)xcalloc(n, sizeof(double));
        g->uhat = (double *)xcalloc(n, sizeof(double));
        g->piv = (int *)xcalloc(n, sizeof(int));
        /* Cholesky ctor pre-computes LLT of the identity (:157-161) */
        for (j = 0; j < n; ++j) { g->Pinv[IX(j, j, n)] = 1.0; g->Lp[IX(j, j, n)] = 1.0; g->Lc[IX(j, j, n)] = 1.0; }
    }
    return cs;
}

static void cond_destroy(orc_condensed *cs) {
    int i;
    if (!cs) return;
    for (i = 0; i < cs->ns; ++i) {
        orc_cseg *g = &cs->seg[i];
        free(g->A); free(g->C); free(g->P); free(g->At); free(g->Pinv); free(g->PC); free(g->PA);
        free(g->D); free(g->LU); free(g->Lp); free(g->Lc); free(g->c); free(g->p); free(g->xhat);
        free(g->uhat); free(g->piv);
    }
    free(cs->seg);
    free(cs);
}

/* update_segment_data(Lxx, A, C, p, c, id)  (LU :64-74, CHOLESKY :183-195) */
static void cond_update_full(orc_condensed *cs, const double *Lxx, int ldL, int off, const double *F,
                             const double *C, const double *p, const double *f, int id) {
    int n = cs->n, i, j, t;
    orc_cseg *g = &cs->seg[id];
    for (j = 0; j < n; ++j)
        for (i = 0; i < n; ++i) {
            double a = 0.0;
            for (t = 0; t < n; ++t) a += Lxx[IX(off + i, off + t, ldL)] * Lxx[IX(off + j, off + t, ldL)];
            g->P[IX(i, j, n)] = a;
        }
    memcpy(g->A, F, sizeof(double) * n * n);
    memcpy(g->C, C, sizeof(double) * n * n);
    memcpy(g->p, p, sizeof(double) * n);
    memcpy(g->c, f, sizeof(double) * n);
    if (cs->type == 1) {
        for (j = 0; j < n; ++j)
            for (i = 0; i < n; ++i) { g->At[IX(i, j, n)] = F[IX(j, i, n)]; g->Pinv[IX(i, j, n)] = (i == j); }
    }
}

/* update_segment_data(p, c, id) (LU :76-80, CHOLESKY :197-201) */
static void cond_update_vec(orc_condensed *cs, const double *p, const double *f, int id) {
    memcpy(cs->seg[id].p, p, sizeof(double) * cs->n);
    memcpy(cs->seg[id].c, f, sizeof(double) * cs->n);
}

/* CondensedSystemLUSolver::backward (condensed_system.hpp:82-103) */
static int cond_lu_backward(orc_condensed *cs) {
    int n = cs->n, i, j, a, b, t;
    for (i = cs->ns - 2; i >= 0; --i) {
        orc_cseg *g = &cs->seg[i], *nx_ = &cs->seg[i + 1];
        for (b = 0; b < n; ++b)
            for (a = 0; a < n; ++a) {
                double s1 = 0.0, s2 = 0.0;
                for (t = 0; t < n; ++t) {
                    s1 += g->C[IX(a, t, n)] * nx_->P[IX(t, b, n)];
                    s2 += nx_->P[IX(a, t, n)] * g->A[IX(t, b, n)];
                }
                g->PC[IX(a, b, n)] = s1 + (a == b ? 1.0 : 0.0);
                g->PA[IX(a, b, n)] = s2;
            }
        memcpy(g->LU, g->PC, sizeof(double) * n * n);
        lu_factor(g->LU, g->piv, n);
        for (j = 0; j < n; ++j) {
            double col[ORC_SMAX];
            for (a = 0; a < n; ++a) col[a] = g->A[IX(a, j, n)];
            lu_solve(g->LU, g->piv, n, col);
            for (a = 0; a < n; ++a) g->D[IX(a, j, n)] = col[a];
        }
        for (b = 0; b < n; ++b)
            for (a = 0; a < n; ++a) {
                double s = 0.0;
                for (t = 0; t < n; ++t) s += g->D[IX(t, a, n)] * g->PA[IX(t, b, n)];
                g->P[IX(a, b, n)] += s;
            }
    }
    return 1;
}

/* CondensedSystemLUSolver::forward (condensed_system.hpp:105-138) */
static void cond_lu_forward(orc_condensed *cs, const double *x0) {
    int n = cs->n, i, a, t;
    double cbar[ORC_SMAX];
    for (i = cs->ns - 2; i >= 0; --i) {
        orc_cseg *g = &cs->seg[i], *nx_ = &cs->seg[i + 1];
        for (a = 0; a < n; ++a) {
            double s = nx_->p[a];
            for (t = 0; t < n; ++t) s += nx_->P[IX(a, t, n)] * g->c[t];
            cbar[a] = s;
        }
        for (a = 0; a < n; ++a) {
            double s = 0.0;
            for (t = 0; t < n; ++t) s += g->D[IX(t, a, n)] * cbar[t];
            g->p[a] += s;
        }
    }
    memcpy(cs->seg[0].xhat, x0, sizeof(double) * n);
    for (i = 0; i < cs->ns - 1; ++i) {
        orc_cseg *g = &cs->seg[i], *nx_ = &cs->seg[i + 1];
        for (a = 0; a < n; ++a) {
            double s = 0.0;
            for (t = 0; t < n; ++t) s += g->A[IX(a, t, n)] * g->xhat[t];
            g->c[a] += s;
        }
        for (a = 0; a < n; ++a) {
            double s = 0.0;
            for (t = 0; t < n; ++t) s += g->C[IX(a, t, n)] * nx_->p[t];
            g->c[a] -= s;
        }
        memcpy(nx_->xhat, g->c, sizeof(double) * n);
        lu_solve(g->LU, g->piv, n, nx_->xhat);
        for (a = 0; a < n; ++a) {
            double s = nx_->p[a];
            for (t = 0; t < n; ++t) s += nx_->P[IX(a, t, n)] * nx_->xhat[t];
            g->uhat[a] = s;
        }
    }
}

static int chol_inv_step(orc_condensed *cs, int i) {
    /* P_chol[i+1] = llt(P_{i+1}); Pinv_{i+1} = P_{i+1}^{-1}; C_i += Pinv; C_chol[i] = llt(C_i)
     * (condensed_system.hpp:218-226 and :235-246) */
    int n = cs->n, j, a;
    orc_cseg *g = &cs->seg[i], *nx_ = &cs->seg[i + 1];
    if (llt_lower(nx_->P, nx_->Lp, n) >= 0) return 0;
    for (j = 0; j < n; ++j) {
        double col[ORC_SMAX];
        for (a = 0; a < n; ++a) col[a] = nx_->Pinv[IX(a, j, n)];
        llt_solve(nx_->Lp, n, col);
        for (a = 0; a < n; ++a) nx_->Pinv[IX(a, j, n)] = col[a];
    }
    for (j = 0; j < n * n; ++j) g->C[j] += nx_->Pinv[j];
    if (llt_lower(g->C, g->Lc, n) >= 0) return 0;
    return 1;
}

/* CondensedSystemCholeskySolver::backward (condensed_system.hpp:203-250) */
static int cond_chol_backward(orc_condensed *cs) {
    int n = cs->n, i, j, a, b, t;
    for (i = cs->ns - 2; i >= 1; --i) {
        orc_cseg *g = &cs->seg[i];
        if (!chol_inv_step(cs, i)) return 0;
        for (j = 0; j < n; ++j) { /* A_i <- C_i^{-1} A_i */
            double col[ORC_SMAX];
            for (a = 0; a < n; ++a) col[a] = g->A[IX(a, j, n)];
            llt_solve(g->Lc, n, col);
            for (a = 0; a < n; ++a) g->A[IX(a, j, n)] = col[a];
        }
        for (b = 0; b < n; ++b) /* P_i += At_i A_i */
            for (a = 0; a < n; ++a) {
                double s = 0.0;
                for (t = 0; t < n; ++t) s += g->At[IX(a, t, n)] * g->A[IX(t, b, n)];
                g->P[IX(a, b, n)] += s;
            }
    }
    return chol_inv_step(cs, 0);
}

/* CondensedSystemCholeskySolver::forward (condensed_system.hpp:252-290) */
static void cond_chol_forward(orc_condensed *cs, const double *x0) {
    int n = cs->n, i, a, t;
    for (i = cs->ns - 2; i >= 1; --i) {
        orc_cseg *g = &cs->seg[i], *nx_ = &cs->seg[i + 1];
        llt_solve(nx_->Lp, n, nx_->p);
        for (a = 0; a < n; ++a) g->c[a] += nx_->p[a];
        for (a = 0; a < n; ++a) {
            double s = 0.0;
            for (t = 0; t < n; ++t) s += g->A[IX(t, a, n)] * g->c[t];
            g->p[a] += s;
        }
    }
    llt_solve(cs->seg[1].Lp, n, cs->seg[1].p);
    for (a = 0; a < n; ++a) cs->seg[0].c[a] += cs->seg[1].p[a];
    memcpy(cs->seg[0].xhat, x0, sizeof(double) * n);
    for (i = 0; i < cs->ns - 1; ++i) {
        orc_cseg *g = &cs->seg[i], *nx_ = &cs->seg[i + 1];
        for (a = 0; a < n; ++a) {
            double s = g->c[a];
            for (t = 0; t < n; ++t) s += g->At[IX(t, a, n)] * g->xhat[t];
            g->uhat[a] = s;
        }
        llt_solve(g->Lc, n, g->uhat);
        for (a = 0; a < n; ++a) {
            double s = -nx_->p[a];
            for (t = 0; t < n; ++t) s += nx_->Pinv[IX(a, t, n)] * g->uhat[t];
            nx_->xhat[a] = s;
        }
    }
}

/* ------------------------------------------------------------------------ */
/* LQRParallelSolver (lqr_solver_parallel.hpp:19-238), single-threaded       */
/* restatement: the OpenMP team is a loop over segments (results do not      */
/* depend on thread scheduling: segments own disjoint workspaces).           */
/* ------------------------------------------------------------------------ */
typedef struct {
    orc_model *md;
    int ns;
    int *idx_start, *Nseg;
    orc_stage **data; /* per segment Nseg+1 stages */
    orc_condensed *cs;
    int last_backward_ok;
    int threads; /* 0: one thread (segments in turn); > 0: OpenMP team of ns threads (CPU baseline (ii)) */
} orc_parallel;

/* Segmentation (lqr_solver_parallel.hpp:64-88): Nseg_i = int(N/(scale+ns-1))
 * for i < ns-1 with scale = 1.55 under load balancing, the last segment takes
 * the remainder.  Returns 0 if any segment would be empty (the reference
 * would then run out of bounds; SURVEY.md section 7 hard part 8). */
int orc_segmentation(int N, int ns, int load_balancing, int *idx_start, int *Nseg) {
    double alpha = 1.55, scale = load_balancing ? alpha : 1.0;
    int i;
    for (i = 0; i < ns; ++i) {
        idx_start[i] = (i == 0) ? 0 : idx_start[i - 1] + Nseg[i - 1];
        Nseg[i] = (i < ns - 1) ? (int)((double)N / (scale + ns - 1)) : N - idx_start[i];
        if (Nseg[i] < 1) return 0;
    }
    return 1;
}

void *orc_parallel_create(int n, int m, int N, const int *nc, const double *E, const double *c, const double *H,
                          const double *h, const double *D, int ns, int load_balancing, int type) {
    orc_parallel *o;
    int i, k;
    if (N < 1 || ns < 1 || n < 1 || m < 1 || n + m > ORC_SMAX) return NULL; /* s <= 256 here */
    if (type == 1 && ns < 2) return NULL; /* CHOLESKY with ns=1 reads out of bounds (condensed_system.hpp:230) */
    o = (orc_parallel *)xcalloc(1, sizeof(orc_parallel));
    o->md = model_create(n, m, N, nc, E, c, H, h, D);
    o->ns = ns;
    o->idx_start = (int *)xcalloc(ns, sizeof(int));
    o->Nseg = (int *)xcalloc(ns, sizeof(int));
    if (!orc_segmentation(N, ns, load_balancing, o->idx_start, o->Nseg)) {
        free(o->idx_start); free(o->Nseg); model_destroy(o->md); free(o);
        return NULL;
    }
    o->data = (orc_stage **)xcalloc(ns, sizeof(orc_stage *));
    for (i = 0; i < ns; ++i) {
        o->data[i] = (orc_stage *)xcalloc(o->Nseg[i] + 1, sizeof(orc_stage));
        for (k = 0; k <= o->Nseg[i]; ++k) {
            int g = o->idx_start[i] + k;
            stage_init(&o->data[i][k], n, m, o->md->nc[g], g == N);
        }
    }
    o->cs = cond_create(n, ns, type);
    return o;
}

void orc_parallel_destroy(void *p) {
    orc_parallel *o = (orc_parallel *)p;
    int i, k;
    if (!o) return;
    for (i = 0; i < o->ns; ++i) {
        for (k = 0; k <= o->Nseg[i]; ++k) stage_free(&o->data[i][k]);
        free(o->data[i]);
    }
    free(o->data); free(o->idx_start); free(o->Nseg);
    cond_destroy(o->cs);
    model_destroy(o->md);
    free(o);
}

void orc_parallel_segments(void *p, int *idx_start, int *Nseg) {
    orc_parallel *o = (orc_parallel *)p;
    memcpy(idx_start, o->idx_start, sizeof(int) * o->ns);
    memcpy(Nseg, o->Nseg, sizeof(int) * o->ns);
}

void orc_parallel_update_problem_data(void *p, const double *ws, const double *ys, const double *zs,
                                      const double *inv_rho, double sigma) { /* :115-140 */
    orc_parallel *o = (orc_parallel *)p;
    int i, k;
    for (i = 0; i < o->ns; ++i)
        for (k = 0; k <= o->Nseg[i]; ++k)
            stage_update(o->md, o->idx_start[i] + k, &o->data[i][k], ws, ys, zs, inv_rho, sigma);
}

static void par_reduction(orc_parallel *o, int tid, const double *rho, int fact) { /* :164-211 */
    int N0 = o->idx_start[tid], Nseg = o->Nseg[tid], N1 = N0 + Nseg, k;
    int last = (tid == o->ns - 1), n = o->md->n;
    orc_stage *d = o->data[tid];
    pk_terminal(o->md, &d[Nseg], rho, last, fact);
    for (k = N1 - 1; k >= N0; --k) pk_step(o->md, k, rho, &d[k - N0 + 1], &d[k - N0], last, fact);
    if (fact)
        cond_update_full(o->cs, d[0].L, d[0].dim, d[0].dim - n, d[0].F, d[0].C, d[0].lp + (d[0].dim - n), d[0].f, tid);
    else
        cond_update_vec(o->cs, d[0].lp + (d[0].dim - n), d[0].f, tid);
}

#ifdef _OPENMP
#include <omp.h>
#define PAR_FOR _Pragma("omp parallel for num_threads(o->ns) schedule(static, 1) if (o->threads > 0)")
#else
#define PAR_FOR
#endif

/* The reference's OpenMP team: num_segments threads, thread tid pinned to core
 * tid (lqr_solver_parallel.hpp:102-112).  Here "core tid" is the tid-th CPU of
 * the process's allowed set (the GPU box grants a CPU share, not cores 0..).
 * Results do not depend on it: segments own disjoint workspaces. */
int orc_parallel_set_threads(void *p, int on, int pin) {
    orc_parallel *o = (orc_parallel *)p;
    int pinned = 0;
    o->threads = on ? o->ns : 0;
#ifdef _OPENMP
    if (on && pin) {
        cpu_set_t allowed;
        if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return 0;
#pragma omp parallel num_threads(o->ns) reduction(+ : pinned)
        {
            int tid = omp_get_thread_num(), cpu, seen = -1;
            for (cpu = 0; cpu < CPU_SETSIZE; ++cpu)
                if (CPU_ISSET(cpu, &allowed) && ++seen == tid) {
                    cpu_set_t one;
                    CPU_ZERO(&one);
                    CPU_SET(cpu, &one);
                    pinned += sched_setaffinity(0, sizeof(one), &one) == 0;
                    break;
                }
        }
    }
#else
    (void)pin;
#endif
    return pinned;
}

void orc_parallel_backward(void *p, const double *rho) { /* :142-146 */
    orc_parallel *o = (orc_parallel *)p;
    int i;
    PAR_FOR
    for (i = 0; i < o->ns; ++i) par_reduction(o, i, rho, 1);
    o->last_backward_ok = (o->cs->type == 0) ? cond_lu_backward(o->cs) : cond_chol_backward(o->cs);
}

void orc_parallel_backward_without_factorization(void *p, const double *rho) { /* :148-154 */
    orc_parallel *o = (orc_parallel *)p;
    int i;
    PAR_FOR
    for (i = 0; i < o->ns; ++i) par_reduction(o, i, rho, 0);
}

int orc_parallel_backward_ok(void *p) { return ((orc_parallel *)p)->last_backward_ok; }

void orc_parallel_forward(void *p, const double *x0, double *ws) { /* :213-238 */
    orc_parallel *o = (orc_parallel *)p;
    int n = o->md->n, m = o->md->m, s = n + m, i;
    if (o->cs->type == 0) cond_lu_forward(o->cs, x0);
    else cond_chol_forward(o->cs, x0);
    PAR_FOR
    for (i = 0; i < o->ns; ++i) {
        int N0 = o->idx_start[i], N1 = N0 + o->Nseg[i], last = (i == o->ns - 1), k, a, t;
        const double *uhat = o->cs->seg[i].uhat;
        memcpy(ws + (size_t)N0 * s + m, o->cs->seg[i].xhat, sizeof(double) * n);
        for (k = N0; k < N1; ++k) {
            orc_stage *st = &o->data[i][k - N0];
            double Gu[ORC_SMAX];
            if (!last)
                for (a = 0; a < m; ++a) {
                    double acc = 0.0;
                    for (t = 0; t < n; ++t) acc += st->G[IX(a, t, m)] * uhat[t];
                    Gu[a] = acc;
                }
            k_forward(o->md, k, st, ws + (size_t)k * s, ws + (size_t)(k + 1) * s, last ? NULL : Gu,
                      last ? 1 : (k < N1 - 1));
        }
    }
}

/* Segment summary accessor for tests: the element (F, C, f, P, p) exported by
 * segment `id` (condensed-solver state after backward). */
void orc_parallel_get_segment(void *p, int id, double *P, double *pv, double *xhat, double *uhat) {
    orc_parallel *o = (orc_parallel *)p;
    orc_cseg *g = &o->cs->seg[id];
    int n = o->md->n;
    if (P) memcpy(P, g->P, sizeof(double) * n * n);
    if (pv) memcpy(pv, g->p, sizeof(double) * n);
    if (xhat) memcpy(xhat, g->xhat, sizeof(double) * n);
    if (uhat) memcpy(uhat, g->uhat, sizeof(double) * n);
}

/* ------------------------------------------------------------------------ */
/* KKT assembly (kkt.hpp) + QDLDL (github.com/osqp/qdldl, unpinned: the      */
/* reference clones master, README.md:24).  QDLDL's published algorithm:     */
/* elimination tree + up-looking LDL^T in natural order + triangular solves. */
/* ------------------------------------------------------------------------ */
typedef struct { int r, c; double v; } trip;

typedef struct {
    orc_model *md;
    int dim;                 /* KKT dimension */
    int nnz;
    int *Ap, *Ai; double *Ax; /* upper CSC */
    int *rho_pos;            /* positions of the y-block diagonals in Ax */
    double *rhs;
    /* factor */
    int *etree, *Lnz, *Lp, *Li; double *Lx, *D, *Dinv; int sumLnz;
    double *x;
} orc_kkt;

static int trip_cmp(const void *a, const void *b) {
    const trip *x = (const trip *)a, *y = (const trip *)b;
    if (x->c != y->c) return x->c - y->c;
    return x->r - y->r;
}

typedef struct { trip *t; int n, cap; } tlist;

static void tpush(tlist *l, int r, int c, double v) {
    if (l->n == l->cap) { l->cap = l->cap ? 2 * l->cap : 1024; l->t = (trip *)realloc(l->t, sizeof(trip) * l->cap); }
    l->t[l->n].r = r; l->t[l->n].c = c; l->t[l->n].v = v; l->n++;
}

/* assign_dense_matrix (utils.hpp:10-34), insert mode */
static void assign_dense(tlist *l, int i0, int j0, const double *M, int rows, int cols, int ld, int transpose,
                         int fill_upper, int ignore_zeros) {
    int i, j;
    for (j = 0; j < cols; ++j)
        for (i = 0; i < rows; ++i) {
            double v = transpose ? M[IX(j, i, ld)] : M[IX(i, j, ld)];
            if (fill_upper && i > j) continue;
            if (ignore_zeros && v == 0.0) continue;
            tpush(l, i0 + i, j0 + j, v);
        }
}

static void assign_diag(tlist *l, int i0, int j0, double v, int size) { /* utils.hpp:51-65 */
    int i;
    for (i = 0; i < size; ++i) tpush(l, i0 + i, j0 + i, v);
}

/* QDLDL_etree */
static int qdldl_etree(int n, const int *Ap, const int *Ai, int *work, int *Lnz, int *etree) {
    int i, j, p, sumLnz = 0;
    for (i = 0; i < n; ++i) { work[i] = 0; Lnz[i] = 0; etree[i] = -1; }
    for (j = 0; j < n; ++j) {
        work[j] = j;
        if (Ap[j] == Ap[j + 1]) return -1;
        for (p = Ap[j]; p < Ap[j + 1]; ++p) {
            i = Ai[p];
            if (i > j) return -1;
            while (work[i] != j) {
                if (etree[i] == -1) etree[i] = j;
                Lnz[i]++;
                work[i] = j;
                i = etree[i];
            }
        }
    }
    for (i = 0; i < n; ++i) sumLnz += Lnz[i];
    return sumLnz;
}

/* QDLDL_factor (up-looking LDL^T). Returns number of positive D or -1. */
static int qdldl_factor(int n, const int *Ap, const int *Ai, const double *Ax, int *Lp, int *Li, double *Lx,
                        double *D, double *Dinv, const int *Lnz, const int *etree) {
    int i, j, k, nnzY, bidx, cidx, nextIdx, nnzE, tmpIdx, pos = 0;
    int *yIdx = (int *)xcalloc(n, sizeof(int)), *elim = (int *)xcalloc(n, sizeof(int));
    int *nextSpace = (int *)xcalloc(n, sizeof(int));
    unsigned char *mark = (unsigned char *)xcalloc(n, 1);
    double *yVals = (double *)xcalloc(n, sizeof(double)), yv;
    Lp[0] = 0;
    for (i = 0; i < n; ++i) { Lp[i + 1] = Lp[i] + Lnz[i]; nextSpace[i] = Lp[i]; D[i] = 0.0; }
    D[0] = Ax[0];
    if (D[0] == 0.0) { pos = -1; goto done; }
    if (D[0] > 0.0) pos++;
    Dinv[0] = 1.0 / D[0];
    for (k = 1; k < n; ++k) {
        nnzY = 0;
        for (i = Ap[k]; i < Ap[k + 1]; ++i) {
            bidx = Ai[i];
            if (bidx == k) { D[k] = Ax[i]; continue; }
            yVals[bidx] = Ax[i];
            nextIdx = bidx;
            if (!mark[nextIdx]) {
                mark[nextIdx] = 1; elim[0] = nextIdx; nnzE = 1;
                nextIdx = etree[bidx];
                while (nextIdx != -1 && nextIdx < k) {
                    if (mark[nextIdx]) break;
                    mark[nextIdx] = 1; elim[nnzE++] = nextIdx; nextIdx = etree[nextIdx];
                }
                while (nnzE) yIdx[nnzY++] = elim[--nnzE];
            }
        }
        for (i = nnzY - 1; i >= 0; --i) {
            cidx = yIdx[i];
            tmpIdx = nextSpace[cidx];
            yv = yVals[cidx];
            for (j = Lp[cidx]; j < tmpIdx; ++j) yVals[Li[j]] -= Lx[j] * yv;
            Li[tmpIdx] = k;
            Lx[tmpIdx] = yv * Dinv[cidx];
            D[k] -= yv * Lx[tmpIdx];
            nextSpace[cidx]++;
            yVals[cidx] = 0.0;
            mark[cidx] = 0;
        }
        if (D[k] == 0.0) { pos = -1; goto done; }
        if (D[k] > 0.0) pos++;
        Dinv[k] = 1.0 / D[k];
    }
done:
    free(yIdx); free(elim); free(nextSpace); free(mark); free(yVals);
    return pos;
}

static void qdldl_solve(int n, const int *Lp, const int *Li, const double *Lx, const double *Dinv, double *x) {
    int i, j;
    for (i = 0; i < n; ++i)
        for (j = Lp[i]; j < Lp[i + 1]; ++j) x[Li[j]] -= Lx[j] * x[i];
    for (i = 0; i < n; ++i) x[i] *= Dinv[i];
    for (i = n - 1; i >= 0; --i)
        for (j = Lp[i]; j < Lp[i + 1]; ++j) x[i] -= Lx[j] * x[Li[j]];
}

/* QDLDLSolver ctor (qdldl_solver.hpp:36-45): KKTSystem (kkt.hpp:45-63),
 * form_KKT_matrix with rho_dyn = sigma = 1e-6 (kkt.hpp:124-205), CSC export
 * (kkt.hpp:302-331), create_workspace -> QDLDL_etree (qdldl_solver.hpp:47-78). */
void *orc_kkt_create(int n, int m, int N, const int *nc, const double *E, const double *c, const double *H,
                     const double *h, const double *D, double rho_dyn, double sigma) {
    orc_kkt *o;
    orc_model *md;
    int s = n + m, k, i, row_offset, col_offset, dim;
    tlist tl = {0, 0, 0};
    double *Hs;
    int *work;
    if (N < 1) return NULL;
    o = (orc_kkt *)xcalloc(1, sizeof(orc_kkt));
    md = o->md = model_create(n, m, N, nc, E, c, H, h, D);
    /* kkt.hpp:47-56: num_rows = (nxu + nc0) + sum_{k=1}^{N-1}(nxu + nc_k + nx) + (nx + nc_N).
     * The primal part holds u0 only for stage 0, so the count equals
     * N*nxu + sum nc + N*nx. */
    dim = N * s;
    for (k = 0; k <= N; ++k) dim += md->nc[k];
    dim += N * n;
    o->dim = dim;
    Hs = (double *)xcalloc((size_t)s * s, sizeof(double));
    row_offset = 0;
    col_offset = N * s;
    { /* stage 0 (kkt.hpp:138-159) */
        int nc0 = md->nc[0];
        const double *Hm = md->H + H_off(md, 0);
        const double *Em = md->E;
        for (i = 0; i < s * s; ++i) Hs[i] = Hm[i];
        for (i = 0; i < s; ++i) Hs[IX(i, i, s)] += sigma;
        assign_dense(&tl, row_offset, row_offset, Hs, m, m, s, 0, 1, 1); /* R0 */
        if (nc0 > 0) assign_dense(&tl, row_offset, col_offset, md->D + md->d_off[0], m, nc0, nc0, 1, 0, 1);
        assign_dense(&tl, row_offset, col_offset + nc0, Em, m, n, n, 1, 0, 0); /* B0^T */
        row_offset += m;
        col_offset += nc0;
    }
    for (k = 1; k < N; ++k) { /* kkt.hpp:161-176 */
        int nck = md->nc[k];
        const double *Hm = md->H + H_off(md, k);
        const double *Em = md->E + (size_t)k * n * s;
        for (i = 0; i < s * s; ++i) Hs[i] = Hm[i];
        for (i = 0; i < s; ++i) Hs[IX(i, i, s)] += sigma;
        /* fill_stage_cost_matrices (kkt.hpp:65-75): Q upper, S^T block, R upper */
        assign_dense(&tl, row_offset, row_offset, Hs + IX(m, m, s), n, n, s, 0, 1, 1);
        assign_dense(&tl, row_offset, row_offset + n, Hs + IX(m, 0, s), n, m, s, 0, 0, 1);
        assign_dense(&tl, row_offset + n, row_offset + n, Hs, m, m, s, 0, 1, 1);
        /* fill_stage_dynamics_matrices (kkt.hpp:77-89) */
        assign_diag(&tl, row_offset, col_offset, -1.0, n);
        assign_dense(&tl, row_offset, col_offset + n + nck, Em + IX(0, m, n), n, n, n, 1, 0, 0); /* A^T */
        assign_dense(&tl, row_offset + n, col_offset + n + nck, Em, m, n, n, 1, 0, 0);            /* B^T */
        /* fill_stage_constraint_matrices (kkt.hpp:91-103) */
        if (nck > 0) {
            const double *Dk = md->D + md->d_off[k];
            assign_dense(&tl, row_offset, col_offset + n, Dk + IX(0, m, nck), n, nck, nck, 1, 0, 1);
            assign_dense(&tl, row_offset + n, col_offset + n, Dk, m, nck, nck, 1, 0, 1);
        }
        row_offset += s;
        col_offset += nck + n;
    }
    { /* terminal (kkt.hpp:178-193) */
        int ncN = md->nc[N];
        const double *Hm = md->H + H_off(md, N);
        double *HN = (double *)xcalloc((size_t)n * n, sizeof(double));
        for (i = 0; i < n * n; ++i) HN[i] = Hm[i];
        for (i = 0; i < n; ++i) HN[IX(i, i, n)] += sigma;
        assign_dense(&tl, row_offset, row_offset, HN, n, n, n, 0, 1, 1);
        assign_diag(&tl, row_offset, col_offset, -1.0, n);
        if (ncN > 0) assign_dense(&tl, row_offset, col_offset + n, md->D + md->d_off[N], n, ncN, ncN, 1, 0, 1);
        row_offset += n;
        free(HN);
    }
    { /* regularization (kkt.hpp:195-204) */
        assign_diag(&tl, row_offset, row_offset, -1.0, md->nc[0]);
        row_offset += md->nc[0];
        for (k = 1; k <= N; ++k) {
            assign_diag(&tl, row_offset, row_offset, -rho_dyn, n);
            row_offset += n;
            assign_diag(&tl, row_offset, row_offset, -1.0, md->nc[k]);
            row_offset += md->nc[k];
        }
    }
    free(Hs);
    /* compress to CSC (sorted rows within a column, as Eigen's compressed form) */
    qsort(tl.t, tl.n, sizeof(trip), trip_cmp);
    o->nnz = tl.n;
    o->Ap = (int *)xcalloc(dim + 1, sizeof(int));
    o->Ai = (int *)xcalloc(tl.n, sizeof(int));
    o->Ax = (double *)xcalloc(tl.n, sizeof(double));
    for (i = 0; i < tl.n; ++i) { o->Ap[tl.t[i].c + 1]++; o->Ai[i] = tl.t[i].r; o->Ax[i] = tl.t[i].v; }
    for (i = 0; i < dim; ++i) o->Ap[i + 1] += o->Ap[i];
    free(tl.t);
    /* positions of the y-block diagonals, for update_rho_vecs (kkt.hpp:105-122) */
    o->rho_pos = (int *)xcalloc(md->y_off[N + 1], sizeof(int));
    {
        int ro = N * s, p;
        for (k = 0; k <= N; ++k) {
            for (i = 0; i < md->nc[k]; ++i) {
                int col = ro + i;
                o->rho_pos[md->y_off[k] + i] = -1;
                for (p = o->Ap[col]; p < o->Ap[col + 1]; ++p)
                    if (o->Ai[p] == col) o->rho_pos[md->y_off[k] + i] = p;
            }
            ro += md->nc[k] + n;
        }
    }
    o->rhs = (double *)xcalloc(dim, sizeof(double));
    o->x = (double *)xcalloc(dim, sizeof(double));
    o->etree = (int *)xcalloc(dim, sizeof(int));
    o->Lnz = (int *)xcalloc(dim, sizeof(int));
    o->Lp = (int *)xcalloc(dim + 1, sizeof(int));
    o->D = (double *)xcalloc(dim, sizeof(double));
    o->Dinv = (double *)xcalloc(dim, sizeof(double));
    work = (int *)xcalloc(3 * (size_t)dim, sizeof(int));
    o->sumLnz = qdldl_etree(dim, o->Ap, o->Ai, work, o->Lnz, o->etree);
    free(work);
    if (o->sumLnz < 0) { o->sumLnz = 0; }
    o->Li = (int *)xcalloc(o->sumLnz, sizeof(int));
    o->Lx = (double *)xcalloc(o->sumLnz, sizeof(double));
    return o;
}

void orc_kkt_destroy(void *p) {
    orc_kkt *o = (orc_kkt *)p;
    if (!o) return;
    free(o->Ap); free(o->Ai); free(o->Ax); free(o->rho_pos); free(o->rhs); free(o->x);
    free(o->etree); free(o->Lnz); free(o->Lp); free(o->Li); free(o->Lx); free(o->D); free(o->Dinv);
    model_destroy(o->md);
    free(o);
}

int orc_kkt_dim(void *p) { return ((orc_kkt *)p)->dim; }
int orc_kkt_nnz(void *p) { return ((orc_kkt *)p)->nnz; }
int orc_kkt_sumLnz(void *p) { return ((orc_kkt *)p)->sumLnz; }

/* KKTSystem::form_rhs (kkt.hpp:224-300) via QDLDLSolver::update_problem_data */
void orc_kkt_update_problem_data(void *p, const double *ws, const double *ys, const double *zs,
                                 const double *inv_rho, double sigma) {
    orc_kkt *o = (orc_kkt *)p;
    orc_model *md = o->md;
    int n = md->n, m = md->m, s = n + m, N = md->N, k, i;
    int r1 = 0, r2 = N * s;
    { /* stage 0 */
        int nc0 = md->nc[0];
        for (i = 0; i < m; ++i) o->rhs[i] = -md->h[i] + sigma * ws[i];
        for (i = 0; i < nc0; ++i) o->rhs[r2 + i] = zs[md->y_off[0] + i] - inv_rho[md->y_off[0] + i] * ys[md->y_off[0] + i];
        for (i = 0; i < n; ++i) o->rhs[r2 + nc0 + i] = -md->c[i];
        r1 += m;
        r2 += nc0 + n;
    }
    for (k = 1; k < N; ++k) {
        int nck = md->nc[k];
        const double *hk = md->h + h_off(md, k), *wk = ws + h_off(md, k);
        for (i = 0; i < n; ++i) o->rhs[r1 + i] = -hk[m + i] + sigma * wk[m + i];
        for (i = 0; i < m; ++i) o->rhs[r1 + n + i] = -hk[i] + sigma * wk[i];
        for (i = 0; i < nck; ++i)
            o->rhs[r2 + i] = zs[md->y_off[k] + i] - inv_rho[md->y_off[k] + i] * ys[md->y_off[k] + i];
        for (i = 0; i < n; ++i) o->rhs[r2 + nck + i] = -md->c[(size_t)k * n + i];
        r1 += s;
        r2 += nck + n;
    }
    {
        int ncN = md->nc[N];
        const double *hN = md->h + h_off(md, N), *wN = ws + h_off(md, N);
        for (i = 0; i < n; ++i) o->rhs[r1 + i] = -hN[i] + sigma * wN[i];
        for (i = 0; i < ncN; ++i)
            o->rhs[r2 + i] = zs[md->y_off[N] + i] - inv_rho[md->y_off[N] + i] * ys[md->y_off[N] + i];
    }
}

/* QDLDLSolver::backward (qdldl_solver.hpp:88-109): update_rho_vecs writes
 * -inv_rho on the y diagonals, then QDLDL_factor.  Returns the factor status. */
int orc_kkt_backward(void *p, const double *inv_rho) {
    orc_kkt *o = (orc_kkt *)p;
    int i, ny = o->md->y_off[o->md->N + 1];
    for (i = 0; i < ny; ++i)
        if (o->rho_pos[i] >= 0) o->Ax[o->rho_pos[i]] = -inv_rho[i];
    return qdldl_factor(o->dim, o->Ap, o->Ai, o->Ax, o->Lp, o->Li, o->Lx, o->D, o->Dinv, o->Lnz, o->etree);
}

/* QDLDLSolver::forward (qdldl_solver.hpp:111-151) */
void orc_kkt_forward(void *p, const double *x0, double *ws) {
    orc_kkt *o = (orc_kkt *)p;
    orc_model *md = o->md;
    int n = md->n, m = md->m, s = n + m, N = md->N, k, i, j, off;
    /* update_rhs_initial_stage (kkt.hpp:207-222): accumulates (+=) */
    for (i = 0; i < m; ++i) {
        double a = 0.0;
        for (j = 0; j < n; ++j) a += md->H[IX(i, m + j, s)] * x0[j]; /* S0 = H.topRightCorner(nu, nx) */
        o->rhs[i] += -a;
    }
    {
        int ro = N * s + md->nc[0];
        for (i = 0; i < n; ++i) {
            double a = 0.0;
            for (j = 0; j < n; ++j) a += md->E[IX(i, m + j, n)] * x0[j];
            o->rhs[ro + i] += -a;
        }
    }
    memcpy(o->x, o->rhs, sizeof(double) * o->dim);
    qdldl_solve(o->dim, o->Lp, o->Li, o->Lx, o->Dinv, o->x);
    memcpy(ws + m, x0, sizeof(double) * n);
    memcpy(ws, o->x, sizeof(double) * m);
    off = m;
    for (k = 1; k < N; ++k) {
        memcpy(ws + (size_t)k * s + m, o->x + off, sizeof(double) * n);
        memcpy(ws + (size_t)k * s, o->x + off + n, sizeof(double) * m);
        off += s;
    }
    memcpy(ws + (size_t)N * s, o->x + off, sizeof(double) * n);
}

/* The KKT right-hand side as the last forward left it (form_rhs plus the
 * accumulated update_rhs_initial_stage terms, kkt.hpp:207-300). */
void orc_kkt_get_rhs(void *p, double *r) {
    orc_kkt *o = (orc_kkt *)p;
    memcpy(r, o->rhs, sizeof(double) * o->dim);
}

/* Full KKT solution vector [primal | dual] after forward. */
void orc_kkt_get_solution(void *p, double *x) {
    orc_kkt *o = (orc_kkt *)p;
    memcpy(x, o->x, sizeof(double) * o->dim);
}

/* Upper-CSC export for tests (kkt.hpp:302-331). */
void orc_kkt_get_csc(void *p, int *Ap, int *Ai, double *Ax) {
    orc_kkt *o = (orc_kkt *)p;
    memcpy(Ap, o->Ap, sizeof(int) * (o->dim + 1));
    memcpy(Ai, o->Ai, sizeof(int) * o->nnz);
    memcpy(Ax, o->Ax, sizeof(double) * o->nnz);
}

/* ------------------------------------------------------------------------ */
/* Batched CPU baseline: independent serial solves over a batch of problems   */
/* (the reference has no batch API; BASELINE.md section 4 variant iii).       */
/* Data is batch-major: problem b's arrays follow each other.  nc = 0.        */
/* ------------------------------------------------------------------------ */
int orc_batched_serial_solve(int n, int m, int N, int batch, const double *E, const double *c, const double *H,
                             const double *h, const double *x0, double sigma, double *ws_out, int threads) {
    int s = n + m;
    size_t nE = (size_t)N * n * s, nc_ = (size_t)N * n, nH = (size_t)N * s * s + (size_t)n * n,
           nh = (size_t)N * s + n;
    int b;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (b = 0; b < batch; ++b) {
        double *zeros = (double *)xcalloc(nh, sizeof(double));
        void *o = orc_serial_create(n, m, N, NULL, E + b * nE, c + b * nc_, H + b * nH, h + b * nh, NULL);
        orc_serial_update_problem_data(o, zeros, NULL, NULL, NULL, sigma);
        orc_serial_backward(o, NULL);
        orc_serial_forward(o, x0 + (size_t)b * n, ws_out + b * nh);
        orc_serial_destroy(o);
        free(zeros);
    }
    (void)threads;
    return 0;
}

int orc_version(void) { return 1; }
