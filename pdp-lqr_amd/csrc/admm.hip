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
//   * k_admm_update (one block per problem, LPS lanes per stage) does the
//     z/y/w step, the termination test AND the next update_problem_data + penalty linear
//     term in the same pass: h~ = h - sigma w^{k+1} - D^T (rho o g^{k+1}),
//     g^{k+1} = z^{k+1} - inv_rho o y^{k+1} -- in the same operation order as
//     k_update_problem_data followed by k_penalty, so the fused and the
//     protocol-level iterations agree bit for bit;
//   * the backward is backward_without_factorization (keep_factors = 1) or
//     the factorizing kernel on the unchanged H~ (keep_factors = 0); at 12/4
//     with 4 constraint rows per stage (the C5 layout) the serial solver runs
//     the update of iteration it INSIDE the streamed backward of it + 1
//     (k_nofact_admm_dma), so no separate update pass touches HBM;
//   * adaptive rho (OSQP's rule, on by default): at a termination test a
//     problem whose normalised residual ratio e = sqrt((r_prim / max(|Dw|,|z|))
//     / (r_dual / |D^T y|)) leaves [1/tol, tol] scales its rho by e (clamped to
//     [1e-6, 1e6]); the next x-update then re-forms H~ and refactors the batch
//     (a problem whose rho did not move gets the same factor back);
//   * the KKT solver re-forms its right-hand side (form_rhs) and re-solves
//     with the factor of the first iteration (the KKT matrix depends on rho
//     only, qdldl_solver.hpp:88-109).
#include <algorithm>

#include "admm.hpp"
#include "device_common.hpp"
#include "solvers.hpp"

namespace pdplqr {

struct AdmmState {
    double *wt = nullptr;  // LQ solution of the current iteration (forward output)
    double *w = nullptr, *y = nullptr, *z = nullptr;
    double *lb = nullptr, *ub = nullptr, *rho = nullptr, *irho = nullptr;
    double *x0 = nullptr;
    double *prim = nullptr, *dual = nullptr;  // [b] residuals at the last check
    double *rscale = nullptr;                 // [b] adaptive-rho factor decided at the last test (1 = keep)
    int32_t *done = nullptr, *iters = nullptr, *conv = nullptr;
    int32_t *active = nullptr;    // [0] problems still iterating, [1] some rho changed
    int32_t *active_h = nullptr;  // pinned copy of active[0..1]
};

// sum over the LPS lanes of one stage (xor butterflies: every lane ends with
// the same bits)
template <int LPS>
__device__ __forceinline__ double stage_sum(double v) {
    if constexpr (LPS == 16) {
        return sum_row16(v);  // DPP form of the same butterfly
    } else {
#pragma unroll
        for (int m = 1; m < LPS; m <<= 1) v += __shfl_xor(v, m, 64);
        return v;
    }
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = fmax(v, __shfl_xor(v, m, 64));
    return v;
}

// One 256-thread block per problem.  A stage takes LPS lanes (one per entry
// of w_k: LPS = 16 for s <= 16, 32 for s <= 32, 64 for s <= 64), so a wave covers 64 / LPS
// consecutive stages with coalesced w / w~ / h loads; the block strides over
// the horizon.  Row r of D_k w~ is a butterfly sum over the stage's lanes;
// every lane then holds the row's new z, y, g and adds its column's share of
// D^T (rho o g), D^T rho (z+ - z), D^T y+ on the spot (no second pass).
// CHECK: the five maxima of the termination test reduce over the block and
// thread 0 decides (OSQP's test, admm.hip header), so there is no separate
// check launch and no atomics on the residuals.
// MNC > 0 (every stage has at most MNC constraint rows): the rows are a
// compile-time loop whose loads are all issued before the arithmetic (a
// runtime row loop waited for each row's loads in turn), and the row results
// are stored after it.  Same operations in the same order either way.
template <int LPS, bool FUSE, bool CHECK, int MNC>
__global__ void __launch_bounds__(256) k_admm_update(AdmmArgs a) {
    const Shape &sh = a.sh;
    const int b = blockIdx.x;
    if (a.done[b]) return;  // block-uniform
    constexpr int SPW = 64 / LPS;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, sub = lane / LPS, j = lane % LPS;
    const double al = a.alpha, bl = 1.0 - a.alpha;
    double rp = 0.0, dwm = 0.0, zm = 0.0, rd = 0.0, dty = 0.0, act = 0.0;
    for (int kb = wv * SPW; kb <= sh.N; kb += 4 * SPW) {
        // wave-uniform trip count: lanes past the horizon idle in the loop
        const int k = kb + sub;
        const bool stg = k <= sh.N;
        const int kk = stg ? k : sh.N;
        const int dim = kk < sh.N ? sh.s : sh.n;
        const bool col = stg && j < dim;
        const long long wo = (long long)b * sh.perh + (long long)kk * sh.s + (j < dim ? j : 0);
        // uniform row layout (a.uni): the offsets are arithmetic, so the trip's
        // loads do not wait on an offset load first
        const int yo0 = a.uni ? kk * a.uni : a.y_off[kk];
        const int nc = !stg ? 0 : (a.uni ? (kk < sh.N ? a.uni : 0) : a.y_off[kk + 1] - yo0);
        const long long yo = (long long)b * sh.ny + yo0;
        const double *Dk = a.D + (long long)b * sh.ndD + (a.uni ? (long long)kk * a.uni * sh.s : a.d_off[kk]);
        const double wtj = col ? a.wt[wo] : 0.0, wj = col ? a.w[wo] : 0.0;
        const double wn = al * wtj + bl * wj;
        double ag = 0.0, ad = 0.0, ay = 0.0;
        if constexpr (MNC > 0) {
            double dr[MNC], zr[MNC], yr[MNC], rr[MNC], ir[MNC], lo[MNC], hi[MNC], zs[MNC], ys[MNC], gs[MNC];
            const long long y0 = (long long)b * sh.ny;  // a valid slot for rows past nc
#pragma unroll
            for (int r = 0; r < MNC; ++r) {
                const bool row = r < nc;
                const long long q = row ? yo + r : y0;
                dr[r] = (row && col) ? Dk[r + j * nc] : 0.0;
                zr[r] = a.z[q];
                yr[r] = a.y[q];
                rr[r] = a.rho[q];
                ir[r] = a.irho[q];
                lo[r] = a.lb[q];
                hi[r] = a.ub[q];
            }
#pragma unroll
            for (int r = 0; r < MNC; ++r) {
                const bool row = r < nc;
                const double d = dr[r];
                const double v = stage_sum<LPS>(d * wtj);
                const double vw = stage_sum<LPS>(d * wj);
                const double vrel = al * v + bl * zr[r];
                const double zn = fmin(fmax(vrel + ir[r] * yr[r], lo[r]), hi[r]);
                const double yn = yr[r] + rr[r] * (vrel - zn);
                const double gn = zn - ir[r] * yn;
                zs[r] = zn;
                ys[r] = yn;
                gs[r] = gn;
                if (row) {
                    if (FUSE) ag += d * (rr[r] * gn);  // k_penalty's order: D[q][i] * (rho_q * g_q)
                    if (CHECK) {
                        const double dwn = al * v + bl * vw;  // D w^{k+1}
                        rp = fmax(rp, fabs(dwn - zn));
                        dwm = fmax(dwm, fabs(dwn));
                        zm = fmax(zm, fabs(zn));
                        ad += d * (rr[r] * (zn - zr[r]));
                        ay += d * yn;
                        if (zn <= lo[r] || zn >= hi[r]) act = 1.0;
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < MNC; ++r)
                if (j == 0 && r < nc) {
                    a.z[yo + r] = zs[r];
                    a.y[yo + r] = ys[r];
                    if (FUSE) a.gw[yo + r] = gs[r];
                }
        } else
        for (int r = 0; r < a.max_nc; ++r) {
            const bool row = r < nc;
            const double d = (row && col) ? Dk[r + j * nc] : 0.0;
            const double v = stage_sum<LPS>(d * wtj);
            const double vw = stage_sum<LPS>(d * wj);
            if (row) {
                const double zr = a.z[yo + r], yr = a.y[yo + r], rr = a.rho[yo + r], ir = a.irho[yo + r];
                const double vrel = al * v + bl * zr;
                const double zn = fmin(fmax(vrel + ir * yr, a.lb[yo + r]), a.ub[yo + r]);
                const double yn = yr + rr * (vrel - zn);
                const double gn = zn - ir * yn;
                if (j == 0) {
                    a.z[yo + r] = zn;
                    a.y[yo + r] = yn;
                    if (FUSE) a.gw[yo + r] = gn;
                }
                if (FUSE) ag += d * (rr * gn);  // k_penalty's order: D[q][i] * (rho_q * g_q)
                if (CHECK) {
                    const double dwn = al * v + bl * vw;  // D w^{k+1}
                    rp = fmax(rp, fabs(dwn - zn));
                    dwm = fmax(dwm, fabs(dwn));
                    zm = fmax(zm, fabs(zn));
                    ad += d * (rr * (zn - zr));
                    ay += d * yn;
                    if (zn <= a.lb[yo + r] || zn >= a.ub[yo + r]) act = 1.0;
                }
            }
        }
        if (col) {
            a.w[wo] = wn;
            if (FUSE) {
                // k_update_problem_data then k_penalty: (h - sigma w) - sum
                double hj = a.hv[wo] - a.sigma * wn;
                if (nc > 0 && !a.no_penalty) hj -= ag;
                a.hw[wo] = hj;
            }
        }
        if (CHECK) {
            rd = fmax(rd, fabs(ad));
            dty = fmax(dty, fabs(ay));
        }
    }
    if (CHECK) {
        __shared__ double red[4][6];
        rp = wave_max(rp);
        dwm = wave_max(dwm);
        zm = wave_max(zm);
        rd = wave_max(rd);
        dty = wave_max(dty);
        act = wave_max(act);
        if (lane == 0) {
            red[wv][0] = rp;
            red[wv][1] = dwm;
            red[wv][2] = zm;
            red[wv][3] = rd;
            red[wv][4] = dty;
            red[wv][5] = act;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
#pragma unroll
            for (int q = 1; q < 4; ++q) {
                rp = fmax(rp, red[q][0]);
                dwm = fmax(dwm, red[q][1]);
                zm = fmax(zm, red[q][2]);
                rd = fmax(rd, red[q][3]);
                dty = fmax(dty, red[q][4]);
                act = fmax(act, red[q][5]);
            }
            admm_decide(a, b, rp, dwm, zm, rd, dty, act);
        }
    }
}

// The same update for 64 < n + m <= 256 (the serial solver's kernels_xl.hip
// shapes): a stage takes the whole wave, lane j holding entries j + 64 e
// (e < EPL); a row of D_k w~ is the lane's partial sum over its entries, then
// the wave butterfly.  Per entry the operations are k_admm_update's, in its
// order (the D^T sums over the rows r in turn).
template <bool FUSE, bool CHECK, int EPL>
__global__ void __launch_bounds__(256) k_admm_update_xl(AdmmArgs a) {
    const Shape &sh = a.sh;
    const int b = blockIdx.x;
    if (a.done[b]) return;  // block-uniform
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const double al = a.alpha, bl = 1.0 - a.alpha;
    double rp = 0.0, dwm = 0.0, zm = 0.0, rd = 0.0, dty = 0.0, act = 0.0;
    for (int k = wv; k <= sh.N; k += 4) {  // wave-uniform
        const int dim = k < sh.N ? sh.s : sh.n;
        const int yo0 = a.uni ? k * a.uni : a.y_off[k];
        const int nc = a.uni ? (k < sh.N ? a.uni : 0) : a.y_off[k + 1] - yo0;
        const long long yo = (long long)b * sh.ny + yo0;
        const double *Dk = a.D + (long long)b * sh.ndD + (a.uni ? (long long)k * a.uni * sh.s : a.d_off[k]);
        bool col[EPL];
        long long wo[EPL];
        double wtj[EPL], wj[EPL], ag[EPL], ad[EPL], ay[EPL];
#pragma unroll
        for (int e = 0; e < EPL; ++e) {
            const int j = lane + 64 * e;
            col[e] = j < dim;
            wo[e] = (long long)b * sh.perh + (long long)k * sh.s + (col[e] ? j : 0);
            wtj[e] = col[e] ? a.wt[wo[e]] : 0.0;
            wj[e] = col[e] ? a.w[wo[e]] : 0.0;
            ag[e] = ad[e] = ay[e] = 0.0;
        }
        for (int r = 0; r < nc; ++r) {
            double d[EPL], pv = 0.0, pw = 0.0;
#pragma unroll
            for (int e = 0; e < EPL; ++e) {
                d[e] = col[e] ? Dk[r + (lane + 64 * e) * nc] : 0.0;
                pv += d[e] * wtj[e];
                pw += d[e] * wj[e];
            }
            const double v = stage_sum<64>(pv), vw = stage_sum<64>(pw);
            const double zr = a.z[yo + r], yr = a.y[yo + r], rr = a.rho[yo + r], ir = a.irho[yo + r];
            const double vrel = al * v + bl * zr;
            const double zn = fmin(fmax(vrel + ir * yr, a.lb[yo + r]), a.ub[yo + r]);
            const double yn = yr + rr * (vrel - zn);
            const double gn = zn - ir * yn;
            if (lane == 0) {
                a.z[yo + r] = zn;
                a.y[yo + r] = yn;
                if (FUSE) a.gw[yo + r] = gn;
            }
#pragma unroll
            for (int e = 0; e < EPL; ++e) {
                if (FUSE) ag[e] += d[e] * (rr * gn);
                if (CHECK) {
                    ad[e] += d[e] * (rr * (zn - zr));
                    ay[e] += d[e] * yn;
                }
            }
            if (CHECK) {
                const double dwn = al * v + bl * vw;
                rp = fmax(rp, fabs(dwn - zn));
                dwm = fmax(dwm, fabs(dwn));
                zm = fmax(zm, fabs(zn));
                if (zn <= a.lb[yo + r] || zn >= a.ub[yo + r]) act = 1.0;
            }
        }
#pragma unroll
        for (int e = 0; e < EPL; ++e) {
            if (col[e]) {
                const double wn = al * wtj[e] + bl * wj[e];
                a.w[wo[e]] = wn;
                if (FUSE) {
                    double hj = a.hv[wo[e]] - a.sigma * wn;
                    if (nc > 0 && !a.no_penalty) hj -= ag[e];
                    a.hw[wo[e]] = hj;
                }
            }
            if (CHECK) {
                rd = fmax(rd, fabs(ad[e]));
                dty = fmax(dty, fabs(ay[e]));
            }
        }
    }
    if (CHECK) {
        __shared__ double red[4][6];
        rp = wave_max(rp);
        dwm = wave_max(dwm);
        zm = wave_max(zm);
        rd = wave_max(rd);
        dty = wave_max(dty);
        act = wave_max(act);
        if (lane == 0) {
            red[wv][0] = rp;
            red[wv][1] = dwm;
            red[wv][2] = zm;
            red[wv][3] = rd;
            red[wv][4] = dty;
            red[wv][5] = act;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
#pragma unroll
            for (int q = 1; q < 4; ++q) {
                rp = fmax(rp, red[q][0]);
                dwm = fmax(dwm, red[q][1]);
                zm = fmax(zm, red[q][2]);
                rd = fmax(rd, red[q][3]);
                dty = fmax(dty, red[q][4]);
                act = fmax(act, red[q][5]);
            }
            admm_decide(a, b, rp, dwm, zm, rd, dty, act);
        }
    }
}

__global__ void k_admm_init(long long ny_total, const double *__restrict__ rho, double *__restrict__ irho) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < ny_total) irho[t] = 1.0 / rho[t];
}

// input check: e_lb <= e_ub and 0 < rho < inf on every row (OSQP's
// validate_data / validate_settings); flag[0] counts violations
__global__ void k_admm_validate(long long ny_total, const double *__restrict__ lb, const double *__restrict__ ub,
                                const double *__restrict__ rho, int32_t *flag) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ny_total) return;
    const double r = rho[t];
    if (!(lb[t] <= ub[t]) || !(r > 0.0 && r < 1.0e300)) atomicAdd(flag, 1);
}

// adaptive rho: every row of problem b scales by rscale[b], clamped to OSQP's
// [RHO_MIN, RHO_MAX] = [1e-6, 1e6]
__global__ void k_admm_rescale(long long ny_total, int ny, const double *__restrict__ rscale, double *__restrict__ rho,
                               double *__restrict__ irho) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ny_total) return;
    const double f = rscale[t / ny];
    if (f == 1.0) return;
    const double r = fmin(fmax(rho[t] * f, 1e-6), 1e6);
    rho[t] = r;
    irho[t] = 1.0 / r;
}

// lanes a stage of k_admm_update takes (past 64: k_admm_update_xl)
static int admm_lps(const Shape &sh) { return sh.s <= 16 ? 16 : (sh.s <= 32 ? 32 : (sh.s <= 64 ? 64 : 256)); }

static int launch_admm_update(const AdmmArgs &a, int lps, bool fuse, bool check, dim3 grid, dim3 blk,
                              hipStream_t S) {
#define PDPLQR_ADMM_LAUNCH(L, F, C) hipLaunchKernelGGL((k_admm_update<L, F, C, 0>), grid, blk, 0, S, a)
#define PDPLQR_ADMM_LAUNCH4(F, C) hipLaunchKernelGGL((k_admm_update<16, F, C, 4>), grid, blk, 0, S, a)
    const bool l16 = lps == 16;
    if (lps > 64) {  // kernels_xl.hip shapes: a wave per stage, up to 4 entries a lane
#define PDPLQR_ADMM_XL(F, C) hipLaunchKernelGGL((k_admm_update_xl<F, C, 4>), grid, blk, 0, S, a)
        if (fuse && check) PDPLQR_ADMM_XL(true, true);
        else if (fuse) PDPLQR_ADMM_XL(true, false);
        else if (check) PDPLQR_ADMM_XL(false, true);
        else PDPLQR_ADMM_XL(false, false);
#undef PDPLQR_ADMM_XL
    } else if (l16 && a.max_nc <= 4) {
        if (fuse && check) PDPLQR_ADMM_LAUNCH4(true, true);
        else if (fuse) PDPLQR_ADMM_LAUNCH4(true, false);
        else if (check) PDPLQR_ADMM_LAUNCH4(false, true);
        else PDPLQR_ADMM_LAUNCH4(false, false);
    } else if (l16) {
        if (fuse && check) PDPLQR_ADMM_LAUNCH(16, true, true);
        else if (fuse) PDPLQR_ADMM_LAUNCH(16, true, false);
        else if (check) PDPLQR_ADMM_LAUNCH(16, false, true);
        else PDPLQR_ADMM_LAUNCH(16, false, false);
    } else if (lps == 32) {
        if (fuse && check) PDPLQR_ADMM_LAUNCH(32, true, true);
        else if (fuse) PDPLQR_ADMM_LAUNCH(32, true, false);
        else if (check) PDPLQR_ADMM_LAUNCH(32, false, true);
        else PDPLQR_ADMM_LAUNCH(32, false, false);
    } else {
        if (fuse && check) PDPLQR_ADMM_LAUNCH(64, true, true);
        else if (fuse) PDPLQR_ADMM_LAUNCH(64, true, false);
        else if (check) PDPLQR_ADMM_LAUNCH(64, false, true);
        else PDPLQR_ADMM_LAUNCH(64, false, false);
    }
#undef PDPLQR_ADMM_LAUNCH
#undef PDPLQR_ADMM_LAUNCH4
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
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
        (rc = aalloc(h, &s->rho, Y)) || (rc = aalloc(h, &s->irho, Y)) ||
        (rc = aalloc(h, &s->x0, B * sh.n)) || (rc = aalloc(h, &s->prim, B)) || (rc = aalloc(h, &s->dual, B)) ||
        (rc = aalloc(h, &s->done, B)) || (rc = aalloc(h, &s->iters, B)) ||
        (rc = aalloc(h, &s->conv, B)) || (rc = aalloc(h, &s->active, 2)) || (rc = aalloc(h, &s->rscale, B)))
        return rc;
    PDPLQR_HIP_TRY(hipHostMalloc((void **)&s->active_h, 2 * sizeof(int32_t), hipHostMallocDefault));
    return PDPLQR_OK;
}

void admm_release(pdplqr_handle h) {
    if (!h->admm) return;
    if (h->admm->active_h) (void)hipHostFree(h->admm->active_h);
    delete h->admm;
    h->admm = nullptr;
}

// admm_solve on a num_devices > 1 handle (multidev.hip): the ADMM vectors and
// the update pass live on the first device; every x-update is the reference
// protocol on the slices -- update_problem_data, then backward (iteration 1 and
// after a rho change) or backward_without_factorization (its exchange is the
// slices' (f, p) only), then forward -- with device pointers on the first
// device (the slices copy their rows peer-to-peer).  The update pass is
// k_admm_update (the unfused form: h~, g are re-formed by the next
// update_problem_data on the slices).
static int md_admm_solve(pdplqr_handle h, const pdplqr_admm_settings *st, const double *x0, const double *lb,
                         const double *ub, const double *rho, double *ws, double *ys, double *zs, int mem) {
    const Shape &sh = h->sh;
    const int dev0 = md_primary_device(h);
    hipStream_t S = reinterpret_cast<hipStream_t>(md_stream(h));
    PDPLQR_HIP_TRY(hipSetDevice(dev0));
    int rc = admm_alloc(h);
    if (rc) return rc;
    AdmmState *s = h->admm;
    const long long B = sh.batch, W = B * sh.perh, Y = B * sh.ny;
    const hipMemcpyKind kin = mem == PDPLQR_MEM_DEVICE ? hipMemcpyDefault : hipMemcpyHostToDevice;
    if (mem == PDPLQR_MEM_DEVICE) PDPLQR_HIP_TRY(hipDeviceSynchronize());  // inputs made on another stream
    PDPLQR_HIP_TRY(hipMemcpyAsync(s->w, ws, W * sizeof(double), kin, S));
    PDPLQR_HIP_TRY(hipMemcpyAsync(s->x0, x0, B * sh.n * sizeof(double), kin, S));
    if (Y > 0) {
        PDPLQR_HIP_TRY(hipMemcpyAsync(s->y, ys, Y * sizeof(double), kin, S));
        PDPLQR_HIP_TRY(hipMemcpyAsync(s->z, zs, Y * sizeof(double), kin, S));
        PDPLQR_HIP_TRY(hipMemcpyAsync(s->lb, lb, Y * sizeof(double), kin, S));
        PDPLQR_HIP_TRY(hipMemcpyAsync(s->ub, ub, Y * sizeof(double), kin, S));
        PDPLQR_HIP_TRY(hipMemcpyAsync(s->rho, rho, Y * sizeof(double), kin, S));
        PDPLQR_HIP_TRY(hipMemsetAsync(s->active, 0, 2 * sizeof(int32_t), S));
        hipLaunchKernelGGL(k_admm_validate, dim3((unsigned)((Y + 255) / 256)), dim3(256), 0, S, Y, s->lb, s->ub,
                           s->rho, s->active);
        hipLaunchKernelGGL(k_admm_init, dim3((unsigned)((Y + 255) / 256)), dim3(256), 0, S, Y, s->rho, s->irho);
        PDPLQR_HIP_TRY(hipGetLastError());
        PDPLQR_HIP_TRY(hipMemcpyAsync(s->active_h, s->active, sizeof(int32_t), hipMemcpyDeviceToHost, S));
        PDPLQR_HIP_TRY(hipStreamSynchronize(S));
        if (s->active_h[0] != 0) {
            set_error("admm_solve: " + std::to_string(s->active_h[0]) +
                      " constraint rows with e_lb > e_ub, or rho not in (0, inf)");
            return PDPLQR_ERR_INVALID;
        }
    }
    PDPLQR_HIP_TRY(hipMemsetAsync(s->done, 0, B * sizeof(int32_t), S));
    PDPLQR_HIP_TRY(hipMemsetAsync(s->conv, 0, B * sizeof(int32_t), S));
    PDPLQR_HIP_TRY(hipMemsetAsync(s->iters, 0, B * sizeof(int32_t), S));
    PDPLQR_HIP_TRY(hipMemsetAsync(s->prim, 0, B * sizeof(double), S));
    PDPLQR_HIP_TRY(hipMemsetAsync(s->dual, 0, B * sizeof(double), S));
    PDPLQR_HIP_TRY(hipStreamSynchronize(S));
    AdmmArgs a;
    a.sh = sh;
    md_admm_view(h, &a.D, &a.d_off, &a.y_off);
    a.hv = nullptr;  // (unfused: h~ and g are re-formed by update_problem_data)
    a.hw = a.gw = nullptr;
    a.wt = s->wt;
    a.lb = s->lb;
    a.ub = s->ub;
    a.rho = s->rho;
    a.irho = s->irho;
    a.w = s->w;
    a.y = s->y;
    a.z = s->z;
    a.done = s->done;
    a.iters = s->iters;
    a.conv = s->conv;
    a.active = s->active;
    a.prim = s->prim;
    a.dual = s->dual;
    a.rscale = s->rscale;
    a.adaptive = st->adaptive_rho ? 1 : 0;
    a.rho_tol = st->adaptive_rho_tolerance;
    a.alpha = st->alpha;
    a.sigma = st->sigma;
    a.eps_abs = st->eps_abs;
    a.eps_rel = st->eps_rel;
    a.max_nc = h->max_nc;
    a.no_penalty = 0;
    {
        const int c0 = sh.N > 0 ? h->ncs[0] : 0;
        bool uni = c0 > 0 && h->ncs[sh.N] == 0;
        for (int k = 0; k < sh.N && uni; ++k) uni = h->ncs[k] == c0;
        a.uni = uni ? c0 : 0;
    }
    const dim3 ugrid((unsigned)B), ublk(256);
    const double *irho_or_null = Y > 0 ? s->irho : nullptr;
    int it = 1, rho_updates = 0;
    bool refactor = true;
    for (;; ++it) {
        if ((rc = md_update(h, s->w, Y > 0 ? s->y : nullptr, Y > 0 ? s->z : nullptr, irho_or_null, st->sigma,
                            PDPLQR_MEM_DEVICE)))
            return rc;
        h->updated = true;
        if ((rc = md_backward(h, Y > 0 ? s->rho : nullptr, PDPLQR_MEM_DEVICE, refactor))) return rc;
        h->factored = true;
        refactor = false;
        if ((rc = md_forward(h, s->x0, s->wt, PDPLQR_MEM_DEVICE))) return rc;  // (returns with the slices drained)
        PDPLQR_HIP_TRY(hipSetDevice(dev0));
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
        a.it = it;
        if (check) PDPLQR_HIP_TRY(hipMemsetAsync(s->active, 0, 2 * sizeof(int32_t), S));
        if ((rc = launch_admm_update(a, admm_lps(sh), false, check, ugrid, ublk, S)))
            return rc;
        if (check) {
            PDPLQR_HIP_TRY(hipMemcpyAsync(s->active_h, s->active, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, S));
            PDPLQR_HIP_TRY(hipStreamSynchronize(S));
            if (s->active_h[0] == 0) break;
            if (s->active_h[1] && !last) {
                hipLaunchKernelGGL(k_admm_rescale, dim3((unsigned)((Y + 255) / 256)), dim3(256), 0, S, Y, sh.ny,
                                   s->rscale, s->rho, s->irho);
                PDPLQR_HIP_TRY(hipGetLastError());
                refactor = true;
                ++rho_updates;
            }
        }
        if (last) break;
        PDPLQR_HIP_TRY(hipStreamSynchronize(S));  // the next update reads w, y, z on the slices' streams
    }
    const hipMemcpyKind kout = mem == PDPLQR_MEM_DEVICE ? hipMemcpyDefault : hipMemcpyDeviceToHost;
    PDPLQR_HIP_TRY(hipMemcpyAsync(ws, s->w, W * sizeof(double), kout, S));
    if (Y > 0) {
        PDPLQR_HIP_TRY(hipMemcpyAsync(ys, s->y, Y * sizeof(double), kout, S));
        PDPLQR_HIP_TRY(hipMemcpyAsync(zs, s->z, Y * sizeof(double), kout, S));
    }
    PDPLQR_HIP_TRY(hipStreamSynchronize(S));
    h->admm_iters = it;
    h->admm_rho_updates = rho_updates;
    return PDPLQR_OK;
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
    s->adaptive_rho = 1;
    s->adaptive_rho_tolerance = 5.0;  // OSQP defaults
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
        !(st->eps_abs >= 0.0) || !(st->eps_rel >= 0.0) || (st->adaptive_rho && !(st->adaptive_rho_tolerance >= 1.0))) {
        set_error("admm_solve: bad settings (max_iter >= 1, check_every >= 1, 0 < alpha < 2, sigma, eps >= 0, "
                  "adaptive_rho_tolerance >= 1)");
        return PDPLQR_ERR_INVALID;
    }
    if (h->md) return md_admm_solve(h, st, x0, lb, ub, rho, ws, ys, zs, mem);
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
        PDPLQR_HIP_TRY(hipMemsetAsync(s->active, 0, 2 * sizeof(int32_t), S));
        hipLaunchKernelGGL(k_admm_validate, dim3((unsigned)((Y + 255) / 256)), dim3(256), 0, S, Y, s->lb, s->ub,
                           s->rho, s->active);
        hipLaunchKernelGGL(k_admm_init, dim3((unsigned)((Y + 255) / 256)), dim3(256), 0, S, Y, s->rho, s->irho);
        PDPLQR_HIP_TRY(hipGetLastError());
        PDPLQR_HIP_TRY(hipMemcpyAsync(s->active_h, s->active, sizeof(int32_t), hipMemcpyDeviceToHost, S));
        PDPLQR_HIP_TRY(hipStreamSynchronize(S));
        if (s->active_h[0] != 0) {
            set_error("admm_solve: " + std::to_string(s->active_h[0]) +
                      " constraint rows with e_lb > e_ub, or rho not in (0, inf)");
            return PDPLQR_ERR_INVALID;
        }
    }
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
    a.hw = h->hw;
    a.gw = h->gw;
    a.d_off = h->d_off;
    a.y_off = h->y_off;
    a.done = s->done;
    a.iters = s->iters;
    a.conv = s->conv;
    a.active = s->active;
    a.prim = s->prim;
    a.dual = s->dual;
    a.rscale = s->rscale;
    a.adaptive = st->adaptive_rho ? 1 : 0;
    a.rho_tol = st->adaptive_rho_tolerance;
    a.alpha = st->alpha;
    a.sigma = st->sigma;
    a.eps_abs = st->eps_abs;
    a.eps_rel = st->eps_rel;
    a.max_nc = h->max_nc;
    a.it = 0;
    // KKT with the factor cache: the update pass also forms the next h~ = h - sigma w
    // and g (the KKT path takes rho through g in its backward, no penalty in h~)
    const bool kkt_lin = kkt && kkt_linear_supported(h);
    a.no_penalty = kkt ? 1 : 0;
    {
        const int c0 = sh.N > 0 ? h->ncs[0] : 0;
        bool uni = c0 > 0 && h->ncs[sh.N] == 0;
        for (int k = 0; k < sh.N && uni; ++k) uni = h->ncs[k] == c0;
        a.uni = uni ? c0 : 0;
    }
    const dim3 ugrid((unsigned)B), ublk(256);
    const double *irho_or_null = Y > 0 ? s->irho : nullptr;
    int it = 1;
    bool refactor = true;  // iteration 1, and after an adaptive rho change
    bool fused = false;    // this iteration's backward already ran inside the fused update
    bool can_fuse = !kkt && Y > 0 && h->Lc != nullptr;  // cleared when the fused kernel does not apply
    // KKT (Riccati-ordered 12/4, C5 rows): rollout + update fused (cleared when it does not apply)
    bool can_fuse_kkt = kkt && kkt_ric_active(h) && a.uni == 4;
    int rho_updates = 0;
    for (;; ++it) {
        // x-update: the reference protocol (iteration 1 and after a rho
        // change: H~ depends on rho), then vectors only
        if (refactor || (kkt && !kkt_lin)) {
            if ((rc = solver_update(h, s->w, s->y, s->z, irho_or_null, st->sigma))) return rc;
            h->updated = true;
        } else if (kkt_lin) {
            // h~, g came from the previous update pass; the x0 sum of the KKT
            // right-hand side restarts as update_problem_data would restart it
            if ((rc = kkt_rhs_restart(h))) return rc;
        }
        // the Riccati-ordered KKT path folds the right-hand side into its
        // elimination (kkt_riccati.hip): with a factor cache (12/4) the later
        // iterations run only its right-hand-side pass, else the whole backward
        if (kkt_lin) {
            if ((rc = refactor ? kkt_backward_cached(h, s->irho) : kkt_backward_linear(h, s->irho))) return rc;
            h->factored = true;
            refactor = false;
        } else if (refactor || (kkt && kkt_ric_active(h))) {
            if ((rc = solver_backward(h, kkt ? s->irho : s->rho))) return rc;
            h->factored = true;
            refactor = false;
        } else if (!kkt && !fused) {
            if ((rc = solver_backward_prepared(h))) return rc;
        }
        fused = false;
        const bool last = it >= st->max_iter;
        const bool check = last || it % st->check_every == 0;
        const bool fuse = (!kkt || kkt_lin) && !last;
        a.it = it;
        if (kkt && Y > 0 && can_fuse_kkt) {
            // the KKT rollout and this iteration's update in one pass (kkt_riccati.hip)
            if (check) PDPLQR_HIP_TRY(hipMemsetAsync(s->active, 0, 2 * sizeof(int32_t), S));
            rc = kkt_forward_admm(h, s->x0, a, fuse, check);
            if (rc == PDPLQR_OK) {
                if (check) {
                    PDPLQR_HIP_TRY(hipMemcpyAsync(s->active_h, s->active, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, S));
                    PDPLQR_HIP_TRY(hipStreamSynchronize(S));
                    if (s->active_h[0] == 0) break;
                    if (s->active_h[1] && !last) {
                        hipLaunchKernelGGL(k_admm_rescale, dim3((unsigned)((Y + 255) / 256)), dim3(256), 0, S, Y, sh.ny,
                                           s->rscale, s->rho, s->irho);
                        PDPLQR_HIP_TRY(hipGetLastError());
                        refactor = true;
                        ++rho_updates;
                    }
                }
                if (last) break;
                continue;
            }
            if (rc != PDPLQR_ERR_UNSUPPORTED) return rc;
            can_fuse_kkt = false;
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
        if (check) PDPLQR_HIP_TRY(hipMemsetAsync(s->active, 0, 2 * sizeof(int32_t), S));
        if (fuse && can_fuse) {
            // the update of this iteration and the backward_without_factorization
            // of the next in one streamed pass (kernels_nofact.hip)
            rc = solver_nofact_admm(h, a, check);
            if (rc == PDPLQR_OK) fused = true;
            else if (rc == PDPLQR_ERR_UNSUPPORTED) can_fuse = false;
            else return rc;
        }
        if (!fused && (rc = launch_admm_update(a, admm_lps(sh), fuse, check, ugrid, ublk, S))) return rc;
        if (check) {
            PDPLQR_HIP_TRY(hipMemcpyAsync(s->active_h, s->active, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, S));
            PDPLQR_HIP_TRY(hipStreamSynchronize(S));
            if (s->active_h[0] == 0) break;
            if (s->active_h[1] && !last) {  // some problem's rho moved: rescale, refactor the batch
                hipLaunchKernelGGL(k_admm_rescale, dim3((unsigned)((Y + 255) / 256)), dim3(256), 0, S, Y, sh.ny,
                                   s->rscale, s->rho, s->irho);
                PDPLQR_HIP_TRY(hipGetLastError());
                refactor = true;
                fused = false;  // the fused backward used the old rho: refactor instead
                ++rho_updates;
            }
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
    h->admm_rho_updates = rho_updates;
    return PDPLQR_OK;
}

int pdplqr_admm_info(pdplqr_handle h, int32_t *iters, int32_t *converged, double *prim_res, double *dual_res,
                     double *rho) {
    if (!h) return PDPLQR_ERR_INVALID;
    if (!h->admm) {
        set_error("admm_info before admm_solve");
        return PDPLQR_ERR_STATE;
    }
    PDPLQR_HIP_TRY(hipSetDevice(h->md ? md_primary_device(h) : h->cfg.device));
    PDPLQR_HIP_TRY(hipStreamSynchronize(h->md ? reinterpret_cast<hipStream_t>(md_stream(h)) : h->stream));
    AdmmState *s = h->admm;
    const size_t B = (size_t)h->sh.batch;
    if (iters) PDPLQR_HIP_TRY(hipMemcpy(iters, s->iters, B * sizeof(int32_t), hipMemcpyDeviceToHost));
    if (converged) PDPLQR_HIP_TRY(hipMemcpy(converged, s->conv, B * sizeof(int32_t), hipMemcpyDeviceToHost));
    if (prim_res) PDPLQR_HIP_TRY(hipMemcpy(prim_res, s->prim, B * sizeof(double), hipMemcpyDeviceToHost));
    if (dual_res) PDPLQR_HIP_TRY(hipMemcpy(dual_res, s->dual, B * sizeof(double), hipMemcpyDeviceToHost));
    if (rho && h->sh.ny > 0)
        PDPLQR_HIP_TRY(hipMemcpy(rho, s->rho, B * h->sh.ny * sizeof(double), hipMemcpyDeviceToHost));
    return h->admm_iters;
}

}  // extern "C"
