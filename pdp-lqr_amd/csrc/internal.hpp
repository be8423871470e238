// internal.hpp -- shared declarations of libpdplqr (MI355X / gfx950, HIP).
//
// Device data layout (HBM), per handle.  Model arrays keep the boundary's
// reference layout (include/pdplqr.h); the workspace is solver-owned:
//   Hw  [b][N*ps + pn]   H~_k = H_k + sigma I (+ rho D^T D), packed lower, column-major
//   hw  [b][N*s + n]     h~_k = h_k - sigma w_k (- D^T rho g)
//   gw  [b][ny]          g_k = z_k - inv_rho o y_k
//   KD  [b][N][s*m + m]  rollout record FR_k = [L_k(:, 0:m) | lu'_k], lu' = Luu^{-1} lu
//   Lc  [b][N*ps + pn]   (keep_factors) Cholesky factor L_k, packed lower
//   lpc [b][N*s + n]     (keep_factors) lp_k = [lu; p]
// with ps = s(s+1)/2 and pn = n(n+1)/2.  One wavefront owns one problem in the
// batched serial kernels (see DESIGN.md for the per-kernel roofline).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <type_traits>
#include <vector>

#include "pdplqr.h"

namespace pdplqr {

void set_error(const std::string &msg);

#define PDPLQR_HIP_TRY(expr)                                                                        \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess) {                                                                     \
            ::pdplqr::set_error(std::string(#expr) + ": " + hipGetErrorString(e_));                 \
            return PDPLQR_ERR_HIP;                                                                  \
        }                                                                                           \
    } while (0)

struct Shape {
    int n, m, N, batch;
    int s, ps, pn;      // s = n + m, packed sizes
    int ny;             // sum_k nc_k
    int ndD;            // sum_k nc_k * dim_k
    long long perE, perc, perH, perh, perHw, perKD;
    int mw = 1;  // PARALLEL: the 4-wave horizon kernels may run (parallel_init's family choice)
    // the batch fits the device's SIMDs once: the one-wave-per-problem kernels
    // launch their one-wave-per-SIMD instance (simd_exclusive, device_common.hpp)
    int x1 = 0;
};

// f(std::true_type{}) or f(std::false_type{}): a launcher's generic lambda picks
// the X1 instance of its kernel from Shape::x1
template <typename F>
inline void with_x1(int x1, F &&f) {
    if (x1) f(std::true_type{});
    else f(std::false_type{});
}
int device_simds(int device);  // SIMDs of the device (4 per CU)
bool one_wave_per_simd(int device, long long waves);  // waves <= SIMDs (PDPLQR_NO_X1: never)

// Riccati (serial, batched) kernels: kernels_riccati.hip
struct RiccatiArgs {
    Shape sh;
    const double *E, *c;   // model
    double *Hw, *hw;       // workspace (read by the backward)
    double *KD;            // out: rollout records
    double *Lc, *lpc;      // factor cache (nullable)
    int32_t *status;       // per-problem factorization status
    const short2 *tab_s;   // packed-lower index tables (i, j)
    const short2 *tab_n;
    // rho penalty fused into the streamed backward (launch_riccati_backward_pen):
    // D, rho, g of a uniform nc rows per stage (k < N), nc_last at the terminal
    const double *D = nullptr, *rho = nullptr, *gw = nullptr;
    const int32_t *d_off = nullptr, *y_off = nullptr;
    int nc_last = 0;
    double *xl_ws = nullptr;  // 64 < n + m <= 256: per-problem workspace of kernels_xl.hip
};
bool xl_shape(const Shape &sh);           // 64 < n + m <= 256 (kernels_xl.hip)
// workspace doubles per problem: V (s x n), two s x s factor buffers and the
// factorisation's input
__host__ __device__ inline long long xl_ws_doubles(const Shape &sh) {
    return (long long)sh.s * sh.n + 3LL * sh.s * sh.s;
}
// KKT_RIC_XL (kernels_xl.hip k_kkt_ric_bwd_xl): XA (n x s), Pt, T0 (n x n), Mb (s x s)
__host__ __device__ inline long long kkt_xl_ws_doubles(const Shape &sh) {
    return (long long)sh.n * sh.s + 2LL * sh.n * sh.n + (long long)sh.s * sh.s;
}

int launch_riccati_backward_xl(const RiccatiArgs &a, hipStream_t st);
int launch_riccati_backward_nofact_xl(const RiccatiArgs &a, hipStream_t st);
int launch_riccati_forward_xl(const Shape &sh, const double *E, const double *c, const double *FR, const double *x0,
                              double *ws, hipStream_t st);

int launch_update_problem_data(const Shape &sh, const double *H, const double *hv, const double *ws,
                               const double *ys, const double *zs, const double *irho, double sigma, double *Hw,
                               double *hw, double *gw, const short2 *tab_s, const short2 *tab_n,
                               hipStream_t st, bool skipH = false);
int launch_penalty(const Shape &sh, const double *D, const double *rho, const double *gw, double *Hw,
                   double *hw, const int32_t *d_off, const int32_t *y_off, const short2 *tab_s,
                   const short2 *tab_n, int with_H, int max_nc, hipStream_t st);
int launch_riccati_backward(const RiccatiArgs &a, hipStream_t st);
int launch_riccati_backward_schur(const RiccatiArgs &a, hipStream_t st);  // ERR_UNSUPPORTED: not applicable
// the rho penalty (lqr_kernel.hpp:82-88,106-112) fused into the 12/4 value-form
// backward, H~ / h~ penalised in place as the reference does; ERR_UNSUPPORTED
// when the shape / row layout needs k_penalty + the plain backward
int launch_riccati_backward_pen(const RiccatiArgs &a, int nc, hipStream_t st);
bool schur_gain_record(const RiccatiArgs &a);  // the backward leaves the gain-form record [K~ | k~]
int launch_rollout_dma(const Shape &sh, const double *E, const double *c, const double *FR, const double *x0,
                       double *ws, hipStream_t st, bool gain = false);  // ERR_UNSUPPORTED: not applicable
int launch_riccati_backward_nofact(const RiccatiArgs &a, hipStream_t st);
// 32 < n + m <= 64 (kernels_big.hip): serial backward with factorization, forward
bool big_shape(const Shape &sh);
int launch_riccati_backward_big(const RiccatiArgs &a, hipStream_t st);
int launch_riccati_forward_big(const Shape &sh, const double *E, const double *c, const double *FR, const double *x0,
                               double *ws, hipStream_t st);
int launch_nofact_dma(const RiccatiArgs &a, hipStream_t st);  // ERR_UNSUPPORTED: not applicable
int launch_riccati_forward(const Shape &sh, const double *E, const double *c, const double *KD, const double *x0,
                           double *ws, hipStream_t st);

}  // namespace pdplqr

namespace pdplqr { struct ParallelState;
struct KKTState;
struct AdmmState;
struct MultiDev;
// one slice of a num_devices split (multidev.hip)
struct MdSlice {
    int N0 = 0, N1 = 0;          // stages [N0, N1)
    bool last = false;           // holds the real terminal
    long long y0 = 0, ny_st = 0; // constraint rows of the slice's stages in the full y vector
    int nc_term = 0;             // rows of the slice's terminal (the last slice: nc_N)
    long long d0 = 0, nd_st = 0; // D entries of the slice's stages in the full D array
    std::vector<int32_t> ncs;    // the slice handle's ncs (N1 - N0 + 1)
};
void md_plan(int N, int R, const std::vector<int32_t> &ncs, int n, int m, std::vector<MdSlice> &out);
}

struct pdplqr_handle_s {
    pdplqr_config cfg;
    std::vector<int32_t> ncs;
    std::vector<int32_t> d_off_h, y_off_h;
    pdplqr::Shape sh;
    int max_nc;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    // model
    double *E = nullptr, *c = nullptr, *H = nullptr, *h = nullptr, *D = nullptr;
    // workspace
    double *Hw = nullptr, *hw = nullptr, *gw = nullptr;
    double *KD = nullptr, *Lc = nullptr, *lpc = nullptr;
    double *xl_ws = nullptr;  // SERIAL, 64 < n + m <= 256 (kernels_xl.hip)
    // H~ = H + sigma I (Hw) depends only on the model and sigma when no stage
    // has constraints (no rho penalty is folded into Hw): kept across
    // update_problem_data calls with the same sigma, re-formed after set_model
    // or clear_workspace
    bool hw_cached = false;
    // the last backward left the gain-form rollout record: the serial path's
    // [K~|k~] (schur_gain_record) or the KKT path's E^ record (kkt_ric_rec_ehat;
    // a cache-writing ADMM backward leaves the P~ record, rec_gain false)
    bool rec_gain = false;
    bool graph_rec_gain = false;  // record form the captured forward graph reads
    double hw_sigma = 0.0;
    int32_t *status = nullptr;
    int32_t *d_off = nullptr, *y_off = nullptr;
    short2 *tab_s = nullptr, *tab_n = nullptr;
    // staging for host inputs / outputs
    double *st_ws = nullptr, *st_y = nullptr, *st_z = nullptr, *st_ir = nullptr, *st_rho = nullptr;
    double *st_x0 = nullptr;
    bool model_set = false, updated = false, factored = false;
    long long model_upload_bytes = 0;  // host -> device model bytes (pdplqr_get_model_upload_bytes)
    bool host_staged = false;  // a host->device copy is in flight on `stream`
    std::vector<void *> allocs;
    pdplqr::ParallelState *par = nullptr;  // PARALLEL solver state (solvers.hip)
    pdplqr::KKTState *kkt = nullptr;       // KKT solver state (kkt.hip)
    pdplqr::AdmmState *admm = nullptr;     // ADMM outer loop state (admm.hip), allocated on first use
    int admm_iters = 0;                    // iterations of the last admm_solve
    int admm_rho_updates = 0;              // adaptive-rho refactorizations of the last admm_solve
    int shard_last = 1;  // last shard_backward's is_last_shard
    pdplqr::MultiDev *md = nullptr;  // num_devices > 1 (multidev.hip): the slices' handles
    // replayable launch sequences of backward / backward_without_factorization /
    // forward (solvers.hip: hipGraph captured on first use per argument set)
    struct Graph {
        hipGraphExec_t exec = nullptr;
        const void *k1 = nullptr, *k2 = nullptr;
        hipStream_t stream = nullptr;
    } graphs[3];
};
