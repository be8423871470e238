// clqr/lqr/lqr_solver_parallel.hpp -- parallel (segmented) Riccati facade (MI355X).
//
// Public surface of the reference's LQRParallelSolver
// (include/clqr/lqr/lqr_solver_parallel.hpp:19-238): the horizon is cut into
// num_segments segments (alpha = 1.55 with load_balancing), each segment is
// summarised as an element (F, C, f, P, p) and the segments are coupled by the
// condensed system.  On the GPU every reference segment is further split into
// sub-segments and the condensed system becomes an associative prefix/suffix
// scan; CondensedSystemSolverType is accepted and validated as in the
// reference.  The OpenMP team / core pinning of the reference has no analogue;
// its multi-core split becomes the optional multi-GPU split (`devices`).
#pragma once

#include <stdexcept>
#include <vector>

#include "clqr/detail/bridge.hpp"

namespace lqr {

enum class CondensedSystemSolverType { LU = PDPLQR_CONDENSED_LU, CHOLESKY = PDPLQR_CONDENSED_CHOLESKY };

class LQRParallelSolver {
public:
    LQRParallelSolver(const LQRModel &model, int num_segments, bool load_balancing = true,
                      CondensedSystemSolverType solver_type = CondensedSystemSolverType::CHOLESKY)
        : LQRParallelSolver(model, num_segments, load_balancing, solver_type, std::vector<int>{}) {}

    // MI355X extension: `devices` (HIP ordinals) splits the horizon into one
    // slice per GPU, driven by this one object -- slice backward on every device,
    // one RCCL all-gather of the slice elements, slice forward (pdplqr.h
    // num_devices; backward_without_factorization exchanges only the slices'
    // (f, p), lqr_solver_parallel.hpp:207-210).
    LQRParallelSolver(const LQRModel &model, int num_segments, bool load_balancing,
                      CondensedSystemSolverType solver_type, const std::vector<int> &devices)
        : model_(model),
          hd_(model, PDPLQR_SOLVER_PARALLEL, num_segments, load_balancing, static_cast<int>(solver_type), true,
              devices),
          num_segments_(num_segments) {
        hd_.upload(model_);
    }

    void update_problem_data(const std::vector<VectorXs> &ws, const std::vector<VectorXs> &ys,
                             const std::vector<VectorXs> &zs, const std::vector<VectorXs> &inv_rho_vecs,
                             const scalar sigma) {
        hd_.sync(model_, PDPLQR_MODEL_H | PDPLQR_MODEL_HV);  // copied into the workspace here (lqr_solver.hpp:41-56)
        hd_.update(ws, ys, zs, inv_rho_vecs, sigma);
    }

    // E, c, D_con are read when the kernels run (lqr_kernel.hpp:106-119,186-188)
    void backward(const std::vector<VectorXs> &rho_vecs) {
        hd_.sync(model_, PDPLQR_MODEL_E | PDPLQR_MODEL_C | PDPLQR_MODEL_D);
        hd_.backward(rho_vecs, true);
    }
    void backward_without_factorization(const std::vector<VectorXs> &rho_vecs) {
        hd_.sync(model_, PDPLQR_MODEL_E | PDPLQR_MODEL_C | PDPLQR_MODEL_D);
        hd_.backward(rho_vecs, false);
    }
    void forward(const VectorXs &x0, std::vector<VectorXs> &ws) {
        hd_.sync(model_, PDPLQR_MODEL_E | PDPLQR_MODEL_C);
        hd_.forward(x0, ws);
    }
    void clear_workspace() { hd_.clear(); }

    // this build: model bytes uploaded host -> device so far (a loop over an
    // unchanged model uploads nothing after the constructor)
    long long model_upload_bytes() const { return hd_.upload_bytes(); }

    // this build: model change tracking.  On (default), every protocol call
    // compares the model arrays it reads with what the device holds (host work
    // O(N s^2), no copy when unchanged).  Off, the calls skip that compare and
    // the caller declares edits: model_changed(PDPLQR_MODEL_E | ...) before the
    // call that should read them (detail::Handle::sync).
    void set_model_tracking(bool on) { hd_.set_tracking(on); }
    void model_changed(int mask = PDPLQR_MODEL_ALL) { hd_.model_changed(mask); }

    int num_segments() const { return num_segments_; }

    // segment boundaries of the reference segmentation (idx_start, Nseg)
    void segments(std::vector<int> &idx_start, std::vector<int> &Nseg) const {
        std::vector<int32_t> a(static_cast<size_t>(num_segments_)), b(static_cast<size_t>(num_segments_));
        detail::check(pdplqr_get_segments(hd_.raw(), a.data(), b.data()), "get_segments");
        idx_start.assign(a.begin(), a.end());
        Nseg.assign(b.begin(), b.end());
    }

private:
    const LQRModel &model_;
    detail::Handle hd_;
    int num_segments_;
};

}  // namespace lqr
