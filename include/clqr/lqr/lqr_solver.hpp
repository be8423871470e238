// clqr/lqr/lqr_solver.hpp -- serial Riccati solver facade (MI355X).
//
// Public surface of the reference's LQRSolver (include/clqr/lqr/lqr_solver.hpp:9-77):
// update_problem_data -> backward -> forward, plus backward_without_factorization
// and clear_workspace.  Every call forwards to libpdplqr's C ABI; the backward
// and the rollout run as HIP kernels on the GPU (no host arithmetic here).
// The model is borrowed, as in the reference, and read lazily as the reference
// reads it: H, h at update_problem_data, E, c, D_con at backward / forward
// (only arrays that changed are re-uploaded: detail::Handle::sync).
#pragma once

#include <vector>

#include "clqr/detail/bridge.hpp"

namespace lqr {

class LQRSolver {
public:
    explicit LQRSolver(const LQRModel &model)
        : model_(model), hd_(model, PDPLQR_SOLVER_SERIAL, 1, true, PDPLQR_CONDENSED_CHOLESKY, true) {
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

    // this build: first stage whose factorisation failed (+1), 0 if none
    int factorization_status() { return hd_.status(); }

private:
    const LQRModel &model_;
    detail::Handle hd_;
};

}  // namespace lqr
