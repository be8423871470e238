// clqr/lqr/lqr_solver.hpp -- serial Riccati solver facade (MI355X).
//
// Public surface of the reference's LQRSolver (include/clqr/lqr/lqr_solver.hpp:9-77):
// update_problem_data -> backward -> forward, plus backward_without_factorization
// and clear_workspace.  Every call forwards to libpdplqr's C ABI; the backward
// and the rollout run as HIP kernels on the GPU (no host arithmetic here).
// The model is borrowed, as in the reference, and re-read on every
// update_problem_data.
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
        hd_.upload(model_);
        hd_.update(ws, ys, zs, inv_rho_vecs, sigma);
    }

    void backward(const std::vector<VectorXs> &rho_vecs) { hd_.backward(rho_vecs, true); }
    void backward_without_factorization(const std::vector<VectorXs> &rho_vecs) { hd_.backward(rho_vecs, false); }
    void forward(const VectorXs &x0, std::vector<VectorXs> &ws) { hd_.forward(x0, ws); }
    void clear_workspace() { hd_.clear(); }

    // this build: first stage whose factorisation failed (+1), 0 if none
    int factorization_status() { return hd_.status(); }

private:
    const LQRModel &model_;
    detail::Handle hd_;
};

}  // namespace lqr
