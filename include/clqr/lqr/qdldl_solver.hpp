// clqr/lqr/qdldl_solver.hpp -- KKT + LDL^T solver facade (MI355X).
//
// Public surface of the reference's QDLDLSolver
// (include/clqr/lqr/qdldl_solver.hpp:14-151).  The KKT matrix of kkt.hpp is
// formed once, at construction, with rho_dyn = sigma = 1e-6; backward takes
// the INVERSE rho vectors and refactors; forward adds -S0 x0, -A0 x0 to the
// stored right-hand side (accumulating, as kkt.hpp:207-222) and solves.  The
// factorisation is libpdplqr's block LDL^T in QDLDL's elimination order
// (csrc/kkt.hip), not the QDLDL library.
#pragma once

#include <stdexcept>
#include <vector>

#include "clqr/detail/bridge.hpp"
#include "clqr/lqr/kkt.hpp"

namespace lqr {

class QDLDLSolver {
public:
    explicit QDLDLSolver(const LQRModel &model)
        : model_(model), hd_(model, PDPLQR_SOLVER_KKT, 1, true, PDPLQR_CONDENSED_CHOLESKY, false) {
        hd_.upload(model_);  // forms the KKT system (the reference's constructor)
    }

    void update_problem_data(const std::vector<VectorXs> &ws, const std::vector<VectorXs> &ys,
                             const std::vector<VectorXs> &zs, const std::vector<VectorXs> &inv_rho_vecs,
                             const scalar sigma) {
        hd_.sync(model_, PDPLQR_MODEL_HV | PDPLQR_MODEL_C);  // form_rhs reads h, c; the matrix stays frozen
        hd_.update(ws, ys, zs, inv_rho_vecs, sigma);
    }

    void backward(const std::vector<VectorXs> &inv_rho_vecs) {
        hd_.backward(inv_rho_vecs, true);
        if (hd_.status() != 0)
            throw std::runtime_error("QDLDL factorization failed with status: " + std::to_string(hd_.status()));
    }

    // update_rhs_initial_stage reads S0 (H) and A0 (E) of the current model (kkt.hpp:207-222)
    void forward(const VectorXs &x0, std::vector<VectorXs> &ws) {
        hd_.sync(model_, PDPLQR_MODEL_E | PDPLQR_MODEL_H);
        hd_.forward(x0, ws);
    }

    long long model_upload_bytes() const { return hd_.upload_bytes(); }

    // this build: model change tracking.  On (default), every protocol call
    // compares the model arrays it reads with what the device holds (host work
    // O(N s^2), no copy when unchanged).  Off, the calls skip that compare and
    // the caller declares edits: model_changed(PDPLQR_MODEL_E | ...) before the
    // call that should read them (detail::Handle::sync).
    void set_model_tracking(bool on) { hd_.set_tracking(on); }
    void model_changed(int mask = PDPLQR_MODEL_ALL) { hd_.model_changed(mask); }

    // qdldl_solver.hpp:19,47-78: the QDLDL workspace (elimination tree, column
    // counts, factor buffers) of a KKT matrix, e.g. KKTSystem::get_KKT_csc_matrix's.
    // Host-side; the GPU factorisation does not use it.
    std::unique_ptr<QDLDLData> create_workspace(const CscMatrix &Kkt) { return detail::create_qdldl_workspace(Kkt); }

private:
    const LQRModel &model_;
    detail::Handle hd_;
};

}  // namespace lqr
