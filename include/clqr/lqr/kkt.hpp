// clqr/lqr/kkt.hpp -- the public KKT assembly of the reference (KKTSystem,
// include/clqr/lqr/kkt.hpp:7-331 there), on the host.
//
// The GPU path of QDLDLSolver never assembles this matrix: csrc/kkt.hip
// condenses the primal blocks per stage and factors the block-tridiagonal dual
// system from tile-packed blocks.  Callers of the reference that use
// KKTSystem directly -- to read the KKT matrix in CSC form or its right-hand
// side, e.g. to hand them to another sparse solver -- get the same matrix here:
//   * variable order: primal [u0, x1,u1, ..., x_{N-1},u_{N-1}, x_N], then dual
//     [y0, lambda1,y1, ..., lambdaN,yN]; within a stage k >= 1, x before u
//     (kkt.hpp:124-205);
//   * upper triangle only; H + sigma I blocks, -I / A^T / B^T dynamics blocks,
//     D^T constraint blocks; zeros of H and D are skipped (ignore_zeros) while
//     those of A, B are kept, exactly as the reference's assign_dense_matrix
//     calls (utils.hpp:10-34);
//   * regularisation diagonal: -1 placeholders on the y rows (replaced by
//     -inv_rho in update_rho_vecs, kkt.hpp:105-122), -rho_dyn on the lambda rows;
//   * CSC in Eigen's compressed order: columns ascending, rows ascending within
//     a column; get_KKT_csc_matrix's pointers stay valid until the next call.
#pragma once

#include <algorithm>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <unordered_map>
#include <vector>

#include "clqr/lqr/qdldl_typedefs.hpp"
#include "clqr/lqr_model.hpp"

namespace lqr {

class KKTSystem {
public:
    KKTSystem(int nx, int nu, int N, const std::vector<int> &ncs) : nx_(nx), nu_(nu), N_(N), ncs_(N + 1) {
        int rows = nx + nu + ncs[0];  // stage 0 (kkt.hpp:45-58)
        ncs_[0] = ncs[0];
        for (int k = 1; k < N; ++k) {
            rows += nx + nu + ncs[k] + nx;
            ncs_[k] = ncs[k];
        }
        rows += nx + ncs[N];
        ncs_[N] = ncs[N];
        dim_ = rows;
        rhs_.resize(rows);
        rhs_.setZero();
    }

    // kkt.hpp:65-75
    void fill_stage_cost_matrices(const MatrixXs &H, int nx, int nu, int row_offset, bool update,
                                  bool ignore_zeros = true) {
        // Q (upper), S^T, R (upper) of H = [R S; S^T Q]
        dense(row_offset, row_offset, H, nu, nu, nx, nx, false, update, true, ignore_zeros);
        dense(row_offset, row_offset + nx, H, nu, 0, nx, nu, false, update, false, ignore_zeros);
        dense(row_offset + nx, row_offset + nx, H, 0, 0, nu, nu, false, update, true, ignore_zeros);
    }

    // kkt.hpp:77-89
    void fill_stage_dynamics_matrices(const MatrixXs &E, int nx, int nu, int nc, int row_offset, int col_offset,
                                      bool update) {
        diag(row_offset, col_offset, -1.0, nx, update);
        dense(row_offset, col_offset + nx + nc, E, 0, nu, nx, nx, true, update, false, false);  // A^T
        dense(row_offset + nx, col_offset + nx + nc, E, 0, 0, nx, nu, true, update, false, false);  // B^T
    }

    // kkt.hpp:91-103
    void fill_stage_constraint_matrices(const MatrixXs &D_con, int nx, int nu, int nc, int row_offset,
                                        int col_offset, bool update, bool ignore_zeros = true) {
        if (nc <= 0) return;
        dense(row_offset, col_offset + nx, D_con, 0, nu, nc, nx, true, update, false, ignore_zeros);  // Dx^T
        dense(row_offset + nx, col_offset + nx, D_con, 0, 0, nc, nu, true, update, false, ignore_zeros);  // Du^T
    }

    // kkt.hpp:105-122: the y diagonal becomes -inv_rho
    void update_rho_vecs(const LQRModel &model, const std::vector<VectorXs> &inv_rho_vecs) {
        int row = N_ * (nx_ + nu_);
        for (int k = 0; k <= N_; ++k) {
            const int nc = model.get_node(k).get_constraint_dim();
            for (int i = 0; i < nc; ++i) set(row + i, row + i, -inv_rho_vecs[k](i), true);
            row += nc + nx_;
        }
    }

    // kkt.hpp:124-205
    void form_KKT_matrix(const LQRModel &model, scalar rho_dyn, scalar sigma, bool update) {
        if (!update) entries_.clear();
        const int nx = nx_, nu = nu_, nxu = nx + nu, N = N_;
        int row = 0, col = N * nxu;
        {  // stage 0: R0, Du0^T, B0^T
            const Node &kp = model.get_node(0);
            const int nc = kp.get_constraint_dim();
            MatrixXs H0 = kp.H;
            for (int i = 0; i < nxu; ++i) H0(i, i) += sigma;
            dense(row, row, H0, 0, 0, nu, nu, false, update, true, true);
            if (nc > 0) dense(row, col, kp.D_con, 0, 0, nc, nu, true, update, false, true);
            dense(row, col + nc, kp.E, 0, 0, nx, nu, true, update, false, false);
            row += nu;
            col += nc;
        }
        for (int k = 1; k < N; ++k) {
            const Node &kp = model.get_node(k);
            const int nc = kp.get_constraint_dim();
            MatrixXs Hk = kp.H;
            for (int i = 0; i < nxu; ++i) Hk(i, i) += sigma;
            fill_stage_cost_matrices(Hk, nx, nu, row, update);
            fill_stage_dynamics_matrices(kp.E, nx, nu, nc, row, col, update);
            fill_stage_constraint_matrices(kp.D_con, nx, nu, nc, row, col, update);
            row += nxu;
            col += nc + nx;
        }
        {  // terminal: Q_N (upper), -I, D_N^T
            const Node &kp = model.get_node(N);
            const int nc = kp.get_constraint_dim();
            MatrixXs HN = kp.H;
            for (int i = 0; i < nx; ++i) HN(i, i) += sigma;
            dense(row, row, HN, 0, 0, nx, nx, false, update, true, true);
            diag(row, col, -1.0, nx, update);
            if (nc > 0) dense(row, col + nx, kp.D_con, 0, 0, nc, nx, true, update, false, true);
            row += nx;
        }
        {  // regularisation
            diag(row, row, -1.0, ncs_[0], update);
            row += ncs_[0];
            for (int k = 1; k <= N; ++k) {
                diag(row, row, -rho_dyn, nx, update);
                row += nx;
                diag(row, row, -1.0, ncs_[k], update);
                row += ncs_[k];
            }
        }
    }

    // kkt.hpp:207-222 (accumulates; stage-0 state constraints are ignored, as there)
    void update_rhs_initial_stage(const LQRModel &model, const VectorXs &x0) {
        const Node &kp = model.get_node(0);
        const int nx = nx_, nu = nu_, nc = kp.get_constraint_dim();
        for (int i = 0; i < nu; ++i) {
            scalar a = 0.0;
            for (int j = 0; j < nx; ++j) a += kp.H(i, nu + j) * x0(j);  // S0 x0
            rhs_(i) += -a;
        }
        const int ro = N_ * (nx + nu) + nc;
        for (int i = 0; i < nx; ++i) {
            scalar a = 0.0;
            for (int j = 0; j < nx; ++j) a += kp.E(i, nu + j) * x0(j);  // A0 x0
            rhs_(ro + i) += -a;
        }
    }

    // kkt.hpp:224-300
    void form_rhs(const LQRModel &model, const std::vector<VectorXs> &ws, const std::vector<VectorXs> &ys,
                  const std::vector<VectorXs> &zs, const std::vector<VectorXs> &inv_rho_vecs, const scalar sigma) {
        const int nx = nx_, nu = nu_, nxu = nx + nu, N = N_;
        int r1 = 0, r2 = N * nxu;
        auto dual = [&](int k, int nc) {
            for (int i = 0; i < nc; ++i) rhs_(r2 + i) = zs[k](i) - inv_rho_vecs[k](i) * ys[k](i);
        };
        {
            const Node &kp = model.get_node(0);
            const int nc = kp.get_constraint_dim();
            for (int i = 0; i < nu; ++i) rhs_(i) = -kp.h(i) + sigma * ws[0](i);
            dual(0, nc);
            for (int i = 0; i < nx; ++i) rhs_(r2 + nc + i) = -kp.c(i);
            r1 += nu;
            r2 += nc + nx;
        }
        for (int k = 1; k < N; ++k) {
            const Node &kp = model.get_node(k);
            const int nc = kp.get_constraint_dim();
            for (int i = 0; i < nx; ++i) rhs_(r1 + i) = -kp.h(nu + i) + sigma * ws[k](nu + i);
            for (int i = 0; i < nu; ++i) rhs_(r1 + nx + i) = -kp.h(i) + sigma * ws[k](i);
            dual(k, nc);
            for (int i = 0; i < nx; ++i) rhs_(r2 + nc + i) = -kp.c(i);
            r1 += nxu;
            r2 += nc + nx;
        }
        {
            const Node &kp = model.get_node(N);
            const int nc = kp.get_constraint_dim();
            for (int i = 0; i < nx; ++i) rhs_(r1 + i) = -kp.h(i) + sigma * ws[N](i);
            dual(N, nc);
        }
    }

    // kkt.hpp:302-331: upper-triangular CSC, Eigen's compressed order
    std::unique_ptr<CscMatrix> get_KKT_csc_matrix() {
        std::vector<std::pair<std::int64_t, scalar>> e(entries_.begin(), entries_.end());
        std::sort(e.begin(), e.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
        csc_p_.assign(static_cast<size_t>(dim_) + 1, 0);
        csc_i_.resize(e.size());
        csc_x_.resize(e.size());
        for (size_t q = 0; q < e.size(); ++q) {
            const int c = static_cast<int>(e[q].first >> 32), r = static_cast<int>(e[q].first & 0xffffffff);
            csc_i_[q] = r;
            csc_x_[q] = e[q].second;
            ++csc_p_[static_cast<size_t>(c) + 1];
        }
        for (int j = 0; j < dim_; ++j) csc_p_[static_cast<size_t>(j) + 1] += csc_p_[static_cast<size_t>(j)];
        auto K = std::make_unique<CscMatrix>();
        K->m = K->n = dim_;
        K->nzmax = static_cast<QDLDL_int>(e.size());
        K->p = csc_p_.data();
        K->i = csc_i_.data();
        K->x = csc_x_.data();
        return K;
    }

    const VectorXs &get_rhs() const { return rhs_; }

private:
    // assign_dense_matrix (utils.hpp:10-34) of the block M(r0 : r0+rows, c0 : c0+cols)
    // or of its transpose (trans), at (i0, j0)
    void dense(int i0, int j0, const MatrixXs &M, int r0, int c0, int rows, int cols, bool trans, bool update,
               bool fill_upper, bool ignore_zeros) {
        const int R = trans ? cols : rows, C = trans ? rows : cols;
        for (int j = 0; j < C; ++j)
            for (int i = 0; i < R; ++i) {
                if (fill_upper && i > j) continue;
                const scalar v = trans ? M(r0 + j, c0 + i) : M(r0 + i, c0 + j);
                if (ignore_zeros && v == scalar(0)) continue;
                set(i0 + i, j0 + j, v, update);
            }
    }
    void diag(int i0, int j0, scalar v, int size, bool update) {
        for (int i = 0; i < size; ++i) set(i0 + i, j0 + i, v, update);
    }
    void set(int r, int c, scalar v, bool /*update: insert and coeffRef both leave v in place*/) {
        entries_[(static_cast<std::int64_t>(c) << 32) | static_cast<std::uint32_t>(r)] = v;
    }

    int nx_, nu_, N_, dim_ = 0;
    std::vector<int> ncs_;
    VectorXs rhs_;
    std::unordered_map<std::int64_t, scalar> entries_;  // (col << 32 | row) -> value
    std::vector<QDLDL_int> csc_p_, csc_i_;
    std::vector<QDLDL_float> csc_x_;
};

namespace detail {

// QDLDL_etree (QDLDL's published elimination-tree / column-count pass, called
// by QDLDLSolver::create_workspace, qdldl_solver.hpp:47-78): -1 if an entry
// lies below the diagonal, -2 on overflow, else sum of the column counts.
inline QDLDL_int qdldl_etree(QDLDL_int n, const QDLDL_int *Ap, const QDLDL_int *Ai, QDLDL_int *work,
                             QDLDL_int *Lnz, QDLDL_int *etree) {
    for (QDLDL_int i = 0; i < n; ++i) {
        work[i] = 0;
        Lnz[i] = 0;
        etree[i] = -1;
    }
    for (QDLDL_int j = 0; j < n; ++j) {
        work[j] = j;
        for (QDLDL_int p = Ap[j]; p < Ap[j + 1]; ++p) {
            QDLDL_int i = Ai[p];
            if (i > j) return -1;
            while (work[i] != j) {
                if (etree[i] == -1) etree[i] = j;
                Lnz[i]++;
                work[i] = j;
                i = etree[i];
            }
        }
    }
    QDLDL_int sum = 0;
    for (QDLDL_int i = 0; i < n; ++i) {
        if (Lnz[i] > (QDLDL_int)0x7fffffffffffffffLL - sum) return -2;
        sum += Lnz[i];
    }
    return sum;
}

// QDLDLSolver::create_workspace (qdldl_solver.hpp:47-78)
inline std::unique_ptr<QDLDLData> create_qdldl_workspace(const CscMatrix &K) {
    auto d = std::make_unique<QDLDLData>();
    const QDLDL_int n = K.n;
    d->Ln = n;
    d->etree = std::make_unique<QDLDL_int[]>(n);
    d->Lnz = std::make_unique<QDLDL_int[]>(n);
    d->Lp = std::make_unique<QDLDL_int[]>(n + 1);
    d->D = std::make_unique<QDLDL_float[]>(n);
    d->Dinv = std::make_unique<QDLDL_float[]>(n);
    d->iwork = std::make_unique<QDLDL_int[]>(3 * n);
    d->bwork = std::make_unique<QDLDL_bool[]>(n);
    d->fwork = std::make_unique<QDLDL_float[]>(n);
    d->sumLnz = qdldl_etree(n, K.p, K.i, d->iwork.get(), d->Lnz.get(), d->etree.get());
    if (d->sumLnz < 0) throw std::runtime_error("Error in QDLDL_etree");
    d->Li = std::make_unique<QDLDL_int[]>(d->sumLnz);
    d->Lx = std::make_unique<QDLDL_float[]>(d->sumLnz);
    d->x = std::make_unique<QDLDL_float[]>(n);
    return d;
}

}  // namespace detail
}  // namespace lqr
