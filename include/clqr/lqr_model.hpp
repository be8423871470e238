// clqr/lqr_model.hpp -- the LQ problem container of the pdpLQR C++ surface.
//
// Same public members and methods as the reference's model header
// (include/clqr/lqr_model.hpp:8-89), so problem-setup code written against the
// reference compiles unchanged:
//   stage k < N   x+ = A x + B u + c,  E = [B A] (n x (m+n)), cost H = [R S; S^T Q], h = [r; q],
//                 e_lb <= D_con [u; x] <= e_ub  (D_con = [Du Dx], n_con rows)
//   terminal N    cost H (n x n), h (n), D_con (n_con x n)
// The solvers (clqr/lqr/*.hpp) read the nodes in add_node order; `ncs` is
// indexed by time_step, as in the reference.
#pragma once

#include <stdexcept>
#include <vector>

#include "clqr/typedefs.hpp"

namespace lqr {

struct Node {
    int n = 0;      // state dimension
    int m = 0;      // control dimension
    int n_con = 0;  // rows of D_con

    MatrixXs E;      // [B A]
    VectorXs c;      // affine dynamics term
    MatrixXs H;      // stage Hessian over [u; x] (terminal: over x)
    VectorXs h;      // stage gradient
    MatrixXs D_con;  // [Du Dx] (terminal: Dx)
    VectorXs e_lb, e_ub;

    bool is_terminal = false;
    int time_step = 0;

    Node(int state_dim, int control_dim, int n_constraints, int stage, bool is_terminal_stage = false)
        : n(state_dim), m(control_dim), n_con(n_constraints), is_terminal(is_terminal_stage), time_step(stage) {
        allocate();
        set_zero();
    }

    int get_constraint_dim() const { return n_con; }

    void set_zero() {
        for (MatrixXs *M : {&E, &H, &D_con}) M->setZero();
        for (VectorXs *v : {&c, &h, &e_lb, &e_ub}) v->setZero();
    }

private:
    void allocate() {
        const int cols = is_terminal ? n : n + m;  // variables this node's blocks act on
        H.resize(cols, cols);
        h.resize(cols);
        if (!is_terminal) {
            E.resize(n, n + m);
            c.resize(n);
        }
        if (n_con > 0) {
            D_con.resize(n_con, cols);
            e_lb.resize(n_con);
            e_ub.resize(n_con);
        }
    }
};

struct LQRModel {
    int n;  // state dimension
    int m;  // control dimension
    int N;  // horizon (number of intervals)

    std::vector<int> ncs;     // constraint rows per time step
    std::vector<Node> nodes;  // N + 1 nodes, the last one terminal

    LQRModel(int state_dim, int control_dim, int horizon) : n(state_dim), m(control_dim), N(horizon) {
        if (N < 1) throw std::runtime_error("Horizon must be at least 1.");
        ncs.assign(static_cast<size_t>(N) + 1, 0);
        nodes.reserve(static_cast<size_t>(N) + 1);
    }

    Node &get_node(int k) { return nodes[static_cast<size_t>(k)]; }
    const Node &get_node(int k) const { return nodes[static_cast<size_t>(k)]; }

    void add_node(int state_dim, int control_dim, int nc, int time_step, bool is_terminal_stage = false) {
        nodes.emplace_back(state_dim, control_dim, nc, time_step, is_terminal_stage);
        ncs[static_cast<size_t>(time_step)] = nc;
    }
};

}  // namespace lqr
