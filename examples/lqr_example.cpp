// lqr_example.cpp -- the reference's quadrotor MPC problem (N = 100, nx = 12,
// nu = 4, constraints disabled) solved through the MI355X build's C++ facade
// with the three solver classes, exactly as reference user code would call
// them (include/clqr/...; the problem data is the one of the reference's
// examples/lqr_example.cpp:53-168).  Each solver runs on the GPU through
// libpdplqr.so; the wall time of backward + forward is printed per solver,
// with u_0..u_4 and x_N for comparison (the three agree to ~2e-5 rel: the
// QDLDL path carries rho_dyn = sigma = 1e-6 in its KKT matrix).
//
//   lqr_example [N]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "clqr/lqr/lqr_solver.hpp"
#include "clqr/lqr/lqr_solver_parallel.hpp"
#include "clqr/lqr/qdldl_solver.hpp"

namespace {

constexpr int kNx = 12, kNu = 4;

// Discretised quadrotor (row-major here; copied into the column-major E = [B A]).
const double kA[kNx][kNx] = {
    {1, 0, 0, 0, 0, 0, 0.1, 0, 0, 0, 0, 0},
    {0, 1, 0, 0, 0, 0, 0, 0.1, 0, 0, 0, 0},
    {0, 0, 1, 0, 0, 0, 0, 0, 0.1, 0, 0, 0},
    {0.0488, 0, 0, 1, 0, 0, 0.0016, 0, 0, 0.0992, 0, 0},
    {0, -0.0488, 0, 0, 1, 0, 0, -0.0016, 0, 0, 0.0992, 0},
    {0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0.0992},
    {0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0},
    {0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0},
    {0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0},
    {0.9734, 0, 0, 0, 0, 0, 0.0488, 0, 0, 0.9846, 0, 0},
    {0, -0.9734, 0, 0, 0, 0, 0, -0.0488, 0, 0, 0.9846, 0},
    {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0.9846}};
const double kB[kNx][kNu] = {
    {0, -0.0726, 0, 0.0726},     {-0.0726, 0, 0.0726, 0},     {-0.0152, 0.0152, -0.0152, 0.0152},
    {0, -0.0006, 0, 0.0006},     {0.0006, 0, -0.0006, 0},     {0.0106, 0.0106, 0.0106, 0.0106},
    {0, -1.4512, 0, 1.4512},     {-1.4512, 0, 1.4512, 0},     {-0.3049, 0.3049, -0.3049, 0.3049},
    {0, -0.0236, 0, 0.0236},     {0.0236, 0, -0.0236, 0},     {0.2107, 0.2107, 0.2107, 0.2107}};
const double kQdiag[kNx] = {0, 0, 10, 10, 10, 10, 0, 0, 0, 5, 5, 5};
const double kRdiag = 0.1;
const double kXref[kNx] = {0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0};

// Stage k of the tracking problem: w = [u; x], H = blkdiag(R, Q), h = [0; -Q x_ref].
void fill_stage(lqr::Node &nd, bool terminal) {
    const int off = terminal ? 0 : kNu;
    if (!terminal) {
        for (int i = 0; i < kNx; ++i) {
            for (int j = 0; j < kNu; ++j) nd.E(i, j) = kB[i][j];
            for (int j = 0; j < kNx; ++j) nd.E(i, kNu + j) = kA[i][j];
            nd.c(i) = 0.0;
        }
        for (int j = 0; j < kNu; ++j) {
            nd.H(j, j) = kRdiag;
            nd.h(j) = 0.0;
        }
    }
    for (int i = 0; i < kNx; ++i) {
        nd.H(off + i, off + i) = kQdiag[i];
        nd.h(off + i) = -kQdiag[i] * kXref[i];
    }
}

std::vector<lqr::VectorXs> sized(int n, int m, int N, int nc_each) {
    std::vector<lqr::VectorXs> v;
    for (int k = 0; k <= N; ++k) {
        lqr::VectorXs x(nc_each < 0 ? (k < N ? n + m : n) : nc_each);
        for (int i = 0; i < x.size(); ++i) x(i) = 0.0;
        v.push_back(x);
    }
    return v;
}

void report(const char *name, double ms, const std::vector<lqr::VectorXs> &ws, int N) {
    std::printf("%-24s %9.3f ms\n", name, ms);
    for (int k = 0; k < 5 && k < N; ++k) {
        std::printf("  u%d =", k);
        for (int i = 0; i < kNu; ++i) std::printf(" % .10f", ws[k](i));
        std::printf("\n");
    }
    std::printf("  x_N =");
    for (int i = 0; i < kNx; ++i) std::printf(" % .7f", ws[N](i));
    std::printf("\n");
}

}  // namespace

int main(int argc, char **argv) {
    const int N = argc > 1 ? std::atoi(argv[1]) : 100;
    lqr::LQRModel model(kNx, kNu, N);
    for (int k = 0; k <= N; ++k) {
        model.add_node(kNx, kNu, 0, k, k == N);
        fill_stage(model.get_node(k), k == N);
    }
    const double sigma = 1e-6;
    auto ws = sized(kNx, kNu, N, -1);
    auto ys = sized(kNx, kNu, N, 0), zs = ys, rho = ys, inv_rho = ys;
    lqr::VectorXs x0(kNx);
    for (int i = 0; i < kNx; ++i) x0(i) = 0.0;

    // one solve = backward + forward, the reference example's timed region
    auto timed = [&](const char *name, const std::function<void(std::vector<lqr::VectorXs> &)> &solve) {
        auto out = ws;
        solve(out);  // first call: device buffers, code objects
        const auto t0 = std::chrono::steady_clock::now();
        solve(out);
        const auto t1 = std::chrono::steady_clock::now();
        report(name, std::chrono::duration<double, std::milli>(t1 - t0).count(), out, N);
    };
    try {
        lqr::QDLDLSolver kkt(model);
        kkt.update_problem_data(ws, ys, zs, inv_rho, sigma);
        timed("QDLDLSolver", [&](std::vector<lqr::VectorXs> &out) {
            kkt.backward(inv_rho);
            kkt.forward(x0, out);
        });
        lqr::LQRSolver serial(model);
        serial.update_problem_data(ws, ys, zs, inv_rho, sigma);
        timed("LQRSolver", [&](std::vector<lqr::VectorXs> &out) {
            serial.backward(rho);
            serial.forward(x0, out);
        });
        lqr::LQRParallelSolver par(model, 4, true, lqr::CondensedSystemSolverType::CHOLESKY);
        par.update_problem_data(ws, ys, zs, inv_rho, sigma);
        timed("LQRParallelSolver(4)", [&](std::vector<lqr::VectorXs> &out) {
            par.backward(rho);
            par.forward(x0, out);
        });
    } catch (const std::exception &e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}
