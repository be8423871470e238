// facade_check.cpp -- drives the C++ facade (include/clqr/...) exactly as a
// reference user would: builds an lqr::LQRModel with add_node, fills the
// Eigen-style blocks element by element, and runs one of the three solver
// classes through update_problem_data -> backward -> forward.
//
//   facade_check <problem.bin> <out.bin> <solver> [num_segments condensed] [nofact|mutate|mpc|declared]
//   solver: serial | parallel | qdldl
// problem.bin (little endian): int32 n, m, N, ncs[N+1]; then float64 arrays in
// the boundary layout of pdplqr.h: E, c, H, h, D, x0, sigma, ws, ys, zs, rho, inv_rho.
// out.bin: float64 w = [u0; x0; ...; xN] (N s + n).  With `nofact` the solve is
// followed by backward_without_factorization + forward on linear data
// perturbed deterministically (w-bar + 0.1), and that second answer is written.
// With `mutate` the model is edited between update_problem_data and backward
// (E of node N/2 scaled by 1.01, H of node 1 doubled): the reference reads E
// at backward / forward and H at update_problem_data, so the answer is that of
// the model with the new E and the old H.  With `mpc` the protocol runs 5 more
// times on the unchanged model and the model bytes uploaded host -> device
// during those iterations are printed ("uploads <bytes>").  With `declared`
// model tracking is off: the same 5 iterations, then the `mutate` edit with only
// E declared (model_changed(PDPLQR_MODEL_E)) before one more solve, whose answer
// is again the model with the new E and the old H.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "clqr/lqr/lqr_solver.hpp"
#include "clqr/lqr/lqr_solver_parallel.hpp"
#include "clqr/lqr/qdldl_solver.hpp"

namespace {

struct Reader {
    std::FILE *f;
    template <typename T>
    std::vector<T> take(size_t k) {
        std::vector<T> v(k);
        if (k && std::fread(v.data(), sizeof(T), k, f) != k) {
            std::fprintf(stderr, "short read\n");
            std::exit(2);
        }
        return v;
    }
};

std::vector<lqr::VectorXs> cut(const std::vector<double> &flat, const std::vector<int> &len) {
    std::vector<lqr::VectorXs> out;
    size_t o = 0;
    for (int l : len) {
        lqr::VectorXs v(l);
        for (int i = 0; i < l; ++i) v(i) = flat[o + static_cast<size_t>(i)];
        o += static_cast<size_t>(l);
        out.push_back(v);
    }
    return out;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s problem.bin out.bin serial|parallel|qdldl [ns condensed] [nofact]\n", argv[0]);
        return 2;
    }
    std::FILE *f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    Reader rd{f};
    const auto hdr = rd.take<int32_t>(3);
    const int n = hdr[0], m = hdr[1], N = hdr[2], s = n + m;
    const auto ncs = rd.take<int32_t>(static_cast<size_t>(N) + 1);
    size_t ndD = 0, ny = 0;
    for (int k = 0; k <= N; ++k) {
        ndD += static_cast<size_t>(ncs[k]) * (k < N ? s : n);
        ny += static_cast<size_t>(ncs[k]);
    }
    const auto E = rd.take<double>(static_cast<size_t>(N) * n * s), c = rd.take<double>(static_cast<size_t>(N) * n);
    const auto H = rd.take<double>(static_cast<size_t>(N) * s * s + static_cast<size_t>(n) * n);
    const auto h = rd.take<double>(static_cast<size_t>(N) * s + n), D = rd.take<double>(ndD);
    const auto x0v = rd.take<double>(n), sig = rd.take<double>(1);
    const auto ws = rd.take<double>(static_cast<size_t>(N) * s + n), ys = rd.take<double>(ny), zs = rd.take<double>(ny);
    const auto rho = rd.take<double>(ny), irho = rd.take<double>(ny);
    std::fclose(f);

    // the model, node by node (reference examples/lqr_example.cpp style)
    lqr::LQRModel model(n, m, N);
    size_t oE = 0, oc = 0, oH = 0, oh = 0, oD = 0;
    for (int k = 0; k <= N; ++k) {
        const bool term = k == N;
        model.add_node(n, m, ncs[k], k, term);
        lqr::Node &nd = model.get_node(k);
        const int dim = term ? n : s;
        if (!term) {
            for (int j = 0; j < s; ++j)
                for (int i = 0; i < n; ++i) nd.E(i, j) = E[oE++];
            for (int i = 0; i < n; ++i) nd.c(i) = c[oc++];
        }
        for (int j = 0; j < dim; ++j)
            for (int i = 0; i < dim; ++i) nd.H(i, j) = H[oH++];
        for (int i = 0; i < dim; ++i) nd.h(i) = h[oh++];
        for (int j = 0; j < dim && ncs[k] > 0; ++j)
            for (int i = 0; i < ncs[k]; ++i) nd.D_con(i, j) = D[oD++];
    }
    std::vector<int> wlen(static_cast<size_t>(N) + 1, s), ylen(ncs.begin(), ncs.end());
    wlen.back() = n;
    auto wsv = cut(ws, wlen), ysv = cut(ys, ylen), zsv = cut(zs, ylen), rhov = cut(rho, ylen),
         irv = cut(irho, ylen);
    lqr::VectorXs x0(n);
    for (int i = 0; i < n; ++i) x0(i) = x0v[i];
    const double sigma = sig[0];
    const std::string kind = argv[3];
    const bool nofact = std::string(argv[argc - 1]) == "nofact";
    const bool mutate = std::string(argv[argc - 1]) == "mutate";
    const bool declared = std::string(argv[argc - 1]) == "declared";
    const bool mpc = declared || std::string(argv[argc - 1]) == "mpc";
    auto edit = [&]() {
        lqr::Node &a = model.get_node(N / 2);
        for (int j = 0; j < s; ++j)
            for (int i = 0; i < n; ++i) a.E(i, j) *= 1.01;
        lqr::Node &b = model.get_node(1);
        for (int j = 0; j < s; ++j)
            for (int i = 0; i < s; ++i) b.H(i, j) *= 2.0;
    };
    long long uploads = -1;
    std::vector<lqr::VectorXs> out = wsv;
    auto ws2 = wsv;
    for (auto &v : ws2)
        for (int i = 0; i < v.size(); ++i) v(i) += 0.1;
    try {
        if (kind == "serial") {
            lqr::LQRSolver sol(model);
            if (declared) sol.set_model_tracking(false);
            sol.update_problem_data(wsv, ysv, zsv, irv, sigma);
            if (mutate) edit();
            sol.backward(rhov);
            sol.forward(x0, out);
            if (mpc) {
                const long long b0 = sol.model_upload_bytes();
                for (int it = 0; it < 5; ++it) {
                    sol.update_problem_data(wsv, ysv, zsv, irv, sigma);
                    sol.backward(rhov);
                    sol.forward(x0, out);
                }
                uploads = sol.model_upload_bytes() - b0;
            }
            if (declared) {
                sol.update_problem_data(wsv, ysv, zsv, irv, sigma);
                edit();
                sol.model_changed(PDPLQR_MODEL_E);  // H's edit is not declared: the device keeps the old H
                sol.backward(rhov);
                sol.forward(x0, out);
            }
            if (nofact) {
                sol.update_problem_data(ws2, ysv, zsv, irv, sigma);
                sol.backward_without_factorization(rhov);
                sol.forward(x0, out);
            }
        } else if (kind == "parallel") {
            const int ns = argc > 4 ? std::atoi(argv[4]) : 4;
            const auto ty = (argc > 5 && std::string(argv[5]) == "LU") ? lqr::CondensedSystemSolverType::LU
                                                                        : lqr::CondensedSystemSolverType::CHOLESKY;
            // devices=0,0,... : the multi-GPU split of the horizon (pdplqr.h num_devices)
            std::vector<int> devs;
            for (int a = 4; a < argc; ++a) {
                const std::string arg = argv[a];
                if (arg.rfind("devices=", 0) != 0) continue;
                size_t p = 8;
                while (p < arg.size()) {
                    const size_t q = arg.find(',', p);
                    devs.push_back(std::atoi(arg.substr(p, q == std::string::npos ? std::string::npos : q - p).c_str()));
                    p = q == std::string::npos ? arg.size() : q + 1;
                }
            }
            lqr::LQRParallelSolver sol(model, ns, true, ty, devs);
            if (declared) sol.set_model_tracking(false);
            sol.update_problem_data(wsv, ysv, zsv, irv, sigma);
            if (mutate) edit();
            sol.backward(rhov);
            sol.forward(x0, out);
            if (mpc) {
                const long long b0 = sol.model_upload_bytes();
                for (int it = 0; it < 5; ++it) {
                    sol.update_problem_data(wsv, ysv, zsv, irv, sigma);
                    sol.backward(rhov);
                    sol.forward(x0, out);
                }
                uploads = sol.model_upload_bytes() - b0;
            }
            if (declared) {
                sol.update_problem_data(wsv, ysv, zsv, irv, sigma);
                edit();
                sol.model_changed(PDPLQR_MODEL_E);  // H's edit is not declared: the device keeps the old H
                sol.backward(rhov);
                sol.forward(x0, out);
            }
            if (nofact) {
                sol.update_problem_data(ws2, ysv, zsv, irv, sigma);
                sol.backward_without_factorization(rhov);
                sol.forward(x0, out);
            }
        } else if (kind == "qdldl") {
            lqr::QDLDLSolver sol(model);
            if (declared) sol.set_model_tracking(false);
            sol.update_problem_data(wsv, ysv, zsv, irv, sigma);
            sol.backward(irv);
            sol.forward(x0, out);
            if (mpc) {
                const long long b0 = sol.model_upload_bytes();
                for (int it = 0; it < 5; ++it) {
                    sol.update_problem_data(wsv, ysv, zsv, irv, sigma);
                    sol.backward(irv);
                    sol.forward(x0, out);
                }
                uploads = sol.model_upload_bytes() - b0;
            }
        } else {
            std::fprintf(stderr, "unknown solver %s\n", kind.c_str());
            return 2;
        }
    } catch (const std::exception &e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 3;
    }
    std::FILE *g = std::fopen(argv[2], "wb");
    if (!g) return 2;
    for (const auto &v : out) std::fwrite(v.data(), sizeof(double), static_cast<size_t>(v.size()), g);
    std::fclose(g);
    std::printf("ok %s u0[0]=%.10f\n", kind.c_str(), out[0](0));
    if (mpc) std::printf("uploads %lld\n", uploads);
    return 0;
}
