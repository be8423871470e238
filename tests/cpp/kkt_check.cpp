// Host-side check of the public KKT surface of the facade (clqr/lqr/kkt.hpp):
// reads a packed problem (written by tests/test_kkt_facade.py), builds an
// lqr::LQRModel node by node, forms the KKT matrix (rho_dyn, sigma) and its
// right-hand side (form_rhs + update_rhs_initial_stage), exports the CSC and
// the QDLDL workspace's elimination tree, and writes them back.  No GPU.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "clqr/lqr/kkt.hpp"

template <class T>
static void rd(FILE *f, T *p, size_t n) {
    if (fread(p, sizeof(T), n, f) != n) {
        fprintf(stderr, "short read\n");
        exit(2);
    }
}

int main(int argc, char **argv) {
    if (argc != 3) return 2;
    FILE *f = fopen(argv[1], "rb");
    int hdr[3];
    rd(f, hdr, 3);
    const int n = hdr[0], m = hdr[1], N = hdr[2], s = n + m;
    std::vector<int> ncs(N + 1);
    rd(f, ncs.data(), N + 1);
    int ny = 0, nD = 0;
    for (int k = 0; k <= N; ++k) {
        ny += ncs[k];
        nD += ncs[k] * (k < N ? s : n);
    }
    std::vector<double> E((size_t)N * n * s), c((size_t)N * n), H((size_t)N * s * s + n * n), h((size_t)N * s + n),
        D(nD), ws((size_t)N * s + n), ys(ny), zs(ny), ir(ny), x0(n), sc(3);
    rd(f, E.data(), E.size());
    rd(f, c.data(), c.size());
    rd(f, H.data(), H.size());
    rd(f, h.data(), h.size());
    rd(f, D.data(), D.size());
    rd(f, ws.data(), ws.size());
    rd(f, ys.data(), ys.size());
    rd(f, zs.data(), zs.size());
    rd(f, ir.data(), ir.size());
    rd(f, x0.data(), x0.size());
    rd(f, sc.data(), 3);  // sigma of the rhs, rho_dyn, sigma frozen into the matrix
    fclose(f);

    lqr::LQRModel model(n, m, N);
    std::vector<lqr::VectorXs> wv, yv, zv, iv;
    int doff = 0, yoff = 0;
    for (int k = 0; k <= N; ++k) {
        const bool term = k == N;
        const int dim = term ? n : s;
        model.add_node(n, m, ncs[k], k, term);
        lqr::Node &nd = model.get_node(k);
        for (int j = 0; j < dim; ++j)
            for (int i = 0; i < dim; ++i) nd.H(i, j) = term ? H[(size_t)N * s * s + i + j * n] : H[(size_t)k * s * s + i + j * s];
        for (int i = 0; i < dim; ++i) nd.h(i) = h[(size_t)k * s + i];
        if (!term) {
            for (int j = 0; j < s; ++j)
                for (int i = 0; i < n; ++i) nd.E(i, j) = E[(size_t)k * n * s + i + j * n];
            for (int i = 0; i < n; ++i) nd.c(i) = c[(size_t)k * n + i];
        }
        for (int j = 0; j < dim; ++j)
            for (int i = 0; i < ncs[k]; ++i) nd.D_con(i, j) = D[doff + i + j * ncs[k]];
        doff += ncs[k] * dim;
        lqr::VectorXs w(dim), y(ncs[k]), z(ncs[k]), r(ncs[k]);
        for (int i = 0; i < dim; ++i) w(i) = ws[(size_t)k * s + i];
        for (int i = 0; i < ncs[k]; ++i) {
            y(i) = ys[yoff + i];
            z(i) = zs[yoff + i];
            r(i) = ir[yoff + i];
        }
        yoff += ncs[k];
        wv.push_back(w);
        yv.push_back(y);
        zv.push_back(z);
        iv.push_back(r);
    }
    lqr::KKTSystem kkt(n, m, N, ncs);
    kkt.form_KKT_matrix(model, sc[1], sc[2], false);  // QDLDLSolver: rho_dyn = sigma = 1e-6 (qdldl_solver.hpp:38-41)
    auto K = kkt.get_KKT_csc_matrix();
    auto ws_ = lqr::detail::create_qdldl_workspace(*K);
    lqr::VectorXs xv(n);
    for (int i = 0; i < n; ++i) xv(i) = x0[i];
    kkt.form_rhs(model, wv, yv, zv, iv, sc[0]);
    kkt.update_rhs_initial_stage(model, xv);
    FILE *o = fopen(argv[2], "wb");
    long long dims[3] = {K->n, K->nzmax, ws_->sumLnz};
    fwrite(dims, sizeof(long long), 3, o);
    fwrite(K->p, sizeof(QDLDL_int), K->n + 1, o);
    fwrite(K->i, sizeof(QDLDL_int), K->nzmax, o);
    fwrite(K->x, sizeof(QDLDL_float), K->nzmax, o);
    fwrite(kkt.get_rhs().data(), sizeof(double), K->n, o);
    fwrite(ws_->Lnz.get(), sizeof(QDLDL_int), K->n, o);
    fwrite(ws_->etree.get(), sizeof(QDLDL_int), K->n, o);
    fclose(o);
    return 0;
}
