// packed_model_check.cpp -- host-only check of the facade's model-change
// detection (clqr/detail/bridge.hpp PackedModel::differs): every array an edit
// touches is reported, nothing else is, and an unchanged model reports 0.
#include <cstdio>

#include "clqr/detail/bridge.hpp"

namespace {
int fails = 0;
void expect(int got, int want, const char *what) {
    if (got != want) {
        std::printf("FAIL %s: got %d want %d\n", what, got, want);
        ++fails;
    }
}
}  // namespace

int main() {
    const int n = 3, m = 2, N = 4, s = n + m;
    lqr::LQRModel model(n, m, N);
    for (int k = 0; k <= N; ++k) {
        const bool term = k == N;
        model.add_node(n, m, k == 1 ? 2 : 0, k, term);
        lqr::Node &nd = model.get_node(k);
        const int dim = term ? n : s;
        if (!term) {
            for (int j = 0; j < s; ++j)
                for (int i = 0; i < n; ++i) nd.E(i, j) = 0.1 * (i + 1) + j + k;
            for (int i = 0; i < n; ++i) nd.c(i) = i - k;
        }
        for (int j = 0; j < dim; ++j)
            for (int i = 0; i < dim; ++i) nd.H(i, j) = (i == j) ? 2.0 + k : 0.01 * (i + j);
        for (int i = 0; i < dim; ++i) nd.h(i) = 0.5 * i + k;
        if (k == 1)
            for (int j = 0; j < dim; ++j)
                for (int i = 0; i < 2; ++i) nd.D_con(i, j) = i + 0.25 * j;
    }
    lqr::detail::PackedModel pk;
    pk.pack(model);
    expect(pk.differs(model, PDPLQR_MODEL_ALL), 0, "unchanged");
    model.get_node(2).E(1, 3) += 1e-12;
    expect(pk.differs(model, PDPLQR_MODEL_ALL), PDPLQR_MODEL_E, "E edit");
    expect(pk.differs(model, PDPLQR_MODEL_H | PDPLQR_MODEL_HV), 0, "E edit outside the mask");
    model.get_node(N).H(2, 2) *= 2.0;  // the terminal block
    model.get_node(1).D_con(1, 4) = -1.0;
    expect(pk.differs(model, PDPLQR_MODEL_ALL), PDPLQR_MODEL_E | PDPLQR_MODEL_H | PDPLQR_MODEL_D, "E, H, D edits");
    pk.pack(model, PDPLQR_MODEL_E | PDPLQR_MODEL_H);
    expect(pk.differs(model, PDPLQR_MODEL_ALL), PDPLQR_MODEL_D, "after re-packing E and H");
    pk.pack(model);
    model.get_node(0).c(0) = 7.0;
    model.get_node(3).h(4) = -3.0;
    expect(pk.differs(model, PDPLQR_MODEL_ALL), PDPLQR_MODEL_C | PDPLQR_MODEL_HV, "c, h edits");
    std::printf(fails ? "FAILED\n" : "ok\n");
    return fails ? 1 : 0;
}
