// clqr/detail/bridge.hpp -- glue between the C++ facade (clqr/lqr/*.hpp) and
// the C ABI of libpdplqr (pdplqr.h): model packing into the boundary layout,
// stage-vector flattening, RAII over pdplqr_handle, error translation.
#pragma once

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "clqr/lqr_model.hpp"
#include "pdplqr.h"

namespace lqr {
namespace detail {

// C ABI status -> exception (the reference throws std::runtime_error)
inline void check(int rc, const char *what) {
    if (rc != PDPLQR_OK) {
        const char *msg = pdplqr_last_error();
        throw std::runtime_error(std::string(what) + ": " + (msg && *msg ? msg : "pdplqr error ") +
                                 " (status " + std::to_string(rc) + ")");
    }
}

template <typename Dense>
inline void append(std::vector<double> &dst, const Dense &a) {
    const size_t k = static_cast<size_t>(a.size());
    if (k) dst.insert(dst.end(), a.data(), a.data() + k);
}

// does `a` equal packed[off, off + a.size())?  advances off
template <typename Dense>
inline bool same_at(const std::vector<double> &packed, size_t &off, const Dense &a) {
    const size_t k = static_cast<size_t>(a.size());
    if (off + k > packed.size()) return false;
    const bool eq = k == 0 || std::memcmp(packed.data() + off, a.data(), k * sizeof(double)) == 0;
    off += k;
    return eq;
}

// The model in the boundary layout of pdplqr.h (Eigen column-major blocks,
// stage-major): E [N][n s], c [N][n], H [N][s s] + [n n], h [N][s] + [n],
// D ragged [nc_k x dim_k].  Node k of the model is nodes[k].
struct PackedModel {
    std::vector<double> E, c, H, h, D;

    // packs the arrays in `mask` (PDPLQR_MODEL_*) only; the others keep their contents
    void pack(const LQRModel &model, int mask = PDPLQR_MODEL_ALL) {
        const int N = model.N;
        if (static_cast<int>(model.nodes.size()) != N + 1)
            throw std::runtime_error("LQRModel: expected N + 1 nodes, got " + std::to_string(model.nodes.size()));
        if (mask & PDPLQR_MODEL_E) E.clear();
        if (mask & PDPLQR_MODEL_C) c.clear();
        if (mask & PDPLQR_MODEL_H) H.clear();
        if (mask & PDPLQR_MODEL_HV) h.clear();
        if (mask & PDPLQR_MODEL_D) D.clear();
        for (int k = 0; k <= N; ++k) {
            const Node &nd = model.nodes[static_cast<size_t>(k)];
            if (k < N) {
                if (mask & PDPLQR_MODEL_E) append(E, nd.E);
                if (mask & PDPLQR_MODEL_C) append(c, nd.c);
            }
            if (mask & PDPLQR_MODEL_H) append(H, nd.H);
            if (mask & PDPLQR_MODEL_HV) append(h, nd.h);
            if ((mask & PDPLQR_MODEL_D) && nd.n_con > 0) append(D, nd.D_con);
        }
    }

    // the arrays in `mask` whose packed contents differ from `model`, compared
    // in place (no packing pass, no allocation; an array stops at its first
    // differing block)
    int differs(const LQRModel &model, int mask) const {
        const int N = model.N;
        if (static_cast<int>(model.nodes.size()) != N + 1) return mask;
        int out = 0;
        size_t oE = 0, oc = 0, oH = 0, oh = 0, oD = 0;
        for (int k = 0; k <= N && (mask & ~out); ++k) {
            const Node &nd = model.nodes[static_cast<size_t>(k)];
            const int live = mask & ~out;
            if (k < N) {
                if ((live & PDPLQR_MODEL_E) && !same_at(E, oE, nd.E)) out |= PDPLQR_MODEL_E;
                if ((live & PDPLQR_MODEL_C) && !same_at(c, oc, nd.c)) out |= PDPLQR_MODEL_C;
            }
            if ((live & PDPLQR_MODEL_H) && !same_at(H, oH, nd.H)) out |= PDPLQR_MODEL_H;
            if ((live & PDPLQR_MODEL_HV) && !same_at(h, oh, nd.h)) out |= PDPLQR_MODEL_HV;
            if ((live & PDPLQR_MODEL_D) && nd.n_con > 0 && !same_at(D, oD, nd.D_con)) out |= PDPLQR_MODEL_D;
        }
        // a model that shrank leaves packed entries unmatched
        if ((mask & PDPLQR_MODEL_E) && oE != E.size()) out |= PDPLQR_MODEL_E;
        if ((mask & PDPLQR_MODEL_C) && oc != c.size()) out |= PDPLQR_MODEL_C;
        if ((mask & PDPLQR_MODEL_H) && oH != H.size()) out |= PDPLQR_MODEL_H;
        if ((mask & PDPLQR_MODEL_HV) && oh != h.size()) out |= PDPLQR_MODEL_HV;
        if ((mask & PDPLQR_MODEL_D) && oD != D.size()) out |= PDPLQR_MODEL_D;
        return out & mask;
    }
};

// stage vectors (ws: s per stage, n at N; ys / zs / rho: nc_k per stage) <-> flat
inline void flatten(const std::vector<VectorXs> &v, std::vector<double> &out) {
    out.clear();
    for (const VectorXs &x : v) append(out, x);
}

inline void unflatten_ws(const std::vector<double> &flat, std::vector<VectorXs> &ws, int n, int m, int N) {
    if (static_cast<int>(ws.size()) < N + 1) throw std::runtime_error("forward: ws must hold N + 1 vectors");
    const int s = n + m;
    for (int k = 0; k <= N; ++k) {
        VectorXs &w = ws[static_cast<size_t>(k)];
        const int len = k < N ? s : n;
        if (w.size() != len) w.resize(len);
        std::memcpy(w.data(), flat.data() + static_cast<size_t>(k) * s, sizeof(double) * static_cast<size_t>(len));
    }
}

// One pdplqr_handle of the requested solver kind for this model (batch 1).
class Handle {
public:
    Handle(const LQRModel &model, int solver, int num_segments = 1, bool load_balancing = true, int condensed = 1,
           bool keep_factors = true, const std::vector<int> &devices = {}) {
        pdplqr_config cfg;
        pdplqr_config_init(&cfg);
        cfg.nx = model.n;
        cfg.nu = model.m;
        cfg.N = model.N;
        cfg.solver = solver;
        cfg.num_segments = num_segments;
        cfg.load_balancing = load_balancing ? 1 : 0;
        cfg.condensed_type = condensed;
        cfg.keep_factors = keep_factors ? 1 : 0;
        ncs_.assign(model.ncs.begin(), model.ncs.end());
        cfg.ncs = ncs_.data();
        devs_.assign(devices.begin(), devices.end());
        if (!devs_.empty()) {  // the horizon split over these GPUs (pdplqr_config.num_devices)
            cfg.num_devices = static_cast<int32_t>(devs_.size());
            cfg.devices = devs_.data();
        }
        check(pdplqr_create(&cfg, &h_), "pdplqr_create");
        n_ = model.n;
        m_ = model.m;
        N_ = model.N;
    }
    ~Handle() { pdplqr_destroy(h_); }
    Handle(const Handle &) = delete;
    Handle &operator=(const Handle &) = delete;

    // Uploads the arrays of `model` in `mask` (PDPLQR_MODEL_*) that differ from
    // what the device holds: the reference reads its model lazily (H, h at
    // update_problem_data, E, c, D_con at backward / forward), so each facade
    // call syncs exactly what that call reads.  With tracking on (the default)
    // an unchanged model costs one in-place compare of the arrays in `mask`
    // (no packing, no host -> device copy); with tracking off the compare is
    // skipped too and only arrays declared by model_changed() are re-read.
    void sync(const LQRModel &model, int mask) {
        if (!synced_) mask = PDPLQR_MODEL_ALL;
        int need;
        if (!synced_) need = PDPLQR_MODEL_ALL;
        else if (tracking_) need = packed_.differs(model, mask);
        else need = pending_ & mask;
        if (!need) return;
        packed_.pack(model, need);
        check(pdplqr_set_model_arrays(h_, need, packed_.E.data(), packed_.c.data(), packed_.H.data(),
                                      packed_.h.data(), packed_.D.empty() ? nullptr : packed_.D.data(),
                                      PDPLQR_MEM_HOST),
              "set_model");
        pending_ &= ~need;
        synced_ = true;
    }
    void upload(const LQRModel &model) { sync(model, PDPLQR_MODEL_ALL); }

    // MPC loops whose model rarely changes: with tracking off the protocol calls
    // do no per-call host work on the model; the caller declares edits with
    // model_changed(mask), and each declared array is re-read at the next call
    // that reads it (the lazy semantics above are kept)
    void set_tracking(bool on) { tracking_ = on; }
    void model_changed(int mask) { pending_ |= mask & PDPLQR_MODEL_ALL; }

    long long upload_bytes() const {
        int64_t b = 0;
        check(pdplqr_get_model_upload_bytes(h_, &b), "get_model_upload_bytes");
        return static_cast<long long>(b);
    }

    void update(const std::vector<VectorXs> &ws, const std::vector<VectorXs> &ys, const std::vector<VectorXs> &zs,
                const std::vector<VectorXs> &inv_rho, scalar sigma) {
        flatten(ws, w_);
        flatten(ys, y_);
        flatten(zs, z_);
        flatten(inv_rho, r_);
        check(pdplqr_update_problem_data(h_, w_.data(), nz(y_), nz(z_), nz(r_), sigma, PDPLQR_MEM_HOST),
              "update_problem_data");
    }

    void backward(const std::vector<VectorXs> &rho, bool factorize) {
        flatten(rho, r_);
        check(factorize ? pdplqr_backward(h_, nz(r_), PDPLQR_MEM_HOST)
                        : pdplqr_backward_without_factorization(h_, nz(r_), PDPLQR_MEM_HOST),
              factorize ? "backward" : "backward_without_factorization");
    }

    void forward(const VectorXs &x0, std::vector<VectorXs> &ws) {
        if (x0.size() != n_) throw std::runtime_error("forward: x0 has the wrong size");
        w_.assign(static_cast<size_t>(N_) * (n_ + m_) + n_, 0.0);
        check(pdplqr_forward(h_, x0.data(), w_.data(), PDPLQR_MEM_HOST), "forward");
        unflatten_ws(w_, ws, n_, m_, N_);
    }

    void clear() { check(pdplqr_clear_workspace(h_), "clear_workspace"); }

    int status() {
        int32_t st = 0;
        check(pdplqr_get_status(h_, &st), "get_status");
        return st;
    }

    pdplqr_handle raw() const { return h_; }

private:
    static const double *nz(const std::vector<double> &v) { return v.empty() ? nullptr : v.data(); }
    pdplqr_handle h_ = nullptr;
    int n_ = 0, m_ = 0, N_ = 0;
    std::vector<int32_t> ncs_, devs_;
    PackedModel packed_;  // what the device holds
    bool synced_ = false, tracking_ = true;
    int pending_ = 0;  // arrays declared changed (tracking off)
    std::vector<double> w_, y_, z_, r_;
};

}  // namespace detail
}  // namespace lqr
