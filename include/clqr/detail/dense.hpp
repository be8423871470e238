// clqr/detail/dense.hpp -- minimal column-major dense containers used as
// lqr::VectorXs / lqr::MatrixXs when Eigen is not installed.
//
// They cover the part of Eigen's interface that callers of the pdpLQR solve
// protocol touch: sizing constructors, resize, element access (i) / (i, j),
// size / rows / cols, data(), setZero / setConstant / setIdentity, and
// contiguous head / tail / segment views of vectors.  Storage is contiguous
// and column-major, exactly Eigen's default, so the facade packs either kind
// with the same code.
#pragma once

#include <algorithm>
#include <cstddef>
#include <stdexcept>
#include <vector>

namespace pdplqr {
namespace dense {

class Vector;

// a contiguous window into a Vector (head / tail / segment)
class VectorView {
public:
    VectorView(double *p, std::ptrdiff_t n) : p_(p), n_(n) {}
    std::ptrdiff_t size() const { return n_; }
    double *data() const { return p_; }
    double &operator()(std::ptrdiff_t i) const { return p_[i]; }
    double &operator[](std::ptrdiff_t i) const { return p_[i]; }
    template <typename V>
    VectorView &operator=(const V &src) {
        if (static_cast<std::ptrdiff_t>(src.size()) != n_) throw std::invalid_argument("VectorView: size mismatch");
        for (std::ptrdiff_t i = 0; i < n_; ++i) p_[i] = src(i);
        return *this;
    }
    VectorView &operator=(const VectorView &src) {
        if (src.size() != n_) throw std::invalid_argument("VectorView: size mismatch");
        std::copy(src.p_, src.p_ + n_, p_);
        return *this;
    }

private:
    double *p_;
    std::ptrdiff_t n_;
};

class Vector {
public:
    Vector() = default;
    explicit Vector(std::ptrdiff_t n) : v_(static_cast<size_t>(n), 0.0) {}
    Vector(const VectorView &w) : v_(w.data(), w.data() + w.size()) {}
    std::ptrdiff_t size() const { return static_cast<std::ptrdiff_t>(v_.size()); }
    std::ptrdiff_t rows() const { return size(); }
    std::ptrdiff_t cols() const { return 1; }
    void resize(std::ptrdiff_t n) { v_.assign(static_cast<size_t>(n), 0.0); }
    double *data() { return v_.data(); }
    const double *data() const { return v_.data(); }
    double &operator()(std::ptrdiff_t i) { return v_[static_cast<size_t>(i)]; }
    double operator()(std::ptrdiff_t i) const { return v_[static_cast<size_t>(i)]; }
    double &operator[](std::ptrdiff_t i) { return v_[static_cast<size_t>(i)]; }
    double operator[](std::ptrdiff_t i) const { return v_[static_cast<size_t>(i)]; }
    Vector &setZero() { return setConstant(0.0); }
    Vector &setConstant(double a) {
        std::fill(v_.begin(), v_.end(), a);
        return *this;
    }
    VectorView head(std::ptrdiff_t k) { return VectorView(data(), k); }
    VectorView tail(std::ptrdiff_t k) { return VectorView(data() + size() - k, k); }
    VectorView segment(std::ptrdiff_t i, std::ptrdiff_t k) { return VectorView(data() + i, k); }
    Vector head(std::ptrdiff_t k) const { return Vector(v_.begin(), v_.begin() + k); }
    Vector tail(std::ptrdiff_t k) const { return Vector(v_.end() - k, v_.end()); }
    Vector segment(std::ptrdiff_t i, std::ptrdiff_t k) const { return Vector(v_.begin() + i, v_.begin() + i + k); }

private:
    template <typename It>
    Vector(It a, It b) : v_(a, b) {}
    std::vector<double> v_;
};

class Matrix {
public:
    Matrix() = default;
    Matrix(std::ptrdiff_t r, std::ptrdiff_t c) : r_(r), c_(c), v_(static_cast<size_t>(r * c), 0.0) {}
    std::ptrdiff_t rows() const { return r_; }
    std::ptrdiff_t cols() const { return c_; }
    std::ptrdiff_t size() const { return r_ * c_; }
    void resize(std::ptrdiff_t r, std::ptrdiff_t c) {
        r_ = r;
        c_ = c;
        v_.assign(static_cast<size_t>(r * c), 0.0);
    }
    double *data() { return v_.data(); }
    const double *data() const { return v_.data(); }
    double &operator()(std::ptrdiff_t i, std::ptrdiff_t j) { return v_[static_cast<size_t>(i + j * r_)]; }
    double operator()(std::ptrdiff_t i, std::ptrdiff_t j) const { return v_[static_cast<size_t>(i + j * r_)]; }
    Matrix &setZero() {
        std::fill(v_.begin(), v_.end(), 0.0);
        return *this;
    }
    Matrix &setIdentity() {
        setZero();
        for (std::ptrdiff_t i = 0; i < std::min(r_, c_); ++i) (*this)(i, i) = 1.0;
        return *this;
    }

private:
    std::ptrdiff_t r_ = 0, c_ = 0;
    std::vector<double> v_;
};

}  // namespace dense
}  // namespace pdplqr
