// clqr/typedefs.hpp -- numeric types of the pdpLQR C++ surface on MI355X.
//
// Drop-in for the reference header of the same name (include/clqr/typedefs.hpp):
// `lqr::scalar` is double and the dense types are Eigen's whenever
// <Eigen/Dense> is on the include path, so existing callers keep compiling.
// On a machine without Eigen (this build's toolchain image) the minimal
// column-major containers of clqr/detail/dense.hpp take their place; define
// PDPLQR_NO_EIGEN to force them, PDPLQR_USE_EIGEN to require Eigen.
#pragma once

#include <limits>

#if defined(PDPLQR_USE_EIGEN)
#define PDPLQR_HAVE_EIGEN 1
#elif !defined(PDPLQR_NO_EIGEN) && defined(__has_include)
#if __has_include(<Eigen/Dense>)
#define PDPLQR_HAVE_EIGEN 1
#endif
#endif

#ifdef PDPLQR_HAVE_EIGEN
#include <Eigen/Dense>
#else
#include "clqr/detail/dense.hpp"
#endif

namespace lqr {

using scalar = double;

#ifdef PDPLQR_HAVE_EIGEN
using VectorXs = Eigen::Matrix<scalar, Eigen::Dynamic, 1>;
using MatrixXs = Eigen::Matrix<scalar, Eigen::Dynamic, Eigen::Dynamic>;
using VectorMap = Eigen::Map<VectorXs>;
using MatrixMap = Eigen::Map<MatrixXs>;
using ConstVectorMap = Eigen::Map<const VectorXs>;
using ConstMatrixMap = Eigen::Map<const MatrixXs>;
using VectorRef = Eigen::Ref<VectorXs>;
using MatrixRef = Eigen::Ref<MatrixXs>;
using ConstVectorRef = Eigen::Ref<const VectorXs>;
using ConstMatrixRef = Eigen::Ref<const MatrixXs>;
#else
using VectorXs = pdplqr::dense::Vector;
using MatrixXs = pdplqr::dense::Matrix;
#endif

inline constexpr scalar LQR_INFTY = std::numeric_limits<scalar>::infinity();
inline constexpr scalar DIVISION_TOL = 1e-20;

}  // namespace lqr
