// clqr/lqr/qdldl_typedefs.hpp -- the CSC / workspace types of the reference's
// QDLDL boundary (include/clqr/lqr/qdldl_typedefs.hpp:8-39 there), for callers
// that use the public KKT accessors (KKTSystem::get_KKT_csc_matrix,
// QDLDLSolver::create_workspace).  The reference takes QDLDL_int / QDLDL_float /
// QDLDL_bool from the QDLDL library's header; this build does not link QDLDL
// (its KKT factorisation runs on the GPU, csrc/kkt.hip), so when <qdldl/qdldl.h>
// is absent they default to QDLDL's default build types (long long, double,
// unsigned char).
#pragma once

#include <memory>

#if defined(__has_include)
#if __has_include(<qdldl/qdldl.h>)
#include <qdldl/qdldl.h>
#define PDPLQR_HAVE_QDLDL 1
#endif
#endif

#ifndef PDPLQR_HAVE_QDLDL
typedef long long QDLDL_int;
typedef double QDLDL_float;
typedef unsigned char QDLDL_bool;
#endif

namespace lqr {

struct CscMatrix {
    QDLDL_int m;           // number of rows
    QDLDL_int n;           // number of cols
    const QDLDL_int *p;    // column pointers (read-only)
    const QDLDL_int *i;    // row indices (read-only)
    const QDLDL_float *x;  // nonzero values (read-only)
    QDLDL_int nzmax;       // number of nonzeros
};

struct QDLDLData {
    // data for L and D factors
    QDLDL_int Ln;
    std::unique_ptr<QDLDL_int[]> Lp;
    std::unique_ptr<QDLDL_int[]> Li;
    std::unique_ptr<QDLDL_float[]> Lx;
    std::unique_ptr<QDLDL_float[]> D;
    std::unique_ptr<QDLDL_float[]> Dinv;
    // data for elim tree calculation
    std::unique_ptr<QDLDL_int[]> etree;
    std::unique_ptr<QDLDL_int[]> Lnz;
    QDLDL_int sumLnz;
    // working data for factorisation
    std::unique_ptr<QDLDL_int[]> iwork;
    std::unique_ptr<QDLDL_bool[]> bwork;
    std::unique_ptr<QDLDL_float[]> fwork;
    // data for results of A\b
    std::unique_ptr<QDLDL_float[]> x;
};

}  // namespace lqr
