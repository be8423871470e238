// device_common.hpp -- device helpers shared by the Riccati kernels (gfx950).
//
// Everything here runs inside ONE wavefront that owns one problem (or one
// horizon segment): stage matrices live in the f64 MFMA C/D layout
// (v_mfma_f64_16x16x4_f64: lane l = 16 g + c holds rows g, g+4, g+8, g+12 of
// column c of a 16x16 tile), padded to P = 16 T.
#pragma once
#include "internal.hpp"

namespace pdplqr {

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ d4 mfma_f64(double a, double b, d4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// acc + sum of three MFMA products on independent accumulators, summed by
// VALU: a dependent f64 MFMA waits ~186 cycles for its predecessor's result,
// independent ones issue every 64 (scripts/ubench/lat_bench.hip), so a
// three-deep accumulation chain becomes one product deep plus two v_add_f64
// (different rounding order from the chain)
__device__ __forceinline__ d4 mfma_f64_x3(double a1, double b1, double a2, double b2, double a3, double b3,
                                          const d4 &acc) {
    const d4 z = {0.0, 0.0, 0.0, 0.0};
    const d4 p1 = mfma_f64(a1, b1, acc), p2 = mfma_f64(a2, b2, z), p3 = mfma_f64(a3, b3, z);
    return (p1 + p2) + p3;
}

// One wave per SIMD (X1).  A one-wave-per-problem kernel whose waves are
// latency-bound runs each problem's stage chain alone on a SIMD when the batch
// fits the device's SIMDs once -- but only if the hardware places the waves
// that way.  With <= 256 registers per wave a SIMD can host two of them, and
// the dispatcher does pair waves on one SIMD while another SIMD of the same CU
// idles (after some preceding kernels, e.g. update_problem_data's: measured
// 65-86 of 1024 SIMDs doubled, those waves 1.3x slower, the kernel span 1.5x;
// scripts/c5_placement.py).  X1 = true makes the wave
// claim the SIMD's whole register file (an AGPR clobber raises the kernel's
// register count past 256), so no second wave fits and the placement is one
// per SIMD by construction.  Launchers pick X1 when grid <= SIMDs (Shape::x1).
template <bool X1>
__device__ __forceinline__ void simd_exclusive() {
    if constexpr (X1) asm volatile("; one wave per SIMD" ::: "a255");
}

// Wave placement probe (diagnostic variant only, -DPDPLQR_HWID_PROBE=1): lane 0
// of every block records where it ran -- (XCC, SE, SH, CU, SIMD) from the
// HW_ID / XCC_ID hardware registers -- its start / end on the 100 MHz
// constant clock and on the shader clock counter (s_memtime: the effective
// core clock is their ratio) into a per-translation-unit device array, read
// back by pdplqr_probe_read_<tu>() (scripts/c5_placement.py).
#ifndef PDPLQR_HWID_PROBE
#define PDPLQR_HWID_PROBE 0
#endif
#if PDPLQR_HWID_PROBE
#define PDPLQR_PROBE_SLOTS 16384
#define PDPLQR_PROBE_FIELDS 5
static __device__ long long g_wave_probe[PDPLQR_PROBE_SLOTS * PDPLQR_PROBE_FIELDS];
#define PDPLQR_PROBE_DEFINE(tu)                                                                    \
    extern "C" int pdplqr_probe_read_##tu(long long *out) {                                       \
        return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_probe), sizeof(g_wave_probe), 0,   \
                                        hipMemcpyDeviceToHost);                                    \
    }
__device__ __forceinline__ long long hw_place() {
    // hwreg(id, offset 0, size 32): id | (size - 1) << 11
    const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));   // HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (3 << 11));  // XCC_ID[3:0]
    // simd [5:4], cu [11:8], sh [12], se [15:13]
    return (long long)(((xcc & 15u) << 16) | (((hw >> 13) & 7u) << 9) | (((hw >> 12) & 1u) << 8) |
                       (((hw >> 8) & 15u) << 4) | ((hw >> 4) & 3u));
}
#define PDPLQR_PROBE_BEGIN                                                                         \
    const long long probe_t0_ = wall_clock64();                                                    \
    const long long probe_c0_ = (long long)__builtin_amdgcn_s_memtime();
#define PDPLQR_PROBE_END(lane, blk)                                                                \
    if ((lane) == 0 && (blk) < PDPLQR_PROBE_SLOTS) {                                               \
        const long long c1_ = (long long)__builtin_amdgcn_s_memtime();                             \
        long long *q_ = g_wave_probe + PDPLQR_PROBE_FIELDS * (blk);                                \
        q_[0] = hw_place();                                                                        \
        q_[1] = probe_t0_;                                                                         \
        q_[2] = wall_clock64();                                                                    \
        q_[3] = probe_c0_;                                                                         \
        q_[4] = c1_;                                                                               \
    }
#else
#define PDPLQR_PROBE_DEFINE(tu)
#define PDPLQR_PROBE_BEGIN
#define PDPLQR_PROBE_END(lane, blk)
#endif

// packed lower (column-major) index of (i, j), i >= j, dimension d
__device__ __forceinline__ int pidx(int i, int j, int d) { return j * d - ((j * (j - 1)) >> 1) + (i - j); }

__device__ __forceinline__ double shfl_xor_f64(double v, int mask) { return __shfl_xor(v, mask, 64); }

// Loads the padded stage matrix H~ into C/D-layout tiles.  Indices in
// [lo, hi) map to the stored packed block (dimension dim, offset off);
// everything else is the identity padding.
template <int T>
__device__ __forceinline__ void load_M(d4 (&M)[T][T], const double *__restrict__ Hp, int dim, int off, int lo, int hi,
                                       int g, int c) {
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int b = 0; b < T; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * a + 4 * r + g, j = 16 * b + c;
                double v;
                if (i >= lo && i < hi && j >= lo && j < hi) {
                    const int ii = i - off, jj = j - off;
                    v = (ii >= jj) ? Hp[pidx(ii, jj, dim)] : Hp[pidx(jj, ii, dim)];
                } else {
                    v = (i == j) ? 1.0 : 0.0;
                }
                M[a][b][r] = v;
            }
}

// Wave-scope ordering of LDS traffic between lanes of ONE wavefront: LDS
// instructions of a wave retire in issue order, so a compiler-level barrier is
// all that is needed (no s_barrier; the workgroup is a single wave).
// threadIdx.x of a one-wavefront block, with its range made known to the
// compiler: index tests on g = lane >> 4 < 4 and c = lane & 15 then fold
// (without it, per-element masks on provably valid tile rows compile to
// exec-masked LDS loads and selects).
__device__ __forceinline__ int wave_lane() {
    const int l = threadIdx.x;
    __builtin_assume(l >= 0 && l < 64);
    return l;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Sum over the four row groups g of a column (lanes c, c+16, c+32, c+48),
// returned on all of them, with gfx950's v_permlane16/32_swap (VALU, no LDS
// round trip like ds_bpermute).  Each swap of two copies of v yields
// (v[l], v[l ^ 16]) in some order per lane; the fp add is commutative, so all
// four groups end with bit-identical sums.
__device__ __forceinline__ double sum_groups(double v) {
    int lo = __double2loint(v), hi = __double2hiint(v);
    auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    v = __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
    lo = __double2loint(v);
    hi = __double2hiint(v);
    a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    return __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
}

// Sum over the 16 lanes of a row (lanes 16 g .. 16 g + 15), returned on all of
// them, with DPP moves (VALU) instead of the four ds_bpermute round trips of an
// xor butterfly.  Bit-identical to v += shfl_xor(v, m) for m = 1, 2, 4, 8:
// quad_perm [1,0,3,2] / [2,3,0,1] are xor 1 / xor 2; after them a quad holds
// one value, and row_half_mirror (l -> 7 - l) / row_mirror (l -> 15 - l) flip
// bit 2 / bit 3 of the lane like xor 4 / xor 8 (the fp add is commutative).
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}

// Masked move: lanes of the DPP rows in ROWS (row = 16-lane group g) and
// banks in BANKS (bank = 4 consecutive lanes of a row) take v, the others keep
// old (quad_perm identity: no data crosses lanes).
template <int ROWS, int BANKS>
__device__ __forceinline__ double dpp_keep(double old, double v) {
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), 0xE4, ROWS, BANKS, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), 0xE4, ROWS, BANKS, false);
    return __hiloint2double(hi, lo);
}

// v[g] on the lanes of row group g (three masked moves instead of three
// selects of two v_cndmask each)
__device__ __forceinline__ double pick_group(const double (&v)[4]) {
    double r = v[0];
    r = dpp_keep<0x2, 0xF>(r, v[1]);
    r = dpp_keep<0x4, 0xF>(r, v[2]);
    r = dpp_keep<0x8, 0xF>(r, v[3]);
    return r;
}

__device__ __forceinline__ double sum_row16(double v) {
    v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp_f64<0x141>(v);  // row_half_mirror
    v += dpp_f64<0x140>(v);  // row_mirror
    return v;
}

// Status semantics of a value-function diagonal (P_k = Lxx Lxx^T): the
// reference's Eigen LLT stops at the first non-positive pivot and the
// remaining columns flow through unfactored (lqr_kernel.hpp:89,126 ignore
// info()), so a positive SEMIdefinite value function -- zero state cost,
// Q_N = 0 with sigma = 0 -- is a valid solve there and is not flagged here.
// Flagged: non-finite values, and diagonals below -PDPLQR_PSD_TOL (an
// indefinite stage matrix).  Control pivots (Muu) must stay positive.
#ifndef PDPLQR_PSD_TOL
#define PDPLQR_PSD_TOL 1e-8
#endif
// Bound below which the Neumann series P~ = sum_{j<8} (-rho_dyn P)^j P is used:
// with e = rho_dyn ||P||_F (>= the spectral radius of rho_dyn P for ANY
// symmetric P) the truncation after J terms is <= e^(J+1) / (1 - e) of ||P~||,
// so at e <= 0.015 eight terms leave < 4e-17.  Above it P~ is formed exactly.
#ifndef PDPLQR_KKT_NEUMANN_MAX
#define PDPLQR_KKT_NEUMANN_MAX 0.015
#endif

// dst[l ldc] = fma(-f, src[l], dst[l ldc]) for l = l0, l0 + st, ... <= lend, in
// groups of four whose loads all precede their stores: the read-modify-writes
// of one LDS array may alias as far as the compiler knows, so written one at a
// time each waits for the previous store (two LDS round trips per entry).
__device__ __forceinline__ void lds_axpy_strided(double *dst, int ldc, const double *src, double f, int l0, int lend,
                                                 int st, int lds = 1) {
    constexpr int G = 4;
    int l = l0;
    for (; l + (G - 1) * st <= lend; l += G * st) {
        double sv[G], dv[G];
#pragma unroll
        for (int u = 0; u < G; ++u) {
            sv[u] = src[(l + u * st) * lds];
            dv[u] = dst[(l + u * st) * ldc];
        }
#pragma unroll
        for (int u = 0; u < G; ++u) dst[(l + u * st) * ldc] = __builtin_fma(-f, sv[u], dv[u]);
    }
    for (; l <= lend; l += st) dst[l * ldc] = __builtin_fma(-f, src[l * lds], dst[l * ldc]);
}

// Two pivots (j, j + 1) of a right-looking elimination in one pass over row
// dst (entries l = l0, l0 + st, ... <= lend, ld ldc): with c0 = column j and
// c1 = column j + 1 before either pivot, a1j = M(j + 1, j), f0 = M(i, j) / d_j
// and f1 = M'(i, j + 1) / d'_{j + 1},
//     t = M(i, l) - f0 M(l, j),  M'(l, j + 1) = M(l, j + 1) - (M(l, j) / d_j) M(j + 1, j),
//     M(i, l) = t - f1 M'(l, j + 1)
// -- the fmas of the two sequential steps, in their order (bit-identical),
// loads of four entries before their stores.
__device__ __forceinline__ void lds_axpy2_strided(double *dst, int ldc, const double *c0, const double *c1, double f0,
                                                  double f1, double inv0, double a1j, int l0, int lend, int st) {
    constexpr int G = 4;
    int l = l0;
    for (; l + (G - 1) * st <= lend; l += G * st) {
        double x0[G], x1[G], dv[G];
#pragma unroll
        for (int u = 0; u < G; ++u) {
            x0[u] = c0[l + u * st];
            x1[u] = c1[l + u * st];
            dv[u] = dst[(l + u * st) * ldc];
        }
#pragma unroll
        for (int u = 0; u < G; ++u) {
            const double t = __builtin_fma(-f0, x0[u], dv[u]);
            const double al = __builtin_fma(-(x0[u] * inv0), a1j, x1[u]);
            dst[(l + u * st) * ldc] = __builtin_fma(-f1, al, t);
        }
    }
    for (; l <= lend; l += st) {
        const double t = __builtin_fma(-f0, c0[l], dst[l * ldc]);
        const double al = __builtin_fma(-(c0[l] * inv0), a1j, c1[l]);
        dst[l * ldc] = __builtin_fma(-f1, al, t);
    }
}

__device__ __forceinline__ bool psd_bad(double v) { return !(v >= -PDPLQR_PSD_TOL && v < 1.0e300); }

__device__ __forceinline__ double readlane_f64(double v, int lane) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}

// LDS-DMA of 16 bytes per lane: LDS[lds_base + 16 lane] <- *src
// (global_load_lds_dwordx4; lds_base is the wave-uniform LDS byte address).
// Issued through inline asm on purpose: the compiler's waitcnt insertion
// treats every later ds_read of the same LDS object as aliasing an in-flight
// builtin DMA and puts s_waitcnt vmcnt(0) in front of it, which serialises the
// prefetch.  Callers own the vmcnt accounting (loads retire in issue order).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is reserved; it is only live inside this asm
__device__ __forceinline__ void dma16(const void *src, const void *lds_dst) {
    const uint32_t base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)lds_dst;
    asm volatile(
        "s_mov_b32 m0, %1\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %0, off" ::"v"(src),
        "s"(__builtin_amdgcn_readfirstlane(base))
        : "memory", "m0");
}
#pragma clang diagnostic pop

// Stores through an explicit global (addrspace 1) pointer.  A store through a
// generic pointer keeps a flat memory operand, and the waitcnt pass then puts
// s_waitcnt vmcnt(0) before every later ds_read (the store "may write LDS"),
// which drains the DMA prefetch queue.
__device__ __forceinline__ void gstore(double *p, double v) { *(__attribute__((address_space(1))) double *)p = v; }
typedef double d2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void gstore2(double *p, d2v v) { *(__attribute__((address_space(1))) d2v *)p = v; }

// 1/sqrt(x): hardware estimate (v_rsq_f64, relative error <= 2^-24, measured
// by tests/test_gpu_combine.py) refined by ONE third-order step
//     r' = r (1 + e/2 + 3 e^2/8),  e = 1 - x r^2
// which cubes the error (full fp64 accuracy) at dependency depth 4, against
// depth 6 for two Newton steps: this sits on every pivot's critical path.
__device__ __forceinline__ double rsqrt_f64(double x) {
    const double r = __builtin_amdgcn_rsq(x);
    const double e = __builtin_fma(-x * r, r, 1.0);
    const double p = __builtin_fma(e, 0.375, 0.5);
    return __builtin_fma(r * e, p, r);
}

// 1/x: hardware estimate (v_rcp_f64) refined by one third-order step
//     r' = r (1 + e + e^2),  e = 1 - x r
// (error cubed: full fp64 accuracy from the ~2^-24 estimate), depth 3.
__device__ __forceinline__ double rcp_f64(double x) {
    const double r = __builtin_amdgcn_rcp(x);
    const double e = __builtin_fma(-x, r, 1.0);
    return __builtin_fma(r, __builtin_fma(e, e, e), r);
}

// Stage-k inputs of one lane, loaded one stage ahead (register prefetch).
template <int T>
struct StageIn {
    double E[4 * T][T];  // MFMA B operand: E[4 cc + g][16 b + c]
    d4 H[T][T];          // MFMA C input: H~[16 a + 4 r + g][16 b + c] (padded)
    double c[4 * T];     // c[4 cc + g]
    double h[T];         // h~[16 b + c]
};

template <int T>
__device__ __forceinline__ void load_stage(StageIn<T> &in, const double *__restrict__ Ek, const double *__restrict__ ck,
                                           const double *__restrict__ Hk, const double *__restrict__ hk, int n,
                                           int s, int g, int c) {
#pragma unroll
    for (int cc = 0; cc < 4 * T; ++cc) {
        const int t = 4 * cc + g;
#pragma unroll
        for (int b = 0; b < T; ++b) {
            const int j = 16 * b + c;
            in.E[cc][b] = (t < n && j < s) ? Ek[t + j * n] : 0.0;
        }
        in.c[cc] = (t < n) ? ck[t] : 0.0;
    }
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int b = 0; b < T; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * a + 4 * r + g, j = 16 * b + c;
                double v;
                if (i < s && j < s)
                    v = (i >= j) ? Hk[pidx(i, j, s)] : Hk[pidx(j, i, s)];
                else
                    v = (i == j) ? 1.0 : 0.0;
                in.H[a][b][r] = v;
            }
#pragma unroll
    for (int b = 0; b < T; ++b) {
        const int j = 16 * b + c;
        in.h[b] = (j < s) ? hk[j] : 0.0;
    }
}

// Position of row/column index i in the pivot broadcast buffer: the 4T rows a
// lane owns (16 a + 4 r + g) are contiguous, so a lane fetches them with
// 128-bit LDS reads.
template <int T>
__device__ __forceinline__ constexpr int colpos(int i) {
    return (i & 3) * (4 * T) + ((i >> 4) << 2) + ((i >> 2) & 3);
}

// Eigen's LLT stop, restated for the right-looking elimination below.  Eigen
// factors small matrices left-looking (llt_inplace::unblocked; the oracle's
// llt_lower, pdplqr_oracle.c:97-116): when the reduced pivot of column j is
// <= 0 it returns with column j and every later column still holding their
// ORIGINAL values, and the reference uses that lower triangle as L
// (lqr_kernel.hpp:89,126 ignore info()).  The right-looking loop has already
// applied the rank-1 updates of the live pivots p < j to that trailing block,
// so they are undone here, in reverse order, with the same products: row p of
// the matrix is still the raw (unscaled) pivot row, 1/d_p = sinv[p]^2.  Only
// the block (i, l >= j) is restored; columns < j keep their factor values.
template <int T>
__device__ __forceinline__ void chol_restore_tail(d4 (&M)[T][T], double *cb, const double *sinv, int jbeg,
                                                            int jdead, int g, int c) {
    double *myslot = cb + g * 16 * T;
#pragma unroll
    for (int tr = T - 1; tr >= 0; --tr)
#pragma unroll
        for (int rr = 3; rr >= 0; --rr) {
#pragma unroll 1
            for (int gj = 3; gj >= 0; --gj) {
                const int p = 16 * tr + 4 * rr + gj;
                if (p < jbeg || p >= jdead) continue;
#pragma unroll
                for (int b = 0; b < T; ++b) {
                    const int jc = 16 * b + c;
                    myslot[colpos<T>(jc)] = (jc > p) ? M[tr][b][rr] : 0.0;
                }
                wave_sync();
                const double *slot = cb + gj * 16 * T;
                const double inv = sinv[p];
                const double inv2 = inv * inv;
                double lc[T];
#pragma unroll
                for (int b = 0; b < T; ++b) {
                    const int jc = 16 * b + c;
                    lc[b] = (jc >= jdead) ? slot[colpos<T>(jc)] * inv2 : 0.0;
                }
#pragma unroll
                for (int a = 0; a < T; ++a)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int i = 16 * a + 4 * r + g;
                        const double li = (i >= jdead) ? slot[colpos<T>(i)] : 0.0;
#pragma unroll
                        for (int b = 0; b < T; ++b) M[a][b][r] = __builtin_fma(li, lc[b], M[a][b][r]);
                    }
                wave_sync();
            }
        }
}

// Right-looking Cholesky of the symmetric padded matrix in C/D layout, pivots
// jbeg..jend-1.  Column j is broadcast through LDS from row j (the row group
// that owns row j holds M[j][*] = M[*][j]; M stays exactly symmetric because
// every update is applied to both triangles with the same products).  The
// owners write zeros for columns <= j, so every lane can update
// M -= raw_i raw_k / M[j][j] without masking; the pivot column itself is left
// unscaled and finalised by finalize_L (L[i][j] = M[i][j] / sqrt(M[j][j]),
// the reciprocal square roots are kept in sinv).  With `aug`, the first `m`
// pivots also eliminate the linear column lpr (the lp_k of
// lqr_kernel.hpp:142-146): lpr_i -= l_ij lu'_j with lu'_j = lp_j / L_jj, which
// is exactly lu <- Luu^{-1} lu followed by p -= Lxu lu.  All lanes of the
// wave run in lock step and LDS ops of one wave retire in order, so no
// barrier is needed between the owners' writes and the readers.
// Returns true if every pivot was positive.
template <int T>
__device__ __forceinline__ bool chol_tiles(d4 (&M)[T][T], double (&lpr)[T][4], double *cb, double *sinv, double *luq,
                                           int jbeg, int jend, int m, bool aug, int g, int c) {
    bool ok = true, live = true;
    int jdead = jend;  // first state pivot <= 0 (wave-uniform)
    // cb holds one 16 T slot per row group: every group writes its own row
    // (no exec-mask branch), readers take the pivot's group slot
    double *myslot = cb + g * 16 * T;
    // pivot j = 16 tr + 4 rr + gj: (tr, rr) unrolled so register indices stay
    // compile-time, the row group gj is a runtime loop (keeps the scheduler
    // from hoisting work across all pivots, which would exhaust registers)
#pragma unroll
    for (int tr = 0; tr < T; ++tr)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
#pragma unroll 1
            for (int gj = 0; gj < 4; ++gj) {
                const int j = 16 * tr + 4 * rr + gj;
                if (j < jbeg || j >= jend) continue;
#pragma unroll
                for (int b = 0; b < T; ++b) {
                    const int jc = 16 * b + c;
                    myslot[colpos<T>(jc)] = (jc > j) ? M[tr][b][rr] : 0.0;
                }
                wave_sync();
                const double *slot = cb + gj * 16 * T;
                const double2 *rows = reinterpret_cast<const double2 *>(slot + g * 4 * T);
                const double djj = readlane_f64(M[tr][tr][rr], (gj << 4) + (j & 15));
                // control pivots (j < m) must be positive; a state pivot <= 0
                // stops the factorisation as Eigen's LLT does (the remaining
                // columns stay unfactored, unscaled), flagged only if clearly
                // negative or not finite (psd_bad)
                ok = ok && (j < m ? djj > 0.0 : !psd_bad(djj));
                if (live && !(j < m || djj > 0.0)) jdead = j;
                live = live && (j < m || djj > 0.0);
                const double inv = live ? rsqrt_f64(djj) : 0.0;
                const double inv2 = inv * inv;
                sinv[j] = live ? inv : 1.0;  // all lanes, same value: no branch
                double lc[T];
#pragma unroll
                for (int b = 0; b < T; ++b) lc[b] = slot[colpos<T>(16 * b + c)] * inv2;
                const bool augj = aug && j < m;
                const double lpj = augj ? readlane_f64(lpr[tr][rr], gj << 4) : 0.0;
                const double qj = lpj * inv2;
                double li[T][4];
#pragma unroll
                for (int q = 0; q < 2 * T; ++q) {
                    const double2 v = rows[q];
                    li[q >> 1][(q & 1) * 2] = v.x;
                    li[q >> 1][(q & 1) * 2 + 1] = v.y;
                }
#pragma unroll
                for (int a = 0; a < T; ++a)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
#pragma unroll
                        for (int b = 0; b < T; ++b) M[a][b][r] = __builtin_fma(-li[a][r], lc[b], M[a][b][r]);
                        // q = lp_j / M[j][j]; lpr_i -= raw_i * q  (raw_i = 0 for i <= j)
                        if (augj) lpr[a][r] = __builtin_fma(-li[a][r], qj, lpr[a][r]);
                    }
                if (augj) luq[j] = lpj * inv;  // uniform condition, all lanes
                wave_sync();
            }
        }
    if (jdead < jend) chol_restore_tail<T>(M, cb, sinv, jbeg, jdead, g, c);  // rare, wave-uniform
    return ok;
}

// L[i][jc] = M[i][jc] / sqrt(M[jc][jc]) below the diagonal, 0 above, for the
// factored columns jbeg <= jc < jend; identity padding elsewhere is left as is.
template <int T>
__device__ __forceinline__ void finalize_L(d4 (&M)[T][T], const double *sinv, int jbeg, int jend, int g, int c) {
#pragma unroll
    for (int b = 0; b < T; ++b) {
        const int jc = 16 * b + c;
        if (jc >= jbeg && jc < jend) {
            const double iv = sinv[jc];
#pragma unroll
            for (int a = 0; a < T; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * a + 4 * r + g;
                    M[a][b][r] = (i >= jc) ? M[a][b][r] * iv : 0.0;
                }
        }
    }
}

template <int T>
struct BwdSmem {
    static constexpr int P = 16 * T;
    static constexpr int LD = P + 1;  // odd leading dimension: conflict-free column reads
    double L[P * LD];                 // L_{k+1} then L_k (padded, column-major, lower, zero upper)
    alignas(16) double col[4 * P];    // Cholesky pivot-row broadcast, one slot per row group (colpos order)
    double inv[P];                    // 1 / sqrt(pivot) per column
    double pbt[P];                    // Pb_tmp = Lxx_next^T c
    double pv[P];                     // p_{k+1}, then p_k
    double lp[P];                     // lp_k (column -> row redistribution)
    double luq[P];                    // lu'_k = Luu^{-1} lu
};

template <int T>
__device__ __forceinline__ void store_L_lds(const d4 (&M)[T][T], double *L, int g, int c) {
    constexpr int LD = 16 * T + 1;
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
        for (int b = 0; b < T; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) L[(16 * a + 4 * r + g) + (16 * b + c) * LD] = M[a][b][r];
}


// One backward stage k (LQRKernel::step_with_factorization, lqr_kernel.hpp:104-147)
// on the padded tiles.  Consumes L_{k+1} (sm.L) and p_{k+1} (sm.pv); produces
// L_k in M (finalised) and sm.L, p_k in sm.pv, lu'_k = Luu^{-1} lu in sm.luq,
// lp_k in lpr (rows of the lane).  Returns false on a non-positive pivot.
template <int T>
__device__ __forceinline__ bool riccati_stage(BwdSmem<T> &sm, const StageIn<T> &cur, d4 (&M)[T][T],
                                             double (&lpr)[T][4], int n, int m, int s, int g, int c) {
    constexpr int LD = 16 * T + 1;
    const int nch = (n + 3) >> 2;
        // ---- A operand: Lxx_next^T, read from LDS (L_{k+1}) ----
        double av[4 * T][T];
#pragma unroll
        for (int cc = 0; cc < 4 * T; ++cc) {
            const int t = 4 * cc + g;
#pragma unroll
            for (int a = 0; a < T; ++a) {
                const int tp = 16 * a + c;
                av[cc][a] = (cc < nch && t < n && tp < n) ? sm.L[(m + t) + (m + tp) * LD] : 0.0;
            }
        }
        // ---- W = Lxx_next^T E  (= V^T, V = E^T Lxx_next, lqr_kernel.hpp:121) ----
        d4 W[T][T];
#pragma unroll
        for (int a = 0; a < T; ++a)
#pragma unroll
            for (int bt = 0; bt < T; ++bt) W[a][bt] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int cc = 0; cc < 4 * T; ++cc)
            if (cc < nch)
#pragma unroll
                for (int a = 0; a < T; ++a)
#pragma unroll
                    for (int bt = 0; bt < T; ++bt) W[a][bt] = mfma_f64(av[cc][a], cur.E[cc][bt], W[a][bt]);
        // ---- Pb_tmp = Lxx_next^T c (lqr_kernel.hpp:138), reduced over row groups ----
#pragma unroll
        for (int a = 0; a < T; ++a) {
            double part = 0.0;
#pragma unroll
            for (int cc = 0; cc < 4 * T; ++cc)
                if (cc < nch) part = __builtin_fma(av[cc][a], cur.c[cc], part);
            part += shfl_xor_f64(part, 16);
            part += shfl_xor_f64(part, 32);
            if (g == 0) sm.pbt[16 * a + c] = part;
        }
        // ---- M = H~ + W^T W  (= H~ + V V^T, lqr_kernel.hpp:123-124) ----
#pragma unroll
        for (int a = 0; a < T; ++a)
#pragma unroll
            for (int bt = 0; bt < T; ++bt) M[a][bt] = cur.H[a][bt];
#pragma unroll
        for (int kc = 0; kc < 4 * T; ++kc)
            if (kc < nch) {
                const int ka = kc >> 2, r = kc & 3;
#pragma unroll
                for (int a = 0; a < T; ++a)
#pragma unroll
                    for (int bt = 0; bt < T; ++bt) M[a][bt] = mfma_f64(W[ka][a][r], W[ka][bt][r], M[a][bt]);
            }
        // ---- lp = h~ + E^T (Lxx_next Pb_tmp + p_next) = h~ + W^T Pb_tmp + E^T p_next
        //      (lqr_kernel.hpp:139-143; E^T Lxx_next = W^T) ----
        wave_sync();
        {
            double part[T];
#pragma unroll
            for (int bt = 0; bt < T; ++bt) part[bt] = 0.0;
#pragma unroll
            for (int kc = 0; kc < 4 * T; ++kc)
                if (kc < nch) {
                    const int t = 4 * kc + g;
                    const double pb = (t < n) ? sm.pbt[t] : 0.0;
                    const double pn = (t < n) ? sm.pv[t] : 0.0;
#pragma unroll
                    for (int bt = 0; bt < T; ++bt) {
                        part[bt] = __builtin_fma(W[kc >> 2][bt][kc & 3], pb, part[bt]);
                        part[bt] = __builtin_fma(cur.E[kc][bt], pn, part[bt]);
                    }
                }
#pragma unroll
            for (int bt = 0; bt < T; ++bt) {
                part[bt] += shfl_xor_f64(part[bt], 16);
                part[bt] += shfl_xor_f64(part[bt], 32);
                if (g == 0) sm.lp[16 * bt + c] = cur.h[bt] + part[bt];
            }
            wave_sync();
#pragma unroll
            for (int a = 0; a < T; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * a + 4 * r + g;
                    lpr[a][r] = (i < s) ? sm.lp[i] : 0.0;
                }
        }
        // ---- L = chol(M) (lqr_kernel.hpp:126) with lu <- Luu^{-1} lu, p -= Lxu lu (:145-146) ----
        const bool ok = chol_tiles<T>(M, lpr, sm.col, sm.inv, sm.luq, 0, s, m, true, g, c);
        finalize_L<T>(M, sm.inv, 0, s, g, c);
        store_L_lds<T>(M, sm.L, g, c);
        // p_k -> LDS (next stage's p_next)
        if (c == 0) {
#pragma unroll
            for (int a = 0; a < T; ++a)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * a + 4 * r + g;
                    if (i >= m && i < s) sm.pv[i - m] = lpr[a][r];
                }
        }
        wave_sync();
        return ok;
}

}  // namespace pdplqr
