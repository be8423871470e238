// kernels_rollout.hip -- batched control rollout (LQRKernel::forward_step,
// lqr_kernel.hpp:181-212) with the stage records streamed through an LDS-DMA
// ring.
//
// The rollout is a serial chain per problem (u_k needs x_k, x_{k+1} needs u_k),
// but everything it reads -- E_k, c_k and the rollout record
// FR_k = [L(:, 0:m) | lu'] -- is known before the chain starts.  One wavefront
// owns one problem and keeps D stage records in flight
// (global_load_lds_dwordx4, no VGPRs), so each stage's HBM latency is hidden
// behind the D-1 stages before it instead of being paid per stage.
//
// Per stage (lane (g, cl) = (lane >> 4, lane & 15)):
//   v   = lu' + Lxu^T x          lanes cl < m, rows 4 q + g, reduced over g
//   u   = -Luu^{-T} v            back substitution, u_i broadcast by readlane;
//                                B u accumulates on the fly (lanes g == 0)
//   x+  = c + A x + B u          lanes cl < n, columns split over g, reduced over g
// vmcnt accounting: each iteration issues exactly NI DMA + 1 store instructions,
// so "stage k has landed" is s_waitcnt vmcnt((NI + 1) (D - 1)).
//
// GAIN: the value-form backward's gain-form record FR_k = [K~ | k~]
// (kernels_schur.hip, K~ = Luu^{-T} Lxu^T, k~ = Luu^{-T} lu'), so
//   u = -(k~ + K~ x)                lanes cl < m, columns 4 q + g, reduced over g
// with no back substitution; 256 doubles per stage = exactly 2 DMA instructions.
#include "device_common.hpp"

#include <stdint.h>
#include <stdlib.h>

namespace pdplqr {

template <int NN, int MM, bool GAIN = false>
struct RollShape {
    static constexpr int n = NN, m = MM, s = NN + MM;
    static constexpr int FS = GAIN ? n * m + m : s * m + m;            // record doubles per stage
    static constexpr int OE = 0, OC = n * s, OF = OC + n, REC = OF + FS;  // doubles per stage
    static constexpr int CH = REC / 2;                                                  // 16-byte chunks
    static constexpr int NI = (CH + 63) / 64;
    static constexpr int TAIL = CH - (NI - 1) * 64;  // active lanes of the last DMA instruction
    static constexpr bool ok = (n * s) % 2 == 0 && n % 2 == 0 && FS % 2 == 0 && s <= 16 && NI >= 2 && NI <= 3;
};

#ifndef PDPLQR_ROLL_DEPTH
#define PDPLQR_ROLL_DEPTH 4
#endif

template <int NN, int MM, int D, bool GAIN = false, bool X1 = false>
__global__ __launch_bounds__(64) void k_rollout_dma(Shape sh, const double *__restrict__ E,
                                                    const double *__restrict__ c, const double *__restrict__ FR,
                                                    const double *__restrict__ x0, double *__restrict__ ws) {
    simd_exclusive<X1>();
    using SH = RollShape<NN, MM, GAIN>;
    constexpr int n = SH::n, m = SH::m, s = SH::s, NI = SH::NI;
    constexpr int NQ = (n + 3) / 4;  // row / column chunks of the x block over g
    static_assert(SH::ok, "rollout DMA layout");
    __shared__ __attribute__((aligned(16))) double ring[D][SH::REC];
    __shared__ double sx[16];
    const int lane = wave_lane(), g = lane >> 4, cl = lane & 15;
    const long long b = blockIdx.x;
    const int N = sh.N;
    const double *Eb = E + b * sh.perE;
    const double *cb = c + b * sh.perc;
    const double *Fb = FR + b * sh.perKD;
    double *wb = ws + b * sh.perh;

    auto dma = [&](int k, int slot) {
#pragma unroll
        for (int q = 0; q < NI; ++q) {
            if (q < NI - 1 || lane < SH::TAIL) {
                const int d = 2 * (q * 64 + lane);
                const double *src = d < SH::OC   ? Eb + (long long)k * (n * s) + d
                                    : d < SH::OF ? cb + (long long)k * n + (d - SH::OC)
                                                 : Fb + (long long)k * SH::FS + (d - SH::OF);
                dma16(src, &ring[slot][q * 128]);
            }
        }
    };

    if (lane < n) sx[lane] = x0[b * n + lane];
#pragma unroll
    for (int j = 0; j < D - 1; ++j) dma(j < N ? j : N - 1, j);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();

    for (int k = 0; k < N; ++k) {
        const int kp = k + D - 1;
        dma(kp < N ? kp : N - 1, kp % D);  // past the end: re-load into a consumed slot (keeps the count uniform)
        if (k < D - 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NI + 1) * (D - 1)) : "memory");
        const double *R = ring[k % D];
        const double *F = R + SH::OF;
        // ---- record reads (independent of the chain).  Addresses are
        // clamped instead of lane-predicated (no exec-mask branches); lanes
        // outside the valid range produce values nobody reads, except the
        // B u term, which only row group 0 may contribute to the sum over g.
        const int cm = cl < m ? cl : m - 1, cn = cl < n ? cl : n - 1;
        const double g0 = (g == 0) ? 1.0 : 0.0;
        double lxu[NQ], ex[NQ], eu[MM], luu[MM], xt[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int t = 4 * q + g, tc = t < n ? t : n - 1;
            const bool tv = (4 * q + 3 < n) || t < n;  // folds to true when n % 4 == 0
            const double l = GAIN ? F[cm * n + tc] : F[cm * s + m + tc], e = R[SH::OE + (m + tc) * n + cn];
            lxu[q] = tv ? l : 0.0;
            ex[q] = tv ? e : 0.0;
        }
#pragma unroll
        for (int i = 0; i < MM; ++i) {
            eu[i] = g0 * R[SH::OE + i * n + cn];
            luu[i] = GAIN ? 0.0 : F[cm * s + i];  // Luu[i][cl] (the record is zero above the diagonal)
        }
        const double lu = GAIN ? F[n * m + cm] : F[s * m + cm];  // k~ / lu'
        const double rdiag = GAIN ? 1.0 : 1.0 / F[cm * s + cm];
        const double cc = R[SH::OC + cn];
        // ---- chain ----
        const int lx = (lane >= m && lane < s) ? lane - m : 0;
        const double xk = sx[lx];  // w_k tail on lanes m..s-1
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int t = 4 * q + g;
            const bool tv = (4 * q + 3 < n) || t < n;
            const double x = sx[t < n ? t : 0];
            xt[q] = tv ? x : 0.0;
        }
        double v = 0.0, a = 0.0;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            v = __builtin_fma(lxu[q], xt[q], v);
            a = __builtin_fma(ex[q], xt[q], a);
        }
        v = sum_groups(v) + lu;
        double acc = 0.0, myu = 0.0;
        if constexpr (GAIN) {
#pragma unroll
            for (int i = 0; i < MM; ++i) {
                const double ui = readlane_f64(-v, i);  // u = -(k~ + K~ x), valid on lane cl == i
                if (cl == i) myu = ui;
                a = __builtin_fma(eu[i], ui, a);  // lanes g == 0: B[cl][i] u_i
            }
        } else
#pragma unroll
        for (int i = m - 1; i >= 0; --i) {
            const double ui = readlane_f64(-(v + acc) * rdiag, i);  // valid on lane cl == i
            if (cl == i) myu = ui;
            acc = __builtin_fma(luu[i], ui, acc);  // lanes cl < i: Luu[i][cl] u_i
            a = __builtin_fma(eu[i], ui, a);       // lanes g == 0: B[cl][i] u_i
        }
        a = sum_groups(a) + cc;
        // w_k = [u_k; x_k]: ONE store instruction per stage (vmcnt accounting above)
        if (lane < s) gstore(wb + (long long)k * s + lane, (lane < m) ? myu : xk);
        wave_sync();  // all reads of x_k done before it is overwritten
        if (g == 0 && cl < n) sx[cl] = a;
        wave_sync();
    }
    if (lane < n) wb[(long long)N * s + lane] = sx[lane];
}

static bool roll_aligned(const Shape &sh, const double *E, const double *c, const double *FR) {
    auto al = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    return al(E) && al(c) && al(FR) && sh.perE % 2 == 0 && sh.perc % 2 == 0 && sh.perKD % 2 == 0;
}

// PDPLQR_ERR_UNSUPPORTED: shape / alignment not covered, caller uses the generic rollout.
// gain: FR holds the gain-form record (only the 12/4 value-form backward writes
// it; no other rollout reads that format, so UNSUPPORTED is then an error).
int launch_rollout_dma(const Shape &sh, const double *E, const double *c, const double *FR, const double *x0,
                       double *ws, hipStream_t st, bool gain) {
    if (gain) {
        if (!(sh.n == 12 && sh.m == 4 && roll_aligned(sh, E, c, FR))) return PDPLQR_ERR_UNSUPPORTED;
        with_x1(sh.x1, [&](auto x1) {
            hipLaunchKernelGGL((k_rollout_dma<12, 4, PDPLQR_ROLL_DEPTH, true, decltype(x1)::value>), dim3(sh.batch),
                               dim3(64), 0, st, sh, E, c, FR, x0, ws);
        });
        PDPLQR_HIP_TRY(hipGetLastError());
        return PDPLQR_OK;
    }
    if (!roll_aligned(sh, E, c, FR)) return PDPLQR_ERR_UNSUPPORTED;
    if (sh.n == 12 && sh.m == 4)
        with_x1(sh.x1, [&](auto x1) {
            hipLaunchKernelGGL((k_rollout_dma<12, 4, PDPLQR_ROLL_DEPTH, false, decltype(x1)::value>), dim3(sh.batch),
                               dim3(64), 0, st, sh, E, c, FR, x0, ws);
        });
    else
        return PDPLQR_ERR_UNSUPPORTED;
    PDPLQR_HIP_TRY(hipGetLastError());
    return PDPLQR_OK;
}

}  // namespace pdplqr
