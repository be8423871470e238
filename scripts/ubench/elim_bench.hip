// Micro-benchmark of the register elimination (combine_tiles.hpp elim_regs):
// one wave per SIMD factors a 16 x 16 SPD tile REP times; prints the median
// core-clock cycles per call (s_memtime) for several variants.  Dev tool only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include "../../pdp-lqr_amd/csrc/combine_tiles.hpp"
using namespace pdplqr;

__global__ __launch_bounds__(64) void k_elim2(const double *A, double *out, long long *cyc, int n, int rep) {
    const int lane = threadIdx.x, g = lane >> 4, c = lane & 15;
    WM<2> M0;
    wm_load<2>(M0, A, 32, n, false, 1.0, g, c);
    d4 acc = {0, 0, 0, 0};
    long long t0 = clock64();
    for (int it = 0; it < rep; ++it) {
        WM<2> M = M0, B = M0;
        M.t[0][0][0] += 1e-12 * it;
        double colinv[2], rowinv[2][4];
        bool ok = elim_regs<2, true>(M, B.t, n, colinv, rowinv, g, c);
        acc += M.t[1][1] + B.t[1][0] + (ok ? 0.0 : 1.0);
    }
    long long t1 = clock64();
    for (int r = 0; r < 4; ++r) out[blockIdx.x * 256 + lane * 4 + r] = acc[r];
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V>
__global__ __launch_bounds__(64) void k_elim(const double *A, double *out, long long *cyc, int n, int rep) {
    const int lane = threadIdx.x, g = lane >> 4, c = lane & 15;
    WM<1> M0;
    wm_load<1>(M0, A, 16, n, false, 1.0, g, c);
    d4 acc = {0, 0, 0, 0};
    long long t0 = clock64(); long long w0 = wall_clock64();
    for (int it = 0; it < rep; ++it) {
        WM<1> M = M0;
        M.t[0][0][0] += 1e-12 * it;
        double colinv[1], rowinv[1][4];
        d4 B[1][2];
        B[0][0] = M0.t[0][0];
        for (int r = 0; r < 4; ++r) B[0][1][r] = (4 * r + g == c) ? 1.0 : 0.0;
        bool ok;
        if (V == 0) ok = elim_regs<1, false, 1>(M, M.t, n, colinv, rowinv, g, c);
        else if (V == 1) ok = elim_regs<1, true, 2>(M, B, n, colinv, rowinv, g, c);
        else if (V == 2) ok = elim_regs_n<1, false, 16, 1>(M, M.t, n, colinv, rowinv, g, c);
        else ok = elim_regs_n<1, true, 16, 2>(M, B, n, colinv, rowinv, g, c);
        acc += M.t[0][0] + B[0][1] + (ok ? 0.0 : 1.0);
    }
    long long t1 = clock64(); long long w1 = wall_clock64();
    for (int r = 0; r < 4; ++r) out[blockIdx.x * 256 + lane * 4 + r] = acc[r];
    if (lane == 0) { cyc[blockIdx.x] = t1 - t0; cyc[blockIdx.x + 1024] = w1 - w0; }
}

int main() {
    const int n = 16, rep = 200, blocks = 1024;
    std::vector<double> A(256, 0.0);
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) A[i + 16 * j] = (i == j ? 20.0 : 0.0) + 1.0 / (1 + i + j);
    double *dA, *dout;
    long long *dc;
    hipMalloc(&dA, 256 * 8);
    hipMalloc(&dout, blocks * 256 * 8);
    hipMalloc(&dc, 2 * blocks * 8);
    hipMemcpy(dA, A.data(), 256 * 8, hipMemcpyHostToDevice);
    std::vector<long long> cy(2 * blocks);
    for (int v = 0; v < 4; ++v) {
        for (int pass = 0; pass < 2; ++pass) {
            if (v == 0) hipLaunchKernelGGL(k_elim<0>, dim3(blocks), dim3(64), 0, 0, dA, dout, dc, n, rep);
            else if (v == 1) hipLaunchKernelGGL(k_elim<1>, dim3(blocks), dim3(64), 0, 0, dA, dout, dc, n, rep);
            else if (v == 2) hipLaunchKernelGGL(k_elim<2>, dim3(blocks), dim3(64), 0, 0, dA, dout, dc, n, rep);
            else hipLaunchKernelGGL(k_elim<3>, dim3(blocks), dim3(64), 0, 0, dA, dout, dc, n, rep);
            hipDeviceSynchronize();
        }
        hipMemcpy(cy.data(), dc, 2 * blocks * 8, hipMemcpyDeviceToHost);
        std::sort(cy.begin(), cy.begin() + blocks);
        std::sort(cy.begin() + blocks, cy.end());
        printf("  wall ticks (100 MHz) per call %.1f -> clock %.0f MHz\n", cy[blocks + blocks / 2] / (double)rep, 100.0 * cy[blocks / 2] / cy[blocks + blocks / 2]);
        printf("variant %d: median %.0f cycles per call (%.0f per pivot)\n", v, cy[blocks / 2] / (double)rep,
               cy[blocks / 2] / (double)rep / n);
    }
    {
        std::vector<double> A2(1024, 0.0);
        for (int i = 0; i < 32; ++i)
            for (int j = 0; j < 32; ++j) A2[i + 32 * j] = (i == j ? 30.0 : 0.0) + 1.0 / (1 + i + j);
        double *dA2;
        hipMalloc(&dA2, 1024 * 8);
        hipMemcpy(dA2, A2.data(), 1024 * 8, hipMemcpyHostToDevice);
        for (int pass = 0; pass < 2; ++pass) {
            hipLaunchKernelGGL(k_elim2, dim3(blocks), dim3(64), 0, 0, dA2, dout, dc, 24, rep);
            hipDeviceSynchronize();
        }
        hipMemcpy(cy.data(), dc, blocks * 8, hipMemcpyDeviceToHost);
        std::sort(cy.begin(), cy.begin() + blocks);
        printf("T=2 n=24 AUG: median %.0f cycles per call (%.0f per pivot)\n", cy[blocks / 2] / (double)rep,
               cy[blocks / 2] / (double)rep / 24);
    }
    return 0;
}
