// Micro-benchmark of the KKT P = 16 serial factor loop structure (kkt.hip
// k_kkt_factor16) on synthetic tiles: cycles per group for variants.  Dev tool.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include "../../pdp-lqr_amd/csrc/combine_tiles.hpp"
using namespace pdplqr;

__device__ __forceinline__ d4 tn_load(const double *tile, int lane) { return *reinterpret_cast<const d4 *>(tile + 4 * lane); }
__device__ __forceinline__ void tn_store(double *tile, int lane, const d4 &v) {
    *(__attribute__((address_space(1))) d4 *)(tile + 4 * lane) = v;
}

template <int V>
__global__ __launch_bounds__(64) void k_f(const double *dpk, const double *dreg, double *fac, long long *cyc, int N) {
    const int lane = threadIdx.x, g = lane >> 4, c = lane & 15;
    const long long b = blockIdx.x;
    const double *tiles = dpk + b * (N + 1) * 512LL;
    const double *dg = dreg + b * (N + 1) * 16LL;
    WM<1> X;
    X.t[0][0] = d4{0.0, 0.0, 0.0, 0.0};
    d4 D1 = tn_load(tiles, lane), B1 = tn_load(tiles + 256, lane);
    d4 D2 = tn_load(tiles + 512, lane), B2 = tn_load(tiles + 768, lane);
    double r1[4], r2[4];
    for (int r = 0; r < 4; ++r) { r1[r] = dg[4 * r + g]; r2[r] = dg[16 + 4 * r + g]; }
    int fail = 0;
    long long t0 = clock64();
    for (int k = 0; k <= N; ++k) {
        WM<1> M, D;
        d4 B[1][2];
        D.t[0][0] = D1;
        B[0][0] = B1;
        for (int r = 0; r < 4; ++r) D.t[0][0][r] += (4 * r + g == c) ? r1[r] : 0.0;
        if (V != 2) {
            D1 = D2; B1 = B2;
            for (int r = 0; r < 4; ++r) r1[r] = r2[r];
            const int kn = min(k + 2, N);
            D2 = tn_load(tiles + kn * 512LL, lane);
            B2 = tn_load(tiles + kn * 512LL + 256, lane);
            for (int r = 0; r < 4; ++r) r2[r] = dg[kn * 16 + 4 * r + g];
        }
        if (k > 0) wm_tn<1>(M, X, X, 16, -1.0e-3, 0.0, &D, g, c);
        else M = D;
        for (int r = 0; r < 4; ++r) B[0][1][r] = (4 * r + g == c) ? 1.0 : 0.0;
        double colinv[1], rowinv[1][4];
        bool ok;
        if (V == 3) ok = elim_regs_n<1, true, 16, 2>(M, B, 16, colinv, rowinv, g, c);
        else ok = elim_regs<1, true, 2>(M, B, 16, colinv, rowinv, g, c);
        if (!ok && !fail) fail = k + 1;
        d4 Linv;
        for (int r = 0; r < 4; ++r) { X.t[0][0][r] = B[0][0][r] * rowinv[0][r]; Linv[r] = B[0][1][r] * rowinv[0][r]; }
        double *fk = fac + (b * (N + 1) + k) * 3LL * 256;
        if (V != 1) { tn_store(fk + 256, lane, X.t[0][0]); tn_store(fk + 512, lane, Linv); }
        else if (k == N) { tn_store(fk + 256, lane, X.t[0][0]); tn_store(fk + 512, lane, Linv); }
    }
    long long t1 = clock64();
    if (lane == 0) { cyc[b] = t1 - t0; fac[b] += fail; }
}

int main() {
    const int N = 512, B = 1024;
    std::vector<double> h((size_t)B * (N + 1) * 512);
    for (size_t t = 0; t < h.size(); ++t) {
        const int e = t % 512, lane = (e % 256) / 4, r = e % 4, i = 4 * r + (lane >> 4), j = lane & 15;
        h[t] = e < 256 ? ((i == j) ? 4.0 : 0.01 * ((i + j) % 5)) : 0.02 * ((i * 3 + j) % 7);
    }
    double *dpk, *dreg, *fac; long long *cyc;
    hipMalloc(&dpk, h.size() * 8); hipMalloc(&dreg, (size_t)B * (N + 1) * 16 * 8);
    hipMalloc(&fac, (size_t)B * (N + 1) * 768 * 8); hipMalloc(&cyc, B * 8);
    hipMemcpy(dpk, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    hipMemset(dreg, 0, (size_t)B * (N + 1) * 16 * 8);
    std::vector<long long> cy(B);
    const char *names[] = {"full", "no stores", "no loads", "compile-time n"};
    for (int v = 0; v < 4; ++v) {
        for (int pass = 0; pass < 2; ++pass) {
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            hipEventRecord(e0);
            if (v == 0) hipLaunchKernelGGL(k_f<0>, dim3(B), dim3(64), 0, 0, dpk, dreg, fac, cyc, N);
            if (v == 1) hipLaunchKernelGGL(k_f<1>, dim3(B), dim3(64), 0, 0, dpk, dreg, fac, cyc, N);
            if (v == 2) hipLaunchKernelGGL(k_f<2>, dim3(B), dim3(64), 0, 0, dpk, dreg, fac, cyc, N);
            if (v == 3) hipLaunchKernelGGL(k_f<3>, dim3(B), dim3(64), 0, 0, dpk, dreg, fac, cyc, N);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            if (pass) {
                hipMemcpy(cy.data(), cyc, B * 8, hipMemcpyDeviceToHost);
                std::sort(cy.begin(), cy.end());
                printf("%-16s %.3f ms, median %.0f cycles per group\n", names[v], ms, cy[B / 2] / (double)(N + 1));
            }
        }
    }
    return 0;
}
