// Wave placement micro-benchmark (gfx950): where does the dispatcher put the
// waves of a latency-bound grid of 1024 one-wave blocks (one per SIMD wanted)
// after differently shaped preceding kernels, and do the remedies hold?
//   A  1024 blocks x 64 threads, ~250 VGPRs (two waves fit a SIMD)
//   B  the same blocks with the register file claimed whole (AGPR clobber)
//   C  256 blocks x 256 threads (4 waves, one problem each) + 96 KB dynamic LDS
//      (one block per CU): are a block's 4 waves on 4 distinct SIMDs?
// Each wave records (XCC, SE, SH, CU, SIMD) and spins ~50 us so that all of
// them are resident together.  Prints, per case and perturbation, the number
// of SIMDs holding 0 / 1 / 2+ waves.
// build: hipcc --offload-arch=gfx950 -O3 -o scripts/ubench/placement scripts/ubench/placement.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <map>
#include <vector>

#define CHECK(x)                                                                    \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            return 1;                                                               \
        }                                                                           \
    } while (0)

__device__ __forceinline__ int hw_place() {
    const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
    const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (3 << 11));
    return (int)(((xcc & 15u) << 16) | (((hw >> 13) & 7u) << 9) | (((hw >> 12) & 1u) << 8) | (((hw >> 8) & 15u) << 4) |
                 ((hw >> 4) & 3u));
}

__device__ __forceinline__ void spin(long long ticks) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

// ~250 arch VGPRs: two waves fit a SIMD (512 registers)
template <bool X1>
__global__ __launch_bounds__(64, 1) void k_one(int *out, long long ticks) {
    if constexpr (X1) asm volatile("; claim" ::: "a255");
    asm volatile("; pressure" ::: "v249");
    spin(ticks);
    if (threadIdx.x == 0) out[blockIdx.x] = hw_place();
}

__global__ __launch_bounds__(256, 1) void k_four(int *out, long long ticks) {
    asm volatile("; pressure" ::: "v249");
    spin(ticks);
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = hw_place();
}

// perturbation: a short kernel of G blocks of T threads
__global__ void k_perturb(double *p, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = p[i] * 1.0000001 + 1.0;
}

static void report(const char *tag, const std::vector<int> &pl, int simds) {
    std::map<int, int> cnt;
    for (int p : pl) cnt[p]++;
    int c1 = 0, c2 = 0;
    for (auto &kv : cnt) (kv.second == 1 ? c1 : c2)++;
    printf("%-28s simds used %4zu  one %4d  two+ %3d  idle %4d\n", tag, cnt.size(), c1, c2, simds - (int)cnt.size());
}

int main(int argc, char **argv) {
    const bool withB = argc > 1 && argv[1][0] == 'B';
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int simds = 4 * cus, W = simds;
    printf("CUs %d SIMDs %d\n", cus, simds);
    int *dout;
    double *buf;
    const int nb = 1 << 24;
    CHECK(hipMalloc(&dout, sizeof(int) * W));
    CHECK(hipMalloc(&buf, sizeof(double) * nb));
    CHECK(hipMemset(buf, 0, sizeof(double) * nb));
    CHECK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_four), hipFuncAttributeMaxDynamicSharedMemorySize,
                              96 * 1024));
    std::vector<int> host(W);
    const long long ticks = 5000;  // 50 us at 100 MHz
    const int pert[][2] = {{0, 0}, {1, 64}, {7, 256}, {100, 256}, {1000, 256}, {4096, 256}, {65536, 256}, {3, 1024}};
    for (auto &pp : pert) {
        for (int mode = 0; mode < 3; ++mode) {
            if ((mode == 1) != withB) continue;
            if (pp[0]) hipLaunchKernelGGL(k_perturb, dim3(pp[0]), dim3(pp[1]), 0, 0, buf, nb);
            if (mode == 0) hipLaunchKernelGGL(k_one<false>, dim3(W), dim3(64), 0, 0, dout, ticks);
            if (mode == 1) hipLaunchKernelGGL(k_one<true>, dim3(W), dim3(64), 0, 0, dout, ticks);
            if (mode == 2) hipLaunchKernelGGL(k_four, dim3(W / 4), dim3(256), 96 * 1024, 0, dout, ticks);
            CHECK(hipGetLastError());
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemcpy(host.data(), dout, sizeof(int) * W, hipMemcpyDeviceToHost));
            char tag[64];
            snprintf(tag, sizeof tag, "%s after %dx%d", mode == 0 ? "A one" : mode == 1 ? "B one+X1" : "C four+LDS",
                     pp[0], pp[1]);
            report(tag, host, simds);
        }
    }
    CHECK(hipFree(dout));
    CHECK(hipFree(buf));
    return 0;
}
