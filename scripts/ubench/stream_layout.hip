// Per-problem streaming pattern of the serial kernels, in isolation: one wave
// per problem walks N stage records from three arrays (+ one small write per
// stage), D stages of loads in flight.  Compares the boundary's problem-major
// layout [b][N][rec] with a stage-major layout [N][b][rec] (all waves of the
// batch then read one contiguous region per stage).  Dev tool:
//   hipcc --offload-arch=gfx950 -O3 -o stream_layout stream_layout.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int LAYOUT, int D>
__global__ __launch_bounds__(256) void k_stream(const double2 *__restrict__ a0, int r0, const double2 *__restrict__ a1,
                                                int r1, const double2 *__restrict__ a2, int r2, double2 *__restrict__ w,
                                                int rw, int P, int N, double *out) {
    const int p = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
    if (p >= P) return;
    auto at = [&](int k, int j, int r) -> size_t {
        return LAYOUT == 0 ? ((size_t)p * N + k) * r + j : ((size_t)k * P + p) * r + j;
    };
    double2 buf[D][6];
    auto load = [&](int d, int k) {
        k = k < N - 1 ? k : N - 1;
        buf[d][0] = a0[at(k, min(l, r0 - 1), r0)];
        buf[d][1] = a0[at(k, min(l + 64, r0 - 1), r0)];
        buf[d][2] = a1[at(k, min(l, r1 - 1), r1)];
        buf[d][3] = a1[at(k, min(l + 64, r1 - 1), r1)];
        buf[d][4] = a2[at(k, min(l, r2 - 1), r2)];
        buf[d][5] = a2[at(k, min(l + 64, r2 - 1), r2)];
    };
#pragma unroll
    for (int d = 0; d < D; ++d) load(d, d);
    double acc = 0.0;
    for (int k = 0; k < N; k += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
#pragma unroll
            for (int i = 0; i < 6; ++i) acc += buf[d][i].x * buf[d][i].y;
            if (l < rw) w[at(k + d, l, rw)] = make_double2(acc, (double)k);
            load(d, k + D + d);
        }
    }
    if (acc == 1234.5) out[0] = acc;
}

template <int LAYOUT, int D>
static float run(const double2 *a0, int r0, const double2 *a1, int r1, const double2 *a2, int r2, double2 *w, int rw,
                 int P, int N, double *o) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e9f;
    for (int r = 0; r < 5; ++r) {
        float ms;
        hipEventRecord(e0);
        hipLaunchKernelGGL((k_stream<LAYOUT, D>), dim3((P + 3) / 4), dim3(256), 0, 0, a0, r0, a1, r1, a2, r2, w, rw, P,
                           N, o);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        if (r && ms < best) best = ms;
    }
    return best;
}

int main() {
    const size_t st = (size_t)4096 * 1024;
    double2 *a0, *a1, *a2, *w;
    double *o;
    const size_t cap = st * 128 * 16;  // every array holds up to 128 16-byte chunks per stage
    if (hipMalloc(&a0, cap) || hipMalloc(&a1, cap) || hipMalloc(&a2, cap) || hipMalloc(&w, st * 34 * 16) ||
        hipMalloc(&o, 8))
        return 1;
    (void)hipMemset(a0, 0, cap);
    (void)hipMemset(a1, 0, cap);
    (void)hipMemset(a2, 0, cap);
    struct Pat {
        const char *name;
        int r0, r1, r2, rw, P;
    } pats[] = {{"forward E|c|rec, w", 96, 6, 34, 8, 4096},
                {"backward E|H+h|c, rec", 96, 76, 6, 34, 4096},
                {"backward reads only", 96, 76, 6, 0, 4096},
                {"forward reads only", 96, 6, 34, 0, 4096},
                {"backward, 2x problems (N/2)", 96, 76, 6, 34, 8192},
                {"backward, 4x problems (N/4)", 96, 76, 6, 34, 16384},
                {"backward reads only, 4x problems", 96, 76, 6, 0, 16384},
                {"full lines 128|128|128 chunks, no write", 128, 128, 128, 0, 4096}};
    for (const Pat &q : pats) {
        const int P = q.P, N = (int)(st / P);
        const double bytes = (double)st * 16.0 * (q.r0 + q.r1 + q.r2 + q.rw);
        float t[2][3];
        t[0][0] = run<0, 2>(a0, q.r0, a1, q.r1, a2, q.r2, w, q.rw, P, N, o);
        t[0][1] = run<0, 4>(a0, q.r0, a1, q.r1, a2, q.r2, w, q.rw, P, N, o);
        t[0][2] = run<0, 8>(a0, q.r0, a1, q.r1, a2, q.r2, w, q.rw, P, N, o);
        t[1][0] = run<1, 2>(a0, q.r0, a1, q.r1, a2, q.r2, w, q.rw, P, N, o);
        t[1][1] = run<1, 4>(a0, q.r0, a1, q.r1, a2, q.r2, w, q.rw, P, N, o);
        t[1][2] = run<1, 8>(a0, q.r0, a1, q.r1, a2, q.r2, w, q.rw, P, N, o);
        for (int L = 0; L < 2; ++L)
            for (int d = 0; d < 3; ++d)
                printf("{\"pattern\": \"%s\", \"layout\": \"%s\", \"depth\": %d, \"ms\": %.4f, \"gbs\": %.0f}\n",
                       q.name, L ? "stage-major [N][b]" : "problem-major [b][N]", 2 << d, t[L][d],
                       bytes / (t[L][d] * 1e-3) / 1e9);
    }
    return 0;
}
