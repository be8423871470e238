// Per-problem streaming pattern of the serial kernels, in isolation: one wave
// per problem walks N stage records from three arrays (+ one small write per
// stage), D stages of loads in flight.  Compares the boundary's problem-major
// layout [b][N][rec] with a stage-major layout [N][b][rec] (all waves of the
// batch then read one contiguous region per stage).  Dev tool:
//   hipcc --offload-arch=gfx950 -O3 -o stream_layout stream_layout.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double nd2 __attribute__((ext_vector_type(2)));

template <int LAYOUT, int D, int WM = 0>
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
            const double2 v = make_double2(acc, (double)k);
            if (WM == 0) {
                if (l < rw) w[at(k + d, l, rw)] = v;
            } else if (WM == 1) {
                if (l < rw) __builtin_nontemporal_store(nd2{v.x, v.y}, reinterpret_cast<nd2 *>(&w[at(k + d, l, rw)]));
            } else if (WM == 2) {
                if (l < rw) w[((size_t)(k + d) * P + p) * rw + l] = v;
            } else if (d == D - 1) {  // WM 3/4: one contiguous write of the last D stages' records
                for (int j = l; j < D * rw; j += 64) {
                    double2 *q = &w[at(k, 0, rw) + j];
                    if (WM == 3) *q = v; else __builtin_nontemporal_store(nd2{v.x, v.y}, reinterpret_cast<nd2 *>(q));
                }
            }
            load(d, k + D + d);
        }
    }
    if (acc == 1234.5) out[0] = acc;
}

template <int LAYOUT, int D, int WM = 0>
static float run(const double2 *a0, int r0, const double2 *a1, int r1, const double2 *a2, int r2, double2 *w, int rw,
                 int P, int N, double *o) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e9f;
    for (int r = 0; r < 5; ++r) {
        float ms;
        hipEventRecord(e0);
        hipLaunchKernelGGL((k_stream<LAYOUT, D, WM>), dim3((P + 3) / 4), dim3(256), 0, 0, a0, r0, a1, r1, a2, r2, w, rw, P,
                           N, o);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        if (r && ms < best) best = ms;
    }
    return best;
}

int main(int argc, char **argv) {
    const bool sweep_layout = argc < 2;
    const size_t st = (size_t)4096 * 1024;
    double2 *a0, *a1, *a2, *w;
    double *o;
    const size_t cap = st * 128 * 16;  // every array holds up to 128 16-byte chunks per stage
    if (hipMalloc(&a0, cap) || hipMalloc(&a1, cap) || hipMalloc(&a2, cap) || hipMalloc(&w, st * 64 * 16) ||
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
        if (!sweep_layout) break;
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
    const char *wm_name[] = {"per-stage store", "per-stage nontemporal store", "stage-major output",
                             "4-stage batched store", "4-stage batched nontemporal"};
    if (argc > 1 && argv[1][0] == 'r') {  // record-size sweep of the backward pattern
        const int P = 4096, N = 1024;
        for (int rw : {0, 8, 16, 26, 31, 32, 34, 36, 40, 48, 64}) {
            const double bytes = (double)st * 16.0 * (96 + 76 + 6 + rw);
            const float t = run<0, 4, 0>(a0, 96, a1, 76, a2, 6, w, rw, P, N, o);
            printf("{\"pattern\": \"backward\", \"record_bytes\": %d, \"ms\": %.4f, \"gbs\": %.0f}\n", 16 * rw, t,
                   bytes / (t * 1e-3) / 1e9);
        }
        return 0;
    }
    for (int pi = 0; pi < 2; ++pi) {
        const Pat &q = pats[pi];
        const int P = q.P, N = (int)(st / P);
        const double bytes = (double)st * 16.0 * (q.r0 + q.r1 + q.r2 + q.rw);
        float t[5];
        t[0] = run<0, 4, 0>(a0, q.r0, a1, q.r1, a2, q.r2, w, q.rw, P, N, o);
        t[1] = run<0, 4, 1>(a0, q.r0, a1, q.r1, a2, q.r2, w, q.rw, P, N, o);
        t[2] = run<0, 4, 2>(a0, q.r0, a1, q.r1, a2, q.r2, w, q.rw, P, N, o);
        t[3] = run<0, 4, 3>(a0, q.r0, a1, q.r1, a2, q.r2, w, q.rw, P, N, o);
        t[4] = run<0, 4, 4>(a0, q.r0, a1, q.r1, a2, q.r2, w, q.rw, P, N, o);
        for (int m = 0; m < 5; ++m)
            printf("{\"pattern\": \"%s\", \"write\": \"%s\", \"ms\": %.4f, \"gbs\": %.0f}\n", q.name, wm_name[m],
                   t[m], bytes / (t[m] * 1e-3) / 1e9);
    }
    return 0;
}
