// Empirical HBM read ceiling on one MI355X: stream a large buffer once with
// 16-B loads (default or non-temporal policy), U loads in flight per lane,
// grid-stride over 1-KiB wave chunks, one double per thread written at the
// end (so nothing is dead code).  The best rate over the configurations is
// the practical ceiling the matVec's roofline fraction is read against
// (DESIGN.md section 3).  Build and run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/hbm_read_peak tools/microbench/hbm_read_peak.hip
//   /tmp/hbm_read_peak [GiB=32]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double d2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_read(const d2 *__restrict__ a, int64_t nchunks, double *out) {
    // a wave reads chunks of 64 d2 (1 KiB); U chunks per step
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t nw = (int64_t)gridDim.x * 4;
    d2 acc = (d2)(0.0);
    for (int64_t c = wave * U; c < nchunks; c += nw * U) {
        d2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t cc = c + u;
            const d2 *p = a + (cc < nchunks ? cc : nchunks - 1) * 64 + lane;
            if constexpr (NT) v[u] = __builtin_nontemporal_load(p);
            else v[u] = *p;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u];
    }
    out[(int64_t)blockIdx.x * 256 + threadIdx.x] = acc.x + acc.y;
}

template <int U, bool NT>
double run(const d2 *a, int64_t nchunks, double *out, int blocks, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_read<U, NT>), dim3(blocks), dim3(256), 0, 0, a, nchunks, out);
    CK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL((k_read<U, NT>), dim3(blocks), dim3(256), 0, 0, a, nchunks, out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float t = 0;
        CK(hipEventElapsedTime(&t, e0, e1));
        ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return (double)nchunks * 1024.0 / (ms[ms.size() / 2] * 1e-3) / 1e9;  // median
}

int main(int argc, char **argv) {
    const double gib = argc > 1 ? std::atof(argv[1]) : 32.0;
    const int64_t bytes = (int64_t)(gib * (1ll << 30)) & ~int64_t(1023);
    const int64_t nchunks = bytes / 1024;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    d2 *a = nullptr;
    double *out = nullptr;
    CK(hipMalloc(&a, bytes));
    CK(hipMemset(a, 0, bytes));
    CK(hipMalloc(&out, (size_t)cus * 16 * 256 * sizeof(double)));
    std::printf("{\"bytes\": %lld, \"cus\": %d, \"results\": [", (long long)bytes, cus);
    bool first = true;
    double best = 0;
    for (int bpc : {1, 2, 4, 8}) {
        const int blocks = bpc * cus;
        const double r4n = run<4, true>(a, nchunks, out, blocks, 5), r8n = run<8, true>(a, nchunks, out, blocks, 5);
        const double r16n = run<16, true>(a, nchunks, out, blocks, 5), r8d = run<8, false>(a, nchunks, out, blocks, 5);
        for (auto [u, nt, g] : {std::tuple<int, int, double>{4, 1, r4n}, {8, 1, r8n}, {16, 1, r16n}, {8, 0, r8d}}) {
            std::printf("%s{\"blocks_per_cu\": %d, \"U\": %d, \"nt\": %d, \"GBps\": %.1f}", first ? "" : ", ", bpc, u,
                        nt, g);
            first = false;
            best = std::max(best, g);
        }
    }
    std::printf("], \"best_GBps\": %.1f}\n", best);
    CK(hipFree(a));
    CK(hipFree(out));
    return 0;
}
