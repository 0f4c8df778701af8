// Empirical HBM ceiling for read/write stream mixes on one MI355X: NR input
// and NW output vectors of `n` doubles, one contiguous grid-stride pass with
// 16-B non-temporal loads and stores, 4 elements pairs per thread in flight.
// The mixes are the Poisson kernels' (k_poisson_p and k_poisson_xr without
// the x update: 2 reads + 1 write; k_poisson_xr with x every iteration: 3 + 2;
// x every other iteration's catch-up: 4 + 2; every third's: 5 + 2) and a
// plain copy (1 + 1).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o /tmp/hbm_mix_peak tools/microbench/hbm_mix_peak.hip
//   /tmp/hbm_mix_peak [n = 67108864]
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

struct Bufs {
    const d2 *in[5];
    d2 *out[2];
};

template <int NR, int NW>
__global__ __launch_bounds__(256) void k_mix(Bufs b, int64_t npairs) {
    constexpr int V = 4;
    const int64_t step = (int64_t)gridDim.x * 256 * V;
    for (int64_t base = (int64_t)blockIdx.x * 256 * V + threadIdx.x; base < npairs; base += step) {
        d2 v[NR][V];
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
            for (int u = 0; u < V; ++u) {
                const int64_t i = base + u * 256;
                v[r][u] = i < npairs ? __builtin_nontemporal_load(b.in[r] + i) : (d2)(0.0);
            }
#pragma unroll
        for (int u = 0; u < V; ++u) {
            const int64_t i = base + u * 256;
            if (i >= npairs) continue;
            d2 s = v[0][u];
#pragma unroll
            for (int r = 1; r < NR; ++r) s = s * 0.5 + v[r][u];
#pragma unroll
            for (int w = 0; w < NW; ++w) __builtin_nontemporal_store(s + (double)w, b.out[w] + i);
        }
    }
}

// The same mix with the next pass's loads issued before this pass's stores
// (two register sets): a wait for a load never covers an earlier store
// (loads and stores share vmcnt), as in a software-pipelined kernel.
template <int NR, int NW>
__global__ __launch_bounds__(256) void k_mix_pipe(Bufs b, int64_t npairs) {
    constexpr int V = 4;
    const int64_t step = (int64_t)gridDim.x * 256 * V;
    int64_t base = (int64_t)blockIdx.x * 256 * V + threadIdx.x;
    d2 v[2][NR][V];
    auto load = [&](d2 (&dst)[NR][V], int64_t bs) {
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
            for (int u = 0; u < V; ++u) {
                const int64_t i = bs + u * 256;
                dst[r][u] = __builtin_nontemporal_load(b.in[r] + (i < npairs ? i : 0));
            }
    };
    auto store = [&](const d2 (&src)[NR][V], int64_t bs) {
#pragma unroll
        for (int u = 0; u < V; ++u) {
            const int64_t i = bs + u * 256;
            d2 s = src[0][u];
#pragma unroll
            for (int r = 1; r < NR; ++r) s = s * 0.5 + src[r][u];
            // past the end: store to element 0 of a spare pair (never read)
#pragma unroll
            for (int w = 0; w < NW; ++w) __builtin_nontemporal_store(s + (double)w, b.out[w] + (i < npairs ? i : npairs));
        }
    };
    if (base >= npairs) return;
    load(v[0], base);
    for (;;) {
        const int64_t nb = base + step;
        load(v[1], nb);
        store(v[0], base);
        if (nb >= npairs) break;
        const int64_t nb2 = nb + step;
        load(v[0], nb2);
        store(v[1], nb);
        if (nb2 >= npairs) break;
        base = nb2;
    }
}

template <int NR, int NW, bool PIPE = false>
double run(const Bufs &b, int64_t npairs, int blocks) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto fn = PIPE ? k_mix_pipe<NR, NW> : k_mix<NR, NW>;
    hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), 0, 0, b, npairs);
    CK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int r = 0; r < 7; ++r) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), 0, 0, b, npairs);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float t = 0;
        CK(hipEventElapsedTime(&t, e0, e1));
        ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return (double)npairs * 16.0 * (NR + NW) / (ms[ms.size() / 2] * 1e-3) / 1e9;
}

int main(int argc, char **argv) {
    const int64_t n = argc > 1 ? std::atoll(argv[1]) : (int64_t)1 << 26;
    const int64_t npairs = n / 2;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    Bufs b;
    for (int i = 0; i < 5; ++i) {
        d2 *p = nullptr;
        CK(hipMalloc(&p, npairs * 16));
        CK(hipMemset(p, 0, npairs * 16));
        b.in[i] = p;
    }
    for (int i = 0; i < 2; ++i) CK(hipMalloc(&b.out[i], (npairs + 1) * 16));  // + a spare pair (k_mix_pipe)
    std::printf("{\"n\": %lld, \"cus\": %d, \"results\": [", (long long)n, cus);
    bool first = true;
    for (int bpc : {1, 2, 3, 4, 8}) {
        const int blocks = bpc * cus;
        const double c11 = run<1, 1>(b, npairs, blocks), c21 = run<2, 1>(b, npairs, blocks);
        const double c32 = run<3, 2>(b, npairs, blocks), c42 = run<4, 2>(b, npairs, blocks);
        const double c52 = run<5, 2>(b, npairs, blocks);
        const double p21 = run<2, 1, true>(b, npairs, blocks), p52 = run<5, 2, true>(b, npairs, blocks);
        std::printf("%s{\"blocks_per_cu\": %d, \"read1_write1_GBps\": %.1f, \"read2_write1_GBps\": %.1f, "
                    "\"read3_write2_GBps\": %.1f, \"read4_write2_GBps\": %.1f, \"read5_write2_GBps\": %.1f, "
                    "\"pipelined_read2_write1_GBps\": %.1f, \"pipelined_read5_write2_GBps\": %.1f}",
                    first ? "" : ", ", bpc, c11, c21, c32, c42, c52, p21, p52);
        first = false;
    }
    std::printf("]}\n");
    return 0;
}
