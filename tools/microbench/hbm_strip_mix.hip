// HBM ceiling of the Poisson kernels' ACCESS PATTERN, without their
// arithmetic: NR input and NW output grids of m x m doubles (row-major, row
// pitch m), walked as k_poisson_* walk them -- work items of (strip of SW
// columns, run of RPI rows), strip-fastest, grid-stride (or XCD-banded: the
// blocks of XCD x take the x-th eighth of the runs), RB rows per step, the
// next step's loads issued before this step's stores (as
// k_poisson_xr_pipe_f64).  A 256-thread block is 4 waves; wave w covers
// columns [w * 128 * CPL, (w + 1) * 128 * CPL) of its strip, load u of a lane
// reads the 16 B at column 128 u + 2 lane, so every load instruction is one
// contiguous KiB.  SW = 512 CPL.  CPL = 1 is the kernels' layout (1-KiB row
// chunks 64 KiB apart, 4 KiB per block-row); CPL = 2 and 4 are the wider
// strips (2 and 4 columns pairs per lane).  Bytes in flight per lane are the
// same for every CPL (RB = 4 / CPL).  m = SW makes the walk contiguous: the
// plain streaming ceiling of the same mix, measured in the same process.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o /tmp/hbm_strip_mix tools/microbench/hbm_strip_mix.hip
//   /tmp/hbm_strip_mix [m = 8192]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double d2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                            \
    do {                                                                 \
        hipError_t e_ = (x);                                             \
        if (e_ != hipSuccess) {                                          \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
            std::exit(1);                                                \
        }                                                                \
    } while (0)

struct Bufs {
    const double *in[5];
    double *out[2];
};

struct Walk {
    int64_t m, nstrips, nitems, spi;  // spi = row steps per item
    int rpi, bands;
};

template <int NR, int NW, int CPL, int RB>
__global__ __launch_bounds__(256) void k_strip(Bufs b, Walk wk) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    constexpr int SW = 512 * CPL;
    // this block's items: v-th item = first + v * stride (v < count)
    int64_t first = blockIdx.x, count = wk.nitems, stride = gridDim.x;
    if (wk.bands) {
        const int64_t nruns = wk.nitems / wk.nstrips, x = blockIdx.x % 8;
        const int64_t r0 = nruns * x / 8, r1 = nruns * (x + 1) / 8;
        first = r0 * wk.nstrips + blockIdx.x / 8;
        count = (r1 - r0) * wk.nstrips;
        stride = gridDim.x / 8;
        count = first - r0 * wk.nstrips < count ? (count - (first - r0 * wk.nstrips) + stride - 1) / stride : 0;
    } else {
        count = first < count ? (count - first + stride - 1) / stride : 0;
    }
    const int64_t nsteps = count * wk.spi;
    if (nsteps == 0) return;
    // element offset of (step g, row t, load u) in every grid
    auto off = [&](int64_t g, int t, int u) -> int64_t {
        const int64_t w = first + (g / wk.spi) * stride;
        const int64_t row = (w / wk.nstrips) * wk.rpi + (g % wk.spi) * RB + t;
        const int64_t col = (w % wk.nstrips) * SW + wv * 128 * CPL + u * 128 + 2 * lane;
        return row * wk.m + col;
    };
    d2 v[2][NR][RB][CPL];
    auto load = [&](d2 (&dst)[NR][RB][CPL], int64_t g) {
#pragma unroll
        for (int t = 0; t < RB; ++t)
#pragma unroll
            for (int u = 0; u < CPL; ++u) {
                const int64_t o = off(g, t, u);
#pragma unroll
                for (int r = 0; r < NR; ++r)
                    dst[r][t][u] = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(b.in[r] + o));
            }
    };
    auto store = [&](const d2 (&src)[NR][RB][CPL], int64_t g) {
#pragma unroll
        for (int t = 0; t < RB; ++t)
#pragma unroll
            for (int u = 0; u < CPL; ++u) {
                const int64_t o = off(g, t, u);
                d2 s = src[0][t][u];
#pragma unroll
                for (int r = 1; r < NR; ++r) s = s * 0.5 + src[r][t][u];
#pragma unroll
                for (int w = 0; w < NW; ++w)
                    __builtin_nontemporal_store(s + (double)w, reinterpret_cast<d2 *>(b.out[w] + o));
            }
    };
    load(v[0], 0);
    for (int64_t g = 0;; g += 2) {
        if (g + 1 < nsteps) load(v[1], g + 1);
        store(v[0], g);
        if (g + 1 >= nsteps) break;
        if (g + 2 < nsteps) load(v[0], g + 2);
        store(v[1], g + 1);
        if (g + 2 >= nsteps) break;
    }
}

template <int NR, int NW, int CPL>
double run(const Bufs &b, int64_t m, int64_t rows, int rpi, int bands, int blocks) {
    constexpr int RB = 4 / CPL;
    Walk wk;
    wk.m = m;
    wk.nstrips = m / (512 * CPL);
    wk.rpi = rpi;
    wk.nitems = (rows / rpi) * wk.nstrips;
    wk.spi = rpi / RB;
    wk.bands = bands;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto fn = k_strip<NR, NW, CPL, RB>;
    hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), 0, 0, b, wk);
    CK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int r = 0; r < 7; ++r) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), 0, 0, b, wk);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float t = 0;
        CK(hipEventElapsedTime(&t, e0, e1));
        ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return (double)(rows / rpi) * rpi * m * 8.0 * (NR + NW) / (ms[ms.size() / 2] * 1e-3) / 1e9;
}

template <int NR, int NW>
void mix(const Bufs &b, int64_t m, int cus, bool &firstline) {
    const int64_t total = m * m;
    for (int bpc : {1, 2}) {
        const int blocks = bpc * cus;
        // contiguous: one strip as wide as a row (rows of SW doubles, back to back)
        const double c1 = run<NR, NW, 1>(b, 512, total / 512, 8, 0, blocks);
        const double c4 = run<NR, NW, 4>(b, 2048, total / 2048, 8, 0, blocks);
        for (int bands : {0, 1}) {
            const double s1 = run<NR, NW, 1>(b, m, m, 8, bands, blocks);
            const double s2 = run<NR, NW, 2>(b, m, m, 8, bands, blocks);
            const double s4 = run<NR, NW, 4>(b, m, m, 8, bands, blocks);
            const double s1r16 = run<NR, NW, 1>(b, m, m, 16, bands, blocks);
            std::printf("%s{\"reads\": %d, \"writes\": %d, \"blocks_per_cu\": %d, \"bands\": %d, "
                        "\"contiguous_GBps\": %.1f, \"contiguous_cpl4_GBps\": %.1f, \"strip512_GBps\": %.1f, "
                        "\"strip1024_GBps\": %.1f, \"strip2048_GBps\": %.1f, \"strip512_rpi16_GBps\": %.1f}",
                        firstline ? "" : ",\n ", NR, NW, bpc, bands, c1, c4, s1, s2, s4, s1r16);
            firstline = false;
            std::fflush(stdout);
        }
    }
}

int main(int argc, char **argv) {
    const int64_t m = argc > 1 ? std::atoll(argv[1]) : 8192;
    if (m % 2048 != 0) {
        std::fprintf(stderr, "m must be a multiple of 2048\n");
        return 1;
    }
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    Bufs b;
    for (int i = 0; i < 5; ++i) {
        double *p = nullptr;
        CK(hipMalloc(&p, m * m * 8));
        CK(hipMemset(p, 0, m * m * 8));
        b.in[i] = p;
    }
    for (int i = 0; i < 2; ++i) CK(hipMalloc(&b.out[i], m * m * 8));
    std::printf("{\"m\": %lld, \"cus\": %d, \"results\": [", (long long)m, cus);
    bool firstline = true;
    mix<5, 2>(b, m, cus, firstline);
    mix<2, 1>(b, m, cus, firstline);
    std::printf("]}\n");
    return 0;
}
