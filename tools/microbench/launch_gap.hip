// Kernel-to-kernel cost of a dependent chain on one stream vs the same chain
// replayed from a hipGraph: decides whether graph replay pays for the CG
// iteration at small N (3 dependent launches per iteration).
// Each kernel reads and writes a small vector (n doubles, 256-thread blocks),
// so consecutive launches depend on each other's data as in the solver.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/launch_gap tools/microbench/launch_gap.hip
//   /tmp/launch_gap [n=8192]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

__global__ __launch_bounds__(256) void k_axpy(int64_t n, double *__restrict__ y, const double *__restrict__ x,
                                              double a) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) y[i] = y[i] * 0.5 + a * x[i];
}

static void chain(hipStream_t s, int64_t n, double *a, double *b, double *c, int iters) {
    const int g = (int)((n + 255) / 256);
    for (int i = 0; i < iters; ++i) {
        k_axpy<<<g, 256, 0, s>>>(n, a, b, 1e-3);
        k_axpy<<<g, 256, 0, s>>>(n, b, c, 1e-3);
        k_axpy<<<g, 256, 0, s>>>(n, c, a, 1e-3);
    }
}

int main(int argc, char **argv) {
    const int64_t n = argc > 1 ? std::atoll(argv[1]) : 8192;
    double *a, *b, *c;
    CK(hipMalloc(&a, n * 8));
    CK(hipMalloc(&b, n * 8));
    CK(hipMalloc(&c, n * 8));
    CK(hipMemset(a, 0, n * 8));
    CK(hipMemset(b, 0, n * 8));
    CK(hipMemset(c, 0, n * 8));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int total = 3000;  // iterations of 3 kernels
    chain(s, n, a, b, c, 50);
    CK(hipStreamSynchronize(s));
    // 1. plain stream launches
    for (int rep = 0; rep < 3; ++rep) {
        auto t0 = std::chrono::steady_clock::now();
        CK(hipEventRecord(e0, s));
        chain(s, n, a, b, c, total);
        CK(hipEventRecord(e1, s));
        auto th = std::chrono::steady_clock::now();
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        double host_us = std::chrono::duration<double, std::micro>(th - t0).count();
        std::printf("{\"mode\": \"stream\", \"n\": %ld, \"us_per_kernel\": %.3f, \"host_enqueue_us_per_kernel\": %.3f}\n",
                    (long)n, ms * 1e3 / (3.0 * total), host_us / (3.0 * total));
    }
    // 2. graphs of G iterations, replayed
    for (int G : {1, 4, 16, 100}) {
        hipGraph_t gr;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        chain(s, n, a, b, c, G);
        CK(hipStreamEndCapture(s, &gr));
        CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        const int reps = total / G;
        for (int rep = 0; rep < 2; ++rep) {
            auto t0 = std::chrono::steady_clock::now();
            CK(hipEventRecord(e0, s));
            for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, s));
            CK(hipEventRecord(e1, s));
            auto th = std::chrono::steady_clock::now();
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            double host_us = std::chrono::duration<double, std::micro>(th - t0).count();
            std::printf("{\"mode\": \"graph\", \"iters_per_graph\": %d, \"n\": %ld, \"us_per_kernel\": %.3f, "
                        "\"host_enqueue_us_per_kernel\": %.3f}\n",
                        G, (long)n, ms * 1e3 / (3.0 * reps * G), host_us / (3.0 * reps * G));
        }
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(gr));
    }
    return 0;
}
