// Host cost of the calls the one-process multi-shard iteration makes
// (cgx_exchange.hip / cgx_iterate.hip), each timed over many back-to-back
// calls with nothing else in flight: hipLaunchKernel with small (16 B) and
// large (272 B: a PeerTable / PeerSum by value) kernel arguments, on one
// stream and round-robin over 8 streams; hipEventRecord; hipStreamWaitEvent.
// Decides whether the pointer tables travel as kernel arguments.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/microbench/_bin/host_enqueue tools/microbench/host_enqueue.hip
//   tools/microbench/_bin/host_enqueue
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

struct Big {
    const char *p[32];
    int cnt;
    double *out;
};

__global__ void k_small(double *y, double a) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && a < 0.0) y[0] = a;
}
__global__ void k_big(Big b, double a) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && a < 0.0) b.out[0] = a;
}

template <typename F>
static double per_call_us(int calls, F f) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < calls; ++i) f(i);
    const auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / calls;
}

int main() {
    const int S = 8, calls = 400;
    double *y;
    CK(hipMalloc(&y, 64));
    std::vector<hipStream_t> st(S);
    std::vector<hipEvent_t> ev(S);
    for (int i = 0; i < S; ++i) {
        CK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
        CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
    }
    Big b{};
    b.cnt = 8;
    b.out = y;
    auto sync = [&] {
        for (auto s : st) CK(hipStreamSynchronize(s));
    };
    // warm up every path once
    hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, st[0], y, 1.0);
    hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, st[0], b, 1.0);
    sync();
    std::printf("{");
    for (int rep = 0; rep < 3; ++rep) {
        sync();
        const double small1 = per_call_us(calls, [&](int) {
            hipLaunchKernelGGL(k_small, dim3(32), dim3(256), 0, st[0], y, 1.0);
        });
        sync();
        const double big1 = per_call_us(calls, [&](int) {
            hipLaunchKernelGGL(k_big, dim3(32), dim3(256), 0, st[0], b, 1.0);
        });
        sync();
        const double small8 = per_call_us(calls, [&](int i) {
            hipLaunchKernelGGL(k_small, dim3(32), dim3(256), 0, st[i % S], y, 1.0);
        });
        sync();
        const double big8 = per_call_us(calls, [&](int i) {
            hipLaunchKernelGGL(k_big, dim3(32), dim3(256), 0, st[i % S], b, 1.0);
        });
        sync();
        const double rec = per_call_us(calls, [&](int i) { CK(hipEventRecord(ev[i % S], st[i % S])); });
        sync();
        const double wait = per_call_us(calls, [&](int i) { CK(hipStreamWaitEvent(st[i % S], ev[(i + 1) % S], 0)); });
        sync();
        std::printf("%s\"rep%d\": {\"launch_16B_1stream_us\": %.2f, \"launch_272B_1stream_us\": %.2f, "
                    "\"launch_16B_8streams_us\": %.2f, \"launch_272B_8streams_us\": %.2f, "
                    "\"event_record_us\": %.2f, \"stream_wait_event_us\": %.2f}",
                    rep ? ", " : "", rep, small1, big1, small8, big8, rec, wait);
    }
    std::printf("}\n");
    return 0;
}
