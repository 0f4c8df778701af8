// The cost of splitting a rank's matVec in two for the exchange overlap
// (DESIGN.md s5): at 8 GPUs a rank owns 8192 rows of the N=65536 system;
// the overlapped iteration multiplies its own 8192-column block while p is
// gathered, then the other 57344 columns (two launches of libcgx's
// matvec_f64_cols), where the unoverlapped one is a single matvec_f64 launch.
// Both are timed here on one GPU with HIP events, interleaved, on the same
// row block (libcgx's own launchers and default plan).
//   hipcc --offload-arch=gfx950 -O2 -I include -I conjugate_gradient_amd/csrc \
//       -o tools/microbench/overlap_split tools/microbench/overlap_split.hip \
//       -L conjugate_gradient_amd/lib -lcgx -Wl,-rpath,$PWD/conjugate_gradient_amd/lib
//   tools/microbench/overlap_split [ranks=8]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "cgx_kernels.h"

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

int main(int argc, char **argv) {
    const int64_t n = 65536, P = argc > 1 ? std::atoi(argv[1]) : 8, rows = n / P, rank = P / 2;
    double *A, *b, *v, *out, *dot;
    cgx::RedWs ws{nullptr, nullptr};
    CK(hipMalloc(&A, (size_t)rows * n * 8));
    CK(hipMalloc(&b, (size_t)rows * 8));
    CK(hipMalloc(&v, (size_t)n * 8));
    CK(hipMalloc(&out, (size_t)rows * 8));
    CK(hipMalloc(&dot, 8));
    CK(hipMalloc(&ws.partials, cgx::kMaxRedBlocks * sizeof(double)));
    CK(hipMalloc(&ws.tickets, cgx::kTickets * sizeof(unsigned)));
    CK(hipMemset(ws.tickets, 0, cgx::kTickets * sizeof(unsigned)));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(cgx::gen_spd_f64(n, n, rank * rows, rows, 42, A, b, s));
    CK(hipMemsetAsync(v, 0, (size_t)n * 8, s));
    CK(cgx::fill_f64(v, n, 1.0, s));
    const cgx::MatvecPlan pl = cgx::plan_matvec_f64(0, rows);
    const double *pown = v + rank * rows;
    auto one = [&] { CK(cgx::matvec_f64(pl, A, n, rows, n, v, out, pown, dot, ws, s)); };
    auto split = [&] {
        CK(cgx::matvec_f64_cols(pl, A, n, rows, n, rank * rows, rows, false, v, out, nullptr, nullptr, ws, s));
        CK(cgx::matvec_f64_cols(pl, A, n, rows, n, (rank + 1) * rows % n, n - rows, true, v, out, pown, dot, ws, s));
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> t1, t2;
    for (int rep = 0; rep < 43; ++rep) {
        for (int which = 0; which < 2; ++which) {
            CK(hipEventRecord(e0, s));
            if (which == 0) one();
            else split();
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep >= 3) (which ? t2 : t1).push_back(ms);
        }
    }
    std::sort(t1.begin(), t1.end());
    std::sort(t2.begin(), t2.end());
    const double m1 = t1[t1.size() / 2], m2 = t2[t2.size() / 2];
    const double bytes = (double)rows * n * 8;
    std::printf("{\"ranks\": %lld, \"rows\": %lld, \"cols\": %lld, \"plan\": {\"R\": %d, \"U\": %d, \"nt\": %d, "
                "\"blocks\": %d}, \"one_launch_us\": %.2f, \"split_us\": %.2f, \"split_cost_us\": %.2f, "
                "\"one_launch_gbps\": %.1f, \"split_gbps\": %.1f}\n",
                (long long)P, (long long)rows, (long long)n, pl.R, pl.U, pl.nt, pl.blocks, 1e3 * m1, 1e3 * m2,
                1e3 * (m2 - m1), bytes / (m1 * 1e-3) / 1e9, bytes / (m2 * 1e-3) / 1e9);
    return 0;
}
