// One rank's share of an N=65536 iteration at G ranks (default 8: an 8192-row
// block), without the collectives: the kernels libcgx's rank mode launches on
// the rank's compute stream for the overlapped dense fp64 iteration
// (cgx_iterate.hip do_iteration + cgx_exchange.hip overlapped_matvec), in the
// same order and with the same launchers and plan:
//   1. matVec over the rank's own 8192-column block (p is local; the p
//      allgather runs beside it on the comm stream)
//   2. matVec over the other columns, accumulating, with the fused p.Ap
//      [allreduce p.Ap]
//   3. k_update_r_f64 (r -= alpha Ap, r.r)
//      [allreduce r.r]
//   4. k_update_xp_f64 (x += alpha p, p = r + beta p)
// Run under `rocprofv3 --kernel-trace` it gives the non-communication budget
// of a G-rank iteration: every kernel's duration and the idle gap before it
// (the two allreduces and the allgather are what a SCALE run adds).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I conjugate_gradient_amd/csrc \
//       -o tools/microbench/rank_iteration tools/microbench/rank_iteration.hip \
//       -L conjugate_gradient_amd/lib -lcgx -Wl,-rpath,$PWD/conjugate_gradient_amd/lib
//   tools/microbench/rank_iteration [ranks=8] [iterations=60]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>

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
    const int iters = argc > 2 ? std::atoi(argv[2]) : 60;
    double *A, *b, *p, *x, *r, *Ap, *scal;
    cgx::RedWs ws{nullptr, nullptr};
    CK(hipMalloc(&A, (size_t)rows * n * 8));
    CK(hipMalloc(&b, (size_t)rows * 8));
    CK(hipMalloc(&p, (size_t)n * 8));
    CK(hipMalloc(&x, (size_t)rows * 8));
    CK(hipMalloc(&r, (size_t)rows * 8));
    CK(hipMalloc(&Ap, (size_t)rows * 8));
    CK(hipMalloc(&scal, 64 * 8));
    CK(hipMalloc(&ws.partials, cgx::kMaxRedBlocks * sizeof(double)));
    CK(hipMalloc(&ws.tickets, cgx::kTickets * sizeof(unsigned)));
    CK(hipMemset(ws.tickets, 0, cgx::kTickets * sizeof(unsigned)));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(cgx::gen_spd_f64(n, n, rank * rows, rows, 42, A, b, s));
    CK(cgx::fill_f64(p, n, 1.0 / n, s));
    CK(cgx::fill_f64(x, rows, 0.0, s));
    CK(hipMemcpyAsync(r, b, rows * 8, hipMemcpyDeviceToDevice, s));
    CK(cgx::fill_f64(scal, 64, 1.0, s));
    // scalar slots: rsold = rr = 1, pAp = 1e6 (alpha small: the vectors stay finite)
    CK(cgx::fill_f64(scal + 1, 1, 1e6, s));
    const cgx::MatvecPlan pl = cgx::plan_matvec_f64(0, rows, 0, 0, -1, 0, n);
    double *pown = p + rank * rows, *rsold = scal, *pAp = scal + 1, *rr = scal + 2;
    auto iteration = [&] {
        CK(cgx::matvec_f64_cols(pl, A, n, rows, n, rank * rows, rows, false, p, Ap, nullptr, nullptr, ws, s));
        CK(cgx::matvec_f64_cols(pl, A, n, rows, n, (rank + 1) * rows % n, n - rows, true, p, Ap, pown, pAp, ws, s));
        CK(cgx::update_r_f64(rows, r, Ap, rsold, pAp, rr, ws, s));
        CK(cgx::update_xp_f64(rows, x, pown, r, rsold, pAp, rr, s));
    };
    for (int i = 0; i < 5; ++i) iteration();
    CK(hipStreamSynchronize(s));
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; ++i) iteration();
    CK(hipStreamSynchronize(s));
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
    std::printf("{\"n\": %lld, \"ranks\": %lld, \"rows_per_rank\": %lld, \"plan\": {\"R\": %d, \"U\": %d, \"nt\": %d, "
                "\"blocks\": %d}, \"iterations\": %d, \"us_per_iteration_without_collectives\": %.2f}\n",
                (long long)n, (long long)P, (long long)rows, pl.R, pl.U, pl.nt, pl.blocks, iters, us);
    return 0;
}
