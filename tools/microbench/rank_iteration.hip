// One rank's share of an N=65536 iteration at G ranks (default 8: an 8192-row
// block), without the collectives: the kernels libcgx's rank mode launches on
// the rank's compute stream for the dense fp64 iteration (cgx_iterate.hip
// do_iteration), in the same order and with the same launchers and plan, in
// the two forms the context chooses between at creation (choose_overlap):
//   split (overlapped exchange):
//     1. matVec over the rank's own 8192-column block (p is local; the p
//        allgather runs beside it on the comm stream)
//     2. matVec over the other columns, accumulating, with the fused p.Ap
//   one (plain exchange: the allgather, then):
//     1. one matVec over the whole row block in the same rotated column order,
//        own block and rest summed apart (the same bits as split)
//   natural (for reference; other bits): one matVec in column order 0..n-1
//   then, both:
//        [allreduce p.Ap]
//     3. k_update_r_f64 (r -= alpha Ap, r.r)
//        [allreduce r.r]
//     4. k_update_xp_f64 (x += alpha p, p = r + beta p)
// The forms run interleaved (blocks of iterations, alternating), and the
// output says whether their Ap agree bit for bit.  Under `rocprofv3
// --kernel-trace` it gives every kernel's duration and the gap before it (the
// two allreduces and the allgather are what a SCALE run adds).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I conjugate_gradient_amd/csrc \
//       -o tools/microbench/rank_iteration tools/microbench/rank_iteration.hip \
//       -L conjugate_gradient_amd/lib -lcgx -Wl,-rpath,$PWD/conjugate_gradient_amd/lib
//   tools/microbench/rank_iteration [ranks=8] [iterations=60] [rank=ranks/2]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
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
    const int64_t n = 65536, P = argc > 1 ? std::atoi(argv[1]) : 8, rows = n / P;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 60;
    const int64_t rank = argc > 3 ? std::atoi(argv[3]) : P / 2;
    double *A, *b, *p, *x, *r, *Ap, *Ap2, *scal;
    cgx::RedWs ws{nullptr, nullptr};
    CK(hipMalloc(&A, (size_t)rows * n * 8));
    CK(hipMalloc(&b, (size_t)rows * 8));
    CK(hipMalloc(&p, (size_t)n * 8));
    CK(hipMalloc(&x, (size_t)rows * 8));
    CK(hipMalloc(&r, (size_t)rows * 8));
    CK(hipMalloc(&Ap, (size_t)rows * 8));
    CK(hipMalloc(&Ap2, (size_t)rows * 8));
    CK(hipMalloc(&scal, 64 * 8));
    CK(hipMalloc(&ws.partials, cgx::kMaxRedBlocks * sizeof(double)));
    CK(hipMalloc(&ws.tickets, cgx::kTickets * sizeof(unsigned)));
    CK(hipMemset(ws.tickets, 0, cgx::kTickets * sizeof(unsigned)));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(cgx::gen_spd_f64(n, n, rank * rows, rows, 42, A, b, s));
    CK(cgx::gen_spd_f64(n, n, 0, 1, 7, p, b, s));  // a p with varied entries (row 0 of another system)
    CK(cgx::fill_f64(x, rows, 0.0, s));
    CK(hipMemcpyAsync(r, b, rows * 8, hipMemcpyDeviceToDevice, s));
    CK(cgx::fill_f64(scal, 64, 1.0, s));
    // scalar slots: rsold = rr = 1, pAp = 1e6 (alpha small: the vectors stay finite)
    CK(cgx::fill_f64(scal + 1, 1, 1e6, s));
    const cgx::MatvecPlan pl = cgx::plan_matvec_f64(0, rows, 0, 0, -1, 0, n);
    double *pown = p + rank * rows, *rsold = scal, *pAp = scal + 1, *rr = scal + 2;
    // the matVec alone in both forms, on the same p: the same bits?
    CK(cgx::matvec_f64_cols(pl, A, n, rows, n, rank * rows, rows, false, p, Ap, nullptr, nullptr, ws, s));
    CK(cgx::matvec_f64_cols(pl, A, n, rows, n, (rank + 1) * rows % n, n - rows, true, p, Ap, nullptr, nullptr, ws, s));
    CK(cgx::matvec_f64_cols(pl, A, n, rows, n, rank * rows, n, false, p, Ap2, nullptr, nullptr, ws, s, nullptr, nullptr,
                            rows));
    CK(hipStreamSynchronize(s));
    std::vector<double> h1(rows), h2(rows);
    CK(hipMemcpy(h1.data(), Ap, rows * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), Ap2, rows * 8, hipMemcpyDeviceToHost));
    const bool same = std::memcmp(h1.data(), h2.data(), rows * 8) == 0;
    CK(cgx::fill_f64(p, n, 1.0 / n, s));
    auto iteration = [&](int form) {
        if (form == 0) {
            CK(cgx::matvec_f64_cols(pl, A, n, rows, n, rank * rows, rows, false, p, Ap, nullptr, nullptr, ws, s));
            CK(cgx::matvec_f64_cols(pl, A, n, rows, n, (rank + 1) * rows % n, n - rows, true, p, Ap, pown, pAp, ws, s));
        } else if (form == 1) {
            CK(cgx::matvec_f64_cols(pl, A, n, rows, n, rank * rows, n, false, p, Ap, pown, pAp, ws, s, nullptr, nullptr,
                                    rows));
        } else {  // column order 0..n-1, one accumulator (the single-GPU kernel; other bits)
            CK(cgx::matvec_f64(pl, A, n, rows, n, p, Ap, pown, pAp, ws, s));
        }
        CK(cgx::update_r_f64(rows, r, Ap, rsold, pAp, rr, ws, s));
        CK(cgx::update_xp_f64(rows, x, pown, r, rsold, pAp, rr, s));
    };
    constexpr int kForms = 3;
    for (int f = 0; f < kForms; ++f)
        for (int i = 0; i < 5; ++i) iteration(f);
    CK(hipStreamSynchronize(s));
    constexpr int kRounds = 5;
    std::vector<double> us[kForms];
    for (int round = 0; round < kRounds; ++round)
        for (int f = 0; f < kForms; ++f) {
            const auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < iters; ++i) iteration(f);
            CK(hipStreamSynchronize(s));
            us[f].push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() /
                            iters);
        }
    auto med = [](std::vector<double> v) {
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
    };
    auto list = [](const std::vector<double> &v) {
        std::string o = "[";
        for (size_t i = 0; i < v.size(); ++i) o += (i ? ", " : "") + std::to_string(v[i]).substr(0, 6);
        return o + "]";
    };
    std::printf("{\"n\": %lld, \"ranks\": %lld, \"rank\": %lld, \"rows_per_rank\": %lld, \"plan\": {\"R\": %d, "
                "\"U\": %d, \"nt\": %d, \"blocks\": %d}, \"iterations\": %d, \"rounds\": %d, "
                "\"us_per_iteration_without_collectives\": {\"split\": %.2f, \"one\": %.2f, \"natural\": %.2f}, "
                "\"split_rounds\": %s, \"one_rounds\": %s, \"natural_rounds\": %s, \"ap_bitwise_equal\": %s}\n",
                (long long)n, (long long)P, (long long)rank, (long long)rows, pl.R, pl.U, pl.nt, pl.blocks, iters,
                kRounds, med(us[0]), med(us[1]), med(us[2]), list(us[0]).c_str(), list(us[1]).c_str(),
                list(us[2]).c_str(), same ? "true" : "false");
    return same ? 0 : 2;
}
