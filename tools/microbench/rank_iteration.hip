// One rank's share of an N=65536 iteration at G ranks (default 8: an 8192-row
// block), without the collectives: the kernels libcgx's rank mode launches
// for the dense fp64 iteration (cgx_iterate.hip do_iteration), with the same
// launchers and plan, in every form of the p exchange:
//   split (round 4's overlap): on the compute stream, the matVec over the
//     rank's own column block (p is local; the allgather runs beside it on the
//     comm stream), then, after the gather, the other columns, accumulating,
//     with the fused p.Ap
//   conc (measured, not adopted): the own-block launch on the compute stream and
//     the rest launch on the comm stream right after the gather, at the same
//     time; then k_matvec_add_f64 adds the two row sums with the fused p.Ap
//   one (plain exchange): the gather, then one matVec over the whole row block
//     in the same rotated column order, own block and rest summed apart
//   natural (for reference; other bits): the gather, then one matVec in
//     column order 0..n-1
// then, every form:   [allreduce p.Ap]  k_update_r_f64 (r -= alpha Ap, r.r)
//                     [allreduce r.r]   k_update_xp_f64 (x += alpha p, p = r + beta p)
// The gather is emulated by a one-wave kernel that waits `gather_us` (0: none)
// on the comm stream (split, conc) or the compute stream (one, natural): the
// allgather's latency over xGMI, which one GPU cannot produce.  The forms run
// interleaved (blocks of iterations, alternating); the output says whether
// split, conc and one give the same Ap bits (and p.Ap).  Under `rocprofv3
// --kernel-trace` it gives every kernel's duration and the gap before it.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I conjugate_gradient_amd/csrc \
//       -o tools/microbench/rank_iteration tools/microbench/rank_iteration.hip \
//       -L conjugate_gradient_amd/lib -lcgx -Wl,-rpath,'$ORIGIN/../../conjugate_gradient_amd/lib'
//   tools/microbench/rank_iteration [ranks=8] [iterations=60] [rank=ranks/2] [gather_us=0]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "cgx_device.h"

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

// The emulated allgather: one wave waits `ticks` of the 100 MHz constant clock.
__global__ void k_wait(int64_t ticks) {
    const int64_t t0 = (int64_t)__builtin_amdgcn_s_memrealtime();
    while ((int64_t)__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

// conc's add (measured and not adopted, round 5): out[i] = own[i] + rest[i]
// (the accumulating rest launch's `out[i] + mine`, the same bits) with the
// fused p.Ap, rows visited by the same (block, wave, lane) as in
// k_matvec_f64<R> on the plan's grid, so p.Ap adds in the matVec's order.
template <int R>
__global__ __launch_bounds__(cgx::kNT) void k_matvec_add_f64(int64_t rows, const double *__restrict__ own,
                                                             const double *__restrict__ rest, double *__restrict__ out,
                                                             const double *__restrict__ pown, double *dot_out,
                                                             double *partials, unsigned *ticket) {
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int64_t ngroups = (rows + R - 1) / R;
    const int64_t wstride = (int64_t)gridDim.x * (cgx::kNT / 64);
    double dacc = 0.0;
    for (int64_t g = (int64_t)blockIdx.x * (cgx::kNT / 64) + wid; g < ngroups; g += wstride) {
        const int64_t i = g * R + lane;
        if (lane < R && i < rows) {
            const double mine = own[i] + rest[i];
            out[i] = mine;
            dacc += pown[i] * mine;
        }
    }
    cgx::grid_sum_last_block(dacc, partials, ticket, dot_out);
}

int main(int argc, char **argv) {
    const int64_t n = 65536, P = argc > 1 ? std::atoi(argv[1]) : 8, rows = n / P;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 60;
    const int64_t rank = argc > 3 ? std::atoi(argv[3]) : P / 2;
    const double gather_us = argc > 4 ? std::atof(argv[4]) : 0.0;
    double *A, *b, *p, *x, *r, *Ap, *Ap2, *Ap3, *Aprest, *scal;
    cgx::RedWs ws{nullptr, nullptr};
    CK(hipMalloc(&A, (size_t)rows * n * 8));
    CK(hipMalloc(&b, (size_t)rows * 8));
    CK(hipMalloc(&p, (size_t)n * 8));
    CK(hipMalloc(&x, (size_t)rows * 8));
    CK(hipMalloc(&r, (size_t)rows * 8));
    CK(hipMalloc(&Ap, (size_t)rows * 8));
    CK(hipMalloc(&Ap2, (size_t)rows * 8));
    CK(hipMalloc(&Ap3, (size_t)rows * 8));
    CK(hipMalloc(&Aprest, (size_t)rows * 8));
    CK(hipMalloc(&scal, 64 * 8));
    CK(hipMalloc(&ws.partials, cgx::kMaxRedBlocks * sizeof(double)));
    CK(hipMalloc(&ws.tickets, cgx::kTickets * sizeof(unsigned)));
    CK(hipMemset(ws.tickets, 0, cgx::kTickets * sizeof(unsigned)));
    hipStream_t s, cs;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    hipEvent_t ev_p, ev_rest;
    CK(hipEventCreateWithFlags(&ev_p, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&ev_rest, hipEventDisableTiming));
    CK(cgx::gen_spd_f64(n, n, rank * rows, rows, 42, A, b, s));
    CK(cgx::gen_spd_f64(n, n, 0, 1, 7, p, b, s));  // a p with varied entries (row 0 of another system)
    CK(cgx::fill_f64(x, rows, 0.0, s));
    CK(hipMemcpyAsync(r, b, rows * 8, hipMemcpyDeviceToDevice, s));
    CK(cgx::fill_f64(scal, 64, 1.0, s));
    // scalar slots: rsold = rr = 1, pAp = 1e6 (alpha small: the vectors stay finite)
    CK(cgx::fill_f64(scal + 1, 1, 1e6, s));
    const cgx::MatvecPlan pl = cgx::plan_matvec_f64(0, rows, 0, 0, -1, 0, n);
    double *pown = p + rank * rows, *rsold = scal, *pAp = scal + 1, *rr = scal + 2;
    const int64_t own0 = rank * rows, rest0 = (rank + 1) * rows % n;
    const int64_t ticks = (int64_t)(gather_us * 100.0);
    auto gather = [&](hipStream_t st) {
        if (ticks > 0) hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, st, ticks);
    };
    // matVec + p.Ap of each form; the result lands in `out`, p.Ap in `dot`
    auto matvec = [&](int form, double *out, double *dot) {
        if (form == 0) {  // split
            CK(hipEventRecord(ev_p, s));
            CK(hipStreamWaitEvent(cs, ev_p, 0));
            gather(cs);
            CK(hipEventRecord(ev_rest, cs));
            CK(cgx::matvec_f64_cols(pl, A, n, rows, n, own0, rows, false, p, out, nullptr, nullptr, ws, s));
            CK(hipStreamWaitEvent(s, ev_rest, 0));
            CK(cgx::matvec_f64_cols(pl, A, n, rows, n, rest0, n - rows, true, p, out, pown, dot, ws, s));
        } else if (form == 1) {  // conc
            CK(hipEventRecord(ev_p, s));
            CK(hipStreamWaitEvent(cs, ev_p, 0));
            gather(cs);
            CK(cgx::matvec_f64_cols(pl, A, n, rows, n, rest0, n - rows, false, p, Aprest, nullptr, nullptr, ws, cs));
            CK(hipEventRecord(ev_rest, cs));
            CK(cgx::matvec_f64_cols(pl, A, n, rows, n, own0, rows, false, p, out, nullptr, nullptr, ws, s));
            CK(hipStreamWaitEvent(s, ev_rest, 0));
            hipLaunchKernelGGL(pl.R == 1 ? k_matvec_add_f64<1> : k_matvec_add_f64<2>, dim3(pl.blocks), dim3(cgx::kNT),
                               0, s, rows, out, Aprest, out, pown, dot, ws.partials, ws.tickets + cgx::T_MATVEC);
            CK(hipGetLastError());
        } else if (form == 2) {  // one
            gather(s);
            CK(cgx::matvec_f64_cols(pl, A, n, rows, n, own0, n, false, p, out, pown, dot, ws, s, nullptr, nullptr, rows));
        } else {  // natural: column order 0..n-1, one accumulator (the single-GPU kernel; other bits)
            gather(s);
            CK(cgx::matvec_f64(pl, A, n, rows, n, p, out, pown, dot, ws, s));
        }
    };
    // the forms on the same p: the same Ap bits and p.Ap?
    matvec(0, Ap, scal + 10);
    matvec(1, Ap2, scal + 11);
    matvec(2, Ap3, scal + 12);
    CK(hipStreamSynchronize(s));
    CK(hipStreamSynchronize(cs));
    std::vector<double> h1(rows), h2(rows), h3(rows), hd(3);
    CK(hipMemcpy(h1.data(), Ap, rows * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), Ap2, rows * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h3.data(), Ap3, rows * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hd.data(), scal + 10, 3 * 8, hipMemcpyDeviceToHost));
    const bool same = std::memcmp(h1.data(), h2.data(), rows * 8) == 0 &&
                      std::memcmp(h1.data(), h3.data(), rows * 8) == 0 && std::memcmp(&hd[0], &hd[1], 8) == 0 &&
                      std::memcmp(&hd[0], &hd[2], 8) == 0;
    CK(cgx::fill_f64(p, n, 1.0 / n, s));
    auto iteration = [&](int form) {
        matvec(form, Ap, pAp);
        CK(cgx::update_r_f64(rows, r, Ap, rsold, pAp, rr, ws, s));
        CK(cgx::update_xp_f64(rows, x, pown, r, rsold, pAp, rr, s));
    };
    constexpr int kForms = 4;
    const char *names[kForms] = {"split", "conc", "one", "natural"};
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
    std::string meds, rounds;
    for (int f = 0; f < kForms; ++f) {
        char buf[64];
        std::snprintf(buf, sizeof buf, "%s\"%s\": %.2f", f ? ", " : "", names[f], med(us[f]));
        meds += buf;
        rounds += std::string(f ? ", " : "") + "\"" + names[f] + "\": [";
        for (size_t i = 0; i < us[f].size(); ++i) {
            std::snprintf(buf, sizeof buf, "%s%.1f", i ? ", " : "", us[f][i]);
            rounds += buf;
        }
        rounds += "]";
    }
    std::printf("{\"n\": %lld, \"ranks\": %lld, \"rank\": %lld, \"rows_per_rank\": %lld, \"gather_us\": %.1f, "
                "\"plan\": {\"R\": %d, \"U\": %d, \"nt\": %d, \"blocks\": %d}, \"iterations\": %d, \"rounds\": %d, "
                "\"us_per_iteration_without_collectives\": {%s}, \"per_round\": {%s}, \"ap_bitwise_equal\": %s}\n",
                (long long)n, (long long)P, (long long)rank, (long long)rows, gather_us, pl.R, pl.U, pl.nt, pl.blocks,
                iters, kRounds, meds.c_str(), rounds.c_str(), same ? "true" : "false");
    return same ? 0 : 2;
}
