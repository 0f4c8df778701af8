// matvec_dyn.hip -- does the dense fp64 matVec lose time to load imbalance
// between waves?  libcgx's k_matvec_f64 hands row groups out statically
// (wave w takes groups w, w + waves, ...), so the launch ends when the slowest
// wave finishes its share.  This variant takes the next row group from a
// global counter (one atomic per group, fetched one group ahead so it is never
// waited for) and is timed against libcgx's default on the same rows,
// interleaved, with HIP events; row sums must be bitwise equal (a row's sum
// does not depend on which wave computes it).  Timing only: no fused p.Ap
// (with dynamic groups its per-block partials would depend on timing).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I conjugate_gradient_amd/csrc \
//       -o tools/microbench/matvec_dyn tools/microbench/matvec_dyn.hip \
//       -L conjugate_gradient_amd/lib -lcgx -Wl,-rpath,$PWD/conjugate_gradient_amd/lib
//   tools/microbench/matvec_dyn rows cols [reps=30]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "cgx_device.h"

#define CK(x)                                                            \
    do {                                                                 \
        hipError_t e_ = (x);                                             \
        if (e_ != hipSuccess) {                                          \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
            std::exit(1);                                                \
        }                                                                \
    } while (0)

using namespace cgx;

namespace {

template <int R, int U>
__device__ __forceinline__ void load_step(const d2 *const (&arow)[R], const d2 *v2, int64_t c, d2 (&pv)[U],
                                          d2 (&av)[R][U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) pv[u] = v2[(c + u) * 64];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u) av[r][u] = __builtin_nontemporal_load(arow[r] + (c + u) * 64);
}

template <int R, int U>
__device__ __forceinline__ void fma_step(const d2 (&pv)[U], const d2 (&av)[R][U], d2 (&acc)[R]) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < R; ++r) {
            acc[r].x = __builtin_fma(av[r][u].x, pv[u].x, acc[r].x);
            acc[r].y = __builtin_fma(av[r][u].y, pv[u].y, acc[r].y);
        }
}

// the same per-group pipeline as libcgx's mv_chunks_pipe (whole U-steps only:
// cols is a multiple of 128 * U here)
template <int R, int U>
__device__ __forceinline__ void chunks_pipe(const d2 *const (&arow)[R], const d2 *v2, int64_t c1, d2 (&acc)[R]) {
    d2 pa[U], aa[R][U], pb[U], ab[R][U];
    int64_t c = 0;
    load_step<R, U>(arow, v2, c, pa, aa);
    while (true) {
        const bool more = c + 2 * U <= c1;
        if (more) load_step<R, U>(arow, v2, c + U, pb, ab);
        fma_step<R, U>(pa, aa, acc);
        c += U;
        if (!more) break;
        const bool more2 = c + 2 * U <= c1;
        if (more2) load_step<R, U>(arow, v2, c + U, pa, aa);
        fma_step<R, U>(pb, ab, acc);
        c += U;
        if (!more2) break;
    }
}

template <int R, int U>
__global__ __launch_bounds__(kNT) void k_mv_dyn(const double *__restrict__ A, int64_t lda, int64_t rows, int64_t cols,
                                                 const double *__restrict__ v, double *__restrict__ out,
                                                 unsigned *counter) {
    const int lane = threadIdx.x & 63;
    const int64_t ngroups = (rows + R - 1) / R;
    const d2 *v2 = reinterpret_cast<const d2 *>(v) + lane;
    unsigned g = 0;
    if (lane == 0) g = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    g = __builtin_amdgcn_readfirstlane(g);
    while ((int64_t)g < ngroups) {
        unsigned gn = 0;  // the next group, fetched before this one's loads
        if (lane == 0) gn = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int64_t r0 = (int64_t)g * R;
        const d2 *arow[R];
        d2 acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int64_t ri = (r0 + r < rows) ? (r0 + r) : (rows - 1);
            arow[r] = reinterpret_cast<const d2 *>(A + ri * lda) + lane;
            acc[r] = (d2)(0.0);
        }
        chunks_pipe<R, U>(arow, v2, cols >> 7, acc);
        double mine = 0.0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const double s = wave_sum(acc[r].x + acc[r].y);
            if (lane == r) mine = s;
        }
        if (lane < R && r0 + lane < rows) out[r0 + lane] = mine;
        g = __builtin_amdgcn_readfirstlane(gn);
    }
}

}  // namespace

int main(int argc, char **argv) {
    const int64_t rows = argc > 1 ? std::atoll(argv[1]) : 16384, cols = argc > 2 ? std::atoll(argv[2]) : 16384;
    const int reps = argc > 3 ? std::atoi(argv[3]) : 30;
    if (cols % 1024) {
        std::fprintf(stderr, "cols must be a multiple of 1024 (whole U=8 steps)\n");
        return 2;
    }
    double *A, *b, *v, *ref, *out;
    unsigned *counters;
    RedWs ws{nullptr, nullptr};
    CK(hipMalloc(&A, (size_t)rows * cols * 8));
    CK(hipMalloc(&b, (size_t)rows * 8));
    CK(hipMalloc(&v, (size_t)cols * 8));
    CK(hipMalloc(&ref, (size_t)rows * 8));
    CK(hipMalloc(&out, (size_t)rows * 8));
    const int ncnt = 4 * (reps + 2);
    CK(hipMalloc(&counters, ncnt * sizeof(unsigned)));
    CK(hipMemset(counters, 0, ncnt * sizeof(unsigned)));
    CK(hipMalloc(&ws.partials, kMaxRedBlocks * sizeof(double)));
    CK(hipMalloc(&ws.tickets, kTickets * sizeof(unsigned)));
    CK(hipMemset(ws.tickets, 0, kTickets * sizeof(unsigned)));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(gen_spd_f64(cols, cols, 0, rows, 42, A, b, s));
    CK(gen_b_f64(cols, 7, v, s));
    const MatvecPlan pl = plan_matvec_f64(0, rows, -1, -1, -1, 0, cols);
    CK(matvec_f64(pl, A, cols, rows, cols, v, ref, nullptr, nullptr, ws, s));
    std::vector<double> href(rows), hout(rows);
    CK(hipMemcpyAsync(href.data(), ref, rows * 8, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = 8.0 * rows * cols + 8.0 * cols + 8.0 * rows;
    int cnt_i = 0;
    for (int R : {1, 2}) {
        const void *fn = R == 1 ? reinterpret_cast<const void *>(k_mv_dyn<1, 8>) : reinterpret_cast<const void *>(k_mv_dyn<2, 8>);
        int per_cu = 0, cus = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kNT, 0));
        CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
        const int blocks = std::max(1, per_cu) * cus;
        auto launch_dyn = [&] {
            unsigned *c = counters + (cnt_i++ % ncnt);
            if (R == 1) hipLaunchKernelGGL((k_mv_dyn<1, 8>), dim3(blocks), dim3(kNT), 0, s, A, cols, rows, cols, v, out, c);
            else hipLaunchKernelGGL((k_mv_dyn<2, 8>), dim3(blocks), dim3(kNT), 0, s, A, cols, rows, cols, v, out, c);
            CK(hipGetLastError());
        };
        auto launch_def = [&] { CK(matvec_f64(pl, A, cols, rows, cols, v, ref, nullptr, nullptr, ws, s)); };
        CK(hipMemset(counters, 0, ncnt * sizeof(unsigned)));
        cnt_i = 0;
        launch_dyn();
        CK(hipMemcpyAsync(hout.data(), out, rows * 8, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        const bool same = std::memcmp(hout.data(), href.data(), rows * 8) == 0;
        std::vector<float> tv, td;
        for (int rep = 0; rep < reps; ++rep)
            for (int which = 0; which < 2; ++which) {
                CK(hipEventRecord(e0, s));
                if (which) launch_def(); else launch_dyn();
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rep) (which ? td : tv).push_back(ms);
            }
        std::sort(tv.begin(), tv.end());
        std::sort(td.begin(), td.end());
        const double mv = tv[tv.size() / 2], md = td[td.size() / 2];
        std::printf("{\"rows\": %lld, \"cols\": %lld, \"dyn_R\": %d, \"dyn_blocks\": %d, \"default_plan\": "
                    "{\"R\": %d, \"U\": %d, \"blocks\": %d}, \"dyn_ms_median\": %.4f, \"dyn_gbps\": %.1f, "
                    "\"dyn_ms_min\": %.4f, \"default_ms_median\": %.4f, \"default_gbps\": %.1f, \"default_ms_min\": %.4f, "
                    "\"bitwise_equal_to_default\": %s}\n",
                    (long long)rows, (long long)cols, R, blocks, pl.R, pl.U, pl.blocks, mv, bytes / mv / 1e6, tv[0], md,
                    bytes / md / 1e6, td[0], same ? "true" : "false");
        std::fflush(stdout);
    }
    return 0;
}
