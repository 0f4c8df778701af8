// HBM read rate by access pattern: how many contiguous streams a CU reads at
// once.  k_symv_f64 streams one contiguous run of tiles per block (one
// stream per CU, 8 KiB per load instruction across the block); the dense
// matVec reads 2 rows per wave (8 streams per CU).  This reads a buffer once
// with nothing but 16-B non-temporal loads, two register slots in flight as
// in both kernels, and splits each block into S groups of waves that each
// stream their own contiguous region (S = 1 is k_symv_f64's pattern).  ALT:
// S = 1, but the two slots alternate between two regions (slot 0 from the
// block's first half, slot 1 from its second).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/hbm_region_read tools/microbench/hbm_region_read.hip
//   /tmp/hbm_region_read [GiB=16]
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

// NT threads, S streams per block (NT/S threads each, whole waves), K 16-B
// loads per thread per step: a step of one stream is (NT/S)*K*16 bytes.
template <int NT, int S, int K, bool ALT>
__global__ __launch_bounds__(NT) void k_region(const d2 *__restrict__ a, int64_t steps, double *out) {
    constexpr int G = NT / S;
    static_assert(G % 64 == 0, "whole waves per stream");
    const int g = threadIdx.x / G, t = threadIdx.x % G;
    const int64_t step_d2 = (int64_t)G * K;
    const d2 *base = a + ((int64_t)blockIdx.x * S + g) * steps * step_d2 + t;
    // ALT: slot 1 walks the region's second half while slot 0 walks the first
    const d2 *base1 = ALT ? base + (steps / 2) * step_d2 : base;
    const int64_t half = ALT ? steps / 2 : steps;
    d2 s0[K], s1[K], acc = (d2)(0.0);
    auto load = [&](d2 *s, const d2 *b, int64_t st, int64_t lim) {
        st = st < lim ? st : lim - 1;  // unconditional: past the end reload the last step
#pragma unroll
        for (int k = 0; k < K; ++k) s[k] = __builtin_nontemporal_load(b + st * step_d2 + k * G);
    };
    if constexpr (ALT) {
        load(s0, base, 0, half);
        for (int64_t st = 0; st < half; ++st) {
            load(s1, base1, st, half);
#pragma unroll
            for (int k = 0; k < K; ++k) acc += s0[k];
            load(s0, base, st + 1, half);
#pragma unroll
            for (int k = 0; k < K; ++k) acc += s1[k];
        }
    } else {
        load(s0, base, 0, steps);
        for (int64_t st = 0; st < steps; st += 2) {
            load(s1, base, st + 1, steps);
#pragma unroll
            for (int k = 0; k < K; ++k) acc += s0[k];
            load(s0, base, st + 2, steps);
#pragma unroll
            for (int k = 0; k < K; ++k) acc += s1[k];
        }
    }
    out[(int64_t)blockIdx.x * NT + threadIdx.x] = acc.x + acc.y;
}

// k_symv_f64's exact load form: one contiguous region per block, each step
// NT * K * 16 bytes read with raw buffer loads (a wave-uniform descriptor per
// step, the lane offset t * 16, the load index in soffset), two slots.
template <int NT, int K>
__global__ __launch_bounds__(NT) void k_region_buf(const d2 *__restrict__ a, int64_t steps, double *out) {
    const int t = threadIdx.x;
    const int64_t step_d2 = (int64_t)NT * K;
    const d2 *base = a + (int64_t)blockIdx.x * steps * step_d2;
    d2 s0[K], s1[K], acc = (d2)(0.0);
    auto load = [&](d2 *s, int64_t st) {
        st = st < steps ? st : steps - 1;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void *)(base + st * step_d2), 0, (int)(step_d2 * 16), 0x00020000);
#pragma unroll
        for (int k = 0; k < K; ++k)
            s[k] = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(rs, t * 16, k * NT * 16, 2));
    };
    load(s0, 0);
    for (int64_t st = 0; st < steps; st += 2) {
        load(s1, st + 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < K; ++k) acc += s0[k];
        load(s0, st + 2);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < K; ++k) acc += s1[k];
    }
    out[(int64_t)blockIdx.x * NT + threadIdx.x] = acc.x + acc.y;
}
template <int NT, int K>
void run_buf(const d2 *a, int64_t total_d2, double *out, int blocks, int reps, bool &first) {
    const int64_t step_d2 = (int64_t)NT * K;
    int64_t steps = total_d2 / ((int64_t)blocks * step_d2);
    steps &= ~int64_t(1);
    const double bytes = (double)steps * blocks * step_d2 * 16.0;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_region_buf<NT, K>), dim3(blocks), dim3(NT), 0, 0, a, steps, out);
    CK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL((k_region_buf<NT, K>), dim3(blocks), dim3(NT), 0, 0, a, steps, out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float tm = 0;
        CK(hipEventElapsedTime(&tm, e0, e1));
        ms.push_back(tm);
    }
    std::sort(ms.begin(), ms.end());
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    const double gbps = bytes / (ms[ms.size() / 2] * 1e-3) / 1e9;
    std::printf("%s\n  {\"threads\": %d, \"streams_per_block\": 1, \"buffer_loads\": 1, \"K\": %d, \"blocks\": %d, "
                "\"step_bytes\": %lld, \"GBps\": %.1f}",
                first ? "" : ",", NT, K, blocks, (long long)(step_d2 * 16), gbps);
    first = false;
}

template <int NT, int S, int K, bool ALT = false>
void run(const d2 *a, int64_t total_d2, double *out, int blocks, int reps, bool &first) {
    const int64_t step_d2 = (int64_t)(NT / S) * K;
    int64_t steps = total_d2 / ((int64_t)blocks * S * step_d2);
    steps &= ~int64_t(1);
    const double bytes = (double)steps * blocks * S * step_d2 * 16.0;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_region<NT, S, K, ALT>), dim3(blocks), dim3(NT), 0, 0, a, steps, out);
    CK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL((k_region<NT, S, K, ALT>), dim3(blocks), dim3(NT), 0, 0, a, steps, out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float t = 0;
        CK(hipEventElapsedTime(&t, e0, e1));
        ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    const double gbps = bytes / (ms[ms.size() / 2] * 1e-3) / 1e9;
    std::printf("%s\n  {\"threads\": %d, \"streams_per_block\": %d, \"alt\": %d, \"K\": %d, \"blocks\": %d, "
                "\"step_bytes\": %lld, \"GBps\": %.1f}",
                first ? "" : ",", NT, S, ALT ? 1 : 0, K, blocks, (long long)(step_d2 * 16), gbps);
    first = false;
}

int main(int argc, char **argv) {
    const double gib = argc > 1 ? std::atof(argv[1]) : 16.0;
    const int64_t bytes = (int64_t)(gib * (1ll << 30)) & ~int64_t(1023);
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    d2 *a = nullptr;
    double *out = nullptr;
    CK(hipMalloc(&a, bytes));
    CK(hipMemset(a, 0, bytes));
    CK(hipMalloc(&out, (size_t)cus * 4 * 512 * sizeof(double)));
    const int64_t n = bytes / 16;
    bool first = true;
    std::printf("{\"bytes\": %lld, \"cus\": %d, \"results\": [", (long long)bytes, cus);
    for (int rep = 0; rep < 2; ++rep) {
        // k_symv_f64's shape: 512 threads, 1 block per CU, 16 loads per thread per step
        run<512, 1, 16>(a, n, out, cus, 5, first);
        run<512, 1, 16, true>(a, n, out, cus, 5, first);
        run<512, 2, 16>(a, n, out, cus, 5, first);
        run<512, 4, 16>(a, n, out, cus, 5, first);
        run<512, 8, 16>(a, n, out, cus, 5, first);
        run<512, 1, 8>(a, n, out, cus, 5, first);
        run<512, 8, 8>(a, n, out, cus, 5, first);
        run<256, 1, 16>(a, n, out, 2 * cus, 5, first);
        run<256, 4, 16>(a, n, out, 2 * cus, 5, first);
        run<256, 4, 16>(a, n, out, cus, 5, first);
        // round 3: k_symv_f64's shape (256 threads, one region per block, one
        // block per CU) with global loads and with its buffer loads
        run<256, 1, 16>(a, n, out, cus, 5, first);
        run_buf<256, 16>(a, n, out, cus, 5, first);
        run_buf<256, 16>(a, n, out, 2 * cus, 5, first);
    }
    std::printf("\n]}\n");
    CK(hipFree(a));
    CK(hipFree(out));
    return 0;
}
