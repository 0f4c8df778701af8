// The cost of one dependent fp32 add on gfx950: the floor of every
// sequential float sum CGX_F32_REF reproduces (serialConjugate.c's matVec
// rows and vecVec).  One wave, N dependent adds:
//   reg    operands in registers (the pure VALU dependency)
//   lds    operands read from LDS as 16-B broadcasts, G quads ahead
// Prints cycles (s_memtime, 100 MHz on gfx950 -> converted by the measured
// kernel time) and ns per add.
//   hipcc --offload-arch=gfx950 -O3 -o tools/microbench/add_chain tools/microbench/add_chain.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            std::exit(1);                                                          \
        }                                                                          \
    } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(64) void k_reg(int n, const float *in, float *out) {
#pragma clang fp contract(off)
    float v[16];
    for (int u = 0; u < 16; ++u) v[u] = in[threadIdx.x + 64 * u];
    float s = 0.0f;
    for (int i = 0; i < n; i += 16) {
#pragma unroll
        for (int u = 0; u < 16; ++u) s = s + v[u];
    }
    out[threadIdx.x] = s;
}

template <int G>
__global__ __launch_bounds__(64) void k_lds(int n, const float *in, float *out) {
#pragma clang fp contract(off)
    __shared__ f4 buf[1024];  // 4096 floats, reread
    for (int i = threadIdx.x; i < 1024; i += 64) buf[i] = *reinterpret_cast<const f4 *>(in + 4 * i);
    __syncthreads();
    float s = 0.0f;
    f4 q[G], qn[G];
#pragma unroll
    for (int u = 0; u < G; ++u) q[u] = buf[u];
    for (int i = 0; i < n / 4; i += 2 * G) {
        const int j = i & 1023;
#pragma unroll
        for (int u = 0; u < G; ++u) qn[u] = buf[(j + G + u) & 1023];
#pragma unroll
        for (int u = 0; u < G; ++u) {
            s = s + q[u].x;
            s = s + q[u].y;
            s = s + q[u].z;
            s = s + q[u].w;
        }
#pragma unroll
        for (int u = 0; u < G; ++u) q[u] = buf[(j + 2 * G + u) & 1023];
#pragma unroll
        for (int u = 0; u < G; ++u) {
            s = s + qn[u].x;
            s = s + qn[u].y;
            s = s + qn[u].z;
            s = s + qn[u].w;
        }
    }
    out[threadIdx.x] = s;
}

template <typename F>
static float time_us(F launch, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1e3f / reps;
}

int main() {
    float *in, *out;
    CK(hipMalloc(&in, 4096 * 4));
    CK(hipMalloc(&out, 64 * 4));
    CK(hipMemset(in, 0, 4096 * 4));
    const int reps = 20;
    for (int n : {8192, 65536, 524288}) {
        const float treg = time_us([&] { hipLaunchKernelGGL(k_reg, dim3(1), dim3(64), 0, 0, n, in, out); }, reps);
        const float t4 = time_us([&] { hipLaunchKernelGGL(k_lds<4>, dim3(1), dim3(64), 0, 0, n, in, out); }, reps);
        const float t8 = time_us([&] { hipLaunchKernelGGL(k_lds<8>, dim3(1), dim3(64), 0, 0, n, in, out); }, reps);
        const float t16 = time_us([&] { hipLaunchKernelGGL(k_lds<16>, dim3(1), dim3(64), 0, 0, n, in, out); }, reps);
        std::printf("{\"adds\": %d, \"reg_us\": %.2f, \"reg_ns_per_add\": %.3f, \"lds_g4_ns_per_add\": %.3f, "
                    "\"lds_g8_ns_per_add\": %.3f, \"lds_g16_ns_per_add\": %.3f}\n",
                    n, treg, treg * 1e3 / n, t4 * 1e3 / n, t8 * 1e3 / n, t16 * 1e3 / n);
    }
    return 0;
}
