// Start-up cost of the HIP runtime on the box, for the CLI's phase
// breakdown: hipGetDeviceCount (runtime init), the first
// hipMalloc and the first kernel launch of a tiny code object.
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/hip_init_time tools/microbench/hip_init_time.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void k_touch(int *p) { p[threadIdx.x] = threadIdx.x; }

int main() {
    using clk = std::chrono::steady_clock;
    auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    const auto t0 = clk::now();
    int n = 0;
    (void)hipGetDeviceCount(&n);
    const auto t1 = clk::now();
    int *p = nullptr;
    (void)hipMalloc(&p, 1 << 20);
    const auto t2 = clk::now();
    k_touch<<<1, 64>>>(p);
    (void)hipDeviceSynchronize();
    const auto t3 = clk::now();
    std::printf("{\"devices\": %d, \"runtime_init_ms\": %.3f, \"first_malloc_ms\": %.3f, \"first_kernel_ms\": %.3f}\n", n,
                ms(t0, t1), ms(t1, t2), ms(t2, t3));
    return 0;
}
