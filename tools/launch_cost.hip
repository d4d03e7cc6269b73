// Host enqueue cost of hipLaunchKernelGGL against the kernel-argument size (the fused forward passes
// Multi<T> structs of up to WD_MULTI jobs: ~2-3 KB).  A spin kernel keeps the GPU busy so that the
// timed launches measure only the host side.  Build: hipcc --offload-arch=gfx950 -O2 launch_cost.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

template <int BYTES> struct Arg { char b[BYTES]; };

template <int BYTES> __global__ void empty_kernel(const Arg<BYTES> a) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && a.b[BYTES - 1] == 123) asm volatile("s_nop 0");
}

__global__ void spin_kernel(long long cycles) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {}
}

template <int BYTES> double time_launches(hipStream_t st, int n, int grid) {
    Arg<BYTES> a{};
    hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, st, 400000000LL);
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL(empty_kernel<BYTES>, dim3(grid), dim3(256), 0, st, a);
    const auto t1 = std::chrono::steady_clock::now();
    hipStreamSynchronize(st);
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main() {
    hipStream_t st;
    hipStreamCreate(&st);
    for (int w = 0; w < 3; ++w) {
        time_launches<64>(st, 50, 256);
        time_launches<2560>(st, 50, 256);
    }
    printf("kernarg   64 B: %.2f us/launch\n", time_launches<64>(st, 400, 256));
    printf("kernarg  512 B: %.2f us/launch\n", time_launches<512>(st, 400, 256));
    printf("kernarg 1024 B: %.2f us/launch\n", time_launches<1024>(st, 400, 256));
    printf("kernarg 2560 B: %.2f us/launch\n", time_launches<2560>(st, 400, 256));
    printf("kernarg 3584 B: %.2f us/launch\n", time_launches<3584>(st, 400, 256));
    hipStreamDestroy(st);
    return 0;
}
