// MFMA issue-rate probe: one workgroup per CU, W waves, each issuing N v_mfma_f32_16x16x32_bf16 on 2 x 5
// accumulators in the layer kernel's order (chains of 6 on one accumulator pair), timed with s_memtime
// (per wave) and hipEvents (whole grid).  hipcc --offload-arch=gfx950 -O3 tools/mfma_rate.hip -o tools/mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
__global__ void probe(float *out, unsigned long long *ticks, int iters) {
    bf16x8 a0, a1, b0, b1;
    for (int i = 0; i < 8; ++i) {
        a0[i] = (__bf16)(threadIdx.x * 0.001f + i); a1[i] = (__bf16)(i * 0.5f);
        b0[i] = (__bf16)(i * 0.25f); b1[i] = (__bf16)(threadIdx.x * 0.002f);
    }
    floatx4 acc[2][5] = {};
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int b = 0; b < 5; ++b)
#pragma unroll
            for (int t = 0; t < 6; ++t) {
                acc[0][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, (t & 1) ? b1 : b0, acc[0][b], 0, 0, 0);
                acc[1][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, (t & 1) ? b0 : b1, acc[1][b], 0, 0, 0);
            }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 5; ++b) s += acc[a][b][0] + acc[a][b][1] + acc[a][b][2] + acc[a][b][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) ticks[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}
int main() {
    const int iters = 100, grid = 256;
    float *out; unsigned long long *ticks;
    hipMalloc(&out, grid * 1024 * 4); hipMalloc(&ticks, grid * 16 * 8);
    for (int waves : {4, 8}) {
        hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
        probe<<<grid, 64 * waves>>>(out, ticks, iters);
        hipEventRecord(e0);
        probe<<<grid, 64 * waves>>>(out, ticks, iters);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        unsigned long long h[16];
        hipMemcpy(h, ticks, sizeof(h), hipMemcpyDeviceToHost);
        const double mf = iters * 60.0;  // MFMAs per wave
        printf("waves/WG %d: %.1f us for %.0f MFMAs per wave -> %.1f ns per MFMA per wave; s_memtime %.1f ticks per MFMA (wave 0); "
               "chip %.0f TFLOP/s bf16\n", waves, ms * 1e3, mf, ms * 1e6 / mf, h[0] / mf,
               grid * waves * mf * 16384.0 / (ms * 1e-3) / 1e12);
    }
    return 0;
}
