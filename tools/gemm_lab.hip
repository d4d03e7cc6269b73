// gemm_lab.hip — standalone timing of the encoder's GEMM kernels at the benchmark shapes (tuning tool,
// not part of the product).  Build: make -C tools gemm_lab (hipcc --offload-arch=gfx950).
// Usage: ./gemm_lab [reps]   -> one line per (shape, kernel): avg µs per launch over `reps` launches,
// cycling through 8 distinct A buffers (an A operand freshly produced by the previous kernel is not
// L2-resident on the reading XCD), plus max normwise error against an fp64 host reference.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "gemm_x6.hpp"

using namespace wd;

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e = (x);                                                                 \
        if (e != hipSuccess) {                                                              \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

struct Shape { const char *name; int M, N, K; };

__global__ void empty_kernel(int *p) {
    if (p && threadIdx.x == 1023) p[blockIdx.x] = 0;
}

// L2 -> LDS streaming ceiling: each workgroup LDS-DMA copies `chunks` x 24 KB (4 waves x 6 x 1 KB per
// chunk) from a buffer of `span` bytes with S LDS stages (S - 1 chunks in flight)
template <int S>
__global__ __launch_bounds__(256) void stream_lds_kernel(const uint8_t *src, size_t span, int chunks, int *sink) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[S * 24576];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t base = ((size_t)blockIdx.x * 24576 * chunks) % span;
    auto issue = [&](int c) {
        uint8_t *st = lds + (c % S) * 24576;
        const size_t off = base + (size_t)c * 24576;
#pragma unroll
        for (int j = 0; j < 6; ++j)
            glds16(src + (off + (size_t)(6 * wave + j) * 1024 + 16 * lane) % span, st + 1024 * (6 * wave + j));
    };
    for (int c = 0; c < S - 1; ++c) issue(c);
    for (int c = 0; c < chunks; ++c) {
        if constexpr (S == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if constexpr (S == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else if constexpr (S == 4) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        issue(c + S - 1);  // past the end: harmless re-reads inside span
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 && lds[blockIdx.x % 1024] == 123 && sink) sink[0] = 1;
}

// same traffic into VGPRs: each lane keeps D float4 loads in flight, waves x 1 KB per instruction
template <int NW, int D>
__global__ __launch_bounds__(64 * NW) void stream_reg_kernel(const uint8_t *src, size_t span, int chunks, int *sink) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t base = ((size_t)blockIdx.x * 24576 * chunks) % span;
    u32x4 acc = {0, 0, 0, 0};
    const int per = 24576 / 1024 / NW;  // wave-instructions per chunk per wave
    for (int c = 0; c < chunks * per; c += D) {
        u32x4 v[D];
#pragma unroll
        for (int d = 0; d < D; ++d)
            v[d] = *reinterpret_cast<const u32x4 *>(src + (base + ((size_t)(c + d) * NW + wave) * 1024 + 16 * lane) % span);
#pragma unroll
        for (int d = 0; d < D; ++d) acc ^= v[d];
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u && sink) sink[0] = 1;
}

// glds with NW waves per workgroup (CB KB per chunk), S stages (S - 1 chunks in flight)
template <int NW, int S, int CB = 24>
__global__ __launch_bounds__(64 * NW) void stream_glds_w_kernel(const uint8_t *src, size_t span, int chunks, int *sink) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[S * CB * 1024];
    constexpr int P = CB / NW;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t base = ((size_t)blockIdx.x * 24576 * chunks) % span;
    auto issue = [&](int c) {
        uint8_t *st = lds + (c % S) * CB * 1024;
        const size_t off = base + (size_t)c * CB * 1024;
#pragma unroll
        for (int j = 0; j < P; ++j)
            glds16(src + (off + (size_t)(P * wave + j) * 1024 + 16 * lane) % span, st + 1024 * (P * wave + j));
    };
    for (int c = 0; c < S - 1; ++c) issue(c);
    for (int c = 0; c < chunks * 24 / CB; ++c) {
        if constexpr (S == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if constexpr (S * P == 9) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
        else if constexpr (S * P == 12) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else if constexpr (S * P == 6) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else if constexpr (S * P == 8) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        issue(c + S - 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 && lds[blockIdx.x % 1024] == 123 && sink) sink[0] = 1;
}

template <typename F>
float time_it(int reps, F &&launch) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 10; ++i) launch(i);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) launch(i);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms * 1000.f / reps;
}


// ---------------------------------------------------------------------------------------------
// Mainloop lab: the fused layer's GEMM phase alone (64 blocks x 128 rows, K = 320 as plane tiles,
// 4 column tiles of 80), wave layouts WM x WN per K-group, KG K-groups (group g multiplies the
// chunks c with c % KG == g; one barrier per KG chunks), DMA / MFMA switchable to find the bound.
// ---------------------------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN, int KG, bool DMA, bool MFMA, int S = 2, bool BPIPE = false, int OCC = 1>
__global__ __launch_bounds__(64 * WM * WN * KG, OCC) void ml_kernel(const uint8_t *A, const uint8_t *Bw, int nkc, int n_tiles,
                                                             float *sink) {
    constexpr int NW = WM * WN * KG, TM = BM / WM / 16, TN = BN / WN / 16;
    constexpr int APL = BM * 64, BPL = BN * 64, STAGE = 3 * APL + 3 * BPL;
    constexpr int AP = 3 * BM / 16, BP = 3 * BN / 16;
    constexpr int APW = (AP + NW - 1) / NW, BPW = (BP + NW - 1) / NW;
    static_assert(KG == 1 || S == 2, "K-groups use two stages");
    __shared__ __attribute__((aligned(16))) uint8_t lds[(S > 2 ? S : 2 * KG) * STAGE];
    const int tile = xcd_tile(blockIdx.x, gridDim.x);
    const int blk = tile / n_tiles, nt = tile % n_tiles;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int grp = wave / (WM * WN), wl = wave % (WM * WN);
    const int wi = wl / WN, wj = wl % WN, g = lane >> 4, i16 = lane & 15;
    int asrc[APW], bsrc[BPW];
#pragma unroll
    for (int j = 0; j < APW; ++j) {
        const int q = 64 * (j * NW + wave) + lane, p = (q / (BM * 4)) % 3, r = (q >> 2) % BM, sl = q & 3;
        asrc[j] = p * APL + r * 64 + 16 * (sl ^ ((r >> 1) & 3));
    }
#pragma unroll
    for (int j = 0; j < BPW; ++j) {
        const int q = 64 * (j * NW + wave) + lane, p = (q / (BN * 4)) % 3, r = (q >> 2) % BN, sl = q & 3;
        bsrc[j] = p * BPL + r * 64 + 16 * (sl ^ ((r >> 1) & 3));
    }
    const uint8_t *ab = A + (size_t)blk * nkc * 3 * APL;
    const uint8_t *bb = Bw + (size_t)nt * nkc * 3 * BPL;
    auto issue = [&](int kc, int buf) {
        if constexpr (DMA) {
            uint8_t *st = lds + buf * STAGE;
#pragma unroll
            for (int j = 0; j < APW; ++j)
                if (AP % NW == 0 || j * NW + wave < AP) glds16(ab + (size_t)kc * 3 * APL + asrc[j], st + 1024 * (j * NW + wave));
#pragma unroll
            for (int j = 0; j < BPW; ++j)
                if (BP % NW == 0 || j * NW + wave < BP)
                    glds16(bb + (size_t)kc * 3 * BPL + bsrc[j], st + 3 * APL + 1024 * (j * NW + wave));
        }
    };
    int ao[TM], bo[TN];
#pragma unroll
    for (int a = 0; a < TM; ++a) ao[a] = x6_slot(wi * (BM / WM) + a * 16 + i16, g);
#pragma unroll
    for (int b = 0; b < TN; ++b) bo[b] = 3 * APL + x6_slot(wj * (BN / WN) + b * 16 + i16, g);
    floatx4 acc[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
    auto compute = [&](const uint8_t *st) {
        constexpr int PA[6] = {0, 0, 1, 0, 2, 1}, PB[6] = {0, 1, 0, 2, 0, 1};
        if constexpr (BPIPE && MFMA) {
            // B fragments one column tile at a time (two in flight): 24 instead of 12 TN registers
            bf16x8 af[TM][3], bq[2][3];
#pragma unroll
            for (int p = 0; p < 3; ++p) {
#pragma unroll
                for (int a = 0; a < TM; ++a) af[a][p] = *reinterpret_cast<const bf16x8 *>(st + p * APL + ao[a]);
                bq[0][p] = *reinterpret_cast<const bf16x8 *>(st + p * BPL + bo[0]);
            }
#pragma unroll
            for (int b = 0; b < TN; ++b) {
                if (b + 1 < TN)
#pragma unroll
                    for (int p = 0; p < 3; ++p) bq[(b + 1) & 1][p] = *reinterpret_cast<const bf16x8 *>(st + p * BPL + bo[b + 1]);
#pragma unroll
                for (int t = 0; t < 6; ++t)
#pragma unroll
                    for (int a = 0; a < TM; ++a)
                        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a][PA[t]], bq[b & 1][PB[t]], acc[a][b], 0, 0, 0);
            }
            return;
        }
        bf16x8 af[TM][3], bfr[TN][3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
#pragma unroll
            for (int a = 0; a < TM; ++a) af[a][p] = *reinterpret_cast<const bf16x8 *>(st + p * APL + ao[a]);
#pragma unroll
            for (int b = 0; b < TN; ++b) bfr[b][p] = *reinterpret_cast<const bf16x8 *>(st + p * BPL + bo[b]);
        }
        if constexpr (MFMA) {
#pragma unroll
            for (int t = 0; t < 6; ++t)
#pragma unroll
                for (int a = 0; a < TM; ++a)
#pragma unroll
                    for (int b = 0; b < TN; ++b)
                        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a][PA[t]], bfr[b][PB[t]], acc[a][b], 0, 0, 0);
        } else {
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b) acc[a][b][0] += (float)(af[a][0][0] + bfr[b][2][1]);
        }
    };
    if constexpr (S > 2) {
        int mine = 0;
#pragma unroll
        for (int j = 0; j < APW; ++j) mine += AP % NW == 0 || j * NW + wave < AP;
#pragma unroll
        for (int j = 0; j < BPW; ++j) mine += BP % NW == 0 || j * NW + wave < BP;
        for (int c = 0; c < S - 1; ++c) issue(c, c);
        for (int kc = 0; kc < nkc; ++kc) {
            wait_vmcnt(min(S - 2, nkc - 1 - kc) * mine);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            if (kc + S - 1 < nkc) issue(kc + S - 1, (kc + S - 1) % S);
            compute(lds + (kc % S) * STAGE);
        }
    }
    const int nsc = S > 2 ? 0 : (nkc + KG - 1) / KG;
    if (S == 2)
        for (int q = 0; q < KG; ++q) issue(q, q);
    for (int sc = 0; sc < nsc; ++sc) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (sc + 1 < nsc)
            for (int q = 0; q < KG; ++q)
                if ((sc + 1) * KG + q < nkc) issue((sc + 1) * KG + q, ((sc + 1) & 1) * KG + q);
        if (sc * KG + grp < nkc) compute(lds + ((sc & 1) * KG + grp) * STAGE);
    }
    float s = 0.f;
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) s += acc[a][b][0] + acc[a][b][3];
    if (s == 1234.5f) sink[threadIdx.x] = s;
}

static void mainloop_lab(int reps) {
    const int nblk = 64, nkc = 10, BM = 128, NTILES = 4;
    const size_t abytes = (size_t)nblk * nkc * 3 * BM * 64, bbytes = (size_t)NTILES * nkc * 3 * 80 * 64;
    const int NA = 8;
    uint8_t *A[NA], *B;
    float *sink;
    for (int i = 0; i < NA; ++i) {
        CK(hipMalloc(&A[i], abytes));
        CK(hipMemset(A[i], 0x3c, abytes));
    }
    CK(hipMalloc(&B, bbytes));
    CK(hipMemset(B, 0x3c, bbytes));
    CK(hipMalloc(&sink, 4096 * 4));
    hipStream_t s2[2];
    CK(hipStreamCreateWithFlags(&s2[0], hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2[1], hipStreamNonBlocking));
    // single: one launch at a time (L2 / MALL state of a rotating A set); pair: two launches in flight on
    // two streams (does a second workgroup per CU co-reside and overlap?), time per launch
    auto run = [&](const char *name, auto kern, int nthreads) {
        hipFuncAttributes fa{};
        CK(hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(kern)));
        float us = time_it(reps, [&](int i) {
            hipLaunchKernelGGL(kern, dim3(nblk * NTILES), dim3(nthreads), 0, 0, A[i % NA], B, nkc, NTILES, sink);
        });
        float usp = 0;
        {
            hipEvent_t a, b;
            CK(hipEventCreate(&a));
            CK(hipEventCreate(&b));
            for (int w = 0; w < 2; ++w) {
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(a, 0));
                CK(hipStreamWaitEvent(s2[0], a, 0));
                CK(hipStreamWaitEvent(s2[1], a, 0));
                for (int i = 0; i < reps; ++i)
                    hipLaunchKernelGGL(kern, dim3(nblk * NTILES), dim3(nthreads), 0, s2[i & 1], A[i % NA], B, nkc, NTILES, sink);
                hipEvent_t e0, e1;
                CK(hipEventCreate(&e0));
                CK(hipEventCreate(&e1));
                CK(hipEventRecord(e0, s2[0]));
                CK(hipEventRecord(e1, s2[1]));
                CK(hipStreamWaitEvent(0, e0, 0));
                CK(hipStreamWaitEvent(0, e1, 0));
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, a, b));
                usp = ms * 1000.f / reps;
                CK(hipEventDestroy(e0));
                CK(hipEventDestroy(e1));
            }
            CK(hipEventDestroy(a));
            CK(hipEventDestroy(b));
        }
        printf("mainloop %-40s %8.2f us  two streams %8.2f us/launch  vgpr %d lds %zu\n", name, us, usp, fa.numRegs,
               fa.sharedSizeBytes);
    };
    run("8x1 KG1 (current)", ml_kernel<128, 80, 8, 1, 1, true, true>, 512);
    run("8x1 KG1 no-DMA", ml_kernel<128, 80, 8, 1, 1, false, true>, 512);
    run("8x1 KG1 DMA-only", ml_kernel<128, 80, 8, 1, 1, true, false>, 512);
    run("8x1 KG1 BP", ml_kernel<128, 80, 8, 1, 1, true, true, 2, true>, 512);
    run("8x1 KG1 BP no-DMA", ml_kernel<128, 80, 8, 1, 1, false, true, 2, true>, 512);
    run("8x1 KG1 BP occ4", ml_kernel<128, 80, 8, 1, 1, true, true, 2, true, 4>, 512);
    run("8x1 KG2 (16 waves)", ml_kernel<128, 80, 8, 1, 2, true, true>, 1024);
    run("8x1 KG2 DMA-only", ml_kernel<128, 80, 8, 1, 2, true, false>, 1024);
    run("4x1 KG2", ml_kernel<128, 80, 4, 1, 2, true, true>, 512);
    run("4x1 KG1 BP", ml_kernel<128, 80, 4, 1, 1, true, true, 2, true>, 256);
    run("8x1 S3", ml_kernel<128, 80, 8, 1, 1, true, true, 3>, 512);
    CK(hipStreamDestroy(s2[0]));
    CK(hipStreamDestroy(s2[1]));
    for (int i = 0; i < NA; ++i) CK(hipFree(A[i]));
    CK(hipFree(B));
    CK(hipFree(sink));
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 200;
    if (argc > 2 && std::string(argv[2]) == "mainloop") {
        mainloop_lab(reps);
        return 0;
    }
    const Shape shapes[] = {{"K32  polymer B64", 6272, 320, 32}, {"K64  polymer B64", 6272, 320, 64},
                            {"W_i  polymer B64", 6272, 320, 160}, {"W_h  polymer B64", 6272, 320, 320},
                            {"W_o  polymer B64", 2304, 320, 480}, {"W_h  zinc B512 H512", 25728, 512, 512}};
    {
        float us = time_it(reps, [&](int) { hipLaunchKernelGGL(empty_kernel, dim3(490), dim3(256), 0, 0, nullptr); });
        printf("%-22s %-26s %8.2f us\n", "launch", "empty 490 x 256", us);
    }
    {
        uint8_t *buf;
        const size_t big = (size_t)512 << 20;
        CK(hipMalloc(&buf, big));
        CK(hipMemset(buf, 1, big));
        auto run_s = [&](const char *nm, auto kern, size_t span, int grid) {
            const int chunks = 20;
            float us = time_it(50, [&](int) { hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, buf, span, chunks, nullptr); });
            const double bytes = (double)grid * chunks * 24576;
            printf("stream %s span %4zu MB grid %4d: %7.2f us  %6.2f TB/s  %6.1f GB/s per CU\n", nm, span >> 20, grid, us,
                   bytes / us * 1e-6, bytes / us * 1e-3 / 256);
        };
        auto run_w = [&](const char *nm, auto kern, int nt, size_t span, int grid) {
            const int chunks = 20;
            float us = time_it(50, [&](int) { hipLaunchKernelGGL(kern, dim3(grid), dim3(nt), 0, 0, buf, span, chunks, nullptr); });
            const double bytes = (double)grid * chunks * 24576;
            printf("stream %s span %4zu MB grid %4d: %7.2f us  %6.2f TB/s  %6.1f GB/s per CU\n", nm, span >> 20, grid, us,
                   bytes / us * 1e-6, bytes / us * 1e-3 / 256);
        };
        for (size_t span : {(size_t)2 << 20, (size_t)64 << 20})
            for (int grid : {256, 512, 1024}) {
                run_s("glds4w S=2", stream_lds_kernel<2>, span, grid);
                run_w("glds8w S=2", stream_glds_w_kernel<8, 2>, 512, span, grid);
                run_w("glds8w S=3", stream_glds_w_kernel<8, 3>, 512, span, grid);
                run_w("glds8w S=4", stream_glds_w_kernel<8, 4>, 512, span, grid);
                run_w("glds8w S=3 36K", stream_glds_w_kernel<8, 3, 32>, 512, span, grid);
                run_w("glds16w S=2", stream_glds_w_kernel<16, 2, 32>, 1024, span, grid);
                run_w("glds16w S=3", stream_glds_w_kernel<16, 3, 32>, 1024, span, grid);
                run_w("reg4w D=2", stream_reg_kernel<4, 2>, 256, span, grid);
                run_w("reg4w D=6", stream_reg_kernel<4, 6>, 256, span, grid);
                run_w("reg8w D=3", stream_reg_kernel<8, 3>, 512, span, grid);
            }
        CK(hipFree(buf));
    }
    if (argc > 2) return 0;  // streaming only
    std::mt19937 rng(1);
    std::uniform_real_distribution<float> U(-1.f, 1.f);
    for (const Shape &S : shapes) {
        const int NA = 8;
        std::vector<float> hA((size_t)S.M * S.K), hB((size_t)S.N * S.K), hR((size_t)S.M * S.N);
        for (auto &v : hA) v = U(rng);
        for (auto &v : hB) v = U(rng) * 0.05f;
        for (auto &v : hR) v = U(rng);
        float *dA[NA], *dB, *dY, *dR;
        for (int i = 0; i < NA; ++i) {
            CK(hipMalloc(&dA[i], hA.size() * 4));
            CK(hipMemcpy(dA[i], hA.data(), hA.size() * 4, hipMemcpyHostToDevice));
        }
        CK(hipMalloc(&dB, hB.size() * 4));
        CK(hipMalloc(&dY, hR.size() * 4));
        CK(hipMalloc(&dR, hR.size() * 4));
        CK(hipMemcpy(dB, hB.data(), hB.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(dR, hR.data(), hR.size() * 4, hipMemcpyHostToDevice));
        // fp64 reference on 64 sampled rows: Y = relu(R + A B^T)
        std::vector<int> rows;
        for (int i = 0; i < 64; ++i) rows.push_back((int)((long long)i * 7919 % S.M));
        std::vector<double> ref(rows.size() * S.N);
        double refmax = 0;
        for (size_t ri = 0; ri < rows.size(); ++ri)
            for (int n = 0; n < S.N; ++n) {
                double s = hR[(size_t)rows[ri] * S.N + n];
                for (int k = 0; k < S.K; ++k) s += (double)hA[(size_t)rows[ri] * S.K + k] * hB[(size_t)n * S.K + k];
                ref[ri * S.N + n] = s > 0 ? s : 0;
                refmax = fmax(refmax, fabs(ref[ri * S.N + n]));
            }
        auto check = [&]() {
            std::vector<float> y(hR.size());
            CK(hipMemcpy(y.data(), dY, y.size() * 4, hipMemcpyDeviceToHost));
            double e = 0;
            for (size_t ri = 0; ri < rows.size(); ++ri)
                for (int n = 0; n < S.N; ++n) e = fmax(e, fabs(y[(size_t)rows[ri] * S.N + n] - ref[ri * S.N + n]));
            return e / refmax;
        };
        Epi epi{};
        epi.kind = EPI_ACT; epi.act = ACT_RELU; epi.resid = dR; epi.Y = dY; epi.ld = S.N;
        // f32 MFMA baseline (gemm_nt16_kernel<64,64,2,2>)
        {
            NtParams P{};
            P.lda0 = S.K; P.ka0 = S.K; P.b = dB; P.ldb = S.K; P.M = S.M; P.N = S.N; P.epi = epi;
            P.tiles_m = S.M / 64; P.tiles_n = S.N / 64;
            float us = time_it(reps, [&](int i) {
                P.a0 = dA[i % NA];
                hipLaunchKernelGGL((gemm_nt16_kernel<64, 64, 2, 2>), dim3(P.tiles_m * P.tiles_n), dim3(256), 0, 0, P);
            });
            printf("%-22s %-26s %8.2f us  err %.2e\n", S.name, "f32 nt16 64x64", us, check());
        }
        auto run_x6 = [&](const char *name, auto kern, int bm) {
            X6Params X{};
            X.lda0 = S.K; X.ka0 = S.K; X.bf = dB; X.ldb = S.K; X.M = S.M; X.N = S.N; X.epi = epi;
            X.tiles_m = S.M / bm; X.tiles_n = S.N / 64;
            float us = time_it(reps, [&](int i) {
                X.a0 = dA[i % NA];
                hipLaunchKernelGGL(kern, dim3(X.tiles_m * X.tiles_n), dim3(4 * bm), 0, 0, X);
            });
            printf("%-22s %-26s %8.2f us  err %.2e\n", S.name, name, us, check());
        };
        run_x6("x6 64x64 k32 split", gemm_x6_kernel<64, 32>, 64);
        if (S.M % 128 == 0) run_x6("x6 128x64 k32 split", gemm_x6_kernel<128, 32>, 128);
        if (S.K % 64 == 0) run_x6("x6 64x64 k64 split", gemm_x6_kernel<64, 64>, 64);
        // both operands pre-split into plane tiles (split once, outside the timing)
        {
            uint8_t *pA[NA], *pB;
            const size_t abytes = (size_t)S.M * S.K * 6, bbytes = (size_t)S.N * S.K * 6;
            for (int i = 0; i < NA; ++i) {
                CK(hipMalloc(&pA[i], abytes));
                hipLaunchKernelGGL(split_tiles_kernel, dim3(1024), dim3(256), 0, 0, dA[i], S.K, S.M, S.K, pA[i]);
            }
            CK(hipMalloc(&pB, bbytes));
            hipLaunchKernelGGL(split_tiles_kernel, dim3(1024), dim3(256), 0, 0, dB, S.K, S.N, S.K, pB);
            CK(hipDeviceSynchronize());
            auto run_p = [&](const char *name, auto kern, int bm, int nthreads) {
                X6PParams X{};
                X.kp0 = S.K; X.ka0 = S.K; X.b = pB; X.kpb = S.K; X.M = S.M; X.N = S.N; X.epi = epi;
                X.tiles_m = S.M / bm; X.tiles_n = S.N / 64;
                float us = time_it(reps, [&](int i) {
                    X.a0 = pA[i % NA];
                    hipLaunchKernelGGL(kern, dim3(X.tiles_m * X.tiles_n), dim3(nthreads), 0, 0, X);
                });
                printf("%-22s %-26s %8.2f us  err %.2e\n", S.name, name, us, check());
            };
            run_p("x6g 64x64 glds 8w", gemm_x6g_kernel, 64, 512);
            // the split itself (what a producer pays to write A as planes instead of fp32)
            float us = time_it(reps, [&](int i) {
                hipLaunchKernelGGL(split_tiles_kernel, dim3(1024), dim3(256), 0, 0, dA[i % NA], S.K, S.M, S.K, pA[i % NA]);
            });
            printf("%-22s %-26s %8.2f us\n", S.name, "split A -> planes", us);
            for (int i = 0; i < NA; ++i) CK(hipFree(pA[i]));
            CK(hipFree(pB));
        }
        fflush(stdout);
        for (int i = 0; i < NA; ++i) CK(hipFree(dA[i]));
        CK(hipFree(dB));
        CK(hipFree(dY));
        CK(hipFree(dR));
    }
    return 0;
}
