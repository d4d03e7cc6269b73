// Round 6 probe: what bounds the layer's chunk loop?  The loop of h2_mainloop_pairs (csrc/gemm_x6.hpp)
// without the layer around it: 512-thread workgroups, waves 4-7 copy each 32-column chunk (A 16 KB: 128 rows
// x 2 fp16 planes; B 10 KB: 80 rows x 2 planes) by LDS-DMA into a ring of NS stages, one s_barrier per chunk;
// waves 0-3 either only pass the barriers (MODE 0) or read their fragments and issue the 30 MFMAs per chunk
// of the layer (MODE 1).  Grid = blocks x 4 column tiles (XCD-grouped as the layer), A per block, B per
// column tile (shared by every block, as W_h).  Reports the launch time (events) and each workgroup's
// loop time (s_memtime, wave 0) per chunk.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ring_probe tools/ring_probe.hip && tools/ring_probe
#include <hip/hip_runtime.h>

#include "../polymer-chemprop_amd/csrc/gemm_x6.hpp"

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                                    \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                            \
        }                                                                                        \
    } while (0)

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ void glds16(const void *g, uint8_t *lds_wave_base) {
    const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void_t *)lds_wave_base);
    uint32_t saved;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(saved) : "s"(l), "v"(g) : "memory");
}

template <int N>
__device__ __forceinline__ void vmwait() {
    static_assert(N >= 0 && N < 64, "vmcnt");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int N = 0>
__device__ __forceinline__ void vmwait_n(int n) {
    if constexpr (N < 63) {
        if (n == N) { vmwait<N>(); return; }
        vmwait_n<N + 1>(n);
    } else {
        vmwait<63>();
    }
}

__device__ __forceinline__ int xcd_tile(int b, int ntiles) {
    const int base = ntiles >> 3, rem = ntiles & 7;
    const int x = b & 7, local = b >> 3;
    return x * base + (x < rem ? x : rem) + local;
}

constexpr int ACH = 16384, BCH = 10240, STAGE = ACH + BCH;

// MODE 0: consumers pass the barriers only; 1: fragment reads + 30 MFMAs per chunk; 2: copies of A only
// (the B pieces skipped); 3: copies of B only
template <int NS, int MODE>
__global__ __launch_bounds__(512, 2) void ring_probe(const uint8_t *A, const uint8_t *B, int nchunks,
                                                   unsigned long long *cyc, float *sink) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, w4 = wave & 3;
    const int tile = xcd_tile(blockIdx.x, gridDim.x), blk = tile >> 2, nt = tile & 3;
    const uint8_t *a_src = A + (size_t)blk * nchunks * ACH, *b_src = B + (size_t)nt * nchunks * BCH;
    const bool loader = wave >= 4;
    constexpr bool DA = MODE != 3, DB = MODE != 2;
    const int mine = (DA ? 4 : 0) + (DB ? (w4 < 2 ? 3 : 2) : 0);
    auto issue = [&](int kc) {
        uint8_t *st = lds + (kc % NS) * STAGE;
        if (DA)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = 4 * j + w4;
                glds16(a_src + (size_t)kc * ACH + c * 1024 + lane * 16, st + c * 1024);
            }
        if (DB)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int c = 4 * j + w4;
                if (c < 10) glds16(b_src + (size_t)kc * BCH + c * 1024 + lane * 16, st + ACH + c * 1024);
            }
    };
    floatx4 acc[2][5];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 5; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
    f16x8 af[2][2], bq[5][2];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (loader)
        for (int c = 0; c < NS - 1 && c < nchunks; ++c) issue(c);
    for (int kc = 0; kc < nchunks; ++kc) {
        if (loader) {
            constexpr int M7 = (DA ? 4 : 0) + (DB ? 3 : 0), M6 = (DA ? 4 : 0) + (DB ? 2 : 0);
            if (nchunks - 1 - kc >= NS - 2 && mine == M7) vmwait<(NS - 2) * M7>();
            else if (nchunks - 1 - kc >= NS - 2 && mine == M6) vmwait<(NS - 2) * M6>();
            else vmwait_n(std::min(NS - 2, nchunks - 1 - kc) * mine);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (loader) {
            if (kc + NS - 1 < nchunks) issue(kc + NS - 1);
        } else if (MODE == 1 || MODE == 4 || MODE == 5) {
            // (4: the B fragments read at chunk 0 only -- no per-chunk B reads; 5: the A fragments likewise)
            const uint8_t *st = lds + (kc % NS) * STAGE, *sb = st + ACH;
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                if (MODE != 5 || kc == 0)
#pragma unroll
                    for (int a = 0; a < 2; ++a)
                        af[a][p] = *reinterpret_cast<const f16x8 *>(st + p * 8192 + wd::x6_slot(32 * w4 + 16 * a + (lane & 15), lane >> 4));
                if (MODE != 4 || kc == 0)
#pragma unroll
                    for (int b = 0; b < 5; ++b)
                        bq[b][p] = *reinterpret_cast<const f16x8 *>(sb + p * 5120 + wd::x6_slot(16 * b + (lane & 15), lane >> 4));
            }
#pragma unroll
            for (int b = 0; b < 5; ++b)
#pragma unroll
                for (int a = 0; a < 2; ++a) {
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[a][0], bq[b][0], acc[a][b], 0, 0, 0);
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[a][0], bq[b][1], acc[a][b], 0, 0, 0);
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[a][1], bq[b][0], acc[a][b], 0, 0, 0);
                }
        }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
    if ((MODE == 1 || MODE == 4 || MODE == 5) && !loader) {
        float s = 0.f;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 5; ++b) s += acc[a][b][0] + acc[a][b][1] + acc[a][b][2] + acc[a][b][3];
        if (s == 12345.f) sink[tid] = s;  // (keeps the MFMAs)
    }
}

// NL loader waves (waves 4 .. 4 + NL - 1) sharing the 26 pieces of a chunk (A 16, B 10): piece c to loader
// wave c % NL; consumers as MODE 1 (or none: MODE 0)
template <int NS, int MODE, int NL, bool CW = false>
__global__ __launch_bounds__(64 * (4 + NL)) void ring_probe_nl(const uint8_t *A, const uint8_t *B, int nchunks,
                                                              unsigned long long *cyc, float *sink) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, w4 = wave & 3;
    const int tile = xcd_tile(blockIdx.x, gridDim.x), blk = tile >> 2, nt = tile & 3;
    const uint8_t *a_src = A + (size_t)blk * nchunks * ACH, *b_src = B + (size_t)nt * nchunks * BCH;
    const bool loader = wave >= 4;
    const int lw = wave - 4;
    constexpr int NP = 26, PMAX = (NP + NL - 1) / NL;
    const int mine = loader ? (NP - lw + NL - 1) / NL : 0;
    auto issue = [&](int kc) {
        uint8_t *st = lds + (kc % NS) * STAGE;
#pragma unroll
        for (int j = 0; j < PMAX; ++j) {
            const int c = lw + NL * j;
            if (c < 16) glds16(a_src + (size_t)kc * ACH + c * 1024 + lane * 16, st + c * 1024);
            else if (c < NP) glds16(b_src + (size_t)kc * BCH + (c - 16) * 1024 + lane * 16, st + ACH + (c - 16) * 1024);
        }
    };
    floatx4 acc[2][5];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 5; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
    f16x8 af[2][2], bq[5][2];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (loader)
        for (int c = 0; c < NS - 1 && c < nchunks; ++c) issue(c);
    const int m_s = __builtin_amdgcn_readfirstlane(mine);
    for (int kc = 0; kc < nchunks; ++kc) {
        if (loader) {
            // (CW: the steady-state counts as constants, as ring_probe's loop)
            constexpr int M7 = (NP + NL - 1) / NL, M6 = NP / NL;
            if (CW && nchunks - 1 - kc >= NS - 2 && m_s == M7) vmwait<(NS - 2) * M7>();
            else if (CW && nchunks - 1 - kc >= NS - 2 && m_s == M6) vmwait<(NS - 2) * M6>();
            else vmwait_n(std::min(NS - 2, nchunks - 1 - kc) * m_s);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (loader) {
            if (kc + NS - 1 < nchunks) issue(kc + NS - 1);
        } else if (MODE == 1) {
            const uint8_t *st = lds + (kc % NS) * STAGE, *sb = st + ACH;
#pragma unroll
            for (int p = 0; p < 2; ++p) {
#pragma unroll
                for (int a = 0; a < 2; ++a)
                    af[a][p] = *reinterpret_cast<const f16x8 *>(st + p * 8192 + wd::x6_slot(32 * w4 + 16 * a + (lane & 15), lane >> 4));
#pragma unroll
                for (int b = 0; b < 5; ++b)
                    bq[b][p] = *reinterpret_cast<const f16x8 *>(sb + p * 5120 + wd::x6_slot(16 * b + (lane & 15), lane >> 4));
            }
#pragma unroll
            for (int b = 0; b < 5; ++b)
#pragma unroll
                for (int a = 0; a < 2; ++a) {
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[a][0], bq[b][0], acc[a][b], 0, 0, 0);
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[a][0], bq[b][1], acc[a][b], 0, 0, 0);
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[a][1], bq[b][0], acc[a][b], 0, 0, 0);
                }
        }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
    if (MODE == 1 && !loader) {
        float s = 0.f;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 5; ++b) s += acc[a][b][0] + acc[a][b][1] + acc[a][b][2] + acc[a][b][3];
        if (s == 12345.f) sink[tid] = s;
    }
}

// the layer's own loop (csrc/gemm_x6.hpp h2_mainloop_pairs<128, 80>), one scale for every chunk
template <int FRAG>
__global__ __launch_bounds__(512, 2) void real_pairs(const uint8_t *A, const uint8_t *B, int nchunks,
                                                   unsigned long long *cyc, float *sink) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[wd::h2p_lds_bytes<128, 80>()];
    const int tid = threadIdx.x, lane = tid & 63;
    const int tile = xcd_tile(blockIdx.x, gridDim.x), blk = tile >> 2, nt = tile & 3;
    const uint32_t wv = lane < 4 ? 0x3f800000u : 0u;
    wd::floatx4 acc[2][5];
    int se;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    wd::h2_mainloop_pairs<128, 80, FRAG>(A + (size_t)blk * nchunks * ACH, B + (size_t)nt * nchunks * BCH, nchunks, 128, wv, 80,
                                   lds, acc, se);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
    if (tid < 256) {
        float s = (float)se;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 5; ++b) s += acc[a][b][0] + acc[a][b][1] + acc[a][b][2] + acc[a][b][3];
        if (s == 12345.f) sink[tid] = s;
    }
}

// the producer of A: every byte written by 16-byte stores, as the layer epilogue writes its pair tiles
__global__ void fill(uint4 *p, size_t n, uint32_t v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4(v, v + 1, v + 2, (uint32_t)i);
}

typedef void (*probe_fn)(const uint8_t *, const uint8_t *, int, unsigned long long *, float *);
int run_k(probe_fn k, int lds, int ns, const char *name, uint8_t *A, uint8_t *B, int nblk, int nchunks, bool fresh,
          unsigned long long *cyc, float *sink, uint4 *fillp, size_t filln, int bytes, int nthr = 512) {
    const int grid = nblk * 4;
    if (lds) CK(hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 30;
    float tot = 0.f;
    std::vector<double> per;
    for (int r = 0; r < reps + 3; ++r) {
        if (fresh) fill<<<1024, 256>>>(fillp, filln, r);
        CK(hipEventRecord(e0));
        k<<<grid, nthr, lds>>>(A, B, nchunks, cyc, sink);
        CK(hipGetLastError());
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 3) {
            tot += ms;
            std::vector<unsigned long long> h(grid);
            CK(hipMemcpy(h.data(), cyc, grid * sizeof(unsigned long long), hipMemcpyDeviceToHost));
            std::sort(h.begin(), h.end());
            per.push_back((double)h[grid / 2] / nchunks);
        }
    }
    std::sort(per.begin(), per.end());
    std::printf("%-28s NS=%d grid=%4d chunks=%2d %-5s  launch %7.2f us  loop/chunk p50 %6.0f cyc  (%.1f B/clk/WG)\n", name, ns,
                grid, nchunks, fresh ? "fresh" : "warm", 1000.f * tot / reps, per[per.size() / 2],
                bytes / per[per.size() / 2]);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return 0;
}
template <int NS, int MODE>
int run(const char *name, uint8_t *A, uint8_t *B, int nblk, int nchunks, bool fresh, unsigned long long *cyc,
        float *sink, uint4 *fillp, size_t filln) {
    return run_k(ring_probe<NS, MODE>, NS * STAGE, NS, name, A, B, nblk, nchunks, fresh, cyc, sink, fillp, filln,
                 MODE == 2 ? ACH : MODE == 3 ? BCH : STAGE);
}

int main() {
    const int maxblk = 128, maxch = 40;
    uint8_t *A, *B;
    unsigned long long *cyc;
    float *sink;
    const size_t abytes = (size_t)maxblk * maxch * ACH, bbytes = (size_t)4 * maxch * BCH;
    CK(hipMalloc(&A, abytes));
    CK(hipMalloc(&B, bbytes));
    CK(hipMalloc(&cyc, 4096 * sizeof(unsigned long long)));
    CK(hipMalloc(&sink, 4096 * sizeof(float)));
    CK(hipMemset(A, 0x3c, abytes));
    CK(hipMemset(B, 0x3c, bbytes));
    uint4 *fp = reinterpret_cast<uint4 *>(A);
    int rc = 0;
    const size_t fn = (size_t)64 * 10 * ACH / 16;  // the A the 64-block, 10-chunk runs read
    for (int fresh = 0; fresh < 1; ++fresh) {
        rc |= run<3, 0>("barriers only", A, B, 64, 10, fresh, cyc, sink, fp, fn);
        rc |= run<3, 1>("copies + MFMA (swizzled)", A, B, 64, 10, fresh, cyc, sink, fp, fn);
        rc |= run_k(real_pairs<0>, 0, 3, "pairs FRAG 0", A, B, 64, 10, fresh, cyc, sink, fp, fn, STAGE);
        rc |= run_k(ring_probe_nl<3, 0, 4>, 3 * STAGE, 3, "NL 4, barriers only", A, B, 64, 10, fresh, cyc, sink, fp, fn, STAGE, 512);
        rc |= run_k(ring_probe_nl<3, 0, 4, true>, 3 * STAGE, 3, "NL 4 CW, barriers only", A, B, 64, 10, fresh, cyc, sink, fp, fn, STAGE, 512);
        rc |= run_k(ring_probe_nl<3, 1, 4, true>, 3 * STAGE, 3, "NL 4 CW, copies + MFMA", A, B, 64, 10, fresh, cyc, sink, fp, fn, STAGE, 512);
        rc |= run_k(ring_probe_nl<3, 1, 6, true>, 3 * STAGE, 3, "NL 6 CW, copies + MFMA", A, B, 64, 10, fresh, cyc, sink, fp, fn, STAGE, 640);
        rc |= run_k(ring_probe_nl<3, 1, 8, true>, 3 * STAGE, 3, "NL 8 CW, copies + MFMA", A, B, 64, 10, fresh, cyc, sink, fp, fn, STAGE, 768);
        rc |= run_k(ring_probe_nl<3, 0, 8, true>, 3 * STAGE, 3, "NL 8 CW, barriers only", A, B, 64, 10, fresh, cyc, sink, fp, fn, STAGE, 768);
    }
    return rc;
}
