// dma_pattern.hip -- memory-side floor of LDS-DMA staging patterns for lane-per-record digests.
// A wave owns 64 records of stride L; a "stage" brings S bytes of every record (S = 64 * BPS) into
// LDS with 4 * BPS buffer_load_dwordx4 ... lds (each instruction: 1024 / S records x S bytes).
// Compared with a contiguous stream of the same bytes.  No hashing: xor of the staged words.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../brb_framework_amd/csrc/gpu dma_pattern.hip -o dmapat
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "dma_stage.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int BPS, int P, int WAVES, bool LINE_ALIGNED = false>
__global__ __launch_bounds__(64 * WAVES) void stage_kernel(const uint8_t *data, uint32_t L, uint64_t n_rec, uint32_t *out)
{
    constexpr int S = 64 * BPS, SLOT = 64 * S, NI = 4 * BPS, RPI = 1024 / S;   // records per instruction
    __shared__ __attribute__((aligned(16))) uint8_t ring[WAVES * P * SLOT];
    const uint32_t lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t n_groups = n_rec / 64, wave0 = uint64_t(blockIdx.x) * WAVES + wv, wstride = uint64_t(gridDim.x) * WAVES;
    if (wave0 >= n_groups) return;
    uint8_t *my = ring + wv * P * SLOT;
    const uint32_t lds0 = uint32_t(reinterpret_cast<uintptr_t>(my));
    // lane j of instruction q: record q*RPI + j/(S/16), granule (j % (S/16)) ^ f(rec)
    constexpr int G = S / 16;
    const uint32_t rec_in = lane / G, gran = lane % G;
    uint32_t vo[NI];
#pragma unroll
    for (int q = 0; q < NI; q++) {
        const uint32_t rec = q * RPI + rec_in;
        const uint32_t f = G == 4 ? (rec >> 2) & 3 : G == 8 ? (rec >> 1) & 7 : rec & 15;
        vo[q] = (LINE_ALIGNED ? (rec * L) & ~127u : rec * L) + ((gran ^ f) % G) * 16;
    }
    const uint32_t nstage = (L / 64) / BPS;
    const uint32_t my_groups = uint32_t((n_groups - wave0 + wstride - 1) / wstride), total = my_groups * nstage;
    uint32_t acc = 0;
    uint64_t g_is = wave0;
    uint32_t st_is = 0;
    auto issue = [&](uint32_t slot) {
        const brb_dma::v4i rs = brb_dma::make_rsrc(data + g_is * 64 * L + st_is * S, ~0ull);
#pragma unroll
        for (int q = 0; q < NI; q++) {
            uint32_t keep;
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(vo[q]), "s"(rs), "s"(lds0 + slot * SLOT + q * 1024) : "memory");
        }
        if (++st_is == nstage) { st_is = 0; g_is += wstride; }
    };
#pragma unroll
    for (int i = 0; i < P - 1; i++) if (uint32_t(i) < total) issue(i);
    uint32_t slot = 0;
    for (uint32_t s = 0; s < total; s++) {
        if (s + P - 1 < total) {
            issue((s + P - 1) % P);
            brb_dma::wait_vmcnt<NI * (P - 1)>();
        } else {
            brb_dma::wait_vmcnt<0>();
        }
        const uint4 *row = reinterpret_cast<const uint4 *>(my + slot * SLOT + lane * S);
#pragma unroll
        for (int k = 0; k < G; k++) { const uint4 v = row[k]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
        slot = slot + 1 == P ? 0 : slot + 1;
    }
    out[(wave0 * 64 + lane) % 65536] = acc;
}

// contiguous streaming reference: each wave reads its group's region in 1 KiB pieces via DMA
template <int P, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void linear_kernel(const uint8_t *data, uint32_t L, uint64_t n_rec, uint32_t *out)
{
    constexpr int SLOT = 4096;
    __shared__ __attribute__((aligned(16))) uint8_t ring[WAVES * P * SLOT];
    const uint32_t lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t n_groups = n_rec / 64, wave0 = uint64_t(blockIdx.x) * WAVES + wv, wstride = uint64_t(gridDim.x) * WAVES;
    if (wave0 >= n_groups) return;
    uint8_t *my = ring + wv * P * SLOT;
    const uint32_t lds0 = uint32_t(reinterpret_cast<uintptr_t>(my));
    const uint32_t nstage = (64 * L) / 4096;
    const uint32_t my_groups = uint32_t((n_groups - wave0 + wstride - 1) / wstride), total = my_groups * nstage;
    uint32_t acc = 0;
    uint64_t g_is = wave0;
    uint32_t st_is = 0;
    auto issue = [&](uint32_t slot) {
        const brb_dma::v4i rs = brb_dma::make_rsrc(data + g_is * 64 * L + st_is * 4096, ~0ull);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            uint32_t keep;
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(q * 1024 + lane * 16), "s"(rs), "s"(lds0 + slot * SLOT + q * 1024) : "memory");
        }
        if (++st_is == nstage) { st_is = 0; g_is += wstride; }
    };
#pragma unroll
    for (int i = 0; i < P - 1; i++) if (uint32_t(i) < total) issue(i);
    uint32_t slot = 0;
    for (uint32_t s = 0; s < total; s++) {
        if (s + P - 1 < total) { issue((s + P - 1) % P); brb_dma::wait_vmcnt<4 * (P - 1)>(); }
        else brb_dma::wait_vmcnt<0>();
        const uint4 *row = reinterpret_cast<const uint4 *>(my + slot * SLOT + lane * 64);
#pragma unroll
        for (int k = 0; k < 4; k++) { const uint4 v = row[k]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
        slot = slot + 1 == P ? 0 : slot + 1;
    }
    out[(wave0 * 64 + lane) % 65536] = acc;
}

using Kern = void (*)(const uint8_t *, uint32_t, uint64_t, uint32_t *);

int main(int argc, char **argv)
{
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 1048576;
    const uint32_t L = argc > 2 ? atoi(argv[2]) : 1536;   // stages = floor(L / S)
    const int nrot = std::max<int>(2, int(700e6 / double(n * L)) + 1);
    std::vector<uint8_t *> d(nrot);
    for (int i = 0; i < nrot; i++) { CK(hipMalloc(&d[i], n * L + 8192)); CK(hipMemset(d[i], i + 1, n * L)); }
    uint32_t *o;
    CK(hipMalloc(&o, 65536 * 4));
    struct V { const char *name; Kern k; int waves; int lds; };
    std::vector<V> vs = {
        {"S=64  P3 (product pattern)", stage_kernel<1, 3, 4>, 4, 4 * 3 * 4096},
        {"S=64  P4", stage_kernel<1, 4, 4>, 4, 4 * 4 * 4096},
        {"S=128 P2", stage_kernel<2, 2, 4>, 4, 4 * 2 * 8192},
        {"S=128 P3", stage_kernel<2, 3, 4>, 4, 4 * 3 * 8192},
        {"S=128 P2 line-aligned", stage_kernel<2, 2, 4, true>, 4, 4 * 2 * 8192},
        {"S=128 P3 line-aligned", stage_kernel<2, 3, 4, true>, 4, 4 * 3 * 8192},
        {"S=256 P2", stage_kernel<4, 2, 4>, 4, 4 * 2 * 16384},
        {"linear 4KiB P3", linear_kernel<3, 4>, 4, 4 * 3 * 4096},
        {"linear 4KiB P4", linear_kernel<4, 4>, 4, 4 * 4 * 4096},
    };
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<std::vector<float>> t(vs.size());
    int it = 0;
    for (int rep = 0; rep < 15; rep++)
        for (size_t v = 0; v < vs.size(); v++) {
            const int per_cu = std::max(1, std::min(8, 160 * 1024 / vs[v].lds));
            const uint64_t groups = n / 64, need = (groups + vs[v].waves - 1) / vs[v].waves;
            const unsigned grid = unsigned(std::min<uint64_t>(need, 256ull * per_cu));
            hipEventRecord(e0);
            hipLaunchKernelGGL(vs[v].k, dim3(grid), dim3(64 * vs[v].waves), 0, 0, d[it++ % nrot], L, n, o);
            hipEventRecord(e1);
            CK(hipEventSynchronize(e1));
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            t[v].push_back(ms * 1e3f);
        }
    printf("n=%llu L=%u (%.1f MB per pass)\n", (unsigned long long)n, L, n * L / 1e6);
    for (size_t v = 0; v < vs.size(); v++) {
        std::sort(t[v].begin(), t[v].end());
        const float med = t[v][t[v].size() / 2];
        printf("%-30s median %8.2f us  min %8.2f  %6.0f GB/s\n", vs[v].name, med, t[v][0], n * L / (med * 1e-6) / 1e9);
    }
    return 0;
}
