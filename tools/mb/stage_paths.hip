// stage_paths.hip -- how fast can one wave per SIMD (cfg2's occupancy) pull 98.3 MB through each
// load path, from HBM (7 rotating copies) and from the Infinity Cache (one copy)?
//   vload: global_load_dwordx4 into VGPRs (xor-reduced), D KiB in flight per wave
//   dma:   buffer_load_dwordx4 ... lds (LDS-DMA, the digest kernels' path), D KiB in flight
// Each wave streams its own contiguous 96 000-byte region (cfg2: 64 records x 1500 B).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 stage_paths.hip -o stagep
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));

// D loads of 1 KiB (64 lanes x 16 B) in flight per wave; region = per-wave bytes
template <int D>
__global__ __launch_bounds__(256) void vload(const uint8_t *data, uint32_t region, uint32_t *out)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w = uint64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
    const v4i *p = reinterpret_cast<const v4i *>(data + w * region);
    const uint32_t n = region / 1024;
    uint32_t acc = 0;
    for (uint32_t i = 0; i < n; i += D) {
        v4i v[D];
#pragma unroll
        for (int j = 0; j < D; j++)
            v[j] = __builtin_nontemporal_load(p + (i + j < n ? i + j : n - 1) * 64 + lane);
#pragma unroll
        for (int j = 0; j < D; j++)
            acc ^= uint32_t(v[j].x ^ v[j].y ^ v[j].z ^ v[j].w);
    }
    if (acc == 0x12345678u)
        out[w * 64 + lane] = acc;
}

template <int D>
__global__ __launch_bounds__(256) void dma(const uint8_t *data, uint32_t region, uint32_t *out)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * D * 1024];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t w = uint64_t(blockIdx.x) * 4 + wv;
    const uint64_t base = reinterpret_cast<uint64_t>(data + w * region);
    v4i rs;
    rs.x = __builtin_amdgcn_readfirstlane(int(uint32_t(base)));
    rs.y = __builtin_amdgcn_readfirstlane(int(uint32_t(base >> 32) & 0xFFFF));
    rs.z = int(region);
    rs.w = 0x00020000;
    const uint32_t n = region / 1024;
    const uint32_t m0 = uint32_t(reinterpret_cast<uintptr_t>(lds)) + wv * D * 1024;
    uint32_t acc = 0;
    for (uint32_t i = 0; i < n; i += D) {
#pragma unroll
        for (int j = 0; j < D; j++) {
            const uint32_t vo = (i + j < n ? i + j : n - 1) * 1024 + lane * 16;
            uint32_t keep;
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                         "buffer_load_dwordx4 %1, %2, 0 offen nt lds\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(vo), "s"(rs), "s"(m0 + j * 1024u) : "memory");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        acc ^= *reinterpret_cast<const uint32_t *>(lds + wv * D * 1024 + lane * 4);
    }
    if (acc == 0x12345678u)
        out[w * 64 + lane] = acc;
}

using Kern = void (*)(const uint8_t *, uint32_t, uint32_t *);

int main()
{
    const uint32_t region = 96000 / 1024 * 1024;     // 93 KiB per wave (whole KiB pieces)
    const int waves = 1024;
    const size_t bytes = size_t(region) * waves;
    const int nrot = 7;
    std::vector<uint8_t *> d(nrot);
    for (auto &p : d) { CK(hipMalloc(&p, bytes)); CK(hipMemset(p, 1, bytes)); }
    uint32_t *o;
    CK(hipMalloc(&o, waves * 64 * 4));
    struct V { const char *name; Kern k; };
    V vs[] = {{"vload D=1 ", vload<1>}, {"vload D=2 ", vload<2>}, {"vload D=4 ", vload<4>}, {"vload D=8 ", vload<8>},
              {"dma   D=2 ", dma<2>},   {"dma   D=4 ", dma<4>},   {"dma   D=8 ", dma<8>},   {"dma   D=16", dma<16>}};
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    int it = 0;
    const int nv = int(sizeof(vs) / sizeof(vs[0]));
    std::vector<float> res[2][16];
    for (int r = 0; r < 3; r++)
        for (int rot = 0; rot < 2; rot++)
            for (int vi = 0; vi < nv; vi++) {
                const int nr = rot ? 1 : nrot;
                for (int rep = 0; rep < 2; rep++) {
                    hipEventRecord(a);
                    for (int i = 0; i < 1000; i++)
                        hipLaunchKernelGGL(vs[vi].k, dim3(waves / 4), dim3(256), 0, 0, d[(it++) % nr], region, o);
                    hipEventRecord(b);
                    CK(hipEventSynchronize(b));
                    float ms;
                    hipEventElapsedTime(&ms, a, b);
                    if (rep)
                        res[rot][vi].push_back(ms * 1e3f / 1000);
                }
            }
    for (int rot = 0; rot < 2; rot++)
        for (int vi = 0; vi < nv; vi++) {
            auto v = res[rot][vi];
            std::sort(v.begin(), v.end());
            printf("%s %s  %.2f us  %.2f TB/s\n", vs[vi].name, rot ? "cache" : "HBM  ", v[1], bytes / (v[1] * 1e-6) / 1e12);
        }
    return 0;
}
