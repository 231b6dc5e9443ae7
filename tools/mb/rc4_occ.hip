// rc4_occ.hip -- is the RC4 keystream chain (rc4_device.h Gen, ~140 cycles per byte in the product)
// set by the LDS round trip of one wave, or by the LDS traffic of the CU's other keystream waves?
// The product's generator alone (no stream I/O), one 4-wave workgroup per CU (a dummy dynamic LDS
// allocation keeps a second one off the CU), of which only NW waves run: the per-byte time at NW =
// 1, 2, 4 keystream waves per CU; and NW = 4 with two workgroups per CU (8 keystream waves).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../brb_framework_amd/csrc/gpu rc4_occ.hip -o rc4_occ
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "rc4_device.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace brb_rc4;

// Gen::step with the start of byte T+1 fenced off from the completion of byte T
// (sched_barrier): the patches and the next j address are issued before the wait for S[j_T], so
// after swap T's writes the read of S[j_{T+1}] goes out at once.
BRB_DEV uint32_t step_fenced(Gen &g)
{
    uint32_t a1 = g.r1;
    a1 = g.qaj == g.ad1 ? g.qa : a1;
    a1 = g.paj == g.ad1 ? g.pa : a1;
    a1 = g.aj == g.ad1 ? g.a : a1;
    const uint32_t aj1 = Gen::ad_plus(g.aj, a1);
    const uint32_t ad3 = Gen::ad_next(g.ad2);
    const uint32_t r3 = g.rd(ad3);
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t b = g.rb;
    g.wr(g.ai, b);
    g.wr(g.aj, g.a);
    const uint32_t rb1 = g.rd(aj1);
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t k = g.rd(g.ad(g.a + b));
    g.qaj = g.paj;
    g.qa = g.pa;
    g.pai = g.ai;
    g.paj = g.aj;
    g.pa = g.a;
    g.a = a1;
    g.rb = rb1;
    g.ai = g.ad1;
    g.aj = aj1;
    g.r1 = g.r2;
    g.ad1 = g.ad2;
    g.r2 = r3;
    g.ad2 = ad3;
    return k;
}

template <int NW, bool FENCE = false>
__global__ __launch_bounds__(256) void gen_only(uint8_t *states, uint32_t L, uint32_t *sink)
{
    __shared__ __attribute__((aligned(16))) uint8_t slot[kSlotLds];
    extern __shared__ uint8_t pad[];
    const uint32_t wv = threadIdx.x >> 6;
    if (wv >= uint32_t(NW))
        return;
    const uint64_t s = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    Gen g;
    g.P.lds = slot;
    g.P.lw = (threadIdx.x & 63) * 4 + wv;
    uint8_t *state = states + s * kStateBytes;
    g.load(state);
    uint32_t acc = 0;
    for (uint32_t b = 0; b < L / 64; b++) {
        uint32_t ks[16];
        if (FENCE) {
            uint32_t kb[64];
#pragma unroll
            for (int t = 0; t < 64; t++)
                kb[t] = step_fenced(g);
#pragma unroll
            for (int w = 0; w < 16; w++)
                ks[w] = kb[4 * w] | (kb[4 * w + 1] << 8) | (kb[4 * w + 2] << 16) | (kb[4 * w + 3] << 24);
        } else {
            g.words(ks);
        }
#pragma unroll
        for (int i = 0; i < 16; i++)
            acc ^= ks[i];
    }
    g.store(state);
    if (acc == 0x12345678u)
        sink[0] = acc + pad[0];
}

int main()
{
    const uint32_t L = 1536;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const uint64_t n = uint64_t(2 * cus) * 256;     // enough states for two workgroups per CU
    uint8_t *st;
    uint32_t *sink;
    CK(hipMalloc(&st, n * kStateBytes));
    CK(hipMalloc(&sink, 64));
    std::vector<uint8_t> h(n * kStateBytes, 0);
    for (uint64_t i = 0; i < n; i++)
        for (int x = 0; x < 256; x++) h[i * kStateBytes + x] = uint8_t((x * 167 + i) & 255);
    CK(hipMemcpy(st, h.data(), h.size(), hipMemcpyHostToDevice));
    struct V { const char *name; void (*f)(uint8_t *, uint32_t, uint32_t *); int nw; unsigned grid; size_t dyn; } vs[] = {
        {"1 wave / CU", gen_only<1>, 1, unsigned(cus), 80 * 1024},
        {"2 waves / CU", gen_only<2>, 2, unsigned(cus), 80 * 1024},
        {"4 waves / CU", gen_only<4>, 4, unsigned(cus), 80 * 1024},
        {"8 waves / CU", gen_only<4>, 4, unsigned(2 * cus), 0},
        {"fenced 1 / CU", gen_only<1, true>, 1, unsigned(cus), 80 * 1024},
        {"fenced 4 / CU", gen_only<4, true>, 4, unsigned(cus), 80 * 1024},
        {"fenced 8 / CU", gen_only<4, true>, 4, unsigned(2 * cus), 0},
    };
    {   // the fenced step must leave the same states as the product's
        std::vector<uint8_t> a(n * kStateBytes), b(n * kStateBytes);
        CK(hipMemcpy(st, h.data(), h.size(), hipMemcpyHostToDevice));
        hipLaunchKernelGGL(gen_only<4>, dim3(2 * cus), dim3(256), 0, 0, st, L, sink);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(a.data(), st, a.size(), hipMemcpyDeviceToHost));
        CK(hipMemcpy(st, h.data(), h.size(), hipMemcpyHostToDevice));
        hipLaunchKernelGGL((gen_only<4, true>), dim3(2 * cus), dim3(256), 0, 0, st, L, sink);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(b.data(), st, b.size(), hipMemcpyDeviceToHost));
        printf("states after %u bytes: %s\n", L, a == b ? "identical" : "DIFFER");
        if (a != b)
            return 2;
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int rep = 0; rep < 3; rep++)
        for (auto &v : vs) {
            for (int w = 0; w < 5; w++) hipLaunchKernelGGL(v.f, dim3(v.grid), dim3(256), v.dyn, 0, st, L, sink);
            CK(hipEventRecord(e0));
            for (int w = 0; w < 20; w++) hipLaunchKernelGGL(v.f, dim3(v.grid), dim3(256), v.dyn, 0, st, L, sink);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1000.0 / 20;
            if (rep == 2)
                printf("%-14s %8.1f us per launch  %.1f ns per byte (x 2.1 GHz = %.0f cycles)\n", v.name, us,
                       us * 1000.0 / L, us * 1000.0 / L * 2.1);
        }
    return 0;
}
