// rc4_parts.hip -- where does the RC4 batch kernel's time go?  65 536 streams x 1500 B, 4-wave
// workgroups (one wave per SIMD), the product's device code (rc4_device.h, byte_stream.h):
//   full      : BlockSrc -> keystream xor -> Snk (the product's rc4_crypt loop)
//   gen only  : keystream of the same length, xor-reduced, no stream I/O
//   io only   : BlockSrc -> xor constant -> Snk, no keystream
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../brb_framework_amd/csrc/gpu rc4_parts.hip -o rc4parts
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "rc4_device.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace brb_rc4;

template <int MODE>   // 0 full, 1 gen only, 2 io only, 3 io only with 16-byte stores, 4 loads only
// 5 product loop (put16, next block taken before the stores), 6 product loop without stores, 7 product loop without loads
__global__ __launch_bounds__(256) void k(uint8_t *states, const uint8_t *in, uint8_t *out, uint32_t L, uint64_t n, uint32_t *sink)
{
    __shared__ __attribute__((aligned(16))) uint8_t slot[kSlotLds];
    const uint64_t s = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    if (s >= n)
        return;
    Gen g;
    g.P.lds = slot;
    g.P.lw = (threadIdx.x & 63) * 4 + (threadIdx.x >> 6);
    uint8_t *state = states + s * kStateBytes;
    if (MODE != 2)
        g.load(state);
    const uint64_t off = s * L;
    brb_io::BlockSrc src;
    brb_io::Snk snk;
    if (MODE != 1) {
        src.init(in + off, L);
        snk.init(out + off, L);
    }
    uint4 *o16 = reinterpret_cast<uint4 *>(out + off);
    uint32_t acc = 0;
    const uint64_t nblk = L / 64;
    if (MODE >= 5) {
        uint32_t c[16];
        if (MODE == 7) {
#pragma unroll
            for (int i = 0; i < 16; i++) c[i] = 0x3C3C3C3Cu + i;
        } else {
            src.fetch(c);
        }
        for (uint64_t b = 0; b < nblk; b++) {
            uint32_t ks[16];
            g.words(ks);
#pragma unroll
            for (int i = 0; i < 16; i++)
                ks[i] ^= c[i];
            if (MODE != 7 && b + 1 < nblk)
                src.fetch(c);
            if (MODE == 6) {
#pragma unroll
                for (int i = 0; i < 16; i++) acc ^= ks[i];
            } else {
                snk.put16(ks);
            }
        }
        snk.flush();
        g.store(state);
        if (acc == 0x12345678u)
            sink[0] = acc;
        return;
    }
    for (uint64_t b = 0; b < nblk; b++) {
        uint32_t c[16], ks[16];
        if (MODE != 1)
            src.fetch(c);
        if (MODE != 2 && MODE != 3 && MODE != 4) {
            g.words(ks);
        } else {
#pragma unroll
            for (int i = 0; i < 16; i++)
                ks[i] = 0x5A5A5A5Au + i;
        }
        if (MODE == 3) {
#pragma unroll
            for (int i = 0; i < 4; i++)
                o16[4 * b + i] = make_uint4(c[4 * i] ^ ks[4 * i], c[4 * i + 1] ^ ks[4 * i + 1], c[4 * i + 2] ^ ks[4 * i + 2],
                                            c[4 * i + 3] ^ ks[4 * i + 3]);
        } else if (MODE == 4) {
#pragma unroll
            for (int i = 0; i < 16; i++)
                acc ^= c[i];
        } else if (MODE != 1) {
#pragma unroll
            for (int i = 0; i < 16; i++)
                snk.put(c[i] ^ ks[i]);
        } else {
#pragma unroll
            for (int i = 0; i < 16; i++)
                acc ^= ks[i];
        }
    }
    if (MODE == 0 || MODE == 2)
        snk.flush();
    if (MODE < 2)
        g.store(state);
    if (acc == 0x12345678u)
        sink[0] = acc;
}

int main()
{
    const uint64_t n = 65536;
    const uint32_t L = 1536;   // whole 64-byte blocks
    uint8_t *st, *in, *out;
    uint32_t *sink;
    CK(hipMalloc(&st, n * kStateBytes));
    CK(hipMalloc(&in, n * L));
    CK(hipMalloc(&out, n * L));
    CK(hipMalloc(&sink, 64));
    std::vector<uint8_t> h(n * kStateBytes);
    for (uint64_t i = 0; i < n; i++) {
        for (int x = 0; x < 256; x++) h[i * kStateBytes + x] = uint8_t((x * 167 + i) & 255);
        for (int x = 256; x < int(kStateBytes); x++) h[i * kStateBytes + x] = 0;
    }
    CK(hipMemcpy(st, h.data(), h.size(), hipMemcpyHostToDevice));
    CK(hipMemset(in, 0x3C, n * L));
    struct V { const char *name; void (*f)(uint8_t *, const uint8_t *, uint8_t *, uint32_t, uint64_t, uint32_t *); } vs[] = {
        {"full", k<0>}, {"gen only", k<1>}, {"io only", k<2>}, {"io 16B st", k<3>}, {"loads only", k<4>}, {"product", k<5>}, {"prod no st", k<6>}, {"prod no ld", k<7>}};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 3; rep++)
        for (auto &v : vs) {
            for (int w = 0; w < 3; w++) hipLaunchKernelGGL(v.f, dim3(n / 256), dim3(256), 0, 0, st, in, out, L, n, sink);
            hipEventRecord(e0);
            for (int w = 0; w < 10; w++) hipLaunchKernelGGL(v.f, dim3(n / 256), dim3(256), 0, 0, st, in, out, L, n, sink);
            hipEventRecord(e1);
            CK(hipEventSynchronize(e1));
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep == 2)
                printf("%-10s %8.1f us per launch  (%.1f ns per byte per stream)\n", v.name, ms * 100, ms * 1e5 / L);
        }
    return 0;
}
