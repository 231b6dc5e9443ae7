// rc4_parts.hip -- where does the RC4 batch kernel's time go?  65 536 streams x 1500 B, 4-wave
// workgroups (one wave per SIMD), the product's device code (rc4_device.h, byte_stream.h):
//   full      : BlockSrc -> keystream xor -> Snk (the product's rc4_crypt loop)
//   gen only  : keystream of the same length, xor-reduced, no stream I/O
//   io only   : BlockSrc -> xor constant -> Snk, no keystream
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../brb_framework_amd/csrc/gpu rc4_parts.hip -o rc4parts
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rc4_device.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace brb_rc4;

// BlockSrc with two blocks in flight (experiment: is the product loop waiting on its loads?)
struct BlockSrc2 {
    const uint32_t *p;
    uint32_t sh;
    uint64_t len, ndw, nb;
    uint32_t prev, A[16], B[16];
    BRB_DEV void load(uint64_t b, uint32_t (&L)[16])
    {
        const uint64_t base = 16 * b + 1;
        if (base + 16 <= ndw) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint4 v = ld16_a4(reinterpret_cast<const uint8_t *>(p + base + 4 * q));
                L[4 * q + 0] = v.x; L[4 * q + 1] = v.y; L[4 * q + 2] = v.z; L[4 * q + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; i++)
                L[i] = base + i < ndw ? ldg(p + base + i) : 0u;
        }
    }
    BRB_DEV void init(const uint8_t *a, uint64_t n)
    {
        const uintptr_t ad = reinterpret_cast<uintptr_t>(a);
        p = reinterpret_cast<const uint32_t *>(ad & ~uintptr_t(3));
        sh = uint32_t(ad & 3) * 8;
        len = n;
        ndw = n ? ((ad & 3) + n + 3) / 4 : 0;
        prev = ndw ? ldg(p) : 0u;
        nb = 0;
        load(0, A);
        load(1, B);
    }
    BRB_DEV void fetch(uint32_t (&c)[16])
    {
#pragma unroll
        for (int i = 0; i < 16; i++)
            c[i] = __builtin_amdgcn_alignbit(A[i], i ? A[i - 1] : prev, sh);
        prev = A[15];
#pragma unroll
        for (int i = 0; i < 16; i++)
            A[i] = B[i];
        ++nb;
        load(nb + 1, B);
    }
};

// Wave-cooperative 64-byte block I/O through LDS (experiment): instruction q moves the blocks of
// lanes 16q .. 16q+15, four lanes per block, so one instruction touches 16 lines instead of 64.
// Exchange row r (lane r's block) keeps its 16-byte chunk c at 16 ((c + (r >> 2)) & 3): conflict-free
// for the row-wise and the chunk-wise access.
BRB_DEV uint32_t xoff(uint32_t r, uint32_t c) { return r * 64 + 16 * ((c + (r >> 2)) & 3); }

__constant__ uint32_t g_stride;   // bytes between stream starts (>= L; 1540 = 4-byte aligned, not 64)

template <int MODE>   // 9 coop loads, 10 coop loads + coop stores; 8 product loop with two blocks in flight; 0 full, 1 gen only, 2 io only, 3 io only with 16-byte stores, 4 loads only
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
    const uint64_t off = s * g_stride;
    brb_io::BlockSrc src;
    brb_io::Snk snk;
    if (MODE != 1) {
        src.init(in + off, L);
        snk.init(out + off, L);
    }
    uint4 *o16 = reinterpret_cast<uint4 *>(out + off);
    uint32_t acc = 0;
    const uint64_t nblk = L / 64;
    if (MODE == 9 || MODE == 10) {
        __shared__ __attribute__((aligned(16))) uint8_t xch[4 * 4096];
        const uint32_t lane = threadIdx.x & 63;
        uint8_t *xw = xch + (threadIdx.x >> 6) * 4096;
        // base addresses of the streams this lane serves in instruction q (stream 16q + lane / 4)
        const uint64_t my_in = reinterpret_cast<uint64_t>(in + off), my_out = reinterpret_cast<uint64_t>(out + off);
        uint64_t qin[4], qout[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int src_lane = 16 * q + (lane >> 2);
            qin[q] = (uint64_t(__shfl(uint32_t(my_in >> 32), src_lane)) << 32) | __shfl(uint32_t(my_in), src_lane);
            qout[q] = (uint64_t(__shfl(uint32_t(my_out >> 32), src_lane)) << 32) | __shfl(uint32_t(my_out), src_lane);
            qin[q] += 16 * (lane & 3);
            qout[q] += 16 * (lane & 3);
        }
        uint4 v[4];
        auto issue = [&](uint64_t b) {
#pragma unroll
            for (int q = 0; q < 4; q++)
                v[q] = ld16_a4(reinterpret_cast<const uint8_t *>(qin[q] + 64 * b));
        };
        auto take = [&](uint32_t (&c)[16]) {
#pragma unroll
            for (int q = 0; q < 4; q++)
                *reinterpret_cast<uint4 *>(xw + xoff(16 * q + (lane >> 2), lane & 3)) = v[q];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint4 t = *reinterpret_cast<const uint4 *>(xw + xoff(lane, k));
                c[4 * k] = t.x; c[4 * k + 1] = t.y; c[4 * k + 2] = t.z; c[4 * k + 3] = t.w;
            }
        };
        uint32_t c[16];
        issue(0);
        take(c);
        if (nblk > 1)
            issue(1);
        for (uint64_t b = 0; b < nblk; b++) {
            uint32_t ks[16];
            g.words(ks);
#pragma unroll
            for (int i = 0; i < 16; i++)
                ks[i] ^= c[i];
            if (b + 1 < nblk) {
                take(c);
                if (b + 2 < nblk)
                    issue(b + 2);
            }
            if (MODE == 9) {
                snk.put16(ks);
            } else {
#pragma unroll
                for (int k = 0; k < 4; k++)
                    *reinterpret_cast<uint4 *>(xw + xoff(lane, k)) = make_uint4(ks[4 * k], ks[4 * k + 1], ks[4 * k + 2], ks[4 * k + 3]);
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint4 t = *reinterpret_cast<const uint4 *>(xw + xoff(16 * q + (lane >> 2), lane & 3));
                    st16_a4(reinterpret_cast<uint8_t *>(qout[q] + 64 * b), t.x, t.y, t.z, t.w);
                }
            }
        }
        if (MODE == 9)
            snk.flush();
        g.store(state);
        return;
    }
    if (MODE == 8) {
        BlockSrc2 s2;
        s2.init(in + off, L);
        uint32_t c[16];
        s2.fetch(c);
        for (uint64_t b = 0; b < nblk; b++) {
            uint32_t ks[16];
            g.words(ks);
#pragma unroll
            for (int i = 0; i < 16; i++)
                ks[i] ^= c[i];
            if (b + 1 < nblk)
                s2.fetch(c);
            snk.put16(ks);
        }
        snk.flush();
        g.store(state);
        return;
    }
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

int main(int argc, char **argv)
{
    const uint64_t n = 65536;
    const uint32_t L = 1536;   // whole 64-byte blocks
    const uint32_t S = argc > 1 ? uint32_t(atoi(argv[1])) : L;
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stride), &S, 4));
    printf("stride %u\n", S);
    uint8_t *st, *in, *out;
    uint32_t *sink;
    CK(hipMalloc(&st, n * kStateBytes));
    CK(hipMalloc(&in, n * S + 64));
    CK(hipMalloc(&out, n * S + 64));
    CK(hipMalloc(&sink, 64));
    std::vector<uint8_t> h(n * kStateBytes);
    for (uint64_t i = 0; i < n; i++) {
        for (int x = 0; x < 256; x++) h[i * kStateBytes + x] = uint8_t((x * 167 + i) & 255);
        for (int x = 256; x < int(kStateBytes); x++) h[i * kStateBytes + x] = 0;
    }
    CK(hipMemcpy(st, h.data(), h.size(), hipMemcpyHostToDevice));
    {
        std::vector<uint8_t> hin(n * S);
        for (size_t i = 0; i < hin.size(); i++) hin[i] = uint8_t(i * 2654435761u >> 13);
        CK(hipMemcpy(in, hin.data(), hin.size(), hipMemcpyHostToDevice));
    }
    struct V { const char *name; void (*f)(uint8_t *, const uint8_t *, uint8_t *, uint32_t, uint64_t, uint32_t *); } vs[] = {
        {"full", k<0>}, {"gen only", k<1>}, {"io only", k<2>}, {"io 16B st", k<3>}, {"loads only", k<4>}, {"product", k<5>}, {"prod no st", k<6>}, {"prod no ld", k<7>}, {"prod 2-ahead", k<8>}, {"coop ld", k<9>}, {"coop ld+st", k<10>}};
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
    // coop variants must write what the product loop writes
    std::vector<uint8_t> ref(n * S), got(n * S);
    CK(hipMemcpy(st, h.data(), h.size(), hipMemcpyHostToDevice));
    CK(hipMemset(out, 0, n * S));
    hipLaunchKernelGGL(k<5>, dim3(n / 256), dim3(256), 0, 0, st, in, out, L, n, sink);
    CK(hipMemcpy(ref.data(), out, n * S, hipMemcpyDeviceToHost));
    for (int m = 9; m <= 10; m++) {
        CK(hipMemcpy(st, h.data(), h.size(), hipMemcpyHostToDevice));
        CK(hipMemset(out, 0, n * S));
        if (m == 9) hipLaunchKernelGGL(k<9>, dim3(n / 256), dim3(256), 0, 0, st, in, out, L, n, sink);
        else hipLaunchKernelGGL(k<10>, dim3(n / 256), dim3(256), 0, 0, st, in, out, L, n, sink);
        CK(hipMemcpy(got.data(), out, n * S, hipMemcpyDeviceToHost));
        printf("mode %d output %s\n", m, got == ref ? "matches" : "DIFFERS");
    }
    return 0;
}
