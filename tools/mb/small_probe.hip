// small_probe.hip -- where the time of 1 Mi x 64-byte MD5 records (cfg3) goes.  One process,
// interleaved variants, medians of 20-launch bursts over 7 rotating copies (HBM-resident):
//   dma     the product's LDS-ring kernel (digest_fixed_dma_kernel, 64-byte stages)
//   direct  per-lane 16-byte buffer loads into VGPRs, next group prefetched (digest_small_kernel)
//   ld      `direct` without hashing (loads, one xor, store)
//   hash    `direct` without loads (words from the lane id)
//   ...     the same at 2 / 4 / 8 waves per SIMD
// Measured (MI355X, medians): dma 25.7 us; direct 26.2 (4/SIMD), 26.6 (2), 27.9 (8), 26.7 (16, one
// group per wave); loads only 22.9 / 23.3; hashing only 23.4 (1/SIMD), 22.4 (2), 22.1 (4), 22.0 (8).
// Hashing alone takes as long at one wave per SIMD as at eight: the MD5 step mix runs at the
// SIMD's VALU throughput (~5 cycles per op at the clock this load holds), not at a lone-wave issue
// limit, and the two halves (22 us each) overlap to 25-26 us.  The product keeps the dma kernel.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../brb_framework_amd/csrc/gpu -I../../include \
//          small_probe.hip -o small_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
#include <cstdio>
#include <vector>

#include "digest_dma.h"
#include "md5_device.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

namespace {
struct Md5Alg {
    using State = Md5State;
    static BRB_DEV State iv() { return md5_iv(); }
    static BRB_DEV void compress(State &st, uint32_t (&w)[16]) { md5_compress(st, w); }
    static BRB_DEV void finish(State &st, uint32_t (&w)[16], uint32_t t, uint64_t len) { md5_finish(st, w, t, len); }
    static BRB_DEV void pad_only(State &st, uint64_t len) { md5_pad_only(st, len); }
    template <bool A>
    static BRB_DEV void store(uint8_t *out, uint64_t r, const State &st)
    {
        reinterpret_cast<uint4 *>(out)[r] = make_uint4(st.a, st.b, st.c, st.d);
    }
};
}  // namespace

// MODE 0 full, 1 loads only, 2 hashing only.  rec_len == 64.
template <int WAVES, int MODE>
__global__ __launch_bounds__(64 * WAVES) void small_k(const uint8_t *__restrict__ data, uint64_t n_rec, uint8_t *__restrict__ out)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t n_groups = (n_rec + 63) / 64;
    const uint64_t wstride = uint64_t(gridDim.x) * WAVES;
    uint64_t g = uint64_t(blockIdx.x) * WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (g >= n_groups)
        return;
    auto load = [&](uint64_t g, uint32_t (&w)[16]) {
        if (MODE == 2) {
#pragma unroll
            for (int i = 0; i < 16; i++)
                w[i] = uint32_t(g) * 977u + lane * 31u + i;
            return;
        }
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(data + g * 4096), 0, 4096, 0x00020000);
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, int(lane * 64 + 16 * q), 0, 2);
            w[4 * q] = v[0];
            w[4 * q + 1] = v[1];
            w[4 * q + 2] = v[2];
            w[4 * q + 3] = v[3];
        }
    };
    uint32_t nx[16];
    load(g, nx);
    for (;;) {
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; i++)
            w[i] = nx[i];
        const uint64_t gn = g + wstride;
        if (gn < n_groups)
            load(gn, nx);
        Md5State st = md5_iv();
        if (MODE == 1) {
#pragma unroll
            for (int i = 0; i < 16; i++)
                st.a ^= w[i];
        } else {
            md5_compress(st, w);
            md5_pad_only(st, 64);
        }
        reinterpret_cast<uint4 *>(out)[g * 64 + lane] = make_uint4(st.a, st.b, st.c, st.d);
        g = gn;
        if (g >= n_groups)
            break;
    }
}

int main()
{
    const uint64_t n = 1 << 20, L = 64, bytes = n * L;
    const int ROT = 7;
    uint8_t *d;
    uint8_t *o;
    CK(hipMalloc(&d, bytes * ROT));
    CK(hipMalloc(&o, n * 16));
    std::vector<uint8_t> h(bytes * ROT);
    for (size_t i = 0; i < h.size(); i++)
        h[i] = uint8_t(i * 2654435761u >> 13);
    CK(hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint64_t groups = n / 64;
    struct V {
        const char *name;
        std::function<void(const uint8_t *)> run;
    };
    auto grid4 = [&](int wpc, int waves) { return unsigned(std::min<uint64_t>(groups / waves, uint64_t(cus) * wpc / waves)); };
    std::vector<V> vs = {
        {"dma (product)", [&](const uint8_t *p) { brb_digest::digest_fixed_dma_kernel<Md5Alg, 4, 2, 1, true><<<1024, 256, 0, s>>>(p, 64, n, o); }},
        {"direct 4/SIMD", [&](const uint8_t *p) { small_k<4, 0><<<grid4(16, 4), 256, 0, s>>>(p, n, o); }},
        {"direct 2/SIMD", [&](const uint8_t *p) { small_k<4, 0><<<grid4(8, 4), 256, 0, s>>>(p, n, o); }},
        {"direct 8/SIMD", [&](const uint8_t *p) { small_k<4, 0><<<grid4(32, 4), 256, 0, s>>>(p, n, o); }},
        {"direct 16/SIMD (1 group/wave)", [&](const uint8_t *p) { small_k<4, 0><<<unsigned(groups / 4), 256, 0, s>>>(p, n, o); }},
        {"ld only 4/SIMD", [&](const uint8_t *p) { small_k<4, 1><<<grid4(16, 4), 256, 0, s>>>(p, n, o); }},
        {"ld only 16/SIMD", [&](const uint8_t *p) { small_k<4, 1><<<unsigned(groups / 4), 256, 0, s>>>(p, n, o); }},
        {"hash only 1/SIMD", [&](const uint8_t *p) { small_k<4, 2><<<grid4(4, 4), 256, 0, s>>>(p, n, o); }},
        {"hash only 2/SIMD", [&](const uint8_t *p) { small_k<4, 2><<<grid4(8, 4), 256, 0, s>>>(p, n, o); }},
        {"hash only 4/SIMD", [&](const uint8_t *p) { small_k<4, 2><<<grid4(16, 4), 256, 0, s>>>(p, n, o); }},
        {"hash only 8/SIMD", [&](const uint8_t *p) { small_k<4, 2><<<grid4(32, 4), 256, 0, s>>>(p, n, o); }},
    };
    std::vector<std::vector<float>> t(vs.size());
    for (int round = 0; round < 8; round++)
        for (size_t v = 0; v < vs.size(); v++) {
            for (int w = 0; w < 3; w++)
                vs[v].run(d + bytes * (w % ROT));
            CK(hipEventRecord(e0, s));
            for (int k = 0; k < 20; k++)
                vs[v].run(d + bytes * (k % ROT));
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t[v].push_back(ms * 1000.f / 20);
        }
    for (size_t v = 0; v < vs.size(); v++) {
        std::sort(t[v].begin(), t[v].end());
        printf("%-32s %7.2f us  (min %.2f)\n", vs[v].name, t[v][t[v].size() / 2], t[v][0]);
    }
    return 0;
}
