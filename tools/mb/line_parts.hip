// line_parts.hip -- cfg2 (65 536 x 1500 B) through the product's line-aligned MD5 kernel with the
// memory side taken away step by step: (a) records rotated over 7 copies (HBM, as bench.py), (b)
// one copy (the 98 MB batch stays in the 256 MiB Infinity Cache), (c)/(d) the same with the
// compression replaced by an xor of the window (staging only).  Interleaved rounds, medians.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../brb_framework_amd/csrc/gpu line_parts.hip -o lparts
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "digest_dma.h"
#include "line3_kernel.h"
#include "md5_device.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct AlgLit {
    using State = Md5State;
    static BRB_DEV State iv() { return md5_iv(); }
    static BRB_DEV void compress(State &st, uint32_t (&w)[16]) { md5_compress(st, w); }
    static BRB_DEV void finish(State &st, uint32_t (&w)[16], uint32_t t, uint64_t len) { md5_finish(st, w, t, len); }
    static BRB_DEV void pad_only(State &st, uint64_t len) { md5_pad_only(st, len); }
    template <bool A> static BRB_DEV void store(uint8_t *out, uint64_t r, const State &st)
    { reinterpret_cast<uint4 *>(out)[r] = make_uint4(st.a, st.b, st.c, st.d); }
};
struct AlgNull : AlgLit {
    static BRB_DEV void compress(State &st, uint32_t (&w)[16])
    {
        uint32_t x = 0;
#pragma unroll
        for (int i = 0; i < 16; i++) x ^= w[i];
        st.a ^= x;
    }
    static BRB_DEV void finish(State &st, uint32_t (&w)[16], uint32_t, uint64_t) { st.b ^= w[0]; }
    static BRB_DEV void pad_only(State &st, uint64_t len) { st.b ^= uint32_t(len); }
};

using Kern = void (*)(const uint8_t *, uint32_t, uint64_t, uint8_t *);

int main(int argc, char **argv)
{
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 65536;
    const uint32_t L = argc > 2 ? atoi(argv[2]) : 1500;
    const int rounds = argc > 3 ? atoi(argv[3]) : 5;
    const int nrot = 7;
    std::vector<uint8_t> h(n * L);
    uint64_t x = 7;
    for (auto &c : h) { x = x * 6364136223846793005ull + 1442695040888963407ull; c = uint8_t(x >> 56); }
    std::vector<uint8_t *> d(nrot);
    for (auto &p : d) { CK(hipMalloc(&p, n * L + 8192)); CK(hipMemcpy(p, h.data(), n * L, hipMemcpyHostToDevice)); }
    uint8_t *o;
    CK(hipMalloc(&o, n * 16));
    const uint64_t groups = (n + 63) / 64;
    struct V { const char *name; const void *k; int rot; int wg; int line3; };
    V vs[] = {{"md5   HBM (7 copies)", (const void *)(Kern)brb_digest::digest_line_kernel<AlgLit, 8, true, true>, nrot, 8, 0},
              {"md5   MALL (1 copy) ", (const void *)(Kern)brb_digest::digest_line_kernel<AlgLit, 8, true, true>, 1, 8, 0},
              {"stage HBM (7 copies)", (const void *)(Kern)brb_digest::digest_line_kernel<AlgNull, 8, true, true>, nrot, 8, 0},
              {"stage MALL (1 copy) ", (const void *)(Kern)brb_digest::digest_line_kernel<AlgNull, 8, true, true>, 1, 8, 0},
              {"md5   HBM line3     ", (const void *)(Kern)brb_digest::digest_line3_kernel<AlgLit, 4, true, true>, nrot, 4, 1},
              {"md5   MALL line3    ", (const void *)(Kern)brb_digest::digest_line3_kernel<AlgLit, 4, true, true>, 1, 4, 1},
              {"md5   HBM line3 late", (const void *)(Kern)brb_digest::digest_line3_kernel<AlgLit, 4, true, false>, nrot, 4, 1},
              {"stage HBM line3     ", (const void *)(Kern)brb_digest::digest_line3_kernel<AlgNull, 4, true, true>, nrot, 4, 1},
              {"stage MALL line3    ", (const void *)(Kern)brb_digest::digest_line3_kernel<AlgNull, 4, true, true>, 1, 4, 1}};
    const int nv = int(sizeof(vs) / sizeof(vs[0]));
    std::vector<std::vector<float>> us(nv);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    int it = 0;
    for (int r = 0; r < rounds; r++)
        for (int vi = 0; vi < nv; vi++) {
            const V &v = vs[vi];
            const unsigned grid = unsigned(std::min<uint64_t>((groups + v.wg - 1) / (v.line3 ? v.wg : 1), 256));
            const unsigned g2 = v.line3 ? grid : unsigned(std::min<uint64_t>(groups, 256));
            for (int rep = 0; rep < 2; rep++) {      // rep 0 warms the clock and the cache
                hipEventRecord(a);
                for (int i = 0; i < 2000; i++) {
                    const uint8_t *src = d[(it++) % v.rot];
                    uint32_t l = L;
                    uint64_t nn = n;
                    void *args[] = {&src, &l, &nn, &o};
                    CK(hipLaunchKernel(v.k, dim3(g2), dim3(64 * v.wg), args, 0, 0));
                }
                hipEventRecord(b);
                CK(hipEventSynchronize(b));
                float ms;
                hipEventElapsedTime(&ms, a, b);
                if (rep)
                    us[vi].push_back(ms * 1e3f / 2000);
            }
        }
    for (int vi = 0; vi < nv; vi++) {
        auto v = us[vi];
        std::sort(v.begin(), v.end());
        printf("%s  median %.2f us  min %.2f  max %.2f  (%d rounds)\n", vs[vi].name, v[v.size() / 2], v.front(), v.back(), int(v.size()));
    }
    return 0;
}
