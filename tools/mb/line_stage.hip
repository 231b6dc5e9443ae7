// line_stage.hip -- where the window read's round trip goes (round 6).  The compression-only probe
//  spends ~10 % of a lone wave's time between "line landed" and "window in VGPRs":
// 32 ds_read_b32, then lgkmcnt(0) before the refill DMA may overwrite the slot.  Variants of
// tools/mb/line_xcd_kernel.h at an even split (which times as the product): STAGE 0 (the product's
// order), 1 (reads, block 2k-2 on the compiler's per-register waits, then the refill DMA, block
// 2k-1), 2 (the refill DMA after step 15 of block 2k-2); and MAP 1 (each workgroup a contiguous block
// of groups instead of every c_x-th).  Digests compared with the product's first.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../brb_framework_amd/csrc/gpu line_stage.hip -o line_stage
// Run:   ./line_stage [n_rec=1048576] [rec_len=1500] [rounds=5] [launches=40]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "digest_line.h"
#include "line_xcd_kernel.h"
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

using K4 = void (*)(const uint8_t *, uint32_t, uint64_t, uint8_t *);
using KX = void (*)(const uint8_t *, uint32_t, uint64_t, uint8_t *, brb_mb_xcd::XSplit, uint64_t *);

static double med(std::vector<double> v)
{
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

template <bool HI>
static const void *kx(int v)
{
    switch (v) {
    case 1: return (const void *)(KX)brb_mb_xcd::digest_line_xcd_kernel<AlgLit, 8, true, HI, 0, 1>;
    case 2: return (const void *)(KX)brb_mb_xcd::digest_line_xcd_kernel<AlgLit, 8, true, HI, 0, 2>;
    case 3: return (const void *)(KX)brb_mb_xcd::digest_line_xcd_kernel<AlgLit, 8, true, HI, 0, 0, 1>;
    default: return (const void *)(KX)brb_mb_xcd::digest_line_xcd_kernel<AlgLit, 8, true, HI, 0, 0>;
    }
}

int main(int argc, char **argv)
{
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 1048576;
    const uint32_t L = argc > 2 ? atoi(argv[2]) : 1500;
    const int rounds = argc > 3 ? atoi(argv[3]) : 5;
    const int nl = argc > 4 ? atoi(argv[4]) : 40;
    if (L <= 64 || (L & 3)) { printf("rec_len must be > 64 and a multiple of 4\n"); return 1; }
    const int nrot = std::max<int>(2, int(700e6 / double(n * L)) + 1);
    std::vector<uint8_t> h(n * L);
    uint64_t x = 11;
    for (auto &c : h) { x = x * 6364136223846793005ull + 1442695040888963407ull; c = uint8_t(x >> 56); }
    std::vector<uint8_t *> d(nrot);
    for (auto &p : d) { CK(hipMalloc(&p, n * L + 8192)); CK(hipMemcpy(p, h.data(), n * L, hipMemcpyHostToDevice)); }
    uint8_t *o;
    CK(hipMalloc(&o, n * 16));
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const uint64_t groups = (n + 63) / 64;
    const unsigned grid = unsigned(std::min<uint64_t>(groups, uint64_t(cus)));
    const bool hi = brb_digest::line_tail_hi(L);
    const void *kp = hi ? (const void *)(K4)brb_digest::digest_line_kernel<AlgLit, 8, true, true>
                        : (const void *)(K4)brb_digest::digest_line_kernel<AlgLit, 8, true, false>;
    // even split over the classes b % 8, in proportion to their workgroup counts
    brb_mb_xcd::XSplit xs;
    {
        uint64_t c[8] = {0};
        for (unsigned b = 0; b < grid; b++) c[b & 7]++;
        xs.s[0] = 0;
        uint64_t acc = 0;
        for (int k = 0; k < 8; k++) {
            acc += c[k];
            xs.s[k + 1] = uint32_t(groups * acc / grid);
        }
    }
    const char *names[5] = {"product", "stage0", "stage1 split", "stage2 hook", "blocked groups"};
    auto run = [&](int v, const uint8_t *src) {
        uint64_t nn = n;
        uint32_t LL = L;
        uint8_t *oo = o;
        uint64_t *st = nullptr;
        if (v == 0) {
            void *a[] = {&src, &LL, &nn, &oo};
            CK(hipLaunchKernel(kp, dim3(grid), dim3(512), a, 0, 0));
        } else {
            void *a[] = {&src, &LL, &nn, &oo, &xs, &st};
            CK(hipLaunchKernel(hi ? kx<true>(v - 1) : kx<false>(v - 1), dim3(grid), dim3(512), a, 0, 0));
        }
    };
    std::vector<uint8_t> ref(n * 16), got(n * 16);
    for (int v = 0; v < 5; v++) {
        CK(hipMemset(o, 0xA5, n * 16));
        run(v, d[0]);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(v ? got.data() : ref.data(), o, n * 16, hipMemcpyDeviceToHost));
        if (v && memcmp(ref.data(), got.data(), n * 16) != 0) {
            printf("MISMATCH %s\n", names[v]);
            return 2;
        }
    }
    printf("n=%llu L=%u grid=%u: digests identical across the five variants\n", (unsigned long long)n, L, grid);
    fflush(stdout);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<std::vector<double>> us(5);
    int it = 0;
    for (int r = 0; r < rounds; r++)
        for (int v = 0; v < 5; v++) {
            float tot = 0;
            while (tot < 300.f) {
                CK(hipEventRecord(a));
                for (int i = 0; i < 20; i++) run(v, d[it++ % nrot]);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                tot += ms;
            }
            CK(hipEventRecord(a));
            for (int i = 0; i < nl; i++) run(v, d[it++ % nrot]);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            us[v].push_back(1000.0 * ms / nl);
            printf("round %d %-12s %.2f us/launch  %.4f of 8 TB/s\n", r, names[v], us[v].back(),
                   double(n) * L / (us[v].back() * 1e-6) / 8e12);
            fflush(stdout);
        }
    for (int v = 0; v < 5; v++)
        printf("MEDIAN %-12s %.2f us  frac %.4f\n", names[v], med(us[v]), double(n) * L / (med(us[v]) * 1e-6) / 8e12);
    return 0;
}
