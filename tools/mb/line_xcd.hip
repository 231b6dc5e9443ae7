// line_xcd.hip -- can the cfg5 shard's cross-XCD spread be recovered by splitting its groups over the
// XCDs by weight?  (Round 6; tools/mb/line_xcd_kernel.h.)  Steps, one process:
//   1. parity: the product kernel vs the weighted kernel at an even and at a skewed split;
//   2. feedback: from an even split, a few rounds of 20 launches; after each round the groups of
//      class x (workgroups blockIdx % 8 = x) are set in proportion to groups_x / T_x, T_x = the mean
//      end of the class's waves from the round's last launch (half-damped);
//   3. interleaved timing: product, even split, weighted split.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../brb_framework_amd/csrc/gpu line_xcd.hip -o line_xcd
// Run:   ./line_xcd [n_rec=1048576] [rec_len=1500] [rounds=5] [launches=40]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
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

// groups per class -> prefix sums
static brb_mb_xcd::XSplit split_of(const std::vector<uint64_t> &gx)
{
    brb_mb_xcd::XSplit s;
    s.s[0] = 0;
    for (int x = 0; x < 8; x++)
        s.s[x + 1] = s.s[x] + uint32_t(gx[x]);
    return s;
}

// shares (any positive weights) -> integer groups per class summing to n_groups
static std::vector<uint64_t> groups_of(const std::vector<double> &wt, uint64_t n_groups)
{
    double tot = 0;
    for (double w : wt) tot += w;
    std::vector<uint64_t> g(8);
    uint64_t used = 0;
    std::vector<std::pair<double, int>> rem;
    for (int x = 0; x < 8; x++) {
        const double e = double(n_groups) * wt[x] / tot;
        g[x] = uint64_t(std::floor(e));
        used += g[x];
        rem.push_back({e - std::floor(e), x});
    }
    std::sort(rem.rbegin(), rem.rend());
    for (uint64_t i = 0; used < n_groups; i++, used++)
        g[rem[i % 8].second]++;
    return g;
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
    const void *kx = hi ? (const void *)(KX)brb_mb_xcd::digest_line_xcd_kernel<AlgLit, 8, true, true>
                        : (const void *)(KX)brb_mb_xcd::digest_line_xcd_kernel<AlgLit, 8, true, false>;
    const uint64_t nwaves = uint64_t(grid) * 8;
    uint64_t *stamp;
    CK(hipMalloc(&stamp, nwaves * 3 * 8));
    auto run_p = [&](const uint8_t *src) {
        uint64_t nn = n;
        uint32_t LL = L;
        uint8_t *oo = o;
        void *a[] = {&src, &LL, &nn, &oo};
        CK(hipLaunchKernel(kp, dim3(grid), dim3(512), a, 0, 0));
    };
    auto run_x = [&](const uint8_t *src, brb_mb_xcd::XSplit s, uint64_t *st) {
        uint64_t nn = n;
        uint32_t LL = L;
        uint8_t *oo = o;
        void *a[] = {&src, &LL, &nn, &oo, &s, &st};
        CK(hipLaunchKernel(kx, dim3(grid), dim3(512), a, 0, 0));
    };
    // classes: workgroups b with b % 8 == x; groups in proportion to the class sizes
    std::vector<double> csize(8, 0.0);
    for (unsigned b = 0; b < grid; b++) csize[b & 7] += 1.0;
    const std::vector<uint64_t> g_even = groups_of(csize, groups);
    // 1. parity
    std::vector<uint8_t> ref(n * 16), got(n * 16);
    CK(hipMemset(o, 0xA5, n * 16));
    run_p(d[0]);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(ref.data(), o, n * 16, hipMemcpyDeviceToHost));
    std::vector<double> skew(8);
    for (int c = 0; c < 8; c++) skew[c] = csize[c] * (1.0 + 0.1 * c);
    for (const auto &gx : {g_even, groups_of(skew, groups)}) {
        CK(hipMemset(o, 0xA5, n * 16));
        run_x(d[0], split_of(gx), nullptr);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got.data(), o, n * 16, hipMemcpyDeviceToHost));
        if (memcmp(ref.data(), got.data(), n * 16) != 0) {
            uint64_t r = 0;
            while (memcmp(&ref[16 * r], &got[16 * r], 16) == 0) r++;
            printf("MISMATCH weighted kernel at record %llu\n", (unsigned long long)r);
            return 2;
        }
    }
    printf("n=%llu L=%u grid=%u: digests identical (product, even split, skewed split)\n", (unsigned long long)n, L, grid);
    fflush(stdout);
    int it = 0;
    // 2. feedback
    std::vector<uint64_t> gx = g_even;
    std::vector<uint64_t> hs(nwaves * 3);
    for (int fr = 0; fr < 8; fr++) {
        for (int i = 0; i < 20; i++) run_x(d[it++ % nrot], split_of(gx), i == 19 ? stamp : nullptr);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(hs.data(), stamp, hs.size() * 8, hipMemcpyDeviceToHost));
        uint64_t t0 = ~0ull, t1 = 0;
        for (uint64_t w = 0; w < nwaves; w++) { t0 = std::min(t0, hs[3 * w]); t1 = std::max(t1, hs[3 * w + 1]); }
        std::vector<double> se(8, 0.0), mx(8, 0.0);
        std::vector<int> cnt(8, 0), match(8, 0);
        for (uint64_t w = 0; w < nwaves; w++) {
            const int c = int((w / 8) & 7);
            const double e = double(hs[3 * w + 1] - t0) * 0.01;   // us
            se[c] += e;
            mx[c] = std::max(mx[c], e);
            cnt[c]++;
            match[c] += hs[3 * w + 2] == uint64_t(c);
        }
        std::vector<double> wt(8);
        printf("feedback %d: span %.1f us |", fr, double(t1 - t0) * 0.01);
        for (int c = 0; c < 8; c++) {
            const double mean = se[c] / cnt[c];
            printf(" c%d %llu g, end %.1f/%.1f%s", c, (unsigned long long)gx[c], mean, mx[c], match[c] == cnt[c] ? "" : " (xcc!=cls)");
            wt[c] = double(gx[c]) / mean;
        }
        printf("\n");
        // half-damped move toward the measured rates
        const std::vector<uint64_t> target = groups_of(wt, groups);
        std::vector<double> mix(8);
        for (int c = 0; c < 8; c++) mix[c] = 0.5 * double(gx[c]) + 0.5 * double(target[c]);
        gx = groups_of(mix, groups);
        fflush(stdout);
    }
    // 3. interleaved timing
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const char *names[3] = {"product", "even split", "weighted split"};
    std::vector<std::vector<double>> us(3);
    for (int r = 0; r < rounds; r++)
        for (int vi = 0; vi < 3; vi++) {
            auto go = [&]() {
                if (vi == 0) run_p(d[it++ % nrot]);
                else run_x(d[it++ % nrot], split_of(vi == 1 ? g_even : gx), nullptr);
            };
            float tot = 0;
            while (tot < 300.f) {
                CK(hipEventRecord(a));
                for (int i = 0; i < 20; i++) go();
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                tot += ms;
            }
            CK(hipEventRecord(a));
            for (int i = 0; i < nl; i++) go();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            us[vi].push_back(1000.0 * ms / nl);
            printf("round %d %-16s %.2f us/launch  %.4f of 8 TB/s\n", r, names[vi], us[vi].back(),
                   double(n) * L / (us[vi].back() * 1e-6) / 8e12);
            fflush(stdout);
        }
    for (int vi = 0; vi < 3; vi++)
        printf("MEDIAN %-16s %.2f us  frac %.4f\n", names[vi], med(us[vi]), double(n) * L / (med(us[vi]) * 1e-6) / 8e12);
    return 0;
}
