// line_ab.hip -- interleaved A/B of the line digest kernel: round 5's form (per-group window and
// DMA-offset setup, per-lane selects; tools/mb/line_r05_kernel.h) against the product's
// (digest_line.h: group-invariant tables built once per wave, launch-uniform choices as template
// arguments / slot parity).  Same MD5 compression, same grid (one 8-wave workgroup per CU), same
// rotated inputs (>= 700 MB, past the Infinity Cache).  Every variant's digests are compared with the
// first variant's before timing.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../brb_framework_amd/csrc/gpu line_ab.hip -o line_ab
// Run:   ./line_ab [n_rec=1048576] [rec_len=1500] [rounds=5] [launches=100]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "digest_line.h"
#include "line3r_kernel.h"
#include "line4_kernel.h"
#include "line_r05_kernel.h"
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
using K6 = void (*)(const uint8_t *, uint32_t, uint64_t, uint8_t *, uint32_t *, uint32_t);

struct Var {
    const char *name;
    const void *k;
    bool six;     // round-5 signature (pool heads, t_own)
    unsigned threads = 512;
    bool one_group = false;   // grid = groups / 4 (one group per wave, 4-wave workgroups)
};

static void launch(const Var &v, unsigned grid, const uint8_t *src, uint32_t L, uint64_t n, uint8_t *o)
{
    if (v.one_group)
        grid = unsigned(((n + 63) / 64 + 3) / 4);
    uint32_t *pool = nullptr;
    uint32_t t_own = 0;
    void *a4[] = {&src, &L, &n, &o};
    void *a6[] = {&src, &L, &n, &o, &pool, &t_own};
    CK(hipLaunchKernel(v.k, dim3(grid), dim3(v.threads), v.six ? a6 : a4, 0, 0));
}

static double med(std::vector<double> v)
{
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char **argv)
{
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 1048576;
    const uint32_t L = argc > 2 ? atoi(argv[2]) : 1500;
    const int rounds = argc > 3 ? atoi(argv[3]) : 5;
    const int nl = argc > 4 ? atoi(argv[4]) : 100;
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
    const Var vs[] = {
        {"r05 per-group setup", (const void *)(K6)brb_mb_r05::digest_line_kernel<AlgLit, 8, true, true, true>, true},
        {"r06 hoisted", hi ? (const void *)(K4)brb_digest::digest_line_kernel<AlgLit, 8, true, true>
                           : (const void *)(K4)brb_digest::digest_line_kernel<AlgLit, 8, true, false>, false},
        {"3-slot ring, 1 group/wave", hi ? (const void *)(K4)brb_mb_l3r::digest_line3r_kernel<AlgLit, true, true>
                                         : (const void *)(K4)brb_mb_l3r::digest_line3r_kernel<AlgLit, true, false>, false, 256, true},
        {"half-line 16 waves", (const void *)(K4)brb_mb_l4::digest_line4_kernel<AlgLit, 16, true>, false, 1024},
        {"half-line 8 waves", (const void *)(K4)brb_mb_l4::digest_line4_kernel<AlgLit, 8, true>, false, 512},
        {"half-line 16 w, all L2", (const void *)(K4)brb_mb_l4::digest_line4_kernel<AlgLit, 16, true, true>, false, 1024},
    };
    const int nv = int(sizeof(vs) / sizeof(vs[0]));
    // parity between the variants, on every copy's first launch
    std::vector<uint8_t> ref(n * 16), got(n * 16);
    for (int vi = 0; vi < nv; vi++) {
        CK(hipMemset(o, 0xA5, n * 16));
        launch(vs[vi], grid, d[0], L, n, o);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(vi ? got.data() : ref.data(), o, n * 16, hipMemcpyDeviceToHost));
        if (vi && memcmp(ref.data(), got.data(), n * 16) != 0) {
            uint64_t r = 0;
            while (memcmp(&ref[16 * r], &got[16 * r], 16) == 0) r++;
            printf("MISMATCH %s vs %s at record %llu\n", vs[vi].name, vs[0].name, (unsigned long long)r);
            return 2;
        }
    }
    printf("n=%llu L=%u grid=%u tail_hi=%d copies=%d: digests identical across variants\n", (unsigned long long)n, L, grid,
           int(hi), nrot);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<std::vector<double>> us(nv);
    int it = 0;
    for (int r = 0; r < rounds; r++)
        for (int vi = 0; vi < nv; vi++) {
            float tot = 0;
            while (tot < 300.f) {       // clocks settle on this variant
                CK(hipEventRecord(a));
                for (int i = 0; i < 20; i++) launch(vs[vi], grid, d[it++ % nrot], L, n, o);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                tot += ms;
            }
            CK(hipEventRecord(a));
            for (int i = 0; i < nl; i++) launch(vs[vi], grid, d[it++ % nrot], L, n, o);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            us[vi].push_back(1000.0 * ms / nl);
            printf("round %d %-22s %.2f us/launch  %.3f of 8 TB/s\n", r, vs[vi].name, us[vi].back(),
                   double(n) * L / (us[vi].back() * 1e-6) / 8e12);
            fflush(stdout);
        }
    for (int vi = 0; vi < nv; vi++)
        printf("MEDIAN %-22s %.2f us  frac %.4f\n", vs[vi].name, med(us[vi]), double(n) * L / (med(us[vi]) * 1e-6) / 8e12);
    return 0;
}
