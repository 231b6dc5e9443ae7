// bf_ab.hip -- A/B of the Blowfish ECB kernels on cfg4 (2^26 blocks = 1 GiB), one process.
// Checks the replicated-table kernels against the simple kernel bit for bit, then times
// encrypt/decrypt pairs interleaved (median per launch).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../brb_framework_amd/csrc/gpu bf_ab.hip -o bfab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "blowfish_device.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void fill(uint64_t *w, uint64_t n, uint64_t seed)
{
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
        uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        w[i] = z ^ (z >> 31);
    }
}

__global__ void diff(const uint64_t *a, const uint64_t *b, uint64_t n, unsigned long long *cnt)
{
    unsigned long long c = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
        c += a[i] != b[i];
    if (c)
        atomicAdd(cnt, c);
}

static unsigned long long count_diff(const uint64_t *a, const uint64_t *b, uint64_t n, unsigned long long *d)
{
    CK(hipMemset(d, 0, 8));
    diff<<<4096, 256>>>(a, b, n, d);
    unsigned long long h;
    CK(hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost));
    return h;
}

typedef void (*Launch)(const uint64_t *, uint64_t *, uint64_t, bool);

static void l_simple(const uint64_t *ctx, uint64_t *w, uint64_t n, bool dec)
{
    const unsigned g = 2048;
    if (dec)
        brb_bf::bf_simple_kernel<256, true><<<g, 256>>>(ctx, reinterpret_cast<uint8_t *>(w), n);
    else
        brb_bf::bf_simple_kernel<256, false><<<g, 256>>>(ctx, reinterpret_cast<uint8_t *>(w), n);
}

template <int ILP>
static void l_rep(const uint64_t *ctx, uint64_t *w, uint64_t n, bool dec)
{
    const uint64_t per = uint64_t(brb_bf::kRepThreads) * ILP;
    const uint64_t want = (n + per - 1) / per;
    const unsigned g = unsigned(std::min<uint64_t>(want, 256));
    if (dec)
        brb_bf::bf_rep_kernel<ILP, true><<<g, brb_bf::kRepThreads>>>(ctx, w, n);
    else
        brb_bf::bf_rep_kernel<ILP, false><<<g, brb_bf::kRepThreads>>>(ctx, w, n);
}

int main(int argc, char **argv)
{
    const uint64_t n_blocks = argc > 1 ? strtoull(argv[1], 0, 0) : (1ull << 26);
    const uint64_t n_words = 2 * n_blocks;
    // a context shaped like an initialised one: random low halves, small high halves
    std::vector<uint64_t> hctx(18 + 1024);
    uint64_t s = 12345;
    for (auto &v : hctx) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        v = (s >> 32) | (((s >> 7) & 0x3FFFF) << 32);
    }
    uint64_t *ctx, *ref, *w, *orig;
    unsigned long long *dcnt;
    CK(hipMalloc(&ctx, hctx.size() * 8));
    CK(hipMemcpy(ctx, hctx.data(), hctx.size() * 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&ref, n_words * 8));
    CK(hipMalloc(&w, n_words * 8));
    CK(hipMalloc(&orig, n_words * 8));
    CK(hipMalloc(&dcnt, 8));
    fill<<<4096, 256>>>(orig, n_words, 7);
    CK(hipMemcpy(ref, orig, n_words * 8, hipMemcpyDeviceToDevice));
    l_simple(ctx, ref, n_blocks, false);

    struct V { const char *name; Launch f; } vs[] = {{"simple", l_simple}, {"rep1", l_rep<1>}, {"rep2", l_rep<2>}, {"rep3", l_rep<3>}, {"rep4", l_rep<4>}};
    const int NV = sizeof(vs) / sizeof(vs[0]);
    for (int v = 0; v < NV; v++) {
        CK(hipMemcpy(w, orig, n_words * 8, hipMemcpyDeviceToDevice));
        vs[v].f(ctx, w, n_blocks, false);
        CK(hipDeviceSynchronize());
        const unsigned long long de = count_diff(w, ref, n_words, dcnt);
        vs[v].f(ctx, w, n_blocks, true);
        CK(hipDeviceSynchronize());
        const unsigned long long dd = count_diff(w, orig, n_words, dcnt);
        printf("%-8s encrypt mismatches %llu, round-trip mismatches %llu\n", vs[v].name, de, dd);
    }

    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(NV);
    for (int rep = 0; rep < 12; rep++)
        for (int v = 0; v < NV; v++)
            for (int dec = 0; dec < 2; dec++) {
                CK(hipEventRecord(e0));
                vs[v].f(ctx, w, n_blocks, dec);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rep >= 2)
                    t[v].push_back(ms);
            }
    for (int v = 0; v < NV; v++) {
        std::sort(t[v].begin(), t[v].end());
        const double us = 1e3 * t[v][t[v].size() / 2];
        printf("%-8s median %.1f us/launch  %.1f GB/s plaintext  %.1f GB/s r+w\n", vs[v].name, us,
               16.0 * n_blocks / us / 1e3, 32.0 * n_blocks / us / 1e3);
    }
    return 0;
}
