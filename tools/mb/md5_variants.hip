// md5_variants.hip -- microbenchmark of MD5 batch kernel structures for cfg2 (65536 x 1500 B).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../brb_framework_amd/csrc/gpu md5_variants.hip -o md5mb
// Every variant's digests are compared with variant 0 (the shipped kernel structure).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#include "md5_device.h"

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

BRB_DEV void put16(uint32_t (&w)[16], uint4 a, uint4 b, uint4 c, uint4 d)
{
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
    w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
    w[8] = c.x; w[9] = c.y; w[10] = c.z; w[11] = c.w;
    w[12] = d.x; w[13] = d.y; w[14] = d.z; w[15] = d.w;
}

BRB_DEV void finish_store(Md5State &st, const uint8_t *p, uint32_t L, uint32_t nfull, uint4 *out, uint64_t r)
{
    uint32_t w[16];
    const uint32_t t = L & 63;
    const uint8_t *pt = p + 64u * nfull;
#pragma unroll
    for (uint32_t i = 0; i < 16; i++)
        w[i] = tail_word_a4(pt, t, i);
    md5_finish(st, w, t, L);
    out[r] = make_uint4(st.a, st.b, st.c, st.d);
}

// ---- direct loads, prefetch depth D blocks (ring in registers, statically indexed) --------------
template <int D>
struct Ring {
    uint4 v[D][4];
};

template <int BLOCK, int D>
__global__ __launch_bounds__(BLOCK) void k_direct(const uint8_t *__restrict__ data, uint32_t L, uint32_t stride, uint64_t n,
                                                  uint4 *__restrict__ out, uint32_t active_lanes)
{
    if ((threadIdx.x & 63) >= active_lanes)
        return;
    const uint64_t r = uint64_t(blockIdx.x) * (BLOCK / 64) * active_lanes + (threadIdx.x / 64) * active_lanes + (threadIdx.x & 63);
    if (r >= n)
        return;
    const uint8_t *p = data + r * stride;
    const uint32_t nfull = L >> 6;
    Md5State st = md5_iv();
    uint32_t w[16];
    uint4 ring[D][4];
#pragma unroll
    for (int i = 0; i < D; i++) {
        const uint8_t *q = p + 64u * min<uint32_t>(i, nfull - 1);
        ring[i][0] = ld16_a4(q); ring[i][1] = ld16_a4(q + 16); ring[i][2] = ld16_a4(q + 32); ring[i][3] = ld16_a4(q + 48);
    }
    uint32_t b = 0;
    for (; b + D <= nfull; b += D) {
#pragma unroll
        for (int i = 0; i < D; i++) {
            put16(w, ring[i][0], ring[i][1], ring[i][2], ring[i][3]);
            const uint8_t *q = p + 64u * min<uint32_t>(b + i + D, nfull - 1);
            ring[i][0] = ld16_a4(q); ring[i][1] = ld16_a4(q + 16); ring[i][2] = ld16_a4(q + 32); ring[i][3] = ld16_a4(q + 48);
            md5_compress(st, w);
        }
    }
#pragma unroll
    for (int i = 0; i < D; i++) {
        if (b + i < nfull) {
            put16(w, ring[i][0], ring[i][1], ring[i][2], ring[i][3]);
            md5_compress(st, w);
        }
    }
    finish_store(st, p, L, nfull, out, r);
}

// ---- LDS-staged, coalesced: a wave stages 4 blocks (256 B) of each of its 64 records ----------
// Workgroup = 1 wave.  Row stride 272 B keeps the per-lane ds_read_b128 conflict-free.
constexpr int kRow = 272;
template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) void k_lds(const uint8_t *__restrict__ data, uint32_t L, uint32_t stride, uint64_t n,
                                                    uint4 *__restrict__ out, uint32_t)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[WAVES][64 * kRow];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t rbase = (uint64_t(blockIdx.x) * WAVES + wv) * 64;
    if (rbase >= n)
        return;
    const uint64_t r = rbase + lane;
    const bool live = r < n;
    const uint32_t nfull = L >> 6;
    const uint32_t nstage = (nfull + 3) / 4;
    uint8_t *my = lds[wv];
    // loader mapping: instruction q covers records rbase + 4q + lane/16, chunk lane%16 of the stage
    const uint32_t lrec = lane >> 4, lchunk = lane & 15;
    uint4 st_regs[16];
    auto issue = [&](uint32_t s) {
        const uint32_t blocks = min<uint32_t>(4, nfull - 4 * s);
        const bool ok = lchunk < 4 * blocks;
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const uint64_t rr = rbase + 4 * q + lrec;
            const uint8_t *src = data + rr * stride + 256u * s + 16u * lchunk;
            st_regs[q] = (ok && rr < n) ? ld16_a4(src) : make_uint4(0, 0, 0, 0);
        }
    };
    Md5State st = md5_iv();
    uint32_t w[16];
    if (nstage)
        issue(0);
    for (uint32_t s = 0; s < nstage; s++) {
#pragma unroll
        for (int q = 0; q < 16; q++)
            *reinterpret_cast<uint4 *>(my + (4 * q + lrec) * kRow + 16 * lchunk) = st_regs[q];
        __syncthreads();
        if (s + 1 < nstage)
            issue(s + 1);
        const uint32_t blocks = min<uint32_t>(4, nfull - 4 * s);
        for (uint32_t b = 0; b < blocks; b++) {
            const uint4 *row = reinterpret_cast<const uint4 *>(my + lane * kRow + 64 * b);
            put16(w, row[0], row[1], row[2], row[3]);
            md5_compress(st, w);
        }
        __syncthreads();
    }
    if (live)
        finish_store(st, data + r * stride, L, nfull, out, r);
}

using Kern = void (*)(const uint8_t *, uint32_t, uint32_t, uint64_t, uint4 *, uint32_t);

struct Variant {
    const char *name;
    Kern k;
    int block;
    int recs_per_block;
    uint32_t active;
    bool alias;     // stride 0: every record reads the same bytes (compute floor)
};

int main(int argc, char **argv)
{
    const uint32_t L = 1500;
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 65536;
    const int reps = 30;
    const int nrot = 7;
    std::vector<uint8_t> h(n * L);
    uint64_t x = 0x1234567;
    for (auto &c : h) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        c = uint8_t(x >> 56);
    }
    uint8_t *d[nrot];
    for (int i = 0; i < nrot; i++) {
        CK(hipMalloc(&d[i], n * L + 256));
        CK(hipMemcpy(d[i], h.data(), n * L, hipMemcpyHostToDevice));
    }
    uint4 *o, *o0;
    CK(hipMalloc(&o, n * 16));
    CK(hipMalloc(&o0, n * 16));

    std::vector<Variant> vs = {
        {"direct D1 b256", k_direct<256, 1>, 256, 256, 64, false},
        {"direct D2 b256", k_direct<256, 2>, 256, 256, 64, false},
        {"direct D3 b256", k_direct<256, 3>, 256, 256, 64, false},
        {"direct D4 b256", k_direct<256, 4>, 256, 256, 64, false},
        {"direct D2 b64", k_direct<64, 2>, 64, 64, 64, false},
        {"direct D4 b64", k_direct<64, 4>, 64, 64, 64, false},
        {"lds 1w", k_lds<1>, 64, 64, 64, false},
        {"lds 4w", k_lds<4>, 256, 256, 64, false},
        {"direct D2 b64 32lanes", k_direct<64, 2>, 64, 32, 32, false},
        {"direct D2 b128 32lanes", k_direct<128, 2>, 128, 64, 32, false},
        {"alias D1 b256 (compute floor)", k_direct<256, 1>, 256, 256, 64, true},
        {"alias D2 b64 (compute floor)", k_direct<64, 2>, 64, 64, 64, true},
        {"alias D2 b64 32lanes (floor)", k_direct<64, 2>, 64, 32, 32, true},
    };
    std::vector<std::vector<float>> t(vs.size());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // reference digests (variant 0)
    hipLaunchKernelGGL(vs[0].k, dim3((n + 255) / 256), dim3(256), 0, 0, d[0], L, L, n, o0, 64u);
    CK(hipDeviceSynchronize());
    std::vector<uint8_t> ref(n * 16), got(n * 16);
    CK(hipMemcpy(ref.data(), o0, n * 16, hipMemcpyDeviceToHost));
    int it = 0;
    for (int rep = 0; rep < reps; rep++) {
        for (size_t v = 0; v < vs.size(); v++) {
            const Variant &V = vs[v];
            const unsigned grid = unsigned((n + V.recs_per_block - 1) / V.recs_per_block);
            const uint8_t *src = d[it++ % nrot];
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(V.k, dim3(grid), dim3(V.block), 0, 0, src, L, V.alias ? 0u : L, n, o, V.active);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t[v].push_back(ms * 1000);
            if (rep == 0 && !V.alias) {
                CK(hipMemcpy(got.data(), o, n * 16, hipMemcpyDeviceToHost));
                if (memcmp(got.data(), ref.data(), n * 16))
                    printf("MISMATCH in %s\n", V.name);
            }
        }
    }
    for (size_t v = 0; v < vs.size(); v++) {
        auto &a = t[v];
        std::sort(a.begin(), a.end());
        printf("%-34s median %8.2f us  min %8.2f us  -> %7.0f GB/s\n", vs[v].name, a[a.size() / 2], a[0],
               n * L / (a[a.size() / 2] * 1e-6) / 1e9);
    }
    return 0;
}
