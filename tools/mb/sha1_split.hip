// sha1_split.hip -- does splitting SHA-1 between two waves pay?  65 536 records x 1500 B (cfg2),
// one record per lane, 64 records per wave:
//   fused : one wave per group does the message schedule and the 80 rounds (4 waves per workgroup,
//           one per SIMD -- the issue-bound shape of the product kernel)
//   split : a producer wave builds the block and its whole schedule W[0..79] and hands it through a
//           double-buffered LDS slot to a consumer wave that runs the rounds (8-wave workgroups:
//           producers are waves 0-3, consumers 4-7, so each SIMD holds one of each); one workgroup
//           barrier per block
// Both read the records with per-lane 16-byte loads, so the difference is the split alone.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../brb_framework_amd/csrc/gpu sha1_split.hip -o sha1split
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "sha1_device.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// Block i of the padded message of record `rec` (L bytes, 4-byte aligned) as big-endian words.
__device__ __forceinline__ void build_block(const uint8_t *rec, uint32_t L, uint32_t i, uint32_t (&w)[16])
{
    const uint32_t nfull = L >> 6, t = L & 63;
    if (i < nfull) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint4 v = ld16_a4(rec + 64 * i + 16 * q);
            w[4 * q] = __builtin_bswap32(v.x);
            w[4 * q + 1] = __builtin_bswap32(v.y);
            w[4 * q + 2] = __builtin_bswap32(v.z);
            w[4 * q + 3] = __builtin_bswap32(v.w);
        }
        return;
    }
    if (i == nfull) {
#pragma unroll
        for (uint32_t k = 0; k < 16; k++)
            w[k] = __builtin_bswap32(tail_word_a4(rec + 64 * nfull, t, k));
    } else {
#pragma unroll
        for (int k = 0; k < 16; k++)
            w[k] = 0;
    }
    const uint64_t len = L;
    if (i == nfull + (t >= 56 ? 1u : 0u)) {
        w[14] = uint32_t(len >> 29) + (len >= (uint64_t(1) << 29) ? 1u : 0u);
        w[15] = uint32_t(len << 3);
    }
}

__device__ __forceinline__ void store_digest(uint8_t *out, uint64_t r, const Sha1State &st)
{
    uint32_t *o = reinterpret_cast<uint32_t *>(out + 20 * r);
    o[0] = __builtin_bswap32(st.a);
    o[1] = __builtin_bswap32(st.b);
    o[2] = __builtin_bswap32(st.c);
    o[3] = __builtin_bswap32(st.d);
    o[4] = __builtin_bswap32(st.e);
}

__global__ __launch_bounds__(256) void sha1_fused(const uint8_t *data, uint32_t L, uint64_t n, uint8_t *out)
{
    const uint64_t r = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    if (r >= n)
        return;
    const uint8_t *rec = data + r * L;
    const uint32_t nb = (L >> 6) + ((L & 63) >= 56 ? 2 : 1);
    Sha1State st = sha1_iv();
    for (uint32_t i = 0; i < nb; i++) {
        uint32_t w[16];
        build_block(rec, L, i, w);
        sha1_compress(st, w);
    }
    store_digest(out, r, st);
}

// The 80 rounds on a precomputed schedule.
__device__ __forceinline__ void sha1_rounds(Sha1State &st, const uint32_t (&W)[80])
{
    uint32_t a = st.a, b = st.b, c = st.c, d = st.d, e = st.e;
    constexpr uint32_t K0 = 0x5A827999u, K1 = 0x6ED9EBA1u, K2 = 0x8F1BBCDCu, K3 = 0xCA62C1D6u;
#define R5(F, K, i)                                  \
    BRB_SHA1_R(F, K, a, b, c, d, e, W[(i) + 0]);     \
    BRB_SHA1_R(F, K, e, a, b, c, d, W[(i) + 1]);     \
    BRB_SHA1_R(F, K, d, e, a, b, c, W[(i) + 2]);     \
    BRB_SHA1_R(F, K, c, d, e, a, b, W[(i) + 3]);     \
    BRB_SHA1_R(F, K, b, c, d, e, a, W[(i) + 4]);
    R5(BRB_SHA1_CH, K0, 0) R5(BRB_SHA1_CH, K0, 5) R5(BRB_SHA1_CH, K0, 10) R5(BRB_SHA1_CH, K0, 15)
    R5(BRB_SHA1_PAR, K1, 20) R5(BRB_SHA1_PAR, K1, 25) R5(BRB_SHA1_PAR, K1, 30) R5(BRB_SHA1_PAR, K1, 35)
    R5(BRB_SHA1_MAJ, K2, 40) R5(BRB_SHA1_MAJ, K2, 45) R5(BRB_SHA1_MAJ, K2, 50) R5(BRB_SHA1_MAJ, K2, 55)
    R5(BRB_SHA1_PAR, K3, 60) R5(BRB_SHA1_PAR, K3, 65) R5(BRB_SHA1_PAR, K3, 70) R5(BRB_SHA1_PAR, K3, 75)
#undef R5
    st.a += a;
    st.b += b;
    st.c += c;
    st.d += d;
    st.e += e;
}

// LDS: [pair 4][buffer 2][20 uint4 rows][64 lanes] = 160 KiB
__global__ __launch_bounds__(512) void sha1_split(const uint8_t *data, uint32_t L, uint64_t n, uint8_t *out)
{
    __shared__ uint4 buf[4][2][20][64];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63, pair = wv & 3;
    const bool prod = wv < 4;
    const uint64_t r = (uint64_t(blockIdx.x) * 4 + pair) * 64 + lane;
    const bool live = r < n;
    const uint8_t *rec = data + (live ? r : 0) * L;
    const uint32_t nb = (L >> 6) + ((L & 63) >= 56 ? 2 : 1);
    Sha1State st = sha1_iv();
    for (uint32_t i = 0; i <= nb; i++) {             // same trip count in every wave: barriers match
        if (prod) {
            if (i < nb) {
                uint32_t W[80];
                uint32_t w[16];
                build_block(rec, L, i, w);
#pragma unroll
                for (int k = 0; k < 16; k++)
                    W[k] = w[k];
#pragma unroll
                for (int k = 16; k < 80; k++)
                    W[k] = rotl<1>(__builtin_amdgcn_bitop3_b32(W[k - 3], W[k - 8], W[k - 14], 0x96) ^ W[k - 16]);
#pragma unroll
                for (int q = 0; q < 20; q++)
                    buf[pair][i & 1][q][lane] = make_uint4(W[4 * q], W[4 * q + 1], W[4 * q + 2], W[4 * q + 3]);
            }
        } else if (i >= 1) {
            uint32_t W[80];
#pragma unroll
            for (int q = 0; q < 20; q++) {
                const uint4 v = buf[pair][(i - 1) & 1][q][lane];
                W[4 * q] = v.x;
                W[4 * q + 1] = v.y;
                W[4 * q + 2] = v.z;
                W[4 * q + 3] = v.w;
            }
            sha1_rounds(st, W);
        }
        __syncthreads();
    }
    if (!prod && live)
        store_digest(out, r, st);
}

int main(int argc, char **argv)
{
    const uint64_t n = argc > 1 ? atoll(argv[1]) : 65536;
    const uint32_t L = argc > 2 ? atoi(argv[2]) : 1500;
    uint8_t *d, *o1, *o2;
    CK(hipMalloc(&d, n * L + 64));
    CK(hipMalloc(&o1, n * 20));
    CK(hipMalloc(&o2, n * 20));
    std::vector<uint8_t> h(n * L);
    for (size_t i = 0; i < h.size(); i++)
        h[i] = uint8_t((i * 2654435761u) >> 11);
    CK(hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const unsigned g_f = unsigned((n + 255) / 256), g_s = unsigned((n + 255) / 256);
    for (int rep = 0; rep < 3; rep++) {
        for (int v = 0; v < 2; v++) {
            for (int w = 0; w < 3; w++) {
                if (v == 0) sha1_fused<<<g_f, 256>>>(d, L, n, o1);
                else sha1_split<<<g_s, 512>>>(d, L, n, o2);
            }
            CK(hipEventRecord(a));
            for (int w = 0; w < 20; w++) {
                if (v == 0) sha1_fused<<<g_f, 256>>>(d, L, n, o1);
                else sha1_split<<<g_s, 512>>>(d, L, n, o2);
            }
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (rep == 2)
                printf("%-6s %8.2f us per launch\n", v ? "split" : "fused", ms * 1e3 / 20);
        }
    }
    std::vector<uint8_t> r1(n * 20), r2(n * 20);
    CK(hipMemcpy(r1.data(), o1, n * 20, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r2.data(), o2, n * 20, hipMemcpyDeviceToHost));
    printf("digests %s\n", r1 == r2 ? "match" : "DIFFER");
    return 0;
}
