// md5_occ.hip -- what one SIMD does with the product's MD5 compression (md5_device.h), data in
// registers, by waves per SIMD (W) and active lanes per wave (A = 64, or 32 with the upper half of
// EXEC clear).  Answers:
//   * the rate of the MD5 instruction mix per SIMD at W = 1, 2, 4 with every wave really resident
//     (round 2's md5_tput.hip launched more waves than fit, so its kernel-time figure of ~4 cycles
//     per VALU mixed waves that ran one after another; its per-wave stamps did not);
//   * whether a wave64 instruction with half of EXEC set costs the SIMD half the time -- if so, two
//     half-waves per SIMD hide each other's dependency stalls at the lone wave's lane throughput.
// Output per configuration: kernel time (hipEvent, best of 3), lane-compressions per SIMD per
// microsecond, shader cycles per wave-instruction per SIMD (clock from s_memtime / s_memrealtime),
// and the overlap of the waves' lifetimes (1.0 = all resident together).
// Also SHA-1 (sha1_device.h) and the all-fast MD5 variant (md5_split).  Build (not through head/pipes:
// a SIGPIPE kills hipcc): hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../brb_framework_amd/csrc/gpu -I../../include \
//          md5_occ.hip -o md5_occ
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "md5_device.h"
#include "sha1_device.h"

// Split-add step (all-fast-ops variant): x = a + (m + K) and y = x + F as plain v_add_u32 (inline asm
// keeps hipcc from fusing them into v_add3_u32), so a step is 5 fast ops + 1 v_alignbit_b32.
#define MB_ADD(d_, x_, y_) asm("v_add_u32 %0, %1, %2" : "=v"(d_) : "v"(x_), "v"(y_))
#define MB_STEP(F, a, b, c, d, m, k, s)                                                  \
    do {                                                                                 \
        const uint32_t mk_ = (m) + (k);                                                  \
        uint32_t x_, y_;                                                                 \
        MB_ADD(x_, a, mk_);                                                              \
        MB_ADD(y_, x_, F((b), (c), (d)));                                                \
        (a) = (b) + rotl<s>(y_);                                                         \
    } while (0)

BRB_DEV void md5_split(Md5State &st, const uint32_t (&m)[16])
{
    uint32_t a = st.a, b = st.b, c = st.c, d = st.d;
#define R1(a, b, c, d, i, k, s) MB_STEP(BRB_MD5_F1, a, b, c, d, m[i], k, s)
#define R2(a, b, c, d, i, k, s) MB_STEP(BRB_MD5_F2, a, b, c, d, m[i], k, s)
#define R3(a, b, c, d, i, k, s) MB_STEP(BRB_MD5_F3, a, b, c, d, m[i], k, s)
#define R4(a, b, c, d, i, k, s) MB_STEP(BRB_MD5_F4, a, b, c, d, m[i], k, s)
    R1(a, b, c, d, 0, 0xd76aa478u, 7); R1(d, a, b, c, 1, 0xe8c7b756u, 12); R1(c, d, a, b, 2, 0x242070dbu, 17); R1(b, c, d, a, 3, 0xc1bdceeeu, 22);
    R1(a, b, c, d, 4, 0xf57c0fafu, 7); R1(d, a, b, c, 5, 0x4787c62au, 12); R1(c, d, a, b, 6, 0xa8304613u, 17); R1(b, c, d, a, 7, 0xfd469501u, 22);
    R1(a, b, c, d, 8, 0x698098d8u, 7); R1(d, a, b, c, 9, 0x8b44f7afu, 12); R1(c, d, a, b, 10, 0xffff5bb1u, 17); R1(b, c, d, a, 11, 0x895cd7beu, 22);
    R1(a, b, c, d, 12, 0x6b901122u, 7); R1(d, a, b, c, 13, 0xfd987193u, 12); R1(c, d, a, b, 14, 0xa679438eu, 17); R1(b, c, d, a, 15, 0x49b40821u, 22);
    R2(a, b, c, d, 1, 0xf61e2562u, 5); R2(d, a, b, c, 6, 0xc040b340u, 9); R2(c, d, a, b, 11, 0x265e5a51u, 14); R2(b, c, d, a, 0, 0xe9b6c7aau, 20);
    R2(a, b, c, d, 5, 0xd62f105du, 5); R2(d, a, b, c, 10, 0x02441453u, 9); R2(c, d, a, b, 15, 0xd8a1e681u, 14); R2(b, c, d, a, 4, 0xe7d3fbc8u, 20);
    R2(a, b, c, d, 9, 0x21e1cde6u, 5); R2(d, a, b, c, 14, 0xc33707d6u, 9); R2(c, d, a, b, 3, 0xf4d50d87u, 14); R2(b, c, d, a, 8, 0x455a14edu, 20);
    R2(a, b, c, d, 13, 0xa9e3e905u, 5); R2(d, a, b, c, 2, 0xfcefa3f8u, 9); R2(c, d, a, b, 7, 0x676f02d9u, 14); R2(b, c, d, a, 12, 0x8d2a4c8au, 20);
    R3(a, b, c, d, 5, 0xfffa3942u, 4); R3(d, a, b, c, 8, 0x8771f681u, 11); R3(c, d, a, b, 11, 0x6d9d6122u, 16); R3(b, c, d, a, 14, 0xfde5380cu, 23);
    R3(a, b, c, d, 1, 0xa4beea44u, 4); R3(d, a, b, c, 4, 0x4bdecfa9u, 11); R3(c, d, a, b, 7, 0xf6bb4b60u, 16); R3(b, c, d, a, 10, 0xbebfbc70u, 23);
    R3(a, b, c, d, 13, 0x289b7ec6u, 4); R3(d, a, b, c, 0, 0xeaa127fau, 11); R3(c, d, a, b, 3, 0xd4ef3085u, 16); R3(b, c, d, a, 6, 0x04881d05u, 23);
    R3(a, b, c, d, 9, 0xd9d4d039u, 4); R3(d, a, b, c, 12, 0xe6db99e5u, 11); R3(c, d, a, b, 15, 0x1fa27cf8u, 16); R3(b, c, d, a, 2, 0xc4ac5665u, 23);
    R4(a, b, c, d, 0, 0xf4292244u, 6); R4(d, a, b, c, 7, 0x432aff97u, 10); R4(c, d, a, b, 14, 0xab9423a7u, 15); R4(b, c, d, a, 5, 0xfc93a039u, 21);
    R4(a, b, c, d, 12, 0x655b59c3u, 6); R4(d, a, b, c, 3, 0x8f0ccc92u, 10); R4(c, d, a, b, 10, 0xffeff47du, 15); R4(b, c, d, a, 1, 0x85845dd1u, 21);
    R4(a, b, c, d, 8, 0x6fa87e4fu, 6); R4(d, a, b, c, 15, 0xfe2ce6e0u, 10); R4(c, d, a, b, 6, 0xa3014314u, 15); R4(b, c, d, a, 13, 0x4e0811a1u, 21);
    R4(a, b, c, d, 4, 0xf7537e82u, 6); R4(d, a, b, c, 11, 0xbd3af235u, 10); R4(c, d, a, b, 2, 0x2ad7d2bbu, 15); R4(b, c, d, a, 9, 0xeb86d391u, 21);
    st.a += a;
    st.b += b;
    st.c += c;
    st.d += d;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int ITERS = 400;
constexpr double VALU_PER_ITER = 326.0;     // hipcc -S: 325 in md5_compress + the xor below
constexpr double VALU_PER_ITER_SPLIT = 390.0;   // md5_split: 64 more v_add_u32 (hipcc -S)
constexpr double VALU_PER_ITER_SHA1 = 600.0;     // sha1_compress + the xor (hipcc -S, loop body)

template <int A, int KIND>
__global__ __launch_bounds__(256) void md5_loop(uint32_t *out, unsigned long long *t, uint32_t seed)
{
    const unsigned lane = threadIdx.x & 63;
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 16; i++)
        m[i] = seed * (i + 1) + threadIdx.x * 7919u + blockIdx.x;
    Md5State st = md5_iv();
    Sha1State s1 = sha1_iv();
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    if (lane < unsigned(A)) {
        for (int it = 0; it < ITERS; it++) {
            if constexpr (KIND == 2) {
                sha1_compress(s1, m);
                m[it & 15] ^= s1.a;
            } else {
                if constexpr (KIND == 1)
                    md5_split(st, m);
                else
                    md5_compress<true>(st, m);
                m[it & 15] ^= st.a;             // keeps the iterations dependent
            }
        }
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = st.a ^ st.b ^ st.c ^ st.d ^ s1.a ^ s1.e;
    if (lane == 0) {
        const unsigned w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        t[4 * w + 0] = c0;
        t[4 * w + 1] = c1;
        t[4 * w + 2] = r0;
        t[4 * w + 3] = r1;
    }
}

template <int A, int KIND = 0>
int run(int W, int cus, double valu_per_iter)
{
    const int blocks = cus * W;                 // 4-wave blocks: W waves per SIMD
    const int nw = blocks * 4;
    uint32_t *o;
    unsigned long long *t;
    CK(hipMalloc(&o, size_t(blocks) * 256 * 4));
    CK(hipMalloc(&t, size_t(nw) * 32));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int rep = 0; rep < 4; rep++) {         // rep 0 warms up
        CK(hipEventRecord(e0));
        md5_loop<A, KIND><<<dim3(blocks), dim3(256)>>>(o, t, 2u + rep);
        CK(hipEventRecord(e1));
        CK(hipDeviceSynchronize());
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep)
            best = std::min(best, ms);
    }
    std::vector<unsigned long long> h(4 * size_t(nw));
    CK(hipMemcpy(h.data(), t, size_t(nw) * 32, hipMemcpyDeviceToHost));
    double cyc = 0, real = 0;
    unsigned long long rmin = ~0ull, rmax = 0;
    for (int w = 0; w < nw; w++) {
        cyc += double(h[4 * w + 1] - h[4 * w + 0]);
        real += double(h[4 * w + 3] - h[4 * w + 2]);
        rmin = std::min(rmin, h[4 * w + 2]);
        rmax = std::max(rmax, h[4 * w + 3]);
    }
    cyc /= nw;
    real /= nw;
    const double ghz = cyc / (real * 10.0);                   // s_memrealtime ticks at 100 MHz
    const double overlap = real / double(rmax - rmin);        // 1.0: every wave alive for the whole span
    const double simd_us = best * 1e3;
    const double lane_comp = double(W) * A * ITERS;           // per SIMD
    const double cpi_simd = simd_us * 1e-6 * ghz * 1e9 / (double(W) * ITERS * valu_per_iter);
    printf("%s W=%d A=%2d  %.2f ns/instr/SIMD  kernel %8.1f us  %7.1f lane-compressions/us/SIMD  %.2f cycles/wave-instr/SIMD  "
           "%.1f cycles/compress/wave  clock %.2f GHz  overlap %.2f\n",
           KIND == 2 ? "sha1 " : KIND == 1 ? "split" : "fused", W, A, simd_us * 1e3 / (double(W) * ITERS * valu_per_iter), simd_us, lane_comp / simd_us, cpi_simd, cyc / ITERS, ghz, overlap);
    hipFree(o);
    hipFree(t);
    return 0;
}

int main()
{
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    for (int W : {1, 2, 4}) {
        if (run<64, 0>(W, cus, VALU_PER_ITER)) return 1;
        if (run<64, 1>(W, cus, VALU_PER_ITER_SPLIT)) return 1;
        if (run<64, 2>(W, cus, VALU_PER_ITER_SHA1)) return 1;
    }
    return 0;
}
