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
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../brb_framework_amd/csrc/gpu -I../../include \
//          md5_occ.hip -o md5_occ
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "md5_device.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int ITERS = 400;
constexpr double VALU_PER_ITER = 326.0;     // hipcc -S: 325 in md5_compress + the xor below

template <int A>
__global__ __launch_bounds__(256) void md5_loop(uint32_t *out, unsigned long long *t, uint32_t seed)
{
    const unsigned lane = threadIdx.x & 63;
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 16; i++)
        m[i] = seed * (i + 1) + threadIdx.x * 7919u + blockIdx.x;
    Md5State st = md5_iv();
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    if (lane < unsigned(A)) {
        for (int it = 0; it < ITERS; it++) {
            md5_compress<true>(st, m);
            m[it & 15] ^= st.a;                 // keeps the iterations dependent
        }
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = st.a ^ st.b ^ st.c ^ st.d;
    if (lane == 0) {
        const unsigned w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        t[4 * w + 0] = c0;
        t[4 * w + 1] = c1;
        t[4 * w + 2] = r0;
        t[4 * w + 3] = r1;
    }
}

template <int A>
int run(int W, int cus)
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
        hipLaunchKernelGGL(md5_loop<A>, dim3(blocks), dim3(256), 0, 0, o, t, 2u + rep);
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
    const double cpi_simd = simd_us * 1e-6 * ghz * 1e9 / (double(W) * ITERS * VALU_PER_ITER);
    printf("W=%d A=%2d  kernel %8.1f us  %7.1f lane-compressions/us/SIMD  %.2f cycles/wave-instr/SIMD  "
           "%.1f cycles/compress/wave  clock %.2f GHz  overlap %.2f\n",
           W, A, simd_us, lane_comp / simd_us, cpi_simd, cyc / ITERS, ghz, overlap);
    hipFree(o);
    hipFree(t);
    return 0;
}

int main()
{
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    for (int W : {1, 2, 4}) {
        if (run<64>(W, cus)) return 1;
        if (run<32>(W, cus)) return 1;
    }
    return 0;
}
