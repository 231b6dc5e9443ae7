// md5_tput.hip -- SIMD throughput of the product's MD5 compression with its data in registers, at
// 1..8 waves per SIMD: shader cycles per VALU instruction per SIMD (s_memtime) and the shader clock
// the load holds (s_memtime ticks / s_memrealtime at 100 MHz).  Answers whether the MD5 step mix
// runs at the per-class VALU rates of tools/mb/valu_tput.hip (add/xor/bitop3 ~2.4 cycles,
// add3/alignbit ~4.4 at >= 2 waves) or at ~5 cycles per instruction, and whether the clock drops.
// Measured (MI355X, profiles/r02d_md5_tput.txt): 4.63 cycles per VALU at one wave per SIMD, 4.24 at
// two, 4.05 at four and eight; the clock holds 2.10-2.21 GHz with every CU busy (2.42 GHz on 8 CUs).
// So the MD5 mix runs at about one VALU per 4 cycles per SIMD at any occupancy: the lone wave of
// cfg2 pays ~14 % over the SIMD's own rate, and the 2.4-cycle classes of valu_tput do not show up.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../brb_framework_amd/csrc/gpu -I../../include \
//          md5_tput.hip -o md5_tput
#include <hip/hip_runtime.h>

#include <cstdio>

#include "md5_device.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int ITERS = 200;

template <int VAR>
__global__ __launch_bounds__(256) void md5_loop(uint32_t *out, unsigned long long *t, uint32_t seed)
{
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 16; i++)
        m[i] = seed * (i + 1) + threadIdx.x * 7919u + blockIdx.x;
    Md5State st = md5_iv();
    __syncthreads();
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; it++) {
        if (VAR == 0)
            md5_compress<true>(st, m);
        else
            md5_compress<false>(st, m);
        m[it & 15] ^= st.a;                     // keeps the iterations dependent
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = st.a ^ st.b ^ st.c ^ st.d;
    if ((threadIdx.x & 63) == 0) {
        const unsigned w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        t[4 * w + 0] = c0;
        t[4 * w + 1] = c1;
        t[4 * w + 2] = r0;
        t[4 * w + 3] = r1;
    }
}

template <int VAR>
int run(int waves_per_simd, int cus)
{
    const int blocks = cus * waves_per_simd;   // 4-wave blocks: one wave per SIMD per block
    const int nw = blocks * 4;
    uint32_t *o;
    unsigned long long *t;
    CK(hipMalloc(&o, size_t(blocks) * 256 * 4));
    CK(hipMalloc(&t, size_t(nw) * 32));
    hipLaunchKernelGGL(md5_loop<VAR>, dim3(blocks), dim3(256), 0, 0, o, t, 1u);   // warm-up
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(md5_loop<VAR>, dim3(blocks), dim3(256), 0, 0, o, t, 2u);
    CK(hipEventRecord(e1));
    CK(hipDeviceSynchronize());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long *h = new unsigned long long[4 * nw];
    CK(hipMemcpy(h, t, size_t(nw) * 32, hipMemcpyDeviceToHost));
    double cyc = 0, real = 0;
    for (int w = 0; w < nw; w++) {
        cyc += double(h[4 * w + 1] - h[4 * w + 0]);
        real += double(h[4 * w + 3] - h[4 * w + 2]);
    }
    cyc /= nw;
    real /= nw;                                 // 100 MHz ticks
    const double ghz = cyc / (real * 10.0);     // cycles per ns
    // VALU per loop iteration, both variants (hipcc -S of this file: 326, the xor included).  Waves
    // of one SIMD do not start together, so the SIMD's rate comes from the kernel time, not from the
    // per-wave stamps: cycles per VALU per SIMD = kernel time x clock / (waves x ITERS x 326).
    const double valu = 326.0;
    const double cpi = ms * 1e-3 * ghz * 1e9 / (double(waves_per_simd) * ITERS * valu);
    printf("var %d  waves/SIMD %d  CUs %3d: %7.1f cycles per compress per wave, %.2f cycles per VALU per SIMD, "
           "clock %.2f GHz, kernel %.1f us\n", VAR, waves_per_simd, cus, cyc / ITERS, cpi, ghz, ms * 1e3);
    delete[] h;
    hipFree(o);
    hipFree(t);
    return 0;
}

int main()
{
    int dev = 0, cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    for (int w : {1, 2, 4, 8}) {
        if (run<0>(w, cus)) return 1;
        if (run<1>(w, cus)) return 1;
    }
    if (run<0>(8, 8)) return 1;                 // 8 CUs only: clock without the chip-wide power draw
    return 0;
}
