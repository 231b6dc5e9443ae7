// valu_tput.hip -- per-SIMD VALU throughput for independent instruction streams at 1..8 waves per
// SIMD: is the integer VALU 2 cycles per wave64 instruction (SIMD-32) when enough waves issue?
// Also v_lshl_add_u64 (the 64-bit add of the Blowfish F function) and v_perm_b32.
// Build: hipcc -O3 --offload-arch=gfx950 valu_tput.hip -o valu_tput
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)
#define R8(x) x x x x x x x x
#define R32(x) R8(x) R8(x) R8(x) R8(x)

constexpr int ITERS = 512;

template <int KIND>
__global__ void k(unsigned *out, unsigned seed)
{
    unsigned a = seed + threadIdx.x, b = a * 3, c = a ^ 5, d = a + 7, e = a * 11, f = a ^ 13, g = a + 17, h = a * 19;
    unsigned long long p = a, q = b, r = c, s = d;
    const unsigned z = seed | 1;
    for (int it = 0; it < ITERS; it++) {
        if constexpr (KIND == 0) {   // 8 independent v_add_u32 per group
            R32(asm volatile("v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
                             "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8"
                             : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "v"(z));)
        } else if constexpr (KIND == 1) {   // 4 independent v_lshl_add_u64 (x2: 8 per group)
            R32(asm volatile("v_lshl_add_u64 %0, %0, 0, %4\n\tv_lshl_add_u64 %1, %1, 0, %4\n\tv_lshl_add_u64 %2, %2, 0, %4\n\tv_lshl_add_u64 %3, %3, 0, %4\n\t"
                             "v_lshl_add_u64 %0, %0, 0, %4\n\tv_lshl_add_u64 %1, %1, 0, %4\n\tv_lshl_add_u64 %2, %2, 0, %4\n\tv_lshl_add_u64 %3, %3, 0, %4"
                             : "+v"(p), "+v"(q), "+v"(r), "+v"(s) : "v"((unsigned long long)z));)
        } else if constexpr (KIND == 2) {   // 8 independent v_perm_b32
            R32(asm volatile("v_perm_b32 %0, %0, %8, %8\n\tv_perm_b32 %1, %1, %8, %8\n\tv_perm_b32 %2, %2, %8, %8\n\tv_perm_b32 %3, %3, %8, %8\n\t"
                             "v_perm_b32 %4, %4, %8, %8\n\tv_perm_b32 %5, %5, %8, %8\n\tv_perm_b32 %6, %6, %8, %8\n\tv_perm_b32 %7, %7, %8, %8"
                             : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "v"(z));)
        } else if constexpr (KIND == 3) {   // 8 independent v_bitop3_b32
            R32(asm volatile("v_bitop3_b32 %0, %0, %8, %1 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %8, %2 bitop3:0x96\n\tv_bitop3_b32 %2, %2, %8, %3 bitop3:0x96\n\tv_bitop3_b32 %3, %3, %8, %4 bitop3:0x96\n\t"
                             "v_bitop3_b32 %4, %4, %8, %5 bitop3:0x96\n\tv_bitop3_b32 %5, %5, %8, %6 bitop3:0x96\n\tv_bitop3_b32 %6, %6, %8, %7 bitop3:0x96\n\tv_bitop3_b32 %7, %7, %8, %0 bitop3:0x96"
                             : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "v"(z));)
        } else if constexpr (KIND == 4) {   // 8 independent v_alignbit_b32
            R32(asm volatile("v_alignbit_b32 %0, %0, %0, 7\n\tv_alignbit_b32 %1, %1, %1, 7\n\tv_alignbit_b32 %2, %2, %2, 7\n\tv_alignbit_b32 %3, %3, %3, 7\n\t"
                             "v_alignbit_b32 %4, %4, %4, 7\n\tv_alignbit_b32 %5, %5, %5, 7\n\tv_alignbit_b32 %6, %6, %6, 7\n\tv_alignbit_b32 %7, %7, %7, 7"
                             : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h));)
        } else if constexpr (KIND == 5) {   // 8 independent v_add3_u32
            R32(asm volatile("v_add3_u32 %0, %0, %8, %1\n\tv_add3_u32 %1, %1, %8, %2\n\tv_add3_u32 %2, %2, %8, %3\n\tv_add3_u32 %3, %3, %8, %4\n\t"
                             "v_add3_u32 %4, %4, %8, %5\n\tv_add3_u32 %5, %5, %8, %6\n\tv_add3_u32 %6, %6, %8, %7\n\tv_add3_u32 %7, %7, %8, %0"
                             : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "v"(z));)
        } else if constexpr (KIND == 6) {   // 8 independent v_mov_b32_sdwa (byte insert, dst preserved)
            R32(asm volatile("v_mov_b32_sdwa %0, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2\n\t"
                             "v_mov_b32_sdwa %1, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_3\n\t"
                             "v_mov_b32_sdwa %2, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\n\t"
                             "v_mov_b32_sdwa %3, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1\n\t"
                             "v_mov_b32_sdwa %4, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2\n\t"
                             "v_mov_b32_sdwa %5, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_3\n\t"
                             "v_mov_b32_sdwa %6, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\n\t"
                             "v_mov_b32_sdwa %7, %8 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1"
                             : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "v"(z));)
        } else if constexpr (KIND == 7) {   // 8 independent v_xor_b32
            R32(asm volatile("v_xor_b32 %0, %0, %8\n\tv_xor_b32 %1, %1, %8\n\tv_xor_b32 %2, %2, %8\n\tv_xor_b32 %3, %3, %8\n\t"
                             "v_xor_b32 %4, %4, %8\n\tv_xor_b32 %5, %5, %8\n\tv_xor_b32 %6, %6, %8\n\tv_xor_b32 %7, %7, %8"
                             : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "v"(z));)
        } else if constexpr (KIND == 8) {   // 4 independent 64-bit adds as v_add_co_u32 + v_addc_co_u32 (VCC)
            R32(asm volatile("v_add_co_u32 %0, vcc, %0, %8\n\tv_addc_co_u32 %1, vcc, %1, %8, vcc\n\t"
                             "v_add_co_u32 %2, vcc, %2, %8\n\tv_addc_co_u32 %3, vcc, %3, %8, vcc\n\t"
                             "v_add_co_u32 %4, vcc, %4, %8\n\tv_addc_co_u32 %5, vcc, %5, %8, vcc\n\t"
                             "v_add_co_u32 %6, vcc, %6, %8\n\tv_addc_co_u32 %7, vcc, %7, %8, vcc"
                             : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "v"(z) : "vcc");)
        } else if constexpr (KIND == 9) {   // 8 independent v_lshl_or_b32 / v_and_or_b32 (VOP3 2-op fusions)
            R32(asm volatile("v_and_or_b32 %0, %0, %8, %1\n\tv_and_or_b32 %1, %1, %8, %2\n\tv_and_or_b32 %2, %2, %8, %3\n\tv_and_or_b32 %3, %3, %8, %4\n\t"
                             "v_and_or_b32 %4, %4, %8, %5\n\tv_and_or_b32 %5, %5, %8, %6\n\tv_and_or_b32 %6, %6, %8, %7\n\tv_and_or_b32 %7, %7, %8, %0"
                             : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "v"(z));)
        } else if constexpr (KIND == 10) {  // v_xad_u32
            R32(asm volatile("v_xad_u32 %0, %0, %8, %1\n\tv_xad_u32 %1, %1, %8, %2\n\tv_xad_u32 %2, %2, %8, %3\n\tv_xad_u32 %3, %3, %8, %4\n\t"
                             "v_xad_u32 %4, %4, %8, %5\n\tv_xad_u32 %5, %5, %8, %6\n\tv_xad_u32 %6, %6, %8, %7\n\tv_xad_u32 %7, %7, %8, %0"
                             : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "v"(z));)
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d + e + f + g + h + unsigned(p + q + r + s);
}

template <int K>
int run(const char *name, int threads)
{
    unsigned *o;
    CK(hipMalloc(&o, 256 * 1024 * 4));
    hipLaunchKernelGGL(k<K>, dim3(256), dim3(threads), 0, 0, o, 1u);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e9f;
    for (int r = 0; r < 5; r++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(k<K>, dim3(256), dim3(threads), 0, 0, o, 2u);
        hipEventRecord(e1);
        CK(hipDeviceSynchronize());
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    const double waves_per_simd = threads / 64.0 / 4.0;
    const double instr_per_wave = double(ITERS) * 32 * 8;
    // per-SIMD cycles per wave-instruction at an assumed 2.4 GHz (report also ns)
    const double ns_per = best * 1e6 / (instr_per_wave * waves_per_simd);
    printf("%-26s waves/SIMD=%4.1f  %6.3f ns per wave-instr per SIMD  (= %.2f cycles @2.4GHz)\n", name, waves_per_simd,
           ns_per, ns_per * 2.4);
    hipFree(o);
    return 0;
}

int main()
{
    // warm the clock
    for (int i = 0; i < 20; i++) run<0>("warm", 1024);
    for (int t : {256, 512, 1024}) {
        run<0>("v_add_u32", t);
        run<1>("v_lshl_add_u64", t);
        run<2>("v_perm_b32", t);
        run<3>("v_bitop3_b32", t);
        run<4>("v_alignbit_b32", t);
        run<5>("v_add3_u32", t);
        run<6>("v_mov_b32_sdwa (byte ins)", t);
        run<7>("v_xor_b32", t);
        run<8>("v_add_co/addc (64b add)", t);
        run<9>("v_and_or_b32", t);
        run<10>("v_xad_u32", t);
    }
    return 0;
}
