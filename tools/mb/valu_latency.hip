// valu_latency.hip -- cycles per VALU instruction for dependent chains and interleaved chains,
// one wave alone on its SIMD (the situation of the cfg2 MD5 kernel: 1024 waves on 1024 SIMDs).
// Build: hipcc -O3 --offload-arch=gfx950 valu_latency.hip -o valu_lat
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

#define R8(x) x x x x x x x x
#define R64(x) R8(R8(x))

constexpr int ITERS = 256;

template <int KIND, bool HALF = false>
__global__ void chain(unsigned *out, unsigned long long *cyc, unsigned seed)
{
    if (HALF && (threadIdx.x & 63) >= 32)        // EXEC = the low 32 lanes of every wave
        return;
    unsigned a = seed + threadIdx.x, b = seed * 3 + 1, c = seed ^ 0x55, d = threadIdx.x * 7, e = 9, f = 11, g = 13, h = 17;
    const unsigned s = seed | 1;
    unsigned long long t0 = clock64();
    for (int it = 0; it < ITERS; it++) {
        if constexpr (KIND == 0) {        // dependent v_add_u32
            R64(asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));)
        } else if constexpr (KIND == 1) { // dependent v_add3_u32
            R64(asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));)
        } else if constexpr (KIND == 2) { // dependent v_alignbit_b32 (rotate)
            R64(asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(a));)
        } else if constexpr (KIND == 3) { // dependent v_bitop3_b32
            R64(asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xac" : "+v"(a) : "v"(b), "v"(c));)
        } else if constexpr (KIND == 4) { // 2 independent add chains interleaved
            R64(asm volatile("v_add_u32 %0, %0, %2\n\tv_add_u32 %1, %1, %2" : "+v"(a), "+v"(d) : "v"(b));)
        } else if constexpr (KIND == 5) { // 4 independent chains
            R64(asm volatile("v_add_u32 %0, %0, %4\n\tv_add_u32 %1, %1, %4\n\tv_add_u32 %2, %2, %4\n\tv_add_u32 %3, %3, %4"
                             : "+v"(a), "+v"(d), "+v"(e), "+v"(f) : "v"(b));)
        } else if constexpr (KIND == 6) { // MD5-like step: bitop3 -> add3(sgpr) -> alignbit -> add, + off-path add
            R64(asm volatile("v_add_u32 %3, %3, %5\n\t"
                             "v_bitop3_b32 %4, %0, %1, %2 bitop3:0xac\n\t"
                             "v_add3_u32 %4, %3, %4, %6\n\t"
                             "v_alignbit_b32 %4, %4, %4, 25\n\t"
                             "v_add_u32 %3, %4, %0"
                             : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e) : "v"(f), "s"(s));)
        } else if constexpr (KIND == 7) { // 8 independent chains (issue rate)
            R64(asm volatile("v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
                             "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8"
                             : "+v"(a), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h), "+v"(c), "+v"(b) : "v"(s));)
        } else if constexpr (KIND == 8) { // dependent v_xor_b32
            R64(asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(b));)
        } else if constexpr (KIND == 9) { // dependent add, VOP3 form with sgpr
            R64(asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a) : "s"(s));)
        }
    }
    unsigned long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d + e + f + g + h;
    if (threadIdx.x == 0)
        cyc[blockIdx.x] = t1 - t0;
}

template <int K, bool HALF = false>
int run(const char *name, int instrs_per_rep, int blocks, int threads)
{
    unsigned *o;
    unsigned long long *c;
    CK(hipMalloc(&o, blocks * threads * 4));
    CK(hipMalloc(&c, blocks * 8));
    hipLaunchKernelGGL((chain<K, HALF>), dim3(blocks), dim3(threads), 0, 0, o, c, 1u);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((chain<K, HALF>), dim3(blocks), dim3(threads), 0, 0, o, c, 2u);
    hipEventRecord(e1);
    CK(hipDeviceSynchronize());
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h;
    CK(hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost));
    double per = double(h) / (ITERS * 64.0 * instrs_per_rep);
    printf("%-48s blocks=%5d thr=%4d  %6.2f clk/instr (clock64), kernel %.1f us\n", name, blocks, threads, per, ms * 1e3);
    hipFree(o);
    hipFree(c);
    return 0;
}

int main()
{
    for (int cfg = 0; cfg < 2; cfg++) {
        int blocks = cfg == 0 ? 1 : 256, threads = cfg == 0 ? 64 : 256;
        run<0>("dep v_add_u32", 1, blocks, threads);
        run<9>("dep v_add_u32_e64 (sgpr)", 1, blocks, threads);
        run<8>("dep v_xor_b32", 1, blocks, threads);
        run<1>("dep v_add3_u32", 1, blocks, threads);
        run<2>("dep v_alignbit_b32", 1, blocks, threads);
        run<3>("dep v_bitop3_b32", 1, blocks, threads);
        run<4>("2 chains v_add_u32", 2, blocks, threads);
        run<5>("4 chains v_add_u32", 4, blocks, threads);
        run<7>("8 chains v_add_u32", 8, blocks, threads);
        run<6>("md5-like step (5 instr)", 5, blocks, threads);
    }
    // clock64 = s_memtime: shader clock.  Also 2 waves per SIMD:
    run<0>("dep v_add_u32, 2 waves/SIMD", 1, 256, 512);
    run<6>("md5-like step, 2 waves/SIMD", 5, 256, 512);
    run<6>("md5-like step, 4 waves/SIMD", 5, 256, 1024);
    // half-filled waves (32 active lanes): does a wave64 op with half EXEC cost less?
    run<6, true>("md5-like step, 1 wave/SIMD, 32 lanes", 5, 256, 256);
    run<6, true>("md5-like step, 2 waves/SIMD, 32 lanes", 5, 256, 512);
    run<0, true>("dep v_add_u32, 2 waves/SIMD, 32 lanes", 1, 256, 512);
    run<7, true>("8 chains v_add_u32, 32 lanes", 8, 256, 256);
    run<7>("8 chains v_add_u32, 64 lanes", 8, 256, 256);
    return 0;
}
