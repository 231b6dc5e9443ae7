// lds_bytes.hip -- LDS throughput of the RC4 access pattern: per-lane random index x, address
// x * 256 + lane * 4 + wave (byte ops) and the 16/32-bit analogues, 4 waves per CU (one per SIMD),
// 256 workgroups.  Reports cycles per LDS instruction per CU (shader clock from s_memtime).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 lds_bytes.hip -o ldsb
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int N = 4096;   // iterations per wave, 8 LDS ops each

template <int MODE, bool LIN = false>   // 0: ds_read_u8, 1: ds_write_b8, 2: ds_read_u16, 3: ds_read_b32, 4: 3 u8 reads + 2 b8 writes
__global__ __launch_bounds__(256) void k(unsigned *out, unsigned long long *cyc)
{
    __shared__ __attribute__((aligned(16))) unsigned char lds[65536];
    const unsigned lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (unsigned i = threadIdx.x; i < 65536 / 4; i += 256) reinterpret_cast<unsigned *>(lds)[i] = i * 2654435761u;
    __syncthreads();
    unsigned x = lane * 977 + wv * 131 + blockIdx.x, acc = 0;
    const unsigned lw = lane * 4 + wv;
    unsigned a[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
        x = x * 1664525u + 1013904223u;
        a[q] = LIN ? (q << 10) + lane * 4 : ((x >> 24) << 8) | lw;   // LIN: consecutive dwords
    }
    unsigned long long t0 = clock64();
    for (int it = 0; it < N; it++) {
#pragma unroll
        for (int q = 0; q < 8; q++)
            asm volatile("" : "+v"(a[q]));
        if (MODE == 0) {
            unsigned v[8];
#pragma unroll
            for (int q = 0; q < 8; q++) asm volatile("ds_read_u8 %0, %1" : "=v"(v[q]) : "v"(a[q]) : "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int q = 0; q < 8; q++) acc += v[q];
        } else if (MODE == 1) {
#pragma unroll
            for (int q = 0; q < 8; q++) asm volatile("ds_write_b8 %0, %1" :: "v"(a[q]), "v"(x) : "memory");
        } else if (MODE == 2) {
            unsigned v[8];
#pragma unroll
            for (int q = 0; q < 8; q++) asm volatile("ds_read_u16 %0, %1" : "=v"(v[q]) : "v"(a[q] & ~1u) : "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int q = 0; q < 8; q++) acc += v[q];
        } else if (MODE == 3) {
            unsigned v[8];
#pragma unroll
            for (int q = 0; q < 8; q++) asm volatile("ds_read_b32 %0, %1" : "=v"(v[q]) : "v"((a[q] & 0xFF00u) | (lane * 4)) : "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int q = 0; q < 8; q++) acc += v[q];
        } else {
            unsigned v[5];
            asm volatile("ds_read_u8 %0, %1" : "=v"(v[0]) : "v"(a[0]) : "memory");
            asm volatile("ds_read_u8 %0, %1" : "=v"(v[1]) : "v"(a[1]) : "memory");
            asm volatile("ds_write_b8 %0, %1" :: "v"(a[2]), "v"(x) : "memory");
            asm volatile("ds_write_b8 %0, %1" :: "v"(a[3]), "v"(x) : "memory");
            asm volatile("ds_read_u8 %0, %1" : "=v"(v[2]) : "v"(a[4]) : "memory");
            asm volatile("ds_read_u8 %0, %1" : "=v"(v[3]) : "v"(a[5]) : "memory");
            asm volatile("ds_write_b8 %0, %1" :: "v"(a[6]), "v"(x) : "memory");
            asm volatile("ds_write_b8 %0, %1" :: "v"(a[7]), "v"(x) : "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            acc += v[0] + v[1] + v[2] + v[3];
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    unsigned long long t1 = clock64();
    if (lane == 0 && wv == 0) cyc[blockIdx.x] = t1 - t0;
    if (acc == 0x12345) out[0] = acc;
}

template <int M, bool LIN = false>
void run(const char *name, unsigned *o, unsigned long long *c)
{
    hipLaunchKernelGGL((k<M, LIN>), dim3(256), dim3(256), 0, 0, o, c);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((k<M, LIN>), dim3(256), dim3(256), 0, 0, o, c);
    hipEventRecord(e1);
    CK(hipEventSynchronize(e1));
    float ms; hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[256];
    CK(hipMemcpy(h, c, sizeof h, hipMemcpyDeviceToHost));
    unsigned long long s = 0; for (auto v : h) s += v;
    const double cyc = double(s) / 256, ops_cu = 4.0 * N * 8;
    printf("%-28s %8.2f cycles per LDS instr per CU (wave clock), kernel %.1f us\n", name, cyc / ops_cu, ms * 1e3);
}

int main()
{
    unsigned *o; unsigned long long *c;
    CK(hipMalloc(&o, 64)); CK(hipMalloc(&c, 256 * 8));
    for (int r = 0; r < 2; r++) {
        run<0>("ds_read_u8 x8", o, c);
        run<1>("ds_write_b8 x8", o, c);
        run<2>("ds_read_u16 x8", o, c);
        run<3>("ds_read_b32 x8", o, c);
        run<4>("4 x u8 read + 4 x b8 write", o, c);
        run<0, true>("ds_read_u8 linear", o, c);
        run<3, true>("ds_read_b32 linear", o, c);
        run<1, true>("ds_write_b8 linear", o, c);
    }
    return 0;
}
