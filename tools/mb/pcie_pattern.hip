// pcie_pattern.hip -- GPU access to page-locked host memory: per-lane vs wave-cooperative 64-byte
// blocks.  n streams of L bytes (one lane per stream, as the batcher's RC4 kernels), each lane
// walking its stream block by block:
//   lane  : each lane loads / stores its own 64-byte block as 4 x 16-byte accesses (BlockSrc, Snk)
//   coop  : instruction q serves the blocks of lanes 16q .. 16q+15, 4 lanes x 16 B per block, so
//           one instruction covers 16 contiguous 64-byte pieces instead of 64 scattered 16-byte ones
// Modes: 0 lane read, 1 coop read, 2 lane write, 3 coop write, 4 lane read+write, 5 coop read+write.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 pcie_pattern.hip -o pciepat
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int MODE>
__global__ __launch_bounds__(256) void k(const uint8_t *in, uint8_t *out, uint32_t L, uint32_t n, uint32_t *sink)
{
    const uint32_t s = blockIdx.x * 256 + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nblk = L / 64;
    const bool rd = MODE == 0 || MODE == 1 || MODE >= 4, wr = MODE >= 2;
    const bool coop = MODE & 1;
    uint32_t acc = 0;
    const uint32_t s0 = s - lane;                   // first stream of this wave
    for (uint32_t b = 0; b < nblk; b++) {
        uint4 v[4];
        if (rd) {
            if (coop) {
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t ss = s0 + 16 * q + (lane >> 2);
                    v[q] = *reinterpret_cast<const uint4 *>(in + uint64_t(ss) * L + 64 * b + 16 * (lane & 3));
                }
            } else {
#pragma unroll
                for (int q = 0; q < 4; q++)
                    v[q] = *reinterpret_cast<const uint4 *>(in + uint64_t(s) * L + 64 * b + 16 * q);
            }
#pragma unroll
            for (int q = 0; q < 4; q++)
                acc ^= v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
        } else {
#pragma unroll
            for (int q = 0; q < 4; q++)
                v[q] = make_uint4(s + b, q, 7, 9);
        }
        if (wr) {
            if (coop) {
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t ss = s0 + 16 * q + (lane >> 2);
                    *reinterpret_cast<uint4 *>(out + uint64_t(ss) * L + 64 * b + 16 * (lane & 3)) = v[q];
                }
            } else {
#pragma unroll
                for (int q = 0; q < 4; q++)
                    *reinterpret_cast<uint4 *>(out + uint64_t(s) * L + 64 * b + 16 * q) = v[q];
            }
        }
    }
    if (acc == 0x12345678u)
        sink[0] = acc;
}

template <int MODE>
float run(const uint8_t *in, uint8_t *out, uint32_t L, uint32_t n, uint32_t *sink, int reps)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> t;
    for (int r = 0; r < reps + 2; r++) {
        CK(hipEventRecord(a));
        k<MODE><<<n / 256, 256>>>(in, out, L, n, sink);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r >= 2)
            t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2] * 1e3f;
}

int main(int argc, char **argv)
{
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 16384, L = argc > 2 ? atoi(argv[2]) : 1536;
    const size_t bytes = size_t(n) * L;
    uint8_t *hin, *hout;
    CK(hipHostMalloc(&hin, bytes, hipHostMallocMapped));
    CK(hipHostMalloc(&hout, bytes, hipHostMallocMapped));
    for (size_t i = 0; i < bytes; i++)
        hin[i] = uint8_t(i * 131);
    uint8_t *din, *dout;
    CK(hipHostGetDevicePointer(reinterpret_cast<void **>(&din), hin, 0));
    CK(hipHostGetDevicePointer(reinterpret_cast<void **>(&dout), hout, 0));
    uint32_t *sink;
    CK(hipMalloc(&sink, 4));
    const double mb = bytes / 1e6;
    const char *names[6] = {"lane read", "coop read", "lane write", "coop write", "lane read+write", "coop read+write"};
    float us[6];
    for (int rep = 0; rep < 2; rep++) {
        us[0] = run<0>(din, dout, L, n, sink, 10);
        us[1] = run<1>(din, dout, L, n, sink, 10);
        us[2] = run<2>(din, dout, L, n, sink, 10);
        us[3] = run<3>(din, dout, L, n, sink, 10);
        us[4] = run<4>(din, dout, L, n, sink, 10);
        us[5] = run<5>(din, dout, L, n, sink, 10);
    }
    for (int m = 0; m < 6; m++)
        printf("%-16s %8.1f us  %6.1f GB/s per direction\n", names[m], us[m], mb / us[m] * 1e3);
    // copy engines for comparison
    uint8_t *dev;
    CK(hipMalloc(&dev, bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int dir = 0; dir < 2; dir++) {
        std::vector<float> t;
        for (int r = 0; r < 12; r++) {
            CK(hipEventRecord(a));
            if (dir == 0)
                CK(hipMemcpyAsync(dev, hin, bytes, hipMemcpyHostToDevice, 0));
            else
                CK(hipMemcpyAsync(hout, dev, bytes, hipMemcpyDeviceToHost, 0));
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (r >= 2)
                t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        printf("%-16s %8.1f us  %6.1f GB/s\n", dir ? "memcpy D2H" : "memcpy H2D", t[5] * 1e3, mb / (t[5] * 1e3) * 1e3);
    }
    return 0;
}
