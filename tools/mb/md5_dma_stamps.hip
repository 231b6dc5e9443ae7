// md5_dma_stamps.hip -- where does a cfg2 MD5 wave spend its time?  Diagnostic build of the
// LDS-DMA kernel with s_memtime stamps (start, after each block, end) per wave.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../brb_framework_amd/csrc/gpu md5_dma_stamps.hip -o md5stamps
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "dma_stage.h"
#include "md5_device.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

BRB_DEV uint64_t stamp()
{
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

template <int WAVES, int P, bool SCHED, bool STAMP>
__global__ __launch_bounds__(64 * WAVES) void k(const uint8_t *__restrict__ data, uint32_t rec_len, uint32_t stride, uint64_t n_rec,
                                                uint4 *__restrict__ out, uint64_t *__restrict__ st_out)
{
    __shared__ __attribute__((aligned(16))) uint8_t ring[WAVES * P * brb_dma::kSlotBytes];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t wid = uint64_t(blockIdx.x) * WAVES + wv;
    const uint64_t rbase = wid * 64;
    if (rbase >= n_rec)
        return;
    uint64_t *so = st_out + wid * 32;
    if (STAMP && lane == 0)
        so[0] = stamp();
    const uint32_t n_wave = 64;
    uint8_t *my = ring + wv * (P * brb_dma::kSlotBytes);
    const uint32_t lds_base = uint32_t(reinterpret_cast<uintptr_t>(my));
    brb_dma::Stager sg;
    sg.init(data + rbase * stride, stride, n_wave, (n_rec - rbase) * stride + 4096, lane);
    const uint32_t nfull = rec_len >> 6;
    Md5State st = md5_iv();
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < P - 1; i++)
        if (uint32_t(i) < nfull)
            sg.issue(lds_base + i * brb_dma::kSlotBytes, i);
    uint32_t slot = 0;
    for (uint32_t b = 0; b < nfull; b++) {
        const uint32_t nb = b + P - 1;
        if (nb < nfull) {
            sg.issue(lds_base + (nb % P) * brb_dma::kSlotBytes, nb);
            brb_dma::wait_vmcnt<4 * (P - 1)>();
        } else {
            brb_dma::wait_vmcnt<0>();
        }
        sg.read(my + slot * brb_dma::kSlotBytes, w);
        slot = slot + 1 == P ? 0 : slot + 1;
        if (SCHED)
            md5_compress_sched(st, w);
        else
            md5_compress(st, w);
        if (STAMP && lane == 0 && b < 28)
            so[1 + b] = stamp();
    }
    for (int i = 0; i < 16; i++)
        w[i] = i == 0 ? 0x80 : 0;
    md5_finish(st, w, 0, rec_len);
    out[rbase + lane] = make_uint4(st.a, st.b, st.c, st.d);
    if (STAMP && lane == 0)
        so[31] = stamp();
}

using Kern = void (*)(const uint8_t *, uint32_t, uint32_t, uint64_t, uint4 *, uint64_t *);

int main()
{
    const uint32_t L = 1536;    // 24 full blocks, no tail: isolates the block loop
    const uint64_t n = 65536;
    std::vector<uint8_t> h(n * L);
    uint64_t x = 99;
    for (auto &c : h) { x = x * 6364136223846793005ull + 1442695040888963407ull; c = uint8_t(x >> 56); }
    const int nrot = 6;
    uint8_t *d[nrot];
    for (int i = 0; i < nrot; i++) {
        CK(hipMalloc(&d[i], n * L + 8192));
        CK(hipMemcpy(d[i], h.data(), n * L, hipMemcpyHostToDevice));
    }
    uint4 *o;
    uint64_t *stp;
    CK(hipMalloc(&o, n * 16));
    CK(hipMalloc(&stp, 1024 * 32 * 8));
    struct V { const char *name; Kern k; int waves; bool alias; };
    std::vector<V> vs = {
        {"P8 W4 sched", k<4, 8, true, false>, 4, false},
        {"P8 W4 plain", k<4, 8, false, false>, 4, false},
        {"P4 W4 sched", k<4, 4, true, false>, 4, false},
        {"P2 W4 sched", k<4, 2, true, false>, 4, false},
        {"P8 W1 sched", k<1, 8, true, false>, 1, false},
        {"P8 W4 sched alias(compute floor)", k<4, 8, true, false>, 4, true},
        {"P8 W4 plain alias(compute floor)", k<4, 8, false, false>, 4, true},
    };
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<std::vector<float>> t(vs.size());
    int it = 0;
    for (int rep = 0; rep < 20; rep++)
        for (size_t v = 0; v < vs.size(); v++) {
            const unsigned grid = unsigned(n / (64 * vs[v].waves));
            hipEventRecord(e0);
            hipLaunchKernelGGL(vs[v].k, dim3(grid), dim3(64 * vs[v].waves), 0, 0, d[it++ % nrot], L, vs[v].alias ? 0u : L, n, o, stp);
            hipEventRecord(e1);
            CK(hipEventSynchronize(e1));
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            t[v].push_back(ms * 1e3f);
        }
    for (size_t v = 0; v < vs.size(); v++) {
        std::sort(t[v].begin(), t[v].end());
        printf("%-36s median %7.2f us  min %7.2f us\n", vs[v].name, t[v][t[v].size() / 2], t[v][0]);
    }
    // stamped runs
    Kern ks[4] = {k<4, 8, true, true>, k<4, 8, true, true>, k<4, 8, false, true>, k<4, 8, false, true>};
    const char *kn[4] = {"STREAM P8 sched", "ALIAS P8 sched", "STREAM P8 plain", "ALIAS P8 plain"};
    for (int a = 0; a < 4; a++) {
        CK(hipMemset(stp, 0, 1024 * 32 * 8));
        hipLaunchKernelGGL(ks[a], dim3(256), dim3(256), 0, 0, d[a % nrot], L, (a & 1) ? 0u : L, n, o, stp);
        CK(hipDeviceSynchronize());
        std::vector<uint64_t> s(1024 * 32);
        CK(hipMemcpy(s.data(), stp, s.size() * 8, hipMemcpyDeviceToHost));
        uint64_t t0 = UINT64_MAX, tend = 0;
        for (int w = 0; w < 1024; w++) { t0 = std::min(t0, s[w * 32]); tend = std::max(tend, s[w * 32 + 31]); }
        printf("\n%s:\n", kn[a]);
        // percentiles of: start offset, time to first block done, per-block time, end
        auto pct = [](std::vector<double> v, double p) { std::sort(v.begin(), v.end()); return v[size_t(p * (v.size() - 1))]; };
        std::vector<double> start, first, mid, last, end;
        for (int w = 0; w < 1024; w++) {
            const uint64_t *q = &s[w * 32];
            start.push_back(double(q[0] - t0));
            first.push_back(double(q[1] - q[0]));
            mid.push_back(double(q[23] - q[2]) / 21.0);
            last.push_back(double(q[24] - q[23]));
            end.push_back(double(q[31] - q[24]));
        }
        printf("  start offset   p0 %8.0f p50 %8.0f p100 %8.0f\n", pct(start, 0), pct(start, .5), pct(start, 1));
        printf("  block 0        p0 %8.0f p50 %8.0f p100 %8.0f\n", pct(first, 0), pct(first, .5), pct(first, 1));
        printf("  blocks 2..23   p0 %8.0f p50 %8.0f p100 %8.0f (per block)\n", pct(mid, 0), pct(mid, .5), pct(mid, 1));
        printf("  finish+store   p0 %8.0f p50 %8.0f p100 %8.0f\n", pct(end, 0), pct(end, .5), pct(end, 1));
        // per-block profile of wave 0
        printf("  wave0 per block:");
        for (int b = 1; b < 25; b++) printf(" %llu", (unsigned long long)(s[b] - s[b - 1]));
        printf("\n");
    }
    return 0;
}
