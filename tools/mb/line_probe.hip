// line_probe.hip -- where does a wave of the line-aligned digest kernel spend its time?
// Per wave: shader-clock and 100 MHz real-time stamps at start and end, and the shader clocks spent
// waiting for its LDS-DMA lines (s_waitcnt vmcnt + the window read).  Prints the clock, the start /
// end skew over waves and the wait fraction.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../brb_framework_amd/csrc/gpu line_probe.hip -o lprobe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <string>
#include <vector>

__device__ uint64_t *g_probe;
__device__ inline uint64_t pr_clk()
{
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
__device__ inline uint64_t pr_rt()
{
    uint64_t t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
#define BRB_LINE_PROBE 1
#define NP 8
#define BRB_LINE_PROBE_DECL uint64_t pr_c0 = 0, pr_r0 = 0, pr_tw = 0, pr_wait = 0, pr_first = 0;
#define BRB_LINE_PROBE(ev)                                                              \
    do {                                                                                \
        if ((ev) == 0) { pr_c0 = pr_clk(); pr_r0 = pr_rt(); }                           \
        if ((ev) == 1) pr_tw = pr_clk();                                                \
        if ((ev) == 2) { pr_wait += pr_clk() - pr_tw; if (!pr_first) pr_first = pr_wait; } \
        if ((ev) == 3 && lane == 0) {                                                   \
            uint64_t *o = g_probe + NP * wave0;                                         \
            o[0] = pr_c0; o[1] = pr_clk(); o[2] = pr_r0; o[3] = pr_rt(); o[4] = pr_wait;\
            o[5] = pr_first;                                                            \
            uint32_t xcc_, hw_;                                                         \
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc_));   \
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_));           \
            o[6] = xcc_; o[7] = hw_;                                                    \
        }                                                                               \
    } while (0)

#include "digest_dma.h"
#include "digest_line.h"
#include "line1_kernel.h"
#include "line_r05_kernel.h"
#include "md5_device.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct AlgLit {
    using State = Md5State;
    static BRB_DEV State iv() { return md5_iv(); }
    static BRB_DEV void compress(State &st, uint32_t (&w)[16]) { md5_compress(st, w); }
    static BRB_DEV void finish(State &st, uint32_t (&w)[16], uint32_t t, uint64_t len) { md5_finish(st, w, t, len); }
    static BRB_DEV void pad_only(State &st, uint64_t len) { md5_pad_only(st, len); }
    template <bool A> static BRB_DEV void store(uint8_t *out, uint64_t r, const State &st)
    { reinterpret_cast<uint4 *>(out)[r] = make_uint4(st.a, st.b, st.c, st.d); }
};
struct AlgNull : AlgLit {
    static BRB_DEV void compress(State &st, uint32_t (&w)[16])
    {
        uint32_t x = 0;
#pragma unroll
        for (int i = 0; i < 16; i++) x ^= w[i];
        st.a ^= x;
    }
    static BRB_DEV void finish(State &st, uint32_t (&w)[16], uint32_t, uint64_t) { st.b ^= w[0]; }
    static BRB_DEV void pad_only(State &st, uint64_t len) { st.b ^= uint32_t(len); }
};

using Kern = void (*)(const uint8_t *, uint32_t, uint64_t, uint8_t *);
using KernL = void (*)(const uint8_t *, uint32_t, uint64_t, uint8_t *, uint32_t *, uint32_t);
// pool heads for the POOL line kernel: a ring of slots, each zeroed by its launch's last workgroup
static uint32_t *g_pool_ring;
static uint64_t g_pool_next;
// launches a kernel of the four arguments (data, rec_len, n_rec, out), or a line kernel of six
// (+ pool slot, owned rounds; pool_rounds < 0: a kernel of four arguments)
static void launch(const void *k, unsigned grid, unsigned bs, const uint8_t *src, uint32_t L, uint64_t n, uint8_t *o,
                   int pool_rounds = -1)
{
    if (pool_rounds < 0) {
        void *args[] = {&src, &L, &n, &o};
        if (hipLaunchKernel(k, dim3(grid), dim3(bs), args, 0, 0) != hipSuccess) { printf("launch failed\n"); exit(1); }
        return;
    }
    const uint64_t groups = (n + 63) / 64, rounds = (groups + grid - 1) / grid;
    uint32_t *slot = g_pool_ring + (g_pool_next++ % brb_mb_r05::kPoolSlots) * brb_mb_r05::kPoolSlotWords;
    uint32_t t_own = uint32_t(rounds - uint64_t(pool_rounds));
    void *args[] = {&src, &L, &n, &o, &slot, &t_own};
    if (hipLaunchKernel(k, dim3(grid), dim3(bs), args, 0, 0) != hipSuccess) { printf("launch failed\n"); exit(1); }
}

static double pct(std::vector<double> v, double p)
{
    std::sort(v.begin(), v.end());
    return v[size_t(p * (v.size() - 1))];
}

int main(int argc, char **argv)
{
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 65536;
    const uint32_t L = argc > 2 ? atoi(argv[2]) : 1500;
    const int nrot = std::max<int>(2, int(700e6 / double(n * L)) + 1);
    std::vector<uint8_t> h(n * L);
    uint64_t x = 7;
    for (auto &c : h) { x = x * 6364136223846793005ull + 1442695040888963407ull; c = uint8_t(x >> 56); }
    std::vector<uint8_t *> d(nrot);
    for (auto &p : d) { CK(hipMalloc(&p, n * L + 8192)); CK(hipMemcpy(p, h.data(), n * L, hipMemcpyHostToDevice)); }
    uint8_t *o;
    CK(hipMalloc(&o, n * 16));
    const uint64_t groups = (n + 63) / 64;
    uint64_t *pr;
    CK(hipMalloc(&pr, 4096 * NP * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_probe), &pr, sizeof(pr)));
    struct V { const char *name; Kern k; };
    struct VG { const char *name; const void *k; int waves; int pool = -1; };
    CK(hipMalloc(&g_pool_ring, size_t(brb_mb_r05::kPoolSlots) * brb_mb_r05::kPoolSlotWords * 4));
    CK(hipMemset(g_pool_ring, 0, size_t(brb_mb_r05::kPoolSlots) * brb_mb_r05::kPoolSlotWords * 4));
    VG vs64[] = {{"DMA64 static 4x4", (const void *)(Kern)brb_digest::digest_fixed_dma_kernel<AlgLit, 4, 2, 1, true>, 4},
                 {"DMA64 dyn16", (const void *)(Kern)brb_digest::digest_fixed_dma_kernel<AlgLit, 16, 2, 1, true, false, true>, 16},
                 {"DMA64 dyn8", (const void *)(Kern)brb_digest::digest_fixed_dma_kernel<AlgLit, 8, 2, 1, true, false, true>, 8},
                 {"DMA64 only", (const void *)(Kern)brb_digest::digest_fixed_dma_kernel<AlgNull, 4, 2, 1, true>, 4}};
    // waves = -4: digest_line1_kernel (one group per wave, 4-wave workgroups, grid = groups / 4)
    // argv[3] = "pool": the product line kernel without and with the tail pool (4 / 8 / 16 rounds),
    // the static split with SIMD partners in lockstep (LOCK) and without, interleaved twice (VERDICT
    // r04 item 2: the workgroup-end spread)
    VG vp[] = {{"LINE nopool", (const void *)(KernL)brb_mb_r05::digest_line_kernel<AlgLit, 8, true, true, true>, 8, 0},
               {"LINE lock", (const void *)(KernL)brb_mb_r05::digest_line_kernel<AlgLit, 8, true, true, false, false, true>, 8, 0},
               {"LINE static", (const void *)(KernL)brb_mb_r05::digest_line_kernel<AlgLit, 8, true, true, false>, 8, 0},
               {"LINE pool8", (const void *)(KernL)brb_mb_r05::digest_line_kernel<AlgLit, 8, true, true, true, true>, 8, 8},
               {"LINE pool4", (const void *)(KernL)brb_mb_r05::digest_line_kernel<AlgLit, 8, true, true, true, true>, 8, 4},
               {"LINE pool16", (const void *)(KernL)brb_mb_r05::digest_line_kernel<AlgLit, 8, true, true, true, true>, 8, 16},
               {"LINE nopool #2", (const void *)(KernL)brb_mb_r05::digest_line_kernel<AlgLit, 8, true, true, true>, 8, 0},
               {"LINE lock #2", (const void *)(KernL)brb_mb_r05::digest_line_kernel<AlgLit, 8, true, true, false, false, true>, 8, 0},
               {"LINE pool8 #2", (const void *)(KernL)brb_mb_r05::digest_line_kernel<AlgLit, 8, true, true, true, true>, 8, 8},
               {"LINE pool4 #2", (const void *)(KernL)brb_mb_r05::digest_line_kernel<AlgLit, 8, true, true, true, true>, 8, 4},
               {"LINE pool16 #2", (const void *)(KernL)brb_mb_r05::digest_line_kernel<AlgLit, 8, true, true, true, true>, 8, 16}};
    VG vs[] = {{"LINE md5 nt dyn8", (const void *)(KernL)brb_mb_r05::digest_line_kernel<AlgLit, 8, true, true, true>, 8, 0},
              {"LINE1 ns3", (const void *)(Kern)brb_digest::digest_line1_kernel<AlgLit, true, true, 3>, -4},
              {"LINE1 ns2", (const void *)(Kern)brb_digest::digest_line1_kernel<AlgLit, true, true, 2>, -4},
              {"LINE1 ns2 u4", (const void *)(Kern)brb_digest::digest_line1_kernel<AlgLit, true, true, 2, false, 4>, -4},
              {"LINE1 ns3 spread", (const void *)(Kern)brb_digest::digest_line1_kernel<AlgLit, true, true, 3, true>, -4},
              {"LINE1 ns2 spread", (const void *)(Kern)brb_digest::digest_line1_kernel<AlgLit, true, true, 2, true>, -4},
              {"LINE md5 nt dyn8 #2", (const void *)(KernL)brb_mb_r05::digest_line_kernel<AlgLit, 8, true, true, true>, 8, 0},
              {"LINE1 ns3 #2", (const void *)(Kern)brb_digest::digest_line1_kernel<AlgLit, true, true, 3>, -4},
              {"LINE1 ns2 #2", (const void *)(Kern)brb_digest::digest_line1_kernel<AlgLit, true, true, 2>, -4},
              {"LINE1 ns2 u4 #2", (const void *)(Kern)brb_digest::digest_line1_kernel<AlgLit, true, true, 2, false, 4>, -4},
              {"LINE1 dma-only ns3", (const void *)(Kern)brb_digest::digest_line1_kernel<AlgNull, true, true, 3>, -4},
              {"LINE dma-only nt dyn8", (const void *)(KernL)brb_mb_r05::digest_line_kernel<AlgNull, 8, true, true, true>, 8, 0}};
    // argv[3] = "r06": the product kernel (digest_line.h, round 6) twice and its DMA-only form
    const bool hi = brb_digest::line_tail_hi(L);
    VG v6[] = {{"r06 product", hi ? (const void *)(Kern)brb_digest::digest_line_kernel<AlgLit, 8, true, true>
                                  : (const void *)(Kern)brb_digest::digest_line_kernel<AlgLit, 8, true, false>, 8},
               {"r06 dma-only", hi ? (const void *)(Kern)brb_digest::digest_line_kernel<AlgNull, 8, true, true>
                                   : (const void *)(Kern)brb_digest::digest_line_kernel<AlgNull, 8, true, false>, 8},
               {"r06 product #2", hi ? (const void *)(Kern)brb_digest::digest_line_kernel<AlgLit, 8, true, true>
                                     : (const void *)(Kern)brb_digest::digest_line_kernel<AlgLit, 8, true, false>, 8}};
    int it = 0;
    const bool small = L <= 64;
    const bool pool = argc > 3 && std::string(argv[3]) == "pool";
    const bool r06 = argc > 3 && std::string(argv[3]) == "r06";
    const int nv = small ? 4 : pool ? int(sizeof(vp) / sizeof(vp[0])) : r06 ? 3 : int(sizeof(vs) / sizeof(vs[0]));
    for (int vi = 0; vi < nv; vi++) {
        const VG &v = small ? vs64[vi] : pool ? vp[vi] : r06 ? v6[vi] : vs[vi];
        // 4-wave workgroups: 2 per CU (4 for <= 64 B records); bigger (dyn): one per CU
        const unsigned grid = v.waves == -4 ? unsigned((groups + 3) / 4)
                              : v.waves == 4 ? unsigned(std::min<uint64_t>((groups + 3) / 4, small ? 1024 : 512))
                                             : unsigned(std::min<uint64_t>(groups, 256));
        const uint64_t waves = std::min<uint64_t>(uint64_t(grid) * (v.waves < 0 ? 4 : v.waves), groups);
        const unsigned bs = 64 * (v.waves < 0 ? 4 : v.waves);
        // warm up >= 0.5 s (clocks), then probe one launch out of a back-to-back burst
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        float tot = 0;
        while (tot < 500.f) {
            hipEventRecord(a);
            for (int i = 0; i < 50; i++) launch(v.k, grid, bs, d[it++ % nrot], L, n, o, v.pool);
            hipEventRecord(b);
            CK(hipEventSynchronize(b));
            float ms;
            hipEventElapsedTime(&ms, a, b);
            tot += ms;
        }
        for (int i = 0; i < 9; i++) launch(v.k, grid, bs, d[it++ % nrot], L, n, o, v.pool);
        CK(hipMemsetAsync(pr, 0, 4096 * NP * 8));
        launch(v.k, grid, bs, d[it++ % nrot], L, n, o, v.pool);
        CK(hipDeviceSynchronize());
        std::vector<uint64_t> all(4096 * NP), hp;
        CK(hipMemcpy(all.data(), pr, all.size() * 8, hipMemcpyDeviceToHost));
        std::vector<uint64_t> widx;
        for (uint64_t w = 0; w < 4096; w++)
            if (all[NP * w + 1]) {
                widx.push_back(w);
                hp.insert(hp.end(), &all[NP * w], &all[NP * w + NP]);
            }
        (void)waves;
        const uint64_t nw = widx.size();
        uint64_t r0 = ~0ull, r1 = 0;
        for (uint64_t w = 0; w < nw; w++) { r0 = std::min(r0, hp[NP * w + 2]); r1 = std::max(r1, hp[NP * w + 3]); }
        std::vector<double> mhz, st, en, dur, wf, fw;
        for (uint64_t w = 0; w < nw; w++) {
            const uint64_t *q = &hp[NP * w];
            const double rt = double(q[3] - q[2]) * 10.0;  // ns (100 MHz)
            mhz.push_back(double(q[1] - q[0]) / (rt * 1e-3));
            st.push_back(double(q[2] - r0) * 10.0 / 1000.0);
            en.push_back(double(q[3] - r0) * 10.0 / 1000.0);
            dur.push_back(rt / 1000.0);
            wf.push_back(double(q[4]) / double(q[1] - q[0]));
            fw.push_back(double(q[5]) / (double(q[1] - q[0]) / dur.back()));   // us
        }
        {   // per-XCD (HW_REG_XCC_ID) median in-kernel clock, mean end, wave count
            printf("  per-XCC (hw): ");
            for (int x = 0; x < 8; x++) {
                std::vector<double> cm, ce;
                for (uint64_t w = 0; w < nw; w++)
                    if (hp[NP * w + 6] == uint64_t(x)) { cm.push_back(mhz[w]); ce.push_back(en[w]); }
                if (cm.empty()) continue;
                double se = 0; for (double e : ce) se += e;
                printf(" x%d: %zu waves %.0f MHz end %.1f |", x, cm.size(), pct(cm, .5), se / ce.size());
            }
            printf("\n");
        }
        {   // per-XCD (blockIdx % 8) mean end time, and a histogram of end times
            double sx[8] = {0}; int cx[8] = {0};
            for (uint64_t w = 0; w < nw; w++) { sx[(widx[w] / (v.waves < 0 ? 4 : v.waves)) % 8] += en[w]; cx[(widx[w] / (v.waves < 0 ? 4 : v.waves)) % 8]++; }
            printf("  waves %llu, per-XCD mean end us:", (unsigned long long)nw);
            for (int i = 0; i < 8; i++) printf(" %.1f", sx[i] / cx[i]);
            printf("\n  end pcts:");
            for (double q : {0.0, 0.1, 0.25, 0.5, 0.75, 0.9, 0.95, 0.99, 1.0}) printf(" p%g=%.1f", q * 100, pct(en, q));
            std::vector<double> by_slot[2];
            for (uint64_t w = 0; w < nw; w++) by_slot[widx[w] / 1024 % 2].push_back(en[w]);
            {   // per workgroup (CU): latest and earliest wave end
                std::vector<double> wmax(4096, 0.0), wmin(4096, 1e30), spread, maxs;
                const int wpb = v.waves < 0 ? 4 : v.waves;
                for (uint64_t w = 0; w < nw; w++) {
                    const uint64_t b = widx[w] / wpb;
                    wmax[b] = std::max(wmax[b], en[w]);
                    wmin[b] = std::min(wmin[b], en[w]);
                }
                for (int b = 0; b < 4096; b++)
                    if (wmax[b] > 0) { maxs.push_back(wmax[b]); spread.push_back(wmax[b] - wmin[b]); }
                printf("\n  per-WG last end p0 %.1f p50 %.1f p100 %.1f | per-WG end spread p10 %.1f p50 %.1f p90 %.1f", pct(maxs, 0),
                       pct(maxs, .5), pct(maxs, 1), pct(spread, .1), pct(spread, .5), pct(spread, .9));
            }
            printf("\n  WG<256 end p50 %.1f p90 %.1f | WG>=256 end p50 %.1f p90 %.1f\n", pct(by_slot[0], .5), pct(by_slot[0], .9),
                   by_slot[1].empty() ? 0.0 : pct(by_slot[1], .5), by_slot[1].empty() ? 0.0 : pct(by_slot[1], .9));
        }
        printf("%-18s n=%llu L=%u  span %.2f us | clock MHz p50 %.0f | start us p0 %.2f p50 %.2f p100 %.2f | end us p0 %.2f p50 %.2f p100 %.2f | wave us p50 %.2f | wait frac p10 %.2f p50 %.2f p90 %.2f\n",
               v.name, (unsigned long long)n, L, double(r1 - r0) * 10.0 / 1000.0, pct(mhz, .5), pct(st, 0), pct(st, .5), pct(st, 1),
               pct(en, 0), pct(en, .5), pct(en, 1), pct(dur, .5), pct(wf, .1), pct(wf, .5), pct(wf, .9));
        printf("  first line-pair wait us p10 %.2f p50 %.2f p90 %.2f p100 %.2f\n", pct(fw, .1), pct(fw, .5), pct(fw, .9), pct(fw, 1));
    }
    return 0;
}
