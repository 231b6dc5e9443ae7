// line1_kernel.h -- EXPERIMENT (not in the product): the line-aligned digest kernel for batches
// of at most one 64-record group per wave, with a ring of NS = 2 or 3 lines per wave.
// Measured with line_probe.hip on cfg2 (65 536 x 1500 B), three runs on two boxes: NS = 3 cuts the
// waves' wait fraction from 14 % to 9 % and streams the DMA-only variant faster (17.0-17.7 vs
// 17.7-19.1 us), but its waves spend ~8 % more cycles per record (42.3-42.8 K vs 39.1 K), so the
// kernel is slower: 21.6-23.4 us against 20.4-21.3 us for NS = 2 (which itself matches the product's
// 8-wave ticketed kernel).  Unrolling NS = 2 to eight compress sites (U = 4) changed nothing, so
// instruction-cache size is not the cause.  Kept for reproduction; DESIGN.md §4.1.
#pragma once

#include "digest_line.h"
#include "line_r05_kernel.h"   // round 5's line_finish / tail_masks signatures

namespace brb_digest {

// One group per wave (batches of at most 4 groups per CU: cfg2's 65 536 records are exactly 1 024
// groups for 256 CUs).  With no next group to prefetch, each wave keeps a THREE-line ring (4 waves
// x 3 x 8 KiB = 96 KiB of LDS, one workgroup per CU): while blocks 2k-2 and 2k-1 are hashed from
// lines k-1 and k, line k+1 is already in flight and line k+2 is requested into the slot of line
// k-1, so a line has two iterations (~3 K cycles) to land instead of one.  Line j sits in slot
// j % 3; the window of iteration k reads lines (k-1, k) through the address table of phase
// (k-1) % 3, and the loop is unrolled by three so that each phase has its own table.
// tools/mb/line_probe.hip (cfg2): with the two-line ring waves spent ~1.1 us per record waiting for
// lines after the first pair.
// NS = ring slots (2 or 3); SPREAD: group of wave wv of workgroup b = b + wv * gridDim.x (a
// workgroup's groups are far apart) instead of 4b + wv.
template <class Alg, bool OUT_ALIGNED, bool NT = false, int NS = 3, bool SPREAD = false, int U = NS>
__global__ __launch_bounds__(256, 1) void digest_line1_kernel(const uint8_t *__restrict__ data, uint32_t rec_len,
                                                              uint64_t n_rec, uint8_t *__restrict__ out)
{
    static_assert(NS == 2 || NS == 3, "ring of two or three lines");
    constexpr uint32_t SLOT = 8192, WAVES = 4;
    __shared__ __attribute__((aligned(16))) uint8_t ring[WAVES * NS * SLOT];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t n_groups = (n_rec + 63) / 64;
    const uint64_t g = SPREAD ? uint64_t(blockIdx.x) + uint64_t(wv) * gridDim.x : uint64_t(blockIdx.x) * WAVES + wv;
    const uint64_t wave0 = g;                                  // (probe hooks)
    if (g >= n_groups)
        return;
    const uint32_t my_off = wv * NS * SLOT;
    const uint32_t lds0 = uint32_t(reinterpret_cast<uintptr_t>(ring)) + my_off;
    const uint32_t nfull = rec_len >> 6, t = rec_len & 63;
    const uint32_t nblk = nfull + (t ? 1 : 0);
    const uint32_t K = (nblk + 1) >> 1;                        // 2-block iterations; K + 1 lines
    const uint64_t dbase = reinterpret_cast<uint64_t>(data);
    const uint64_t end_line = (dbase + n_rec * rec_len + 127) & ~uint64_t(127);
    auto swz = [](uint32_t row) { return (row >> 1) & 7; };

    // DMA issue: as digest_line_kernel (descriptor 4 KiB below the line, one M0 write per 4 DMAs)
    const uint64_t r0 = g * 64;
    const uint32_t last = uint32_t(n_rec - r0 < 64 ? n_rec - r0 - 1 : 63);
    const uint64_t a0 = dbase + r0 * rec_len;
    const uint32_t o0 = uint32_t(a0) & 127;
    uint32_t vq[8];
    brb_dma::v4i rs;
    {
        const uint64_t gbase = (a0 & ~uint64_t(127)) - 4096;
        const uint64_t gleft = end_line - gbase;
        rs.x = __builtin_amdgcn_readfirstlane(int(uint32_t(gbase)));
        rs.y = __builtin_amdgcn_readfirstlane(int(uint32_t(gbase >> 32) & 0xFFFF));
        rs.z = __builtin_amdgcn_readfirstlane(int(gleft > 0x7FFFFFFFull ? 0x7FFFFFFFu : uint32_t(gleft)));
        rs.w = 0x00020000;
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const uint32_t row = 8 * q + (lane >> 3);
            const uint32_t rr = row < last ? row : last;
            vq[q] = ((o0 + rr * rec_len) & ~127u) + 16 * ((lane & 7) ^ swz(row)) + 4096u - 1024u * (q & 3);
        }
    }
    auto issue = [&](uint32_t slot) {                          // the next line -> slot
        const uint32_t m = lds0 + slot * SLOT;
        uint32_t keep;
#define BRB_LINE1_DMA8(POL)                                                                     \
    asm volatile("s_mov_b32 %0, m0\n\t"                                                          \
                 "s_mov_b32 m0, %10\n\t"                                                         \
                 "s_nop 0\n\t"                                                                   \
                 "buffer_load_dwordx4 %1, %9, 0 offen " POL "lds\n\t"                            \
                 "buffer_load_dwordx4 %2, %9, 0 offen offset:1024 " POL "lds\n\t"                \
                 "buffer_load_dwordx4 %3, %9, 0 offen offset:2048 " POL "lds\n\t"                \
                 "buffer_load_dwordx4 %4, %9, 0 offen offset:3072 " POL "lds\n\t"                \
                 "s_mov_b32 m0, %11\n\t"                                                         \
                 "s_nop 0\n\t"                                                                   \
                 "buffer_load_dwordx4 %5, %9, 0 offen " POL "lds\n\t"                            \
                 "buffer_load_dwordx4 %6, %9, 0 offen offset:1024 " POL "lds\n\t"                \
                 "buffer_load_dwordx4 %7, %9, 0 offen offset:2048 " POL "lds\n\t"                \
                 "buffer_load_dwordx4 %8, %9, 0 offen offset:3072 " POL "lds\n\t"                \
                 "s_mov_b32 m0, %0"                                                               \
                 : "=&s"(keep)                                                                    \
                 : "v"(vq[0]), "v"(vq[1]), "v"(vq[2]), "v"(vq[3]), "v"(vq[4]), "v"(vq[5]), "v"(vq[6]), \
                   "v"(vq[7]), "s"(rs), "s"(m), "s"(m + 4096u)                                    \
                 : "memory")
        if constexpr (NT)
            BRB_LINE1_DMA8("nt ");
        else
            BRB_LINE1_DMA8("");
#undef BRB_LINE1_DMA8
        const uint64_t b = ((uint64_t(uint32_t(rs.y)) << 32) | uint32_t(rs.x)) + 128u;
        rs.x = int(uint32_t(b));
        rs.y = int(uint32_t(b >> 32));
        int z = rs.z;
        asm("s_sub_i32 %0, %0, 0x80\n\ts_max_i32 %0, %0, 0" : "+s"(z) : : "scc");
        rs.z = z;
    };

    // window address tables: phase v reads lines (k-1, k) from slots (v, (v + 1) % 3)
    uint32_t t0[32], t1[32], t2[32];
    {
        const uint32_t rr = lane < last ? lane : last;
        const uint32_t sh = ((o0 + rr * rec_len) & 127) >> 2;
        const uint32_t f = swz(lane), row = my_off + lane * 128;
#pragma unroll
        for (uint32_t i = 0; i < 32; i++) {
            const uint32_t q = sh + i, qq = q & 31;
            const uint32_t a = row + ((((qq >> 2) ^ f) << 4) | ((qq & 3) << 2));
            const bool hi = q >= 32;
            t0[i] = a + (hi ? SLOT : 0u);
            t1[i] = NS == 3 ? a + (hi ? 2 * SLOT : SLOT) : a + (hi ? 0u : SLOT);
            t2[i] = a + (hi ? 0u : 2 * SLOT);
            asm volatile("" : "+v"(t1[i]), "+v"(t2[i]));       // separate tables, not re-derived per use
        }
    }
    uint32_t w0[16], w1[16];
    auto read_window = [&](const uint32_t (&ad)[32]) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            w0[i] = *reinterpret_cast<const uint32_t *>(ring + ad[i]);
            w1[i] = *reinterpret_cast<const uint32_t *>(ring + ad[16 + i]);
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);                    // lgkmcnt(0): window in VGPRs
    };

    BRB_LINE_PROBE_DECL
    BRB_LINE_PROBE(0);
    issue(0);
    issue(1);
    if (NS == 3 && K >= 2)
        issue(2);
    typename Alg::State st = Alg::iv();
    // iteration k: line k landed (line k+1 may still be in flight), window (k-1, k), line k+2 into
    // the slot of line k-1, blocks 2k-2 and 2k-1
    auto step = [&](uint32_t k, const uint32_t (&ad)[32], uint32_t refill) {
        BRB_LINE_PROBE(1);
        if (NS == 3 && k < K)
            brb_dma::wait_vmcnt<8>();
        else
            brb_dma::wait_vmcnt<0>();
        read_window(ad);
        BRB_LINE_PROBE(2);
        if (k + NS - 1 <= K)
            issue(refill);
        const uint32_t b = 2 * k - 2;
        if (b < nfull)
            Alg::compress(st, w0);
        if (b + 1 < nfull)
            Alg::compress(st, w1);
    };
    for (uint32_t k = 1;; k += U) {
        step(k, t0, 0);
        if (k == K)
            break;
        step(k + 1, t1, 1);
        if (k + 1 == K)
            break;
        if constexpr (NS == 3) {
            step(k + 2, t2, 2);
            if (k + 2 == K)
                break;
        }
        if constexpr (NS == 2 && U == 4) {                     // (code-size experiment: eight sites)
            step(k + 2, t0, 0);
            if (k + 2 == K)
                break;
            step(k + 3, t1, 1);
            if (k + 3 == K)
                break;
        }
    }
    uint32_t tm[16], tp[16];
    brb_mb_r05::tail_masks(t, tm, tp);
    brb_mb_r05::line_finish<Alg, OUT_ALIGNED>(st, w0, w1, tm, tp, t, nfull, K, rec_len, out, r0 + lane, n_rec);
    BRB_LINE_PROBE(3);
}

}  // namespace brb_digest
