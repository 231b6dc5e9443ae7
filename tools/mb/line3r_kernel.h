// line3r_kernel.h -- experiment (round 6): the product line kernel (digest_line.h) with a THREE-slot
// ring, for launches of one group per wave (cfg2: 65 536 records = 1 024 groups = one wave per
// SIMD, four waves per CU, 24 KiB of LDS each).
//
// The per-wave probe puts cfg2 between its compression alone (17.3 us) and its
// staging alone (16.4 us) at 20-21 us: a lone wave waits for line k at the top of iteration k, and
// line k was issued only one iteration (two compressions, ~1.4 us) earlier.  Here line k+2 goes into
// the slot of line k-1 right after window k is read, so a line has two iterations to land.  Round 3
// measured a three-slot ring built on round 3's kernel (per-group setup, window reads behind the
// compression) slower; this one is the round-6 kernel with only the ring depth changed: three
// window-address tables (slot pairs (0,1), (1,2), (2,0)), the loop unrolled by three, wait_vmcnt<8>
// (line k+1 may still be in flight).  Used by tools/mb/line_ab.hip.
#pragma once

#include "digest_line.h"

namespace brb_mb_l3r {

template <class Alg, bool OUT_ALIGNED, bool TAIL_HI>
__global__ __launch_bounds__(256, 1) void digest_line3r_kernel(const uint8_t *__restrict__ data, uint32_t rec_len,
                                                               uint64_t n_rec, uint8_t *__restrict__ out)
{
    constexpr int WAVES = 4;
    constexpr uint32_t SLOT = 8192;
    __shared__ __attribute__((aligned(16))) uint8_t ring[WAVES * 3 * SLOT];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t n_groups = (n_rec + 63) / 64;
    const uint64_t g = uint64_t(blockIdx.x) * WAVES + wv;     // one group per wave
    if (g >= n_groups)
        return;
    const uint32_t my_off = wv * 3 * SLOT;
    const uint32_t lds0 = uint32_t(reinterpret_cast<uintptr_t>(ring)) + my_off;
    const uint32_t nfull = rec_len >> 6, t = rec_len & 63;
    const uint32_t nblk = nfull + (t ? 1 : 0);
    const uint32_t K = (nblk + 1) >> 1;                        // lines 0 .. K; line j in slot j % 3
    const uint64_t dbase = reinterpret_cast<uint64_t>(data);
    const uint64_t end_line = (dbase + n_rec * rec_len + 127) & ~uint64_t(127);
    const uint64_t gbytes = uint64_t(rec_len) * 64;
    const uint32_t o0 = uint32_t(dbase) & 127;
    auto swz = [](uint32_t row) { return (row >> 1) & 7; };
    uint32_t vq[8];
    {
        const uint32_t l3 = lane >> 3;
        const uint32_t base = o0 + l3 * rec_len;
        const uint32_t g0 = 16u * ((lane & 7) ^ (l3 >> 1));
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const uint32_t x = base + 8u * q * rec_len;
            vq[q] = ((x & ~127u) | (q & 1 ? g0 ^ 64u : g0)) + (4096u - 1024u * (q & 3));
        }
    }
    brb_dma::v4i rs;
    {
        const uint64_t gbase = ((dbase + g * gbytes) & ~uint64_t(127)) - 4096;
        const uint64_t gleft = end_line - gbase;
        rs.x = __builtin_amdgcn_readfirstlane(int(uint32_t(gbase)));
        rs.y = __builtin_amdgcn_readfirstlane(int(uint32_t(gbase >> 32) & 0xFFFF));
        rs.z = __builtin_amdgcn_readfirstlane(int(gleft > 0x7FFFFFFFull ? 0x7FFFFFFFu : uint32_t(gleft)));
        rs.w = 0x00020000;
    }
    uint32_t so = 0;
    auto issue = [&](uint32_t slot, bool keep_l2) {
        const uint32_t m = __builtin_amdgcn_readfirstlane(lds0 + slot * SLOT);
        const uint32_t sof = __builtin_amdgcn_readfirstlane(so);
        uint32_t keep;
#define BRB_L3R_DMA8(POL)                                                                       \
    asm volatile("s_mov_b32 %0, m0\n\t"                                                          \
                 "s_mov_b32 m0, %10\n\t"                                                         \
                 "s_nop 0\n\t"                                                                   \
                 "buffer_load_dwordx4 %1, %9, %12 offen " POL "lds\n\t"                         \
                 "buffer_load_dwordx4 %2, %9, %12 offen offset:1024 " POL "lds\n\t"             \
                 "buffer_load_dwordx4 %3, %9, %12 offen offset:2048 " POL "lds\n\t"             \
                 "buffer_load_dwordx4 %4, %9, %12 offen offset:3072 " POL "lds\n\t"             \
                 "s_mov_b32 m0, %11\n\t"                                                         \
                 "s_nop 0\n\t"                                                                   \
                 "buffer_load_dwordx4 %5, %9, %12 offen " POL "lds\n\t"                         \
                 "buffer_load_dwordx4 %6, %9, %12 offen offset:1024 " POL "lds\n\t"             \
                 "buffer_load_dwordx4 %7, %9, %12 offen offset:2048 " POL "lds\n\t"             \
                 "buffer_load_dwordx4 %8, %9, %12 offen offset:3072 " POL "lds\n\t"             \
                 "s_mov_b32 m0, %0"                                                               \
                 : "=&s"(keep)                                                                    \
                 : "v"(vq[0]), "v"(vq[1]), "v"(vq[2]), "v"(vq[3]), "v"(vq[4]), "v"(vq[5]), "v"(vq[6]), \
                   "v"(vq[7]), "s"(rs), "s"(m), "s"(m + 4096u), "s"(sof)                          \
                 : "memory")
        if (keep_l2)
            BRB_L3R_DMA8("");
        else
            BRB_L3R_DMA8("nt ");
#undef BRB_L3R_DMA8
        so += 128;
    };
    // lines 0, 1, 2 in flight before anything else
    issue(0, true);
    issue(1, true);
    if (K >= 2)
        issue(2, false);
    __builtin_amdgcn_sched_barrier(0);
    // window tables: lines (k-1, k) in slots (s, s+1 mod 3), s = (k-1) mod 3
    uint32_t t0[32], t1[32], t2[32];
    {
        const uint32_t sh4 = (o0 + lane * rec_len) & 127;
        const uint32_t fr = (my_off + lane * 128) | (swz(lane) << 4);
#pragma unroll
        for (uint32_t i = 0; i < 32; i++) {
            const uint32_t q4 = sh4 + 4 * i;
            const uint32_t in = (q4 & 124u) ^ fr, hi = (q4 & 128u) != 0;
            t0[i] = in + (hi ? 1u : 0u) * SLOT;                // slots 0, 1
            t1[i] = in + (hi ? 2u : 1u) * SLOT;                // slots 1, 2
            t2[i] = in + (hi ? 0u : 2u) * SLOT;                // slots 2, 0
            asm volatile("" : "+v"(t0[i]), "+v"(t1[i]), "+v"(t2[i]));
        }
    }
    uint32_t tm[16], tp[16];
    brb_digest::tail_masks(t, tm, tp);
    uint32_t w0[16], w1[16];
    auto read_window = [&](const uint32_t (&ad)[32]) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            w0[i] = *reinterpret_cast<const uint32_t *>(ring + ad[i]);
            w1[i] = *reinterpret_cast<const uint32_t *>(ring + ad[16 + i]);
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
    };
    typename Alg::State st = Alg::iv();
    // iteration k < K: wait for line k (line k+1 may be in flight: vmcnt <= 8), read lines k-1, k,
    // refill the slot of line k-1 with line k+2 (if any), hash blocks 2k-2, 2k-1
    auto full_step = [&](uint32_t k, const uint32_t (&ad)[32]) {
        brb_dma::wait_vmcnt<8>();
        read_window(ad);
        if (k + 2 <= K)
            issue((k + 2) % 3, false);
        __builtin_amdgcn_sched_barrier(0);
        Alg::compress(st, w0);
        Alg::compress(st, w1);
        __builtin_amdgcn_sched_barrier(0);
    };
    uint32_t k = 1;
    for (; k + 3 <= K; k += 3) {
        full_step(k, t0);                                      // (k-1) % 3 == 0
        full_step(k + 1, t1);
        full_step(k + 2, t2);
    }
    for (; k < K; k++) {                                       // at most two: uniform branches
        const uint32_t r = (k - 1) % 3;
        if (r == 0)
            full_step(k, t0);
        else if (r == 1)
            full_step(k, t1);
        else
            full_step(k, t2);
    }
    // iteration K: lines K-1, K; nothing left to issue
    brb_dma::wait_vmcnt<0>();
    {
        const uint32_t r = (K - 1) % 3;
        if (r == 0)
            read_window(t0);
        else if (r == 1)
            read_window(t1);
        else
            read_window(t2);
    }
    if (2 * K - 2 < nfull)
        Alg::compress(st, w0);
    if (2 * K - 1 < nfull)
        Alg::compress(st, w1);
    brb_digest::line_finish<Alg, OUT_ALIGNED, TAIL_HI>(st, w0, w1, tm, tp, t, rec_len, out, g * 64 + lane, n_rec);
}

}  // namespace brb_mb_l3r
