// line4_kernel.h -- experiment (round 6): the line digest kernel at FOUR waves per SIMD.
//
// digest_line.h stages 128-byte lines into a two-slot ring of 8 KiB slots, so a wave holds 16 KiB
// of LDS and a CU fits 8 waves (two per SIMD).  The MD5 mix issues at 4.02 cycles per instruction
// per SIMD with two waves and 3.72 with four, so this form stages 64-byte
// HALF-lines instead: a slot is 64 rows x 64 B = 4 KiB, a wave 8 KiB, 16 waves per CU.  Iteration
// b reads the 16-dword window of block b from half-lines b and b+1 (the record's dword shift
// sh = (address mod 64) / 4 < 16) and refills half-line b's slot with half-line b+2; one block per
// iteration, four DMAs of 1 KiB per half-line under one M0 write.  Everything else as digest_line.h:
// group-invariant tables built once per wave, per-workgroup tickets, the last iteration peeled, the
// slot parity chosen so that it reads slots 0, 1.
// Used by tools/mb/line_ab.hip only.
#pragma once

#include "digest_line.h"

namespace brb_mb_l4 {

template <class Alg, int WAVES, bool OUT_ALIGNED, bool ALL_L2 = false>
__global__ __launch_bounds__(64 * WAVES, 1) void digest_line4_kernel(const uint8_t *__restrict__ data,
                                                                    uint32_t rec_len, uint64_t n_rec,
                                                                    uint8_t *__restrict__ out)
{
    constexpr uint32_t SLOT = 4096;                            // 64 rows x one 64-byte half-line
    __shared__ __attribute__((aligned(16))) uint8_t ring[WAVES * 2 * SLOT];
    __shared__ uint32_t next_ticket;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t n_groups = (n_rec + 63) / 64;
    if (threadIdx.x == 0)
        next_ticket = WAVES;
    __syncthreads();
    auto take = [&]() -> uint64_t {
        uint32_t tk = 0;
        if (lane == 0)
            tk = __hip_atomic_fetch_add(&next_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        tk = __builtin_amdgcn_readfirstlane(tk);
        return uint64_t(blockIdx.x) + uint64_t(tk) * gridDim.x;
    };
    uint64_t g = uint64_t(blockIdx.x) + uint64_t(wv) * gridDim.x;
    if (g >= n_groups)
        return;
    const uint32_t my_off = wv * 2 * SLOT;                     // slot 1 = slot 0 + SLOT (bit 12 clear)
    const uint32_t lds0 = uint32_t(reinterpret_cast<uintptr_t>(ring)) + my_off;
    const uint32_t nfull = rec_len >> 6, t = rec_len & 63;
    const uint32_t nblk = nfull + (t ? 1 : 0);                 // >= 2 (rec_len > 64); half-lines 0 .. nblk
    const uint32_t P = (nblk + 1) & 1;                          // half-line j in slot (j + P) & 1
    const uint64_t dbase = reinterpret_cast<uint64_t>(data);
    const uint64_t end_line = (dbase + n_rec * rec_len + 63) & ~uint64_t(63);
    const uint64_t gbytes = uint64_t(rec_len) * 64;
    const uint32_t o0 = uint32_t(dbase) & 63;
    // 16-byte granule swizzle of a 64-byte row (on the DMA source; the reads use the same map)
    auto swz = [](uint32_t row) { return (row >> 1) & 3; };

    // DMA q (0..3), lane j: granule j & 3 of row 16 q + j / 4's half-line
    uint32_t vq[4];
    {
        const uint32_t r4 = lane >> 2;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t row = 16u * q + r4;
            const uint32_t x = o0 + row * rec_len;
            vq[q] = ((x & ~63u) | (16u * ((lane & 3) ^ swz(row)))) + (4096u - 1024u * q);
        }
    }
    brb_dma::v4i rs, rsn;
    auto desc = [&](uint64_t g, brb_dma::v4i &rs) {
        const uint64_t gbase = ((dbase + g * gbytes) & ~uint64_t(63)) - 4096;
        const uint64_t gleft = end_line - gbase;
        rs.x = __builtin_amdgcn_readfirstlane(int(uint32_t(gbase)));
        rs.y = __builtin_amdgcn_readfirstlane(int(uint32_t(gbase >> 32) & 0xFFFF));
        rs.z = __builtin_amdgcn_readfirstlane(int(gleft > 0x7FFFFFFFull ? 0x7FFFFFFFu : uint32_t(gleft)));
        rs.w = 0x00020000;
    };
    uint32_t so = 0, son = 0;
    auto issue = [&](const brb_dma::v4i &rs, uint32_t &so, uint32_t slot, bool keep_l2 = false) {
        const uint32_t m = lds0 + slot * SLOT;
        uint32_t keep;
#define BRB_L4_DMA4(POL)                                                                        \
    asm volatile("s_mov_b32 %0, m0\n\t"                                                          \
                 "s_mov_b32 m0, %6\n\t"                                                          \
                 "s_nop 0\n\t"                                                                   \
                 "buffer_load_dwordx4 %1, %5, %7 offen " POL "lds\n\t"                          \
                 "buffer_load_dwordx4 %2, %5, %7 offen offset:1024 " POL "lds\n\t"              \
                 "buffer_load_dwordx4 %3, %5, %7 offen offset:2048 " POL "lds\n\t"              \
                 "buffer_load_dwordx4 %4, %5, %7 offen offset:3072 " POL "lds\n\t"              \
                 "s_mov_b32 m0, %0"                                                               \
                 : "=&s"(keep)                                                                    \
                 : "v"(vq[0]), "v"(vq[1]), "v"(vq[2]), "v"(vq[3]), "s"(rs), "s"(m), "s"(so)      \
                 : "memory")
        if (!keep_l2 && !ALL_L2)
            BRB_L4_DMA4("nt ");
        else
            BRB_L4_DMA4("");
#undef BRB_L4_DMA4
        so += 64;
    };

    uint32_t ae[16], ao[16];
    uint32_t w[16];
    auto read_window = [&](const uint32_t (&ad)[16]) {
#pragma unroll
        for (int i = 0; i < 16; i++)
            w[i] = *reinterpret_cast<const uint32_t *>(ring + ad[i]);
        __builtin_amdgcn_s_waitcnt(0xC07F);
    };

    desc(g, rs);
    issue(rs, so, P, true);
    issue(rs, so, P ^ 1, true);
    __builtin_amdgcn_sched_barrier(0);
    uint64_t gn = take();
    {
        const uint32_t sh4 = (o0 + lane * rec_len) & 63;       // 4 x the record's dword shift (< 64)
        const uint32_t fr = my_off + lane * 64;
        const uint32_t sz = swz(lane) << 4;
#pragma unroll
        for (uint32_t i = 0; i < 16; i++) {
            const uint32_t q4 = sh4 + 4 * i;                   // < 128: half-line b (< 64) or b+1
            ae[i] = (fr | (((q4 & 60u) ^ sz))) | ((q4 & 64u) << 6);   // SLOT = 64 << 6
            ao[i] = ae[i] ^ SLOT;
            asm volatile("" : "+v"(ae[i]), "+v"(ao[i]));
        }
    }
    uint32_t tm[16], tp[16];
    brb_digest::tail_masks(t, tm, tp);
    auto full_step = [&](typename Alg::State &st, const uint32_t (&ad)[16], uint32_t refill_slot) {
        brb_dma::wait_vmcnt<0>();
        read_window(ad);
        issue(rs, so, refill_slot);
        __builtin_amdgcn_sched_barrier(0);
        Alg::compress(st, w);
        __builtin_amdgcn_sched_barrier(0);
    };
    for (;;) {
        typename Alg::State st = Alg::iv();
        uint32_t b = 0;
        if (P) {                                               // nblk even: iteration 0 is odd-slotted
            full_step(st, ao, 1);
            b = 1;
        }
        for (; b + 2 <= nblk - 1; b += 2) {
            full_step(st, ae, 0);
            full_step(st, ao, 1);
        }
        {   // iteration nblk - 1: half-lines nblk-1, nblk in slots 0, 1
            brb_dma::wait_vmcnt<0>();
            read_window(ae);
            if (gn < n_groups) {
                desc(gn, rsn);
                son = 0;
                issue(rsn, son, P, true);
                issue(rsn, son, P ^ 1, true);
            }
            if (t == 0) {
                Alg::compress(st, w);
                Alg::pad_only(st, rec_len);
            } else {
#pragma unroll
                for (int i = 0; i < 16; i++)
                    w[i] = (w[i] & tm[i]) | tp[i];
                Alg::finish(st, w, t, rec_len);
            }
            const uint64_t r = g * 64 + lane;
            if (r < n_rec)
                Alg::template store<OUT_ALIGNED>(out, r, st);
        }
        g = gn;
        if (g >= n_groups)
            break;
        gn = take();
        rs = rsn;
        so = son;
    }
}

}  // namespace brb_mb_l4
