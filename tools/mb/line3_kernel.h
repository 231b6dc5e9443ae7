// line3_kernel.h (tools/mb; measured slower, not in the library) -- the line-aligned digest kernel of digest_line.h with a THREE-slot LDS ring and
// the window reads software-pipelined behind the compressions.  For batches of at most one group
// of 64 records per SIMD (cfg2: 65 536 records = 1 024 groups = one wave per SIMD), where no second
// wave hides a wave's own waits.
//
// Why (round 3, cfg2 PMC, profiles/r03_pmc_cfg2_md5.txt): a wave of digest_line_kernel spends ~22 %
// of its cycles in s_waitcnt.  Each of its iterations waits for line k, reads the 32-dword window
// (lines k-1, k) and waits for those reads before any VALU of the two compressions can issue, and
// line k+1 -- issued into the slot of line k-1 only once that window is in VGPRs -- has one
// iteration to arrive.  Here:
//   * line k+2 goes into the slot of line k-1 at the start of iteration k (three slots: lines k-1,
//     k, k+1 resident or in flight), so a line has two iterations (~2.8 us) to land;
//   * window k+1 is read while block 2k-1 of window k is compressed (its reads land during the
//     ~1 400 cycles of that compression), so the ds_read latency is off the issue path.
// The cost is LDS: 24 KiB per wave, 4 waves per CU (one per SIMD).
//
// Slot of line j = j mod 3.  Window k (lines k-1, k) at position s = (k-1) mod 3 reads slots
// (s, s+1 mod 3): tables T0 (slots 0, 1; at LDS offset +0 for s = 0 and +SLOT for s = 1, the
// immediate offset of ds_read_b32) and T2 (slots 2, 0).
//
// Record r's digest = BRB_MD5Init/Update/Final (md5.c:38-168) or BrbSha1_Do (sha1.c:203-216) of
// data[r * rec_len .. (r + 1) * rec_len), exactly as digest_line_kernel.
#pragma once

#include "digest_line.h"
#include "line_r05_kernel.h"   // round 5's line_finish / tail_masks signatures

namespace brb_digest {

template <class Alg, int WAVES, bool OUT_ALIGNED, bool EARLY>
__global__ __launch_bounds__(64 * WAVES, 1) void digest_line3_kernel(const uint8_t *__restrict__ data,
                                                                      uint32_t rec_len, uint64_t n_rec,
                                                                      uint8_t *__restrict__ out)
{
    constexpr uint32_t SLOT = 8192;                            // 64 rows x one 128-byte line
    __shared__ __attribute__((aligned(16))) uint8_t ring[WAVES * 3 * SLOT];
    __shared__ uint32_t next_ticket;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t n_groups = (n_rec + 63) / 64;
    if (threadIdx.x == 0)
        next_ticket = WAVES;                                   // tickets 0 .. WAVES-1: one per wave
    __syncthreads();
    auto take = [&]() -> uint64_t {                            // the next group of this workgroup
        uint32_t tk = 0;
        if (lane == 0)
            tk = __hip_atomic_fetch_add(&next_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        tk = __builtin_amdgcn_readfirstlane(tk);
        return uint64_t(blockIdx.x) + uint64_t(tk) * gridDim.x;
    };
    uint64_t g = uint64_t(blockIdx.x) + uint64_t(wv) * gridDim.x;
    if (g >= n_groups)
        return;
    const uint32_t my_off = wv * 3 * SLOT;
    const uint32_t lds0 = uint32_t(reinterpret_cast<uintptr_t>(ring)) + my_off;
    const uint32_t nfull = rec_len >> 6, t = rec_len & 63;
    const uint32_t nblk = nfull + (t ? 1 : 0);
    const uint32_t K = (nblk + 1) >> 1;                        // 2-block iterations per group; K + 1 lines
    const bool line2 = K >= 2;                                 // a group has a line 2
    const uint64_t dbase = reinterpret_cast<uint64_t>(data);
    const uint64_t end_line = (dbase + n_rec * rec_len + 127) & ~uint64_t(127);
    auto swz = [](uint32_t row) { return (row >> 1) & 7; };

    // ---- issue side (as digest_line_kernel: descriptor 4 KiB below the group's first line, line j
    // at soffset 128 j, one M0 write per four DMAs)
    uint32_t vq[8], vqn[8];
    brb_dma::v4i rs, rsn;
    auto dma_setup = [&](uint64_t g, uint32_t (&vq)[8], brb_dma::v4i &rs) {
        const uint64_t r0 = g * 64;
        const uint32_t last = uint32_t(n_rec - r0 < 64 ? n_rec - r0 - 1 : 63);
        const uint64_t a0 = dbase + r0 * rec_len;
        const uint64_t gbase = (a0 & ~uint64_t(127)) - 4096;
        const uint64_t gleft = end_line - gbase;
        rs.x = __builtin_amdgcn_readfirstlane(int(uint32_t(gbase)));
        rs.y = __builtin_amdgcn_readfirstlane(int(uint32_t(gbase >> 32) & 0xFFFF));
        rs.z = __builtin_amdgcn_readfirstlane(int(gleft > 0x7FFFFFFFull ? 0x7FFFFFFFu : uint32_t(gleft)));
        rs.w = 0x00020000;
        const uint32_t o0 = uint32_t(a0) & 127;
        const uint32_t l3 = lane >> 3;
        const uint32_t base = o0 + l3 * rec_len, cap = o0 + last * rec_len;
        const uint32_t g0 = 16u * ((lane & 7) ^ (l3 >> 1));
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const uint32_t x = base + 8u * q * rec_len;
            vq[q] = (((x < cap ? x : cap) & ~127u) | (q & 1 ? g0 ^ 64u : g0)) + (4096u - 1024u * (q & 3));
        }
    };
    uint32_t so = 0, son = 0;
    // lines 0 and 1 of a group through the L2 with the normal policy (the neighbour record's
    // last line is the same memory line), the others non-temporal
    auto issue = [&](const uint32_t (&vq)[8], const brb_dma::v4i &rs, uint32_t &so, uint32_t slot, bool keep_l2) {
        const uint32_t m = lds0 + slot * SLOT;
        uint32_t keep;
        const uint32_t sso = __builtin_amdgcn_readfirstlane(so);   // an SGPR, never a literal soffset
#define BRB_LINE3_DMA8(POL)                                                                     \
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
                   "v"(vq[7]), "s"(rs), "s"(m), "s"(m + 4096u), "s"(sso)                          \
                 : "memory")
        if (keep_l2)
            BRB_LINE3_DMA8("");
        else
            BRB_LINE3_DMA8("nt ");
#undef BRB_LINE3_DMA8
        so += 128;
    };
    // lines 0, 1 (and 2) of a group into slots 0, 1 (and 2)
    auto issue_first = [&](const uint32_t (&vq)[8], const brb_dma::v4i &rs, uint32_t &so) {
        issue(vq, rs, so, 0, true);
        issue(vq, rs, so, 1, true);
        if (line2)
            issue(vq, rs, so, 2, false);
    };
    // lines 0 and 1 of a group landed (line 2 may still be in flight)
    auto wait_first = [&]() {
        if (line2)
            brb_dma::wait_vmcnt<8>();
        else
            brb_dma::wait_vmcnt<0>();
    };

    // ---- read side: window dword i -> LDS offset; T0: line k-1 in slot 0, line k in slot 1;
    // T2: line k-1 in slot 2, line k in slot 0
    uint32_t t0[32], t2[32];
    auto win_setup = [&](uint64_t g) {
        const uint64_t r0 = g * 64;
        const uint32_t last = uint32_t(n_rec - r0 < 64 ? n_rec - r0 - 1 : 63);
        const uint32_t o0 = uint32_t(dbase + r0 * rec_len) & 127;
        const uint32_t rr = lane < last ? lane : last;
        const uint32_t sh4 = (o0 + rr * rec_len) & 127;        // 4 x the record's dword shift
        const uint32_t fr = (my_off + lane * 128) | (swz(lane) << 4);
#pragma unroll
        for (uint32_t i = 0; i < 32; i++) {
            const uint32_t q4 = sh4 + 4 * i;                   // < 256
            const uint32_t a = (q4 & 124u) ^ fr;
            t0[i] = a + ((q4 & 128u) << 6);                    // SLOT = 128 << 6
            t2[i] = a + (q4 & 128u ? 0u : 2 * SLOT);
            asm volatile("" : "+v"(t0[i]), "+v"(t2[i]));       // keep both tables
        }
    };
    // window dwords at table + a compile-time offset (ds_read_b32's immediate)
    auto read_window = [&](const uint32_t (&ad)[32], uint32_t imm, uint32_t (&n0)[16], uint32_t (&n1)[16]) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            n0[i] = *reinterpret_cast<const uint32_t *>(ring + imm + ad[i]);
            n1[i] = *reinterpret_cast<const uint32_t *>(ring + imm + ad[16 + i]);
        }
    };
    auto wait_reads = []() { __builtin_amdgcn_s_waitcnt(0xC07F); };   // lgkmcnt(0)

    uint32_t w0[16], w1[16];                                   // window k
    uint32_t n0[16], n1[16];                                   // window k+1, in flight
    dma_setup(g, vq, rs);
    issue_first(vq, rs, so);
    __builtin_amdgcn_sched_barrier(0);
    uint64_t gn = take();
    win_setup(g);
    uint32_t tm[16], tp[16];
    brb_mb_r05::tail_masks(t, tm, tp);
    wait_first();
    read_window(t0, 0, w0, w1);
    wait_reads();

    // Iteration k < K at position S = (k-1) mod 3: line k+2 (if the group has it) into slot S,
    // block 2k-2, wait for line k+1, read window k+1 (position S+1), block 2k-1, reads landed.
    auto body = [&](typename Alg::State &st, uint32_t k, auto S_) {
        constexpr uint32_t S = decltype(S_)::value;
        const bool more = k + 2 <= K;                          // uniform
        if (more)
            issue(vq, rs, so, S, false);
        __builtin_amdgcn_sched_barrier(0);
        Alg::compress(st, w0);
        if constexpr (!EARLY) {
            __builtin_amdgcn_sched_barrier(0);
            Alg::compress(st, w1);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (more)
            brb_dma::wait_vmcnt<8>();
        else
            brb_dma::wait_vmcnt<0>();
        if constexpr (S == 0)
            read_window(t0, SLOT, n0, n1);                     // window k+1 at position 1
        else if constexpr (S == 1)
            read_window(t2, 0, n0, n1);                        // position 2
        else
            read_window(t0, 0, n0, n1);                        // position 0
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (EARLY) {
            Alg::compress(st, w1);
            __builtin_amdgcn_sched_barrier(0);
        }
        wait_reads();
#pragma unroll
        for (int i = 0; i < 16; i++) {
            w0[i] = n0[i];
            w1[i] = n1[i];
        }
    };
    using P0 = std::integral_constant<uint32_t, 0>;
    using P1 = std::integral_constant<uint32_t, 1>;
    using P2 = std::integral_constant<uint32_t, 2>;
    for (;;) {
        typename Alg::State st = Alg::iv();
        // iterations 1 .. K-1 (every one hashes two whole blocks: 2k - 1 <= 2K - 3 < nfull)
        for (uint32_t k = 1; k < K;) {
            body(st, k, P0{});
            if (++k >= K)
                break;
            body(st, k, P1{});
            if (++k >= K)
                break;
            body(st, k, P2{});
            ++k;
        }
        // iteration K: window K is in VGPRs, every slot is free -> the next group's first lines
        const bool next = gn < n_groups;
        if (next) {
            dma_setup(gn, vqn, rsn);
            son = 0;
            issue_first(vqn, rsn, son);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (2 * K - 2 < nfull)
            Alg::compress(st, w0);
        uint32_t tw0[16], tw1[16];                             // this group's last window
#pragma unroll
        for (int i = 0; i < 16; i++) {
            tw0[i] = w0[i];
            tw1[i] = w1[i];
        }
        if (next) {
            win_setup(gn);
            wait_first();
            read_window(t0, 0, w0, w1);                        // the next group's window 1
        }
        __builtin_amdgcn_sched_barrier(0);
        if (2 * K - 1 < nfull)
            Alg::compress(st, tw1);
        brb_mb_r05::line_finish<Alg, OUT_ALIGNED>(st, tw0, tw1, tm, tp, t, nfull, K, rec_len, out, g * 64 + lane, n_rec);
        if (!next)
            break;
        wait_reads();
        g = gn;
        gn = take();
#pragma unroll
        for (int q = 0; q < 8; q++)
            vq[q] = vqn[q];
        rs = rsn;
        so = son;
    }
}

// One 4-wave workgroup per CU (96 KiB of LDS: one wave per SIMD), persistent, tickets.
template <class Alg>
hipError_t launch_fixed_line3(const uint8_t *data, uint32_t rec_len, uint64_t n_rec, uint8_t *out, bool out_al,
                              hipStream_t s, bool early)
{
    constexpr int W = 4;
    const uint64_t groups = (n_rec + 63) / 64;
    const uint64_t wgs = (groups + W - 1) / W;
    const unsigned g = unsigned(wgs < device_cu_count() ? wgs : device_cu_count());
    if (early) {
        if (out_al)
            digest_line3_kernel<Alg, W, true, true><<<g, 64 * W, 0, s>>>(data, rec_len, n_rec, out);
        else
            digest_line3_kernel<Alg, W, false, true><<<g, 64 * W, 0, s>>>(data, rec_len, n_rec, out);
    } else {
        if (out_al)
            digest_line3_kernel<Alg, W, true, false><<<g, 64 * W, 0, s>>>(data, rec_len, n_rec, out);
        else
            digest_line3_kernel<Alg, W, false, false><<<g, 64 * W, 0, s>>>(data, rec_len, n_rec, out);
    }
    return hipGetLastError();
}

}  // namespace brb_digest
