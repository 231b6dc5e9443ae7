// digest_line_pair.h -- the fixed-stride line-staged digest (digest_line.h) as wave pairs, for
// launches with one group of 64 records per SIMD (cfg2: 65 536 x 1500 B = 1 024 groups).
//
// digest_line_kernel runs one wave per SIMD there.  That wave issues the DMA of every line, waits for
// it, reads the shifted window with 32 ds_read_b32 per two blocks and compresses; a lone wave pays
// each LDS and memory round trip in full and issues at the lone-wave rate (the
// compression with its window reads takes ~18 us of the ~21 us launch).  Here a group belongs to a
// pair of waves on one SIMD (waves p and p + NP of the workgroup):
//   stager   stages the records' lines by LDS-DMA into a three-slot ring (two lines in flight),
//            reads each two-block window with the per-lane shift (address tables, as
//            digest_line_kernel) and drops the blocks into a three-block ring in a lane-contiguous
//            layout: 16-byte granule q of lane l's block at ((slot * 4 + q) * 64 + l) * 16;
//   hasher   reads each block with four ds_read_b128 at the same offset for every lane (the next
//            block's reads issued before the current block is compressed), compresses, pads the
//            tail (the tail block's bytes past the record masked, as line_finish) and stores.
// Two LDS counts per pair order the hand-offs: blocks staged (stager -> hasher, release after the
// ring writes) and blocks taken (hasher -> stager); both run over the pair's whole group sequence,
// and every wait is bounded (pair_sync.h).
#pragma once

#include <type_traits>

#include "digest_line.h"
#include "pair_sync.h"
#include "test_options.h"

namespace brb_digest {

template <class Alg, int NP, bool OUT_ALIGNED>
__global__ __launch_bounds__(128 * NP) void digest_line_pair_kernel(const uint8_t *__restrict__ data, uint32_t rec_len,
                                                                    uint64_t n_rec, uint8_t *__restrict__ out)
{
    using brb_line::pc_load;
    using brb_line::pc_publish;
    constexpr uint32_t SLOT = 8192;                            // 64 rows x one 128-byte line
    constexpr uint32_t NS = 3;                                 // line slots per pair
    constexpr uint32_t RB = 3;                                 // ring blocks per pair (4 KiB each)
    __shared__ __attribute__((aligned(16))) uint8_t lines[NP * NS * SLOT];
    __shared__ __attribute__((aligned(16))) uint8_t blocks[NP * RB * 4096];
    __shared__ uint32_t cnt[NP][2];                            // blocks staged, blocks taken
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t pr = wv % NP;
    if (threadIdx.x < 2 * NP)
        (&cnt[0][0])[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t n_groups = (n_rec + 63) / 64;
    const uint64_t gstride = uint64_t(gridDim.x) * NP;
    const uint32_t nfull = rec_len >> 6, t = rec_len & 63;
    const uint32_t nblk = nfull + (t ? 1 : 0);
    const uint32_t K = (nblk + 1) >> 1;                        // two-block windows per group; K + 1 lines
    const uint32_t nb = 2 * K;                                 // blocks handed over per group
    uint8_t *const ring = blocks + pr * RB * 4096;
    const uint32_t ring0 = uint32_t(reinterpret_cast<uintptr_t>(ring));

    if (wv >= NP) {
        // ---------------- hasher ----------------
        uint32_t tm[16], tp[16];
        tail_masks(t, tm, tp);
        uint32_t taken = 0;                                    // blocks taken over all groups so far
        auto ready = [&](uint32_t b) { return brb_line::pc_wait_ge(&cnt[pr][0], b); };
        auto read_block = [&](uint32_t b, uint32_t (&w)[16]) {
            const uint32_t base = ring0 + (b % RB) * 4096 + lane * 16;
            typedef uint32_t v4u __attribute__((ext_vector_type(4)));
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const v4u v = *reinterpret_cast<const __attribute__((address_space(3))) v4u *>(base + q * 1024);
                w[4 * q + 0] = v.x;
                w[4 * q + 1] = v.y;
                w[4 * q + 2] = v.z;
                w[4 * q + 3] = v.w;
            }
        };
        for (uint64_t g = uint64_t(blockIdx.x) * NP + pr; g < n_groups; g += gstride) {
            typename Alg::State st = Alg::iv();
            uint32_t w[16], tail[16];
#pragma unroll
            for (int i = 0; i < 16; i++)
                tail[i] = 0;
            if (!ready(taken + 1))
                return;                                        // a protocol fault: no digests, no hang
            read_block(taken, w);
            __builtin_amdgcn_s_waitcnt(0xC07F);
            pc_publish(&cnt[pr][1], ++taken);
            for (uint32_t b = 0; b < nb; b++) {
                uint32_t wn[16];
                const bool more = b + 1 < nb;
                if (more) {                                    // the next block's reads fly during this one
                    if (!ready(taken + 1))
                        return;
                    read_block(taken, wn);
                }
                if (b < nfull)
                    Alg::compress(st, w);
                else if (b == nfull) {
#pragma unroll
                    for (int i = 0; i < 16; i++)
                        tail[i] = w[i];
                }
                if (more) {
                    __builtin_amdgcn_s_waitcnt(0xC07F);
                    pc_publish(&cnt[pr][1], ++taken);
#pragma unroll
                    for (int i = 0; i < 16; i++)
                        w[i] = wn[i];
                }
            }
            if (t == 0) {
                Alg::pad_only(st, rec_len);                    // the padding block is a constant
            } else {
#pragma unroll
                for (int i = 0; i < 16; i++)
                    tail[i] = (tail[i] & tm[i]) | tp[i];
                Alg::finish(st, tail, t, rec_len);
            }
            const uint64_t r = g * 64 + lane;
            if (r < n_rec)
                Alg::template store<OUT_ALIGNED>(out, r, st);
        }
        return;
    }

    // ---------------- stager ----------------
    const uint32_t my_off = pr * NS * SLOT;
    const uint32_t lds0 = uint32_t(reinterpret_cast<uintptr_t>(lines)) + my_off;
    const uint64_t dbase = reinterpret_cast<uint64_t>(data);
    const uint64_t end_line = (dbase + n_rec * rec_len + 127) & ~uint64_t(127);
    auto swz = [](uint32_t row) { return (row >> 1) & 7; };
    uint32_t vq[8];
    brb_dma::v4i rs;
    uint32_t so = 0;
    // as digest_line_kernel::dma_setup: DMA q stages row 8q + lane / 8 of the group's next line
    auto dma_setup = [&](uint64_t g) {
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
        so = 0;
    };
    auto issue = [&](uint32_t slot, bool nt) {                 // the group's next line -> slot
        const uint32_t m = lds0 + slot * SLOT;
        uint32_t keep;
#define BRB_PAIR_DMA8(POL)                                                                      \
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
                   "v"(vq[7]), "s"(rs), "s"(m), "s"(m + 4096u), "s"(so)                           \
                 : "memory")
        if (nt)
            BRB_PAIR_DMA8("nt ");
        else
            BRB_PAIR_DMA8("");
#undef BRB_PAIR_DMA8
        so += 128;
    };
    // window dword i of this lane -> row-relative LDS offset; tA: lines k-1, k in consecutive slots
    // (s, s + 1), tW: in slots (2, 0) (the ring's wrap); both plus the first slot's base
    uint32_t tA[32], tW[32];
    auto win_setup = [&](uint64_t g) {
        const uint64_t r0 = g * 64;
        const uint32_t last = uint32_t(n_rec - r0 < 64 ? n_rec - r0 - 1 : 63);
        const uint32_t o0 = uint32_t(dbase + r0 * rec_len) & 127;
        const uint32_t rr = lane < last ? lane : last;
        const uint32_t sh4 = (o0 + rr * rec_len) & 127;
        const uint32_t fr = lane * 128 | (swz(lane) << 4);
#pragma unroll
        for (uint32_t i = 0; i < 32; i++) {
            const uint32_t q4 = sh4 + 4 * i;                   // < 256
            const uint32_t rp = ((q4 & 124u) ^ fr) + lds0;
            tA[i] = rp + (q4 & 128u ? SLOT : 0u);
            tW[i] = rp + (q4 & 128u ? 0u : 2 * SLOT);          // first line in slot 2, second in slot 0
            asm volatile("" : "+v"(tA[i]), "+v"(tW[i]));
        }
    };
    // the window (lines k-1, k) with line k-1 in slot SA: the slot's base is an immediate offset
    auto read_win = [&](auto SA, uint32_t (&w0)[16], uint32_t (&w1)[16]) {
        constexpr uint32_t sa_c = decltype(SA)::value;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const uint32_t a0 = sa_c == 2 ? tW[i] : tA[i] + sa_c * SLOT;
            const uint32_t a1 = sa_c == 2 ? tW[16 + i] : tA[16 + i] + sa_c * SLOT;
            w0[i] = *reinterpret_cast<const __attribute__((address_space(3))) uint32_t *>(a0);
            w1[i] = *reinterpret_cast<const __attribute__((address_space(3))) uint32_t *>(a1);
        }
    };
    uint32_t staged = 0;                                       // blocks staged over all groups so far
    auto put_block = [&](const uint32_t (&w)[16]) -> bool {    // into ring block `staged`
        if (!brb_line::pc_wait_ge(&cnt[pr][1], staged + 1 > RB ? staged + 1 - RB : 0u))
            return false;
        const uint32_t base = ring0 + (staged % RB) * 4096 + lane * 16;
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int q = 0; q < 4; q++) {
            v4u v;
            v.x = w[4 * q + 0];
            v.y = w[4 * q + 1];
            v.z = w[4 * q + 2];
            v.w = w[4 * q + 3];
            *reinterpret_cast<__attribute__((address_space(3))) v4u *>(base + q * 1024) = v;
        }
        pc_publish(&cnt[pr][0], ++staged);
        return true;
    };
    for (uint64_t g = uint64_t(blockIdx.x) * NP + pr; g < n_groups; g += gstride) {
        dma_setup(g);
        issue(0, false);                                       // lines 0, 1 keep the L2 policy (the
        issue(1, false);                                       // previous record's tail lines), as in
        if (K >= 2)                                            // digest_line_kernel
            issue(2, true);
        win_setup(g);
        for (uint32_t k = 1; k <= K; k++) {
            const uint32_t sa = (k - 1) % NS;                  // line k-1's slot
            // line k landed; line k + 1 (issued at k - 1) may fly
            if (k + 1 <= K)
                brb_dma::wait_vmcnt<8>();
            else
                brb_dma::wait_vmcnt<0>();
            uint32_t w0[16], w1[16];
            if (sa == 0)
                read_win(std::integral_constant<uint32_t, 0>{}, w0, w1);
            else if (sa == 1)
                read_win(std::integral_constant<uint32_t, 1>{}, w0, w1);
            else
                read_win(std::integral_constant<uint32_t, 2>{}, w0, w1);
            __builtin_amdgcn_s_waitcnt(0xC07F);                // the window is in; line k-1's slot is free
            if (k + 2 <= K)
                issue(sa, true);                               // line k + 2 into line k - 1's slot
            if (!put_block(w0) || !put_block(w1)) {
                brb_dma::wait_vmcnt<0>();
                return;
            }
        }
        brb_dma::wait_vmcnt<0>();
    }
}

// One 8-wave workgroup per CU (128 KiB of LDS), persistent, groups handed out by tickets (DYN), DMA
// with the non-temporal policy (every line is read exactly once).  Measured with
// tools/mb/md5_ab.hip, MD5, medians of 20-launch bursts:
//   1 Mi x 1500 B: 316 us static 4-wave workgroups -> 300 us (read floor of the same bytes: 261 us nt)
//   cfg2 65 536 x 1500 B: 25.3 us (record-relative 128-byte stages) -> 24.9 us
// Launches with at most one group per SIMD (cfg2) take the wave pairs above (test option
// "line_pair" 0 keeps the single-wave kernel there); larger ones keep two compressing waves per SIMD.
template <class Alg>
hipError_t launch_fixed_line(const uint8_t *data, uint32_t rec_len, uint64_t n_rec, uint8_t *out, bool out_al,
                             hipStream_t s)
{
    constexpr int W = 8;
    const uint64_t groups = (n_rec + 63) / 64;
    if (groups <= 4 * uint64_t(device_cu_count()) && brb_opt::get(brb_opt::kLinePair) != 0) {
        constexpr int NP = 4;                              // 4 pairs, 144 KiB of LDS: one workgroup per CU
        const uint64_t wgs = (groups + NP - 1) / NP;
        const unsigned grid = unsigned(wgs < device_cu_count() ? wgs : device_cu_count());
        if (out_al)
            digest_line_pair_kernel<Alg, NP, true><<<grid, 128 * NP, 0, s>>>(data, rec_len, n_rec, out);
        else
            digest_line_pair_kernel<Alg, NP, false><<<grid, 128 * NP, 0, s>>>(data, rec_len, n_rec, out);
        return hipGetLastError();
    }
    const unsigned g = unsigned(groups < device_cu_count() ? groups : device_cu_count());
    if (out_al)
        digest_line_kernel<Alg, W, true, true, true><<<g, 64 * W, 0, s>>>(data, rec_len, n_rec, out);
    else
        digest_line_kernel<Alg, W, false, true, true><<<g, 64 * W, 0, s>>>(data, rec_len, n_rec, out);
    return hipGetLastError();
}

}  // namespace brb_digest
