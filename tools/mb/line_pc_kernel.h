// line_pc_kernel.h (tools/mb; measured slower, not in the library) -- the line-aligned digest kernel of digest_line.h with the LDS-DMA issued by a
// separate PRODUCER wave: each workgroup holds C consumer waves (one group of 64 records each at a
// time, as digest_line_kernel's waves) and one producer wave that stages every consumer's lines.
//
// Why (round 3, cfg2, tools/mb/line_probe.hip, profiles/r03/line_probe_cfg2*.txt): a lone wave of
// digest_line_kernel issues 16.6 us of instructions per 1 500-byte record when it also issues its
// own DMA, 15.3 us when the DMA is compiled out -- the 104 `buffer_load ... lds` per record cost the
// compressing wave ~1.2 us of issue beyond their instruction count.  A producer wave on the same CU
// takes that off the consumers' instruction streams (the SIMD issues its VMEM beside their VALU),
// keeps up to NS lines per consumer in flight, and starts every consumer's first lines while the
// consumers set up.
//
// Protocol (all in LDS, per consumer c; line numbers run on across c's groups):
//   ready[c] = number of c's lines landed (written by the producer after s_waitcnt vmcnt);
//   freed[c] = number of c's lines whose slot may be refilled (written by the consumer after its
//              window reads landed: window k reads lines k-1 and k, so afterwards lines < k are free).
// Line n of consumer c lives in slot n mod NS of c's ring.  The producer issues line n once
// freed[c] >= n - NS + 1, one line per consumer per round, and marks a round ready when the next
// round is in flight.  Every wait is a bounded poll (s_sleep between reads), so a protocol error
// ends the kernel with wrong digests (which the parity tests catch), never with a hang.
//
// Groups are assigned statically: consumer c of workgroup b takes groups b + G c, b + G (c + C),
// ... (G = gridDim.x), which the producer walks in the same order.
//
// Record r's digest = BRB_MD5Init/Update/Final (md5.c:38-168) or BrbSha1_Do (sha1.c:203-216) of
// data[r * rec_len .. (r + 1) * rec_len), exactly as digest_line_kernel.
#pragma once

#include "digest_line.h"
#include "line_r05_kernel.h"   // round 5's line_finish / tail_masks signatures

namespace brb_digest {

constexpr uint32_t kPcPollCap = 1u << 22;     // ~4 M polls of >= 64 cycles: seconds, never reached

template <class Alg, int C, int NS, bool OUT_ALIGNED>
__global__ __launch_bounds__(64 * (C + 1), 1) void digest_line_pc_kernel(const uint8_t *__restrict__ data,
                                                                          uint32_t rec_len, uint64_t n_rec,
                                                                          uint8_t *__restrict__ out)
{
    constexpr uint32_t SLOT = 8192;                            // 64 rows x one 128-byte line
    static_assert(NS >= 2 && NS <= 4, "ring of 2..4 lines");
    __shared__ __attribute__((aligned(16))) uint8_t ring[C * NS * SLOT];
    __shared__ uint32_t ready[C], freed[C], fifo[8];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t n_groups = (n_rec + 63) / 64;
    const uint64_t G = gridDim.x;
    if (threadIdx.x < C) {
        ready[threadIdx.x] = 0;
        freed[threadIdx.x] = 0;
    }
    __syncthreads();
    const uint32_t nfull = rec_len >> 6, t = rec_len & 63;
    const uint32_t nblk = nfull + (t ? 1 : 0);
    const uint32_t K = (nblk + 1) >> 1;                        // 2-block iterations per group; K + 1 lines
    const uint64_t dbase = reinterpret_cast<uint64_t>(data);
    const uint32_t ring0 = uint32_t(reinterpret_cast<uintptr_t>(ring));
    auto lds_load = [](const uint32_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
    auto lds_store = [](uint32_t *p, uint32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };

    if (wv == C) {
        // ================= producer =================
        const uint64_t end_line = (dbase + n_rec * rec_len + 127) & ~uint64_t(127);
        struct Feed {
            uint32_t vq[8];
            brb_dma::v4i rs;
        };
        // descriptor and DMA offsets of group g (as digest_line_kernel's dma_setup)
        auto dma_setup = [&](uint64_t g, Feed &f) {
            const uint64_t r0 = g * 64;
            const uint32_t last = uint32_t(n_rec - r0 < 64 ? n_rec - r0 - 1 : 63);
            const uint64_t a0 = dbase + r0 * rec_len;
            const uint64_t gbase = (a0 & ~uint64_t(127)) - 4096;
            const uint64_t gleft = end_line - gbase;
            f.rs.x = __builtin_amdgcn_readfirstlane(int(uint32_t(gbase)));
            f.rs.y = __builtin_amdgcn_readfirstlane(int(uint32_t(gbase >> 32) & 0xFFFF));
            f.rs.z = __builtin_amdgcn_readfirstlane(int(gleft > 0x7FFFFFFFull ? 0x7FFFFFFFu : uint32_t(gleft)));
            f.rs.w = 0x00020000;
            const uint32_t o0 = uint32_t(a0) & 127;
            const uint32_t l3 = lane >> 3;
            const uint32_t base = o0 + l3 * rec_len, cap = o0 + last * rec_len;
            const uint32_t g0 = 16u * ((lane & 7) ^ (l3 >> 1));
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const uint32_t x = base + 8u * q * rec_len;
                f.vq[q] = (((x < cap ? x : cap) & ~127u) | (q & 1 ? g0 ^ 64u : g0)) + (4096u - 1024u * (q & 3));
            }
        };
        // line j of the group f into LDS byte address m (lines 0 and 1 keep the L2 policy)
        auto issue = [&](const Feed &f, uint32_t j, uint32_t m) {
            const uint32_t so = __builtin_amdgcn_readfirstlane(128u * j);
            brb_dma::v4i rs;                                   // in SGPRs whatever hipcc did with feed[]
            rs.x = __builtin_amdgcn_readfirstlane(f.rs.x);
            rs.y = __builtin_amdgcn_readfirstlane(f.rs.y);
            rs.z = __builtin_amdgcn_readfirstlane(f.rs.z);
            rs.w = __builtin_amdgcn_readfirstlane(f.rs.w);
            const uint32_t mm = __builtin_amdgcn_readfirstlane(m);
            uint32_t keep;
#define BRB_PC_DMA8(POL)                                                                        \
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
                 : "v"(f.vq[0]), "v"(f.vq[1]), "v"(f.vq[2]), "v"(f.vq[3]), "v"(f.vq[4]), "v"(f.vq[5]), \
                   "v"(f.vq[6]), "v"(f.vq[7]), "s"(rs), "s"(mm), "s"(mm + 4096u), "s"(so)          \
                 : "memory")
            if (j < 2)
                BRB_PC_DMA8("");
            else
                BRB_PC_DMA8("nt ");
#undef BRB_PC_DMA8
        };
        // Per consumer: the group being fed, its next line j, the virtual line number of the next
        // issue (each group starts at a multiple of NS, so a consumer's window k always reads the
        // slots (k-1, k) mod NS), what the ring's slots hold (used[s] = last line in slot s, + 1),
        // the issued and the published counts.
        Feed feed[C];
        uint64_t grp[C];
        uint32_t nxt[C], vline[C], used[C][NS];
#pragma unroll
        for (int c = 0; c < C; c++) {
            grp[c] = uint64_t(blockIdx.x) + G * c;
            nxt[c] = 0;
            vline[c] = 0;
#pragma unroll
            for (int q = 0; q < NS; q++)
                used[c][q] = 0;
            if (grp[c] < n_groups)
                dma_setup(grp[c], feed[c]);
        }
        // Issue whatever a consumer's free slots allow (never blocking on a consumer), keep the
        // issued lines in a FIFO (in LDS) and publish them in issue order as they land: vmcnt is
        // in order, so waiting for all but the 8 (t - h - 1) youngest DMAs lands the oldest line.
        // At most 7 lines are outstanding (vmcnt counts to 63).
        uint32_t h = 0, tl = 0;
        for (;;) {
            bool left = false;
#pragma unroll
            for (int c = 0; c < C; c++) {
                if (grp[c] >= n_groups)
                    continue;
                left = true;
                if (tl - h >= 7)
                    continue;
                const uint32_t n = vline[c], q = n % NS;
                uint32_t busy = 0;                             // used[c][q], statically indexed
#pragma unroll
                for (int qq = 0; qq < NS; qq++)
                    busy = qq == int(q) ? used[c][qq] : busy;
                if (__builtin_amdgcn_readfirstlane(lds_load(&freed[c])) < busy)
                    continue;
                issue(feed[c], nxt[c], ring0 + (c * NS + q) * SLOT);
#pragma unroll
                for (int qq = 0; qq < NS; qq++)
                    used[c][qq] = qq == int(q) ? n + 1 : used[c][qq];
                lds_store(&fifo[tl % 8], (uint32_t(c) << 24) | (n + 1));
                tl++;
                vline[c] = n + 1;
                if (++nxt[c] > K) {                            // group done: the consumer's next group
                    nxt[c] = 0;
                    vline[c] = (vline[c] + NS - 1) / NS * NS;
                    grp[c] += G * C;
                    if (grp[c] < n_groups)
                        dma_setup(grp[c], feed[c]);
                }
            }
            if (tl == h) {
                if (!left)
                    break;
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            switch (tl - h) {                                  // the oldest outstanding line landed
            case 1: brb_dma::wait_vmcnt<0>(); break;
            case 2: brb_dma::wait_vmcnt<8>(); break;
            case 3: brb_dma::wait_vmcnt<16>(); break;
            case 4: brb_dma::wait_vmcnt<24>(); break;
            case 5: brb_dma::wait_vmcnt<32>(); break;
            case 6: brb_dma::wait_vmcnt<40>(); break;
            default: brb_dma::wait_vmcnt<48>(); break;
            }
            const uint32_t e = __builtin_amdgcn_readfirstlane(lds_load(&fifo[h % 8]));
            h++;
            lds_store(&ready[e >> 24], e & 0xFFFFFFu);
        }
        return;
    }

    // ================= consumer wave c = wv =================
    static_assert(NS == 3, "consumer tables written for a ring of 3");
    const uint32_t c = wv;
    uint64_t g = uint64_t(blockIdx.x) + G * c;
    if (g >= n_groups)
        return;
    const uint32_t my_off = c * NS * SLOT;
    auto swz = [](uint32_t row) { return (row >> 1) & 7; };
    // window dword i of this lane -> LDS offset: t0 for lines (k-1, k) in slots (0, 1) (and, with
    // +SLOT as ds_read's immediate offset, slots (1, 2)); t2 for slots (2, 0)
    uint32_t t0[32], t2[32];
    auto win_setup = [&](uint64_t g) {
        const uint64_t r0 = g * 64;
        const uint32_t last = uint32_t(n_rec - r0 < 64 ? n_rec - r0 - 1 : 63);
        const uint32_t o0 = uint32_t(dbase + r0 * rec_len) & 127;
        const uint32_t rr = lane < last ? lane : last;
        const uint32_t sh4 = (o0 + rr * rec_len) & 127;
        const uint32_t fr = (my_off + lane * 128) | (swz(lane) << 4);
#pragma unroll
        for (uint32_t i = 0; i < 32; i++) {
            const uint32_t q4 = sh4 + 4 * i;
            const uint32_t a = (q4 & 124u) ^ fr;
            t0[i] = a + ((q4 & 128u) << 6);                    // SLOT = 128 << 6
            t2[i] = a + (q4 & 128u ? 0u : 2 * SLOT);
            asm volatile("" : "+v"(t0[i]), "+v"(t2[i]));
        }
    };
    uint32_t tm[16], tp[16];
    brb_mb_r05::tail_masks(t, tm, tp);
    uint32_t w0[16], w1[16];
    auto wait_ready = [&](uint32_t need) {
        uint32_t polls = 0;
        while (__builtin_amdgcn_readfirstlane(lds_load(&ready[c])) < need && ++polls < kPcPollCap)
            __builtin_amdgcn_s_sleep(1);
    };
    auto read_window = [&](const uint32_t (&ad)[32], uint32_t imm) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            w0[i] = *reinterpret_cast<const uint32_t *>(ring + imm + ad[i]);
            w1[i] = *reinterpret_cast<const uint32_t *>(ring + imm + ad[16 + i]);
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);                    // lgkmcnt(0): the window is in VGPRs
    };
    auto set_freed = [&](uint32_t v) {
        if (lane == 0)
            lds_store(&freed[c], v);
    };
    uint32_t v0 = 0;                                           // virtual number of the group's line 0
    for (;;) {
        win_setup(g);
        typename Alg::State st = Alg::iv();
        // window k (k < K) at position P = (k - 1) mod 3: wait for line v0 + k, read, free lines
        // below it, hash two whole blocks
        auto body = [&](uint32_t k, auto P_) {
            constexpr uint32_t P = decltype(P_)::value;
            wait_ready(v0 + k + 1);
            if constexpr (P == 0)
                read_window(t0, 0);
            else if constexpr (P == 1)
                read_window(t0, SLOT);
            else
                read_window(t2, 0);
            set_freed(v0 + k);
            __builtin_amdgcn_sched_barrier(0);
            Alg::compress(st, w0);
            Alg::compress(st, w1);
            __builtin_amdgcn_sched_barrier(0);
        };
        using P0 = std::integral_constant<uint32_t, 0>;
        using P1 = std::integral_constant<uint32_t, 1>;
        using P2 = std::integral_constant<uint32_t, 2>;
        for (uint32_t k = 1; k < K;) {
            body(k, P0{});
            if (++k >= K)
                break;
            body(k, P1{});
            if (++k >= K)
                break;
            body(k, P2{});
            ++k;
        }
        {   // window K at position (K - 1) mod 3, table picked once per group
            const uint32_t P = (K - 1) % 3;
            uint32_t al[32];
#pragma unroll
            for (int i = 0; i < 32; i++)
                al[i] = P == 2 ? t2[i] : t0[i] + P * SLOT;
            wait_ready(v0 + K + 1);
            read_window(al, 0);
            set_freed(v0 + K + 1);                             // every line of the group is free
            __builtin_amdgcn_sched_barrier(0);
            if (2 * K - 2 < nfull)
                Alg::compress(st, w0);
            if (2 * K - 1 < nfull)
                Alg::compress(st, w1);
        }
        brb_mb_r05::line_finish<Alg, OUT_ALIGNED>(st, w0, w1, tm, tp, t, nfull, K, rec_len, out, g * 64 + lane, n_rec);
        v0 = (v0 + K + 1 + NS - 1) / NS * NS;
        g += G * C;
        if (g >= n_groups)
            break;
    }
}

// One (C + 1)-wave workgroup per CU: C = 4 consumers (one per SIMD) + the producer.
template <class Alg>
hipError_t launch_fixed_line_pc(const uint8_t *data, uint32_t rec_len, uint64_t n_rec, uint8_t *out, bool out_al,
                                hipStream_t s)
{
    constexpr int C = 4, NS = 3;
    const uint64_t groups = (n_rec + 63) / 64;
    const uint64_t wgs = (groups + C - 1) / C;
    const unsigned g = unsigned(wgs < device_cu_count() ? wgs : device_cu_count());
    if (out_al)
        digest_line_pc_kernel<Alg, C, NS, true><<<g, 64 * (C + 1), 0, s>>>(data, rec_len, n_rec, out);
    else
        digest_line_pc_kernel<Alg, C, NS, false><<<g, 64 * (C + 1), 0, s>>>(data, rec_len, n_rec, out);
    return hipGetLastError();
}

}  // namespace brb_digest
