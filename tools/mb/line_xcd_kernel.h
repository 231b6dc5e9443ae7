// line_xcd_kernel.h -- experiment (round 6): the product line kernel (digest_line.h) with its
// groups split over the eight XCDs by weight instead of evenly.
//
// The per-wave probe (tools/gpu_r06_probe.sh) shows the XCDs of one MI355X holding
// different clocks under the MD5 load (1 778 .. 1 932 MHz in one run) and ending the cfg5 shard in
// exactly that order, 14-16 us apart: each CU gets 64 groups whatever its XCD's clock.  Here the
// workgroups of class x = blockIdx % 8 (the dispatcher's round-robin over XCDs) share the group range
// [xs[x], xs[x+1]) -- workgroup j of the class takes xs[x] + j + t * c_x for its tickets t -- and the
// host chooses xs from the previous launches' per-XCD end times.  Every wave stamps its end
// (s_memrealtime) into stamp[wave] and its XCC id, for that feedback.  Used by tools/mb/line_xcd.hip.
#pragma once

#include "digest_line.h"
#include "md5_device.h"

namespace brb_mb_xcd {

struct XSplit {
    uint32_t s[9];    // prefix sums of groups per class; s[8] = n_groups
};

// MD5 compression with a hook after step 15 (round 1 has consumed m[0..15] in order): the
// STAGE 2 form of the kernel below issues its refill DMA there.
template <class Hook>
BRB_DEV void md5_compress_hk(Md5State &st, const uint32_t (&m)[16], Hook hook)
{
    uint32_t a = st.a, b = st.b, c = st.c, d = st.d;
    BRB_MD5_STEP(BRB_MD5_F1, a, b, c, d, m[0], 0xd76aa478u, 7);
    BRB_MD5_STEP(BRB_MD5_F1, d, a, b, c, m[1], 0xe8c7b756u, 12);
    BRB_MD5_STEP(BRB_MD5_F1, c, d, a, b, m[2], 0x242070dbu, 17);
    BRB_MD5_STEP(BRB_MD5_F1, b, c, d, a, m[3], 0xc1bdceeeu, 22);
    BRB_MD5_STEP(BRB_MD5_F1, a, b, c, d, m[4], 0xf57c0fafu, 7);
    BRB_MD5_STEP(BRB_MD5_F1, d, a, b, c, m[5], 0x4787c62au, 12);
    BRB_MD5_STEP(BRB_MD5_F1, c, d, a, b, m[6], 0xa8304613u, 17);
    BRB_MD5_STEP(BRB_MD5_F1, b, c, d, a, m[7], 0xfd469501u, 22);
    BRB_MD5_STEP(BRB_MD5_F1, a, b, c, d, m[8], 0x698098d8u, 7);
    BRB_MD5_STEP(BRB_MD5_F1, d, a, b, c, m[9], 0x8b44f7afu, 12);
    BRB_MD5_STEP(BRB_MD5_F1, c, d, a, b, m[10], 0xffff5bb1u, 17);
    BRB_MD5_STEP(BRB_MD5_F1, b, c, d, a, m[11], 0x895cd7beu, 22);
    BRB_MD5_STEP(BRB_MD5_F1, a, b, c, d, m[12], 0x6b901122u, 7);
    BRB_MD5_STEP(BRB_MD5_F1, d, a, b, c, m[13], 0xfd987193u, 12);
    BRB_MD5_STEP(BRB_MD5_F1, c, d, a, b, m[14], 0xa679438eu, 17);
    BRB_MD5_STEP(BRB_MD5_F1, b, c, d, a, m[15], 0x49b40821u, 22);
    __builtin_amdgcn_sched_barrier(0);
    hook();
    __builtin_amdgcn_sched_barrier(0);
    BRB_MD5_STEP(BRB_MD5_F2, a, b, c, d, m[1], 0xf61e2562u, 5);
    BRB_MD5_STEP(BRB_MD5_F2, d, a, b, c, m[6], 0xc040b340u, 9);
    BRB_MD5_STEP(BRB_MD5_F2, c, d, a, b, m[11], 0x265e5a51u, 14);
    BRB_MD5_STEP(BRB_MD5_F2, b, c, d, a, m[0], 0xe9b6c7aau, 20);
    BRB_MD5_STEP(BRB_MD5_F2, a, b, c, d, m[5], 0xd62f105du, 5);
    BRB_MD5_STEP(BRB_MD5_F2, d, a, b, c, m[10], 0x02441453u, 9);
    BRB_MD5_STEP(BRB_MD5_F2, c, d, a, b, m[15], 0xd8a1e681u, 14);
    BRB_MD5_STEP(BRB_MD5_F2, b, c, d, a, m[4], 0xe7d3fbc8u, 20);
    BRB_MD5_STEP(BRB_MD5_F2, a, b, c, d, m[9], 0x21e1cde6u, 5);
    BRB_MD5_STEP(BRB_MD5_F2, d, a, b, c, m[14], 0xc33707d6u, 9);
    BRB_MD5_STEP(BRB_MD5_F2, c, d, a, b, m[3], 0xf4d50d87u, 14);
    BRB_MD5_STEP(BRB_MD5_F2, b, c, d, a, m[8], 0x455a14edu, 20);
    BRB_MD5_STEP(BRB_MD5_F2, a, b, c, d, m[13], 0xa9e3e905u, 5);
    BRB_MD5_STEP(BRB_MD5_F2, d, a, b, c, m[2], 0xfcefa3f8u, 9);
    BRB_MD5_STEP(BRB_MD5_F2, c, d, a, b, m[7], 0x676f02d9u, 14);
    BRB_MD5_STEP(BRB_MD5_F2, b, c, d, a, m[12], 0x8d2a4c8au, 20);
    BRB_MD5_STEP3X(a, b, c, d, m[5], 0xfffa3942u, 4);
    BRB_MD5_STEP3X(d, a, b, c, m[8], 0x8771f681u, 11);
    BRB_MD5_STEP3X(c, d, a, b, m[11], 0x6d9d6122u, 16);
    BRB_MD5_STEP3X(b, c, d, a, m[14], 0xfde5380cu, 23);
    BRB_MD5_STEP3X(a, b, c, d, m[1], 0xa4beea44u, 4);
    BRB_MD5_STEP3X(d, a, b, c, m[4], 0x4bdecfa9u, 11);
    BRB_MD5_STEP3X(c, d, a, b, m[7], 0xf6bb4b60u, 16);
    BRB_MD5_STEP3X(b, c, d, a, m[10], 0xbebfbc70u, 23);
    BRB_MD5_STEP3X(a, b, c, d, m[13], 0x289b7ec6u, 4);
    BRB_MD5_STEP3X(d, a, b, c, m[0], 0xeaa127fau, 11);
    BRB_MD5_STEP3X(c, d, a, b, m[3], 0xd4ef3085u, 16);
    BRB_MD5_STEP3X(b, c, d, a, m[6], 0x04881d05u, 23);
    BRB_MD5_STEP3X(a, b, c, d, m[9], 0xd9d4d039u, 4);
    BRB_MD5_STEP3X(d, a, b, c, m[12], 0xe6db99e5u, 11);
    BRB_MD5_STEP3X(c, d, a, b, m[15], 0x1fa27cf8u, 16);
    BRB_MD5_STEP3X(b, c, d, a, m[2], 0xc4ac5665u, 23);
    BRB_MD5_STEP(BRB_MD5_F4, a, b, c, d, m[0], 0xf4292244u, 6);
    BRB_MD5_STEP(BRB_MD5_F4, d, a, b, c, m[7], 0x432aff97u, 10);
    BRB_MD5_STEP(BRB_MD5_F4, c, d, a, b, m[14], 0xab9423a7u, 15);
    BRB_MD5_STEP(BRB_MD5_F4, b, c, d, a, m[5], 0xfc93a039u, 21);
    BRB_MD5_STEP(BRB_MD5_F4, a, b, c, d, m[12], 0x655b59c3u, 6);
    BRB_MD5_STEP(BRB_MD5_F4, d, a, b, c, m[3], 0x8f0ccc92u, 10);
    BRB_MD5_STEP(BRB_MD5_F4, c, d, a, b, m[10], 0xffeff47du, 15);
    BRB_MD5_STEP(BRB_MD5_F4, b, c, d, a, m[1], 0x85845dd1u, 21);
    BRB_MD5_STEP(BRB_MD5_F4, a, b, c, d, m[8], 0x6fa87e4fu, 6);
    BRB_MD5_STEP(BRB_MD5_F4, d, a, b, c, m[15], 0xfe2ce6e0u, 10);
    BRB_MD5_STEP(BRB_MD5_F4, c, d, a, b, m[6], 0xa3014314u, 15);
    BRB_MD5_STEP(BRB_MD5_F4, b, c, d, a, m[13], 0x4e0811a1u, 21);
    BRB_MD5_STEP(BRB_MD5_F4, a, b, c, d, m[4], 0xf7537e82u, 6);
    BRB_MD5_STEP(BRB_MD5_F4, d, a, b, c, m[11], 0xbd3af235u, 10);
    BRB_MD5_STEP(BRB_MD5_F4, c, d, a, b, m[2], 0x2ad7d2bbu, 15);
    BRB_MD5_STEP(BRB_MD5_F4, b, c, d, a, m[9], 0xeb86d391u, 21);
    st.a += a;
    st.b += b;
    st.c += c;
    st.d += d;
}

BRB_DEV inline uint64_t rt_now()
{
    uint64_t t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

// POL (streamed lines 2..K of a group): 0 nt (the product's), 1 nt sc1, 2 sc1, 3 sc0 sc1, 4 nt sc0 sc1
// STAGE (full iterations): 0 the product's (32 window reads, lgkmcnt(0), refill DMA, two compressions);
// 1 the reads without the wait (the compiler's per-register waits), block 2k-2 hashed, then
// lgkmcnt(0) and the refill DMA, then block 2k-1; 2 the same with the refill DMA after step 15 of
// block 2k-2 (md5_compress_hk; MD5 only)
// MAP: 0 workgroup j of a class takes groups g_lo + j + t c_x (interleaved, the product's); 1 it takes
// a contiguous block of the class's range (the CU's eight waves work on neighbouring groups)
template <class Alg, int WAVES, bool OUT_ALIGNED, bool TAIL_HI, int POL = 0, int STAGE = 0, int MAP = 0>
__global__ __launch_bounds__(64 * WAVES, 2) void digest_line_xcd_kernel(const uint8_t *__restrict__ data,
                                                                       uint32_t rec_len, uint64_t n_rec,
                                                                       uint8_t *__restrict__ out, XSplit xs,
                                                                       uint64_t *__restrict__ stamp)
{
    constexpr uint32_t SLOT = 8192;
    __shared__ __attribute__((aligned(16))) uint8_t ring[WAVES * 2 * SLOT];
    __shared__ uint32_t next_ticket;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t cls = blockIdx.x & 7, jx = blockIdx.x >> 3;
    const uint32_t cx = (gridDim.x - cls + 7) >> 3;            // workgroups of this class
    const uint64_t c_lo = xs.s[cls], c_hi = xs.s[cls + 1];
    const uint64_t g_lo = MAP ? c_lo + (uint64_t(jx) * (c_hi - c_lo)) / cx : c_lo;
    const uint64_t g_hi = MAP ? c_lo + (uint64_t(jx + 1) * (c_hi - c_lo)) / cx : c_hi;
    const uint64_t g_first = MAP ? g_lo : g_lo + jx, g_step = MAP ? 1 : cx;
    const uint64_t t0 = stamp ? rt_now() : 0;
    if (threadIdx.x == 0)
        next_ticket = WAVES;
    __syncthreads();
    auto take = [&]() -> uint64_t {
        uint32_t tk = 0;
        if (lane == 0)
            tk = __hip_atomic_fetch_add(&next_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        tk = __builtin_amdgcn_readfirstlane(tk);
        return g_first + uint64_t(tk) * g_step;
    };
    auto finish_stamp = [&]() {
        if (stamp && lane == 0) {
            uint32_t xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
            const uint64_t w = uint64_t(blockIdx.x) * WAVES + wv;
            stamp[3 * w] = t0;
            stamp[3 * w + 1] = rt_now();
            stamp[3 * w + 2] = xcc;
        }
    };
    uint64_t g = g_first + uint64_t(wv) * g_step;
    if (g >= g_hi) {
        finish_stamp();
        return;
    }
    const uint32_t my_off = wv * 2 * SLOT;
    const uint32_t lds0 = uint32_t(reinterpret_cast<uintptr_t>(ring)) + my_off;
    const uint32_t nfull = rec_len >> 6, t = rec_len & 63;
    const uint32_t nblk = nfull + (t ? 1 : 0);
    const uint32_t K = (nblk + 1) >> 1;
    const uint32_t P = (K & 1) ^ 1;
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
    brb_dma::v4i rs, rsn;
    auto desc = [&](uint64_t g, brb_dma::v4i &rs) {
        const uint64_t gbase = ((dbase + g * gbytes) & ~uint64_t(127)) - 4096;
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
#define BRB_XCD_DMA8(POL)                                                                       \
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
        if (keep_l2)
            BRB_XCD_DMA8("");
        else if (POL == 1)
            BRB_XCD_DMA8("nt sc1 ");
        else if (POL == 2)
            BRB_XCD_DMA8("sc1 ");
        else if (POL == 3)
            BRB_XCD_DMA8("sc0 sc1 ");
        else if (POL == 4)
            BRB_XCD_DMA8("nt sc0 sc1 ");
        else
            BRB_XCD_DMA8("nt ");
#undef BRB_XCD_DMA8
        so += 128;
    };
    uint32_t ae[32], ao[32];
    uint32_t w0[16], w1[16];
    auto read_window = [&](const uint32_t (&ad)[32]) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            w0[i] = *reinterpret_cast<const uint32_t *>(ring + ad[i]);
            w1[i] = *reinterpret_cast<const uint32_t *>(ring + ad[16 + i]);
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
    };
    desc(g, rs);
    issue(rs, so, P, true);
    issue(rs, so, P ^ 1, true);
    __builtin_amdgcn_sched_barrier(0);
    uint64_t gn = take();
    {
        const uint32_t sh4 = (o0 + lane * rec_len) & 127;
        const uint32_t fr = (my_off + lane * 128) | (swz(lane) << 4);
#pragma unroll
        for (uint32_t i = 0; i < 32; i++) {
            const uint32_t q4 = sh4 + 4 * i;
            ae[i] = ((q4 & 124u) ^ fr) | ((q4 & 128u) << 6);
            ao[i] = ae[i] ^ SLOT;
            asm volatile("" : "+v"(ae[i]), "+v"(ao[i]));
        }
    }
    uint32_t tm[16], tp[16];
    brb_digest::tail_masks(t, tm, tp);
    auto full_step = [&](typename Alg::State &st, const uint32_t (&ad)[32], uint32_t refill_slot) {
        brb_dma::wait_vmcnt<0>();
        if constexpr (STAGE == 0) {
            read_window(ad);
            issue(rs, so, refill_slot);
            __builtin_amdgcn_sched_barrier(0);
            Alg::compress(st, w0);
            Alg::compress(st, w1);
        } else {
#pragma unroll
            for (int i = 0; i < 16; i++)
                w0[i] = *reinterpret_cast<const uint32_t *>(ring + ad[i]);
#pragma unroll
            for (int i = 0; i < 16; i++)
                w1[i] = *reinterpret_cast<const uint32_t *>(ring + ad[16 + i]);
            __builtin_amdgcn_sched_barrier(0);
            auto refill = [&]() {
                __builtin_amdgcn_s_waitcnt(0xC07F);             // every window read has landed
                issue(rs, so, refill_slot);
            };
            if constexpr (STAGE == 1) {
                Alg::compress(st, w0);
                __builtin_amdgcn_sched_barrier(0);
                refill();
                __builtin_amdgcn_sched_barrier(0);
            } else {
                md5_compress_hk(st, w0, refill);
                __builtin_amdgcn_sched_barrier(0);
            }
            Alg::compress(st, w1);
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    for (;;) {
        typename Alg::State st = Alg::iv();
        uint32_t k = 1;
        if (P) {
            full_step(st, ao, 1);
            k = 2;
        }
        for (; k + 2 <= K; k += 2) {
            full_step(st, ae, 0);
            full_step(st, ao, 1);
        }
        {
            brb_dma::wait_vmcnt<0>();
            read_window(ae);
            if (gn < g_hi) {
                desc(gn, rsn);
                son = 0;
                issue(rsn, son, P, true);
                issue(rsn, son, P ^ 1, true);
            }
            if (2 * K - 2 < nfull)
                Alg::compress(st, w0);
            if (2 * K - 1 < nfull)
                Alg::compress(st, w1);
        }
        brb_digest::line_finish<Alg, OUT_ALIGNED, TAIL_HI>(st, w0, w1, tm, tp, t, rec_len, out, g * 64 + lane, n_rec);
        g = gn;
        if (g >= g_hi)
            break;
        gn = take();
        rs = rsn;
        so = son;
    }
    finish_stamp();
}

}  // namespace brb_mb_xcd
