// digest_line.h -- fixed-stride, lane-per-record digest kernel (MD5, SHA-1) with LINE-ALIGNED
// LDS-DMA staging.  Used when every record starts on a 4-byte boundary (data 4-aligned and
// rec_len % 4 == 0, e.g. the 1500-byte records of SURVEY §8(d) configs 2 and 5).
//
// Why line-aligned: a record of 1500 B starts anywhere inside a 128-byte memory line, so a
// 128-byte stage taken at the record's own offset straddles two lines and every line is requested
// twice.  Measured on the staging alone (tools/mb/dma_pattern.hip, 1 Mi x 1500 B): 5.8 TB/s with
// record-relative 128-byte pieces, 6.5 TB/s with line-aligned ones (a contiguous stream: 6.3).
//
// Stage k of lane l's record = the k-th 128-byte line from the line holding the record's first
// byte.  The record starts sh = (address mod 128) / 4 dwords into its first line, so message blocks
// 2k-2 and 2k-1 (stream dwords sh + 32(k-1) .. sh + 32k - 1) lie in lines k-1 and k.  Lines k-1
// and k sit in the two slots of the wave's LDS ring; each lane reads its 32 shifted dwords with
// ds_read_b32 at per-lane addresses that are fixed for the whole record (one address table per
// slot parity), so the shift costs no VALU.  Once the window is in VGPRs, the slot of line k-1 is
// refilled with line k+1 while blocks 2k-2 and 2k-1 are hashed.
//
// Safety: every line read holds at least one byte of the batch (the line of a record's first byte,
// the lines after it up to the line of the batch's last byte); lines past that are cut off by the
// buffer descriptor's range check and read as zeros.  Bytes of a line outside the record are
// masked by the padding step, as the tail of any record.
//
// Record r's digest = BRB_MD5Init/Update/Final (md5.c:38-168) or BrbSha1_Do (sha1.c:203-216) of
// data[r * rec_len .. (r + 1) * rec_len).
#pragma once

#include "dma_stage.h"

// Diagnostic hooks (tools/mb/line_probe.hip defines them; empty in the product build).
#ifndef BRB_LINE_PROBE
#define BRB_LINE_PROBE_DECL
#define BRB_LINE_PROBE(ev) ((void)0)
#endif

namespace brb_digest {

// Padding, digest and store of one group: the record's tail block (if any) is window half
// nfull - (2K - 2) of the last iteration; bytes past the record are masked (md5.c:134-168).
template <class Alg, bool OUT_ALIGNED>
BRB_DEV void line_finish(typename Alg::State &st, const uint32_t (&w0)[16], const uint32_t (&w1)[16], uint32_t t,
                         uint32_t nfull, uint32_t K, uint32_t rec_len, uint8_t *out, uint64_t r, uint64_t n_rec)
{
    uint32_t tt = t;
    asm volatile("" : "+s"(tt));                               // keep the tail math here, once per group
    if (tt == 0) {
        Alg::pad_only(st, rec_len);                            // the padding block is a constant
        if (r < n_rec)
            Alg::template store<OUT_ALIGNED>(out, r, st);
        return;
    }
    uint32_t w[16];
    if (nfull + 2 - 2 * K) {
#pragma unroll
        for (int i = 0; i < 16; i++)
            w[i] = w1[i];
    } else {
#pragma unroll
        for (int i = 0; i < 16; i++)
            w[i] = w0[i];
    }
#pragma unroll
    for (uint32_t i = 0; i < 16; i++) {
        const uint32_t o = 4 * i;
        const uint32_t keep = tt > o ? (tt - o < 4 ? tt - o : 4) : 0;
        uint32_t v = w[i] & uint32_t((uint64_t(1) << (8 * keep)) - 1);
        if (tt >= o && tt < o + 4)
            v |= 0x80u << (8 * (tt - o));
        w[i] = v;
    }
    Alg::finish(st, w, t, rec_len);
    if (r < n_rec)
        Alg::template store<OUT_ALIGNED>(out, r, st);
}

// Group assignment.  Static (DYN = false): wave w of the grid takes groups w, w + W_total, ...
// Dynamic (DYN = true): workgroup b owns groups b, b + G, b + 2G, ... (G = gridDim.x) and its waves
// take them one at a time from an LDS ticket counter.  Why: with two waves per SIMD the older wave
// wins the issue arbitration, so under a static split the first workgroup of every CU finished its
// share at ~190 us and the second one ran alone (at the lone-wave issue rate) until ~300 us
// (1 Mi x 1500 B, tools/mb/line_probe.hip); with tickets the faster wave simply takes more groups.
// launch_bounds: two waves per SIMD (4-wave workgroups: two per CU, 64 KiB of LDS each; 8-wave
// workgroups: one per CU, 128 KiB).
template <class Alg, int WAVES, bool OUT_ALIGNED, bool NT = false, bool DYN = false>
__global__ __launch_bounds__(64 * WAVES, 2) void digest_line_kernel(const uint8_t *__restrict__ data,
                                                                             uint32_t rec_len, uint64_t n_rec,
                                                                             uint8_t *__restrict__ out)
{
    constexpr uint32_t SLOT = 8192;                            // 64 rows x one 128-byte line
    __shared__ __attribute__((aligned(16))) uint8_t ring[WAVES * 2 * SLOT];
    __shared__ uint32_t next_ticket;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t n_groups = (n_rec + 63) / 64;
    const uint64_t wave0 = uint64_t(blockIdx.x) * WAVES + wv;
    const uint64_t wstride = uint64_t(gridDim.x) * WAVES;
    if (DYN) {
        if (threadIdx.x == 0)
            next_ticket = WAVES;                               // tickets 0 .. WAVES-1: one per wave
        __syncthreads();
    }
    auto take = [&]() -> uint64_t {                            // DYN: the next group of this workgroup
        uint32_t tk = 0;
        if (lane == 0)
            tk = __hip_atomic_fetch_add(&next_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        tk = __builtin_amdgcn_readfirstlane(tk);
        return uint64_t(blockIdx.x) + uint64_t(tk) * gridDim.x;
    };
    uint64_t g = DYN ? uint64_t(blockIdx.x) + uint64_t(wv) * gridDim.x : wave0;
    if (g >= n_groups)
        return;
    uint64_t gn = DYN ? take() : g + wstride;                  // the group after g

    const uint32_t my_off = wv * 2 * SLOT;                     // slot 0; slot 1 = my_off + SLOT (bit 13 clear)
    const uint32_t lds0 = uint32_t(reinterpret_cast<uintptr_t>(ring)) + my_off;
    const uint32_t nfull = rec_len >> 6, t = rec_len & 63;
    const uint32_t nblk = nfull + (t ? 1 : 0);
    const uint32_t K = (nblk + 1) >> 1;                        // 2-block iterations per group; K + 1 lines
    const uint64_t dbase = reinterpret_cast<uint64_t>(data);
    const uint64_t end_line = (dbase + n_rec * rec_len + 127) & ~uint64_t(127);
    // 16-byte granule swizzle of a 128-byte row (applied on the DMA source): ds_read_b128 of one
    // logical granule by all lanes is conflict-free, ds_read_b32 of one logical dword 4-way at worst.
    auto swz = [](uint32_t row) { return (row >> 1) & 7; };

    // ---- issue side: DMA lane j of instruction q stages granule j % 8 of row 8q + j / 8
    uint32_t vq[8];
    uint64_t gline = 0;                                        // first line of the issuing group
    uint64_t gleft = 0;                                        // bytes from gline to end_line
    // fastq: DMA q carries the instruction offset 1024 (q % 4), which lands in the LDS address as
    // well, so one M0 write serves four DMAs; the voffset is lowered by the same amount.  Needs
    // every voffset >= 3072 where q % 4 == 3: full groups and records of at least 160 bytes.
    bool fastq = false;
    auto dma_setup = [&](uint64_t g) {
        const uint64_t r0 = g * 64;
        const uint32_t last = uint32_t(n_rec - r0 < 64 ? n_rec - r0 - 1 : 63);
        const uint64_t a0 = dbase + r0 * rec_len;
        gline = a0 & ~uint64_t(127);
        gleft = end_line - gline;
        const uint32_t o0 = uint32_t(a0) & 127;
        fastq = last == 63 && rec_len >= 160;
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const uint32_t row = 8 * q + (lane >> 3);
            const uint32_t rr = row < last ? row : last;
            vq[q] = ((o0 + rr * rec_len) & ~127u) + 16 * ((lane & 7) ^ swz(row)) - (fastq ? 1024u * (q & 3) : 0u);
        }
    };
    auto issue = [&](uint32_t slot, uint32_t k) {              // line k of the issuing group -> slot
        // descriptor of line k: base gline + 128 k, num_records = bytes left to end_line clamped to
        // [0, 2^31 - 1], in 32-bit scalar ops (gfx950 has no 64-bit ordered scalar compare)
        const uint64_t base = gline + 128ull * k;
        const int64_t left = int64_t(gleft) - int64_t(128u * k);
        const int32_t lhi = int32_t(uint64_t(left) >> 32);
        const uint32_t llo = uint32_t(left);
        const uint32_t nrec = lhi < 0 ? 0u : (lhi > 0 || llo > 0x7FFFFFFFu) ? 0x7FFFFFFFu : llo;
        brb_dma::v4i rs;
        rs.x = int(uint32_t(base));
        rs.y = int(uint32_t(base >> 32) & 0xFFFF);
        rs.z = int(nrec);
        rs.w = 0x00020000;
        const uint32_t m = lds0 + slot * SLOT;
        if (fastq) {
#define BRB_LINE_DMA8(POL)                                                                      \
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
            uint32_t keep;
            if constexpr (NT)
                BRB_LINE_DMA8("nt ");
            else
                BRB_LINE_DMA8("");
#undef BRB_LINE_DMA8
            return;
        }
#define BRB_LINE_DMA(POL)                                                  \
    asm volatile("s_mov_b32 %0, m0\n\t"                                     \
                 "s_mov_b32 m0, %3\n\t"                                     \
                 "s_nop 0\n\t"                                              \
                 "buffer_load_dwordx4 %1, %2, 0 offen " POL "lds\n\t"       \
                 "s_mov_b32 m0, %0"                                          \
                 : "=&s"(keep)                                               \
                 : "v"(vq[q]), "s"(rs), "s"(m + 1024u * q)                   \
                 : "memory")
#pragma unroll
        for (int q = 0; q < 8; q++) {
            uint32_t keep;
            if constexpr (NT)
                BRB_LINE_DMA("nt ");
            else
                BRB_LINE_DMA("");
        }
#undef BRB_LINE_DMA
    };

    // ---- read side: window dword i of this lane -> LDS offset, for lines (k-1, k) in slots
    // (0, 1) ["ae", k odd] and (1, 0) ["ao", k even]
    uint32_t ae[32], ao[32];
    auto win_setup = [&](uint64_t g) {
        const uint64_t r0 = g * 64;
        const uint32_t last = uint32_t(n_rec - r0 < 64 ? n_rec - r0 - 1 : 63);
        const uint32_t o0 = uint32_t(dbase + r0 * rec_len) & 127;
        const uint32_t rr = lane < last ? lane : last;
        const uint32_t sh = ((o0 + rr * rec_len) & 127) >> 2;
        const uint32_t f = swz(lane), row = my_off + lane * 128;
#pragma unroll
        for (uint32_t i = 0; i < 32; i++) {
            const uint32_t q = sh + i, qq = q & 31;
            const uint32_t a = row + ((((qq >> 2) ^ f) << 4) | ((qq & 3) << 2));
            ae[i] = q >= 32 ? a + SLOT : a;
            ao[i] = q >= 32 ? a : a + SLOT;
        }
    };

    uint32_t w0[16], w1[16];
    auto read_window = [&](const uint32_t (&ad)[32]) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            w0[i] = *reinterpret_cast<const uint32_t *>(ring + ad[i]);
            w1[i] = *reinterpret_cast<const uint32_t *>(ring + ad[16 + i]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // window in VGPRs before its slot is refilled
    };

    BRB_LINE_PROBE_DECL
    BRB_LINE_PROBE(0);
    dma_setup(g);
    issue(0, 0);
    issue(1, 1);
    win_setup(g);
    for (;;) {
        typename Alg::State st = Alg::iv();
        // one iteration: wait for line k, read the window, refill the slot of line k-1 (or start
        // the next group), hash blocks 2k-2 and 2k-1
        // one compress site per block (the code must stay small: one wave per SIMD runs out of
        // the shared instruction cache at once when the loop body is unrolled)
        for (uint32_t k = 1; k <= K; k++) {
            BRB_LINE_PROBE(1);
            brb_dma::wait_vmcnt<0>();
            if (k & 1)
                read_window(ae);
            else
                read_window(ao);
            BRB_LINE_PROBE(2);
            if (k < K) {
                issue((k + 1) & 1, k + 1);
            } else if (gn < n_groups) {
                dma_setup(gn);
                issue(0, 0);
                issue(1, 1);
            }
            const uint32_t b = 2 * k - 2;
            if (b < nfull)
                Alg::compress(st, w0);
            if (b + 1 < nfull)
                Alg::compress(st, w1);
        }
        line_finish<Alg, OUT_ALIGNED>(st, w0, w1, t, nfull, K, rec_len, out, g * 64 + lane, n_rec);
        g = gn;
        if (g >= n_groups)
            break;
        gn = DYN ? take() : g + wstride;
        win_setup(g);
    }
    BRB_LINE_PROBE(3);
}

// Line-aligned staging needs 4-byte record bases (the window shift is whole dwords).
inline bool line_supported(const uint8_t *data, uint32_t rec_len)
{
    return rec_len > 64 && (rec_len & 3) == 0 && (reinterpret_cast<uintptr_t>(data) & 3) == 0 &&
           uint64_t(rec_len) * 64 + 256 < (uint64_t(1) << 31);
}

inline unsigned device_cu_count()
{
    static const unsigned n = [] {
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
            c = 256;
        return unsigned(c);
    }();
    return n;
}

// One 8-wave workgroup per CU (128 KiB of LDS), persistent, groups handed out by tickets (DYN), DMA
// with the non-temporal policy (every line is read exactly once).  Measured with
// tools/mb/md5_ab.hip, MD5, medians of 20-launch bursts:
//   1 Mi x 1500 B: 316 us static 4-wave workgroups -> 300 us (read floor of the same bytes: 261 us nt)
//   cfg2 65 536 x 1500 B: 25.3 us (record-relative 128-byte stages) -> 24.9 us
template <class Alg>
hipError_t launch_fixed_line(const uint8_t *data, uint32_t rec_len, uint64_t n_rec, uint8_t *out, bool out_al,
                             hipStream_t s)
{
    constexpr int W = 8;
    const uint64_t groups = (n_rec + 63) / 64;
    const unsigned g = unsigned(groups < device_cu_count() ? groups : device_cu_count());
    if (out_al)
        digest_line_kernel<Alg, W, true, true, true><<<g, 64 * W, 0, s>>>(data, rec_len, n_rec, out);
    else
        digest_line_kernel<Alg, W, false, true, true><<<g, 64 * W, 0, s>>>(data, rec_len, n_rec, out);
    return hipGetLastError();
}

}  // namespace brb_digest
