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
// Group-invariant setup (round 6).  rec_len % 4 == 0, so a group of 64
// records spans 64 * rec_len bytes, a multiple of 256: every group starts at the same offset
// o0 = data mod 128 inside its first line, and record l of any group sits at o0 + l * rec_len from
// that line.  The two window-address tables and the eight DMA offsets of a lane are therefore the
// same for every group and are built once per wave; a group costs its buffer descriptor (scalar).
// Lanes past a partial last group keep their full-group addresses: their DMA rows lie past the
// batch (range-checked to zeros), their window reads stay inside their own LDS row, and their
// digests are not stored.  The launch-uniform choices are template arguments or slot parity, not
// per-lane selects: TAIL_HI (the record's tail block is the second block of the last iteration)
// and P, the slot that takes a group's line 0, chosen so that the last iteration always reads
// lines K-1, K from slots 0, 1 (one table, no select).
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
#include "test_options.h"

// Diagnostic hooks (tools/mb/line_probe.hip defines them; empty in the product build).
#ifndef BRB_LINE_PROBE
#define BRB_LINE_PROBE_DECL
#define BRB_LINE_PROBE(ev) ((void)0)
#endif

namespace brb_digest {

// Padding, digest and store of one group: the record's tail block (if any) is the last
// iteration's block 2K-1 (TAIL_HI, w1) or 2K-2 (w0); bytes past the record are masked
// (md5.c:134-168).  The tail's per-dword keep masks and 0x80 marker (tm, tp) depend only on
// rec_len: they are built once per wave (tail_masks), so a group pays 16 v_and_or here.
template <class Alg, bool OUT_ALIGNED, bool TAIL_HI>
BRB_DEV void line_finish(typename Alg::State &st, const uint32_t (&w0)[16], const uint32_t (&w1)[16],
                         const uint32_t (&tm)[16], const uint32_t (&tp)[16], uint32_t t, uint32_t rec_len,
                         uint8_t *out, uint64_t r, uint64_t n_rec)
{
    if (t == 0) {
        Alg::pad_only(st, rec_len);                            // the padding block is a constant
        if (r < n_rec)
            Alg::template store<OUT_ALIGNED>(out, r, st);
        return;
    }
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++)
        w[i] = ((TAIL_HI ? w1[i] : w0[i]) & tm[i]) | tp[i];
    Alg::finish(st, w, t, rec_len);
    if (r < n_rec)
        Alg::template store<OUT_ALIGNED>(out, r, st);
}

// Keep mask and marker of tail dword i for a tail of t bytes (0 < t < 64): bytes below t kept,
// 0x80 at byte t, zeros after.  Kept in VGPRs (asm barrier) so that no group recomputes them.
BRB_DEV void tail_masks(uint32_t t, uint32_t (&tm)[16], uint32_t (&tp)[16])
{
#pragma unroll
    for (uint32_t i = 0; i < 16; i++) {
        const uint32_t o = 4 * i;
        const uint32_t keep = t > o ? (t - o < 4 ? t - o : 4) : 0;
        tm[i] = uint32_t((uint64_t(1) << (8 * keep)) - 1);
        tp[i] = t >= o && t < o + 4 ? 0x80u << (8 * (t - o)) : 0u;
        asm volatile("" : "+v"(tm[i]), "+v"(tp[i]));
    }
}

// Which half of the last iteration's window holds the tail block of a rec_len-byte record (t > 0):
// blocks 0 .. nfull-1 are whole and the tail is block nfull; the last iteration K = (nfull + 2) / 2
// holds blocks 2K-2 and 2K-1, so the tail is its second block exactly when nfull is odd.
inline bool line_tail_hi(uint32_t rec_len)
{
    return ((rec_len >> 6) & 1) != 0;
}

// Group assignment: workgroup b owns groups b, b + G, b + 2G, ... (G = gridDim.x) and its waves
// take them one at a time from an LDS ticket counter.  Why: with two waves per SIMD the older wave
// wins the issue arbitration, so under a static split the first workgroup of every CU finished its
// share at ~190 us and the second one ran alone (at the lone-wave issue rate) until ~300 us
// (1 Mi x 1500 B, tools/mb/line_probe.hip); with tickets the faster wave simply takes more groups.
// One 8-wave workgroup per CU (128 KiB of LDS), two waves per SIMD.  Two ways of evening out the
// end of a launch measured slower and live in tools/mb/line_r05_kernel.h: a chip-wide tail pool
// and SIMD partners in lockstep.  Round 6: one ticket counter per SIMD (SIMD s of
// a workgroup owning its rounds s, s + 4, ...) measured the same on the cfg5 shard (289.95 vs
// 290.45 us) and 1 % slower at 300 001 records (profiles/r06/line_ab_*_box4_simd_tickets.txt).
// Loading one dword of each row's line k+2 right after line k+1's DMA (temporal policy, into an LDS
// scratch row) so that its DMA would hit the L2 one iteration later: cfg5 297.0 -> 322.0 us, cfg2
// 21.3 -> 24.1 us (profiles/r06/line_ab_*_box5_l2prefetch.txt): not kept.
template <class Alg, int WAVES, bool OUT_ALIGNED, bool TAIL_HI>
__global__ __launch_bounds__(64 * WAVES, 2) void digest_line_kernel(const uint8_t *__restrict__ data,
                                                                             uint32_t rec_len, uint64_t n_rec,
                                                                             uint8_t *__restrict__ out)
{
    constexpr uint32_t SLOT = 8192;                            // 64 rows x one 128-byte line
    __shared__ __attribute__((aligned(16))) uint8_t ring[WAVES * 2 * SLOT];
    __shared__ uint32_t next_ticket;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    [[maybe_unused]] const uint64_t wave0 = uint64_t(blockIdx.x) * WAVES + wv;   // probe builds
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
    const uint32_t my_off = wv * 2 * SLOT;                     // slot 0; slot 1 = my_off + SLOT (bit 13 clear)
    const uint32_t lds0 = uint32_t(reinterpret_cast<uintptr_t>(ring)) + my_off;
    const uint32_t nfull = rec_len >> 6, t = rec_len & 63;
    const uint32_t nblk = nfull + (t ? 1 : 0);
    const uint32_t K = (nblk + 1) >> 1;                        // 2-block iterations per group; K + 1 lines
    // Line j of a group goes to slot (j + P) & 1: iteration k reads lines k-1, k from slots
    // (k-1+P) & 1, (k+P) & 1, which at k = K are 0, 1 for either parity of K.
    const uint32_t P = (K & 1) ^ 1;
    const uint64_t dbase = reinterpret_cast<uint64_t>(data);
    const uint64_t end_line = (dbase + n_rec * rec_len + 127) & ~uint64_t(127);
    const uint64_t gbytes = uint64_t(rec_len) * 64;            // a multiple of 256
    const uint32_t o0 = uint32_t(dbase) & 127;                 // every group's first-byte offset in its line
    // 16-byte granule swizzle of a 128-byte row (applied on the DMA source): ds_read_b128 of one
    // logical granule by all lanes is conflict-free, ds_read_b32 of one logical dword 4-way at worst.
    auto swz = [](uint32_t row) { return (row >> 1) & 7; };

    // ---- issue side: DMA lane j of instruction q stages granule j % 8 of row 8q + j / 8 of the
    // issuing group's next line.  One M0 write serves four DMAs: DMA q carries the instruction
    // offset 1024 (q % 4), which lands in the LDS address as well, and its voffset is lowered by the
    // same amount.  The descriptor base sits 4 KiB below the group's first line (and num_records
    // 4 KiB above the bytes left), so every voffset stays >= 1024 whatever the record length: one
    // DMA form for every line, no per-DMA M0 writes.  Row 8q + l3's line offset from the group's
    // first line is (o0 + row * rec_len) & ~127 for every group (see the header), so the offsets
    // are built here, once per wave; swz(8q + l3) = (l3 >> 1) ^ 4(q & 1) takes two values.
    uint32_t vq[8];
    {
        const uint32_t l3 = lane >> 3;
        const uint32_t base = o0 + l3 * rec_len;
        const uint32_t g0 = 16u * ((lane & 7) ^ (l3 >> 1));
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const uint32_t x = base + 8u * q * rec_len;        // < 2^27: rec_len <= 1 MiB
            vq[q] = ((x & ~127u) | (q & 1 ? g0 ^ 64u : g0)) + (4096u - 1024u * (q & 3));
        }
    }
    // Descriptor of a group: base = the group's first line - 4096, num_records = 4096 + bytes from
    // that line to end_line, clamped to [0, 2^31 - 1]; line j of the group is addressed by
    // soffset = 128 j.  A group at least 2^31 - 4097 bytes from the end has num_records 2^31 - 1,
    // above every offset of its K + 1 lines (line_supported caps rec_len at 1 MiB: < 64 MiB + 8 KiB).
    // Scalar only.  The next group's descriptor goes to rsn and is taken over once per group.
    brb_dma::v4i rs, rsn;
    auto desc = [&](uint64_t g, brb_dma::v4i &rs) {
        const uint64_t gbase = ((dbase + g * gbytes) & ~uint64_t(127)) - 4096;
        const uint64_t gleft = end_line - gbase;
        rs.x = __builtin_amdgcn_readfirstlane(int(uint32_t(gbase)));
        rs.y = __builtin_amdgcn_readfirstlane(int(uint32_t(gbase >> 32) & 0xFFFF));
        rs.z = __builtin_amdgcn_readfirstlane(int(gleft > 0x7FFFFFFFull ? 0x7FFFFFFFu : uint32_t(gleft)));
        rs.w = 0x00020000;
    };
    // Lines 0 and 1 of a group go through the L2 with the normal (temporal) policy, the others
    // non-temporal: record r's last line or two are record r+1's first ones, read by the same wave
    // ~17 us later, and with every line nt the L2 had dropped them (cfg2 fetched 105.3 MB for 98.3 MB
    // of records).  Round 3: 94.9 MB fetched, cfg2 21.49 -> 20.99 us, the 1 Mi-record shard 300.4 ->
    // 288.7 us (interleaved A/B).
    // soffset of the next line to issue (the descriptor stays put for the whole group; the range
    // check covers voffset + soffset + the instruction offset, per dword: tools/mb/buf_range.hip).
    uint32_t so = 0, son = 0;
    auto issue = [&](const brb_dma::v4i &rs, uint32_t &so, uint32_t slot, bool keep_l2 = false) {   // next line -> slot
#ifdef BRB_LINE_NO_DMA      // diagnostic builds only (tools/mb/line_parts.hip): hash stale LDS
        return;
#endif
        const uint32_t m = lds0 + slot * SLOT;
        uint32_t keep;
#define BRB_LINE_DMA8(POL)                                                                      \
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
        if (!keep_l2)
            BRB_LINE_DMA8("nt ");
        else
            BRB_LINE_DMA8("");
#undef BRB_LINE_DMA8
        so += 128;                                             // the line after the issued one
    };

    // ---- read side: window dword i of this lane -> LDS offset, for lines (k-1, k) in slots
    // (0, 1) ["ae"] and (1, 0) ["ao"].  Built once per wave, behind the first DMA (below): lane l's
    // shift is that of record l of every group.
    uint32_t ae[32], ao[32];

    uint32_t w0[16], w1[16];
    auto read_window = [&](const uint32_t (&ad)[32]) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            w0[i] = *reinterpret_cast<const uint32_t *>(ring + ad[i]);
            w1[i] = *reinterpret_cast<const uint32_t *>(ring + ad[16 + i]);
        }
        // window in VGPRs before its slot is refilled: lgkmcnt(0) (vmcnt 63, expcnt 7 = no wait).
        // The builtin, not inline asm: the compiler's waitcnt pass then knows the reads are done and
        // inserts no waits of its own before their uses.
        __builtin_amdgcn_s_waitcnt(0xC07F);
    };

    BRB_LINE_PROBE_DECL
    BRB_LINE_PROBE(0);
    // (Round 6: issuing this first line pair before the workgroup barrier that publishes the ticket
    // counter measured 297-301 us against 295-297 us on the cfg5 shard, cfg2 unchanged: not kept,
    // profiles/r06/early_dma_ab.txt.)
    desc(g, rs);
    issue(rs, so, P, true);
    issue(rs, so, P ^ 1, true);
    // Everything else of the prologue runs while the first two lines are in flight: without the
    // barrier hipcc hoisted the window tables (~300 VALU) above the first DMA.
    __builtin_amdgcn_sched_barrier(0);
    uint64_t gn = take();                                      // the group after g
    {
        const uint32_t sh4 = (o0 + lane * rec_len) & 127;      // 4 x the record's dword shift
        // Stream dword q = sh + i sits at row byte ((4q mod 128) ^ 16 swz) of slot q >= 32: with
        // fr = row base | 16 swz (disjoint bits), one xor, one or and the slot bit.
        const uint32_t fr = (my_off + lane * 128) | (swz(lane) << 4);
#pragma unroll
        for (uint32_t i = 0; i < 32; i++) {
            const uint32_t q4 = sh4 + 4 * i;                   // < 256
            ae[i] = ((q4 & 124u) ^ fr) | ((q4 & 128u) << 6);   // SLOT = 128 << 6
            ao[i] = ae[i] ^ SLOT;                              // slot 0 has bit 13 clear
            asm volatile("" : "+v"(ae[i]), "+v"(ao[i]));       // keep both tables in VGPRs
        }
    }
    uint32_t tm[16], tp[16];
    tail_masks(t, tm, tp);
    // One iteration k (1 <= k <= K): wait for line k, read the window (lines k-1, k), refill the
    // slot of line k-1 with line k+1 (at k = K: start the next group's lines 0 and 1), hash blocks
    // 2k-2 and 2k-1.  Iterations k < K always refill and always hash two whole blocks
    // (2k - 1 <= 2K - 3 < nfull), so they run branch-free in a loop unrolled by two (each parity
    // reads with its own address table: four compress sites, which the shared instruction cache
    // holds; unrolling the whole record did not fit).  With K even (P = 1) iteration 1
    // reads with "ao" and runs before the loop.  The last iteration is peeled: it alone starts the
    // next group and checks which blocks are whole.  Round 3: the peeled form issues ~18 fewer
    // scalar/branch instructions per iteration than one loop with the checks.
    auto full_step = [&](typename Alg::State &st, const uint32_t (&ad)[32], uint32_t refill_slot) {
        BRB_LINE_PROBE(1);
        brb_dma::wait_vmcnt<0>();
        read_window(ad);
        BRB_LINE_PROBE(2);
        issue(rs, so, refill_slot);
        // Without branches between the steps hipcc interleaved the compressions with the window
        // reads (one s_waitcnt per dword) and hoisted the next window read above them.
        __builtin_amdgcn_sched_barrier(0);
        Alg::compress(st, w0);
        Alg::compress(st, w1);
        __builtin_amdgcn_sched_barrier(0);
    };
    for (;;) {
        typename Alg::State st = Alg::iv();
        uint32_t k = 1;
        if (P) {                                               // K even: iteration 1 is odd-slotted
            full_step(st, ao, 1);
            k = 2;
        }
        for (; k + 2 <= K; k += 2) {
            full_step(st, ae, 0);                              // lines k-1, k in slots 0, 1: refill 0
            full_step(st, ao, 1);                              // lines k-1, k in slots 1, 0: refill 1
        }
        {   // iteration K: lines K-1, K in slots 0, 1
            BRB_LINE_PROBE(1);
            brb_dma::wait_vmcnt<0>();
            read_window(ae);
            BRB_LINE_PROBE(2);
            if (gn < n_groups) {
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
        line_finish<Alg, OUT_ALIGNED, TAIL_HI>(st, w0, w1, tm, tp, t, rec_len, out, g * 64 + lane, n_rec);
        g = gn;
        if (g >= n_groups)
            break;
        gn = take();
        rs = rsn;
        so = son;
    }
    BRB_LINE_PROBE(3);
}

// Line-aligned staging needs 4-byte record bases (the window shift is whole dwords).
inline bool line_supported(const uint8_t *data, uint32_t rec_len)
{
    return rec_len > 64 && rec_len <= (1u << 20) && (rec_len & 3) == 0 && (reinterpret_cast<uintptr_t>(data) & 3) == 0;
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

// One 8-wave workgroup per CU (128 KiB of LDS), persistent, groups handed out by tickets, DMA with
// the non-temporal policy past each group's first two lines.  Measured with tools/mb/md5_ab.hip,
// MD5, medians of 20-launch bursts:
//   1 Mi x 1500 B: 316 us static 4-wave workgroups -> 300 us (read floor of the same bytes: 261 us nt)
//   cfg2 65 536 x 1500 B: 25.3 us (record-relative 128-byte stages) -> 24.9 us
// (later rounds: DESIGN.md §4.1 and §5).
template <class Alg>
hipError_t launch_fixed_line(const uint8_t *data, uint32_t rec_len, uint64_t n_rec, uint8_t *out, bool out_al,
                             hipStream_t s)
{
    constexpr int W = 8;
    const uint64_t groups = (n_rec + 63) / 64;
    const unsigned g = unsigned(groups < device_cu_count() ? groups : device_cu_count());
    const bool hi = line_tail_hi(rec_len);
    if (out_al && hi)
        digest_line_kernel<Alg, W, true, true><<<g, 64 * W, 0, s>>>(data, rec_len, n_rec, out);
    else if (out_al)
        digest_line_kernel<Alg, W, true, false><<<g, 64 * W, 0, s>>>(data, rec_len, n_rec, out);
    else if (hi)
        digest_line_kernel<Alg, W, false, true><<<g, 64 * W, 0, s>>>(data, rec_len, n_rec, out);
    else
        digest_line_kernel<Alg, W, false, false><<<g, 64 * W, 0, s>>>(data, rec_len, n_rec, out);
    return hipGetLastError();
}

}  // namespace brb_digest
