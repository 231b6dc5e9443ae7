// line_stream.h -- per-lane byte streams staged through the line-aligned LDS-DMA ring, for the
// MD5 kernels whose message is a lane's own sequence of byte ranges: the segment lists of
// BRB_MD5BatchSegments (md5_seg_kernels.hip) and the item data of MetaData packs
// (metadata_kernels.hip; meta_data.c:145-290, 397-433).
//
// The fixed-stride and variable-length digests (digest_line.h, digest_var_line.h) stage a lane's
// record as 128-byte memory lines, 64 rows (one per lane) x one line per ring slot, by LDS-DMA
// (buffer_load_dwordx4 ... lds): no VGPRs in flight, whole lines requested once, the next line
// landing while the lane hashes the previous one.  Here a lane's lines form a VIRTUAL line sequence
// -- its segments' lines one after another (a segment's lines are contiguous in memory; the next
// segment's first line may be anywhere) -- so every stage gathers each row's next line offset
// from its lane (8 ds_bpermute) instead of advancing one shared descriptor.  The descriptor's base
// is 4 KiB below the group's lowest line; a group whose lines span 2 GiB or more (32-bit voffsets)
// takes the per-lane block path instead.
//
// Consumption: iteration k reads the 33-dword window of lines k-1 and k (slots (k-1) & 1, k & 1)
// and EMITS the message words of the lane's current range that start in line k-1, into the lane's
// 64-word funnel ring (md5_funnel.h FunnelT<64>); whole 16-word blocks are then compressed from the
// ring.  A range is read on a word grid that starts e = (message bytes before it) mod 4 bytes
// before the range (as the per-lane kernels do), so message words are one v_alignbit of two window
// dwords each and the first word's low e bytes are the carried ones (Funnel::head).  A word is
// emitted in the line that holds its first byte (a range's first word: in the line that holds the
// range's first byte), so at most 33 words leave one line, and a word that runs into line k reads
// it from the window (line k is the next line of the same range whenever a range continues).
#pragma once

#include "digest_line.h"
#include "md5_funnel.h"
#include "pair_sync.h"

namespace brb_line {

constexpr uint32_t kSlot = 8192;          // one ring slot: 64 rows x one 128-byte line
constexpr uint32_t kSlots = 3;            // line j in slot j % 3: line k+1 lands during line k-1's work
constexpr uint32_t kOOB = 0x80000000u;    // a voffset past every descriptor's range (DMA returns 0)
constexpr uint32_t kRingWords = 32;       // funnel ring words per lane (8 KiB per wave)

// A lane's view of its rows in the ring.  Row `lane` of a slot holds the lane's line at granule
// positions swizzled by swz(row) = (row >> 1) & 7 (applied on the DMA source side).  Every lane reads
// the same window granule at the same time (the window always starts at its line's first byte), so
// the window is read with ds_read_b128: per 16-lane group the granules sit in 16 distinct bank
// quads (rows alternate halves of the 64 banks, swz spreads the eight positions), conflict-free --
// with ds_read_b32 the 32 lanes of a group met on 8 banks (4-way: 3.2 M conflict cycles per launch,
// round-4 PMC), and 33 reads became 9.
struct Win {
    uint32_t fr;                               // the lane's row offset in a slot, OR its granule swizzle
    BRB_DEV void init(uint32_t lane)
    {
        fr = (lane * 128) | (((lane >> 1) & 7) << 4);
    }
    // window granule G (0..8) / dword j (0..63): line k-1 in the slot at LDS address sa, line k at sb
    BRB_DEV uint32_t granule(uint32_t G, uint32_t sa, uint32_t sb) const
    {
        return (((16 * G) & 112u) ^ fr) + (G < 8 ? sa : sb);
    }
    BRB_DEV uint32_t dword_addr(uint32_t j, uint32_t sa, uint32_t sb) const
    {
        return (((4 * j) & 124u) ^ fr) + (j < 32 ? sa : sb);
    }
};

BRB_DEV uint32_t lds_ld(uint32_t a) { return *reinterpret_cast<const __attribute__((address_space(3))) uint32_t *>(a); }

// The window's first 36 dwords (33 are used: line k-1 and line k's first dword); returns once they
// are in registers (lgkmcnt(0)), so the slot of line k-1 may be refilled right after.
BRB_DEV void read_window(const Win &w, uint32_t sa, uint32_t sb, uint32_t (&dw)[36])
{
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
#pragma unroll
    for (uint32_t G = 0; G < 9; G++) {
        const v4u v = *reinterpret_cast<const __attribute__((address_space(3))) v4u *>(w.granule(G, sa, sb));
        dw[4 * G + 0] = v.x;
        dw[4 * G + 1] = v.y;
        dw[4 * G + 2] = v.z;
        dw[4 * G + 3] = v.w;
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
}

// Window dword j (0..63) at a lane-varying j.
BRB_DEV uint32_t win_dword(const Win &w, uint32_t j, uint32_t sa, uint32_t sb)
{
    return lds_ld(w.dword_addr(j, sa, sb));
}

// Stage one line per row into the slot at LDS address `lm`: row r's line is `rel` of lane r
// (its offset from the group's lowest line, a multiple of 128), or kOOB for none.  DMA lane
// (q, l3 = lane >> 3) moves granule (lane & 7) ^ swz(row) of row 8q + l3's line; the descriptor's
// base is 4 KiB below the lowest line and four DMAs share one M0 through their instruction offsets.
// prep_rows gathers the rows' offsets (8 ds_bpermute) -- early, so their LDS round trip overlaps
// the wait for the current line; fire_rows issues the DMAs.
struct RowsV {
    uint32_t v[8];
};

// A row's offset is a multiple of 128 (a line) or kOOB, and its granule's byte offset is below 128,
// so the voffset is one add of a per-(q mod 4) lane constant; a kOOB row stays >= 2^31, past every
// descriptor's range (num_records <= 2^31 - 1), so its DMA still returns zeros -- no compare and
// select per DMA (round 5: 4 VALU -> 1 per DMA, 24 per line).
BRB_DEV RowsV prep_rows(uint32_t rel, uint32_t lane)
{
    const uint32_t l3 = lane >> 3;
    const uint32_t g0 = 16u * ((lane & 7) ^ (l3 >> 1));   // swz(8q + l3) = (l3 >> 1) ^ 4 (q & 1)
    RowsV r;
#pragma unroll
    for (int q = 0; q < 8; q++) {
        const uint32_t rr = uint32_t(__builtin_amdgcn_ds_bpermute(int(8 * q + l3) * 4, int(rel)));
        r.v[q] = rr + ((q & 1 ? g0 ^ 64u : g0) + (4096u - 1024u * (q & 3)));
    }
    return r;
}

BRB_DEV void fire_rows(const brb_dma::v4i &rs, uint32_t lm_, const RowsV &r)
{
    const uint32_t lm = __builtin_amdgcn_readfirstlane(lm_);   // wave-uniform; says so to the compiler
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\t"
                 "s_mov_b32 m0, %10\n\t"
                 "s_nop 0\n\t"
                 "buffer_load_dwordx4 %1, %9, 0 offen nt lds\n\t"
                 "buffer_load_dwordx4 %2, %9, 0 offen offset:1024 nt lds\n\t"
                 "buffer_load_dwordx4 %3, %9, 0 offen offset:2048 nt lds\n\t"
                 "buffer_load_dwordx4 %4, %9, 0 offen offset:3072 nt lds\n\t"
                 "s_mov_b32 m0, %11\n\t"
                 "s_nop 0\n\t"
                 "buffer_load_dwordx4 %5, %9, 0 offen nt lds\n\t"
                 "buffer_load_dwordx4 %6, %9, 0 offen offset:1024 nt lds\n\t"
                 "buffer_load_dwordx4 %7, %9, 0 offen offset:2048 nt lds\n\t"
                 "buffer_load_dwordx4 %8, %9, 0 offen offset:3072 nt lds\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(r.v[0]), "v"(r.v[1]), "v"(r.v[2]), "v"(r.v[3]), "v"(r.v[4]), "v"(r.v[5]), "v"(r.v[6]),
                   "v"(r.v[7]), "s"(rs), "s"(lm), "s"(lm + 4096u)
                 : "memory");
}

BRB_DEV void issue_rows(const brb_dma::v4i &rs, uint32_t lm, uint32_t rel, uint32_t lane)
{
    fire_rows(rs, lm, prep_rows(rel, lane));
}

// Descriptor for a group whose lines lie in [lo, hi) (128-byte aligned absolute addresses).
BRB_DEV brb_dma::v4i group_rsrc(uint64_t lo, uint64_t hi)
{
    const uint64_t base = lo - 4096;
    const uint64_t left = hi - base;
    brb_dma::v4i r;
    r.x = __builtin_amdgcn_readfirstlane(int(uint32_t(base)));
    r.y = __builtin_amdgcn_readfirstlane(int(uint32_t(base >> 32) & 0xFFFF));
    r.z = __builtin_amdgcn_readfirstlane(int(left > 0x7FFFFFFFull ? 0x7FFFFFFFu : uint32_t(left)));
    r.w = 0x00020000;
    return r;
}

// The range a staged line belongs to, in offsets from the group's lowest line: the line itself, the
// range's first byte and its end.  line == kOOB: the lane has no line in this slot.
struct LineDesc {
    uint32_t line, ss, se;
};

// The message words of one range that start in the window's line k-1 (see the file comment), in
// line-relative byte coordinates:
//   first  the range starts in this line, at byte ss (0..127); else it started in an earlier line
//   endr   the range's end (exclusive), line-relative, > 0 (clamped: 4096 = "well past this line")
//   b      the lane's word-grid phase inside lines (0..3), set at the range's first line
// Word i (-1..31) of the line's grid = window bytes b + 4i .. + 3; words i0 <= i < iw are whole and
// go to ring position wpos0 + i - i0; when the range's last word starts in this line (ends), the
// bytes of a last partial word (word it) become the carry.  Emitted in two halves (i < 16, i >= 16)
// with the ring pumped between them, so a 32-word ring holds a line's words: before a half at most
// 15 words wait, a half adds at most 17.
// Every word of a half is written, unconditionally: a word before i0 to slot wpos0 (word i0
// overwrites it later in program order), a word past the range to the first slot after the half's
// words (free, and never one still waiting: a half that fills the ring has no such word) -- one
// v_med3 on the address instead of a branch per word.  The first word's carried bytes (head) and
// the last partial word (tail) are built once, from the two window dwords each reads back by
// address (edge_words) before the line's slot is refilled.
struct Emit {
    int i0, iw, it;
    uint32_t sh, hmask, carry, rem, wpos0, abase, alo;
    uint32_t head, tail;            // word i0 with the carried bytes in, word it (raw)
    bool ends, any;
};

template <uint32_t RW>
BRB_DEV void plan_range(const brb_md5::FunnelT<RW> &f, bool first, uint32_t ss, uint32_t endr, uint32_t &b, Emit &p)
{
    int o;                                                    // grid offset of the first word (-3..127)
    uint32_t e = 0;
    if (first) {
        e = f.nacc;
        o = int(ss) - int(e);
        b = uint32_t(o) & 3u;
    } else {
        o = int(b);
    }
    p.any = int(endr) > o;                                    // else its last word started in the line before
    p.i0 = o >> 2;                                            // -1 .. 31
    const int span = int(endr) - int(b);                      // > 4 i0 when any
    p.iw = span >> 2 < 32 ? span >> 2 : 32;                   // whole words: i0 <= i < iw
    p.ends = p.any && span <= 128;                            // the range's last word starts here
    p.rem = uint32_t(span) & 3u;                              // bytes of a last partial word
    p.it = span >> 2;                                         // its index (when ends && rem)
    p.sh = 8 * b;
    p.carry = uint32_t(f.acc);
    p.hmask = e ? (1u << (8 * e)) - 1u : 0u;
    p.wpos0 = f.wpos;
    if (!p.any) {                                             // nothing to write
        p.i0 = 0;
        p.iw = 0;
        p.it = -2;
    }
    p.abase = f.lane4 + ((f.wpos - uint32_t(p.i0)) << 8);
    p.alo = f.lane4 + (f.wpos << 8);
    p.head = 0;
    p.tail = 0;
}

// Words i0 and it of a planned range, from the window dwords by address (line k-1 at sa, line k at
// sb), before the slot of line k-1 is refilled.
BRB_DEV void edge_words(const Win &w, uint32_t sa, uint32_t sb, Emit &p)
{
    const uint32_t j0 = p.i0 < 0 ? 0u : uint32_t(p.i0);       // i0 = -1: the dword below the line holds
    const uint32_t jt = p.it < 0 ? 0u : p.it > 31 ? 31u : uint32_t(p.it);   // only carried bytes
    const uint32_t h1 = win_dword(w, uint32_t(p.i0 + 1), sa, sb);
    const uint32_t h0 = p.i0 < 0 ? h1 : win_dword(w, j0, sa, sb);
    const uint32_t t0 = win_dword(w, jt, sa, sb), t1 = win_dword(w, jt + 1, sa, sb);
    const uint32_t raw = __builtin_amdgcn_alignbit(h1, h0, p.sh);
    p.head = (raw & ~p.hmask) | (p.carry & p.hmask);
    p.tail = p.it == p.i0 ? p.head : __builtin_amdgcn_alignbit(t1, t0, p.sh);
}

// A line wholly inside the lane's current range, not its first line and not the line of its last
// word (the common case): 32 whole words, no head, no tail.
template <uint32_t RW>
BRB_DEV void plan_whole(const brb_md5::FunnelT<RW> &f, uint32_t b, Emit &p)
{
    p.any = true;
    p.i0 = 0;
    p.iw = 32;
    p.it = -2;
    p.ends = false;
    p.rem = 0;
    p.sh = 8 * b;
    p.carry = 0;
    p.hmask = 0;
    p.wpos0 = f.wpos;
    p.abase = f.lane4 + (f.wpos << 8);
    p.alo = p.abase;
    p.head = 0;
    p.tail = 0;
}

// Round 6: when no writing lane's half wraps around its ring, the words go
// out without the wrap mask -- a whole half as one base address and the ds_write instruction
// offsets (1 VALU per word: the funnel shift), a boundary half with the clamp on unmasked ring
// addresses (3 instead of 4).  Whether any lane wraps is one ballot per half (wave-uniform branch);
// with RW = 64 a whole half wraps in at most one of four consecutive halves.
template <uint32_t RW, int H, bool WHOLE>
BRB_DEV void emit_half(brb_md5::FunnelT<RW> &f, Emit &p, const uint32_t (&dw)[36])
{
    constexpr int lo = H ? 16 : -1, hi = H ? 32 : 16;
    constexpr uint32_t M = brb_md5::FunnelT<RW>::kMask;
    // words written after this half: [i0, min(iw, hi)); the first slot after them (a whole line:
    // words 0 .. 31, so 16 after the first half and 32 after the second)
    const int top = p.iw < hi ? p.iw : hi;
    const uint32_t n = WHOLE ? uint32_t(H ? 32 : 16) : uint32_t(top > p.i0 ? top - p.i0 : 0);
    const uint32_t ahi = p.alo + (n << 8);
    const uint32_t s0 = p.wpos0 & (RW - 1);                   // ring slot of word i0 (whole: word 0)
    if (WHOLE) {
        // this half's 16 words go to slots s0 + 16 H .. + 15
        const uint32_t s = (s0 + 16u * H) & (RW - 1);
        if (__builtin_amdgcn_ballot_w64(s > RW - 16) == 0) {
            const uint32_t base = f.ring | (f.lane4 + (s << 8));
#pragma unroll
            for (int i = lo < 0 ? 0 : lo; i < hi; i++)
                brb_md5::FunnelT<RW>::lds_st(base + uint32_t((i - (lo < 0 ? 0 : lo)) << 8),
                                             __builtin_amdgcn_alignbit(dw[i + 1], dw[i], p.sh));
            f.wpos = p.wpos0 + n;
            return;
        }
    } else if (__builtin_amdgcn_ballot_w64(s0 + n > RW - 1) == 0) {
        // slots s0 .. s0 + n (the last one the clamp's free slot) lie inside the ring: clamp on
        // unmasked addresses (signed: a word before i0 may compute below the ring's base)
        const int alo = int(f.ring | (f.lane4 + (s0 << 8)));
        const int ahi2 = alo + int(n << 8);
        const int abase = alo - (p.i0 << 8);
#pragma unroll
        for (int i = lo; i < hi; i++) {
            const uint32_t v = __builtin_amdgcn_alignbit(dw[i + 1], dw[i < 0 ? 0 : i], p.sh);
            int a = abase + (i << 8);
            asm("v_med3_i32 %0, %1, %2, %3" : "=v"(a) : "v"(a), "v"(alo), "v"(ahi2));   // before i0 -> wpos0, past the range -> free slot
            brb_md5::FunnelT<RW>::lds_st(uint32_t(a), v);
        }
        if (p.hmask && p.i0 >= lo && p.i0 < hi && p.i0 < p.iw)   // the head, over word i0's slot
            brb_md5::FunnelT<RW>::lds_st(uint32_t(alo), p.head);
        f.wpos = p.wpos0 + n;
        return;
    }
#pragma unroll
    for (int i = lo; i < hi; i++) {
        if (WHOLE && i < 0)
            continue;
        const uint32_t v = __builtin_amdgcn_alignbit(dw[i + 1], dw[i < 0 ? 0 : i], p.sh);
        uint32_t a = p.abase + uint32_t(i << 8);
        if (!WHOLE)
            asm("v_med3_u32 %0, %1, %2, %3" : "=v"(a) : "v"(a), "v"(p.alo), "v"(ahi));   // before i0 -> wpos0, past the range -> free slot (alo <= ahi)
        brb_md5::FunnelT<RW>::lds_st((a & M) | f.ring, v);
    }
    if (!WHOLE && p.hmask && p.i0 >= lo && p.i0 < hi && p.i0 < p.iw)   // the head, over word i0's slot
        brb_md5::FunnelT<RW>::lds_st((p.alo & M) | f.ring, p.head);
    f.wpos = p.wpos0 + n;
}

template <uint32_t RW>
BRB_DEV void emit_finish(brb_md5::FunnelT<RW> &f, const Emit &p)
{
    if (p.ends) {
        f.nacc = p.rem;
        f.acc = p.rem ? (p.tail & ((1u << (8 * p.rem)) - 1u)) : 0u;
    }
}

// ---- producer / consumer wave pairs (md5_seg_pc_kernel, metadata_line_kernel<..., PC>) ----------
// A pair's two waves share a funnel ring: the producer stages lines and emits message words, the
// consumer compresses them (pair_sync.h for the hand-off primitives).

// Producer side, per lane: wait until the lane's ring has room for a half-line of words (at most
// 17, plus the free slot past them that emit_half's clamp may write): wpos - cpos <= RW - 18, cpos
// being the consumer's published count of compressed words.  Lanes that will not write pass.
template <uint32_t RW>
BRB_DEV bool pc_room(uint32_t *cpx, uint32_t wpos, bool writes, uint64_t *idle = nullptr)
{
    for (uint32_t spin = 0; spin < (1u << 22); spin++) {
        const bool full = writes && wpos - pc_load(cpx) > RW - 18;
        if (__builtin_amdgcn_ballot_w64(full) == 0)
            return true;
        const uint64_t t = idle ? __builtin_amdgcn_s_memtime() : 0;
        __builtin_amdgcn_s_sleep(1);
        if (idle)
            *idle += __builtin_amdgcn_s_memtime() - t;
    }
    return false;
}

// Compresses every whole block waiting in the ring (one compress site per call; at most two blocks
// wait after a half).
template <uint32_t RW>
BRB_DEV void pump_all(brb_md5::FunnelT<RW> &f)
{
    while (f.wpos - f.cpos >= 16)
        f.pump();
}

// One line's emission in two halves (the range planned in e).  Alone (PC = false): whole blocks are
// compressed after each half (a 32-word ring).  Producer (PC = true): before each half, room in the
// pair's ring (pc_room); after it, the word count posted to the consumer (wpx).  `writes`: this lane
// has words in the line.  False when a wait timed out.
template <uint32_t RW, bool WHOLE, bool PC>
BRB_DEV bool emit_line(brb_md5::FunnelT<RW> &f, Emit &e, const uint32_t (&dw)[36], bool writes, uint32_t *cpx,
                       uint32_t *wpx, uint64_t *idle = nullptr)
{
    if (PC && !pc_room<RW>(cpx, f.wpos, writes, idle))
        return false;
    if (writes)
        emit_half<RW, 0, WHOLE>(f, e, dw);
    if (PC)
        pc_publish(wpx, f.wpos);
    else
        pump_all(f);
    if (PC && !pc_room<RW>(cpx, f.wpos, writes, idle))
        return false;
    if (writes) {
        emit_half<RW, 1, WHOLE>(f, e, dw);
        emit_finish(f, e);
    }
    if (PC)
        pc_publish(wpx, f.wpos);
    else
        pump_all(f);
    return true;
}

// Consumer: compresses the lane's words as the producer posts them (wpx), posting its own count
// (cpx), until the producer's event count reaches `end` (its last post is in by then).  False when
// the producer stopped (2^22 sleeps with no word, no end and no beat of hb: a protocol fault; the
// launch's digests are then wrong, but it ends, and the caller reports it: pair_fault.h).
template <uint32_t RW>
BRB_DEV bool pc_consume(brb_md5::FunnelT<RW> &f, uint32_t *ev_p, uint32_t end, uint32_t *wpx, uint32_t *cpx,
                        uint32_t *hb, uint64_t *idle = nullptr)
{
    uint32_t last = pc_beat_of(hb);
    for (uint32_t spin = 0; spin < (1u << 22); spin++) {
        const bool ended = __builtin_amdgcn_readfirstlane(pc_load(ev_p)) >= end;   // before wpos: the last post is in
        f.wpos = pc_load(wpx);
        if (__builtin_amdgcn_ballot_w64(f.wpos - f.cpos >= 16) != 0) {
            pump_all(f);
            pc_publish(cpx, f.cpos);
            spin = 0;
        } else if (ended) {
            return true;
        } else {
            const uint32_t h = pc_beat_of(hb);
            if (h != last) {
                last = h;
                spin = 0;
            }
            const uint64_t t = idle ? __builtin_amdgcn_s_memtime() : 0;
            __builtin_amdgcn_s_sleep(1);
            if (idle)
                *idle += __builtin_amdgcn_s_memtime() - t;
        }
    }
    return false;
}

}  // namespace brb_line
