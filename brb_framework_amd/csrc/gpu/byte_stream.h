// byte_stream.h -- per-lane sequential access to byte ranges at arbitrary addresses.
//
// Records, streams and segments start at any byte offset.  Src reads a range as 4-byte chunks
// using aligned dword loads and a funnel shift (v_alignbit_b32), loading each dword once; Snk
// writes a range as 4-byte chunks with aligned dword stores and byte stores only for the partial
// dwords at its two ends.  Neither touches a dword that holds none of the range's bytes, so ranges
// packed back to back are safe to process from different lanes at once.
#pragma once

#include "brb_gpu_common.h"

namespace brb_io {

// Sequential 4-byte chunks of a byte range at any address; bytes past the range read as 0.
struct Src {
    const uint32_t *p;
    uint32_t sh;     // 8 * (address & 3)
    uint32_t lo;     // dword at p
    uint64_t rem;    // bytes left from the current position

    BRB_DEV void init(const uint8_t *a, uint64_t n)
    {
        const uintptr_t ad = reinterpret_cast<uintptr_t>(a);
        p = reinterpret_cast<const uint32_t *>(ad & ~uintptr_t(3));
        sh = uint32_t(ad & 3) * 8;
        rem = n;
        lo = n ? ldg(p) : 0u;
    }

    BRB_DEV uint32_t next()
    {
        const uint32_t o = sh >> 3;
        const uint32_t hi = rem > 4 - o ? ldg(p + 1) : 0u;     // the next dword holds a byte of the range
        uint32_t v = __builtin_amdgcn_alignbit(hi, lo, sh);
        if (rem < 4)
            v &= (1u << (8 * uint32_t(rem))) - 1u;
        ++p;
        lo = hi;
        rem = rem > 4 ? rem - 4 : 0;
        return v;
    }
};

// Sequential 4-byte chunks into a byte range at any address (exactly `n` bytes are written).
struct Snk {
    uint32_t *p;
    uint32_t o;        // address & 3
    uint32_t carry;    // bytes of the dword at p that the previous chunk produced (positions 0..o-1)
    uint32_t carry_n;
    uint64_t rem;
    bool first;

    BRB_DEV void init(uint8_t *a, uint64_t n)
    {
        const uintptr_t ad = reinterpret_cast<uintptr_t>(a);
        p = reinterpret_cast<uint32_t *>(ad & ~uintptr_t(3));
        o = uint32_t(ad & 3);
        carry = 0;
        carry_n = 0;
        rem = n;
        first = true;
    }

    static BRB_DEV void part(uint32_t *q, uint32_t w, uint32_t lo, uint32_t hi)
    {
        if (lo == 0 && hi == 3) {
            stg(q, w);
            return;
        }
        uint8_t *b = reinterpret_cast<uint8_t *>(q);
        for (uint32_t k = lo; k <= hi; k++)
            stg8(b + k, w >> (8 * k));
    }

    BRB_DEV void put(uint32_t v)
    {
        if (rem == 0)
            return;
        const uint32_t n = rem < 4 ? uint32_t(rem) : 4u;
        const uint32_t w0 = o ? (carry | (v << (8 * o))) : v;
        const uint32_t hi = o + n - 1 < 3 ? o + n - 1 : 3u;
        part(p, w0, first ? o : 0u, hi);
        carry = o ? (v >> (32 - 8 * o)) : 0u;
        carry_n = o + n > 4 ? o + n - 4 : 0u;
        ++p;
        first = false;
        rem -= n;
    }

    BRB_DEV void flush()
    {
        if (carry_n)
            part(p, carry, 0, carry_n - 1);
        carry_n = 0;
    }

    // 16 chunks, the same bytes as 16 put() calls.  Past the range's first dword and with at least
    // 64 bytes left, every destination dword is whole: they are written as four 16-byte stores at
    // 4-byte alignment (gfx950 runs in unaligned-access mode) instead of 16 dword stores.  Dword
    // stores scattered one per lane over 64 lines left a 65 536-stream RC4 pass at 133 us of pure
    // stream I/O per 98 MB each way; 16-byte stores, 54 us (tools/mb/rc4_parts.hip).
    BRB_DEV void put16(const uint32_t (&v)[16])
    {
        if (first || rem < 64) {
#pragma unroll
            for (int k = 0; k < 16; k++)
                put(v[k]);
            return;
        }
        // out_k = (v_k << 8 o) | (v_{k-1} >> (32 - 8 o)) as one v_perm_b32: byte b of the result is
        // byte 4 + b - o of {v_k : v_{k-1}} (selector values 4..7 pick v_k, 1..3 pick v_{k-1})
        const uint32_t sel = 0x07060504u - 0x01010101u * o;
        uint32_t w[16];
        uint32_t prev = o ? carry << (8 * (4 - o)) : 0u;   // the carried bytes on top of a virtual v_{-1}
#pragma unroll
        for (int k = 0; k < 16; k++) {
            w[k] = __builtin_amdgcn_perm(v[k], prev, sel);
            prev = v[k];
        }
#pragma unroll
        for (int q = 0; q < 4; q++)
            st16_a4(reinterpret_cast<uint8_t *>(p + 4 * q), w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
        p += 16;
        carry = o ? (v[15] >> (32 - 8 * o)) : 0u;
        carry_n = o;
        rem -= 64;
    }
};

// Snk whose middle goes out as whole, aligned 64-byte memory sectors.  A stream starting at a
// 4-byte offset inside a sector writes each sector in two pieces one 64-byte block apart (with
// Snk::put16: four 16-byte stores at the stream's own alignment), and the L2 wrote most of them
// back to HBM twice: the RC4 pass wrote 190.9 MB for 115.6 MB of output (profiles/
// r01_pmc_f1_rc4.txt).  Here put16's memory-aligned dwords go into the lane's LDS row -- two
// sectors, circular by absolute dword index -- and the sector the block completes is read back with
// four ds_read_b128 and stored with four aligned 16-byte stores.  The stream's first partial sector
// (shared with the previous stream) is stored dword by dword, and the dwords left in the row are
// stored dword by dword before the byte-exact tail (drain).  Rows are 144 bytes apart (36 banks):
// lanes writing the same row position meet at most 4-way.
struct SectorSnk {
    static constexpr uint32_t kRowBytes = 144;
    Snk s;                     // the byte-exact ends and the current position
    uint32_t ta[16], tb[16];   // LDS addresses of row positions (u + i) & 31 for (u & 16) = 0 / 16
    uint32_t rowb;             // LDS address of the row
    uint32_t pend;             // dwords in the row not yet stored (0..15), ending at the position u
    bool whole;                // the pending dwords start at a sector boundary (not the stream's first)

    // `row` = this lane's 144-byte LDS row (16-byte aligned), as an LDS address
    BRB_DEV void init(uint8_t *a, uint64_t n, uint32_t row)
    {
        s.init(a, n);
        rowb = row;
        pend = 0;
        whole = false;
        const uint32_t d = uint32_t(reinterpret_cast<uintptr_t>(s.p) >> 2) & 15;
#pragma unroll
        for (uint32_t i = 0; i < 16; i++) {
            ta[i] = row + 4 * ((d + i) & 31);
            tb[i] = row + 4 * ((d + 16 + i) & 31);
        }
    }

    static BRB_DEV uint32_t lds_ld(uint32_t a) { return *reinterpret_cast<const __attribute__((address_space(3))) uint32_t *>(a); }
    static BRB_DEV void lds_st(uint32_t a, uint32_t v) { *reinterpret_cast<__attribute__((address_space(3))) uint32_t *>(a) = v; }

    // stores the `pend` dwords before the current position that are only in the row
    BRB_DEV void drain()
    {
        const uint32_t u = uint32_t(reinterpret_cast<uintptr_t>(s.p) >> 2);
#pragma unroll
        for (uint32_t i = 1; i <= 15; i++)
            if (i <= pend)
                stg(s.p - i, lds_ld(rowb + 4 * ((u - i) & 31)));
        pend = 0;
    }

    BRB_DEV void put(uint32_t v)
    {
        if (pend)
            drain();
        s.put(v);
    }

    BRB_DEV void flush()
    {
        if (pend)
            drain();
        s.flush();
    }

    BRB_DEV void put16(const uint32_t (&v)[16])
    {
        if (s.first || s.rem < 64) {
#pragma unroll
            for (int k = 0; k < 16; k++)
                put(v[k]);
            return;
        }
        const uint32_t o = s.o;
        const uint32_t sel = 0x07060504u - 0x01010101u * o;    // as Snk::put16
        uint32_t w[16];
        uint32_t prev = o ? s.carry << (8 * (4 - o)) : 0u;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            w[k] = __builtin_amdgcn_perm(v[k], prev, sel);
            prev = v[k];
        }
        const uint32_t u = uint32_t(reinterpret_cast<uintptr_t>(s.p) >> 2);   // absolute dword index
        if (u & 16) {
#pragma unroll
            for (int i = 0; i < 16; i++)
                lds_st(tb[i], w[i]);
        } else {
#pragma unroll
            for (int i = 0; i < 16; i++)
                lds_st(ta[i], w[i]);
        }
        // the sector holding dword u is complete: its dwords before u came with the previous block
        // (pend of them; none of a stream's first sector went through the row)
        const uint32_t d = u & 15;
        const uint32_t half = rowb + 64 * ((u >> 4) & 1);
        uint32_t *sec = s.p - d;
        if (whole || d == 0) {
#pragma unroll
            for (uint32_t q = 0; q < 4; q++) {
                typedef uint32_t v4u __attribute__((ext_vector_type(4)));
                const v4u x = *reinterpret_cast<const __attribute__((address_space(3))) v4u *>(half + 16 * q);
                st16_a4(reinterpret_cast<uint8_t *>(sec + 4 * q), x.x, x.y, x.z, x.w);
            }
        } else {
#pragma unroll
            for (uint32_t i = 0; i < 16; i++)
                if (i >= d)
                    stg(sec + i, lds_ld(half + 4 * i));
        }
        whole = true;
        pend = d;
        s.p += 16;
        s.carry = o ? (v[15] >> (32 - 8 * o)) : 0u;
        s.carry_n = o;
        s.rem -= 64;
    }
};

// 64-byte blocks of a byte range at any address, the next block always in flight: a lane that
// consumes one block per few thousand cycles (RC4, a digest) never waits on HBM latency.  Block b
// is 16 little-endian chunks, chunk i = range bytes 64 b + 4 i .. + 3; bytes past the range are 0.
// Loads are aligned-dword based (4 x global_load_dwordx4 at 4-byte alignment for a block that lies
// inside the range's dwords, guarded single dwords at the end), funnel-shifted with v_alignbit_b32.
struct BlockSrc {
    const uint32_t *p;   // dword holding the range's first byte
    uint32_t sh;         // 8 * (address & 3)
    uint64_t len, ndw;   // range bytes; dwords holding any of them
    uint64_t nb;         // block returned by the next fetch()
    uint32_t prev;       // dword 16 nb (last dword of the previous load)
    uint32_t L[16];      // dwords 16 nb + 1 .. 16 nb + 16, in flight

    BRB_DEV void load(uint64_t b)
    {
        const uint64_t base = 16 * b + 1;
        if (base + 16 <= ndw) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint4 v = ld16_a4(reinterpret_cast<const uint8_t *>(p + base + 4 * q));
                L[4 * q + 0] = v.x;
                L[4 * q + 1] = v.y;
                L[4 * q + 2] = v.z;
                L[4 * q + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; i++)
                L[i] = base + i < ndw ? ldg(p + base + i) : 0u;
        }
    }

    // `lo` (optional): the range's bytes below lo are not memory to read (md5_seg_kernel starts a
    // segment's range up to 3 bytes early and overwrites those bytes); a first dword wholly below
    // lo's dword reads as 0.  Only that dword can lie below: load() starts at dword 1.
    BRB_DEV void init(const uint8_t *a, uint64_t n, const uint8_t *lo = nullptr)
    {
        const uintptr_t ad = reinterpret_cast<uintptr_t>(a);
        p = reinterpret_cast<const uint32_t *>(ad & ~uintptr_t(3));
        sh = uint32_t(ad & 3) * 8;
        len = n;
        ndw = n ? ((ad & 3) + n + 3) / 4 : 0;
        const bool below = lo && (ad & ~uintptr_t(3)) < (reinterpret_cast<uintptr_t>(lo) & ~uintptr_t(3));
        prev = ndw && !below ? ldg(p) : 0u;
        nb = 0;
        load(0);
    }

    // chunks of block nb; starts the load of block nb + 1.  The block in flight is consumed BEFORE
    // the next load is issued: the two load paths (whole block / guarded dwords) leave hipcc unsure
    // of the pending count, and a wait placed after the new load would wait for it too (one HBM
    // round trip per block: 98 -> 138 us for 65 536 RC4 streams of 1500 B).
    BRB_DEV void fetch(uint32_t (&c)[16])
    {
#pragma unroll
        for (int i = 0; i < 16; i++)
            c[i] = __builtin_amdgcn_alignbit(L[i], i ? L[i - 1] : prev, sh);
        prev = L[15];
        const uint64_t pos = 64 * nb;
        if (pos + 64 > len) {
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const uint64_t q = pos + 4 * i;
                c[i] = q >= len ? 0u : q + 4 <= len ? c[i] : c[i] & ((1u << (8 * uint32_t(len - q))) - 1u);
            }
        }
        ++nb;
        load(nb);
    }
};

// BlockSrc for a whole wave: the same blocks, loaded cooperatively.  Instruction q of a load moves
// the blocks of lanes 16q .. 16q+15, four lanes per block (16 bytes each), so one instruction
// touches 16 memory lines instead of 64; the blocks are handed to their lanes through a 4 KiB LDS
// exchange per wave.  A per-lane load of 64 scattered 16-byte pieces keeps the texture path busy for
// ~150 cycles per instruction, and a lone wave per SIMD waits on it: 65 536 RC4 streams x 1536 B,
// 121 -> 111 us per pass (tools/mb/rc4_parts.hip).
// init() and fetch() must be called by all 64 lanes of the wave in uniform control flow, the same
// number of times; a lane with a shorter (or empty) range receives zero blocks past its end.
struct BlockSrcW {
    const uint32_t *p;   // dword holding the range's first byte
    uint32_t sh;         // 8 * (address & 3)
    uint64_t len, ndw;   // range bytes; dwords holding any of them
    uint64_t nb;         // block returned by the next fetch()
    uint32_t prev;       // dword 16 nb of this lane's range
    uint8_t *xw;         // this wave's exchange rows: row r = lane r's block
    uint32_t lane;
    uint64_t qa[4];      // address of dword 1 + 4 (lane & 3) of the range of lane 16q + lane / 4
    uint64_t qrem[4];    // dwords of that range from there on
    uint4 v[4];          // in flight: chunk lane & 3 of block nb of lane 16q + lane / 4

    // chunk c of row r sits at 16 ((c + (r >> 2)) & 3): the row-wise reads and the chunk-wise
    // writes are both free of bank conflicts
    static BRB_DEV uint32_t xoff(uint32_t r, uint32_t c) { return r * 64 + 16 * ((c + (r >> 2)) & 3); }

    BRB_DEV void issue(uint64_t b)
    {
        const uint64_t base = 16 * b;
        // the common block: every chunk this lane loads lies inside its range -- four plain loads
        // behind one branch, as StepSrcW::issue (RC4 pass 118.1 -> 115.4 us)
        if (base + 4 <= qrem[0] && base + 4 <= qrem[1] && base + 4 <= qrem[2] && base + 4 <= qrem[3]) {
#pragma unroll
            for (int q = 0; q < 4; q++)
                v[q] = ld16_a4(reinterpret_cast<const uint8_t *>(qa[q] + 4 * base));
            return;
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (base + 4 <= qrem[q]) {
                v[q] = ld16_a4(reinterpret_cast<const uint8_t *>(qa[q] + 4 * base));
            } else {
                const uint32_t *d = reinterpret_cast<const uint32_t *>(qa[q]) + base;
                v[q].x = base + 0 < qrem[q] ? ldg(d + 0) : 0u;
                v[q].y = base + 1 < qrem[q] ? ldg(d + 1) : 0u;
                v[q].z = base + 2 < qrem[q] ? ldg(d + 2) : 0u;
                v[q].w = base + 3 < qrem[q] ? ldg(d + 3) : 0u;
            }
        }
    }

    BRB_DEV void init(const uint8_t *a, uint64_t n, uint8_t *exchange)
    {
        const uintptr_t ad = reinterpret_cast<uintptr_t>(a);
        p = reinterpret_cast<const uint32_t *>(ad & ~uintptr_t(3));
        sh = uint32_t(ad & 3) * 8;
        len = n;
        ndw = n ? ((ad & 3) + n + 3) / 4 : 0;
        prev = ndw ? ldg(p) : 0u;
        nb = 0;
        xw = exchange;
        lane = threadIdx.x & 63;
        const uint64_t pa = reinterpret_cast<uint64_t>(p);
        const uint32_t c = lane & 3;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int src = 16 * q + int(lane >> 2);
            const uint64_t a_r = (uint64_t(uint32_t(__shfl(int(pa >> 32), src))) << 32) | uint32_t(__shfl(int(uint32_t(pa)), src));
            const uint64_t n_r = (uint64_t(uint32_t(__shfl(int(ndw >> 32), src))) << 32) | uint32_t(__shfl(int(uint32_t(ndw)), src));
            qa[q] = a_r + 4 * (1 + 4 * c);
            qrem[q] = n_r > 1 + 4 * c ? n_r - 1 - 4 * c : 0;
        }
        issue(0);
    }

    BRB_DEV void fetch(uint32_t (&c)[16])
    {
#pragma unroll
        for (int q = 0; q < 4; q++)
            *reinterpret_cast<uint4 *>(xw + xoff(16 * q + (lane >> 2), lane & 3)) = v[q];
        uint32_t L[16];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint4 t = *reinterpret_cast<const uint4 *>(xw + xoff(lane, k));
            L[4 * k] = t.x;
            L[4 * k + 1] = t.y;
            L[4 * k + 2] = t.z;
            L[4 * k + 3] = t.w;
        }
#pragma unroll
        for (int i = 0; i < 16; i++)
            c[i] = __builtin_amdgcn_alignbit(L[i], i ? L[i - 1] : prev, sh);
        prev = L[15];
        const uint64_t pos = 64 * nb;
        if (pos + 64 > len) {
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const uint64_t q = pos + 4 * i;
                c[i] = q >= len ? 0u : q + 4 <= len ? c[i] : c[i] & ((1u << (8 * uint32_t(len - q))) - 1u);
            }
        }
        ++nb;
        issue(nb);
    }
};

// The 0x80 end marker of MD5 / SHA-1 padding at byte len % 64 of a (zero-filled) tail block.
BRB_DEV void add_marker(uint32_t (&w)[16], uint64_t len)
{
    const uint32_t t = uint32_t(len & 63), m = 0x80u << (8 * (t & 3));
#pragma unroll
    for (uint32_t i = 0; i < 16; i++)
        w[i] |= i == (t >> 2) ? m : 0u;
}

}  // namespace brb_io
