// rc4_device.h -- device code of the batched RC4 and RC4+MD5 framing kernels.
//
// RC4 (libbrb_core/crypto/rc4.c:64-87) is a byte-serial chain over a 256-byte permutation that
// every byte mutates, so the parallelism is across connections: one lane owns one stream, and the
// 64 lanes of a wave keep their 64 permutations in one 16 KiB LDS slot laid out so that every access
// of lane l lands in bank l, whatever the index:
//
//   byte x of lane l's permutation  ->  LDS byte (x >> 2) * 256 + l * 4 + (x & 3)
//
// (64 rows of one dword per lane).  Random indices therefore never conflict.  Per keystream byte:
// S[j] is the only read on the dependency chain; S[i + 1] is read ahead before the swap is written
// and patched when the swap moved it (j == i + 1); S[S[i] + S[j]] is read after the swap.
//
// Memory side: streams start at arbitrary byte offsets, so inputs are read as aligned dwords and
// funnel-shifted (Src), outputs are written as aligned dwords with byte stores only for the partial
// dwords at the two ends of a stream (Snk).  No access touches a dword that holds none of the
// stream's bytes, so streams packed back to back never race.
#pragma once

#include "brb_gpu_common.h"
#include "md5_device.h"

namespace brb_rc4 {

constexpr uint32_t kStateBytes = 264;   // sizeof(BRB_RC4_State), libbrb_data.h:887-897
constexpr uint32_t kWaveLds = 16384;    // 64 lanes x 256-byte permutation
constexpr uint32_t kHeader = 30;        // salt(8) "HASH:"(5) MD5(16) NUL(1), ev_kq_aio_transform.c:224-227

struct Perm {
    uint8_t *lds;   // the wave's 16 KiB slot
    uint32_t lb;    // lane * 4

    BRB_DEV uint32_t addr(uint32_t x) const { return ((x << 6) & 0x3F00u) | (x & 3u) | lb; }
    BRB_DEV uint32_t rd(uint32_t x) const { return lds[addr(x)]; }
    BRB_DEV void wr(uint32_t x, uint32_t v) const { lds[addr(x)] = uint8_t(v); }
    BRB_DEV uint32_t &row(uint32_t k) const { return *reinterpret_cast<uint32_t *>(lds + (k << 8) + lb); }
};

// Keystream generator: BRB_RC4_Crypt's index1/index2 walk (rc4.c:71-82).
struct Gen {
    Perm P;
    uint32_t i, j;   // index1, index2
    uint32_t si;     // S[(i + 1) & 255], read ahead
    uint32_t tail;   // dword 64 of the state: index1, index2 and the two bytes after them

    // BRB_RC4_State (4-byte aligned) -> LDS slot + registers
    BRB_DEV void load(const uint8_t *st)
    {
        const uint32_t *w = reinterpret_cast<const uint32_t *>(st);
#pragma unroll 8
        for (uint32_t k = 0; k < 64; k++)
            P.row(k) = w[k];
        tail = w[64];
        i = tail & 255u;
        j = (tail >> 8) & 255u;
        si = P.rd((i + 1) & 255u);
    }

    BRB_DEV void store(uint8_t *st) const
    {
        uint32_t *w = reinterpret_cast<uint32_t *>(st);
#pragma unroll 8
        for (uint32_t k = 0; k < 64; k++)
            w[k] = P.row(k);
        w[64] = (tail & 0xFFFF0000u) | (j << 8) | i;
    }

    BRB_DEV uint32_t next()
    {
        i = (i + 1) & 255u;
        const uint32_t a = si;                      // S[i]
        j = (j + a) & 255u;
        const uint32_t b = P.rd(j);                 // S[j]
        const uint32_t i1 = (i + 1) & 255u;
        const uint32_t n = P.rd(i1);                // S[i + 1] before the swap
        P.wr(i, b);
        P.wr(j, a);
        const uint32_t k = P.rd((a + b) & 255u);    // S[S[i] + S[j]] after the swap
        si = i1 == j ? a : n;
        return k;
    }

    BRB_DEV uint32_t next4()
    {
        const uint32_t b0 = next(), b1 = next(), b2 = next(), b3 = next();
        return b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
    }

    // nb (0..4) keystream bytes, little-endian in the low bytes; the state advances by exactly nb
    BRB_DEV uint32_t next_n(uint32_t nb)
    {
        if (nb >= 4)
            return next4();
        uint32_t v = 0;
        for (uint32_t b = 0; b < nb; b++)
            v |= next() << (8 * b);
        return v;
    }
};

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
        lo = n ? p[0] : 0u;
    }

    BRB_DEV uint32_t next()
    {
        const uint32_t o = sh >> 3;
        const uint32_t hi = rem > 4 - o ? p[1] : 0u;     // the next dword holds a byte of the range
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
            *q = w;
            return;
        }
        uint8_t *b = reinterpret_cast<uint8_t *>(q);
        for (uint32_t k = lo; k <= hi; k++)
            b[k] = uint8_t(w >> (8 * k));
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
};

// Word w of the MD5-padded message of `len` bytes, given the raw data word (zeros past the end).
BRB_DEV uint32_t md5_pad_word(uint32_t raw, uint64_t w, uint64_t len, uint64_t n_words)
{
    uint32_t v = raw;
    if (w == (len >> 2))
        v |= 0x80u << (8 * uint32_t(len & 3));
    if (w == n_words - 2)
        v = uint32_t(len << 3);
    if (w == n_words - 1)
        v = uint32_t(len >> 29);
    return v;
}

// number of 64-byte MD5 blocks of a `len`-byte message including the padding
BRB_DEV uint64_t md5_blocks(uint64_t len) { return (len + 72) >> 6; }

}  // namespace brb_rc4
