// rc4_device.h -- device code of the batched RC4 and RC4+MD5 framing kernels.
//
// RC4 (libbrb_core/crypto/rc4.c:64-87) is a byte-serial chain over a 256-byte permutation that
// every byte mutates, so the parallelism is across connections: one lane owns one stream.  A
// workgroup of 4 waves keeps its 256 permutations in one 64 KiB LDS image laid out so that every
// access of lane l lands in bank l, whatever the index, and costs one VALU op to address:
//
//   byte x of the permutation of (wave w, lane l)  ->  LDS byte  x * 256 + l * 4 + w
//
// (256 rows, one dword per lane, one byte of it per wave).  Random indices never conflict, and an
// address is a single v_lshl_or_b32 of the 8-bit index.  Per keystream byte: S[j] is the only read
// on the dependency chain; S[i + 1] is read ahead before the swap is written and patched when the
// swap moved it (j == i + 1); S[S[i] + S[j]] is read after the swap.
//
// Memory side: byte_stream.h (aligned-dword Src / Snk for streams at arbitrary byte offsets).
#pragma once

#include "brb_gpu_common.h"
#include "byte_stream.h"
#include "md5_device.h"

namespace brb_rc4 {

using brb_io::Snk;
using brb_io::Src;

constexpr uint32_t kStateBytes = 264;   // sizeof(BRB_RC4_State), libbrb_data.h:887-897
constexpr uint32_t kWaves = 4;          // waves per workgroup
constexpr uint32_t kSlotLds = 65536;    // 256 rows x 64 lanes x 4 waves
constexpr uint32_t kHeader = 30;        // salt(8) "HASH:"(5) MD5(16) NUL(1), ev_kq_aio_transform.c:224-227

struct Perm {
    uint8_t *lds;   // the workgroup's 64 KiB image
    uint32_t lw;    // lane * 4 + wave

    BRB_DEV uint32_t addr(uint32_t x) const { return (x << 8) | lw; }
    BRB_DEV uint32_t rd(uint32_t x) const { return lds[addr(x)]; }
    BRB_DEV void wr(uint32_t x, uint32_t v) const { lds[addr(x)] = uint8_t(v); }
};

// Keystream generator: BRB_RC4_Crypt's index1/index2 walk (rc4.c:71-82).
struct Gen {
    Perm P;
    uint32_t i, j;   // index1, index2
    uint32_t si;     // S[(i + 1) & 255], read ahead
    uint32_t tail;   // dword 64 of the state: index1, index2 and the two bytes after them

    // BRB_RC4_State (4-byte aligned) -> LDS image + registers
    BRB_DEV void load(const uint8_t *st)
    {
        const uint32_t *w = reinterpret_cast<const uint32_t *>(st);
#pragma unroll 8
        for (uint32_t k = 0; k < 64; k++) {
            const uint32_t v = w[k];
#pragma unroll
            for (uint32_t b = 0; b < 4; b++)
                P.wr(4 * k + b, v >> (8 * b));
        }
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
            w[k] = P.rd(4 * k) | (P.rd(4 * k + 1) << 8) | (P.rd(4 * k + 2) << 16) | (P.rd(4 * k + 3) << 24);
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
