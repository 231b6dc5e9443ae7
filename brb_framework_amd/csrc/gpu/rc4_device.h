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

// Keystream generator: BRB_RC4_Crypt's index1/index2 walk (rc4.c:71-82), software-pipelined.
//
// The serial form of byte t is  i += 1; a = S[i]; j += a; b = S[j]; S[i] = b; S[j] = a;
// k = S[a + b].  step() STARTS byte T+1 (a, j, the S[j] address) and then COMPLETES byte T (write
// its swap, read S[j_{T+1}] and k_T):
//   * S[j_{T+1}] is read right after swap T is written, so it is exact: the one LDS write -> read
//     round trip per byte on the chain is covered by the rest of the step;
//   * S[i] is read two bytes ahead (positions i+1, i+2 in flight), before the swap of its step is
//     written; a raw S[i_{T+1}] missed swaps T-2, T-1 and T, and since i_s != i_{T+1} for those,
//     only j_s == i_{T+1} -> a_s applies (three compare/select pairs).
// So j_{T+1} = j_T + a_{T+1} is pure VALU.  Indices live only as their LDS addresses, 16-bit values
// index << 8 | column (round 6): the next i is one v_pk_add_u16 of 256 and the
// next j one v_pk_mad_u16 (a_{T+1} * 256 + address of j_T).  The low halves wrap mod 2^16, i.e. the
// index mod 256, and the high halves add zeros, so the result stays a clean 16-bit address
// (tools/mb/u16_check.hip; the plain v_add_u16 / v_mad_u16 leave the destination's high half as it
// was on gfx950).  Round 5 kept running 32-bit sums and paid an add and a v_perm_b32 for each.  The patches compare addresses, so no masking op is needed
// anywhere.
// Before the first byte the "previous swaps" are identity swaps (S[ci] = S[ci], S[cj] = S[cj]),
// which patch nothing wrongly, so there is no special case.  One byte is always started ahead of
// the last one returned; store() drops it (its swap was never written), so the state advances by
// exactly the bytes returned.
// Measured (65 536 streams x 1500 B, MI355X): 188 us serial form -> 170 us pipelined with S[j]
// read before swap T and patched (two more pairs); hand-scheduled inline asm variants with one and
// two steps of read-ahead ran 178 and 195 us.  Round 2 (session 4), interleaved A/B (rocprofv3): reading
// S[j] after the swap instead of patching it took the RC4 pass 123.0 -> 117.4 us, the frame kernel
// 141.2 -> 130.0 us and the open kernel 138.1 -> 124.7 us; moving the S[i] read after the swap too
// (one pair fewer) ran 128 us: the read then lands too late for the step that needs it.  Round 6,
// with the 16-bit address ops (11.3 VALU per byte): reading S[j_{T+1}] before swap T again (patched
// with swap T-1 at completion, 15.3 VALU per byte) ran 102.5 -> 125.9 us (interleaved, three
// rounds, profiles/r06/ab_rc4.txt); the exact read after the swap stays.
struct Gen {
    Perm P;
    // Every index is kept as its LDS address.  Two indices are equal mod 256 iff their addresses
    // are (same lane column), so all compares are on addresses.
    // started byte T: S[i_T], raw S[j_T], addresses of S[i_T] and S[j_T]
    uint32_t a, rb, ai, aj;
    // swap T-1 (written): addresses of i and j, a; swap T-2: address of j, a
    uint32_t pai, paj, pa, qaj, qa;
    // S[i] read ahead: positions i_T + 1 and i_T + 2: raw values, addresses
    uint32_t r1, ad1, r2, ad2;
    uint32_t tail;     // dword 64 of the state: index1, index2 and the two bytes after them

    // LDS address of index x (low byte of x): byte 1 = x, byte 0 = the lane's column
    BRB_DEV uint32_t ad(uint32_t x) const { return __builtin_amdgcn_perm(x, P.lw, 0x0C0C0400u); }
    // address of the index after the one at address x: (x + 256) mod 2^16 (x < 2^16)
    static BRB_DEV uint32_t ad_next(uint32_t x)
    {
        uint32_t r;
        asm("v_pk_add_u16 %0, %1, %2" : "=v"(r) : "v"(x), "s"(256u));
        return r;
    }
    // address of (the index at address x) + v: (v * 256 + x) mod 2^16 (x < 2^16, v < 2^16)
    static BRB_DEV uint32_t ad_plus(uint32_t x, uint32_t v)
    {
        uint32_t r;
        asm("v_pk_mad_u16 %0, %1, %2, %3" : "=v"(r) : "v"(v), "s"(256u), "v"(x));
        return r;
    }
    BRB_DEV uint32_t rd(uint32_t a_) const { return P.lds[a_]; }
    BRB_DEV void wr(uint32_t a_, uint32_t v) const { P.lds[a_] = uint8_t(v); }

    // BRB_RC4_State (4-byte aligned) -> LDS image + registers; starts byte 0
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
        const uint32_t ci = tail & 255u, cj = (tail >> 8) & 255u;
        pai = ad(ci);                  // identity swaps before byte 0: S[ci] = S[ci], S[cj] = S[cj]
        paj = ad(cj);
        pa = rd(paj);
        qaj = paj;
        qa = pa;
        ai = ad(ci + 1);
        a = rd(ai);
        aj = ad(cj + a);
        rb = rd(aj);
        ad1 = ad(ci + 2);
        r1 = rd(ad1);
        ad2 = ad(ci + 3);
        r2 = rd(ad2);
    }

    BRB_DEV void store(uint8_t *st) const
    {
        uint32_t *w = reinterpret_cast<uint32_t *>(st);
#pragma unroll 8
        for (uint32_t k = 0; k < 64; k++)
            w[k] = P.rd(4 * k) | (P.rd(4 * k + 1) << 8) | (P.rd(4 * k + 2) << 16) | (P.rd(4 * k + 3) << 24);
        // indices of the last completed byte = byte 1 of its addresses
        w[64] = (tail & 0xFFFF0000u) | (paj & 0xFF00u) | ((pai >> 8) & 255u);
    }

    // Completes byte T (returns its keystream byte) and starts byte T+1.
    BRB_DEV uint32_t step()
    {
        // ---- start byte T+1 at address ad1
        uint32_t a1 = r1;                    // read before swap T-2 was written
        a1 = qaj == ad1 ? qa : a1;           // swap T-2
        a1 = paj == ad1 ? pa : a1;           // swap T-1
        a1 = aj == ad1 ? a : a1;             // swap T (not written yet)
        const uint32_t aj1 = ad_plus(aj, a1);   // j_{T+1} = j_T + a_{T+1}
        const uint32_t ad3 = ad_next(ad2);
        const uint32_t r3 = rd(ad3);         // S[i_{T+1} + 2], sees swaps <= T-1
        // ---- complete byte T
        const uint32_t b = rb;               // S[j_T], read after swap T-1 was written: exact
        wr(ai, b);                           // S[i] = S[j]
        wr(aj, a);                           // S[j] = S[i]   (rc4.c:76-78)
        const uint32_t rb1 = rd(aj1);        // S[j_{T+1}] after swap T: exact
        const uint32_t k = rd(ad(a + b));    // S[S[i] + S[j]]
        // ---- shift the pipeline
        qaj = paj;
        qa = pa;
        pai = ai;
        paj = aj;
        pa = a;
        a = a1;
        rb = rb1;
        ai = ad1;
        aj = aj1;
        r1 = r2;
        ad1 = ad2;
        r2 = r3;
        ad2 = ad3;
        return k;
    }

    // NW keystream words; the bytes are packed after all NW * 4 steps are issued
    template <int NW>
    BRB_DEV void words(uint32_t (&ks)[NW])
    {
        uint32_t kb[4 * NW];
#pragma unroll
        for (int t = 0; t < 4 * NW; t++)
            kb[t] = step();
#pragma unroll
        for (int w = 0; w < NW; w++)
            ks[w] = kb[4 * w] | (kb[4 * w + 1] << 8) | (kb[4 * w + 2] << 16) | (kb[4 * w + 3] << 24);
    }

    BRB_DEV uint32_t next4()
    {
        const uint32_t b0 = step(), b1 = step(), b2 = step(), b3 = step();
        return b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
    }

    // nb (0..4) keystream bytes, little-endian in the low bytes; the state advances by exactly nb
    BRB_DEV uint32_t next_n(uint32_t nb)
    {
        if (nb >= 4)
            return next4();
        uint32_t v = 0;
        for (uint32_t b = 0; b < nb; b++)
            v |= step() << (8 * b);
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

// Words 16b .. 16b + 15 of the MD5-padded message, in place over the raw words: a block wholly
// inside the message is its raw words (one compare per block instead of three 64-bit compares and
// selects per word); only the last one or two blocks take md5_pad_word.
BRB_DEV void md5_pad_block(uint32_t (&m)[16], uint64_t b, uint64_t len, uint64_t n_words)
{
    if (64 * (b + 1) <= len)
        return;
#pragma unroll
    for (uint32_t i = 0; i < 16; i++)
        m[i] = md5_pad_word(m[i], 16 * b + i, len, n_words);
}

// number of 64-byte MD5 blocks of a `len`-byte message including the padding
BRB_DEV uint64_t md5_blocks(uint64_t len) { return (len + 72) >> 6; }

}  // namespace brb_rc4
