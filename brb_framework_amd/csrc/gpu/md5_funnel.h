// md5_funnel.h -- one lane's streaming MD5 over bytes that arrive in pieces of 1..4 bytes at any
// message position (BRB_MD5Init, BRB_MD5UpdateBig per piece, BRB_MD5Final: md5.c:38-168).
//
// A carry holds the 0..3 message bytes left over from the previous piece; whole 32-bit message
// words go to the lane's private 32-word ring in LDS, word k of lane l at (k * 64 + l) * 4 -- every
// access of lane l hits bank l.  The callers read each piece from `nacc` bytes before it, so its
// words already fall on message word boundaries (head/put16w/put_tail below); pump() compresses the
// oldest 16 once they are there, and must run at least once per 16 words written.  Keeping the
// compression out of the puts leaves one compress site per caller loop: with it inside, a loop of
// 16 unrolled puts inlined 16 copies of the compression (52 KB of code for metadata_unpack_kernel).
// Used by md5_seg_kernel (a record's segments) and metadata_unpack_kernel (a pack's items).
#pragma once

#include "md5_device.h"

namespace brb_md5 {

constexpr uint32_t kRingWords = 32;

// RW ring words per lane (a multiple of 16, a power of two): the wave's ring is RW x 64 dwords at an
// RW * 256-byte aligned LDS address.  The line-staged kernels (line_stream.h) put up to 33 words per
// 128-byte line and take RW = 64; the per-lane block kernels put 16 per block and take 32.
template <uint32_t RW>
struct FunnelT {
    static constexpr uint32_t kMask = RW * 256 - 1;
    uint32_t *bb;       // ring word k of this lane at bb[64 k] (LDS)
    uint32_t ring;      // LDS address of this wave's ring (RW * 256-byte aligned), OR'd into word addresses
    uint32_t lane4;     // 4 x lane: the lane's byte within a ring row
    Md5State st;
    uint64_t acc, total; // the carried bytes (low nacc bytes), message bytes so far (the caller's)
    uint32_t nacc;      // bytes held in acc (0..3)
    uint32_t wpos;      // words written
    uint32_t cpos;      // words compressed (a multiple of 16)

    // lane_words = &ring[0][lane] of a [RW][64] uint32 array at an RW * 256-byte aligned LDS
    // address, so a word's address is one and-or of its ring offset
    BRB_DEV void init(uint32_t *lane_words)
    {
        bb = lane_words;
        const uint32_t a = uint32_t(reinterpret_cast<uintptr_t>(lane_words));
        ring = a & ~kMask;
        lane4 = a & 0xFFu;
        st = md5_iv();
        acc = total = 0;
        nacc = wpos = cpos = 0;
    }

    static BRB_DEV void lds_st(uint32_t a, uint32_t v) { *reinterpret_cast<__attribute__((address_space(3))) uint32_t *>(a) = v; }

    // word at ring position wpos + i (mod RW): (lane4 + 256 (wpos + i)) mod (RW * 256), in the wave's ring
    BRB_DEV void word_at(uint32_t i, uint32_t w) const
    {
        lds_st(((lane4 + ((wpos + i) << 8)) & kMask) | ring, w);
    }
    BRB_DEV void word(uint32_t w)
    {
        word_at(0, w);
        ++wpos;
    }

    // Word-aligned input (metadata_unpack_kernel): the caller reads the next piece starting nacc
    // bytes early, so its words fall on MD5 word boundaries; the low nacc bytes of its first word
    // are replaced by the carried bytes (head), whole words go straight to the ring (put16w,
    // put_tail), and the bytes of a last partial word become the carry.  `total` is the caller's.
    BRB_DEV uint32_t head(uint32_t w0) const
    {
        return nacc ? (w0 & ~((1u << (8 * nacc)) - 1u)) | uint32_t(acc) : w0;
    }
    BRB_DEV void put16w(const uint32_t (&w)[16])
    {
#pragma unroll
        for (uint32_t i = 0; i < 16; i++)
            word_at(i, w[i]);
        wpos += 16;
    }
    // the first `left` (< 64) bytes of w: whole words to the ring, the rest (zeros past it) carried
    BRB_DEV void put_tail(const uint32_t (&w)[16], uint32_t left)
    {
#pragma unroll
        for (uint32_t i = 0; i < 16; i++)
            if (4 * i + 4 <= left)
                word(w[i]);
        const uint32_t k = left >> 2;
        uint32_t t = 0;
#pragma unroll
        for (uint32_t i = 0; i < 16; i++)
            t = i == k ? w[i] : t;
        nacc = left & 3;
        acc = nacc ? t : 0u;
    }

    // cpos is a multiple of 16, so the 16 words never wrap: one base, immediate offsets
    BRB_DEV void load16(uint32_t (&w)[16]) const
    {
        const uint32_t *b = bb + 64 * (cpos & (RW - 16));
#pragma unroll
        for (uint32_t i = 0; i < 16; i++)
            w[i] = b[64 * i];
    }

    BRB_DEV void pump()
    {
        if (wpos - cpos >= 16) {
            uint32_t w[16];
            load16(w);
            md5_compress(st, w);
            cpos += 16;
        }
    }

    // BRB_MD5Final (md5.c:134-168): 0x80, zeros, the 64-bit bit count
    BRB_DEV Md5State finish()
    {
        pump();
        const uint32_t r = wpos - cpos;                   // whole words not yet compressed (0..15)
        uint32_t w[16];
        load16(w);
        const uint32_t tail = uint32_t(acc | (uint64_t(0x80) << (8 * nacc)));
#pragma unroll
        for (uint32_t i = 0; i < 16; i++)
            w[i] = i < r ? w[i] : i == r ? tail : 0u;
        if (r + 1 > 14) {
            md5_compress(st, w);
#pragma unroll
            for (int i = 0; i < 16; i++)
                w[i] = 0;
        }
        w[14] = uint32_t(total << 3);
        w[15] = uint32_t(total >> 29);
        md5_compress(st, w);
        return st;
    }
};

using Funnel = FunnelT<kRingWords>;

}  // namespace brb_md5
