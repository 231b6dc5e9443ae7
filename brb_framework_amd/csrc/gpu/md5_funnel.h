// md5_funnel.h -- one lane's streaming MD5 over bytes that arrive in pieces of 1..4 bytes at any
// message position (BRB_MD5Init, BRB_MD5UpdateBig per piece, BRB_MD5Final: md5.c:38-168).
//
// A 64-bit carry holds the 0..3 message bytes left over from the previous piece; whole 32-bit
// message words go to the lane's private 64-byte block buffer in LDS, word k of lane l at
// (k * 64 + l) * 4 -- every access of lane l hits bank l -- and a full block is compressed from
// there.  Used by md5_seg_kernel (a record's segments) and metadata_unpack_kernel (the items of a
// MetaData pack).
#pragma once

#include "md5_device.h"

namespace brb_md5 {

struct Funnel {
    uint32_t *bb;       // word k of this lane's block at bb[64 k] (LDS)
    Md5State st;
    uint64_t acc, total;
    uint32_t nacc, wpos;

    BRB_DEV void init(uint32_t *lane_words)
    {
        bb = lane_words;
        st = md5_iv();
        acc = total = 0;
        nacc = wpos = 0;
    }

    // appends the low `nb` (1..4) bytes of v, least significant first
    BRB_DEV void put(uint32_t v, uint32_t nb)
    {
        total += nb;
        acc |= uint64_t(v) << (8 * nacc);
        nacc += nb;
        if (nacc >= 4) {
            bb[64 * wpos] = uint32_t(acc);
            acc >>= 32;
            nacc -= 4;
            if (++wpos == 16) {
                uint32_t w[16];
#pragma unroll
                for (int i = 0; i < 16; i++)
                    w[i] = bb[64 * i];
                md5_compress(st, w);
                wpos = 0;
            }
        }
    }

    // BRB_MD5Final (md5.c:134-168): 0x80, zeros, the 64-bit bit count
    BRB_DEV Md5State finish()
    {
        uint32_t w[16];
        bb[64 * wpos] = uint32_t(acc | (uint64_t(0x80) << (8 * nacc)));
        ++wpos;
#pragma unroll
        for (uint32_t i = 0; i < 16; i++)
            w[i] = i < wpos ? bb[64 * i] : 0u;
        if (wpos > 14) {
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

}  // namespace brb_md5
