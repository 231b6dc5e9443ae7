// md5_device.h -- MD5 compression for gfx950, one record per lane.
//
// Same function as BRB_MD5Transform (libbrb_core/crypto/md5.c:170-253; step macro
// libbrb_data.h:851).  Each of the 64 steps lowers to five VALU ops on gfx950:
//   v_add_u32 (m + K, literal K)  ->  v_bitop3_b32 (F)  ->  v_add3_u32 (a + F + mK)
//   ->  v_alignbit_b32 (rotate)  ->  v_add_u32 (+ b)
#pragma once

#include "brb_gpu_common.h"

#define BRB_MD5_F1(x, y, z) ((z) ^ ((x) & ((y) ^ (z))))
#define BRB_MD5_F2(x, y, z) ((y) ^ ((z) & ((x) ^ (y))))
#define BRB_MD5_F3(x, y, z) __builtin_amdgcn_bitop3_b32((x), (y), (z), 0x96)   // x ^ y ^ z
#define BRB_MD5_F4(x, y, z) ((y) ^ ((x) | ~(z)))
#define BRB_MD5_STEP(F, a, b, c, d, m, k, s) (a) = (b) + rotl<s>((a) + F((b), (c), (d)) + ((m) + (k)))

struct Md5State {
    uint32_t a, b, c, d;
};

BRB_DEV Md5State md5_iv()
{
    return Md5State{0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
}

// Round-3 step (F3 = b ^ c ^ d) with v_xad_u32 = (b ^ cd) + x: cd = c ^ d and x = a + m + K do not
// depend on b, so the step's dependent chain is xad -> alignbit -> add (3 ops, 5 VALU per step)
// instead of xor -> add3 -> alignbit -> add (hipcc's lowering of the plain macro, 6 VALU).
#define BRB_MD5_STEP3X(a, b, c, d, m, k, s)                                               \
    do {                                                                                 \
        const uint32_t x_ = (a) + (m) + (k), cd_ = (c) ^ (d);                            \
        uint32_t f_;                                                                     \
        asm("v_xad_u32 %0, %1, %2, %3" : "=v"(f_) : "v"(b), "v"(cd_), "v"(x_));          \
        (a) = (b) + rotl<s>(f_);                                                         \
    } while (0)

template <bool XAD = true>
BRB_DEV void md5_compress(Md5State &st, const uint32_t (&m)[16])
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

    if constexpr (XAD) BRB_MD5_STEP3X(a, b, c, d, m[5], 0xfffa3942u, 4); else BRB_MD5_STEP(BRB_MD5_F3, a, b, c, d, m[5], 0xfffa3942u, 4);
    if constexpr (XAD) BRB_MD5_STEP3X(d, a, b, c, m[8], 0x8771f681u, 11); else BRB_MD5_STEP(BRB_MD5_F3, d, a, b, c, m[8], 0x8771f681u, 11);
    if constexpr (XAD) BRB_MD5_STEP3X(c, d, a, b, m[11], 0x6d9d6122u, 16); else BRB_MD5_STEP(BRB_MD5_F3, c, d, a, b, m[11], 0x6d9d6122u, 16);
    if constexpr (XAD) BRB_MD5_STEP3X(b, c, d, a, m[14], 0xfde5380cu, 23); else BRB_MD5_STEP(BRB_MD5_F3, b, c, d, a, m[14], 0xfde5380cu, 23);
    if constexpr (XAD) BRB_MD5_STEP3X(a, b, c, d, m[1], 0xa4beea44u, 4); else BRB_MD5_STEP(BRB_MD5_F3, a, b, c, d, m[1], 0xa4beea44u, 4);
    if constexpr (XAD) BRB_MD5_STEP3X(d, a, b, c, m[4], 0x4bdecfa9u, 11); else BRB_MD5_STEP(BRB_MD5_F3, d, a, b, c, m[4], 0x4bdecfa9u, 11);
    if constexpr (XAD) BRB_MD5_STEP3X(c, d, a, b, m[7], 0xf6bb4b60u, 16); else BRB_MD5_STEP(BRB_MD5_F3, c, d, a, b, m[7], 0xf6bb4b60u, 16);
    if constexpr (XAD) BRB_MD5_STEP3X(b, c, d, a, m[10], 0xbebfbc70u, 23); else BRB_MD5_STEP(BRB_MD5_F3, b, c, d, a, m[10], 0xbebfbc70u, 23);
    if constexpr (XAD) BRB_MD5_STEP3X(a, b, c, d, m[13], 0x289b7ec6u, 4); else BRB_MD5_STEP(BRB_MD5_F3, a, b, c, d, m[13], 0x289b7ec6u, 4);
    if constexpr (XAD) BRB_MD5_STEP3X(d, a, b, c, m[0], 0xeaa127fau, 11); else BRB_MD5_STEP(BRB_MD5_F3, d, a, b, c, m[0], 0xeaa127fau, 11);
    if constexpr (XAD) BRB_MD5_STEP3X(c, d, a, b, m[3], 0xd4ef3085u, 16); else BRB_MD5_STEP(BRB_MD5_F3, c, d, a, b, m[3], 0xd4ef3085u, 16);
    if constexpr (XAD) BRB_MD5_STEP3X(b, c, d, a, m[6], 0x04881d05u, 23); else BRB_MD5_STEP(BRB_MD5_F3, b, c, d, a, m[6], 0x04881d05u, 23);
    if constexpr (XAD) BRB_MD5_STEP3X(a, b, c, d, m[9], 0xd9d4d039u, 4); else BRB_MD5_STEP(BRB_MD5_F3, a, b, c, d, m[9], 0xd9d4d039u, 4);
    if constexpr (XAD) BRB_MD5_STEP3X(d, a, b, c, m[12], 0xe6db99e5u, 11); else BRB_MD5_STEP(BRB_MD5_F3, d, a, b, c, m[12], 0xe6db99e5u, 11);
    if constexpr (XAD) BRB_MD5_STEP3X(c, d, a, b, m[15], 0x1fa27cf8u, 16); else BRB_MD5_STEP(BRB_MD5_F3, c, d, a, b, m[15], 0x1fa27cf8u, 16);
    if constexpr (XAD) BRB_MD5_STEP3X(b, c, d, a, m[2], 0xc4ac5665u, 23); else BRB_MD5_STEP(BRB_MD5_F3, b, c, d, a, m[2], 0xc4ac5665u, 23);

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

// Padding blocks of a message whose last partial block holds `t` (< 64) bytes; `wtail` is that
// partial block with the 0x80 marker already placed (tail_word_a4 / word_any).  Appends the
// 64-bit bit length (md5.c:158-159: in[14] = bytes << 3, in[15] = bytes >> 29) and compresses
// one or two blocks (md5.c:147-153).
BRB_DEV void md5_finish(Md5State &st, uint32_t (&w)[16], uint32_t t, uint64_t total_len)
{
    if (t >= 56) {
        md5_compress(st, w);
#pragma unroll
        for (int i = 0; i < 14; i++)
            w[i] = 0;
    }
    w[14] = uint32_t(total_len << 3);
    w[15] = uint32_t(total_len >> 29);
    md5_compress(st, w);
}

// The padding block of a message whose length is a multiple of 64 (md5.c:134-168 with t = 0):
// 0x80, zeros, the bit length.  Compile-time words except the length (wave-uniform), so m + K folds
// into constants and each step is 4 VALU instead of 5.  Round 3 takes the plain form here
// (bitop3 xor3 -> add3 with the folded constant): with no message add to hide, v_xad would cost
// the c ^ d op on top.
BRB_DEV void md5_pad_only(Md5State &st, uint64_t total_len)
{
    uint32_t w[16] = {0x80u};
    w[14] = uint32_t(total_len << 3);
    w[15] = uint32_t(total_len >> 29);
    md5_compress<false>(st, w);
}
