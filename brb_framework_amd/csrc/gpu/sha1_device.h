// sha1_device.h -- SHA-1 compression for gfx950, one record per lane.
//
// Same function as BrbSha1_Transform (libbrb_core/crypto/sha1.c:75-130): big-endian message
// words (blk0, :46-47 -> one v_perm_b32), 16-word circular schedule (blk, :49-50 -> v_xor3 +
// v_alignbit), rounds R0..R4 (:54-58 -> v_bitop3 + v_add3 + v_alignbit).  The batch kernels keep
// the schedule in registers and never write it back to the input (the compat surface does).
#pragma once

#include "brb_gpu_common.h"

struct Sha1State {
    uint32_t a, b, c, d, e;
};

BRB_DEV Sha1State sha1_iv()
{
    return Sha1State{0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
}

// Each round function is one v_bitop3_b32 (truth table indexed by b << 2 | c << 1 | d).  Written
// with the builtin: hipcc lowers the plain C forms of Parity and Maj to two ops (xor + xor,
// bfi + xor), and the schedule's four-way xor to three xors.
#define BRB_SHA1_CH(b, c, d) __builtin_amdgcn_bitop3_b32((b), (c), (d), 0xCA)
#define BRB_SHA1_PAR(b, c, d) __builtin_amdgcn_bitop3_b32((b), (c), (d), 0x96)
#define BRB_SHA1_MAJ(b, c, d) __builtin_amdgcn_bitop3_b32((b), (c), (d), 0xE8)
#define BRB_SHA1_W(i) \
    (w[(i) & 15] = rotl<1>(__builtin_amdgcn_bitop3_b32(w[((i) + 13) & 15], w[((i) + 8) & 15], w[((i) + 2) & 15], 0x96) ^ w[(i) & 15]))
// round with the roles of (a..e) rotated by the caller, as the reference's R0..R4 macros do
#define BRB_SHA1_R(F, K, v, x, y, z, u, wi)                    \
    do {                                                       \
        (u) += F((x), (y), (z)) + (wi) + (K) + rotl<5>(v);     \
        (x) = rotl<30>(x);                                     \
    } while (0)

// `w` holds the 16 message words already converted to big-endian values; it is consumed.
BRB_DEV void sha1_compress(Sha1State &st, uint32_t (&w)[16])
{
    uint32_t a = st.a, b = st.b, c = st.c, d = st.d, e = st.e;
    constexpr uint32_t K0 = 0x5A827999u, K1 = 0x6ED9EBA1u, K2 = 0x8F1BBCDCu, K3 = 0xCA62C1D6u;

#define R5(F, K, i, W)                                   \
    BRB_SHA1_R(F, K, a, b, c, d, e, W(i + 0));           \
    BRB_SHA1_R(F, K, e, a, b, c, d, W(i + 1));           \
    BRB_SHA1_R(F, K, d, e, a, b, c, W(i + 2));           \
    BRB_SHA1_R(F, K, c, d, e, a, b, W(i + 3));           \
    BRB_SHA1_R(F, K, b, c, d, e, a, W(i + 4));
#define W0(i) w[(i)]
#define WX(i) BRB_SHA1_W(i)
    R5(BRB_SHA1_CH, K0, 0, W0) R5(BRB_SHA1_CH, K0, 5, W0) R5(BRB_SHA1_CH, K0, 10, W0)
    BRB_SHA1_R(BRB_SHA1_CH, K0, a, b, c, d, e, w[15]);
    BRB_SHA1_R(BRB_SHA1_CH, K0, e, a, b, c, d, WX(16));
    BRB_SHA1_R(BRB_SHA1_CH, K0, d, e, a, b, c, WX(17));
    BRB_SHA1_R(BRB_SHA1_CH, K0, c, d, e, a, b, WX(18));
    BRB_SHA1_R(BRB_SHA1_CH, K0, b, c, d, e, a, WX(19));
    R5(BRB_SHA1_PAR, K1, 20, WX) R5(BRB_SHA1_PAR, K1, 25, WX) R5(BRB_SHA1_PAR, K1, 30, WX) R5(BRB_SHA1_PAR, K1, 35, WX)
    R5(BRB_SHA1_MAJ, K2, 40, WX) R5(BRB_SHA1_MAJ, K2, 45, WX) R5(BRB_SHA1_MAJ, K2, 50, WX) R5(BRB_SHA1_MAJ, K2, 55, WX)
    R5(BRB_SHA1_PAR, K3, 60, WX) R5(BRB_SHA1_PAR, K3, 65, WX) R5(BRB_SHA1_PAR, K3, 70, WX) R5(BRB_SHA1_PAR, K3, 75, WX)
#undef W0
#undef WX
#undef R5

    st.a += a;
    st.b += b;
    st.c += c;
    st.d += d;
    st.e += e;
}

// Final padding of a message whose last partial block holds t (< 64) bytes; `w` holds that block
// as LITTLE-endian words with the 0x80 marker placed.  The 64-bit bit count is the reference's
// counter pair (sha1.c:151-152 for ONE update of `len` bytes, then Final's finalcount, :177-179):
//   count[0] = (len << 3) mod 2^32,  count[1] = (len >> 29) + (len >= 2^29)   <- extra carry quirk
BRB_DEV void sha1_finish(Sha1State &st, uint32_t (&w)[16], uint32_t t, uint64_t len)
{
#pragma unroll
    for (int i = 0; i < 16; i++)
        w[i] = __builtin_bswap32(w[i]);
    if (t >= 56) {
        sha1_compress(st, w);
#pragma unroll
        for (int i = 0; i < 14; i++)
            w[i] = 0;
    }
    w[14] = uint32_t(len >> 29) + (len >= (uint64_t(1) << 29) ? 1u : 0u);
    w[15] = uint32_t(len << 3);
    sha1_compress(st, w);
}

// The padding block of a message whose length is a multiple of 64 (t = 0 in sha1_finish): the
// block and its whole schedule are constants except the two wave-uniform length words.
BRB_DEV void sha1_pad_only(Sha1State &st, uint64_t len)
{
    uint32_t w[16] = {0x80000000u};
    w[14] = uint32_t(len >> 29) + (len >= (uint64_t(1) << 29) ? 1u : 0u);
    w[15] = uint32_t(len << 3);
    sha1_compress(st, w);
}
