/*
 * brb_blowfish.c -- compat Blowfish surface of libbrb_crypto_gpu.so (host).
 *
 * Behaviour follows libbrb_core/crypto/blowfish.c (reference @ 2024_10_08), which is Kocher's
 * Blowfish with every word an LP64 `unsigned long`:
 *   * _F (blowfish.c:445-462) adds and xors 64-bit S-box entries with no 32-bit wrap, so carries
 *     accumulate in the high halves; the S-box index bytes come from bits 0..31 only;
 *   * Encrypt/Decrypt (:312-380) run 16 Feistel rounds on two 64-bit words;
 *   * Init (:382-443) xors P with the key cycled big-endian 4 bytes at a time and refills P and
 *     then S with 521 chained encryptions of a running (L, R) = (0, 0).
 * The low 32 bits of every word equal standard Blowfish; the high 32 bits are the reference's
 * deterministic carries.  Initial P/S = hex digits of pi (tools/gen_pi_tables.py).
 */
#include "brb_crypto.h"

#include "../common/blowfish_pi.h"

_Static_assert(sizeof(unsigned long) == 8, "the reference's Blowfish needs LP64");
_Static_assert(sizeof(BRB_BLOWFISH_CTX) == 8336, "BRB_BLOWFISH_CTX ABI");

static inline unsigned long bf_f(const BRB_BLOWFISH_CTX *ctx, unsigned long x)
{
    uint32_t lo = (uint32_t)x;
    unsigned long y = ctx->S[0][lo >> 24] + ctx->S[1][(lo >> 16) & 0xFF];
    y ^= ctx->S[2][(lo >> 8) & 0xFF];
    return y + ctx->S[3][lo & 0xFF];
}

void BRB_Blowfish_Encrypt(BRB_BLOWFISH_CTX *ctx, unsigned long *xl, unsigned long *xr)
{
    unsigned long L = *xl, R = *xr;

    /* two rounds per iteration: the swap is folded into the register naming */
    for (int i = 0; i < 16; i += 2) {
        L ^= ctx->P[i];
        R ^= bf_f(ctx, L);
        R ^= ctx->P[i + 1];
        L ^= bf_f(ctx, R);
    }
    /* after 16 rounds (even) plus the final undo-swap: out_l = R ^ P[17], out_r = L ^ P[16] */
    *xl = R ^ ctx->P[17];
    *xr = L ^ ctx->P[16];
}

void BRB_Blowfish_Decrypt(BRB_BLOWFISH_CTX *ctx, unsigned long *xl, unsigned long *xr)
{
    unsigned long L = *xl, R = *xr;

    for (int i = 17; i > 1; i -= 2) {
        L ^= ctx->P[i];
        R ^= bf_f(ctx, L);
        R ^= ctx->P[i - 1];
        L ^= bf_f(ctx, R);
    }
    *xl = R ^ ctx->P[0];
    *xr = L ^ ctx->P[1];
}

void BRB_Blowfish_Init(BRB_BLOWFISH_CTX *ctx, unsigned char *key, int keyLen)
{
    int j = 0;
    unsigned long L = 0, R = 0;

    for (int s = 0; s < 4; s++)
        for (int i = 0; i < 256; i++)
            ctx->S[s][i] = BRB_BF_PI_S[s][i];

    for (int i = 0; i < 18; i++) {
        unsigned long data = 0;
        for (int k = 0; k < 4; k++) {
            data = (data << 8) | key[j];
            if (++j >= keyLen)
                j = 0;
        }
        ctx->P[i] = (unsigned long)BRB_BF_PI_P[i] ^ data;
    }

    for (int i = 0; i < 18; i += 2) {
        BRB_Blowfish_Encrypt(ctx, &L, &R);
        ctx->P[i] = L;
        ctx->P[i + 1] = R;
    }
    for (int s = 0; s < 4; s++)
        for (int i = 0; i < 256; i += 2) {
            BRB_Blowfish_Encrypt(ctx, &L, &R);
            ctx->S[s][i] = L;
            ctx->S[s][i + 1] = R;
        }
}
