/*
 * brb_rc4.c -- compat RC4 surface of libbrb_crypto_gpu.so (host).
 *
 * Behaviour follows libbrb_core/crypto/rc4.c (reference @ 2024_10_08), which is the textbook
 * RC4 on BRB_RC4_State (libbrb_data.h:887-897):
 *   * Init (rc4.c:40-62): identity permutation, index1 = index2 = 0, one key-scheduling sweep
 *     with the key cycled by i % keylen; `flags` is not touched;
 *   * Crypt (rc4.c:64-87): per byte index1 += 1, index2 += perm[index1], swap the two entries,
 *     out = in ^ perm[perm[index1] + perm[index2]] (8-bit arithmetic); in == out is allowed.
 * A single connection's stream is a serial chain, so this stays on the calling CPU thread; many
 * connections at once go to BRB_RC4_CryptBatch (GPU).
 */
#include <stddef.h>

#include "brb_crypto.h"

_Static_assert(sizeof(BRB_RC4_State) == 264, "BRB_RC4_State ABI");
_Static_assert(offsetof(BRB_RC4_State, index1) == 256 && offsetof(BRB_RC4_State, index2) == 257,
               "BRB_RC4_State ABI");

void BRB_RC4_Init(BRB_RC4_State *state, const unsigned char *key, int keylen)
{
    unsigned char *S = state->perm;
    for (int k = 0; k < 256; k++)
        S[k] = (unsigned char)k;
    state->index1 = 0;
    state->index2 = 0;
    unsigned char j = 0;
    for (int k = 0; k < 256; k++) {
        const unsigned char t = S[k];
        j = (unsigned char)(j + t + key[k % keylen]);
        S[k] = S[j];
        S[j] = t;
    }
}

void BRB_RC4_Crypt(BRB_RC4_State *state, const unsigned char *inbuf, unsigned char *outbuf, int buflen)
{
    unsigned char *S = state->perm;
    unsigned char i = state->index1, j = state->index2;
    for (int k = 0; k < buflen; k++) {
        i = (unsigned char)(i + 1);
        const unsigned char a = S[i];
        j = (unsigned char)(j + a);
        const unsigned char b = S[j];
        S[i] = b;
        S[j] = a;
        outbuf[k] = inbuf[k] ^ S[(unsigned char)(a + b)];
    }
    state->index1 = i;
    state->index2 = j;
}
