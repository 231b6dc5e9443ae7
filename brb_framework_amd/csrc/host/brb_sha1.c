/*
 * brb_sha1.c -- compat SHA-1 surface of libbrb_crypto_gpu.so (host, one streaming context).
 *
 * Behaviour follows libbrb_core/crypto/sha1.c (reference @ 2024_10_08), including its two
 * observable quirks:
 *   * in-place schedule: SHA1HANDSOFF is undefined (sha1.c:84-90), so the compression works inside
 *     the block it is given and leaves W[64..79] (host byte order) there.  Update hands it the
 *     caller's own bytes for every full block after the first fill (sha1.c:157-158), so those
 *     bytes are rewritten, exactly as the reference does;
 *   * bit counter: `count[0] += len << 3` is compared against the size_t `len << 3`
 *     (sha1.c:151), which adds one spurious carry for a single update of >= 2^29 bytes.
 * BrbSha1_Final pads byte-wise through Update (sha1.c:180-184) and wipes the context (:192-194).
 */
#include "brb_crypto.h"

#include <string.h>

_Static_assert(sizeof(BrbSha1Ctx) == 92, "BrbSha1Ctx ABI");

#define ROL(x, s) (((x) << (s)) | ((x) >> (32 - (s))))

static inline uint32_t be32(uint32_t v)
{
    return __builtin_bswap32(v);
}

/* 80-step compression on a 16-word circular schedule held IN the block (as the reference). */
static void sha1_compress_inplace(uint32_t st[5], uint32_t *w)
{
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], t;

#define SCHED(i) (w[(i) & 15] = ROL(w[((i) + 13) & 15] ^ w[((i) + 8) & 15] ^ w[((i) + 2) & 15] ^ w[(i) & 15], 1))
#define ROUND(i, fexpr, k, wexpr)                          \
    do {                                                   \
        t = ROL(a, 5) + (fexpr) + e + (k) + (wexpr);       \
        e = d;                                             \
        d = c;                                             \
        c = ROL(b, 30);                                    \
        b = a;                                             \
        a = t;                                             \
    } while (0)

    for (int i = 0; i < 16; i++) {
        w[i] = be32(w[i]);
        ROUND(i, d ^ (b & (c ^ d)), 0x5A827999u, w[i]);
    }
    for (int i = 16; i < 20; i++)
        ROUND(i, d ^ (b & (c ^ d)), 0x5A827999u, SCHED(i));
    for (int i = 20; i < 40; i++)
        ROUND(i, b ^ c ^ d, 0x6ED9EBA1u, SCHED(i));
    for (int i = 40; i < 60; i++)
        ROUND(i, (b & c) | (d & (b | c)), 0x8F1BBCDCu, SCHED(i));
    for (int i = 60; i < 80; i++)
        ROUND(i, b ^ c ^ d, 0xCA62C1D6u, SCHED(i));
#undef ROUND
#undef SCHED

    st[0] += a;
    st[1] += b;
    st[2] += c;
    st[3] += d;
    st[4] += e;
}

/* One block at an arbitrary address, written back like the reference's union cast would. */
static void sha1_block(uint32_t st[5], uint8_t *blk)
{
    uint32_t w[16];
    memcpy(w, blk, 64);
    sha1_compress_inplace(st, w);
    memcpy(blk, w, 64);
}

void BrbSha1_Transform(uint32_t state[5], const uint8_t buffer[64])
{
    sha1_block(state, (uint8_t *)buffer);
}

void BrbSha1_Init(BrbSha1Ctx *context)
{
    context->state[0] = 0x67452301u;
    context->state[1] = 0xEFCDAB89u;
    context->state[2] = 0x98BADCFEu;
    context->state[3] = 0x10325476u;
    context->state[4] = 0xC3D2E1F0u;
    context->count[0] = context->count[1] = 0;
}

void BrbSha1_Update(BrbSha1Ctx *context, const uint8_t *data, const size_t len)
{
    size_t i, j = (context->count[0] >> 3) & 63;

    context->count[0] += (uint32_t)(len << 3);
    if ((size_t)context->count[0] < (len << 3))
        context->count[1]++;
    context->count[1] += (uint32_t)(len >> 29);

    if (j + len > 63) {
        i = 64 - j;
        memcpy(&context->buffer[j], data, i);
        sha1_block(context->state, context->buffer);
        for (; i + 63 < len; i += 64)
            sha1_block(context->state, (uint8_t *)data + i);
        j = 0;
    } else {
        i = 0;
    }
    memcpy(&context->buffer[j], &data[i], len - i);
}

void BrbSha1_Final(BrbSha1Ctx *context, uint8_t digest[BRB_SHA1_DIGEST_SIZE])
{
    uint8_t finalcount[8];
    static const uint8_t pad80 = 0x80, pad00 = 0x00;

    for (int i = 0; i < 8; i++)
        finalcount[i] = (uint8_t)(context->count[i >= 4 ? 0 : 1] >> ((3 - (i & 3)) * 8));
    BrbSha1_Update(context, &pad80, 1);
    while ((context->count[0] & 504) != 448)
        BrbSha1_Update(context, &pad00, 1);
    BrbSha1_Update(context, finalcount, 8);
    for (int i = 0; i < BRB_SHA1_DIGEST_SIZE; i++)
        digest[i] = (uint8_t)(context->state[i >> 2] >> ((3 - (i & 3)) * 8));

    memset(context->buffer, 0, 64);
    memset(context->state, 0, 20);
    memset(context->count, 0, 8);
}

int BrbSha1_Do(const uint8_t *in_ptr, int in_len, char *dig_str)
{
    BrbSha1Ctx ctx;

    if (!in_ptr || !dig_str)
        return -1;

    BrbSha1_Init(&ctx);
    BrbSha1_Update(&ctx, in_ptr, (size_t)in_len);    /* int -> size_t as in sha1.c:213 */
    BrbSha1_Final(&ctx, (uint8_t *)dig_str);
    return 0;
}
