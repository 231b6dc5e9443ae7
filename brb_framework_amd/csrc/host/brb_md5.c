/*
 * brb_md5.c -- compat MD5 surface of libbrb_crypto_gpu.so (host, one streaming context).
 *
 * Behaviour follows libbrb_core/crypto/md5.c (reference @ 2024_10_08):
 *   BRB_MD5Init md5.c:38, UpdateBig :49 (65 535-byte chunks), Update :72 (32-bit byte counter
 *   with carry into bytes[1]), UpdateLowerText :112, Final :134 (0x80, zero pad, 64-bit bit
 *   length, digest, lowercase hex string), Transform :170, LateInitDigestString :255, ToStr :264.
 * Context layout is BRB_MD5_CTX of libbrb_data.h:854-860 (checked by static asserts).
 */
#include "brb_crypto.h"

#include <string.h>

_Static_assert(sizeof(BRB_MD5_CTX) == 168, "BRB_MD5_CTX ABI");
_Static_assert(offsetof(BRB_MD5_CTX, in) == 24 && offsetof(BRB_MD5_CTX, digest) == 88 &&
               offsetof(BRB_MD5_CTX, string) == 104, "BRB_MD5_CTX ABI");

#define ROTL(x, s) (((x) << (s)) | ((x) >> (32 - (s))))
#define MD5_F(x, y, z) ((z) ^ ((x) & ((y) ^ (z))))
#define MD5_G(x, y, z) ((y) ^ ((z) & ((x) ^ (y))))
#define MD5_H(x, y, z) ((x) ^ (y) ^ (z))
#define MD5_I(x, y, z) ((y) ^ ((x) | ~(z)))
#define STEP(fn, a, b, c, d, m, k, s)          \
    do {                                       \
        (a) += fn((b), (c), (d)) + (m) + (k);  \
        (a) = ROTL((a), (s)) + (b);            \
    } while (0)

static void md5_compress(uint32_t st[4], const uint32_t *m)
{
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];

    STEP(MD5_F, a, b, c, d, m[0], 0xd76aa478u, 7);   STEP(MD5_F, d, a, b, c, m[1], 0xe8c7b756u, 12);
    STEP(MD5_F, c, d, a, b, m[2], 0x242070dbu, 17);  STEP(MD5_F, b, c, d, a, m[3], 0xc1bdceeeu, 22);
    STEP(MD5_F, a, b, c, d, m[4], 0xf57c0fafu, 7);   STEP(MD5_F, d, a, b, c, m[5], 0x4787c62au, 12);
    STEP(MD5_F, c, d, a, b, m[6], 0xa8304613u, 17);  STEP(MD5_F, b, c, d, a, m[7], 0xfd469501u, 22);
    STEP(MD5_F, a, b, c, d, m[8], 0x698098d8u, 7);   STEP(MD5_F, d, a, b, c, m[9], 0x8b44f7afu, 12);
    STEP(MD5_F, c, d, a, b, m[10], 0xffff5bb1u, 17); STEP(MD5_F, b, c, d, a, m[11], 0x895cd7beu, 22);
    STEP(MD5_F, a, b, c, d, m[12], 0x6b901122u, 7);  STEP(MD5_F, d, a, b, c, m[13], 0xfd987193u, 12);
    STEP(MD5_F, c, d, a, b, m[14], 0xa679438eu, 17); STEP(MD5_F, b, c, d, a, m[15], 0x49b40821u, 22);

    STEP(MD5_G, a, b, c, d, m[1], 0xf61e2562u, 5);   STEP(MD5_G, d, a, b, c, m[6], 0xc040b340u, 9);
    STEP(MD5_G, c, d, a, b, m[11], 0x265e5a51u, 14); STEP(MD5_G, b, c, d, a, m[0], 0xe9b6c7aau, 20);
    STEP(MD5_G, a, b, c, d, m[5], 0xd62f105du, 5);   STEP(MD5_G, d, a, b, c, m[10], 0x02441453u, 9);
    STEP(MD5_G, c, d, a, b, m[15], 0xd8a1e681u, 14); STEP(MD5_G, b, c, d, a, m[4], 0xe7d3fbc8u, 20);
    STEP(MD5_G, a, b, c, d, m[9], 0x21e1cde6u, 5);   STEP(MD5_G, d, a, b, c, m[14], 0xc33707d6u, 9);
    STEP(MD5_G, c, d, a, b, m[3], 0xf4d50d87u, 14);  STEP(MD5_G, b, c, d, a, m[8], 0x455a14edu, 20);
    STEP(MD5_G, a, b, c, d, m[13], 0xa9e3e905u, 5);  STEP(MD5_G, d, a, b, c, m[2], 0xfcefa3f8u, 9);
    STEP(MD5_G, c, d, a, b, m[7], 0x676f02d9u, 14);  STEP(MD5_G, b, c, d, a, m[12], 0x8d2a4c8au, 20);

    STEP(MD5_H, a, b, c, d, m[5], 0xfffa3942u, 4);   STEP(MD5_H, d, a, b, c, m[8], 0x8771f681u, 11);
    STEP(MD5_H, c, d, a, b, m[11], 0x6d9d6122u, 16); STEP(MD5_H, b, c, d, a, m[14], 0xfde5380cu, 23);
    STEP(MD5_H, a, b, c, d, m[1], 0xa4beea44u, 4);   STEP(MD5_H, d, a, b, c, m[4], 0x4bdecfa9u, 11);
    STEP(MD5_H, c, d, a, b, m[7], 0xf6bb4b60u, 16);  STEP(MD5_H, b, c, d, a, m[10], 0xbebfbc70u, 23);
    STEP(MD5_H, a, b, c, d, m[13], 0x289b7ec6u, 4);  STEP(MD5_H, d, a, b, c, m[0], 0xeaa127fau, 11);
    STEP(MD5_H, c, d, a, b, m[3], 0xd4ef3085u, 16);  STEP(MD5_H, b, c, d, a, m[6], 0x04881d05u, 23);
    STEP(MD5_H, a, b, c, d, m[9], 0xd9d4d039u, 4);   STEP(MD5_H, d, a, b, c, m[12], 0xe6db99e5u, 11);
    STEP(MD5_H, c, d, a, b, m[15], 0x1fa27cf8u, 16); STEP(MD5_H, b, c, d, a, m[2], 0xc4ac5665u, 23);

    STEP(MD5_I, a, b, c, d, m[0], 0xf4292244u, 6);   STEP(MD5_I, d, a, b, c, m[7], 0x432aff97u, 10);
    STEP(MD5_I, c, d, a, b, m[14], 0xab9423a7u, 15); STEP(MD5_I, b, c, d, a, m[5], 0xfc93a039u, 21);
    STEP(MD5_I, a, b, c, d, m[12], 0x655b59c3u, 6);  STEP(MD5_I, d, a, b, c, m[3], 0x8f0ccc92u, 10);
    STEP(MD5_I, c, d, a, b, m[10], 0xffeff47du, 15); STEP(MD5_I, b, c, d, a, m[1], 0x85845dd1u, 21);
    STEP(MD5_I, a, b, c, d, m[8], 0x6fa87e4fu, 6);   STEP(MD5_I, d, a, b, c, m[15], 0xfe2ce6e0u, 10);
    STEP(MD5_I, c, d, a, b, m[6], 0xa3014314u, 15);  STEP(MD5_I, b, c, d, a, m[13], 0x4e0811a1u, 21);
    STEP(MD5_I, a, b, c, d, m[4], 0xf7537e82u, 6);   STEP(MD5_I, d, a, b, c, m[11], 0xbd3af235u, 10);
    STEP(MD5_I, c, d, a, b, m[2], 0x2ad7d2bbu, 15);  STEP(MD5_I, b, c, d, a, m[9], 0xeb86d391u, 21);

    st[0] += a;
    st[1] += b;
    st[2] += c;
    st[3] += d;
}

void BRB_MD5Init(BRB_MD5_CTX *ctx)
{
    ctx->buf[0] = 0x67452301u;
    ctx->buf[1] = 0xefcdab89u;
    ctx->buf[2] = 0x98badcfeu;
    ctx->buf[3] = 0x10325476u;
    ctx->bytes[0] = 0;
    ctx->bytes[1] = 0;
}

void BRB_MD5Transform(BRB_MD5_CTX *ctx)
{
    md5_compress(ctx->buf, ctx->in);
}

void BRB_MD5Update(BRB_MD5_CTX *ctx, const void *_buf, unsigned long len)
{
    const uint8_t *p = (const uint8_t *)_buf;
    unsigned long have = ctx->bytes[0];
    unsigned long room;

    ctx->bytes[0] = (uint32_t)(have + len);
    if ((unsigned long)ctx->bytes[0] < have)
        ctx->bytes[1]++;

    room = 64 - (have & 0x3f);
    if (room > len) {
        memcpy((uint8_t *)ctx->in + 64 - room, p, len);
        return;
    }
    memcpy((uint8_t *)ctx->in + 64 - room, p, room);
    md5_compress(ctx->buf, ctx->in);
    p += room;
    len -= room;

    while (len >= 64) {
        /* the reference copies every block through ctx->in; the state after the call is the same
         * except for the stale copy in ctx->in, which is overwritten below exactly as md5.c:109 */
        uint32_t w[16];
        memcpy(w, p, 64);
        md5_compress(ctx->buf, w);
        if (len < 128)
            memcpy(ctx->in, w, 64);
        p += 64;
        len -= 64;
    }
    memcpy(ctx->in, p, len);
}

void BRB_MD5UpdateBig(BRB_MD5_CTX *ctx, const void *_buf, unsigned long len)
{
    const char *p = (const char *)_buf;
    while (len >= 65535) {
        BRB_MD5Update(ctx, p, 65535);
        p += 65535;
        len -= 65535;
    }
    if (len > 0)
        BRB_MD5Update(ctx, p, len);
}

void BRB_MD5UpdateLowerText(BRB_MD5_CTX *md5_context, char *key_ptr, int key_sz)
{
    char piece[128];
    int done = 0;

    if (!key_ptr || key_sz <= 0)
        return;

    while (done < key_sz) {
        int n = key_sz - done < 128 ? key_sz - done : 128;
        for (int i = 0; i < n; i++) {
            char ch = key_ptr[done + i];
            piece[i] = (ch >= 'A' && ch <= 'Z') ? (char)(ch + 32) : ch;
        }
        BRB_MD5Update(md5_context, piece, (unsigned long)n);
        done += n;
    }
}

static void hex16(const unsigned char *d, unsigned char *out)
{
    static const char hx[] = "0123456789abcdef";
    for (int i = 0; i < 16; i++) {
        out[2 * i] = (unsigned char)hx[d[i] >> 4];
        out[2 * i + 1] = (unsigned char)hx[d[i] & 15];
    }
    out[32] = 0;
}

void BRB_MD5LateInitDigestString(BRB_MD5_CTX *ret)
{
    hex16(ret->digest, ret->string);
}

void BRB_MD5ToStr(unsigned char *bin_digest, unsigned char *ret_buf_str)
{
    hex16(bin_digest, ret_buf_str);
}

void BRB_MD5Final(BRB_MD5_CTX *ctx)
{
    unsigned used = ctx->bytes[0] & 0x3f;
    uint8_t *in = (uint8_t *)ctx->in;

    in[used++] = 0x80;
    if (used > 56) {
        memset(in + used, 0, 64 - used);
        md5_compress(ctx->buf, ctx->in);
        used = 0;
    }
    memset(in + used, 0, 56 - used);
    ctx->in[14] = ctx->bytes[0] << 3;
    ctx->in[15] = (ctx->bytes[1] << 3) | (ctx->bytes[0] >> 29);
    md5_compress(ctx->buf, ctx->in);

    memcpy(ctx->digest, ctx->buf, 16);
    BRB_MD5LateInitDigestString(ctx);
}
