/*
 * brb_oracle.c -- CPU ORACLE (test infrastructure only; see brb_oracle.h for who may use it and
 * how its parity is pinned).  Deliberately written as plain loops over tables, not as the
 * unrolled macro form of the reference, so that it is an independent restatement.
 */
#include "brb_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

static uint32_t rotl32(uint32_t x, unsigned s) { return (x << s) | (x >> ((32 - s) & 31)); }

/* =========================================================================================== */
/* MD5 -- libbrb_core/crypto/md5.c                                                              */
/* =========================================================================================== */

/* RFC 1321 §3.4: T[i] = floor(|sin(i + 1)| * 2^32); per-round shift amounts.  The reference
 * writes the same 64 constants as literals in BRB_MD5Transform (md5.c:179-245). */
static uint32_t md5_T[64];
static const unsigned md5_shift[4][4] = {{7, 12, 17, 22}, {5, 9, 14, 20}, {4, 11, 16, 23}, {6, 10, 15, 21}};
static pthread_once_t md5_once = PTHREAD_ONCE_INIT;

static void md5_tables(void)
{
    for (int i = 0; i < 64; i++)
        md5_T[i] = (uint32_t)(uint64_t)floor(fabs(sin((double)(i + 1))) * 4294967296.0);
}

/* Message word of step i: RFC 1321 §3.4's per-round index progressions. */
static int md5_word(int i)
{
    switch (i >> 4) {
    case 0: return i;
    case 1: return (5 * i + 1) & 15;
    case 2: return (3 * i + 5) & 15;
    default: return (7 * i) & 15;
    }
}

/* One compression of c->in into c->buf (md5.c:170-253). */
static void orc_md5_transform(orc_md5_ctx *c)
{
    uint32_t a = c->buf[0], b = c->buf[1], cc = c->buf[2], d = c->buf[3];
    for (int i = 0; i < 64; i++) {
        int r = i >> 4;
        uint32_t f;
        switch (r) {       /* F1..F4 of libbrb_data.h:845-848 */
        case 0: f = d ^ (b & (cc ^ d)); break;
        case 1: f = cc ^ (d & (b ^ cc)); break;
        case 2: f = b ^ cc ^ d; break;
        default: f = cc ^ (b | ~d); break;
        }
        uint32_t t = a + f + c->in[md5_word(i)] + md5_T[i];     /* MD5STEP, libbrb_data.h:851 */
        a = d;
        d = cc;
        cc = b;
        b = b + rotl32(t, md5_shift[r][i & 3]);
    }
    c->buf[0] += a;
    c->buf[1] += b;
    c->buf[2] += cc;
    c->buf[3] += d;
}

void orc_md5_init(orc_md5_ctx *c)                       /* md5.c:38-47 */
{
    pthread_once(&md5_once, md5_tables);
    c->buf[0] = 0x67452301u;
    c->buf[1] = 0xefcdab89u;
    c->buf[2] = 0x98badcfeu;
    c->buf[3] = 0x10325476u;
    c->bytes[0] = c->bytes[1] = 0;
}

void orc_md5_update(orc_md5_ctx *c, const void *p, unsigned long len)   /* md5.c:72-110 */
{
    const uint8_t *s = (const uint8_t *)p;
    unsigned long t = c->bytes[0];
    c->bytes[0] = (uint32_t)(t + len);
    if ((unsigned long)c->bytes[0] < t)           /* 32-bit carry into bytes[1] (md5.c:80-81) */
        c->bytes[1]++;
    unsigned long room = 64 - (t & 0x3f);
    uint8_t *in = (uint8_t *)c->in;
    if (room > len) {
        memcpy(in + 64 - room, s, len);
        return;
    }
    memcpy(in + 64 - room, s, room);
    orc_md5_transform(c);
    s += room;
    len -= room;
    for (; len >= 64; s += 64, len -= 64) {
        memcpy(in, s, 64);
        orc_md5_transform(c);
    }
    memcpy(in, s, len);
}

void orc_md5_update_big(orc_md5_ctx *c, const void *p, unsigned long len)   /* md5.c:49-70 */
{
    const uint8_t *s = (const uint8_t *)p;
    while (len >= 65535) {
        orc_md5_update(c, s, 65535);
        s += 65535;
        len -= 65535;
    }
    if (len)
        orc_md5_update(c, s, len);
}

void orc_md5_final(orc_md5_ctx *c)                     /* md5.c:134-168 */
{
    static const char hx[] = "0123456789abcdef";
    int count = c->bytes[0] & 0x3f;
    uint8_t *in = (uint8_t *)c->in;
    in[count] = 0x80;
    if (count + 1 > 56) {                    /* padding forces an extra block (md5.c:147-153) */
        memset(in + count + 1, 0, 63 - count);
        orc_md5_transform(c);
        memset(in, 0, 56);
    } else {
        memset(in + count + 1, 0, 55 - count);
    }
    c->in[14] = c->bytes[0] << 3;
    c->in[15] = (c->bytes[1] << 3) | (c->bytes[0] >> 29);
    orc_md5_transform(c);
    memcpy(c->digest, c->buf, 16);
    for (int i = 0; i < 16; i++) {           /* lowercase hex, md5.c:255-262 */
        c->string[2 * i] = (unsigned char)hx[c->digest[i] >> 4];
        c->string[2 * i + 1] = (unsigned char)hx[c->digest[i] & 15];
    }
    c->string[32] = 0;
}

void orc_md5(const void *p, uint64_t len, uint8_t out[16])
{
    orc_md5_ctx c;
    orc_md5_init(&c);
    orc_md5_update_big(&c, p, (unsigned long)len);
    orc_md5_final(&c);
    memcpy(out, c.digest, 16);
}

/* =========================================================================================== */
/* SHA-1 -- libbrb_core/crypto/sha1.c                                                           */
/* =========================================================================================== */

/* FIPS 180-1 round constants, one per 20 steps (the reference's R0/R1..R4 macros, sha1.c:54-58). */
static const uint32_t sha1_K[4] = {0x5A827999u, 0x6ED9EBA1u, 0x8F1BBCDCu, 0xCA62C1D6u};

/* Compression of one 64-byte block (sha1.c:75-130).  With SHA1HANDSOFF undefined the reference
 * expands the schedule inside the caller's block: on return the block holds W[64..79] in host
 * (little-endian) order.  `block` is mutated the same way here. */
static void orc_sha1_transform_x(uint32_t st[5], uint8_t *block, int mutate)
{
    uint32_t W[80];
    for (int i = 0; i < 16; i++)
        W[i] = ((uint32_t)block[4 * i] << 24) | ((uint32_t)block[4 * i + 1] << 16) |
               ((uint32_t)block[4 * i + 2] << 8) | (uint32_t)block[4 * i + 3];
    for (int i = 16; i < 80; i++)
        W[i] = rotl32(W[i - 3] ^ W[i - 8] ^ W[i - 14] ^ W[i - 16], 1);
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4];
    for (int i = 0; i < 80; i++) {
        uint32_t f;
        const uint32_t k = sha1_K[i / 20];
        if (i < 20) f = (b & c) | (~b & d);
        else if (i < 40) f = b ^ c ^ d;
        else if (i < 60) f = (b & c) | (b & d) | (c & d);
        else f = b ^ c ^ d;
        uint32_t t = rotl32(a, 5) + f + e + k + W[i];
        e = d;
        d = c;
        c = rotl32(b, 30);
        b = a;
        a = t;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e;
    if (mutate)
        memcpy(block, &W[64], 64);           /* the in-place side effect, native byte order */
}

static void orc_sha1_transform(uint32_t st[5], uint8_t *block) { orc_sha1_transform_x(st, block, 1); }

void orc_sha1_init(orc_sha1_ctx *c)                     /* sha1.c:132-141 */
{
    c->state[0] = 0x67452301u;
    c->state[1] = 0xEFCDAB89u;
    c->state[2] = 0x98BADCFEu;
    c->state[3] = 0x10325476u;
    c->state[4] = 0xC3D2E1F0u;
    c->count[0] = c->count[1] = 0;
}

static void sha1_update_x(orc_sha1_ctx *c, uint8_t *data, size_t len, int mutate)   /* sha1.c:143-169 */
{
    size_t i, j = (c->count[0] >> 3) & 63;
    /* Counter arithmetic exactly as sha1.c:151-152: the carry test compares the 32-bit sum with
     * the size_t (len << 3), so len >= 2^29 always adds one extra carry. */
    c->count[0] += (uint32_t)(len << 3);
    if ((size_t)c->count[0] < (len << 3))
        c->count[1]++;
    c->count[1] += (uint32_t)(len >> 29);
    if (j + len > 63) {
        i = 64 - j;
        memcpy(&c->buffer[j], data, i);
        orc_sha1_transform(c->state, c->buffer);
        for (; i + 63 < len; i += 64)
            orc_sha1_transform_x(c->state, data + i, mutate);   /* mutates data[i .. i+63] */
        j = 0;
    } else {
        i = 0;
    }
    memcpy(&c->buffer[j], data + i, len - i);
}

void orc_sha1_update(orc_sha1_ctx *c, uint8_t *data, size_t len) { sha1_update_x(c, data, len, 1); }

void orc_sha1_final(orc_sha1_ctx *c, uint8_t out[20])   /* sha1.c:171-200 */
{
    uint8_t fc[8], b80 = 0x80, b00 = 0;
    for (int i = 0; i < 8; i++)
        fc[i] = (uint8_t)(c->count[i >= 4 ? 0 : 1] >> ((3 - (i & 3)) * 8));
    orc_sha1_update(c, &b80, 1);
    while ((c->count[0] & 504) != 448)
        orc_sha1_update(c, &b00, 1);
    orc_sha1_update(c, fc, 8);
    for (int i = 0; i < 20; i++)
        out[i] = (uint8_t)(c->state[i >> 2] >> ((3 - (i & 3)) * 8));
    memset(c, 0, sizeof(*c));
}

void orc_sha1(const void *p, uint64_t len, uint8_t out[20])
{
    /* BrbSha1_Do semantics (sha1.c:203-216: Init, ONE Update of len, Final) but without writing
     * the schedule back into the caller's bytes (the batch surface never mutates its input). */
    orc_sha1_ctx c;
    orc_sha1_init(&c);
    sha1_update_x(&c, (uint8_t *)p, (size_t)len, 0);
    orc_sha1_final(&c, out);
}

/* =========================================================================================== */
/* Blowfish -- libbrb_core/crypto/blowfish.c, with 64-bit unsigned long words                   */
/* =========================================================================================== */

/* Hex digit extraction of pi (Bailey-Borwein-Plouffe).  Returns frac(16^n * S_j) pieces. */
static long double bbp_series(int j, long n)
{
    long double s = 0.0L;
    for (long k = 0; k <= n; k++) {
        uint64_t m = (uint64_t)(8 * k + j), r = 1 % m, b = 16 % m;
        for (uint64_t e = (uint64_t)(n - k); e; e >>= 1) {       /* 16^(n-k) mod m, exact */
            if (e & 1) r = (r * b) % m;
            b = (b * b) % m;
        }
        s += (long double)r / (long double)m;
        s -= floorl(s);
    }
    for (long k = n + 1; k <= n + 24; k++) {
        s += powl(16.0L, (long double)(n - k)) / (long double)(8 * k + j);
    }
    return s - floorl(s);
}

static uint32_t pi_word(long idx)        /* hex digits [8 idx, 8 idx + 8) after the point */
{
    long n = 8 * idx;
    long double x = 4 * bbp_series(1, n) - 2 * bbp_series(4, n) - bbp_series(5, n) - bbp_series(6, n);
    x -= floorl(x);
    uint32_t w = 0;
    for (int i = 0; i < 8; i++) {
        x *= 16.0L;
        int dgt = (int)x;
        w = (w << 4) | (uint32_t)dgt;
        x -= dgt;
    }
    return w;
}

static uint32_t bf_pi[1042];
static pthread_once_t bf_once = PTHREAD_ONCE_INIT;
static void bf_pi_init(void)
{
    for (long i = 0; i < 1042; i++)
        bf_pi[i] = pi_word(i);
}

void orc_bf_pi_words(uint32_t out[1042])
{
    pthread_once(&bf_once, bf_pi_init);
    memcpy(out, bf_pi, sizeof(bf_pi));
}

static uint64_t bf_F(const orc_bf_ctx *c, uint64_t x)   /* _F, blowfish.c:445-462 */
{
    unsigned a = (unsigned)(x >> 24) & 0xFF, b = (unsigned)(x >> 16) & 0xFF;
    unsigned cc = (unsigned)(x >> 8) & 0xFF, d = (unsigned)x & 0xFF;
    return ((c->S[0][a] + c->S[1][b]) ^ c->S[2][cc]) + c->S[3][d];   /* 64-bit, no 32-bit wrap */
}

void orc_bf_encrypt(const orc_bf_ctx *c, uint64_t *xl, uint64_t *xr)   /* blowfish.c:312-345 */
{
    uint64_t L = *xl, R = *xr, t;
    for (int i = 0; i < 16; i++) {
        L ^= c->P[i];
        R ^= bf_F(c, L);
        t = L; L = R; R = t;
    }
    t = L; L = R; R = t;
    R ^= c->P[16];
    L ^= c->P[17];
    *xl = L;
    *xr = R;
}

void orc_bf_decrypt(const orc_bf_ctx *c, uint64_t *xl, uint64_t *xr)   /* blowfish.c:347-380 */
{
    uint64_t L = *xl, R = *xr, t;
    for (int i = 17; i > 1; i--) {
        L ^= c->P[i];
        R ^= bf_F(c, L);
        t = L; L = R; R = t;
    }
    t = L; L = R; R = t;
    R ^= c->P[1];
    L ^= c->P[0];
    *xl = L;
    *xr = R;
}

void orc_bf_init(orc_bf_ctx *c, const unsigned char *key, int key_len)   /* blowfish.c:382-443 */
{
    pthread_once(&bf_once, bf_pi_init);
    for (int s = 0; s < 4; s++)
        for (int i = 0; i < 256; i++)
            c->S[s][i] = bf_pi[18 + 256 * s + i];
    int j = 0;
    for (int i = 0; i < 18; i++) {
        uint64_t data = 0;
        for (int k = 0; k < 4; k++) {
            data = (data << 8) | key[j];
            j++;
            if (j >= key_len)            /* key_len <= 0 therefore always re-reads key[0] */
                j = 0;
        }
        c->P[i] = (uint64_t)bf_pi[i] ^ data;
    }
    uint64_t L = 0, R = 0;
    for (int i = 0; i < 18; i += 2) {
        orc_bf_encrypt(c, &L, &R);
        c->P[i] = L;
        c->P[i + 1] = R;
    }
    for (int s = 0; s < 4; s++)
        for (int i = 0; i < 256; i += 2) {
            orc_bf_encrypt(c, &L, &R);
            c->S[s][i] = L;
            c->S[s][i + 1] = R;
        }
}

typedef struct {
    const orc_bf_ctx *c;
    uint64_t *w;
    uint64_t b0, b1;
    int dec;
} bf_job;

static void *bf_worker(void *arg)
{
    bf_job *j = (bf_job *)arg;
    for (uint64_t b = j->b0; b < j->b1; b++) {
        if (j->dec) orc_bf_decrypt(j->c, &j->w[2 * b], &j->w[2 * b + 1]);
        else orc_bf_encrypt(j->c, &j->w[2 * b], &j->w[2 * b + 1]);
    }
    return NULL;
}

void orc_bf_ecb(const orc_bf_ctx *c, uint64_t *words, uint64_t n_blocks, int decrypt, int n_threads)
{
    if (n_threads < 1) n_threads = 1;
    if (n_threads > 256) n_threads = 256;
    pthread_t th[256];
    bf_job jobs[256];
    for (int t = 0; t < n_threads; t++) {
        jobs[t].c = c;
        jobs[t].w = words;
        jobs[t].b0 = n_blocks * (uint64_t)t / (uint64_t)n_threads;
        jobs[t].b1 = n_blocks * (uint64_t)(t + 1) / (uint64_t)n_threads;
        jobs[t].dec = decrypt;
    }
    if (n_threads == 1) { bf_worker(&jobs[0]); return; }
    for (int t = 0; t < n_threads; t++) pthread_create(&th[t], NULL, bf_worker, &jobs[t]);
    for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
}

/* MemBuffer Blowfish wrappers, mem_buf.c:1499-1617 ------------------------------------------- */
void orc_membuf_key(unsigned int seed, unsigned int key[16])       /* mem_buf.c:1511-1515 */
{
    for (unsigned long i = 0; i < 16; i++) {
        key[i] = (unsigned int)(((i + seed) * seed) + (13 * i));
        seed = key[i] * seed;
    }
}

static uint64_t ld64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }
static void st64(uint8_t *p, uint64_t v) { memcpy(p, &v, 8); }

uint64_t orc_membuf_encrypt(uint8_t *buf, uint64_t size, unsigned int seed, uint64_t offset)
{
    unsigned int key[16];
    orc_bf_ctx c;
    uint64_t blocks = (size + offset) / 8 + 2;            /* mem_buf.c:1503-1504, :1518 */
    orc_membuf_key(seed, key);
    orc_bf_init(&c, (const unsigned char *)key, 4);      /* sizeof(enc_key[16]) == 4, :1528 */
    uint8_t *raw = buf + offset;
    uint64_t i;
    for (i = 0; i < blocks; i += 2) {                     /* :1538-1539 */
        uint64_t l = ld64(raw + 8 * i), r = ld64(raw + 8 * (i + 1));
        orc_bf_encrypt(&c, &l, &r);
        st64(raw + 8 * i, l);
        st64(raw + 8 * (i + 1), r);
    }
    return i * 8 + offset;                                /* :1542 */
}

uint64_t orc_membuf_decrypt(uint8_t *buf, uint64_t size, unsigned int seed, uint64_t offset)
{
    unsigned int key[16];
    orc_bf_ctx c;
    uint64_t blocks = (size - offset) / 8 + 2;            /* mem_buf.c:1557-1558, :1571 */
    orc_membuf_key(seed, key);
    orc_bf_init(&c, (const unsigned char *)key, 64);     /* sizeof(enc_key) == 64, :1582 */
    uint8_t *raw = buf + offset;
    uint64_t i;
    for (i = 0; i < blocks; i += 2) {
        uint64_t l = ld64(raw + 8 * i), r = ld64(raw + 8 * (i + 1));
        if (l == 0 || r == 0)                             /* "padding gremlin", :1595-1596 */
            break;
        orc_bf_decrypt(&c, &l, &r);
        st64(raw + 8 * i, l);
        st64(raw + 8 * (i + 1), r);
    }
    return i * 8 + offset;                                /* :1609 */
}

/* =========================================================================================== */
/* Batches                                                                                       */
/* =========================================================================================== */
typedef struct {
    const uint8_t *data;
    uint32_t L;
    uint64_t r0, r1;
    uint8_t *out;
    int sha;
} dig_job;

static void *dig_worker(void *arg)
{
    dig_job *j = (dig_job *)arg;
    for (uint64_t r = j->r0; r < j->r1; r++) {
        if (j->sha) orc_sha1(j->data + r * j->L, j->L, j->out + 20 * r);
        else orc_md5(j->data + r * j->L, j->L, j->out + 16 * r);
    }
    return NULL;
}

static void dig_fixed(const uint8_t *data, uint32_t L, uint64_t n, uint8_t *out, int n_threads, int sha)
{
    if (n_threads < 1) n_threads = 1;
    if (n_threads > 256) n_threads = 256;
    pthread_t th[256];
    dig_job jobs[256];
    for (int t = 0; t < n_threads; t++) {
        jobs[t].data = data;
        jobs[t].L = L;
        jobs[t].r0 = n * (uint64_t)t / (uint64_t)n_threads;
        jobs[t].r1 = n * (uint64_t)(t + 1) / (uint64_t)n_threads;
        jobs[t].out = out;
        jobs[t].sha = sha;
    }
    if (n_threads == 1) { dig_worker(&jobs[0]); return; }
    for (int t = 0; t < n_threads; t++) pthread_create(&th[t], NULL, dig_worker, &jobs[t]);
    for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
}

void orc_md5_batch_fixed(const uint8_t *data, uint32_t L, uint64_t n, uint8_t *out16, int n_threads)
{
    pthread_once(&md5_once, md5_tables);
    dig_fixed(data, L, n, out16, n_threads, 0);
}

void orc_sha1_batch_fixed(const uint8_t *data, uint32_t L, uint64_t n, uint8_t *out20, int n_threads)
{
    dig_fixed(data, L, n, out20, n_threads, 1);
}

void orc_md5_batch(const uint8_t *data, const uint64_t *off, const uint32_t *len, uint64_t n, uint8_t *out16)
{
    for (uint64_t r = 0; r < n; r++) orc_md5(data + off[r], len[r], out16 + 16 * r);
}

void orc_sha1_batch(const uint8_t *data, const uint64_t *off, const uint32_t *len, uint64_t n, uint8_t *out20)
{
    for (uint64_t r = 0; r < n; r++) orc_sha1(data + off[r], len[r], out20 + 20 * r);
}

/* The same on n_threads pthreads over contiguous record ranges (bench.py's cpu_baseline of the
 * variable-length legs). */
typedef struct {
    const uint8_t *data;
    const uint64_t *off;
    const uint32_t *len;
    uint64_t r0, r1;
    uint8_t *out;
    int sha;
} var_job;

static void *var_worker(void *arg)
{
    var_job *j = (var_job *)arg;
    if (j->sha) orc_sha1_batch(j->data, j->off + j->r0, j->len + j->r0, j->r1 - j->r0, j->out + 20 * j->r0);
    else orc_md5_batch(j->data, j->off + j->r0, j->len + j->r0, j->r1 - j->r0, j->out + 16 * j->r0);
    return NULL;
}

static void var_run(const uint8_t *data, const uint64_t *off, const uint32_t *len, uint64_t n, uint8_t *out,
                    int n_threads, int sha)
{
    pthread_once(&md5_once, md5_tables);
    if (n_threads < 1) n_threads = 1;
    if (n_threads > 256) n_threads = 256;
    pthread_t th[256];
    var_job jobs[256];
    for (int t = 0; t < n_threads; t++) {
        jobs[t] = (var_job){data, off, len, n * (uint64_t)t / (uint64_t)n_threads,
                            n * (uint64_t)(t + 1) / (uint64_t)n_threads, out, sha};
    }
    if (n_threads == 1) { var_worker(&jobs[0]); return; }
    for (int t = 0; t < n_threads; t++) pthread_create(&th[t], NULL, var_worker, &jobs[t]);
    for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
}

void orc_md5_batch_mt(const uint8_t *data, const uint64_t *off, const uint32_t *len, uint64_t n, uint8_t *out16,
                      int n_threads)
{
    var_run(data, off, len, n, out16, n_threads, 0);
}

void orc_sha1_batch_mt(const uint8_t *data, const uint64_t *off, const uint32_t *len, uint64_t n, uint8_t *out20,
                       int n_threads)
{
    var_run(data, off, len, n, out20, n_threads, 1);
}

/* =========================================================================================== */
/* RC4 -- libbrb_core/crypto/rc4.c                                                               */
/* =========================================================================================== */

/* rc4.c:40-62: identity permutation, indices zeroed, then one key-scheduling sweep with an 8-bit
 * accumulator j and key bytes cycled by i % keylen.  `flags` is left as it was. */
void orc_rc4_init(orc_rc4_state *s, const unsigned char *key, int keylen)
{
    for (int i = 0; i < 256; i++) s->perm[i] = (unsigned char)i;
    s->index1 = 0;
    s->index2 = 0;
    unsigned j = 0;
    for (int i = 0; i < 256; i++) {
        j = (j + s->perm[i] + key[i % keylen]) & 255u;
        unsigned char t = s->perm[i];
        s->perm[i] = s->perm[j];
        s->perm[j] = t;
    }
}

/* rc4.c:64-87: per byte, index1 += 1, index2 += perm[index1], swap, out = in ^ perm[perm[index1] +
 * perm[index2]] (all 8-bit).  in == out is allowed. */
void orc_rc4_crypt(orc_rc4_state *s, const unsigned char *in, unsigned char *out, int n)
{
    unsigned a = s->index1, b = s->index2;
    for (int k = 0; k < n; k++) {
        a = (a + 1) & 255u;
        b = (b + s->perm[a]) & 255u;
        unsigned char t = s->perm[a];
        s->perm[a] = s->perm[b];
        s->perm[b] = t;
        out[k] = in[k] ^ s->perm[(s->perm[a] + s->perm[b]) & 255u];
    }
    s->index1 = (unsigned char)a;
    s->index2 = (unsigned char)b;
}

/* RC4 over more than INT_MAX bytes in int-sized pieces (the keystream is position-only). */
static void rc4_crypt_big(orc_rc4_state *s, const uint8_t *in, uint8_t *out, uint64_t n)
{
    while (n) {
        int piece = n > (1u << 30) ? (1 << 30) : (int)n;
        orc_rc4_crypt(s, in, out, piece);
        in += piece;
        out += piece;
        n -= (uint64_t)piece;
    }
}

/* ev_kq_aio_transform.c:212-230 then :281-283 (WRITE side). */
void orc_rc4md5_frame(orc_rc4_state *s, const uint8_t *payload, uint64_t len, uint64_t salt, uint8_t *frame)
{
    uint8_t dig[16];
    orc_md5(payload, len, dig);
    memcpy(frame, &salt, 8);                /* MemBufferAdd(&random_salt, sizeof(unsigned long)) */
    memcpy(frame + 8, "HASH:", 5);
    memcpy(frame + 13, dig, 16);
    frame[29] = 0;
    memcpy(frame + ORC_RC4MD5_HDR, payload, len);
    rc4_crypt_big(s, frame, frame, ORC_RC4MD5_HDR + len);
}

/* ev_kq_aio_transform.c:270-279 (READ side, in place) then DataValidate (:158-184). */
int orc_rc4md5_open(orc_rc4_state *s, uint8_t *frame, uint64_t frame_len)
{
    rc4_crypt_big(s, frame, frame, frame_len);
    if (frame_len < ORC_RC4MD5_HDR) return 0;
    if (memcmp(frame + 8, "HASH:", 5)) return 0;
    uint8_t dig[16];
    orc_md5(frame + ORC_RC4MD5_HDR, frame_len - ORC_RC4MD5_HDR, dig);
    return memcmp(dig, frame + 13, 16) == 0;
}

typedef struct {
    orc_rc4_state *s;
    const uint8_t *payload;
    uint8_t *frames;
    const uint64_t *off, *foff, *salts;
    const uint32_t *len;
    uint8_t *valid;
    uint64_t r0, r1;
} rc4_job;

static void *rc4_frame_worker(void *arg)
{
    rc4_job *j = (rc4_job *)arg;
    for (uint64_t r = j->r0; r < j->r1; r++)
        orc_rc4md5_frame(&j->s[r], j->payload + j->off[r], j->len[r], j->salts[r], j->frames + j->foff[r]);
    return NULL;
}

static void *rc4_open_worker(void *arg)
{
    rc4_job *j = (rc4_job *)arg;
    for (uint64_t r = j->r0; r < j->r1; r++)
        j->valid[r] = (uint8_t)orc_rc4md5_open(&j->s[r], j->frames + j->off[r], j->len[r]);
    return NULL;
}

static void rc4_run(rc4_job proto, uint64_t n, int n_threads, void *(*fn)(void *))
{
    pthread_once(&md5_once, md5_tables);
    if (n_threads < 1) n_threads = 1;
    if (n_threads > 256) n_threads = 256;
    pthread_t th[256];
    rc4_job jobs[256];
    for (int t = 0; t < n_threads; t++) {
        jobs[t] = proto;
        jobs[t].r0 = n * (uint64_t)t / (uint64_t)n_threads;
        jobs[t].r1 = n * (uint64_t)(t + 1) / (uint64_t)n_threads;
    }
    if (n_threads == 1) { fn(&jobs[0]); return; }
    for (int t = 0; t < n_threads; t++) pthread_create(&th[t], NULL, fn, &jobs[t]);
    for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
}

static void *rc4_crypt_worker(void *arg)
{
    rc4_job *j = (rc4_job *)arg;
    for (uint64_t r = j->r0; r < j->r1; r++)
        orc_rc4_crypt(&j->s[r], j->frames + j->off[r], j->frames + j->off[r], (int)j->len[r]);
    return NULL;
}

/* BRB_RC4_Crypt in place on n streams (stream r = data[off[r] .. + len[r]) with state s[r]). */
void orc_rc4_crypt_batch(orc_rc4_state *s, uint8_t *data, const uint64_t *off, const uint32_t *len, uint64_t n,
                         int n_threads)
{
    rc4_job p = {s, NULL, data, off, NULL, NULL, len, NULL, 0, 0};
    rc4_run(p, n, n_threads, rc4_crypt_worker);
}

void orc_rc4md5_frame_batch(orc_rc4_state *s, const uint8_t *payload, const uint64_t *off, const uint32_t *len,
                            const uint64_t *salts, uint8_t *frames, const uint64_t *foff, uint64_t n, int n_threads)
{
    rc4_job p = {s, payload, frames, off, foff, salts, len, NULL, 0, 0};
    rc4_run(p, n, n_threads, rc4_frame_worker);
}

void orc_rc4md5_open_batch(orc_rc4_state *s, uint8_t *frames, const uint64_t *off, const uint32_t *len, uint64_t n,
                           uint8_t *valid, int n_threads)
{
    rc4_job p = {s, NULL, frames, off, NULL, NULL, len, valid, 0, 0};
    rc4_run(p, n, n_threads, rc4_open_worker);
}

/* =========================================================================================== */
/* base64 -- libbrb_core/crypto/base64.c                                                         */
/* =========================================================================================== */
static const char b64_code[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

/* base64.c:304-361: 3 bytes -> 4 characters; a 1- or 2-byte tail is shifted up and padded */
uint64_t orc_b64_encode(const uint8_t *in, uint64_t len, char *out)
{
    uint64_t o = 0, k = 0;
    for (; k + 3 <= len; k += 3) {
        uint32_t v = ((uint32_t)in[k] << 16) | ((uint32_t)in[k + 1] << 8) | in[k + 2];
        out[o++] = b64_code[v >> 18];
        out[o++] = b64_code[(v >> 12) & 63];
        out[o++] = b64_code[(v >> 6) & 63];
        out[o++] = b64_code[v & 63];
    }
    uint64_t t = len - k;
    if (t) {
        uint32_t v = (uint32_t)in[k] << 16;
        if (t == 2) v |= (uint32_t)in[k + 1] << 8;
        out[o++] = b64_code[v >> 18];
        out[o++] = b64_code[(v >> 12) & 63];
        out[o++] = t == 2 ? b64_code[(v >> 6) & 63] : '=';
        out[o++] = '=';
    }
    return o;
}

/* base64.c:363-376 value table: the alphabet, '=' -> 0, everything else -> skipped */
static int b64_value(unsigned char c)
{
    if (c == '=') return 0;
    const char *p = memchr(b64_code, c, 64);
    return (c && p) ? (int)(p - b64_code) : -1;
}

/* base64.c:131-179 */
uint64_t orc_b64_decode(const char *in, uint64_t len, uint8_t *out)
{
    uint64_t o = 0;
    uint32_t val = 0, c = 0;
    for (uint64_t k = 0; k < len && in[k]; k++) {
        int v = b64_value((unsigned char)in[k]);
        if (v < 0) continue;
        val = (val << 6) + (uint32_t)v;
        if (++c < 4) continue;
        out[o++] = (uint8_t)(val >> 16);
        out[o++] = (uint8_t)(val >> 8);
        out[o++] = (uint8_t)val;
        val = c = 0;
    }
    return o;
}

/* =========================================================================================== */
/* MetaData packs -- libbrb_core/data/utils/meta_data.c, libbrb_data.h:291-330 (LP64)           */
/* =========================================================================================== */
/* header: int version @0, int item_count @4, unsigned long size @8, "BRB_META" @16, MD5 @24,
 * 24 reserved bytes @40; item: unsigned long item_id, item_sub_id, sz; data; 0x1F */
static void put_le(uint8_t *p, uint64_t v, int n)
{
    for (int k = 0; k < n; k++)
        p[k] = (uint8_t)(v >> (8 * k));
}

/* MetaDataPack (meta_data.c:104-140) with MetaDataHeaderLoadData (:397-433): returns the bytes written */
uint64_t orc_metadata_pack(const uint8_t *data, const uint64_t *off, const uint64_t *len, const uint64_t *id,
                           const uint64_t *sub, uint64_t n_items, uint8_t *out)
{
    orc_md5_ctx c;
    memset(&c, 0, sizeof(c));
    orc_md5_init(&c);
    uint64_t size = 0;
    for (uint64_t i = 0; i < n_items; i++) {
        orc_md5_update_big(&c, data + off[i], (unsigned long)len[i]);
        size += len[i] + 24 + 1;
    }
    orc_md5_final(&c);
    memset(out, 0, 64);
    put_le(out + 4, (uint32_t)(int32_t)n_items, 4);
    put_le(out + 8, size, 8);
    memcpy(out + 16, "BRB_META", 8);
    memcpy(out + 24, c.digest, 16);
    uint64_t o = 64;
    for (uint64_t i = 0; i < n_items; i++) {
        put_le(out + o, id[i], 8);
        put_le(out + o + 8, sub[i], 8);
        put_le(out + o + 16, len[i], 8);
        memcpy(out + o + 24, data + off[i], len[i]);
        out[o + 24 + len[i]] = 0x1F;
        o += 24 + len[i] + 1;
    }
    return o;
}

/* a byte of the pack, 0 past its end (the reference reads whatever its MemBuffer holds there) */
static uint8_t md_byte(const uint8_t *b, uint64_t size, uint64_t pos) { return pos < size ? b[pos] : 0; }
static uint64_t md_u64(const uint8_t *b, uint64_t size, uint64_t pos)
{
    uint64_t v = 0;
    for (int k = 0; k < 8; k++)
        v |= (uint64_t)md_byte(b, size, pos + (uint64_t)k) << (8 * k);
    return v;
}

/* MetaDataUnpack (meta_data.c:145-328) of a MemBuffer holding the pack at offset 0; info = the
 * MetaDataUnpackerInfo fields plus the count of items unpacked.  Returns error_code. */
int orc_metadata_unpack(const uint8_t *b, uint64_t size, orc_md_info *info)
{
    uint64_t cur_offset = 0, cur_remaining = 0, cur_needed = 0, pos = 0;
    uint32_t items = 0;
    int code = 7;                                                    /* METADATA_UNPACK_SUCCESS */
    const int32_t item_count = (int32_t)(uint32_t)(md_u64(b, size, 0) >> 32);
    if (md_u64(b, size, 16) != md_u64((const uint8_t *)"BRB_META", 8, 0)) {   /* :183-195 */
        code = 0;
        goto out;
    }
    orc_md5_ctx c;
    memset(&c, 0, sizeof(c));
    orc_md5_init(&c);
    pos = 64;                                                        /* :198-199 */
    cur_offset += 64;
    for (int32_t i = 0; i < item_count; i++) {                       /* :202 */
        cur_remaining = size - pos;                                  /* :213 */
        if (cur_remaining < 32) {                                    /* :216-224, sizeof(MetaDataItem) */
            cur_needed = 32 - cur_remaining;
            code = 5;
            goto out;
        }
        const uint64_t sz = md_u64(b, size, pos + 16);
        pos += 24;                                                   /* :227-232 */
        cur_offset += 24;
        cur_remaining -= 24;
        if (cur_remaining < sz + 1 || sz > size) {                   /* :237-246 */
            cur_needed = sz + 1 - cur_remaining;
            code = 6;
            goto out;
        }
        if (pos + sz <= size) {                                      /* :249-254 */
            orc_md5_update_big(&c, b + pos, (unsigned long)sz);
        } else {                                                     /* past the pack: zeros */
            for (uint64_t k = 0; k < sz; k++) {
                uint8_t v = md_byte(b, size, pos + k);
                orc_md5_update_big(&c, &v, 1);
            }
        }
        pos += sz;
        cur_offset += sz;
        cur_remaining -= sz;
        if (md_byte(b, size, pos) != 0x1F) {                         /* :258-268 */
            code = 3;
            goto out;
        }
        pos += 1;                                                    /* :271-277 */
        cur_offset += 1;
        cur_remaining -= 1;
        items++;
        if (pos == size)                                             /* :280-281 */
            break;
    }
    orc_md5_final(&c);                                               /* :285-298 */
    for (int k = 0; k < 16; k++)
        if (c.digest[k] != md_byte(b, size, 24 + (uint64_t)k)) {
            code = 4;
            break;
        }
out:
    info->error_code = code;
    info->item_count = items;
    info->cur_offset = cur_offset;
    info->cur_remaining = cur_remaining;
    info->cur_needed = cur_needed;
    return code;
}

typedef struct {
    const uint8_t *data;
    const uint64_t *off;
    const uint32_t *len;
    uint64_t p0, p1;
    orc_md_info *info;
} md_job;

static void *md_worker(void *arg)
{
    md_job *j = (md_job *)arg;
    for (uint64_t p = j->p0; p < j->p1; p++)
        orc_metadata_unpack(j->data + j->off[p], j->len[p], &j->info[p]);
    return NULL;
}

/* orc_metadata_unpack of n packs on n_threads pthreads (the CPU baseline of bench.py --op metadata) */
void orc_metadata_unpack_batch(const uint8_t *data, const uint64_t *off, const uint32_t *len, uint64_t n,
                               orc_md_info *info, int n_threads)
{
    pthread_once(&md5_once, md5_tables);
    if (n_threads < 1) n_threads = 1;
    if (n_threads > 256) n_threads = 256;
    pthread_t th[256];
    md_job jobs[256];
    for (int t = 0; t < n_threads; t++) {
        jobs[t] = (md_job){data, off, len, n * (uint64_t)t / (uint64_t)n_threads,
                           n * (uint64_t)(t + 1) / (uint64_t)n_threads, info};
    }
    if (n_threads == 1) { md_worker(&jobs[0]); return; }
    for (int t = 0; t < n_threads; t++) pthread_create(&th[t], NULL, md_worker, &jobs[t]);
    for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
}

/* =========================================================================================== */
/* Generator                                                                                     */
/* =========================================================================================== */
uint64_t orc_splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void orc_gen_records(uint64_t seed, uint64_t r0, uint64_t n, uint32_t L, uint8_t *out)
{
    for (uint64_t i = 0; i < n; i++) {
        uint64_t r = r0 + i;
        uint64_t base = seed ^ (r * 0x9E3779B97F4A7C15ull);
        uint8_t *o = out + i * L;
        for (uint32_t k = 0; k < L; k += 8) {
            uint64_t v = orc_splitmix64(base ^ (uint64_t)(k >> 3));
            for (uint32_t b = 0; b < 8 && k + b < L; b++)
                o[k + b] = (uint8_t)(v >> (8 * b));
        }
    }
}

/* The constants the restatement uses, for tests/test_ref_tables.py (pinned to the reference's
 * source text through tests/golden/ref_tables.json): MD5 T, message word and rotation per step and
 * the IV; SHA-1 round constant per step and the IV. */
void orc_md5_consts(uint32_t T[64], uint32_t word[64], uint32_t rot[64], uint32_t iv[4])
{
    orc_md5_ctx c;
    orc_md5_init(&c);
    for (int i = 0; i < 64; i++) {
        T[i] = md5_T[i];
        word[i] = (uint32_t)md5_word(i);
        rot[i] = md5_shift[i >> 4][i & 3];
    }
    memcpy(iv, c.buf, 16);
}

void orc_sha1_consts(uint32_t k80[80], uint32_t iv[5])
{
    orc_sha1_ctx c;
    orc_sha1_init(&c);
    for (int i = 0; i < 80; i++)
        k80[i] = sha1_K[i / 20];
    memcpy(iv, c.state, 20);
}
