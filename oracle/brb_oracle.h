/*
 * brb_oracle.h -- CPU ORACLE for the libbrb_core/crypto hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * This is a plain-C restatement of the reference's algorithms, written from reading
 *   libbrb_core/crypto/md5.c       (BRB_MD5*,           reference @ 2024_10_08)
 *   libbrb_core/crypto/sha1.c      (BrbSha1_*)
 *   libbrb_core/crypto/blowfish.c  (BRB_Blowfish_*, 64-bit `unsigned long` words)
 *   libbrb_core/data/core/mem_buf.c:1499-1617 (MemBuffer Blowfish wrappers)
 * Each function cites the reference file:line it follows.
 *
 * Who may use it: tests/ (as the checker), __graft_entry__.smoke() (as the checker) and the
 * `cpu_baseline` leg of bench.py.  The product library (brb_framework_amd/libbrb_crypto_gpu.so)
 * never links, loads or calls this code.
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   * The reference build is UNBUILDABLE here: every crypto unit includes libbrb_data.h, which needs
 *     <bsd/string.h>/<bsd/stdlib.h> (libbsd-dev, absent), and stand-in headers are not allowed.
 *   * MD5 / SHA-1: pinned by RFC 1321 A.5 and FIPS 180-1 known answers plus Python hashlib
 *     (OpenSSL), which the survey verified equal to the reference on 20 edge lengths.
 *   * Blowfish: the low 32 bits of every word are pinned by the published Blowfish known answers
 *     (Kocher "TESTKEY", Eric Young ECB set) and by OpenSSL BF_encrypt over random keys.
 *     The HIGH 32 bits (the reference's 64-bit carries) are pinned only by this restatement:
 *     "parity unpinned" for the high halves.
 */
#ifndef BRB_ORACLE_H
#define BRB_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- MD5 (md5.c) -------------------------------------------------------------------------- */
typedef struct {                 /* same field order as BRB_MD5_CTX, libbrb_data.h:854-860 */
    uint32_t buf[4];
    uint32_t bytes[2];
    uint32_t in[16];
    unsigned char digest[16];
    unsigned char string[64];
} orc_md5_ctx;

void orc_md5_init(orc_md5_ctx *c);
void orc_md5_update(orc_md5_ctx *c, const void *p, unsigned long len);
void orc_md5_update_big(orc_md5_ctx *c, const void *p, unsigned long len);
void orc_md5_final(orc_md5_ctx *c);
void orc_md5(const void *p, uint64_t len, uint8_t out[16]);

/* ---- SHA-1 (sha1.c) ----------------------------------------------------------------------- */
typedef struct {                 /* same field order as BrbSha1Ctx, libbrb_data.h:1937-1943 */
    uint32_t state[5];
    uint32_t count[2];
    uint8_t buffer[64];
} orc_sha1_ctx;

void orc_sha1_init(orc_sha1_ctx *c);
/* Streaming update with the reference's in-place mutation of `data` (sha1.c:84-90,157-158). */
void orc_sha1_update(orc_sha1_ctx *c, uint8_t *data, size_t len);
void orc_sha1_final(orc_sha1_ctx *c, uint8_t out[20]);
/* One-shot digest WITHOUT touching the input (batch semantics: digest of a private copy). */
void orc_sha1(const void *p, uint64_t len, uint8_t out[20]);

/* ---- Blowfish (blowfish.c), 64-bit words ------------------------------------------------- */
typedef struct {                 /* same layout as BRB_BLOWFISH_CTX, libbrb_data.h:876-879 */
    uint64_t P[18];
    uint64_t S[4][256];
} orc_bf_ctx;

/* pi-derived tables by BBP digit extraction (independent of tools/gen_pi_tables.py) */
void orc_bf_pi_words(uint32_t out[1042]);
void orc_md5_consts(uint32_t T[64], uint32_t word[64], uint32_t rot[64], uint32_t iv[4]);
void orc_sha1_consts(uint32_t k80[80], uint32_t iv[5]);
void orc_bf_init(orc_bf_ctx *c, const unsigned char *key, int key_len);
void orc_bf_encrypt(const orc_bf_ctx *c, uint64_t *xl, uint64_t *xr);
void orc_bf_decrypt(const orc_bf_ctx *c, uint64_t *xl, uint64_t *xr);
/* ECB over n_blocks (xl, xr) pairs in place; decrypt != 0 selects decryption. */
void orc_bf_ecb(const orc_bf_ctx *c, uint64_t *words, uint64_t n_blocks, int decrypt, int n_threads);

/* MemBuffer semantics (mem_buf.c:1499-1617): key derivation and the size/loop rules.
 * `buf` must have room for ((size + offset)/8 + 3) * 8 bytes, zero-filled past `size`.
 * Returns the new MemBuffer size the reference would store. */
void orc_membuf_key(unsigned int seed, unsigned int key_out[16]);
uint64_t orc_membuf_encrypt(uint8_t *buf, uint64_t size, unsigned int seed, uint64_t offset);
uint64_t orc_membuf_decrypt(uint8_t *buf, uint64_t size, unsigned int seed, uint64_t offset);

/* ---- RC4 -- libbrb_core/crypto/rc4.c ------------------------------------------------------
 * State layout = BRB_RC4_State (libbrb_data.h:887-897): perm[256], index1, index2, flags. */
typedef struct {
    unsigned char perm[256];
    unsigned char index1;
    unsigned char index2;
    struct { unsigned int initialized : 1; } flags;
} orc_rc4_state;

void orc_rc4_init(orc_rc4_state *s, const unsigned char *key, int keylen);            /* rc4.c:40-62 */
void orc_rc4_crypt(orc_rc4_state *s, const unsigned char *in, unsigned char *out, int n); /* rc4.c:64-87 */

/* ---- RC4+MD5 framing -- EvAIOReqTransform_CryptoRaw, ev_kq_aio_transform.c:189-288 --------
 * WRITE (:212-230, :281-283): frame = salt (8 B, LP64 unsigned long) | "HASH:" | MD5(payload) |
 *   NUL | payload, then RC4 with the write state.  `frame` receives 30 + len bytes.
 * READ (:232-236, :270-279): RC4 with the read state over the whole received buffer, in place.
 * VALIDATE (EvAIOReqTransform_RC4_MD5_DataValidate, :158-184): "HASH:" at 8 and MD5 of bytes
 *   [30, size) equal to bytes [13, 29).  Frames shorter than 30 B are reported invalid (the
 *   reference would read past the frame and digest ~2^64 bytes: undefined). */
#define ORC_RC4MD5_HDR 30
void orc_rc4md5_frame(orc_rc4_state *s, const uint8_t *payload, uint64_t len, uint64_t salt, uint8_t *frame);
int orc_rc4md5_open(orc_rc4_state *s, uint8_t *frame, uint64_t frame_len);
/* n connections (pthreads over contiguous connection ranges; bench.py's cpu_baseline) */
void orc_rc4_crypt_batch(orc_rc4_state *s, uint8_t *data, const uint64_t *off, const uint32_t *len, uint64_t n,
                         int n_threads);
void orc_rc4md5_frame_batch(orc_rc4_state *s, const uint8_t *payload, const uint64_t *off, const uint32_t *len,
                            const uint64_t *salts, uint8_t *frames, const uint64_t *foff, uint64_t n, int n_threads);
void orc_rc4md5_open_batch(orc_rc4_state *s, uint8_t *frames, const uint64_t *off, const uint32_t *len, uint64_t n,
                           uint8_t *valid, int n_threads);

/* ---- base64 -- libbrb_core/crypto/base64.c --------------------------------------------------
 * encode = brb_base64_encode_to_mb (base64.c:304-361): standard alphabet, '=' padding, no cap.
 * decode = brb_base64_decode_to_mb (:131-179): stops at NUL or after len bytes, skips bytes outside
 *   the alphabet, '=' counts as value 0 (:363-376), each 4 counted characters give 3 bytes, a
 *   trailing partial group is dropped.  Both return the output length. */
uint64_t orc_b64_encode(const uint8_t *in, uint64_t len, char *out);
uint64_t orc_b64_decode(const char *in, uint64_t len, uint8_t *out);

/* ---- Batches (used by tests and by bench.py's cpu_baseline) ------------------------------- */
void orc_md5_batch_fixed(const uint8_t *data, uint32_t rec_len, uint64_t n, uint8_t *out16, int n_threads);
void orc_sha1_batch_fixed(const uint8_t *data, uint32_t rec_len, uint64_t n, uint8_t *out20, int n_threads);
void orc_md5_batch(const uint8_t *data, const uint64_t *off, const uint32_t *len, uint64_t n, uint8_t *out16);
void orc_sha1_batch(const uint8_t *data, const uint64_t *off, const uint32_t *len, uint64_t n, uint8_t *out20);
void orc_md5_batch_mt(const uint8_t *data, const uint64_t *off, const uint32_t *len, uint64_t n, uint8_t *out16,
                      int n_threads);
void orc_sha1_batch_mt(const uint8_t *data, const uint64_t *off, const uint32_t *len, uint64_t n, uint8_t *out20,
                       int n_threads);

/* ---- Deterministic input generator --------------------------------------
 * byte(r, k) = byte (k mod 8), little-endian, of splitmix64(seed ^ (r * 0x9E3779B97F4A7C15) ^ (k >> 3))
 * splitmix64(x): z = x + 0x9E3779B97F4A7C15; z = (z ^ z>>30) * 0xBF58476D1CE4E5B9;
 *                z = (z ^ z>>27) * 0x94D049BB133111EB; return z ^ z>>31.                      */
uint64_t orc_splitmix64(uint64_t x);
void orc_gen_records(uint64_t seed, uint64_t r0, uint64_t n, uint32_t rec_len, uint8_t *out);

/* MetaData packs (meta_data.c:104-140, 145-328, 397-433) */
typedef struct {
    int32_t error_code;
    uint32_t item_count;
    uint64_t cur_offset, cur_remaining, cur_needed;
} orc_md_info;
uint64_t orc_metadata_pack(const uint8_t *data, const uint64_t *off, const uint64_t *len, const uint64_t *id,
                           const uint64_t *sub, uint64_t n_items, uint8_t *out);
int orc_metadata_unpack(const uint8_t *b, uint64_t size, orc_md_info *info);
void orc_metadata_unpack_batch(const uint8_t *data, const uint64_t *off, const uint32_t *len, uint64_t n,
                               orc_md_info *info, int n_threads);

#ifdef __cplusplus
}
#endif
#endif
