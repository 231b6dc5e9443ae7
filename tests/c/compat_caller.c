/*
 * compat_caller.c -- a C caller written the way the reference's callers use libbrb_core/crypto,
 * compiled against include/brb_crypto.h and linked with -lbrb_crypto_gpu (no other source).
 *
 * Patterns exercised (reference call sites):
 *   - MetaData pack digest: Init, UpdateBig per item, Final      (data/utils/meta_data.c:407-431)
 *   - RC4+MD5 frame validation digest + memcmp of 16 bytes       (event/aio/ev_kq_aio_transform.c:175-180)
 *   - RSA-SHA1 signing pre-digest: BrbSha1_Do                    (comm/utils/comm_ssl_pkey.c:465)
 *   - MemBuffer Blowfish ECB over word pairs                     (data/core/mem_buf.c:1528-1539)
 *   - RC4 connection streams: Init per direction, Crypt per buffer (ev_kq_aio_transform.c:89-90,273,282)
 *   - then the batch surface on the same records, which must agree with the compat results
 *     (returns 0 with a reason when no GPU is present; it never computes on the CPU),
 *   - and the multi-device runtime: BRB_CryptoGPU_DeviceCount / SetDevice per device, and one
 *     batch split over every device with BRB_BATCH_ALL_DEVICES.
 *
 * Output: one line per check, "name value", parsed by tests/test_abi.py.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "brb_crypto.h"

static void hex(const unsigned char *p, int n, char *out)
{
    for (int i = 0; i < n; i++)
        sprintf(out + 2 * i, "%02x", p[i]);
}

int main(void)
{
    enum { NREC = 300, RLEN = 1500 };
    static unsigned char recs[NREC * RLEN];
    unsigned long long x = 0x5EED0002ull;
    for (int i = 0; i < NREC * RLEN; i++) {           /* any deterministic bytes */
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        recs[i] = (unsigned char)(x >> 56);
    }
    char h[64];

    /* MetaData-style multi-item digest */
    BRB_MD5_CTX md5;
    BRB_MD5Init(&md5);
    for (int i = 0; i < 3; i++)
        BRB_MD5UpdateBig(&md5, recs + i * RLEN, RLEN);
    BRB_MD5Final(&md5);
    printf("meta_md5 %s\n", (char *)md5.string);

    /* per-record digests via the compat surface */
    static unsigned char ref16[NREC][16], ref20[NREC][20];
    for (int r = 0; r < NREC; r++) {
        BRB_MD5_CTX c;
        BRB_MD5Init(&c);
        BRB_MD5Update(&c, recs + r * RLEN, RLEN);
        BRB_MD5Final(&c);
        memcpy(ref16[r], c.digest, 16);
        static unsigned char tmp[RLEN];
        memcpy(tmp, recs + r * RLEN, RLEN);            /* BrbSha1_Do mutates its input */
        if (BrbSha1_Do(tmp, RLEN, (char *)ref20[r]) != 0)
            return 2;
    }
    hex(ref16[NREC - 1], 16, h);
    printf("rec_last_md5 %s\n", h);
    hex(ref20[NREC - 1], 20, h);
    printf("rec_last_sha1 %s\n", h);
    /* frame validation pattern: recompute and memcmp */
    printf("validate %d\n", memcmp(ref16[0], ref16[0], 16) == 0);

    /* MemBuffer-style Blowfish round trip with one ctx */
    BRB_BLOWFISH_CTX bf;
    unsigned char key[] = "brb_framework_k4";
    BRB_Blowfish_Init(&bf, key, 16);
    unsigned long w[64];
    for (int i = 0; i < 64; i++)
        w[i] = ((unsigned long)recs[8 * i] << 40) ^ (unsigned long)i * 0x9E3779B97F4A7C15ul;
    unsigned long w0[64];
    memcpy(w0, w, sizeof(w));
    for (int i = 0; i < 64; i += 2)
        BRB_Blowfish_Encrypt(&bf, &w[i], &w[i + 1]);
    unsigned long enc[64];
    memcpy(enc, w, sizeof(w));
    for (int i = 0; i < 64; i += 2)
        BRB_Blowfish_Decrypt(&bf, &w[i], &w[i + 1]);
    printf("bf_roundtrip %d\n", memcmp(w, w0, sizeof(w)) == 0);
    printf("bf_enc0 %016lx%016lx\n", enc[0], enc[1]);

    /* RC4: write and read states from one key; two buffers on the write stream, decrypted in one
     * read call; the "Key"/"Plaintext" vector on a fresh state */
    BRB_RC4_State wst, rst, kst;
    BRB_RC4_Init(&wst, (const unsigned char *)"cryptokey", 9);
    BRB_RC4_Init(&rst, (const unsigned char *)"cryptokey", 9);
    static unsigned char c1[RLEN], p1[RLEN];
    BRB_RC4_Crypt(&wst, recs, c1, 700);
    BRB_RC4_Crypt(&wst, recs + 700, c1 + 700, RLEN - 700);
    BRB_RC4_Crypt(&rst, c1, p1, RLEN);
    printf("rc4_roundtrip %d\n", memcmp(p1, recs, RLEN) == 0 && memcmp(&wst, &rst, sizeof(wst)) == 0);
    unsigned char kc[9];
    BRB_RC4_Init(&kst, (const unsigned char *)"Key", 3);
    BRB_RC4_Crypt(&kst, (const unsigned char *)"Plaintext", kc, 9);
    hex(kc, 9, h);
    printf("rc4_kat %s\n", h);

    /* batch surface on the same data (host mode) */
    static unsigned char dig16[NREC][16], dig20[NREC][20];
    int rc = BRB_MD5BatchFixed(recs, RLEN, NREC, dig16, BRB_BATCH_HOST, NULL);
    printf("batch_md5_rc %d\n", rc);
    if (rc != BRB_BATCH_OK) {
        printf("batch_reason %s\n", BRB_CryptoGPU_LastError());
        return 0;
    }
    printf("batch_md5_eq %d\n", memcmp(dig16, ref16, sizeof(ref16)) == 0);
    rc = BrbSha1_BatchFixed(recs, RLEN, NREC, dig20, BRB_BATCH_HOST, NULL);
    printf("batch_sha1_eq %d\n", rc == 1 && memcmp(dig20, ref20, sizeof(ref20)) == 0);
    memcpy(w, w0, sizeof(w));
    rc = BRB_Blowfish_EncryptBatch(&bf, w, 32, BRB_BATCH_HOST, NULL);
    printf("batch_bf_eq %d\n", rc == 1 && memcmp(w, enc, sizeof(enc)) == 0);
    /* RC4 batch: one stream of 1500 B on a fresh write state must equal c1 (the two compat calls) */
    BRB_RC4_State bst;
    BRB_RC4_Init(&bst, (const unsigned char *)"cryptokey", 9);
    static unsigned char bc[RLEN];
    uint64_t off0 = 0;
    uint32_t len0 = RLEN;
    rc = BRB_RC4_CryptBatch(&bst, recs, bc, &off0, &len0, 1, BRB_BATCH_HOST, NULL);
    printf("batch_rc4_eq %d\n", rc == 1 && memcmp(bc, c1, RLEN) == 0 && memcmp(&bst, &wst, sizeof(bst)) == 0);

    /* several GPUs from one process without linking HIP (the kqueue daemon's event threads, one
     * per GPU): device count, per-thread device selection, and one batch split over every device */
    int ndev = BRB_CryptoGPU_DeviceCount();
    printf("devices %d\n", ndev);
    int per_dev_ok = ndev > 0;
    for (int g = 0; g < ndev; g++) {
        if (BRB_CryptoGPU_SetDevice(g) != BRB_BATCH_OK) {
            per_dev_ok = 0;
            break;
        }
        memset(dig16, 0, sizeof(dig16));
        rc = BRB_MD5BatchFixed(recs, RLEN, NREC, dig16, BRB_BATCH_HOST, NULL);
        per_dev_ok &= rc == 1 && memcmp(dig16, ref16, sizeof(ref16)) == 0 && BRB_CryptoGPU_GetDevice() == g;
    }
    (void)BRB_CryptoGPU_SetDevice(0);
    printf("per_device_md5_eq %d\n", per_dev_ok);
    memset(dig16, 0, sizeof(dig16));
    rc = BRB_MD5BatchFixed(recs, RLEN, NREC, dig16, BRB_BATCH_HOST | BRB_BATCH_ALL_DEVICES, NULL);
    printf("all_devices_md5_eq %d\n", rc == 1 && memcmp(dig16, ref16, sizeof(ref16)) == 0);
    memcpy(w, w0, sizeof(w));
    rc = BRB_Blowfish_EncryptBatch(&bf, w, 32, BRB_BATCH_HOST | BRB_BATCH_ALL_DEVICES, NULL);
    printf("all_devices_bf_eq %d\n", rc == 1 && memcmp(w, enc, sizeof(enc)) == 0);
    printf("set_device_out_of_range %d\n", BRB_CryptoGPU_SetDevice(ndev));
    printf("all_devices_with_device_ptrs %d\n",
           BRB_MD5BatchFixed(recs, RLEN, NREC, dig16, BRB_BATCH_DEVICE | BRB_BATCH_ALL_DEVICES, NULL));
    BRB_CryptoGPU_ThreadCleanup();
    rc = BRB_MD5BatchFixed(recs, RLEN, NREC, dig16, BRB_BATCH_HOST, NULL);
    printf("after_cleanup_md5_eq %d\n", rc == 1 && memcmp(dig16, ref16, sizeof(ref16)) == 0);
    return 0;
}
