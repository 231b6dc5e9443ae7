/*
 * brb_crypto.h -- C ABI of libbrb_crypto_gpu.so, the MI355X-native replacement for
 * libbrb_core/crypto (BrByte brb_framework @ 2024_10_08).
 *
 * Two surfaces:
 *
 *  1. COMPAT (drop-in): the reference's crypto prototypes with the same names, argument types,
 *     struct layouts and side effects, so the callers in libbrb_core/comm and libbrb_core/data link
 *     unchanged (list in INTEGRATION.md).  They run on the calling CPU thread: a single streaming
 *     context is a serial chain and does not belong on a GPU.
 *
 *  2. BATCH (new): many independent records per call, executed by hand-written gfx950 HIP
 *     kernels.  This is the hot path.  It never falls back to a CPU implementation: if no HIP
 *     device is usable the call returns 0 and BRB_CryptoGPU_LastError() says why.
 *
 * LP64 is assumed, exactly as the reference assumes it (`unsigned long` = 8 bytes inside
 * BRB_BLOWFISH_CTX).
 */
#ifndef BRB_CRYPTO_H
#define BRB_CRYPTO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ============================================================================================ */
/* 1. COMPAT SURFACE                                                                              */
/* ============================================================================================ */
/* A translation unit that already includes the reference's libbrb_data.h (guard LIBBRB_DATA_H_)
 * gets these types and prototypes from there; the definitions below are the same ABI. */
#ifndef LIBBRB_DATA_H_

/* ---- MD5 -- replaces libbrb_core/crypto/md5.c; prototypes libbrb_data.h:862-869 ------------ */
#define MD5_DIGEST_LENGTH 16                      /* libbrb_data.h:852 */

typedef struct _BRB_MD5_CTX {                     /* libbrb_data.h:854-860, sizeof == 168 */
    uint32_t buf[4];
    uint32_t bytes[2];
    uint32_t in[16];
    unsigned char digest[16];
    unsigned char string[64];                     /* lowercase hex + NUL after Final */
} BRB_MD5_CTX;

void BRB_MD5Init(BRB_MD5_CTX *ctx);                                             /* md5.c:38  */
void BRB_MD5UpdateBig(BRB_MD5_CTX *ctx, const void *_buf, unsigned long len);   /* md5.c:49  */
void BRB_MD5Update(BRB_MD5_CTX *ctx, const void *_buf, unsigned long len);      /* md5.c:72  */
/* md5.c:112.  The reference lowercases into a 128-byte stack buffer and overflows it when
 * key_sz > 128; this version lowercases in 128-byte pieces (same digest, no overflow). */
void BRB_MD5UpdateLowerText(BRB_MD5_CTX *md5_context, char *key_ptr, int key_sz);
void BRB_MD5Final(BRB_MD5_CTX *ctx);                                            /* md5.c:134 */
void BRB_MD5Transform(BRB_MD5_CTX *ctx);                                        /* md5.c:170 */
void BRB_MD5LateInitDigestString(BRB_MD5_CTX *ret);                             /* md5.c:255 */
void BRB_MD5ToStr(unsigned char *bin_digest, unsigned char *ret_buf_str);       /* md5.c:264 */

/* ---- SHA-1 -- replaces libbrb_core/crypto/sha1.c; prototypes libbrb_data.h:1947-1951 ------- */
typedef struct {                                  /* libbrb_data.h:1937-1943, sizeof == 92 */
    uint32_t state[5];
    uint32_t count[2];
    uint8_t buffer[64];
} BrbSha1Ctx;

#define BRB_SHA1_DIGEST_SIZE 20                   /* libbrb_data.h:1945 */

void BrbSha1_Init(BrbSha1Ctx *context);                                          /* sha1.c:132 */
/* sha1.c:143.  Like the reference (SHA1HANDSOFF undefined, sha1.c:84-90) every full 64-byte block
 * transformed directly from `data` is overwritten with message-schedule words W[64..79]. */
void BrbSha1_Update(BrbSha1Ctx *context, const uint8_t *data, const size_t len);
void BrbSha1_Final(BrbSha1Ctx *context, uint8_t digest[BRB_SHA1_DIGEST_SIZE]);   /* sha1.c:171 */
void BrbSha1_Transform(uint32_t state[5], const uint8_t buffer[64]);             /* sha1.c:75  */
int BrbSha1_Do(const uint8_t *in_ptr, int in_len, char *dig_str);                /* sha1.c:203 */

/* ---- Blowfish -- replaces libbrb_core/crypto/blowfish.c; prototypes libbrb_data.h:881-883 -- */
typedef struct _BRB_BLOWFISH_CTX {                /* libbrb_data.h:876-879, sizeof == 8336 */
    unsigned long P[16 + 2];
    unsigned long S[4][256];
} BRB_BLOWFISH_CTX;

void BRB_Blowfish_Init(BRB_BLOWFISH_CTX *ctx, unsigned char *key, int keyLen);         /* :382 */
void BRB_Blowfish_Encrypt(BRB_BLOWFISH_CTX *ctx, unsigned long *xl, unsigned long *xr); /* :312 */
void BRB_Blowfish_Decrypt(BRB_BLOWFISH_CTX *ctx, unsigned long *xl, unsigned long *xr); /* :347 */

/* ---- RC4 -- replaces libbrb_core/crypto/rc4.c; prototypes libbrb_data.h:899-900 ------------ */
typedef struct _BRB_RC4_State {                   /* libbrb_data.h:887-897, sizeof == 264 */
    unsigned char perm[256];
    unsigned char index1;
    unsigned char index2;
    struct {
        unsigned int initialized : 1;
    } flags;
} BRB_RC4_State;

void BRB_RC4_Init(BRB_RC4_State *state, const unsigned char *key, int keylen);            /* rc4.c:40 */
void BRB_RC4_Crypt(BRB_RC4_State *state, const unsigned char *inbuf, unsigned char *outbuf,
                   int buflen);                                                          /* rc4.c:64 */
#endif /* LIBBRB_DATA_H_ */

/* ============================================================================================ */
/* 2. BATCH SURFACE (GPU)                                                                         */
/* ============================================================================================ */

/* Return codes follow the reference's transform-hook convention (ev_kq_aio_transform.c:52-57):
 *   1  done
 *   0  not done: no usable HIP device, device error, or unsupported request
 *      (BRB_CryptoGPU_LastError() has the reason; nothing was computed on the CPU)
 *  -1  bad arguments (NULL pointer where one is required, length out of range)         */
#define BRB_BATCH_OK        1
#define BRB_BATCH_NOT_DONE  0
#define BRB_BATCH_BADARG   (-1)
#define BRB_BATCH_DROPPED  (-2)   /* transform batcher: a round was dropped (see Flush)         */
#define BRB_BATCH_PARTIAL  (-3)   /* all-devices transform batcher: some parts delivered their
                                     buffers, others could not select their device and keep their
                                     rounds pending (see Flush)                                  */
#define BRB_BATCH_FAULT    (-4)   /* segment digests, MetaData unpack, RC4 pass, RC4+MD5 frame /
                                     open: a wave-pair kernel's bounded wait on its partner wave
                                     gave up (a protocol fault; never a hang).  The call's outputs,
                                     and for RC4 the states, are wrong.  Returned by synchronous
                                     calls; a device-mode BRB_BATCH_ASYNC call cannot know yet and
                                     returns 1: BRB_CryptoGPU_AsyncFaultCheck() reports it after the
                                     caller has synchronised its stream.  A transform batcher round
                                     with a fault is dropped (Flush returns BRB_BATCH_DROPPED).
                                     Test option pair_stall injects one.                         */

/* flags */
#define BRB_BATCH_HOST      0x0u   /* pointers are host memory: copied in and out by the call      */
#define BRB_BATCH_DEVICE    0x1u   /* every pointer (data, offsets, lengths, digests, ctx, words)
                                      is device memory (HBM-resident); nothing crosses PCIe       */
#define BRB_BATCH_ASYNC     0x2u   /* with BRB_BATCH_DEVICE: enqueue on `hip_stream` and return
                                      without waiting; the caller synchronises the stream and then
                                      calls BRB_CryptoGPU_AsyncFaultCheck() (same thread) before it
                                      trusts the outputs of wave-pair calls (BRB_BATCH_FAULT)     */
#define BRB_BATCH_ALL_DEVICES 0x4u /* host mode only (every batch call except MemBuffer):
                                      split the records (blocks, streams, packs) into contiguous
                                      ranges [g*n/G, (g+1)*n/G), one per visible device g < G, run
                                      them concurrently and return when all are done (SURVEY §8(e):
                                      no collective); the RC4 states go with their streams.  Calls
                                      that write a byte span back (RC4, frames, base64 outputs)
                                      split only when the ranges' spans do not interleave across
                                      parts (ranges in submission order); otherwise they run on the
                                      calling thread's device.  With BRB_BATCH_DEVICE: -1.           */

/* Device mode: `hip_stream` is a hipStream_t (NULL = the legacy default stream of the current
 * device) and the work runs on the caller's current HIP device (BRB_CryptoGPU_SetDevice,
 * hipSetDevice or torch.cuda.set_device).
 * DEVICE-MODE CONTRACT: the library cannot see how large a device allocation is, so in device mode
 * every offset, length and count is the caller's promise that the range lies inside its allocation
 * (data, offsets/lengths arrays, digests, outputs, states).  A range past the end is not detected
 * and not answered with -1: the kernel's access faults and the HIP context is lost ("illegal memory
 * access", every later call on that device fails).  Host mode copies exactly the ranges given, so
 * there a bad range is an ordinary out-of-bounds read of the caller's host memory.  Host mode: the call runs on the caller's current device
 * (or on every device with BRB_BATCH_ALL_DEVICES), copies straight from and to the caller's memory
 * (pageable or page-locked) in chunks so that copies in both directions overlap the kernels, and
 * returns when the results are in host memory; `hip_stream` is not used. */

/* MD5 of n_rec records of rec_len bytes each, stored back to back: record i is
 * data[i*rec_len .. (i+1)*rec_len).  digests[i] = BRB_MD5Init/Update/Final of record i. */
int BRB_MD5BatchFixed(const void *data, uint32_t rec_len, uint64_t n_rec,
                      unsigned char (*digests)[16], unsigned flags, void *hip_stream);

/* MD5 of n_rec records of arbitrary byte offset and length (record i = data[offsets[i] ..
 * offsets[i] + lengths[i])).  Records may overlap and need no alignment. */
int BRB_MD5Batch(const void *data, const uint64_t *offsets, const uint32_t *lengths,
                 uint64_t n_rec, unsigned char (*digests)[16], unsigned flags, void *hip_stream);

/* MD5 of segment lists: record i is the concatenation of segments
 * rec_first_seg[i] .. rec_first_seg[i + 1] - 1 (rec_first_seg has n_rec + 1 entries), segment k =
 * data[seg_offsets[k] .. + seg_lengths[k]).  digests[i] = BRB_MD5Init, BRB_MD5UpdateBig per segment,
 * BRB_MD5Final -- the MetaData pack digest of meta_data.c:397-433 with one record per MetaData. */
int BRB_MD5BatchSegments(const void *data, const uint64_t *seg_offsets, const uint32_t *seg_lengths,
                         const uint64_t *rec_first_seg, uint64_t n_rec, unsigned char (*digests)[16],
                         unsigned flags, void *hip_stream);

/* MetaData packs (the format of meta_data.c:104-140, libbrb_data.h:291-330, LP64):
 * a 64-byte header {int version; int item_count; unsigned long size; "BRB_META"; 16-byte MD5 of
 * the items' data; 24 reserved bytes}, then per item {unsigned long item_id, item_sub_id, sz;
 * sz data bytes; 0x1F}.  BRB_MetaDataUnpackBatch checks pack i = data[offsets[i] .. + lengths[i])
 * exactly as MetaDataUnpack (meta_data.c:145-328) checks a MemBuffer holding it at offset 0, and
 * writes the MetaDataUnpackerInfo fields (libbrb_data.h:332-344) plus the number of items unpacked:
 * error_code is a BRB_METADATA_UNPACK_* value (the reference's MetaDataUnpackReturnCode), SUCCESS
 * only if every canary holds and the MD5 of the items read equals the header's digest.  Quirks kept:
 * an item is only read with sizeof(MetaDataItem) = 32 bytes left (24 are its header), so a pack whose
 * last item holds 0..6 data bytes reports NEED_MORE_DATA_METAITEM; the walk stops after item_count
 * items or at the pack's end, whichever comes first.  Where the reference reads past its buffer
 * (packs shorter than the header, a size field beyond the pack), bytes past the pack read as 0 and
 * an item larger than the whole pack reports NEED_MORE_DATA_OBJECT without being read. */
#define BRB_METADATA_UNPACK_FAILED_INVALID_HEADER_MAGIC 0
#define BRB_METADATA_UNPACK_FAILED_CORRUPTED_CANARY 3
#define BRB_METADATA_UNPACK_FAILED_DIGEST_INVALID 4
#define BRB_METADATA_UNPACK_FAILED_NEED_MORE_DATA_METAITEM 5
#define BRB_METADATA_UNPACK_FAILED_NEED_MORE_DATA_OBJECT 6
#define BRB_METADATA_UNPACK_SUCCESS 7
#define BRB_METADATA_HEADER_SIZE 64
#define BRB_METADATA_ITEM_RAW_SIZE 24
typedef struct BRB_MetaDataUnpackInfo {
    int32_t error_code;       /* MetaDataUnpackReturnCode */
    uint32_t item_count;      /* items whose canary was checked before error_code was decided */
    uint64_t cur_offset;      /* MetaDataUnpackerInfo.cur_offset / cur_remaining / cur_needed */
    uint64_t cur_remaining;
    uint64_t cur_needed;
} BRB_MetaDataUnpackInfo;
int BRB_MetaDataUnpackBatch(const void *data, const uint64_t *offsets, const uint32_t *lengths, uint64_t n_packs,
                            BRB_MetaDataUnpackInfo *info, unsigned flags, void *hip_stream);

/* SHA-1 batches: digests[i] = BrbSha1_Do(record i) (20 raw big-endian bytes).  Unlike
 * BrbSha1_Update the batch surface never writes into the input records. */
int BrbSha1_BatchFixed(const void *data, uint32_t rec_len, uint64_t n_rec,
                       uint8_t (*digests)[20], unsigned flags, void *hip_stream);
int BrbSha1_Batch(const void *data, const uint64_t *offsets, const uint32_t *lengths,
                  uint64_t n_rec, uint8_t (*digests)[20], unsigned flags, void *hip_stream);

/* Blowfish ECB over n_blocks blocks in place.  A block is the reference's (xl, xr) pair of
 * 64-bit `unsigned long` words (blowfish.c:312, mem_buf.c:1538-1539): words[2i] = xl,
 * words[2i+1] = xr.  The result equals BRB_Blowfish_Encrypt/Decrypt(ctx, &w[2i], &w[2i+1])
 * for every i, bit for bit in all 64 bits.  With BRB_BATCH_DEVICE, ctx is a device copy of the
 * 8336-byte BRB_BLOWFISH_CTX. */
int BRB_Blowfish_EncryptBatch(const BRB_BLOWFISH_CTX *ctx, unsigned long *words, uint64_t n_blocks,
                              unsigned flags, void *hip_stream);
int BRB_Blowfish_DecryptBatch(const BRB_BLOWFISH_CTX *ctx, unsigned long *words, uint64_t n_blocks,
                              unsigned flags, void *hip_stream);

/* ---- RC4 and the RC4+MD5 frame of the comm transform -------------------------
 * One stream per connection; states[i] is that connection's BRB_RC4_State (an array of n
 * contiguous 264-byte states) and advances exactly as the scalar calls would.  Streams of one
 * call must belong to different connections (a connection's buffers are sequential). */

/* out[offsets[i] .. + lengths[i]) = BRB_RC4_Crypt(&states[i], in + offsets[i], ..., lengths[i]).
 * out may equal in (in place); otherwise the ranges of in and out must not overlap. */
int BRB_RC4_CryptBatch(BRB_RC4_State *states, const void *in, void *out, const uint64_t *offsets,
                       const uint32_t *lengths, uint64_t n_streams, unsigned flags, void *hip_stream);

/* Bytes before the payload in a frame: salt (8) "HASH:" (5) MD5 (16) NUL (1). */
#define BRB_RC4MD5_HEADER 30

/* WRITE side of EvAIOReqTransform_CryptoRaw(COMM_CRYPTO_FUNC_RC4_MD5) (ev_kq_aio_transform.c:
 * 212-230, 281-283) for n connections: with payload i = payload[offsets[i] .. + lengths[i]),
 *   frames[frame_offsets[i] .. + 30 + lengths[i]) =
 *       RC4(states[i], salts[i] as 8 LE bytes | "HASH:" | MD5(payload i) | NUL | payload i).
 * salts[i] is the caller's arc4random() value (the reference's `unsigned long random_salt`).
 * The frames must not overlap each other or the payloads. */
int BRB_RC4MD5_FrameBatch(BRB_RC4_State *states, const void *payload, const uint64_t *offsets,
                          const uint32_t *lengths, const uint64_t *salts, void *frames,
                          const uint64_t *frame_offsets, uint64_t n, unsigned flags, void *hip_stream);

/* READ side (ev_kq_aio_transform.c:270-279) followed by EvAIOReqTransform_RC4_MD5_DataValidate
 * (:158-184): frame i = frames[offsets[i] .. + lengths[i]) is RC4-decrypted with states[i] into
 * out at the same offset (out may equal frames), and valid[i] = 1 if bytes 8..12 are "HASH:" and
 * bytes 13..28 are the MD5 of bytes 30.., else 0.  A frame shorter than 30 bytes is decrypted and
 * reported invalid (the reference would digest past the end of the buffer). */
int BRB_RC4MD5_OpenBatch(BRB_RC4_State *states, const void *frames, void *out, const uint64_t *offsets,
                         const uint32_t *lengths, uint64_t n, uint8_t *valid, unsigned flags,
                         void *hip_stream);

/* ---- Receive-loop batching ------------------------------------------------------
 * The comm layer calls the transform hook once per buffer on the thread that owns the connection
 * (EvAIOReqTransform_ReadData / _WriteData, ev_kq_aio_transform.c:42-70, from comm_tcp_server.c:1749,
 * 1773, comm_tcp_client_read.c:176, 203, comm_tcp_server_conn.c:932).  A transform batcher takes the
 * buffers of one event-loop round from many connections and runs them as one GPU call per
 * direction.  It owns the read and write RC4 states of up to max_conns connections in HBM
 * (CommEvCryptoInfo, libbrb_ev_comm.h:206-236).  Usage per round: Read/Write for every buffer,
 * then Flush, which delivers every result through the callback in submission order.
 * A connection's buffers stay in order: two buffers of one connection and direction in one round
 * run as consecutive sub-rounds.
 *   READ  (RC4_MD5): out = the decrypted frame, valid = EvAIOReqTransform_RC4_MD5_DataValidate;
 *         the payload starts at out + BRB_RC4MD5_HEADER (the reference's MemBufferOffsetSet(30)).
 *   WRITE (RC4_MD5): out = the 30 + len byte frame, salt = the caller's arc4random() value.
 *   RC4: out = the RC4 stream of the buffer in either direction, valid = 1. */
#define BRB_CRYPTO_FUNC_RC4       1       /* COMM_CRYPTO_FUNC_RC4, libbrb_ev_comm.h:166 */
#define BRB_CRYPTO_FUNC_RC4_MD5   2       /* COMM_CRYPTO_FUNC_RC4_MD5, :167 */
#define BRB_CRYPTO_OP_READ        0       /* CRYPTO_OPERATION_READ, libbrb_ev_aio.h:101 */
#define BRB_CRYPTO_OP_WRITE       1       /* CRYPTO_OPERATION_WRITE, :102 */
/* OR into `algo` at Create: zero-copy rounds.  Read/Write keep a reference to `data` instead of
 * copying it: the bytes must lie in page-locked memory (BRB_CryptoGPU_HostRegister, or allocated
 * page-locked by HIP) and stay unchanged until Flush returns.  The kernels read the buffers over
 * PCIe and write the results into the batcher's page-locked output arena: no staging memcpy on the
 * CPU, no bulk H2D/D2H copies.  Read/Write return -1 for a buffer outside page-locked memory. */
#define BRB_BATCHER_ZERO_COPY     0x100
/* OR into `algo` at Create: pipelined rounds.  The batcher owns two rounds' arenas, so the loop fills
 * round k+1 while the GPU runs round k (BRB_TransformBatcherFlushAsync).  Twice the arena memory. */
#define BRB_BATCHER_PIPELINED     0x200
/* OR into `algo` at Create: all devices (the daemon's multi-threaded engine spreading connections,
 * ev_kq_base.c:95).  Connection c lives on device c % G (G = visible devices) with its read and
 * write states; Read/Write/Enable/GetState route by connection, and one Flush / FlushAsync enqueues
 * every device's round before it waits for any, so the devices run concurrently.  Callbacks come on
 * the calling thread, device by device: each connection's buffers keep their order, buffers of
 * connections on different devices are not interleaved in submission order.  With one device (or
 * max_conns < G) this is a plain batcher. */
#define BRB_BATCHER_ALL_DEVICES   0x400
typedef struct BRB_TransformBatcher BRB_TransformBatcher;
typedef void (*BRB_TransformDone)(void *user, uint32_t conn, int op, const void *out, uint32_t out_len, int valid);
/* `valid` of a buffer whose round was dropped (out = NULL, out_len = 0): see Flush. */
#define BRB_TRANSFORM_DROPPED (-1)
/* NULL on failure (reason in BRB_CryptoGPU_LastError).  A round holds at most max_round_bytes of
 * input and 4 * max_conns buffers; Read/Write return 0 when it is full (Flush, then submit again). */
BRB_TransformBatcher *BRB_TransformBatcherCreate(uint32_t max_conns, uint64_t max_round_bytes, int algo);
void BRB_TransformBatcherDestroy(BRB_TransformBatcher *b);
/* EvAIOReqTransform_CryptoEnable (ev_kq_aio_transform.c:71-105): both states of `conn` = BRB_RC4_Init(key). */
int BRB_TransformBatcherEnable(BRB_TransformBatcher *b, uint32_t conn, const void *key, int key_sz);
/* Read/Write may run concurrently on several threads (the reference's mt_engine, ev_kq_base.c:95)
 * as long as each connection is submitted from one thread; results come back in each connection's
 * order.  Flush/FlushAsync/Enable must not overlap them.  A thread reserves slots and arena bytes in
 * chunks, so a round shared by T threads may report full up to T chunks (64 buffers, 128 KiB) early. */
int BRB_TransformBatcherRead(BRB_TransformBatcher *b, uint32_t conn, const void *data, uint32_t len);
int BRB_TransformBatcherWrite(BRB_TransformBatcher *b, uint32_t conn, const void *data, uint32_t len, uint64_t salt);
/* Runs the round; returns the number of buffers delivered, or -1 for bad arguments.  All-devices
 * batcher: a part that cannot select its device (hipSetDevice fails) keeps its round pending and
 * delivers nothing, while the other parts deliver as usual; the call then returns
 * BRB_BATCH_PARTIAL (-3) if some buffers were delivered, 0 if none, with the parts and the
 * delivered count in LastError -- Flush again once the device is back.  A round that
 * fails on the device is dropped and never re-run (kernels launched before the failure may have
 * advanced their connections' states; running them again would advance them twice): each of its
 * buffers still gets its callback, in order, with valid = BRB_TRANSFORM_DROPPED, out = NULL and
 * out_len = 0, and the call returns BRB_BATCH_DROPPED (-2) with the reason in LastError -- also when
 * another round was delivered in the same call, whose buffers came back through their callbacks as
 * usual (and BRB_BATCH_PARTIAL when, besides, a part's round stays pending).  A round in which a
 * wave-pair kernel reports a protocol fault (BRB_BATCH_FAULT above) is dropped the same way, so no
 * output, frame or valid flag computed over wrong bytes is ever delivered.  The connections of a round
 * dropped on the device (a completion error or a wave-pair fault) are out of step with their peers, as
 * after a lost buffer in the reference, and stay poisoned until Enable re-keys them: their buffers
 * already launched behind the dropped round (pipelined FlushAsync) and those still waiting in the
 * filling round come back BRB_TRANSFORM_DROPPED (the call returns BRB_BATCH_DROPPED), and Read/Write
 * refuse them (BRB_BATCH_BADARG) until then.  A round whose kernel launch failed on the host is
 * dropped without poisoning (only the groups launched before the failure ran, once each).  On a
 * pipelined batcher Flush first delivers the round
 * FlushAsync left running, so Flush drains everything.  A batcher's calls run on the device it was
 * created on and leave the calling thread's current device unchanged. */
int64_t BRB_TransformBatcherFlush(BRB_TransformBatcher *b, BRB_TransformDone done, void *user);
/* Pipelined rounds: enqueues the current round and returns without waiting for it, after delivering
 * the previous round (if one is running) in submission order; Read/Write then fill the other arena.
 * Returns the number of buffers delivered (those of the previous round), or -1 / 0 as Flush.  A
 * connection's streams stay in order across rounds (one HIP stream).  In zero-copy mode a buffer
 * must stay unchanged until its round is delivered.  Without BRB_BATCHER_PIPELINED this is Flush. */
int64_t BRB_TransformBatcherFlushAsync(BRB_TransformBatcher *b, BRB_TransformDone done, void *user);
/* Copies a connection's current state (op = READ or WRITE) back to the host (tests, migration). */
int BRB_TransformBatcherGetState(BRB_TransformBatcher *b, uint32_t conn, int op, BRB_RC4_State *out);
/* Test support, not for production use: from now on the `launch`-th kernel launch (0-based) of every
 * round reports a failure without running, so a test can watch a round being dropped; -1 turns it
 * off.  Returns 1, or -1 for a NULL batcher.  (Replaces round 2's BRB_TEST_BATCHER_FAULT variable:
 * the library reads no environment variable.) */
int BRB_TransformBatcherInjectFault(BRB_TransformBatcher *b, int launch);

/* ---- base64 -----------------------------------------------------------------------
 * Encode = brb_base64_encode_to_mb (base64.c:304-361) for n records: record i = data[offsets[i] ..
 * + lengths[i]) -> out[out_offsets[i] .. + 4 * ceil(lengths[i] / 3)), standard alphabet, '='
 * padding, no NUL written.  (brb_base64_encode_bin's static 131 070-byte result buffer cap is a
 * property of that buffer, not of the encoding, and is not reproduced.) */
int BRB_Base64EncodeBatch(const void *data, const uint64_t *offsets, const uint32_t *lengths, uint64_t n,
                          void *out, const uint64_t *out_offsets, unsigned flags, void *hip_stream);
/* Decode = brb_base64_decode_to_mb (base64.c:131-179) for n records: record i = text[offsets[i] ..
 * + lengths[i]) read as a C string (a NUL ends it); bytes outside the alphabet are skipped, '='
 * counts as the value 0 (base64.c:374), every 4 counted characters give 3 bytes, a trailing
 * partial group is dropped.  out_lengths[i] = bytes written at out + out_offsets[i]; the caller
 * reserves 3 * (lengths[i] / 4) bytes there. */
int BRB_Base64DecodeBatch(const void *text, const uint64_t *offsets, const uint32_t *lengths, uint64_t n,
                          void *out, const uint64_t *out_offsets, uint32_t *out_lengths, unsigned flags,
                          void *hip_stream);

/* ---- MemBuffer Blowfish -------------------------------------------------------
 * MemBufferEncryptData / MemBufferDecryptData (mem_buf.c:1499-1617) on the bytes of a MemBuffer:
 * buf = MemBufferDeref(mb) with mb->offset == 0, size = MemBufferGetSize(mb).  Reproduced exactly:
 *   key[i] = (i + seed) * seed + 13 i, seed = key[i] * seed            (mem_buf.c:1511-1515)
 *   encrypt: Blowfish keyLen 4 (sizeof(enc_key[16])), pairs of 64-bit words from buf + offset,
 *            (size + offset) / 8 + 2 words rounded up to pairs; new size = 8 * words + offset
 *   decrypt: keyLen 64 (sizeof(enc_key)), (size - offset) / 8 + 2 words, stops at the first pair
 *            holding a zero word; new size = 8 * words decrypted + offset
 * (so decrypt(encrypt(x)) does not restore x, as in the reference).  The caller grows the buffer
 * first, as MemBufferCheckForGrow does (mem_buf.c:1525, 1585): buf must hold
 * offset + BRB_MEMBUF_SPAN(size + offset) bytes to encrypt, offset + BRB_MEMBUF_SPAN(size - offset)
 * bytes to decrypt.  The Blowfish context is built on the host; the
 * ECB pass (and the zero-pair scan) run on the GPU.  Device mode needs buf + offset 8-byte
 * aligned.  Both calls return when *new_size is known (ASYNC is ignored). */
#define BRB_MEMBUF_SPAN(data_size) ((((data_size) / 8 + 3) / 2) * 16)
void BRB_MemBufferKey(unsigned int seed, unsigned int key[16]);
int BRB_MemBufferEncrypt(void *buf, unsigned long size, unsigned int seed, unsigned long offset,
                         unsigned long *new_size, unsigned flags, void *hip_stream);
int BRB_MemBufferDecrypt(void *buf, unsigned long size, unsigned int seed, unsigned long offset,
                         unsigned long *new_size, unsigned flags, void *hip_stream);

/* ---- runtime ---------------------------------------------------------------------------- */
/* 1 if a HIP device is usable from this process, else 0 (reason in LastError). */
int BRB_CryptoGPU_Available(void);
/* Number of visible HIP devices (probed once per process); 0 if none (reason in LastError). */
int BRB_CryptoGPU_DeviceCount(void);
/* Makes `dev` the calling thread's current device for the batch calls, so a C caller that does not
 * link HIP itself can drive several GPUs (e.g. one event thread per GPU): 1 = done, 0 = no device /
 * HIP error, -1 = dev out of range. */
int BRB_CryptoGPU_SetDevice(int dev);
/* The calling thread's current device, or -1 (reason in LastError). */
int BRB_CryptoGPU_GetDevice(void);
/* Frees the calling thread's host-mode scratch (device workspaces, streams, events) now instead of
 * at thread exit.  Call it with no batch call of this thread running.  If the thread made
 * device-mode BRB_BATCH_ASYNC calls of wave-pair kernels, their devices are synchronised first
 * (hipDeviceSynchronize), since those kernels may still write the thread's fault word. */
void BRB_CryptoGPU_ThreadCleanup(void);
/* Last error of the calling thread ("" if none). */
const char *BRB_CryptoGPU_LastError(void);
/* Wave-pair faults of the calling thread's device-mode BRB_BATCH_ASYNC calls: 1 if none of the
 * wave-pair kernels they enqueued since the last check reported a protocol fault, BRB_BATCH_FAULT
 * (-4) if one did (reason in LastError; the report is cleared).  Call it after synchronising the
 * streams those calls used: a kernel still running has not reported yet. */
int BRB_CryptoGPU_AsyncFaultCheck(void);
/* Page-lock [p, p + len) for the GPU (hipHostRegister, mapped) so that zero-copy batchers can read
 * it: 1 = done, 0 = no device / HIP error (LastError), -1 = bad arguments.  Unregister takes the
 * same `p`. */
int BRB_CryptoGPU_HostRegister(void *p, uint64_t len);
int BRB_CryptoGPU_HostUnregister(void *p);
/* Test support, not for production use: process-wide A/B switches of the kernel selection, the only
 * way to change them (the library reads no environment variable).  "rc4_sector" -1/0/1 (launcher's
 * choice / force the per-stream sink / force the whole-sector sink of the RC4 pass), "var_line" 1/0
 * (variable-length digests on the line kernel / on the per-lane kernel), "fixed_var_line" 1/0
 * (unaligned fixed-stride records on the line kernel / record-relative kernel), "var_sort" 1/0
 * (variable-length batches bucketed by length / in caller order; 2 keeps the first round of groups in
 * caller order), "devices" 0/k (all-devices calls and batchers on every visible device / forced into k <= 16
 * parts, part g on device g % count; an all-devices batcher takes at most 16 parts either way), "b64_group" -1/0..6 (base64 lanes per record: launcher's choice /
 * forced to 2^value), "host_chunk_mib" / "host_digest_chunk_mib" 0/k (host-mode chunks of the default
 * 16 / 32 MiB, or k MiB; chunk-size sweeps), "seg_line" 2/1/0 (segment digests and MetaData unpack on the
 * line-staged producer / consumer wave pairs, the line-staged single waves, the per-lane kernels), "b64_kernel" 2/3/1/0 (64-byte fixed-stride records on
 * the register-buffered kernel at 8 / 4 waves per SIMD, the two-slot kernel, the generic one),
 * "line_slots" 0/2/3 (LDS-DMA ring slots of the line-staged segment and MetaData kernels: each
 * kernel's default, or forced), "rc4md5_pair" 1/0 (BRB_RC4MD5_FrameBatch / OpenBatch on keystream +
 * partner wave pairs / one wave per connection), "rc4_pair" 1/0 (BRB_RC4_CryptBatch likewise; a forced
 * "rc4_sector" value selects the one-wave kernel), "pair_stall" 0/1 (1: the segment, MetaData, RC4
 * pass and RC4+MD5 frame / open wave pairs get a protocol fault injected, so the call returns
 * BRB_BATCH_FAULT, an async call's check reports it and a batcher round is dropped).  Returns 1 and the previous
 * value in *old (if not NULL), or -1 for an unknown name or a value out of range. */
int BRB_CryptoGPU_TestOption(const char *name, int value, int *old);
/* Library version string. */
const char *BRB_CryptoGPU_Version(void);

#ifdef __cplusplus
}
#endif
#endif /* BRB_CRYPTO_H */
