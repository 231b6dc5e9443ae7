/*
 * batcher_bench.c -- host-inclusive benchmark of the receive-loop transform batcher
 * as a C event loop would drive it: per round, every connection receives one RC4+MD5 frame written
 * by its peer and sends one payload; each buffer is one BRB_TransformBatcherRead/Write call, then
 * one Flush delivers the results.  The peer side is built with the library's own compat surface
 * (BRB_RC4_Crypt + BRB_MD5*), for every round before the timed region.  Prints one JSON object;
 * payload_gib_s is over the whole timed window (R rounds of submit + flush, drained at both ends).
 *
 * Build: gcc -O2 -pthread -I include tools/batcher_bench.c -L brb_framework_amd -lbrb_crypto_gpu \
 *            -Wl,-rpath,$PWD/brb_framework_amd -o tools/batcher_bench
 * Run:   tools/batcher_bench [connections=16384] [bytes=1500] [rounds=20] [warmup=3] [zero_copy=0] [pipelined=0] [submit_threads=1]
 *
 * zero_copy=1: the batcher is created with BRB_BATCHER_ZERO_COPY and the frame / payload buffers
 * (the loop's socket buffers) are page-locked once with BRB_CryptoGPU_HostRegister.
 * pipelined=1: BRB_BATCHER_PIPELINED, each round started with FlushAsync: the loop submits round
 * k+1 while the GPU runs round k (every round has its own frames, so a running round's buffers stay
 * unchanged, as zero-copy requires).
 * submit_threads=T: T threads (the reference's mt_engine) submit disjoint connection ranges into the
 * same round at once; the main thread is thread 0 and flushes after all T have finished.
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "brb_crypto.h"

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

typedef struct {
    unsigned long long delivered, valid, bytes;
} Tally;

static void on_done(void *user, uint32_t conn, int op, const void *out, uint32_t out_len, int valid)
{
    Tally *t = (Tally *)user;
    (void)conn;
    (void)op;
    (void)out;
    t->delivered++;
    t->valid += valid != 0;
    t->bytes += out_len;
}

/* submit threads: thread t submits connections [t*C/T, (t+1)*C/T) of the current round */
typedef struct {
    BRB_TransformBatcher *b;
    const unsigned char *frames, *payload;
    uint32_t C, L, F, T;
    int rounds;                 /* rounds the workers take part in */
    pthread_barrier_t start, end;
    int failed;
} Submit;

static void submit_range(Submit *S, uint32_t t)
{
    const uint32_t c0 = (uint32_t)((uint64_t)S->C * t / S->T), c1 = (uint32_t)((uint64_t)S->C * (t + 1) / S->T);
    for (uint32_t c = c0; c < c1; c++)
        if (BRB_TransformBatcherRead(S->b, c, S->frames + (size_t)c * S->F, S->F) != BRB_BATCH_OK ||
            BRB_TransformBatcherWrite(S->b, c, S->payload + (size_t)c * S->L, S->L, c) != BRB_BATCH_OK)
            __atomic_store_n(&S->failed, 1, __ATOMIC_RELAXED);
}

typedef struct {
    Submit *S;
    uint32_t t;
} Worker;

static void *worker(void *arg)
{
    Worker *w = (Worker *)arg;
    for (int r = 0; r < w->S->rounds; r++) {
        pthread_barrier_wait(&w->S->start);
        submit_range(w->S, w->t);
        pthread_barrier_wait(&w->S->end);
    }
    return NULL;
}

static int cmp_d(const void *a, const void *b)
{
    double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

int main(int argc, char **argv)
{
    const uint32_t C = argc > 1 ? (uint32_t)atoi(argv[1]) : 16384;
    const uint32_t L = argc > 2 ? (uint32_t)atoi(argv[2]) : 1500;
    const int R = argc > 3 ? atoi(argv[3]) : 20, W = argc > 4 ? atoi(argv[4]) : 3;
    const int zc = argc > 5 ? atoi(argv[5]) : 0;
    const int pipelined = argc > 6 ? atoi(argv[6]) : 0;
    const uint32_t T = argc > 7 && atoi(argv[7]) > 0 ? (uint32_t)atoi(argv[7]) : 1;
    const int algo = argc > 8 && atoi(argv[8]) == 1 ? BRB_CRYPTO_FUNC_RC4 : BRB_CRYPTO_FUNC_RC4_MD5;
    /* every round's frames are built before timing (each depends on the peer's RC4 state) */
    const int NR = W + R;
    const uint32_t F = L + BRB_RC4MD5_HEADER;
    const size_t pl_sz = ((size_t)C * L + 4095) & ~(size_t)4095, fr_sz = ((size_t)C * F + 4095) & ~(size_t)4095;
    unsigned char *payload = aligned_alloc(4096, pl_sz), *frames = aligned_alloc(4096, fr_sz);
    BRB_RC4_State *peer = malloc(sizeof(BRB_RC4_State) * C);
    unsigned char key[16];
    unsigned long long x = 0x5EED00F2ull;
    for (size_t i = 0; i < (size_t)C * L; i++) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        payload[i] = (unsigned char)(x >> 56);
    }
    if (zc && (BRB_CryptoGPU_HostRegister(payload, pl_sz) != BRB_BATCH_OK ||
               BRB_CryptoGPU_HostRegister(frames, fr_sz) != BRB_BATCH_OK)) {
        printf("{\"error\": \"%s\"}\n", BRB_CryptoGPU_LastError());
        return 1;
    }
    BRB_TransformBatcher *b = BRB_TransformBatcherCreate(C, (uint64_t)C * (L + F) * 102 / 100 + (uint64_t)T * (256 << 10) + 4096,
                                                         algo | (zc ? BRB_BATCHER_ZERO_COPY : 0) |
                                                             (pipelined ? BRB_BATCHER_PIPELINED : 0));
    if (!b) {
        printf("{\"error\": \"%s\"}\n", BRB_CryptoGPU_LastError());
        return 1;
    }
    for (uint32_t c = 0; c < C; c++) {
        for (int k = 0; k < 16; k++)
            key[k] = (unsigned char)(c * 131 + k * 7);
        memset(&peer[c], 0, sizeof(peer[c]));
        BRB_RC4_Init(&peer[c], key, 16);
        if (BRB_TransformBatcherEnable(b, c, key, 16) != BRB_BATCH_OK) {
            printf("{\"error\": \"%s\"}\n", BRB_CryptoGPU_LastError());
            return 1;
        }
    }
    /* the peers' frames for every round, built before timing (ev_kq_aio_transform.c:212-230 +
     * :281-283): a pipelined round keeps its buffers until the next round delivers it */
    unsigned char *frames_all = frames;
    {
        frames_all = aligned_alloc(4096, fr_sz * NR);
        if (!frames_all || (zc && BRB_CryptoGPU_HostRegister(frames_all, fr_sz * NR) != BRB_BATCH_OK)) {
            printf("{\"error\": \"frame arena: %s\"}\n", BRB_CryptoGPU_LastError());
            return 1;
        }
    }
    for (int r = 0; r < W + R; r++)
        for (uint32_t c = 0; c < C; c++) {
            unsigned char *f = frames_all + (size_t)r * fr_sz + (size_t)c * F;
            BRB_MD5_CTX m;
            BRB_MD5Init(&m);
            BRB_MD5Update(&m, payload + (size_t)c * L, L);
            BRB_MD5Final(&m);
            unsigned long salt = (unsigned long)(r * 1000003u + c);
            memcpy(f, &salt, 8);
            memcpy(f + 8, "HASH:", 5);
            memcpy(f + 13, m.digest, 16);
            f[29] = 0;
            memcpy(f + 30, payload + (size_t)c * L, L);
            BRB_RC4_Crypt(&peer[c], f, f, (int)F);
        }
    double *t = malloc(sizeof(double) * R), *ts = malloc(sizeof(double) * R);
    Tally tally = {0, 0, 0};
    double t_start = 0;
    Submit S;
    memset(&S, 0, sizeof(S));
    S.b = b;
    S.payload = payload;
    S.C = C;
    S.L = L;
    S.F = F;
    S.T = T;
    S.rounds = W + R;
    pthread_barrier_init(&S.start, NULL, T);
    pthread_barrier_init(&S.end, NULL, T);
    pthread_t *th = malloc(sizeof(pthread_t) * T);
    Worker *wk = malloc(sizeof(Worker) * T);
    for (uint32_t i = 1; i < T; i++) {
        wk[i].S = &S;
        wk[i].t = i;
        pthread_create(&th[i], NULL, worker, &wk[i]);
    }
    for (int r = 0; r < W + R; r++) {
        if (r == W) {   /* drain the warm-up rounds, then time R rounds of submit + flush */
            if (BRB_TransformBatcherFlush(b, on_done, &tally) < 0) {
                printf("{\"error\": \"drain: %s\"}\n", BRB_CryptoGPU_LastError());
                return 1;
            }
            t_start = now();
        }
        const unsigned char *fr = frames_all + (size_t)r * fr_sz;
        const double t0 = now();
        S.frames = fr;
        if (T > 1)
            pthread_barrier_wait(&S.start);
        submit_range(&S, 0);
        if (T > 1)
            pthread_barrier_wait(&S.end);
        const double t1 = now();
        if (S.failed) {
            printf("{\"error\": \"round %d: submit failed: %s\"}\n", r, BRB_CryptoGPU_LastError());
            return 1;
        }
        const int64_t n = pipelined ? BRB_TransformBatcherFlushAsync(b, on_done, &tally)
                                    : BRB_TransformBatcherFlush(b, on_done, &tally);
        if (r >= W) {
            ts[r - W] = t1 - t0;
            t[r - W] = now() - t0;
        }
        if (n < 0 || n != (pipelined && (r == 0 || r == W) ? 0 : 2 * (int64_t)C)) {
            printf("{\"error\": \"round %d: %lld delivered: %s\"}\n", r, (long long)n, BRB_CryptoGPU_LastError());
            return 1;
        }
    }
    if (BRB_TransformBatcherFlush(b, on_done, &tally) < 0) {
        printf("{\"error\": \"final flush: %s\"}\n", BRB_CryptoGPU_LastError());
        return 1;
    }
    const double total = now() - t_start, mean = total / R;
    if (tally.delivered != 2ull * C * (W + R) || tally.valid != tally.delivered) {
        printf("{\"error\": \"%llu delivered, %llu valid, expected %llu\"}\n", tally.delivered, tally.valid,
               2ull * C * (W + R));
        return 1;
    }
    qsort(t, R, sizeof(double), cmp_d);
    qsort(ts, R, sizeof(double), cmp_d);
    for (uint32_t i = 1; i < T; i++)
        pthread_join(th[i], NULL);
    printf("{\"zero_copy\": %d, \"pipelined\": %d, \"submit_threads\": %u, \"connections\": %u, \"bytes\": %u, \"rounds\": %d, "
           "\"round_ms_mean\": %.3f, \"round_ms_median\": %.3f, \"round_ms_min\": %.3f, "
           "\"submit_ms_median\": %.3f, \"payload_gib_s\": %.3f, \"buffers_per_s\": %.0f, \"valid\": %llu, \"delivered\": %llu}\n",
           zc, pipelined, T, C, L, R, mean * 1e3, t[R / 2] * 1e3, t[0] * 1e3, ts[R / 2] * 1e3,
           2.0 * C * L / mean / (1 << 30), 2.0 * C / mean, tally.valid, tally.delivered);
    BRB_TransformBatcherDestroy(b);
    if (zc) {
        BRB_CryptoGPU_HostUnregister(payload);
        BRB_CryptoGPU_HostUnregister(frames);
        if (frames_all != frames)
            BRB_CryptoGPU_HostUnregister(frames_all);
    }
    return 0;
}
