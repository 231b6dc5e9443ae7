// call_latency.cpp -- per-call cost of BRB_MD5BatchFixed for the small batches a kqueue round hands
// over, called through the C ABI as a C caller would (no Python).
// For n = 1 .. 65 536 records of 1500 B: host mode from pageable memory, host mode from page-locked
// memory (BRB_CryptoGPU_HostRegister), device mode synchronous, device mode asynchronous (K calls
// back to back, one sync).  Median of R timed calls after W warm-up calls; the first call of the
// process (workspace and stream creation) is reported separately.  One JSON object per line.
// Build: hipcc -O2 -std=c++17 -I include tools/call_latency.cpp -L brb_framework_amd -lbrb_crypto_gpu \
//          -Wl,-rpath,$PWD/brb_framework_amd -o tools/call_latency
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "brb_crypto.h"

static double now_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double median(std::vector<double> v)
{
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main()
{
    const uint32_t L = 1500;
    const uint64_t NMAX = 65536;
    std::vector<uint8_t> host(NMAX * L);
    for (size_t i = 0; i < host.size(); i++)
        host[i] = uint8_t(i * 2654435761u >> 11);
    std::vector<uint8_t> out(NMAX * 16);
    uint8_t *pinned = static_cast<uint8_t *>(aligned_alloc(4096, NMAX * L));
    memcpy(pinned, host.data(), NMAX * L);
    uint8_t *pout = static_cast<uint8_t *>(aligned_alloc(4096, 1 << 20));
    uint8_t *dbuf = nullptr, *dout = nullptr;
    hipStream_t s;
    if (hipMalloc(&dbuf, NMAX * L) != hipSuccess || hipMalloc(&dout, NMAX * 16) != hipSuccess ||
        hipMemcpy(dbuf, host.data(), NMAX * L, hipMemcpyHostToDevice) != hipSuccess || hipStreamCreate(&s) != hipSuccess) {
        printf("{\"error\": \"hip setup\"}\n");
        return 1;
    }
    auto digests = [](uint8_t *p) { return reinterpret_cast<unsigned char (*)[16]>(p); };
    {   // first call of the process: per-thread workspace and streams are created here
        const double t0 = now_us();
        const int rc = BRB_MD5BatchFixed(host.data(), L, 64, digests(out.data()), BRB_BATCH_HOST, nullptr);
        printf("{\"what\": \"first host-mode call (64 records)\", \"us\": %.1f, \"rc\": %d}\n", now_us() - t0, rc);
    }
    if (BRB_CryptoGPU_HostRegister(pinned, NMAX * L) != BRB_BATCH_OK || BRB_CryptoGPU_HostRegister(pout, 1 << 20) != BRB_BATCH_OK) {
        printf("{\"error\": \"%s\"}\n", BRB_CryptoGPU_LastError());
        return 1;
    }
    for (uint64_t n : {1ull, 4ull, 16ull, 64ull, 256ull, 1024ull, 4096ull, 16384ull, 65536ull}) {
        const int W = 20, R = n <= 4096 ? 200 : 50;
        struct Mode {
            const char *name;
            int (*call)(uint64_t, void *);
        };
        std::vector<double> t;
        auto time_it = [&](auto &&fn) {
            for (int i = 0; i < W; i++)
                fn();
            t.clear();
            for (int i = 0; i < R; i++) {
                const double t0 = now_us();
                fn();
                t.push_back(now_us() - t0);
            }
            return median(t);
        };
        int bad = 0;
        const double hp = time_it([&] {
            bad |= BRB_MD5BatchFixed(host.data(), L, n, digests(out.data()), BRB_BATCH_HOST, nullptr) != BRB_BATCH_OK;
        });
        const double hl = time_it([&] {
            bad |= BRB_MD5BatchFixed(pinned, L, n, digests(pout), BRB_BATCH_HOST, nullptr) != BRB_BATCH_OK;
        });
        const double ds = time_it([&] {
            bad |= BRB_MD5BatchFixed(dbuf, L, n, digests(dout), BRB_BATCH_DEVICE, s) != BRB_BATCH_OK;
        });
        // asynchronous: K calls back to back on one stream, then one synchronize
        const int K = 100;
        for (int i = 0; i < W; i++)
            bad |= BRB_MD5BatchFixed(dbuf, L, n, digests(dout), BRB_BATCH_DEVICE | BRB_BATCH_ASYNC, s) != BRB_BATCH_OK;
        (void)hipStreamSynchronize(s);
        const double t0 = now_us();
        for (int i = 0; i < K; i++)
            bad |= BRB_MD5BatchFixed(dbuf, L, n, digests(dout), BRB_BATCH_DEVICE | BRB_BATCH_ASYNC, s) != BRB_BATCH_OK;
        const double enq = (now_us() - t0) / K;
        (void)hipStreamSynchronize(s);
        const double da = (now_us() - t0) / K;
        printf("{\"records\": %llu, \"bytes\": %llu, \"host_pageable_us\": %.1f, \"host_pagelocked_us\": %.1f, "
               "\"device_sync_us\": %.1f, \"device_async_us_per_call\": %.2f, \"async_enqueue_us_per_call\": %.2f, "
               "\"host_pageable_GBs\": %.2f, \"ok\": %s}\n",
               (unsigned long long)n, (unsigned long long)(n * L), hp, hl, ds, da, enq, n * L / hp / 1e3, bad ? "false" : "true");
        fflush(stdout);
    }
    BRB_CryptoGPU_HostUnregister(pinned);
    BRB_CryptoGPU_HostUnregister(pout);
    return 0;
}
