// host_pipe.hip -- chunked, overlapped host-mode execution and the all-devices split (host_pipe.h).
//
// Measured on the MI355X box (tools/mb/host_copy.cpp): a pageable hipMemcpy already
// runs at the PCIe rate (56.5 GB/s H2D vs 57.3 GB/s from page-locked memory), page-locking a fresh
// buffer costs as long as copying it (≈ 17 ms per GiB), and H2D and D2H together reach ≈ 48.5 GB/s
// each way, but an H2D or D2H from pageable memory holds the calling thread until it is done.  So a
// host-mode call copies straight from and to the caller's memory in chunks: the calling thread
// issues the H2D copies (chunk k+1 travels while the kernel runs on chunk k), and for outputs as
// large as the inputs (Blowfish in place) a per-device worker thread issues the D2H copies, so both
// PCIe directions run at once.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "api_util.h"
#include "brb_kernels.h"
#include "host_pipe.h"
#include "test_options.h"

namespace {

using brb_api::DeviceGuard;
using brb_api::fail_hip;
using brb_api::set_err;

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Input bytes per chunk.  Every pageable chunk copy pays a fixed cost (8 MiB pieces copy at
// 52 GB/s, one 98 MB copy at 56.5 GB/s), while only the first chunk's H2D and the last chunk's D2H
// go un-overlapped.  Blowfish returns as many bytes as it sends, so its ends are whole chunks:
// 16 MiB.  Digest batches return 16-20 B per record, so their chunks can be larger: 32 MiB.
// Test options "host_chunk_mib" / "host_digest_chunk_mib" (0 = these defaults) change them for
// sweeps (tools/host_sweep.py); the library reads no environment variable.
size_t chunk_bytes()
{
    const int mib = brb_opt::get(brb_opt::kHostChunkMiB);
    return (mib > 0 ? size_t(mib) : size_t(16)) << 20;
}
size_t digest_chunk_bytes()
{
    const int mib = brb_opt::get(brb_opt::kHostDigestChunkMiB);
    return (mib > 0 ? size_t(mib) : size_t(32)) << 20;
}

// Posts "wait for `ev` on `s_out`, then copy [src, src + bytes) to host `dst`" to the device's D2H
// worker: a D2H copy into pageable memory holds its thread until done, and on the worker it runs
// while the calling thread goes on issuing H2D copies, so both PCIe directions are busy.
class Pending;
void post_d2h(int dev, Pending &pending, hipStream_t s_out, hipEvent_t ev, void *dst, const void *src, size_t bytes);

// ---- persistent worker threads -------------------------------------------------------------------
// One per (part or device, role): role 0 runs part g of an all-devices split on device g % count,
// role 1 issues a device's D2H copies.  They live for the whole process (never joined: nothing may
// wait on a GPU runtime that is being torn down at exit).
class Worker {
public:
    explicit Worker(int dev) : dev_(dev) { std::thread([this] { run(); }).detach(); }
    void post(std::function<void()> f)
    {
        {
            std::lock_guard<std::mutex> lk(mu_);
            q_.push_back(std::move(f));
        }
        cv_.notify_one();
    }

private:
    void run()
    {
        (void)hipSetDevice(dev_);
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [this] { return !q_.empty(); });
                f = std::move(q_.front());
                q_.pop_front();
            }
            f();
        }
    }
    int dev_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
};

// `idx`: the part (role 0) or the device (role 1); the thread runs on device `dev`.
Worker &worker(int idx, int role, int dev)
{
    static std::mutex mu;
    static auto *pool = new std::vector<Worker *>;   // intentionally never destroyed
    std::lock_guard<std::mutex> lk(mu);
    const size_t i = size_t(idx) * 2 + size_t(role);
    if (pool->size() <= i)
        pool->resize(i + 1, nullptr);
    if (!(*pool)[i])
        (*pool)[i] = new Worker(dev);
    return *(*pool)[i];
}

// Counts posted jobs up and finished jobs down; wait() returns once every posted job has finished.
class Pending {
public:
    void add()
    {
        std::lock_guard<std::mutex> lk(mu_);
        ++n_;
    }
    void done(int rc, const std::string &err)
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (rc != BRB_BATCH_OK && rc_ == BRB_BATCH_OK) {
            rc_ = rc;
            err_ = err;
        }
        if (--n_ == 0)
            cv_.notify_all();
    }
    bool failed()
    {
        std::lock_guard<std::mutex> lk(mu_);
        return rc_ != BRB_BATCH_OK;
    }
    int wait(std::string *err)
    {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return n_ == 0; });
        *err = err_;
        return rc_;
    }

private:
    std::mutex mu_;
    std::condition_variable cv_;
    uint64_t n_ = 0;
    int rc_ = BRB_BATCH_OK;
    std::string err_;
};

void post_d2h(int dev, Pending &pending, hipStream_t s_out, hipEvent_t ev, void *dst, const void *src, size_t bytes)
{
    pending.add();
    worker(dev, 1, dev).post([=, &pending] {
        hipError_t x;
        int r = BRB_BATCH_OK;
        std::string why;
        if ((x = hipStreamWaitEvent(s_out, ev, 0)) != hipSuccess ||
            (x = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s_out)) != hipSuccess) {
            r = fail_hip("hipMemcpyAsync D2H", x);
            why = brb_api::t_err;
        }
        pending.done(r, why);
    });
}

// ---- per-thread, per-device streams and events ---------------------------------------------------
constexpr int kEvents = 64;   // reused round-robin; a wait on a later record of the same event only
                              // waits longer (later chunks follow on the same stream)
struct Pipe {
    hipStream_t s_in = nullptr, s_k = nullptr, s_out = nullptr;
    hipEvent_t ev_in[kEvents] = {}, ev_k[kEvents] = {};
};
struct Pipes {
    std::vector<Pipe *> by_dev;
    ~Pipes() { release(); }
    void release()
    {
        for (size_t d = 0; d < by_dev.size(); d++)
            if (Pipe *p = by_dev[d]) {
                DeviceGuard g{int(d)};
                for (hipStream_t q : {p->s_in, p->s_k, p->s_out})
                    if (q) {
                        (void)hipStreamSynchronize(q);
                        (void)hipStreamDestroy(q);
                    }
                for (int i = 0; i < kEvents; i++) {
                    if (p->ev_in[i])
                        (void)hipEventDestroy(p->ev_in[i]);
                    if (p->ev_k[i])
                        (void)hipEventDestroy(p->ev_k[i]);
                }
                delete p;
                by_dev[d] = nullptr;
            }
    }
};
thread_local Pipes t_pipes;

Pipe *pipe_for(int dev, hipError_t *e)
{
    if (t_pipes.by_dev.size() <= size_t(dev))
        t_pipes.by_dev.resize(dev + 1, nullptr);
    if (Pipe *p = t_pipes.by_dev[dev])
        return p;
    auto *p = new Pipe;
    *e = hipSuccess;
    for (hipStream_t *q : {&p->s_in, &p->s_k, &p->s_out})
        if (*e == hipSuccess)
            *e = hipStreamCreateWithFlags(q, hipStreamNonBlocking);
    for (int i = 0; i < kEvents && *e == hipSuccess; i++)
        if ((*e = hipEventCreateWithFlags(&p->ev_in[i], hipEventDisableTiming)) == hipSuccess)
            *e = hipEventCreateWithFlags(&p->ev_k[i], hipEventDisableTiming);
    t_pipes.by_dev[dev] = p;   // released at thread exit even if creation failed halfway
    return *e == hipSuccess ? p : nullptr;
}

// Drains the pipe's streams (every exit of a pipeline does this, so no copy is still in flight
// into the per-thread workspace when the next call reuses or regrows it).  rc in, rc out.
int drain(Pipe *p, int rc)
{
    for (hipStream_t q : {p->s_in, p->s_k, p->s_out}) {
        const hipError_t e = hipStreamSynchronize(q);
        if (e != hipSuccess && rc == BRB_BATCH_OK)
            rc = fail_hip("hipStreamSynchronize", e);
    }
    return rc;
}

// One device's share of a fixed-stride digest batch: H2D chunk by chunk on s_in (calling thread),
// one kernel per chunk on s_k once its bytes have landed, and each chunk's digests back through the
// device's D2H worker while later chunks are still going up (cfg3's 64-byte records return a
// quarter of their bytes as digests).
int digest_part(brb_host::FixedLauncher launch, size_t dig, const uint8_t *data, uint32_t L, uint64_t n,
                uint8_t *digests)
{
    hipError_t e;
    int dev = 0;
    if ((e = hipGetDevice(&dev)) != hipSuccess)
        return fail_hip("hipGetDevice", e);
    Pipe *p = pipe_for(dev, &e);
    if (!p)
        return fail_hip("host pipeline streams", e);
    const size_t in_bytes = size_t(L) * n, off_out = align_up(in_bytes, 256);
    uint8_t *ws = static_cast<uint8_t *>(brb_api::workspace(off_out + dig * n, &e));
    if (!ws)
        return fail_hip("device workspace", e);
    const uint64_t per = L ? std::max<uint64_t>(1, digest_chunk_bytes() / L) : n;
    if (per >= n) {
        // one chunk: nothing to overlap, so no worker hand-off and no events -- H2D, kernel and D2H
        // in order on one stream (tools/call_latency.cpp: the pipeline's machinery cost ~48 us per
        // call on batches of 1..1024 records)
        if (L && (e = hipMemcpyAsync(ws, data, n * L, hipMemcpyHostToDevice, p->s_k)) != hipSuccess)
            return drain(p, fail_hip("hipMemcpyAsync H2D", e));
        if ((e = launch(ws, L, n, ws + off_out, p->s_k)) != hipSuccess)
            return drain(p, fail_hip("kernel launch", e));
        if ((e = hipMemcpyAsync(digests, ws + off_out, dig * n, hipMemcpyDeviceToHost, p->s_k)) != hipSuccess)
            return drain(p, fail_hip("hipMemcpyAsync D2H", e));
        if ((e = hipStreamSynchronize(p->s_k)) != hipSuccess)
            return drain(p, fail_hip("hipStreamSynchronize", e));
        return BRB_BATCH_OK;
    }
    Pending pending;
    int rc = BRB_BATCH_OK;
    uint64_t c = 0;
    for (uint64_t i = 0; i < n && rc == BRB_BATCH_OK && !pending.failed(); i += per, c++) {
        const uint64_t m = std::min(per, n - i);
        hipEvent_t ev_in = p->ev_in[c % kEvents], ev_k = p->ev_k[c % kEvents];
        if (L && (e = hipMemcpyAsync(ws + i * L, data + i * L, m * L, hipMemcpyHostToDevice, p->s_in)) != hipSuccess)
            rc = fail_hip("hipMemcpyAsync H2D", e);
        else if ((e = hipEventRecord(ev_in, p->s_in)) != hipSuccess || (e = hipStreamWaitEvent(p->s_k, ev_in, 0)) != hipSuccess)
            rc = fail_hip("chunk event", e);
        else if ((e = launch(ws + i * L, L, m, ws + off_out + i * dig, p->s_k)) != hipSuccess)
            rc = fail_hip("kernel launch", e);
        else if ((e = hipEventRecord(ev_k, p->s_k)) != hipSuccess)
            rc = fail_hip("chunk event", e);
        else
            post_d2h(dev, pending, p->s_out, ev_k, digests + i * dig, ws + off_out + i * dig, dig * m);
    }
    std::string why;
    const int rc_out = pending.wait(&why);
    if (rc == BRB_BATCH_OK && rc_out != BRB_BATCH_OK) {
        brb_api::t_err = why;
        rc = rc_out;
    }
    return drain(p, rc);
}

// One device's share of a Blowfish batch: the words go up chunk by chunk on s_in (calling thread),
// each chunk is enciphered on s_k, and the device's D2H worker brings it back on s_out while later
// chunks are still going up.
int blowfish_part(const BRB_BLOWFISH_CTX *ctx, uint64_t *words, uint64_t nb, bool decrypt)
{
    hipError_t e;
    int dev = 0;
    if ((e = hipGetDevice(&dev)) != hipSuccess)
        return fail_hip("hipGetDevice", e);
    Pipe *p = pipe_for(dev, &e);
    if (!p)
        return fail_hip("host pipeline streams", e);
    const size_t ctx_bytes = align_up(sizeof(BRB_BLOWFISH_CTX), 256);
    uint8_t *ws = static_cast<uint8_t *>(brb_api::workspace(ctx_bytes + 16 * size_t(nb), &e));
    if (!ws)
        return fail_hip("device workspace", e);
    const uint64_t *dctx = reinterpret_cast<const uint64_t *>(ws);
    uint64_t *dw = reinterpret_cast<uint64_t *>(ws + ctx_bytes);
    const uint64_t per = std::max<uint64_t>(1, chunk_bytes() / 16);
    if (per >= nb) {                                           // one chunk: one stream, one sync
        if ((e = hipMemcpyAsync(ws, ctx, sizeof(BRB_BLOWFISH_CTX), hipMemcpyHostToDevice, p->s_k)) != hipSuccess ||
            (e = hipMemcpyAsync(dw, words, 16 * nb, hipMemcpyHostToDevice, p->s_k)) != hipSuccess ||
            (e = brb::launch_blowfish(dctx, dw, nb, decrypt, p->s_k)) != hipSuccess ||
            (e = hipMemcpyAsync(words, dw, 16 * nb, hipMemcpyDeviceToHost, p->s_k)) != hipSuccess ||
            (e = hipStreamSynchronize(p->s_k)) != hipSuccess)
            return drain(p, fail_hip("single-chunk Blowfish batch", e));
        return BRB_BATCH_OK;
    }
    if ((e = hipMemcpyAsync(ws, ctx, sizeof(BRB_BLOWFISH_CTX), hipMemcpyHostToDevice, p->s_in)) != hipSuccess)
        return drain(p, fail_hip("hipMemcpyAsync H2D", e));
    Pending pending;
    int rc = BRB_BATCH_OK;
    uint64_t c = 0;
    for (uint64_t i = 0; i < nb && rc == BRB_BATCH_OK && !pending.failed(); i += per, c++) {
        const uint64_t m = std::min(per, nb - i);
        hipEvent_t ev_in = p->ev_in[c % kEvents], ev_k = p->ev_k[c % kEvents];
        if ((e = hipMemcpyAsync(dw + 2 * i, words + 2 * i, 16 * m, hipMemcpyHostToDevice, p->s_in)) != hipSuccess)
            rc = fail_hip("hipMemcpyAsync H2D", e);
        else if ((e = hipEventRecord(ev_in, p->s_in)) != hipSuccess || (e = hipStreamWaitEvent(p->s_k, ev_in, 0)) != hipSuccess)
            rc = fail_hip("chunk event", e);
        else if ((e = brb::launch_blowfish(dctx, dw + 2 * i, m, decrypt, p->s_k)) != hipSuccess)
            rc = fail_hip("kernel launch", e);
        else if ((e = hipEventRecord(ev_k, p->s_k)) != hipSuccess)
            rc = fail_hip("chunk event", e);
        else
            post_d2h(dev, pending, p->s_out, ev_k, words + 2 * i, dw + 2 * i, 16 * m);
    }
    std::string why;
    const int rc_out = pending.wait(&why);
    if (rc == BRB_BATCH_OK && rc_out != BRB_BATCH_OK) {
        brb_api::t_err = why;
        rc = rc_out;
    }
    return drain(p, rc);
}

}  // namespace

namespace brb_host {

void release_thread_pipes()
{
    t_pipes.release();
}

int split_parts()
{
    const int forced = brb_opt::get(brb_opt::kDevices);
    return forced > 0 ? forced : brb_api::device_count();
}

int part_device(int g)
{
    const int n = brb_api::device_count();
    return n > 0 ? g % n : 0;
}

int split_devices(uint64_t n, const std::function<int(int, uint64_t, uint64_t)> &part)
{
    const int G = split_parts();
    if (G <= 1 || n < uint64_t(G)) {
        DeviceGuard g(0);
        if (g.error() != hipSuccess)
            return fail_hip("hipSetDevice", g.error());
        return part(0, 0, n);
    }
    struct Result {
        int rc = BRB_BATCH_OK;
        std::string err;
    };
    std::vector<Result> res(G);
    Pending pending;
    for (int g = 0; g < G; g++) {
        const uint64_t lo = n * uint64_t(g) / uint64_t(G), hi = n * uint64_t(g + 1) / uint64_t(G);
        pending.add();
        const int dev = part_device(g);
        worker(g, 0, dev).post([&, g, dev, lo, hi] {
            brb_api::clear_err();
            DeviceGuard dg{dev};                       // the worker selected dev at start; a failure there shows here
            res[g].rc = dg.error() != hipSuccess ? fail_hip("hipSetDevice", dg.error()) : part(dev, lo, hi);
            if (res[g].rc != BRB_BATCH_OK)
                res[g].err = brb_api::t_err;
            pending.done(BRB_BATCH_OK, std::string());
        });
    }
    std::string unused;
    pending.wait(&unused);
    for (int g = 0; g < G; g++)
        if (res[g].rc != BRB_BATCH_OK) {
            set_err("device %d: %s", g, res[g].err.c_str());
            return res[g].rc;
        }
    return BRB_BATCH_OK;
}

int digest_fixed(FixedLauncher launch, size_t dig, const uint8_t *data, uint32_t L, uint64_t n, uint8_t *digests,
                 unsigned flags, hipStream_t)
{
    if (flags & BRB_BATCH_ALL_DEVICES)
        return split_devices(n, [&](int, uint64_t lo, uint64_t hi) {
            return digest_part(launch, dig, data + lo * L, L, hi - lo, digests + lo * dig);
        });
    return digest_part(launch, dig, data, L, n, digests);
}

int blowfish(const BRB_BLOWFISH_CTX *ctx, uint64_t *words, uint64_t nb, bool decrypt, unsigned flags, hipStream_t)
{
    if (flags & BRB_BATCH_ALL_DEVICES)
        return split_devices(nb, [&](int, uint64_t lo, uint64_t hi) {
            return blowfish_part(ctx, words + 2 * lo, hi - lo, decrypt);
        });
    return blowfish_part(ctx, words, nb, decrypt);
}

}  // namespace brb_host
