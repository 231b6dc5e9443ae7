// batch_api.hip -- the exported C ABI of the batch (GPU) surface; see include/brb_crypto.h.
//
// Host mode (BRB_BATCH_HOST): inputs are copied into a per-thread device workspace, the kernel
// runs, results are copied back, and the call returns after the stream has drained.
// Device mode (BRB_BATCH_DEVICE): the caller's HBM-resident buffers are used in place.
// There is no CPU fallback anywhere in this file: a missing or failing device returns
// BRB_BATCH_NOT_DONE with the reason in BRB_CryptoGPU_LastError().
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <mutex>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "brb_crypto.h"
#include "api_util.h"
#include "brb_kernels.h"
#include "host_pipe.h"
#include "test_options.h"

namespace brb_api {

thread_local std::string t_err;

void clear_err()
{
    t_err.clear();
}

void set_err(const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    t_err = buf;
}

int fail_hip(const char *what, hipError_t e)
{
    set_err("%s: %s (%d)", what, hipGetErrorString(e), int(e));
    return BRB_BATCH_NOT_DONE;
}

// The device count is cached once a probe has found a device: a batch call from the event loop
// should not pay a runtime query per call, and the set of visible devices does not change while a
// process runs.  A failed probe is not cached (a transient hipGetDeviceCount error must not disable
// the library for the rest of the process): the next call probes again.
namespace {
std::atomic<int> g_count{0};
std::mutex g_count_mu;
}  // namespace

int device_count()
{
    const int n = g_count.load(std::memory_order_acquire);
    if (n > 0)
        return n;
    std::lock_guard<std::mutex> lk(g_count_mu);
    if (g_count.load(std::memory_order_relaxed) > 0)
        return g_count.load(std::memory_order_relaxed);
    int m = 0;
    if (hipGetDeviceCount(&m) != hipSuccess || m < 0)
        m = 0;
    if (m > 0)
        g_count.store(m, std::memory_order_release);
    return m;
}

int device_ok()
{
    if (device_count() > 0)
        return BRB_BATCH_OK;
    int n = 0;
    const hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess)
        set_err("hipGetDeviceCount: %s (%d)", hipGetErrorString(e), int(e));
    else
        set_err("no HIP device visible to this process");
    (void)hipGetLastError();
    return BRB_BATCH_NOT_DONE;
}

}  // namespace brb_api

namespace {

using brb_api::device_ok;
using brb_api::fail_hip;
using brb_api::set_err;
using brb_api::t_err;

}  // namespace

namespace brb_api {

// Per-thread, per-device grow-only scratch for host-mode batches.  Freed when the thread exits
// (an event thread that ends returns its HBM) or by BRB_CryptoGPU_ThreadCleanup().
struct Workspaces {
    std::vector<std::pair<void *, size_t>> by_dev;   // (ptr, capacity) per device ordinal
    uint32_t *fault_word = nullptr;                   // pair_fault.h: the thread's fault word
    uint32_t *async_word = nullptr;                   // ... and its sticky word for ASYNC calls
    // Devices on which a device-mode ASYNC call armed async_word (bit d; bit 63 also stands for every
    // device >= 63).  Those calls return before their kernels run, so a pair kernel may still write
    // the word after the thread cleans up: release() first drains these devices.
    uint64_t async_devs = 0;
    void release()
    {
        for (size_t d = 0; d < by_dev.size(); d++)
            if (by_dev[d].first) {
                brb_api::DeviceGuard g{int(d)};
                (void)hipFree(by_dev[d].first);
                by_dev[d] = {nullptr, 0};
            }
        if (async_word && async_devs) {
            int n = 0;
            if (hipGetDeviceCount(&n) != hipSuccess)
                n = 0;
            for (int d = 0; d < n; d++)
                if (async_devs & (uint64_t(1) << (d < 63 ? d : 63))) {
                    brb_api::DeviceGuard g{d};
                    if (g.error() == hipSuccess)
                        (void)hipDeviceSynchronize();
                }
            (void)hipGetLastError();
            async_devs = 0;
        }
        for (uint32_t **w : {&fault_word, &async_word})
            if (*w) {
                (void)hipHostFree(*w);
                *w = nullptr;
            }
    }
    ~Workspaces() { release(); }
};
thread_local Workspaces t_ws;
thread_local uint32_t *t_fault_armed = nullptr;       // the word the pair kernels' launchers pass

// The calling thread's fault word: page-locked, device-mapped, coherent host memory, portable to
// every device (one word serves the thread whatever device it calls on; the kernel's store is visible
// once the stream has drained).  Allocated on the thread's first armed call; nullptr if it cannot be
// had.  The word is 0 between calls (check() clears it), so arming a call is one thread-local store
// and nothing runs between the caller and the launch (the bench's events see no host work).
uint32_t *alloc_fault_word(uint32_t **slot)
{
    if (!*slot) {
        void *p = nullptr;
        if (hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        *slot = static_cast<uint32_t *>(p);
        **slot = 0;
    }
    return *slot;
}
uint32_t *fault_word() { return alloc_fault_word(&t_ws.fault_word); }

// Arms the thread's fault word for one synchronous call (pair_fault.h); check() after the stream
// has drained turns a fault into BRB_BATCH_FAULT.  A device-mode async call returns before its
// kernels run: it arms the thread's sticky async word instead, which BRB_CryptoGPU_AsyncFaultCheck
// reads (and clears) once the caller has synchronised its streams.
struct PairFault {
    uint32_t *w = nullptr;
    explicit PairFault(unsigned flags)
    {
        if ((flags & BRB_BATCH_DEVICE) && (flags & BRB_BATCH_ASYNC)) {
            t_fault_armed = alloc_fault_word(&t_ws.async_word);
            int dev = 0;
            if (t_fault_armed && hipGetDevice(&dev) == hipSuccess && dev >= 0)
                t_ws.async_devs |= uint64_t(1) << (dev < 63 ? dev : 63);
            return;
        }
        w = fault_word();
        t_fault_armed = w;
    }
    ~PairFault() { t_fault_armed = nullptr; }
    PairFault(const PairFault &) = delete;
    PairFault &operator=(const PairFault &) = delete;
    int check(int rc) const
    {
        if (!w || __atomic_load_n(w, __ATOMIC_ACQUIRE) == 0)
            return rc;
        __atomic_store_n(w, 0u, __ATOMIC_RELAXED);      // clean for the thread's next call
        if (rc != BRB_BATCH_OK)
            return rc;
        set_err("wave-pair protocol fault: a kernel's bounded wait on its partner wave gave up; the "
                "outputs (and RC4 states) of this call are wrong");
        return BRB_BATCH_FAULT;
    }
};

void release_thread_resources()
{
    // host-mode calls have drained their streams before returning; device-mode ASYNC calls may not
    // have, and release() drains the devices they armed the async fault word on before freeing it
    if (device_count() > 0) {
        t_ws.release();
        brb_host::release_thread_pipes();
    }
}

// Every host-mode call synchronises its stream before it returns (also on its error paths), so a
// workspace is never freed or regrown while a copy into it is still in flight.
void *workspace(size_t bytes, hipError_t *err)
{
    int dev = 0;
    *err = hipGetDevice(&dev);
    if (*err != hipSuccess)
        return nullptr;
    if (t_ws.by_dev.size() <= size_t(dev))
        t_ws.by_dev.resize(dev + 1, {nullptr, 0});
    auto &w = t_ws.by_dev[dev];
    if (w.first && w.second < bytes) {
        (void)hipFree(w.first);
        w = {nullptr, 0};
    }
    if (!w.first) {
        size_t cap = std::max<size_t>(bytes, size_t(1) << 20);
        void *p = nullptr;
        *err = hipMalloc(&p, cap);
        if (*err != hipSuccess)
            return nullptr;
        w = {p, cap};
    }
    return w.first;
}

}  // namespace brb_api

namespace brb {
uint32_t *pair_fault_word()
{
    return brb_api::t_fault_armed;
}
uint32_t *pair_fault_arm(uint32_t *w)
{
    uint32_t *prev = brb_api::t_fault_armed;
    brb_api::t_fault_armed = w;
    return prev;
}
}  // namespace brb

namespace {

using brb_api::PairFault;
using brb_api::workspace;

inline size_t align_up(size_t x, size_t a)
{
    return (x + a - 1) / a * a;
}

// One-lane-per-item kernels (variable-length digests, RC4 streams, segments, base64) launch one
// work-item per item, and a launch holds fewer than 2^32 work-items per dimension.
constexpr uint64_t kMaxItems = (uint64_t(1) << 32) - (uint64_t(1) << 16);

bool items_ok(uint64_t n)
{
    if (n <= kMaxItems)
        return true;
    set_err("%llu items in one call (at most %llu): split the batch", (unsigned long long)n,
            (unsigned long long)kMaxItems);
    return false;
}

// BRB_BATCH_ALL_DEVICES splits host-mode batches only (device pointers belong to one device).
bool flags_ok(unsigned flags)
{
    if ((flags & BRB_BATCH_ALL_DEVICES) && (flags & BRB_BATCH_DEVICE)) {
        set_err("BRB_BATCH_ALL_DEVICES needs host pointers (device pointers belong to one device)");
        return false;
    }
    return true;
}

int finish(hipStream_t s, unsigned flags)
{
    if ((flags & BRB_BATCH_DEVICE) && (flags & BRB_BATCH_ASYNC))
        return BRB_BATCH_OK;
    hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess)
        return fail_hip("hipStreamSynchronize", e);
    return BRB_BATCH_OK;
}

using FixedLauncher = hipError_t (*)(const uint8_t *, uint32_t, uint64_t, uint8_t *, hipStream_t);
using VarLauncher = hipError_t (*)(const uint8_t *, const uint64_t *, const uint32_t *, uint64_t, uint8_t *,
                                   hipStream_t);

int digest_fixed(FixedLauncher launch, size_t dig_len, const void *data, uint32_t rec_len, uint64_t n_rec,
                 void *digests, unsigned flags, void *stream)
{
    t_err.clear();
    if (n_rec == 0)
        return BRB_BATCH_OK;
    if (!digests || (!data && rec_len)) {
        set_err("NULL data or digests");
        return BRB_BATCH_BADARG;
    }
    if ((rec_len == 0 && !items_ok(n_rec)) || !flags_ok(flags))   // empty records: one-lane-per-record kernel
        return BRB_BATCH_BADARG;
    if (int ok = device_ok(); ok != BRB_BATCH_OK)
        return ok;
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipError_t e;
    if (flags & BRB_BATCH_DEVICE) {
        e = launch(static_cast<const uint8_t *>(data), rec_len, n_rec, static_cast<uint8_t *>(digests), s);
        if (e != hipSuccess)
            return fail_hip("kernel launch", e);
        return finish(s, flags);
    }
    return brb_host::digest_fixed(launch, dig_len, static_cast<const uint8_t *>(data), rec_len, n_rec,
                                  static_cast<uint8_t *>(digests), flags, s);
}

int digest_var(VarLauncher launch, size_t dig_len, const void *data, const uint64_t *offsets,
               const uint32_t *lengths, uint64_t n_rec, void *digests, unsigned flags, void *stream)
{
    t_err.clear();
    if (n_rec == 0)
        return BRB_BATCH_OK;
    if (!digests || !offsets || !lengths || !data) {
        set_err("NULL data, offsets, lengths or digests");
        return BRB_BATCH_BADARG;
    }
    if (!items_ok(n_rec) || !flags_ok(flags))
        return BRB_BATCH_BADARG;
    if (int ok = device_ok(); ok != BRB_BATCH_OK)
        return ok;
    if (flags & BRB_BATCH_ALL_DEVICES)   // contiguous record ranges, one per device
        return brb_host::split_devices(n_rec, [&](int, uint64_t lo, uint64_t hi) {
            return digest_var(launch, dig_len, data, offsets + lo, lengths + lo, hi - lo,
                              static_cast<uint8_t *>(digests) + lo * dig_len, flags & ~BRB_BATCH_ALL_DEVICES, nullptr);
        });
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipError_t e;
    if (flags & BRB_BATCH_DEVICE) {
        e = launch(static_cast<const uint8_t *>(data), offsets, lengths, n_rec, static_cast<uint8_t *>(digests), s);
        if (e != hipSuccess)
            return fail_hip("kernel launch", e);
        return finish(s, flags);
    }
    // host mode: copy the byte range the records cover, rebased to its first byte
    uint64_t lo = UINT64_MAX, hi = 0;
    for (uint64_t i = 0; i < n_rec; i++) {
        if (lengths[i] == 0)
            continue;
        if (offsets[i] > UINT64_MAX - lengths[i]) {
            set_err("record %llu: offset + length wraps", (unsigned long long)i);
            return BRB_BATCH_BADARG;
        }
        lo = std::min(lo, offsets[i]);
        hi = std::max(hi, offsets[i] + lengths[i]);
    }
    if (lo == UINT64_MAX)
        lo = hi = 0;
    const size_t span = size_t(hi - lo);
    const size_t o_off = align_up(span, 256);
    const size_t o_len = align_up(o_off + 8 * n_rec, 256);
    const size_t o_dig = align_up(o_len + 4 * n_rec, 256);
    uint8_t *ws = static_cast<uint8_t *>(workspace(o_dig + dig_len * n_rec, &e));
    if (!ws)
        return fail_hip("device workspace", e);
    uint64_t *rebased = static_cast<uint64_t *>(malloc(8 * n_rec));
    if (!rebased) {
        set_err("out of host memory");
        return BRB_BATCH_NOT_DONE;
    }
    for (uint64_t i = 0; i < n_rec; i++)
        rebased[i] = lengths[i] ? offsets[i] - lo : 0;
    int rc = BRB_BATCH_OK;
    if (span && (e = hipMemcpyAsync(ws, static_cast<const uint8_t *>(data) + lo, span, hipMemcpyHostToDevice, s)) != hipSuccess)
        rc = fail_hip("hipMemcpyAsync H2D", e);
    else if ((e = hipMemcpyAsync(ws + o_off, rebased, 8 * n_rec, hipMemcpyHostToDevice, s)) != hipSuccess)
        rc = fail_hip("hipMemcpyAsync H2D", e);
    else if ((e = hipMemcpyAsync(ws + o_len, lengths, 4 * n_rec, hipMemcpyHostToDevice, s)) != hipSuccess)
        rc = fail_hip("hipMemcpyAsync H2D", e);
    else if ((e = launch(ws, reinterpret_cast<const uint64_t *>(ws + o_off), reinterpret_cast<const uint32_t *>(ws + o_len),
                         n_rec, ws + o_dig, s)) != hipSuccess)
        rc = fail_hip("kernel launch", e);
    else if ((e = hipMemcpyAsync(digests, ws + o_dig, dig_len * n_rec, hipMemcpyDeviceToHost, s)) != hipSuccess)
        rc = fail_hip("hipMemcpyAsync D2H", e);
    if (rc == BRB_BATCH_OK)
        rc = finish(s, flags & ~BRB_BATCH_ASYNC);
    else
        (void)hipStreamSynchronize(s);
    free(rebased);
    return rc;
}

int blowfish_batch(const BRB_BLOWFISH_CTX *ctx, unsigned long *words, uint64_t n_blocks, unsigned flags,
                   void *stream, bool decrypt)
{
    t_err.clear();
    if (n_blocks == 0)
        return BRB_BATCH_OK;
    if (!ctx || !words) {
        set_err("NULL ctx or words");
        return BRB_BATCH_BADARG;
    }
    if (!flags_ok(flags))
        return BRB_BATCH_BADARG;
    if (int ok = device_ok(); ok != BRB_BATCH_OK)
        return ok;
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipError_t e;
    if (flags & BRB_BATCH_DEVICE) {
        e = brb::launch_blowfish(reinterpret_cast<const uint64_t *>(ctx), reinterpret_cast<uint64_t *>(words), n_blocks,
                                 decrypt, s);
        if (e != hipSuccess)
            return fail_hip("kernel launch", e);
        return finish(s, flags);
    }
    return brb_host::blowfish(ctx, reinterpret_cast<uint64_t *>(words), n_blocks, decrypt, flags, s);
}

// ---- host-mode staging for the multi-buffer (RC4) batches --------------------------------------
// Segments are laid out back to back (256-B aligned) in the per-thread workspace; `in` segments are
// copied H2D before the launch, `out` segments D2H after it (a segment may be both).
struct Staging {
    struct Seg {
        const void *h_in;
        void *h_out;
        size_t bytes, off;
    };
    std::vector<Seg> segs;
    size_t total = 0;
    uint8_t *ws = nullptr;

    size_t add(const void *h_in, void *h_out, size_t bytes)
    {
        segs.push_back({h_in, h_out, bytes, total});
        total = align_up(total + bytes, 256);
        return segs.size() - 1;
    }
    uint8_t *dev(size_t i) const { return ws + segs[i].off; }

    int upload(hipStream_t s)
    {
        hipError_t e;
        ws = static_cast<uint8_t *>(workspace(std::max<size_t>(total, 256), &e));
        if (!ws)
            return fail_hip("device workspace", e);
        for (const Seg &g : segs)
            if (g.h_in && g.bytes && (e = hipMemcpyAsync(ws + g.off, g.h_in, g.bytes, hipMemcpyHostToDevice, s)) != hipSuccess)
                return fail_hip("hipMemcpyAsync H2D", e);
        return BRB_BATCH_OK;
    }
    int download(hipStream_t s)
    {
        hipError_t e;
        for (const Seg &g : segs)
            if (g.h_out && g.bytes && (e = hipMemcpyAsync(g.h_out, ws + g.off, g.bytes, hipMemcpyDeviceToHost, s)) != hipSuccess)
                return fail_hip("hipMemcpyAsync D2H", e);
        return finish(s, 0);
    }
};

// [lo, hi) covered by ranges offsets[i] .. + lengths[i] + extra (empty ranges ignored); false (and
// the error set) when a range wraps the address space
bool span_of(const uint64_t *offs, const uint32_t *lens, uint64_t n, uint64_t extra, uint64_t &lo, uint64_t &hi)
{
    lo = UINT64_MAX;
    hi = 0;
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t len = uint64_t(lens[i]) + extra;
        if (!len)
            continue;
        if (offs[i] > UINT64_MAX - len) {
            set_err("range %llu: offset %llu + %llu bytes wraps", (unsigned long long)i, (unsigned long long)offs[i],
                    (unsigned long long)len);
            return false;
        }
        lo = std::min(lo, offs[i]);
        hi = std::max(hi, offs[i] + len);
    }
    if (lo == UINT64_MAX)
        lo = hi = 0;
    return true;
}

std::vector<uint64_t> rebase(const uint64_t *offs, uint64_t n, uint64_t lo)
{
    std::vector<uint64_t> r(n);
    for (uint64_t i = 0; i < n; i++)
        r[i] = offs[i] >= lo ? offs[i] - lo : 0;
    return r;
}

// BRB_BATCH_ALL_DEVICES for the multi-range calls whose host-mode parts write a byte span back
// (RC4 streams, frames, base64 outputs): part g stages and returns the span its ranges
// [g n/G, (g+1) n/G) cover, so the split is taken only when those spans are pairwise disjoint --
// otherwise a part would write back bytes of another part's ranges.  Streams of different
// connections are disjoint by contract; ranges in submission order give disjoint spans.  Ranges
// in any other order run on the calling thread's device (same results, one device).
bool parts_disjoint(const uint64_t *offs, const uint32_t *lens, uint64_t n, uint64_t extra, const uint32_t *lens_out = nullptr)
{
    const int G = brb_host::split_parts();
    if (G <= 1 || n < uint64_t(G))
        return false;
    std::vector<std::pair<uint64_t, uint64_t>> sp;
    for (int g = 0; g < G; g++) {
        const uint64_t a = n * uint64_t(g) / uint64_t(G), b = n * uint64_t(g + 1) / uint64_t(G);
        uint64_t lo, hi;
        if (!span_of(offs + a, lens_out ? lens_out + a : lens + a, b - a, extra, lo, hi))
            return false;
        if (hi > lo)
            sp.push_back({lo, hi});
    }
    std::sort(sp.begin(), sp.end());
    for (size_t i = 1; i < sp.size(); i++)
        if (sp[i].first < sp[i - 1].second)
            return false;
    return true;
}

int rc4_crypt_batch(BRB_RC4_State *states, const void *in, void *out, const uint64_t *offsets, const uint32_t *lengths,
                    uint64_t n, unsigned flags, void *stream)
{
    t_err.clear();
    if (n == 0)
        return BRB_BATCH_OK;
    if (!states || !in || !out || !offsets || !lengths) {
        set_err("NULL states, in, out, offsets or lengths");
        return BRB_BATCH_BADARG;
    }
    if (!items_ok(n) || !flags_ok(flags))
        return BRB_BATCH_BADARG;
    if (int ok = device_ok(); ok != BRB_BATCH_OK)
        return ok;
    if (flags & BRB_BATCH_ALL_DEVICES) {   // connections split over the devices, states with them
        flags &= ~BRB_BATCH_ALL_DEVICES;
        if (parts_disjoint(offsets, lengths, n, 0))
            return brb_host::split_devices(n, [&](int, uint64_t lo, uint64_t hi) {
                return rc4_crypt_batch(states + lo, in, out, offsets + lo, lengths + lo, hi - lo, flags, nullptr);
            });
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    const PairFault pf(flags);                       // pair_fault.h
    hipError_t e;
    if (flags & BRB_BATCH_DEVICE) {
        e = brb::launch_rc4_crypt(reinterpret_cast<uint8_t *>(states), static_cast<const uint8_t *>(in),
                                  static_cast<uint8_t *>(out), offsets, lengths, n, s);
        if (e != hipSuccess)
            return fail_hip("kernel launch", e);
        return pf.check(finish(s, flags));
    }
    uint64_t lo, hi;
    if (!span_of(offsets, lengths, n, 0, lo, hi))
        return BRB_BATCH_BADARG;
    const std::vector<uint64_t> roff = rebase(offsets, n, lo);
    const size_t span = size_t(hi - lo);
    Staging st;
    const size_t i_st = st.add(states, states, sizeof(BRB_RC4_State) * n);
    const size_t i_in = st.add(static_cast<const uint8_t *>(in) + lo, in == out ? static_cast<uint8_t *>(out) + lo : nullptr, span);
    // a separate output buffer is staged with its current bytes so that bytes outside the streams survive
    const size_t i_out = in == out ? i_in : st.add(static_cast<uint8_t *>(out) + lo, static_cast<uint8_t *>(out) + lo, span);
    const size_t i_off = st.add(roff.data(), nullptr, 8 * n);
    const size_t i_len = st.add(lengths, nullptr, 4 * n);
    int rc = st.upload(s);
    if (rc == BRB_BATCH_OK &&
        (e = brb::launch_rc4_crypt(st.dev(i_st), st.dev(i_in), st.dev(i_out), reinterpret_cast<const uint64_t *>(st.dev(i_off)),
                                   reinterpret_cast<const uint32_t *>(st.dev(i_len)), n, s)) != hipSuccess)
        rc = fail_hip("kernel launch", e);
    if (rc == BRB_BATCH_OK)
        return pf.check(st.download(s));
    (void)hipStreamSynchronize(s);
    return rc;
}

int rc4md5_frame_batch(BRB_RC4_State *states, const void *payload, const uint64_t *offsets, const uint32_t *lengths,
                       const uint64_t *salts, void *frames, const uint64_t *frame_offsets, uint64_t n, unsigned flags,
                       void *stream)
{
    t_err.clear();
    if (n == 0)
        return BRB_BATCH_OK;
    if (!states || !payload || !offsets || !lengths || !salts || !frames || !frame_offsets) {
        set_err("NULL states, payload, offsets, lengths, salts, frames or frame_offsets");
        return BRB_BATCH_BADARG;
    }
    if (!items_ok(n) || !flags_ok(flags))
        return BRB_BATCH_BADARG;
    if (int ok = device_ok(); ok != BRB_BATCH_OK)
        return ok;
    if (flags & BRB_BATCH_ALL_DEVICES) {   // frames are written back: their spans must not interleave
        flags &= ~BRB_BATCH_ALL_DEVICES;
        if (parts_disjoint(frame_offsets, lengths, n, BRB_RC4MD5_HEADER))
            return brb_host::split_devices(n, [&](int, uint64_t lo, uint64_t hi) {
                return rc4md5_frame_batch(states + lo, payload, offsets + lo, lengths + lo, salts + lo, frames,
                                          frame_offsets + lo, hi - lo, flags, nullptr);
            });
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    const PairFault pf(flags);                       // pair_fault.h
    hipError_t e;
    if (flags & BRB_BATCH_DEVICE) {
        e = brb::launch_rc4md5_frame(reinterpret_cast<uint8_t *>(states), static_cast<const uint8_t *>(payload), offsets,
                                     lengths, salts, static_cast<uint8_t *>(frames), frame_offsets, n, s);
        if (e != hipSuccess)
            return fail_hip("kernel launch", e);
        return pf.check(finish(s, flags));
    }
    uint64_t plo, phi, flo, fhi;
    if (!span_of(offsets, lengths, n, 0, plo, phi) || !span_of(frame_offsets, lengths, n, BRB_RC4MD5_HEADER, flo, fhi))
        return BRB_BATCH_BADARG;
    const std::vector<uint64_t> poff = rebase(offsets, n, plo), foff = rebase(frame_offsets, n, flo);
    Staging st;
    const size_t i_st = st.add(states, states, sizeof(BRB_RC4_State) * n);
    const size_t i_pl = st.add(static_cast<const uint8_t *>(payload) + plo, nullptr, size_t(phi - plo));
    const size_t i_fr = st.add(static_cast<uint8_t *>(frames) + flo, static_cast<uint8_t *>(frames) + flo, size_t(fhi - flo));
    const size_t i_po = st.add(poff.data(), nullptr, 8 * n);
    const size_t i_fo = st.add(foff.data(), nullptr, 8 * n);
    const size_t i_len = st.add(lengths, nullptr, 4 * n);
    const size_t i_salt = st.add(salts, nullptr, 8 * n);
    int rc = st.upload(s);
    if (rc == BRB_BATCH_OK &&
        (e = brb::launch_rc4md5_frame(st.dev(i_st), st.dev(i_pl), reinterpret_cast<const uint64_t *>(st.dev(i_po)),
                                      reinterpret_cast<const uint32_t *>(st.dev(i_len)),
                                      reinterpret_cast<const uint64_t *>(st.dev(i_salt)), st.dev(i_fr),
                                      reinterpret_cast<const uint64_t *>(st.dev(i_fo)), n, s)) != hipSuccess)
        rc = fail_hip("kernel launch", e);
    if (rc == BRB_BATCH_OK)
        return pf.check(st.download(s));
    (void)hipStreamSynchronize(s);
    return rc;
}

int rc4md5_open_batch(BRB_RC4_State *states, const void *frames, void *out, const uint64_t *offsets,
                      const uint32_t *lengths, uint64_t n, uint8_t *valid, unsigned flags, void *stream)
{
    t_err.clear();
    if (n == 0)
        return BRB_BATCH_OK;
    if (!states || !frames || !out || !offsets || !lengths || !valid) {
        set_err("NULL states, frames, out, offsets, lengths or valid");
        return BRB_BATCH_BADARG;
    }
    if (!items_ok(n) || !flags_ok(flags))
        return BRB_BATCH_BADARG;
    if (int ok = device_ok(); ok != BRB_BATCH_OK)
        return ok;
    if (flags & BRB_BATCH_ALL_DEVICES) {
        flags &= ~BRB_BATCH_ALL_DEVICES;
        if (parts_disjoint(offsets, lengths, n, 0))
            return brb_host::split_devices(n, [&](int, uint64_t lo, uint64_t hi) {
                return rc4md5_open_batch(states + lo, frames, out, offsets + lo, lengths + lo, hi - lo, valid + lo, flags,
                                         nullptr);
            });
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    const PairFault pf(flags);                       // pair_fault.h
    hipError_t e;
    if (flags & BRB_BATCH_DEVICE) {
        e = brb::launch_rc4md5_open(reinterpret_cast<uint8_t *>(states), static_cast<const uint8_t *>(frames),
                                    static_cast<uint8_t *>(out), offsets, lengths, n, valid, s);
        if (e != hipSuccess)
            return fail_hip("kernel launch", e);
        return pf.check(finish(s, flags));
    }
    uint64_t lo, hi;
    if (!span_of(offsets, lengths, n, 0, lo, hi))
        return BRB_BATCH_BADARG;
    const std::vector<uint64_t> roff = rebase(offsets, n, lo);
    const size_t span = size_t(hi - lo);
    Staging st;
    const size_t i_st = st.add(states, states, sizeof(BRB_RC4_State) * n);
    const size_t i_in = st.add(static_cast<const uint8_t *>(frames) + lo, frames == out ? static_cast<uint8_t *>(out) + lo : nullptr, span);
    const size_t i_out = frames == out ? i_in : st.add(static_cast<uint8_t *>(out) + lo, static_cast<uint8_t *>(out) + lo, span);
    const size_t i_off = st.add(roff.data(), nullptr, 8 * n);
    const size_t i_len = st.add(lengths, nullptr, 4 * n);
    const size_t i_val = st.add(nullptr, valid, n);
    int rc = st.upload(s);
    if (rc == BRB_BATCH_OK &&
        (e = brb::launch_rc4md5_open(st.dev(i_st), st.dev(i_in), st.dev(i_out), reinterpret_cast<const uint64_t *>(st.dev(i_off)),
                                     reinterpret_cast<const uint32_t *>(st.dev(i_len)), n, st.dev(i_val), s)) != hipSuccess)
        rc = fail_hip("kernel launch", e);
    if (rc == BRB_BATCH_OK)
        return pf.check(st.download(s));
    (void)hipStreamSynchronize(s);
    return rc;
}

int md5_segments(const void *data, const uint64_t *soff, const uint32_t *slen, const uint64_t *first, uint64_t n_rec,
                 void *digests, unsigned flags, void *stream)
{
    t_err.clear();
    if (n_rec == 0)
        return BRB_BATCH_OK;
    if (!digests || !first || (!data || !soff || !slen)) {
        set_err("NULL data, seg_offsets, seg_lengths, rec_first_seg or digests");
        return BRB_BATCH_BADARG;
    }
    if (!items_ok(n_rec) || !flags_ok(flags))
        return BRB_BATCH_BADARG;
    if (int ok = device_ok(); ok != BRB_BATCH_OK)
        return ok;
    if (flags & BRB_BATCH_ALL_DEVICES)   // contiguous record ranges (segment lists with them), one per device
        return brb_host::split_devices(n_rec, [&](int, uint64_t lo, uint64_t hi) {
            return md5_segments(data, soff, slen, first + lo, hi - lo, static_cast<uint8_t *>(digests) + 16 * lo,
                                flags & ~BRB_BATCH_ALL_DEVICES, nullptr);
        });
    hipStream_t s = static_cast<hipStream_t>(stream);
    const PairFault pf(flags);                       // pair_fault.h
    hipError_t e;
    if (flags & BRB_BATCH_DEVICE) {
        e = brb::launch_md5_segments(static_cast<const uint8_t *>(data), soff, slen, first, n_rec,
                                     static_cast<uint8_t *>(digests), s);
        if (e != hipSuccess)
            return fail_hip("kernel launch", e);
        return pf.check(finish(s, flags));
    }
    // host mode: rebase the segment lists to start at 0 and copy the byte span they cover
    const uint64_t k0 = first[0], nseg = first[n_rec] - k0;
    for (uint64_t i = 0; i < n_rec; i++)
        if (first[i + 1] < first[i]) {
            set_err("rec_first_seg is not non-decreasing at %llu", (unsigned long long)i);
            return BRB_BATCH_BADARG;
        }
    uint64_t lo, hi;
    if (!span_of(soff + k0, slen + k0, nseg, 0, lo, hi))
        return BRB_BATCH_BADARG;
    const std::vector<uint64_t> roff = rebase(soff + k0, nseg, lo);
    std::vector<uint64_t> rfirst(first, first + n_rec + 1);
    for (uint64_t &f : rfirst)
        f -= k0;
    Staging st;
    const size_t i_d = st.add(static_cast<const uint8_t *>(data) + lo, nullptr, size_t(hi - lo));
    const size_t i_o = st.add(roff.data(), nullptr, 8 * nseg);
    const size_t i_l = st.add(slen + k0, nullptr, 4 * nseg);
    const size_t i_f = st.add(rfirst.data(), nullptr, 8 * (n_rec + 1));
    const size_t i_out = st.add(nullptr, digests, 16 * n_rec);
    int rc = st.upload(s);
    if (rc == BRB_BATCH_OK &&
        (e = brb::launch_md5_segments(st.dev(i_d), reinterpret_cast<const uint64_t *>(st.dev(i_o)),
                                      reinterpret_cast<const uint32_t *>(st.dev(i_l)),
                                      reinterpret_cast<const uint64_t *>(st.dev(i_f)), n_rec, st.dev(i_out), s)) != hipSuccess)
        rc = fail_hip("kernel launch", e);
    if (rc == BRB_BATCH_OK)
        return pf.check(st.download(s));
    (void)hipStreamSynchronize(s);
    return rc;
}

// ---- MetaData packs ------------------------------------------------------------
int metadata_unpack(const void *data, const uint64_t *offs, const uint32_t *lens, uint64_t n,
                    BRB_MetaDataUnpackInfo *info, unsigned flags, void *stream)
{
    t_err.clear();
    if (n == 0)
        return BRB_BATCH_OK;
    if (!data || !offs || !lens || !info) {
        set_err("NULL data, offsets, lengths or info");
        return BRB_BATCH_BADARG;
    }
    if (!items_ok(n) || !flags_ok(flags))
        return BRB_BATCH_BADARG;
    if (int ok = device_ok(); ok != BRB_BATCH_OK)
        return ok;
    if (flags & BRB_BATCH_ALL_DEVICES)   // contiguous pack ranges, one per device
        return brb_host::split_devices(n, [&](int, uint64_t lo, uint64_t hi) {
            return metadata_unpack(data, offs + lo, lens + lo, hi - lo, info + lo, flags & ~BRB_BATCH_ALL_DEVICES, nullptr);
        });
    hipStream_t s = static_cast<hipStream_t>(stream);
    const PairFault pf(flags);                       // pair_fault.h
    hipError_t e;
    if (flags & BRB_BATCH_DEVICE) {
        if ((e = brb::launch_metadata_unpack(static_cast<const uint8_t *>(data), offs, lens, n, info, s)) != hipSuccess)
            return fail_hip("kernel launch", e);
        return pf.check(finish(s, flags));
    }
    // host mode: copy the byte span the packs cover, with the offsets rebased to it
    uint64_t lo, hi;
    if (!span_of(offs, lens, n, 0, lo, hi))
        return BRB_BATCH_BADARG;
    const std::vector<uint64_t> roff = rebase(offs, n, lo);
    Staging st;
    const size_t i_d = st.add(static_cast<const uint8_t *>(data) + lo, nullptr, size_t(hi - lo));
    const size_t i_o = st.add(roff.data(), nullptr, 8 * n);
    const size_t i_l = st.add(lens, nullptr, 4 * n);
    const size_t i_out = st.add(nullptr, info, sizeof(BRB_MetaDataUnpackInfo) * n);
    int rc = st.upload(s);
    if (rc == BRB_BATCH_OK &&
        (e = brb::launch_metadata_unpack(st.dev(i_d), reinterpret_cast<const uint64_t *>(st.dev(i_o)),
                                         reinterpret_cast<const uint32_t *>(st.dev(i_l)), n,
                                         reinterpret_cast<BRB_MetaDataUnpackInfo *>(st.dev(i_out)), s)) != hipSuccess)
        rc = fail_hip("kernel launch", e);
    if (rc == BRB_BATCH_OK)
        return pf.check(st.download(s));
    (void)hipStreamSynchronize(s);
    return rc;
}

// ---- base64 --------------------------------------------------------------------
int b64_batch(bool decode, const void *in, const uint64_t *offs, const uint32_t *lens, uint64_t n, void *out,
              const uint64_t *ooffs, uint32_t *olens, unsigned flags, void *stream)
{
    t_err.clear();
    if (n == 0)
        return BRB_BATCH_OK;
    if (!in || !offs || !lens || !out || !ooffs || (decode && !olens)) {
        set_err("NULL data, offsets, lengths, out, out_offsets or out_lengths");
        return BRB_BATCH_BADARG;
    }
    if (!items_ok(n) || !flags_ok(flags))
        return BRB_BATCH_BADARG;
    if (int ok = device_ok(); ok != BRB_BATCH_OK)
        return ok;
    if (flags & BRB_BATCH_ALL_DEVICES) {   // outputs are written back: their spans must not interleave
        flags &= ~BRB_BATCH_ALL_DEVICES;
        std::vector<uint32_t> omax(n);
        for (uint64_t i = 0; i < n; i++)
            omax[i] = decode ? 3u * (lens[i] / 4) : 4u * ((lens[i] + 2) / 3);
        if (parts_disjoint(ooffs, lens, n, 0, omax.data()))
            return brb_host::split_devices(n, [&](int, uint64_t lo, uint64_t hi) {
                return b64_batch(decode, in, offs + lo, lens + lo, hi - lo, out, ooffs + lo, olens ? olens + lo : nullptr,
                                 flags, nullptr);
            });
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipError_t e;
    uint64_t mean_len = 0;                      // unknown in device mode (the lengths are device memory)
    if (!(flags & BRB_BATCH_DEVICE)) {
        uint64_t sum = 0;
        for (uint64_t i = 0; i < n; i++)
            sum += lens[i];
        mean_len = sum / n + 1;
    }
    auto launch = [&](const uint8_t *i, const uint64_t *o, const uint32_t *l, uint8_t *d, const uint64_t *oo,
                      uint32_t *ol) {
        return decode ? brb::launch_b64_decode(i, o, l, n, d, oo, ol, mean_len, s)
                      : brb::launch_b64_encode(i, o, l, n, d, oo, mean_len, s);
    };
    if (flags & BRB_BATCH_DEVICE) {
        if ((e = launch(static_cast<const uint8_t *>(in), offs, lens, static_cast<uint8_t *>(out), ooffs, olens)) != hipSuccess)
            return fail_hip("kernel launch", e);
        return finish(s, flags);
    }
    // output extents: encode 4 * ceil(len / 3), decode at most 3 * (len / 4)
    std::vector<uint32_t> olen_max(n);
    for (uint64_t i = 0; i < n; i++)
        olen_max[i] = decode ? 3u * (lens[i] / 4) : 4u * ((lens[i] + 2) / 3);
    uint64_t lo, hi, olo, ohi;
    if (!span_of(offs, lens, n, 0, lo, hi) || !span_of(ooffs, olen_max.data(), n, 0, olo, ohi))
        return BRB_BATCH_BADARG;
    const std::vector<uint64_t> roff = rebase(offs, n, lo), rooff = rebase(ooffs, n, olo);
    Staging st;
    const size_t i_in = st.add(static_cast<const uint8_t *>(in) + lo, nullptr, size_t(hi - lo));
    const size_t i_out = st.add(static_cast<uint8_t *>(out) + olo, static_cast<uint8_t *>(out) + olo, size_t(ohi - olo));
    const size_t i_o = st.add(roff.data(), nullptr, 8 * n);
    const size_t i_l = st.add(lens, nullptr, 4 * n);
    const size_t i_oo = st.add(rooff.data(), nullptr, 8 * n);
    const size_t i_ol = decode ? st.add(nullptr, olens, 4 * n) : 0;
    int rc = st.upload(s);
    if (rc == BRB_BATCH_OK &&
        (e = launch(st.dev(i_in), reinterpret_cast<const uint64_t *>(st.dev(i_o)), reinterpret_cast<const uint32_t *>(st.dev(i_l)),
                    st.dev(i_out), reinterpret_cast<const uint64_t *>(st.dev(i_oo)),
                    decode ? reinterpret_cast<uint32_t *>(st.dev(i_ol)) : nullptr)) != hipSuccess)
        rc = fail_hip("kernel launch", e);
    if (rc == BRB_BATCH_OK)
        return st.download(s);
    (void)hipStreamSynchronize(s);
    return rc;
}

// ---- MemBuffer Blowfish -------------------------------------------------------
int membuf_crypt(void *buf, unsigned long size, unsigned int seed, unsigned long offset, unsigned long *new_size,
                 unsigned flags, void *stream, bool decrypt)
{
    t_err.clear();
    if (!buf || !new_size) {
        set_err("NULL buf or new_size");
        return BRB_BATCH_BADARG;
    }
    if (decrypt && size < offset) {
        set_err("size %lu < offset %lu (the reference would walk ~2^61 words)", size, offset);
        return BRB_BATCH_BADARG;
    }
    uint8_t *raw = static_cast<uint8_t *>(buf) + offset;
    if ((flags & BRB_BATCH_DEVICE) && (reinterpret_cast<uintptr_t>(raw) & 7)) {
        set_err("device mode needs buf + offset 8-byte aligned");
        return BRB_BATCH_BADARG;
    }
    if (int ok = device_ok(); ok != BRB_BATCH_OK)
        return ok;
    // host side: key (mem_buf.c:1511-1515) and the reference's keyLen quirk (:1528 vs :1582)
    unsigned int key[16];
    BRB_MemBufferKey(seed, key);
    BRB_BLOWFISH_CTX *ctx = static_cast<BRB_BLOWFISH_CTX *>(malloc(sizeof(BRB_BLOWFISH_CTX)));
    if (!ctx) {
        set_err("out of host memory");
        return BRB_BATCH_NOT_DONE;
    }
    BRB_Blowfish_Init(ctx, reinterpret_cast<unsigned char *>(key), decrypt ? int(sizeof(key)) : int(sizeof(key[0])));
    const uint64_t words = (decrypt ? (size - offset) : (size + offset)) / 8 + 2;
    const uint64_t pairs = (words + 1) / 2;
    const size_t span = size_t(16) * pairs;
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipError_t e;
    Staging st;
    const size_t i_ctx = st.add(ctx, nullptr, sizeof(BRB_BLOWFISH_CTX));
    const size_t i_first = st.add(nullptr, nullptr, 8);
    const size_t i_w = (flags & BRB_BATCH_DEVICE) ? 0 : st.add(raw, raw, span);
    int rc = st.upload(s);
    uint64_t *w = (flags & BRB_BATCH_DEVICE) ? reinterpret_cast<uint64_t *>(raw) : reinterpret_cast<uint64_t *>(st.dev(i_w));
    unsigned long long done = pairs;
    if (rc == BRB_BATCH_OK && decrypt) {
        unsigned long long *first = reinterpret_cast<unsigned long long *>(st.dev(i_first));
        if ((e = hipMemcpyAsync(first, &done, 8, hipMemcpyHostToDevice, s)) != hipSuccess)
            rc = fail_hip("hipMemcpyAsync H2D", e);
        else if ((e = brb::launch_first_zero_pair(w, pairs, first, s)) != hipSuccess)
            rc = fail_hip("kernel launch", e);
        else if ((e = hipMemcpyAsync(&done, first, 8, hipMemcpyDeviceToHost, s)) != hipSuccess ||
                 (e = hipStreamSynchronize(s)) != hipSuccess)
            rc = fail_hip("zero-pair scan", e);
    }
    if (rc == BRB_BATCH_OK &&
        (e = brb::launch_blowfish(reinterpret_cast<const uint64_t *>(st.dev(i_ctx)), w, done, decrypt, s)) != hipSuccess)
        rc = fail_hip("kernel launch", e);
    if (rc == BRB_BATCH_OK)
        rc = st.download(s);        // host mode: the staged words back; always: synchronise
    else
        (void)hipStreamSynchronize(s);
    free(ctx);
    if (rc == BRB_BATCH_OK)
        *new_size = static_cast<unsigned long>(16 * done + offset);
    return rc;
}

}  // namespace

extern "C" {

int BRB_Base64EncodeBatch(const void *data, const uint64_t *offsets, const uint32_t *lengths, uint64_t n, void *out,
                          const uint64_t *out_offsets, unsigned flags, void *hip_stream)
{
    return b64_batch(false, data, offsets, lengths, n, out, out_offsets, nullptr, flags, hip_stream);
}

int BRB_Base64DecodeBatch(const void *text, const uint64_t *offsets, const uint32_t *lengths, uint64_t n, void *out,
                          const uint64_t *out_offsets, uint32_t *out_lengths, unsigned flags, void *hip_stream)
{
    return b64_batch(true, text, offsets, lengths, n, out, out_offsets, out_lengths, flags, hip_stream);
}

void BRB_MemBufferKey(unsigned int seed, unsigned int key[16])
{
    for (unsigned long i = 0; i < 16; i++) {          // mem_buf.c:1511-1515 (unsigned long i)
        key[i] = static_cast<unsigned int>(((i + seed) * seed) + (13 * i));
        seed = key[i] * seed;
    }
}

int BRB_MemBufferEncrypt(void *buf, unsigned long size, unsigned int seed, unsigned long offset, unsigned long *new_size,
                         unsigned flags, void *hip_stream)
{
    return membuf_crypt(buf, size, seed, offset, new_size, flags, hip_stream, false);
}

int BRB_MemBufferDecrypt(void *buf, unsigned long size, unsigned int seed, unsigned long offset, unsigned long *new_size,
                         unsigned flags, void *hip_stream)
{
    return membuf_crypt(buf, size, seed, offset, new_size, flags, hip_stream, true);
}

int BRB_MD5BatchFixed(const void *data, uint32_t rec_len, uint64_t n_rec, unsigned char (*digests)[16], unsigned flags,
                      void *hip_stream)
{
    return digest_fixed(brb::launch_md5_fixed, 16, data, rec_len, n_rec, digests, flags, hip_stream);
}

int BRB_MD5Batch(const void *data, const uint64_t *offsets, const uint32_t *lengths, uint64_t n_rec,
                 unsigned char (*digests)[16], unsigned flags, void *hip_stream)
{
    return digest_var(brb::launch_md5_var, 16, data, offsets, lengths, n_rec, digests, flags, hip_stream);
}

int BRB_MD5BatchSegments(const void *data, const uint64_t *seg_offsets, const uint32_t *seg_lengths,
                         const uint64_t *rec_first_seg, uint64_t n_rec, unsigned char (*digests)[16], unsigned flags,
                         void *hip_stream)
{
    return md5_segments(data, seg_offsets, seg_lengths, rec_first_seg, n_rec, digests, flags, hip_stream);
}

int BRB_MetaDataUnpackBatch(const void *data, const uint64_t *offsets, const uint32_t *lengths, uint64_t n_packs,
                            BRB_MetaDataUnpackInfo *info, unsigned flags, void *hip_stream)
{
    return metadata_unpack(data, offsets, lengths, n_packs, info, flags, hip_stream);
}

int BrbSha1_BatchFixed(const void *data, uint32_t rec_len, uint64_t n_rec, uint8_t (*digests)[20], unsigned flags,
                       void *hip_stream)
{
    return digest_fixed(brb::launch_sha1_fixed, 20, data, rec_len, n_rec, digests, flags, hip_stream);
}

int BrbSha1_Batch(const void *data, const uint64_t *offsets, const uint32_t *lengths, uint64_t n_rec,
                  uint8_t (*digests)[20], unsigned flags, void *hip_stream)
{
    return digest_var(brb::launch_sha1_var, 20, data, offsets, lengths, n_rec, digests, flags, hip_stream);
}

int BRB_Blowfish_EncryptBatch(const BRB_BLOWFISH_CTX *ctx, unsigned long *words, uint64_t n_blocks, unsigned flags,
                              void *hip_stream)
{
    return blowfish_batch(ctx, words, n_blocks, flags, hip_stream, false);
}

int BRB_Blowfish_DecryptBatch(const BRB_BLOWFISH_CTX *ctx, unsigned long *words, uint64_t n_blocks, unsigned flags,
                              void *hip_stream)
{
    return blowfish_batch(ctx, words, n_blocks, flags, hip_stream, true);
}

int BRB_RC4_CryptBatch(BRB_RC4_State *states, const void *in, void *out, const uint64_t *offsets, const uint32_t *lengths,
                       uint64_t n_streams, unsigned flags, void *hip_stream)
{
    return rc4_crypt_batch(states, in, out, offsets, lengths, n_streams, flags, hip_stream);
}

int BRB_RC4MD5_FrameBatch(BRB_RC4_State *states, const void *payload, const uint64_t *offsets, const uint32_t *lengths,
                          const uint64_t *salts, void *frames, const uint64_t *frame_offsets, uint64_t n, unsigned flags,
                          void *hip_stream)
{
    return rc4md5_frame_batch(states, payload, offsets, lengths, salts, frames, frame_offsets, n, flags, hip_stream);
}

int BRB_RC4MD5_OpenBatch(BRB_RC4_State *states, const void *frames, void *out, const uint64_t *offsets,
                         const uint32_t *lengths, uint64_t n, uint8_t *valid, unsigned flags, void *hip_stream)
{
    return rc4md5_open_batch(states, frames, out, offsets, lengths, n, valid, flags, hip_stream);
}

int BRB_CryptoGPU_Available(void)
{
    t_err.clear();
    return device_ok() == BRB_BATCH_OK ? 1 : 0;
}

int BRB_CryptoGPU_DeviceCount(void)
{
    t_err.clear();
    const int n = brb_api::device_count();
    if (n == 0)
        (void)device_ok();   // sets the reason
    return n;
}

int BRB_CryptoGPU_SetDevice(int dev)
{
    t_err.clear();
    if (int ok = device_ok(); ok != BRB_BATCH_OK)
        return ok;
    if (dev < 0 || dev >= brb_api::device_count()) {
        set_err("device %d out of range (%d visible)", dev, brb_api::device_count());
        return BRB_BATCH_BADARG;
    }
    hipError_t e = hipSetDevice(dev);
    return e == hipSuccess ? BRB_BATCH_OK : fail_hip("hipSetDevice", e);
}

int BRB_CryptoGPU_GetDevice(void)
{
    t_err.clear();
    if (device_ok() != BRB_BATCH_OK)
        return -1;
    int dev = -1;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) {
        fail_hip("hipGetDevice", e);
        return -1;
    }
    return dev;
}

void BRB_CryptoGPU_ThreadCleanup(void)
{
    t_err.clear();
    brb_api::release_thread_resources();
}

const char *BRB_CryptoGPU_LastError(void)
{
    return t_err.c_str();
}

int BRB_CryptoGPU_AsyncFaultCheck(void)
{
    brb_api::clear_err();
    uint32_t *w = brb_api::t_ws.async_word;
    if (!w || __atomic_load_n(w, __ATOMIC_ACQUIRE) == 0)
        return BRB_BATCH_OK;
    __atomic_store_n(w, 0u, __ATOMIC_RELAXED);
    set_err("wave-pair protocol fault in a device-mode BRB_BATCH_ASYNC call of this thread since the last check: "
            "that call's outputs (and RC4 states) are wrong");
    return BRB_BATCH_FAULT;
}

const char *BRB_CryptoGPU_Version(void)
{
    return "brb_crypto_gpu 0.1 (gfx950)";
}

}  // extern "C"

extern "C" int BRB_CryptoGPU_TestOption(const char *name, int value, int *old)
{
    brb_api::clear_err();
    static const struct {
        const char *name;
        brb_opt::Opt opt;
        int lo, hi;
    } known[] = {{"rc4_sector", brb_opt::kRc4Sector, -1, 1},
                 {"var_line", brb_opt::kVarLine, 0, 1},
                 {"fixed_var_line", brb_opt::kFixedVarLine, 0, 1},
                 {"var_sort", brb_opt::kVarSort, 0, 2},
                 {"devices", brb_opt::kDevices, 0, 16},   // an all-devices batcher takes at most 16 parts
                 {"b64_group", brb_opt::kB64Group, -1, 6},
                 {"host_chunk_mib", brb_opt::kHostChunkMiB, 0, 1024},
                 {"host_digest_chunk_mib", brb_opt::kHostDigestChunkMiB, 0, 1024},
                 {"seg_line", brb_opt::kSegLine, 0, 2},
                 {"b64_kernel", brb_opt::kB64Kernel, 0, 3},
                 {"line_slots", brb_opt::kLineSlots, 0, 3},
                 {"rc4md5_pair", brb_opt::kRc4Pair, 0, 1},
                 {"rc4_pair", brb_opt::kRc4CryptPair, 0, 1},
                 {"pair_stall", brb_opt::kPairStall, 0, 1}};
    if (!name) {
        set_err("NULL option name");
        return BRB_BATCH_BADARG;
    }
    for (const auto &k : known)
        if (strcmp(name, k.name) == 0) {
            if (value < k.lo || value > k.hi) {
                set_err("test option %s: value %d out of [%d, %d]", name, value, k.lo, k.hi);
                return BRB_BATCH_BADARG;
            }
            const int prev = brb_opt::g_opt[k.opt].exchange(value, std::memory_order_relaxed);
            if (old)
                *old = prev;
            return BRB_BATCH_OK;
        }
    set_err("unknown test option '%s'", name);
    return BRB_BATCH_BADARG;
}
