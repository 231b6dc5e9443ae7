// transform_batcher.hip -- receive-loop batching of the comm transform.
//
// The reference calls the transform hook per buffer on the connection's event thread
// (EvAIOReqTransform_ReadData / _WriteData, ev_kq_aio_transform.c:42-70).  The batcher collects the
// buffers of one event-loop round from many connections in a pinned host arena, runs the round as
// one H2D copy, one kernel per direction and sub-round, one D2H copy, and hands every result back
// in submission order.  The connections' RC4 states (CommEvCryptoInfo's read and write
// BRB_RC4_State, libbrb_ev_comm.h:206-236) stay resident in HBM; the kernels address them through a
// connection table (launch_rc4_* `sidx`).
//
// Ordering: a connection's buffers in one direction form one RC4 stream, so a round may hold at
// most one of them per sub-round; the k-th buffer of a connection in a round runs in sub-round k.
//
// Zero-copy rounds (BRB_BATCHER_ZERO_COPY): the callers' buffers are page-locked, Read/Write keep a
// reference instead of copying them into the arena, the kernels read them over PCIe and write the
// results straight into the page-locked output arena.  The copy mode spent ~60 % of a round in the
// submit memcpy (4.9 of 8.1 ms for 16 384 connections x 2 buffers, tools/batcher_bench.c).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "api_util.h"
#include "brb_crypto.h"
#include "brb_kernels.h"
#include "host_pipe.h"

using brb_api::DeviceGuard;
using brb_api::fail_hip;
using brb_api::set_err;

namespace {

constexpr uint32_t kHdr = BRB_RC4MD5_HEADER;
constexpr size_t kAlign = 256;    // arenas
constexpr size_t kMetaItem = 80;  // metadata bytes budgeted per buffer: 32 of arrays + up to 40 of padding + valid

inline size_t up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct Item {
    uint32_t conn;
    int op;
    uint64_t in_off;  // copy mode: offset in the input arena; zero-copy: device address of the buffer
    uint32_t in_len;
    uint64_t out_off;
    uint32_t out_len;
    uint64_t salt;
    uint32_t round;   // sub-round
    uint32_t epoch;   // the connection's key epoch at submission (BRB_TransformBatcher::epoch)
};

// Page-locked host ranges registered through BRB_CryptoGPU_HostRegister: host base, length, the
// device address of the base.  Sorted by host base.
struct HostRange {
    uintptr_t h;
    uint64_t len;
    uintptr_t d;
};
std::mutex g_ranges_mu;
std::vector<HostRange> g_ranges;
std::atomic<uint64_t> g_ranges_gen{1};          // bumped by every unregister
constexpr int kHits = 4;                         // a loop's read pool, write pool, ...
thread_local HostRange t_last[kHits];            // this thread's last hits, valid while gen matches
thread_local unsigned t_next = 0;
thread_local uint64_t t_last_gen = 0;

// Device address of [p, p + len) if it lies in page-locked memory the GPU can read (device `dev`).
bool host_to_device(const void *p, uint64_t len, uintptr_t *d, int dev)
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    // a receive loop submits buffers from the same few regions (reads and writes alternate between
    // two pools): a few compares instead of the lock, which several submitting threads would share
    if (t_last_gen == g_ranges_gen.load(std::memory_order_acquire))
        for (const HostRange &r : t_last)
            if (a >= r.h && a - r.h + len <= r.len && r.len) {
                *d = r.d + (a - r.h);
                return true;
            }
    {
        std::lock_guard<std::mutex> lk(g_ranges_mu);
        auto it = std::upper_bound(g_ranges.begin(), g_ranges.end(), a,
                                   [](uintptr_t x, const HostRange &r) { return x < r.h; });
        if (it != g_ranges.begin()) {
            --it;
            if (a >= it->h && a - it->h + len <= it->len) {
                *d = it->d + (a - it->h);
                const uint64_t gen = g_ranges_gen.load(std::memory_order_relaxed);
                if (t_last_gen != gen) {
                    for (HostRange &r : t_last)
                        r = HostRange{0, 0, 0};
                    t_last_gen = gen;
                }
                t_last[t_next++ % kHits] = *it;
                return true;
            }
        }
    }
    void *dp = nullptr;                      // page-locked by HIP itself (hipHostMalloc)
    DeviceGuard g(dev);
    if (g.error() == hipSuccess && hipHostGetDevicePointer(&dp, const_cast<void *>(p), 0) == hipSuccess && dp) {
        *d = reinterpret_cast<uintptr_t>(dp);
        return true;
    }
    (void)hipGetLastError();
    return false;
}

std::atomic<uint64_t> g_round_gen{1};   // round generations, unique across batchers

// Takes up to `want` (at least `need`) units from the shared counter `c` bounded by `cap`; returns
// the first unit and sets *got, or returns UINT64_MAX when fewer than `need` are left.  The unused
// tail [ret, ret_end) of the caller's previous chunk is handed back first when nothing was taken
// after it (always, with one submitting thread), so a lone thread wastes no capacity.
uint64_t take(std::atomic<uint64_t> &c, uint64_t cap, uint64_t need, uint64_t want, uint64_t *got, uint64_t ret = 0,
              uint64_t ret_end = 0)
{
    if (ret < ret_end) {
        uint64_t top = ret_end;
        c.compare_exchange_strong(top, ret, std::memory_order_relaxed);
    }
    uint64_t cur = c.load(std::memory_order_relaxed);
    for (;;) {
        if (cur > cap || cap - cur < need)
            return UINT64_MAX;
        const uint64_t n = std::min(std::max(need, want), cap - cur);
        if (c.compare_exchange_weak(cur, cur + n, std::memory_order_relaxed)) {
            *got = n;
            return cur;
        }
    }
}

// A submitting thread's reserved chunk of one round: slots and arena bytes handed out without
// touching the shared counters (which bounce between cores when several event threads submit).
struct Chunk {
    uint64_t gen = 0;
    uint64_t slot = 0, slot_end = 0, in = 0, in_end = 0, out = 0, out_end = 0;
};
// One entry per round this thread submits into: an all-devices batcher's Read/Write alternate
// between its parts' rounds, and with a single entry every switch abandoned the chunk just taken
// (its slots became holes and a part's round reported full after a few dozen buffers).
constexpr int kChunks = 16;
thread_local Chunk t_chunks[kChunks];
thread_local unsigned t_chunk_next = 0;

Chunk &chunk_for(uint64_t gen)
{
    for (Chunk &c : t_chunks)
        if (c.gen == gen)
            return c;
    Chunk &c = t_chunks[t_chunk_next++ % kChunks];   // oldest entry: its unused slots stay holes
    c = Chunk{gen, 0, 0, 0, 0, 0, 0};
    return c;
}
constexpr uint64_t kChunkSlots = 64, kChunkBytes = 128 << 10;

// One round's arenas and bookkeeping.  A pipelined batcher (BRB_BATCHER_PIPELINED) owns two, so the
// event loop fills one while the GPU runs the other.
struct Round {
    uint8_t *h_in = nullptr, *h_out = nullptr, *h_meta = nullptr;   // pinned
    uint8_t *d_in = nullptr, *d_out = nullptr, *d_meta = nullptr;
    uintptr_t out_dev = 0, meta_dev = 0;   // device addresses of h_out, h_meta
    // Read/Write reserve a slot and arena bytes with atomics, so several event threads may submit
    // into one round at once (their copies run in parallel); a failed reservation leaves a hole.
    std::vector<Item> slots;               // max_items
    std::atomic<uint64_t> n_slots{0}, in_used{0}, out_used{0};
    std::atomic<uint64_t> gen{0};          // new value at every reset: invalidates threads' chunks
    std::vector<Item> items;               // the launched round's buffers, in slot order
    // filled by launch_round, read by deliver_round
    std::vector<int64_t> group_of;         // (sub-round, op) -> group
    std::vector<size_t> group_valid;       // group -> offset of its valid flags in h_meta
    hipEvent_t done = nullptr;
    hipEvent_t ev_h2d = nullptr, ev_kern = nullptr;   // pipelined: inputs landed, kernels finished
    // pair_fault.h: the round's fault word (page-locked, mapped), armed around its kernel launches and
    // read once the round is done; cleared before every launch of the round
    uint32_t *fault = nullptr;
    bool in_flight = false;

    void release()
    {
        (void)hipFree(d_in);
        (void)hipFree(d_out);
        (void)hipFree(d_meta);
        (void)hipHostFree(h_in);
        (void)hipHostFree(h_out);
        (void)hipHostFree(h_meta);
        (void)hipHostFree(fault);
        for (hipEvent_t ev : {done, ev_h2d, ev_kern})
            if (ev)
                (void)hipEventDestroy(ev);
    }
    void reset()
    {
        items.clear();
        n_slots = 0;
        in_used = 0;
        out_used = 0;
        in_flight = false;
        gen = g_round_gen.fetch_add(1, std::memory_order_relaxed);
    }
    bool empty() const { return n_slots.load(std::memory_order_relaxed) == 0; }
};

constexpr uint32_t kHole = 0xFFFFFFFFu;   // Item::conn of a slot whose reservation failed

}  // namespace

struct BRB_TransformBatcher {
    uint32_t max_conns = 0;
    uint64_t cap = 0;          // input bytes per round
    int algo = 0;
    bool zc = false;           // zero-copy rounds
    int n_rounds = 1;          // 2 when pipelined
    int cur = 0;               // the round Read/Write fill
    int dev = 0;
    // test support (BRB_TransformBatcherInjectFault): the k-th kernel launch of every round is
    // reported as failed without running, so the tests can check that a failed round is dropped
    // exactly once (the groups launched before it ran; nothing runs twice)
    int fault_launch = -1;
    hipStream_t stream = nullptr;          // kernels (and Enable/GetState), in round order
    // Pipelined: round k+1's H2D and round k's D2H run on their own streams, so the two copy
    // directions overlap each other and the kernels.  One-round batchers use `stream` for all.
    hipStream_t s_h2d = nullptr, s_d2h = nullptr;
    uint8_t *d_states = nullptr;           // [2][max_conns] x 264 B: read states, then write states
    size_t out_cap = 0, meta_cap = 0;
    uint64_t max_items = 0;    // buffers per round: 4 per connection on average
    Round r[2];
    std::vector<uint8_t> enabled;
    // Key epochs: Enable starts a connection's next epoch; a round dropped for a device
    // fault leaves the states of its connections out of step, so their epoch is poisoned
    // (poison_upto[c] = the last poisoned epoch).  A buffer of a poisoned epoch is never delivered as
    // data: one already launched behind the faulted round (pipelined FlushAsync) comes back
    // BRB_TRANSFORM_DROPPED, one still waiting in the filling round is dropped without running, and
    // Read/Write refuse the connection until Enable re-keys it.  Atomics: submitting threads read
    // them while a Flush on another thread poisons.
    std::vector<uint32_t> epoch, poison_upto;
    // BRB_BATCHER_ALL_DEVICES: the connections are partitioned over G sub-batchers, connection c
    // in sub c % G as its connection c / G, sub g on device g % (visible devices); this object then
    // only routes (no collective -- a connection's states live on its device).
    std::vector<BRB_TransformBatcher *> subs;

    ~BRB_TransformBatcher()
    {
        for (BRB_TransformBatcher *sb : subs)
            delete sb;
        if (!subs.empty())
            return;
        DeviceGuard g(dev);
        for (hipStream_t q : {s_h2d, s_d2h, stream})
            if (q)
                (void)hipStreamSynchronize(q);
        (void)hipFree(d_states);
        for (Round &x : r)
            x.release();
        for (hipStream_t q : {s_h2d, s_d2h, stream})
            if (q)
                (void)hipStreamDestroy(q);
    }

    uint8_t *state(uint32_t conn, int op) { return d_states + (size_t(op) * max_conns + conn) * sizeof(BRB_RC4_State); }

    hipError_t alloc_round(Round &x)
    {
        hipError_t e;
        void *od = nullptr, *md = nullptr, *fw = nullptr;
        if ((e = hipMalloc(&x.d_in, up(cap, kAlign))) != hipSuccess || (e = hipMalloc(&x.d_out, out_cap)) != hipSuccess ||
            (e = hipMalloc(&x.d_meta, meta_cap)) != hipSuccess ||
            (e = hipHostMalloc(&x.h_in, up(cap, kAlign), hipHostMallocDefault)) != hipSuccess ||
            (e = hipHostMalloc(&x.h_out, out_cap, hipHostMallocDefault)) != hipSuccess ||
            (e = hipHostMalloc(&x.h_meta, meta_cap, hipHostMallocDefault)) != hipSuccess ||
            (e = hipHostGetDevicePointer(&od, x.h_out, 0)) != hipSuccess ||
            (e = hipHostGetDevicePointer(&md, x.h_meta, 0)) != hipSuccess ||
            (e = hipHostMalloc(&fw, 64, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&x.done, hipEventDisableTiming)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&x.ev_h2d, hipEventDisableTiming)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&x.ev_kern, hipEventDisableTiming)) != hipSuccess)
            return e;
        x.fault = static_cast<uint32_t *>(fw);
        __atomic_store_n(x.fault, 0u, __ATOMIC_RELAXED);
        x.out_dev = reinterpret_cast<uintptr_t>(od);
        x.meta_dev = reinterpret_cast<uintptr_t>(md);
        x.slots.resize(max_items);
        x.gen = g_round_gen.fetch_add(1, std::memory_order_relaxed);
        return hipSuccess;
    }
};

extern "C" {

BRB_TransformBatcher *BRB_TransformBatcherCreate(uint32_t max_conns, uint64_t max_round_bytes, int algo)
{
    brb_api::clear_err();
    if (algo & BRB_BATCHER_ALL_DEVICES) {
        algo &= ~BRB_BATCHER_ALL_DEVICES;
        if (brb_api::device_ok() != BRB_BATCH_OK)
            return nullptr;
        // at most kChunks parts: a thread keeps one chunk entry per part's round (with
        // more parts than entries every round-robin submit evicted a live chunk)
        const int G = std::min(brb_host::split_parts(), kChunks);
        if (G > 1 && max_conns >= uint32_t(G)) {
            auto *m = new BRB_TransformBatcher;
            m->max_conns = max_conns;
            m->algo = algo;
            for (int g = 0; g < G; g++) {
                DeviceGuard dg(brb_host::part_device(g));
                BRB_TransformBatcher *sb = dg.error() == hipSuccess
                                               ? BRB_TransformBatcherCreate((max_conns - uint32_t(g) + uint32_t(G) - 1) / uint32_t(G),
                                                                            max_round_bytes, algo)
                                               : nullptr;
                if (!sb) {
                    if (dg.error() != hipSuccess)
                        fail_hip("hipSetDevice", dg.error());
                    const std::string why = brb_api::t_err;
                    delete m;
                    set_err("all-devices batcher, part %d: %s", g, why.c_str());
                    return nullptr;
                }
                m->subs.push_back(sb);
            }
            return m;
        }
    }
    const bool zc = (algo & BRB_BATCHER_ZERO_COPY) != 0;
    const bool pipelined = (algo & BRB_BATCHER_PIPELINED) != 0;
    algo &= ~(BRB_BATCHER_ZERO_COPY | BRB_BATCHER_PIPELINED);
    if (max_conns == 0 || max_round_bytes == 0 || (algo != BRB_CRYPTO_FUNC_RC4 && algo != BRB_CRYPTO_FUNC_RC4_MD5)) {
        set_err("max_conns and max_round_bytes must be > 0 and algo RC4 (1) or RC4_MD5 (2)");
        return nullptr;
    }
    if (uint64_t(max_conns) * 4 > (uint64_t(1) << 32) - (uint64_t(1) << 16)) {
        set_err("max_conns %u: a round holds up to 4 buffers per connection, at most 2^32 - 2^16", max_conns);
        return nullptr;
    }
    if (brb_api::device_ok() != BRB_BATCH_OK)
        return nullptr;
    auto *b = new BRB_TransformBatcher;
    b->max_conns = max_conns;
    b->cap = max_round_bytes;
    b->algo = algo;
    b->zc = zc;
    b->n_rounds = pipelined ? 2 : 1;
    b->enabled.assign(max_conns, 0);
    b->epoch.assign(max_conns, 0);
    b->poison_upto.assign(max_conns, 0);
    // outputs: every buffer may grow by a frame header; metadata: per item and sub-round arrays
    b->max_items = 4 * uint64_t(max_conns);
    b->out_cap = up(max_round_bytes + kHdr * b->max_items, kAlign);
    b->meta_cap = up(kMetaItem * b->max_items + 4096, kAlign);
    hipError_t e;
    if ((e = hipGetDevice(&b->dev)) != hipSuccess || (e = hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipMalloc(&b->d_states, size_t(2) * max_conns * sizeof(BRB_RC4_State))) != hipSuccess ||
        // On the batcher's own stream and drained here.  A plain hipMemset runs on the legacy default
        // stream, which the non-blocking `stream` does not wait for: behind other work on the default
        // stream it could land after Enable's state copies and a round's kernels, zeroing live states
        // (the all-zero state of tests/test_batcher.py::test_states_survive_busy_default_stream).
        (e = hipMemsetAsync(b->d_states, 0, size_t(2) * max_conns * sizeof(BRB_RC4_State), b->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(b->stream)) != hipSuccess) {
        fail_hip("transform batcher allocation", e);
        delete b;
        return nullptr;
    }
    if (pipelined && ((e = hipStreamCreateWithFlags(&b->s_h2d, hipStreamNonBlocking)) != hipSuccess ||
                      (e = hipStreamCreateWithFlags(&b->s_d2h, hipStreamNonBlocking)) != hipSuccess)) {
        fail_hip("transform batcher copy streams", e);
        delete b;
        return nullptr;
    }
    for (int i = 0; i < b->n_rounds; i++)
        if ((e = b->alloc_round(b->r[i])) != hipSuccess) {
            fail_hip("transform batcher round allocation", e);
            delete b;
            return nullptr;
        }
    return b;
}

void BRB_TransformBatcherDestroy(BRB_TransformBatcher *b)
{
    delete b;
}

int BRB_TransformBatcherEnable(BRB_TransformBatcher *b, uint32_t conn, const void *key, int key_sz)
{
    brb_api::clear_err();
    if (!b || !key || key_sz <= 0 || conn >= b->max_conns) {
        set_err("bad batcher, key or connection id");
        return BRB_BATCH_BADARG;
    }
    if (!b->subs.empty())
        return BRB_TransformBatcherEnable(b->subs[conn % b->subs.size()], conn / uint32_t(b->subs.size()), key, key_sz);
    BRB_RC4_State st;
    memset(&st, 0, sizeof(st));              // ev_kq_aio_transform.c:78 memset of the crypto states
    BRB_RC4_Init(&st, static_cast<const unsigned char *>(key), key_sz);
    DeviceGuard g(b->dev);
    hipError_t e;
    if ((e = g.error()) != hipSuccess)
        return fail_hip("hipSetDevice", e);
    for (int op = 0; op < 2; op++)
        if ((e = hipMemcpyAsync(b->state(conn, op), &st, sizeof(st), hipMemcpyHostToDevice, b->stream)) != hipSuccess)
            return fail_hip("hipMemcpyAsync H2D", e);
    if ((e = hipStreamSynchronize(b->stream)) != hipSuccess)
        return fail_hip("hipStreamSynchronize", e);
    b->enabled[conn] = 1;
    __atomic_fetch_add(&b->epoch[conn], 1u, __ATOMIC_RELEASE);   // buffers from here on: the fresh key
    return BRB_BATCH_OK;
}

static int submit(BRB_TransformBatcher *b, uint32_t conn, int op, const void *data, uint32_t len, uint64_t salt)
{
    brb_api::clear_err();
    if (b && !b->subs.empty() && conn < b->max_conns)
        return submit(b->subs[conn % b->subs.size()], conn / uint32_t(b->subs.size()), op, data, len, salt);
    if (!b || (!data && len) || conn >= b->max_conns || !b->enabled[conn]) {
        set_err("bad batcher, data or connection (not enabled?)");
        return BRB_BATCH_BADARG;
    }
    const uint32_t ep = __atomic_load_n(&b->epoch[conn], __ATOMIC_ACQUIRE);
    if (ep <= __atomic_load_n(&b->poison_upto[conn], __ATOMIC_ACQUIRE)) {
        set_err("connection %u: its RC4 states are out of step after a round dropped for a device fault; re-key it "
                "with Enable", conn);
        return BRB_BATCH_BADARG;
    }
    Round &R = b->r[b->cur];
    const uint32_t out_len = len + (b->algo == BRB_CRYPTO_FUNC_RC4_MD5 && op == BRB_CRYPTO_OP_WRITE ? kHdr : 0);
    // Slot order is delivery order.  A thread's slots and bytes come from its own chunks, taken in
    // increasing order, so the buffers of a connection (owned by one thread) keep their order.
    // Slots of a chunk left unused stay holes; the metadata arrays fit max_items slots.
    const uint64_t gen = R.gen.load(std::memory_order_relaxed);
    Chunk &k = chunk_for(gen);
    uint64_t got;
    if (k.slot == k.slot_end) {
        const uint64_t s0 = take(R.n_slots, b->max_items, 1, kChunkSlots, &got);
        if (s0 == UINT64_MAX) {
            set_err("round is full: flush first");
            return BRB_BATCH_NOT_DONE;
        }
        for (uint64_t i = s0; i < s0 + got; i++)
            R.slots[i].conn = kHole;
        k.slot = s0;
        k.slot_end = s0 + got;
    }
    if (k.in_end - k.in < len) {
        const uint64_t i0 = take(R.in_used, b->cap, len, kChunkBytes, &got, k.in, k.in_end);
        if (i0 == UINT64_MAX) {
            k.in = k.in_end = 0;   // the tail may have been handed back: never reuse it
            set_err("round is full: flush first");
            return BRB_BATCH_NOT_DONE;
        }
        k.in = i0;
        k.in_end = i0 + got;
    }
    if (k.out_end - k.out < out_len) {
        const uint64_t o0 = take(R.out_used, b->out_cap, out_len, kChunkBytes, &got, k.out, k.out_end);
        if (o0 == UINT64_MAX) {
            k.out = k.out_end = 0;
            set_err("round is full: flush first");
            return BRB_BATCH_NOT_DONE;
        }
        k.out = o0;
        k.out_end = o0 + got;
    }
    Item &it = R.slots[k.slot];
    const uint64_t in_off = k.in, out_off = k.out;
    it = Item{conn, op, in_off, len, out_off, out_len, salt, 0, ep};
    if (b->zc) {
        uintptr_t d = 0;
        if (len && !host_to_device(data, len, &d, b->dev)) {
            it.conn = kHole;   // this thread's next buffer takes the slot and the bytes
            set_err("zero-copy batcher: buffer is not in page-locked memory (BRB_CryptoGPU_HostRegister)");
            return BRB_BATCH_BADARG;
        }
        it.in_off = d;
    } else if (len) {
        memcpy(R.h_in + in_off, data, len);
    }
    k.slot++;
    k.in += len;
    k.out += out_len;
    return BRB_BATCH_OK;
}

int BRB_TransformBatcherRead(BRB_TransformBatcher *b, uint32_t conn, const void *data, uint32_t len)
{
    return submit(b, conn, BRB_CRYPTO_OP_READ, data, len, 0);
}

int BRB_TransformBatcherWrite(BRB_TransformBatcher *b, uint32_t conn, const void *data, uint32_t len, uint64_t salt)
{
    return submit(b, conn, BRB_CRYPTO_OP_WRITE, data, len, salt);
}

}  // extern "C"

// A buffer of a poisoned key epoch (its connection's states went out of step in a dropped round).
static bool poisoned(const BRB_TransformBatcher *b, const Item &it)
{
    return it.epoch <= __atomic_load_n(&b->poison_upto[it.conn], __ATOMIC_ACQUIRE);
}

// A round dropped for a device fault: every connection it holds is poisoned up to the epoch its
// buffers were submitted under (a later Enable has already started a fresh one).
static void poison_round(BRB_TransformBatcher *b, const Round &R)
{
    for (const Item &it : R.items)
        if (__atomic_load_n(&b->poison_upto[it.conn], __ATOMIC_RELAXED) < it.epoch)
            __atomic_store_n(&b->poison_upto[it.conn], it.epoch, __ATOMIC_RELEASE);
}

// The round's buffers in slot order, holes dropped.  Called once no Read/Write is running on R.
// Buffers of poisoned epochs (submitted before a fault was found) go to *stale instead: they must
// not run, since they would advance the states an Enable re-keys.
static size_t collect(BRB_TransformBatcher *b, Round &R, std::vector<Item> *stale)
{
    const uint64_t n = std::min<uint64_t>(R.n_slots, b->max_items);
    R.items.clear();
    stale->clear();
    for (uint64_t i = 0; i < n; i++)
        if (R.slots[i].conn != kHole)
            (poisoned(b, R.slots[i]) ? *stale : R.items).push_back(R.slots[i]);
    return R.items.size();
}

// Enqueues round R on the batcher's stream: metadata, H2D, the kernels, D2H, then R.done.  Nothing
// waits here; the stream keeps rounds (and so every connection's RC4 stream) in order.  *started is
// set once the first copy has been enqueued.
static int enqueue_round(BRB_TransformBatcher *b, Round &R, bool *started)
{
    hipError_t e;
    // arena bytes past the last successful reservation belong to failed ones: not copied
    const uint64_t in_used = std::min<uint64_t>(R.in_used, b->cap), out_used = std::min<uint64_t>(R.out_used, b->out_cap);
    // sub-round of every item: its rank among the same connection's items in the same direction
    std::vector<uint32_t> seen(size_t(2) * b->max_conns, 0);
    uint32_t rounds = 0;
    for (Item &it : R.items) {
        it.round = seen[size_t(it.op) * b->max_conns + it.conn]++;
        rounds = std::max(rounds, it.round + 1);
    }
    // metadata: per (sub-round, op) a contiguous group: sidx u32[], offs u64[], lens u32[], ooffs u64[], salts u64[]
    struct Group {
        int op;
        uint32_t count;
        size_t o_sidx, o_offs, o_lens, o_ooffs, o_salts;
    };
    std::vector<Group> groups;
    R.group_of.assign(size_t(rounds) * 2, -1);
    size_t m = 0;
    for (uint32_t r = 0; r < rounds; r++)
        for (int op = 0; op < 2; op++) {
            uint32_t c = 0;
            for (const Item &it : R.items)
                c += it.round == r && it.op == op;
            if (!c)
                continue;
            Group g{op, c, 0, 0, 0, 0, 0};
            g.o_sidx = m;
            m = up(m + 4 * size_t(c), 8);
            g.o_offs = m;
            m = up(m + 8 * size_t(c), 8);
            g.o_lens = m;
            m = up(m + 4 * size_t(c), 8);
            g.o_ooffs = m;
            m = up(m + 8 * size_t(c), 8);
            g.o_salts = m;
            m = up(m + 8 * size_t(c), 8);
            if (m > b->meta_cap) {
                set_err("metadata overflow");
                return BRB_BATCH_NOT_DONE;
            }
            uint32_t k = 0;
            for (const Item &it : R.items) {
                if (it.round != r || it.op != op)
                    continue;
                reinterpret_cast<uint32_t *>(R.h_meta + g.o_sidx)[k] = uint32_t(op) * b->max_conns + it.conn;
                // zero-copy: kernels address input buffers as out_dev + (device address - out_dev)
                reinterpret_cast<uint64_t *>(R.h_meta + g.o_offs)[k] = b->zc ? it.in_off - uint64_t(R.out_dev) : it.in_off;
                reinterpret_cast<uint32_t *>(R.h_meta + g.o_lens)[k] = it.in_len;
                reinterpret_cast<uint64_t *>(R.h_meta + g.o_ooffs)[k] = it.out_off;
                reinterpret_cast<uint64_t *>(R.h_meta + g.o_salts)[k] = it.salt;
                ++k;
            }
            R.group_of[size_t(r) * 2 + op] = int64_t(groups.size());
            groups.push_back(g);
        }
    // valid flags: one byte per item of each read group, after the metadata
    const size_t o_valid = m;
    if (o_valid + R.items.size() > b->meta_cap) {
        set_err("metadata overflow");
        return BRB_BATCH_NOT_DONE;
    }
    hipStream_t s = b->stream;
    const bool split = b->s_h2d != nullptr;
    // the arena's previous round was delivered (its done event waited on) before it was refilled
    hipStream_t sh = split ? b->s_h2d : s;
    *started = true;
    if ((!b->zc && (e = hipMemcpyAsync(R.d_in, R.h_in, in_used, hipMemcpyHostToDevice, sh)) != hipSuccess) ||
        (e = hipMemcpyAsync(R.d_meta, R.h_meta, m, hipMemcpyHostToDevice, sh)) != hipSuccess)
        return fail_hip("hipMemcpyAsync H2D", e);
    if (split && ((e = hipEventRecord(R.ev_h2d, sh)) != hipSuccess || (e = hipStreamWaitEvent(s, R.ev_h2d, 0)) != hipSuccess))
        return fail_hip("H2D event", e);
    // the round's pair kernels report a protocol fault into R.fault (pair_fault.h); the word's last
    // reader was this round's previous delivery, so no kernel still writes it
    __atomic_store_n(R.fault, 0u, __ATOMIC_RELAXED);
    struct Arm {
        uint32_t *prev;
        explicit Arm(uint32_t *w) : prev(brb::pair_fault_arm(w)) {}
        ~Arm() { brb::pair_fault_arm(prev); }
    } arm(R.fault);
    uint8_t *zbase = reinterpret_cast<uint8_t *>(R.out_dev);   // zero-copy: inputs and outputs
    uint8_t *zvalid = reinterpret_cast<uint8_t *>(R.meta_dev);
    size_t vpos = o_valid;
    R.group_valid.assign(groups.size(), 0);
    for (size_t gi = 0; gi < groups.size(); gi++) {
        const Group &g = groups[gi];
        const uint32_t *sidx = reinterpret_cast<const uint32_t *>(R.d_meta + g.o_sidx);
        const uint64_t *offs = reinterpret_cast<const uint64_t *>(R.d_meta + g.o_offs);
        const uint32_t *lens = reinterpret_cast<const uint32_t *>(R.d_meta + g.o_lens);
        const uint64_t *ooffs = reinterpret_cast<const uint64_t *>(R.d_meta + g.o_ooffs);
        const uint64_t *salts = reinterpret_cast<const uint64_t *>(R.d_meta + g.o_salts);
        if (int64_t(gi) == b->fault_launch)
            return fail_hip("kernel launch (injected fault)", hipErrorLaunchFailure);
        if (b->zc) {
            // inputs read in place over PCIe, outputs written into the page-locked output arena
            if (b->algo == BRB_CRYPTO_FUNC_RC4) {
                e = brb::launch_rc4_crypt(b->d_states, zbase, zbase, offs, lens, g.count, s, sidx, ooffs, true);
            } else if (g.op == BRB_CRYPTO_OP_WRITE) {
                e = brb::launch_rc4md5_frame(b->d_states, zbase, offs, lens, salts, zbase, ooffs, g.count, s, sidx);
            } else {
                R.group_valid[gi] = vpos;
                e = brb::launch_rc4md5_open(b->d_states, zbase, zbase, offs, lens, g.count, zvalid + vpos, s, sidx, ooffs);
                vpos += g.count;
            }
        } else if (b->algo == BRB_CRYPTO_FUNC_RC4) {
            // the output arena mirrors the input arena for RC4 (same offsets, same lengths)
            e = brb::launch_rc4_crypt(b->d_states, R.d_in, R.d_out, offs, lens, g.count, s, sidx);
        } else if (g.op == BRB_CRYPTO_OP_WRITE) {
            e = brb::launch_rc4md5_frame(b->d_states, R.d_in, offs, lens, salts, R.d_out, ooffs, g.count, s, sidx);
        } else {
            // decrypt in place in the input arena, then the frames are copied out with it
            R.group_valid[gi] = vpos;
            e = brb::launch_rc4md5_open(b->d_states, R.d_in, R.d_in, offs, lens, g.count, R.d_meta + vpos, s, sidx);
            vpos += g.count;
        }
        if (e != hipSuccess)
            return fail_hip("kernel launch", e);
    }
    hipStream_t sd = split ? b->s_d2h : s;
    if (split && ((e = hipEventRecord(R.ev_kern, s)) != hipSuccess || (e = hipStreamWaitEvent(sd, R.ev_kern, 0)) != hipSuccess))
        return fail_hip("kernel event", e);
    if (!b->zc && ((e = hipMemcpyAsync(R.h_out, R.d_out, out_used, hipMemcpyDeviceToHost, sd)) != hipSuccess ||
                   (b->algo == BRB_CRYPTO_FUNC_RC4_MD5 &&
                    (e = hipMemcpyAsync(R.h_in, R.d_in, in_used, hipMemcpyDeviceToHost, sd)) != hipSuccess) ||
                   (vpos > o_valid && (e = hipMemcpyAsync(R.h_meta + o_valid, R.d_meta + o_valid, vpos - o_valid,
                                                          hipMemcpyDeviceToHost, sd)) != hipSuccess)))
        return fail_hip("round D2H", e);
    if ((e = hipEventRecord(R.done, sd)) != hipSuccess)
        return fail_hip("hipEventRecord", e);
    R.in_flight = true;
    return BRB_BATCH_OK;
}

// A dropped round: every buffer's callback fires with valid = BRB_TRANSFORM_DROPPED (no output), in
// submission order, so an event loop learns which buffers were lost without parsing LastError.
static void drop_round(Round &R, BRB_TransformDone done, void *user)
{
    if (done)
        for (const Item &it : R.items)
            done(user, it.conn, it.op, nullptr, 0, BRB_TRANSFORM_DROPPED);
    R.reset();
}

// enqueue_round, and on failure drop the round: it is never retried, because the groups enqueued
// before the failure may already have advanced their connections' RC4 states and running them again
// would advance those states twice.  The streams are drained first, so no copy still reads an arena
// that the next round refills.  Returns BRB_BATCH_OK, or BRB_BATCH_DROPPED after the dropped
// buffers' callbacks (reason in LastError).
static int launch_round(BRB_TransformBatcher *b, Round &R, BRB_TransformDone done, void *user)
{
    bool started = false;
    if (enqueue_round(b, R, &started) == BRB_BATCH_OK)
        return BRB_BATCH_OK;
    if (started)
        for (hipStream_t q : {b->s_h2d, b->s_d2h, b->stream})
            if (q)
                (void)hipStreamSynchronize(q);
    const std::string why = brb_api::t_err;
    set_err("%s; round of %zu buffers dropped%s", why.c_str(), R.items.size(),
            started ? " (groups launched before the failure have advanced their connections' states)" : "");
    drop_round(R, done, user);
    return BRB_BATCH_DROPPED;
}

// Waits for round R and hands every result back in submission order; the k-th read item of a
// group has valid flag k of that group.  Returns the number of buffers delivered, or -1 when the
// round failed on the device (dropped: drop_round's callbacks, its connections poisoned; reason in
// LastError).  Buffers of connections poisoned after R was launched come back
// BRB_TRANSFORM_DROPPED and are counted in *n_stale.
static int64_t deliver_round(BRB_TransformBatcher *b, Round &R, BRB_TransformDone done, void *user, int64_t *n_stale)
{
    hipError_t e;
    *n_stale = 0;
    if ((e = hipEventSynchronize(R.done)) != hipSuccess) {
        fail_hip("round completion", e);
        const std::string why = brb_api::t_err;
        set_err("%s; round of %zu buffers dropped (its connections' states are out of step: re-key them with Enable)",
                why.c_str(), R.items.size());
        poison_round(b, R);
        drop_round(R, done, user);
        return -1;
    }
    if (__atomic_load_n(R.fault, __ATOMIC_ACQUIRE) != 0) {
        // a pair kernel's bounded wait gave up: its outputs, valid flags and the RC4 states it
        // advanced are wrong, so nothing of the round is delivered as data (the reference's only
        // integrity check, ev_kq_aio_transform.c:157-184, must never pass over wrong bytes)
        set_err("wave-pair protocol fault: a kernel of the round gave up waiting on its partner wave; round of %zu "
                "buffers dropped (its connections' states are out of step: re-key them with Enable)",
                R.items.size());
        poison_round(b, R);
        drop_round(R, done, user);
        return -1;
    }
    std::vector<uint32_t> next_in_group(R.group_valid.size(), 0);
    int64_t delivered = 0;
    for (const Item &it : R.items) {
        const int64_t gi = R.group_of[size_t(it.round) * 2 + it.op];
        const uint32_t k = next_in_group[gi]++;
        if (poisoned(b, it)) {          // ran on states a faulted round before it left out of step
            ++*n_stale;
            if (done)
                done(user, it.conn, it.op, nullptr, 0, BRB_TRANSFORM_DROPPED);
            continue;
        }
        ++delivered;
        int valid = 1;
        const uint8_t *out;
        if (b->zc) {
            out = R.h_out + it.out_off;
            if (b->algo == BRB_CRYPTO_FUNC_RC4_MD5 && it.op == BRB_CRYPTO_OP_READ)
                valid = R.h_meta[R.group_valid[gi] + k];
        } else if (b->algo == BRB_CRYPTO_FUNC_RC4) {
            out = R.h_out + it.in_off;
        } else if (it.op == BRB_CRYPTO_OP_WRITE) {
            out = R.h_out + it.out_off;
        } else {
            out = R.h_in + it.in_off;
            valid = R.h_meta[R.group_valid[gi] + k];
        }
        if (done)
            done(user, it.conn, it.op, out, it.out_len, valid);
    }
    if (*n_stale)
        set_err("%lld buffers of connections whose states a faulted round left out of step were dropped (re-key "
                "them with Enable)", (long long)*n_stale);
    R.reset();
    return delivered;
}

// ---- Flush / FlushAsync in phases, so that an all-devices batcher can enqueue every device's
// round before it waits for any of them (the devices run concurrently; the callbacks still come on
// the calling thread, device by device, each device's buffers in submission order).
//   Flush:      deliver the round FlushAsync left running (pipelined) | launch the current round |
//               deliver it
//   FlushAsync: launch the current round and switch arenas | deliver the previous round
struct Phase {
    BRB_TransformBatcher *b;
    BRB_TransformDone done;
    void *user;
    Round *prev = nullptr;     // FlushAsync: the round to deliver after the launches
    int64_t n = 0;             // buffers delivered
    std::vector<Item> stale;   // the launched round's buffers of poisoned epochs (phase_stale)
    bool dropped = false;
    bool failed = false;       // hipSetDevice failed: the round stays pending
};

// the batcher's connection ids -> the caller's (all-devices: sub g's connection c is c * G + g)
struct Tramp {
    BRB_TransformDone done;
    void *user;
    uint32_t G, g;
    static void call(void *u, uint32_t conn, int op, const void *out, uint32_t len, int valid)
    {
        const Tramp *t = static_cast<const Tramp *>(u);
        t->done(t->user, conn * t->G + t->g, op, out, len, valid);
    }
};

static void phase_deliver(Phase &p, Round &R)
{
    if (!R.in_flight)
        return;
    DeviceGuard g(p.b->dev);
    if (g.error() != hipSuccess) {      // the round stays in flight: a later Flush delivers it
        fail_hip("hipSetDevice", g.error());
        p.failed = true;
        return;
    }
    int64_t stale = 0;
    const int64_t n = deliver_round(p.b, R, p.done, p.user, &stale);
    if (n < 0 || stale)
        p.dropped = true;
    if (n > 0)
        p.n += n;
}

static void phase_launch(Phase &p, bool async)
{
    BRB_TransformBatcher *b = p.b;
    DeviceGuard g(b->dev);
    if (g.error() != hipSuccess) {
        fail_hip("hipSetDevice", g.error());
        p.failed = true;
        return;
    }
    Round &R = b->r[b->cur];
    p.prev = async && b->n_rounds == 2 ? &b->r[b->cur ^ 1] : nullptr;
    const size_t n = collect(b, R, &p.stale);
    if (n == 0)
        R.reset();
    else if (launch_round(b, R, p.done, p.user) != BRB_BATCH_OK)   // dropped: its callbacks have fired
        p.dropped = true;
    if (async && b->n_rounds == 2 && R.in_flight)
        b->cur ^= 1;        // Read/Write now fill the other arena (the previous round's, once delivered)
}

// The buffers phase_launch left out (submitted under a poisoned epoch, never run): their callbacks
// fire after the round before theirs was delivered and before their own round's results, so every
// connection still sees its buffers in submission order.
static void phase_stale(Phase &p)
{
    if (p.stale.empty())
        return;
    if (p.done)
        for (const Item &it : p.stale)
            p.done(p.user, it.conn, it.op, nullptr, 0, BRB_TRANSFORM_DROPPED);
    set_err("%zu buffers of connections whose states a faulted round left out of step were dropped without running "
            "(re-key them with Enable)", p.stale.size());
    p.dropped = true;
    p.stale.clear();
}

static int64_t flush_all(BRB_TransformBatcher *b, BRB_TransformDone done, void *user, bool async)
{
    std::vector<BRB_TransformBatcher *> parts = b->subs;
    if (parts.empty())
        parts.push_back(b);
    const uint32_t G = uint32_t(parts.size());
    std::vector<Tramp> tr(G);
    std::vector<Phase> ph;
    for (uint32_t g = 0; g < G; g++) {
        tr[g] = Tramp{done, user, G, g};
        ph.push_back(Phase{parts[g], done ? (b->subs.empty() ? done : &Tramp::call) : nullptr,
                           b->subs.empty() ? user : static_cast<void *>(&tr[g])});
    }
    const bool pipelined = parts[0]->n_rounds == 2;
    if (!async || !pipelined) {
        if (pipelined)
            for (Phase &p : ph)   // the rounds FlushAsync left running come first
                phase_deliver(p, p.b->r[p.b->cur ^ 1]);
        for (Phase &p : ph)
            phase_launch(p, false);
        for (Phase &p : ph) {
            phase_stale(p);
            phase_deliver(p, p.b->r[p.b->cur]);
        }
    } else {
        for (Phase &p : ph)
            phase_launch(p, true);
        for (Phase &p : ph) {
            if (p.prev)
                phase_deliver(p, *p.prev);
            phase_stale(p);
        }
    }
    int64_t total = 0;
    bool dropped = false;
    uint32_t failed = 0;
    for (const Phase &p : ph) {
        total += p.n;
        dropped |= p.dropped;
        failed += p.failed ? 1u : 0u;
    }
    if (failed) {
        // parts that could not select their device keep their rounds pending, while the
        // other parts' buffers were delivered (callbacks fired, states advanced): say so instead of
        // returning "not done" for the whole call.  ADVICE r04: a round of another part dropped in the
        // same call is reported with it, not instead of it -- DROPPED tells the caller that nothing is
        // pending, and the pending parts' rounds still read their zero-copy inputs in place.
        const std::string why = brb_api::t_err;
        set_err("%u of %u parts could not select their device (%s); their rounds stay pending, %lld buffers of "
                "the other parts were delivered%s; Flush again",
                failed, G, why.c_str(), (long long)total,
                dropped ? " and a round of another part was dropped (its buffers came back as BRB_TRANSFORM_DROPPED)"
                        : "");
        return total || dropped ? BRB_BATCH_PARTIAL : BRB_BATCH_NOT_DONE;
    }
    if (dropped)
        return BRB_BATCH_DROPPED;
    return total;
}

extern "C" {

int64_t BRB_TransformBatcherFlush(BRB_TransformBatcher *b, BRB_TransformDone done, void *user)
{
    brb_api::clear_err();
    if (!b) {
        set_err("NULL batcher");
        return BRB_BATCH_BADARG;
    }
    return flush_all(b, done, user, false);
}

int64_t BRB_TransformBatcherFlushAsync(BRB_TransformBatcher *b, BRB_TransformDone done, void *user)
{
    brb_api::clear_err();
    if (!b) {
        set_err("NULL batcher");
        return BRB_BATCH_BADARG;
    }
    return flush_all(b, done, user, true);
}

int BRB_TransformBatcherInjectFault(BRB_TransformBatcher *b, int launch)
{
    brb_api::clear_err();
    if (!b) {
        set_err("NULL batcher");
        return BRB_BATCH_BADARG;
    }
    b->fault_launch = launch;
    for (BRB_TransformBatcher *sb : b->subs)
        sb->fault_launch = launch;
    return BRB_BATCH_OK;
}

}  // extern "C"

extern "C" {

int BRB_CryptoGPU_HostRegister(void *p, uint64_t len)
{
    brb_api::clear_err();
    if (!p || !len) {
        set_err("NULL or empty host range");
        return BRB_BATCH_BADARG;
    }
    if (int ok = brb_api::device_ok(); ok != BRB_BATCH_OK)
        return ok;
    hipError_t e = hipHostRegister(p, len, hipHostRegisterMapped | hipHostRegisterPortable);   // every device
    if (e != hipSuccess)
        return fail_hip("hipHostRegister", e);
    void *dp = nullptr;
    if ((e = hipHostGetDevicePointer(&dp, p, 0)) != hipSuccess) {
        (void)hipHostUnregister(p);
        return fail_hip("hipHostGetDevicePointer", e);
    }
    std::lock_guard<std::mutex> lk(g_ranges_mu);
    const HostRange r{reinterpret_cast<uintptr_t>(p), len, reinterpret_cast<uintptr_t>(dp)};
    g_ranges.insert(std::upper_bound(g_ranges.begin(), g_ranges.end(), r.h,
                                     [](uintptr_t x, const HostRange &q) { return x < q.h; }),
                    r);
    return BRB_BATCH_OK;
}

int BRB_CryptoGPU_HostUnregister(void *p)
{
    brb_api::clear_err();
    std::lock_guard<std::mutex> lk(g_ranges_mu);
    for (auto it = g_ranges.begin(); it != g_ranges.end(); ++it)
        if (it->h == reinterpret_cast<uintptr_t>(p)) {
            g_ranges.erase(it);
            g_ranges_gen.fetch_add(1, std::memory_order_acq_rel);
            hipError_t e = hipHostUnregister(p);
            return e == hipSuccess ? BRB_BATCH_OK : fail_hip("hipHostUnregister", e);
        }
    set_err("host range was not registered");
    return BRB_BATCH_BADARG;
}

int BRB_TransformBatcherGetState(BRB_TransformBatcher *b, uint32_t conn, int op, BRB_RC4_State *out)
{
    brb_api::clear_err();
    if (!b || !out || conn >= b->max_conns || (op != BRB_CRYPTO_OP_READ && op != BRB_CRYPTO_OP_WRITE)) {
        set_err("bad batcher, connection or op");
        return BRB_BATCH_BADARG;
    }
    if (!b->subs.empty())
        return BRB_TransformBatcherGetState(b->subs[conn % b->subs.size()], conn / uint32_t(b->subs.size()), op, out);
    DeviceGuard g(b->dev);
    hipError_t e;
    if ((e = g.error()) != hipSuccess ||
        (e = hipMemcpyAsync(out, b->state(conn, op), sizeof(*out), hipMemcpyDeviceToHost, b->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(b->stream)) != hipSuccess)
        return fail_hip("state copy", e);
    return BRB_BATCH_OK;
}

}  // extern "C"
