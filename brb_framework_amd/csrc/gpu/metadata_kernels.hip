// metadata_kernels.hip -- batched MetaDataUnpack (libbrb_core/data/utils/meta_data.c:145-328) over
// many MetaData packs (the mmap'd file cache and encrypted K/V files keep their
// objects as packs whose MD5 covers the items' data).
//
// One lane per pack.  A pack is one sequential byte stream -- header, then per item three 8-byte
// fields, the data, the 0x1F canary -- whose every position depends on the sizes before it, so the
// lane's loads form a chain.  The chain is kept off the critical path: the header comes with the
// first item's fields in one read, an item's data streams in 64-byte blocks with the next block in
// flight (brb_io::BlockSrc), and the 25 bytes after the data (the canary and the next item's
// fields) are loaded before the data is hashed (Ahead).  The data feeds the lane's MD5
// (md5_funnel.h).  The control flow and the
// unsigned-long arithmetic of cur_offset / cur_remaining / cur_needed are the reference's; see
// include/brb_crypto.h for the two rules where the reference reads past its buffer.
#include "brb_kernels.h"
#include "byte_stream.h"
#include "digest_var_line.h"
#include "line_stream.h"
#include "md5_funnel.h"
#include "test_options.h"

namespace {

constexpr int kBlock = 256;
constexpr uint64_t kMagic = 0x4154454D5F425242ull;   // "BRB_META" as a little-endian unsigned long
constexpr uint64_t kItemStruct = 32;                  // sizeof(MetaDataItem): 3 unsigned longs + a pointer
constexpr uint64_t kItemRaw = 24;                     // METADATA_ITEM_RAW_SZ (libbrb_data.h:297)

// N little-endian dwords of the pack from byte q (any alignment): the N + 1 aligned dwords that
// hold pack bytes are loaded together (the others read as 0), funnel-shifted, and bytes at or past
// `size` are zeroed.  Issued early, they land while the lane hashes the item before them.
template <int N>
struct Ahead {
    uint32_t d[N + 1];
    uint32_t sh;
    uint64_t q, size;

    BRB_DEV void issue(const uint8_t *base, uint64_t size_, uint64_t q_)
    {
        q = q_;
        size = size_;
        const uintptr_t a = reinterpret_cast<uintptr_t>(base) + q;
        const uint32_t *p = reinterpret_cast<const uint32_t *>(a & ~uintptr_t(3));
        sh = uint32_t(a & 3) * 8;
        const uint64_t first = q - (a & 3);                   // pack byte of dword 0 (may be q - 3 .. q)
#pragma unroll
        for (int i = 0; i < N + 1; i++) {
            // dword i starts at pack byte b (b in -3 .. -1, wrapped, for a dword that starts before
            // the pack): it is loaded iff it holds a pack byte
            const uint64_t b = first + 4 * uint64_t(i);
            d[i] = size && (b < size || b > ~uint64_t(0) - 3) ? ldg(p + i) : 0u;
        }
    }
    BRB_DEV uint32_t dw(int i) const                          // pack bytes q + 4i .. q + 4i + 3
    {
        const uint32_t v = __builtin_amdgcn_alignbit(d[i + 1], d[i], sh);
        const uint64_t at = q + 4 * uint64_t(i);
        if (at >= size)
            return 0u;
        const uint64_t left = size - at;
        return left >= 4 ? v : v & ((1u << (8 * uint32_t(left))) - 1u);
    }
    BRB_DEV uint64_t qw(int i) const { return uint64_t(dw(i)) | (uint64_t(dw(i + 1)) << 32); }
};

// MetaDataUnpack of one pack by one lane with per-lane loads (the round-3 kernel's walk): groups
// whose packs span 2 GiB or more take it inside the line-staged kernel, and the round-3 kernel
// (test option seg_line = 0) is this function per lane.
template <uint32_t RW, class Beat = brb_line::NoBeat>
BRB_DEV BRB_MetaDataUnpackInfo unpack_lane(brb_md5::FunnelT<RW> &f, const uint8_t *base, uint64_t size,
                                           Beat beat = Beat())
{
    int32_t code;
    uint32_t items = 0;
    uint64_t offset = 0, remaining = 0, needed = 0;   // cur_offset starts at the MemBuffer offset, 0

    // MetaDataHeader (libbrb_data.h:322-330) and the first item's three fields: bytes 0 .. 87
    Ahead<22> hd;
    hd.issue(base, size, 0);
    const int32_t item_count = int32_t(hd.dw(1));
    const uint64_t magic = hd.qw(4);
    const uint32_t dig[4] = {hd.dw(6), hd.dw(7), hd.dw(8), hd.dw(9)};
    if (magic != kMagic) {                                  // meta_data.c:183-195
        code = BRB_METADATA_UNPACK_FAILED_INVALID_HEADER_MAGIC;
    } else {
        offset = BRB_METADATA_HEADER_SIZE;                  // :198-199
        code = BRB_METADATA_UNPACK_SUCCESS;
        uint64_t sz = hd.qw(20);                            // item 0's sz (bytes 80..87)
        for (int32_t i = 0; i < item_count; i++) {          // :202
            beat();                                         // per item: an empty one runs no block
            remaining = size - offset;                      // :213 (unsigned long)
            if (remaining < kItemStruct) {                  // :216-224
                needed = kItemStruct - remaining;
                code = BRB_METADATA_UNPACK_FAILED_NEED_MORE_DATA_METAITEM;
                break;
            }
            offset += kItemRaw;                             // :227-232 (item_id, item_sub_id skipped)
            remaining -= kItemRaw;
            if (remaining < sz + 1 || sz > size) {          // :237-246 (sz > size: never read, see header)
                needed = sz + 1 - remaining;
                code = BRB_METADATA_UNPACK_FAILED_NEED_MORE_DATA_OBJECT;
                break;
            }
            // the canary and the next item's fields (bytes offset + sz .. + 24) load while the data
            // is hashed; the data comes in 64-byte blocks with the next one in flight
            Ahead<7> nx;
            nx.issue(base, size, offset + sz);
            // The data is read from e = (bytes digested so far) mod 4 bytes before it (the item's
            // own fields, offset >= 88 > e), so its words fall on the digest's word boundaries: one
            // funnel shift per word (in BlockSrc) and no carry shifting (md5_funnel.h put16w); the
            // first word's e low bytes are the carried ones.  Here sz + 1 <= size - offset.
            const uint32_t e = f.nacc;
            const uint64_t n = sz + e;
            brb_io::BlockSrc bs;   // two blocks in flight (registers copied per block): 75.7 -> 81.4 us
            bs.init(base + offset - e, n);
            for (uint64_t c = 0; c < n; c += 64) {          // :249-254 BRB_MD5UpdateBig of the data
                uint32_t w[16];
                bs.fetch(w);
                if (c == 0)
                    w[0] = f.head(w[0]);
                const uint64_t left = n - c;
                if (left >= 64)
                    f.put16w(w);
                else
                    f.put_tail(w, uint32_t(left));
                f.pump();
                beat();
            }
            if ((n & 63) == 0) {                            // ended on a whole block: nothing carried
                f.acc = 0;
                f.nacc = 0;
            }
            f.total += sz;
            offset += sz;
            remaining -= sz;
            if ((nx.dw(0) & 0xFFu) != 0x1Fu) {              // :258-268
                code = BRB_METADATA_UNPACK_FAILED_CORRUPTED_CANARY;
                break;
            }
            offset += 1;                                    // :271-277
            remaining -= 1;
            items++;
            if (offset == size)                             // :280-281
                break;
            // next item's sz: pack bytes offset + 16 .. + 23 = bytes 17 .. 24 of nx
            sz = uint64_t(__builtin_amdgcn_alignbit(nx.dw(5), nx.dw(4), 8)) |
                 (uint64_t(__builtin_amdgcn_alignbit(nx.dw(6), nx.dw(5), 8)) << 32);
        }
        if (code == BRB_METADATA_UNPACK_SUCCESS) {          // :287-298
            const Md5State st = f.finish();
            if (st.a != dig[0] || st.b != dig[1] || st.c != dig[2] || st.d != dig[3])
                code = BRB_METADATA_UNPACK_FAILED_DIGEST_INVALID;
        }
    }
    BRB_MetaDataUnpackInfo o;
    o.error_code = code;
    o.item_count = items;
    o.cur_offset = offset;
    o.cur_remaining = remaining;
    o.cur_needed = needed;
    return o;
}

__global__ __launch_bounds__(kBlock) void metadata_unpack_kernel(const uint8_t *__restrict__ data,
                                                                 const uint64_t *__restrict__ offs,
                                                                 const uint32_t *__restrict__ lens, uint64_t n,
                                                                 BRB_MetaDataUnpackInfo *__restrict__ info)
{
    __shared__ __attribute__((aligned(8192))) uint32_t blk[kBlock / 64][brb_md5::kRingWords][64];   // 8 KiB per wave
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t r = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (r >= n)
        return;
    brb_md5::Funnel f;
    f.init(&blk[wave][0][lane]);
    info[r] = unpack_lane(f, data + offs[r], lens[r]);
}

// Line-staged MetaDataUnpack (round 4; line_stream.h).  A wave unpacks groups of 64 packs, one per
// lane; a pack's 128-byte lines stream through the LDS-DMA ring, and the lane walks its pack out of
// the window (lines k-1, k) as a state machine over the reference's loop (meta_data.c:202-282):
//   FIELDS at `offset`: the loop's checks, sz from the item's fields (window bytes), -> DATA
//   DATA [ds, de):       the item's words that start in line k-1 emitted into the funnel ring;
//                        -> CANARY once its last word is out
//   CANARY at de:        the 0x1F check, items++, offset == size stops the walk, -> FIELDS
// Every event is handled in the line that holds its first byte, so the window always holds what it
// reads; the whole line's reads happen before that line's slot is refilled.  NS ring slots (three:
// line k+1 is in flight during line k-1's work).  The return codes and the unsigned long arithmetic
// of cur_offset / cur_remaining / cur_needed are unpack_lane's (the reference's).
// PC = false: the walking wave also compresses (a 32-word funnel ring, whole blocks compressed after
// each half-line).  PC = true: wave pairs as md5_seg_pc_kernel (md5_seg_kernels.hip): the walking
// wave (the producer) emits the words into the pair's 64-word ring; its partner on the same SIMD
// (wave W + p) compresses them, pads, checks the digest and writes the info (two ring slots, so that
// four pairs fit a CU's LDS).
// STALL: test option pair_stall (pair_fault.h), PC only.
template <int W, int NS, bool PC, bool STALL = false>
__global__ __launch_bounds__(64 * W * (PC ? 2 : 1)) void metadata_line_kernel(const uint8_t *__restrict__ data,
                                                                               const uint64_t *__restrict__ offs,
                                                                               const uint32_t *__restrict__ lens, uint64_t n,
                                                                               BRB_MetaDataUnpackInfo *__restrict__ info,
                                                                               uint32_t *fault)
{
    using namespace brb_line;
    constexpr uint32_t RW = PC ? 64 : brb_line::kRingWords;
    constexpr int WP = PC ? W : 1;                      // pairs' mailbox arrays (1: unused)
    enum : uint32_t { kFields = 0, kData = 1, kCanary = 2, kDone = 3 };
    static_assert(NS == 2 || NS == 3, "two or three ring slots");
    static_assert(!PC || NS == 2, "wave pairs: two slots");
    __shared__ __attribute__((aligned(16384))) uint8_t ring[W * NS * kSlot];
    __shared__ __attribute__((aligned(RW * 256))) uint32_t fring[W][RW][64];
    __shared__ uint32_t wpx[WP][64], cpx[WP][64];       // pairs: words written, words compressed
    __shared__ uint32_t fin[WP][15][64];                // pairs: the walk's results for the consumer
    __shared__ uint32_t ev[WP][4];                      // pairs: producer events, consumer events, plan, heartbeat
    __shared__ uint32_t *fault_at;                      // pairs: pair_sync.h pc_fault_from
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t pr = PC ? wv % W : wv;
    const uint64_t n_groups = (n + 63) / 64;
    const uint64_t gstride = uint64_t(gridDim.x) * W;
    if (PC) {
        if (threadIdx.x == 0)
            fault_at = fault;
        if (threadIdx.x < WP * 4)
            (&ev[0][0])[threadIdx.x] = 0;
        if (threadIdx.x < WP * 64) {
            (&wpx[0][0])[threadIdx.x] = 0;
            (&cpx[0][0])[threadIdx.x] = 0;
        }
        __syncthreads();
    }
    if (PC && wv >= W) {
        // ---------------- consumer ----------------
        uint32_t pseen = 0, cev = 0;
        for (uint64_t g = uint64_t(blockIdx.x) * W + pr; g < n_groups; g += gstride) {
            if (!pc_wait_ge(&ev[pr][0], pseen + 1, &ev[pr][3])) {
                pc_fault_from(&fault_at);
                return;
            }
            pseen++;
            const uint32_t K = __builtin_amdgcn_readfirstlane(ev[pr][2]);
            pc_publish(&ev[pr][1], ++cev);              // plan read
            if (K == 0)
                continue;                               // the producer runs this group alone
            brb_md5::FunnelT<RW> f;
            f.init(&fring[pr][0][lane]);
            if (!pc_consume(f, &ev[pr][0], pseen + 1, &wpx[pr][lane], &cpx[pr][lane], &ev[pr][3])) {
                pc_fault_from(&fault_at);
                return;
            }
            pseen++;
            uint32_t v[15];
#pragma unroll
            for (int q = 0; q < 15; q++)
                v[q] = fin[pr][q][lane];
            f.acc = v[0] & 0xFFFFFFu;
            f.nacc = v[0] >> 24;
            f.total = uint64_t(v[1]) | (uint64_t(v[2]) << 32);
            int32_t code = int32_t(v[3]);
            if (code == BRB_METADATA_UNPACK_SUCCESS) {  // :287-298
                const Md5State st = f.finish();
                if (st.a != v[4] || st.b != v[5] || st.c != v[6] || st.d != v[7])
                    code = BRB_METADATA_UNPACK_FAILED_DIGEST_INVALID;
            }
            pc_publish(&cpx[pr][lane], 0u);
            pc_publish(&ev[pr][1], ++cev);              // group done: ring, fin and cpos free
            const uint64_t r = g * 64 + lane;
            if (r < n) {
                BRB_MetaDataUnpackInfo o;
                o.error_code = code;
                o.item_count = v[8];
                o.cur_offset = uint64_t(v[9]) | (uint64_t(v[10]) << 32);
                o.cur_remaining = uint64_t(v[11]) | (uint64_t(v[12]) << 32);
                o.cur_needed = uint64_t(v[13]) | (uint64_t(v[14]) << 32);
                info[r] = o;
            }
        }
        return;
    }

    const uint32_t lds0 = uint32_t(reinterpret_cast<uintptr_t>(ring)) + pr * NS * kSlot;
    const uint64_t dbase = reinterpret_cast<uint64_t>(data);
    uint32_t *const my_cpx = &cpx[PC ? pr : 0][lane];
    uint32_t *const my_wpx = &wpx[PC ? pr : 0][lane];
    Win win;
    win.init(lane);
    uint32_t pev = 0, cexp = 0;                         // pairs: events published, consumer events expected
    uint32_t beats = 0;                                 // pairs: heartbeat, one per line

    for (uint64_t g = uint64_t(blockIdx.x) * W + pr; g < n_groups; g += gstride) {
        if (PC && !pc_wait_ge(&ev[pr][1], cexp))        // every earlier event acknowledged (a fault: the
            return;                                       // consumer, waiting on this wave, reports it)
        const uint64_t r = g * 64 + lane;
        const bool valid = r < n;
        const uint64_t base = valid ? dbase + offs[r] : dbase;
        const uint64_t size = valid ? lens[r] : 0;
        const uint32_t a0 = uint32_t(base & 127);
        const uint32_t nl = size ? uint32_t((a0 + size + 127) >> 7) : 0u;
        const uint64_t line0 = base & ~uint64_t(127);
        const uint64_t lo = brb_digest::uniform64(brb_digest::wave_min64(nl ? line0 : ~uint64_t(0)));
        const uint64_t hi = brb_digest::uniform64(brb_digest::wave_max64(nl ? line0 + 128 * uint64_t(nl) : 0));
        const uint32_t Kl = __builtin_amdgcn_readfirstlane(uint32_t(brb_digest::wave_max64(nl)));
        const uint32_t K = Kl ? Kl : 1u;                  // iteration 1 reads every header
        brb_md5::FunnelT<RW> f;
        f.init(&fring[pr][0][lane]);
        if (!(hi > lo && hi - lo < (uint64_t(1) << 31) - (uint64_t(1) << 16))) {   // no line, or too wide
            if (PC) {                                     // the per-lane path, this wave only
                ev[pr][2] = 0;
                pc_publish(&ev[pr][0], ++pev);
                cexp += 1;
            }
            if (valid) {
                if (PC)
                    info[r] = unpack_lane(f, reinterpret_cast<const uint8_t *>(base), size, brb_line::HbBeat{&ev[pr][3], 0});
                else
                    info[r] = unpack_lane(f, reinterpret_cast<const uint8_t *>(base), size);
            }
            continue;
        }
        if (PC) {
            *my_wpx = 0;                                  // the consumer reads it only after the plan
            ev[pr][2] = K;
            if (STALL && blockIdx.x == 0 && pr == 0 && pev == 0)
                ++pev;                                    // test option pair_stall: the plan is never posted
            else
                pc_publish(&ev[pr][0], ++pev);
            cexp += 2;
        }
        const brb_dma::v4i rs = group_rsrc(lo, hi);
        const uint32_t rel0 = nl ? uint32_t(line0 - lo) : kOOB;
        auto line_rel = [&](uint32_t j) { return j < nl ? rel0 + 128 * j : kOOB; };
        issue_rows(rs, lds0, line_rel(0), lane);
        issue_rows(rs, lds0 + kSlot, line_rel(1), lane);
        if (NS == 3)
            issue_rows(rs, lds0 + 2 * kSlot, line_rel(2), lane);

        int32_t code = BRB_METADATA_UNPACK_SUCCESS, item_count = 0, item = 0;
        uint32_t items = 0, phase = kDone, b = 0, dig[4] = {0, 0, 0, 0};
        uint64_t offset = 0, remaining = 0, needed = 0, ds = 0, de = 0;
        bool ok = true;

        // The walk's events whose first byte lies before pack byte L1, line k-1 = pack bytes [L0, L1)
        // in the window.  drain: after the last line, the events a pack shorter than its header
        // still reaches past its end (every byte there reads as 0: sz 0, no canary).
        auto events = [&](int64_t L0, int64_t L1, uint32_t sa, uint32_t sb, const uint32_t (&dw)[36], bool drain) {
            auto rd32 = [&](int64_t p) -> uint32_t {           // pack bytes p .. p + 3, 0 past the pack
                if (drain || uint64_t(p) >= size)
                    return 0u;
                const uint32_t wb = uint32_t(p - L0);
                const uint32_t v = __builtin_amdgcn_alignbit(win_dword(win, (wb >> 2) + 1, sa, sb),
                                                             win_dword(win, wb >> 2, sa, sb), 8 * (wb & 3));
                const uint64_t left = size - uint64_t(p);
                return left >= 4 ? v : v & ((1u << (8 * uint32_t(left))) - 1u);
            };
            bool more = phase != kDone;
            while (more) {
                more = false;
                if (phase == kFields && int64_t(offset) < L1) {  // :202-246, the loop's top
                    if (item >= item_count) {
                        phase = kDone;
                    } else {
                        remaining = size - offset;               // :213
                        if (remaining < kItemStruct) {           // :216-224
                            needed = kItemStruct - remaining;
                            code = BRB_METADATA_UNPACK_FAILED_NEED_MORE_DATA_METAITEM;
                            phase = kDone;
                        } else {
                            const uint64_t sz = uint64_t(rd32(int64_t(offset) + 16)) |
                                                (uint64_t(rd32(int64_t(offset) + 20)) << 32);
                            offset += kItemRaw;                  // :227-232
                            remaining -= kItemRaw;
                            if (remaining < sz + 1 || sz > size) {   // :237-246
                                needed = sz + 1 - remaining;
                                code = BRB_METADATA_UNPACK_FAILED_NEED_MORE_DATA_OBJECT;
                                phase = kDone;
                            } else {
                                ds = offset;
                                de = offset + sz;
                                f.total += sz;
                                offset += sz;                    // :249-256 (the walk's values after the data)
                                remaining -= sz;
                                phase = kData;
                                more = true;
                            }
                        }
                    }
                }
                if (phase == kData && int64_t(ds) < L1) {        // :249-254 BRB_MD5UpdateBig of the data
                    const bool first = int64_t(ds) >= L0;
                    const int64_t er = int64_t(de) - L0;
                    bool done = de == ds || drain;
                    if (!done) {
                        Emit e;
                        plan_range(f, first, uint32_t(int64_t(ds) - L0), er < 4096 ? uint32_t(er) : 4096u, b, e);
                        edge_words(win, sa, sb, e);
                        ok = emit_line<RW, false, PC>(f, e, dw, true, my_cpx, my_wpx) && ok;
                        done = !e.any || e.ends;
                    }
                    more = done;                                 // else the line is used up (no second emission)
                    if (done)
                        phase = kCanary;
                }
                if (phase == kCanary && int64_t(de) < L1) {      // :258-281
                    if ((rd32(int64_t(de)) & 0xFFu) != 0x1Fu) {
                        code = BRB_METADATA_UNPACK_FAILED_CORRUPTED_CANARY;
                        phase = kDone;
                    } else {
                        offset += 1;
                        remaining -= 1;
                        items++;
                        item++;
                        phase = offset == size ? kDone : kFields;
                        more = phase != kDone;
                    }
                }
            }
        };
        uint32_t sa = 0;                                         // byte offset of line k-1's slot (uniform)
        for (uint32_t k = 1; k <= K; k++) {
            const uint32_t sb = sa == (NS - 1) * kSlot ? 0u : sa + kSlot;  // line k's slot
            brb_dma::wait_vmcnt<NS == 3 ? 8 : 0>();              // line k landed (NS = 3: line k+1 may fly)
            uint32_t dw[36];
            read_window(win, lds0 + sa, lds0 + sb, dw);
            // pack byte p sits at window byte p - L0 while L0 <= p < L0 + 256
            const int64_t L0 = int64_t(128) * int64_t(k - 1) - int64_t(a0);
            if (k == 1 && valid) {                               // MetaDataHeader (libbrb_data.h:322-330)
                auto hd32 = [&](uint32_t p) -> uint32_t {        // header bytes: 0 past the pack
                    if (p >= size)
                        return 0u;
                    const uint32_t wb = p + a0;
                    const uint32_t v = __builtin_amdgcn_alignbit(win_dword(win, (wb >> 2) + 1, lds0 + sa, lds0 + sb),
                                                                 win_dword(win, wb >> 2, lds0 + sa, lds0 + sb), 8 * (wb & 3));
                    const uint64_t left = size - p;
                    return left >= 4 ? v : v & ((1u << (8 * uint32_t(left))) - 1u);
                };
                item_count = int32_t(hd32(4));
                const uint64_t magic = uint64_t(hd32(16)) | (uint64_t(hd32(20)) << 32);
#pragma unroll
                for (int q = 0; q < 4; q++)
                    dig[q] = hd32(24 + 4 * q);
                if (magic != kMagic) {                           // meta_data.c:183-195
                    code = BRB_METADATA_UNPACK_FAILED_INVALID_HEADER_MAGIC;
                } else {
                    offset = BRB_METADATA_HEADER_SIZE;           // :198-199
                    phase = kFields;
                }
            }
            // the common line: every walking lane is inside an item's data that covers the whole
            // line and goes on past its 32 words (not its first line, not the line of its last word,
            // where the carry is set) -> 32 whole words, no event to look for
            const bool whole = phase == kDone ||
                               (phase == kData && int64_t(ds) < L0 && int64_t(de) - L0 > 128 + int64_t(b));
            if (k > 1 && __builtin_amdgcn_ballot_w64(!whole) == 0) {
                // line k+NS-1 into line k-1's slot at once: the emission reads the window registers only
                issue_rows(rs, lds0 + sa, phase == kDone ? kOOB : line_rel(k + NS - 1), lane);
                Emit e;
                plan_whole(f, b, e);
                ok = emit_line<RW, true, PC>(f, e, dw, phase == kData, my_cpx, my_wpx) && ok;
            } else {
                events(L0, L0 + 128, lds0 + sa, lds0 + sb, dw, false);
                // line k+NS-1 into line k-1's slot (its window reads are done)
                issue_rows(rs, lds0 + sa, phase == kDone ? kOOB : line_rel(k + NS - 1), lane);
            }
            sa = sb;
            if (PC) {
                pc_beat(&ev[pr][3], ++beats);
                if (__builtin_amdgcn_ballot_w64(!ok) != 0)
                    break;
            }
        }
        brb_dma::wait_vmcnt<0>();                                // the stray stages, before the slots are reused
        if (PC && __builtin_amdgcn_ballot_w64(!ok) != 0)
            return;                                              // a protocol fault: the consumer reports it
        if (phase != kDone) {                                    // a pack shorter than its header
            uint32_t dw[36] = {};
            events(int64_t(1) << 62, int64_t(1) << 62, 0, 0, dw, true);
        }
        if (PC) {
            const uint32_t v[15] = {uint32_t(f.acc) | (f.nacc << 24), uint32_t(f.total), uint32_t(f.total >> 32),
                                    uint32_t(code), dig[0], dig[1], dig[2], dig[3], items,
                                    uint32_t(offset), uint32_t(offset >> 32), uint32_t(remaining),
                                    uint32_t(remaining >> 32), uint32_t(needed), uint32_t(needed >> 32)};
#pragma unroll
            for (int q = 0; q < 15; q++)
                fin[pr][q][lane] = v[q];
            pc_publish(&ev[pr][0], ++pev);                       // the group's end
            continue;
        }
        if (!valid)
            continue;
        if (code == BRB_METADATA_UNPACK_SUCCESS) {               // :287-298
            const Md5State st = f.finish();
            if (st.a != dig[0] || st.b != dig[1] || st.c != dig[2] || st.d != dig[3])
                code = BRB_METADATA_UNPACK_FAILED_DIGEST_INVALID;
        }
        BRB_MetaDataUnpackInfo o;
        o.error_code = code;
        o.item_count = items;
        o.cur_offset = offset;
        o.cur_remaining = remaining;
        o.cur_needed = needed;
        info[r] = o;
    }
}

}  // namespace

namespace brb {

hipError_t launch_metadata_unpack(const uint8_t *data, const uint64_t *offs, const uint32_t *lens, uint64_t n,
                                  BRB_MetaDataUnpackInfo *info, hipStream_t s)
{
    if (n == 0)
        return hipSuccess;
    if (brb_opt::get(brb_opt::kSegLine) == 0) {
        metadata_unpack_kernel<<<unsigned((n + kBlock - 1) / kBlock), kBlock, 0, s>>>(data, offs, lens, n, info);
        return hipGetLastError();
    }
    constexpr int W = 4;                               // 4 walking waves: one workgroup per CU
    const uint64_t groups = (n + 63) / 64;
    const uint64_t wgs = (groups + W - 1) / W;
    const unsigned grid = unsigned(wgs < brb_digest::device_cu_count() ? wgs : brb_digest::device_cu_count());
    if (brb_opt::get(brb_opt::kSegLine) == 2) {        // wave pairs
        if (brb_opt::get(brb_opt::kPairStall) != 0)
            metadata_line_kernel<W, 2, true, true><<<grid, 128 * W, 0, s>>>(data, offs, lens, n, info, brb::pair_fault_word());
        else
            metadata_line_kernel<W, 2, true><<<grid, 128 * W, 0, s>>>(data, offs, lens, n, info, brb::pair_fault_word());
    } else if (brb_opt::get(brb_opt::kLineSlots) == 2) {
        // three slots by default: 43.6 vs 49.3 us with two (bench --op metadata, interleaved A/B,
        // profiles/r04/ab/r04s_md); test option line_slots 2 for the other
        metadata_line_kernel<W, 2, false><<<grid, 64 * W, 0, s>>>(data, offs, lens, n, info, nullptr);
    } else {
        metadata_line_kernel<W, 3, false><<<grid, 64 * W, 0, s>>>(data, offs, lens, n, info, nullptr);
    }
    return hipGetLastError();
}

}  // namespace brb
