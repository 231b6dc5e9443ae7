// md5_seg_kernels.hip -- MD5 of a list of byte segments per record.
//
// MetaDataHeaderLoadData (libbrb_core/data/utils/meta_data.c:397-433) digests the items of one
// MetaData as BRB_MD5Init, one BRB_MD5UpdateBig per item, BRB_MD5Final: the MD5 of the items'
// concatenation, the items scattered in memory.  Batched: one record (one MetaData) per lane, its
// segments (items) walked in order in 64-byte blocks (brb_io::BlockSrc, the next block in flight,
// and the next segment's first block in flight while the current one is hashed), their bytes
// funnelled into the lane's MD5 (md5_funnel.h).
#include "brb_kernels.h"
#include "byte_stream.h"
#include "digest_var_line.h"
#include "line_stream.h"
#include "md5_funnel.h"
#include "test_options.h"

namespace {

constexpr int kBlock = 256;

// The per-lane block path: record r's segments read in 64-byte blocks (brb_io::BlockSrc, the next
// block in flight, the next segment's first block in flight while the current one is hashed) and
// funnelled into the lane's MD5.  Segment k is read as a range starting e_k = (bytes before it)
// mod 4 bytes before it, so its words fall on the digest's word boundaries (Funnel::head); those e
// bytes are the carried ones, never loaded from below the segment.  Used for groups whose lines span
// 2 GiB or more, and by the round-3 kernel kept for A/B (test option seg_line = 0).
template <uint32_t RW, class Beat = brb_line::NoBeat>
BRB_DEV void seg_lane(brb_md5::FunnelT<RW> &f, const uint8_t *__restrict__ data, const uint64_t *__restrict__ soff,
                      const uint32_t *__restrict__ slen, uint64_t k, uint64_t k1, Beat beat = Beat())
{
    uint64_t before = 0;
    auto skip_empty = [&](uint64_t kk) {                // the next segment with bytes (an empty one's
        while (kk < k1 && slen[kk] == 0) {              // address need not be memory); a beat per
            kk++;                                       // skipped segment: a million-long run of empty
            beat();                                     // ones outlasts the partner's idle budget
        }
        return kk;
    };
    auto start = [&](brb_io::BlockSrc &src, uint64_t kk, uint64_t pre, uint64_t &len) {
        len = slen[kk];
        const uint8_t *a = data + soff[kk];
        const uint32_t e = uint32_t(pre & 3);
        src.init(a - e, len + e, a);
    };
    auto run = [&](brb_io::BlockSrc &src, uint64_t len) {   // 64-byte blocks, the next one in flight
        const uint32_t e = f.nacc;
        const uint64_t n = len + e;
        for (uint64_t c = 0; c < n; c += 64) {
            uint32_t w[16];
            src.fetch(w);
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
        f.total += len;
    };
    brb_io::BlockSrc sa, sb;
    uint64_t la = 0, lb = 0;
    k = skip_empty(k);
    if (k < k1)
        start(sa, k, before, la);
    while (k < k1) {
        uint64_t kb = skip_empty(k + 1);
        if (kb < k1)
            start(sb, kb, before + la, lb);
        run(sa, la);
        before += la;
        if (kb >= k1)
            break;
        k = skip_empty(kb + 1);
        if (k < k1)
            start(sa, k, before + lb, la);
        run(sb, lb);
        before += lb;
    }
}

BRB_DEV void store_digest(uint8_t *out, uint64_t r, const Md5State &st)
{
    const uint4 v = make_uint4(st.a, st.b, st.c, st.d);
    __builtin_memcpy(out + 16 * r, &v, 16);
}

// Round-3 kernel (one record per lane, per-lane block loads), kept for A/B runs.
__global__ __launch_bounds__(kBlock) void md5_seg_kernel(const uint8_t *__restrict__ data,
                                                         const uint64_t *__restrict__ soff,
                                                         const uint32_t *__restrict__ slen,
                                                         const uint64_t *__restrict__ first, uint64_t n_rec,
                                                         uint8_t *__restrict__ out)
{
    __shared__ __attribute__((aligned(8192))) uint32_t blk[kBlock / 64][brb_md5::kRingWords][64];   // 8 KiB per wave
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t r = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (r >= n_rec)
        return;
    brb_md5::Funnel f;
    f.init(&blk[wave][0][lane]);
    seg_lane(f, data, soff, slen, first[r], first[r + 1]);
    store_digest(out, r, f.finish());
}

// A group's segments in the wave's LDS table, and its line plan (both line-staged kernels).  The
// group's segments are one contiguous range of the arrays (first[] is monotone): [s0, s1).  They go
// to the table with coalesced loads, so the stage cursor reads them with LDS latency and no
// vector-memory load ever sits between a wave's DMA issues (a per-lane load there made hipcc wait
// for it right before the DMA).  plan() is false when the group takes the per-lane path: more
// segments than the table holds, no line at all, or lines spanning 2 GiB or more (32-bit voffsets).
template <uint32_t kTab>
struct SegGroup {
    uint64_t *off;          // this wave's table
    uint32_t *len;
    uint32_t t0, t1;        // the lane's entries
    uint32_t K;             // stages of the group's longest lane (an empty segment costs one)
    uint64_t lo, hi;        // the group's 128-byte-aligned line span

    BRB_DEV bool plan(const uint64_t *__restrict__ soff, const uint32_t *__restrict__ slen, uint64_t k0, uint64_t k1,
                      bool valid, uint64_t dbase, uint32_t lane)
    {
        const uint64_t s0 = brb_digest::uniform64(brb_digest::wave_min64(valid ? k0 : ~uint64_t(0)));
        const uint64_t s1 = brb_digest::uniform64(brb_digest::wave_max64(valid ? k1 : 0));
        const uint64_t S = s1 > s0 ? s1 - s0 : 0;
        if (S > kTab)
            return false;
        for (uint32_t i = lane; i < uint32_t(S); i += 64) {
            off[i] = soff[s0 + i];
            len[i] = slen[s0 + i];
        }
        __builtin_amdgcn_s_waitcnt(0);                  // the table is in LDS, every load of it done
        __builtin_amdgcn_wave_barrier();
        t0 = uint32_t(k0 - (valid ? s0 : k0));
        t1 = uint32_t(k1 - (valid ? s0 : k1));
        uint64_t l = ~uint64_t(0), h = 0;
        uint32_t nl = 0;
        for (uint32_t t = t0; t < t1; t++) {
            const uint32_t n = len[t];
            if (!n) {
                nl++;
                continue;
            }
            const uint64_t a = dbase + off[t];
            const uint64_t l0 = a & ~uint64_t(127), l1 = (a + n + 127) & ~uint64_t(127);
            l = l0 < l ? l0 : l;
            h = l1 > h ? l1 : h;
            nl += uint32_t((l1 - l0) >> 7);
        }
        lo = brb_digest::uniform64(brb_digest::wave_min64(l));
        hi = brb_digest::uniform64(brb_digest::wave_max64(h));
        K = __builtin_amdgcn_readfirstlane(uint32_t(brb_digest::wave_max64(nl)));
        return hi > lo && hi - lo < (uint64_t(1) << 31) - (uint64_t(1) << 16);   // K >= 1 then
    }
};

// Stage cursor over a lane's segments: the line to stage next (offset from the group's lowest line;
// kEnd: the cursor must enter the next segment first) and its segment; nt = the next table entry.
struct SegCursor {
    static constexpr uint32_t kEnd = 0xFFFFFFFFu;
    const uint64_t *off;
    const uint32_t *len;
    uint64_t base;          // dbase - lo
    uint32_t nt, t1;
    uint32_t c_line = kEnd, c_last = 0, c_ss = 0, c_se = 0;

    BRB_DEV brb_line::LineDesc next()                   // this stage's line; the cursor moves on
    {
        if (c_line == kEnd && nt < t1) {                // enter segment nt
            const uint32_t n = len[nt];
            if (n) {
                c_ss = uint32_t(base + off[nt]);
                c_se = c_ss + n;
                c_line = c_ss & ~127u;
                c_last = (c_se - 1) & ~127u;
            }
            nt++;
        }
        const brb_line::LineDesc d{c_line == kEnd ? brb_line::kOOB : c_line, c_ss, c_se};
        if (c_line != kEnd)
            c_line = c_line == c_last ? kEnd : c_line + 128;
        return d;
    }
};

// Line-staged kernel (round 4; line_stream.h).  A wave digests groups of 64 records, one per lane;
// a lane's VIRTUAL lines are its non-empty segments' 128-byte memory lines in order, staged by
// LDS-DMA into a three-slot ring: at iteration k the window is lines (k-1, k), line k+1 is in flight
// since iteration k-1, and line k+2 goes into line k-1's slot once the window is read.  The
// segment's words that start in line k-1 go to the lane's 32-word funnel ring in two halves, whole
// blocks compressed after each.  W waves per workgroup, W * 38 KiB of LDS; groups strided over the
// grid.
template <int W, int NS>
__global__ __launch_bounds__(64 * W) void md5_seg_line_kernel(const uint8_t *__restrict__ data,
                                                               const uint64_t *__restrict__ soff,
                                                               const uint32_t *__restrict__ slen,
                                                               const uint64_t *__restrict__ first, uint64_t n_rec,
                                                               uint8_t *__restrict__ out)
{
    using namespace brb_line;
    constexpr uint32_t RW = brb_line::kRingWords;
    constexpr uint32_t kTab = 512;                      // segments per group held in LDS (8 per record)
    static_assert(NS == 2 || NS == 3, "two or three ring slots");
    __shared__ __attribute__((aligned(16384))) uint8_t ring[W * NS * kSlot];
    __shared__ __attribute__((aligned(8192))) uint32_t fring[W][RW][64];
    __shared__ uint64_t tab_off[W][kTab];
    __shared__ uint32_t tab_len[W][kTab];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t n_groups = (n_rec + 63) / 64;
    const uint32_t lds0 = uint32_t(reinterpret_cast<uintptr_t>(ring)) + wv * NS * kSlot;
    const uint64_t dbase = reinterpret_cast<uint64_t>(data);
    Win win;
    win.init(lane);

    for (uint64_t g = uint64_t(blockIdx.x) * W + wv; g < n_groups; g += uint64_t(gridDim.x) * W) {
        const uint64_t rec = g * 64 + lane;
        const bool valid = rec < n_rec;
        const uint64_t k0 = valid ? first[rec] : 0, k1 = valid ? first[rec + 1] : 0;
        brb_md5::FunnelT<RW> f;
        f.init(&fring[wv][0][lane]);
        SegGroup<kTab> sg{tab_off[wv], tab_len[wv]};
        if (!sg.plan(soff, slen, k0, k1, valid, dbase, lane)) {   // the per-lane path
            if (valid) {
                seg_lane(f, data, soff, slen, k0, k1);
                store_digest(out, rec, f.finish());
            }
            continue;
        }
        const uint32_t K = sg.K;
        const brb_dma::v4i rs = group_rsrc(sg.lo, sg.hi);
        SegCursor cur{sg.off, sg.len, dbase - sg.lo, sg.t0, sg.t1};
        auto stage_line = [&]() { return cur.next(); };
        // lines 0 .. NS-1 -> slots 0 .. NS-1; dA, dB (, dC): the lines k-1, k (, k+1) at iteration k
        LineDesc dA = stage_line(), dB = stage_line(), dC = dB;
        issue_rows(rs, lds0, dA.line, lane);
        issue_rows(rs, lds0 + kSlot, dB.line, lane);
        if (NS == 3) {
            dC = stage_line();
            issue_rows(rs, lds0 + 2 * kSlot, dC.line, lane);
        }
        uint32_t b = 0;
        uint32_t sa = 0;                                // byte offset of line k-1's slot (uniform)
#ifdef BRB_LINE_STAMPS    // diagnostic builds only (make -C brb_framework_amd diag; tools/seg_probe.py)
        uint64_t acc_wait = 0, acc_win = 0, acc_stage = 0, acc_emit = 0, acc_pump = 0;
        const uint64_t t_start = __builtin_amdgcn_s_memtime();
#define BRB_STAMP(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#else
#define BRB_STAMP(v)
#endif
        for (uint32_t k = 1; k <= K; k++) {
            const uint32_t sb = sa == (NS - 1) * kSlot ? 0u : sa + kSlot;   // line k's slot
            BRB_STAMP(t0);
            const LineDesc dn = stage_line();           // line k+NS-1 (kOOB rows past the end): its
            const RowsV rv = prep_rows(dn.line, lane);  // rows' offsets gathered while line k lands
            brb_dma::wait_vmcnt<NS == 3 ? 8 : 0>();     // line k landed (NS = 3: line k+1's 8 DMAs may fly)
            BRB_STAMP(t1);
            uint32_t dw[36];
            read_window(win, lds0 + sa, lds0 + sb, dw);
            BRB_STAMP(t2);
            const LineDesc d = dA;                      // line k-1
            dA = dB;
            if (NS == 3) {
                dB = dC;
                dC = dn;
            } else {
                dB = dn;
            }
            const bool has = d.line != kOOB;
            // whole line inside the segment, and not the line of its last word (the carry is set there)
            const bool whole = has && d.ss < d.line && d.se - d.line > 128u + b;
            const bool all_whole = __builtin_amdgcn_ballot_w64(has && !whole) == 0;
            Emit e;
            if (all_whole) {
                plan_whole(f, b, e);
            } else {
                const bool fst = d.ss >= d.line;
                if (has && fst)
                    f.total += d.se - d.ss;
                plan_range(f, fst, d.ss - d.line, d.se - d.line < 4096u ? d.se - d.line : 4096u, b, e);
                if (has)
                    edge_words(win, lds0 + sa, lds0 + sb, e);
                __builtin_amdgcn_s_waitcnt(0xC07F);     // those reads are in before the slot is refilled
            }
            fire_rows(rs, lds0 + sa, rv);               // line k+NS-1 into line k-1's slot
            BRB_STAMP(t3);
            if (!has) {                                 // no line for this lane: nothing to write
                e.any = false;
                e.ends = false;
                e.i0 = 0;
                e.iw = 0;
                e.it = -2;
            }
            if (has) {
                if (all_whole)
                    emit_half<RW, 0, true>(f, e, dw);
                else
                    emit_half<RW, 0, false>(f, e, dw);
            }
            BRB_STAMP(t4);
            pump_all(f);
            BRB_STAMP(t5);
            if (has) {
                if (all_whole)
                    emit_half<RW, 1, true>(f, e, dw);
                else
                    emit_half<RW, 1, false>(f, e, dw);
                emit_finish(f, e);
            }
            BRB_STAMP(t6);
            pump_all(f);
            BRB_STAMP(t7);
#ifdef BRB_LINE_STAMPS
            acc_wait += t1 - t0;
            acc_win += t2 - t1;
            acc_stage += t3 - t2;
            acc_emit += (t4 - t3) + (t6 - t5);
            acc_pump += (t5 - t4) + (t7 - t6);
#endif
            sa = sb;
        }
        brb_dma::wait_vmcnt<0>();                       // the stray stages past K, before the slots are reused
#ifdef BRB_LINE_STAMPS
        // lane 0's digest slot: wait, window, stage, emit; lane 1's: pump, total, K, 0 (cycles)
        const uint64_t t_end = __builtin_amdgcn_s_memtime();
        if (lane < 2 && valid) {
            const uint4 v = lane == 0 ? make_uint4(uint32_t(acc_wait), uint32_t(acc_win), uint32_t(acc_stage), uint32_t(acc_emit))
                                      : make_uint4(uint32_t(acc_pump), uint32_t(t_end - t_start), K, 0u);
            __builtin_memcpy(out + 16 * rec, &v, 16);
        }
        continue;
#endif
        if (valid)
            store_digest(out, rec, f.finish());
    }
}

// Producer / consumer form of the line-staged kernel.  With one 64-record group per SIMD (the
// md5seg bench shape: 1 024 groups on 1 024 SIMDs) the lone wave of md5_seg_line_kernel pays the
// lone-wave issue rate and every LDS round trip of its staging, emission and window reads (in-kernel
// stamps, tools/seg_probe.py: 47 % compression, 53 % the rest).  Here a group belongs to a PAIR of
// waves: the producer (waves 0..NP-1) walks the group's lines as md5_seg_line_kernel does (segment
// table, DMA ring of two slots, window, emission) but never compresses; the consumer (wave NP + p)
// compresses the words from the pair's 64-word funnel ring.  Both waves share a SIMD (8 waves per
// CU), so the consumer's compression fills the producer's LDS and DMA waits and the two instruction
// streams pair in the SIMD's issue.
// Protocol, per lane, through LDS mailboxes (line_stream.h pc_*): the producer posts its word count
// wpos after each half-line (release store) and waits, before a half, until the consumer's posted
// compressed count cpos leaves room in the ring (pc_room); the consumer polls wpos, compresses every
// whole block, posts cpos.  Per group, two event counts order the rest: the producer publishes the
// group's plan (K lines, or 0: the per-lane path, run by the producer alone) and its end (the carried
// bytes and the length in `fin`); the consumer acknowledges the plan and, after the digest, the end
// (its cpos back to 0).  A producer starts a group only once every earlier event is acknowledged.
// STALL: test option pair_stall (pair_fault.h), a separate instantiation so the product kernel
// carries no test code.
template <int NP, bool STALL>
__global__ __launch_bounds__(128 * NP) void md5_seg_pc_kernel(const uint8_t *__restrict__ data,
                                                             const uint64_t *__restrict__ soff,
                                                             const uint32_t *__restrict__ slen,
                                                             const uint64_t *__restrict__ first, uint64_t n_rec,
                                                             uint8_t *__restrict__ out, uint32_t *fault)
{
    using namespace brb_line;
    constexpr uint32_t RW = 64;                         // funnel ring words per lane (16 KiB per pair)
    constexpr uint32_t kTab = 512;
    __shared__ __attribute__((aligned(16384))) uint8_t ring[NP * 2 * kSlot];
    __shared__ __attribute__((aligned(16384))) uint32_t fring[NP][RW][64];
    __shared__ uint64_t tab_off[NP][kTab];
    __shared__ uint32_t tab_len[NP][kTab];
    __shared__ uint32_t wpx[NP][64], cpx[NP][64];       // the mailboxes: words written, words compressed
    __shared__ uint32_t fin[NP][3][64];                 // carried bytes | count << 24, length lo / hi
    __shared__ uint32_t ev[NP][4];                      // producer events, consumer events, plan, heartbeat
    __shared__ uint32_t *fault_at;                      // pair_sync.h pc_fault_from
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t pr = wv % NP;
    const bool producer = wv < NP;
    if (threadIdx.x == 0)
        fault_at = fault;
    if (threadIdx.x < NP * 4)
        (&ev[0][0])[threadIdx.x] = 0;
    if (threadIdx.x < NP * 64) {
        (&wpx[0][0])[threadIdx.x] = 0;
        (&cpx[0][0])[threadIdx.x] = 0;
    }
    __syncthreads();
    const uint64_t n_groups = (n_rec + 63) / 64;
    const uint64_t gstride = uint64_t(gridDim.x) * NP;

    if (!producer) {
        // ---------------- consumer ----------------
        uint32_t pseen = 0, cev = 0;
#ifdef BRB_LINE_STAMPS    // diagnostic builds only (tools/seg_probe.py --pc): cycles without a block to compress
        uint64_t c_wait = 0;
        const uint64_t c_t0 = __builtin_amdgcn_s_memtime();
#endif
        for (uint64_t g = uint64_t(blockIdx.x) * NP + pr; g < n_groups; g += gstride) {
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
#ifdef BRB_LINE_STAMPS
            if (!pc_consume(f, &ev[pr][0], pseen + 1, &wpx[pr][lane], &cpx[pr][lane], &ev[pr][3], &c_wait)) {
                pc_fault_from(&fault_at);
                return;
            }
#else
            if (!pc_consume(f, &ev[pr][0], pseen + 1, &wpx[pr][lane], &cpx[pr][lane], &ev[pr][3])) {
                pc_fault_from(&fault_at);
                return;
            }
#endif
            pseen++;
            const uint32_t a = fin[pr][0][lane];
            f.acc = a & 0xFFFFFFu;
            f.nacc = a >> 24;
            f.total = uint64_t(fin[pr][1][lane]) | (uint64_t(fin[pr][2][lane]) << 32);
            const Md5State st = f.finish();
            pc_publish(&cpx[pr][lane], 0u);
            pc_publish(&ev[pr][1], ++cev);              // group done: ring, fin and cpos free
            const uint64_t rec = g * 64 + lane;
#ifdef BRB_LINE_STAMPS
            if (lane == 1 && rec < n_rec) {
                const uint4 v = make_uint4(uint32_t(c_wait), uint32_t(__builtin_amdgcn_s_memtime() - c_t0), K, 0u);
                __builtin_memcpy(out + 16 * rec, &v, 16);
            }
            if (lane < 2)
                continue;
#endif
            if (rec < n_rec)
                store_digest(out, rec, st);
        }
        return;
    }

    // ---------------- producer ----------------
    const uint32_t lds0 = uint32_t(reinterpret_cast<uintptr_t>(ring)) + pr * 2 * kSlot;
    const uint64_t dbase = reinterpret_cast<uint64_t>(data);
    Win win;
    win.init(lane);
    uint32_t pev = 0, cexp = 0;                         // events published; consumer events expected so far
    uint32_t beats = 0;                                 // heartbeat: one per line
#ifdef BRB_LINE_STAMPS    // the producer's waits for ring room and for its DMA
    uint64_t p_wait = 0, p_dma = 0;
    const uint64_t p_t0 = __builtin_amdgcn_s_memtime();
#endif
    for (uint64_t g = uint64_t(blockIdx.x) * NP + pr; g < n_groups; g += gstride) {
        if (!pc_wait_ge(&ev[pr][1], cexp))             // every earlier event acknowledged (a fault: the
            return;                                     // consumer, waiting on this wave, reports it)
        const uint64_t rec = g * 64 + lane;
        const bool valid = rec < n_rec;
        const uint64_t k0 = valid ? first[rec] : 0, k1 = valid ? first[rec + 1] : 0;
        brb_md5::FunnelT<RW> f;
        f.init(&fring[pr][0][lane]);
        auto alone = [&]() {                            // the per-lane path, this wave only
            ev[pr][2] = 0;
            pc_publish(&ev[pr][0], ++pev);
            cexp += 1;
            if (valid) {
                seg_lane(f, data, soff, slen, k0, k1, brb_line::HbBeat{&ev[pr][3], 0});
                store_digest(out, rec, f.finish());
            }
        };
        SegGroup<kTab> sg{tab_off[pr], tab_len[pr]};
        if (!sg.plan(soff, slen, k0, k1, valid, dbase, lane)) {
            alone();
            continue;
        }
        const uint32_t K = sg.K;
        wpx[pr][lane] = 0;                              // the consumer reads it only after the plan
        ev[pr][2] = K;                                  // the plan (K >= 1)
        if (STALL && blockIdx.x == 0 && pr == 0 && pev == 0)
            ++pev;                                      // test option pair_stall: the plan is never posted
        else
            pc_publish(&ev[pr][0], ++pev);
        cexp += 2;
        const brb_dma::v4i rs = group_rsrc(sg.lo, sg.hi);
        SegCursor cur{sg.off, sg.len, dbase - sg.lo, sg.t0, sg.t1};
        auto stage_line = [&]() { return cur.next(); };
        LineDesc dA = stage_line(), dB = stage_line();
        issue_rows(rs, lds0, dA.line, lane);
        issue_rows(rs, lds0 + kSlot, dB.line, lane);
        uint32_t b = 0, sa = 0;
        bool ok = true;
        for (uint32_t k = 1; k <= K; k++) {
            const uint32_t sb = sa ^ kSlot;             // line k's slot
            const LineDesc dn = stage_line();           // line k+1
            const RowsV rv = prep_rows(dn.line, lane);
#ifdef BRB_LINE_STAMPS
            const uint64_t _d0 = __builtin_amdgcn_s_memtime();
            brb_dma::wait_vmcnt<0>();
            p_dma += __builtin_amdgcn_s_memtime() - _d0;
#else
            brb_dma::wait_vmcnt<0>();                   // line k landed
#endif
            uint32_t dw[36];
            read_window(win, lds0 + sa, lds0 + sb, dw);
            const LineDesc d = dA;
            dA = dB;
            dB = dn;
            const bool has = d.line != kOOB;
            const bool whole = has && d.ss < d.line && d.se - d.line > 128u + b;
            const bool all_whole = __builtin_amdgcn_ballot_w64(has && !whole) == 0;
            Emit e;
            if (all_whole) {
                plan_whole(f, b, e);
            } else {
                const bool fst = d.ss >= d.line;
                if (has && fst)
                    f.total += d.se - d.ss;
                plan_range(f, fst, d.ss - d.line, d.se - d.line < 4096u ? d.se - d.line : 4096u, b, e);
                if (has)
                    edge_words(win, lds0 + sa, lds0 + sb, e);
                __builtin_amdgcn_s_waitcnt(0xC07F);
            }
            fire_rows(rs, lds0 + sa, rv);               // line k+1 into line k-1's slot
#ifdef BRB_LINE_STAMPS
            uint64_t *idle = &p_wait;
#else
            uint64_t *idle = nullptr;
#endif
            const bool emitted = all_whole ? emit_line<RW, true, true>(f, e, dw, has, &cpx[pr][lane], &wpx[pr][lane], idle)
                                           : emit_line<RW, false, true>(f, e, dw, has, &cpx[pr][lane], &wpx[pr][lane], idle);
            if (!emitted) {
                ok = false;
                break;
            }
            pc_beat(&ev[pr][3], ++beats);
            sa = sb;
        }
        brb_dma::wait_vmcnt<0>();                       // the stray stage past K, before the slots are reused
        if (!ok)
            return;                                     // reported by the consumer (it stops getting words)
        fin[pr][0][lane] = uint32_t(f.acc) | (f.nacc << 24);
        fin[pr][1][lane] = uint32_t(f.total);
        fin[pr][2][lane] = uint32_t(f.total >> 32);
        pc_publish(&ev[pr][0], ++pev);                  // the group's end
#ifdef BRB_LINE_STAMPS
        if (lane == 0 && valid) {
            const uint4 v = make_uint4(uint32_t(p_wait), uint32_t(p_dma), uint32_t(__builtin_amdgcn_s_memtime() - p_t0), K);
            __builtin_memcpy(out + 16 * rec, &v, 16);
        }
#endif
    }
}

}  // namespace

namespace brb {

hipError_t launch_md5_segments(const uint8_t *data, const uint64_t *soff, const uint32_t *slen, const uint64_t *first,
                               uint64_t n_rec, uint8_t *out, hipStream_t s)
{
    if (n_rec == 0)
        return hipSuccess;
    if (brb_opt::get(brb_opt::kSegLine) == 0) {
        md5_seg_kernel<<<unsigned((n_rec + kBlock - 1) / kBlock), kBlock, 0, s>>>(data, soff, slen, first, n_rec, out);
        return hipGetLastError();
    }
    const uint64_t groups = (n_rec + 63) / 64;
    if (brb_opt::get(brb_opt::kSegLine) == 2) {
        constexpr int NP = 4;                          // 4 pairs, 159 KiB of LDS: one workgroup per CU
        const uint64_t wgs = (groups + NP - 1) / NP;
        const unsigned grid = unsigned(wgs < brb_digest::device_cu_count() ? wgs : brb_digest::device_cu_count());
        if (brb_opt::get(brb_opt::kPairStall) != 0)
            md5_seg_pc_kernel<NP, true><<<grid, 128 * NP, 0, s>>>(data, soff, slen, first, n_rec, out, brb::pair_fault_word());
        else
            md5_seg_pc_kernel<NP, false><<<grid, 128 * NP, 0, s>>>(data, soff, slen, first, n_rec, out, brb::pair_fault_word());
        return hipGetLastError();
    }
    constexpr int W = 4;                               // 4 x (8 NS + 14) KiB of LDS: one workgroup per CU
    const uint64_t wgs = (groups + W - 1) / W;
    const unsigned grid = unsigned(wgs < brb_digest::device_cu_count() ? wgs : brb_digest::device_cu_count());
    // two slots by default: 40.6 vs 41.2 us with three (bench --op md5seg, interleaved A/B,
    // gpurun_out/r04s_seg); test option line_slots 3 for the other
    if (brb_opt::get(brb_opt::kLineSlots) != 3)
        md5_seg_line_kernel<W, 2><<<grid, 64 * W, 0, s>>>(data, soff, slen, first, n_rec, out);
    else
        md5_seg_line_kernel<W, 3><<<grid, 64 * W, 0, s>>>(data, soff, slen, first, n_rec, out);
    return hipGetLastError();
}

}  // namespace brb
