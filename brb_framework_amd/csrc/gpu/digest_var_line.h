// digest_var_line.h -- lane-per-record digest (MD5, SHA-1) of records given by byte offsets and
// lengths (BRB_MD5Batch / BrbSha1_Batch), with the line-aligned LDS-DMA staging of digest_line.h.
//
// What differs from the fixed-stride kernel:
//  * Each group of 64 records gets its own buffer descriptor, 4 KiB below the lowest 128-byte line
//    its records touch; a DMA lane learns its row's line and line count from that row's lane
//    (ds_bpermute).  A group whose lines span 2 GiB or more (32-bit voffsets) is digested by the
//    per-lane block reader instead (digest_lane).
//  * Records start at any byte: the window is read one dword wider and funnel-shifted by the
//    record's byte offset (one v_alignbit_b32 per word; a 4-byte aligned record shifts by 0).
//  * Records have their own lengths: the group runs to its longest record; a row whose record has
//    no line left gets an out-of-range voffset (the DMA returns zeros without touching memory), a
//    lane compresses only its own blocks, and the tail block (if any) is stashed in registers when
//    it passes through the window and finished for all lanes at the end of the group.
// Record r's digest = BRB_MD5Init/Update/Final (md5.c:38-168) or BrbSha1_Do (sha1.c:203-216) of
// data[offs[r] .. offs[r] + lens[r]).
#pragma once

#include "byte_stream.h"
#include "digest_line.h"
#include "test_options.h"

namespace brb_digest {

// The per-lane path (and the fallback of the line kernel): 64-byte blocks, the next one in flight.
template <class Alg>
BRB_DEV typename Alg::State digest_lane(const uint8_t *a, uint64_t len)
{
    typename Alg::State st = Alg::iv();
    brb_io::BlockSrc src;
    src.init(a, len);
    uint32_t w[16];
    for (uint64_t b = 0; b < (len >> 6); ++b) {
        src.fetch(w);
        Alg::compress(st, w);
    }
    src.fetch(w);                   // tail (bytes past the record read as 0)
    brb_io::add_marker(w, len);
    Alg::finish(st, w, uint32_t(len & 63), len);
    return st;
}

BRB_DEV uint64_t uniform64(uint64_t v)
{
    return (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(v >> 32))))) << 32) |
           uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(v))));
}

BRB_DEV uint64_t wave_min64(uint64_t v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const uint64_t o = __shfl_xor(v, m, 64);
        v = o < v ? o : v;
    }
    return v;
}

BRB_DEV uint64_t wave_max64(uint64_t v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const uint64_t o = __shfl_xor(v, m, 64);
        v = o > v ? o : v;
    }
    return v;
}

// ---- Bucketing of variable-length batches by length (SURVEY §7 "Hard parts").  A group of 64 lanes
// runs to its longest record, so 64 consecutive records of lengths U[1000, 2000] cost ~1.33x their
// mean.  Records are therefore grouped by length inside CHUNKS of CG groups (64 CG consecutive
// records): the chunk's records are ranked by a bucket of their 2-block iteration count (stable:
// equal buckets keep record order), and group j of the chunk takes ranks [64 j, 64 j + 64).  Every
// wave that takes a group of the chunk computes the same ranking on its own -- ballots, mbcnt and
// scalar popcounts are deterministic -- so no wave waits for another and the ticketed groups stay
// as they are.  Digests go to each record's own slot (caller order).  Cost: one coalesced load of
// the chunk's lengths, NB x CG ballots, one LDS scatter/gather per group (~200 instructions against
// ~8 000 per group of 1 500-byte records).
constexpr uint32_t kSortCG = 4;       // groups per chunk: 256 records
constexpr uint32_t kSortNB = 8;       // buckets

// Record of lane `lane` in group g (chunk c = g / kSortCG, j = g % kSortCG), or ~0 when that rank
// holds no record (past n_rec).  `scratch`: this wave's 4 * 64 * kSortCG bytes of LDS.
// The slice a group takes is rotated by its round t = g / gridDim.x: workgroup b owns groups
// b + t gridDim.x, all with the same g mod kSortCG (gridDim.x is a multiple of it), so without the
// rotation one workgroup in kSortCG took every chunk's longest slice in every round and set the
// kernel time (measured: no gain at all on 524 288 records).  The groups of one chunk share t, so
// the rotation is a bijection of the slices the chunk's groups take -- of all kSortCG in a whole
// chunk, and of slices 0 .. pc-1 in a last chunk of pc < kSortCG groups: its records rank first
// (a missing record is keyed into the last bucket, behind every real one of that bucket), so they
// fill exactly slices 0 .. pc-1.  (Rotating over all kSortCG there sent a group to an empty slice
// and left a slice of real records undigested)
BRB_DEV uint64_t sorted_record(uint64_t g, uint32_t lane, const uint32_t *__restrict__ lens, uint64_t n_rec,
                               uint32_t *scratch)
{
    const uint64_t cg = (g / kSortCG) * kSortCG;              // the chunk's first group
    const uint64_t c0 = cg * 64;
    const uint64_t left = (n_rec + 63) / 64 - cg;             // groups of this chunk (>= 1)
    const uint32_t pc = left < kSortCG ? uint32_t(left) : kSortCG;
    const uint32_t j = uint32_t((g % kSortCG + g / gridDim.x) % pc);
    uint32_t it[kSortCG];
    bool ok[kSortCG];
    uint32_t lo = 0xFFFFFFFFu, hi = 0;
#pragma unroll
    for (uint32_t v = 0; v < kSortCG; v++) {
        const uint64_t idx = c0 + 64 * v + lane;
        ok[v] = idx < n_rec;
        const uint32_t len = ok[v] ? lens[idx] : 0u;
        const uint32_t nb = (len >> 6) + ((len & 63) ? 1u : 0u);
        it[v] = (nb >> 1) + (nb & 1);                          // the record's 2-block iterations
        lo = ok[v] && it[v] < lo ? it[v] : lo;
        hi = ok[v] && it[v] > hi ? it[v] : hi;
    }
    // wave-uniform range of the chunk's iteration counts
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const uint32_t a = uint32_t(__shfl_xor(int(lo), m, 64)), b = uint32_t(__shfl_xor(int(hi), m, 64));
        lo = a < lo ? a : lo;
        hi = b > hi ? b : hi;
    }
    lo = __builtin_amdgcn_readfirstlane(lo);
    hi = __builtin_amdgcn_readfirstlane(hi);
    const uint32_t span = hi > lo ? hi - lo : 0u;
    // bucket: iterations above the chunk's minimum, scaled onto kSortNB buckets when they span more
    // (one float multiply; the same inputs give every wave the same buckets); no record: last
    const float scale = span < kSortNB ? 1.0f : float(kSortNB - 1) / float(span);
    uint32_t key[kSortCG], pos[kSortCG];
#pragma unroll
    for (uint32_t v = 0; v < kSortCG; v++) {
        const uint32_t d = it[v] - lo;
        const uint32_t q = uint32_t(float(d) * scale + 0.5f);
        key[v] = !ok[v] ? kSortNB - 1 : (q < kSortNB ? q : kSortNB - 1);
        pos[v] = 0;
    }
    uint32_t base = 0;                                         // uniform: records in buckets < k
#pragma unroll
    for (uint32_t k = 0; k < kSortNB; k++) {
#pragma unroll
        for (uint32_t v = 0; v < kSortCG; v++) {
            const uint64_t m = __builtin_amdgcn_ballot_w64(key[v] == k);
            const uint32_t below = __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
            pos[v] = key[v] == k ? base + below : pos[v];
            base += uint32_t(__builtin_popcountll(m));
        }
    }
    // rank -> record through the wave's scratch
#pragma unroll
    for (uint32_t v = 0; v < kSortCG; v++)
        scratch[pos[v]] = ok[v] ? 64 * v + lane : 0xFFFFFFFFu;
    __builtin_amdgcn_s_waitcnt(0xC07F);                        // lgkmcnt(0): the scatter has landed
    __builtin_amdgcn_wave_barrier();
    const uint32_t e = scratch[64 * j + lane];
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    return e == 0xFFFFFFFFu ? ~uint64_t(0) : c0 + e;
}

// FIXED: record r = data[r * rec_len .. + rec_len) (offs / lens unused) -- fixed-stride batches
// whose records are not 4-byte aligned, which digest_line_kernel's dword window cannot take.
// SORT: groups bucketed by length inside chunks of kSortCG groups (sorted_record).
template <class Alg, int WAVES, bool OUT_ALIGNED, bool FIXED = false, bool SORT = false>
__global__ __launch_bounds__(64 * WAVES, 2) void digest_var_line_kernel(const uint8_t *__restrict__ data,
                                                                        const uint64_t *__restrict__ offs,
                                                                        const uint32_t *__restrict__ lens,
                                                                        uint32_t rec_len, uint64_t n_rec,
                                                                        uint8_t *__restrict__ out,
                                                                        uint64_t brb_first_sorted = 0)
{
    constexpr uint32_t SLOT = 8192;                            // 64 rows x one 128-byte line
    constexpr uint32_t OOB = 0x80000000u;                      // a voffset past every descriptor's range
    __shared__ __attribute__((aligned(16))) uint8_t ring[WAVES * 2 * SLOT];
    __shared__ uint32_t sort_scratch[SORT ? WAVES * 64 * kSortCG : 1];
    __shared__ uint32_t next_ticket;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t n_groups = (n_rec + 63) / 64;
    if (threadIdx.x == 0)
        next_ticket = WAVES;                                   // tickets 0 .. WAVES-1: one per wave
    __syncthreads();
    auto take = [&]() -> uint64_t {
        uint32_t tk = 0;
        if (lane == 0)
            tk = __hip_atomic_fetch_add(&next_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        tk = __builtin_amdgcn_readfirstlane(tk);
        return uint64_t(blockIdx.x) + uint64_t(tk) * gridDim.x;
    };
    uint64_t g = uint64_t(blockIdx.x) + uint64_t(wv) * gridDim.x;
    if (g >= n_groups)
        return;
    const uint32_t my_off = wv * 2 * SLOT;
    const uint32_t lds0 = uint32_t(reinterpret_cast<uintptr_t>(ring)) + my_off;
    const uint64_t dbase = reinterpret_cast<uint64_t>(data);
    auto swz = [](uint32_t row) { return (row >> 1) & 7; };

    // ---- one group's layout (Grp): this lane's record, and the group's descriptor and DMA lanes
    struct Grp {
        uint64_t a;          // address of this lane's record
        uint64_t r;          // its index (the digest's slot), ~0 for none
        uint32_t len;
        uint32_t K;          // 2-block iterations of the group (its longest record)
        bool line;           // false: the group's lines span >= 2 GiB, use digest_lane
        brb_dma::v4i rs;     // descriptor of the next line to issue
        uint32_t vq[8];      // DMA voffsets of rows 8q + lane / 8 (line 0 relative to the descriptor)
        uint32_t lq[8];      // lines of those rows' records
    };
    // Record of this lane in group g: caller order (64 g + lane), or, for SORT groups from
    // first_sorted on (0, or the end of the first round of tickets, 8 x gridDim.x: whole chunks
    // either way, gridDim.x being a multiple of kSortCG), the length-bucketed order of
    // sorted_record.  A group's ranking is computed while the group before it runs (the first
    // group's before its first DMA).  ~0: no record (past n_rec).
    const uint64_t first_sorted = brb_first_sorted;
    auto record_of = [&](uint64_t g) -> uint64_t {
        if (SORT && g >= first_sorted && g < n_groups)
            return sorted_record(g, lane, lens, n_rec, sort_scratch + wv * (64 * kSortCG));
        return g * 64 + lane < n_rec ? g * 64 + lane : ~uint64_t(0);
    };
    auto setup = [&](uint64_t g, uint64_t rec, Grp &G) {
        const uint64_t r = rec != ~uint64_t(0) ? rec : uniform64(g * 64);   // no record: empty, valid offset
        G.r = rec;
        G.a = dbase + (FIXED ? r * rec_len : offs[r]);
        G.len = FIXED ? rec_len : (rec != ~uint64_t(0) ? lens[r] : 0u);
        const uint64_t line = G.a & ~uint64_t(127);
        const uint32_t lines = G.len ? uint32_t(((G.a & 127) + G.len + 127) >> 7) : 0u;
        const uint32_t nblk = (G.len >> 6) + ((G.len & 63) ? 1u : 0u);
        // empty records touch no line (their offsets may point anywhere): they do not widen the span
        // (every lane holds the reduced values; readfirstlane tells the compiler they are uniform, so
        // the descriptor and the branches on them stay scalar)
        const uint64_t lo = uniform64(wave_min64(G.len ? line : ~uint64_t(0)));
        const uint64_t hi = uniform64(wave_max64(G.len ? line + 128 * uint64_t(lines) : 0));
        G.K = __builtin_amdgcn_readfirstlane(uint32_t(wave_max64((nblk + 1) >> 1)));
        G.line = hi > lo && hi - lo < (uint64_t(1) << 31) - (uint64_t(1) << 16);   // all empty: lane path
        const uint64_t base = lo - 4096;
        const uint64_t left = hi - base;
        G.rs.x = __builtin_amdgcn_readfirstlane(int(uint32_t(base)));
        G.rs.y = __builtin_amdgcn_readfirstlane(int(uint32_t(base >> 32) & 0xFFFF));
        G.rs.z = __builtin_amdgcn_readfirstlane(int(left > 0x7FFFFFFFull ? 0x7FFFFFFFu : uint32_t(left)));
        G.rs.w = 0x00020000;
        const uint32_t rel = uint32_t(line - lo);              // < 2^31 when G.line
        const uint32_t l3 = lane >> 3;
        const uint32_t g0 = 16u * ((lane & 7) ^ (l3 >> 1));   // swz(8q + l3) = (l3 >> 1) ^ 4 (q & 1)
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const int src = int(8 * q + l3) * 4;               // ds_bpermute byte address of row 8q + l3
            const uint32_t rrel = uint32_t(__builtin_amdgcn_ds_bpermute(src, int(rel)));
            G.lq[q] = uint32_t(__builtin_amdgcn_ds_bpermute(src, int(lines)));
            G.vq[q] = (rrel | (q & 1 ? g0 ^ 64u : g0)) + (4096u - 1024u * (q & 3));
        }
    };
    // keep_l2 (fixed stride only): a group's lines 0 and 1 use the temporal policy -- the previous
    // record's last lines are the same memory lines, read ~a group later (digest_line.h); the others
    // nt.  Measured: 1 501-byte records 24.5 -> 24.2 us; on the variable-length batch (random
    // offsets, no shared lines) 32.24 -> 32.33 us, so variable-length groups keep nt throughout.
    auto issue = [&](Grp &G, uint32_t m, uint32_t slot, bool keep_l2 = false) {   // line m of every row -> slot
        const uint32_t lm = lds0 + slot * SLOT;
        uint32_t v[8];
#pragma unroll
        for (int q = 0; q < 8; q++)
            v[q] = m < G.lq[q] ? G.vq[q] : OOB;
        uint32_t keep;
#define BRB_VLINE_DMA8(POL)                                                                     \
        asm volatile("s_mov_b32 %0, m0\n\t"                                                    \
                     "s_mov_b32 m0, %10\n\t"                                                   \
                     "s_nop 0\n\t"                                                             \
                     "buffer_load_dwordx4 %1, %9, 0 offen " POL "lds\n\t"                      \
                     "buffer_load_dwordx4 %2, %9, 0 offen offset:1024 " POL "lds\n\t"          \
                     "buffer_load_dwordx4 %3, %9, 0 offen offset:2048 " POL "lds\n\t"          \
                     "buffer_load_dwordx4 %4, %9, 0 offen offset:3072 " POL "lds\n\t"          \
                     "s_mov_b32 m0, %11\n\t"                                                   \
                     "s_nop 0\n\t"                                                             \
                     "buffer_load_dwordx4 %5, %9, 0 offen " POL "lds\n\t"                      \
                     "buffer_load_dwordx4 %6, %9, 0 offen offset:1024 " POL "lds\n\t"          \
                     "buffer_load_dwordx4 %7, %9, 0 offen offset:2048 " POL "lds\n\t"          \
                     "buffer_load_dwordx4 %8, %9, 0 offen offset:3072 " POL "lds\n\t"          \
                     "s_mov_b32 m0, %0"                                                         \
                     : "=&s"(keep)                                                              \
                     : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]), \
                       "s"(G.rs), "s"(lm), "s"(lm + 4096u)                                      \
                     : "memory")
        if (keep_l2)
            BRB_VLINE_DMA8("");
        else
            BRB_VLINE_DMA8("nt ");
#undef BRB_VLINE_DMA8
        const uint64_t b = ((uint64_t(uint32_t(G.rs.y)) << 32) | uint32_t(G.rs.x)) + 128u;
        G.rs.x = int(uint32_t(b));
        G.rs.y = int(uint32_t(b >> 32));
        int z = G.rs.z;
        asm("s_sub_i32 %0, %0, 0x80\n\ts_max_i32 %0, %0, 0" : "+s"(z) : : "scc");
        G.rs.z = z;
    };
    auto start = [&](Grp &G) {                                 // lines 0 and 1 of a line group
        if (G.line) {
            issue(G, 0, 0, FIXED);
            issue(G, 1, 1, FIXED);
        }
    };

    // window dword i (0..32) of this lane for lines (k-1, k) in slots (0, 1) [ae] and (1, 0) [ao]
    uint32_t ae[33], ao[33];
    auto win_setup = [&](const Grp &G) {
        const uint32_t sh4 = uint32_t(G.a) & 124u;
        const uint32_t fr = (my_off + lane * 128) | (swz(lane) << 4);
#pragma unroll
        for (uint32_t i = 0; i < 33; i++) {
            const uint32_t q4 = sh4 + 4 * i;                   // < 256
            ae[i] = ((q4 & 124u) ^ fr) | ((q4 & 128u) << 6);
            ao[i] = ae[i] ^ SLOT;
            asm volatile("" : "+v"(ao[i]));
        }
    };
    uint32_t w0[16], w1[16];
    auto read_window = [&](const uint32_t (&ad)[33], uint32_t fb) {
        uint32_t d[33];
#pragma unroll
        for (int i = 0; i < 33; i++)
            d[i] = *reinterpret_cast<const uint32_t *>(ring + ad[i]);
        __builtin_amdgcn_s_waitcnt(0xC07F);
#pragma unroll
        for (int i = 0; i < 16; i++) {
            w0[i] = __builtin_amdgcn_alignbit(d[i + 1], d[i], fb);
            w1[i] = __builtin_amdgcn_alignbit(d[i + 17], d[i + 16], fb);
        }
    };

    Grp G, Gn;
    setup(g, record_of(g), G);
    start(G);
    __builtin_amdgcn_sched_barrier(0);
    for (;;) {
        const uint64_t gn = take();
        const uint64_t rn = record_of(gn);                     // ranking of the next group, if sorted
        const uint64_t r = G.r;
        typename Alg::State st;
        if (!G.line) {
            st = digest_lane<Alg>(reinterpret_cast<const uint8_t *>(G.a), G.len);
            if (gn < n_groups) {
                setup(gn, rn, Gn);
                start(Gn);
            }
        } else {
            win_setup(G);
            const uint32_t fb = (uint32_t(G.a) & 3u) * 8u;
            const uint32_t nfull = G.len >> 6, t = G.len & 63;
            const uint32_t tb = t ? nfull : 0xFFFFFFFFu;       // the block holding the tail bytes
            uint32_t wt[16];                                   // that block, stashed as it passes
#pragma unroll
            for (int i = 0; i < 16; i++)
                wt[i] = 0;
            st = Alg::iv();
            const uint32_t K = G.K;
            auto step = [&](uint32_t k, const uint32_t (&ad)[33], uint32_t refill_slot) {
                brb_dma::wait_vmcnt<0>();
                read_window(ad, fb);
                if (k < K) {
                    issue(G, k + 1, refill_slot);
                } else if (gn < n_groups) {
                    setup(gn, rn, Gn);
                    start(Gn);
                }
                const uint32_t b = 2 * k - 2;
                if (b < nfull)
                    Alg::compress(st, w0);
                if (b + 1 < nfull)
                    Alg::compress(st, w1);
                if (__builtin_amdgcn_ballot_w64(tb - b < 2) != 0) {   // some lane's tail is in the window
#pragma unroll
                    for (int i = 0; i < 16; i++)
                        wt[i] = tb == b ? w0[i] : tb == b + 1 ? w1[i] : wt[i];
                }
            };
            if (K == 0) {                                      // every record of the group is empty
                brb_dma::wait_vmcnt<0>();
                if (gn < n_groups) {
                    setup(gn, rn, Gn);
                    start(Gn);
                }
            }
            for (uint32_t k = 1; k <= K; k += 2) {
                step(k, ae, 0);                                // odd k: line k+1 goes to slot 0
                if (k == K)
                    break;
                step(k + 1, ao, 1);                            // even k: line k+1 goes to slot 1
            }
            // padding, digest (md5.c:134-168): the lane's own tail length
            if (t == 0) {
                Alg::pad_only(st, G.len);
            } else {
#pragma unroll
                for (uint32_t i = 0; i < 16; i++) {
                    const uint32_t o = 4 * i;
                    const uint32_t keep = t > o ? (t - o < 4 ? t - o : 4) : 0;
                    uint32_t v = keep == 4 ? wt[i] : wt[i] & ((1u << (8 * keep)) - 1u);
                    if (t >= o && t < o + 4)
                        v |= 0x80u << (8 * (t - o));
                    wt[i] = v;
                }
                Alg::finish(st, wt, t, G.len);
            }
        }
        if (r != ~uint64_t(0))
            Alg::template store<OUT_ALIGNED>(out, r, st);
        g = gn;
        if (g >= n_groups)
            break;
        G = Gn;
    }
}

// One 8-wave workgroup per CU (128 KiB of LDS), groups handed out by tickets.
template <class Alg>
hipError_t launch_var_line(const uint8_t *data, const uint64_t *offs, const uint32_t *lens, uint64_t n_rec, uint8_t *out,
                           bool out_al, hipStream_t s)
{
    constexpr int W = 8;
    const uint64_t groups = (n_rec + 63) / 64;
    const unsigned g = unsigned(groups < device_cu_count() ? groups : device_cu_count());
    // bucketing pays only where waves take several groups (with one group per wave the batch's
    // longest record sets the time whatever the grouping): groups past the first round of tickets
    // (sorted_record's slice rotation needs whole chunks per round: gridDim.x % kSortCG == 0)
    const bool sort = brb_opt::get(brb_opt::kVarSort) != 0 && groups > uint64_t(g) * W && g % kSortCG == 0;
    // every group is bucketed, the first round of tickets too (measured on 524 288 records, bimodal
    // lengths: 698 us unsorted, 438 us with the first round in caller order, 372 us all sorted;
    // U[1000, 2000]: 200.8 / 200.0 / 197.5 us); test option var_sort = 2 keeps the first round in
    // caller order (A/B)
    const uint64_t first = brb_opt::get(brb_opt::kVarSort) == 2 ? uint64_t(g) * W : 0;
    if (sort && out_al)
        digest_var_line_kernel<Alg, W, true, false, true><<<g, 64 * W, 0, s>>>(data, offs, lens, 0, n_rec, out, first);
    else if (sort)
        digest_var_line_kernel<Alg, W, false, false, true><<<g, 64 * W, 0, s>>>(data, offs, lens, 0, n_rec, out, first);
    else if (out_al)
        digest_var_line_kernel<Alg, W, true><<<g, 64 * W, 0, s>>>(data, offs, lens, 0, n_rec, out);
    else
        digest_var_line_kernel<Alg, W, false><<<g, 64 * W, 0, s>>>(data, offs, lens, 0, n_rec, out);
    return hipGetLastError();
}

template <class Alg>
hipError_t launch_fixed_var_line(const uint8_t *data, uint32_t rec_len, uint64_t n_rec, uint8_t *out, bool out_al,
                                 hipStream_t s)
{
    constexpr int W = 8;
    const uint64_t groups = (n_rec + 63) / 64;
    const unsigned g = unsigned(groups < device_cu_count() ? groups : device_cu_count());
    if (out_al)
        digest_var_line_kernel<Alg, W, true, true><<<g, 64 * W, 0, s>>>(data, nullptr, nullptr, rec_len, n_rec, out);
    else
        digest_var_line_kernel<Alg, W, false, true><<<g, 64 * W, 0, s>>>(data, nullptr, nullptr, rec_len, n_rec, out);
    return hipGetLastError();
}

// Test option "var_line" = 0 keeps variable-length batches on the per-lane kernel (A/B measurements).
inline bool var_line_enabled()
{
    return brb_opt::get(brb_opt::kVarLine) != 0;
}

}  // namespace brb_digest
