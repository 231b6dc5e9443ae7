// line_r05_kernel.h -- the round-5 line digest kernel, frozen for A/B measurements (tools/mb only;
// the library does not include it).  It still carries the two forms that measured slower and left
// the product in round 6: POOL, the chip-wide tail pool (profiles/r05/ab/pool:
// 286.7 us without, 288.5-291.3 us with 4-16 rounds pooled), and LOCK, SIMD partners in lockstep
// (profiles/r05/ab/lock*: within 0.4-0.7 %, box noise).  It also keeps round 5's per-group window
// and DMA-offset setup, the baseline of round 6's hoisted form.
//
// Kernel arguments as in round 5: (data, rec_len, n_rec, out, pool heads, t_own).
#pragma once

#include <atomic>
#include <mutex>

#include "dma_stage.h"
#include "test_options.h"

// Diagnostic hooks (tools/mb/line_probe.hip defines them; empty in the product build).
#ifndef BRB_LINE_PROBE
#define BRB_LINE_PROBE_DECL
#define BRB_LINE_PROBE(ev) ((void)0)
#endif

namespace brb_mb_r05 {

// Padding, digest and store of one group: the record's tail block (if any) is window half
// nfull - (2K - 2) of the last iteration; bytes past the record are masked (md5.c:134-168).  The
// tail's per-dword keep masks and 0x80 marker (tm, tp) depend only on rec_len: they are built once
// per wave (tail_masks) while the first lines are in flight, so a group pays 16 v_and_or here.
template <class Alg, bool OUT_ALIGNED>
BRB_DEV void line_finish(typename Alg::State &st, const uint32_t (&w0)[16], const uint32_t (&w1)[16],
                         const uint32_t (&tm)[16], const uint32_t (&tp)[16], uint32_t t, uint32_t nfull, uint32_t K,
                         uint32_t rec_len, uint8_t *out, uint64_t r, uint64_t n_rec)
{
    if (t == 0) {
        Alg::pad_only(st, rec_len);                            // the padding block is a constant
        if (r < n_rec)
            Alg::template store<OUT_ALIGNED>(out, r, st);
        return;
    }
    uint32_t w[16];
    const bool second = nfull + 2 - 2 * K;                     // uniform: which half holds the tail
#pragma unroll
    for (int i = 0; i < 16; i++)
        w[i] = ((second ? w1[i] : w0[i]) & tm[i]) | tp[i];
    Alg::finish(st, w, t, rec_len);
    if (r < n_rec)
        Alg::template store<OUT_ALIGNED>(out, r, st);
}

// Keep mask and marker of tail dword i for a tail of t bytes (0 < t < 64): bytes below t kept,
// 0x80 at byte t, zeros after.  Kept in VGPRs (asm barrier) so that no group recomputes them.
BRB_DEV void tail_masks(uint32_t t, uint32_t (&tm)[16], uint32_t (&tp)[16])
{
#pragma unroll
    for (uint32_t i = 0; i < 16; i++) {
        const uint32_t o = 4 * i;
        const uint32_t keep = t > o ? (t - o < 4 ? t - o : 4) : 0;
        tm[i] = uint32_t((uint64_t(1) << (8 * keep)) - 1);
        tp[i] = t >= o && t < o + 4 ? 0x80u << (8 * (t - o)) : 0u;
        asm volatile("" : "+v"(tm[i]), "+v"(tp[i]));
    }
}

// Group assignment.  Static (DYN = false): wave w of the grid takes groups w, w + W_total, ...
// Dynamic (DYN = true): workgroup b owns groups b, b + G, b + 2G, ... (G = gridDim.x) and its waves
// take them one at a time from an LDS ticket counter.  Why: with two waves per SIMD the older wave
// wins the issue arbitration, so under a static split the first workgroup of every CU finished its
// share at ~190 us and the second one ran alone (at the lone-wave issue rate) until ~300 us
// (1 Mi x 1500 B, tools/mb/line_probe.hip); with tickets the faster wave simply takes more groups.
// launch_bounds: two waves per SIMD (4-wave workgroups: two per CU, 64 KiB of LDS each; 8-wave
// workgroups: one per CU, 128 KiB).
//
// POOL (with DYN; round 5): the tail of the batch is balanced across the chip.
// A workgroup's LDS tickets cover only its first `t_own` rounds of groups (b + t G, t < t_own); the
// groups after them form a pool split over kPoolHeads heads in HBM (pool_head), head h holding pool
// groups h, h + 8, ...  A wave whose workgroup has no ticket left takes pool groups from the head
// of its own XCD (HW_REG_XCC_ID) and, once that one is empty, sweeps the other heads (an LDS mask
// of heads the workgroup found empty saves the repeat).  Why: the workgroups of a static split end
// between 257 and 291 us (1 Mi x 1500 B, profiles/r03/line_probe_cfg5.txt), the odd XCDs 5-13 us
// behind the even ones, while the kernel is issue-bound: a CU that is done early idles its SIMDs.
// Round 3's pool (one head, one device-scope atomic per group, its return waited on with the first
// line pair) cost 3-22 us; here the first pool ticket of a group is requested right after iteration
// 1's refill, so its return lands while blocks 0-1 are hashed, and 8 heads spread the atomics.
// The heads of a launch are zeroed by its last workgroup (one device-scope count per workgroup), so
// the next launch given the same slot (launch_fixed_line: a ring of kPoolSlots per device) starts
// from zero.
constexpr uint32_t kPoolHeads = 8;
constexpr uint32_t kPoolStride = 64;                           // u32: heads 256 B apart
constexpr uint32_t kPoolSlotWords = (kPoolHeads + 1) * kPoolStride;   // the heads, then the done count
constexpr uint32_t kPoolSlots = 512;

// LOCK (with a static split, DYN = false; round 5): the two waves that share a SIMD progress in
// lockstep.  Each wave publishes its iteration count in LDS and reads its SIMD partner's (the other
// wave of the workgroup with the same HW_REG_HW_ID SIMD id) once per iteration; the wave that is
// ahead by more than one iteration drops to issue priority 0, the one behind rises to 2.  Why: at
// two waves per SIMD the older wave wins the issue arbitration, and a static split then ends with
// one wave of every SIMD running alone; with tickets (DYN) the last groups are handed out a group
// early and the workgroup's waves end one group-time apart (profiles/r05/ab/pool/lprobe_pool.txt:
// per-WG end spread p50 30 us).  With equal shares (groups a multiple of the grid's waves) and
// equal progress every wave of a CU ends at about the same time.
template <class Alg, int WAVES, bool OUT_ALIGNED, bool NT = false, bool DYN = false, bool POOL = false,
          bool LOCK = false>
__global__ __launch_bounds__(64 * WAVES, 2) void digest_line_kernel(const uint8_t *__restrict__ data,
                                                                             uint32_t rec_len, uint64_t n_rec,
                                                                             uint8_t *__restrict__ out,
                                                                             uint32_t *__restrict__ pool,
                                                                             uint32_t t_own)
{
    constexpr uint32_t SLOT = 8192;                            // 64 rows x one 128-byte line
    __shared__ __attribute__((aligned(16))) uint8_t ring[WAVES * 2 * SLOT];
    __shared__ uint32_t next_ticket;
    __shared__ uint32_t pool_empty, waves_done;                // POOL: heads found empty; waves finished
    __shared__ uint32_t lock_simd[WAVES], lock_prog[WAVES];    // LOCK: each wave's SIMD and iterations
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t partner = WAVES;                                  // LOCK: the wave sharing this SIMD (WAVES: none)
    uint32_t prog = 0;
    if (LOCK) {
        uint32_t hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        if (lane == 0) {
            lock_simd[wv] = (__builtin_amdgcn_readfirstlane(hw) >> 4) & 3u;
            lock_prog[wv] = 0;
        }
        __syncthreads();
        const uint32_t me = lock_simd[wv];
        for (uint32_t w = 0; w < uint32_t(WAVES); w++)
            if (w != wv && lock_simd[w] == me && partner == uint32_t(WAVES))
                partner = w;
        partner = __builtin_amdgcn_readfirstlane(partner);
    }
    // LOCK: publish this wave's progress and read the partner's (issued before the iteration's waits,
    // used after its window read); then set the issue priority from the difference
    auto lock_pub = [&]() -> uint32_t {
        if (!LOCK || partner >= uint32_t(WAVES))
            return 0;
        ++prog;
        __hip_atomic_store(&lock_prog[wv], prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return __hip_atomic_load(&lock_prog[partner], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    // The lower-numbered wave of a pair is held `t_own` iterations ahead of its partner, not level
    // with it: level partners wait for their lines at the same moments, apart each one's wait falls
    // in the other's compression (cfg5: level 289.9 -> 290.1 us, one iteration 285.5 -> 283.5 us).
    // LOCK: t_own = lead (iterations, bits 0-7) | slack << 8 (the drift left to the arbitration)
    const int lock_target = wv < partner ? int(t_own & 255u) : -int(t_own & 255u);
    const int lock_slack = int(t_own >> 8);
    auto lock_prio = [&](uint32_t other) {
        if (!LOCK || partner >= uint32_t(WAVES))
            return;
        const int d = int(prog - __builtin_amdgcn_readfirstlane(other)) - lock_target;
        if (d > lock_slack)
            __builtin_amdgcn_s_setprio(0);
        else if (d < -lock_slack)
            __builtin_amdgcn_s_setprio(2);
        else
            __builtin_amdgcn_s_setprio(1);
    };
    const uint64_t n_groups = (n_rec + 63) / 64;
    const uint64_t wave0 = uint64_t(blockIdx.x) * WAVES + wv;
    const uint64_t wstride = uint64_t(gridDim.x) * WAVES;
    if (DYN) {
        if (threadIdx.x == 0) {
            next_ticket = WAVES;                               // tickets 0 .. WAVES-1: one per wave
            pool_empty = 0;
            waves_done = 0;
        }
        __syncthreads();
    }
    // POOL: groups [own_end, n_groups) are pooled; pool group p = own_end + p, head p % 8.
    const uint64_t own_end = POOL ? uint64_t(t_own) * gridDim.x : n_groups;
    const uint64_t pool_n = POOL && own_end < n_groups ? n_groups - own_end : 0;
    uint32_t home = 0;
    if (POOL)
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(home));
    home = __builtin_amdgcn_readfirstlane(home) & (kPoolHeads - 1);
    // One pool ticket from head h (lane 0's vector atomic, device scope): the returned index, or
    // UINT32_MAX past the head's share.  Its return is waited on where the value is first used.
    auto pool_fetch = [&](uint32_t h) -> uint32_t {
        uint32_t v = 0;
        if (lane == 0)
            v = __hip_atomic_fetch_add(pool + h * kPoolStride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return v;
    };
    auto pool_group = [&](uint32_t h, uint32_t v) -> uint64_t {   // n_groups when head h is exhausted
        v = __builtin_amdgcn_readfirstlane(v);
        const uint64_t p = uint64_t(v) * kPoolHeads + h;
        const uint64_t r = p < pool_n ? own_end + p : n_groups;
        return (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(r >> 32))))) << 32) |
               uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(r))));
    };
    auto home_open = [&]() {                                   // home head not yet found empty
        return !(__builtin_amdgcn_readfirstlane(__hip_atomic_load(&pool_empty, __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_WORKGROUP)) & (1u << home));
    };
    // The rest of the sweep, synchronous (only once the home head is empty: the end of the launch).
    auto pool_sweep = [&](uint32_t h0) -> uint64_t {
        __hip_atomic_fetch_or(&pool_empty, 1u << h0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        uint64_t gp = n_groups;
        for (uint32_t i = 1; i < kPoolHeads; i++) {
            const uint32_t h = (h0 + i) & (kPoolHeads - 1);
            const uint32_t known = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(&pool_empty, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
            if (gp < n_groups || (known & (1u << h)))
                continue;
            gp = pool_group(h, pool_fetch(h));
            if (gp >= n_groups)                                // every lane: an idempotent LDS or
                __hip_atomic_fetch_or(&pool_empty, 1u << h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        return gp;
    };
    auto take = [&]() -> uint64_t {                            // DYN: the next group of this workgroup
        uint32_t tk = 0;
        if (lane == 0)
            tk = __hip_atomic_fetch_add(&next_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        tk = __builtin_amdgcn_readfirstlane(tk);
        const uint64_t gt = uint64_t(blockIdx.x) + uint64_t(tk) * gridDim.x;
        return POOL && gt >= own_end ? ~uint64_t(0) : gt;     // POOL: ~0 = "from the pool"
    };
    // POOL epilogue: every wave counts itself out; the workgroup's last wave counts the workgroup out
    // and the launch's last workgroup zeroes the heads and the count for the slot's next launch.
    auto pool_done = [&]() {
        if (!POOL)
            return;
        uint32_t last = 0;
        if (lane == 0)
            last = __hip_atomic_fetch_add(&waves_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == WAVES - 1;
        if (!__builtin_amdgcn_readfirstlane(last))
            return;
        uint32_t wg_last = 0;
        if (lane == 0)
            wg_last = __hip_atomic_fetch_add(pool + kPoolHeads * kPoolStride, 1u, __ATOMIC_ACQ_REL,
                                             __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
        if (__builtin_amdgcn_readfirstlane(wg_last) && lane <= kPoolHeads)
            __hip_atomic_store(pool + lane * kPoolStride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    uint64_t g = DYN ? uint64_t(blockIdx.x) + uint64_t(wv) * gridDim.x : wave0;
    if (POOL && g >= own_end && g < n_groups) {               // fewer own rounds than waves
        g = pool_group(home, pool_fetch(home));
        if (g >= n_groups)
            g = pool_sweep(home);
    }
    if (g >= n_groups) {
        pool_done();
        return;
    }
    const uint32_t my_off = wv * 2 * SLOT;                     // slot 0; slot 1 = my_off + SLOT (bit 13 clear)
    const uint32_t lds0 = uint32_t(reinterpret_cast<uintptr_t>(ring)) + my_off;
    const uint32_t nfull = rec_len >> 6, t = rec_len & 63;
    const uint32_t nblk = nfull + (t ? 1 : 0);
    const uint32_t K = (nblk + 1) >> 1;                        // 2-block iterations per group; K + 1 lines
    const uint64_t dbase = reinterpret_cast<uint64_t>(data);
    const uint64_t end_line = (dbase + n_rec * rec_len + 127) & ~uint64_t(127);
    // 16-byte granule swizzle of a 128-byte row (applied on the DMA source): ds_read_b128 of one
    // logical granule by all lanes is conflict-free, ds_read_b32 of one logical dword 4-way at worst.
    auto swz = [](uint32_t row) { return (row >> 1) & 7; };

    // ---- issue side: DMA lane j of instruction q stages granule j % 8 of row 8q + j / 8 of the
    // issuing group's next line.  One M0 write serves four DMAs: DMA q carries the instruction
    // offset 1024 (q % 4), which lands in the LDS address as well, and its voffset is lowered by the
    // same amount.  The descriptor base sits 4 KiB below the line (and num_records 4 KiB above the
    // bytes left), so every voffset stays >= 1024 whatever the record length or group size: one DMA
    // form for every group, no per-DMA M0 writes.
    uint32_t vq[8], vqn[8];                                    // this group's, the next group's
    // Descriptor of a group: base = the group's first line - 4096, num_records = 4096 + bytes from
    // that line to end_line, clamped to [0, 2^31 - 1].  Set once per group (dma_setup); line j of
    // the group is addressed by soffset = 128 j, one scalar add per issue (round 3: the per-line
    // descriptor advance took four scalar ops plus hipcc's copies).  A group at least 2^31 - 4097
    // bytes from the end has num_records 2^31 - 1, above every offset of its K + 1 lines
    // (line_supported caps rec_len at 1 MiB: offsets < 64 MiB + 8 KiB).
    brb_dma::v4i rs, rsn;
    // The next group's offsets and descriptor go to vqn / rsn (taken over once per group): written
    // into vq / rs inside the loop, they made hipcc copy all eight offsets on every iteration.
    auto dma_setup = [&](uint64_t g, uint32_t (&vq)[8], brb_dma::v4i &rs) {
        const uint64_t r0 = g * 64;
        const uint32_t last = uint32_t(n_rec - r0 < 64 ? n_rec - r0 - 1 : 63);
        const uint64_t a0 = dbase + r0 * rec_len;
        const uint64_t gbase = (a0 & ~uint64_t(127)) - 4096;
        const uint64_t gleft = end_line - gbase;
        rs.x = __builtin_amdgcn_readfirstlane(int(uint32_t(gbase)));
        rs.y = __builtin_amdgcn_readfirstlane(int(uint32_t(gbase >> 32) & 0xFFFF));
        rs.z = __builtin_amdgcn_readfirstlane(int(gleft > 0x7FFFFFFFull ? 0x7FFFFFFFu : uint32_t(gleft)));
        rs.w = 0x00020000;
        // DMA q stages row 8q + lane/8 (rows past `last` re-stage row `last`): its line offset is
        // min(row, last) * rec_len = min(row * rec_len, last * rec_len), one multiply per group; and
        // swz(8q + l3) = (l3 >> 1) ^ 4(q & 1), so the granule swizzle takes two values.  4 VALU per DMA.
        const uint32_t o0 = uint32_t(a0) & 127;
        const uint32_t l3 = lane >> 3;
        const uint32_t base = o0 + l3 * rec_len, cap = o0 + last * rec_len;
        const uint32_t g0 = 16u * ((lane & 7) ^ (l3 >> 1));
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const uint32_t x = base + 8u * q * rec_len;
            vq[q] = (((x < cap ? x : cap) & ~127u) | (q & 1 ? g0 ^ 64u : g0)) + (4096u - 1024u * (q & 3));
        }
    };
    // Lines 0 and 1 of a group go through the L2 with the normal (temporal) policy, the others
    // non-temporal: record r's last line or two are record r+1's first ones, read by the same wave
    // ~17 us later, and with every line nt the L2 had dropped them (cfg2 fetched 105.3 MB for 98.3 MB
    // of records).  Round 3: 94.9 MB fetched, cfg2 21.49 -> 20.99 us, the 1 Mi-record shard 300.4 ->
    // 288.7 us (interleaved A/B).
    // soffset of the next line to issue (the descriptor stays put for the whole group; the range
    // check covers voffset + soffset + the instruction offset, per dword: tools/mb/buf_range.hip).
    uint32_t so = 0, son = 0;
    auto issue = [&](const uint32_t (&vq)[8], const brb_dma::v4i &rs, uint32_t &so, uint32_t slot, bool keep_l2 = false) {   // next line -> slot
#ifdef BRB_LINE_NO_DMA      // diagnostic builds only (tools/mb/line_parts.hip): hash stale LDS
        return;
#endif
        const uint32_t m = lds0 + slot * SLOT;
        uint32_t keep;
#define BRB_LINE_DMA8(POL)                                                                      \
    asm volatile("s_mov_b32 %0, m0\n\t"                                                          \
                 "s_mov_b32 m0, %10\n\t"                                                         \
                 "s_nop 0\n\t"                                                                   \
                 "buffer_load_dwordx4 %1, %9, %12 offen " POL "lds\n\t"                         \
                 "buffer_load_dwordx4 %2, %9, %12 offen offset:1024 " POL "lds\n\t"             \
                 "buffer_load_dwordx4 %3, %9, %12 offen offset:2048 " POL "lds\n\t"             \
                 "buffer_load_dwordx4 %4, %9, %12 offen offset:3072 " POL "lds\n\t"             \
                 "s_mov_b32 m0, %11\n\t"                                                         \
                 "s_nop 0\n\t"                                                                   \
                 "buffer_load_dwordx4 %5, %9, %12 offen " POL "lds\n\t"                         \
                 "buffer_load_dwordx4 %6, %9, %12 offen offset:1024 " POL "lds\n\t"             \
                 "buffer_load_dwordx4 %7, %9, %12 offen offset:2048 " POL "lds\n\t"             \
                 "buffer_load_dwordx4 %8, %9, %12 offen offset:3072 " POL "lds\n\t"             \
                 "s_mov_b32 m0, %0"                                                               \
                 : "=&s"(keep)                                                                    \
                 : "v"(vq[0]), "v"(vq[1]), "v"(vq[2]), "v"(vq[3]), "v"(vq[4]), "v"(vq[5]), "v"(vq[6]), \
                   "v"(vq[7]), "s"(rs), "s"(m), "s"(m + 4096u), "s"(so)                           \
                 : "memory")
        if (NT && !keep_l2)
            BRB_LINE_DMA8("nt ");
        else
            BRB_LINE_DMA8("");
#undef BRB_LINE_DMA8
        so += 128;                                             // the line after the issued one
    };

    // ---- read side: window dword i of this lane -> LDS offset, for lines (k-1, k) in slots
    // (0, 1) ["ae", k odd] and (1, 0) ["ao", k even]
    uint32_t ae[32], ao[32];
    auto win_setup = [&](uint64_t g) {
        const uint64_t r0 = g * 64;
        const uint32_t last = uint32_t(n_rec - r0 < 64 ? n_rec - r0 - 1 : 63);
        const uint32_t o0 = uint32_t(dbase + r0 * rec_len) & 127;
        const uint32_t rr = lane < last ? lane : last;
        const uint32_t sh4 = (o0 + rr * rec_len) & 127;        // 4 x the record's dword shift
        // Stream dword q = sh + i sits at row byte ((4q mod 128) ^ 16 swz) of slot q >= 32: with
        // fr = row base | 16 swz (disjoint bits), one xor, one or and the slot bit.
        const uint32_t fr = (my_off + lane * 128) | (swz(lane) << 4);
#pragma unroll
        for (uint32_t i = 0; i < 32; i++) {
            const uint32_t q4 = sh4 + 4 * i;                   // < 256
            ae[i] = ((q4 & 124u) ^ fr) | ((q4 & 128u) << 6);   // SLOT = 128 << 6
            ao[i] = ae[i] ^ SLOT;                              // slot 0 has bit 13 clear
            asm volatile("" : "+v"(ao[i]));                    // keep both tables (hipcc would re-derive
        }                                                      // ao with 32 XORs per iteration)
    };

    uint32_t w0[16], w1[16];
    auto read_window = [&](const uint32_t (&ad)[32]) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            w0[i] = *reinterpret_cast<const uint32_t *>(ring + ad[i]);
            w1[i] = *reinterpret_cast<const uint32_t *>(ring + ad[16 + i]);
        }
        // window in VGPRs before its slot is refilled: lgkmcnt(0) (vmcnt 63, expcnt 7 = no wait).
        // The builtin, not inline asm: the compiler's waitcnt pass then knows the reads are done and
        // inserts no waits of its own before their uses.
        __builtin_amdgcn_s_waitcnt(0xC07F);
    };

    BRB_LINE_PROBE_DECL
    BRB_LINE_PROBE(0);
    dma_setup(g, vq, rs);
    issue(vq, rs, so, 0, true);
    issue(vq, rs, so, 1, true);
    // Everything else of the prologue runs while the first two lines are in flight: without the
    // barrier hipcc hoisted the window tables (~300 VALU) above the first DMA.
    __builtin_amdgcn_sched_barrier(0);
    uint64_t gn = DYN ? take() : g + wstride;                  // the group after g
    // POOL: gn == ~0 -> the head's ticket is requested in iteration 1 (pv) and resolved at the end
    uint32_t pv = 0;
    bool pv_pending = false;
    win_setup(g);
    uint32_t tm[16], tp[16];
    tail_masks(t, tm, tp);
    // One iteration k (1 <= k <= K): wait for line k, read the window (lines k-1, k), refill the
    // slot of line k-1 with line k+1 (at k = K: start the next group's lines 0 and 1), hash blocks
    // 2k-2 and 2k-1.  Iterations k < K always refill and always hash two whole blocks
    // (2k - 1 <= 2K - 3 < nfull), so they run branch-free in a loop unrolled by two (each parity
    // reads with its own address table: four compress sites, which the shared instruction cache
    // holds; unrolling the whole record did not fit).  The last iteration is peeled:
    // it alone starts the next group and checks which blocks are whole.  Round 3: the peeled form
    // issues ~18 fewer scalar/branch instructions per iteration than one loop with the checks.
    auto full_step = [&](typename Alg::State &st, const uint32_t (&ad)[32], uint32_t refill_slot) {
        BRB_LINE_PROBE(1);
        const uint32_t other = lock_pub();
        brb_dma::wait_vmcnt<0>();
        read_window(ad);
        lock_prio(other);
        BRB_LINE_PROBE(2);
        issue(vq, rs, so, refill_slot);
        // Without branches between the steps hipcc interleaved the compressions with the window
        // reads (one s_waitcnt per dword) and hoisted the next window read above them.
        __builtin_amdgcn_sched_barrier(0);
        Alg::compress(st, w0);
        Alg::compress(st, w1);
        __builtin_amdgcn_sched_barrier(0);
    };
    for (;;) {
        typename Alg::State st = Alg::iv();
        uint32_t k = 1;
        if (POOL && gn == ~uint64_t(0) && K >= 2) {
            // iteration 1 with the pool ticket requested behind its refill: the return is waited on
            // with iteration 2's line, after blocks 0 and 1 are hashed
            BRB_LINE_PROBE(1);
            brb_dma::wait_vmcnt<0>();
            read_window(ae);
            BRB_LINE_PROBE(2);
            issue(vq, rs, so, 0);
            pv_pending = home_open();
            if (pv_pending)
                pv = pool_fetch(home);
            __builtin_amdgcn_sched_barrier(0);
            Alg::compress(st, w0);
            Alg::compress(st, w1);
            __builtin_amdgcn_sched_barrier(0);
            k = 2;
            if (k < K) {                                       // iteration 2 (even) is a full step too:
                full_step(st, ao, 1);                          // the loop below then starts at odd k
                k = 3;
            }
        }
        for (; k + 2 <= K; k += 2) {
            full_step(st, ae, 0);                              // odd k: line k+1 goes to slot 0
            full_step(st, ao, 1);                              // even k: line k+1 goes to slot 1
        }
        if (k < K) {                                           // K even: iteration K-1 (odd) is left
            full_step(st, ae, 0);
        }
        {   // iteration K: the window table of its parity, selected once per group
            uint32_t al[32];
#pragma unroll
            for (int i = 0; i < 32; i++)
                al[i] = (K & 1) ? ae[i] : ao[i];
            BRB_LINE_PROBE(1);
            const uint32_t other = lock_pub();
            brb_dma::wait_vmcnt<0>();
            read_window(al);
            lock_prio(other);
            BRB_LINE_PROBE(2);
            if (POOL && gn == ~uint64_t(0)) {                  // the pool ticket (K = 1: taken here)
                gn = pv_pending || home_open() ? pool_group(home, pv_pending ? pv : pool_fetch(home)) : n_groups;
                pv_pending = false;
                if (gn >= n_groups)
                    gn = pool_sweep(home);
            }
            if (gn < n_groups) {
                dma_setup(gn, vqn, rsn);
                son = 0;
                issue(vqn, rsn, son, 0, true);
                issue(vqn, rsn, son, 1, true);
            }
            if (2 * K - 2 < nfull)
                Alg::compress(st, w0);
            if (2 * K - 1 < nfull)
                Alg::compress(st, w1);
        }
        line_finish<Alg, OUT_ALIGNED>(st, w0, w1, tm, tp, t, nfull, K, rec_len, out, g * 64 + lane, n_rec);
        g = gn;
        if (g >= n_groups)
            break;
        gn = DYN ? take() : g + wstride;
#pragma unroll
        for (int q = 0; q < 8; q++)
            vq[q] = vqn[q];
        rs = rsn;
        so = son;
        win_setup(g);
    }
    BRB_LINE_PROBE(3);
    pool_done();
}

}  // namespace brb_mb_r05
