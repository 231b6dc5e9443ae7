// digest_dma.h -- the fixed-stride, LDS-DMA staged, lane-per-record digest kernel shared by MD5
// and SHA-1.  `Alg` supplies State, iv(), compress(st, w) on little-endian message words,
// finish(st, w, t, len) on the padded tail block, pad_only(st, len) for the constant padding block
// of a record whose length is a multiple of 64, and store<ALIGNED>(out, r, st).
//
// Persistent waves: wave w digests record groups w, w + W_total, w + 2 W_total, ... (64 records
// per group, one per lane).  A wave's work is one flat sequence of "stages" (group, block); the
// LDS ring prefetches P-1 stages ahead ACROSS group boundaries, so only the wave's very first block
// pays the HBM latency.  Record r's digest = BRB_MD5Init/Update/Final (md5.c:38-168) or
// BrbSha1_Do (sha1.c:203-216) of data[r * rec_len .. (r + 1) * rec_len).
#pragma once

#include "digest_line.h"
#include "digest_var_line.h"
#include "dma_stage.h"

namespace brb_digest {

// Group assignment as in digest_line.h: static (wave w takes groups w, w + W_total, ...) or, with
// DYN, workgroup b owns groups b, b + G, ... and its waves take them from an LDS ticket counter (the
// older wave of a SIMD wins the issue arbitration, so a static split leaves the younger waves
// running alone at the end).  DYN needs a ring of 2: each slot remembers the group of its stage.
template <class Alg, int WAVES, int P, int BPS, bool OUT_ALIGNED, bool NT = false, bool DYN = false>
__global__ __launch_bounds__(64 * WAVES) void digest_fixed_dma_kernel(const uint8_t *__restrict__ data, uint32_t rec_len,
                                                                       uint64_t n_rec, uint8_t *__restrict__ out)
{
    static_assert(!DYN || P == 2, "ticketed groups are implemented for a ring of 2");
    using SG = brb_dma::Stager<BPS, NT>;
    __shared__ __attribute__((aligned(16))) uint8_t ring[WAVES * P * SG::SLOT];
    __shared__ uint32_t next_ticket;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t n_groups = (n_rec + 63) / 64;
    const uint64_t wave0 = uint64_t(blockIdx.x) * WAVES + wv;
    const uint64_t wstride = uint64_t(gridDim.x) * WAVES;
    if (DYN) {
        if (threadIdx.x == 0)
            next_ticket = WAVES;                               // tickets 0 .. WAVES-1: one per wave
        __syncthreads();
    }
    auto take = [&]() -> uint64_t {
        uint32_t tk = 0;
        if (lane == 0)
            tk = __hip_atomic_fetch_add(&next_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        tk = __builtin_amdgcn_readfirstlane(tk);
        return uint64_t(blockIdx.x) + uint64_t(tk) * gridDim.x;
    };
    const uint64_t g0 = DYN ? uint64_t(blockIdx.x) + uint64_t(wv) * gridDim.x : wave0;
    if (g0 >= n_groups)
        return;

    uint8_t *my = ring + wv * (P * SG::SLOT);
    const uint32_t lds_base = uint32_t(reinterpret_cast<uintptr_t>(my));
    const uint32_t lds_last = lds_base + (P - 1) * SG::SLOT;

    const uint32_t nfull = rec_len >> 6, t = rec_len & 63;
    const uint32_t nblk = nfull + (t ? 1 : 0);                // blocks holding record bytes (>= 1)
    const uint32_t nstage = (nblk + BPS - 1) / BPS;           // stages per group
    const bool fast = rec_len >= 64 * BPS;                    // inst_offset form of the issue

    // ---- issue cursor: runs P-1 stages ahead of the compute cursor, across group boundaries.
    // The descriptor base points at the stage being issued and num_records at the bytes left to
    // the end of the batch, so the range check zeroes exactly the bytes past the batch end.
    uint64_t is_g = g0;                                        // group of the next stage to issue
    uint64_t is_left = (n_rec - g0 * 64) * rec_len;
    const uint8_t *is_base = data + g0 * 64 * rec_len;
    uint32_t is_stage = 0, is_slot = lds_base;
    uint32_t pending = 0;                                      // stages issued, not yet hashed
    uint64_t slot_g0 = g0, slot_g1 = g0;                       // DYN: group of the stage in each slot
    SG sg;
    sg.init(rec_len, uint32_t(n_rec - g0 * 64 < 64 ? n_rec - g0 * 64 : 64), lane, fast);
    brb_dma::v4i rs = brb_dma::make_rsrc(is_base, is_left);
    auto issue_next = [&]() {                                  // precondition: is_g < n_groups
        if (fast)
            sg.issue_fast(rs, is_slot);
        else
            sg.issue_slow(rs, is_slot);
        if (DYN) {
            if (is_slot == lds_base)
                slot_g0 = is_g;
            else
                slot_g1 = is_g;
        }
        ++pending;
        is_slot = is_slot == lds_last ? lds_base : is_slot + SG::SLOT;
        if (++is_stage < nstage) {
            is_base += SG::S;
            is_left -= SG::S;
        } else {                                              // this wave's next group
            is_stage = 0;
            is_g = DYN ? take() : is_g + wstride;
            const uint64_t r0 = is_g * 64;
            is_base = data + r0 * rec_len;
            is_left = is_g < n_groups ? (n_rec - r0) * rec_len : 0;
            if (is_g < n_groups && n_rec - r0 < 64)
                sg.group_offsets(rec_len, uint32_t(n_rec - r0), fast);
        }
        rs = brb_dma::make_rsrc(is_base, is_left);
    };
#pragma unroll
    for (int i = 0; i < P - 1; i++)
        if (is_g < n_groups)
            issue_next();

    typename Alg::State st = Alg::iv();
    uint32_t w[16];
    uint64_t rb = g0 * 64;                                     // compute cursor: first record of group
    uint32_t cs = 0, slot = lds_base;
    BRB_LINE_PROBE_DECL
    BRB_LINE_PROBE(0);
    while (pending) {
        if (is_g < n_groups) {
            issue_next();
            BRB_LINE_PROBE(1);
            brb_dma::wait_vmcnt<SG::NI * (P - 1)>();
        } else {
            BRB_LINE_PROBE(1);
            brb_dma::wait_vmcnt<0>();
        }
        BRB_LINE_PROBE(2);
        --pending;
        if (DYN)
            rb = (slot == lds_base ? slot_g0 : slot_g1) * 64;
        const uint8_t *sp = my + (slot - lds_base);
        slot = slot == lds_last ? lds_base : slot + SG::SLOT;
        const uint32_t b0 = cs * BPS;
#pragma unroll
        for (uint32_t j = 0; j < BPS; j++) {
            if (b0 + j < nfull) {
                sg.read(sp, j, w);
                Alg::compress(st, w);
            }
        }
        if (++cs < nstage)
            continue;
        // ---- last stage of this group: padding, digest, store
        // `tt` is laundered through an empty asm so that everything derived from it below is
        // computed here, once per group, instead of being hoisted out of the loop into live SGPRs
        // (the hoisted form spilled ~200 SGPRs to VGPR lanes).
        uint32_t tt = t;
        asm volatile("" : "+s"(tt));
        const uint64_t r = rb + lane;
        if (tt == 0) {                                        // the padding block is a constant
            Alg::pad_only(st, rec_len);
        } else {
        if (tt) {
            sg.read(sp, nfull - b0, w);                       // the tail block of this stage
        } else {
#pragma unroll
            for (uint32_t i = 0; i < 16; i++)
                w[i] = 0;
        }
        // records ending within 3 bytes of the batch end: a staged dword of their tail may
        // straddle the end of the batch and was range-checked to zero -> re-read byte by byte
        if (tt && r < n_rec && (n_rec - 1 - r) * rec_len < 4) {
            const uint8_t *a = data + r * rec_len + 64u * nfull;
#pragma unroll
            for (uint32_t i = 0; i < 16; i++) {
                uint32_t v = 0;
#pragma unroll
                for (uint32_t k = 0; k < 4; k++)
                    if (4 * i + k < tt)
                        v |= uint32_t(a[4 * i + k]) << (8 * k);
                w[i] = v;
            }
        }
        // keep the t tail bytes, place the 0x80 marker, zero the rest
#pragma unroll
        for (uint32_t i = 0; i < 16; i++) {
            const uint32_t o = 4 * i;
            const uint32_t keep = tt > o ? (tt - o < 4 ? tt - o : 4) : 0;
            uint32_t v = w[i] & uint32_t((uint64_t(1) << (8 * keep)) - 1);
            if (tt >= o && tt < o + 4)
                v |= 0x80u << (8 * (tt - o));
            w[i] = v;
        }
        Alg::finish(st, w, t, rec_len);
        }
        if (r < n_rec)
            Alg::template store<OUT_ALIGNED>(out, r, st);
        st = Alg::iv();
        cs = 0;
        if (!DYN)
            rb += wstride * 64;
    }
    BRB_LINE_PROBE(3);
}

// Records of exactly 64 bytes (cfg3: 1 Mi x 64 B): one data block and the constant padding block
// per record, one 64-byte stage per group.  The generic kernel above spends ~100 scalar
// instructions per group on its stage cursor (64-bit multiplies by the runtime record length, the
// group-boundary bookkeeping of multi-stage records, the tail machinery) -- 1.70 M SALU per launch,
// 17 % of the VALU count, issued by the same four waves per SIMD that the VALU-bound compression
// keeps busy (profiles/r03_pmc_cfg3_md5.txt).  Here a wave walks its groups
// w, w + W_total, ... with the byte stride between them fixed once, so a group costs one 64-bit add
// and subtract, the descriptor and four DMAs.
template <class Alg, int WAVES, bool OUT_ALIGNED>
__global__ __launch_bounds__(64 * WAVES) void digest_b64_kernel(const uint8_t *__restrict__ data, uint64_t n_rec,
                                                                uint8_t *__restrict__ out)
{
    using SG = brb_dma::Stager<1, false>;                     // 64-byte rows, 4 DMAs per stage
    __shared__ __attribute__((aligned(16))) uint8_t ring[WAVES * 2 * SG::SLOT];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t n_groups = (n_rec + 63) / 64;
    uint64_t g = uint64_t(blockIdx.x) * WAVES + wv;
    const uint64_t wstride = uint64_t(gridDim.x) * WAVES;
    if (g >= n_groups)
        return;
    uint8_t *my = ring + wv * (2 * SG::SLOT);
    const uint32_t lds0 = uint32_t(reinterpret_cast<uintptr_t>(my));
    const uint64_t last_full = n_rec / 64;                    // groups below this one hold 64 records
    SG sg;
    sg.init(64, uint32_t(g < last_full ? 64 : n_rec - g * 64), lane, true);
    const uint64_t gbytes = wstride * 4096;                   // bytes from one of this wave's groups to the next
    const uint8_t *base = data + g * 4096;
    uint64_t left = (n_rec - g * 64) * 64;
    sg.issue_fast(brb_dma::make_rsrc(base, left), lds0);
    uint32_t slot = 0;
    for (;;) {
        const uint64_t gn = g + wstride;
        const bool more = gn < n_groups;
        if (more) {
            base += gbytes;
            left -= gbytes;
            if (gn >= last_full)                              // the batch's partial last group
                sg.group_offsets(64, uint32_t(n_rec - gn * 64), true);
            sg.issue_fast(brb_dma::make_rsrc(base, left), slot ? lds0 : lds0 + SG::SLOT);
            brb_dma::wait_vmcnt<SG::NI>();
        } else {
            brb_dma::wait_vmcnt<0>();
        }
        uint32_t w[16];
        sg.read(my + slot * SG::SLOT, 0, w);
        typename Alg::State st = Alg::iv();
        Alg::compress(st, w);
        Alg::pad_only(st, 64);
        const uint64_t r = g * 64 + lane;
        if (g < last_full || r < n_rec)
            Alg::template store<OUT_ALIGNED>(out, r, st);
        if (!more)
            break;
        g = gn;
        slot ^= 1;
    }
}

// Same work with one LDS slot per wave: a group's 16 words go to registers, and the next group's
// DMA is issued into the same slot before the compression starts, so the registers are the second
// buffer.  4 KiB of LDS per wave (50 VGPRs) lets 8 waves share a SIMD instead of 4.  A group's
// digest is stored one iteration later, after that iteration's window read: the only VMEM
// operation older than the DMA a wave waits for is then a store issued a whole compression
// earlier, so the wait (vmcnt 0) never waits on a fresh write's acknowledgement.
template <class Alg, int WAVES, bool OUT_ALIGNED>
__global__ __launch_bounds__(64 * WAVES) void digest_b64r_kernel(const uint8_t *__restrict__ data, uint64_t n_rec,
                                                                 uint8_t *__restrict__ out)
{
    using SG = brb_dma::Stager<1, false>;
    __shared__ __attribute__((aligned(16))) uint8_t ring[WAVES * SG::SLOT];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t n_groups = (n_rec + 63) / 64;
    uint64_t g = uint64_t(blockIdx.x) * WAVES + wv;
    const uint64_t wstride = uint64_t(gridDim.x) * WAVES;
    if (g >= n_groups)
        return;
    uint8_t *my = ring + wv * SG::SLOT;
    const uint32_t lds0 = uint32_t(reinterpret_cast<uintptr_t>(my));
    const uint64_t last_full = n_rec / 64;
    SG sg;
    sg.init(64, uint32_t(g < last_full ? 64 : n_rec - g * 64), lane, true);
    const uint64_t gbytes = wstride * 4096;
    const uint8_t *base = data + g * 4096;
    uint64_t left = (n_rec - g * 64) * 64;
    sg.issue_fast(brb_dma::make_rsrc(base, left), lds0);
    typename Alg::State prev;
    uint64_t rprev = ~uint64_t(0);                            // no digest pending
    for (;;) {
        brb_dma::wait_vmcnt<0>();
        uint32_t w[16];
        sg.read(my, 0, w);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");    // the slot is free for the next DMA
        if (rprev < n_rec)
            Alg::template store<OUT_ALIGNED>(out, rprev, prev);
        const uint64_t gn = g + wstride;
        const bool more = gn < n_groups;
        if (more) {
            base += gbytes;
            left -= gbytes;
            if (gn >= last_full)
                sg.group_offsets(64, uint32_t(n_rec - gn * 64), true);
            sg.issue_fast(brb_dma::make_rsrc(base, left), lds0);
        }
        prev = Alg::iv();
        Alg::compress(prev, w);
        Alg::pad_only(prev, 64);
        rprev = g * 64 + lane;
        if (!more)
            break;
        g = gn;
    }
    if (rprev < n_rec)
        Alg::template store<OUT_ALIGNED>(out, rprev, prev);
}

// Host-side launch.
inline bool dma_supported(uint32_t rec_len)
{
    return rec_len > 0 && uint64_t(rec_len) * 64 + 64 < (uint64_t(1) << 31);
}

// Test option "fixed_var_line" = 0 keeps byte-aligned fixed-stride records on the record-relative
// kernel (A/B measurements).
inline bool fixed_var_line_enabled()
{
    return brb_opt::get(brb_opt::kFixedVarLine) != 0;
}

template <class Alg>
hipError_t launch_fixed_dma(const uint8_t *data, uint32_t rec_len, uint64_t n_rec, uint8_t *out, bool out_al,
                            hipStream_t s)
{
    // Shapes measured with tools/mb/md5_ab.hip (interleaved, one process):
    //  * records > 64 B at any alignment: 128-byte stages, ring of 2 (16 KiB per wave): 1 Mi x
    //    1500 B 335 us vs 388 us with 64-byte stages;
    //  * records <= 64 B (one block + padding): 64-byte stages, ring of 2, 4 workgroups per CU.
    // Persistent beyond the resident grid (waves loop over groups of 64 records).
    constexpr int W = 4;
    const uint64_t groups = (n_rec + 63) / 64;
    const uint64_t wgs_needed = (groups + W - 1) / W;
    // 4-byte record bases and lengths over 64 B: line-aligned staging, digest_line.h (every line
    // is read once; no 128-byte piece straddles two lines).  1 Mi x 1500 B: 343 -> 300 us,
    // cfg2: 25.3 -> 24.9 us (tools/mb/md5_ab.hip).
    if (line_supported(data, rec_len))
        return launch_fixed_line<Alg>(data, rec_len, n_rec, out, out_al, s);
    if (rec_len > 64 && rec_len <= (1u << 20) && fixed_var_line_enabled())
        return launch_fixed_var_line<Alg>(data, rec_len, n_rec, out, out_al, s);   // any byte alignment
    if (rec_len > 64) {
        // one 8-wave workgroup per CU (two waves per SIMD, 128 KiB of LDS), persistent, groups
        // handed out by tickets, 128-byte stages, ring of 2
        const unsigned g = unsigned(groups < device_cu_count() ? groups : device_cu_count());
        if (out_al)
            digest_fixed_dma_kernel<Alg, 8, 2, 2, true, false, true><<<g, 512, 0, s>>>(data, rec_len, n_rec, out);
        else
            digest_fixed_dma_kernel<Alg, 8, 2, 2, false, false, true><<<g, 512, 0, s>>>(data, rec_len, n_rec, out);
    } else if (rec_len == 64 && brb_opt::get(brb_opt::kB64Kernel) >= 2) {
        // register-buffered 64-byte kernel: 16 KiB per workgroup; option 2: 8 workgroups per CU
        // (8 waves per SIMD), option 3: 4 per CU
        const unsigned cap = brb_opt::get(brb_opt::kB64Kernel) == 2 ? 2048u : 1024u;
        const unsigned g = unsigned(wgs_needed < cap ? wgs_needed : cap);
        if (out_al)
            digest_b64r_kernel<Alg, W, true><<<g, 64 * W, 0, s>>>(data, n_rec, out);
        else
            digest_b64r_kernel<Alg, W, false><<<g, 64 * W, 0, s>>>(data, n_rec, out);
    } else if (rec_len == 64 && brb_opt::get(brb_opt::kB64Kernel) != 0) {
        // the lean 64-byte kernel, same shape as below (4 workgroups of 4 waves per CU, 32 KiB each)
        const unsigned g = unsigned(wgs_needed < 1024 ? wgs_needed : 1024);
        if (out_al)
            digest_b64_kernel<Alg, W, true><<<g, 64 * W, 0, s>>>(data, n_rec, out);
        else
            digest_b64_kernel<Alg, W, false><<<g, 64 * W, 0, s>>>(data, n_rec, out);
    } else {
        // 4 workgroups per CU (32 KiB each), static groups: 1 Mi x 64 B = 16 384 groups = exactly 4
        // per wave.  Measured (md5_ab, 1 Mi x 64 B): 24.6 us; one 16-wave workgroup per CU with
        // tickets 25.3 us; a ring of 3 at 3 workgroups per CU 26.1 us.
        const unsigned g = unsigned(wgs_needed < 1024 ? wgs_needed : 1024);
        if (out_al)
            digest_fixed_dma_kernel<Alg, W, 2, 1, true><<<g, 64 * W, 0, s>>>(data, rec_len, n_rec, out);
        else
            digest_fixed_dma_kernel<Alg, W, 2, 1, false><<<g, 64 * W, 0, s>>>(data, rec_len, n_rec, out);
    }
    return hipGetLastError();
}

}  // namespace brb_digest
