// dma_stage.h -- LDS-DMA staging of fixed-stride records for the lane-per-record digest kernels.
//
// A wave digests groups of 64 consecutive records, one record per lane.  A "stage" brings S bytes
// (S = 64 * BPS, BPS message blocks) of all 64 records of a group into a private LDS ring slot with
// 4 * BPS `buffer_load_dwordx4 ... lds` instructions (LDS-DMA: no VGPR destination, no ds_write,
// unaligned sources allowed).  One instruction covers 1024 / S records x S contiguous bytes.
// Why S = 128 (BPS = 2) and not 64: records of 1500 B are only 4-byte aligned, so a 64-byte piece
// straddles two 64-byte memory sectors; at S = 64 the staging alone streams at 4.5 TB/s on a
// 1 Mi-record batch, at S = 128 at 5.5 TB/s, against 6.4 TB/s for a contiguous copy
// (tools/mb/dma_pattern.hip, 1 048 576 x 1500 B).
//
// The LDS image is lane-linear per instruction, so the bank swizzle is applied to the SOURCE
// address (cdna_hip_programming.md rule 21): a slot row is one record's S bytes = G = S / 16
// granules of 16 B; logical granule k of record r sits at physical granule k ^ f(r) with
//   f(r) = (r >> 2) & 3  (G = 4)     f(r) = (r >> 1) & 7  (G = 8)
// which makes ds_read_b128 of one granule by all 64 lanes conflict-free (SQ_LDS_BANK_CONFLICT = 0).
//
// The stage base is a buffer descriptor (SGPRs) whose num_records is the byte count to the end of
// the batch, each lane's record row + granule a 32-bit voffset: staging costs no VALU per stage,
// and the hardware range check (voffset + inst_offset against num_records) returns zeros for bytes
// past the batch end instead of faulting.
//
// NT = true sets the non-temporal policy (nt) on the DMA: the records are read exactly once.
#pragma once

#include "brb_gpu_common.h"

namespace brb_dma {

typedef int v4i __attribute__((ext_vector_type(4)));

// gfx950 raw buffer descriptor (stride 0): base, num_records (bytes), DATA_FORMAT=32 flags.
BRB_DEV v4i make_rsrc(const uint8_t *base, uint64_t extent)
{
    const uint64_t a = reinterpret_cast<uint64_t>(base);
    v4i r;
    r.x = __builtin_amdgcn_readfirstlane(int(uint32_t(a)));
    r.y = __builtin_amdgcn_readfirstlane(int(uint32_t(a >> 32) & 0xFFFF));
    r.z = __builtin_amdgcn_readfirstlane(int(extent > 0x7FFFFFFFull ? 0x7FFFFFFFu : uint32_t(extent)));
    r.w = 0x00020000;
    return r;
}

template <int BPS, bool NT = false>
struct Stager {
    static constexpr int S = 64 * BPS;          // bytes of one record per stage
    static constexpr int G = S / 16;            // 16-byte granules per record row
    static constexpr int NI = 4 * BPS;          // DMA instructions per stage (1 KiB each)
    static constexpr int RPI = 1024 / S;        // records per instruction
    static constexpr int SLOT = 64 * S;         // LDS bytes per stage
    static_assert(BPS == 1 || BPS == 2, "swizzle defined for 64- and 128-byte rows");

    uint32_t vq[NI];                 // per-lane source offset of instruction q (minus 1024 (q % 4))
    uint32_t lane;

    static BRB_DEV uint32_t swz(uint32_t r) { return G == 4 ? (r >> 2) & 3 : (r >> 1) & 7; }

    // Offsets for a group of n_grp records (n_grp < 64: lanes past the end re-read the last one).
    // fast (stride >= 128): instruction q carries inst_offset 1024 (q % 4), cancelled here.
    BRB_DEV void group_offsets(uint32_t stride, uint32_t n_grp, bool fast)
    {
        const uint32_t last = n_grp - 1, sub = lane / G, gran = lane % G;
#pragma unroll
        for (int q = 0; q < NI; q++) {
            const uint32_t row = uint32_t(q * RPI) + sub;                  // LDS slot row
            const uint32_t rec = min(row, last);
            const uint32_t logical = gran ^ swz(row);
            vq[q] = rec * stride + logical * 16 - (fast ? 1024u * (q & 3) : 0u);
        }
    }

    BRB_DEV void init(uint32_t stride, uint32_t n_grp, uint32_t lane_, bool fast)
    {
        lane = lane_;
        group_offsets(stride, n_grp, fast);
    }

    // Issue one stage into the LDS slot at byte address slot_lds (wave-uniform).  Inline asm on
    // purpose: hipcc, seeing an LDS-DMA builtin, drains the whole ring with vmcnt(0) before every
    // ds_read; the counted waits are placed by hand instead (wait_vmcnt).  M0 (the LDS base of a
    // DMA) is compiler-reserved, so it is saved and restored inside the statement.
    BRB_DEV void issue_fast(const v4i &rsrc, uint32_t slot_lds) const
    {
#define BRB_DMA_FAST(POL)                                                                              \
    asm volatile("s_mov_b32 %0, m0\n\t"                                                                 \
                 "s_mov_b32 m0, %6\n\t"                                                                 \
                 "s_nop 0\n\t"                                                                          \
                 "buffer_load_dwordx4 %1, %5, 0 offen " POL "lds\n\t"                                   \
                 "buffer_load_dwordx4 %2, %5, 0 offen offset:1024 " POL "lds\n\t"                       \
                 "buffer_load_dwordx4 %3, %5, 0 offen offset:2048 " POL "lds\n\t"                       \
                 "buffer_load_dwordx4 %4, %5, 0 offen offset:3072 " POL "lds\n\t"                       \
                 "s_mov_b32 m0, %0"                                                                      \
                 : "=&s"(keep)                                                                           \
                 : "v"(vq[4 * h]), "v"(vq[4 * h + 1]), "v"(vq[4 * h + 2]), "v"(vq[4 * h + 3]), "s"(rsrc), \
                   "s"(slot_lds + 4096u * h)                                                             \
                 : "memory")
#pragma unroll
        for (int h = 0; h < BPS; h++) {
            uint32_t keep;
            if constexpr (NT)
                BRB_DMA_FAST("nt ");
            else
                BRB_DMA_FAST("");
        }
#undef BRB_DMA_FAST
    }

    // Same, one M0 write per instruction (strides below 128, where the inst_offset trick would
    // need negative voffsets).
    BRB_DEV void issue_slow(const v4i &rsrc, uint32_t slot_lds) const
    {
#define BRB_DMA_SLOW(POL)                                                \
    asm volatile("s_mov_b32 %0, m0\n\t"                                   \
                 "s_mov_b32 m0, %3\n\t"                                   \
                 "s_nop 0\n\t"                                            \
                 "buffer_load_dwordx4 %1, %2, 0 offen " POL "lds\n\t"     \
                 "s_mov_b32 m0, %0"                                        \
                 : "=&s"(keep)                                             \
                 : "v"(vq[q]), "s"(rsrc), "s"(slot_lds + 1024u * q)        \
                 : "memory")
#pragma unroll
        for (int q = 0; q < NI; q++) {
            uint32_t keep;
            if constexpr (NT)
                BRB_DMA_SLOW("nt ");
            else
                BRB_DMA_SLOW("");
        }
#undef BRB_DMA_SLOW
    }

    // Read this lane's block j (0 <= j < BPS) of the stage in `slot` as 16 little-endian words.
    BRB_DEV void read(const uint8_t *slot, uint32_t j, uint32_t (&w)[16]) const
    {
        const uint32_t f = swz(lane);
        const uint8_t *row = slot + lane * S;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t k = 4 * j + c;
            const uint4 v = *reinterpret_cast<const uint4 *>(row + ((k ^ f) << 4));
            w[4 * c + 0] = v.x;
            w[4 * c + 1] = v.y;
            w[4 * c + 2] = v.z;
            w[4 * c + 3] = v.w;
        }
    }
};

// s_waitcnt vmcnt(N): the LDS-DMA of all but the N youngest VMEM operations of this wave landed.
template <int N>
BRB_DEV void wait_vmcnt()
{
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

}  // namespace brb_dma
