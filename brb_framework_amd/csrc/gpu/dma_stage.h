// dma_stage.h -- LDS-DMA staging of fixed-stride records for the lane-per-record digest kernels.
//
// A wave digests groups of 64 consecutive records, one record per lane.  Message block `blk` of
// all 64 records of a group (4 KiB) is brought into a private LDS ring slot by four
// `buffer_load_dwordx4 ... lds` instructions (LDS-DMA: no VGPR destination, no ds_write,
// unaligned sources allowed).  One instruction covers 16 records x 64 contiguous bytes, so L2/HBM
// see 64-byte segments instead of the 16-byte per-lane scatter of direct loads.  The LDS image is
// lane-linear per instruction, so the bank swizzle is applied to the SOURCE address
// (cdna_hip_programming.md rule 21): slot j of instruction q holds record 16q + j/4, chunk
// (j & 3) ^ ((j >> 4) & 3); lane r then reads chunk c of its record at
//   r * 64 + (c ^ ((r >> 2) & 3)) * 16
// which is conflict-free for ds_read_b128's four 16-lane groups (SQ_LDS_BANK_CONFLICT = 0).
//
// The group base is a buffer descriptor (SGPRs), each lane's record row + chunk a 32-bit voffset,
// the block index the scalar soffset: staging costs no VALU work per block.
#pragma once

#include "brb_gpu_common.h"

namespace brb_dma {

constexpr int kSlotBytes = 4096;     // one 64-byte block of 64 records

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

struct Stager {
    uint32_t voff[4];                // per-lane source offset of instruction q (record row + chunk)
    uint32_t lane_row;               // this lane's record row inside a slot
    uint32_t chunk, lane;

    BRB_DEV void init(uint32_t stride, uint32_t lane_)
    {
        lane = lane_;
        chunk = (lane & 3) ^ ((lane >> 4) & 3);
#pragma unroll
        for (int q = 0; q < 4; q++)
            voff[q] = (16 * q + (lane >> 2)) * stride + chunk * 16;
        lane_row = lane * 64;
    }

    // Issue the 4 DMAs of block `blk` of the group at `base` (n_grp records, `extent` bytes to the
    // end of the batch) into the LDS slot at byte address `slot_lds` (wave-uniform).
    // Inline asm on purpose: hipcc, seeing an LDS-DMA builtin, drains the whole ring with
    // vmcnt(0) before every ds_read; the counted waits are placed by hand instead (wait_vmcnt).
    // M0 is saved and restored inside the statement (it is compiler-reserved).
    BRB_DEV void issue(const uint8_t *base, uint32_t stride, uint32_t n_grp, uint64_t extent, uint32_t slot_lds,
                       uint32_t blk) const
    {
        const v4i rsrc = make_rsrc(base, extent);
        uint32_t v0 = voff[0], v1 = voff[1], v2 = voff[2], v3 = voff[3];
        if (n_grp < 64) {                                    // partial last group: re-read a valid record
            const uint32_t last = n_grp - 1, r = lane >> 2, c16 = chunk * 16;
            v0 = min(r, last) * stride + c16;
            v1 = min(16 + r, last) * stride + c16;
            v2 = min(32 + r, last) * stride + c16;
            v3 = min(48 + r, last) * stride + c16;
        }
        const uint32_t soff = __builtin_amdgcn_readfirstlane(blk * 64);
        const uint32_t m = __builtin_amdgcn_readfirstlane(slot_lds);
        uint32_t keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\t"
            "s_mov_b32 m0, %7\n\t"
            "s_nop 0\n\t"
            "buffer_load_dwordx4 %1, %5, %6 offen lds\n\t"
            "s_add_u32 m0, m0, 0x400\n\t"
            "s_nop 0\n\t"
            "buffer_load_dwordx4 %2, %5, %6 offen lds\n\t"
            "s_add_u32 m0, m0, 0x400\n\t"
            "s_nop 0\n\t"
            "buffer_load_dwordx4 %3, %5, %6 offen lds\n\t"
            "s_add_u32 m0, m0, 0x400\n\t"
            "s_nop 0\n\t"
            "buffer_load_dwordx4 %4, %5, %6 offen lds\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(v0), "v"(v1), "v"(v2), "v"(v3), "s"(rsrc), "s"(soff), "s"(m)
            : "memory", "scc");
    }

    // Same as issue(), for stride >= 64: one M0 write per block.  The instruction offset field
    // (applied to both the LDS destination and the global address) selects the 1 KiB quarter of
    // the slot; the per-lane voffsets carry -1024 q to cancel it on the global side.
    BRB_DEV void issue_fast(const v4i &rsrc, const uint32_t (&vq)[4], uint32_t slot_lds) const
    {
        uint32_t keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\t"
            "s_mov_b32 m0, %6\n\t"
            "s_nop 0\n\t"
            "buffer_load_dwordx4 %1, %5, 0 offen lds\n\t"
            "buffer_load_dwordx4 %2, %5, 0 offen offset:1024 lds\n\t"
            "buffer_load_dwordx4 %3, %5, 0 offen offset:2048 lds\n\t"
            "buffer_load_dwordx4 %4, %5, 0 offen offset:3072 lds\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(vq[0]), "v"(vq[1]), "v"(vq[2]), "v"(vq[3]), "s"(rsrc), "s"(slot_lds)
            : "memory");
    }

    // Per-lane voffsets of issue_fast for a group of n_grp records (n_grp < 64: clamp to the last).
    BRB_DEV void group_offsets(uint32_t stride, uint32_t n_grp, uint32_t (&vq)[4]) const
    {
        const uint32_t last = n_grp - 1, r = lane >> 2, c16 = chunk * 16;
#pragma unroll
        for (int q = 0; q < 4; q++)
            vq[q] = min(16u * q + r, last) * stride + c16 - 1024u * q;
    }

    // Read this lane's 16 little-endian words of the block in `slot`.
    BRB_DEV void read(const uint8_t *slot, uint32_t (&w)[16]) const
    {
        const uint32_t sw = (lane >> 2) & 3;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint4 v = *reinterpret_cast<const uint4 *>(slot + lane_row + ((c ^ sw) << 4));
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
