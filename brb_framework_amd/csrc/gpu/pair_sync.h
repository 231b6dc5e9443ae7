// pair_sync.h -- LDS hand-off between the two waves of a producer / consumer pair sharing one SIMD
// (md5_seg_pc_kernel, metadata_line_kernel<..., PC>, the RC4+MD5 frame / open pairs).
// One writer per counter or mailbox: release store after the data it covers, acquire load before
// the reads it guards (workgroup scope: both waves are in one workgroup, so LDS and the CU's L1 are
// shared).  Every wait is bounded (~2^22 sleeps without progress from the other wave): a protocol
// fault never hangs a wave; its outputs are wrong, and the wave that gives up stores 1 into the
// call's fault word (pc_fault; pair_fault.h), so the batch call fails instead of returning them.
#pragma once

#include "brb_gpu_common.h"

namespace brb_line {

BRB_DEV uint32_t pc_load(uint32_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// A heartbeat: the working wave bumps it as it goes (no ordering needed, so a relaxed store: no
// wait for its own LDS writes), and a waiting wave's budget counts only sleeps with no beat.  So a
// legitimately long stretch (a lane's multi-GiB record on the per-lane path, thousands of lines of
// empty items) never times out, while a wave whose partner stopped still ends.
BRB_DEV void pc_beat(uint32_t *hb, uint32_t v)
{
    __hip_atomic_store(hb, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

BRB_DEV uint32_t pc_beat_of(uint32_t *hb)
{
    return hb ? __builtin_amdgcn_readfirstlane(__hip_atomic_load(hb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) : 0u;
}

// Per-block beat hooks for code shared with the single-wave kernels (seg_lane, unpack_lane).
struct NoBeat {
    BRB_DEV void operator()() {}
};
struct HbBeat {
    uint32_t *hb;
    uint32_t n;
    BRB_DEV void operator()() { pc_beat(hb, ++n); }
};

// Waits until *ctr >= target; false after 2^22 sleeps without a beat of *hb (if given).
BRB_DEV bool pc_wait_ge(uint32_t *ctr, uint32_t target, uint32_t *hb = nullptr)
{
    uint32_t last = pc_beat_of(hb);
    for (uint32_t spin = 0; spin < (1u << 22); spin++) {
        const uint32_t v = __hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (__builtin_amdgcn_readfirstlane(v) >= target)
            return true;
        const uint32_t h = pc_beat_of(hb);
        if (h != last) {
            last = h;
            spin = 0;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    return false;
}

BRB_DEV void pc_publish(uint32_t *ctr, uint32_t v)
{
    __hip_atomic_store(ctr, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// A bounded wait gave up: flag the call (a word of page-locked host memory, pair_fault.h; nullptr
// when the call is not armed).  A vector store at system scope, read by the host after the launch
// has completed.
BRB_DEV void pc_fault(uint32_t *fault)
{
    if (fault)   // a global (not flat) store: no flat access anywhere in the pair kernels
        __hip_atomic_store((__attribute__((address_space(1))) uint32_t *)fault, 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

// The pair kernels keep the fault word's address in LDS (`fault_at`, written by thread 0 before the
// kernel's first barrier) and read it back only when a wait gives up: a kernel argument live for the
// whole kernel holds an SGPR pair (md5_seg_pc_kernel: SGPR spills 39 -> 47).  Both accesses are
// typed (ds_read, global_store): a generic pointer made them flat_load / flat_store, and one flat
// access in these LDS-heavy kernels made hipcc's wait-count insertion conservative everywhere --
// md5seg 34.3 -> 35.1 us, MetaData 38.5 -> 38.9 us, with the flat ops on cold paths only.
BRB_DEV void pc_fault_from(uint32_t **fault_at)
{
    pc_fault(__hip_atomic_load(fault_at, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}

}  // namespace brb_line
