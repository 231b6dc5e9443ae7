// pair_sync.h -- LDS hand-off between the two waves of a producer / consumer pair sharing one SIMD
// (md5_seg_pc_kernel, metadata_line_kernel<..., PC>, the RC4+MD5 frame / open pairs).
// One writer per counter or mailbox: release store after the data it covers, acquire load before
// the reads it guards (workgroup scope: both waves are in one workgroup, so LDS and the CU's L1 are
// shared).  Every wait is bounded (~2^22 sleeps, far beyond any launch): a protocol fault gives
// wrong results, never a hung wave.
#pragma once

#include "brb_gpu_common.h"

namespace brb_line {

BRB_DEV bool pc_wait_ge(uint32_t *ctr, uint32_t target)
{
    for (uint32_t spin = 0; spin < (1u << 22); spin++) {
        const uint32_t v = __hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (__builtin_amdgcn_readfirstlane(v) >= target)
            return true;
        __builtin_amdgcn_s_sleep(1);
    }
    return false;
}

BRB_DEV void pc_publish(uint32_t *ctr, uint32_t v)
{
    __hip_atomic_store(ctr, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

BRB_DEV uint32_t pc_load(uint32_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

}  // namespace brb_line
