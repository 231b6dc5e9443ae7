// brb_gpu_common.h -- device helpers shared by the gfx950 crypto kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define BRB_DEV __device__ __forceinline__

// 32-bit rotate left by a compile-time amount: one v_alignbit_b32.
template <int S>
BRB_DEV uint32_t rotl(uint32_t x)
{
    return __builtin_amdgcn_alignbit(x, x, 32 - S);
}

// Funnel shift: bits [sh, sh+32) of the 64-bit value {hi:lo}; sh in [0, 31].  v_alignbit_b32.
BRB_DEV uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t sh)
{
    return __builtin_amdgcn_alignbit(hi, lo, sh);
}

// Global-memory accessors.  Pointers rebuilt from integers (byte offsets rounded to dwords) lose
// their address space, and hipcc then emits FLAT instructions, which count in LGKM_CNT as well as
// VM_CNT: every LDS wait of a kernel (the RC4 generator's) would also wait for its HBM loads and
// stores.  These casts keep them global_load / global_store.
#define BRB_GLOBAL __attribute__((address_space(1)))
#define BRB_GPTR(T, p) ((BRB_GLOBAL T *)(uintptr_t)(p))
typedef uint32_t brb_v4u_a4 __attribute__((ext_vector_type(4), aligned(4)));

// 16-byte load from a 4-byte-aligned global address (gfx950 runs in unaligned-access mode; one
// global_load_dwordx4).
BRB_DEV uint4 ld16_a4(const uint8_t *p)
{
    const brb_v4u_a4 v = *BRB_GPTR(const brb_v4u_a4, p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

BRB_DEV void st16_a4(uint8_t *p, uint32_t a, uint32_t b, uint32_t c, uint32_t d)
{
    brb_v4u_a4 v;
    v.x = a;
    v.y = b;
    v.z = c;
    v.w = d;
    *BRB_GPTR(brb_v4u_a4, p) = v;
}

BRB_DEV uint32_t ld4_a4(const uint8_t *p)
{
    return *BRB_GPTR(const uint32_t, p);
}

BRB_DEV uint32_t ldg(const uint32_t *p)
{
    return *BRB_GPTR(const uint32_t, p);
}

BRB_DEV void stg(uint32_t *p, uint32_t v)
{
    *BRB_GPTR(uint32_t, p) = v;
}

BRB_DEV uint32_t ldg8(const uint8_t *p)
{
    return *BRB_GPTR(const uint8_t, p);
}

BRB_DEV void stg8(uint8_t *p, uint32_t v)
{
    *BRB_GPTR(uint8_t, p) = uint8_t(v);
}

// Little-endian word i (bytes [4i, 4i+4)) of a message tail of `t` valid bytes (t < 64) followed by
// the MD5/SHA-1 padding byte 0x80 and zeros.  `p` is 4-byte aligned; a dword is read only when it
// holds at least one valid byte, so nothing past the record's last dword is touched.
BRB_DEV uint32_t tail_word_a4(const uint8_t *p, uint32_t t, uint32_t i)
{
    const uint32_t o = 4 * i;
    uint32_t v = 0;
    if (o < t)
        v = ld4_a4(p + o);
    if (o + 4 <= t)
        return v;
    if (o > t)
        return 0;
    // this word holds the end of the data and the 0x80 marker: keep (t - o) bytes
    const uint32_t keep = t - o;                 // 0..3
    const uint32_t mask = keep ? (0xFFFFFFFFu >> (32 - 8 * keep)) : 0u;
    return (v & mask) | (0x80u << (8 * keep));
}

// Byte-aligned variant: the record starts at an arbitrary address `a` with `len` bytes; returns
// little-endian word i of the 64-byte block that starts at byte `blk_off` of the record, with the
// padding applied past `len` (pass pad = false for blocks known to be full).
BRB_DEV uint32_t word_any(const uint8_t *a, uint64_t len, uint64_t blk_off, uint32_t i)
{
    const uint64_t o = blk_off + 4 * i;
    if (o + 4 <= len) {
        const uintptr_t addr = reinterpret_cast<uintptr_t>(a) + o;
        const uintptr_t a0 = addr & ~uintptr_t(3);
        const uint32_t sh = uint32_t(addr & 3) * 8;
        const uint32_t lo = ldg(reinterpret_cast<const uint32_t *>(a0));
        // the second dword is read only if it holds a byte of this word (sh != 0)
        const uint32_t hi = sh ? ldg(reinterpret_cast<const uint32_t *>(a0 + 4)) : 0u;
        return funnel(hi, lo, sh);
    }
    uint32_t v = 0;
    for (uint32_t k = 0; k < 4; k++) {
        const uint64_t ob = o + k;
        uint32_t byte = 0;
        if (ob < len)
            byte = ldg8(a + ob);
        else if (ob == len)
            byte = 0x80u;
        v |= byte << (8 * k);
    }
    return v;
}
