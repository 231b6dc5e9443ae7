// byte_stream.h -- per-lane sequential access to byte ranges at arbitrary addresses.
//
// Records, streams and segments start at any byte offset.  Src reads a range as 4-byte chunks
// using aligned dword loads and a funnel shift (v_alignbit_b32), loading each dword once; Snk
// writes a range as 4-byte chunks with aligned dword stores and byte stores only for the partial
// dwords at its two ends.  Neither touches a dword that holds none of the range's bytes, so ranges
// packed back to back are safe to process from different lanes at once.
#pragma once

#include "brb_gpu_common.h"

namespace brb_io {

// Sequential 4-byte chunks of a byte range at any address; bytes past the range read as 0.
struct Src {
    const uint32_t *p;
    uint32_t sh;     // 8 * (address & 3)
    uint32_t lo;     // dword at p
    uint64_t rem;    // bytes left from the current position

    BRB_DEV void init(const uint8_t *a, uint64_t n)
    {
        const uintptr_t ad = reinterpret_cast<uintptr_t>(a);
        p = reinterpret_cast<const uint32_t *>(ad & ~uintptr_t(3));
        sh = uint32_t(ad & 3) * 8;
        rem = n;
        lo = n ? p[0] : 0u;
    }

    BRB_DEV uint32_t next()
    {
        const uint32_t o = sh >> 3;
        const uint32_t hi = rem > 4 - o ? p[1] : 0u;     // the next dword holds a byte of the range
        uint32_t v = __builtin_amdgcn_alignbit(hi, lo, sh);
        if (rem < 4)
            v &= (1u << (8 * uint32_t(rem))) - 1u;
        ++p;
        lo = hi;
        rem = rem > 4 ? rem - 4 : 0;
        return v;
    }
};

// Sequential 4-byte chunks into a byte range at any address (exactly `n` bytes are written).
struct Snk {
    uint32_t *p;
    uint32_t o;        // address & 3
    uint32_t carry;    // bytes of the dword at p that the previous chunk produced (positions 0..o-1)
    uint32_t carry_n;
    uint64_t rem;
    bool first;

    BRB_DEV void init(uint8_t *a, uint64_t n)
    {
        const uintptr_t ad = reinterpret_cast<uintptr_t>(a);
        p = reinterpret_cast<uint32_t *>(ad & ~uintptr_t(3));
        o = uint32_t(ad & 3);
        carry = 0;
        carry_n = 0;
        rem = n;
        first = true;
    }

    static BRB_DEV void part(uint32_t *q, uint32_t w, uint32_t lo, uint32_t hi)
    {
        if (lo == 0 && hi == 3) {
            *q = w;
            return;
        }
        uint8_t *b = reinterpret_cast<uint8_t *>(q);
        for (uint32_t k = lo; k <= hi; k++)
            b[k] = uint8_t(w >> (8 * k));
    }

    BRB_DEV void put(uint32_t v)
    {
        if (rem == 0)
            return;
        const uint32_t n = rem < 4 ? uint32_t(rem) : 4u;
        const uint32_t w0 = o ? (carry | (v << (8 * o))) : v;
        const uint32_t hi = o + n - 1 < 3 ? o + n - 1 : 3u;
        part(p, w0, first ? o : 0u, hi);
        carry = o ? (v >> (32 - 8 * o)) : 0u;
        carry_n = o + n > 4 ? o + n - 4 : 0u;
        ++p;
        first = false;
        rem -= n;
    }

    BRB_DEV void flush()
    {
        if (carry_n)
            part(p, carry, 0, carry_n - 1);
        carry_n = 0;
    }
};

}  // namespace brb_io
