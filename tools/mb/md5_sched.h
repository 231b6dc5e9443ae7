// md5_sched.h -- hand-scheduled MD5 compression (inline asm), kept for the microbenchmarks
// (tools/mb/md5_ab.hip, md5_dma_stamps.hip).  It measured 6-13 % slower than hipcc's schedule of
// md5_compress and is not part of the product.
#pragma once

#include "md5_device.h"

// ---- hand-scheduled compression for the latency-bound regime (one wave per SIMD) ----------------
// With ~one wave per SIMD (cfg2: 65 536 records = 1 024 waves on 1 024 SIMDs) a step costs its
// dependent-chain latency, ~8.3 cycles per dependent VALU op on gfx950 (tools/mb/valu_latency.hip),
// not its issue slots.  hipcc schedules the off-chain add (a + m + K) between F and the add that
// consumes it, which puts it on the chain (~37 cycles/step measured).  These steps fix the order:
//   bitop3 F(b,c,d) | add3 next X = d + m' + K' (off-chain) | add F + X | alignbit | add b
// = 4 chain ops (33 cycles), and for the F3 = b^c^d rounds
//   xad (b ^ cd) + X | add3 next X | alignbit | xor next cd = b ^ c (off-chain) | add b
// = 3 chain ops (25 cycles).  Same function as md5_compress (bit-exact, tested).
// v_bitop3 truth tables (index = b<<2 | c<<1 | d): F1 = 0xCA, F2 = 0xE4, F4 = 0x39.
template <int IMM, int S, bool CD, bool NEXT>
BRB_DEV void md5_step_bitop(uint32_t &a, uint32_t b, uint32_t c, uint32_t d, uint32_t &cd, uint32_t &x, uint32_t an,
                            uint32_t mn, uint32_t kn)
{
    uint32_t f, xn, cdn;
    if constexpr (NEXT && CD) {
        asm volatile("v_bitop3_b32 %[f], %[b], %[c], %[d] bitop3:%[imm]\n\t"
                     "v_add3_u32 %[xn], %[an], %[mn], %[kn]\n\t"
                     "v_add_u32 %[f], %[f], %[x]\n\t"
                     "v_xor_b32 %[cdn], %[b], %[c]\n\t"
                     "v_alignbit_b32 %[f], %[f], %[f], %[rs]\n\t"
                     "v_add_u32 %[a], %[f], %[b]"
                     : [a] "=v"(a), [f] "=&v"(f), [xn] "=&v"(xn), [cdn] "=&v"(cdn)
                     : [b] "v"(b), [c] "v"(c), [d] "v"(d), [x] "v"(x), [an] "v"(an), [mn] "v"(mn), [kn] "s"(kn),
                       [imm] "i"(IMM), [rs] "i"(32 - S));
        x = xn;
        cd = cdn;
    } else if constexpr (NEXT) {
        asm volatile("v_bitop3_b32 %[f], %[b], %[c], %[d] bitop3:%[imm]\n\t"
                     "v_add3_u32 %[xn], %[an], %[mn], %[kn]\n\t"
                     "v_add_u32 %[f], %[f], %[x]\n\t"
                     "v_alignbit_b32 %[f], %[f], %[f], %[rs]\n\t"
                     "v_add_u32 %[a], %[f], %[b]"
                     : [a] "=v"(a), [f] "=&v"(f), [xn] "=&v"(xn)
                     : [b] "v"(b), [c] "v"(c), [d] "v"(d), [x] "v"(x), [an] "v"(an), [mn] "v"(mn), [kn] "s"(kn),
                       [imm] "i"(IMM), [rs] "i"(32 - S));
        x = xn;
    } else {
        asm volatile("v_bitop3_b32 %[f], %[b], %[c], %[d] bitop3:%[imm]\n\t"
                     "v_add_u32 %[f], %[f], %[x]\n\t"
                     "v_alignbit_b32 %[f], %[f], %[f], %[rs]\n\t"
                     "v_add_u32 %[a], %[f], %[b]"
                     : [a] "=v"(a), [f] "=&v"(f)
                     : [b] "v"(b), [c] "v"(c), [d] "v"(d), [x] "v"(x), [imm] "i"(IMM), [rs] "i"(32 - S));
        (void)an, (void)mn, (void)kn, (void)cd;
    }
}

template <int S, bool CD, bool NEXT>
BRB_DEV void md5_step_xad(uint32_t &a, uint32_t b, uint32_t c, uint32_t &cd, uint32_t &x, uint32_t an, uint32_t mn,
                          uint32_t kn)
{
    static_assert(NEXT, "the last MD5 step is an F4 step");
    uint32_t f, xn, cdn;
    if constexpr (CD) {
        asm volatile("v_xad_u32 %[f], %[b], %[cd], %[x]\n\t"
                     "v_add3_u32 %[xn], %[an], %[mn], %[kn]\n\t"
                     "v_alignbit_b32 %[f], %[f], %[f], %[rs]\n\t"
                     "v_xor_b32 %[cdn], %[b], %[c]\n\t"
                     "v_add_u32 %[a], %[f], %[b]"
                     : [a] "=v"(a), [f] "=&v"(f), [xn] "=&v"(xn), [cdn] "=&v"(cdn)
                     : [b] "v"(b), [c] "v"(c), [cd] "v"(cd), [x] "v"(x), [an] "v"(an), [mn] "v"(mn), [kn] "s"(kn),
                       [rs] "i"(32 - S));
        cd = cdn;
    } else {
        asm volatile("v_xad_u32 %[f], %[b], %[cd], %[x]\n\t"
                     "v_add3_u32 %[xn], %[an], %[mn], %[kn]\n\t"
                     "v_alignbit_b32 %[f], %[f], %[f], %[rs]\n\t"
                     "v_add_u32 %[a], %[f], %[b]"
                     : [a] "=v"(a), [f] "=&v"(f), [xn] "=&v"(xn)
                     : [b] "v"(b), [cd] "v"(cd), [x] "v"(x), [an] "v"(an), [mn] "v"(mn), [kn] "s"(kn), [rs] "i"(32 - S));
        (void)c;
    }
    x = xn;
}

BRB_DEV void md5_compress_sched(Md5State &st, const uint32_t (&m)[16])
{
    uint32_t a = st.a, b = st.b, c = st.c, d = st.d;
    uint32_t cd = 0;
    uint32_t x = a + m[0] + 0xd76aa478u;
    md5_step_bitop<0xCA, 7, false, true>(a, b, c, d, cd, x, d, m[1], 0xe8c7b756u);
    md5_step_bitop<0xCA, 12, false, true>(d, a, b, c, cd, x, c, m[2], 0x242070dbu);
    md5_step_bitop<0xCA, 17, false, true>(c, d, a, b, cd, x, b, m[3], 0xc1bdceeeu);
    md5_step_bitop<0xCA, 22, false, true>(b, c, d, a, cd, x, a, m[4], 0xf57c0fafu);
    md5_step_bitop<0xCA, 7, false, true>(a, b, c, d, cd, x, d, m[5], 0x4787c62au);
    md5_step_bitop<0xCA, 12, false, true>(d, a, b, c, cd, x, c, m[6], 0xa8304613u);
    md5_step_bitop<0xCA, 17, false, true>(c, d, a, b, cd, x, b, m[7], 0xfd469501u);
    md5_step_bitop<0xCA, 22, false, true>(b, c, d, a, cd, x, a, m[8], 0x698098d8u);
    md5_step_bitop<0xCA, 7, false, true>(a, b, c, d, cd, x, d, m[9], 0x8b44f7afu);
    md5_step_bitop<0xCA, 12, false, true>(d, a, b, c, cd, x, c, m[10], 0xffff5bb1u);
    md5_step_bitop<0xCA, 17, false, true>(c, d, a, b, cd, x, b, m[11], 0x895cd7beu);
    md5_step_bitop<0xCA, 22, false, true>(b, c, d, a, cd, x, a, m[12], 0x6b901122u);
    md5_step_bitop<0xCA, 7, false, true>(a, b, c, d, cd, x, d, m[13], 0xfd987193u);
    md5_step_bitop<0xCA, 12, false, true>(d, a, b, c, cd, x, c, m[14], 0xa679438eu);
    md5_step_bitop<0xCA, 17, false, true>(c, d, a, b, cd, x, b, m[15], 0x49b40821u);
    md5_step_bitop<0xCA, 22, false, true>(b, c, d, a, cd, x, a, m[1], 0xf61e2562u);
    md5_step_bitop<0xE4, 5, false, true>(a, b, c, d, cd, x, d, m[6], 0xc040b340u);
    md5_step_bitop<0xE4, 9, false, true>(d, a, b, c, cd, x, c, m[11], 0x265e5a51u);
    md5_step_bitop<0xE4, 14, false, true>(c, d, a, b, cd, x, b, m[0], 0xe9b6c7aau);
    md5_step_bitop<0xE4, 20, false, true>(b, c, d, a, cd, x, a, m[5], 0xd62f105du);
    md5_step_bitop<0xE4, 5, false, true>(a, b, c, d, cd, x, d, m[10], 0x02441453u);
    md5_step_bitop<0xE4, 9, false, true>(d, a, b, c, cd, x, c, m[15], 0xd8a1e681u);
    md5_step_bitop<0xE4, 14, false, true>(c, d, a, b, cd, x, b, m[4], 0xe7d3fbc8u);
    md5_step_bitop<0xE4, 20, false, true>(b, c, d, a, cd, x, a, m[9], 0x21e1cde6u);
    md5_step_bitop<0xE4, 5, false, true>(a, b, c, d, cd, x, d, m[14], 0xc33707d6u);
    md5_step_bitop<0xE4, 9, false, true>(d, a, b, c, cd, x, c, m[3], 0xf4d50d87u);
    md5_step_bitop<0xE4, 14, false, true>(c, d, a, b, cd, x, b, m[8], 0x455a14edu);
    md5_step_bitop<0xE4, 20, false, true>(b, c, d, a, cd, x, a, m[13], 0xa9e3e905u);
    md5_step_bitop<0xE4, 5, false, true>(a, b, c, d, cd, x, d, m[2], 0xfcefa3f8u);
    md5_step_bitop<0xE4, 9, false, true>(d, a, b, c, cd, x, c, m[7], 0x676f02d9u);
    md5_step_bitop<0xE4, 14, false, true>(c, d, a, b, cd, x, b, m[12], 0x8d2a4c8au);
    md5_step_bitop<0xE4, 20, true, true>(b, c, d, a, cd, x, a, m[5], 0xfffa3942u);
    md5_step_xad<4, true, true>(a, b, c, cd, x, d, m[8], 0x8771f681u);
    md5_step_xad<11, true, true>(d, a, b, cd, x, c, m[11], 0x6d9d6122u);
    md5_step_xad<16, true, true>(c, d, a, cd, x, b, m[14], 0xfde5380cu);
    md5_step_xad<23, true, true>(b, c, d, cd, x, a, m[1], 0xa4beea44u);
    md5_step_xad<4, true, true>(a, b, c, cd, x, d, m[4], 0x4bdecfa9u);
    md5_step_xad<11, true, true>(d, a, b, cd, x, c, m[7], 0xf6bb4b60u);
    md5_step_xad<16, true, true>(c, d, a, cd, x, b, m[10], 0xbebfbc70u);
    md5_step_xad<23, true, true>(b, c, d, cd, x, a, m[13], 0x289b7ec6u);
    md5_step_xad<4, true, true>(a, b, c, cd, x, d, m[0], 0xeaa127fau);
    md5_step_xad<11, true, true>(d, a, b, cd, x, c, m[3], 0xd4ef3085u);
    md5_step_xad<16, true, true>(c, d, a, cd, x, b, m[6], 0x04881d05u);
    md5_step_xad<23, true, true>(b, c, d, cd, x, a, m[9], 0xd9d4d039u);
    md5_step_xad<4, true, true>(a, b, c, cd, x, d, m[12], 0xe6db99e5u);
    md5_step_xad<11, true, true>(d, a, b, cd, x, c, m[15], 0x1fa27cf8u);
    md5_step_xad<16, true, true>(c, d, a, cd, x, b, m[2], 0xc4ac5665u);
    md5_step_xad<23, false, true>(b, c, d, cd, x, a, m[0], 0xf4292244u);
    md5_step_bitop<0x39, 6, false, true>(a, b, c, d, cd, x, d, m[7], 0x432aff97u);
    md5_step_bitop<0x39, 10, false, true>(d, a, b, c, cd, x, c, m[14], 0xab9423a7u);
    md5_step_bitop<0x39, 15, false, true>(c, d, a, b, cd, x, b, m[5], 0xfc93a039u);
    md5_step_bitop<0x39, 21, false, true>(b, c, d, a, cd, x, a, m[12], 0x655b59c3u);
    md5_step_bitop<0x39, 6, false, true>(a, b, c, d, cd, x, d, m[3], 0x8f0ccc92u);
    md5_step_bitop<0x39, 10, false, true>(d, a, b, c, cd, x, c, m[10], 0xffeff47du);
    md5_step_bitop<0x39, 15, false, true>(c, d, a, b, cd, x, b, m[1], 0x85845dd1u);
    md5_step_bitop<0x39, 21, false, true>(b, c, d, a, cd, x, a, m[8], 0x6fa87e4fu);
    md5_step_bitop<0x39, 6, false, true>(a, b, c, d, cd, x, d, m[15], 0xfe2ce6e0u);
    md5_step_bitop<0x39, 10, false, true>(d, a, b, c, cd, x, c, m[6], 0xa3014314u);
    md5_step_bitop<0x39, 15, false, true>(c, d, a, b, cd, x, b, m[13], 0x4e0811a1u);
    md5_step_bitop<0x39, 21, false, true>(b, c, d, a, cd, x, a, m[4], 0xf7537e82u);
    md5_step_bitop<0x39, 6, false, true>(a, b, c, d, cd, x, d, m[11], 0xbd3af235u);
    md5_step_bitop<0x39, 10, false, true>(d, a, b, c, cd, x, c, m[2], 0x2ad7d2bbu);
    md5_step_bitop<0x39, 15, false, true>(c, d, a, b, cd, x, b, m[9], 0xeb86d391u);
    md5_step_bitop<0x39, 21, false, false>(b, c, d, a, cd, x, 0u, 0u, 0u);

    st.a += a;
    st.b += b;
    st.c += c;
    st.d += d;
}

