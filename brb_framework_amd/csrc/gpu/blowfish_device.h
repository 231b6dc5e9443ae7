// blowfish_device.h -- device code of the batched Blowfish ECB kernels (64-bit reference words).
//
// Bit-exact to BRB_Blowfish_Encrypt/Decrypt (libbrb_core/crypto/blowfish.c:312-380) with _F
// (:445-462) evaluated on 64-bit words: ((S0[a] + S1[b]) ^ S2[c]) + S3[d], carries kept, the
// indices taken from the low 32 bits only.  A block is one (xl, xr) pair = 16 bytes; blocks are
// independent (ECB, mem_buf.c:1538-1539).
//
// The path is bound by the S-box gathers: 64 random 8-byte LDS reads per 16-byte block.  A
// `ds_read_b64` is serviced in two lane groups of 32, and a bank pair hit by two different
// addresses of one group costs an extra LDS cycle.  One shared 8 KiB table measured 3.15 LDS cycles
// per group instead of 1 (SQ_LDS_BANK_CONFLICT, profiles/r01_pmc_cfg4_blowfish.txt).
//
// bf_rep_kernel replicates the tables 16 times in a 128 KiB LDS image laid out so that the bank
// pair a lane hits depends only on its copy and its half, never on the index:
//
//   byte address = region * 64 KiB + index * 256 + half * 128 + copy * 8
//   region 0: half 0 = S0, half 1 = S1        region 1: half 0 = S2, half 1 = S3
//   copy = lane & 15  ->  bank pair = copy + 16 * half
//
// Lanes j and j + 16 of a group share a copy.  For the S0 / S1 gathers they are sent to opposite
// halves: lanes with h = (lane >> 4) & 1 == 0 read S0[a] in the first instruction and S1[b] in the
// second, lanes with h == 1 the other way round; S0[a] + S1[b] is commutative, so the two results
// are simply added.  Those two gathers are conflict-free (1 cycle per group); the S2 and S3 gathers
// are 2-way (2 cycles per group): 12 LDS cycles per F instead of about 25.
//
// An address is one v_perm_b32: byte 1 <- the index byte of x, bytes 0 and 2 <- a per-lane base
// (copy * 8 + half * 128, region), byte 3 <- 0.  The S3 half is the instruction offset 128.
#pragma once

#include "brb_gpu_common.h"

namespace brb_bf {

// ------------------------------------------------------------------------------------------------
// simple form: one 8 KiB table per workgroup (kept as the A/B baseline, tools/mb/bf_ab.hip)
// ------------------------------------------------------------------------------------------------
BRB_DEV uint64_t f_simple(const uint64_t *__restrict__ S, uint64_t x)
{
    const uint32_t lo = uint32_t(x);
    uint64_t y = S[lo >> 24] + S[256 + ((lo >> 16) & 0xFF)];
    y ^= S[512 + ((lo >> 8) & 0xFF)];
    return y + S[768 + (lo & 0xFF)];
}

template <bool DECRYPT>
BRB_DEV void block_simple(const uint64_t *__restrict__ S, const uint64_t (&P)[18], uint64_t &xl, uint64_t &xr)
{
    uint64_t L = xl, R = xr;
    if (!DECRYPT) {
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
            L ^= P[i];
            R ^= f_simple(S, L);
            R ^= P[i + 1];
            L ^= f_simple(S, R);
        }
        xl = R ^ P[17];
        xr = L ^ P[16];
    } else {
#pragma unroll
        for (int i = 17; i > 1; i -= 2) {
            L ^= P[i];
            R ^= f_simple(S, L);
            R ^= P[i - 1];
            L ^= f_simple(S, R);
        }
        xl = R ^ P[0];
        xr = L ^ P[1];
    }
}

template <int BLOCK, bool DECRYPT>
__global__ __launch_bounds__(BLOCK) void bf_simple_kernel(const uint64_t *__restrict__ ctx, uint8_t *__restrict__ words,
                                                          uint64_t n_blocks)
{
    __shared__ uint64_t S[1024];
    for (int i = threadIdx.x; i < 1024; i += BLOCK)
        S[i] = ctx[18 + i];
    uint64_t P[18];
#pragma unroll
    for (int i = 0; i < 18; i++)
        P[i] = ctx[i];
    __syncthreads();

    const uint64_t stride = uint64_t(gridDim.x) * BLOCK;
    for (uint64_t b = uint64_t(blockIdx.x) * BLOCK + threadIdx.x; b < n_blocks; b += stride) {
        uint64_t v[2];
        __builtin_memcpy(v, __builtin_assume_aligned(words + 16 * b, 8), 16);
        block_simple<DECRYPT>(S, P, v[0], v[1]);
        __builtin_memcpy(__builtin_assume_aligned(words + 16 * b, 8), v, 16);
    }
}

// ------------------------------------------------------------------------------------------------
// replicated form
// ------------------------------------------------------------------------------------------------
constexpr int kRepThreads = 1024;                 // one workgroup per CU (128 KiB of LDS), 4 waves/SIMD
constexpr uint32_t kRepLdsBytes = 128u * 1024u;
constexpr uint32_t kRepQwords = kRepLdsBytes / 8;

// v_perm_b32 selector: byte 0 <- base byte 0, byte 1 <- byte k of x, byte 2 <- base byte 2, byte 3 <- 0.
// Selector values 0-3 pick bytes of the second operand (base), 4-7 bytes of the first (x), 12 = 0x00.
constexpr uint32_t sel_byte(int k) { return (0x0Cu << 24) | (2u << 16) | (uint32_t(4 + k) << 8) | 0u; }

struct RepLane {
    uint32_t cbA, cbB, cbC;    // per-lane bases: copy * 8 | half * 128 | region << 16
    uint32_t selA, selB;       // per-lane selectors of the S0/S1 gathers (swapped for h == 1)

    BRB_DEV void init(uint32_t lane)
    {
        const uint32_t c = lane & 15, h = (lane >> 4) & 1;
        cbA = (c << 3) | (h << 7);
        cbB = (c << 3) | ((h ^ 1) << 7);
        cbC = (c << 3) | (1u << 16);
        selA = h ? sel_byte(2) : sel_byte(3);
        selB = h ? sel_byte(3) : sel_byte(2);
    }
};

// a ^ b ^ c as two v_bitop3_b32 (truth table 0x96); hipcc leaves 64-bit xor chains as v_xor pairs
BRB_DEV uint64_t xor3(uint64_t a, uint64_t b, uint64_t c)
{
    const uint32_t lo = __builtin_amdgcn_bitop3_b32(uint32_t(a), uint32_t(b), uint32_t(c), 0x96);
    const uint32_t hi = __builtin_amdgcn_bitop3_b32(uint32_t(a >> 32), uint32_t(b >> 32), uint32_t(c >> 32), 0x96);
    return (uint64_t(hi) << 32) | lo;
}

BRB_DEV uint64_t lds_q(const uint8_t *lds, uint32_t addr)
{
    return *reinterpret_cast<const uint64_t *>(lds + addr);
}

// F of the low 32 bits x (blowfish.c:445-462 on 64-bit words), split in its gathers and its
// arithmetic so that the gathers of all ILP chains are issued before any chain waits
struct Gath {
    uint64_t A, B, C, D;
};

BRB_DEV Gath gather(const uint8_t *lds, const RepLane &ln, uint32_t x)
{
    Gath g;
    g.A = lds_q(lds, __builtin_amdgcn_perm(x, ln.cbA, ln.selA));          // S0[a] or S1[b]
    g.B = lds_q(lds, __builtin_amdgcn_perm(x, ln.cbB, ln.selB));          // S1[b] or S0[a]
    g.C = lds_q(lds, __builtin_amdgcn_perm(x, ln.cbC, sel_byte(1)));      // S2[c]
    g.D = lds_q(lds, __builtin_amdgcn_perm(x, ln.cbC, sel_byte(0)) + 128); // S3[d]
    return g;
}

BRB_DEV uint64_t f_of(const Gath &g) { return ((g.A + g.B) ^ g.C) + g.D; }

// One half-round on ILP chains: Y ^= F(X) ^ p.
template <int ILP>
BRB_DEV void half_round(const uint8_t *lds, const RepLane &ln, const uint64_t (&X)[ILP], uint64_t (&Y)[ILP],
                        uint64_t p)
{
    Gath g[ILP];
#pragma unroll
    for (int k = 0; k < ILP; k++)
        g[k] = gather(lds, ln, uint32_t(X[k]));
    if (ILP > 1)
        __builtin_amdgcn_sched_barrier(0);   // keep the chains' gathers together (hipcc serialises them)
#pragma unroll
    for (int k = 0; k < ILP; k++)
        Y[k] = xor3(Y[k], f_of(g[k]), p);
}

// ILP independent blocks per lane.  P is the schedule in application order: encrypt P[0..17],
// decrypt P[17..0] (blowfish.c:347-380 walks P backwards).
template <int ILP>
BRB_DEV void blocks_rep(const uint8_t *lds, const RepLane &ln, const uint64_t (&P)[18], uint64_t (&L)[ILP],
                        uint64_t (&R)[ILP])
{
#pragma unroll
    for (int k = 0; k < ILP; k++)
        L[k] ^= P[0];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        half_round<ILP>(lds, ln, L, R, P[2 * j + 1]);
        half_round<ILP>(lds, ln, R, L, P[2 * j + 2]);
    }
    // final swap: (xl, xr) = (R ^ P[17], L) -- L already carries P[16]
#pragma unroll
    for (int k = 0; k < ILP; k++) {
        const uint64_t t = R[k] ^ P[17];
        R[k] = L[k];
        L[k] = t;
    }
}

// Persistent grid, one workgroup per CU.  Iteration: the workgroup takes kRepThreads * ILP
// consecutive blocks, lane t of the workgroup blocks t, t + 1024, ... (each load instruction is one
// contiguous KiB per wave); the next iteration's blocks are loaded before this one's rounds.
template <int ILP, bool DECRYPT>
__global__ __launch_bounds__(kRepThreads) void bf_rep_kernel(const uint64_t *__restrict__ ctx,
                                                             uint64_t *__restrict__ words, uint64_t n_blocks)
{
    __shared__ __attribute__((aligned(16))) uint64_t tab[kRepQwords];
    const uint32_t tid = threadIdx.x;
    for (uint32_t q = tid; q < kRepQwords; q += kRepThreads) {
        const uint32_t region = q >> 13, row = (q >> 5) & 255, half = (q >> 4) & 1;
        tab[q] = ctx[18 + (2 * region + half) * 256 + row];
    }
    uint64_t P[18];
#pragma unroll
    for (int i = 0; i < 18; i++)
        P[i] = ctx[DECRYPT ? 17 - i : i];
    RepLane ln;
    ln.init(tid & 63);
    __syncthreads();
    const uint8_t *lds = reinterpret_cast<const uint8_t *>(tab);

    constexpr uint64_t kPer = uint64_t(kRepThreads) * ILP;
    const uint64_t stride = uint64_t(gridDim.x) * kPer;
    uint64_t base = uint64_t(blockIdx.x) * kPer;
    // Loads are unconditional (a lane past the end re-reads the last block) so that hipcc issues the
    // next iteration's loads before the rounds instead of waiting inside a branch; stores are guarded.
    const uint64_t last = n_blocks - 1;
    uint64_t cl[ILP], cr[ILP];
#pragma unroll
    for (int k = 0; k < ILP; k++) {
        const uint64_t b = min(base + uint64_t(k) * kRepThreads + tid, last);
        cl[k] = words[2 * b];
        cr[k] = words[2 * b + 1];
    }
    while (base < n_blocks) {
        const uint64_t nb = base + stride;
        uint64_t nl[ILP], nr[ILP];
#pragma unroll
        for (int k = 0; k < ILP; k++) {
            const uint64_t b = min(nb + uint64_t(k) * kRepThreads + tid, last);
            nl[k] = words[2 * b];
            nr[k] = words[2 * b + 1];
        }
        blocks_rep<ILP>(lds, ln, P, cl, cr);
        // all ILP chains complete here: otherwise hipcc sinks chain k > 0 below the guarded store of
        // chain 0 and runs the chains one after the other
#pragma unroll
        for (int k = 0; k < ILP; k++)
            asm volatile("" ::"v"(cl[k]), "v"(cr[k]));
#pragma unroll
        for (int k = 0; k < ILP; k++) {
            const uint64_t b = base + uint64_t(k) * kRepThreads + tid;
            if (b < n_blocks) {
                words[2 * b] = cl[k];
                words[2 * b + 1] = cr[k];
            }
            cl[k] = nl[k];
            cr[k] = nr[k];
        }
        base = nb;
    }
}

}  // namespace brb_bf
