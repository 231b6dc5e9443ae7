// blowfish_kernels.hip -- batched Blowfish ECB for gfx950 (MI355X), 64-bit reference words.
//
// Bit-exact to BRB_Blowfish_Encrypt/Decrypt (libbrb_core/crypto/blowfish.c:312-380) with _F
// (:445-462) evaluated on 64-bit words: ((S0[a] + S1[b]) ^ S2[c]) + S3[d] with carries kept.
// A block is one (xl, xr) pair = 16 bytes; blocks are independent (ECB, mem_buf.c:1538-1539),
// so one lane owns one block at a time and a workgroup sweeps a grid-stride range of them.
// The 8 KiB of 64-bit S-boxes live in LDS (one copy per workgroup, loaded once); P[18] is
// wave-uniform and stays in SGPRs.
#include "brb_kernels.h"

namespace {

BRB_DEV uint64_t bf_f(const uint64_t *__restrict__ S, uint64_t x)
{
    const uint32_t lo = uint32_t(x);
    uint64_t y = S[lo >> 24] + S[256 + ((lo >> 16) & 0xFF)];
    y ^= S[512 + ((lo >> 8) & 0xFF)];
    return y + S[768 + (lo & 0xFF)];
}

template <bool DECRYPT>
BRB_DEV void bf_block(const uint64_t *__restrict__ S, const uint64_t (&P)[18], uint64_t &xl, uint64_t &xr)
{
    uint64_t L = xl, R = xr;
    if (!DECRYPT) {
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
            L ^= P[i];
            R ^= bf_f(S, L);
            R ^= P[i + 1];
            L ^= bf_f(S, R);
        }
        xl = R ^ P[17];
        xr = L ^ P[16];
    } else {
#pragma unroll
        for (int i = 17; i > 1; i -= 2) {
            L ^= P[i];
            R ^= bf_f(S, L);
            R ^= P[i - 1];
            L ^= bf_f(S, R);
        }
        xl = R ^ P[0];
        xr = L ^ P[1];
    }
}

template <int BLOCK, bool DECRYPT>
__global__ __launch_bounds__(BLOCK) void bf_ecb_kernel(const uint64_t *__restrict__ ctx, uint8_t *__restrict__ words,
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
        bf_block<DECRYPT>(S, P, v[0], v[1]);
        __builtin_memcpy(__builtin_assume_aligned(words + 16 * b, 8), v, 16);
    }
}

constexpr int kBlock = 256;

}  // namespace

namespace brb {

hipError_t launch_blowfish(const uint64_t *ctx_dev, uint64_t *words, uint64_t n_blocks, bool decrypt, hipStream_t s)
{
    if (n_blocks == 0)
        return hipSuccess;
    uint64_t want = (n_blocks + kBlock - 1) / kBlock;
    // grid-stride: enough workgroups to fill 256 CUs several times, each amortising its S-box load
    const uint64_t cap = 256 * 8;
    const unsigned g = unsigned(want < cap ? want : cap);
    uint8_t *w = reinterpret_cast<uint8_t *>(words);
    if (decrypt)
        bf_ecb_kernel<kBlock, true><<<g, kBlock, 0, s>>>(ctx_dev, w, n_blocks);
    else
        bf_ecb_kernel<kBlock, false><<<g, kBlock, 0, s>>>(ctx_dev, w, n_blocks);
    return hipGetLastError();
}

}  // namespace brb
