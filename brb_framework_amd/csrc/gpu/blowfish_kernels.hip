// blowfish_kernels.hip -- batched Blowfish ECB for gfx950 (MI355X), 64-bit reference words.
//
// Launches brb_bf::bf_rep_kernel (blowfish_device.h): S-boxes replicated 16x in a bank-aware
// 128 KiB LDS image, one 1024-thread workgroup per CU, two blocks per lane, P in SGPRs.
// Bit-exact to BRB_Blowfish_Encrypt/Decrypt (libbrb_core/crypto/blowfish.c:312-380).
#include "blowfish_device.h"
#include "brb_kernels.h"

namespace {

constexpr int kIlp = 2;   // tools/mb/bf_ab.hip: ILP 1/2/3/4 = 520/499/519/525 us per GiB

int cu_count()
{
    static int n = 0;
    if (n == 0) {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
            n = v;
        else
            n = 256;
    }
    return n;
}

// MemBufferDecryptData's "padding gremlin" stop (mem_buf.c:1595-1596): first pair with a zero word
__global__ __launch_bounds__(256) void first_zero_pair_kernel(const uint64_t *__restrict__ w, uint64_t n,
                                                              unsigned long long *first)
{
    unsigned long long best = ~0ull;
    for (uint64_t b = uint64_t(blockIdx.x) * 256 + threadIdx.x; b < n; b += uint64_t(gridDim.x) * 256)
        if (w[2 * b] == 0 || w[2 * b + 1] == 0) {
            best = b;
            break;        // later b of this lane are larger
        }
    if (best != ~0ull)
        atomicMin(first, best);
}

}  // namespace

namespace brb {

hipError_t launch_first_zero_pair(const uint64_t *words, uint64_t n_blocks, unsigned long long *first, hipStream_t s)
{
    if (n_blocks == 0)
        return hipSuccess;
    const uint64_t want = (n_blocks + 255) / 256;
    const unsigned g = unsigned(want < 2048 ? want : 2048);
    first_zero_pair_kernel<<<g, 256, 0, s>>>(words, n_blocks, first);
    return hipGetLastError();
}

hipError_t launch_blowfish(const uint64_t *ctx_dev, uint64_t *words, uint64_t n_blocks, bool decrypt, hipStream_t s)
{
    if (n_blocks == 0)
        return hipSuccess;
    const uint64_t per = uint64_t(brb_bf::kRepThreads) * kIlp;
    const uint64_t want = (n_blocks + per - 1) / per;
    const uint64_t cap = uint64_t(cu_count());   // persistent: one workgroup per CU (128 KiB LDS each)
    const unsigned g = unsigned(want < cap ? want : cap);
    if (decrypt)
        brb_bf::bf_rep_kernel<kIlp, true><<<g, brb_bf::kRepThreads, 0, s>>>(ctx_dev, words, n_blocks);
    else
        brb_bf::bf_rep_kernel<kIlp, false><<<g, brb_bf::kRepThreads, 0, s>>>(ctx_dev, words, n_blocks);
    return hipGetLastError();
}

}  // namespace brb
