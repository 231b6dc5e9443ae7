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

}  // namespace

namespace brb {

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
