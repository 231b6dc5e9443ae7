// md5_seg_kernels.hip -- MD5 of a list of byte segments per record.
//
// MetaDataHeaderLoadData (libbrb_core/data/utils/meta_data.c:397-433) digests the items of one
// MetaData as BRB_MD5Init, one BRB_MD5UpdateBig per item, BRB_MD5Final: the MD5 of the items'
// concatenation, the items scattered in memory.  Batched: one record (one MetaData) per lane, its
// segments (items) walked in order in 64-byte blocks (brb_io::BlockSrc, the next block in flight),
// their bytes funnelled into the lane's MD5 (md5_funnel.h).
#include "brb_kernels.h"
#include "byte_stream.h"
#include "md5_funnel.h"

namespace {

constexpr int kBlock = 256;

__global__ __launch_bounds__(kBlock) void md5_seg_kernel(const uint8_t *__restrict__ data,
                                                         const uint64_t *__restrict__ soff,
                                                         const uint32_t *__restrict__ slen,
                                                         const uint64_t *__restrict__ first, uint64_t n_rec,
                                                         uint8_t *__restrict__ out)
{
    __shared__ uint32_t blk[kBlock / 64][brb_md5::kRingWords][64];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t r = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (r >= n_rec)
        return;
    brb_md5::Funnel f;
    f.init(&blk[wave][0][lane]);
    const uint64_t k1 = first[r + 1];
    for (uint64_t k = first[r]; k < k1; k++) {         // 64-byte blocks, the next one in flight
        const uint64_t len = slen[k];
        brb_io::BlockSrc src;
        src.init(data + soff[k], len);
        for (uint64_t c = 0; c < len; c += 64) {
            uint32_t w[16];
            src.fetch(w);
            const uint64_t left = len - c;
            if (left >= 64) {
#pragma unroll
                for (int i = 0; i < 16; i++)
                    f.put4(w[i]);
            } else {
#pragma unroll
                for (uint32_t i = 0; i < 16; i++)
                    if (4 * i < left)
                        f.put(w[i], left - 4 * i >= 4 ? 4u : uint32_t(left - 4 * i));
            }
            f.pump();
        }
    }
    const Md5State st = f.finish();
    const uint4 v = make_uint4(st.a, st.b, st.c, st.d);
    __builtin_memcpy(out + 16 * r, &v, 16);
}

}  // namespace

namespace brb {

hipError_t launch_md5_segments(const uint8_t *data, const uint64_t *soff, const uint32_t *slen, const uint64_t *first,
                               uint64_t n_rec, uint8_t *out, hipStream_t s)
{
    if (n_rec == 0)
        return hipSuccess;
    md5_seg_kernel<<<unsigned((n_rec + kBlock - 1) / kBlock), kBlock, 0, s>>>(data, soff, slen, first, n_rec, out);
    return hipGetLastError();
}

}  // namespace brb
