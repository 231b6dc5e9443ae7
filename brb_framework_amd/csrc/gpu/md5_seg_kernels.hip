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
    __shared__ __attribute__((aligned(8192))) uint32_t blk[kBlock / 64][brb_md5::kRingWords][64];   // 8 KiB per wave
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t r = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (r >= n_rec)
        return;
    brb_md5::Funnel f;
    f.init(&blk[wave][0][lane]);
    const uint64_t k1 = first[r + 1];
    for (uint64_t k = first[r]; k < k1; k++) {         // 64-byte blocks, the next one in flight
        // The segment is read as a range starting e = (bytes digested so far) mod 4 bytes before
        // it, so its words fall on the digest's word boundaries (as metadata_unpack_kernel): those
        // e bytes are the carried ones (Funnel::head), never loaded from below the segment.
        const uint64_t len = slen[k];
        if (len == 0)                                   // no bytes: its address need not be memory
            continue;
        const uint8_t *a = data + soff[k];
        const uint32_t e = f.nacc;
        const uint64_t n = len + e;
        brb_io::BlockSrc src;
        src.init(a - e, n, a);
        for (uint64_t c = 0; c < n; c += 64) {
            uint32_t w[16];
            src.fetch(w);
            if (c == 0)
                w[0] = f.head(w[0]);
            const uint64_t left = n - c;
            if (left >= 64)
                f.put16w(w);
            else
                f.put_tail(w, uint32_t(left));
            f.pump();
        }
        if ((n & 63) == 0) {                            // ended on a whole block: nothing carried
            f.acc = 0;
            f.nacc = 0;
        }
        f.total += len;
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
