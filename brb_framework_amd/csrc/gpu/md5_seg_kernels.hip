// md5_seg_kernels.hip -- MD5 of a list of byte segments per record.
//
// MetaDataHeaderLoadData (libbrb_core/data/utils/meta_data.c:397-433) digests the items of one
// MetaData as BRB_MD5Init, one BRB_MD5UpdateBig per item, BRB_MD5Final: the MD5 of the items'
// concatenation, the items scattered in memory.  Batched: one record (one MetaData) per lane, its
// segments (items) walked in order in 64-byte blocks (brb_io::BlockSrc, the next block in flight,
// and the next segment's first block in flight while the current one is hashed), their bytes
// funnelled into the lane's MD5 (md5_funnel.h).
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
    // Segment k is read as a range starting e_k = (bytes before it) mod 4 bytes before it, so its
    // words fall on the digest's word boundaries (as metadata_unpack_kernel): those e bytes are the
    // carried ones (Funnel::head), never loaded from below the segment.  e_k depends only on the
    // lengths, so segment k + 1's source starts (its first block in flight) before segment k is
    // hashed: the two sources alternate (sa, sb: no register copies), and a segment's first block no
    // longer waits a whole HBM round trip after the previous segment's last one.
    uint64_t k = first[r], before = 0;
    auto skip_empty = [&](uint64_t kk) {                // the next segment with bytes (an empty one's
        while (kk < k1 && slen[kk] == 0)                // address need not be memory)
            kk++;
        return kk;
    };
    auto start = [&](brb_io::BlockSrc &src, uint64_t kk, uint64_t pre, uint64_t &len) {
        len = slen[kk];
        const uint8_t *a = data + soff[kk];
        const uint32_t e = uint32_t(pre & 3);
        src.init(a - e, len + e, a);
    };
    auto run = [&](brb_io::BlockSrc &src, uint64_t len) {   // 64-byte blocks, the next one in flight
        const uint32_t e = f.nacc;
        const uint64_t n = len + e;
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
    };
    brb_io::BlockSrc sa, sb;
    uint64_t la = 0, lb = 0;
    k = skip_empty(k);
    if (k < k1)
        start(sa, k, before, la);
    while (k < k1) {
        uint64_t kb = skip_empty(k + 1);
        if (kb < k1)
            start(sb, kb, before + la, lb);
        run(sa, la);
        before += la;
        if (kb >= k1)
            break;
        k = skip_empty(kb + 1);
        if (k < k1)
            start(sa, k, before + lb, la);
        run(sb, lb);
        before += lb;
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
