// md5_seg_kernels.hip -- MD5 of a list of byte segments per record.
//
// MetaDataHeaderLoadData (libbrb_core/data/utils/meta_data.c:397-433) digests the items of one
// MetaData as BRB_MD5Init, one BRB_MD5UpdateBig per item, BRB_MD5Final: the MD5 of the items'
// concatenation, the items scattered in memory.  Batched: one record (one MetaData) per lane, its
// segments (items) walked in order.  Segments start and end at any byte, so each lane funnels its
// bytes into whole 32-bit words (a 64-bit carry holds the 0..3 bytes left over from the previous
// segment) and parks them in a private 64-byte block buffer in LDS, word k of lane l at
// (k * 64 + l) * 4 -- every access of lane l hits bank l.  A full block is compressed from there.
#include "brb_kernels.h"
#include "byte_stream.h"
#include "md5_device.h"

namespace {

constexpr int kBlock = 256;

__global__ __launch_bounds__(kBlock) void md5_seg_kernel(const uint8_t *__restrict__ data,
                                                         const uint64_t *__restrict__ soff,
                                                         const uint32_t *__restrict__ slen,
                                                         const uint64_t *__restrict__ first, uint64_t n_rec,
                                                         uint8_t *__restrict__ out)
{
    __shared__ uint32_t blk[kBlock / 64][16][64];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t r = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (r >= n_rec)
        return;
    uint32_t *bb = &blk[wave][0][lane];   // word k at bb[64 k]
    Md5State st = md5_iv();
    uint32_t w[16];
    uint64_t acc = 0, total = 0;
    uint32_t nacc = 0, wpos = 0;
    const uint64_t k1 = first[r + 1];
    for (uint64_t k = first[r]; k < k1; k++) {
        const uint64_t len = slen[k];
        total += len;
        brb_io::Src src;
        src.init(data + soff[k], len);
        for (uint64_t c = 0; c < len; c += 4) {
            const uint32_t nb = len - c >= 4 ? 4u : uint32_t(len - c);
            acc |= uint64_t(src.next()) << (8 * nacc);
            nacc += nb;
            if (nacc >= 4) {
                bb[64 * wpos] = uint32_t(acc);
                acc >>= 32;
                nacc -= 4;
                if (++wpos == 16) {
#pragma unroll
                    for (int i = 0; i < 16; i++)
                        w[i] = bb[64 * i];
                    md5_compress(st, w);
                    wpos = 0;
                }
            }
        }
    }
    // BRB_MD5Final (md5.c:134-168): 0x80, zeros, 64-bit bit count
    bb[64 * wpos] = uint32_t(acc | (uint64_t(0x80) << (8 * nacc)));
    ++wpos;
#pragma unroll
    for (uint32_t i = 0; i < 16; i++)
        w[i] = i < wpos ? bb[64 * i] : 0u;
    if (wpos > 14) {
        md5_compress(st, w);
#pragma unroll
        for (int i = 0; i < 16; i++)
            w[i] = 0;
    }
    w[14] = uint32_t(total << 3);
    w[15] = uint32_t(total >> 29);
    md5_compress(st, w);
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
