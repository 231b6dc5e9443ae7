// md5_kernels.hip -- batched MD5 for gfx950 (MI355X).
//
// One record per lane: a digest is a serial Merkle-Damgard chain (md5.c:98-106), so the
// parallelism is across records.  Each lane streams its own record through registers with a
// one-block software prefetch; the record's 16 message words are consumed straight from VGPRs.
// Digest of record r = BRB_MD5Init + BRB_MD5Update(record) + BRB_MD5Final (md5.c:38-168).
#include "brb_kernels.h"
#include "byte_stream.h"
#include "digest_dma.h"
#include "digest_var_line.h"
#include "md5_device.h"

namespace {

struct Md5Alg;

struct Out16 {
    template <bool ALIGNED>
    static BRB_DEV void store(uint8_t *out, uint64_t r, const Md5State &st)
    {
        const uint4 v = make_uint4(st.a, st.b, st.c, st.d);
        if (ALIGNED)
            reinterpret_cast<uint4 *>(out)[r] = v;
        else
            __builtin_memcpy(out + 16 * r, &v, 16);
    }
};

struct Md5Alg {
    using State = Md5State;
    static BRB_DEV State iv() { return md5_iv(); }
    static BRB_DEV void compress(State &st, uint32_t (&w)[16]) { md5_compress(st, w); }
    static BRB_DEV void finish(State &st, uint32_t (&w)[16], uint32_t t, uint64_t len) { md5_finish(st, w, t, len); }
    static BRB_DEV void pad_only(State &st, uint64_t len) { md5_pad_only(st, len); }
    template <bool ALIGNED>
    static BRB_DEV void store(uint8_t *out, uint64_t r, const State &st) { Out16::store<ALIGNED>(out, r, st); }
};

// Fixed-stride records, record base 4-byte aligned (data 4-aligned and rec_len % 4 == 0).
template <int BLOCK, bool OUT_ALIGNED>
__global__ __launch_bounds__(BLOCK) void md5_fixed_a4_kernel(const uint8_t *__restrict__ data, uint32_t rec_len,
                                                              uint64_t n_rec, uint8_t *__restrict__ out)
{
    const uint64_t r = uint64_t(blockIdx.x) * BLOCK + threadIdx.x;
    if (r >= n_rec)
        return;
    const uint8_t *p = data + r * rec_len;
    const uint32_t nfull = rec_len >> 6;
    Md5State st = md5_iv();
    uint32_t w[16];

    if (nfull) {
        uint4 n0 = ld16_a4(p), n1 = ld16_a4(p + 16), n2 = ld16_a4(p + 32), n3 = ld16_a4(p + 48);
        for (uint32_t b = 0; b < nfull; ++b) {
            const uint4 c0 = n0, c1 = n1, c2 = n2, c3 = n3;
            // prefetch the next block (the last iteration re-reads its own block: in bounds)
            const uint8_t *q = p + 64u * (b + 1 < nfull ? b + 1 : b);
            n0 = ld16_a4(q);
            n1 = ld16_a4(q + 16);
            n2 = ld16_a4(q + 32);
            n3 = ld16_a4(q + 48);
            w[0] = c0.x; w[1] = c0.y; w[2] = c0.z; w[3] = c0.w;
            w[4] = c1.x; w[5] = c1.y; w[6] = c1.z; w[7] = c1.w;
            w[8] = c2.x; w[9] = c2.y; w[10] = c2.z; w[11] = c2.w;
            w[12] = c3.x; w[13] = c3.y; w[14] = c3.z; w[15] = c3.w;
            md5_compress(st, w);
        }
    }
    const uint32_t t = rec_len & 63;
    const uint8_t *pt = p + 64u * nfull;
#pragma unroll
    for (uint32_t i = 0; i < 16; i++)
        w[i] = tail_word_a4(pt, t, i);
    md5_finish(st, w, t, rec_len);
    Out16::store<OUT_ALIGNED>(out, r, st);
}

// General records: byte offsets and lengths, any alignment.  FIXED: offset = r * rec_len.
template <int BLOCK, bool FIXED, bool OUT_ALIGNED>
__global__ __launch_bounds__(BLOCK) void md5_any_kernel(const uint8_t *__restrict__ data, const uint64_t *__restrict__ offs,
                                                         const uint32_t *__restrict__ lens, uint32_t rec_len,
                                                         uint64_t n_rec, uint8_t *__restrict__ out)
{
    const uint64_t r = uint64_t(blockIdx.x) * BLOCK + threadIdx.x;
    if (r >= n_rec)
        return;
    const uint8_t *a = data + (FIXED ? r * rec_len : offs[r]);
    const uint64_t len = FIXED ? rec_len : lens[r];
    const uint64_t nfull = len >> 6;
    Md5State st = md5_iv();
    uint32_t w[16];
    brb_io::BlockSrc src;           // the next 64-byte block is always in flight
    src.init(a, len);
    for (uint64_t b = 0; b < nfull; ++b) {
        src.fetch(w);
        md5_compress(st, w);
    }
    src.fetch(w);                   // tail (bytes past the record read as 0)
    brb_io::add_marker(w, len);
    md5_finish(st, w, uint32_t(len & 63), len);
    Out16::store<OUT_ALIGNED>(out, r, st);
}

constexpr int kBlock = 256;

inline unsigned grid_for(uint64_t n)
{
    return unsigned((n + kBlock - 1) / kBlock);
}

}  // namespace

namespace brb {

hipError_t launch_md5_fixed(const uint8_t *data, uint32_t rec_len, uint64_t n_rec, uint8_t *out, hipStream_t s)
{
    if (n_rec == 0)
        return hipSuccess;
    const bool out_al = (reinterpret_cast<uintptr_t>(out) & 15) == 0;
    const bool in_a4 = (reinterpret_cast<uintptr_t>(data) & 3) == 0 && (rec_len & 3) == 0;
    const unsigned g = grid_for(n_rec);
    if (brb_digest::dma_supported(rec_len))
        return brb_digest::launch_fixed_dma<Md5Alg>(data, rec_len, n_rec, out, out_al, s);
    if (in_a4) {
        if (out_al)
            md5_fixed_a4_kernel<kBlock, true><<<g, kBlock, 0, s>>>(data, rec_len, n_rec, out);
        else
            md5_fixed_a4_kernel<kBlock, false><<<g, kBlock, 0, s>>>(data, rec_len, n_rec, out);
    } else {
        if (out_al)
            md5_any_kernel<kBlock, true, true><<<g, kBlock, 0, s>>>(data, nullptr, nullptr, rec_len, n_rec, out);
        else
            md5_any_kernel<kBlock, true, false><<<g, kBlock, 0, s>>>(data, nullptr, nullptr, rec_len, n_rec, out);
    }
    return hipGetLastError();
}

hipError_t launch_md5_var(const uint8_t *data, const uint64_t *offs, const uint32_t *lens, uint64_t n_rec,
                          uint8_t *out, hipStream_t s)
{
    if (n_rec == 0)
        return hipSuccess;
    const bool out_al = (reinterpret_cast<uintptr_t>(out) & 15) == 0;
    // line-aligned LDS-DMA staging (digest_var_line.h); the per-lane kernel below is its A/B baseline
    if (brb_digest::var_line_enabled())
        return brb_digest::launch_var_line<Md5Alg>(data, offs, lens, n_rec, out, out_al, s);
    const unsigned g = grid_for(n_rec);
    if (out_al)
        md5_any_kernel<kBlock, false, true><<<g, kBlock, 0, s>>>(data, offs, lens, 0, n_rec, out);
    else
        md5_any_kernel<kBlock, false, false><<<g, kBlock, 0, s>>>(data, offs, lens, 0, n_rec, out);
    return hipGetLastError();
}

}  // namespace brb
