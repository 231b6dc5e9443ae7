// sha1_kernels.hip -- batched SHA-1 for gfx950 (MI355X), one record per lane.
// Digest of record r = BrbSha1_Do(record) (libbrb_core/crypto/sha1.c:203-216): 20 raw bytes,
// big-endian state words (sha1.c:185-188).
#include "brb_kernels.h"
#include "byte_stream.h"
#include "digest_dma.h"
#include "digest_var_line.h"
#include "sha1_device.h"

namespace {

template <bool ALIGNED>
BRB_DEV void store20(uint8_t *out, uint64_t r, const Sha1State &st)
{
    const uint32_t v[5] = {__builtin_bswap32(st.a), __builtin_bswap32(st.b), __builtin_bswap32(st.c),
                           __builtin_bswap32(st.d), __builtin_bswap32(st.e)};
    uint8_t *o = out + 20 * r;
    if (ALIGNED) {
        uint32_t *o32 = reinterpret_cast<uint32_t *>(o);
#pragma unroll
        for (int i = 0; i < 5; i++)
            o32[i] = v[i];
    } else {
        __builtin_memcpy(o, v, 20);
    }
}

struct Sha1Alg {
    using State = Sha1State;
    static BRB_DEV State iv() { return sha1_iv(); }
    static BRB_DEV void compress(State &st, uint32_t (&w)[16])
    {
#pragma unroll
        for (int i = 0; i < 16; i++)
            w[i] = __builtin_bswap32(w[i]);
        sha1_compress(st, w);
    }
    static BRB_DEV void finish(State &st, uint32_t (&w)[16], uint32_t t, uint64_t len) { sha1_finish(st, w, t, len); }
    static BRB_DEV void pad_only(State &st, uint64_t len) { sha1_pad_only(st, len); }
    template <bool ALIGNED>
    static BRB_DEV void store(uint8_t *out, uint64_t r, const State &st) { store20<ALIGNED>(out, r, st); }
};

template <int BLOCK, bool OUT_ALIGNED>
__global__ __launch_bounds__(BLOCK) void sha1_fixed_a4_kernel(const uint8_t *__restrict__ data, uint32_t rec_len,
                                                               uint64_t n_rec, uint8_t *__restrict__ out)
{
    const uint64_t r = uint64_t(blockIdx.x) * BLOCK + threadIdx.x;
    if (r >= n_rec)
        return;
    const uint8_t *p = data + r * rec_len;
    const uint32_t nfull = rec_len >> 6;
    Sha1State st = sha1_iv();
    uint32_t w[16];

    if (nfull) {
        uint4 n0 = ld16_a4(p), n1 = ld16_a4(p + 16), n2 = ld16_a4(p + 32), n3 = ld16_a4(p + 48);
        for (uint32_t b = 0; b < nfull; ++b) {
            const uint4 c0 = n0, c1 = n1, c2 = n2, c3 = n3;
            const uint8_t *q = p + 64u * (b + 1 < nfull ? b + 1 : b);
            n0 = ld16_a4(q);
            n1 = ld16_a4(q + 16);
            n2 = ld16_a4(q + 32);
            n3 = ld16_a4(q + 48);
            w[0] = c0.x; w[1] = c0.y; w[2] = c0.z; w[3] = c0.w;
            w[4] = c1.x; w[5] = c1.y; w[6] = c1.z; w[7] = c1.w;
            w[8] = c2.x; w[9] = c2.y; w[10] = c2.z; w[11] = c2.w;
            w[12] = c3.x; w[13] = c3.y; w[14] = c3.z; w[15] = c3.w;
#pragma unroll
            for (int i = 0; i < 16; i++)
                w[i] = __builtin_bswap32(w[i]);
            sha1_compress(st, w);
        }
    }
    const uint32_t t = rec_len & 63;
    const uint8_t *pt = p + 64u * nfull;
#pragma unroll
    for (uint32_t i = 0; i < 16; i++)
        w[i] = tail_word_a4(pt, t, i);
    sha1_finish(st, w, t, rec_len);
    store20<OUT_ALIGNED>(out, r, st);
}

template <int BLOCK, bool FIXED, bool OUT_ALIGNED>
__global__ __launch_bounds__(BLOCK) void sha1_any_kernel(const uint8_t *__restrict__ data, const uint64_t *__restrict__ offs,
                                                          const uint32_t *__restrict__ lens, uint32_t rec_len,
                                                          uint64_t n_rec, uint8_t *__restrict__ out)
{
    const uint64_t r = uint64_t(blockIdx.x) * BLOCK + threadIdx.x;
    if (r >= n_rec)
        return;
    const uint8_t *a = data + (FIXED ? r * rec_len : offs[r]);
    const uint64_t len = FIXED ? rec_len : lens[r];
    const uint64_t nfull = len >> 6;
    Sha1State st = sha1_iv();
    uint32_t w[16];
    brb_io::BlockSrc src;           // the next 64-byte block is always in flight
    src.init(a, len);
    for (uint64_t b = 0; b < nfull; ++b) {
        src.fetch(w);
#pragma unroll
        for (uint32_t i = 0; i < 16; i++)
            w[i] = __builtin_bswap32(w[i]);
        sha1_compress(st, w);
    }
    src.fetch(w);                   // tail (bytes past the record read as 0)
    brb_io::add_marker(w, len);
    sha1_finish(st, w, uint32_t(len & 63), len);
    store20<OUT_ALIGNED>(out, r, st);
}

constexpr int kBlock = 256;

inline unsigned grid_for(uint64_t n)
{
    return unsigned((n + kBlock - 1) / kBlock);
}

}  // namespace

namespace brb {

hipError_t launch_sha1_fixed(const uint8_t *data, uint32_t rec_len, uint64_t n_rec, uint8_t *out, hipStream_t s)
{
    if (n_rec == 0)
        return hipSuccess;
    const bool out_al = (reinterpret_cast<uintptr_t>(out) & 3) == 0;
    const bool in_a4 = (reinterpret_cast<uintptr_t>(data) & 3) == 0 && (rec_len & 3) == 0;
    const unsigned g = grid_for(n_rec);
    if (brb_digest::dma_supported(rec_len))
        return brb_digest::launch_fixed_dma<Sha1Alg>(data, rec_len, n_rec, out, out_al, s);
    if (in_a4) {
        if (out_al)
            sha1_fixed_a4_kernel<kBlock, true><<<g, kBlock, 0, s>>>(data, rec_len, n_rec, out);
        else
            sha1_fixed_a4_kernel<kBlock, false><<<g, kBlock, 0, s>>>(data, rec_len, n_rec, out);
    } else {
        if (out_al)
            sha1_any_kernel<kBlock, true, true><<<g, kBlock, 0, s>>>(data, nullptr, nullptr, rec_len, n_rec, out);
        else
            sha1_any_kernel<kBlock, true, false><<<g, kBlock, 0, s>>>(data, nullptr, nullptr, rec_len, n_rec, out);
    }
    return hipGetLastError();
}

hipError_t launch_sha1_var(const uint8_t *data, const uint64_t *offs, const uint32_t *lens, uint64_t n_rec,
                           uint8_t *out, hipStream_t s)
{
    if (n_rec == 0)
        return hipSuccess;
    const bool out_al = (reinterpret_cast<uintptr_t>(out) & 3) == 0;
    // line-aligned LDS-DMA staging (digest_var_line.h); the per-lane kernel below is its A/B baseline
    if (brb_digest::var_line_enabled())
        return brb_digest::launch_var_line<Sha1Alg>(data, offs, lens, n_rec, out, out_al, s);
    const unsigned g = grid_for(n_rec);
    if (out_al)
        sha1_any_kernel<kBlock, false, true><<<g, kBlock, 0, s>>>(data, offs, lens, 0, n_rec, out);
    else
        sha1_any_kernel<kBlock, false, false><<<g, kBlock, 0, s>>>(data, offs, lens, 0, n_rec, out);
    return hipGetLastError();
}

}  // namespace brb
