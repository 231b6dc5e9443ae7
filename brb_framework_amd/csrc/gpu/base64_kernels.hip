// base64_kernels.hip -- batched base64 codec, one record per lane.
//
//   encode = brb_base64_encode_to_mb (libbrb_core/crypto/base64.c:304-361): every 3 input bytes
//            -> 4 characters of the standard alphabet, a 1- or 2-byte tail padded with '='.
//   decode = brb_base64_decode_to_mb (:131-179): the record is a C string (a NUL ends it), bytes
//            outside the alphabet are skipped, '=' counts as 0 (:363-376), every 4 counted
//            characters give 3 bytes, a trailing partial group is dropped.
//
// A lane streams its record like the RC4 pass (rc4_kernels.hip): 64-byte input blocks with the
// next one in flight (brb_io::BlockSrc) and 16-byte output stores (brb_io::Snk::put16).  Encode
// works in steps of 192 input bytes (48 dwords = 16 quanta triples -> 64 output dwords), each 24-bit
// quantum one v_perm_b32 and two lookups in a 12-bit -> 2-character LDS table.  Decode takes steps
// of 256 characters while every character is in the alphabet or '=' (then the groups sit at fixed
// positions: 64 groups -> 192 bytes); at the first step holding a skipped byte or a NUL it falls
// back to the reference's character-serial rules for the rest of the record.  The per-lane dword
// reader of the first version (one dword in flight) left both at ~1.2 ms per round trip of
// 65 536 x 1500 bytes.
#include "brb_kernels.h"
#include "byte_stream.h"

namespace {

constexpr int kBlock = 256;

BRB_DEV uint32_t alpha(uint32_t i)   // base64.c:42
{
    return i < 26 ? 'A' + i : i < 52 ? 'a' + (i - 26) : i < 62 ? '0' + (i - 52) : i == 62 ? '+' : '/';
}

// big-endian 24-bit quantum q (0..3) of the 12 bytes d0|d1|d2 (v_perm selectors: 0-3 = src1 bytes,
// 4-7 = src0 bytes, 0x0C = 0)
BRB_DEV uint32_t quantum(uint32_t d0, uint32_t d1, uint32_t d2, int q)
{
    switch (q) {
    case 0: return __builtin_amdgcn_perm(d0, d0, 0x0C000102u);
    case 1: return __builtin_amdgcn_perm(d1, d0, 0x0C030405u);
    case 2: return __builtin_amdgcn_perm(d2, d1, 0x0C020304u);
    default: return __builtin_amdgcn_perm(d2, d2, 0x0C010203u);
    }
}

// the 4 characters of quantum v: two lookups of 12 bits each
BRB_DEV uint32_t chars4(const uint16_t *pair, uint32_t v)
{
    return uint32_t(pair[v >> 12]) | (uint32_t(pair[v & 4095u]) << 16);
}

template <int I>
BRB_DEV uint32_t pick(const uint32_t (&a)[16], const uint32_t (&b)[16], const uint32_t (&c)[16])
{
    return I < 16 ? a[I & 15] : I < 32 ? b[I & 15] : c[I & 15];
}

// the 16 output dwords of triples 4h .. 4h + 3 of a 48-dword step
template <int H>
BRB_DEV void encode16(const uint16_t *pair, const uint32_t (&a)[16], const uint32_t (&b)[16], const uint32_t (&c)[16],
                      uint32_t (&o)[16])
{
#pragma unroll
    for (int g = 0; g < 4; g++) {
        const int t = 4 * H + g;
        uint32_t d0, d1, d2;
        switch (t) {   // compile-time register indices
#define BRB_T(T) case T: d0 = pick<3 * T>(a, b, c); d1 = pick<3 * T + 1>(a, b, c); d2 = pick<3 * T + 2>(a, b, c); break;
            BRB_T(0) BRB_T(1) BRB_T(2) BRB_T(3) BRB_T(4) BRB_T(5) BRB_T(6) BRB_T(7)
            BRB_T(8) BRB_T(9) BRB_T(10) BRB_T(11) BRB_T(12) BRB_T(13) BRB_T(14) default: BRB_T(15)
#undef BRB_T
        }
#pragma unroll
        for (int q = 0; q < 4; q++)
            o[4 * g + q] = chars4(pair, quantum(d0, d1, d2, q));
    }
}

__global__ __launch_bounds__(kBlock) void b64_encode_kernel(const uint8_t *__restrict__ in,
                                                            const uint64_t *__restrict__ offs,
                                                            const uint32_t *__restrict__ lens, uint64_t n,
                                                            uint8_t *__restrict__ out,
                                                            const uint64_t *__restrict__ ooffs)
{
    __shared__ uint16_t pair[4096];
    for (uint32_t e = threadIdx.x; e < 4096; e += kBlock)
        pair[e] = uint16_t(alpha(e >> 6) | (alpha(e & 63) << 8));
    __syncthreads();
    const uint64_t r = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (r >= n)
        return;
    const uint64_t len = lens[r];
    const uint64_t olen = 4 * ((len + 2) / 3);
    brb_io::BlockSrc src;
    brb_io::Snk snk;
    src.init(in + offs[r], len);
    snk.init(out + ooffs[r], olen);
    uint32_t a[16], b[16], c[16], o[16];
    const uint64_t steps = len / 192;
    for (uint64_t st = 0; st < steps; st++) {
        src.fetch(a);
        src.fetch(b);
        src.fetch(c);
        encode16<0>(pair, a, b, c, o);
        snk.put16(o);
        encode16<1>(pair, a, b, c, o);
        snk.put16(o);
        encode16<2>(pair, a, b, c, o);
        snk.put16(o);
        encode16<3>(pair, a, b, c, o);
        snk.put16(o);
    }
    const uint32_t t = uint32_t(len - 192 * steps);           // 0..191 tail bytes (zeros past them)
    if (t) {
        src.fetch(a);
        if (t > 64)
            src.fetch(b);
        else
#pragma unroll
            for (int i = 0; i < 16; i++)
                b[i] = 0;
        if (t > 128)
            src.fetch(c);
        else
#pragma unroll
            for (int i = 0; i < 16; i++)
                c[i] = 0;
        const uint32_t full = t / 3, rest = t % 3;            // quantum `full` holds the 1- or 2-byte tail
        // the padding rule of base64.c:335-352 (bytes past the record read as 0 above)
        auto pad = [&](uint32_t v, uint32_t u) {
            return u == full && rest ? (rest == 1 ? (v & 0x0000FFFFu) | 0x3D3D0000u : (v & 0x00FFFFFFu) | 0x3D000000u) : v;
        };
        encode16<0>(pair, a, b, c, o);
#pragma unroll
        for (int k = 0; k < 16; k++)
            o[k] = pad(o[k], k);
        snk.put16(o);                                         // Snk writes no byte past olen
        if (t > 48) {
            encode16<1>(pair, a, b, c, o);
#pragma unroll
            for (int k = 0; k < 16; k++)
                o[k] = pad(o[k], 16 + k);
            snk.put16(o);
        }
        if (t > 96) {
            encode16<2>(pair, a, b, c, o);
#pragma unroll
            for (int k = 0; k < 16; k++)
                o[k] = pad(o[k], 32 + k);
            snk.put16(o);
        }
        if (t > 144) {
            encode16<3>(pair, a, b, c, o);
#pragma unroll
            for (int k = 0; k < 16; k++)
                o[k] = pad(o[k], 48 + k);
            snk.put16(o);
        }
    }
    snk.flush();
}

// base64.c:363-376: alphabet value, 0 for '=', -1 for anything else (NUL included)
BRB_DEV int b64_value(uint32_t c)
{
    if (c - 'A' < 26u)
        return int(c - 'A');
    if (c - 'a' < 26u)
        return int(c - 'a' + 26);
    if (c - '0' < 10u)
        return int(c - '0' + 52);
    if (c == '+')
        return 62;
    if (c == '/')
        return 63;
    return c == '=' ? 0 : -1;
}

// 4 characters (one dword) -> their 3 bytes in output order (b0 | b1 << 8 | b2 << 16), bit 31 set
// if any character is outside the alphabet / '=' (256-byte table: one dword per LDS bank)
BRB_DEV uint32_t group3(const int8_t *val, uint32_t ch)
{
    const int v0 = val[ch & 255u], v1 = val[(ch >> 8) & 255u], v2 = val[(ch >> 16) & 255u], v3 = val[ch >> 24];
    const uint32_t w = (uint32_t(v0) << 18) | (uint32_t(v1) << 12) | (uint32_t(v2) << 6) | uint32_t(v3 & 63);
    const uint32_t s = __builtin_amdgcn_perm(w, w, 0x0C000102u);   // bytes w2 w1 w0 -> output order
    return s | (uint32_t(v0 | v1 | v2 | v3) & 0x80000000u);
}

// 16 groups (one 64-character block) -> 12 output dwords at o[12 k ..]; returns the OR of the flags
BRB_DEV uint32_t decode_block(const int8_t *val, const uint32_t (&c)[16], uint32_t (&o)[48], int k)
{
    uint32_t bad = 0;
#pragma unroll
    for (int g = 0; g < 16; g += 4) {
        const uint32_t s0 = group3(val, c[g]), s1 = group3(val, c[g + 1]), s2 = group3(val, c[g + 2]),
                       s3 = group3(val, c[g + 3]);
        bad |= s0 | s1 | s2 | s3;
        const int q = 12 * k + 3 * (g / 4);
        o[q] = (s0 & 0xFFFFFFu) | (s1 << 24);
        o[q + 1] = ((s1 & 0xFFFFFFu) >> 8) | (s2 << 16);
        o[q + 2] = ((s2 & 0xFFFFFFu) >> 16) | (s3 << 8);
    }
    return bad;
}

__global__ __launch_bounds__(kBlock) void b64_decode_kernel(const uint8_t *__restrict__ in,
                                                            const uint64_t *__restrict__ offs,
                                                            const uint32_t *__restrict__ lens, uint64_t n,
                                                            uint8_t *__restrict__ out,
                                                            const uint64_t *__restrict__ ooffs,
                                                            uint32_t *__restrict__ olens)
{
    __shared__ int8_t val[256];
    for (uint32_t e = threadIdx.x; e < 256; e += kBlock)
        val[e] = int8_t(b64_value(e));
    __syncthreads();
    const uint64_t r = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (r >= n)
        return;
    const uint64_t len = lens[r];
    const uint8_t *a = in + offs[r];
    brb_io::Snk snk;
    snk.init(out + ooffs[r], 3 * (len / 4));
    uint64_t pos = 0;
    uint32_t produced = 0;
    if (len >= 256) {
        // steps of 256 characters while every one of them is in the alphabet or '=': 64 whole groups
        brb_io::BlockSrc src;
        src.init(a, len);
        uint32_t c0[16], c1[16], c2[16], c3[16], o[48];
        for (; pos + 256 <= len; pos += 256) {
            src.fetch(c0);
            src.fetch(c1);
            src.fetch(c2);
            src.fetch(c3);
            const uint32_t bad = decode_block(val, c0, o, 0) | decode_block(val, c1, o, 1) |
                                 decode_block(val, c2, o, 2) | decode_block(val, c3, o, 3);
            if (bad & 0x80000000u)
                break;                                        // skipped bytes or a NUL: serial from pos
            uint32_t h[16];
#pragma unroll
            for (int q = 0; q < 3; q++) {
#pragma unroll
                for (int i = 0; i < 16; i++)
                    h[i] = o[16 * q + i];
                snk.put16(h);
            }
            produced += 192;
        }
    }
    // base64.c:131-179, character by character, from pos (a group boundary: val = cnt = 0)
    brb_io::Src src;
    src.init(a + pos, len - pos);
    uint32_t val4 = 0, cnt = 0, outn = 0;
    uint64_t outacc = 0;
    bool live = true;
    for (uint64_t c4 = pos; c4 < len && live; c4 += 4) {
        const uint32_t chunk = src.next();
        const uint32_t nb = len - c4 >= 4 ? 4u : uint32_t(len - c4);
        for (uint32_t b = 0; b < nb; b++) {
            const uint32_t ch = (chunk >> (8 * b)) & 0xFFu;
            if (ch == 0) {              // C-string end (base64.c:146)
                live = false;
                break;
            }
            const int v = val[ch];
            if (v < 0)
                continue;
            val4 = (val4 << 6) | uint32_t(v);
            if (++cnt < 4)
                continue;
            const uint32_t t = ((val4 >> 16) & 0xFFu) | (val4 & 0xFF00u) | ((val4 & 0xFFu) << 16);
            outacc |= uint64_t(t) << (8 * outn);
            outn += 3;
            produced += 3;
            val4 = cnt = 0;
            if (outn >= 4) {
                snk.put(uint32_t(outacc));
                outacc >>= 32;
                outn -= 4;
            }
        }
    }
    if (outn) {
        snk.rem = outn;
        snk.put(uint32_t(outacc));
    }
    snk.flush();
    olens[r] = produced;
}

inline unsigned grid_for(uint64_t n) { return unsigned((n + kBlock - 1) / kBlock); }

}  // namespace

namespace brb {

hipError_t launch_b64_encode(const uint8_t *in, const uint64_t *offs, const uint32_t *lens, uint64_t n, uint8_t *out,
                             const uint64_t *ooffs, hipStream_t s)
{
    if (n == 0)
        return hipSuccess;
    b64_encode_kernel<<<grid_for(n), kBlock, 0, s>>>(in, offs, lens, n, out, ooffs);
    return hipGetLastError();
}

hipError_t launch_b64_decode(const uint8_t *in, const uint64_t *offs, const uint32_t *lens, uint64_t n, uint8_t *out,
                             const uint64_t *ooffs, uint32_t *olens, hipStream_t s)
{
    if (n == 0)
        return hipSuccess;
    b64_decode_kernel<<<grid_for(n), kBlock, 0, s>>>(in, offs, lens, n, out, ooffs, olens);
    return hipGetLastError();
}

}  // namespace brb
