// base64_kernels.hip -- batched base64 codec, one record per lane.
//
//   encode = brb_base64_encode_to_mb (libbrb_core/crypto/base64.c:304-361): every 3 input bytes
//            -> 4 characters of the standard alphabet, a 1- or 2-byte tail padded with '='.  Each
//            3-byte quantum is exactly one 4-character output dword, built with v_perm_b32 from the
//            input dwords and a 64-byte alphabet table in LDS (16 dwords in 16 banks: no conflicts).
//   decode = brb_base64_decode_to_mb (:131-179): the record is a C string (a NUL ends it), bytes
//            outside the alphabet are skipped, '=' counts as 0 (:363-376), every 4 counted
//            characters give 3 bytes, a trailing partial group is dropped.
#include "brb_kernels.h"
#include "byte_stream.h"

namespace {

constexpr int kBlock = 256;

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

BRB_DEV uint32_t chars4(const uint8_t *alpha, uint32_t v)
{
    return uint32_t(alpha[v >> 18]) | (uint32_t(alpha[(v >> 12) & 63]) << 8) | (uint32_t(alpha[(v >> 6) & 63]) << 16) |
           (uint32_t(alpha[v & 63]) << 24);
}

__global__ __launch_bounds__(kBlock) void b64_encode_kernel(const uint8_t *__restrict__ in,
                                                            const uint64_t *__restrict__ offs,
                                                            const uint32_t *__restrict__ lens, uint64_t n,
                                                            uint8_t *__restrict__ out,
                                                            const uint64_t *__restrict__ ooffs)
{
    __shared__ uint8_t alpha[64];
    if (threadIdx.x < 64) {
        const uint32_t i = threadIdx.x;   // base64.c:42
        alpha[i] = uint8_t(i < 26 ? 'A' + i : i < 52 ? 'a' + (i - 26) : i < 62 ? '0' + (i - 52) : i == 62 ? '+' : '/');
    }
    __syncthreads();
    const uint64_t r = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (r >= n)
        return;
    const uint64_t len = lens[r];
    const uint64_t olen = 4 * ((len + 2) / 3);
    brb_io::Src src;
    brb_io::Snk snk;
    src.init(in + offs[r], len);
    snk.init(out + ooffs[r], olen);
    const uint64_t groups = len / 12;
    for (uint64_t g = 0; g < groups; g++) {
        const uint32_t d0 = src.next(), d1 = src.next(), d2 = src.next();
#pragma unroll
        for (int q = 0; q < 4; q++)
            snk.put(chars4(alpha, quantum(d0, d1, d2, q)));
    }
    const uint32_t t = uint32_t(len - 12 * groups);          // 0..11 tail bytes
    if (t) {
        const uint32_t d0 = src.next(), d1 = t > 4 ? src.next() : 0u, d2 = t > 8 ? src.next() : 0u;
        const uint32_t full = t / 3, rest = t % 3;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (uint32_t(q) < full) {
                snk.put(chars4(alpha, quantum(d0, d1, d2, q)));
            } else if (uint32_t(q) == full && rest) {
                // bytes past the record read as 0 (Src masks them): the tail rule of base64.c:335-352
                uint32_t c = chars4(alpha, quantum(d0, d1, d2, q));
                c = rest == 1 ? (c & 0x0000FFFFu) | 0x3D3D0000u : (c & 0x00FFFFFFu) | 0x3D000000u;
                snk.put(c);
            }
        }
    }
    snk.flush();
}

// base64.c:363-376: alphabet value, 0 for '=', -1 for anything else
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

__global__ __launch_bounds__(kBlock) void b64_decode_kernel(const uint8_t *__restrict__ in,
                                                            const uint64_t *__restrict__ offs,
                                                            const uint32_t *__restrict__ lens, uint64_t n,
                                                            uint8_t *__restrict__ out,
                                                            const uint64_t *__restrict__ ooffs,
                                                            uint32_t *__restrict__ olens)
{
    const uint64_t r = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (r >= n)
        return;
    const uint64_t len = lens[r];
    brb_io::Src src;
    brb_io::Snk snk;
    src.init(in + offs[r], len);
    snk.init(out + ooffs[r], 3 * (len / 4));
    uint32_t val = 0, cnt = 0, produced = 0, outn = 0;
    uint64_t outacc = 0;
    bool live = true;
    for (uint64_t c4 = 0; c4 < len && live; c4 += 4) {
        const uint32_t chunk = src.next();
        const uint32_t nb = len - c4 >= 4 ? 4u : uint32_t(len - c4);
        for (uint32_t b = 0; b < nb; b++) {
            const uint32_t ch = (chunk >> (8 * b)) & 0xFFu;
            if (ch == 0) {              // C-string end (base64.c:146)
                live = false;
                break;
            }
            const int v = b64_value(ch);
            if (v < 0)
                continue;
            val = (val << 6) | uint32_t(v);
            if (++cnt < 4)
                continue;
            const uint32_t t = ((val >> 16) & 0xFFu) | (val & 0xFF00u) | ((val & 0xFFu) << 16);
            outacc |= uint64_t(t) << (8 * outn);
            outn += 3;
            produced += 3;
            val = cnt = 0;
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
