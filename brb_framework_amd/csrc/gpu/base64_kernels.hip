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
#include "test_options.h"

namespace {

constexpr int kBlock = 256;
constexpr uint32_t kWaves = kBlock / 64;
constexpr uint32_t kXch = 4096;                 // per-wave exchange of the cooperative loads / stores

// Wave-uniform maximum (loop bounds of the cooperative loads and stores).
BRB_DEV uint32_t wave_max(uint32_t x)
{
#pragma unroll
    for (int o = 32; o; o >>= 1) {
        const uint32_t y = uint32_t(__shfl_xor(int(x), o));
        x = y > x ? y : x;
    }
    return __builtin_amdgcn_readfirstlane(x);
}

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

// P pieces per record (lanes P r .. P r + P - 1): encoding has no chain -- every 3 input bytes give
// their 4 characters on their own -- so a record is cut into P pieces whose lengths are multiples
// of 3 (all but the last), each encoded by its own lane exactly as a record of its own (only the
// last piece can end in a partial quantum, and it gets the padding).  65 536 records then fill P
// waves per SIMD instead of one, whose loads and stores hide each other's latency; adjacent lanes
// also read adjacent bytes.
template <int P>
__global__ __launch_bounds__(kBlock) void b64_encode_kernel(const uint8_t *__restrict__ in,
                                                            const uint64_t *__restrict__ offs,
                                                            const uint32_t *__restrict__ lens, uint64_t n,
                                                            uint8_t *__restrict__ out,
                                                            const uint64_t *__restrict__ ooffs)
{
    __shared__ uint16_t pair[4096];
    __shared__ __attribute__((aligned(16))) uint8_t xin[kWaves * kXch], xout[kWaves * kXch];
    for (uint32_t e = threadIdx.x; e < 4096; e += kBlock)
        pair[e] = uint16_t(alpha(e >> 6) | (alpha(e & 63) << 8));
    __syncthreads();
    const uint64_t gid = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
    const uint64_t r = gid / P;
    const uint32_t j = uint32_t(gid % P);
    const bool live = r < n;                      // lanes past n only take part in the wave's loads/stores
    const uint64_t rlen = live ? lens[r] : 0;
    const uint64_t S = 3 * ((rlen + 3 * P - 1) / (3 * P));  // piece bytes, a multiple of 3
    const uint64_t lo = j * S < rlen ? j * S : rlen;
    const uint64_t len = (rlen - lo < S ? rlen - lo : S);   // this lane's piece
    const uint64_t olen = 4 * ((len + 2) / 3);
    const uint32_t wv = threadIdx.x >> 6;
    brb_io::StepSrcW<3> src;
    brb_io::SnkW snk;
    src.init(in + (live ? offs[r] + lo : 0), len, xin + wv * kXch);
    snk.init(out + (live ? ooffs[r] + 4 * (lo / 3) : 0), olen, xout + wv * kXch);
    // step st: input bytes [192 st, 192 st + 192) -> characters [256 st, 256 st + 256) = output
    // blocks 4 st .. 4 st + 3; the last step of a record holds its 0..191-byte tail
    const uint64_t full = len / 192;
    const uint32_t t = uint32_t(len - 192 * full);            // 0..191 tail bytes (zeros past them)
    const uint32_t qfull = t / 3, rest = t % 3;               // quantum qfull holds the 1- or 2-byte tail
    const uint32_t nloop = wave_max(uint32_t(full + (t ? 1 : 0)));
    uint32_t blk[3][16], o[4][16];
    if (nloop) {
        src.issue(0);
        src.take(blk);
    }
    for (uint32_t st = 0; st < nloop; st++) {
        if (st + 1 < nloop)
            src.issue(st + 1);                                // in flight while step st is encoded
        const bool in_full = st < full, in_tail = st == full && t;
        // the padding rule of base64.c:335-352 (bytes past the record read as 0 above)
        auto pad = [&](uint32_t v, uint32_t u) {
            return in_tail && u == qfull && rest ? (rest == 1 ? (v & 0x0000FFFFu) | 0x3D3D0000u : (v & 0x00FFFFFFu) | 0x3D000000u) : v;
        };
#define BRB_ENC(H)                                                                          \
        encode16<H>(pair, blk[0], blk[1], blk[2], o[H]);                                    \
        _Pragma("unroll") for (int k = 0; k < 16; k++) o[H][k] = pad(o[H][k], 16 * H + k);
        BRB_ENC(0) BRB_ENC(1) BRB_ENC(2) BRB_ENC(3)
#undef BRB_ENC
        if (st + 1 < nloop)
            src.take(blk);                                    // before this step's stores (StepSrcW)
#pragma unroll
        for (int h = 0; h < 4; h++)
            snk.put16(o[h], 4 * st + h, in_full || (in_tail && t > 48u * h));
    }
    if (live)
        snk.flush();                                          // Snk writes no byte past olen
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

// 16 groups (one 64-character block) -> 12 output dwords at o[12 k ..]; flag word q (bit 31 set: a
// character outside the alphabet / '=') covers groups 4q .. 4q + 3, one bit 31 per group in
// bits 31, 30, 29, 28 so that a partial step can ignore the groups past its end (group_mask)
BRB_DEV void decode_block4(const int8_t *val, const uint32_t (&c)[16], uint32_t (&o)[48], int k, uint32_t (&f)[4])
{
#pragma unroll
    for (int g = 0; g < 16; g += 4) {
        const uint32_t s0 = group3(val, c[g]), s1 = group3(val, c[g + 1]), s2 = group3(val, c[g + 2]),
                       s3 = group3(val, c[g + 3]);
        f[g / 4] = (s0 & 0x80000000u) | ((s1 >> 1) & 0x40000000u) | ((s2 >> 2) & 0x20000000u) | ((s3 >> 3) & 0x10000000u);
        const int q = 12 * k + 3 * (g / 4);
        o[q] = (s0 & 0xFFFFFFu) | (s1 << 24);
        o[q + 1] = ((s1 & 0xFFFFFFu) >> 8) | (s2 << 16);
        o[q + 2] = ((s2 & 0xFFFFFFu) >> 16) | (s3 << 8);
    }
}

// flags of the first m (>= 1) groups of a flag word, folded onto bit 31
BRB_DEV uint32_t group_mask(uint32_t m)
{
    return m >= 4 ? 0xF0000000u : (0xF0000000u << (4 - m)) & 0xF0000000u;
}

__global__ __launch_bounds__(kBlock) void b64_decode_kernel(const uint8_t *__restrict__ in,
                                                            const uint64_t *__restrict__ offs,
                                                            const uint32_t *__restrict__ lens, uint64_t n,
                                                            uint8_t *__restrict__ out,
                                                            const uint64_t *__restrict__ ooffs,
                                                            uint32_t *__restrict__ olens)
{
    __shared__ int8_t val[256];
    __shared__ __attribute__((aligned(16))) uint8_t xin[kWaves * kXch], xout[kWaves * kXch];
    for (uint32_t e = threadIdx.x; e < 256; e += kBlock)
        val[e] = int8_t(b64_value(e));
    __syncthreads();
    const uint64_t r = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
    const bool live = r < n;                      // lanes past n only take part in the wave's loads/stores
    const uint64_t len = live ? lens[r] : 0;
    const uint8_t *a = in + (live ? offs[r] : 0);
    const uint32_t wv = threadIdx.x >> 6;
    brb_io::SnkW snk;
    snk.init(out + (live ? ooffs[r] : 0), 3 * (len / 4), xout + wv * kXch);
    // Steps of 256 characters (4 input blocks -> 64 groups -> 3 output blocks) in one wave-uniform
    // loop.  A lane's last step may be partial: its whole groups decode the same way and a trailing
    // partial group is dropped (base64.c:171-175).  At the first step whose whole groups hold a byte
    // outside the alphabet / '=' (a skipped byte or a NUL), the lane leaves the loop's output and
    // finishes with the reference's character-serial rules from that step's start.
    uint64_t pos = 0;
    uint32_t produced = 0;
    bool fast = true;
    {
        brb_io::StepSrcW<4> src;
        src.init(a, len, xin + wv * kXch);
        const uint32_t nloop = wave_max(uint32_t((len + 255) / 256));
        uint32_t c[4][16], o[48];
        if (nloop) {
            src.issue(0);
            src.take(c);
        }
        for (uint32_t st = 0; st < nloop; st++) {
            if (st + 1 < nloop)
                src.issue(st + 1);
            const uint64_t p0 = 256ull * st;
            const uint32_t nch = fast && p0 < len ? uint32_t(len - p0 < 256 ? len - p0 : 256) : 0u;
            const uint32_t ng = nch / 4;                          // whole groups of this step
            uint32_t bad = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                uint32_t b4[4];
                decode_block4(val, c[k], o, k, b4);
#pragma unroll
                for (int q = 0; q < 4; q++)
                    bad |= 16u * k + 4u * q < ng ? b4[q] & group_mask(ng - 16u * k - 4u * q) : 0u;
            }
            const bool act = nch && !bad;
            if (nch && !act) {
                fast = false;                                     // serial from this step's start
                pos = p0;
            }
            if (act) {
                pos = p0 + nch;
                produced += 3 * ng;
            }
            if (st + 1 < nloop)
                src.take(c);
#pragma unroll
            for (int q = 0; q < 3; q++) {
                uint32_t h[16];
#pragma unroll
                for (int i = 0; i < 16; i++)
                    h[i] = o[16 * q + i];
                snk.put16(h, 3 * st + q, act && 3 * ng > 64u * q);
            }
        }
    }
    if (!live)
        return;
    // base64.c:131-179, character by character, from pos (a group boundary: val = cnt = 0); after
    // the fast loop only a lane that met a skipped byte or a NUL, or a trailing partial group, is left
    brb_io::Snk &ss = snk.s;
    brb_io::Src src;
    src.init(a + pos, len - pos);
    uint32_t val4 = 0, cnt = 0, outn = 0;
    uint64_t outacc = 0;
    bool on = !fast;
    for (uint64_t c4 = pos; c4 < len && on; c4 += 4) {
        const uint32_t chunk = src.next();
        const uint32_t nb = len - c4 >= 4 ? 4u : uint32_t(len - c4);
        for (uint32_t b = 0; b < nb; b++) {
            const uint32_t ch = (chunk >> (8 * b)) & 0xFFu;
            if (ch == 0) {              // C-string end (base64.c:146)
                on = false;
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
                ss.put(uint32_t(outacc));
                outacc >>= 32;
                outn -= 4;
            }
        }
    }
    if (outn) {
        ss.rem = outn;
        ss.put(uint32_t(outacc));
    }
    ss.flush();
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
    // one lane per record: two pieces per record (two waves per SIMD at 246 VGPRs) measured slower,
    // 153.8 -> 167.8 us per 65 536 x 1 500 B round trip (interleaved, gpurun_out/r03b64); test
    // option b64_pieces = 2 keeps them for A/B
    const bool two = brb_opt::get(brb_opt::kB64Pieces) == 2;
    if (two)
        b64_encode_kernel<2><<<unsigned((2 * n + kBlock - 1) / kBlock), kBlock, 0, s>>>(in, offs, lens, n, out, ooffs);
    else
        b64_encode_kernel<1><<<grid_for(n), kBlock, 0, s>>>(in, offs, lens, n, out, ooffs);
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
