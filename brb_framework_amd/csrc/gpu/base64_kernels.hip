// base64_kernels.hip -- batched base64 codec, a group of lanes per record.
//
//   encode = brb_base64_encode_to_mb (libbrb_core/crypto/base64.c:304-361): every 3 input bytes
//            -> 4 characters of the standard alphabet, a 1- or 2-byte tail padded with '='.
//   decode = brb_base64_decode_to_mb (:131-179): the record is a C string (a NUL ends it), bytes
//            outside the alphabet are skipped, '=' counts as 0 (:363-376), every 4 counted
//            characters give 3 bytes, a trailing partial group is dropped.
//
// History (65 536 x 1500 B round trip): one lane per record with a per-lane dword reader, ~1.2 ms;
// per-lane 64-byte blocks, 235 us (round 2); wave-cooperative 192/256-byte steps through a per-wave
// LDS exchange, 154 us (round 3, 1 wave per SIMD at 246-497 VGPRs); the group kernels below, 91 us.
#include "brb_kernels.h"
#include "byte_stream.h"
#include "test_options.h"

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

// ---- group kernels: G lanes per record, 12 / 16-byte pieces -------------------------------------
//
// Neither direction of the codec carries state along a record (every 3 bytes <-> 4 characters on
// their own, while the characters are clean), so a record is cut into pieces: encode 12 input bytes
// -> 16 characters, decode 16 characters -> 12 bytes.  G lanes (a power of two, 1..64) work on one
// record, lane j of the group on pieces j, j + G, ...; a piece is one 16/12-byte access at a lane
// stride of 12/16 bytes, so a group's loads and stores are contiguous runs of 12 G / 16 G bytes,
// and the kernels hold 46 (encode) / 64 (decode) VGPRs -- 8 waves per SIMD instead of the
// lane-per-record kernels' 1 to 2, which waited on memory 36 % of the time.  The grid is persistent
// (kPersist workgroups): group k walks records k, k + groups, ...

constexpr unsigned kPersist = 2048;              // 8 workgroups of 4 waves on each of 256 CUs

// bytes [a, a + m) (m <= 16) as 4 little-endian dwords, zeros past m.  Reads only dwords that hold
// a byte of the range (so never past the end of a buffer); one 16-byte load when aligned and whole.
BRB_DEV void load_piece(const uint8_t *a, uint32_t m, uint32_t (&d)[4])
{
    const uintptr_t ad = reinterpret_cast<uintptr_t>(a);
    const uint32_t s = uint32_t(ad & 3);
    if (s == 0 && m == 16) {
        const uint4 v = ld16_a4(a);
        d[0] = v.x;
        d[1] = v.y;
        d[2] = v.z;
        d[3] = v.w;
        return;
    }
    const uint8_t *a0 = a - s;
    uint32_t w[5];
#pragma unroll
    for (int k = 0; k < 5; k++)
        w[k] = m && 4u * k < s + m ? ld4_a4(a0 + 4 * k) : 0u;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t v = funnel(w[k + 1], w[k], 8 * s);
        const uint32_t lo = 4u * k;
        d[k] = m >= lo + 4 ? v : m > lo ? v & (0xFFFFFFFFu >> (32 - 8 * (m - lo))) : 0u;
    }
}

// 12 bytes [a, a + 12), 4-byte aligned: three dword loads the compiler merges into one dwordx3
BRB_DEV void load12_a4(const uint8_t *a, uint32_t (&d)[4])
{
    d[0] = ld4_a4(a);
    d[1] = ld4_a4(a + 4);
    d[2] = ld4_a4(a + 8);
    d[3] = 0;
}

// the q (<= 16) bytes of v -> [o, o + q), writing no byte outside it: aligned dwords that the range
// covers whole go out as dword (or one 16-byte) stores, the partial dwords at its ends byte by byte
BRB_DEV void store_piece(uint8_t *o, uint32_t q, const uint32_t (&v)[4])
{
    const uintptr_t ad = reinterpret_cast<uintptr_t>(o);
    const uint32_t s = uint32_t(ad & 3);
    if (s == 0 && q == 16) {
        st16_a4(o, v[0], v[1], v[2], v[3]);
        return;
    }
    if (s == 0 && q == 12) {
        stg(reinterpret_cast<uint32_t *>(o), v[0]);
        stg(reinterpret_cast<uint32_t *>(o + 4), v[1]);
        stg(reinterpret_cast<uint32_t *>(o + 8), v[2]);
        return;
    }
    uint8_t *a0 = o - s;
    // aligned dword k holds range bytes 4k - s .. 4k - s + 3: byte b = byte 4 + b - s of {v_k : v_k-1}
    const uint32_t sel = 0x07060504u - 0x01010101u * s;
#pragma unroll
    for (int k = 0; k < 5; k++) {
        const uint32_t first = 4u * k;                       // position of the dword in [a0, ...)
        if (first >= s + q)
            break;
        const uint32_t w = __builtin_amdgcn_perm(k < 4 ? v[k] : 0u, k > 0 ? v[k - 1] : 0u, sel);
        const uint32_t lo = first < s ? s - first : 0u;      // 0, or s in dword 0
        const uint32_t end = s + q - first;                  // bytes of this dword before the end
        const uint32_t hi = end >= 4 ? 3u : end - 1;
        if (lo == 0 && hi == 3) {
            stg(reinterpret_cast<uint32_t *>(a0 + first), w);
        } else {
#pragma unroll
            for (uint32_t b = 0; b < 4; b++)
                if (b >= lo && b <= hi)
                    stg8(a0 + first + b, w >> (8 * b));
        }
    }
}

// one encode piece: m (1..12) input bytes in d[0..2] (zeros past m) -> 4 * ceil(m / 3) characters
BRB_DEV uint32_t encode_piece(const uint16_t *pair, const uint32_t (&d)[4], uint32_t m, uint32_t (&c)[4])
{
#pragma unroll
    for (int q = 0; q < 4; q++)
        c[q] = chars4(pair, quantum(d[0], d[1], d[2], q));
    if (m < 12) {                                             // the record's last piece
        const uint32_t nq = (m + 2) / 3, rest = m % 3;        // base64.c:335-352 padding
        if (rest) {
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (uint32_t(q) == nq - 1)
                    c[q] = rest == 1 ? (c[q] & 0x0000FFFFu) | 0x3D3D0000u : (c[q] & 0x00FFFFFFu) | 0x3D000000u;
        }
        return 4 * nq;
    }
    return 16;
}

__global__ __launch_bounds__(kBlock) void b64_encode_group_kernel(const uint8_t *__restrict__ in,
                                                                  const uint64_t *__restrict__ offs,
                                                                  const uint32_t *__restrict__ lens, uint64_t n,
                                                                  uint8_t *__restrict__ out,
                                                                  const uint64_t *__restrict__ ooffs, uint32_t lg)
{
    __shared__ uint16_t pair[4096];
    for (uint32_t e = threadIdx.x; e < 4096; e += kBlock)
        pair[e] = uint16_t(alpha(e >> 6) | (alpha(e & 63) << 8));
    __syncthreads();
    const uint32_t G = 1u << lg, sub = threadIdx.x & (G - 1);
    const uint64_t groups = uint64_t(gridDim.x) * (kBlock >> lg);
    for (uint64_t r = (uint64_t(blockIdx.x) * kBlock + threadIdx.x) >> lg; r < n; r += groups) {
        const uint64_t len = lens[r];
        const uint8_t *a = in + offs[r];
        uint8_t *o = out + ooffs[r];
        const uint64_t np = (len + 11) / 12;
        const bool al = (reinterpret_cast<uintptr_t>(a) & 3) == 0;
        // two pieces per lane per pass (p, p + G): both loads in flight before either is encoded (four
        // measured slower: 88 VGPRs, 5 waves per SIMD)
        for (uint64_t p = sub; p < np; p += 2 * G) {
            uint32_t d[2][4], m[2];
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const uint64_t pu = p + u * G;
                m[u] = pu < np ? (len - 12 * pu >= 12 ? 12u : uint32_t(len - 12 * pu)) : 0u;
                if (al && m[u] == 12)
                    load12_a4(a + 12 * pu, d[u]);
                else
                    load_piece(a + 12 * pu, m[u], d[u]);      // m == 0: nothing is read
            }
#pragma unroll
            for (int u = 0; u < 2; u++) {
                if (m[u]) {
                    uint32_t c[4];
                    const uint32_t q = encode_piece(pair, d[u], m[u], c);
                    store_piece(o + 16 * (p + u * G), q, c);
                }
            }
        }
    }
}

// one decode piece: the 16 characters in d; returns the flags of its first `groups` groups (bit 31
// set: a character outside the alphabet / '=' among them) and the 12 bytes in b[0..2]
BRB_DEV uint32_t decode_piece(const int8_t *val, const uint32_t (&d)[4], uint32_t groups, uint32_t (&b)[4])
{
    const uint32_t s0 = group3(val, d[0]), s1 = group3(val, d[1]), s2 = group3(val, d[2]), s3 = group3(val, d[3]);
    b[0] = (s0 & 0xFFFFFFu) | (s1 << 24);
    b[1] = ((s1 & 0xFFFFFFu) >> 8) | (s2 << 16);
    b[2] = ((s2 & 0xFFFFFFu) >> 16) | (s3 << 8);
    b[3] = 0;
    const uint32_t f = (s0 & (groups > 0 ? 0x80000000u : 0u)) | (s1 & (groups > 1 ? 0x80000000u : 0u)) |
                       (s2 & (groups > 2 ? 0x80000000u : 0u)) | (s3 & (groups > 3 ? 0x80000000u : 0u));
    return f;
}

// base64.c:131-179 character by character from character `pos` of a record (a group boundary,
// val = cnt = 0 there) with `produced` bytes already written; returns the record's output length
BRB_DEV uint32_t decode_serial(const int8_t *val, const uint8_t *a, uint64_t len, uint64_t pos, uint8_t *o,
                               uint32_t produced)
{
    brb_io::Snk ss;
    ss.init(o + produced, 3 * (len / 4) - produced);
    brb_io::Src src;
    src.init(a + pos, len - pos);
    uint32_t val4 = 0, cnt = 0, outn = 0;
    uint64_t outacc = 0;
    bool on = true;
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
    return produced;
}

// Pieces before a record's first piece with a character outside the alphabet / '=' in its whole
// groups decode at fixed positions; from that piece's start the group's first lane finishes the
// record with the reference's serial rules (a skipped byte shifts every later group; a NUL ends
// the string).  The group finds that piece with one ballot per half pass, so no lane stores a
// piece at or after it.  Characters of a trailing partial group never produce output.
__global__ __launch_bounds__(kBlock) void b64_decode_group_kernel(const uint8_t *__restrict__ in,
                                                                  const uint64_t *__restrict__ offs,
                                                                  const uint32_t *__restrict__ lens, uint64_t n,
                                                                  uint8_t *__restrict__ out,
                                                                  const uint64_t *__restrict__ ooffs,
                                                                  uint32_t *__restrict__ olens, uint32_t lg)
{
    __shared__ int8_t val[256];
    for (uint32_t e = threadIdx.x; e < 256; e += kBlock)
        val[e] = int8_t(b64_value(e));
    __syncthreads();
    const uint32_t G = 1u << lg, lane = threadIdx.x & 63, sub = lane & (G - 1), gbase = lane - sub;
    const uint64_t gmask = G == 64 ? ~0ull : ((1ull << G) - 1) << gbase;
    const uint64_t groups = uint64_t(gridDim.x) * (kBlock >> lg);
    for (uint64_t r = (uint64_t(blockIdx.x) * kBlock + threadIdx.x) >> lg; r < n; r += groups) {
        const uint64_t len = lens[r];
        const uint8_t *a = in + offs[r];
        uint8_t *o = out + ooffs[r];
        const uint64_t ng = len / 4;                          // whole groups
        const uint64_t np = (ng + 3) / 4;                     // pieces holding a whole group
        uint64_t dirty = ~0ull;                               // first piece with a skipped byte / NUL
        for (uint64_t p = sub; p < np; p += 2 * G) {         // pieces p and p + G: both loads in flight
            const uint64_t p1 = p + G;
            const uint32_t g0 = ng - 4 * p >= 4 ? 4u : uint32_t(ng - 4 * p);
            const uint32_t g1 = p1 < np ? (ng - 4 * p1 >= 4 ? 4u : uint32_t(ng - 4 * p1)) : 0u;
            uint32_t d0[4], d1[4], b0[4], b1[4];
            load_piece(a + 16 * p, 4 * g0, d0);
            load_piece(a + 16 * p1, 4 * g1, d1);              // g1 == 0: nothing is read
            const uint32_t f0 = decode_piece(val, d0, g0, b0), f1 = decode_piece(val, d1, g1, b1);
            const uint64_t m0 = (__builtin_amdgcn_ballot_w64(f0 != 0) & gmask) >> gbase;
            const uint64_t m1 = (__builtin_amdgcn_ballot_w64(f1 != 0) & gmask) >> gbase;
            const uint64_t base = p - sub;
            if (m0 | m1)
                dirty = m0 ? base + __builtin_ctzll(m0) : base + G + __builtin_ctzll(m1);
            if (p < dirty)
                store_piece(o + 12 * p, 3 * g0, b0);
            if (g1 && p1 < dirty)
                store_piece(o + 12 * p1, 3 * g1, b1);
            if (dirty != ~0ull)
                break;                                        // group-uniform
        }
        if (sub == 0)
            olens[r] = dirty == ~0ull ? uint32_t(3 * ng) : decode_serial(val, a, len, 16 * dirty, o, uint32_t(12 * dirty));
    }
}

// log2 of the lanes per record: an average record takes two passes of two pieces per lane, at most
// 32 lanes (measured on 65 536 x 1500 B: 16 / 32 / 64 lanes 96.0 / 90.7 / 92.2 us per round trip);
// mean_len 0 = unknown (device mode): 32 lanes.  The test option forces it.
uint32_t group_lg(uint64_t mean_len, uint32_t piece)
{
    const int forced = brb_opt::get(brb_opt::kB64Group);
    if (forced >= 0 && forced <= 6)
        return uint32_t(forced);
    if (mean_len == 0)
        return 5;
    const uint64_t quarter = (mean_len + 4 * piece - 1) / (4 * piece);
    uint32_t lg = 0;
    while (lg < 5 && (1ull << lg) < quarter)
        lg++;
    return lg;
}

unsigned group_grid(uint64_t n, uint32_t lg)
{
    const uint64_t blocks = ((n << lg) + kBlock - 1) / kBlock;
    return unsigned(blocks < kPersist ? blocks : kPersist);
}

}  // namespace

namespace brb {

hipError_t launch_b64_encode(const uint8_t *in, const uint64_t *offs, const uint32_t *lens, uint64_t n, uint8_t *out,
                             const uint64_t *ooffs, uint64_t mean_len, hipStream_t s)
{
    if (n == 0)
        return hipSuccess;
    const uint32_t lg = group_lg(mean_len, 12);
    b64_encode_group_kernel<<<group_grid(n, lg), kBlock, 0, s>>>(in, offs, lens, n, out, ooffs, lg);
    return hipGetLastError();
}

hipError_t launch_b64_decode(const uint8_t *in, const uint64_t *offs, const uint32_t *lens, uint64_t n, uint8_t *out,
                             const uint64_t *ooffs, uint32_t *olens, uint64_t mean_len, hipStream_t s)
{
    if (n == 0)
        return hipSuccess;
    const uint32_t lg = group_lg(mean_len, 16);
    b64_decode_group_kernel<<<group_grid(n, lg), kBlock, 0, s>>>(in, offs, lens, n, out, ooffs, olens, lg);
    return hipGetLastError();
}

}  // namespace brb
