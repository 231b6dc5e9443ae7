// rc4_kernels.hip -- batched RC4 and RC4+MD5 framing for gfx950.
//
// One lane per connection stream, one wave per workgroup, the wave's 64 permutations in a 16 KiB
// LDS slot (rc4_device.h).  Lanes touch only their own LDS bytes, so no barrier is needed.
//
//   rc4_crypt_kernel   BRB_RC4_Crypt on every stream                          (rc4.c:64-87)
//   rc4md5_frame_kernel  WRITE side of EvAIOReqTransform_CryptoRaw(RC4_MD5):  one pass over the
//                      payload feeds MD5 and the RC4 stream; the 30-byte header, which holds the
//                      digest, is encrypted with keystream bytes 0..29 saved up front and written
//                      last                                (ev_kq_aio_transform.c:212-230, 281-283)
//   rc4md5_open_kernel READ side + EvAIOReqTransform_RC4_MD5_DataValidate: one pass decrypts the
//                      frame and feeds the decrypted payload to MD5       (:270-279, :158-184)
#include "brb_kernels.h"
#include "rc4_device.h"

namespace {

using namespace brb_rc4;

constexpr int kWave = 64;

BRB_DEV uint32_t clamp4(uint64_t left) { return left >= 4 ? 4u : uint32_t(left); }

__global__ __launch_bounds__(kWave) void rc4_crypt_kernel(uint8_t *__restrict__ states, const uint8_t *in, uint8_t *out,
                                                          const uint64_t *__restrict__ offs,
                                                          const uint32_t *__restrict__ lens, uint64_t n)
{
    __shared__ __attribute__((aligned(16))) uint8_t slot[kWaveLds];
    const uint32_t lane = threadIdx.x;
    const uint64_t s = uint64_t(blockIdx.x) * kWave + lane;
    if (s >= n)
        return;
    Gen g;
    g.P.lds = slot;
    g.P.lb = lane * 4;
    g.load(states + s * kStateBytes);
    const uint64_t off = offs[s], len = lens[s];
    Src src;
    Snk snk;
    src.init(in + off, len);
    snk.init(out + off, len);
    const uint64_t full = len >> 2;
    for (uint64_t c = 0; c < full; c++) {
        const uint32_t v = src.next();
        snk.put(v ^ g.next4());
    }
    if (len & 3) {
        const uint32_t v = src.next();
        snk.put(v ^ g.next_n(uint32_t(len & 3)));
    }
    snk.flush();
    g.store(states + s * kStateBytes);
}

__global__ __launch_bounds__(kWave) void rc4md5_frame_kernel(uint8_t *__restrict__ states, const uint8_t *__restrict__ payload,
                                                             const uint64_t *__restrict__ offs,
                                                             const uint32_t *__restrict__ lens,
                                                             const uint64_t *__restrict__ salts, uint8_t *frames,
                                                             const uint64_t *__restrict__ foffs, uint64_t n)
{
    __shared__ __attribute__((aligned(16))) uint8_t slot[kWaveLds];
    const uint32_t lane = threadIdx.x;
    const uint64_t s = uint64_t(blockIdx.x) * kWave + lane;
    if (s >= n)
        return;
    Gen g;
    g.P.lds = slot;
    g.P.lb = lane * 4;
    g.load(states + s * kStateBytes);
    const uint64_t len = lens[s];
    const uint64_t F = kHeader + len;            // frame bytes
    uint8_t *frame = frames + foffs[s];

    // keystream of frame chunks 0..7 (bytes 0..31; chunk 7 = digest[15], NUL, payload[0..1])
    uint32_t kh[8];
#pragma unroll
    for (int k = 0; k < 7; k++)
        kh[k] = g.next4();
    kh[7] = g.next_n(clamp4(F - 28));

    Src src;
    src.init(payload + offs[s], len);
    Snk snk;                                      // frame bytes 32..F-1
    snk.init(frame + 32, F > 32 ? F - 32 : 0);
    Md5State st = md5_iv();
    const uint64_t nblk = md5_blocks(len), nw = 16 * nblk;
    uint32_t prev = 0, first = 0;
    for (uint64_t b = 0; b < nblk; b++) {
        uint32_t m[16];
#pragma unroll
        for (uint32_t i = 0; i < 16; i++) {
            const uint64_t w = 16 * b + i;
            const uint32_t raw = src.next();
            if (w == 0) {
                first = raw;
            } else {
                // frame chunk w + 7 = payload bytes 4w - 2 .. 4w + 1
                const uint64_t fb = 4 * (w + 7);
                if (fb < F)
                    snk.put(__builtin_amdgcn_alignbit(raw, prev, 16) ^ g.next_n(clamp4(F - fb)));
            }
            prev = raw;
            m[i] = md5_pad_word(raw, w, len, nw);
        }
        md5_compress(st, m);
    }
    snk.flush();

    // header: salt (LE unsigned long), "HASH:", digest, NUL, then payload[0..1] in chunk 7
    const uint64_t salt = salts[s];
    uint32_t h[8];
    h[0] = uint32_t(salt);
    h[1] = uint32_t(salt >> 32);
    h[2] = 0x48534148u;                           // "HASH"
    h[3] = 0x3Au | (st.a << 8);                   // ':' + digest[0..2]
    h[4] = __builtin_amdgcn_alignbit(st.b, st.a, 24);
    h[5] = __builtin_amdgcn_alignbit(st.c, st.b, 24);
    h[6] = __builtin_amdgcn_alignbit(st.d, st.c, 24);
    h[7] = (st.d >> 24) | (first << 16);          // digest[15], NUL, payload[0], payload[1]
    Snk hs;
    hs.init(frame, F < 32 ? F : 32);
#pragma unroll
    for (int k = 0; k < 8; k++)
        hs.put(h[k] ^ kh[k]);
    hs.flush();
    g.store(states + s * kStateBytes);
}

__global__ __launch_bounds__(kWave) void rc4md5_open_kernel(uint8_t *__restrict__ states, const uint8_t *in, uint8_t *out,
                                                            const uint64_t *__restrict__ offs,
                                                            const uint32_t *__restrict__ lens, uint64_t n,
                                                            uint8_t *__restrict__ valid)
{
    __shared__ __attribute__((aligned(16))) uint8_t slot[kWaveLds];
    const uint32_t lane = threadIdx.x;
    const uint64_t s = uint64_t(blockIdx.x) * kWave + lane;
    if (s >= n)
        return;
    Gen g;
    g.P.lds = slot;
    g.P.lb = lane * 4;
    g.load(states + s * kStateBytes);
    const uint64_t off = offs[s], F = lens[s];
    Src src;
    Snk snk;
    src.init(in + off, F);
    snk.init(out + off, F);

    // header chunks 0..7 (frame bytes 0..31)
    uint32_t hd[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint64_t fb = 4 * uint64_t(k);
        const uint32_t nb = fb < F ? clamp4(F - fb) : 0u;
        const uint32_t raw = src.next();
        hd[k] = raw ^ (nb ? g.next_n(nb) : 0u);
        snk.put(hd[k]);
    }

    uint32_t ok = 0;
    if (F >= kHeader) {
        // payload word w = frame bytes 30 + 4w .. 33 + 4w = chunks w + 7 (high half) and w + 8 (low half)
        const uint64_t len = F - kHeader;
        const uint64_t nblk = md5_blocks(len), nw = 16 * nblk;
        Md5State st = md5_iv();
        uint32_t prev = hd[7];
        for (uint64_t b = 0; b < nblk; b++) {
            uint32_t m[16];
#pragma unroll
            for (uint32_t i = 0; i < 16; i++) {
                const uint64_t w = 16 * b + i;
                const uint64_t fb = 4 * (w + 8);
                uint32_t pt = 0;
                if (fb < F) {
                    pt = src.next() ^ g.next_n(clamp4(F - fb));
                    snk.put(pt);
                }
                m[i] = md5_pad_word(__builtin_amdgcn_alignbit(pt, prev, 16), w, len, nw);
                prev = pt;
            }
            md5_compress(st, m);
        }
        const bool tag = hd[2] == 0x48534148u && (hd[3] & 0xFFu) == 0x3Au;   // "HASH:" at 8..12
        const bool dig = __builtin_amdgcn_alignbit(hd[4], hd[3], 8) == st.a &&
                         __builtin_amdgcn_alignbit(hd[5], hd[4], 8) == st.b &&
                         __builtin_amdgcn_alignbit(hd[6], hd[5], 8) == st.c &&
                         __builtin_amdgcn_alignbit(hd[7], hd[6], 8) == st.d;
        ok = tag && dig;
    }
    snk.flush();
    valid[s] = uint8_t(ok);
    g.store(states + s * kStateBytes);
}

inline unsigned grid_for(uint64_t n) { return unsigned((n + kWave - 1) / kWave); }

}  // namespace

namespace brb {

hipError_t launch_rc4_crypt(uint8_t *states, const uint8_t *in, uint8_t *out, const uint64_t *offs,
                            const uint32_t *lens, uint64_t n, hipStream_t s)
{
    if (n == 0)
        return hipSuccess;
    rc4_crypt_kernel<<<grid_for(n), kWave, 0, s>>>(states, in, out, offs, lens, n);
    return hipGetLastError();
}

hipError_t launch_rc4md5_frame(uint8_t *states, const uint8_t *payload, const uint64_t *offs, const uint32_t *lens,
                               const uint64_t *salts, uint8_t *frames, const uint64_t *foffs, uint64_t n,
                               hipStream_t s)
{
    if (n == 0)
        return hipSuccess;
    rc4md5_frame_kernel<<<grid_for(n), kWave, 0, s>>>(states, payload, offs, lens, salts, frames, foffs, n);
    return hipGetLastError();
}

hipError_t launch_rc4md5_open(uint8_t *states, const uint8_t *in, uint8_t *out, const uint64_t *offs,
                              const uint32_t *lens, uint64_t n, uint8_t *valid, hipStream_t s)
{
    if (n == 0)
        return hipSuccess;
    rc4md5_open_kernel<<<grid_for(n), kWave, 0, s>>>(states, in, out, offs, lens, n, valid);
    return hipGetLastError();
}

}  // namespace brb
