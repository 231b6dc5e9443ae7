// rc4_kernels.hip -- batched RC4 and RC4+MD5 framing for gfx950.
//
// One lane per connection stream, 4 waves per workgroup, the workgroup's 256 permutations in a
// 64 KiB LDS image (rc4_device.h).  Lanes touch only their own LDS bytes, so no barrier is needed.
//
//   rc4_crypt_kernel   BRB_RC4_Crypt on every stream                          (rc4.c:64-87)
//   rc4md5_frame_kernel  WRITE side of EvAIOReqTransform_CryptoRaw(RC4_MD5):  one pass over the
//                      payload feeds MD5 and the RC4 stream; the 30-byte header, which holds the
//                      digest, is encrypted with keystream bytes 0..29 saved up front and written
//                      last                                (ev_kq_aio_transform.c:212-230, 281-283)
//   rc4md5_open_kernel READ side + EvAIOReqTransform_RC4_MD5_DataValidate: one pass decrypts the
//                      frame and feeds the decrypted payload to MD5       (:270-279, :158-184)
#include <type_traits>

#include "brb_kernels.h"
#include "pair_sync.h"
#include "rc4_device.h"
#include "test_options.h"

namespace {

using namespace brb_rc4;

constexpr int kWave = 64 * int(kWaves);   // threads per workgroup

BRB_DEV uint32_t clamp4(uint64_t left) { return left >= 4 ? 4u : uint32_t(left); }

// Wave-uniform maximum (loop bounds of the cooperative block loads).
BRB_DEV uint32_t wave_max(uint32_t x)
{
#pragma unroll
    for (int o = 32; o; o >>= 1) {
        const uint32_t y = uint32_t(__shfl_xor(int(x), o));
        x = y > x ? y : x;
    }
    return __builtin_amdgcn_readfirstlane(x);
}

// BlockSrcW exchange per wave.  Only the plain RC4 pass loads cooperatively: 65 536 x 1500 B,
// 135 -> 124 us.  The frame and open kernels, whose MD5 work per block hides the per-lane loads,
// measured slower with it (frame 141 -> 150 us, open 139 -> 143 us, rocprofv3, tools/gpu_ab_prof.sh).
constexpr uint32_t kXchBytes = 4096;

// Decrypt frame block b (chunks 16b .. 16b + 15 of a frame of F bytes, fetched into c) into pt and
// the sink.
BRB_DEV void decrypt_block(const uint32_t (&c)[16], Snk &snk, Gen &g, uint64_t F, uint64_t b, uint32_t (&pt)[16])
{
    const uint64_t pos = 64 * b;
    if (pos + 64 <= F) {
        uint32_t ks[16];
        g.words(ks);
#pragma unroll
        for (int i = 0; i < 16; i++)
            pt[i] = c[i] ^ ks[i];
        snk.put16(pt);
    } else {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const uint64_t q = pos + 4 * i;
            pt[i] = 0;
            if (q < F) {
                pt[i] = c[i] ^ g.next_n(clamp4(F - q));
                snk.put(pt[i]);
            }
        }
    }
}

BRB_DEV void decrypt_block(brb_io::BlockSrc &src, Snk &snk, Gen &g, uint64_t F, uint64_t b, uint32_t (&pt)[16])
{
    uint32_t c[16];
    src.fetch(c);
    decrypt_block(c, snk, g, F, b, pt);
}

// SECTOR: outputs through brb_io::SectorSnk (whole aligned 64-byte sectors) instead of Snk.
// Measured with the first pipelined generator (tools/gpu_rc4_sector.sh, 65 536 x 1500 B, two
// interleaved rounds): HBM outputs 123.0 -> 128.3 us per pass (the sink's LDS row and address selects
// add ~50 VALU per block to ~1 100 for the keystream) for 190.9 -> 152.8 MB written; zero-copy batcher
// rounds (outputs into page-locked host memory over PCIe) 1.87 -> 1.81 ms pipelined.  With the
// session-4 generator (S[j] read after the swap, rc4_device.h), whose steps wait on LDS as much as on
// issue, the sink's extra VALU fit in those waits: HBM outputs 120.9 -> 118.2 us (three interleaved
// rounds, the rc4_sector test option) and 187 -> 152 MB written (PMC WRITE_SIZE), so
// every RC4 pass output now takes SectorSnk.  The open kernel, whose MD5 work already fills those
// waits, measured slower with it (125.4 -> 134.9 us, interleaved, a build with these kernels templated on
// the sink; not kept), so the frame and
// open kernels keep Snk.
template <bool SECTOR>
__global__ __launch_bounds__(kWave) void rc4_crypt_kernel(uint8_t *__restrict__ states, const uint8_t *in, uint8_t *out,
                                                          const uint64_t *__restrict__ offs,
                                                          const uint32_t *__restrict__ lens, uint64_t n,
                                                          const uint32_t *__restrict__ sidx,
                                                          const uint64_t *__restrict__ ooffs)
{
    __shared__ __attribute__((aligned(16))) uint8_t slot[kSlotLds];
    __shared__ __attribute__((aligned(16))) uint8_t xch[kWaves * kXchBytes];
    __shared__ __attribute__((aligned(16))) uint8_t rows[SECTOR ? kWave * brb_io::SectorSnk::kRowBytes : 16];
    const uint64_t s = uint64_t(blockIdx.x) * kWave + threadIdx.x;
    const bool live = s < n;                     // lanes past n only help with the block loads
    Gen g;
    g.P.lds = slot;
    g.P.lw = (threadIdx.x & 63) * 4 + (threadIdx.x >> 6);
    uint8_t *state = nullptr;
    uint64_t off = 0, len = 0, ooff = 0;
    if (live) {
        state = states + uint64_t(sidx ? sidx[s] : s) * kStateBytes;   // sidx: connection table
        g.load(state);
        off = offs[s];
        len = lens[s];
        ooff = ooffs ? ooffs[s] : off;
    }
    brb_io::BlockSrcW src;
    std::conditional_t<SECTOR, brb_io::SectorSnk, Snk> snk;
    src.init(in + off, len, xch + (threadIdx.x >> 6) * kXchBytes);
    if constexpr (SECTOR)
        snk.init(out + ooff, len, uint32_t(reinterpret_cast<uintptr_t>(rows)) + threadIdx.x * brb_io::SectorSnk::kRowBytes);
    else
        snk.init(out + ooff, len);
    const uint64_t nblk = (len + 63) >> 6;
    const uint32_t nloop = wave_max(uint32_t(nblk));
    uint32_t c[16];
    if (nloop)
        src.fetch(c);
    for (uint32_t b = 0; b < nloop; b++) {
        const uint64_t pos = 64ull * b;
        const bool full = pos + 64 <= len;
        uint32_t ks[16];
        if (full) {
            g.words(ks);
#pragma unroll
            for (int i = 0; i < 16; i++)
                ks[i] ^= c[i];
        } else if (pos < len) {
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const uint64_t q = pos + 4 * i;
                if (q < len)
                    snk.put(c[i] ^ g.next_n(clamp4(len - q)));
            }
        }
        // the next block is taken (and the one after it requested) before this block's stores go
        // out, so the wait for it never includes them
        if (b + 1 < nloop)
            src.fetch(c);
        if (full)
            snk.put16(ks);
    }
    if (live) {
        snk.flush();
        g.store(state);
    }
}

__global__ __launch_bounds__(kWave) void rc4md5_frame_kernel(uint8_t *__restrict__ states, const uint8_t *__restrict__ payload,
                                                             const uint64_t *__restrict__ offs,
                                                             const uint32_t *__restrict__ lens,
                                                             const uint64_t *__restrict__ salts, uint8_t *frames,
                                                             const uint64_t *__restrict__ foffs, uint64_t n,
                                                             const uint32_t *__restrict__ sidx)
{
    __shared__ __attribute__((aligned(16))) uint8_t slot[kSlotLds];
    const uint64_t s = uint64_t(blockIdx.x) * kWave + threadIdx.x;
    if (s >= n)
        return;
    Gen g;
    g.P.lds = slot;
    g.P.lw = (threadIdx.x & 63) * 4 + (threadIdx.x >> 6);
    uint8_t *state = states + uint64_t(sidx ? sidx[s] : s) * kStateBytes;   // sidx: connection table
    g.load(state);
    const uint64_t len = lens[s];
    const uint64_t F = kHeader + len;            // frame bytes
    uint8_t *frame = frames + foffs[s];

    // keystream of frame chunks 0..7 (bytes 0..31; chunk 7 = digest[15], NUL, payload[0..1])
    uint32_t kh[8];
#pragma unroll
    for (int k = 0; k < 7; k++)
        kh[k] = g.next4();
    kh[7] = g.next_n(clamp4(F - 28));

    brb_io::BlockSrc src;
    src.init(payload + offs[s], len);
    Snk snk;                                      // frame bytes 32..F-1
    snk.init(frame + 32, F > 32 ? F - 32 : 0);
    Md5State st = md5_iv();
    const uint64_t nblk = md5_blocks(len), nw = 16 * nblk;
    uint32_t prev = 0, first = 0;
    for (uint64_t b = 0; b < nblk; b++) {
        uint32_t m[16], rw[16];
        src.fetch(rw);
        // frame chunks 16b + 7 .. 16b + 22 (payload words 16b .. 16b + 15; word 0 lives in the
        // header chunk 7): when all of them lie inside the frame, their keystream is one run
        if (4 * (16 * b + 23) <= F) {
            uint32_t ks[16];
            if (b == 0) {
                uint32_t k15[15];
                g.words(k15);
#pragma unroll
                for (int i = 0; i < 15; i++)
                    ks[i + 1] = k15[i];
                ks[0] = 0;
            } else {
                g.words(ks);
            }
            uint32_t ct[16];
#pragma unroll
            for (uint32_t i = 0; i < 16; i++) {
                const uint64_t w = 16 * b + i;
                const uint32_t raw = rw[i];
                if (w == 0)
                    first = raw;
                ct[i] = __builtin_amdgcn_alignbit(raw, prev, 16) ^ ks[i];
                prev = raw;
                m[i] = raw;
            }
            md5_pad_block(m, b, len, nw);
            if (b == 0) {
#pragma unroll
                for (int i = 1; i < 16; i++)
                    snk.put(ct[i]);
            } else {
                snk.put16(ct);
            }
        } else {
#pragma unroll
            for (uint32_t i = 0; i < 16; i++) {
                const uint64_t w = 16 * b + i;
                const uint32_t raw = rw[i];
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
    g.store(state);
}

__global__ __launch_bounds__(kWave) void rc4md5_open_kernel(uint8_t *__restrict__ states, const uint8_t *in, uint8_t *out,
                                                            const uint64_t *__restrict__ offs,
                                                            const uint32_t *__restrict__ lens, uint64_t n,
                                                            uint8_t *__restrict__ valid,
                                                            const uint32_t *__restrict__ sidx,
                                                            const uint64_t *__restrict__ ooffs)
{
    __shared__ __attribute__((aligned(16))) uint8_t slot[kSlotLds];
    const uint64_t s = uint64_t(blockIdx.x) * kWave + threadIdx.x;
    if (s >= n)
        return;
    Gen g;
    g.P.lds = slot;
    g.P.lw = (threadIdx.x & 63) * 4 + (threadIdx.x >> 6);
    uint8_t *state = states + uint64_t(sidx ? sidx[s] : s) * kStateBytes;   // sidx: connection table
    g.load(state);
    const uint64_t off = offs[s], F = lens[s];
    brb_io::BlockSrc src;
    Snk snk;
    src.init(in + off, F);
    snk.init(out + (ooffs ? ooffs[s] : off), F);

    // frame block 0 = chunks 0..15; the header is chunks 0..7 (frame bytes 0..31)
    uint32_t cur[16];
    decrypt_block(src, snk, g, F, 0, cur);
    uint32_t ok = 0;
    if (F >= kHeader) {
        // payload word w = frame bytes 30 + 4w .. 33 + 4w: the high half of chunk w + 7 and the low
        // half of chunk w + 8; MD5 block b needs chunks 16b + 7 .. 16b + 23 = frame blocks b, b + 1
        const uint64_t len = F - kHeader;
        const uint64_t nblk = md5_blocks(len), nw = 16 * nblk;
        const uint32_t h2 = cur[2], h3 = cur[3], h4 = cur[4], h5 = cur[5], h6 = cur[6], h7 = cur[7];
        Md5State st = md5_iv();
        for (uint64_t b = 0; b < nblk; b++) {
            uint32_t nxt[16], m[16];
            decrypt_block(src, snk, g, F, b + 1, nxt);
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const uint32_t lo = i + 7 < 16 ? cur[i + 7] : nxt[i - 9];
                const uint32_t hi = i + 8 < 16 ? cur[i + 8] : nxt[i - 8];
                m[i] = __builtin_amdgcn_alignbit(hi, lo, 16);
            }
            md5_pad_block(m, b, len, nw);
            md5_compress(st, m);
#pragma unroll
            for (int i = 0; i < 16; i++)
                cur[i] = nxt[i];
        }
        const bool tag = h2 == 0x48534148u && (h3 & 0xFFu) == 0x3Au;   // "HASH:" at 8..12
        const bool dig = __builtin_amdgcn_alignbit(h4, h3, 8) == st.a && __builtin_amdgcn_alignbit(h5, h4, 8) == st.b &&
                         __builtin_amdgcn_alignbit(h6, h5, 8) == st.c && __builtin_amdgcn_alignbit(h7, h6, 8) == st.d;
        ok = tag && dig;
    }
    snk.flush();
    valid[s] = uint8_t(ok);
    g.store(state);
}

// The RC4 pass as wave pairs (round 4).  rc4_crypt_kernel's lone wave per SIMD spends its issue on
// the keystream chain (97 us of the 115 us pass with the I/O compiled out, tools/mb/rc4_parts.hip)
// plus the block loads, their exchange and the sink.  Here the 4 keystream waves of a workgroup
// each get an I/O wave (wave w + 4): it loads the streams' 64-byte blocks cooperatively
// (BlockSrcW) into a two-block LDS ring per lane, and stores the results the keystream wave leaves
// in a second ring; per-lane mailbox counts (staged, taken, produced, stored) order the hand-offs.
struct Rc4Mail {
    uint32_t *in_cnt, *in_used, *out_cnt, *out_used;   // this lane's
};

// false after 2^22 sleeps in which the wave's open lanes saw no progress
template <class F>
BRB_DEV bool rc4_wait(F blocked)
{
    for (uint32_t spin = 0; spin < (1u << 22); spin++) {
        if (__builtin_amdgcn_ballot_w64(blocked()) == 0)
            return true;
        __builtin_amdgcn_s_sleep(1);
    }
    return false;
}

// STALL: test option pair_stall (pair_fault.h), a separate instantiation so the product kernel
// carries no test code.
template <bool STALL>
__global__ __launch_bounds__(2 * kWave) void rc4_crypt_pair_kernel(uint8_t *__restrict__ states, const uint8_t *in,
                                                                   uint8_t *out, const uint64_t *__restrict__ offs,
                                                                   const uint32_t *__restrict__ lens, uint64_t n,
                                                                   const uint32_t *__restrict__ sidx,
                                                                   const uint64_t *__restrict__ ooffs, uint32_t *fault)
{
    using brb_line::pc_fault_from;
    using brb_line::pc_load;
    using brb_line::pc_publish;
    __shared__ __attribute__((aligned(16))) uint8_t slot[kSlotLds];
    __shared__ uint32_t rin[kWaves][2][16][64];         // staged input blocks, word i of lane l at [.][i][l]
    __shared__ uint32_t rout[kWaves][2][16][64];        // produced output blocks
    __shared__ __attribute__((aligned(16))) uint8_t xch[kWaves * kXchBytes];
    __shared__ uint32_t mb[kWaves][4][64];              // staged, taken, produced, stored (blocks)
    __shared__ uint32_t *fault_at;                      // pair_sync.h pc_fault_from
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t w4 = wv % kWaves;
    for (uint32_t i = threadIdx.x; i < kWaves * 4 * 64; i += 2 * kWave)
        (&mb[0][0][0])[i] = 0;
    if (threadIdx.x == 0)
        fault_at = fault;
    __syncthreads();
    const uint64_t s = uint64_t(blockIdx.x) * kWave + w4 * 64 + lane;
    const bool live = s < n;                           // lanes past n only help with the block loads
    const uint64_t len = live ? lens[s] : 0;
    const uint32_t nblk = uint32_t((len + 63) >> 6);
    const uint32_t nloop = wave_max(nblk);
    const Rc4Mail m{&mb[w4][0][lane], &mb[w4][1][lane], &mb[w4][2][lane], &mb[w4][3][lane]};
    if (wv >= kWaves) {
        // ---- I/O wave
        const uint64_t off = live ? offs[s] : 0;
        brb_io::BlockSrcW src;
        src.init(in + off, len, xch + w4 * kXchBytes);
        Snk snk;
        snk.init(out + (live && ooffs ? ooffs[s] : off), len);
        // test option pair_stall: the first workgroup's first I/O wave never hands a block over
        const bool stalled = STALL && blockIdx.x == 0 && w4 == 0;
        uint32_t bi = 0, bo = 0;
        for (uint32_t idle = 0; bo < nloop && idle < (1u << 22);) {
            // stage block bi once the keystream wave has taken block bi - 2 (its slot is free)
            if (bi < nloop && __builtin_amdgcn_ballot_w64(bi < nblk && pc_load(m.in_used) + 2 <= bi) == 0) {
                uint32_t c[16];
                src.fetch(c);                          // every lane: the loads are cooperative
                if (bi < nblk && !stalled) {
#pragma unroll
                    for (int i = 0; i < 16; i++)
                        rin[w4][bi & 1][i][lane] = c[i];
                    pc_publish(m.in_cnt, bi + 1);
                }
                bi++;
                idle = 0;
                continue;
            }
            // store block bo once produced
            if (__builtin_amdgcn_ballot_w64(bo < nblk && pc_load(m.out_cnt) < bo + 1) == 0) {
                if (bo < nblk) {
                    uint32_t w[16];
#pragma unroll
                    for (int i = 0; i < 16; i++)
                        w[i] = rout[w4][bo & 1][i][lane];
                    pc_publish(m.out_used, bo + 1);
                    if (64ull * bo + 64 <= len) {
                        snk.put16(w);
                    } else {
#pragma unroll
                        for (int i = 0; i < 16; i++)
                            if (64ull * bo + 4 * i < len)
                                snk.put(w[i]);
                    }
                }
                bo++;
                idle = 0;
                continue;
            }
            __builtin_amdgcn_s_sleep(1);
            idle++;
        }
        if (bo < nloop)
            pc_fault_from(&fault_at);                 // a protocol fault: reported, never a hang
        if (live)
            snk.flush();
        return;
    }
    // ---- keystream wave (issue priority: its chain is the critical path)
    __builtin_amdgcn_s_setprio(3);
    Gen g;
    g.P.lds = slot;
    g.P.lw = lane * 4 + w4;
    uint8_t *state = live ? states + uint64_t(sidx ? sidx[s] : s) * kStateBytes : nullptr;
    if (live)
        g.load(state);
    for (uint32_t b = 0; b < nloop; b++) {
        if (!rc4_wait([&] { return b < nblk && pc_load(m.in_cnt) < b + 1; }))
            break;                                     // a protocol fault: the I/O wave reports it
        if (b >= nblk)
            continue;
        uint32_t c[16];
#pragma unroll
        for (int i = 0; i < 16; i++)
            c[i] = rin[w4][b & 1][i][lane];
        pc_publish(m.in_used, b + 1);
        const uint64_t pos = 64ull * b;
        uint32_t o[16];
        if (pos + 64 <= len) {
            uint32_t ks[16];
            g.words(ks);
#pragma unroll
            for (int i = 0; i < 16; i++)
                o[i] = c[i] ^ ks[i];
        } else {
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const uint64_t q = pos + 4 * i;
                o[i] = q < len ? c[i] ^ g.next_n(clamp4(len - q)) : 0u;
            }
        }
        if (!rc4_wait([&] { return pc_load(m.out_used) + 2 <= b; }))
            break;
#pragma unroll
        for (int i = 0; i < 16; i++)
            rout[w4][b & 1][i][lane] = o[i];
        pc_publish(m.out_cnt, b + 1);
    }
    if (live)
        g.store(state);
}

// RC4 + MD5 frames as wave pairs (round 4).  The fused kernels run one wave per SIMD that does the
// keystream chain, the MD5 and the I/O.  Here each keystream wave (waves 0..3) gets a partner
// (wave w + 4) that does everything else: it loads the blocks cooperatively (BlockSrcW) into a
// two-block LDS ring per lane, computes the MD5, and stores what the keystream wave leaves in a
// second ring; the mailbox counts of rc4_crypt_pair_kernel order the hand-offs.  The keystream
// wave keeps the SIMD's issue priority: its chain is the critical path.
//   frame (write side, ev_kq_aio_transform.c:212-230, 281-283): the partner stages the payload
//     blocks and digests them; the keystream wave encrypts them (frame chunks 7.., payload shifted
//     by 2 bytes) and, once the digest is posted, writes the encrypted header;
//   open (read side + DataValidate, :158-184, 270-279): the partner stages the frame blocks; the
//     keystream wave decrypts them; the partner stores the plaintext, digests the payload words
//     (frame bytes 30 + 4w, two plaintext blocks funnel-shifted), checks "HASH:" and the digest and
//     writes the valid flag.
// Earlier forms measured (rocprofv3, 65 536 x 1 530-byte frames): fused frame 128.1 us / open
// 122.9 us; the MD5 alone on the partner with the keystream wave doing the I/O: frame 127.2 us, open
// 111.1 us.

// The I/O side of a pair: stage input block bi once block bi - 2 is taken; hand back output block bo
// once produced.  `stage(c, b)` gets every lane's block b (lanes past their count included: the
// loads are cooperative); `drain(b)` runs for the lanes whose block b is out.  Returns when every
// output block is drained (true), or after 2^22 idle sleeps (false: a protocol fault, no hang).
template <class Stage, class Drain>
BRB_DEV bool pair_io(const Rc4Mail &m, uint32_t nblk, uint32_t nloop, brb_io::BlockSrcW &src, Stage stage, Drain drain)
{
    using brb_line::pc_load;
    uint32_t bi = 0, bo = 0;
    for (uint32_t idle = 0; bo < nloop && idle < (1u << 22);) {
        if (bi < nloop && __builtin_amdgcn_ballot_w64(bi < nblk && pc_load(m.in_used) + 2 <= bi) == 0) {
            uint32_t c[16];
            src.fetch(c);
            stage(c, bi);
            bi++;
            idle = 0;
            continue;
        }
        if (__builtin_amdgcn_ballot_w64(bo < nblk && pc_load(m.out_cnt) < bo + 1) == 0) {
            if (bo < nblk)
                drain(bo);
            bo++;
            idle = 0;
            continue;
        }
        __builtin_amdgcn_s_sleep(1);
        idle++;
    }
    return bo >= nloop;
}

// STALL (both pair kernels): test option pair_stall, as rc4_crypt_pair_kernel -- the first workgroup's
// first partner wave stages its blocks but never hands one over, so both waves' bounded waits give up.
template <bool STALL>
__global__ __launch_bounds__(2 * kWave) void rc4md5_frame_pair_kernel(uint8_t *__restrict__ states,
                                                                      const uint8_t *__restrict__ payload,
                                                                      const uint64_t *__restrict__ offs,
                                                                      const uint32_t *__restrict__ lens,
                                                                      const uint64_t *__restrict__ salts, uint8_t *frames,
                                                                      const uint64_t *__restrict__ foffs, uint64_t n,
                                                                      const uint32_t *__restrict__ sidx, uint32_t *fault)
{
    using brb_line::pc_fault_from;
    using brb_line::pc_load;
    using brb_line::pc_publish;
    __shared__ __attribute__((aligned(16))) uint8_t slot[kSlotLds];
    __shared__ uint32_t rin[kWaves][2][16][64];
    __shared__ uint32_t rout[kWaves][2][16][64];
    __shared__ __attribute__((aligned(16))) uint8_t xch[kWaves * kXchBytes];
    __shared__ uint32_t mb[kWaves][4][64];
    __shared__ uint32_t *fault_at;                      // pair_sync.h pc_fault_from
    __shared__ uint32_t dg[kWaves][4][64];        // the digests
    __shared__ uint32_t posted[kWaves];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t w4 = wv % kWaves;
    for (uint32_t i = threadIdx.x; i < kWaves * 4 * 64; i += 2 * kWave)
        (&mb[0][0][0])[i] = 0;
    if (threadIdx.x < kWaves)
        posted[threadIdx.x] = 0;
    if (threadIdx.x == 0)
        fault_at = fault;
    __syncthreads();
    const uint64_t s = uint64_t(blockIdx.x) * kWave + w4 * 64 + lane;
    const bool live = s < n;
    const uint64_t len = live ? lens[s] : 0;
    const uint64_t F = kHeader + len;              // frame bytes
    const uint32_t nblk = live ? uint32_t(md5_blocks(len)) : 0u;
    const uint32_t nloop = wave_max(nblk);
    const Rc4Mail m{&mb[w4][0][lane], &mb[w4][1][lane], &mb[w4][2][lane], &mb[w4][3][lane]};
    if (wv >= kWaves) {
        // ---- partner: payload blocks in, MD5 (ev_kq_aio_transform.c:218-222), ciphertext out
        brb_io::BlockSrcW src;
        src.init(payload + (live ? offs[s] : 0), len, xch + w4 * kXchBytes);
        Snk snk;                                  // frame bytes 32..F-1
        snk.init(live ? frames + foffs[s] + 32 : nullptr, live && F > 32 ? F - 32 : 0);
        Md5State st = md5_iv();
        const uint64_t nw = 16 * uint64_t(nblk);
        const bool stalled = STALL && blockIdx.x == 0 && w4 == 0;
        const bool io_ok = pair_io(
            m, nblk, nloop, src,
            [&](const uint32_t (&c)[16], uint32_t b) {
                if (b < nblk) {
#pragma unroll
                    for (int i = 0; i < 16; i++)
                        rin[w4][b & 1][i][lane] = c[i];
                    if (!stalled)
                        pc_publish(m.in_cnt, b + 1);
                    uint32_t w[16];
#pragma unroll
                    for (int i = 0; i < 16; i++)
                        w[i] = c[i];
                    md5_pad_block(w, b, len, nw);
                    md5_compress(st, w);
                }
                if (b + 1 == nloop) {             // every block digested: the header can go
                    dg[w4][0][lane] = st.a;
                    dg[w4][1][lane] = st.b;
                    dg[w4][2][lane] = st.c;
                    dg[w4][3][lane] = st.d;
                    pc_publish(&posted[w4], 1u);
                }
            },
            [&](uint32_t b) {
                uint32_t ct[16];
#pragma unroll
                for (int i = 0; i < 16; i++)
                    ct[i] = rout[w4][b & 1][i][lane];
                pc_publish(m.out_used, b + 1);
                if (4 * (16 * uint64_t(b) + 23) <= F) {
                    if (b == 0) {
#pragma unroll
                        for (int i = 1; i < 16; i++)
                            snk.put(ct[i]);
                    } else {
                        snk.put16(ct);
                    }
                } else {
#pragma unroll
                    for (uint32_t i = 0; i < 16; i++) {
                        const uint64_t w = 16 * uint64_t(b) + i;
                        if (w != 0 && 4 * (w + 7) < F)
                            snk.put(ct[i]);
                    }
                }
            });
        if (!io_ok)
            pc_fault_from(&fault_at);
        if (nloop == 0)
            pc_publish(&posted[w4], 1u);
        if (live)
            snk.flush();
        return;
    }
    // ---- keystream wave
    __builtin_amdgcn_s_setprio(3);
    Gen g;
    g.P.lds = slot;
    g.P.lw = lane * 4 + w4;
    uint8_t *state = live ? states + uint64_t(sidx ? sidx[s] : s) * kStateBytes : nullptr;
    uint32_t kh[8];                               // keystream of frame chunks 0..7 (the header)
    if (live) {
        g.load(state);
#pragma unroll
        for (int k = 0; k < 7; k++)
            kh[k] = g.next4();
        kh[7] = g.next_n(clamp4(F - 28));
    }
    uint32_t prev = 0, first = 0;
    bool ok = true;
    for (uint32_t b = 0; b < nloop && ok; b++) {
        ok = rc4_wait([&] { return b < nblk && pc_load(m.in_cnt) < b + 1; });
        if (b >= nblk || !ok)
            continue;
        uint32_t rw[16], ct[16];
#pragma unroll
        for (int i = 0; i < 16; i++)
            rw[i] = rin[w4][b & 1][i][lane];
        pc_publish(m.in_used, b + 1);
        if (4 * (16 * uint64_t(b) + 23) <= F) {
            uint32_t ks[16];
            if (b == 0) {
                uint32_t k15[15];
                g.words(k15);
#pragma unroll
                for (int i = 0; i < 15; i++)
                    ks[i + 1] = k15[i];
                ks[0] = 0;
                first = rw[0];
            } else {
                g.words(ks);
            }
#pragma unroll
            for (uint32_t i = 0; i < 16; i++) {
                ct[i] = __builtin_amdgcn_alignbit(rw[i], prev, 16) ^ ks[i];
                prev = rw[i];
            }
        } else {
#pragma unroll
            for (uint32_t i = 0; i < 16; i++) {
                const uint64_t w = 16 * uint64_t(b) + i;
                const uint32_t raw = rw[i];
                ct[i] = 0;
                if (w == 0) {
                    first = raw;
                } else {
                    const uint64_t fb = 4 * (w + 7);   // frame chunk w + 7 = payload bytes 4w - 2 .. 4w + 1
                    if (fb < F)
                        ct[i] = __builtin_amdgcn_alignbit(raw, prev, 16) ^ g.next_n(clamp4(F - fb));
                }
                prev = raw;
            }
        }
        ok = rc4_wait([&] { return pc_load(m.out_used) + 2 <= b; });
#pragma unroll
        for (int i = 0; i < 16; i++)
            rout[w4][b & 1][i][lane] = ct[i];
        pc_publish(m.out_cnt, b + 1);
    }
    if (!live)
        return;
    const bool got = brb_line::pc_wait_ge(&posted[w4], 1u) && ok;
    Md5State st;
    st.a = dg[w4][0][lane];
    st.b = dg[w4][1][lane];
    st.c = dg[w4][2][lane];
    st.d = dg[w4][3][lane];
    if (!got)
        st.a = ~st.a;                             // a protocol fault (a wrong header; the partner reports it)
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
    hs.init(frames + foffs[s], F < 32 ? F : 32);
#pragma unroll
    for (int k = 0; k < 8; k++)
        hs.put(h[k] ^ kh[k]);
    hs.flush();
    g.store(state);
}

template <bool STALL>
__global__ __launch_bounds__(2 * kWave) void rc4md5_open_pair_kernel(uint8_t *__restrict__ states, const uint8_t *in,
                                                                     uint8_t *out, const uint64_t *__restrict__ offs,
                                                                     const uint32_t *__restrict__ lens, uint64_t n,
                                                                     uint8_t *__restrict__ valid,
                                                                     const uint32_t *__restrict__ sidx,
                                                                     const uint64_t *__restrict__ ooffs, uint32_t *fault)
{
    using brb_line::pc_fault_from;
    using brb_line::pc_load;
    using brb_line::pc_publish;
    __shared__ __attribute__((aligned(16))) uint8_t slot[kSlotLds];
    __shared__ uint32_t rin[kWaves][2][16][64];
    __shared__ uint32_t rout[kWaves][2][16][64];
    __shared__ __attribute__((aligned(16))) uint8_t xch[kWaves * kXchBytes];
    __shared__ uint32_t mb[kWaves][4][64];
    __shared__ uint32_t *fault_at;                      // pair_sync.h pc_fault_from
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t w4 = wv % kWaves;
    for (uint32_t i = threadIdx.x; i < kWaves * 4 * 64; i += 2 * kWave)
        (&mb[0][0][0])[i] = 0;
    if (threadIdx.x == 0)
        fault_at = fault;
    __syncthreads();
    const uint64_t s = uint64_t(blockIdx.x) * kWave + w4 * 64 + lane;
    const bool live = s < n;
    const uint64_t off = live ? offs[s] : 0, F = live ? lens[s] : 0;
    const bool framed = live && F >= kHeader;
    const uint64_t len = framed ? F - kHeader : 0;
    // frame blocks 0 .. nfb-1: block 0 (the header and payload bytes 0..33), then block b + 1 for
    // every MD5 block b, as rc4md5_open_kernel
    const uint32_t nmd = framed ? uint32_t(md5_blocks(len)) : 0u;
    const uint32_t nfb = live ? 1 + nmd : 0u;
    const uint32_t nloop = wave_max(nfb);
    const Rc4Mail m{&mb[w4][0][lane], &mb[w4][1][lane], &mb[w4][2][lane], &mb[w4][3][lane]};
    if (wv >= kWaves) {
        // ---- partner: frame blocks in, plaintext out, MD5 of the payload and the check
        brb_io::BlockSrcW src;
        src.init(in + off, F, xch + w4 * kXchBytes);
        Snk snk;
        snk.init(live ? out + (ooffs ? ooffs[s] : off) : nullptr, F);
        Md5State st = md5_iv();
        const uint64_t nw = 16 * uint64_t(nmd);
        uint32_t cur[16], h[6] = {0, 0, 0, 0, 0, 0};
        const bool stalled = STALL && blockIdx.x == 0 && w4 == 0;
        const bool io_ok = pair_io(
            m, nfb, nloop, src,
            [&](const uint32_t (&c)[16], uint32_t b) {
                if (b < nfb && !stalled) {
#pragma unroll
                    for (int i = 0; i < 16; i++)
                        rin[w4][b & 1][i][lane] = c[i];
                    pc_publish(m.in_cnt, b + 1);
                }
            },
            [&](uint32_t j) {
                uint32_t pt[16];
#pragma unroll
                for (int i = 0; i < 16; i++)
                    pt[i] = rout[w4][j & 1][i][lane];
                pc_publish(m.out_used, j + 1);
                const uint64_t pos = 64 * uint64_t(j);
                if (pos + 64 <= F) {
                    snk.put16(pt);
                } else {
#pragma unroll
                    for (int i = 0; i < 16; i++)
                        if (pos + 4 * i < F)
                            snk.put(pt[i]);
                }
                if (j == 0) {
#pragma unroll
                    for (int q = 0; q < 6; q++)
                        h[q] = pt[2 + q];
                } else {                          // MD5 block j - 1: frame blocks j - 1 (cur) and j
                    uint32_t w[16];
#pragma unroll
                    for (int i = 0; i < 16; i++) {
                        const uint32_t lo = i + 7 < 16 ? cur[i + 7] : pt[i - 9];
                        const uint32_t hi = i + 8 < 16 ? cur[i + 8] : pt[i - 8];
                        w[i] = __builtin_amdgcn_alignbit(hi, lo, 16);
                    }
                    md5_pad_block(w, j - 1, len, nw);
                    md5_compress(st, w);
                }
#pragma unroll
                for (int i = 0; i < 16; i++)
                    cur[i] = pt[i];
            });
        if (!io_ok)
            pc_fault_from(&fault_at);
        if (live) {
            snk.flush();
            const bool tag = h[0] == 0x48534148u && (h[1] & 0xFFu) == 0x3Au;   // "HASH:" at 8..12
            const bool dig = __builtin_amdgcn_alignbit(h[2], h[1], 8) == st.a &&
                             __builtin_amdgcn_alignbit(h[3], h[2], 8) == st.b &&
                             __builtin_amdgcn_alignbit(h[4], h[3], 8) == st.c &&
                             __builtin_amdgcn_alignbit(h[5], h[4], 8) == st.d;
            valid[s] = uint8_t(framed && tag && dig);
        }
        return;
    }
    // ---- keystream wave
    __builtin_amdgcn_s_setprio(3);
    Gen g;
    g.P.lds = slot;
    g.P.lw = lane * 4 + w4;
    uint8_t *state = live ? states + uint64_t(sidx ? sidx[s] : s) * kStateBytes : nullptr;
    if (live)
        g.load(state);
    bool ok = true;
    for (uint32_t j = 0; j < nloop && ok; j++) {
        ok = rc4_wait([&] { return j < nfb && pc_load(m.in_cnt) < j + 1; });
        if (j >= nfb || !ok)
            continue;
        uint32_t c[16], pt[16];
#pragma unroll
        for (int i = 0; i < 16; i++)
            c[i] = rin[w4][j & 1][i][lane];
        pc_publish(m.in_used, j + 1);
        const uint64_t pos = 64 * uint64_t(j);
        if (pos + 64 <= F) {
            uint32_t ks[16];
            g.words(ks);
#pragma unroll
            for (int i = 0; i < 16; i++)
                pt[i] = c[i] ^ ks[i];
        } else {
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const uint64_t q = pos + 4 * i;
                pt[i] = q < F ? c[i] ^ g.next_n(clamp4(F - q)) : 0u;
            }
        }
        ok = rc4_wait([&] { return pc_load(m.out_used) + 2 <= j; });
#pragma unroll
        for (int i = 0; i < 16; i++)
            rout[w4][j & 1][i][lane] = pt[i];
        pc_publish(m.out_cnt, j + 1);
    }
    if (live)
        g.store(state);
}

inline unsigned grid_for(uint64_t n) { return unsigned((n + kWave - 1) / kWave); }

}  // namespace

namespace brb {

hipError_t launch_rc4_crypt(uint8_t *states, const uint8_t *in, uint8_t *out, const uint64_t *offs,
                            const uint32_t *lens, uint64_t n, hipStream_t s, const uint32_t *sidx,
                            const uint64_t *ooffs, bool sector_out)
{
    if (n == 0)
        return hipSuccess;
    // test option "rc4_sector" = 0/1 forces the sink for A/B measurements and tests
    const int force = brb_opt::get(brb_opt::kRc4Sector);
    if (force >= 0)
        sector_out = force == 1;
    if (brb_opt::get(brb_opt::kRc4CryptPair) != 0 && force < 0) {
        if (brb_opt::get(brb_opt::kPairStall) != 0)
            rc4_crypt_pair_kernel<true><<<grid_for(n), 2 * kWave, 0, s>>>(states, in, out, offs, lens, n, sidx, ooffs,
                                                                          brb::pair_fault_word());
        else
            rc4_crypt_pair_kernel<false><<<grid_for(n), 2 * kWave, 0, s>>>(states, in, out, offs, lens, n, sidx, ooffs,
                                                                           brb::pair_fault_word());
    } else if (sector_out)
        rc4_crypt_kernel<true><<<grid_for(n), kWave, 0, s>>>(states, in, out, offs, lens, n, sidx, ooffs);
    else
        rc4_crypt_kernel<false><<<grid_for(n), kWave, 0, s>>>(states, in, out, offs, lens, n, sidx, ooffs);
    return hipGetLastError();
}

hipError_t launch_rc4md5_frame(uint8_t *states, const uint8_t *payload, const uint64_t *offs, const uint32_t *lens,
                               const uint64_t *salts, uint8_t *frames, const uint64_t *foffs, uint64_t n,
                               hipStream_t s, const uint32_t *sidx)
{
    if (n == 0)
        return hipSuccess;
    if (brb_opt::get(brb_opt::kRc4Pair) != 0) {
        if (brb_opt::get(brb_opt::kPairStall) != 0)
            rc4md5_frame_pair_kernel<true><<<grid_for(n), 2 * kWave, 0, s>>>(states, payload, offs, lens, salts, frames,
                                                                             foffs, n, sidx, brb::pair_fault_word());
        else
            rc4md5_frame_pair_kernel<false><<<grid_for(n), 2 * kWave, 0, s>>>(states, payload, offs, lens, salts, frames,
                                                                              foffs, n, sidx, brb::pair_fault_word());
    } else
        rc4md5_frame_kernel<<<grid_for(n), kWave, 0, s>>>(states, payload, offs, lens, salts, frames, foffs, n, sidx);
    return hipGetLastError();
}

hipError_t launch_rc4md5_open(uint8_t *states, const uint8_t *in, uint8_t *out, const uint64_t *offs,
                              const uint32_t *lens, uint64_t n, uint8_t *valid, hipStream_t s, const uint32_t *sidx,
                              const uint64_t *ooffs)
{
    if (n == 0)
        return hipSuccess;
    if (brb_opt::get(brb_opt::kRc4Pair) != 0) {
        if (brb_opt::get(brb_opt::kPairStall) != 0)
            rc4md5_open_pair_kernel<true><<<grid_for(n), 2 * kWave, 0, s>>>(states, in, out, offs, lens, n, valid, sidx,
                                                                            ooffs, brb::pair_fault_word());
        else
            rc4md5_open_pair_kernel<false><<<grid_for(n), 2 * kWave, 0, s>>>(states, in, out, offs, lens, n, valid, sidx,
                                                                             ooffs, brb::pair_fault_word());
    } else
        rc4md5_open_kernel<<<grid_for(n), kWave, 0, s>>>(states, in, out, offs, lens, n, valid, sidx, ooffs);
    return hipGetLastError();
}

}  // namespace brb
