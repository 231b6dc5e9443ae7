// brb_kernels.h -- internal launchers of the gfx950 crypto kernels (C++ linkage, not exported).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "brb_crypto.h"
#include "brb_gpu_common.h"
#include "pair_fault.h"

namespace brb {

// All pointers are device pointers; launches are asynchronous on `s`.
hipError_t launch_md5_fixed(const uint8_t *data, uint32_t rec_len, uint64_t n_rec, uint8_t *out, hipStream_t s);
hipError_t launch_md5_var(const uint8_t *data, const uint64_t *offs, const uint32_t *lens, uint64_t n_rec,
                          uint8_t *out, hipStream_t s);
hipError_t launch_sha1_fixed(const uint8_t *data, uint32_t rec_len, uint64_t n_rec, uint8_t *out, hipStream_t s);
hipError_t launch_sha1_var(const uint8_t *data, const uint64_t *offs, const uint32_t *lens, uint64_t n_rec,
                           uint8_t *out, hipStream_t s);
// ctx_dev: device copy of BRB_BLOWFISH_CTX (P[18] then S[4][256], 64-bit words)
hipError_t launch_blowfish(const uint64_t *ctx_dev, uint64_t *words, uint64_t n_blocks, bool decrypt, hipStream_t s);
// *first = min(*first, index of the first block (xl, xr) with a zero word); *first preset by the caller
hipError_t launch_first_zero_pair(const uint64_t *words, uint64_t n_blocks, unsigned long long *first, hipStream_t s);

// MD5 of segment lists (md5_seg_kernels.hip): record r = segments first[r] .. first[r + 1] - 1
hipError_t launch_md5_segments(const uint8_t *data, const uint64_t *soff, const uint32_t *slen, const uint64_t *first,
                               uint64_t n_rec, uint8_t *out, hipStream_t s);

// MetaDataUnpack of whole packs (metadata_kernels.hip): pack r = data[offs[r] .. + lens[r])
hipError_t launch_metadata_unpack(const uint8_t *data, const uint64_t *offs, const uint32_t *lens, uint64_t n,
                                  BRB_MetaDataUnpackInfo *info, hipStream_t s);

// base64 (base64_kernels.hip)
hipError_t launch_b64_encode(const uint8_t *in, const uint64_t *offs, const uint32_t *lens, uint64_t n, uint8_t *out,
                             const uint64_t *ooffs, uint64_t mean_len, hipStream_t s);
hipError_t launch_b64_decode(const uint8_t *in, const uint64_t *offs, const uint32_t *lens, uint64_t n, uint8_t *out,
                             const uint64_t *ooffs, uint32_t *olens, uint64_t mean_len, hipStream_t s);

// RC4 (rc4_kernels.hip): 264-byte BRB_RC4_State records, updated in place.  Stream i uses
// states[sidx ? sidx[i] : i] (sidx: a connection table, the transform batcher's indirection).
// ooffs: output offsets (nullptr = the input offsets, out mirrors in)
// sector_out: write whole aligned 64-byte sectors (brb_io::SectorSnk); the default for HBM and host
// outputs alike since the session-4 generator (rc4_kernels.hip); false = per-stream 16-byte pieces (Snk)
hipError_t launch_rc4_crypt(uint8_t *states, const uint8_t *in, uint8_t *out, const uint64_t *offs,
                            const uint32_t *lens, uint64_t n, hipStream_t s, const uint32_t *sidx = nullptr,
                            const uint64_t *ooffs = nullptr, bool sector_out = true);
hipError_t launch_rc4md5_frame(uint8_t *states, const uint8_t *payload, const uint64_t *offs, const uint32_t *lens,
                               const uint64_t *salts, uint8_t *frames, const uint64_t *foffs, uint64_t n,
                               hipStream_t s, const uint32_t *sidx = nullptr);
hipError_t launch_rc4md5_open(uint8_t *states, const uint8_t *in, uint8_t *out, const uint64_t *offs,
                              const uint32_t *lens, uint64_t n, uint8_t *valid, hipStream_t s,
                              const uint32_t *sidx = nullptr, const uint64_t *ooffs = nullptr);

}  // namespace brb
