// host_pipe.h -- host-mode execution of the batch calls (internal, not exported).
//
// A host-mode call starts and ends in the caller's host memory (the kqueue receive path's socket
// buffers, mem_buf.c:1224-1254 recv() into a calloc'd MemBuffer), so it is bound by PCIe, not HBM.
// These functions cut a batch into chunks and overlap the H2D copy of chunk k with the kernel on
// chunk k-1 and the D2H copy of chunk k-2, straight from and to the caller's memory (pageable or
// page-locked), and with BRB_BATCH_ALL_DEVICES split the batch into contiguous record ranges over
// every visible device (no collective).  DESIGN.md §5 has the measured rates.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <functional>

#include "brb_crypto.h"

namespace brb_api {
// Per-thread, per-device grow-only device scratch (batch_api.hip).
void *workspace(size_t bytes, hipError_t *err);
}  // namespace brb_api

namespace brb_host {

using FixedLauncher = hipError_t (*)(const uint8_t *, uint32_t, uint64_t, uint8_t *, hipStream_t);

// Fixed-stride digests (BRB_MD5BatchFixed / BrbSha1_BatchFixed) in host mode.
int digest_fixed(FixedLauncher launch, size_t dig_len, const uint8_t *data, uint32_t rec_len, uint64_t n_rec,
                 uint8_t *digests, unsigned flags, hipStream_t s);

// Blowfish ECB in place (BRB_Blowfish_EncryptBatch / DecryptBatch) in host mode.
int blowfish(const BRB_BLOWFISH_CTX *ctx, uint64_t *words, uint64_t n_items, bool decrypt, unsigned flags,
             hipStream_t s);

// Runs part(dev, lo, hi) for the contiguous ranges [g*n/G, (g+1)*n/G) of n items over G parts,
// concurrently (one persistent worker thread per part, current device = dev = part_device(g)), and
// returns BRB_BATCH_OK or the first failing part's code with "device g: <reason>" in LastError.
// G = the visible devices, or the "devices" test option (parts mapped onto the visible devices).
int split_devices(uint64_t n, const std::function<int(int dev, uint64_t lo, uint64_t hi)> &part);
int split_parts();                 // G
int part_device(int g);            // the device of part g

// Destroys the calling thread's pipeline streams and events (BRB_CryptoGPU_ThreadCleanup).
void release_thread_pipes();

}  // namespace brb_host
