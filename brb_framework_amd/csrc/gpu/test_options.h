// test_options.h -- process-wide A/B and test switches, set only through the exported test-support
// call BRB_CryptoGPU_TestOption (batch_api.hip).  The library reads no environment variable: a
// stray variable in a production process cannot change a code path.
#pragma once

#include <atomic>

namespace brb_opt {

enum Opt {
    kRc4Sector = 0,     // -1: the launcher's choice; 0/1 force Snk / SectorSnk for the RC4 pass
    kVarLine = 1,       // 1: variable-length digests on the line kernel; 0: per-lane kernel
    kFixedVarLine = 2,  // 1: byte-aligned fixed-stride records on the var-line kernel; 0: record-relative
    kVarSort = 3,       // 1: variable-length batches bucketed by block count; 0: caller order
    kDevices = 4,       // 0: BRB_BATCH_ALL_DEVICES / all-devices batchers use every visible device;
                        // k > 0: they split into k parts, part g on device g % (visible devices) --
                        // the concurrent multi-device paths exercised on a one-GPU box
    kB64Group = 5,      // -1: the launcher's choice; 0..6: log2 of the base64 lanes per record
    kHostChunkMiB = 6,  // 0: host-mode Blowfish/RC4 chunks of 16 MiB; k: k MiB (tools/host_sweep.py)
    kHostDigestChunkMiB = 7,   // 0: host-mode digest chunks of 32 MiB; k: k MiB
    kSegLine = 8,       // segment digests / MetaData unpack: 2 line-staged wave pairs (default), 1 line-staged
                        // single waves, 0 the per-lane kernels
    kB64Kernel = 9,     // 64-byte fixed-stride records: 2 digest_b64r_kernel at 8 waves per SIMD (default), 3 the same
                        // at 4, 1 digest_b64_kernel (two LDS slots), 0 the generic DMA kernel
    kLineSlots = 10,    // LDS-DMA ring slots of the line-staged kernels: 2 or 3; 0 = each kernel's default
    kRc4Pair = 11,      // 1: RC4+MD5 frame / open on keystream + partner wave pairs (default); 0: one wave
    kRc4CryptPair = 12, // 1: the RC4 pass on keystream + I/O wave pairs; 0: one wave per stream does both
    kPairStall = 13,    // 1: inject a protocol fault into the segment-digest, MetaData, RC4-pass and frame/open wave pairs
                        // (the first workgroup's first pair never hands over its first plan / block), so the
                        // tests see a bounded wait give up and the call report it (pair_fault.h); 0: off
    kCount = 14
};

inline std::atomic<int> g_opt[kCount] = {-1, 1, 1, 1, 0, -1, 0, 0, 2, 2, 0, 1, 1, 0};

inline int get(Opt o) { return g_opt[o].load(std::memory_order_relaxed); }

}  // namespace brb_opt
