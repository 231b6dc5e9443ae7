// pair_fault.h -- how a wave-pair kernel's protocol fault reaches the batch call that launched it.
//
// The wave-pair kernels (md5_seg_pc_kernel, metadata_line_kernel<..., PC>, rc4_crypt_pair_kernel,
// rc4md5_frame_pair_kernel, rc4md5_open_pair_kernel) bound every wait on their partner wave, so a
// protocol fault ends the launch instead of hanging it, with wrong outputs.  The consumer / I/O wave
// of a pair, whose waits give up whenever its partner's do (a partner that gives up stops feeding
// it), stores 1 into the call's fault word (pc_fault_from, pair_sync.h); the producer and keystream
// waves carry no fault code, so their loops compile as before.  The word is 32 bits of page-locked,
// device-mapped, portable host memory, one per calling thread, 0 between calls.  A synchronous batch
// call arms it (PairFault in batch_api.hip: one thread-local store, nothing between the caller and
// the launch) and reads it once the stream has drained: a set word turns the call into
// BRB_BATCH_FAULT (-4) with "wave-pair protocol fault" in BRB_CryptoGPU_LastError().  Calls that return before the stream drains (device mode with
// BRB_BATCH_ASYNC) and the transform batcher's rounds are not armed: their launches get nullptr and
// store nothing.
#pragma once

#include <cstdint>

namespace brb {

// The word armed on the calling thread (device-visible address), or nullptr.  Read by the
// launchers of the pair kernels.
uint32_t *pair_fault_word();

}  // namespace brb
