// pair_fault.h -- how a wave-pair kernel's protocol fault reaches the call that launched it.
//
// The wave-pair kernels (md5_seg_pc_kernel, metadata_line_kernel<..., PC>, rc4_crypt_pair_kernel,
// rc4md5_frame_pair_kernel, rc4md5_open_pair_kernel) bound every wait on their partner wave, so a
// protocol fault ends the launch instead of hanging it, with wrong outputs.  The consumer / I/O wave
// of a pair, whose waits give up whenever its partner's do (a partner that gives up stops feeding
// it), stores 1 into the armed fault word (pc_fault_from, pair_sync.h); the producer and keystream
// waves carry no fault code, so their loops compile as before.  A fault word is 32 bits of
// page-locked, device-mapped, portable host memory, and the launchers pass whichever word is armed
// on the launching thread:
//   * a synchronous batch call arms the thread's call word (PairFault in batch_api.hip: one
//     thread-local store, nothing between the caller and the launch) and reads it once the stream
//     has drained: a set word turns the call into BRB_BATCH_FAULT (-4) with "wave-pair protocol
//     fault" in BRB_CryptoGPU_LastError();
//   * a device-mode BRB_BATCH_ASYNC call arms the thread's sticky async word, which
//     BRB_CryptoGPU_AsyncFaultCheck() reads and clears after the caller has synchronised its streams;
//   * a transform batcher round arms its own round word (pair_fault_arm) around its launches and
//     reads it when the round completes: a set word drops the round (BRB_BATCH_DROPPED, every buffer
//     delivered as BRB_TRANSFORM_DROPPED), so no wrong plaintext, frame or valid flag is delivered.
#pragma once

#include <cstdint>

namespace brb {

// The word armed on the calling thread (device-visible address), or nullptr.  Read by the
// launchers of the pair kernels.
uint32_t *pair_fault_word();

// Arms `w` on the calling thread (nullptr disarms); returns the word armed before.
uint32_t *pair_fault_arm(uint32_t *w);

}  // namespace brb
