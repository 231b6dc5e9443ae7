// pair_fault.h -- how a wave-pair kernel's protocol fault reaches the batch call that launched it.
//
// The wave-pair kernels (md5_seg_pc_kernel, metadata_line_kernel<..., PC>, rc4_crypt_pair_kernel,
// rc4md5_frame_pair_kernel, rc4md5_open_pair_kernel) bound every wait on their partner wave, so a
// protocol fault ends the launch instead of hanging it, with wrong outputs.  The wave that gives up
// stores 1 into the call's fault word (pc_fault, pair_sync.h): one 32-bit word of page-locked,
// device-mapped host memory per calling thread and device.  A synchronous batch call arms its
// thread's word before the launch (PairFault in batch_api.hip) and reads it once the stream has
// drained: a set word turns the call into BRB_BATCH_FAULT (-4) with "wave-pair protocol fault" in
// BRB_CryptoGPU_LastError().  Calls that return before the stream drains (device mode with
// BRB_BATCH_ASYNC) and the transform batcher's rounds are not armed: their launches get nullptr and
// store nothing.
#pragma once

#include <cstdint>

namespace brb {

// The word armed on the calling thread (device-visible address), or nullptr.  Read by the
// launchers of the pair kernels.
uint32_t *pair_fault_word();

}  // namespace brb
