// api_util.h -- error reporting shared by the C-ABI translation units (batch_api.hip,
// transform_batcher.hip).  The message is per thread and read by BRB_CryptoGPU_LastError().
#pragma once

#include <hip/hip_runtime.h>

#include <string>

namespace brb_api {

extern thread_local std::string t_err;
void clear_err();
void set_err(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
int fail_hip(const char *what, hipError_t e);   // sets the message, returns BRB_BATCH_NOT_DONE
int device_ok();                                // BRB_BATCH_OK if a HIP device is visible

}  // namespace brb_api
