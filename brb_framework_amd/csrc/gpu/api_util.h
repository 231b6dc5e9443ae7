// api_util.h -- error reporting and device selection shared by the C-ABI translation units
// (batch_api.hip, host_pipe.hip, transform_batcher.hip).  The message is per thread and read by
// BRB_CryptoGPU_LastError().
#pragma once

#include <hip/hip_runtime.h>

#include <string>

namespace brb_api {

extern thread_local std::string t_err;
void clear_err();
void set_err(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
int fail_hip(const char *what, hipError_t e);   // sets the message, returns BRB_BATCH_NOT_DONE
int device_ok();                                // BRB_BATCH_OK if a HIP device is visible
int device_count();                             // visible HIP devices (probed once per process), 0 if none
void release_thread_resources();                // the calling thread's workspaces, streams and events

// Makes `dev` the calling thread's current HIP device for one scope and restores the caller's
// device on exit: every batch call runs on the caller's current device, so library code that
// switches devices (a batcher created on another GPU, an all-devices split) must switch back.
class DeviceGuard {
public:
    explicit DeviceGuard(int dev)
    {
        int cur = -1;
        if ((err_ = hipGetDevice(&cur)) != hipSuccess)
            return;
        if (cur != dev) {
            if ((err_ = hipSetDevice(dev)) != hipSuccess)
                return;
            prev_ = cur;
        }
    }
    ~DeviceGuard()
    {
        if (prev_ >= 0)
            (void)hipSetDevice(prev_);
    }
    hipError_t error() const { return err_; }
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;

private:
    int prev_ = -1;
    hipError_t err_ = hipSuccess;
};

}  // namespace brb_api
