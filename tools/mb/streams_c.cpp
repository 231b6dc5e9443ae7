// streams_c.cpp -- K back-to-back BRB_MD5BatchFixed calls (device mode, async) on 1 or 2 HIP streams.
// Build: hipcc -O2 -I../../include streams_c.cpp -L../../brb_framework_amd -lbrb_crypto_gpu -Wl,-rpath,$PWD/../../brb_framework_amd -o streams_c
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>
#include "brb_crypto.h"
int main() {
    const uint32_t L = 1500; const uint64_t n = 65536; const int nrot = 6, K = 200;
    std::vector<uint8_t> h(n * L, 7);
    uint8_t *d[nrot]; unsigned char (*o[3])[16];
    for (int i = 0; i < nrot; i++) { hipMalloc(&d[i], n * L); hipMemcpy(d[i], h.data(), n * L, hipMemcpyHostToDevice); }
    for (int i = 0; i < 3; i++) hipMalloc(&o[i], n * 16);
    hipStream_t s[2]; for (int i = 0; i < 2; i++) hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking);
    for (int ns = 1; ns <= 2; ns++) for (int rep = 0; rep < 3; rep++) {
        hipDeviceSynchronize();
        auto t0 = std::chrono::steady_clock::now();
        for (int k = 0; k < K; k++) {
            int rc = BRB_MD5BatchFixed(d[k % nrot], L, n, o[k % ns], BRB_BATCH_DEVICE | BRB_BATCH_ASYNC, s[k % ns]);
            if (rc != 1) { printf("rc %d %s\n", rc, BRB_CryptoGPU_LastError()); return 1; }
        }
        hipDeviceSynchronize();
        double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / K;
        printf("streams=%d  %.2f us/step  %.0f GB/s\n", ns, us, n * L / us / 1e3);
    }
    // null stream
    hipDeviceSynchronize();
    auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < K; k++) BRB_MD5BatchFixed(d[k % nrot], L, n, o[0], BRB_BATCH_DEVICE | BRB_BATCH_ASYNC, nullptr);
    hipDeviceSynchronize();
    double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / K;
    printf("null stream  %.2f us/step\n", us);
    return 0;
}
