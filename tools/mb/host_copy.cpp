// host_copy.cpp -- what a host-mode batch call can reach from pageable memory.
// Measures, for a 98 MB (cfg2) and a 1 GiB (cfg4) buffer:
//   H2D from pageable memory (HIP's own staging), H2D from pinned memory,
//   hipHostRegister + H2D + hipHostUnregister of the pageable buffer,
//   memcpy pageable -> pinned with 1/2/4/8/16 threads,
//   D2H into pageable and into pinned memory.
// build: hipcc -O2 -std=c++17 -pthread tools/mb/host_copy.cpp -o tools/mb/host_copy
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

static double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void par_copy(void *dst, const void *src, size_t n, int th)
{
    std::vector<std::thread> t;
    const size_t per = (n / th + 4095) & ~size_t(4095);
    for (int i = 0; i < th; i++) {
        size_t a = per * i, b = std::min(n, a + per);
        if (a >= b)
            break;
        t.emplace_back([=] { memcpy(static_cast<char *>(dst) + a, static_cast<const char *>(src) + a, b - a); });
    }
    for (auto &x : t)
        x.join();
}

int main()
{
    for (size_t n : {size_t(98304000), size_t(1) << 30}) {
        char *pg = static_cast<char *>(aligned_alloc(4096, n));
        char *pg2 = static_cast<char *>(aligned_alloc(4096, n));
        memset(pg, 1, n);
        memset(pg2, 2, n);
        char *pin;
        CK(hipHostMalloc(reinterpret_cast<void **>(&pin), n, hipHostMallocDefault));
        memset(pin, 3, n);
        void *d;
        CK(hipMalloc(&d, n));
        auto rate = [&](const char *what, auto fn) {
            fn();
            double best = 1e9;
            for (int r = 0; r < 5; r++) {
                double t = now();
                fn();
                best = std::min(best, now() - t);
            }
            printf("{\"bytes\": %zu, \"what\": \"%s\", \"ms\": %.3f, \"GB_s\": %.2f}\n", n, what, best * 1e3, n / best / 1e9);
            fflush(stdout);
        };
        rate("H2D pageable (hipMemcpy)", [&] { CK(hipMemcpy(d, pg, n, hipMemcpyHostToDevice)); });
        rate("H2D pinned (hipMemcpy)", [&] { CK(hipMemcpy(d, pin, n, hipMemcpyHostToDevice)); });
        rate("D2H pageable (hipMemcpy)", [&] { CK(hipMemcpy(pg2, d, n, hipMemcpyDeviceToHost)); });
        rate("D2H pinned (hipMemcpy)", [&] { CK(hipMemcpy(pin, d, n, hipMemcpyDeviceToHost)); });
        rate("hipHostRegister + H2D + Unregister", [&] {
            CK(hipHostRegister(pg, n, hipHostRegisterDefault));
            CK(hipMemcpy(d, pg, n, hipMemcpyHostToDevice));
            CK(hipHostUnregister(pg));
        });
        rate("hipHostRegister + Unregister only", [&] {
            CK(hipHostRegister(pg, n, hipHostRegisterDefault));
            CK(hipHostUnregister(pg));
        });
        // registration of memory never registered before (a caller's fresh buffer)
        {
            double tr = 0, tu = 0;
            for (int r = 0; r < 3; r++) {
                char *f = static_cast<char *>(aligned_alloc(4096, n));
                memset(f, 5, n);
                double t = now();
                CK(hipHostRegister(f, n, hipHostRegisterDefault));
                tr += now() - t;
                t = now();
                CK(hipMemcpy(d, f, n, hipMemcpyHostToDevice));
                double tc = now() - t;
                t = now();
                CK(hipHostUnregister(f));
                tu += now() - t;
                printf("{\"bytes\": %zu, \"what\": \"fresh register / H2D after it\", \"register_ms\": %.3f, \"h2d_GB_s\": %.2f}\n", n, 0.0 + tr * 1e3 / (r + 1), n / tc / 1e9);
                free(f);
            }
            printf("{\"bytes\": %zu, \"what\": \"fresh register avg\", \"register_ms\": %.3f, \"unregister_ms\": %.3f}\n", n, tr / 3 * 1e3, tu / 3 * 1e3);
        }
        // fresh pageable buffer straight through hipMemcpy (no reuse of a buffer HIP has seen)
        {
            char *f = static_cast<char *>(aligned_alloc(4096, n));
            memset(f, 6, n);
            double t = now();
            CK(hipMemcpy(d, f, n, hipMemcpyHostToDevice));
            double tc = now() - t;
            printf("{\"bytes\": %zu, \"what\": \"H2D fresh pageable (first use)\", \"ms\": %.3f, \"GB_s\": %.2f}\n", n, tc * 1e3, n / tc / 1e9);
            free(f);
        }
        // full duplex: pinned H2D and D2H at once on two streams
        {
            char *pin2;
            void *d2;
            CK(hipHostMalloc(reinterpret_cast<void **>(&pin2), n, hipHostMallocDefault));
            CK(hipMalloc(&d2, n));
            hipStream_t a, b;
            CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
            CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
            rate("duplex pinned H2D || D2H (bytes each way)", [&] {
                CK(hipMemcpyAsync(d, pin, n, hipMemcpyHostToDevice, a));
                CK(hipMemcpyAsync(pin2, d2, n, hipMemcpyDeviceToHost, b));
                CK(hipStreamSynchronize(a));
                CK(hipStreamSynchronize(b));
            });
            rate("chunked pinned H2D 8 MiB pieces on one stream", [&] {
                for (size_t o = 0; o < n; o += 8 << 20)
                    CK(hipMemcpyAsync(static_cast<char *>(d) + o, pin + o, std::min(n - o, size_t(8) << 20), hipMemcpyHostToDevice, a));
                CK(hipStreamSynchronize(a));
            });
            rate("pageable hipMemcpyAsync H2D, 8 MiB pieces, host time to enqueue+sync", [&] {
                for (size_t o = 0; o < n; o += 8 << 20)
                    CK(hipMemcpyAsync(static_cast<char *>(d) + o, pg + o, std::min(n - o, size_t(8) << 20), hipMemcpyHostToDevice, a));
                CK(hipStreamSynchronize(a));
            });
            {
                double t = now();
                for (size_t o = 0; o < n; o += 8 << 20)
                    CK(hipMemcpyAsync(static_cast<char *>(d) + o, pg + o, std::min(n - o, size_t(8) << 20), hipMemcpyHostToDevice, a));
                double te = now() - t;
                CK(hipStreamSynchronize(a));
                printf("{\"bytes\": %zu, \"what\": \"pageable async H2D: enqueue returns after\", \"ms\": %.3f, \"total_ms\": %.3f}\n", n, te * 1e3, (now() - t) * 1e3);
            }
            rate("duplex pageable H2D || D2H from two host threads", [&] {
                std::thread t1([&] { CK(hipMemcpyAsync(d, pg, n, hipMemcpyHostToDevice, a)); CK(hipStreamSynchronize(a)); });
                std::thread t2([&] { CK(hipMemcpyAsync(pg2, d2, n, hipMemcpyDeviceToHost, b)); CK(hipStreamSynchronize(b)); });
                t1.join();
                t2.join();
            });
            CK(hipStreamDestroy(a));
            CK(hipStreamDestroy(b));
            CK(hipFree(d2));
            CK(hipHostFree(pin2));
        }
        for (int th : {1, 2, 4, 8, 16}) {
            char name[64];
            snprintf(name, sizeof name, "memcpy pageable->pinned %d thr", th);
            rate(name, [&] { par_copy(pin, pg, n, th); });
        }
        for (int th : {1, 4, 8}) {
            char name[64];
            snprintf(name, sizeof name, "memcpy pinned->pageable %d thr", th);
            rate(name, [&] { par_copy(pg2, pin, n, th); });
        }
        CK(hipFree(d));
        CK(hipHostFree(pin));
        free(pg);
        free(pg2);
    }
    return 0;
}
