// Open's setup costs, one at a time, in a fresh process (tools/setup_xp.sh):
// HIP's initialisation, gck_ctx_create x4, and 512 MiB of page-locked staging
// (16 x 32 MiB) by hipHostMalloc and by malloc + hipHostRegister, with and
// without huge pages.  Measurement aid, not product code.
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "gocask_hip.h"

static double ms(std::chrono::steady_clock::time_point a) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
}

int main(int argc, char **argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    const size_t chunk = 32ull << 20;
    const int nbuf = 16;
    auto t = std::chrono::steady_clock::now();
    size_t fr = 0, tot = 0;
    (void)hipMemGetInfo(&fr, &tot);
    printf("{\"mode\": %d, \"hip_init_ms\": %.2f", mode, ms(t));
    t = std::chrono::steady_clock::now();
    if (mode == 0) {  // contexts
        gck_ctx *c[4];
        for (int i = 0; i < 4; ++i) {
            auto t1 = std::chrono::steady_clock::now();
            if (gck_ctx_create(nullptr, &c[i])) return 1;
            printf(", \"ctx%d_ms\": %.2f", i, ms(t1));
        }
        printf(", \"ctx_total_ms\": %.2f", ms(t));
        for (auto *x : c) gck_ctx_destroy(x);
    } else if (mode == 1) {  // hipHostMalloc
        std::vector<void *> b(nbuf);
        for (auto &p : b)
            if (hipHostMalloc(&p, chunk, hipHostMallocDefault) != hipSuccess) return 1;
        printf(", \"hostmalloc_ms\": %.2f", ms(t));
    } else if (mode == 2 || mode == 3) {  // malloc (+ huge pages) + touch + register
        std::vector<void *> b(nbuf);
        for (auto &p : b) {
            p = aligned_alloc(2u << 20, chunk);
            if (mode == 3) (void)madvise(p, chunk, MADV_HUGEPAGE);
            memset(p, 0, chunk);
        }
        const double touch = ms(t);
        auto t1 = std::chrono::steady_clock::now();
        for (auto &p : b)
            if (hipHostRegister(p, chunk, hipHostRegisterDefault) != hipSuccess) return 1;
        printf(", \"touch_ms\": %.2f, \"register_ms\": %.2f, \"huge\": %d", touch, ms(t1), mode == 3);
    } else if (mode == 4) {  // hipHostMalloc on 4 threads
        std::vector<void *> b(nbuf);
        std::vector<std::thread> th;
        for (int k = 0; k < 4; ++k)
            th.emplace_back([&, k] {
                for (int i = k; i < nbuf; i += 4) (void)hipHostMalloc(&b[i], chunk, hipHostMallocDefault);
            });
        for (auto &x : th) x.join();
        printf(", \"hostmalloc_4threads_ms\": %.2f", ms(t));
    } else if (mode == 6) {  // gck_ctx_create's HIP calls one by one, then the context itself
        auto step = [&](const char *name) {
            printf(", \"%s_ms\": %.2f", name, ms(t));
            t = std::chrono::steady_clock::now();
        };
        hipDeviceProp_t prop;
        (void)hipGetDeviceProperties(&prop, 0);
        step("props");
        hipStream_t s;
        (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
        step("stream");
        hipEvent_t ev[16];
        for (auto &e : ev) (void)hipEventCreate(&e);
        step("events");
        void *d = nullptr, *h = nullptr;
        (void)hipMalloc(&d, 1 << 20);
        step("malloc");
        std::vector<char> src(1 << 16, 1);
        (void)hipMemcpy(d, src.data(), src.size(), hipMemcpyHostToDevice);
        step("memcpy");
        (void)hipHostMalloc(&h, 128, hipHostMallocMapped | hipHostMallocCoherent);
        step("hostmalloc128");
        (void)hipMemsetAsync(d, 0, 1 << 20, s);
        (void)hipStreamSynchronize(s);
        step("memset");
        gck_ctx *c = nullptr;
        if (gck_ctx_create(nullptr, &c)) return 1;
        step("ctx_after");
        gck_ctx_destroy(c);
    } else if (mode == 5) {  // contexts and staging together, as Open does
        std::vector<void *> b(nbuf);
        std::thread pre([&] {
            for (auto &p : b) (void)hipHostMalloc(&p, chunk, hipHostMallocDefault);
        });
        gck_ctx *c[4];
        for (int i = 0; i < 4; ++i)
            if (gck_ctx_create(nullptr, &c[i])) return 1;
        printf(", \"ctx_ms\": %.2f", ms(t));
        pre.join();
        printf(", \"both_ms\": %.2f", ms(t));
    }
    printf("}\n");
    return 0;
}
