// h2d_probe: host-to-device copy paths for the end-to-end build's residues
// (DESIGN.md §7): pageable hipMemcpy, hipHostMalloc'ed (pinned) source, a
// hipHostRegister'ed malloc buffer, and a memchr scan, each timed on the host.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 201309633ull;
    void* d = nullptr;
    double t = now_ms();
    CK(hipMalloc(&d, n));
    std::printf("hipMalloc %zu B: %.2f ms\n", n, now_ms() - t);
    std::vector<uint8_t> pg(n);
    for (size_t i = 0; i < n; ++i) pg[i] = (uint8_t)('A' + i % 20);
    for (int r = 0; r < 3; ++r) {
        t = now_ms();
        CK(hipMemcpy(d, pg.data(), n, hipMemcpyHostToDevice));
        const double ms = now_ms() - t;
        std::printf("pageable hipMemcpy: %.2f ms (%.1f GB/s)\n", ms, n / ms / 1e6);
    }
    t = now_ms();
    const void* q = std::memchr(pg.data(), '[', n);
    std::printf("memchr one thread: %.2f ms (%p)\n", now_ms() - t, q);
    for (int r = 0; r < 2; ++r) {
        void* hp = nullptr;
        t = now_ms();
        CK(hipHostMalloc(&hp, n, hipHostMallocDefault));
        const double ta = now_ms() - t;
        t = now_ms();
        std::memcpy(hp, pg.data(), n);
        const double tc = now_ms() - t;
        t = now_ms();
        CK(hipMemcpy(d, hp, n, hipMemcpyHostToDevice));
        const double ms = now_ms() - t;
        t = now_ms();
        CK(hipHostFree(hp));
        std::printf("hipHostMalloc %.2f ms, first touch memcpy %.2f ms, pinned hipMemcpy %.2f ms (%.1f GB/s), free %.2f ms\n",
                    ta, tc, ms, n / ms / 1e6, now_ms() - t);
    }
    for (int r = 0; r < 2; ++r) {
        uint8_t* m = (uint8_t*)std::malloc(n);
        std::memcpy(m, pg.data(), n);
        t = now_ms();
        CK(hipHostRegister(m, n, hipHostRegisterDefault));
        const double tr = now_ms() - t;
        t = now_ms();
        CK(hipMemcpy(d, m, n, hipMemcpyHostToDevice));
        const double ms = now_ms() - t;
        t = now_ms();
        CK(hipHostUnregister(m));
        std::printf("hipHostRegister %.2f ms, registered hipMemcpy %.2f ms (%.1f GB/s), unregister %.2f ms\n", tr, ms,
                    n / ms / 1e6, now_ms() - t);
        std::free(m);
    }
    // device allocation cost by size (the one-off build's buffers), hipMalloc vs the stream-ordered pool
    {
        const size_t sizes[] = {1u << 20, 64u << 20, 512u << 20, 1024ull << 20, 4096ull << 20};
        for (size_t sz : sizes) {
            void* p[3];
            double ta = 0, tf = 0;
            for (int k = 0; k < 3; ++k) {
                t = now_ms();
                CK(hipMalloc(&p[k], sz));
                ta += now_ms() - t;
            }
            for (int k = 0; k < 3; ++k) {
                t = now_ms();
                CK(hipFree(p[k]));
                tf += now_ms() - t;
            }
            std::printf("hipMalloc %zu MiB: %.3f ms, hipFree %.3f ms (avg of 3)\n", sz >> 20, ta / 3, tf / 3);
        }
        hipStream_t s2;
        CK(hipStreamCreate(&s2));
        for (int r = 0; r < 2; ++r) {
            void* q[4];
            t = now_ms();
            for (int k = 0; k < 4; ++k) CK(hipMallocAsync(&q[k], 1024ull << 20, s2));
            CK(hipStreamSynchronize(s2));
            const double ta = now_ms() - t;
            t = now_ms();
            for (int k = 0; k < 4; ++k) CK(hipFreeAsync(q[k], s2));
            CK(hipStreamSynchronize(s2));
            std::printf("hipMallocAsync 4 x 1 GiB (round %d): %.3f ms, hipFreeAsync %.3f ms\n", r, ta, now_ms() - t);
        }
        t = now_ms();
        hipStream_t s3;
        CK(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));
        std::printf("hipStreamCreate: %.3f ms\n", now_ms() - t);
        t = now_ms();
        hipEvent_t evs[96];
        for (auto& e : evs) CK(hipEventCreate(&e));
        std::printf("96 x hipEventCreate: %.3f ms\n", now_ms() - t);
    }
    // pinned staging ring: 4 MiB chunks, 16 threads memcpy into two pinned halves
    {
        const size_t C = 8u << 20;
        void* st[2];
        CK(hipHostMalloc(&st[0], C, hipHostMallocDefault));
        CK(hipHostMalloc(&st[1], C, hipHostMallocDefault));
        hipStream_t s;
        CK(hipStreamCreate(&s));
        hipEvent_t ev[2];
        CK(hipEventCreate(&ev[0]));
        CK(hipEventCreate(&ev[1]));
        for (int r = 0; r < 3; ++r) {
            t = now_ms();
            for (size_t o = 0, k = 0; o < n; o += C, ++k) {
                const size_t b = k & 1, len = std::min(C, n - o);
                if (k >= 2) CK(hipEventSynchronize(ev[b]));
                const int T = 8;
                std::vector<std::thread> th;
                for (int i = 0; i < T; ++i)
                    th.emplace_back([&, i] {
                        const size_t a = len * i / T, e = len * (i + 1) / T;
                        std::memcpy((uint8_t*)st[b] + a, pg.data() + o + a, e - a);
                    });
                for (auto& x : th) x.join();
                CK(hipMemcpyAsync((uint8_t*)d + o, st[b], len, hipMemcpyHostToDevice, s));
                CK(hipEventRecord(ev[b], s));
            }
            CK(hipStreamSynchronize(s));
            const double ms = now_ms() - t;
            std::printf("staged ring (8 MiB x 2, 8 memcpy threads): %.2f ms (%.1f GB/s)\n", ms, n / ms / 1e6);
        }
    }
    return 0;
}
