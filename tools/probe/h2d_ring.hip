// h2d_ring: the end-to-end build's residue upload (dbi_engine.hip
// upload_residues) by variant, each from a FRESH host buffer (malloc'ed and
// written untimed, as the FASTA parser leaves its output): pageable hipMemcpy,
// pageable async pieces, and staged rings of pinned slots (slice size x host
// threads x DMA streams).  Times on the host; the ring's registration apart.
#include <hip/hip_runtime.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sys/mman.h>
#include <thread>
#include <vector>

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

static uint8_t* fresh(size_t n, bool huge = false) {
    uint8_t* p = nullptr;
    if (huge) {  // as the FASTA parser allocates its output (alloc_big)
        void* q = nullptr;
        if (posix_memalign(&q, 2u << 20, n)) std::exit(1);
        madvise(q, (n + (2u << 20) - 1) & ~size_t((2u << 20) - 1), MADV_HUGEPAGE);
        p = (uint8_t*)q;
    } else {
        p = (uint8_t*)std::malloc(n);
    }
    std::vector<std::thread> th;
    for (int t = 0; t < 16; ++t)
        th.emplace_back([=] {
            for (size_t i = n * t / 16; i < n * (t + 1) / 16; ++i) p[i] = (uint8_t)('A' + i % 20);
        });
    for (auto& x : th) x.join();
    return p;
}

struct Ring {
    uint8_t* host = nullptr;
    size_t slice = 0;
    int threads = 0, nstreams = 0;
    std::vector<hipEvent_t> ev;
    std::vector<hipStream_t> st;
    double reg_ms = 0;
    Ring(size_t sl, int T, int S) : slice(sl), threads(T), nstreams(S) {
        const size_t bytes = sl * 2 * T;
        void* p = nullptr;
        if (posix_memalign(&p, 2u << 20, bytes)) std::exit(1);
        madvise(p, bytes, MADV_HUGEPAGE);
        const double t = now_ms();
        CK(hipHostRegister(p, bytes, hipHostRegisterDefault));
        reg_ms = now_ms() - t;
        host = (uint8_t*)p;
        ev.resize(2 * T);
        for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        st.resize(S);
        for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    }
    void upload(uint8_t* d, const uint8_t* src, size_t n) {
        const size_t ns = (n + slice - 1) / slice;
        auto work = [&](int t) {
            uint32_t k = 0;
            for (size_t c = t; c < ns; c += threads, ++k) {
                const int slot = 2 * t + (int)(k & 1u);
                uint8_t* sp = host + slice * slot;
                const size_t a = c * slice, len = std::min(slice, n - a);
                if (k >= 2) CK(hipEventSynchronize(ev[slot]));
                std::memcpy(sp, src + a, len);
                hipStream_t s = st[t % nstreams];
                CK(hipMemcpyAsync(d + a, sp, len, hipMemcpyHostToDevice, s));
                CK(hipEventRecord(ev[slot], s));
            }
        };
        std::vector<std::thread> th;
        for (int t = 1; t < threads; ++t) th.emplace_back(work, t);
        work(0);
        for (auto& x : th) x.join();
        for (auto s : st) CK(hipStreamSynchronize(s));
    }
};

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 201309633ull;
    uint8_t* d = nullptr;
    CK(hipMalloc((void**)&d, n));
    {   // warm the runtime's pageable path once (the e2e process has copied before)
        uint8_t* w = fresh(64u << 20);
        double t = now_ms();
        CK(hipMemcpy(d, w, 64u << 20, hipMemcpyHostToDevice));
        std::printf("warm-up pageable 64 MiB: %.2f ms\n", now_ms() - t);
        std::free(w);
    }
    for (int r = 0; r < 2; ++r) {
        uint8_t* p = fresh(n);
        double t = now_ms();
        CK(hipMemcpy(d, p, n, hipMemcpyHostToDevice));
        double ms = now_ms() - t;
        std::printf("pageable hipMemcpy, fresh buffer: %.2f ms (%.1f GB/s)\n", ms, n / ms / 1e6);
        t = now_ms();
        CK(hipMemcpy(d, p, n, hipMemcpyHostToDevice));
        ms = now_ms() - t;
        std::printf("pageable hipMemcpy, same buffer again: %.2f ms (%.1f GB/s)\n", ms, n / ms / 1e6);
        std::free(p);
    }
    // the caller's buffer registered in page-aligned chunks by T threads in
    // parallel, each chunk's DMA queued as soon as it is registered
    for (int huge = 0; huge < 2; ++huge)
    for (int T : {1, 4, 8, 16}) {
        for (size_t chunk : {size_t(8) << 20, size_t(32) << 20}) {
            hipStream_t s;
            CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            double best = 1e30, first = 0, reg_sum = 0;
            for (int r = 0; r < 3; ++r) {
                uint8_t* p = fresh(n, huge);
                const uintptr_t base = (uintptr_t)p & ~uintptr_t(4095);
                const size_t span = ((uintptr_t)p + n + 4095 - base) & ~size_t(4095);
                const size_t nc = (span + chunk - 1) / chunk;
                std::atomic<double> regt{0};
                const double t = now_ms();
                std::vector<std::thread> th;
                for (int k = 0; k < T; ++k)
                    th.emplace_back([&, k] {
                        for (size_t c = k; c < nc; c += T) {
                            uint8_t* a = (uint8_t*)(base + c * chunk);
                            const size_t len = std::min(chunk, span - c * chunk);
                            const double t0 = now_ms();
                            CK(hipHostRegister(a, len, hipHostRegisterDefault));
                            double old = regt.load();
                            while (!regt.compare_exchange_weak(old, old + now_ms() - t0)) {}
                            // the residues inside this chunk
                            const uint8_t* lo = std::max((const uint8_t*)a, (const uint8_t*)p);
                            const uint8_t* hi = std::min((const uint8_t*)a + len, (const uint8_t*)p + n);
                            if (hi > lo) CK(hipMemcpyAsync(d + (lo - p), lo, hi - lo, hipMemcpyHostToDevice, s));
                        }
                    });
                for (auto& x : th) x.join();
                CK(hipStreamSynchronize(s));
                const double ms = now_ms() - t;
                for (size_t c = 0; c < nc; ++c) CK(hipHostUnregister((void*)(base + c * chunk)));
                if (r == 0) first = ms;
                best = std::min(best, ms);
                reg_sum += regt.load();
                std::free(p);
            }
            std::printf("register caller buffer (%s pages): %zu MiB chunks x %d threads: first %.2f ms, best %.2f ms (%.1f GB/s), "
                        "registration %.2f ms of thread time per run\n", huge ? "2 MiB" : "4 KiB", chunk >> 20, T, first, best, n / best / 1e6, reg_sum / 3);
        }
    }
    struct V { size_t slice; int T, S; };
    const V vs[] = {{1u << 20, 8, 1}, {1u << 20, 8, 2}, {2u << 20, 8, 1}, {2u << 20, 8, 2}, {4u << 20, 8, 1},
                    {4u << 20, 8, 2}, {4u << 20, 4, 2}, {2u << 20, 16, 2}, {8u << 20, 4, 2}, {2u << 20, 8, 4}};
    for (const V& v : vs) {
        Ring ring(v.slice, v.T, v.S);
        double best = 1e30, first = 0;
        for (int r = 0; r < 3; ++r) {
            uint8_t* p = fresh(n);
            const double t = now_ms();
            ring.upload(d, p, n);
            const double ms = now_ms() - t;
            if (r == 0) first = ms;
            best = std::min(best, ms);
            std::free(p);
        }
        std::printf("ring %zu MiB x %d threads x %d streams (%zu MiB pinned, register %.2f ms): first %.2f ms, best %.2f ms "
                    "(%.1f GB/s)\n", v.slice >> 20, v.T, v.S, (v.slice * 2 * v.T) >> 20, ring.reg_ms, first, best,
                    n / best / 1e6);
    }
    return 0;
}
