// Copy-kernel shapes for dbi_hbm_copy_bandwidth (the measured HBM ceiling the
// bench prints): grid-stride vs one-shot blocks, default vs nontemporal.
// Build: hipcc --offload-arch=gfx950 -O3 tools/copy_probe.hip -o tools/copy_probe.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void __launch_bounds__(256) grid_stride(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const uint4 a = in[i], b = in[i + stride], c = in[i + 2 * stride], d = in[i + 3 * stride];
        out[i] = a; out[i + stride] = b; out[i + 2 * stride] = c; out[i + 3 * stride] = d;
    }
    for (; i < n; i += stride) out[i] = in[i];
}

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ void __launch_bounds__(256) one_shot(const v4u* __restrict__ in, v4u* __restrict__ out, uint64_t n) {
    const uint64_t base = (uint64_t)blockIdx.x * 256u * U + threadIdx.x;
    v4u v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const uint64_t i = base + (uint64_t)k * 256u;
        if (i < n) v[k] = NT ? __builtin_nontemporal_load(in + i) : in[i];
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const uint64_t i = base + (uint64_t)k * 256u;
        if (i < n) {
            if (NT) __builtin_nontemporal_store(v[k], out + i);
            else out[i] = v[k];
        }
    }
}

template <typename F>
static void timeit(const char* name, F launch, uint64_t n16) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    launch();
    hipEventRecord(e0);
    const int reps = 10;
    for (int r = 0; r < reps; ++r) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-24s %8.1f GB/s\n", name, 2.0 * 16.0 * n16 * reps / (ms * 1e-3) / 1e9);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main() {
    const uint64_t bytes = 1ull << 31, n16 = bytes / 16;
    uint4 *a, *b;
    if (hipMalloc(&a, bytes) || hipMalloc(&b, bytes)) return 1;
    hipMemset(a, 1, bytes);
    hipMemset(b, 2, bytes);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (int per : {4, 8, 16, 32}) {
        char nm[64];
        snprintf(nm, sizeof nm, "grid_stride x%d/CU", per);
        timeit(nm, [&] { grid_stride<<<cus * per, 256>>>(a, b, n16); }, n16);
    }
    timeit("one_shot U4", [&] { one_shot<4, false><<<(n16 + 1023) / 1024, 256>>>((const v4u*)a, (v4u*)b, n16); }, n16);
    timeit("one_shot U8", [&] { one_shot<8, false><<<(n16 + 2047) / 2048, 256>>>((const v4u*)a, (v4u*)b, n16); }, n16);
    timeit("one_shot U4 nt", [&] { one_shot<4, true><<<(n16 + 1023) / 1024, 256>>>((const v4u*)a, (v4u*)b, n16); }, n16);
    timeit("one_shot U8 nt", [&] { one_shot<8, true><<<(n16 + 2047) / 2048, 256>>>((const v4u*)a, (v4u*)b, n16); }, n16);
    timeit("one_shot U2", [&] { one_shot<2, false><<<(n16 + 511) / 512, 256>>>((const v4u*)a, (v4u*)b, n16); }, n16);
    timeit("hipMemcpyAsync d2d", [&] { hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0); }, n16);
    hipDeviceSynchronize();
    hipFree(a);
    hipFree(b);
    return 0;
}
