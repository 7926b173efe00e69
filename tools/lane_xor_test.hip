// Device check of dbi::lane_xor<M> (dbindex_amd/csrc/dbi_lane.h) against
// __shfl_xor for every mask the bitonic networks use.  Build + run:
//   hipcc --offload-arch=gfx950 -O3 -I dbindex_amd/csrc tools/lane_xor_test.hip -o /tmp/lane_xor_test && /tmp/lane_xor_test
#include <cstdio>
#include "dbi_lane.h"

template <int M>
__device__ void check(uint32_t* bad, int slot) {
    const uint64_t v = 0x9E3779B97F4A7C15ull * (threadIdx.x + 1) ^ ((uint64_t)threadIdx.x << 40);
    const uint64_t want = __shfl_xor(v, M, 64);
    if (dbi::lane_xor64<M>(v) != want) atomicAdd(&bad[slot], 1u);
}

__global__ void k_test(uint32_t* bad) {
    check<1>(bad, 0); check<2>(bad, 1); check<3>(bad, 2); check<4>(bad, 3); check<7>(bad, 4); check<8>(bad, 5);
    check<15>(bad, 6); check<16>(bad, 7); check<31>(bad, 8); check<32>(bad, 9); check<63>(bad, 10);
}

int main() {
    uint32_t* d;
    const int masks[11] = {1, 2, 3, 4, 7, 8, 15, 16, 31, 32, 63};
    if (hipMalloc(&d, 4 * 11) != hipSuccess || hipMemset(d, 0, 4 * 11) != hipSuccess) return 2;
    hipLaunchKernelGGL(k_test, dim3(4), dim3(256), 0, 0, d);
    uint32_t h[11] = {};
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    int bad = 0;
    for (int i = 0; i < 11; ++i) {
        printf("lane ^ %2d: %u mismatches\n", masks[i], h[i]);
        bad += h[i] != 0;
    }
    return bad ? 1 : 0;
}
