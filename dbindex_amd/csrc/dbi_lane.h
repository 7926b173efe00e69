// Cross-lane exchange inside a wave64 without LDS: lane_xor<M>(v) returns v of
// lane (lane ^ M), from DPP row permutes (quad_perm, row_half_mirror,
// row_mirror, row_ror) and the gfx950 row swaps v_permlane16_swap /
// v_permlane32_swap -- a few VALU cycles instead of a ds_bpermute round trip.
// M: 1, 2, 3, 4, 7, 8, 15, 16, 31, 32, 63 (the lane masks of a bitonic
// network: half-cleaners j and flips k-1).  tools/lane_xor_test.hip checks
// every mask against __shfl_xor on the device.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace dbi {

template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}

constexpr int DPP_QUAD_1032 = 0xB1;   // quad_perm [1,0,3,2]: lane ^ 1
constexpr int DPP_QUAD_2301 = 0x4E;   // quad_perm [2,3,0,1]: lane ^ 2
constexpr int DPP_QUAD_3210 = 0x1B;   // quad_perm [3,2,1,0]: lane ^ 3
constexpr int DPP_ROW_ROR8 = 0x128;   // row_ror:8: lane ^ 8
constexpr int DPP_ROW_MIRROR = 0x140;       // lane ^ 15
constexpr int DPP_ROW_HALF_MIRROR = 0x141;  // lane ^ 7

// rows r and r ^ 1 (16 lanes each) exchanged
__device__ __forceinline__ uint32_t swap16(uint32_t v) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (__lane_id() & 16) ? r[0] : r[1];
}

// halves exchanged (lane ^ 32)
__device__ __forceinline__ uint32_t swap32(uint32_t v) {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (__lane_id() & 32) ? r[0] : r[1];
}

template <int M>
__device__ __forceinline__ uint32_t lane_xor(uint32_t v) {
    if constexpr (M == 1) return dpp32<DPP_QUAD_1032>(v);
    else if constexpr (M == 2) return dpp32<DPP_QUAD_2301>(v);
    else if constexpr (M == 3) return dpp32<DPP_QUAD_3210>(v);
    else if constexpr (M == 4) return dpp32<DPP_QUAD_3210>(dpp32<DPP_ROW_HALF_MIRROR>(v));  // 3 ^ 7
    else if constexpr (M == 7) return dpp32<DPP_ROW_HALF_MIRROR>(v);
    else if constexpr (M == 8) return dpp32<DPP_ROW_ROR8>(v);
    else if constexpr (M == 15) return dpp32<DPP_ROW_MIRROR>(v);
    else if constexpr (M == 16) return swap16(v);
    else if constexpr (M == 31) return swap16(dpp32<DPP_ROW_MIRROR>(v));
    else if constexpr (M == 32) return swap32(v);
    else if constexpr (M == 63) return swap32(swap16(dpp32<DPP_ROW_MIRROR>(v)));
    else {
        static_assert(M == 1, "lane_xor: unsupported mask");
        return v;
    }
}

template <int M>
__device__ __forceinline__ uint64_t lane_xor64(uint64_t v) {
    const uint32_t lo = lane_xor<M>((uint32_t)v), hi = lane_xor<M>((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

}  // namespace dbi
