// Wavefront reductions through cross-lane moves (gfx950): DPP quad_perm /
// row_half_mirror / row_mirror inside each 16-lane row, ds_swizzle (xor 16, no LDS
// storage) across the two rows of a 32-lane half, v_readlane for the two halves.
// No LDS buffer and no workgroup barrier per step; every lane of a pair combines the
// same two values, so all lanes agree after each step and the combination order is
// fixed: results are bit-identical run to run.  Used where a workgroup folds
// per-thread partials (channel mean, scanner window statistics, display autoscale).
#pragma once
#include <hip/hip_runtime.h>

namespace rfa {

__device__ __forceinline__ int dpp_i(int v, int ctrl_id) {
    switch (ctrl_id) {  // compile-time after inlining
    case 0: return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true);   // quad_perm [1,0,3,2]: lane ^ 1
    case 1: return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true);   // quad_perm [2,3,0,1]: lane ^ 2
    case 2: return __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, true);  // row_half_mirror: i <-> 7 - i
    case 3: return __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, true);  // row_mirror: i <-> 15 - i
    default: return __builtin_amdgcn_ds_swizzle(v, 0x401F);             // bitmask mode: lane ^ 16 (in 32)
    }
}
template <typename T>
__device__ __forceinline__ T xlane(T v, int ctrl_id) {
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "32- or 64-bit values");
    if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, dpp_i(__builtin_bit_cast(int, v), ctrl_id));
    } else {
        const long long b = __builtin_bit_cast(long long, v);
        const int lo = dpp_i((int)(b & 0xffffffffll), ctrl_id), hi = dpp_i((int)(b >> 32), ctrl_id);
        return __builtin_bit_cast(T, ((long long)hi << 32) | (unsigned)lo);
    }
}
template <typename T>
__device__ __forceinline__ T readlane_t(T v, int lane) {
    if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
    } else {
        const long long b = __builtin_bit_cast(long long, v);
        const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
        const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
        return __builtin_bit_cast(T, ((long long)hi << 32) | (unsigned)lo);
    }
}

// op over the 64 lanes of a wave (all lanes active); the result is wave-uniform.
template <typename T, typename Op>
__device__ __forceinline__ T wave_reduce(T x, Op op) {
#pragma unroll
    for (int c = 0; c < 5; c++) x = op(x, xlane(x, c));
    return op(readlane_t(x, 0), readlane_t(x, 32));
}

}  // namespace rfa
