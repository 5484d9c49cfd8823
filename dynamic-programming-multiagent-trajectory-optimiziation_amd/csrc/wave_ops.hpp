// Wave-level helpers for one-agent-per-wavefront kernels (gfx950, wave64, float64).
//
// A workgroup is exactly one 64-lane wavefront.  LDS instructions of one wave execute in issue
// order, so lanes of the wave exchange data through LDS without a hardware barrier: a phase
// boundary only needs the compiler not to move LDS accesses across it (wsync).
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif

namespace scvx {

constexpr int WAVE = 64;

// Phase boundary inside a one-wave workgroup: a compiler-level LDS fence (the LDS counter need
// not be drained: DS instructions of one wave are processed in order).
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// 64-bit DPP move (two 32-bit halves).  All 64 lanes must be active.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double readlane_d(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}

// Lane l (< 16) of this lane's 16-lane row, broadcast by a 64-bit DPP move (row_newbcast, gfx90a+):
// one VALU op with no SGPR round trip.  l must fold to a constant (unrolled loops).
template <int L>
__device__ __forceinline__ double row_bcast_c(double v) {
    static_assert(L >= 0 && L < 16, "row lane");
    return __builtin_amdgcn_mov_dpp(v, 0x150 + L, 0xF, 0xF, false);   // every lane written: no `old` to set up
}
__device__ __forceinline__ double row_bcast_d(double v, int l) {
    switch (l) {
        case 0: return row_bcast_c<0>(v);
        case 1: return row_bcast_c<1>(v);
        case 2: return row_bcast_c<2>(v);
        case 3: return row_bcast_c<3>(v);
        case 4: return row_bcast_c<4>(v);
        case 5: return row_bcast_c<5>(v);
        case 6: return row_bcast_c<6>(v);
        case 7: return row_bcast_c<7>(v);
        case 8: return row_bcast_c<8>(v);
        case 9: return row_bcast_c<9>(v);
        case 10: return row_bcast_c<10>(v);
        case 11: return row_bcast_c<11>(v);
        case 12: return row_bcast_c<12>(v);
        case 13: return row_bcast_c<13>(v);
        case 14: return row_bcast_c<14>(v);
        default: return row_bcast_c<15>(v);
    }
}

// Lane L (< 8) of this lane's 8-lane group (lanes 8g .. 8g+7), broadcast by two bank-masked 64-bit DPP
// row_newbcast moves: banks 0-1 of each 16-lane row (its lanes 0-7) take row lane L, banks 2-3 (lanes 8-15)
// take row lane 8 + L.  Eight independent groups exchange in two VALU ops.
template <int L>
__device__ __forceinline__ double oct_bcast_c(double v) {
    static_assert(L >= 0 && L < 8, "group lane");
    const double lo = __builtin_amdgcn_mov_dpp(v, 0x150 + L, 0xF, 0x3, false);
    return __builtin_amdgcn_update_dpp(lo, v, 0x158 + L, 0xF, 0xC, false);
}
__device__ __forceinline__ double oct_bcast_d(double v, int l) {
    switch (l) {
        case 0: return oct_bcast_c<0>(v);
        case 1: return oct_bcast_c<1>(v);
        case 2: return oct_bcast_c<2>(v);
        case 3: return oct_bcast_c<3>(v);
        case 4: return oct_bcast_c<4>(v);
        case 5: return oct_bcast_c<5>(v);
        case 6: return oct_bcast_c<6>(v);
        default: return oct_bcast_c<7>(v);
    }
}

// Reductions over the 64 lanes (result uniform): DPP inside each 16-lane row (quad xor 1, quad
// xor 2, half-row mirror, row mirror), then the four row results through readlane.
#define SCVX_WAVE_REDUCE(NAME, OP)                                     \
    __device__ __forceinline__ double NAME(double v) {                 \
        v = OP(v, dpp_d<0xB1>(v));  /* quad_perm [1,0,3,2] */          \
        v = OP(v, dpp_d<0x4E>(v));  /* quad_perm [2,3,0,1] */          \
        v = OP(v, dpp_d<0x141>(v)); /* row_half_mirror */              \
        v = OP(v, dpp_d<0x140>(v)); /* row_mirror */                   \
        return OP(OP(readlane_d(v, 0), readlane_d(v, 16)),             \
                  OP(readlane_d(v, 32), readlane_d(v, 48)));           \
    }
__device__ __forceinline__ double op_add(double a, double b) { return a + b; }
SCVX_WAVE_REDUCE(wave_sum, op_add)
SCVX_WAVE_REDUCE(wave_max, fmax)
SCVX_WAVE_REDUCE(wave_min, fmin)
#undef SCVX_WAVE_REDUCE

}  // namespace scvx
