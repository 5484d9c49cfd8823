// Wave-level helpers for one-agent-per-wavefront kernels (gfx950, wave64, float64).
//
// A workgroup is exactly one 64-lane wavefront.  LDS instructions of one wave execute in issue
// order, so lanes of the wave exchange data through LDS without a hardware barrier: a phase
// boundary only needs the compiler not to move LDS accesses across it (wsync).
#pragma once
#include <hip/hip_runtime.h>

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
