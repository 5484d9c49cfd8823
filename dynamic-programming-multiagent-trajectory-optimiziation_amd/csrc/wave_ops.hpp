// Wave-level helpers for one-agent-per-wavefront kernels (gfx950, wave64, float64).
//
// A workgroup is exactly one 64-lane wavefront, so __syncthreads() is a cheap s_barrier that
// also orders LDS and global traffic between the lanes of the wave.  Small dense matrices
// (<= 16x16) live in LDS row-major; element-parallel ops give every lane one (or a few) output
// elements.
#pragma once
#include <hip/hip_runtime.h>

namespace scvx {

constexpr int WAVE = 64;

// LDS-only barrier for a one-wavefront workgroup.  __syncthreads() emits s_waitcnt vmcnt(0)
// (it fences global memory too), which would drain every prefetch load and every store in flight
// at each phase of a sequential sweep.  Lanes of one wave exchange data through LDS in issue
// order, so a phase boundary only needs the LDS counter drained plus a compiler barrier.
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0) only (vmcnt, expcnt left at max)
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, WAVE));
    return v;
}
__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, WAVE));
    return v;
}

// out[i][j] (R x C) = (add ? add[i][j] : 0) + alpha * sum_k op(A)[i][k] op(B)[k][j]
// op(A) is R x KK: TA ? A stored KK x R : A stored R x KK.  op(B) is KK x C similarly.
template <int R, int C, int KK, bool TA, bool TB>
__device__ __forceinline__ void mm(double* __restrict__ out, const double* __restrict__ A,
                                   const double* __restrict__ B, const double* add, double alpha, int lane) {
    for (int e = lane; e < R * C; e += WAVE) {
        const int i = e / C, j = e % C;
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < KK; ++k) {
            const double a = TA ? A[k * R + i] : A[i * KK + k];
            const double b = TB ? B[j * KK + k] : B[k * C + j];
            acc = fma(a, b, acc);
        }
        out[e] = (add ? add[e] : 0.0) + alpha * acc;
    }
}

// y (R) = (add ? add : 0) + alpha * op(A) x,   op(A) R x C
template <int R, int C, bool TA>
__device__ __forceinline__ void mv(double* __restrict__ y, const double* __restrict__ A, const double* __restrict__ x,
                                   const double* add, double alpha, int lane) {
    if (lane < R) {
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < C; ++k) acc = fma(TA ? A[k * R + lane] : A[lane * C + k], x[k], acc);
        y[lane] = (add ? add[lane] : 0.0) + alpha * acc;
    }
}

}  // namespace scvx
