// Micro-benchmark (diagnostics only; round-6 verdict item: FP64 MFMA for the n = 12 Riccati stage products).
// A dependent chain M <- A' M of 12 x 12 FP64 products -- the shape and dependency of the n = 12 factor's
// T1 = P'A / W1 = A'Pi' / Qh = Q + A'T1 phases, one product per stage on the sweep's critical path -- in one wave per
// SIMD with every SIMD of the chip busy (1024 workgroups of 64, as the C5 QP launch), timed with s_memtime:
//   valu: the QP kernel's pattern -- 144 outputs over 64 lanes (3 repetitions), each a 12-term dot product of two
//         contiguous LDS vectors, written back to LDS, wave barrier;
//   mfma: v_mfma_f64_16x16x4f64 on zero-padded 16 x 16 tiles -- 3 MFMAs (K = 12 in steps of 4), operands one
//         ds_read_b64 each per lane, 4 results per lane written back to LDS, wave barrier.
// Both produce the same product (checked on the host against a CPU reference).
// build: hipcc -O3 --offload-arch=gfx950 tools/ubench/mfma_stage.hip -o tools/ubench/mfma_stage
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

typedef double v4d __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// LDS: At row-major 16 x 16 (At[i][k] = A[k][i], zero padded), M[2] row-major 16 x 16 (ping-pong)
__global__ __launch_bounds__(64) void k_valu(const double* A, const double* M0, double* out, long long* cyc, int n) {
    __shared__ double At[256], M[2][256];
    const int l = threadIdx.x;
    for (int e = l; e < 256; e += 64) { At[e] = A[e]; M[0][e] = M0[e]; M[1][e] = 0.0; }
    __syncthreads();
    // a column-major copy of M makes every dot product two contiguous vectors (the QP kernel's packet layout)
    __shared__ double Mcm[2][256];
    for (int e = l; e < 256; e += 64) { Mcm[0][e] = M[0][(e % 16) * 16 + e / 16]; Mcm[1][e] = 0.0; }
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < n; ++s) {
        const double* src = Mcm[s & 1];
        double* dst = Mcm[(s + 1) & 1];
        double v[3];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const int o = l + 64 * r, oo = o < 144 ? o : 0, i = oo / 12, j = oo % 12;
            const double* a = At + i * 16;    // row i of A' (row-major At: contiguous)
            const double* b = src + j * 16;   // column j of M (column-major copy: contiguous)
            double a0 = 0.0, a1 = 0.0;
#pragma unroll
            for (int k = 0; k < 12; ++k) { if (k & 1) a1 = fma(a[k], b[k], a1); else a0 = fma(a[k], b[k], a0); }
            v[r] = a0 + a1;
        }
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const int o = l + 64 * r, oo = o < 144 ? o : 0, i = oo / 12, j = oo % 12;
            dst[o < 144 ? j * 16 + i : 255] = v[r] * 0.25;
        }
        wsync();
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    for (int e = l; e < 256; e += 64) out[blockIdx.x * 256 + e] = Mcm[n & 1][(e % 16) * 16 + e / 16];
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(64) void k_mfma(const double* A, const double* M0, double* out, long long* cyc, int n) {
    __shared__ double At[256], M[2][256];
    const int l = threadIdx.x;
    for (int e = l; e < 256; e += 64) { At[e] = A[e]; M[0][e] = M0[e]; M[1][e] = 0.0; }
    __syncthreads();
    const int r16 = l & 15, q = l >> 4;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < n; ++s) {
        const double* src = M[s & 1];
        double* dst = M[(s + 1) & 1];
        v4d c = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kk = 0; kk < 3; ++kk) {
            const double a = At[r16 * 16 + 4 * kk + q];     // A' (16 x K): row r16, k = 4 kk + q
            const double b = src[(4 * kk + q) * 16 + r16];  // M (K x 16): row k, column r16
            c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) dst[(q + 4 * r) * 16 + r16] = c[r] * 0.25;   // D: row q + 4 r, column r16
        wsync();
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    for (int e = l; e < 256; e += 64) out[blockIdx.x * 256 + e] = M[n & 1][e];
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

static void cpu_ref(const std::vector<double>& A, std::vector<double> R, int n, std::vector<double>& out) {
    std::vector<double> T(256);
    for (int s = 0; s < n; ++s) {
        for (int i = 0; i < 16; ++i)
            for (int j = 0; j < 16; ++j) {
                double v = 0.0;
                for (int k = 0; k < 12; ++k) v += A[i * 16 + k] * R[k * 16 + j];
                T[i * 16 + j] = (i < 12 && j < 12) ? 0.25 * v : 0.0;
            }
        R = T;
    }
    out = R;
}

int main() {
    const int G = 1024;
    std::vector<double> A(256, 0.0), M0(256, 0.0);
    for (int k = 0; k < 12; ++k)
        for (int i = 0; i < 12; ++i) {
            A[i * 16 + k] = std::sin(1.0 + i + 3.0 * k) * 0.5 + (i == k ? 1.0 : 0.0);   // At[i][k] = A[k][i]
            M0[k * 16 + i] = std::cos(0.3 * i + k);
        }
    double *dA, *dM, *dO;
    long long* dC;
    hipMalloc(&dA, 256 * 8); hipMalloc(&dM, 256 * 8); hipMalloc(&dO, (size_t)G * 256 * 8); hipMalloc(&dC, G * 8);
    hipMemcpy(dA, A.data(), 256 * 8, hipMemcpyHostToDevice);
    hipMemcpy(dM, M0.data(), 256 * 8, hipMemcpyHostToDevice);
    std::vector<double> O((size_t)G * 256), R;
    std::vector<long long> C(G);
    for (int rep = 0; rep < 3; ++rep)
        for (int v = 0; v < 2; ++v)
            for (int n : {6, 2000}) {
                if (v == 0) hipLaunchKernelGGL(k_valu, dim3(G), dim3(64), 0, 0, dA, dM, dO, dC, n);
                else hipLaunchKernelGGL(k_mfma, dim3(G), dim3(64), 0, 0, dA, dM, dO, dC, n);
                hipDeviceSynchronize();
                hipMemcpy(O.data(), dO, O.size() * 8, hipMemcpyDeviceToHost);
                hipMemcpy(C.data(), dC, G * 8, hipMemcpyDeviceToHost);
                if (n == 6) {
                    cpu_ref(A, M0, n, R);
                    double err = 0.0, ref = 0.0;
                    for (int e = 0; e < 256; ++e) {   // the 12 x 12 block (the VALU form parks its idle lanes' stores in (15, 15))
                        if (e / 16 >= 12 || e % 16 >= 12) continue;
                        err = std::fmax(err, std::fabs(O[e] - R[e]));
                        ref = std::fmax(ref, std::fabs(R[e]));
                    }
                    printf("%s: 6 chained products, max |err| %.2e of max |M| %.2e\n", v ? "mfma" : "valu", err, ref);
                    continue;
                }
                double cs = 0.0;
                for (long long c : C) cs += (double)c;
                printf("%s: %.1f cycles per 12x12 product (mean over %d waves, %d chained products)\n", v ? "mfma" : "valu",
                       cs / G / n, G, n);
            }
    return 0;
}
