// Micro-benchmarks (diagnostics only): latencies of the primitives the QP chain steps use, one
// wave per SIMD, measured with s_memtime inside the kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ double rl(double v, int l) {
    int lo = __builtin_amdgcn_readlane(__double2loint(v), l), hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}

__global__ __launch_bounds__(64) void k_chain_rl(double* out, long long* cyc, int n, const double* A) {
    const int lane = threadIdx.x;
    double a[6];
    for (int k = 0; k < 6; ++k) a[k] = A[lane * 6 + k] * 0.1;
    double p = lane < 6 ? 1.0 + lane : 0.0;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < n; ++s) {
        double v0 = 0.5, v1 = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k) { double pk = rl(p, k); if (k & 1) v1 = fma(a[k], pk, v1); else v0 = fma(a[k], pk, v0); }
        p = v0 + v1;
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + lane] = p;
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(64) void k_chain_lds(double* out, long long* cyc, int n, const double* A) {
    __shared__ double x[2][8];
    const int lane = threadIdx.x;
    double a[6];
    for (int k = 0; k < 6; ++k) a[k] = A[lane * 6 + k] * 0.1;
    if (lane < 8) x[0][lane] = 1.0 + lane;
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < n; ++s) {
        const double* xs = x[s & 1];
        double v0 = 0.5, v1 = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k) { double pk = xs[k]; if (k & 1) v1 = fma(a[k], pk, v1); else v0 = fma(a[k], pk, v0); }
        if (lane < 6) x[(s + 1) & 1][lane] = v0 + v1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + lane] = x[n & 1][lane & 7];
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

// dependent FP64 FMA chain
__global__ __launch_bounds__(64) void k_fma(double* out, long long* cyc, int n, const double* A) {
    double v = A[threadIdx.x], a = A[threadIdx.x + 64];
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < n; ++s) {
#pragma unroll
        for (int k = 0; k < 16; ++k) v = fma(v, a, 0.25);
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = v;
    if (threadIdx.x == 0) cyc[blockIdx.x] = (t1 - t0);
}

// dependent LDS load chain (pointer chasing)
__global__ __launch_bounds__(64) void k_lds(double* out, long long* cyc, int n, const double* A) {
    __shared__ int nx[64];
    nx[threadIdx.x] = (threadIdx.x + 1) & 63;
    __syncthreads();
    int p = threadIdx.x;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < n; ++s) {
#pragma unroll
        for (int k = 0; k < 16; ++k) p = nx[p];
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = p;
    if (threadIdx.x == 0) cyc[blockIdx.x] = (t1 - t0);
}

// dependent global load chain over a small (L2 resident) or large buffer
__global__ __launch_bounds__(64) void k_glob(double* out, long long* cyc, int n, const int* nxt) {
    int p = (blockIdx.x * 64 + threadIdx.x) * 16;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < n; ++s) p = nxt[p];
    long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = p;
    if (threadIdx.x == 0) cyc[blockIdx.x] = (t1 - t0);
}

int main() {
    const int NB = 1024, n = 1000;
    double *out, *A; long long* cyc; int* nxt;
    hipMalloc(&out, NB * 64 * 8); hipMalloc(&A, 4096 * 8); hipMalloc(&cyc, NB * 8);
    std::vector<double> hA(4096); for (int i = 0; i < 4096; ++i) hA[i] = 0.5 + 0.001 * i;
    hipMemcpy(A, hA.data(), 4096 * 8, hipMemcpyHostToDevice);
    const size_t big = 64ull << 20;  // ints
    hipMalloc(&nxt, big * 4);
    std::vector<int> hn(big);
    auto run = [&](const char* name, void (*k)(double*, long long*, int, const double*), int grid, int nsteps, double per) {
        hipLaunchKernelGGL(k, dim3(grid), dim3(64), 0, 0, out, cyc, 10, A);
        hipDeviceSynchronize();
        hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k, dim3(grid), dim3(64), 0, 0, out, cyc, nsteps, A);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        std::vector<long long> hc(grid); hipMemcpy(hc.data(), cyc, grid * 8, hipMemcpyDeviceToHost);
        double c = 0; for (auto v : hc) c += v; c /= grid;
        printf("%-28s grid %5d: %8.1f cycles per step (memtime), kernel %.3f ms -> %.2f GHz\n", name, grid, c / (nsteps * per), ms, c / (ms * 1e6));
    };
    run("chain readlane (6x6)", k_chain_rl, 1, n, 1); run("chain readlane (6x6)", k_chain_rl, NB, n, 1);
    run("chain LDS (6x6)", k_chain_lds, 1, n, 1); run("chain LDS (6x6)", k_chain_lds, NB, n, 1);
    run("fp64 fma dep", k_fma, 1, n, 16); run("fp64 fma dep", k_fma, NB, n, 16);
    run("lds load dep", k_lds, 1, n, 16); run("lds load dep", k_lds, NB, n, 16);
    for (size_t span : {size_t(1) << 16, size_t(16) << 20, size_t(64) << 20}) {
        // random cyclic permutation over `span` ints with stride 16 ints (64 B) per node
        size_t m = span / 16;
        std::vector<size_t> perm(m); for (size_t i = 0; i < m; ++i) perm[i] = i;
        unsigned long long s = 12345; for (size_t i = m - 1; i > 0; --i) { s = s * 6364136223846793005ull + 1; size_t j = (s >> 33) % (i + 1); std::swap(perm[i], perm[j]); }
        for (size_t i = 0; i < m; ++i) hn[perm[i] * 16] = (int)(perm[(i + 1) % m] * 16);
        hipMemcpy(nxt, hn.data(), span * 4, hipMemcpyHostToDevice);
        for (int grid : {1, NB}) {
            hipLaunchKernelGGL(k_glob, dim3(grid), dim3(64), 0, 0, out, cyc, 10, nxt);
            hipDeviceSynchronize();
            hipLaunchKernelGGL(k_glob, dim3(grid), dim3(64), 0, 0, out, cyc, 200, nxt);
            hipDeviceSynchronize();
            std::vector<long long> hc(grid); hipMemcpy(hc.data(), cyc, grid * 8, hipMemcpyDeviceToHost);
            double c = 0; for (auto v : hc) c += v; c /= grid;
            printf("global load dep span %6zu KB grid %5d: %8.1f cycles per load\n", span * 4 / 1024, grid, c / 200);
        }
    }
    return 0;
}
