// FOH and nonlinear roll-out kernel bodies, templated on the model (gfx950, float64).
//
// Shared by the built-in models (csrc/foh.hip: compiled with the library) and by runtime-compiled
// user models (csrc/foh_rtc.hip: this file is embedded in the library as text and handed to hipRTC
// as a header, so both paths run the same integrator).  Self-contained: no other header of the
// library is visible to hipRTC.
//
// A model is a struct with
//   static constexpr int N, M;                                   state / input dimension
//   __device__ static void f (x, u, o, P)      o = f(x,u)                     (n)
//   __device__ static void Av(x, u, v, o, P)   o = (df/dx)(x,u) v            (n)
//   __device__ static void Bw(x, u, w, o, P)   o = (df/du)(x,u) w            (n)
// the contract of the reference's BaseModel.get_equations (SCvx/models/base_model.py:16-24) with the
// Jacobians applied to a vector instead of materialised.
//
// foh_body.  Replaces FirstOrderHold.calculate_discretization (first_order_hold.py:52-87).  The
// reference integrates the augmented ODE [x, Phi, Phi^-1 B alpha, ...] with LSODA and inverts Phi on
// every right-hand-side call (:108).  We integrate the equivalent forward-sensitivity system, which
// needs no inverse:
//     x'   = sigma f(x,u)
//     col' = sigma A(x,u) (col - d_z x) + sigma B(x,u) w_c + d_S f(x,u)
// where the "columns" of one interval are the n columns of Phi (w=0), the m columns of
// P_B = Phi*Btil (w = alpha e_j), of P_C (w = beta e_j), P_S (d_S = 1) and P_z
// (d_z = 1, w = -u).  At t = dt: A_k = Phi, B_k = P_B, ..., z_k = P_z -- exactly the reference's
// Phi@B_mat, Phi@C_mat, ... (:80-85).  Classical RK4 with `nsub` fixed substeps (exact for the
// double integrator with nsub = 1).
//
// Mapping.  One lane per (agent, interval, column): every lane re-integrates the interval's
// nominal state x(t) in registers (identical bits in all lanes of the interval) next to its own
// n-vector column, so there is no cross-lane traffic at all.  With the output laid out
// agent-major as out[N][K-1][n*(n+2m+2)] (column-major blocks, the reference's order='F'),
// lane `tid` owns exactly out[tid*n .. tid*n+n): consecutive lanes store consecutive bytes.
// The kernel is HBM-write bound: per interval it reads (n + 2m) doubles and writes
// n*(n+2m+2) doubles.
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif
#include <type_traits>

namespace scvx {

// a model may provide fab(x, u, v, w, f_out, Av_out, Bw_out, P): f, (df/dx) v and (df/du) w in one call sharing its
// common subexpressions (the quadrotor's sines and cosines); the integrator then calls it instead of f, Av, Bw
template <class M, class = void>
struct foh_has_fab : std::false_type {};
template <class M>
struct foh_has_fab<M, std::void_t<decltype(&M::fab)>> : std::true_type {};

#define SCVX_MAX_MODEL_PARAMS 16

struct ModelParams {
    double p[SCVX_MAX_MODEL_PARAMS];  // quadrotor: mass, g, Jx, Jy, Jz; user models: their own
};

// blockDim.x == 256 (the launchers' block); stage: __shared__ double[256 * Mdl::N]
template <class Mdl>
__device__ __forceinline__ void foh_body(const double* __restrict__ X, const double* __restrict__ U,
                                         const double* __restrict__ sigma, double* __restrict__ out, int K, int N,
                                         int nsub, const ModelParams& P, double* stage) {
    constexpr int n = Mdl::N, m = Mdl::M, ncol = n + 2 * m + 2;
    const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long total = (long long)N * (K - 1) * ncol;
    const bool live = tid < total;
    const long long tidc = live ? tid : total - 1;  // dead lanes recompute a valid column, store nothing
    const int col = (int)(tidc % ncol);
    const long long iv = tidc / ncol;  // agent * (K-1) + interval
    const int k = (int)(iv % (K - 1));
    const long long agent = iv / (K - 1);

    const double* xk = X + (agent * K + k) * n;
    const double* u0p = U + (agent * K + k) * m;
    const double s = sigma[agent];
    double x[n], c[n], u0[m], du[m];
#pragma unroll
    for (int i = 0; i < n; ++i) { x[i] = xk[i]; c[i] = (col == i) ? 1.0 : 0.0; }
#pragma unroll
    for (int j = 0; j < m; ++j) { u0[j] = u0p[j]; du[j] = u0p[m + j] - u0[j]; }

    // column kind -> (w selector, d_S, d_z)
    const bool isB = (col >= n) && (col < n + m);
    const bool isC = (col >= n + m) && (col < n + 2 * m);
    const int jcol = isB ? col - n : (isC ? col - n - m : -1);
    const double dS = (col == n + 2 * m) ? 1.0 : 0.0;
    const double dZ = (col == n + 2 * m + 1) ? 1.0 : 0.0;

    const double dt = 1.0 / (K - 1), h = dt / nsub;

    auto rhs = [&](double t, const double* xs, const double* cs, double* dx, double* dc) {
        const double beta = t / dt, alpha = 1.0 - beta;
        double u[m], w[m], fv[n], tmp[n], Aw[n], Bwv[n];
#pragma unroll
        for (int j = 0; j < m; ++j) {
            u[j] = u0[j] + beta * du[j];
            const double e = (j == jcol) ? 1.0 : 0.0;
            w[j] = isB ? alpha * e : (isC ? beta * e : -dZ * u[j]);
        }
#pragma unroll
        for (int i = 0; i < n; ++i) tmp[i] = cs[i] - dZ * xs[i];
        if constexpr (foh_has_fab<Mdl>::value) {
            Mdl::fab(xs, u, tmp, w, fv, Aw, Bwv, P);
        } else {
            Mdl::f(xs, u, fv, P);
            Mdl::Av(xs, u, tmp, Aw, P);
            Mdl::Bw(xs, u, w, Bwv, P);
        }
#pragma unroll
        for (int i = 0; i < n; ++i) {
            dx[i] = s * fv[i];
            dc[i] = s * (Aw[i] + Bwv[i]) + dS * fv[i];
        }
    };

    for (int sstep = 0; sstep < nsub; ++sstep) {
        const double t = sstep * h;
        double kx[n], kc[n], ax[n], ac[n], xt[n], ct[n];
        rhs(t, x, c, kx, kc);
#pragma unroll
        for (int i = 0; i < n; ++i) {
            ax[i] = kx[i]; ac[i] = kc[i];
            xt[i] = x[i] + 0.5 * h * kx[i]; ct[i] = c[i] + 0.5 * h * kc[i];
        }
        rhs(t + 0.5 * h, xt, ct, kx, kc);
#pragma unroll
        for (int i = 0; i < n; ++i) {
            ax[i] += 2.0 * kx[i]; ac[i] += 2.0 * kc[i];
            xt[i] = x[i] + 0.5 * h * kx[i]; ct[i] = c[i] + 0.5 * h * kc[i];
        }
        rhs(t + 0.5 * h, xt, ct, kx, kc);
#pragma unroll
        for (int i = 0; i < n; ++i) {
            ax[i] += 2.0 * kx[i]; ac[i] += 2.0 * kc[i];
            xt[i] = x[i] + h * kx[i]; ct[i] = c[i] + h * kc[i];
        }
        rhs(t + h, xt, ct, kx, kc);
#pragma unroll
        for (int i = 0; i < n; ++i) {
            x[i] += h / 6.0 * (ax[i] + kx[i]);
            c[i] += h / 6.0 * (ac[i] + kc[i]);
        }
    }
    // the block's columns are one contiguous range of out: stage them in LDS, then store with
    // consecutive lanes on consecutive doubles (full-line coalesced writes)
#pragma unroll
    for (int i = 0; i < n; ++i) stage[threadIdx.x * n + i] = c[i];
    __syncthreads();
    const long long base = (long long)blockIdx.x * blockDim.x * n;
    const long long lim = total * n - base;
#pragma unroll
    for (int i = 0; i < n; ++i) {
        const int e = i * (int)blockDim.x + threadIdx.x;
        if (e < lim) out[base + e] = stage[e];
    }
}

// integrate_nonlinear_piecewise (first_order_hold.py:127-140): one lane per (agent, interval),
// restart from X[:,k] each interval, physical time [0, dt*sigma], u interpolated by t/(dt*sigma).
// integrate_nonlinear_full (:142-155): one lane per agent, chained over the intervals.
template <class Mdl>
__device__ __forceinline__ void nonlinear_body(const double* __restrict__ X, const double* __restrict__ U,
                                               const double* __restrict__ sigma, double* __restrict__ Xout, int K,
                                               int N, int nsub, int piecewise, const ModelParams& P) {
    constexpr int n = Mdl::N, m = Mdl::M;
    const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long nwork = piecewise ? (long long)N * (K - 1) : (long long)N;
    if (tid >= nwork) return;
    const long long agent = piecewise ? tid / (K - 1) : tid;
    const int k0 = piecewise ? (int)(tid % (K - 1)) : 0;
    const int k1 = piecewise ? k0 + 1 : K - 1;
    const double T = sigma[agent] / (K - 1), h = T / nsub;
    double x[n];
#pragma unroll
    for (int i = 0; i < n; ++i) x[i] = X[(agent * K + k0) * n + i];
    if (!piecewise || k0 == 0) {
#pragma unroll
        for (int i = 0; i < n; ++i) Xout[agent * K * n + i] = x[i];
    }
    for (int k = k0; k < k1; ++k) {
        const double* u0p = U + (agent * K + k) * m;
        double u0[m], du[m];
#pragma unroll
        for (int j = 0; j < m; ++j) { u0[j] = u0p[j]; du[j] = u0p[m + j] - u0[j]; }
        auto fx = [&](double t, const double* xs, double* o) {
            double u[m];
#pragma unroll
            for (int j = 0; j < m; ++j) u[j] = u0[j] + (t / T) * du[j];
            Mdl::f(xs, u, o, P);
        };
        for (int sstep = 0; sstep < nsub; ++sstep) {
            const double t = sstep * h;
            double k_[n], acc[n], xt[n];
            fx(t, x, k_);
#pragma unroll
            for (int i = 0; i < n; ++i) { acc[i] = k_[i]; xt[i] = x[i] + 0.5 * h * k_[i]; }
            fx(t + 0.5 * h, xt, k_);
#pragma unroll
            for (int i = 0; i < n; ++i) { acc[i] += 2.0 * k_[i]; xt[i] = x[i] + 0.5 * h * k_[i]; }
            fx(t + 0.5 * h, xt, k_);
#pragma unroll
            for (int i = 0; i < n; ++i) { acc[i] += 2.0 * k_[i]; xt[i] = x[i] + h * k_[i]; }
            fx(t + h, xt, k_);
#pragma unroll
            for (int i = 0; i < n; ++i) x[i] += h / 6.0 * (acc[i] + k_[i]);
        }
#pragma unroll
        for (int i = 0; i < n; ++i) Xout[(agent * K + k + 1) * n + i] = x[i];
    }
}

}  // namespace scvx
