// Batched First-Order-Hold discretization (MI355X / gfx950, float64).
//
// Replaces FirstOrderHold.calculate_discretization (SCvx/discretization/first_order_hold.py:52-87)
// and its nonlinear roll-outs (:127-162) for N agents at once.
//
// Algorithm.  The reference integrates the augmented ODE [x, Phi, Phi^-1 B alpha, ...] with LSODA
// and inverts Phi on every right-hand-side call (:108).  We integrate the equivalent
// forward-sensitivity system, which needs no inverse:
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
#include <hip/hip_runtime.h>

#include "models.hpp"
#include "scvx_hip.h"
#include "common.hpp"

namespace scvx {

template <class Mdl>
__global__ __launch_bounds__(256) void foh_kernel(const double* __restrict__ X, const double* __restrict__ U,
                                                  const double* __restrict__ sigma, double* __restrict__ out,
                                                  int K, int N, int nsub, ModelParams P) {
    constexpr int n = Mdl::N, m = Mdl::M, ncol = n + 2 * m + 2;
    __shared__ double stage[256 * n];
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
        Mdl::f(xs, u, fv, P);
#pragma unroll
        for (int i = 0; i < n; ++i) tmp[i] = cs[i] - dZ * xs[i];
        Mdl::Av(xs, u, tmp, Aw, P);
        Mdl::Bw(xs, u, w, Bwv, P);
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
__global__ __launch_bounds__(256) void nonlinear_kernel(const double* __restrict__ X, const double* __restrict__ U,
                                                        const double* __restrict__ sigma, double* __restrict__ Xout,
                                                        int K, int N, int nsub, int piecewise, ModelParams P) {
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
    if (piecewise && k0 == 0) {
#pragma unroll
        for (int i = 0; i < n; ++i) Xout[agent * K * n + i] = x[i];
    }
    if (!piecewise) {
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

template <class Mdl>
static int launch_foh(const double* X, const double* U, const double* sigma, double* out, int K, int N,
                      int nsub, const ModelParams& P, hipStream_t st) {
    constexpr int ncol = Mdl::N + 2 * Mdl::M + 2;
    const long long total = (long long)N * (K - 1) * ncol;
    const int block = 256;
    const long long grid = (total + block - 1) / block;
    hipLaunchKernelGGL(foh_kernel<Mdl>, dim3((unsigned)grid), dim3(block), 0, st, X, U, sigma, out, K, N, nsub, P);
    return check_launch("foh_kernel");
}

template <class Mdl>
static int launch_nl(const double* X, const double* U, const double* sigma, double* Xout, int K, int N,
                     int nsub, int piecewise, const ModelParams& P, hipStream_t st) {
    const long long total = piecewise ? (long long)N * (K - 1) : (long long)N;
    const int block = piecewise ? 256 : 64;
    const long long grid = (total + block - 1) / block;
    hipLaunchKernelGGL(nonlinear_kernel<Mdl>, dim3((unsigned)grid), dim3(block), 0, st, X, U, sigma, Xout, K, N,
                       nsub, piecewise, P);
    return check_launch("nonlinear_kernel");
}

static ModelParams make_params(int model_id, const double* params) {
    ModelParams P{};
    if (model_id == Quadrotor12::ID) {
        const double dflt[5] = {1.0, 9.81, 0.02, 0.02, 0.04};
        for (int i = 0; i < 5; ++i) P.p[i] = params ? params[i] : dflt[i];
    }
    return P;
}

}  // namespace scvx

using namespace scvx;

extern "C" int scvx_foh_batched(int model_id, const double* params, int K, int N, const double* X, const double* U,
                                const double* sigma, int nsub, double* out, void* stream) {
    if (K < 2 || N < 0 || nsub < 1 || !X || !U || !sigma || !out) return set_error(SCVX_EINVAL, "foh: bad args");
    if (N == 0) return SCVX_OK;
    const ModelParams P = make_params(model_id, params);
    hipStream_t st = (hipStream_t)stream;
    switch (model_id) {
        case DoubleIntegrator3D::ID: return launch_foh<DoubleIntegrator3D>(X, U, sigma, out, K, N, nsub, P, st);
        case Unicycle::ID: return launch_foh<Unicycle>(X, U, sigma, out, K, N, nsub, P, st);
        case SingleIntegrator3D::ID: return launch_foh<SingleIntegrator3D>(X, U, sigma, out, K, N, nsub, P, st);
        case Quadrotor12::ID: return launch_foh<Quadrotor12>(X, U, sigma, out, K, N, nsub, P, st);
        default: return set_error(SCVX_EUNSUPPORTED, "foh: unknown model id");
    }
}

extern "C" int scvx_integrate_nonlinear_batched(int model_id, const double* params, int K, int N, const double* X,
                                                const double* U, const double* sigma, int nsub, int piecewise,
                                                double* Xout, void* stream) {
    if (K < 2 || N < 0 || nsub < 1 || !X || !U || !sigma || !Xout) return set_error(SCVX_EINVAL, "nl: bad args");
    if (N == 0) return SCVX_OK;
    const ModelParams P = make_params(model_id, params);
    hipStream_t st = (hipStream_t)stream;
    switch (model_id) {
        case DoubleIntegrator3D::ID: return launch_nl<DoubleIntegrator3D>(X, U, sigma, Xout, K, N, nsub, piecewise, P, st);
        case Unicycle::ID: return launch_nl<Unicycle>(X, U, sigma, Xout, K, N, nsub, piecewise, P, st);
        case SingleIntegrator3D::ID: return launch_nl<SingleIntegrator3D>(X, U, sigma, Xout, K, N, nsub, piecewise, P, st);
        case Quadrotor12::ID: return launch_nl<Quadrotor12>(X, U, sigma, Xout, K, N, nsub, piecewise, P, st);
        default: return set_error(SCVX_EUNSUPPORTED, "nl: unknown model id");
    }
}
