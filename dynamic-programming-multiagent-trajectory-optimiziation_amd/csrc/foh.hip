// Batched First-Order-Hold discretization and nonlinear roll-outs of the built-in models
// (MI355X / gfx950, float64).  The integrator bodies (algorithm, lane mapping, roofline) live in
// csrc/foh_body.hpp, shared with the runtime-compiled user models of csrc/foh_rtc.hip.
#include <hip/hip_runtime.h>

#include "models.hpp"
#include "scvx_hip.h"
#include "common.hpp"

namespace scvx {

// FOH_MIN_WAVES: minimum waves per SIMD the register allocation must allow (diagnostics A/B; the quadrotor's kernel
// takes 356 of 512 registers, one wave per SIMD)
#ifndef FOH_MIN_WAVES
#define FOH_MIN_WAVES 1
#endif
template <class Mdl>
__global__ __launch_bounds__(256, FOH_MIN_WAVES) void foh_kernel(const double* __restrict__ X, const double* __restrict__ U,
                                                  const double* __restrict__ sigma, double* __restrict__ out,
                                                  int K, int N, int nsub, ModelParams P) {
    __shared__ double stage[256 * Mdl::N];
    foh_body<Mdl>(X, U, sigma, out, K, N, nsub, P, stage);
}

template <class Mdl>
__global__ __launch_bounds__(256) void nonlinear_kernel(const double* __restrict__ X, const double* __restrict__ U,
                                                        const double* __restrict__ sigma, double* __restrict__ Xout,
                                                        int K, int N, int nsub, int piecewise, ModelParams P) {
    nonlinear_body<Mdl>(X, U, sigma, Xout, K, N, nsub, piecewise, P);
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
