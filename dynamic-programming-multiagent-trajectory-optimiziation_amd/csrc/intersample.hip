// Batched inter-sample obstacle clearance for MI355X (gfx950, float64): the built-in models' launches of the
// kernel body in csrc/intersample_body.hpp (runtime-compiled user models: csrc/foh_rtc.hip).
#include <hip/hip_runtime.h>

#include <cmath>

#include "common.hpp"
#include "intersample_body.hpp"
#include "models.hpp"
#include "scvx_hip.h"

namespace scvx {
namespace {

template <class Mdl>
__global__ __launch_bounds__(256) void intersample_kernel(ISArgs a) {
    intersample_body<Mdl>(a);
}

template <class Mdl>
int launch_is(const ISArgs& a, hipStream_t st) {
    const long long nwork = (long long)a.N * (a.K - 1) * a.T.n_obs;
    const int block = 256;
    const long long grid = (nwork + block - 1) / block;
    hipLaunchKernelGGL(intersample_kernel<Mdl>, dim3((unsigned)grid), dim3(block), 0, st, a);
    return check_launch("intersample_kernel");
}

}  // namespace
}  // namespace scvx

using namespace scvx;

extern "C" int scvx_intersample_batched(const scvx_intersample_template* tpl, const double* params, int K, int N,
                                        const double* X, const double* U, const double* sigma, int32_t* n_crit,
                                        double* t_crit, double* h0, double* grad_x, double* grad_u, void* stream) {
    if (!tpl) return set_error(SCVX_EINVAL, "intersample: bad template / sizes");
    const scvx_intersample_template& T = *tpl;
    if (const char* bad = intersample_check(T, K, N, 0)) return set_error(SCVX_EINVAL, bad);
    if (N == 0 || T.n_obs == 0) return SCVX_OK;
    if (!X || !U || !sigma || !n_crit || !t_crit || !h0 || !grad_x || !grad_u)
        return set_error(SCVX_EINVAL, "intersample: null buffer");
    ISArgs a{};
    a.T = T;
    a.K = K; a.N = N;
    a.X = X; a.U = U; a.sigma = sigma;
    a.n_crit = n_crit; a.t_crit = t_crit; a.h0 = h0; a.grad_x = grad_x; a.grad_u = grad_u;
    a.P = model_params(T.model_id, params);
    hipStream_t st = (hipStream_t)stream;
    switch (T.model_id) {
        case DoubleIntegrator3D::ID: return launch_is<DoubleIntegrator3D>(a, st);
        case Unicycle::ID: return launch_is<Unicycle>(a, st);
        case SingleIntegrator3D::ID: return launch_is<SingleIntegrator3D>(a, st);
        case Quadrotor12::ID: return launch_is<Quadrotor12>(a, st);
        default: return set_error(SCVX_EUNSUPPORTED, "intersample: unknown model id");
    }
}
