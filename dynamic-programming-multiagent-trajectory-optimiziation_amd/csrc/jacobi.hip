// Fused bookkeeping of one Jacobi SCvx iteration (per-agent trust-region rule), device-resident.
//
// Replaces the per-step tensor ops of scvx_hip/scvx.py JacobiSCvx.step for tr_rule="per_agent":
//   * X_out / U_out: an agent whose subproblem failed (status 2) keeps its iterate X / U, the others
//     take the solution
//     (the update X_traj += s of Distributed_opt/dist_scvx_3d.py:113-118, with the solved trajectory);
//   * cost_i = sum_{t<K-1} ||u_t||^2 of the new inputs (cost_fcn, dist_scvx_3d.py:131-138);
//   * tr_i halves when cost_i > prev_cost_i (1 + tie_rtol) (the rule of dist_scvx_3d.py:248-252 applied
//     per agent; tie_rtol > 0 keeps a converged agent, whose successive costs agree to rounding, from
//     halving on the rounding of its cost sum), then a failed agent's radius halves (grow = 0) or doubles
//     (grow = 1, every radius then capped at tr_max);
//   * prev_cost_i = cost_i.
// One wave per agent: coalesced copies of the agent's X / U slabs, the cost by a wave reduction,
// lane 0 updates the radius.  Replaces ~10 small elementwise launches per SCvx iteration.
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "scvx_hip.h"
#include "wave_ops.hpp"

namespace scvx {

__global__ __launch_bounds__(64) void jacobi_update_kernel(int K, int n, int m, const int32_t* __restrict__ status,
                                                           const double* __restrict__ X_sol,
                                                           const double* __restrict__ U_sol, const double* X,
                                                           const double* U, double* X_out, double* U_out,
                                                           double* __restrict__ tr,
                                                           double* __restrict__ prev_cost, int grow, double tr_max,
                                                           double tie_rtol) {
    const long long a = blockIdx.x;
    const int lane = threadIdx.x;
    const bool ok = status[a] != SCVX_STATUS_NUMERICAL;
    const long long xo = a * K * n, uo = a * K * m;
    // (X_out may alias X: every element is read and written by the same lane)
    for (int e = lane; e < K * n; e += WAVE) X_out[xo + e] = ok ? X_sol[xo + e] : X[xo + e];
    double c = 0.0;
    for (int e = lane; e < K * m; e += WAVE) {
        const double u = ok ? U_sol[uo + e] : U[uo + e];
        U_out[uo + e] = u;
        if (e < (K - 1) * m) c = fma(u, u, c);
    }
    c = wave_sum(c);
    if (lane == 0) {
        double r = tr[a];
        if (c > prev_cost[a] * (1.0 + tie_rtol)) r *= 0.5;
        if (!ok) r = grow ? 2.0 * r : 0.5 * r;
        if (grow) r = fmin(r, tr_max);  // the driver's rule caps every radius at tr_max in grow mode
        tr[a] = r;
        prev_cost[a] = c;
    }
}

}  // namespace scvx

extern "C" int scvx_jacobi_update_batched(int N, int K, int n_x, int n_u, const int32_t* status, const double* X_sol,
                                          const double* U_sol, const double* X, const double* U, double* X_out,
                                          double* U_out, double* tr, double* prev_cost, int grow, double tr_max,
                                          double tie_rtol, void* stream) {
    if (N < 0 || K < 2 || n_x < 1 || n_u < 1 || !status || !X_sol || !U_sol || !X || !U || !X_out || !U_out || !tr ||
        !prev_cost || !(tie_rtol >= 0.0))
        return scvx::set_error(SCVX_EINVAL, "jacobi_update: bad args");
    if (N == 0) return SCVX_OK;
    hipLaunchKernelGGL(scvx::jacobi_update_kernel, dim3((unsigned)N), dim3(scvx::WAVE), 0, (hipStream_t)stream, K, n_x,
                       n_u, status, X_sol, U_sol, X, U, X_out, U_out, tr, prev_cost, grow, tr_max, tie_rtol);
    return scvx::check_launch("jacobi_update_kernel");
}
