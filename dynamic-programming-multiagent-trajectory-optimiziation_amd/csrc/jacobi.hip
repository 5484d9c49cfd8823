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
//
// The global rule (the reference's: one radius for all agents, halved when the SUMMED cost rises,
// dist_scvx_3d.py:248-252) in two launches (round 6): jacobi_update_kernel with cost_out set writes each
// agent's cost and leaves the radii alone; jacobi_global_rule_kernel (one workgroup) sums the costs in a fixed
// order, compares the total with the previous one (the reference's strict test), scales every radius, applies the
// failure rule and stores the total.  At world > 1 the local total is all-reduced in between (mode 0 sums, mode 2
// applies a given total).
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
                                                           double tie_rtol, double* __restrict__ cost_out) {
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
    if (cost_out) {   // global rule: the radii change in jacobi_global_rule_kernel
        if (lane == 0) cost_out[a] = c;
        return;
    }
    if (lane == 0) {
        double r = tr[a];
        if (c > prev_cost[a] * (1.0 + tie_rtol)) r *= 0.5;
        if (!ok) r = grow ? 2.0 * r : 0.5 * r;
        if (grow) r = fmin(r, tr_max);  // the driver's rule caps every radius at tr_max in grow mode
        tr[a] = r;
        prev_cost[a] = c;
    }
}

// The global rule over N agents' costs, one workgroup of GR_THREADS: thread i sums agents i, i + GR_THREADS, ...
// in index order, then a fixed-shape tree (the same total for the same costs on every run).  mode 0: write the
// local total only; 1: sum, then apply; 2: apply the given total_in (the all-reduced sum of every rank's totals).
// Apply: shrink = total > prev_total (strict, dist_scvx_3d.py:250); tr_i *= 0.5 if shrink; a failed agent's radius
// then halves (grow = 0) or doubles (grow = 1, capped at tr_max) -- JacobiSCvx.step's tensor rule; prev_total = total.
constexpr int GR_THREADS = 256;
__global__ __launch_bounds__(GR_THREADS) void jacobi_global_rule_kernel(int N, int mode, const int32_t* __restrict__ status,
                                                                        const double* __restrict__ cost,
                                                                        const double* __restrict__ total_in,
                                                                        double* __restrict__ total_out,
                                                                        double* __restrict__ tr, double* prev_total,
                                                                        int grow, double tr_max) {
    __shared__ double part[GR_THREADS];
    const int i = threadIdx.x;
    double total;
    if (mode == 2) {
        total = *total_in;
    } else {
        double v = 0.0;
        for (int a = i; a < N; a += GR_THREADS) v += cost[a];
        part[i] = v;
        __syncthreads();
        for (int w = GR_THREADS / 2; w > 0; w >>= 1) {
            if (i < w) part[i] += part[i + w];
            __syncthreads();
        }
        total = part[0];
        if (mode == 0) {
            if (i == 0) *total_out = total;
            return;
        }
    }
    const double prev = *prev_total;
    const bool shrink = total > prev;
    for (int a = i; a < N; a += GR_THREADS) {
        double r = tr[a];
        if (shrink) r *= 0.5;
        if (status[a] == SCVX_STATUS_NUMERICAL) r = grow ? 2.0 * r : 0.5 * r;
        if (grow) r = fmin(r, tr_max);
        tr[a] = r;
    }
    __syncthreads();   // every thread has read prev_total
    if (i == 0) {
        *prev_total = total;
        if (total_out) *total_out = total;
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
                       n_u, status, X_sol, U_sol, X, U, X_out, U_out, tr, prev_cost, grow, tr_max, tie_rtol,
                       (double*)nullptr);
    return scvx::check_launch("jacobi_update_kernel");
}

extern "C" int scvx_jacobi_update_costs_batched(int N, int K, int n_x, int n_u, const int32_t* status,
                                                const double* X_sol, const double* U_sol, const double* X,
                                                const double* U, double* X_out, double* U_out, double* cost,
                                                void* stream) {
    if (N < 0 || K < 2 || n_x < 1 || n_u < 1 || !status || !X_sol || !U_sol || !X || !U || !X_out || !U_out || !cost)
        return scvx::set_error(SCVX_EINVAL, "jacobi_update_costs: bad args");
    if (N == 0) return SCVX_OK;
    hipLaunchKernelGGL(scvx::jacobi_update_kernel, dim3((unsigned)N), dim3(scvx::WAVE), 0, (hipStream_t)stream, K, n_x,
                       n_u, status, X_sol, U_sol, X, U, X_out, U_out, (double*)nullptr, (double*)nullptr, 0, 0.0, 0.0,
                       cost);
    return scvx::check_launch("jacobi_update_kernel");
}

extern "C" int scvx_jacobi_global_rule(int N, int mode, const int32_t* status, const double* cost,
                                       const double* total_in, double* total_out, double* tr, double* prev_total,
                                       int grow, double tr_max, void* stream) {
    if (N < 0 || mode < 0 || mode > 2 || (mode != 2 && !cost) || (mode == 2 && !total_in) || (mode == 0 && !total_out) ||
        (mode != 0 && (!status || !tr || !prev_total)))
        return scvx::set_error(SCVX_EINVAL, "jacobi_global_rule: bad args");
    hipLaunchKernelGGL(scvx::jacobi_global_rule_kernel, dim3(1), dim3(scvx::GR_THREADS), 0, (hipStream_t)stream, N, mode,
                       status, cost, total_in, total_out, tr, prev_total, grow, tr_max);
    return scvx::check_launch("jacobi_global_rule_kernel");
}
