// Batched ADMM consensus / dual update of the multi-agent coordinators.
//
// Replaces the host loop of SCvx/optimization/admm_coordinator.py:80-96 (and the same step of
// si_admm_coordinator.py:91-102): for every agent i and neighbour slot s (neighbour j = nbr[i][s]),
// with p_j the neighbour's new positions (rows 0..pos_dim-1 of its state trajectory):
//     Y_new = (Y + p_j) / 2,   Lam += rho (p_j - Y_new),
//     primal = ||p_j - Y_new||_F,   dual = ||Y_new - Y||_F            (admm_utils.py:20-38)
// All element updates are single IEEE operations in the reference's order (no contraction), so the
// consensus and dual variables are bit-identical to the numpy loop; the residual norms sum in a
// different order (last-bit differences in the logged means only).
//
// Mapping: one 64-lane wavefront per (agent, slot); lanes stride the K x pos_dim block (node-major,
// pos_dim minor -- the layout the SCP kernel reads nbr_Y / nbr_Lam in); the two norms are wave
// reductions.  Bytes per slot: read Y, Lam, p (24 K pos_dim / 3 B), write Y, Lam -- HBM-bound and tiny
// (one launch per ADMM round instead of N (N-1) host updates and a host round trip).
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "scvx_hip.h"
#include "wave_ops.hpp"

namespace scvx {

#pragma clang fp contract(off)
__global__ __launch_bounds__(64) void admm_consensus_kernel(int N, int n_nbr, int K, int pos_dim, int n_x,
                                                            const double* __restrict__ X_new,
                                                            const int32_t* __restrict__ nbr, double rho,
                                                            double* __restrict__ Y, double* __restrict__ Lam,
                                                            double* __restrict__ primal, double* __restrict__ dual) {
    const int slot = blockIdx.x;  // agent * n_nbr + s
    const int lane = threadIdx.x;
    const int j = nbr[slot];
    const int L = K * pos_dim;
    double* y = Y + (long long)slot * L;
    double* lam = Lam + (long long)slot * L;
    const double* xj = X_new + (long long)j * K * n_x;
    double pr = 0.0, du = 0.0;
    for (int e = lane; e < L; e += WAVE) {
        const int k = e / pos_dim, d = e - k * pos_dim;
        const double p = xj[k * n_x + d];
        const double yo = y[e];
        const double yn = 0.5 * (yo + p);
        const double r = p - yn;
        lam[e] = lam[e] + rho * r;
        y[e] = yn;
        const double dd = yn - yo;
        pr += r * r;
        du += dd * dd;
    }
    pr = wave_sum(pr);
    du = wave_sum(du);
    if (lane == 0) {
        primal[slot] = sqrt(pr);
        dual[slot] = sqrt(du);
    }
}
#pragma clang fp contract(on)

}  // namespace scvx

extern "C" int scvx_admm_consensus_batched(int N, int n_nbr, int K, int pos_dim, int n_x, const double* X_new,
                                           const int32_t* nbr, double rho, double* Y, double* Lam, double* primal,
                                           double* dual, void* stream) {
    if (N < 0 || n_nbr < 0 || K < 1 || pos_dim < 1 || pos_dim > n_x || !X_new || !nbr || !Y || !Lam || !primal ||
        !dual)
        return scvx::set_error(SCVX_EINVAL, "admm_consensus: bad args");
    if (N == 0 || n_nbr == 0) return SCVX_OK;
    hipLaunchKernelGGL(scvx::admm_consensus_kernel, dim3((unsigned)(N * n_nbr)), dim3(64), 0, (hipStream_t)stream, N,
                       n_nbr, K, pos_dim, n_x, X_new, nbr, rho, Y, Lam, primal, dual);
    return scvx::check_launch("admm_consensus_kernel");
}
