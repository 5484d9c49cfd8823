// Batched SCvx convex subproblem (SCProblem / AgentSolver) for MI355X (gfx950), float64.
//
// Replaces the CVXPY+ECOS solve of SCvx/optimization/sc_problem.py:15-105 (SCVXSolver's subproblem,
// scvx_solver.py:55-71) and of AgentSolver.setup/solve (agent_solver.py:43-117,
// si_agent_solver.py:39-105), batched over N agents; the problem is stated in include/scvx_hip.h.
// oracle/scp_cpu.py is the line-by-line CPU restatement of this kernel, oracle/scp_dense.py the
// independent reference-formulation checker.
//
// Reformulation (exact), per node k: z_k = [xi_k (n) | g (4) | u_k (m) | nu_k (n)] with
//   xi_k = x_k - C_{k-1} u_k            (FOH transform: the dynamics lose the u_{k+1} term)
//   g    = (sigma, tau_x, tau_u, tau_nu) augmented Riccati state, g_{k+1} = g_k
// The induced 1-norms become L1-ball facets s'(x_k - xbar_k) <= tau_x, s'(u_k - ubar_k) <= tau_u,
// s'nu_k <= tau_nu with |sigma - sigma_ref| + tau_x + tau_u <= tr at node 0; x_{K-1} = x_final is
// eliminated by substituting nu_{K-2} from the K-2 dynamics into its facets (the K-2 dynamics then
// pin xi_{K-1}); u_0, u_{K-1}, nu_{K-1} (absent) and nu_{K-2} are pinned inputs; x_0 = x_init is the
// Riccati initial state with g_0 free.  Soft rows (obstacles, ADMM collision rows) keep their slack,
// eliminated per row.  Every cost term is divided by an objective scale cs so the duals are O(1).
//
// Mapping: one agent per workgroup of NW waves (NW = 2 when K > 64 and the launch leaves SIMDs idle, e.g.
// a single-agent SCVXSolver or Nash call; 1 otherwise).  Node phases are parallel over the nodes (thread
// tid: nodes tid, tid + 64 NW, ...); the Riccati factor sweep is sequential over nodes and
// element-parallel over wave 0's lanes, with the stage matrices in LDS.  The LQ solve is the same sweep
// form for NW = 1 and the closed-loop form (two NXA-vector chains, the rest lane-parallel) for NW = 2.
// Per-node data (rows in z coordinates, iterates, scaling, factor outputs) lives in an agent-private
// workspace block per node.  Problems are small (K <= 256, |z| <= 16): this kernel serves the
// reference's SCVXSolver / ADMM / Nash subproblems, not the batched headline path (csrc/qp_ipm.hpp).
//
// The kernel itself is csrc/scp_kernel.hpp (also compiled at run time for user models).
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "scp_kernel.hpp"
#include "scvx_hip.h"
#include "subproblem_rtc.hpp"
#include "wave_ops.hpp"


using namespace scvx;

extern "C" size_t scvx_scp_workspace_bytes(const scvx_scp_template* T, int N) {
    if (!T || N < 0) return 0;
    const SCPLay L = scp_layout(*T);
    return sizeof(double) * (size_t)N * (size_t)L.stride * (size_t)(T->K + 1);  // + the per-lane junk block
}


static int scp_launch(const scvx_scp_template* T, int N, const double* disc, const double* Xref, const double* Uref,
                      const double* sigma_ref, const double* tr, const double* x_init, const double* x_final,
                      const double* nbr_pos, const double* nbr_Y, const double* nbr_Lam, const double* X_prev,
                      const double* slab_z, const double* slab_P, double* X, double* U, double* nu, double* sigma,
                      double* s_obs, double* s_nbr, double* obj, int32_t* status, int32_t* iters, void* workspace,
                      size_t workspace_bytes, void* stream) {
    if (!T || N < 0) return set_error(SCVX_EINVAL, "scp: null template");
    if (N == 0) return SCVX_OK;
    if (T->K < 3 || T->K > SCP_KMAX) return set_error(SCVX_EUNSUPPORTED, "scp: K must be in [3, 256]");
    if (T->pos_dim < 1 || T->pos_dim > 3 || T->pos_dim > T->n_x) return set_error(SCVX_EINVAL, "scp: pos_dim");
    if (T->n_ubound < 0 || T->n_ubound > SCVX_MAX_BOX || T->n_xbound < 0 || T->n_xbound > SCVX_MAX_BOX ||
        T->n_obs < 0 || T->n_obs > SCVX_MAX_OBS || T->n_nbr < 0 || T->n_nbr > SCVX_MAX_NBR)
        return set_error(SCVX_EINVAL, "scp: bound / obstacle / neighbour counts");
    for (int b = 0; b < T->n_ubound; ++b)
        if (T->ub_idx[b] < 0 || T->ub_idx[b] >= T->n_u) return set_error(SCVX_EINVAL, "scp: input bound index");
    for (int b = 0; b < T->n_xbound; ++b)
        if (T->xb_idx[b] < 0 || T->xb_idx[b] >= T->n_x) return set_error(SCVX_EINVAL, "scp: state bound index");
    if (T->has_final && !T->pin_u_last) return set_error(SCVX_EUNSUPPORTED, "scp: has_final requires pin_u_last");
    if (T->max_iter < 1) return set_error(SCVX_EINVAL, "scp: max_iter");
    if (T->waves_per_agent < 0 || T->waves_per_agent > 2) return set_error(SCVX_EINVAL, "scp: waves_per_agent (0, 1, 2)");
    if (!disc || !Xref || !Uref || !sigma_ref || !tr || !x_init || !x_final || !X || !U || !nu || !sigma || !obj ||
        !status || !iters || (T->n_obs && !s_obs) || (T->n_nbr && (!nbr_pos || !nbr_Y || !nbr_Lam || !s_nbr)))
        return set_error(SCVX_EINVAL, "scp: null buffer");
    if (T->game) {
        if (T->n_nbr != 0) return set_error(SCVX_EUNSUPPORTED, "scp game: no ADMM terms (n_nbr must be 0)");
        if (T->n_slab < 0 || T->n_slab > SCVX_MAX_NBR) return set_error(SCVX_EINVAL, "scp game: n_slab");
        if (T->theta_idx >= T->n_x) return set_error(SCVX_EINVAL, "scp game: theta_idx");
        if (!(T->w_u2 >= 0.0) || !(T->w_du >= 0.0) || !(T->w_dth >= 0.0) || !(T->w_in >= 0.0))
            return set_error(SCVX_EINVAL, "scp game: negative weight");
        if ((T->w_in > 0.0 && !X_prev) || (T->n_slab && (!slab_z || !slab_P)))
            return set_error(SCVX_EINVAL, "scp game: null buffer");
    }
    const size_t need = scvx_scp_workspace_bytes(T, N);
    if (!workspace || workspace_bytes < need) return set_error(SCVX_EWORKSPACE, "scp: workspace too small");
    SCPArgs a{};
    a.T = *T;
    a.N = N;
    a.disc = disc; a.Xref = Xref; a.Uref = Uref; a.sigma_ref = sigma_ref; a.tr = tr; a.x_init = x_init;
    a.x_final = x_final; a.nbr_pos = nbr_pos; a.nbr_Y = nbr_Y; a.nbr_Lam = nbr_Lam;
    a.X_prev = X_prev; a.slab_z = slab_z; a.slab_P = slab_P;
    a.X = X; a.U = U; a.nu = nu; a.sigma = sigma; a.s_obs = s_obs; a.s_nbr = s_nbr; a.obj = obj;
    a.status = status; a.iters = iters;
    a.ws = (double*)workspace;
    a.ws_agent = (long long)scp_layout(*T).stride * (T->K + 1);
    hipStream_t st = (hipStream_t)stream;
    const int ne = scp_ne(*T);
    // two waves per agent (node phases in one pass over K <= 128 nodes) when the launch leaves SIMDs idle:
    // the kernel holds a SIMD's whole register file, so at most one wave per SIMD runs
    static int simds = 0;
    if (!simds) {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
            simds = 4 * cus;
        if (simds <= 0) simds = 1024;
    }
    // the template's own mapping: 0 automatic, 1 or 2 forced
    const int wsel = T->waves_per_agent;
    const bool two = wsel == 2 || (wsel == 0 && T->K > WAVE && 2LL * N <= simds);
    if (T->model_id == SCVX_MODEL_UNICYCLE && T->n_x == 3 && T->n_u == 2) {
        if (T->has_soc) return set_error(SCVX_EUNSUPPORTED, "scp: SOC rows need n_u + 1 <= 4");
        if (ne == 0)
            { if (two) hipLaunchKernelGGL((scp_ipm_kernel<3, 2, 0, 2>), dim3(N), dim3(2 * WAVE), 0, st, a, a.ws, a.disc); else hipLaunchKernelGGL((scp_ipm_kernel<3, 2, 0, 1>), dim3(N), dim3(WAVE), 0, st, a, a.ws, a.disc); }
        else if (ne == 3)
            { if (two) hipLaunchKernelGGL((scp_ipm_kernel<3, 2, 3, 2>), dim3(N), dim3(2 * WAVE), 0, st, a, a.ws, a.disc); else hipLaunchKernelGGL((scp_ipm_kernel<3, 2, 3, 1>), dim3(N), dim3(WAVE), 0, st, a, a.ws, a.disc); }
        else
            return set_error(SCVX_EUNSUPPORTED, "scp game: unicycle needs theta_idx = 2");
    } else if (T->model_id == SCVX_MODEL_SINGLE_INTEGRATOR && T->n_x == 3 && T->n_u == 3) {
        if (ne == 0)
            { if (two) hipLaunchKernelGGL((scp_ipm_kernel<3, 3, 0, 2>), dim3(N), dim3(2 * WAVE), 0, st, a, a.ws, a.disc); else hipLaunchKernelGGL((scp_ipm_kernel<3, 3, 0, 1>), dim3(N), dim3(WAVE), 0, st, a, a.ws, a.disc); }
        else if (ne == 3)
            { if (two) hipLaunchKernelGGL((scp_ipm_kernel<3, 3, 3, 2>), dim3(N), dim3(2 * WAVE), 0, st, a, a.ws, a.disc); else hipLaunchKernelGGL((scp_ipm_kernel<3, 3, 3, 1>), dim3(N), dim3(WAVE), 0, st, a, a.ws, a.disc); }
        else
            return set_error(SCVX_EUNSUPPORTED, "scp game: single integrator has no heading (theta_idx = -1)");
    } else if (T->model_id == SCVX_MODEL_RUNTIME) {
        // any other model (its FOH from scvx_rtc_model_create): the kernel instantiated for (n_x, n_u) at the
        // first solve; the node vector z = [xi | g | game states | u | nu] stays within the kernel's 16
        if (const char* bad = rtc_scp_class_error(T->n_x, T->n_u, ne)) return set_error(SCVX_EUNSUPPORTED, bad);
        if (T->has_soc && T->n_u > 3) return set_error(SCVX_EUNSUPPORTED, "scp: SOC rows need n_u + 1 <= 4");
        return rtc_scp_launch(a, ne, two ? 2 : 1, st);
    } else {
        return set_error(SCVX_EUNSUPPORTED, "scp: model (unicycle n=3 m=2, single integrator n=3 m=3, or "
                                            "SCVX_MODEL_RUNTIME)");
    }
    return check_launch("scp_ipm_kernel");
}


extern "C" int scvx_scp_solve_batched(const scvx_scp_template* T, int N, const double* disc, const double* Xref,
                                      const double* Uref, const double* sigma_ref, const double* tr,
                                      const double* x_init, const double* x_final, const double* nbr_pos,
                                      const double* nbr_Y, const double* nbr_Lam, double* X, double* U, double* nu,
                                      double* sigma, double* s_obs, double* s_nbr, double* obj, int32_t* status,
                                      int32_t* iters, void* workspace, size_t workspace_bytes, void* stream) {
    if (T && T->game) return set_error(SCVX_EINVAL, "scp: game template: use scvx_scp_game_solve_batched");
    return scp_launch(T, N, disc, Xref, Uref, sigma_ref, tr, x_init, x_final, nbr_pos, nbr_Y, nbr_Lam, nullptr,
                      nullptr, nullptr, X, U, nu, sigma, s_obs, s_nbr, obj, status, iters, workspace, workspace_bytes,
                      stream);
}

extern "C" int scvx_scp_game_solve_batched(const scvx_scp_template* T, int N, const double* disc, const double* Xref,
                                           const double* Uref, const double* sigma_ref, const double* tr,
                                           const double* x_init, const double* x_final, const double* X_prev,
                                           const double* slab_z, const double* slab_P, double* X, double* U,
                                           double* nu, double* sigma, double* s_obs, double* obj, int32_t* status,
                                           int32_t* iters, void* workspace, size_t workspace_bytes, void* stream) {
    if (!T || !T->game) return set_error(SCVX_EINVAL, "scp game: template without game = 1");
    return scp_launch(T, N, disc, Xref, Uref, sigma_ref, tr, x_init, x_final, nullptr, nullptr, nullptr, X_prev,
                      slab_z, slab_P, X, U, nu, sigma, s_obs, nullptr, obj, status, iters, workspace, workspace_bytes,
                      stream);
}

// ---------------------------------------------------------------------------------------------
// ACS slab update (game_model.py:54-66): z = d/||d|| (0 when ||d|| < 1e-6), one lane per (agent, j, k)
namespace scvx {
namespace {
__global__ __launch_bounds__(256) void slab_update_kernel(int N, int n_slab, int K, int pd, int n_x,
                                                          const double* __restrict__ p, const double* __restrict__ P,
                                                          double* __restrict__ z) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long total = (long long)N * n_slab * K;
    if (e >= total) return;
    const int k = (int)(e % K);
    const long long a = e / ((long long)n_slab * K);
    double d[3] = {0.0, 0.0, 0.0}, nn = 0.0;
    for (int i = 0; i < pd; ++i) {
        d[i] = p[(a * K + k) * n_x + i] - P[e * pd + i];
        nn += d[i] * d[i];
    }
    nn = sqrt(nn);
    for (int i = 0; i < pd; ++i) z[e * pd + i] = nn < 1e-6 ? 0.0 : d[i] / nn;
}
}  // namespace
}  // namespace scvx

extern "C" int scvx_slab_update_batched(int N, int n_slab, int K, int pos_dim, int n_x, const double* p,
                                        const double* P, double* z, void* stream) {
    if (N < 0 || n_slab < 0 || K < 1 || pos_dim < 1 || pos_dim > 3 || pos_dim > n_x || !p || !P || !z)
        return set_error(SCVX_EINVAL, "slab_update: bad args");
    const long long total = (long long)N * n_slab * K;
    if (total == 0) return SCVX_OK;
    hipLaunchKernelGGL(slab_update_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       N, n_slab, K, pos_dim, n_x, p, P, z);
    return check_launch("slab_update_kernel");
}
