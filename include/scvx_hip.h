/*
 * libscvx_hip.so -- C-ABI of the MI355X-native batched SCvx inner loop.
 *
 * Every pointer argument of a compute entry point is a CALLER-OWNED DEVICE buffer (e.g. a
 * PyTorch-ROCm tensor's data_ptr()); `stream` is a hipStream_t (NULL = default stream).  The
 * library never allocates caller-visible memory, never synchronises the stream and never throws:
 * every function returns SCVX_OK (0) or a negative SCVX_E* code, with a message available from
 * scvx_last_error().  Per-agent solver outcomes are reported in `status` arrays
 * (SCVX_STATUS_*), which the Python layer maps to CVXPY status strings.
 *
 * Layouts are agent-major (agent = outermost index) so that one agent's data is contiguous:
 *   X      [N][K][n]        == per agent the reference's X (n,K) in order='F'
 *   U      [N][K][m]
 *   disc   [N][K-1][n*(n+2m+2)]   per interval vec_F(A_k) | vec_F(B_k) | vec_F(C_k) | S_k | z_k
 *          == columns k of the reference's (A_bar, B_bar, C_bar, S_bar, z_bar)
 *          (SCvx/discretization/first_order_hold.py:20-24, 75-85).
 */
#ifndef SCVX_HIP_H
#define SCVX_HIP_H

#ifndef __HIPCC_RTC__  /* hipRTC (runtime-compiled kernels of user models) provides size_t itself */
#include <stddef.h>
#endif
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SCVX_HIP_VERSION 6   /* 6: scvx_jacobi_update_costs_batched + scvx_jacobi_global_rule (the global rule fused) */

#define SCVX_OK 0
#define SCVX_EINVAL (-1)
#define SCVX_EUNSUPPORTED (-2)
#define SCVX_ELAUNCH (-3)
#define SCVX_EWORKSPACE (-4)

/* model ids (csrc/models.hpp) */
#define SCVX_MODEL_DOUBLE_INTEGRATOR 0 /* n=6,  m=3  Distributed_opt/dist_scvx_3d.py:10-21 */
#define SCVX_MODEL_UNICYCLE 1          /* n=3,  m=2  SCvx/models/unicycle_model.py:54-63   */
#define SCVX_MODEL_SINGLE_INTEGRATOR 2 /* n=3,  m=3  SCvx/models/single_integrator_model.py:54-57 */
#define SCVX_MODEL_QUADROTOR 3         /* n=12, m=4  build-defined           */
/* any other model: n_x / n_u taken from the template; the subproblem kernels (QP, SCP) are compiled for
   those dimensions at the first solve (hipRTC) -- the user-model path of scvx_rtc_model_create */
#define SCVX_MODEL_RUNTIME 255

/* per-agent solver status (maps to cvxpy.OPTIMAL / OPTIMAL_INACCURATE / ...) */
#define SCVX_STATUS_OPTIMAL 0
#define SCVX_STATUS_MAX_ITER 1
#define SCVX_STATUS_NUMERICAL 2

int scvx_version(void);
const char* scvx_last_error(void);

/*
 * Batched FOH discretization.  Replaces FirstOrderHold.calculate_discretization
 * (SCvx/discretization/first_order_hold.py:52-87) for N agents in one launch.
 *   X [N][K][n], U [N][K][m], sigma [N]  ->  out [N][K-1][n*(n+2m+2)]
 * nsub = RK4 substeps per interval (1 is exact for the double integrator).
 * params: model parameters (quadrotor: mass, g, Jx, Jy, Jz) or NULL for defaults.
 */
int scvx_foh_batched(int model_id, const double* params, int K, int N, const double* X, const double* U,
                     const double* sigma, int nsub, double* out, void* stream);

/*
 * Batched nonlinear roll-outs: FirstOrderHold.integrate_nonlinear_piecewise (piecewise=1) and
 * integrate_nonlinear_full (piecewise=0) (first_order_hold.py:127-155).  Xout [N][K][n].
 */
int scvx_integrate_nonlinear_batched(int model_id, const double* params, int K, int N, const double* X,
                                     const double* U, const double* sigma, int nsub, int piecewise,
                                     double* Xout, void* stream);

/* ------------------------------------------------------------------------------------------
 * Runtime-compiled user models (hipRTC).  The reference's FirstOrderHold(model, K) integrates ANY
 * BaseModel through its numpy f/A/B callables (SCvx/discretization/first_order_hold.py:13-50,
 * 89-125; SCvx/models/base_model.py:16-24).  Here a user model is given as C expressions and
 * compiled for gfx950 at run time into the same RK4 forward-sensitivity kernel the built-in models
 * use (csrc/foh_body.hpp); no CPU path exists.
 *
 * Expressions are HIP C++ double expressions in x[0..n_x), u[0..n_u), p[0..SCVX_MAX_MODEL_PARAMS)
 * (the params array of the launch) and any name the prelude defines:
 *   f_exprs  n_x entries         f_i(x, u)
 *   A_exprs  n_x*n_x, row-major  dA_ij = d f_i / d x_j
 *   B_exprs  n_x*n_u, row-major  dB_ij = d f_i / d u_j
 * A NULL entry, "" or "0" is a structural zero (skipped in the generated matrix-vector products).
 * prelude: optional statements (e.g. `const double c2 = cos(x[2]);`) evaluated before the
 * expressions in each of f, A and B.  n_x <= 16, n_u <= 8.
 *
 * scvx_rtc_model_create compiles (no GPU needed); the code object is loaded on the calling
 * thread's current device at the first launch.  On a compile error it returns SCVX_EINVAL with
 * *out set to a model that holds only the generated source and the compiler log (read them with
 * scvx_rtc_model_source / _log, then destroy it; launches on it fail); other errors leave *out NULL.
 * ------------------------------------------------------------------------------------------ */
#define SCVX_MAX_MODEL_PARAMS 16
#define SCVX_RTC_MAX_NX 16
#define SCVX_RTC_MAX_NU 8
typedef struct scvx_rtc_model scvx_rtc_model;

int scvx_rtc_model_create(int n_x, int n_u, const char* const* f_exprs, const char* const* A_exprs,
                          const char* const* B_exprs, const char* prelude, scvx_rtc_model** out);
/* generated HIP source (for inspection) and the last compile log; buffers are the model's */
const char* scvx_rtc_model_source(const scvx_rtc_model* model);
const char* scvx_rtc_model_log(const scvx_rtc_model* model);
int scvx_rtc_model_destroy(scvx_rtc_model* model);

/* as scvx_foh_batched / scvx_integrate_nonlinear_batched; params: n_params <= SCVX_MAX_MODEL_PARAMS
 * doubles (host memory, copied into the launch), p[i] = 0 beyond n_params */
int scvx_rtc_foh_batched(const scvx_rtc_model* model, const double* params, int n_params, int K, int N,
                         const double* X, const double* U, const double* sigma, int nsub, double* out,
                         void* stream);
int scvx_rtc_integrate_nonlinear_batched(const scvx_rtc_model* model, const double* params, int n_params,
                                         int K, int N, const double* X, const double* U, const double* sigma,
                                         int nsub, int piecewise, double* Xout, void* stream);

/* Compile (no GPU needed) the subproblem kernel a SCVX_MODEL_RUNTIME template is served by, into the
 * process-wide code-object cache the first solve would fill (a warm-up / a build check of user classes):
 *   kind 0  the trust-region QP (scvx_qp_solve_batched), cls = {n_x, n_u, n_box, n_obs, j_max class, VC}
 *   kind 1  the SCProblem (scvx_scp_solve_batched),       cls = {n_x, n_u, n_extra, waves per agent}
 * (the class ints of csrc/qp_capi.hip / csrc/scp_ipm.hip).  *code_bytes (optional) = code-object size.
 * SCVX_EINVAL with the compiler log in scvx_last_error() on a compile error. */
int scvx_rtc_subproblem_compile(int kind, const int* cls, int ncls, size_t* code_bytes);

/* ------------------------------------------------------------------------------------------
 * Batched trust-region subproblem (one per agent), the convex solve the reference hands to
 * CVXPY+Clarabel in Distributed_opt/dist_scvx_3d.py:51-111 (x_traj_opt), written in absolute
 * variables x_t = xbar_t + d_t, u_t = ubar_t + w_t:
 *
 *   min  sum_{t<K-1} ||u_t||^2 + w_last ||u_{K-1}||^2 + w_coll sum_t S_t + w_obs sum_{t,o} s_{t,o}
 *   s.t. x_0 = x_init                                                    (:73, d_0 = 0)
 *        x_{t+1} = A_t x_t + B_t u_t + C_t u_{t+1} + S_t sigma + z_t      (:80-83; FOH form)
 *        x_{K-1} = x_final                     if has_final               (:74)
 *        u_{K-1} = ubar_{K-1}                  if fix_last_input          (:63, unused w row)
 *   for nodes t < K-1 (and t = K-1 if ineq_last):
 *        ||u_t - ubar_t||_1 <= tr                                        (:84)
 *        box_lo[i] <= x_t[box_idx[i]] <= box_hi[i]                         (:87-90)
 *        b_j - g_j' p_t <= S_t (j < coll_count[t]),  S_t >= 0           (:93-107, shared slack)
 *        a_o' (p_t - c_o) >= r_o - s_{t,o},  s_{t,o} >= 0,
 *           a_o = (pbar_t - c_o)/(||pbar_t - c_o|| + 1e-6)   (single_integrator_model.py:113-126)
 *        ||u_t||_2 <= u_max                    if has_soc                 (single_integrator_model.py:103-104)
 * with p_t = x_t[0:pos_dim].  With w_nu > 0 (virtual control, the SCvx subproblem form of
 * SCvx/optimization/sc_problem.py:60-68) every dynamics row carries nu_t (t < K-1):
 *        x_{t+1} = A_t x_t + B_t u_t + C_t u_{t+1} + S_t sigma + z_t + nu_t,
 * and the objective gains the exact penalty w_nu sum_t ||nu_t||_1 (node-separable; the reference's
 * SCProblem prices max_t ||nu_t||_1, scvx_scp_solve_batched below), so the subproblem stays feasible
 * whatever the linearisation point (nonlinear models under the Jacobi update).  With w_prox > 0 the
 * objective also gains w_prox sum_t ||x_t - xbar_t||^2, a soft trust region on the states (the trust
 * region above bounds only the inputs, which leaves the states of a long integrator chain free).  Solved by a batched primal-dual interior-point method (Mehrotra
 * predictor-corrector, Nesterov-Todd scaling for the SOC) whose KKT systems are factored by a
 * Riccati recursion over the K nodes.
 * ------------------------------------------------------------------------------------------ */
#define SCVX_MAX_BOX 4
#define SCVX_MAX_OBS 16

typedef struct scvx_qp_template {
    int32_t model_id;       /* only used for n_x/n_u consistency checks */
    int32_t n_x, n_u, K;
    int32_t pos_dim;        /* 2 or 3 */
    int32_t has_final;
    int32_t fix_last_input;
    int32_t ineq_last;
    double w_last;
    int32_t n_box;
    int32_t box_idx[SCVX_MAX_BOX];
    double box_lo[SCVX_MAX_BOX];
    double box_hi[SCVX_MAX_BOX];
    int32_t n_obs;
    double obs_center[SCVX_MAX_OBS][3];
    double obs_radius[SCVX_MAX_OBS];
    double w_obs;
    int32_t j_max;          /* collision rows per node (0 = no coupling) */
    double w_coll;
    int32_t has_soc;
    double u_max;
    int32_t max_iter;
    double tol;
    double w_final;         /* has_final = 0 and w_final > 0: soft terminal w_final ||x_{K-1} - x_final||^2 */
    double w_nu;            /* > 0: virtual control nu_t with penalty w_nu sum_t ||nu_t||_1 (0: none) */
    double w_prox;          /* > 0: proximal term w_prox sum_t ||x_t - xbar_t||^2 (a soft state trust region) */
} scvx_qp_template;

/*
 * Inputs (device, agent-major):
 *   disc [N][K-1][n(n+2m+2)], sigma [N], Xref [N][K][n], Uref [N][K][m], x_init [N][n],
 *   x_final [N][n] (ignored unless has_final or w_final > 0), tr [N],
 *   coll_rows [N][K][j_max][pos_dim+1] rows (g, b), coll_count [N][K] (both ignored if j_max=0)
 * Outputs (device):
 *   X [N][K][n], U [N][K][m], slack_coll [N][K] (S_t, zeros if j_max = 0),
 *   nu [N][K-1][n] (virtual control; required iff w_nu > 0, may be NULL otherwise), obj [N],
 *   status [N], iters [N]
 * warm [N] (device int32, may be NULL): agents with warm[a] != 0 start from the primal-dual point their
 *   previous solve left in this workspace (same template, same agent slot): z, the multipliers and the
 *   inequality duals are kept, the slacks recomputed from the new rows, every slack / dual floored
 *   inside its cone.  The optimum and the stopping rule are unchanged; the Jacobi SCvx loop, which
 *   re-solves each agent re-linearised at its own solution, needs ~2.4x fewer IPM iterations (C3).
 *   Requires K >= 2 n_x.  warm = NULL (or all 0): the CVXOPT-style cold start.
 * workspace: caller-owned device scratch of at least scvx_qp_workspace_bytes(tpl, N) bytes.
 * Limits: 2 <= K <= 64 (one node per lane), n_u <= 4, <= 64 inequality rows per node.
 */
int scvx_qp_solve_batched(const scvx_qp_template* tpl, int N, const double* disc, const double* sigma,
                          const double* Xref, const double* Uref, const double* x_init, const double* x_final,
                          const double* tr, const double* coll_rows, const int32_t* coll_count, double* X,
                          double* U, double* slack_coll, double* nu, double* obj, int32_t* status, int32_t* iters,
                          const int32_t* warm, void* workspace, size_t workspace_bytes, void* stream);

/* scvx_qp_solve_batched with a dispatch order (replaces the same call, qp_capi.hip; the reference has no
 * counterpart -- its agents' subproblems are solved one by one, dist_scvx_3d.py:110): workgroup b solves agent
 * order[b] (device int32 [N], a permutation of 0..N-1; NULL = agent b).  A non-permutation is undefined
 * behaviour: an entry outside [0, N) is replaced by b, which can duplicate an agent (two workgroups then share
 * its workspace and outputs) and leave another unsolved.
 * Workgroups start in index order as slots free up, so when the agents outnumber the resident waves the
 * longest solves dealt first shorten the launch (JacobiSCvx orders by the last step's IPM iterations).
 * Results do not depend on the order. */
int scvx_qp_solve_batched_ordered(const scvx_qp_template* tpl, int N, const double* disc, const double* sigma,
                                  const double* Xref, const double* Uref, const double* x_init,
                                  const double* x_final, const double* tr, const double* coll_rows,
                                  const int32_t* coll_count, double* X, double* U, double* slack_coll, double* nu,
                                  double* obj, int32_t* status, int32_t* iters, const int32_t* warm,
                                  const int32_t* order, void* workspace, size_t workspace_bytes, void* stream);

/* Bytes of caller-owned device scratch scvx_qp_solve_batched needs for N agents. */
size_t scvx_qp_workspace_bytes(const scvx_qp_template* tpl, int N);

/* Diagnostics hook: later solves write 8 doubles per IPM iteration of agent `agent`
 * (pres, dres, gap, pobj, alpha_aff, alpha, sigma, mu) into device buffer `buf` (cap iterations).
 * buf = NULL disables.  Not needed for normal use. */
int scvx_qp_set_trace(double* buf, int agent, int cap);

/*
 * Pairwise collision linearization for the Jacobi coupling (Distributed_opt/dist_scvx_3d.py:93-107):
 * for local agents i0..i0+N_local-1 of the all-gathered states X_all [N_total][K][n_x] and nodes
 * t < K-1, rows (g, b) with g = (p_i - p_j)/|p_i - p_j|, b = 2R - |p_i - p_j| + g' p_i, i.e.
 * b - g' p_t <= S_t.  cull_radius <= 0 keeps every neighbour; otherwise only |p_i - p_j| < cull_radius.
 * At most j_max rows per node (largest 2R - |.| kept).  rows [N_local][K][j_max][pos_dim+1],
 * count [N_local][K].
 */
int scvx_collision_rows_batched(int K, int pos_dim, int n_x, int N_total, const double* X_all, int i0,
                                int N_local, double R, double cull_radius, int j_max, double* rows,
                                int32_t* count, void* stream);

/*
 * The same rows for an arbitrary subset of agents: local agent a (< N_sel) is global agent idx[a] of X_all
 * (idx: device int32 [N_sel], distinct values in [0, N_total)).  rows [N_sel][K][j_max][pos_dim+1],
 * count [N_sel][K].  Used for the agents the full-row check below found violating.
 */
int scvx_collision_rows_indexed(int K, int pos_dim, int n_x, int N_total, const double* X_all, const int32_t* idx,
                                int N_sel, double R, double cull_radius, int j_max, double* rows, int32_t* count,
                                void* stream);

/*
 * A-posteriori check of the reference's FULL collision row set at a solution (replaces nothing in the
 * reference, which always solves with every row: Distributed_opt/dist_scvx_3d.py:93-107).  For every
 * local agent i, node t < K-1 and every j != i of X_all (the linearisation point):
 *     v = (2R - |pbar_i - pbar_j|) - g_ij' (p_t - pbar_i) - S_t,   g_ij = (pbar_i - pbar_j)/|.|
 * with p_t = X_new[i][t][0:pos_dim], S_t = slack[i][t].  Outputs viol [N_local][K] = #{j : v > tol}
 * and vmax [N_local][K] = max_j v (0 at t = K-1).  A culled solve (j_max < N_total-1) is the
 * reference's solution iff no row is violated: the culled problem is a relaxation of the full one.
 */
int scvx_collision_check_batched(int K, int pos_dim, int n_x, int N_total, const double* X_all, int i0,
                                 int N_local, double R, const double* X_new, const double* slack, double tol,
                                 int32_t* viol, double* vmax, void* stream);

/* ------------------------------------------------------------------------------------------
 * Batched SCvx convex subproblem: the reference's SCProblem (SCvx/optimization/sc_problem.py:15-83)
 * with the constraints of its models (unicycle_model.py:88-114, single_integrator_model.py:80-126)
 * and, when n_nbr > 0, the ADMM terms of AgentSolver (agent_solver.py:78-102, si_agent_solver.py:70-92):
 *
 *   min  w_nu ||nu||_{1,ind} + w_slack sum_{o,k} s'_{o,k} + w_sigma sigma
 *        + sum_j [ sum Lam_j o (p - Y_j) + rho/2 ||p - Y_j||_F^2 + w_coll sum_k S_{j,k} ]
 *   s.t. x_{k+1} = A_k x_k + B_k u_k + C_k u_{k+1} + S_k sigma + z_k + nu_k      (:53-68)
 *        ||X - Xref||_{1,ind} + ||U - Uref||_{1,ind} + |sigma - sigma_ref| <= tr    (:71-74)
 *        sigma >= 0; x_0 = x_init; x_{K-1} = x_final (has_final); u_0 = 0 (pin_u_first);
 *        u_{K-1} = 0 (pin_u_last); ub_lo <= u_k[ub_idx] <= ub_hi; xb_lo <= x_k[xb_idx] <= xb_hi;
 *        ||u_k||_2 <= u_max (has_soc); a_{o,k}'(p_k - c_o) >= r_o - s'_{o,k}, s' >= 0 with
 *        a_{o,k} = (pbar_k - c_o)/(||pbar_k - c_o|| + 1e-6);  a_{j,k}'(p_k - Y_{j,k}) + S_{j,k} >= d_min,
 *        S >= 0 with a_{j,k} = (pbar_k - P_{j,k})/(||pbar_k - P_{j,k}|| + 1e-6) (multi_agent_model.py:61-79),
 * p_k = x_k[0:pos_dim], ||M||_{1,ind} = max_k ||M[:,k]||_1 (the induced norm cvx.norm(M, 1) computes).
 * Solved by a primal-dual interior-point method (Mehrotra, Nesterov-Todd SOC scaling) whose Newton
 * systems go through a Riccati recursion with (sigma, tau_x, tau_u, tau_nu) as augmented states.
 * Supported models: unicycle (n=3, m=2), single integrator (n=3, m=3).  K <= 256.
 * ------------------------------------------------------------------------------------------ */
#define SCVX_MAX_NBR 32

typedef struct scvx_scp_template {
    int32_t model_id;
    int32_t n_x, n_u, K;
    int32_t pos_dim;
    int32_t has_final;      /* X[:,-1] == x_final (requires pin_u_last) */
    int32_t pin_u_first;    /* U[:,0] == 0  */
    int32_t pin_u_last;     /* U[:,-1] == 0 */
    int32_t n_ubound;
    int32_t ub_idx[SCVX_MAX_BOX];
    int32_t ub_has_lo[SCVX_MAX_BOX];
    int32_t ub_has_hi[SCVX_MAX_BOX];
    double ub_lo[SCVX_MAX_BOX];
    double ub_hi[SCVX_MAX_BOX];
    int32_t has_soc;
    double u_max;
    int32_t n_xbound;
    int32_t xb_idx[SCVX_MAX_BOX];
    double xb_lo[SCVX_MAX_BOX];
    double xb_hi[SCVX_MAX_BOX];
    int32_t n_obs;
    double obs_center[SCVX_MAX_OBS][3];
    double obs_radius[SCVX_MAX_OBS];   /* total clearance r_o (obstacle + robot radius [+ margin]) */
    double w_nu, w_slack, w_sigma;
    int32_t n_nbr;
    double rho, d_min, w_coll;
    int32_t max_iter;
    double tol;
    double reg;             /* primal regularisation of the Newton systems (scaled units), e.g. 1e-10 */
    /* Nash best-response terms (scvx_scp_game_solve_batched; zero for SCProblem / AgentSolver) */
    int32_t game;           /* 1: the terms below are active */
    int32_t sigma_fixed;    /* sigma == sigma_ref (agent_best_response.py:77) */
    double w_u2;            /* control_weight       * ||U||_F^2                       (game_model.py:88) */
    double w_du;            /* control_rate_weight  * sum_k ||u_{k+1} - u_k||^2       (:91-93) */
    double w_dth;           /* curvature_weight     * sum_k (x_{k+1}[th] - x_k[th])^2 (:94-96) */
    int32_t theta_idx;      /* state index of th (unicycle 2), -1: no curvature state */
    double w_in;            /* inertia_weight       * ||X - X_prev||_F^2              (:99-100) */
    int32_t n_slab;         /* slab rows z_{j,k}'(p_k - P_{j,k}) >= r_slab per node (:121-124), <= SCVX_MAX_NBR */
    double r_slab;          /* collision_radius */
    /* launch mapping of this template's solves (version 4; version 5 dropped the process-wide default setter):
     * 0 = automatic -- two waves per agent when K > 64 and the launch leaves SIMDs idle (2 N <= 4 x CUs), so the
     * node phases of a K <= 128 agent run in one pass; 1 or 2 waves per agent forced */
    int32_t waves_per_agent;
} scvx_scp_template;

/*
 * Inputs (device, agent-major): disc [N][K-1][n(n+2m+2)], Xref [N][K][n], Uref [N][K][m],
 *   sigma_ref [N], tr [N], x_init [N][n], x_final [N][n],
 *   nbr_pos / nbr_Y / nbr_Lam [N][n_nbr][K][pos_dim]  (neighbour reference positions X_ref_j[0:pd],
 *   consensus Y_j, duals Lambda_j; ignored when n_nbr = 0).
 * Outputs (device): X [N][K][n], U [N][K][m], nu [N][K-1][n], sigma [N], s_obs [N][n_obs][K],
 *   s_nbr [N][n_nbr][K], obj [N] (the reference objective at the solution), status [N], iters [N].
 */
int scvx_scp_solve_batched(const scvx_scp_template* tpl, int N, const double* disc, const double* Xref,
                           const double* Uref, const double* sigma_ref, const double* tr, const double* x_init,
                           const double* x_final, const double* nbr_pos, const double* nbr_Y, const double* nbr_Lam,
                           double* X, double* U, double* nu, double* sigma, double* s_obs, double* s_nbr, double* obj,
                           int32_t* status, int32_t* iters, void* workspace, size_t workspace_bytes, void* stream);

/* Bytes of caller-owned device scratch scvx_scp_solve_batched / scvx_scp_game_solve_batched need for
 * N agents (depends on the game fields: the game kernel carries extra Riccati states). */
size_t scvx_scp_workspace_bytes(const scvx_scp_template* tpl, int N);



/* ------------------------------------------------------------------------------------------
 * Batched Nash best response: AgentBestResponse.setup/solve (SCvx/optimization/agent_best_response.py:
 * 35-113, si_agent_best_response.py:36-127) = the SCProblem above (without ADMM terms) plus the
 * GameUnicycleModel / GameSIModel cost and slab constraints (game_model.py:68-126,
 * game_si_model.py:90-136) and sigma == sigma_ref:
 *
 *   + w_u2 ||U||_F^2 + w_du sum_k ||u_{k+1} - u_k||^2 + w_dth sum_k (th_{k+1} - th_k)^2
 *   + w_in ||X - X_prev||_F^2,      s.t.  z_{j,k}'(p_k - P_{j,k}) >= r_slab   (j < n_slab, every k)
 *
 * The cross-node terms ride on augmented Riccati states u~_k = u_{k-1}, th~_k = th_{k-1}.
 * Extra inputs (device): X_prev [N][K][n] (read when w_in > 0), slab_z / slab_P
 * [N][n_slab][K][pos_dim] (the slab normals z and neighbour positions P).  obj includes the game
 * cost and w_sigma sigma_ref.  Requires tpl->game = 1 and tpl->n_nbr = 0; models as above.
 * ------------------------------------------------------------------------------------------ */
int scvx_scp_game_solve_batched(const scvx_scp_template* tpl, int N, const double* disc, const double* Xref,
                                const double* Uref, const double* sigma_ref, const double* tr,
                                const double* x_init, const double* x_final, const double* X_prev,
                                const double* slab_z, const double* slab_P, double* X, double* U, double* nu,
                                double* sigma, double* s_obs, double* obj, int32_t* status, int32_t* iters,
                                void* workspace, size_t workspace_bytes, void* stream);

/* Slab normals of the ACS dual update (GameUnicycleModel.update_slabs, game_model.py:54-66 /
 * game_si_model.py:69-88): z[a][j][k] = d / ||d|| with d = p[a][k] - P[a][j][k], 0 when ||d|| < 1e-6.
 * p [N][K][n_x] (positions = the first pos_dim states), P [N][n_slab][K][pos_dim], z likewise. */
int scvx_slab_update_batched(int N, int n_slab, int K, int pos_dim, int n_x, const double* p, const double* P,
                             double* z, void* stream);

/* ------------------------------------------------------------------------------------------
 * Batched inter-sample obstacle clearance: SCvx/utils/intersample_collision.py (make_segment_f
 * :104-126, h_i :7-26, find_critical_times :29-67, linearize_h :70-101) for every (agent, segment k,
 * obstacle) of N agents, as called per segment by SCvx/models/game_si_model.py:156-176.
 * For segment k of agent a: x(t) rolls out dx/dtau = f(x, u_k + tau/dt_phys (u_{k+1} - u_k)) from
 * X[a][k] to tau = t dt_phys (dt_phys = seg_dt * sigma[a]; FirstOrderHold._dx); h(t) = ||proj x(t) -
 * c_o|| - r_o; the interior minima t* in (0, dt) of h are located by the reference's scan
 * (num_samples central differences phi with step eps on [eps, dt - eps], bisection to tol, phi2 > 0);
 * at each t*: h0 = h(t*), grad_x = central differences of h w.r.t. x_k, grad_u = 0 (the segment
 * roll-out ignores u_k, as in the reference).
 * ------------------------------------------------------------------------------------------ */
#define SCVX_IS_MAX_PROJ 3
#define SCVX_IS_MAX_STATE 12

typedef struct scvx_intersample_template {
    int32_t model_id;
    int32_t n_obs;
    double obs_center[SCVX_MAX_OBS][SCVX_IS_MAX_PROJ];
    double obs_radius[SCVX_MAX_OBS];
    int32_t proj_rows;                                   /* rows of T (projection), <= 3 */
    double proj[SCVX_IS_MAX_PROJ * SCVX_IS_MAX_STATE];   /* T row-major, row stride SCVX_IS_MAX_STATE */
    double dt;            /* find_critical_times' dt (normalised segment length; the reference passes 1.0) */
    double seg_dt;        /* FirstOrderHold.dt = 1 / (K_foh - 1) */
    double eps;           /* central-difference step (reference 1e-4) */
    double tol;           /* bisection tolerance (reference 1e-6) */
    int32_t num_samples;  /* scan points (reference 100) */
    int32_t max_crit;     /* minima stored per (agent, segment, obstacle) */
    int32_t nsub;         /* RK4 steps per roll-out */
} scvx_intersample_template;

/*
 * Inputs (device): X [N][K][n], U [N][K][m], sigma [N]; params as scvx_foh_batched.
 * Outputs (device): n_crit [N][K-1][n_obs] (minima found; only the first max_crit are stored),
 *   t_crit / h0 [N][K-1][n_obs][max_crit], grad_x [..][max_crit][n], grad_u [..][max_crit][m].
 */
int scvx_intersample_batched(const scvx_intersample_template* tpl, const double* params, int K, int N,
                             const double* X, const double* U, const double* sigma, int32_t* n_crit,
                             double* t_crit, double* h0, double* grad_x, double* grad_u, void* stream);

/* scvx_intersample_batched for a runtime-compiled user model (scvx_rtc_model_create; n_x <= SCVX_IS_MAX_STATE):
 * the same scan on the model's own f, so the inter-sample search of any BaseModel runs on the GPU (the reference's
 * SCvx/utils/intersample_collision.py:104-126 integrates model.get_equations()'s f with odeint for any model).
 * tpl->model_id is ignored; params / n_params as scvx_rtc_foh_batched.  (version 5) */
int scvx_rtc_intersample_batched(const scvx_rtc_model* model, const double* params, int n_params,
                                 const scvx_intersample_template* tpl, int K, int N, const double* X, const double* U,
                                 const double* sigma, int32_t* n_crit, double* t_crit, double* h0, double* grad_x,
                                 double* grad_u, void* stream);

/* ------------------------------------------------------------------------------------------
 * ADMM consensus / dual update of the multi-agent coordinators: replaces the host loop of
 * SCvx/optimization/admm_coordinator.py:80-96 (si_admm_coordinator.py:91-102).  For agent i and
 * neighbour slot s (j = nbr[i][s]), p_j = X_new[j][:, 0:pos_dim]:
 *     Y_new = (Y + p_j) / 2;  Lam += rho (p_j - Y_new);
 *     primal[i][s] = ||p_j - Y_new||_F;  dual[i][s] = ||Y_new - Y||_F   (admm_utils.py:20-38)
 * Device buffers: X_new [N][K][n_x], nbr [N][n_nbr] int32, Y / Lam [N][n_nbr][K][pos_dim] (updated in
 * place; the layout of scvx_scp_solve_batched's nbr_Y / nbr_Lam), primal / dual [N][n_nbr].  The
 * element updates are bit-identical to the reference's numpy expressions.
 */
int scvx_admm_consensus_batched(int N, int n_nbr, int K, int pos_dim, int n_x, const double* X_new,
                                const int32_t* nbr, double rho, double* Y, double* Lam, double* primal,
                                double* dual, void* stream);

/* ------------------------------------------------------------------------------------------
 * Bookkeeping of one Jacobi SCvx iteration with the per-agent trust-region rule (the tensor ops of
 * scvx_hip/scvx.py JacobiSCvx.step, fused): per agent i, (X_out[i], U_out[i]) = (X_sol[i], U_sol[i]) if
 * status[i] != 2, else (X[i], U[i]) (Distributed_opt/dist_scvx_3d.py:113-118; X_out may alias X);
 * cost = sum_{t<K-1} ||U_out[i][t]||^2
 * (cost_fcn, :131-138); tr[i] *= 0.5 if cost > prev_cost[i] (1 + tie_rtol) (:248-252, per agent;
 * tie_rtol >= 0, e.g. 1e-9: successive costs of a converged agent agree only to rounding, so the
 * reference's strict test (tie_rtol = 0) would halve on the rounding of the sum); a failed agent's
 * radius then halves (grow = 0) or doubles (grow = 1; every radius is then capped at tr_max);
 * prev_cost[i] = cost.
 * Device buffers: status [N] int32, X_sol / X / X_out [N][K][n_x], U_sol / U / U_out [N][K][n_u],
 * tr / prev_cost [N] (updated in place).
 */
int scvx_jacobi_update_batched(int N, int K, int n_x, int n_u, const int32_t* status, const double* X_sol,
                               const double* U_sol, const double* X, const double* U, double* X_out, double* U_out,
                               double* tr, double* prev_cost, int grow, double tr_max, double tie_rtol,
                               void* stream);

/*
 * The same bookkeeping under the reference's GLOBAL trust-region rule (Distributed_opt/dist_scvx_3d.py:242-252:
 * one radius, halved when the summed cost_fcn rises; ABI 6), in two calls:
 *   scvx_jacobi_update_costs_batched: X_out / U_out as scvx_jacobi_update_batched, cost[i] = sum_{t<K-1}
 *     ||U_out[i][t]||^2; the radii are not touched.
 *   scvx_jacobi_global_rule: total = sum_i cost[i] (fixed summation order); mode 0 writes it to total_out only (a
 *     rank's share, to be all-reduced by the caller), mode 1 sums and applies, mode 2 applies *total_in (the
 *     all-reduced total).  Apply: tr[i] *= 0.5 for every agent if total > *prev_total (the reference's strict test),
 *     then a failed agent's radius halves (grow = 0) or doubles (grow = 1, capped at tr_max); *prev_total = total
 *     (and *total_out when given).
 * Device buffers: cost / tr [N], status [N] int32, total_in / total_out / prev_total one double each.
 */
int scvx_jacobi_update_costs_batched(int N, int K, int n_x, int n_u, const int32_t* status, const double* X_sol,
                                     const double* U_sol, const double* X, const double* U, double* X_out,
                                     double* U_out, double* cost, void* stream);
int scvx_jacobi_global_rule(int N, int mode, const int32_t* status, const double* cost, const double* total_in,
                            double* total_out, double* tr, double* prev_total, int grow, double tr_max, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SCVX_HIP_H */
