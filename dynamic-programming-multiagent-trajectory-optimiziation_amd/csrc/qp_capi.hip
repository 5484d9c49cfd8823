// C-ABI of the batched trust-region QP (include/scvx_hip.h): argument checks, row-capacity class
// selection (qp_caps.hpp), workspace sizing and the launch of the matching qp_ipm_kernel
// instantiation (qp_inst_*.hip).
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "qp_caps.hpp"
#include "qp_ipm.hpp"
#include "scvx_hip.h"
#include "subproblem_rtc.hpp"

namespace scvx {
int qp_launch_di(int idx, const QPArgs& a, hipStream_t st);
int qp_launch_unicycle(int idx, const QPArgs& a, hipStream_t st);
int qp_launch_si(int idx, const QPArgs& a, hipStream_t st);
int qp_launch_quad(int idx, const QPArgs& a, hipStream_t st);
}  // namespace scvx

using namespace scvx;

namespace {
double* g_trace = nullptr;
int g_trace_agent = 0, g_trace_cap = 0;

constexpr int kCapsDI[] = {SCVX_CAPS_DI};
constexpr int kCapsUni[] = {SCVX_CAPS_UNICYCLE};
constexpr int kCapsSI[] = {SCVX_CAPS_SI};
constexpr int kCapsQuad[] = {SCVX_CAPS_QUAD};

struct ModelTable {
    int nx, nu;
    const int* caps;
    int ncaps;
    int (*launch)(int, const QPArgs&, hipStream_t);
};

// model table entry for the template (nullptr: unknown model / dimensions)
const ModelTable* model_of(const scvx_qp_template& T) {
    static const ModelTable tab[] = {
        {6, 3, kCapsDI, (int)(sizeof(kCapsDI) / sizeof(int) / QP_CAPS_W), qp_launch_di},
        {3, 2, kCapsUni, (int)(sizeof(kCapsUni) / sizeof(int) / QP_CAPS_W), qp_launch_unicycle},
        {3, 3, kCapsSI, (int)(sizeof(kCapsSI) / sizeof(int) / QP_CAPS_W), qp_launch_si},
        {12, 4, kCapsQuad, (int)(sizeof(kCapsQuad) / sizeof(int) / QP_CAPS_W), qp_launch_quad},
    };
    const int ids[] = {SCVX_MODEL_DOUBLE_INTEGRATOR, SCVX_MODEL_UNICYCLE, SCVX_MODEL_SINGLE_INTEGRATOR, SCVX_MODEL_QUADROTOR};
    for (int i = 0; i < 4; ++i)
        if (T.model_id == ids[i] && T.n_x == tab[i].nx && T.n_u == tab[i].nu) return &tab[i];
    return nullptr;
}

// the kernel class of a template: a compiled row-capacity class of a built-in model (mt, cls), or -- for
// model_id = SCVX_MODEL_RUNTIME -- the exact class (n_x, n_u, n_box, n_obs, j_max, VC) compiled at run time
struct QPClass {
    const ModelTable* mt = nullptr;
    int cls = -1;
    bool rt = false;
    int nx = 0, nu = 0, nb = 0, no = 0, nc = 0, vc = 0;
};

// validates the template; on success sets the class
int qp_check(const scvx_qp_template* T, int N, QPClass& c) {
    if (!T || N < 0) return set_error(SCVX_EINVAL, "qp: null template");
    if (T->K < 2 || T->K > WAVE) return set_error(SCVX_EUNSUPPORTED, "qp: K must be in [2, 64]");
    if (T->pos_dim < 1 || T->pos_dim > 3 || T->pos_dim > T->n_x) return set_error(SCVX_EINVAL, "qp: pos_dim");
    if (T->n_box < 0 || T->n_box > SCVX_MAX_BOX || T->n_obs < 0 || T->n_obs > SCVX_MAX_OBS || T->j_max < 0)
        return set_error(SCVX_EINVAL, "qp: box/obstacle/collision counts");
    for (int b = 0; b < T->n_box; ++b)
        if (T->box_idx[b] < 0 || T->box_idx[b] >= T->n_x) return set_error(SCVX_EINVAL, "qp: box index");
    if (T->max_iter < 1) return set_error(SCVX_EINVAL, "qp: max_iter");
    if (T->w_nu < 0.0 || T->w_prox < 0.0) return set_error(SCVX_EINVAL, "qp: w_nu / w_prox must be >= 0");
    c = QPClass{};
    c.nx = T->n_x; c.nu = T->n_u;
    if (T->model_id == SCVX_MODEL_RUNTIME) {
        // the kernel's limits (subproblem_rtc.hpp, shared with scvx_rtc_subproblem_compile)
        if (const char* bad = rtc_qp_class_error(T->n_x, T->n_u, T->n_box, T->n_obs, T->j_max, T->w_nu > 0.0 ? 1 : 0,
                                                 T->K))
            return set_error(SCVX_EUNSUPPORTED, bad);
        c.rt = true;
        c.nb = T->n_box; c.no = T->n_obs; c.nc = T->j_max; c.vc = T->w_nu > 0.0 ? 1 : 0;
        return SCVX_OK;
    }
    c.mt = model_of(*T);
    if (!c.mt) return set_error(SCVX_EUNSUPPORTED, "qp: model id / dimensions");
    c.cls = qp_pick_caps(c.mt->caps, c.mt->ncaps, *T);
    if (c.cls < 0)
        return set_error(SCVX_EUNSUPPORTED, T->w_nu > 0.0
            ? "qp: no virtual-control class for this model / row counts (w_nu > 0: quad n_box <= 4, n_obs <= 16, j_max <= 32; di n_box <= 2, n_obs <= 8, no coupling)"
            : "qp: more box / obstacle / collision rows than the largest capacity class (j_max <= 32, n_obs <= 16)");
    const int* cp = c.mt->caps + QP_CAPS_W * c.cls;
    c.nb = cp[0]; c.no = cp[1]; c.nc = cp[2]; c.vc = cp[3];
    return SCVX_OK;
}

size_t ws_bytes(const QPClass& c, int N, int K) {
    const int nv = c.vc ? c.nx : 0, ns = c.no + c.nc, ng = c.no + (c.nc > 0 ? 1 : 0);
    return sizeof(double) * (size_t)N * (size_t)qp_ws_doubles(c.nx, c.nu, c.nb, ns, ng, K, nv, c.nc);
}
}  // namespace

// Diagnostics hook (not part of the solve contract): subsequent scvx_qp_solve_batched launches write
// 8 doubles per IPM iteration of agent `agent` into the device buffer (pres, dres, gap, pobj,
// alpha_aff, alpha, sigma, mu), then 4 doubles (factor cycles, solve cycles, total cycles, fail code).
// agent < 0: one double per agent instead, its exit code (0 converged, 1 start-point factorization,
// 2 terminal Schur complement, 3 non-finite residual, 4 non-finite direction, 5 iteration cap,
// 6 stall at reduced accuracy).
extern "C" int scvx_qp_set_trace(double* buf, int agent, int cap) {
    g_trace = buf; g_trace_agent = agent; g_trace_cap = buf ? cap : 0;
    return SCVX_OK;
}

extern "C" size_t scvx_qp_workspace_bytes(const scvx_qp_template* tpl, int N) {
    QPClass c;
    if (N <= 0 || qp_check(tpl, N, c) != SCVX_OK) return 0;
    return ws_bytes(c, N, tpl->K);
}

extern "C" int scvx_qp_solve_batched_ordered(const scvx_qp_template* tpl, int N, const double* disc,
                                             const double* sigma, const double* Xref, const double* Uref,
                                             const double* x_init, const double* x_final, const double* tr,
                                             const double* coll_rows, const int32_t* coll_count, double* X, double* U,
                                             double* slack_coll, double* nu, double* obj, int32_t* status,
                                             int32_t* iters, const int32_t* warm, const int32_t* order,
                                             void* workspace, size_t workspace_bytes, void* stream) {
    QPClass c;
    int rc = qp_check(tpl, N, c);
    if (rc != SCVX_OK) return rc;
    if (N == 0) return SCVX_OK;
    if (!disc || !sigma || !Xref || !Uref || !x_init || !tr || !X || !U || !slack_coll || !obj || !status || !iters)
        return set_error(SCVX_EINVAL, "qp: null buffer");
    if ((tpl->has_final || tpl->w_final > 0.0) && !x_final) return set_error(SCVX_EINVAL, "qp: x_final required");
    if (tpl->w_final < 0.0 || (tpl->w_final > 0.0 && tpl->has_final))
        return set_error(SCVX_EINVAL, "qp: w_final > 0 (soft terminal) needs has_final = 0");
    if (tpl->j_max > 0 && (!coll_rows || !coll_count)) return set_error(SCVX_EINVAL, "qp: collision rows required");
    if (tpl->w_nu > 0.0 && !nu) return set_error(SCVX_EINVAL, "qp: nu output required (w_nu > 0)");
    if (warm && tpl->K < 2 * tpl->n_x) return set_error(SCVX_EUNSUPPORTED, "qp: warm start needs K >= 2 n_x");
    const size_t need = ws_bytes(c, N, tpl->K);
    if (!workspace || workspace_bytes < need) return set_error(SCVX_EWORKSPACE, "qp: workspace too small");
    QPArgs a{};
    a.T = *tpl;
    a.N = N;
    a.disc = disc; a.sigma = sigma; a.Xref = Xref; a.Uref = Uref; a.x_init = x_init; a.x_final = x_final;
    a.tr = tr; a.coll_rows = coll_rows; a.coll_count = coll_count; a.warm = warm;
    a.X = X; a.U = U; a.slack_coll = slack_coll; a.nu = nu; a.obj = obj; a.status = status; a.iters = iters;
    a.ws = (double*)workspace;
    a.ws_agent = (long long)(need / sizeof(double) / (size_t)N);
    a.trace = g_trace; a.trace_agent = g_trace_agent; a.trace_cap = g_trace_cap;
    a.order = order;
    if (c.rt) return rtc_qp_launch(a, c.nb, c.no, c.nc, c.vc, (hipStream_t)stream);
    return c.mt->launch(c.cls, a, (hipStream_t)stream);
}

extern "C" int scvx_qp_solve_batched(const scvx_qp_template* tpl, int N, const double* disc, const double* sigma,
                                     const double* Xref, const double* Uref, const double* x_init,
                                     const double* x_final, const double* tr, const double* coll_rows,
                                     const int32_t* coll_count, double* X, double* U, double* slack_coll,
                                     double* nu, double* obj, int32_t* status, int32_t* iters,
                                     const int32_t* warm, void* workspace,
                                     size_t workspace_bytes, void* stream) {
    return scvx_qp_solve_batched_ordered(tpl, N, disc, sigma, Xref, Uref, x_init, x_final, tr, coll_rows, coll_count,
                                         X, U, slack_coll, nu, obj, status, iters, warm, nullptr, workspace,
                                         workspace_bytes, stream);
}
