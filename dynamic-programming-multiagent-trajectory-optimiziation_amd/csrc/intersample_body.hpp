// Inter-sample obstacle clearance kernel body, templated on the model (gfx950, float64).
//
// Shared by the built-in models (csrc/intersample.hip, compiled with the library) and by runtime-compiled user
// models (csrc/foh_rtc.hip: embedded as text and compiled by hipRTC next to the model's f), so the scan of any
// BaseModel runs the same arithmetic -- the reference's scan is model-agnostic (it integrates
// model.get_equations()'s f with odeint, SCvx/utils/intersample_collision.py:104-126).
//
// Replaces, for every (agent, segment k, obstacle) at once, the reference's per-segment Python loop
// of SCvx/models/game_si_model.py:156-176 over SCvx/utils/intersample_collision.py:
//   make_segment_f (:104-126)      x(t) = roll-out of dx/dtau = f(x, u0 + tau/dt_phys (u1 - u0)) from
//                                  x_k over tau in [0, t dt_phys], dt_phys = dt_foh * sigma
//                                  (FirstOrderHold._dx, first_order_hold.py:157-162);
//   h_i (:7-26)                    h(t) = ||T x(t) - c|| - r;
//   find_critical_times (:29-67)   phi = central difference of h (step eps) on num_samples points of
//                                  [eps, dt - eps]; bisection (<= 30 halvings, |b - a| < tol) on every
//                                  bracket with phi_i == 0 or a sign change; keep roots in (0, dt)
//                                  with phi2 > 0 (central difference of phi);
//   linearize_h (:70-101)          h0 and central-difference gradients w.r.t. x_k and u_k (the segment
//                                  roll-out ignores its u argument, so grad_u is identically 0, as in
//                                  the reference).
// The reference integrates with LSODA (odeint, rtol = atol = 1.49e-8); here each roll-out is fixed-step
// RK4 with nsub steps (exact for the single integrator, whose x(t) is quadratic).
//
// Mapping: one lane per (agent, k, obstacle); everything a lane needs (x_k, u_k, u_{k+1}, T, the
// obstacle) sits in registers, each roll-out restarts from x_k (the reference's semantics: odeint
// from 0 to t for every evaluation).  Lanes of a wave take consecutive obstacles / segments of one
// agent, so the loads of x_k, u_k are broadcast-friendly; there is no inter-lane communication.
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>

#include <cmath>
#endif

#include "foh_body.hpp"   // ModelParams
#include "scvx_hip.h"     // scvx_intersample_template

namespace scvx {

struct ISArgs {
    scvx_intersample_template T;
    int K, N;
    const double *X, *U, *sigma;
    int32_t* n_crit;
    double *t_crit, *h0, *grad_x, *grad_u;
    ModelParams P;
};

// One lane per (agent, segment k, obstacle); blockDim.x == 256 (the launchers' block).
template <class Mdl>
__device__ __forceinline__ void intersample_body(const ISArgs& a) {
    constexpr int n = Mdl::N, m = Mdl::M;
    static_assert(n <= SCVX_IS_MAX_STATE, "the projection rows hold SCVX_IS_MAX_STATE states");
    const auto& T = a.T;
    const int O = T.n_obs;
    const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long nwork = (long long)a.N * (a.K - 1) * O;
    if (tid >= nwork) return;
    const int o = (int)(tid % O);
    const long long seg = tid / O;  // agent * (K-1) + k
    const long long agent = seg / (a.K - 1);
    const int k = (int)(seg % (a.K - 1));
    double xk[n], u0[m], du[m];
#pragma unroll
    for (int i = 0; i < n; ++i) xk[i] = a.X[(agent * a.K + k) * n + i];
#pragma unroll
    for (int j = 0; j < m; ++j) {
        u0[j] = a.U[(agent * a.K + k) * m + j];
        du[j] = a.U[(agent * a.K + k + 1) * m + j] - u0[j];
    }
    const double dtp = T.seg_dt * a.sigma[agent];  // dt_phys of make_segment_f
    const int pd = T.proj_rows;
    double c[SCVX_IS_MAX_PROJ];
    for (int i = 0; i < pd; ++i) c[i] = T.obs_center[o][i];
    const double r = T.obs_radius[o];
    const int nsub = T.nsub;

    // h(x0, t): roll-out to tau = t * dtp, projection, clearance
    auto h = [&](const double* x0, double t) -> double {
        double x[n];
#pragma unroll
        for (int i = 0; i < n; ++i) x[i] = x0[i];
        const double hs = t * dtp / nsub;
        auto fx = [&](double tau, const double* xs, double* out) {
            double u[m];
            const double w = tau / dtp;
#pragma unroll
            for (int j = 0; j < m; ++j) u[j] = u0[j] + w * du[j];
            Mdl::f(xs, u, out, a.P);
        };
        for (int s = 0; s < nsub; ++s) {
            const double tau = s * hs;
            double kk[n], acc[n], xt[n];
            fx(tau, x, kk);
#pragma unroll
            for (int i = 0; i < n; ++i) { acc[i] = kk[i]; xt[i] = x[i] + 0.5 * hs * kk[i]; }
            fx(tau + 0.5 * hs, xt, kk);
#pragma unroll
            for (int i = 0; i < n; ++i) { acc[i] += 2.0 * kk[i]; xt[i] = x[i] + 0.5 * hs * kk[i]; }
            fx(tau + 0.5 * hs, xt, kk);
#pragma unroll
            for (int i = 0; i < n; ++i) { acc[i] += 2.0 * kk[i]; xt[i] = x[i] + hs * kk[i]; }
            fx(tau + hs, xt, kk);
#pragma unroll
            for (int i = 0; i < n; ++i) x[i] += (hs / 6.0) * (acc[i] + kk[i]);
        }
        double d2 = 0.0;
        for (int i = 0; i < pd; ++i) {
            double p = -c[i];
#pragma unroll
            for (int j = 0; j < n; ++j) p += T.proj[i * SCVX_IS_MAX_STATE + j] * x[j];
            d2 += p * p;
        }
        return sqrt(d2) - r;
    };
    const double eps = T.eps;
    auto phi = [&](double t) -> double { return (h(xk, t + eps) - h(xk, t - eps)) / (2.0 * eps); };

    const long long slot = seg * O + o;
    const int MC = T.max_crit;
    int found = 0;
    // sample grid ts = linspace(eps, dt - eps, num_samples)
    const int ns = T.num_samples;
    const double t0 = eps, t1 = T.dt - eps;
    const double step = ns > 1 ? (t1 - t0) / (ns - 1) : 0.0;
    auto ts = [&](int i) -> double { return (i == ns - 1) ? t1 : t0 + i * step; };
    double pc = phi(ts(0));
    for (int i = 0; i + 1 < ns; ++i) {
        const double pn = phi(ts(i + 1));
        if (pc == 0.0 || pc * pn < 0.0) {
            double lo = ts(i), hi = ts(i + 1);
            for (int it = 0; it < 30; ++it) {
                const double mid = 0.5 * (lo + hi);
                if (phi(lo) * phi(mid) <= 0.0) hi = mid; else lo = mid;
                if (fabs(hi - lo) < T.tol) break;
            }
            const double root = 0.5 * (lo + hi);
            const double p2 = (phi(root + eps) - phi(root - eps)) / (2.0 * eps);
            if (root > 0.0 && root < T.dt && p2 > 0.0) {
                if (found < MC) {
                    const long long q = slot * MC + found;
                    a.t_crit[q] = root;
                    a.h0[q] = h(xk, root);
                    double xp[n];
#pragma unroll
                    for (int j = 0; j < n; ++j) xp[j] = xk[j];
                    for (int j = 0; j < n; ++j) {
                        xp[j] = xk[j] + eps;
                        const double hp = h(xp, root);
                        xp[j] = xk[j] - eps;
                        const double hm = h(xp, root);
                        xp[j] = xk[j];
                        a.grad_x[q * n + j] = (hp - hm) / (2.0 * eps);
                    }
#pragma unroll
                    for (int j = 0; j < m; ++j) a.grad_u[q * m + j] = 0.0;
                }
                ++found;
            }
        }
        pc = pn;
    }
    a.n_crit[slot] = found;
}


#ifndef __HIPCC_RTC__
// host-side checks shared by scvx_intersample_batched and scvx_rtc_intersample_batched: nullptr when valid
inline const char* intersample_check(const scvx_intersample_template& T, int K, int N, int n_x) {
    if (K < 2 || N < 0) return "intersample: bad template / sizes";
    if (n_x > SCVX_IS_MAX_STATE) return "intersample: n_x > SCVX_IS_MAX_STATE";
    if (T.n_obs < 0 || T.n_obs > SCVX_MAX_OBS) return "intersample: n_obs";
    if (T.proj_rows < 1 || T.proj_rows > SCVX_IS_MAX_PROJ) return "intersample: proj_rows";
    if (T.num_samples < 2 || T.max_crit < 1 || T.nsub < 1 || !(T.eps > 0.0) || !(T.dt > 2.0 * T.eps) ||
        !(T.seg_dt > 0.0) || !(T.tol > 0.0))
        return "intersample: num_samples / max_crit / nsub / eps / dt / seg_dt / tol";
    return nullptr;
}
#endif

}  // namespace scvx
