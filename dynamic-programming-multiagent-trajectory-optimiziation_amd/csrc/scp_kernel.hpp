// SCP kernel (device code and the layout shared with the host) -- see csrc/scp_ipm.hip for the C-ABI.
// Batched SCvx convex subproblem (SCProblem / AgentSolver) for MI355X (gfx950), float64.
//
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
// Also compiled at run time for user models (csrc/subproblem_rtc.hip embeds this file): no host-only header
// below is visible to hipRTC.
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>

#include <cmath>
#endif

#include "scvx_hip.h"
#include "wave_ops.hpp"

// end-game step fraction (see the step rule in the iteration)
constexpr double SCP_TAU_END = 0.99999;

#if defined(__HIPCC_RTC__) && !defined(INFINITY)
#define INFINITY __builtin_huge_valf()
#endif

namespace scvx {


constexpr int SCP_NG = 4;
constexpr int SCP_KMAX = 256;

struct SCPArgs {
    scvx_scp_template T;
    int N;
    const double *disc, *Xref, *Uref, *sigma_ref, *tr, *x_init, *x_final, *nbr_pos, *nbr_Y, *nbr_Lam;
    const double *X_prev, *slab_z, *slab_P;  // Nash best response (T.game)
    double *X, *U, *nu, *sigma, *s_obs, *s_nbr, *obj;
    int32_t *status, *iters;
    double* ws;
    long long ws_agent;
};

// node-block layout (doubles); counts are runtime (rows depend on the template)
struct SCPLay {
    int RH, NS, Q, RL, ROWS, stride;
    int o_rows, o_q, o_P, o_At, o_Bt, o_ct, o_z, o_sig, o_s, o_lam, o_wl, o_sw, o_lt, o_H, o_f, o_rd, o_rc, o_rsig,
        o_t, o_rho, o_rhs, o_dz, o_dsig, o_ds, o_dl, o_dsa, o_dla, o_y, o_yp, o_rp, o_K, o_Pr, o_pv, o_kv, o_LD, o_nh,
        o_zb, o_sgb, o_Acl, o_g, o_w, o_e;
};

// augmented game states: u~_k = u_{k-1} (m), th~_k = th_{k-1} (1 when the model has a heading)
__host__ __device__ inline int scp_ne(const scvx_scp_template& T) {
    return T.game ? T.n_u + (T.theta_idx >= 0 ? 1 : 0) : 0;
}

__host__ __device__ inline SCPLay scp_layout(const scvx_scp_template& T) {
    const int n = T.n_x, m = T.n_u;
    const int NXA = n + SCP_NG + scp_ne(T), NUA = m + n, NZ = NXA + NUA;
    SCPLay L{};
    int sides = 0;
    for (int b = 0; b < T.n_ubound; ++b) sides += (T.ub_has_lo[b] ? 1 : 0) + (T.ub_has_hi[b] ? 1 : 0);
    L.RH = (1 << n) + (1 << m) + (1 << n) + sides + 2 * T.n_xbound + 3 + (T.game ? T.n_slab : 0);
    L.NS = T.n_obs + T.n_nbr;
    L.Q = T.has_soc ? m + 1 : 0;
    L.RL = L.RH + 2 * L.NS + L.Q;
    L.ROWS = L.RH + L.NS + L.Q;
    int o = 0;
    auto take = [&](int sz) { const int r = o; o += sz; return r; };
    L.o_rows = take(L.ROWS * (NZ + 1));
    L.o_q = take(NZ);
    L.o_P = take(NZ * NZ);
    L.o_At = take(NXA * NXA);
    L.o_Bt = take(NXA * NUA);
    L.o_ct = take(NXA);
    L.o_z = take(NZ);
    L.o_sig = take(L.NS);
    L.o_s = take(L.RL);
    L.o_lam = take(L.RL);
    L.o_wl = take(L.RH + 2 * L.NS);
    L.o_sw = take(L.Q + 1);
    L.o_lt = take(L.RL);
    L.o_H = take(NZ * NZ);
    L.o_f = take(NZ);
    L.o_rd = take(NZ);
    L.o_rc = take(L.RL);
    L.o_rsig = take(L.NS);
    L.o_t = take(L.RL);
    L.o_rho = take(L.RL);
    L.o_rhs = take(L.NS);
    L.o_dz = take(NZ);
    L.o_dsig = take(L.NS);
    L.o_ds = take(L.RL);
    L.o_dl = take(L.RL);
    L.o_dsa = take(L.RL);
    L.o_dla = take(L.RL);
    L.o_y = take(NXA);
    L.o_yp = take(NXA);
    L.o_rp = take(NXA);
    L.o_K = take(NUA * NXA);
    L.o_Pr = take(NXA * NXA);
    L.o_pv = take(NXA);
    L.o_kv = take(NUA);
    L.o_LD = take(NUA * NUA);
    L.o_nh = take(1);
    L.o_zb = take(NZ);       // best iterate (z, soft slacks) once the reduced tolerances hold
    L.o_sgb = take(L.NS);
    L.o_Acl = take(NXA * NXA);  // closed-loop Acl = At + Bt K (row-major), LQ chain offsets g, w, e
    L.o_g = take(NXA);
    L.o_w = take(NXA);
    L.o_e = take(NXA);
    L.stride = (o + 7) & ~7;
    if (L.stride < 64) L.stride = 64;  // the junk block after the K node blocks holds one slot per lane
    return L;
}

// LDL' of a small symmetric block in registers, pivots clamped at rel * max|diag| (the dynamic
// regularisation of oracle/scp_cpu.py:ldl_solve); Lm holds L below the diagonal and 1/d on it.
template <int D>
__device__ __forceinline__ void ldl_factor(double (&Lm)[D * D], int nn) {
    double dmax = 0.0;
    for (int j = 0; j < nn; ++j) dmax = fmax(dmax, fabs(Lm[j * D + j]));
    const double dmin = 1e-13 * dmax + 1e-300;
    double dg[D];
    for (int j = 0; j < nn; ++j) {
        double d = Lm[j * D + j];
        for (int k = 0; k < j; ++k) d -= Lm[j * D + k] * Lm[j * D + k] * dg[k];
        d = d > dmin ? d : dmin;
        dg[j] = d;
        const double inv = 1.0 / d;
        for (int i = j + 1; i < nn; ++i) {
            double v = Lm[i * D + j];
            for (int k = 0; k < j; ++k) v -= Lm[i * D + k] * Lm[j * D + k] * dg[k];
            Lm[i * D + j] = v * inv;
        }
        Lm[j * D + j] = inv;
    }
}
template <int D>
__device__ __forceinline__ void ldl_solve(const double (&Lm)[D * D], int nn, double (&x)[D]) {
    for (int i = 0; i < nn; ++i)
        for (int k = 0; k < i; ++k) x[i] -= Lm[i * D + k] * x[k];
    for (int i = 0; i < nn; ++i) x[i] *= Lm[i * D + i];
    for (int i = nn - 1; i >= 0; --i)
        for (int k = i + 1; k < nn; ++k) x[i] -= Lm[k * D + i] * x[k];
}

// keep a value opaque to the optimiser: per-sweep decoded offsets derived from it are then computed
// where the sweep starts instead of being hoisted out of the IPM loop (and held live across it)
__device__ __forceinline__ int scp_opaque(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

// ---- second-order cone algebra (dimension Q = m + 1 <= 4), hyperbolic-rotation NT scaling
template <int QM>
struct Soc {
    // W v and W^-1 v from (w, eta)
    __device__ __forceinline__ static void wmul(const double* w, double eta, const double* vin, double* out, int Q, bool inv) {
        double v[QM];
        for (int i = 0; i < Q; ++i) v[i] = vin[i];
        double w1v1 = 0.0;
        for (int i = 1; i < Q; ++i) w1v1 += w[i] * v[i];
        const double sgn = inv ? -1.0 : 1.0;
        const double sc = inv ? 1.0 / eta : eta;
        out[0] = sc * (w[0] * v[0] + sgn * w1v1);
        const double c = sgn * v[0] + w1v1 / (1.0 + w[0]);
        for (int i = 1; i < Q; ++i) out[i] = sc * (v[i] + c * w[i]);
    }
    __device__ __forceinline__ static void nt(const double* s, const double* z, double* w, double& eta, int Q) {
        double js = s[0] * s[0], jz = z[0] * z[0];
        for (int i = 1; i < Q; ++i) { js -= s[i] * s[i]; jz -= z[i] * z[i]; }
        const double rs = 1.0 / sqrt(js), rz = 1.0 / sqrt(jz);
        double sz = 0.0;
        for (int i = 0; i < Q; ++i) sz += s[i] * rs * z[i] * rz;
        const double gam = sqrt(0.5 * (1.0 + sz));
        const double ig = 0.5 / gam;
        w[0] = (s[0] * rs + z[0] * rz) * ig;
        for (int i = 1; i < Q; ++i) w[i] = (s[i] * rs - z[i] * rz) * ig;
        eta = sqrt(sqrt(js / jz));
    }
    __device__ __forceinline__ static void jprod(const double* a, const double* b, double* out, int Q) {
        double d = 0.0;
        for (int i = 0; i < Q; ++i) d += a[i] * b[i];
        const double a0 = a[0], b0 = b[0];
        for (int i = 1; i < Q; ++i) out[i] = a0 * b[i] + b0 * a[i];
        out[0] = d;
    }
    __device__ __forceinline__ static void jdiv(const double* x, const double* r, double* out, int Q) {
        double d = x[0] * x[0], xr = x[0] * r[0];
        for (int i = 1; i < Q; ++i) { d -= x[i] * x[i]; xr -= x[i] * r[i]; }
        const double r0 = xr / d;
        for (int i = 1; i < Q; ++i) out[i] = (r[i] - r0 * x[i]) / x[0];
        out[0] = r0;
    }
    __device__ __forceinline__ static double step(const double* x, const double* dx, int Q) {
        double qa = dx[0] * dx[0], qb = x[0] * dx[0], qc = x[0] * x[0];
        for (int i = 1; i < Q; ++i) { qa -= dx[i] * dx[i]; qb -= x[i] * dx[i]; qc -= x[i] * x[i]; }
        qb *= 2.0;
        double a = INFINITY;
        if (fabs(qa) > 1e-300) {
            const double disc = qb * qb - 4.0 * qa * qc;
            if (disc >= 0.0) {
                const double sq = sqrt(disc);
                const double r1 = (-qb - sq) / (2.0 * qa), r2 = (-qb + sq) / (2.0 * qa);
                if (r1 > 0.0 && x[0] + r1 * dx[0] >= -1e-14) a = fmin(a, r1);
                if (r2 > 0.0 && x[0] + r2 * dx[0] >= -1e-14) a = fmin(a, r2);
            }
        } else if (qb != 0.0 && -qc / qb > 0.0) {
            a = fmin(a, -qc / qb);
        }
        if (dx[0] < 0.0) a = fmin(a, -x[0] / dx[0]);
        return a;
    }
    __device__ __forceinline__ static double mineig(const double* x, int Q) {
        double nr = 0.0;
        for (int i = 1; i < Q; ++i) nr += x[i] * x[i];
        return x[0] - sqrt(nr);
    }
};

// ---- hot row loops of the node phases, as functions with __restrict__ operands: inlined, the
// parameters' noalias becomes scoped alias metadata, so the compiler may move the next row's loads
// above this row's stores (the layout offsets are runtime values and would otherwise alias) and
// unroll with the loads of several rows in flight.  Arithmetic and accumulation order are unchanged.
// residual, hard rows: rd += a_r l_r, rc_r = a_r z + s_r - h_r
template <int NZ>
__device__ __forceinline__ void rows_residual(const double* __restrict__ rows, const double* __restrict__ lam,
                                              const double* __restrict__ sl, double* __restrict__ rc, int nh,
                                              const double (&z)[NZ], double (&rd)[NZ], double& presl, double& gapl) {
    constexpr int RS = NZ + 1;
    #pragma unroll 2
    for (int r = 0; r < nh; ++r) {
        const double* ar = rows + r * RS;
        const double l = lam[r], s = sl[r];
        #pragma unroll
        for (int i = 0; i < NZ; ++i) rd[i] += ar[i] * l;
        double v = 0.0;
        #pragma unroll
        for (int i = 0; i < NZ; ++i) v += ar[i] * z[i];
        const double rcv = v + s - ar[NZ];
        rc[r] = rcv;
        presl = fmax(presl, fabs(rcv));
        gapl += s * l;
    }
}
// direction, LP rows: rho = rcomp / lt, t = rho / wl + rc / wl^2 (stored); f += a_r t_r on hard rows
template <int NZ>
__device__ __forceinline__ void rows_direction(const double* __restrict__ rows, const double* __restrict__ lt_,
                                               const double* __restrict__ wl_, const double* __restrict__ dsa,
                                               const double* __restrict__ dla, const double* __restrict__ rc,
                                               double* __restrict__ rho_, double* __restrict__ t_, int r0, int r1,
                                               bool hard, bool corr, double sgmu, double (&f)[NZ]) {
    constexpr int RS = NZ + 1;
    #pragma unroll 2
    for (int r = r0; r < r1; ++r) {
        const double lt = lt_[r], wl = wl_[r];
        double rcv = -lt * lt;
        if (corr) rcv += -(dsa[r] * dla[r]) + sgmu;
        const double rho = rcv / lt;
        const double tv = rho / wl + rc[r] / (wl * wl);
        rho_[r] = rho;
        t_[r] = tv;
        if (hard) {
            const double* ar = rows + r * RS;
            #pragma unroll
            for (int i = 0; i < NZ; ++i) f[i] += ar[i] * tv;
        }
    }
}
// step recovery, hard rows: ds = -rc - a_r dz, dl = rho / wl + (rc + a_r dz) / wl^2, ratio test
template <int NZ>
__device__ __forceinline__ void rows_step(const double* __restrict__ rows, const double* __restrict__ wl_,
                                          const double* __restrict__ rc_, const double* __restrict__ rho_,
                                          const double* __restrict__ sl, const double* __restrict__ lam,
                                          double* __restrict__ ds_, double* __restrict__ dl_, int nh,
                                          const double (&dz)[NZ], double& amax) {
    constexpr int RS = NZ + 1;
    #pragma unroll 2
    for (int r = 0; r < nh; ++r) {
        const double* ar = rows + r * RS;
        double gdz = 0.0;
        #pragma unroll
        for (int i = 0; i < NZ; ++i) gdz += ar[i] * dz[i];
        const double wl = wl_[r], rc = rc_[r];
        const double ds = -rc - gdz;
        const double dl = rho_[r] / wl + (rc + gdz) / (wl * wl);
        ds_[r] = ds;
        dl_[r] = dl;
        if (ds < 0.0) amax = fmin(amax, -sl[r] / ds);
        if (dl < 0.0) amax = fmin(amax, -lam[r] / dl);
    }
}

// LP-row scaling: wl = sqrt(s / l), lt = sqrt(s l) on rows [r0, r1)
__device__ __forceinline__ void rows_scale(const double* __restrict__ sl, const double* __restrict__ lam,
                                           double* __restrict__ wl, double* __restrict__ lt, int r0, int r1) {
    #pragma unroll 4
    for (int r = r0; r < r1; ++r) {
        const double s = sl[r], l = lam[r];
        wl[r] = sqrt(s / l);
        lt[r] = sqrt(s * l);
    }
}
// predictor complementarity sum_r (s + aa ds)(l + aa dl) on rows [r0, r1) (accumulated in row order)
__device__ __forceinline__ void rows_mu(const double* __restrict__ sl, const double* __restrict__ lam,
                                        const double* __restrict__ ds, const double* __restrict__ dl, int r0, int r1,
                                        double aa, double& mual) {
    #pragma unroll 4
    for (int r = r0; r < r1; ++r) mual += (sl[r] + aa * ds[r]) * (lam[r] + aa * dl[r]);
}
// y[r] = x[r] on rows [0, n)
__device__ __forceinline__ void rows_copy2(const double* __restrict__ x1, const double* __restrict__ x2,
                                           double* __restrict__ y1, double* __restrict__ y2, int n) {
    #pragma unroll 4
    for (int r = 0; r < n; ++r) { y1[r] = x1[r]; y2[r] = x2[r]; }
}
// s += al ds, l += al dl on rows [r0, r1)
__device__ __forceinline__ void rows_update(double* __restrict__ sl, double* __restrict__ lam,
                                            const double* __restrict__ ds, const double* __restrict__ dl, int r0,
                                            int r1, double al) {
    #pragma unroll 4
    for (int r = r0; r < r1; ++r) { sl[r] += al * ds[r]; lam[r] += al * dl[r]; }
}

template <int NX, int NU, int NE, int NW>
__global__ __launch_bounds__(64 * NW) void scp_ipm_kernel(SCPArgs a, double* __restrict__ ws_all, const double* __restrict__ disc_all) {
    // workspace and disc come in as kernel pointer arguments (known global address space): read out
    // of the by-value struct they would be FLAT accesses, which also count against lgkmcnt, so every
    // LDS wait would drain the outstanding global loads
    constexpr int NXA = NX + SCP_NG + NE, NUA = NU + NX, NZ = NXA + NUA, RS = NZ + 1;
    constexpr int SIG = NX, TX = NX + 1, TU = NX + 2, TN = NX + 3, E0 = NX + SCP_NG, ZU = NXA, ZN = ZU + NU;
    // game terms (NE > 0): E0..E0+NU-1 = u~, E0+NU = th~ (when T.theta_idx >= 0)
    constexpr int QM = NU + 1;
    const scvx_scp_template& T = a.T;
    __shared__ double sRed[NW];
    // reductions over the agent's threads (result uniform across its waves)
    auto blk_red = [&](double v, int op) -> double {
        v = op == 0 ? wave_sum(v) : (op == 1 ? wave_max(v) : wave_min(v));
        if constexpr (NW > 1) {
            if ((threadIdx.x & (WAVE - 1)) == 0) sRed[threadIdx.x / WAVE] = v;
            __syncthreads();
            double r = sRed[0];
            #pragma unroll
            for (int w = 1; w < NW; ++w) r = op == 0 ? r + sRed[w] : (op == 1 ? fmax(r, sRed[w]) : fmin(r, sRed[w]));
            __syncthreads();
            v = r;
        }
        return v;
    };
    auto blk_sum = [&](double v) { return blk_red(v, 0); };
    auto blk_max = [&](double v) { return blk_red(v, 1); };
    auto blk_min = [&](double v) { return blk_red(v, 2); };
    const bool sfix = NE > 0 && T.sigma_fixed != 0;
    // NW waves per agent: node phases over all NW * 64 threads (thread tid: nodes tid, tid + NT, ...); the
    // sequential sweeps (factor, LQ chains) on wave 0 while the others wait at the next block barrier
    constexpr int NT = NW * WAVE;
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), wid = tid / WAVE;
    const int K = T.K, pd = T.pos_dim;
    const long long agent = blockIdx.x;
    const SCPLay Ly = scp_layout(T);
    const int RH = Ly.RH, NS = Ly.NS, Q = Ly.Q, RL = Ly.RL, NLP = RH + 2 * NS;
    double* ws = ws_all + agent * a.ws_agent;
    auto nb = [&](int t) -> double* { return ws + (long long)t * Ly.stride; };
    // per-lane junk slot after the K node blocks: lanes without an output of their own store there, so
    // every global store of the sweeps is unconditional (a store under a divergent branch makes the
    // compiler's vmcnt accounting fall back to vmcnt(0), draining the next stage's prefetched packet)
    double* const jnk = ws + (long long)K * Ly.stride + lane;
    const double* disc = disc_all + agent * (long long)(K - 1) * (NX * (NX + 2 * NU + 2));
    constexpr int DSTR = NX * (NX + 2 * NU + 2);
    const double trv = a.tr[agent], sref = a.sigma_ref[agent];
    const double* xinit = a.x_init + agent * NX;
    const double* xfin = a.x_final + agent * NX;
    const bool fin = T.has_final != 0;

    __shared__ double sP[NXA * NXA], sPAB[NXA * (NXA + NUA)], sQxx[NXA * NXA], sQuxC[NUA * NXA],
        sQuu[NUA * NUA], sKC[NUA * NXA], sXi[NXA], sMisc[32];
    __shared__ double sPv[NXA], sV[NXA], sQ[NZ], sU[NUA], sXw[2][NXA];  // sweep-form LQ solve (NW = 1)
    // sMisc: 0..NX-1 r_init, 8..8+NX-1 y0+, 16.. scalars
    auto pinned = [&](int t, int i) -> bool {  // i: z index
        if (i >= ZU && i < ZN) return (t == 0 && T.pin_u_first) || (t == K - 1 && T.pin_u_last);
        if (i >= ZN) return t == K - 1 || (fin && t == K - 2);
        return false;
    };
    auto Cprev = [&](int t, int i, int j) -> double {  // C_{t-1}[i][j]
        return t > 0 ? disc[(long long)(t - 1) * DSTR + NX * NX + NX * NU + j * NX + i] : 0.0;
    };

    // ------------------------------------------------------------------ setup (rows, dynamics)
    // objective scale: every cost term / cs (oracle/scp_cpu.py build_nodes)
    double csl = 0.0;
    for (int t = tid; t < K; t += NT) {
        for (int j = 0; j < T.n_nbr; ++j)
            for (int i = 0; i < pd; ++i) {
                const long long o = ((agent * T.n_nbr + j) * K + t) * pd + i;
                csl = fmax(csl, fabs(a.nbr_Lam[o] - T.rho * a.nbr_Y[o]));
            }
    }
    double cs = blk_max(csl);
    cs = fmax(cs, fmax(1.0, fmax(T.w_nu, T.w_sigma)));
    if (T.n_obs > 0) cs = fmax(cs, T.w_slack);
    if (T.n_nbr > 0) cs = fmax(cs, fmax(T.w_coll, T.rho));
    const double ics = 1.0 / cs;
    const double w_obs = T.w_slack * ics, w_col = T.w_coll * ics;
    double hmax = 0.0, qmax = 0.0, degl = 0.0;
    for (int t = tid; t < K; t += NT) {
        double* B = nb(t);
        double xb[NX], ub[NU];
        #pragma unroll
        for (int i = 0; i < NX; ++i) xb[i] = a.Xref[(agent * K + t) * NX + i];
        #pragma unroll
        for (int j = 0; j < NU; ++j) ub[j] = a.Uref[(agent * K + t) * NU + j];
        double Cp[NX * NU];
        #pragma unroll
        for (int i = 0; i < NX; ++i)
            #pragma unroll
            for (int j = 0; j < NU; ++j) Cp[i * NU + j] = Cprev(t, i, j);
        const bool subst = fin && t == K - 2;
        const double* dk = disc + (long long)t * DSTR;  // only read when t < K-1
        // write one row given v-coordinate coefficients
        auto put = [&](int r, double* av, double h) {
            if (subst) {  // nu_{K-2} = x_final - (A x + B u + S sigma + z)   (u_{K-1} pinned at 0)
                double an[NX];
                #pragma unroll
                for (int i = 0; i < NX; ++i) an[i] = av[ZN + i];
                for (int l = 0; l < NX; ++l) {
                    double v = 0.0;
                    #pragma unroll
                    for (int i = 0; i < NX; ++i) v += dk[l * NX + i] * an[i];  // (A' an)_l, A col-major
                    av[l] -= v;
                }
                #pragma unroll
                for (int j = 0; j < NU; ++j) {
                    double v = 0.0;
                    #pragma unroll
                    for (int i = 0; i < NX; ++i) v += dk[NX * NX + j * NX + i] * an[i];
                    av[ZU + j] -= v;
                }
                double sv = 0.0, hz = 0.0;
                #pragma unroll
                for (int i = 0; i < NX; ++i) {
                    sv += dk[NX * NX + 2 * NX * NU + i] * an[i];
                    hz += an[i] * (xfin[i] - dk[NX * NX + 2 * NX * NU + NX + i]);
                    av[ZN + i] = 0.0;
                }
                av[SIG] -= sv;
                h -= hz;
            }
            if (sfix) { h -= av[SIG] * sref; av[SIG] = 0.0; }  // sigma == sigma_ref is data
            // FOH transform: a_u += C_{t-1}' a_x
            #pragma unroll
            for (int j = 0; j < NU; ++j) {
                double v = 0.0;
                #pragma unroll
                for (int i = 0; i < NX; ++i) v += Cp[i * NU + j] * av[i];
                av[ZU + j] += v;
            }
            double* rp = B + Ly.o_rows + r * RS;
            #pragma unroll
            for (int i = 0; i < NZ; ++i) rp[i] = av[i];
            rp[NZ] = h;
            hmax = fmax(hmax, fabs(h));
        };
        double av[NZ];
        auto clr = [&]() { for (int i = 0; i < NZ; ++i) av[i] = 0.0; };
        int r = 0;
        for (int s = 0; s < (1 << NX); ++s) {  // TR facets on x
            clr();
            double h = 0.0;
            #pragma unroll
            for (int i = 0; i < NX; ++i) { const double sg = (s >> (NX - 1 - i)) & 1 ? -1.0 : 1.0; av[i] = sg; h += sg * xb[i]; }
            av[TX] = -1.0;
            put(r++, av, h);
        }
        for (int s = 0; s < (1 << NU); ++s) {  // TR facets on u
            clr();
            double h = 0.0;
            #pragma unroll
            for (int j = 0; j < NU; ++j) { const double sg = (s >> (NU - 1 - j)) & 1 ? -1.0 : 1.0; av[ZU + j] = sg; h += sg * ub[j]; }
            av[TU] = -1.0;
            put(r++, av, h);
        }
        if (t < K - 1)
            for (int s = 0; s < (1 << NX); ++s) {  // ||nu_t||_1 <= tau_nu facets
                clr();
                #pragma unroll
                for (int i = 0; i < NX; ++i) av[ZN + i] = (s >> (NX - 1 - i)) & 1 ? -1.0 : 1.0;
                av[TN] = -1.0;
                put(r++, av, 0.0);
            }
        for (int b = 0; b < T.n_ubound; ++b) {
            const int j = T.ub_idx[b];
            // a bound on a pinned input (u_0 = u_{K-1} = 0) is a constant row; keeping it would give
            // the IPM an empty-interior block (s -> 0, lambda -> inf) whenever the bound is 0
            if (pinned(t, ZU + j)) continue;
            if (T.ub_has_hi[b]) { clr(); av[ZU + j] = 1.0; put(r++, av, T.ub_hi[b]); }
            if (T.ub_has_lo[b]) { clr(); av[ZU + j] = -1.0; put(r++, av, -T.ub_lo[b]); }
        }
        for (int b = 0; b < T.n_xbound; ++b) {
            const int i = T.xb_idx[b];
            clr(); av[i] = 1.0; put(r++, av, T.xb_hi[b]);
            clr(); av[i] = -1.0; put(r++, av, -T.xb_lo[b]);
        }
        if (NE > 0)  // slab rows -z'p_k <= -r - z'P_k (game_model.py:121-124)
            for (int j = 0; j < T.n_slab; ++j) {
                clr();
                const long long base = ((agent * T.n_slab + j) * K + t) * pd;
                double h = -T.r_slab;
                for (int i = 0; i < pd; ++i) { av[i] = -a.slab_z[base + i]; h -= a.slab_z[base + i] * a.slab_P[base + i]; }
                put(r++, av, h);
            }
        if (t == 0) {
            if (sfix) {  // |sigma - sigma_ref| = 0: tau_x + tau_u <= tr
                clr(); av[TX] = 1.0; av[TU] = 1.0; put(r++, av, trv);
            } else {
                clr(); av[SIG] = -1.0; put(r++, av, 0.0);
                clr(); av[SIG] = 1.0; av[TX] = 1.0; av[TU] = 1.0; put(r++, av, trv + sref);
                clr(); av[SIG] = -1.0; av[TX] = 1.0; av[TU] = 1.0; put(r++, av, trv - sref);
            }
        }
        B[Ly.o_nh] = (double)r;
        degl += r + 2 * NS + (Q > 0 ? 1 : 0);
        // soft rows: obstacles, then ADMM collision rows
        for (int o = 0; o < T.n_obs; ++o) {
            clr();
            double nr = 0.0, d[3] = {0, 0, 0};
            for (int i = 0; i < pd; ++i) { d[i] = xb[i] - T.obs_center[o][i]; nr += d[i] * d[i]; }
            nr = sqrt(nr) + 1e-6;
            double ac = 0.0;
            for (int i = 0; i < pd; ++i) { av[i] = -d[i] / nr; ac += d[i] / nr * T.obs_center[o][i]; }
            put(RH + o, av, -T.obs_radius[o] - ac);
        }
        for (int j = 0; j < T.n_nbr; ++j) {
            clr();
            const long long base = ((agent * T.n_nbr + j) * K + t) * pd;
            double nr = 0.0, d[3] = {0, 0, 0};
            for (int i = 0; i < pd; ++i) { d[i] = xb[i] - a.nbr_pos[base + i]; nr += d[i] * d[i]; }
            nr = sqrt(nr) + 1e-6;
            double ay = 0.0;
            for (int i = 0; i < pd; ++i) { av[i] = -d[i] / nr; ay += d[i] / nr * a.nbr_Y[base + i]; }
            put(RH + T.n_obs + j, av, -T.d_min - ay);
        }
        if (Q > 0) {
            clr(); put(RH + NS, av, T.u_max);
            #pragma unroll
            for (int j = 0; j < NU; ++j) { clr(); av[ZU + j] = -1.0; put(RH + NS + 1 + j, av, 0.0); }
        }
        // linear / quadratic cost (z coordinates)
        double qv[NZ];
        #pragma unroll
        for (int i = 0; i < NZ; ++i) qv[i] = 0.0;
        if (t == 0) { qv[SIG] = sfix ? 0.0 : T.w_sigma * ics; qv[TN] = T.w_nu * ics; }
        if (NE > 0 && T.w_in > 0.0)  // inertia: w_in ||x_t - xprev_t||^2 -> q_x = -2 w_in xprev_t
            #pragma unroll
            for (int i = 0; i < NX; ++i) qv[i] -= 2.0 * T.w_in * ics * a.X_prev[(agent * K + t) * NX + i];
        double pv = 0.0;
        for (int j = 0; j < T.n_nbr; ++j) {
            const long long base = ((agent * T.n_nbr + j) * K + t) * pd;
            for (int i = 0; i < pd; ++i) qv[i] += (a.nbr_Lam[base + i] - T.rho * a.nbr_Y[base + i]) * ics;
            pv += T.rho * ics;
        }
        #pragma unroll
        for (int j = 0; j < NU; ++j) {
            double v = 0.0;
            #pragma unroll
            for (int i = 0; i < NX; ++i) v += Cp[i * NU + j] * qv[i];
            qv[ZU + j] += v;
        }
        #pragma unroll
        for (int i = 0; i < NZ; ++i) { B[Ly.o_q + i] = qv[i]; qmax = fmax(qmax, fabs(qv[i])); }
        // P_z = T' diag(pv on positions) T
        #pragma unroll
        for (int i = 0; i < NZ; ++i)
            #pragma unroll
            for (int j = 0; j < NZ; ++j) {
                double v = 0.0;
                for (int l = 0; l < pd; ++l) {
                    const double ti = i == l ? 1.0 : (i >= ZU && i < ZN ? Cp[l * NU + (i - ZU)] : 0.0);
                    const double tj = j == l ? 1.0 : (j >= ZU && j < ZN ? Cp[l * NU + (j - ZU)] : 0.0);
                    v += ti * pv * tj;
                }
                B[Ly.o_P + i * NZ + j] = v;
            }
        if (NE > 0) {
            // game_model.py:87-100 in z coordinates (x_t = xi_t + C_{t-1} u_t), each term / cs
            auto padd = [&](int i, int j, double v) { B[Ly.o_P + i * NZ + j] += v; };
            const double cu = 2.0 * T.w_u2 * ics, cr = 2.0 * T.w_du * ics, cth = 2.0 * T.w_dth * ics,
                         ci = 2.0 * T.w_in * ics;
            #pragma unroll
            for (int j = 0; j < NU; ++j) padd(ZU + j, ZU + j, cu);
            if (t > 0) {
                #pragma unroll
                for (int j = 0; j < NU; ++j) {  // (u_t - u~_t)^2
                    padd(ZU + j, ZU + j, cr); padd(E0 + j, E0 + j, cr);
                    padd(ZU + j, E0 + j, -cr); padd(E0 + j, ZU + j, -cr);
                }
                if (NE > NU && T.theta_idx >= 0) {  // (th_t - th~_t)^2, th_t = xi[th] + C[th,:] u_t
                    const int th = T.theta_idx;
                    double c[NZ];
                    #pragma unroll
                    for (int i = 0; i < NZ; ++i) c[i] = 0.0;
                    c[th] = 1.0;
                    c[E0 + NU] = -1.0;
                    #pragma unroll
                    for (int j = 0; j < NU; ++j) c[ZU + j] = Cp[th * NU + j];
                    #pragma unroll
                    for (int i = 0; i < NZ; ++i)
                        #pragma unroll
                        for (int j = 0; j < NZ; ++j)
                            if (c[i] != 0.0 && c[j] != 0.0) padd(i, j, cth * c[i] * c[j]);
                }
            }
            if (T.w_in > 0.0)  // ||x_t - xprev_t||^2: T'T with T = [I 0 0 C 0]
                #pragma unroll
                for (int i = 0; i < NZ; ++i)
                    #pragma unroll
                    for (int j = 0; j < NZ; ++j) {
                        const bool xi = i < NX, xj = j < NX, ui = i >= ZU && i < ZN, uj = j >= ZU && j < ZN;
                        if (!((xi || ui) && (xj || uj))) continue;
                        double v = 0.0;
                        for (int l = 0; l < NX; ++l) {
                            const double ti = xi ? (i == l ? 1.0 : 0.0) : Cp[l * NU + (i - ZU)];
                            const double tj = xj ? (j == l ? 1.0 : 0.0) : Cp[l * NU + (j - ZU)];
                            v += ti * tj;
                        }
                        padd(i, j, ci * v);
                    }
            if (sfix && t == 0) padd(SIG, SIG, 1.0);  // sigma is data: a decoupled z_sigma -> 0
        }
        // dynamics to node t+1 (Riccati coordinates)
        if (t < K - 1) {
            double* At = B + Ly.o_At;
            double* Bt = B + Ly.o_Bt;
            double* ct = B + Ly.o_ct;
            #pragma unroll
            for (int e = 0; e < NXA * NXA; ++e) At[e] = 0.0;
            #pragma unroll
            for (int e = 0; e < NXA * NUA; ++e) Bt[e] = 0.0;
            for (int g = 0; g < SCP_NG; ++g) { At[(NX + g) * NXA + NX + g] = 1.0; ct[NX + g] = 0.0; }
            if (subst) {
                #pragma unroll
                for (int i = 0; i < NX; ++i) ct[i] = xfin[i];
            } else {
                #pragma unroll
                for (int i = 0; i < NX; ++i) {
                    for (int l = 0; l < NX; ++l) At[i * NXA + l] = dk[l * NX + i];
                    At[i * NXA + SIG] = dk[NX * NX + 2 * NX * NU + i];
                    #pragma unroll
                    for (int j = 0; j < NU; ++j) {
                        double v = dk[NX * NX + j * NX + i];
                        for (int l = 0; l < NX; ++l) v += dk[l * NX + i] * Cp[l * NU + j];
                        Bt[i * NUA + j] = v;
                    }
                    Bt[i * NUA + NU + i] = 1.0;
                    ct[i] = dk[NX * NX + 2 * NX * NU + NX + i];
                    if (sfix) { ct[i] += At[i * NXA + SIG] * sref; At[i * NXA + SIG] = 0.0; }
                }
            }
            if (NE > 0) {  // u~_{t+1} = u_t; th~_{t+1} = th_t = xi_t[th] + C_{t-1}[th,:] u_t
                #pragma unroll
                for (int j = 0; j < NU; ++j) { Bt[(E0 + j) * NUA + j] = 1.0; ct[E0 + j] = 0.0; }
                if (NE > NU) {
                    const int th = T.theta_idx;
                    At[(E0 + NU) * NXA + th] = 1.0;
                    #pragma unroll
                    for (int j = 0; j < NU; ++j) Bt[(E0 + NU) * NUA + j] = Cp[th * NU + j];
                    ct[E0 + NU] = 0.0;
                }
            }
            #pragma unroll
            for (int i = 0; i < NXA; ++i) hmax = fmax(hmax, fabs(ct[i]));
        }
    }
    if (lane < NX) hmax = fmax(hmax, fabs(xinit[lane]));
    const double pscale = 1.0 + blk_max(hmax);
    double dsc = blk_max(qmax);
    if (T.n_obs > 0) dsc = fmax(dsc, w_obs);
    if (T.n_nbr > 0) dsc = fmax(dsc, w_col);
    const double dscale = 1.0 + dsc;
    const double deg = blk_sum(degl);
    __syncthreads();

    auto soft_w = [&](int r) -> double { return r < T.n_obs ? w_obs : w_col; };
    // the node cost Hessian P is identically zero for the plain SCProblem (an LP: no ADMM, no game
    // terms); its loads are skipped then (uniform)
    const bool hasP = T.n_nbr > 0 || NE > 0;

    // ------------------------------------------------------------------ stage packets
    // The Riccati sweeps are sequential over nodes, so every global load inside a stage is exposed
    // latency.  Each sweep instead gathers the next stage's operands (a packet of node-block elements)
    // into registers at the top of the current stage and parks them in an LDS ring slot at its end; the
    // stage itself reads only LDS.  Each lane's packet elements are mapped to (node delta, node-block
    // offset) once per sweep, so a stage's gather is PF loads at stage-invariant offsets.  Loads are
    // unconditional (node clamped to [0, K-1], lanes past the packet re-read an element into the slot
    // tail) and the sweeps use LDS-only wave barriers, so nothing drains the prefetch.
    constexpr int NAB = NXA + NUA;
    constexpr int PK_F = NZ * NZ + NXA * NAB;                                               // factor
    constexpr int PK_B = NXA * NXA + NXA + NZ + NXA * NXA + NXA * NUA + NUA * NUA + NUA * NXA;  // LQ backward
    constexpr int PK_W = NUA + NUA * NXA + NXA + NXA * NXA + NXA * NUA + NXA + NXA * NXA;   // LQ forward
    constexpr int PK_MAX = PK_F > PK_B ? (PK_F > PK_W ? PK_F : PK_W) : (PK_B > PK_W ? PK_B : PK_W);
    constexpr int PF = (PK_MAX + WAVE - 1) / WAVE;
    __shared__ double sRing[2][PF * WAVE];
    __shared__ double sSink[WAVE];  // LDS stores of lanes without an output element
    double pf[PF];
    // segments: {node offset (0 or +1), node-block offset, length} -> per-lane element map (sweep-form LQ)
    auto seg_map = [&](const int (&dn)[7], const int (&off)[7], const int (&len)[7], int nseg, int (&fo)[PF],
                       int (&fd)[PF]) {
        #pragma unroll
        for (int c = 0; c < PF; ++c) {
            const int e = lane + c * WAVE;
            int o = off[0], d = dn[0], acc = 0;
            #pragma unroll
            for (int sg = 0; sg < 7; ++sg) {
                if (sg < nseg && e >= acc && e < acc + len[sg]) { o = off[sg] + (e - acc); d = dn[sg]; }
                if (sg < nseg) acc += len[sg];
            }
            fo[c] = o;
            fd[c] = d;
        }
    };
    auto gather = [&](int t, const int (&fo)[PF], const int (&fd)[PF]) {
        #pragma unroll
        for (int c = 0; c < PF; ++c) {
            int tn = t + fd[c];
            tn = tn < 0 ? 0 : (tn > K - 1 ? K - 1 : tn);
            pf[c] = ws[(long long)tn * Ly.stride + fo[c]];
        }
    };
    auto park = [&](int slot) {
        #pragma unroll
        for (int c = 0; c < PF; ++c) sRing[slot][lane + c * WAVE] = pf[c];
    };

    // ------------------------------------------------------------------ Riccati factor (uses o_H)
    // Stage packet: H (NZ x NZ) | [At Bt] column-major (column j of [At Bt] is NXA contiguous doubles),
    // so every product of the stage is a dot product of two contiguous LDS vectors.  Four straight-line
    // phases per stage, each lane's operand offsets decoded once per sweep (the packet slot alternates,
    // the offsets within it do not); no divergent branches:
    //   1: PAB = P [At Bt]                       (column-major, NXA x NAB)
    //   2: Qxx = H_xx + At'PA (upper triangle), Qux = H_ux + Bt'PA (column-major), Quu = H_uu + Bt'PB
    //   3: Quu = L D L' in registers (every lane); K = -Quu^-1 Qux, lane c < NXA solves column c
    //   4: P = Qxx + Qux'K (symmetric: the upper element for both halves)
    // Every accumulation runs in the order of oracle/scp_cpu.py's restatement (and of the previous
    // element-loop form of this sweep): sequential k, starting from the H element.
    auto factor = [&]() __attribute__((always_inline)) {
      if (wid == 0) {  // the sweep: wave 0
        const int lane = scp_opaque(threadIdx.x);
        constexpr int R1 = (NXA * NAB + WAVE - 1) / WAVE;
        constexpr int E2 = NXA * NXA + NXA * NUA + NUA * NUA, R2 = (E2 + WAVE - 1) / WAVE;
        constexpr int R4 = (NXA * NXA + WAVE - 1) / WAVE;
        int fo[PF], fd[PF];
        #pragma unroll
        for (int c = 0; c < PF; ++c) {
            const int e = lane + c * WAVE;
            fd[c] = 0;
            if (e < NZ * NZ) {
                fo[c] = Ly.o_H + e;
            } else if (e < PK_F) {
                const int c2 = e - NZ * NZ, j = c2 / NXA, k = c2 - j * NXA;
                fo[c] = j < NXA ? Ly.o_At + k * NXA + j : Ly.o_Bt + k * NUA + (j - NXA);
            } else {
                fo[c] = Ly.o_H;
            }
        }
        // phase 1: out PAB[o] (o = j NXA + i) = P row i . [At Bt] column j
        int l1[R1], r1[R1];
        double* o1[R1];
        #pragma unroll
        for (int r = 0; r < R1; ++r) {
            const int o = lane + r * WAVE;
            const bool ok = o < NXA * NAB;
            const int oo = ok ? o : 0, j = oo / NXA, i = oo - j * NXA;
            l1[r] = i * NXA;
            r1[r] = NZ * NZ + j * NXA;
            o1[r] = ok ? sPAB + oo : sSink + lane;
        }
        // phase 2: column a of [At Bt] . PAB column b, + H[hi][hj]; pin classes (0 state, 1 input, 2 nu)
        int a2[R2], b2[R2], h2[R2], ci2[R2], cj2[R2], kd2[R2];
        double* o2[R2];
        #pragma unroll
        for (int r = 0; r < R2; ++r) {
            const int o = lane + r * WAVE;
            int a = 0, b = 0, hi = 0, hj = 0, ci = 0, cj = 0, kd = 0;
            double* out = sSink + lane;
            if (o < NXA * NXA) {  // Qxx (p, q) = (min, max)
                const int i = o / NXA, j = o - i * NXA, p = i < j ? i : j, q = i < j ? j : i;
                a = p; b = q; hi = p; hj = q; out = sQxx + o;
            } else if (o < NXA * NXA + NXA * NUA) {  // Qux column-major: element (i, j) at j NUA + i
                const int o2_ = o - NXA * NXA, j = o2_ / NUA, i = o2_ - j * NUA;
                a = NXA + i; b = j; hi = NXA + i; hj = j; ci = i < NU ? 1 : 2; kd = 1; out = sQuxC + o2_;
            } else if (o < E2) {  // Quu (i, j)
                const int o3 = o - NXA * NXA - NXA * NUA, i = o3 / NUA, j = o3 - i * NUA;
                a = NXA + i; b = NXA + j; hi = NXA + i; hj = NXA + j;
                ci = i < NU ? 1 : 2; cj = j < NU ? 1 : 2; kd = i == j ? 3 : 2; out = sQuu + o3;
            }
            a2[r] = NZ * NZ + a * NXA; b2[r] = b * NXA; h2[r] = hi * NZ + hj;
            ci2[r] = ci; cj2[r] = cj; kd2[r] = kd; o2[r] = out;
        }
        const bool kl = lane < NXA;
        const int kc = kl ? lane : 0;
        for (int e = lane; e < NXA * NXA; e += WAVE) sP[e] = 0.0;
        gather(K - 1, fo, fd);
        park(0);
        wsync();
        for (int t = K - 1; t >= 0; --t) {
            const int slot = (K - 1 - t) & 1;
            gather(t - 1, fo, fd);
            const double* pk = sRing[slot];
            const bool dyn = t < K - 1;
            const bool pinU = (t == 0 && T.pin_u_first) || (t == K - 1 && T.pin_u_last);
            const bool pinN = t == K - 1 || (fin && t == K - 2);
            #pragma unroll
            for (int r = 0; r < R1; ++r) {
                double v = 0.0;
                #pragma unroll
                for (int k = 0; k < NXA; ++k) v += sP[l1[r] + k] * pk[r1[r] + k];
                *o1[r] = v;
            }
            wsync();
            #pragma unroll
            for (int r = 0; r < R2; ++r) {
                double v = pk[h2[r]];
                double d = v;
                #pragma unroll
                for (int k = 0; k < NXA; ++k) d += pk[a2[r] + k] * sPAB[b2[r] + k];
                v = dyn ? d : v;
                const bool pi = ci2[r] == 1 ? pinU : (ci2[r] == 2 ? pinN : false);
                const bool pj = cj2[r] == 1 ? pinU : (cj2[r] == 2 ? pinN : false);
                if (kd2[r] == 1) v = pi ? 0.0 : v;
                if (kd2[r] >= 2) v = (pi || pj) ? (kd2[r] == 3 ? 1.0 : 0.0) : v;
                *o2[r] = v;
            }
            wsync();
            double Lm[NUA * NUA];
            #pragma unroll
            for (int e = 0; e < NUA * NUA; ++e) Lm[e] = sQuu[e];
            ldl_factor<NUA>(Lm, NUA);
            {  // every lane solves (lanes >= NXA on a copy of column 0, stored to the sinks)
                double x[NUA];
                #pragma unroll
                for (int i = 0; i < NUA; ++i) x[i] = -sQuxC[kc * NUA + i];
                ldl_solve<NUA>(Lm, NUA, x);
                #pragma unroll
                for (int i = 0; i < NUA; ++i) {
                    *(kl ? sKC + kc * NUA + i : sSink + lane) = x[i];
                    *(kl ? nb(t) + Ly.o_K + i * NXA + lane : jnk) = x[i];
                }
                double lv = 0.0;  // element `lane` of the factor (select chain: no dynamic register index)
                #pragma unroll
                for (int e = 0; e < NUA * NUA; ++e) lv = (e == lane) ? Lm[e] : lv;
                *(lane < NUA * NUA ? nb(t) + Ly.o_LD + lane : jnk) = lv;
            }
            wsync();
            #pragma unroll
            for (int rep = 0; rep < R4; ++rep) {
                const int e = lane + rep * WAVE;
                const bool ok = e < NXA * NXA;
                const int ee = ok ? e : 0;
                const int i = ee / NXA, j = ee % NXA, p = i < j ? i : j, q = i < j ? j : i;
                double v = sQxx[p * NXA + q];
                #pragma unroll
                for (int k = 0; k < NUA; ++k) v += sQuxC[p * NUA + k] * sKC[q * NUA + k];
                *(ok ? sP + e : sSink + lane) = v;
                *(ok ? nb(t) + Ly.o_Pr + e : jnk) = v;
            }
            park(slot ^ 1);
            wsync();
        }
      }
        __syncthreads();
        // closed-loop Acl_t = At_t + Bt_t K_t (row-major), the LQ chains' matrices: lane-parallel over nodes
        if constexpr (NW > 1)
        for (int t = tid; t < K - 1; t += NT) {
            double* B = nb(t);
            double Kt[NUA * NXA];
            #pragma unroll
            for (int e = 0; e < NUA * NXA; ++e) Kt[e] = B[Ly.o_K + e];
            #pragma unroll
            for (int i = 0; i < NXA; ++i) {
                double bi[NUA];
                #pragma unroll
                for (int k = 0; k < NUA; ++k) bi[k] = B[Ly.o_Bt + i * NUA + k];
                #pragma unroll
                for (int j = 0; j < NXA; ++j) {
                    double v = B[Ly.o_At + i * NXA + j];
                    #pragma unroll
                    for (int k = 0; k < NUA; ++k) v += bi[k] * Kt[k * NXA + j];
                    B[Ly.o_Acl + i * NXA + j] = v;
                }
            }
        }
        __syncthreads();
    };

    // ------------------------------------------------------------------ LQ solve, sweep form (one wave per agent)
    // The element-parallel Riccati sweeps of rounds 1-2 (the recursion below stage by stage, the stage
    // operands gathered a stage ahead into an LDS ring): used when the launch fills every SIMD (NW = 1),
    // where the closed-loop form's lane-parallel passes (P, Acl and K of every node re-read under
    // full-chip contention) measured slower (batched game launch 61.9 vs 70.9 ms).
    // In: o_f (per node), o_rp (t < K-1), sMisc[0..NX) = r_init.  Out: o_dz, o_yp (costates y+),
    // sMisc[8..8+NX) = y0+.
    auto lqsolve_sweep = [&]() __attribute__((always_inline)) {
        // backward: v = P_{t+1} rp_t + p_{t+1}; qx = fx + At'v; qu = fu + Bt'v; k = -Quu^-1 qu; p = qx + K'qu
        constexpr int B_PR = 0, B_RP = B_PR + NXA * NXA, B_F = B_RP + NXA, B_AT = B_F + NZ, B_BT = B_AT + NXA * NXA,
                      B_LD = B_BT + NXA * NUA, B_K = B_LD + NUA * NUA;
        {
            const int dn[7] = {1, 0, 0, 0, 0, 0, 0};
            const int off[7] = {Ly.o_Pr, Ly.o_rp, Ly.o_f, Ly.o_At, Ly.o_Bt, Ly.o_LD, Ly.o_K};
            const int len[7] = {NXA * NXA, NXA, NZ, NXA * NXA, NXA * NUA, NUA * NUA, NUA * NXA};
            int fo[PF], fd[PF];
            seg_map(dn, off, len, 7, fo, fd);
            gather(K - 1, fo, fd);
            park(0);
            wsync();
            for (int t = K - 1; t >= 0; --t) {
                const int slot = (K - 1 - t) & 1;
                gather(t - 1, fo, fd);
                const double* pk = sRing[slot];
                const bool dyn = t < K - 1;
                if (lane < NXA) {
                    double v = 0.0;
                    if (dyn) {
                        v = sPv[lane];
                        for (int k = 0; k < NXA; ++k) v += pk[B_PR + lane * NXA + k] * pk[B_RP + k];
                    }
                    sV[lane] = v;
                }
                wsync();
                if (lane < NZ) {
                    double v = pk[B_F + lane];
                    if (dyn) {
                        if (lane < NXA)
                            for (int k = 0; k < NXA; ++k) v += pk[B_AT + k * NXA + lane] * sV[k];
                        else
                            for (int k = 0; k < NXA; ++k) v += pk[B_BT + k * NUA + lane - NXA] * sV[k];
                    }
                    if (pinned(t, lane)) v = 0.0;
                    sQ[lane] = v;
                }
                wsync();
                {
                    double Lm[NUA * NUA], x[NUA];
                    #pragma unroll
                    for (int e = 0; e < NUA * NUA; ++e) Lm[e] = pk[B_LD + e];
                    #pragma unroll
                    for (int i = 0; i < NUA; ++i) x[i] = -sQ[NXA + i];
                    ldl_solve<NUA>(Lm, NUA, x);
                    // (select x[lane] without dynamic register indexing)
                    double xv = 0.0;
                    #pragma unroll
                    for (int i = 0; i < NUA; ++i) xv = (i == lane) ? x[i] : xv;
                    *(lane < NUA ? nb(t) + Ly.o_kv + lane : jnk) = xv;
                }
                double pn;
                {
                    const int li = lane < NXA ? lane : 0;
                    pn = sQ[li];
                    for (int k = 0; k < NUA; ++k) pn += pk[B_K + k * NXA + li] * sQ[NXA + k];
                    *(lane < NXA ? nb(t) + Ly.o_pv + lane : jnk) = pn;
                }
                wsync();
                if (lane < NXA) sPv[lane] = pn;
                park(slot ^ 1);
                wsync();
            }
        }
        __syncthreads();
        // stage 0: x part fixed (-r_init), g part free: P_gg dg = -(p_g + P_gx dx)
        {
            const double* B0 = nb(0);
            double dx[NX];
            #pragma unroll
            for (int i = 0; i < NX; ++i) dx[i] = -sMisc[i];
            double Lm[SCP_NG * SCP_NG], g[SCP_NG];
            for (int i = 0; i < SCP_NG; ++i) {
                double v = B0[Ly.o_pv + NX + i];
                for (int k = 0; k < NX; ++k) v += B0[Ly.o_Pr + (NX + i) * NXA + k] * dx[k];
                g[i] = -v;
                for (int j = 0; j < SCP_NG; ++j) Lm[i * SCP_NG + j] = B0[Ly.o_Pr + (NX + i) * NXA + NX + j];
            }
            ldl_factor<SCP_NG>(Lm, SCP_NG);
            ldl_solve<SCP_NG>(Lm, SCP_NG, g);
            #pragma unroll
            for (int i = 0; i < NX; ++i)
                if (lane == i) sXw[0][lane] = dx[i];
            for (int i = 0; i < SCP_NG; ++i)
                if (lane == NX + i) sXw[0][lane] = g[i];
            if (lane >= E0 && lane < NXA) sXw[0][lane] = 0.0;  // u~_0, th~_0: no predecessor, no cost
            __syncthreads();
            if (lane < NX) {
                double v = B0[Ly.o_pv + lane];
                for (int k = 0; k < NXA; ++k) v += B0[Ly.o_Pr + lane * NXA + k] * sXw[0][k];
                sMisc[8 + lane] = v;
            }
        }
        __syncthreads();
        // forward: u = kv + K xi; xi+ = rp + At xi + Bt u; y+ = p_{t+1} + P_{t+1} xi+
        {
            constexpr int W_KV = 0, W_K = W_KV + NUA, W_RP = W_K + NUA * NXA, W_AT = W_RP + NXA,
                          W_BT = W_AT + NXA * NXA, W_PV1 = W_BT + NXA * NUA, W_PR1 = W_PV1 + NXA;
            const int dn[7] = {0, 0, 0, 0, 0, 1, 1};
            const int off[7] = {Ly.o_kv, Ly.o_K, Ly.o_rp, Ly.o_At, Ly.o_Bt, Ly.o_pv, Ly.o_Pr};
            const int len[7] = {NUA, NUA * NXA, NXA, NXA * NXA, NXA * NUA, NXA, NXA * NXA};
            int fo[PF], fd[PF];
            seg_map(dn, off, len, 7, fo, fd);
            gather(0, fo, fd);
            park(0);
            wsync();
            int cur = 0;
            for (int t = 0; t < K; ++t) {
                const int slot = t & 1;
                gather(t + 1, fo, fd);
                const double* pk = sRing[slot];
                double* B = nb(t);
                {
                    const int lu = lane < NUA ? lane : 0;
                    double v = pk[W_KV + lu];
                    for (int k = 0; k < NXA; ++k) v += pk[W_K + lu * NXA + k] * sXw[cur][k];
                    if (lane < NUA) sU[lane] = v;
                    *(lane < NUA ? B + Ly.o_dz + NXA + lane : jnk) = v;
                }
                *(lane < NXA ? B + Ly.o_dz + lane : jnk) = sXw[cur][lane < NXA ? lane : 0];
                wsync();
                if (t < K - 1) {
                    if (lane < NXA) {
                        double v = pk[W_RP + lane];
                        for (int k = 0; k < NXA; ++k) v += pk[W_AT + lane * NXA + k] * sXw[cur][k];
                        for (int k = 0; k < NUA; ++k) v += pk[W_BT + lane * NUA + k] * sU[k];
                        sXw[cur ^ 1][lane] = v;
                    }
                    wsync();
                    cur ^= 1;
                    {
                        const int li = lane < NXA ? lane : 0;
                        double v = pk[W_PV1 + li];
                        for (int k = 0; k < NXA; ++k) v += pk[W_PR1 + li * NXA + k] * sXw[cur][k];
                        *(lane < NXA ? B + Ly.o_yp + lane : jnk) = v;
                    }
                }
                park(slot ^ 1);
                wsync();
            }
        }
        __syncthreads();
    };

    // ------------------------------------------------------------------ LQ solve
    // In: o_f (per node), o_rp (t < K-1), sMisc[0..NX) = r_init.  Out: o_dz, o_yp (costates y+),
    // sMisc[8..8+NX) = y0+.
    // Closed-loop form: with Acl_t = At_t + Bt_t K_t (the factor's output) the backward recursion
    //   v = P_{t+1} rp_t + p_{t+1}; q = f + [At Bt]'v; k_t = -Quu^-1 q_u; p_t = q_x + K_t'q_u
    // is p_t = Acl_t' p_{t+1} + g_t with g_t = f_x + K_t'f_u + Acl_t' P_{t+1} rp_t (K_t's pinned rows are 0),
    // and the forward one xi_{t+1} = Acl_t xi_t + e_t with e_t = rp_t + Bt_t k_t.  Only these two NXA-vector
    // recursions are sequential: each step is one NXA-term dot product per lane (lane i: element i), the
    // previous vector broadcast by 64-bit DPP row_newbcast, operands prefetched four steps ahead.  g_t,
    // k_t, e_t and the outputs u_t, y+_t are lane-parallel passes over the nodes.
    auto lqsolve = [&]() __attribute__((always_inline)) {
        const int li = scp_opaque(lane < NXA ? lane : 0);
        // ---- backward pre-pass: w_t = P_{t+1} rp_t, g_t
        for (int t = tid; t < K; t += NT) {
            double* B = nb(t);
            const bool dyn = t < K - 1;
            double w[NXA], g[NXA], fu[NUA];
            #pragma unroll
            for (int j = 0; j < NUA; ++j) fu[j] = B[Ly.o_f + NXA + j];
            #pragma unroll
            for (int i = 0; i < NXA; ++i) {
                double v = B[Ly.o_f + i];
                #pragma unroll
                for (int j = 0; j < NUA; ++j) v += B[Ly.o_K + j * NXA + i] * fu[j];
                g[i] = v;
            }
            if (dyn) {
                const double* Bn = nb(t + 1);
                double rp[NXA];
                #pragma unroll
                for (int k = 0; k < NXA; ++k) rp[k] = B[Ly.o_rp + k];
                #pragma unroll
                for (int i = 0; i < NXA; ++i) {
                    double v = 0.0;
                    #pragma unroll
                    for (int k = 0; k < NXA; ++k) v += Bn[Ly.o_Pr + i * NXA + k] * rp[k];
                    w[i] = v;
                    B[Ly.o_w + i] = v;
                }
                #pragma unroll
                for (int i = 0; i < NXA; ++i) {
                    double v = g[i];
                    #pragma unroll
                    for (int k = 0; k < NXA; ++k) v += B[Ly.o_Acl + k * NXA + i] * w[k];
                    g[i] = v;
                }
            }
            #pragma unroll
            for (int i = 0; i < NXA; ++i) B[Ly.o_g + i] = g[i];
        }
        __syncthreads();
        // ---- backward chain p_t = Acl_t' p_{t+1} + g_t  (lane i < NXA: element i; column i of Acl_t)
        if (wid == 0) {
            double ca[4][NXA], cg[4];
            auto ld = [&](int t, double (&c)[NXA], double& gv) __attribute__((always_inline)) {
                const double* B = nb(t > 0 ? t : 0);
                #pragma unroll
                for (int k = 0; k < NXA; ++k) c[k] = B[Ly.o_Acl + k * NXA + li];
                gv = B[Ly.o_g + li];
            };
            double p = nb(K - 1)[Ly.o_g + li];
            *(lane < NXA ? nb(K - 1) + Ly.o_pv + lane : jnk) = p;
            ld(K - 2, ca[0], cg[0]);
            ld(K - 3, ca[1], cg[1]);
            ld(K - 4, ca[2], cg[2]);
            ld(K - 5, ca[3], cg[3]);
            auto step = [&](int t, double (&c)[NXA], double gv, double (&nc)[NXA], double& ng) __attribute__((always_inline)) {
                double v = gv;
                #pragma unroll
                for (int k = 0; k < NXA; ++k) v += c[k] * row_bcast_d(p, k);
                p = v;
                *(lane < NXA ? nb(t) + Ly.o_pv + lane : jnk) = v;
                ld(t - 4, nc, ng);  // stage t-4 into the slot just consumed
            };
            int t = K - 2;
            while (true) {
                step(t, ca[0], cg[0], ca[0], cg[0]); if (--t < 0) break;
                step(t, ca[1], cg[1], ca[1], cg[1]); if (--t < 0) break;
                step(t, ca[2], cg[2], ca[2], cg[2]); if (--t < 0) break;
                step(t, ca[3], cg[3], ca[3], cg[3]); if (--t < 0) break;
            }
        }
        __syncthreads();
        // ---- backward post-pass: k_t = -Quu^-1 (f_u + Bt'(p_{t+1} + w_t)); e_t = rp_t + Bt k_t
        for (int t = tid; t < K; t += NT) {
            double* B = nb(t);
            const bool dyn = t < K - 1;
            double v[NXA], x[NUA], Lm[NUA * NUA];
            #pragma unroll
            for (int k = 0; k < NXA; ++k) v[k] = dyn ? nb(t + 1)[Ly.o_pv + k] + B[Ly.o_w + k] : 0.0;
            #pragma unroll
            for (int j = 0; j < NUA; ++j) {
                double q = B[Ly.o_f + NXA + j];
                if (dyn)
                    #pragma unroll
                    for (int k = 0; k < NXA; ++k) q += B[Ly.o_Bt + k * NUA + j] * v[k];
                x[j] = pinned(t, NXA + j) ? 0.0 : -q;
            }
            #pragma unroll
            for (int e = 0; e < NUA * NUA; ++e) Lm[e] = B[Ly.o_LD + e];
            ldl_solve<NUA>(Lm, NUA, x);
            #pragma unroll
            for (int j = 0; j < NUA; ++j) B[Ly.o_kv + j] = x[j];
            if (dyn)
                #pragma unroll
                for (int i = 0; i < NXA; ++i) {
                    double e = B[Ly.o_rp + i];
                    #pragma unroll
                    for (int j = 0; j < NUA; ++j) e += B[Ly.o_Bt + i * NUA + j] * x[j];
                    B[Ly.o_e + i] = e;
                }
        }
        __syncthreads();
        // stage 0: x part fixed (-r_init), g part free: P_gg dg = -(p_g + P_gx dx)
        {
            const double* B0 = nb(0);
            double dx[NX];
            #pragma unroll
            for (int i = 0; i < NX; ++i) dx[i] = -sMisc[i];
            double Lm[SCP_NG * SCP_NG], g[SCP_NG];
            for (int i = 0; i < SCP_NG; ++i) {
                double v = B0[Ly.o_pv + NX + i];
                for (int k = 0; k < NX; ++k) v += B0[Ly.o_Pr + (NX + i) * NXA + k] * dx[k];
                g[i] = -v;
                for (int j = 0; j < SCP_NG; ++j) Lm[i * SCP_NG + j] = B0[Ly.o_Pr + (NX + i) * NXA + NX + j];
            }
            ldl_factor<SCP_NG>(Lm, SCP_NG);
            ldl_solve<SCP_NG>(Lm, SCP_NG, g);
            #pragma unroll
            for (int i = 0; i < NX; ++i)
                if (lane == i) sXi[lane] = dx[i];
            for (int i = 0; i < SCP_NG; ++i)
                if (lane == NX + i) sXi[lane] = g[i];
            if (lane >= E0 && lane < NXA) sXi[lane] = 0.0;  // u~_0, th~_0: no predecessor, no cost
            __syncthreads();
            if (lane < NX) {
                double v = B0[Ly.o_pv + lane];
                for (int k = 0; k < NXA; ++k) v += B0[Ly.o_Pr + lane * NXA + k] * sXi[k];
                sMisc[8 + lane] = v;
            }
        }
        __syncthreads();
        // ---- forward chain xi_{t+1} = Acl_t xi_t + e_t  (lane i < NXA: element i; row i of Acl_t)
        if (wid == 0) {
            double ca[4][NXA], ce[4];
            auto ld = [&](int t, double (&c)[NXA], double& ev) __attribute__((always_inline)) {
                const double* B = nb(t < K - 2 ? t : K - 2);
                #pragma unroll
                for (int k = 0; k < NXA; ++k) c[k] = B[Ly.o_Acl + li * NXA + k];
                ev = B[Ly.o_e + li];
            };
            double xi = sXi[li];
            *(lane < NXA ? nb(0) + Ly.o_dz + lane : jnk) = xi;
            ld(0, ca[0], ce[0]);
            ld(1, ca[1], ce[1]);
            ld(2, ca[2], ce[2]);
            ld(3, ca[3], ce[3]);
            auto step = [&](int t, double (&c)[NXA], double ev, double (&nc)[NXA], double& ne) __attribute__((always_inline)) {
                double v = ev;
                #pragma unroll
                for (int k = 0; k < NXA; ++k) v += c[k] * row_bcast_d(xi, k);
                xi = v;
                *(lane < NXA ? nb(t + 1) + Ly.o_dz + lane : jnk) = v;
                ld(t + 4, nc, ne);
            };
            int t = 0;
            while (true) {
                if (t > K - 2) break;
                step(t, ca[0], ce[0], ca[0], ce[0]); if (++t > K - 2) break;
                step(t, ca[1], ce[1], ca[1], ce[1]); if (++t > K - 2) break;
                step(t, ca[2], ce[2], ca[2], ce[2]); if (++t > K - 2) break;
                step(t, ca[3], ce[3], ca[3], ce[3]); ++t;
            }
        }
        __syncthreads();
        // ---- forward post-pass: u_t = k_t + K_t xi_t; y+_t = p_{t+1} + P_{t+1} xi_{t+1}
        for (int t = tid; t < K; t += NT) {
            double* B = nb(t);
            double xi[NXA];
            #pragma unroll
            for (int k = 0; k < NXA; ++k) xi[k] = B[Ly.o_dz + k];
            #pragma unroll
            for (int j = 0; j < NUA; ++j) {
                double v = B[Ly.o_kv + j];
                #pragma unroll
                for (int k = 0; k < NXA; ++k) v += B[Ly.o_K + j * NXA + k] * xi[k];
                B[Ly.o_dz + NXA + j] = v;
            }
            if (t < K - 1) {
                const double* Bn = nb(t + 1);
                double x1[NXA];
                #pragma unroll
                for (int k = 0; k < NXA; ++k) x1[k] = Bn[Ly.o_dz + k];
                #pragma unroll
                for (int i = 0; i < NXA; ++i) {
                    double v = Bn[Ly.o_pv + i];
                    #pragma unroll
                    for (int k = 0; k < NXA; ++k) v += Bn[Ly.o_Pr + i * NXA + k] * x1[k];
                    B[Ly.o_yp + i] = v;
                }
            }
        }
        __syncthreads();
    };

    // row helpers (node t, block B)
    auto rowp = [&](const double* B, int r) -> const double* { return B + Ly.o_rows + r * RS; };
    auto dot = [&](const double* a0, const double* z) -> double {
        double v = 0.0;
        #pragma unroll
        for (int i = 0; i < NZ; ++i) v += a0[i] * z[i];
        return v;
    };

    // ------------------------------------------------------------------ starting point (W = I)
    for (int t = tid; t < K; t += NT) {
        double* B = nb(t);
        const int nh = (int)B[Ly.o_nh];
        double Hu[NZ * NZ], f[NZ];
        #pragma unroll
        for (int e = 0; e < NZ * NZ; ++e) Hu[e] = hasP ? B[Ly.o_P + e] : 0.0;
        #pragma unroll
        for (int i = 0; i < NZ; ++i) f[i] = B[Ly.o_q + i];
        for (int r = 0; r < nh; ++r) {
            const double* ar = rowp(B, r);
            const double h = ar[NZ];
            #pragma unroll
            for (int i = 0; i < NZ; ++i) {
                f[i] -= ar[i] * h;
                #pragma unroll
                for (int j = i; j < NZ; ++j) Hu[i * NZ + j] += ar[i] * ar[j];
            }
        }
        for (int r = 0; r < NS; ++r) {
            const double* ar = rowp(B, RH + r);
            const double h = ar[NZ];
            const double rhs = -soft_w(r) - h;
            B[Ly.o_rhs + r] = rhs;
            #pragma unroll
            for (int i = 0; i < NZ; ++i) {
                f[i] -= ar[i] * (h + 0.5 * rhs);
                #pragma unroll
                for (int j = i; j < NZ; ++j) Hu[i * NZ + j] += 0.5 * ar[i] * ar[j];
            }
        }
        for (int r = 0; r < Q; ++r) {
            const double* ar = rowp(B, RH + NS + r);
            const double h = ar[NZ];
            #pragma unroll
            for (int i = 0; i < NZ; ++i) {
                f[i] -= ar[i] * h;
                #pragma unroll
                for (int j = i; j < NZ; ++j) Hu[i * NZ + j] += ar[i] * ar[j];
            }
        }
        #pragma unroll
        for (int i = 0; i < NZ; ++i) Hu[i * NZ + i] += T.reg;
        #pragma unroll
        for (int e = 0; e < NZ * NZ; ++e) B[Ly.o_H + e] = Hu[e / NZ <= e % NZ ? e : (e % NZ) * NZ + e / NZ];  // upper triangle, mirrored
        #pragma unroll
        for (int i = 0; i < NZ; ++i) B[Ly.o_f + i] = f[i];
        if (t < K - 1)
            #pragma unroll
            for (int i = 0; i < NXA; ++i) B[Ly.o_rp + i] = B[Ly.o_ct + i];
    }
    if (tid < NX) sMisc[tid] = -xinit[tid];
    __syncthreads();
    factor();
    if constexpr (NW == 1) lqsolve_sweep(); else lqsolve();
    double mins = INFINITY, minl = INFINITY;
    for (int t = tid; t < K; t += NT) {
        double* B = nb(t);
        const int nh = (int)B[Ly.o_nh];
        double z[NZ];
        #pragma unroll
        for (int i = 0; i < NZ; ++i) { z[i] = B[Ly.o_dz + i]; B[Ly.o_z + i] = z[i]; }
        for (int r = 0; r < nh; ++r) {
            const double* ar = rowp(B, r);
            const double sv = ar[NZ] - dot(ar, z);
            B[Ly.o_s + r] = sv; B[Ly.o_lam + r] = -sv;
            mins = fmin(mins, sv); minl = fmin(minl, -sv);
        }
        for (int r = 0; r < NS; ++r) {
            const double* ar = rowp(B, RH + r);
            const double az = dot(ar, z);
            const double sg = 0.5 * (B[Ly.o_rhs + r] + az);
            B[Ly.o_sig + r] = sg;
            const double s1 = ar[NZ] - az + sg, s2 = sg;
            B[Ly.o_s + RH + 2 * r] = s1; B[Ly.o_lam + RH + 2 * r] = -s1;
            B[Ly.o_s + RH + 2 * r + 1] = s2; B[Ly.o_lam + RH + 2 * r + 1] = -s2;
            mins = fmin(mins, fmin(s1, s2)); minl = fmin(minl, fmin(-s1, -s2));
        }
        if (Q > 0) {
            double sv[QM], lv[QM];
            for (int r = 0; r < Q; ++r) {
                const double* ar = rowp(B, RH + NS + r);
                sv[r] = ar[NZ] - dot(ar, z);
                lv[r] = -sv[r];
                B[Ly.o_s + NLP + r] = sv[r]; B[Ly.o_lam + NLP + r] = lv[r];
            }
            mins = fmin(mins, Soc<QM>::mineig(sv, Q));
            minl = fmin(minl, Soc<QM>::mineig(lv, Q));
        }
        #pragma unroll
        for (int i = 0; i < NXA; ++i) B[Ly.o_y + i] = 0.0;
    }
    {
        const double as = blk_min(mins), al = blk_min(minl);
        const double sh_s = fmax(0.0, 1.0 - as), sh_l = fmax(0.0, 1.0 - al);
        for (int t = tid; t < K; t += NT) {
            double* B = nb(t);
            const int nh = (int)B[Ly.o_nh];
            for (int r = 0; r < NLP; ++r) {
                if (r >= nh && r < RH) continue;
                B[Ly.o_s + r] += sh_s; B[Ly.o_lam + r] += sh_l;
            }
            if (Q > 0) { B[Ly.o_s + NLP] += sh_s; B[Ly.o_lam + NLP] += sh_l; }
        }
    }
    double y0[NX];
    #pragma unroll
    for (int i = 0; i < NX; ++i) y0[i] = 0.0;
    __syncthreads();

    // ------------------------------------------------------------------ IPM iterations
    int status = 1, it = 0;
    bool near_ok = false;
    // primal regularisation of the iteration's Newton systems: raised x100 to retry an iteration whose
    // direction broke down (Riccati overflow in the end-game), relaxed x0.01 after every taken step
    double regv = T.reg;
    double pres_best = INFINITY, dres_best = INFINITY;
    double score_best = INFINITY;  // max(pres/pscale, dres/dscale, gap/max(1,|pobj|)) of the snapshot (o_zb / o_sgb)
    bool restore = false;
#ifdef SCP_TRACE
    long long tr_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    long long tr_last = __builtin_amdgcn_s_memtime();
#define SCP_TR(i) { const long long now_ = __builtin_amdgcn_s_memtime(); tr_acc[i] += now_ - tr_last; tr_last = now_; }
#else
#define SCP_TR(i)
#endif
    for (it = 0; it < T.max_iter; ++it) {
        // ---- residuals (node-parallel); rp needs xi~_{t+1}
        double gapl = 0.0, pobjl = 0.0, presl = 0.0, dresl = 0.0;
        for (int t = tid; t < K; t += NT) {
            double* B = nb(t);
            const int nh = (int)B[Ly.o_nh];
            double z[NZ], rd[NZ];
            #pragma unroll
            for (int i = 0; i < NZ; ++i) z[i] = B[Ly.o_z + i];
            #pragma unroll
            for (int i = 0; i < NZ; ++i) {
                double v = B[Ly.o_q + i];
                if (hasP)
                    #pragma unroll
                    for (int j = 0; j < NZ; ++j) v += B[Ly.o_P + i * NZ + j] * z[j];
                pobjl += z[i] * (B[Ly.o_q + i] + 0.5 * (v - B[Ly.o_q + i]));
                rd[i] = v;
            }
            rows_residual<NZ>(B + Ly.o_rows, B + Ly.o_lam, B + Ly.o_s, B + Ly.o_rc, nh, z, rd, presl, gapl);
            for (int r = 0; r < NS; ++r) {
                const double* ar = rowp(B, RH + r);
                const double l1 = B[Ly.o_lam + RH + 2 * r], l2 = B[Ly.o_lam + RH + 2 * r + 1];
                const double s1 = B[Ly.o_s + RH + 2 * r], s2 = B[Ly.o_s + RH + 2 * r + 1];
                const double sg = B[Ly.o_sig + r];
                #pragma unroll
                for (int i = 0; i < NZ; ++i) rd[i] += ar[i] * l1;
                const double rs = soft_w(r) - l1 - l2;
                B[Ly.o_rsig + r] = rs;
                dresl = fmax(dresl, fabs(rs));
                const double rc1 = dot(ar, z) - sg + s1 - ar[NZ], rc2 = -sg + s2;
                B[Ly.o_rc + RH + 2 * r] = rc1; B[Ly.o_rc + RH + 2 * r + 1] = rc2;
                presl = fmax(presl, fmax(fabs(rc1), fabs(rc2)));
                gapl += s1 * l1 + s2 * l2;
                pobjl += soft_w(r) * sg;
            }
            for (int r = 0; r < Q; ++r) {
                const double* ar = rowp(B, RH + NS + r);
                const double l = B[Ly.o_lam + NLP + r], s = B[Ly.o_s + NLP + r];
                #pragma unroll
                for (int i = 0; i < NZ; ++i) rd[i] += ar[i] * l;
                const double rc = dot(ar, z) + s - ar[NZ];
                B[Ly.o_rc + NLP + r] = rc;
                presl = fmax(presl, fabs(rc));
                gapl += s * l;
            }
            // rd0 (no multipliers) -> o_rd; the full residual adds the dynamics multipliers
            #pragma unroll
            for (int i = 0; i < NZ; ++i) B[Ly.o_rd + i] = pinned(t, i) ? 0.0 : rd[i];
            if (t < K - 1) {
                double y[NXA];
                #pragma unroll
                for (int i = 0; i < NXA; ++i) y[i] = B[Ly.o_y + i];
                #pragma unroll
                for (int j = 0; j < NXA; ++j)
                    #pragma unroll
                    for (int i = 0; i < NXA; ++i) rd[j] += B[Ly.o_At + i * NXA + j] * y[i];
                #pragma unroll
                for (int j = 0; j < NUA; ++j)
                    #pragma unroll
                    for (int i = 0; i < NXA; ++i) rd[NXA + j] += B[Ly.o_Bt + i * NUA + j] * y[i];
                const double* Bn = nb(t + 1);
                #pragma unroll
                for (int i = 0; i < NXA; ++i) {
                    double v = B[Ly.o_ct + i] - Bn[Ly.o_z + i];
                    for (int k = 0; k < NXA; ++k) v += B[Ly.o_At + i * NXA + k] * z[k];
                    for (int k = 0; k < NUA; ++k) v += B[Ly.o_Bt + i * NUA + k] * z[NXA + k];
                    B[Ly.o_rp + i] = v;
                    presl = fmax(presl, fabs(v));
                }
            }
            if (t > 0) {
                const double* Bp = nb(t - 1);
                #pragma unroll
                for (int i = 0; i < NXA; ++i) rd[i] -= Bp[Ly.o_y + i];
            } else {
                #pragma unroll
                for (int i = 0; i < NX; ++i) {
                    rd[i] -= y0[i];
                    const double ri = z[i] - xinit[i];
                    presl = fmax(presl, fabs(ri));
                }
            }
            #pragma unroll
            for (int i = 0; i < NZ; ++i)
                if (!pinned(t, i)) dresl = fmax(dresl, fabs(rd[i]));
        }
        SCP_TR(0)
        const double gap = blk_sum(gapl), pobj = blk_sum(pobjl), pres = blk_max(presl), dres = blk_max(dresl);
        if (!(gap == gap) || !(pres == pres) || !(dres == dres)) { status = 2; break; }
        if (pres < T.tol * pscale && dres < T.tol * dscale && gap < T.tol * fmax(1.0, fabs(pobj))) { status = 0; break; }
        // ECOS-style reduced tolerances: an iterate meeting them is reported "optimal_inaccurate"
        // if the iteration cap or a numerical breakdown ends the solve before full accuracy
        near_ok = pres < fmax(1e-4, T.tol) * pscale && dres < fmax(1e-4, T.tol) * dscale &&
                  gap < fmax(5e-5, T.tol) * fmax(1.0, fabs(pobj));  // ECOS reduced tolerances
        // insufficient progress (ECOS's end-game exit): once the reduced tolerances hold, a residual
        // that jumps 100x above its best (the Newton systems' accuracy floor, barrier ratios ~1e16) ends
        // the solve as optimal_inaccurate instead of letting the iterate drift away
        // ... on the best iterate seen since they first held (ECOS restores its best iterate there)
        if (near_ok && (pres > fmax(100.0 * pres_best, T.tol * pscale) || dres > fmax(100.0 * dres_best, T.tol * dscale))) {
            status = 1;
            restore = score_best < INFINITY;
            break;
        }
        pres_best = fmin(pres_best, pres);
        dres_best = fmin(dres_best, dres);
        {
            const double score = fmax(fmax(pres / pscale, dres / dscale), gap / fmax(1.0, fabs(pobj)));
            if (near_ok && score < score_best) {  // snapshot (uniform branch: the scores are wave reductions)
                score_best = score;
                for (int t = tid; t < K; t += NT) {
                    double* B = nb(t);
                    #pragma unroll
                    for (int i = 0; i < NZ; ++i) B[Ly.o_zb + i] = B[Ly.o_z + i];
                    for (int r = 0; r < NS; ++r) B[Ly.o_sgb + r] = B[Ly.o_sig + r];
                }
            }
        }
        const double mu = gap / deg;
        if (tid < NX) sMisc[tid] = nb(0)[Ly.o_z + tid] - xinit[tid];  // r_init
        // ---- scaling and node Hessians
        for (int t = tid; t < K; t += NT) {
            double* B = nb(t);
            const int nh = (int)B[Ly.o_nh];
            double Hu[NZ * NZ];
            #pragma unroll
            for (int e = 0; e < NZ * NZ; ++e) Hu[e] = hasP ? B[Ly.o_P + e] : 0.0;
            rows_scale(B + Ly.o_s, B + Ly.o_lam, B + Ly.o_wl, B + Ly.o_lt, 0, nh);
            rows_scale(B + Ly.o_s, B + Ly.o_lam, B + Ly.o_wl, B + Ly.o_lt, RH, NLP);
            for (int r = 0; r < nh; ++r) {
                const double* ar = rowp(B, r);
                const double d = B[Ly.o_lam + r] / B[Ly.o_s + r];
                #pragma unroll
                for (int i = 0; i < NZ; ++i) {
                    const double di = d * ar[i];
                    #pragma unroll
                    for (int j = i; j < NZ; ++j) Hu[i * NZ + j] += di * ar[j];
                }
            }
            for (int r = 0; r < NS; ++r) {
                const double* ar = rowp(B, RH + r);
                const double d1 = B[Ly.o_lam + RH + 2 * r] / B[Ly.o_s + RH + 2 * r];
                const double d2 = B[Ly.o_lam + RH + 2 * r + 1] / B[Ly.o_s + RH + 2 * r + 1];
                const double d = d1 * d2 / (d1 + d2);
                #pragma unroll
                for (int i = 0; i < NZ; ++i) {
                    const double di = d * ar[i];
                    #pragma unroll
                    for (int j = i; j < NZ; ++j) Hu[i * NZ + j] += di * ar[j];
                }
            }
            if (Q > 0) {
                double s[QM], l[QM], w[QM], eta;
                for (int r = 0; r < Q; ++r) { s[r] = B[Ly.o_s + NLP + r]; l[r] = B[Ly.o_lam + NLP + r]; }
                Soc<QM>::nt(s, l, w, eta, Q);
                for (int r = 0; r < Q; ++r) B[Ly.o_sw + r] = w[r];
                B[Ly.o_sw + Q] = eta;
                double lt[QM];
                Soc<QM>::wmul(w, eta, l, lt, Q, false);
                for (int r = 0; r < Q; ++r) B[Ly.o_lt + NLP + r] = lt[r];
                // Wi^2 (Q x Q) column by column, then H += Gs' Wi^2 Gs
                double M[QM * QM];
                for (int c = 0; c < Q; ++c) {
                    double e[QM], t1[QM], t2[QM];
                    for (int r = 0; r < Q; ++r) e[r] = r == c ? 1.0 : 0.0;
                    Soc<QM>::wmul(w, eta, e, t1, Q, true);
                    Soc<QM>::wmul(w, eta, t1, t2, Q, true);
                    for (int r = 0; r < Q; ++r) M[r * QM + c] = t2[r];
                }
                for (int r1 = 0; r1 < Q; ++r1) {
                    const double* a1 = rowp(B, RH + NS + r1);
                    for (int r2 = 0; r2 < Q; ++r2) {
                        const double* a2 = rowp(B, RH + NS + r2);
                        const double mm = M[r1 * QM + r2];
                        if (mm == 0.0) continue;
                        #pragma unroll
                        for (int i = 0; i < NZ; ++i) {
                            const double di = mm * a1[i];
                            #pragma unroll
                            for (int j = i; j < NZ; ++j) Hu[i * NZ + j] += di * a2[j];
                        }
                    }
                }
            }
            #pragma unroll
            for (int i = 0; i < NZ; ++i) Hu[i * NZ + i] += regv;
            #pragma unroll
            for (int e = 0; e < NZ * NZ; ++e) B[Ly.o_H + e] = Hu[e / NZ <= e % NZ ? e : (e % NZ) * NZ + e / NZ];  // upper triangle, mirrored
        }
        __syncthreads();
        SCP_TR(1)
        factor();
        SCP_TR(2)

        // ---- one Newton direction: corrector = false -> affine (predictor)
        auto direction = [&](bool corr, double sgmu) __attribute__((always_inline)) -> double {
            for (int t = tid; t < K; t += NT) {
                double* B = nb(t);
                const int nh = (int)B[Ly.o_nh];
                double f[NZ];
                #pragma unroll
                for (int i = 0; i < NZ; ++i) f[i] = B[Ly.o_rd + i];
                // LP rows: lt = sqrt(s l), wl = sqrt(s/l); rcomp = -lt^2 [- (ds_a/wl)(wl dl_a) + sg mu]
                rows_direction<NZ>(B + Ly.o_rows, B + Ly.o_lt, B + Ly.o_wl, B + Ly.o_dsa, B + Ly.o_dla, B + Ly.o_rc,
                                   B + Ly.o_rho, B + Ly.o_t, 0, nh, true, corr, sgmu, f);
                rows_direction<NZ>(B + Ly.o_rows, B + Ly.o_lt, B + Ly.o_wl, B + Ly.o_dsa, B + Ly.o_dla, B + Ly.o_rc,
                                   B + Ly.o_rho, B + Ly.o_t, RH, NLP, false, corr, sgmu, f);
                for (int r = 0; r < NS; ++r) {
                    const double* ar = rowp(B, RH + r);
                    const double wl1 = B[Ly.o_wl + RH + 2 * r], wl2 = B[Ly.o_wl + RH + 2 * r + 1];
                    const double d1 = 1.0 / (wl1 * wl1), d2 = 1.0 / (wl2 * wl2);
                    const double t1 = B[Ly.o_t + RH + 2 * r], t2 = B[Ly.o_t + RH + 2 * r + 1];
                    const double rhs = -B[Ly.o_rsig + r] + t1 + t2;
                    B[Ly.o_rhs + r] = rhs;
                    const double c = t1 - d1 * rhs / (d1 + d2);
                    #pragma unroll
                    for (int i = 0; i < NZ; ++i) f[i] += ar[i] * c;
                }
                if (Q > 0) {
                    double w[QM], lt[QM], rc[QM], rcv[QM], rho[QM], tmp[QM], tv[QM];
                    for (int r = 0; r < Q; ++r) {
                        w[r] = B[Ly.o_sw + r]; lt[r] = B[Ly.o_lt + NLP + r]; rc[r] = B[Ly.o_rc + NLP + r];
                    }
                    const double eta = B[Ly.o_sw + Q];
                    Soc<QM>::jprod(lt, lt, rcv, Q);
                    for (int r = 0; r < Q; ++r) rcv[r] = -rcv[r];
                    if (corr) {
                        double dsa[QM], dla[QM], u1[QM], u2[QM], cp[QM];
                        for (int r = 0; r < Q; ++r) { dsa[r] = B[Ly.o_dsa + NLP + r]; dla[r] = B[Ly.o_dla + NLP + r]; }
                        Soc<QM>::wmul(w, eta, dsa, u1, Q, true);
                        Soc<QM>::wmul(w, eta, dla, u2, Q, false);
                        Soc<QM>::jprod(u1, u2, cp, Q);
                        for (int r = 0; r < Q; ++r) rcv[r] -= cp[r];
                        rcv[0] += sgmu;
                    }
                    Soc<QM>::jdiv(lt, rcv, rho, Q);
                    Soc<QM>::wmul(w, eta, rho, tv, Q, true);
                    Soc<QM>::wmul(w, eta, rc, tmp, Q, true);
                    Soc<QM>::wmul(w, eta, tmp, tmp, Q, true);
                    for (int r = 0; r < Q; ++r) {
                        tv[r] += tmp[r];
                        B[Ly.o_rho + NLP + r] = rho[r];
                        B[Ly.o_t + NLP + r] = tv[r];
                        const double* ar = rowp(B, RH + NS + r);
                        #pragma unroll
                        for (int i = 0; i < NZ; ++i) f[i] += ar[i] * tv[r];
                    }
                }
                #pragma unroll
                for (int i = 0; i < NZ; ++i) B[Ly.o_f + i] = pinned(t, i) ? 0.0 : f[i];
            }
            __syncthreads();
            SCP_TR(3)
            if constexpr (NW == 1) lqsolve_sweep(); else lqsolve();
            SCP_TR(4)
            // recover slack steps, step length
            double amax = INFINITY;
            for (int t = tid; t < K; t += NT) {
                double* B = nb(t);
                const int nh = (int)B[Ly.o_nh];
                double dz[NZ];
                #pragma unroll
                for (int i = 0; i < NZ; ++i) dz[i] = B[Ly.o_dz + i];
                auto lpstep = [&](int r, double gdz) {
                    const double wl = B[Ly.o_wl + r];
                    const double rc = B[Ly.o_rc + r];
                    const double ds = -rc - gdz;
                    const double dl = B[Ly.o_rho + r] / wl + (rc + gdz) / (wl * wl);
                    B[Ly.o_ds + r] = ds; B[Ly.o_dl + r] = dl;
                    if (ds < 0.0) amax = fmin(amax, -B[Ly.o_s + r] / ds);
                    if (dl < 0.0) amax = fmin(amax, -B[Ly.o_lam + r] / dl);
                };
                rows_step<NZ>(B + Ly.o_rows, B + Ly.o_wl, B + Ly.o_rc, B + Ly.o_rho, B + Ly.o_s, B + Ly.o_lam, B + Ly.o_ds,
                              B + Ly.o_dl, nh, dz, amax);
                for (int r = 0; r < NS; ++r) {
                    const double* ar = rowp(B, RH + r);
                    const double wl1 = B[Ly.o_wl + RH + 2 * r], wl2 = B[Ly.o_wl + RH + 2 * r + 1];
                    const double d1 = 1.0 / (wl1 * wl1), d2 = 1.0 / (wl2 * wl2);
                    const double adz = dot(ar, dz);
                    const double dsg = (B[Ly.o_rhs + r] + d1 * adz) / (d1 + d2);
                    B[Ly.o_dsig + r] = dsg;
                    lpstep(RH + 2 * r, adz - dsg);
                    lpstep(RH + 2 * r + 1, -dsg);
                }
                if (Q > 0) {
                    double w[QM], gdz[QM], rc[QM], rho[QM], ds[QM], dl[QM], tmp[QM], sv[QM], lv[QM];
                    for (int r = 0; r < Q; ++r) {
                        w[r] = B[Ly.o_sw + r];
                        gdz[r] = dot(rowp(B, RH + NS + r), dz);
                        rc[r] = B[Ly.o_rc + NLP + r];
                        rho[r] = B[Ly.o_rho + NLP + r];
                        sv[r] = B[Ly.o_s + NLP + r];
                        lv[r] = B[Ly.o_lam + NLP + r];
                    }
                    const double eta = B[Ly.o_sw + Q];
                    for (int r = 0; r < Q; ++r) { ds[r] = -rc[r] - gdz[r]; tmp[r] = rc[r] + gdz[r]; }
                    Soc<QM>::wmul(w, eta, tmp, tmp, Q, true);
                    Soc<QM>::wmul(w, eta, tmp, tmp, Q, true);
                    Soc<QM>::wmul(w, eta, rho, dl, Q, true);
                    for (int r = 0; r < Q; ++r) {
                        dl[r] += tmp[r];
                        B[Ly.o_ds + NLP + r] = ds[r];
                        B[Ly.o_dl + NLP + r] = dl[r];
                    }
                    amax = fmin(amax, fmin(Soc<QM>::step(sv, ds, Q), Soc<QM>::step(lv, dl, Q)));
                }
            }
            const double am = blk_min(amax);
            SCP_TR(5)
            return am;
        };

        const double aa = fmin(1.0, direction(false, 0.0));
        double mual = 0.0;
        for (int t = tid; t < K; t += NT) {
            double* B = nb(t);
            const int nh = (int)B[Ly.o_nh];
            rows_mu(B + Ly.o_s, B + Ly.o_lam, B + Ly.o_ds, B + Ly.o_dl, 0, nh, aa, mual);
            rows_mu(B + Ly.o_s, B + Ly.o_lam, B + Ly.o_ds, B + Ly.o_dl, RH, RL, aa, mual);
            // Mehrotra corrector terms in scaled coordinates: LP (ds_a / wl) * (wl dl_a) = ds_a dl_a;
            // SOC: keep ds_a, dl_a raw (scaled inside direction())
            rows_copy2(B + Ly.o_ds, B + Ly.o_dl, B + Ly.o_dsa, B + Ly.o_dla, RL);
        }
        const double mu_a = blk_sum(mual) / deg;
        const double sg = (mu_a / mu) * (mu_a / mu) * (mu_a / mu);
#ifdef SCP_DEGEN
        {   // diagnostics: which rows carry the predicted complementarity (s + aa ds)(l + aa dl) of the affine step, by
            // row type (x / u / nu trust-region facets, bounds + slabs + node-0 rows, soft rows); "deg" counts rows whose
            // slack and dual both fall to at least a quarter of their value (products >= 0.05 s l)
            double share[5] = {0, 0, 0, 0, 0}, cntd[5] = {0, 0, 0, 0, 0};
            for (int t = tid; t < K; t += NT) {
                double* B = nb(t);
                const int nh = (int)B[Ly.o_nh];
                for (int r = 0; r < RL; ++r) {
                    if (r >= nh && r < RH) continue;
                    int ty = 4;
                    if (r < RH) {
                        const int q = r - (1 << NX) - (1 << NU);
                        ty = r < (1 << NX) ? 0 : (q < 0 ? 1 : ((t < K - 1 && q < (1 << NX)) ? 2 : 3));
                    }
                    const double sv = B[Ly.o_s + r], lv = B[Ly.o_lam + r], ds = B[Ly.o_dsa + r], dl = B[Ly.o_dla + r];
                    const double c = (sv + aa * ds) * (lv + aa * dl);
                    if (agent == 0 && it >= 16 && t == 50 && c >= 0.05 * sv * lv) {
                        const double* ar = B + Ly.o_rows + r * (NZ + 1);
                        int nzi[4] = {-1, -1, -1, -1}, k = 0;
                        for (int i = 0; i < NZ && k < 4; ++i)
                            if (ar[i] != 0.0) nzi[k++] = i;
                        printf("SCP_DEGEN_ROW it %d t %d r %d ty %d s %.3e l %.3e ds %.3e dl %.3e | nz %d %d %d %d coef %.3e h %.3e\n",
                               it, t, r, ty, sv, lv, ds, dl, nzi[0], nzi[1], nzi[2], nzi[3], nzi[0] >= 0 ? ar[nzi[0]] : 0.0,
                               ar[NZ]);
                    }
                    for (int q = 0; q < 5; ++q) {
                        share[q] += q == ty ? c : 0.0;
                        cntd[q] += (q == ty && c >= 0.05 * sv * lv) ? 1.0 : 0.0;
                    }
                }
            }
            for (int q = 0; q < 5; ++q) { share[q] = blk_sum(share[q]); cntd[q] = blk_sum(cntd[q]); }
            if (agent == 0 && tid == 0)
                printf("SCP_DEGEN it %d mu %.3e mu_aff/mu %.3f aa %.4f | share x %.3f u %.3f nu %.3f bnd %.3f soft %.3f | "
                       "deg rows x %d u %d nu %d bnd %d soft %d\n", it, mu, mu_a / mu, aa, share[0] / (mu_a * deg),
                       share[1] / (mu_a * deg), share[2] / (mu_a * deg), share[3] / (mu_a * deg), share[4] / (mu_a * deg),
                       (int)cntd[0], (int)cntd[1], (int)cntd[2], (int)cntd[3], (int)cntd[4]);
        }
#endif
        __syncthreads();
        // step fraction 0.99, or 1 - 1e-5 once the affine predictor takes a (nearly) full step: the end game,
        // where a fixed 0.99 caps the gap reduction at 100x per iteration (qp_ipm.hpp QP_TAU_END, the same rule)
        const double al = fmin(1.0, (aa >= 0.99 ? SCP_TAU_END : 0.99) * direction(true, sg * mu));
#ifdef SCP_ITRACE
        if (agent == 0 && tid == 0)
            printf("SCP_ITRACE it %d pres %.3e dres %.3e gap %.3e pobj %.9e aa %.4f al %.4f sg %.2e mu %.3e ps %.2e ds %.2e near %d reg %.1e\n",
                   it, pres, dres, gap, pobj, aa, al, sg, mu, pscale, dscale, (int)near_ok, regv);
#endif
        // ---- breakdown guard: a non-finite direction (Riccati overflow in the end-game) ends the
        // solve on the current, finite iterate instead of corrupting it
        double badl = (al > 0.0) ? 0.0 : 1.0;
        for (int t = tid; t < K; t += NT) {
            const double* B = nb(t);
            const int nh = (int)B[Ly.o_nh];
            double acc = 0.0;
            #pragma unroll
            for (int i = 0; i < NZ; ++i) acc += B[Ly.o_dz + i];
            for (int r = 0; r < NS; ++r) acc += B[Ly.o_dsig + r];
            for (int r = 0; r < RL; ++r) {
                if (r >= nh && r < RH) continue;
                acc += B[Ly.o_ds + r] + B[Ly.o_dl + r];
            }
            if (t < K - 1)
                #pragma unroll
                for (int i = 0; i < NXA; ++i) acc += B[Ly.o_yp + i];
            if (!(fabs(acc) < INFINITY)) badl = 1.0;
        }
        #pragma unroll
        for (int i = 0; i < NX; ++i)
            if (!(fabs(sMisc[8 + i]) < INFINITY)) badl = 1.0;
        if (blk_max(badl) > 0.0) {
            if (regv < 1e-5) { regv *= 100.0; __syncthreads(); continue; }   // retry, stiffer
            status = near_ok ? 1 : 2;
            break;
        }
        // ---- update
        for (int t = tid; t < K; t += NT) {
            double* B = nb(t);
            const int nh = (int)B[Ly.o_nh];
            #pragma unroll
            for (int i = 0; i < NZ; ++i) B[Ly.o_z + i] += al * B[Ly.o_dz + i];
            for (int r = 0; r < NS; ++r) B[Ly.o_sig + r] += al * B[Ly.o_dsig + r];
            rows_update(B + Ly.o_s, B + Ly.o_lam, B + Ly.o_ds, B + Ly.o_dl, 0, nh, al);
            rows_update(B + Ly.o_s, B + Ly.o_lam, B + Ly.o_ds, B + Ly.o_dl, RH, RL, al);
            if (t < K - 1)
                #pragma unroll
                for (int i = 0; i < NXA; ++i) B[Ly.o_y + i] += al * (B[Ly.o_yp + i] - B[Ly.o_y + i]);
        }
        #pragma unroll
        for (int i = 0; i < NX; ++i) y0[i] += al * (sMisc[8 + i] - y0[i]);
        regv = fmax(T.reg, 0.01 * regv);
        __syncthreads();
        SCP_TR(6)
    }
#ifdef SCP_TRACE
    if (agent == 0 && tid == 0)
        printf("SCP_TRACE it=%d res=%lld hess=%lld factor=%lld dirnode=%lld lqsolve=%lld step=%lld upd=%lld\n", it,
               tr_acc[0], tr_acc[1], tr_acc[2], tr_acc[3], tr_acc[4], tr_acc[5], tr_acc[6]);
#endif

    if (status == 1 && it == T.max_iter && !near_ok) status = 2;   // cap reached far from optimal
    if (restore) {
        for (int t = tid; t < K; t += NT) {
            double* B = nb(t);
            #pragma unroll
            for (int i = 0; i < NZ; ++i) B[Ly.o_z + i] = B[Ly.o_zb + i];
            for (int r = 0; r < NS; ++r) B[Ly.o_sig + r] = B[Ly.o_sgb + r];
        }
        __syncthreads();
    }
    // ------------------------------------------------------------------ outputs
    double sigv = sfix ? sref : nb(0)[Ly.o_z + SIG];
    double numaxl = 0.0, softl = 0.0, admml = 0.0;
    for (int t = tid; t < K; t += NT) {
        double* B = nb(t);
        double u[NU], x[NX];
        #pragma unroll
        for (int j = 0; j < NU; ++j) u[j] = B[Ly.o_z + ZU + j];
        #pragma unroll
        for (int i = 0; i < NX; ++i) {
            double v = B[Ly.o_z + i];
            #pragma unroll
            for (int j = 0; j < NU; ++j) v += Cprev(t, i, j) * u[j];
            x[i] = v;
            a.X[(agent * K + t) * NX + i] = v;
        }
        #pragma unroll
        for (int j = 0; j < NU; ++j) a.U[(agent * K + t) * NU + j] = u[j];
        for (int o = 0; o < T.n_obs; ++o) {
            const double sg = B[Ly.o_sig + o];
            a.s_obs[(agent * T.n_obs + o) * K + t] = sg;
            softl += T.w_slack * sg;
        }
        for (int j = 0; j < T.n_nbr; ++j) {
            const double sg = B[Ly.o_sig + T.n_obs + j];
            a.s_nbr[(agent * T.n_nbr + j) * K + t] = sg;
            softl += T.w_coll * sg;
            const long long base = ((agent * T.n_nbr + j) * K + t) * pd;
            for (int i = 0; i < pd; ++i) {
                const double df = x[i] - a.nbr_Y[base + i];
                admml += a.nbr_Lam[base + i] * df + 0.5 * T.rho * df * df;
            }
        }
        if (t < K - 1 && !(fin && t == K - 2)) {
            double s1 = 0.0;
            #pragma unroll
            for (int i = 0; i < NX; ++i) {
                const double v = B[Ly.o_z + ZN + i];
                a.nu[(agent * (K - 1) + t) * NX + i] = v;
                s1 += fabs(v);
            }
            numaxl = fmax(numaxl, s1);
        }
    }
    __syncthreads();
    // nu_{K-2} from the dynamics (x_{K-1} = x_final)
    if (fin && K >= 2 && tid == 0) {
        const int t = K - 2;
        const double* dk = disc + (long long)t * DSTR;
        const double* xk = a.X + (agent * K + t) * NX;
        const double* uk = a.U + (agent * K + t) * NU;
        const double* uk1 = a.U + (agent * K + t + 1) * NU;
        double s1 = 0.0;
        #pragma unroll
        for (int i = 0; i < NX; ++i) {
            double v = xfin[i] - dk[NX * NX + 2 * NX * NU + i] * sigv - dk[NX * NX + 2 * NX * NU + NX + i];
            for (int l = 0; l < NX; ++l) v -= dk[l * NX + i] * xk[l];
            #pragma unroll
            for (int j = 0; j < NU; ++j) v -= dk[NX * NX + j * NX + i] * uk[j] + dk[NX * NX + NX * NU + j * NX + i] * uk1[j];
            a.nu[(agent * (K - 1) + t) * NX + i] = v;
            s1 += fabs(v);
        }
        numaxl = fmax(numaxl, s1);
    }
    double gamel = 0.0;
    if (NE > 0) {  // the game cost at the solution (game_model.py:87-100)
        __syncthreads();
        for (int t = tid; t < K; t += NT) {
            const double* x = a.X + (agent * K + t) * NX;
            const double* u = a.U + (agent * K + t) * NU;
            #pragma unroll
            for (int j = 0; j < NU; ++j) gamel += T.w_u2 * u[j] * u[j];
            if (T.w_in > 0.0)
                #pragma unroll
                for (int i = 0; i < NX; ++i) {
                    const double d = x[i] - a.X_prev[(agent * K + t) * NX + i];
                    gamel += T.w_in * d * d;
                }
            if (t > 0) {
                #pragma unroll
                for (int j = 0; j < NU; ++j) { const double d = u[j] - u[j - NU]; gamel += T.w_du * d * d; }
                if (T.theta_idx >= 0) {
                    const double d = x[T.theta_idx] - x[T.theta_idx - NX];
                    gamel += T.w_dth * d * d;
                }
            }
        }
    }
    const double numax = blk_max(numaxl), soft = blk_sum(softl), admm = blk_sum(admml), game = blk_sum(gamel);
    if (tid == 0) {
        a.sigma[agent] = sigv;
        a.obj[agent] = T.w_nu * numax + soft + T.w_sigma * sigv + admm + game;
        a.status[agent] = status;
        a.iters[agent] = it;
    }
}


}  // namespace scvx
