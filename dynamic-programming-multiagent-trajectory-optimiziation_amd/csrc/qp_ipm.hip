// Batched trust-region QP/SOCP solve for the SCvx inner loop (MI355X / gfx950, float64).
//
// Replaces the per-agent CVXPY+Clarabel solve of Distributed_opt/dist_scvx_3d.py:51-111
// (x_traj_opt), batched over N agents; the problem is stated in include/scvx_hip.h.
//
// Algorithm: primal-dual interior point, Mehrotra predictor-corrector, Nesterov-Todd scaling
// for the per-node second-order cone ||u_t|| <= u_max, CVXOPT-style starting point.  Each
// Newton system
//      [H  A'] [dz]   [r1]
//      [A  0 ] [dy] = [r2]       (A: initial state, dynamics, terminal state)
// is solved by a Riccati recursion over the K nodes in the FOH-transformed state
// xi_t = x_t - C_{t-1} u_t (so x_{t+1} = A_t x_t + B_t u_t + C_t u_{t+1} + c_t becomes a
// standard xi_{t+1} = A_t xi_t + (B_t + A_t C_{t-1}) u_t + c_t); the terminal equality is
// handled by an n x n Schur complement on its multiplier, accumulated in the same backward
// sweep (M = sum_t W2_t' kappa_t).  The node-local slack variables of the soft constraints
// (obstacle slacks, the shared collision slack S_t of dist_scvx_3d.py:93-107) are eliminated
// per node before the sweep.
//
// Mapping (one agent per 64-lane wavefront = one workgroup):
//   * node phases   -- lane t owns node t: its primal z_t, slacks s, duals lambda and SOC pair
//                      live in registers for the whole solve; residuals, NT scaling, node
//                      Hessians and step lengths are computed lane-parallel over the nodes;
//   * Riccati sweeps -- sequential over the nodes, element-parallel over the lanes: every small
//                      matrix product of a stage is spread one output element per lane
//                      through LDS (wave_ops.hpp).
// Per-stage factors go to an agent-private global workspace (L2-resident between the
// factor sweep and the two solve sweeps of an iteration).
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "scvx_hip.h"
#include "wave_ops.hpp"

namespace scvx {

struct QPArgs {
    scvx_qp_template T;
    int N;
    const double* disc;
    const double* sigma;
    const double* Xref;
    const double* Uref;
    const double* x_init;
    const double* x_final;
    const double* tr;
    const double* coll_rows;
    const int32_t* coll_count;
    double* X;
    double* U;
    double* slack_coll;
    double* obj;
    int32_t* status;
    int32_t* iters;
    double* ws;          // workspace
    long long ws_agent;  // doubles per agent
    double* trace;       // optional per-iteration diagnostics of agent `trace_agent` (or nullptr)
    int trace_agent, trace_cap;
    int rows_max;        // orthant rows per node (upper bound over nodes)
    int gmax;            // slack groups per node (>= 1)
};

// per-stage block layout in the agent workspace
template <int NX, int NU>
struct StageLayout {
    static constexpr int Q = 0;
    static constexpr int S = Q + NX * NX;           // NX x NU
    static constexpr int R = S + NX * NU;           // NU x NU
    static constexpr int q = R + NU * NU;           // NX
    static constexpr int r = q + NX;                // NU
    static constexpr int e = r + NU;                // NX
    static constexpr int Bt = e + NX;               // NX x NU
    static constexpr int Kg = Bt + NX * NU;         // NU x NX
    static constexpr int L = Kg + NU * NX;          // NU x NU
    static constexpr int kap = L + NU * NU;         // NU x NX
    static constexpr int W2 = kap + NU * NX;        // NU x NX
    static constexpr int P = W2 + NU * NX;          // NX x NX
    static constexpr int Pi = P + NX * NX;          // NX x NX
    static constexpr int k0 = Pi + NX * NX;         // NU
    static constexpr int p0 = k0 + NU;              // NX
    static constexpr int size = p0 + NX;
};

static void qp_row_counts(const scvx_qp_template& T, int& rows, int& ngroups) {
    ngroups = T.n_obs + (T.j_max > 0 ? 1 : 0);
    rows = (1 << T.n_u) + 2 * T.n_box + T.n_obs + T.j_max + ngroups;
}

// agent workspace: stage blocks | soft rows [q][i][lane] | row columns [4][rows][lane] |
// group columns [8][groups][lane]   (column layouts: lane-contiguous, coalesced over nodes)
static long long qp_ws_doubles_per_agent(const scvx_qp_template& T, int nx, int nu) {
    const int SB = 4 * nx * nx + 6 * nx * nu + 2 * nu * nu + 4 * nx + 3 * nu;
    int rows, ng;
    qp_row_counts(T, rows, ng);
    const int soft = T.n_obs + T.j_max;
    const int gmax = ng > 0 ? ng : 1;
    return (long long)T.K * SB + (long long)soft * (T.pos_dim + 1) * 64 + 4LL * rows * 64 + 8LL * gmax * 64 + 64;
}

template <int NX, int NU>
__global__ __launch_bounds__(64) void qp_ipm_kernel(QPArgs a) {
    using SL = StageLayout<NX, NU>;
    constexpr int NZ = NX + NU;
    constexpr int NQ = NU + 1;   // SOC dimension
    constexpr int NTR = 1 << NU; // L1-ball facets
    const scvx_qp_template& T = a.T;
    const int K = T.K, pd = T.pos_dim, lane = threadIdx.x, t = lane;
    const long long agent = blockIdx.x;
    const bool act = t < K;
    const bool ineq = act && ((t < K - 1) || T.ineq_last);
    const bool fin = T.has_final != 0;
    const bool soc = ineq && T.has_soc;
    const int ngroups = T.n_obs + (T.j_max > 0 ? 1 : 0);
    const int ccount = (ineq && T.j_max > 0) ? min((int)a.coll_count[agent * K + t], T.j_max) : 0;
    const int nsoft = ineq ? T.n_obs + ccount : 0;
    const int r_box0 = NTR, r_soft0 = NTR + 2 * T.n_box, r_grp0 = r_soft0 + nsoft;
    const int nrows = ineq ? r_grp0 + ngroups : 0;
    const int na = ineq ? ngroups : 0;
    const double trv = a.tr[agent];
    const double sig = a.sigma[agent];
    const int DSTR = NX * (NX + 2 * NU + 2);
    const double* disc = a.disc + agent * (long long)(K - 1) * DSTR;
    double* ws = a.ws + agent * a.ws_agent;
    double* stage = ws;
    const int softmax = T.n_obs + T.j_max;
    double* soft = ws + (long long)K * SL::size;                     // [q][i][lane]
    double* rowc = soft + (long long)softmax * (pd + 1) * WAVE;       // [4][rows][lane]
    double* grpc = rowc + 4LL * a.rows_max * WAVE;                     // [8][groups][lane]
    // node-private columns (element k of this lane at ptr[k * WAVE])
    double* cS = rowc + lane;                         // slacks s_r
    double* cL = rowc + 1LL * a.rows_max * WAVE + lane;  // duals lambda_r
    double* cP = rowc + 2LL * a.rows_max * WAVE + lane;  // predictor products ds_r dl_r
    double* cR = rowc + 3LL * a.rows_max * WAVE + lane;  // residuals rc_r
    double* gA = grpc + lane;                               // slack variables a_g
    double* gHaa = grpc + 1LL * a.gmax * WAVE + lane;       // eliminated block H_aa
    double* gH0 = grpc + 2LL * a.gmax * WAVE + lane;        // H_pa (3 columns)
    double* gRd = grpc + 5LL * a.gmax * WAVE + lane;        // dual residual (aux part)
    double* gR1 = grpc + 6LL * a.gmax * WAVE + lane;        // Newton rhs (aux part)
    double* gDa = grpc + 7LL * a.gmax * WAVE + lane;        // aux direction

    __shared__ double sA[NX * NX], sBt[NX * NU], sQ[NX * NX], sS[NX * NU], sR[NU * NU];
    __shared__ double sPp[NX * NX], sPip[NX * NX], sT1[NX * NX], sT2[NX * NU], sW1[NX * NX], sW2[NU * NX];
    __shared__ double sQh[NX * NX], sSh[NU * NX], sRh[NU * NU], sKk[NU * 2 * NX], sM[NX * NX];
    __shared__ double sv[8][16];
    __shared__ int spiv[NX];
    __shared__ double sz[WAVE][NZ], sy[WAVE][NX], sdz[WAVE][NZ], sdy[WAVE][NX];
    __shared__ double syi[NX], syf[NX], sdyi[NX], sdyf[NX], sflag[4];
    __shared__ double sStamp[16];
    __shared__ double sRing[3 * (StageLayout<NX, NU>::size + NX * NX + NX * NU)];

    // ------------------------------------------------------------------ node constants
    double xb[NX], ub[NU], Cp[NX * NU];  // reference point, C_{t-1} (column-major as disc)
#pragma unroll
    for (int i = 0; i < NX; ++i) xb[i] = act ? a.Xref[(agent * K + t) * NX + i] : 0.0;
#pragma unroll
    for (int j = 0; j < NU; ++j) ub[j] = act ? a.Uref[(agent * K + t) * NU + j] : 0.0;
#pragma unroll
    for (int e = 0; e < NX * NU; ++e) Cp[e] = (act && t > 0) ? disc[(t - 1) * DSTR + NX * NX + NX * NU + e] : 0.0;
    const double wu = (t < K - 1) ? 1.0 : T.w_last;
    const bool fixed_u = act && (t == K - 1) && T.fix_last_input;

    // soft rows (g, b): obstacle linearisations (single_integrator_model.py:113-126), then the
    // collision rows of dist_scvx_3d.py:93-107 supplied by the caller
    auto softp = [&](int q, int i) __attribute__((always_inline)) -> double& { return soft[((long long)q * (pd + 1) + i) * WAVE + lane]; };
    if (ineq) {
        for (int o = 0; o < T.n_obs; ++o) {
            double d[3] = {0, 0, 0}, nr = 0.0, bo = T.obs_radius[o];
            for (int i = 0; i < pd; ++i) { d[i] = xb[i] - T.obs_center[o][i]; nr += d[i] * d[i]; }
            nr = sqrt(nr) + 1e-6;
            for (int i = 0; i < pd; ++i) { softp(o, i) = d[i] / nr; bo += d[i] / nr * T.obs_center[o][i]; }
            softp(o, pd) = bo;
        }
        for (int j = 0; j < ccount; ++j) {
            const double* src = a.coll_rows + ((agent * K + t) * T.j_max + j) * (pd + 1);
            for (int i = 0; i <= pd; ++i) softp(T.n_obs + j, i) = src[i];
        }
    }
    auto soft_row = [&](int q, double* g, double& b) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 3; ++i) g[i] = (i < pd) ? softp(q, i) : 0.0;
        b = softp(q, pd);
    };
    auto group_of = [&](int q) __attribute__((always_inline)) { return q < T.n_obs ? q : T.n_obs; };

    // G_r [z; aux] and h_r of orthant row r at this node (aux: a group column pointer)
    auto row_eval = [&](int r, const double* z, const double* auxc, double& gz, double& h) __attribute__((always_inline)) {
        if (r < NTR) {
            gz = 0.0; h = trv;
#pragma unroll
            for (int j = 0; j < NU; ++j) {
                const double sg = ((r >> j) & 1) ? -1.0 : 1.0;
                gz += sg * z[NX + j]; h += sg * ub[j];
            }
        } else if (r < r_soft0) {
            const int b = (r - r_box0) >> 1, lo = (r - r_box0) & 1, idx = T.box_idx[b];
            double xi = 0.0;
#pragma unroll
            for (int i = 0; i < NX; ++i) xi = (i == idx) ? z[i] : xi;
            gz = lo ? -xi : xi; h = lo ? -T.box_lo[b] : T.box_hi[b];
        } else if (r < r_grp0) {
            double g[3], b;
            const int q = r - r_soft0;
            soft_row(q, g, b);
            gz = -(g[0] * z[0] + g[1] * z[1] + g[2] * (pd > 2 ? z[2] : 0.0)) - auxc[group_of(q) * WAVE];
            h = -b;
        } else {
            gz = -auxc[(r - r_grp0) * WAVE]; h = 0.0;
        }
    };
    // gzv += c * G_r'|_z ; gav column += c * G_r'|_aux
    auto row_accT = [&](int r, double c, double* gzv, double* gav) __attribute__((always_inline)) {
        if (r < NTR) {
#pragma unroll
            for (int j = 0; j < NU; ++j) gzv[NX + j] += (((r >> j) & 1) ? -c : c);
        } else if (r < r_soft0) {
            const int b = (r - r_box0) >> 1, lo = (r - r_box0) & 1, idx = T.box_idx[b];
#pragma unroll
            for (int i = 0; i < NX; ++i) gzv[i] += (i == idx) ? (lo ? -c : c) : 0.0;
        } else if (r < r_grp0) {
            double g[3], b;
            const int q = r - r_soft0;
            soft_row(q, g, b);
            gzv[0] -= c * g[0]; gzv[1] -= c * g[1];
            if (pd > 2) gzv[2] -= c * g[2];
            gav[group_of(q) * WAVE] -= c;
        } else {
            gav[(r - r_grp0) * WAVE] -= c;
        }
    };

    // ------------------------------------------------------------------ primal/dual state
    double z[NZ], sq[NQ], lq[NQ];
#pragma unroll
    for (int i = 0; i < NX; ++i) z[i] = xb[i];
#pragma unroll
    for (int j = 0; j < NU; ++j) z[NX + j] = ub[j];
    for (int g = 0; g < a.gmax; ++g) gA[g * WAVE] = 0.0;
#pragma unroll
    for (int j = 0; j < NQ; ++j) { sq[j] = 0.0; lq[j] = 0.0; }
    if (lane < NX) { syi[lane] = 0.0; syf[lane] = 0.0; }
#pragma unroll
    for (int i = 0; i < NX; ++i) sy[lane][i] = 0.0;
    __syncthreads();

    // per-iteration node quantities (registers)
    double rd[NZ], rcq[NQ], rp[NX];
    double W[NQ * NQ], Wi[NQ * NQ], ltq[NQ];  // SOC NT scaling, scaled point

    // ---------------------------------------------------------------- Riccati machinery
    // Stage packets: [stage block (SL) | A_t (disc, col-major) | C_{t-1} (disc, col-major)], streamed
    // from the agent workspace into a 3-slot LDS ring one stage ahead of the sweep, so the
    // sequential chain only ever waits on LDS (the global loads of stage t-+1 fly during stage t).
    // Each phase of a stage is straight-line: a lane picks its output element(s) (pointer/stride
    // selection only), then one shared dot-product body runs for every output kind, so a phase
    // costs one LDS round trip plus a short FMA chain.
    constexpr int PKT = SL::size + NX * NX + NX * NU;
    constexpr int PFN = (PKT + WAVE - 1) / WAVE;
    constexpr int OA = SL::size, OC = SL::size + NX * NX;
    const bool stamp_on = a.trace && agent == a.trace_agent;
    auto slot = [&](int ts) __attribute__((always_inline)) -> double* { return sRing + (ts % 3) * PKT; };
    auto pf_issue = [&](int ts, double* r) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < PFN; ++k) {
            const int e = lane + WAVE * k;
            const double* src = stage + (long long)ts * SL::size + e;
            if (e >= SL::size && e < OC) src = disc + (long long)(ts < K - 1 ? ts : 0) * DSTR + (e - OA);
            if (e >= OC) src = disc + (long long)(ts > 0 ? ts - 1 : 0) * DSTR + NX * NX + NX * NU + (e - OC);
            const bool zero = (e >= SL::size && e < OC && ts >= K - 1) || (e >= OC && ts == 0);
            r[k] = (e < PKT && !zero) ? *src : 0.0;
        }
    };
    auto pf_commit = [&](int ts, const double* r) __attribute__((always_inline)) {
        double* d = slot(ts);
#pragma unroll
        for (int k = 0; k < PFN; ++k) {
            const int e = lane + WAVE * k;
            if (e < PKT) d[e] = r[k];
        }
    };
    constexpr int E1 = 2 * NX * NX + 2 * NX * NU;   // phase-1 outputs: P'A, P'Bt, A'Pi', Bt'Pi'
    constexpr int E2 = NX * NX + NU * NX + NU * NU; // phase-2 outputs: Qh, Sh, Rh
    constexpr int E4 = 3 * NX * NX;                 // phase-4 outputs: P, Pi, M-increment
    // factor: node Hessians (Q,S,R) of all stages already in the stage buffers
    auto factor = [&]() __attribute__((always_inline)) -> bool {
        double pf[PFN];
        for (int e = lane; e < NX * NX; e += WAVE) { sM[e] = 0.0; sPp[e] = 0.0; sPip[e] = 0.0; }
        if (lane == 0) sflag[0] = 0.0;
        __syncthreads();  // stage buffers were written by other lanes (global)
        pf_issue(K - 1, pf);
        pf_commit(K - 1, pf);
        wsync();
        for (int ts = K - 1; ts >= 0; --ts) {
            if (stamp_on && ts == 25 && lane == 0) sStamp[0] = (double)__builtin_amdgcn_s_memtime();
            if (ts > 0) pf_issue(ts - 1, pf);
            double* pk = slot(ts);
            double* stg = stage + (long long)ts * SL::size;  // global outputs
            const bool last = ts == K - 1;
            // ---- phase 1: T1 = P'A, T2 = P'Bt, W1 = A'Pi', W2 = Bt'Pi'   (zero / C' at the last stage)
#pragma unroll
            for (int rep = 0; rep < (E1 + WAVE - 1) / WAVE; ++rep) {
                int off = lane + rep * WAVE;
                if (off < E1) {
                    const double *Lp, *Rp;
                    int lsk, rsk;
                    double* out;
                    double base = 0.0;
                    if (off < NX * NX) {
                        const int i = off / NX, j = off % NX;
                        Lp = sPp + i * NX; lsk = 1; Rp = pk + OA + j * NX; rsk = 1; out = sT1 + off;
                    } else if ((off -= NX * NX) < NX * NU) {
                        const int i = off / NU, j = off % NU;
                        Lp = sPp + i * NX; lsk = 1; Rp = pk + SL::Bt + j; rsk = NU; out = sT2 + off;
                    } else if ((off -= NX * NU) < NX * NX) {
                        const int i = off / NX, j = off % NX;
                        Lp = pk + OA + i * NX; lsk = 1; Rp = sPip + j; rsk = NX; out = sW1 + off;
                        if (last) base = (i == j) ? 1.0 : 0.0;
                    } else {
                        off -= NX * NX;
                        const int i = off / NX, j = off % NX;
                        Lp = pk + SL::Bt + i; lsk = NU; Rp = sPip + j; rsk = NX; out = sW2 + off;
                        if (last) base = pk[OC + i * NX + j];  // C_{K-2}' (M += W2' kappa -> C_{K-2} kappa)
                    }
                    double acc = 0.0;
                    if (!last) {
#pragma unroll
                        for (int k = 0; k < NX; ++k) acc = fma(Lp[k * lsk], Rp[k * rsk], acc);
                    }
                    *out = base + acc;
                }
            }
            wsync();
            if (stamp_on && ts == 25 && lane == 0) sStamp[1] = (double)__builtin_amdgcn_s_memtime();
            // ---- phase 2: Qh = Q + A'T1, Sh = S' + Bt'T1, Rh = R + Bt'T2
#pragma unroll
            for (int rep = 0; rep < (E2 + WAVE - 1) / WAVE; ++rep) {
                int off = lane + rep * WAVE;
                if (off < E2) {
                    const double *Lp, *Rp;
                    int lsk, rsk;
                    double* out;
                    double base;
                    if (off < NX * NX) {
                        const int i = off / NX, j = off % NX;
                        Lp = pk + OA + i * NX; lsk = 1; Rp = sT1 + j; rsk = NX; out = sQh + off; base = pk[SL::Q + off];
                    } else if ((off -= NX * NX) < NU * NX) {
                        const int i = off / NX, j = off % NX;
                        Lp = pk + SL::Bt + i; lsk = NU; Rp = sT1 + j; rsk = NX; out = sSh + off; base = pk[SL::S + j * NU + i];
                    } else {
                        off -= NU * NX;
                        const int i = off / NU, j = off % NU;
                        Lp = pk + SL::Bt + i; lsk = NU; Rp = sT2 + j; rsk = NU; out = sRh + off; base = pk[SL::R + off];
                    }
                    double acc = 0.0;
                    if (!last) {
#pragma unroll
                        for (int k = 0; k < NX; ++k) acc = fma(Lp[k * lsk], Rp[k * rsk], acc);
                    }
                    *out = base + acc;
                }
            }
            wsync();
            if (stamp_on && ts == 25 && lane == 0) sStamp[2] = (double)__builtin_amdgcn_s_memtime();
            // ---- phase 3: Cholesky of Rhat in registers (every lane), [K | kappa] = -Rhat^-1 [Sh | W2]
            const bool fx = last && T.fix_last_input;
            double Lr[NU * NU], id[NU];
#pragma unroll
            for (int e = 0; e < NU * NU; ++e) Lr[e] = fx ? ((e / NU == e % NU) ? 1.0 : 0.0) : sRh[e];
            // pivots that rounding pushed below 1e-13 * max diag (Rhat = R + Bt'P'Bt with P' a Schur
            // complement loses definiteness at ~1e15 barrier scalings) are clamped, not fatal
            double dmax = 0.0;
#pragma unroll
            for (int j = 0; j < NU; ++j) dmax = fmax(dmax, fabs(Lr[j * NU + j]));
            const double dmin = 1e-13 * dmax + 1e-300;
            bool bad = (dmax != dmax);
#pragma unroll
            for (int j = 0; j < NU; ++j) {
                double d = Lr[j * NU + j];
#pragma unroll
                for (int k = 0; k < j; ++k) d -= Lr[j * NU + k] * Lr[j * NU + k];
                bad |= (d != d);
                d = sqrt(d > dmin ? d : dmin);
                Lr[j * NU + j] = d;
                id[j] = 1.0 / d;
#pragma unroll
                for (int i = j + 1; i < NU; ++i) {
                    double v = Lr[i * NU + j];
#pragma unroll
                    for (int k = 0; k < j; ++k) v -= Lr[i * NU + k] * Lr[j * NU + k];
                    Lr[i * NU + j] = v * id[j];
                }
            }
            if (bad && lane == 0) sflag[0] = 1.0;
            if (lane < 2 * NX) {
                const int c = lane;
                const bool isk = c < NX;
                double col[NU];
#pragma unroll
                for (int i = 0; i < NU; ++i) col[i] = fx ? 0.0 : (isk ? sSh[i * NX + c] : (fin ? sW2[i * NX + c - NX] : 0.0));
#pragma unroll
                for (int i = 0; i < NU; ++i) {
                    double v = col[i];
#pragma unroll
                    for (int k = 0; k < i; ++k) v -= Lr[i * NU + k] * col[k];
                    col[i] = v * id[i];
                }
#pragma unroll
                for (int i = NU - 1; i >= 0; --i) {
                    double v = col[i];
#pragma unroll
                    for (int k = i + 1; k < NU; ++k) v -= Lr[k * NU + i] * col[k];
                    col[i] = v * id[i];
                }
#pragma unroll
                for (int i = 0; i < NU; ++i) {
                    sKk[i * 2 * NX + c] = -col[i];
                    (isk ? stg[SL::Kg + i * NX + c] : stg[SL::kap + i * NX + c - NX]) = -col[i];
                }
            }
            if (lane < NU * NU) stg[SL::L + lane] = Lr[lane];
            wsync();
            if (stamp_on && ts == 25 && lane == 0) sStamp[3] = (double)__builtin_amdgcn_s_memtime();
            // ---- phase 4: P = Qh + Sh'K (symmetrised in-lane), Pi = W1 + Sh'kappa, M += W2'kappa
#pragma unroll
            for (int rep = 0; rep < (E4 + WAVE - 1) / WAVE; ++rep) {
                int off = lane + rep * WAVE;
                if (off < E4) {
                    const int grp = off / (NX * NX), o = off % (NX * NX), i = o / NX, j = o % NX;
                    if (grp == 0) {
                        double p = sQh[o], pt = sQh[j * NX + i];
#pragma unroll
                        for (int k = 0; k < NU; ++k) {
                            const double shk_i = fx ? 0.0 : sSh[k * NX + i], shk_j = fx ? 0.0 : sSh[k * NX + j];
                            p = fma(shk_i, sKk[k * 2 * NX + j], p);
                            pt = fma(shk_j, sKk[k * 2 * NX + i], pt);
                        }
                        p = 0.5 * (p + pt);
                        sPp[o] = p;
                        stg[SL::P + o] = p;
                    } else if (grp == 1) {
                        double pi = sW1[o];
#pragma unroll
                        for (int k = 0; k < NU; ++k) pi = fma(fx ? 0.0 : sSh[k * NX + i], sKk[k * 2 * NX + NX + j], pi);
                        sPip[o] = pi;
                        stg[SL::Pi + o] = pi;
                    } else if (fin) {
                        double mm_ = 0.0;
#pragma unroll
                        for (int k = 0; k < NU; ++k) mm_ = fma(sW2[k * NX + i], sKk[k * 2 * NX + NX + j], mm_);
                        sM[o] += mm_;
                    }
                }
            }
            for (int e = lane; e < NU * NX; e += WAVE) stg[SL::W2 + e] = sW2[e];
            if (ts > 0) pf_commit(ts - 1, pf);
            wsync();
            if (stamp_on && ts == 25 && lane == 0) sStamp[4] = (double)__builtin_amdgcn_s_memtime();
        }
        // LU with partial pivoting of M (lane 0, in registers; NX <= 12)
        if (fin && lane == 0) {
            double Mr[NX * NX];
#pragma unroll
            for (int e = 0; e < NX * NX; ++e) Mr[e] = sM[e];
#pragma unroll
            for (int k = 0; k < NX; ++k) {
                int p = k;
                double best = fabs(Mr[k * NX + k]);
#pragma unroll
                for (int i = k + 1; i < NX; ++i) {
                    const double v = fabs(Mr[i * NX + k]);
                    if (v > best) { best = v; p = i; }
                }
                spiv[k] = p;
#pragma unroll
                for (int i = k + 1; i < NX; ++i) {
                    if (i == p) {
#pragma unroll
                        for (int j = 0; j < NX; ++j) { const double tmp = Mr[k * NX + j]; Mr[k * NX + j] = Mr[i * NX + j]; Mr[i * NX + j] = tmp; }
                    }
                }
                const double d = Mr[k * NX + k];
                if (d == 0.0) sflag[0] = 2.0;
                const double inv = d != 0.0 ? 1.0 / d : 0.0;
#pragma unroll
                for (int i = k + 1; i < NX; ++i) {
                    const double f = Mr[i * NX + k] * inv;
                    Mr[i * NX + k] = f;
#pragma unroll
                    for (int j = k + 1; j < NX; ++j) Mr[i * NX + j] -= f * Mr[k * NX + j];
                }
            }
#pragma unroll
            for (int e = 0; e < NX * NX; ++e) sM[e] = Mr[e];
        }
        wsync();
        return sflag[0] == 0.0;
    };

    // solve: stage q,r,e buffers filled; xi0 = sv[0], r2f = sv[1] (LDS).  Outputs sdz, sdy, sdyi, sdyf.
    // LDS vector slots: sv[0] xi0, sv[1] r2f, sv[2] xi, sv[3] xi', sv[4] qh|rh / v, sv[5] p', sv[6] xacc, sv[7] mu
    auto solve = [&]() __attribute__((always_inline)) {
        double* xi = sv[2]; double* xin = sv[3]; double* qr = sv[4]; double* pp = sv[5];
        double* xacc = sv[6]; double* mu = sv[7];
        double pf[PFN];
        if (lane < NX) { pp[lane] = 0.0; xacc[lane] = 0.0; }
        __syncthreads();  // q, r, e were written by other lanes (global)
        pf_issue(K - 1, pf);
        pf_commit(K - 1, pf);
        wsync();
        for (int ts = K - 1; ts >= 0; --ts) {
            if (ts > 0) pf_issue(ts - 1, pf);
            const double* pk = slot(ts);
            const double* pkn = slot(ts + 1);
            double* stg = stage + (long long)ts * SL::size;
            const bool last = ts == K - 1;
            // ---- phase 1: h = P_{t+1} e + p' (every lane, redundantly); lanes 0..NX-1: qh = q + A'h,
            //      lanes NX..NX+NU-1: rh = r + Bt'h
            if (lane < NX + NU) {
                double h[NX];
#pragma unroll
                for (int i = 0; i < NX; ++i) {
                    double v = pp[i];
                    if (!last) {
#pragma unroll
                        for (int k = 0; k < NX; ++k) v = fma(pkn[SL::P + i * NX + k], pk[SL::e + k], v);
                    }
                    h[i] = last ? 0.0 : v;
                }
                const bool isq = lane < NX;
                const int j = isq ? lane : lane - NX;
                double v = isq ? pk[SL::q + j] : pk[SL::r + j];
#pragma unroll
                for (int k = 0; k < NX; ++k) v = fma(isq ? pk[OA + j * NX + k] : pk[SL::Bt + k * NU + j], h[k], v);
                qr[lane] = v;
            }
            wsync();
            // ---- phase 2: k = -Rhat^-1 rh (every lane), p = qh + K'rh, xacc += W2'k + Pi_{t+1}'e
            const bool fx = last && T.fix_last_input;
            double kv[NU], rh[NU], Lr[NU * NU];
#pragma unroll
            for (int e = 0; e < NU * NU; ++e) Lr[e] = pk[SL::L + e];
#pragma unroll
            for (int i = 0; i < NU; ++i) { rh[i] = fx ? 0.0 : qr[NX + i]; kv[i] = rh[i]; }
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                double v = kv[i];
#pragma unroll
                for (int k = 0; k < i; ++k) v -= Lr[i * NU + k] * kv[k];
                kv[i] = v / Lr[i * NU + i];
            }
#pragma unroll
            for (int i = NU - 1; i >= 0; --i) {
                double v = kv[i];
#pragma unroll
                for (int k = i + 1; k < NU; ++k) v -= Lr[k * NU + i] * kv[k];
                kv[i] = v / Lr[i * NU + i];
            }
            if (lane < NX) {
                double p = qr[lane], xa = 0.0;
#pragma unroll
                for (int k = 0; k < NU; ++k) {
                    p = fma(pk[SL::Kg + k * NX + lane], rh[k], p);
                    xa = fma(pk[SL::W2 + k * NX + lane], -kv[k], xa);
                }
                if (!last) {
#pragma unroll
                    for (int k = 0; k < NX; ++k) xa = fma(pkn[SL::Pi + k * NX + lane], pk[SL::e + k], xa);
                }
                stg[SL::p0 + lane] = p;
                pp[lane] = p;   // p' of stage ts-1
                xacc[lane] += xa;
                if (lane < NU) stg[SL::k0 + lane] = -kv[lane];
            }
            if (ts > 0) pf_commit(ts - 1, pf);
            wsync();
        }
        // terminal multiplier mu = M^{-1} (r2f - xacc - Pi_0' xi0)   (Pi_0 from slot(0))
        if (lane == 0) {
            const double* pk0 = slot(0);
            double b[NX];
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                double v = sv[1][i] - xacc[i];
#pragma unroll
                for (int k = 0; k < NX; ++k) v -= pk0[SL::Pi + k * NX + i] * sv[0][k];
                b[i] = fin ? v : 0.0;
            }
            if (fin) {
                // getrf storage: apply every row interchange first, then unit-lower substitution
#pragma unroll
                for (int k = 0; k < NX; ++k) {
                    const int p = spiv[k];
#pragma unroll
                    for (int i = 0; i < NX; ++i)
                        if (i == p && p != k) { const double tmp = b[k]; b[k] = b[i]; b[i] = tmp; }
                }
#pragma unroll
                for (int k = 0; k < NX; ++k)
#pragma unroll
                    for (int i = k + 1; i < NX; ++i) b[i] -= sM[i * NX + k] * b[k];
#pragma unroll
                for (int i = NX - 1; i >= 0; --i) {
                    double v = b[i];
#pragma unroll
                    for (int j = i + 1; j < NX; ++j) v -= sM[i * NX + j] * b[j];
                    b[i] = v / sM[i * NX + i];
                }
            }
#pragma unroll
            for (int i = 0; i < NX; ++i) mu[i] = b[i];
        }
        // forward sweep (slots t, t+1 ring-buffered; k0/p0 were just written by the backward sweep)
        __syncthreads();
        pf_issue(0, pf);
        pf_commit(0, pf);
        if (K > 1) { pf_issue(1, pf); pf_commit(1, pf); }
        if (lane < NX) xi[lane] = sv[0][lane];
        wsync();
        for (int ts = 0; ts < K; ++ts) {
            if (ts + 2 < K) pf_issue(ts + 2, pf);
            const double* pk = slot(ts);
            // ---- phase a: v = K xi + k0 + kappa mu (lanes 0..NU-1); y_{t-1} = -(P_t xi + p0_t + Pi_t mu)
            //      (lanes 32..32+NX-1; y_{-1} is the initial-state multiplier)
            if (lane < NU) {
                double v = pk[SL::k0 + lane];
#pragma unroll
                for (int k = 0; k < NX; ++k) v += pk[SL::Kg + lane * NX + k] * xi[k] + pk[SL::kap + lane * NX + k] * mu[k];
                qr[lane] = v;
            } else if (lane >= 32 && lane < 32 + NX) {
                const int i = lane - 32;
                double v = pk[SL::p0 + i];
#pragma unroll
                for (int k = 0; k < NX; ++k) v += pk[SL::P + i * NX + k] * xi[k] + pk[SL::Pi + i * NX + k] * mu[k];
                if (ts == 0) { sdyi[i] = -v; sdyf[i] = mu[i]; }
                else sdy[ts - 1][i] = -v;
            }
            wsync();
            // ---- phase b: dx_t = xi + C_{t-1} v, du_t = v, xi' = A xi + Bt v + e
            if (lane < NX) {
                double dx = xi[lane];
#pragma unroll
                for (int j = 0; j < NU; ++j) dx += pk[OC + j * NX + lane] * qr[j];  // C_{t-1} (zero at t = 0)
                sdz[ts][lane] = dx;
                double xn = pk[SL::e + lane];
#pragma unroll
                for (int k = 0; k < NX; ++k) xn += pk[OA + k * NX + lane] * xi[k];
#pragma unroll
                for (int j = 0; j < NU; ++j) xn += pk[SL::Bt + lane * NU + j] * qr[j];
                xin[lane] = xn;
            } else if (lane >= 32 && lane < 32 + NU) {
                sdz[ts][NX + lane - 32] = qr[lane - 32];
            }
            if (ts + 2 < K) pf_commit(ts + 2, pf);
            wsync();
            if (lane < NX) xi[lane] = xin[lane];
            wsync();
        }
    };

    // ------------------------------------------------------------------ node phase helpers
    auto exchange_z = [&]() __attribute__((always_inline)) {
        if (act) {
#pragma unroll
            for (int i = 0; i < NZ; ++i) sz[t][i] = z[i];
        }
        __syncthreads();
    };
    // write node Hessian blocks (Q, S, R in xi/v coordinates): Hxx = diag(dbox) + embed(Hpp),
    // Huu dense, H_xu = 0.
    auto write_hessian = [&](const double* dbox, double (*Hpp)[3], const double* Huu) __attribute__((always_inline)) {
        if (!act) return;
        double* st = stage + (long long)t * SL::size;
#pragma unroll
        for (int i = 0; i < NX; ++i)
#pragma unroll
            for (int j = 0; j < NX; ++j) {
                double v = (i == j) ? dbox[i] : 0.0;
                if (i < pd && j < pd) v += Hpp[i][j];
                st[SL::Q + i * NX + j] = v;
            }
        double Sx[NX * NU];
#pragma unroll
        for (int i = 0; i < NX; ++i)
#pragma unroll
            for (int j = 0; j < NU; ++j) {
                double v = dbox[i] * Cp[j * NX + i];
#pragma unroll
                for (int k = 0; k < 3; ++k)
                    if (i < pd && k < pd) v += Hpp[i < 3 ? i : 0][k] * Cp[j * NX + k];
                Sx[i * NU + j] = v;
                st[SL::S + i * NU + j] = v;
            }
#pragma unroll
        for (int i = 0; i < NU; ++i)
#pragma unroll
            for (int j = 0; j < NU; ++j) {
                double v = Huu[i * NU + j];
#pragma unroll
                for (int k = 0; k < NX; ++k) v += Cp[i * NX + k] * Sx[k * NU + j];
                st[SL::R + i * NU + j] = v;
            }
    };
    // linear terms q = -r1x, r = -(Cp' r1x + r1u), e = -rp for this node
    auto write_rhs = [&](const double* r1) __attribute__((always_inline)) {
        if (!act) return;
        double* st = stage + (long long)t * SL::size;
#pragma unroll
        for (int i = 0; i < NX; ++i) st[SL::q + i] = -r1[i];
#pragma unroll
        for (int j = 0; j < NU; ++j) {
            double v = r1[NX + j];
#pragma unroll
            for (int k = 0; k < NX; ++k) v += Cp[j * NX + k] * r1[k];
            st[SL::r + j] = fixed_u ? 0.0 : -v;
        }
        if (t < K - 1) {
#pragma unroll
            for (int i = 0; i < NX; ++i) st[SL::e + i] = -rp[i];
        }
    };
    // Bt_t = B_t + A_t C_{t-1}
    auto write_Bt = [&]() __attribute__((always_inline)) {
        if (!(act && t < K - 1)) return;
        const double* d = disc + (long long)t * DSTR;
        double* st = stage + (long long)t * SL::size;
#pragma unroll
        for (int i = 0; i < NX; ++i)
#pragma unroll
            for (int j = 0; j < NU; ++j) {
                double v = d[NX * NX + j * NX + i];
#pragma unroll
                for (int k = 0; k < NX; ++k) v += d[k * NX + i] * Cp[j * NX + k];
                st[SL::Bt + i * NU + j] = v;
            }
    };
    // dynamics residual rp_t = x_{t+1} - A x_t - B u_t - C u_{t+1} - c_t (needs sz filled)
    auto dyn_residual = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < NX; ++i) rp[i] = 0.0;
        if (!(act && t < K - 1)) return;
        const double* d = disc + (long long)t * DSTR;
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            double v = sz[t + 1][i] - (d[NX * NX + 2 * NX * NU + i] * sig + d[NX * NX + 2 * NX * NU + NX + i]);
#pragma unroll
            for (int k = 0; k < NX; ++k) v -= d[k * NX + i] * z[k];
#pragma unroll
            for (int j = 0; j < NU; ++j) v -= d[NX * NX + j * NX + i] * z[NX + j] + d[NX * NX + NX * NU + j * NX + i] * sz[t + 1][NX + j];
            rp[i] = v;
        }
    };
    // r1 (position part) -= sum_g Hpa[g] r1a[g] / Haa[g]
    auto eliminate_rhs = [&](double* r1) __attribute__((always_inline)) {
        for (int g = 0; g < na; ++g) {
            const double f = gR1[g * WAVE] / gHaa[g * WAVE];
#pragma unroll
            for (int i = 0; i < 3; ++i)
                if (i < pd) r1[i] -= gH0[(3 * g + i) * WAVE] * f;
        }
    };
    // node Hessian for scaling D_r (unit = true: D = 1, W = I) ; fills group columns Haa, Hpa
    auto assemble_hessian = [&](bool unit, const double* Wi2uu) __attribute__((always_inline)) {
        double dbox[NX], Hpp[3][3], Huu[NU * NU];
#pragma unroll
        for (int i = 0; i < NX; ++i) dbox[i] = 0.0;
#pragma unroll
        for (int i = 0; i < 3; ++i) Hpp[i][0] = Hpp[i][1] = Hpp[i][2] = 0.0;
#pragma unroll
        for (int i = 0; i < NU; ++i)
#pragma unroll
            for (int j = 0; j < NU; ++j) Huu[i * NU + j] = (i == j ? 2.0 * wu : 0.0) + (soc ? Wi2uu[i * NU + j] : 0.0);
        for (int g = 0; g < na; ++g) {
            gHaa[g * WAVE] = 0.0;
#pragma unroll
            for (int i = 0; i < 3; ++i) gH0[(3 * g + i) * WAVE] = 0.0;
        }
        for (int r = 0; r < nrows; ++r) {
            const double Dr = unit ? 1.0 : cL[r * WAVE] / cS[r * WAVE];
            if (r < NTR) {
#pragma unroll
                for (int i = 0; i < NU; ++i)
#pragma unroll
                    for (int j = 0; j < NU; ++j) {
                        const double si = ((r >> i) & 1) ? -1.0 : 1.0, sj = ((r >> j) & 1) ? -1.0 : 1.0;
                        Huu[i * NU + j] += Dr * si * sj;
                    }
            } else if (r < r_soft0) {
                const int idx = T.box_idx[(r - r_box0) >> 1];
#pragma unroll
                for (int i = 0; i < NX; ++i) dbox[i] += (i == idx) ? Dr : 0.0;
            } else if (r < r_grp0) {
                double g[3], b;
                const int q = r - r_soft0, gr = group_of(q);
                soft_row(q, g, b);
#pragma unroll
                for (int i = 0; i < 3; ++i)
#pragma unroll
                    for (int j = 0; j < 3; ++j) Hpp[i][j] += Dr * g[i] * g[j];
                gHaa[gr * WAVE] += Dr;
#pragma unroll
                for (int i = 0; i < 3; ++i) gH0[(3 * gr + i) * WAVE] += Dr * g[i];
            } else {
                gHaa[(r - r_grp0) * WAVE] += Dr;
            }
        }
        for (int g = 0; g < na; ++g) {
            const double ih = 1.0 / gHaa[g * WAVE];
            double hp[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) hp[i] = gH0[(3 * g + i) * WAVE];
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) Hpp[i][j] -= hp[i] * hp[j] * ih;
        }
        write_hessian(dbox, Hpp, Huu);
    };
    // aux direction from the position direction: da_g = (r1a_g - Hpa_g' dp) / Haa_g
    auto recover_aux = [&](const double* dzl) __attribute__((always_inline)) {
        for (int g = 0; g < a.gmax; ++g) {
            double v = 0.0;
            if (g < na) {
                v = gR1[g * WAVE];
#pragma unroll
                for (int i = 0; i < 3; ++i)
                    if (i < pd) v -= gH0[(3 * g + i) * WAVE] * dzl[i];
                v /= gHaa[g * WAVE];
            }
            gDa[g * WAVE] = v;
        }
    };
    auto set_boundary_rhs = [&]() __attribute__((always_inline)) {
        if (lane < NX) {
            sv[0][lane] = a.x_init[agent * NX + lane] - sz[0][lane];
            sv[1][lane] = fin ? a.x_final[agent * NX + lane] - sz[K - 1][lane] : 0.0;
        }
        __syncthreads();
    };

    // ------------------------------------------------------------------ starting point
    // minimiser of 1/2 z'Pz + q'z + 1/2||Gz - h||^2 s.t. Az = b from z_ref (aux = 0), unit scaling
    // (the CVXOPT coneqp initialisation; oracle/qp_dense.py does the same on the dense form)
    int status = SCVX_STATUS_MAX_ITER;
    int it = 0;
    {
        double Wu[NU * NU];
#pragma unroll
        for (int e = 0; e < NU * NU; ++e) Wu[e] = (e / NU == e % NU) ? 1.0 : 0.0;
        write_Bt();
        assemble_hessian(true, Wu);
        exchange_z();
        dyn_residual();
        double r1[NZ];
#pragma unroll
        for (int i = 0; i < NX; ++i) r1[i] = 0.0;
#pragma unroll
        for (int j = 0; j < NU; ++j) r1[NX + j] = -2.0 * wu * z[NX + j] - (soc ? z[NX + j] : 0.0);
        for (int g = 0; g < na; ++g) gR1[g * WAVE] = -((g < T.n_obs) ? T.w_obs : T.w_coll);
        for (int r = 0; r < nrows; ++r) {
            double gz, h;
            row_eval(r, z, gA, gz, h);
            row_accT(r, -(gz - h), r1, gR1);
        }
        if (fixed_u) {
#pragma unroll
            for (int j = 0; j < NU; ++j) r1[NX + j] = 0.0;
        }
        eliminate_rhs(r1);
        write_rhs(r1);
        set_boundary_rhs();
        if (!factor()) status = SCVX_STATUS_NUMERICAL;
        solve();
        double dzl[NZ];
#pragma unroll
        for (int i = 0; i < NZ; ++i) dzl[i] = act ? sdz[t][i] : 0.0;
        recover_aux(dzl);
        if (act) {
#pragma unroll
            for (int i = 0; i < NZ; ++i) z[i] += dzl[i];
            for (int g = 0; g < na; ++g) gA[g * WAVE] += gDa[g * WAVE];
        }
        double smin = 1e300, lmin = 1e300;
        for (int r = 0; r < nrows; ++r) {
            double gz, h;
            row_eval(r, z, gA, gz, h);
            cS[r * WAVE] = h - gz; cL[r * WAVE] = gz - h;
            smin = fmin(smin, h - gz); lmin = fmin(lmin, gz - h);
        }
        if (soc) {
            double nu2 = 0.0;
            sq[0] = T.u_max; lq[0] = -T.u_max;
#pragma unroll
            for (int j = 0; j < NU; ++j) { sq[1 + j] = z[NX + j]; lq[1 + j] = -z[NX + j]; nu2 += z[NX + j] * z[NX + j]; }
            smin = fmin(smin, T.u_max - sqrt(nu2));
            lmin = fmin(lmin, -T.u_max - sqrt(nu2));
        }
        smin = wave_min(smin); lmin = wave_min(lmin);
        const double shs = fmax(0.0, 1.0 - smin), shl = fmax(0.0, 1.0 - lmin);
        for (int r = 0; r < nrows; ++r) { cS[r * WAVE] += shs; cL[r * WAVE] += shl; }
        if (soc) { sq[0] += shs; lq[0] += shl; }
    }
    int deg = nrows + (soc ? 1 : 0);
    deg = (int)wave_sum((double)deg);
    const double tol = T.tol > 0 ? T.tol : 1e-9;

    auto soc_step = [&](const double* x, const double* dx) __attribute__((always_inline)) {
        double qa = dx[0] * dx[0], qb = x[0] * dx[0], qc = x[0] * x[0];
#pragma unroll
        for (int j = 1; j < NQ; ++j) { qa -= dx[j] * dx[j]; qb -= x[j] * dx[j]; qc -= x[j] * x[j]; }
        qb *= 2.0;
        double best = 1e300;
        if (fabs(qa) < 1e-300) {
            if (qb < 0) best = fmin(best, -qc / qb);
        } else {
            const double disc_ = qb * qb - 4 * qa * qc;
            if (disc_ >= 0) {
                const double sqd = sqrt(disc_), q1 = (-qb - sqd) / (2 * qa), q2 = (-qb + sqd) / (2 * qa);
                if (q1 > 0) best = fmin(best, q1);
                if (q2 > 0) best = fmin(best, q2);
            }
        }
        if (dx[0] < 0) best = fmin(best, -x[0] / dx[0]);
        return best;
    };

    // ------------------------------------------------------------------ IPM iterations
    long long cyc_factor = 0, cyc_solve = 0, cyc_all0 = __builtin_amdgcn_s_memtime();
    double fail_code = 0.0;
    for (it = 0; it < T.max_iter && status != SCVX_STATUS_NUMERICAL; ++it) {
        exchange_z();
        dyn_residual();
        double pres = 0.0, dres = 0.0, gap = 0.0, hsc = 1.0, qsc = 1.0, pobj = 0.0;
#pragma unroll
        for (int i = 0; i < NX; ++i) pres = fmax(pres, fabs(rp[i]));
        if (t == 0) {
#pragma unroll
            for (int i = 0; i < NX; ++i) pres = fmax(pres, fabs(z[i] - a.x_init[agent * NX + i]));
        }
        if (act && t == K - 1 && fin) {
#pragma unroll
            for (int i = 0; i < NX; ++i) pres = fmax(pres, fabs(z[i] - a.x_final[agent * NX + i]));
        }
        // dual residual rd = Pz + q + A'y + G'lam ; row residuals rc = Gz + s - h
#pragma unroll
        for (int i = 0; i < NX; ++i) rd[i] = 0.0;
#pragma unroll
        for (int j = 0; j < NU; ++j) rd[NX + j] = 2.0 * wu * z[NX + j];
        for (int g = 0; g < na; ++g) gRd[g * WAVE] = (g < T.n_obs) ? T.w_obs : T.w_coll;
        if (na > 0) qsc = fmax(qsc, fmax(T.n_obs > 0 ? T.w_obs : 0.0, T.j_max > 0 ? T.w_coll : 0.0));
        for (int r = 0; r < nrows; ++r) {
            double gz, h;
            row_eval(r, z, gA, gz, h);
            const double sr = cS[r * WAVE], lr = cL[r * WAVE];
            const double rcr = gz + sr - h;
            cR[r * WAVE] = rcr;
            pres = fmax(pres, fabs(rcr));
            hsc = fmax(hsc, fabs(h));
            gap += sr * lr;
            row_accT(r, lr, rd, gRd);
        }
        if (soc) {
            rcq[0] = sq[0] - T.u_max;
#pragma unroll
            for (int j = 0; j < NU; ++j) { rcq[1 + j] = sq[1 + j] - z[NX + j]; rd[NX + j] -= lq[1 + j]; }
#pragma unroll
            for (int j = 0; j < NQ; ++j) { pres = fmax(pres, fabs(rcq[j])); gap += sq[j] * lq[j]; }
            hsc = fmax(hsc, T.u_max);
        } else {
#pragma unroll
            for (int j = 0; j < NQ; ++j) rcq[j] = 0.0;
        }
        if (act) {
            if (t == 0) {
#pragma unroll
                for (int i = 0; i < NX; ++i) rd[i] += syi[i];
            }
            if (t == K - 1 && fin) {
#pragma unroll
                for (int i = 0; i < NX; ++i) rd[i] += syf[i];
            }
            if (t >= 1) {
#pragma unroll
                for (int i = 0; i < NX; ++i) rd[i] += sy[t - 1][i];
#pragma unroll
                for (int j = 0; j < NU; ++j)
#pragma unroll
                    for (int i = 0; i < NX; ++i) rd[NX + j] -= Cp[j * NX + i] * sy[t - 1][i];
            }
            if (t < K - 1) {
                const double* d = disc + (long long)t * DSTR;
#pragma unroll
                for (int k = 0; k < NX; ++k)
#pragma unroll
                    for (int i = 0; i < NX; ++i) rd[k] -= d[k * NX + i] * sy[t][i];
#pragma unroll
                for (int j = 0; j < NU; ++j)
#pragma unroll
                    for (int i = 0; i < NX; ++i) rd[NX + j] -= d[NX * NX + j * NX + i] * sy[t][i];
            }
            if (fixed_u) {
#pragma unroll
                for (int j = 0; j < NU; ++j) rd[NX + j] = 0.0;
            }
#pragma unroll
            for (int i = 0; i < NZ; ++i) dres = fmax(dres, fabs(rd[i]));
            for (int g = 0; g < na; ++g) dres = fmax(dres, fabs(gRd[g * WAVE]));
#pragma unroll
            for (int j = 0; j < NU; ++j) pobj += wu * z[NX + j] * z[NX + j];
            for (int g = 0; g < na; ++g) pobj += ((g < T.n_obs) ? T.w_obs : T.w_coll) * gA[g * WAVE];
        }
        pres = wave_max(pres); dres = wave_max(dres); hsc = wave_max(hsc); qsc = wave_max(qsc);
        gap = wave_sum(gap); pobj = wave_sum(pobj);
        const double mu = gap / fmax((double)deg, 1.0);
        if (!isfinite(pres + dres + mu)) { status = SCVX_STATUS_NUMERICAL; fail_code = 3.0; break; }
        if (pres <= tol * hsc && dres <= tol * qsc && gap <= tol * fmax(1.0, fabs(pobj))) {
            status = SCVX_STATUS_OPTIMAL;
            break;
        }
        // ECOS-style reduced accuracy: what a numerical breakdown below leaves is still usable
        const bool near = pres <= 1e-6 * hsc && dres <= 1e-6 * qsc && gap <= 1e-6 * fmax(1.0, fabs(pobj));
        // SOC Nesterov-Todd scaling (hyperbolic-rotation form, W z = W^-1 s)
        double Wi2uu[NU * NU];
        if (soc) {
            // J(x) = (x0 - |x1|)(x0 + |x1|): no catastrophic cancellation next to the cone boundary
            double n1s = 0.0, n1z = 0.0;
#pragma unroll
            for (int j = 1; j < NQ; ++j) { n1s += sq[j] * sq[j]; n1z += lq[j] * lq[j]; }
            n1s = sqrt(n1s); n1z = sqrt(n1z);
            const double Js = fmax((sq[0] - n1s) * (sq[0] + n1s), 1e-300), Jz = fmax((lq[0] - n1z) * (lq[0] + n1z), 1e-300);
            const double ns = sqrt(Js), nz = sqrt(Jz);
            double sb[NQ], zb[NQ], w[NQ], dot = 0.0;
#pragma unroll
            for (int j = 0; j < NQ; ++j) { sb[j] = sq[j] / ns; zb[j] = lq[j] / nz; dot += sb[j] * zb[j]; }
            const double gam = sqrt((1.0 + dot) / 2.0);
#pragma unroll
            for (int j = 0; j < NQ; ++j) w[j] = (sb[j] + (j == 0 ? zb[j] : -zb[j])) / (2.0 * gam);
            const double eta = sqrt(sqrt(Js / Jz));
            W[0] = eta * w[0]; Wi[0] = w[0] / eta;
#pragma unroll
            for (int i = 1; i < NQ; ++i) {
                W[i] = W[i * NQ] = eta * w[i];
                Wi[i] = Wi[i * NQ] = -w[i] / eta;
#pragma unroll
                for (int j = 1; j < NQ; ++j) {
                    const double v = (i == j ? 1.0 : 0.0) + w[i] * w[j] / (1.0 + w[0]);
                    W[i * NQ + j] = eta * v; Wi[i * NQ + j] = v / eta;
                }
            }
#pragma unroll
            for (int i = 0; i < NQ; ++i) {
                double v = 0.0;
#pragma unroll
                for (int j = 0; j < NQ; ++j) v += W[i * NQ + j] * lq[j];
                ltq[i] = v;
            }
#pragma unroll
            for (int i = 0; i < NU; ++i)
#pragma unroll
                for (int j = 0; j < NU; ++j) {
                    double v = 0.0;
#pragma unroll
                    for (int k = 0; k < NQ; ++k) v += Wi[(1 + i) * NQ + k] * Wi[k * NQ + 1 + j];
                    Wi2uu[i * NU + j] = v;
                }
        } else {
#pragma unroll
            for (int e = 0; e < NU * NU; ++e) Wi2uu[e] = 0.0;
#pragma unroll
            for (int e = 0; e < NQ * NQ; ++e) { W[e] = 0.0; Wi[e] = 0.0; }
#pragma unroll
            for (int j = 0; j < NQ; ++j) ltq[j] = 0.0;
        }
        assemble_hessian(false, Wi2uu);
        __syncthreads();
        long long st0 = __builtin_amdgcn_s_memtime();
        if (!factor()) { status = near ? SCVX_STATUS_MAX_ITER : SCVX_STATUS_NUMERICAL; fail_code = sflag[0]; break; }
        cyc_factor += __builtin_amdgcn_s_memtime() - st0;

        // complementarity rhs of row r: predictor -s l ; corrector -s l - ds_a dl_a + sig mu
        double sgmu = 0.0;
        bool corr = false;
        auto rco_of = [&](int r) __attribute__((always_inline)) {
            const double v = -cS[r * WAVE] * cL[r * WAVE];
            return corr ? v - cP[r * WAVE] + sgmu : v;
        };
        // Newton direction: dz, dy -> LDS; aux -> gDa; SOC pieces -> dsq/dlq.  Returns dzl.
        double dzl[NZ], dsq[NQ], dlq[NQ], rho[NQ];
        auto newton = [&](const double* rcq2) __attribute__((always_inline)) {
            double r1[NZ];
#pragma unroll
            for (int i = 0; i < NZ; ++i) r1[i] = -rd[i];
            for (int g = 0; g < na; ++g) gR1[g * WAVE] = -gRd[g * WAVE];
            for (int r = 0; r < nrows; ++r)
                row_accT(r, -(rco_of(r) + cL[r * WAVE] * cR[r * WAVE]) / cS[r * WAVE], r1, gR1);
#pragma unroll
            for (int j = 0; j < NQ; ++j) rho[j] = 0.0;
            if (soc) {
                // rho = ltq o^-1 rcq2 ; G' (Wi rho + Wi^2 rcq) on u = -(...)[1:]
                double J = ltq[0] * ltq[0], r0 = ltq[0] * rcq2[0], w2[NQ];
#pragma unroll
                for (int j = 1; j < NQ; ++j) { J -= ltq[j] * ltq[j]; r0 -= ltq[j] * rcq2[j]; }
                r0 /= J;
                rho[0] = r0;
#pragma unroll
                for (int j = 1; j < NQ; ++j) rho[j] = (rcq2[j] - r0 * ltq[j]) / ltq[0];
#pragma unroll
                for (int i = 0; i < NQ; ++i) {
                    double v = 0.0;
#pragma unroll
                    for (int j = 0; j < NQ; ++j) v += Wi[i * NQ + j] * rcq[j];
                    w2[i] = v;
                }
#pragma unroll
                for (int i = 0; i < NU; ++i) {
                    double v = 0.0;
#pragma unroll
                    for (int j = 0; j < NQ; ++j) v += Wi[(1 + i) * NQ + j] * (rho[j] + w2[j]);
                    r1[NX + i] += v;
                }
            }
            if (fixed_u) {
#pragma unroll
                for (int j = 0; j < NU; ++j) r1[NX + j] = 0.0;
            }
            eliminate_rhs(r1);
            write_rhs(r1);
            set_boundary_rhs();
            long long st1 = __builtin_amdgcn_s_memtime();
            solve();
            cyc_solve += __builtin_amdgcn_s_memtime() - st1;
#pragma unroll
            for (int i = 0; i < NZ; ++i) dzl[i] = act ? sdz[t][i] : 0.0;
            recover_aux(dzl);
            if (soc) {
                double v2[NQ], w2[NQ];
                dsq[0] = -rcq[0];
                v2[0] = rcq[0];
#pragma unroll
                for (int j = 1; j < NQ; ++j) { dsq[j] = -rcq[j] + dzl[NX + j - 1]; v2[j] = rcq[j] - dzl[NX + j - 1]; }
#pragma unroll
                for (int i = 0; i < NQ; ++i) {
                    double v = 0.0;
#pragma unroll
                    for (int j = 0; j < NQ; ++j) v += Wi[i * NQ + j] * v2[j];
                    w2[i] = v;
                }
#pragma unroll
                for (int i = 0; i < NQ; ++i) {
                    double v = 0.0;
#pragma unroll
                    for (int j = 0; j < NQ; ++j) v += Wi[i * NQ + j] * (rho[j] + w2[j]);
                    dlq[i] = v;
                }
            } else {
#pragma unroll
                for (int j = 0; j < NQ; ++j) { dsq[j] = 0.0; dlq[j] = 0.0; }
            }
        };
        // row directions ds = -rc - G d, dl = (rco + l (rc + G d)) / s
        auto row_dir = [&](int r, double& dsr, double& dlr) __attribute__((always_inline)) {
            double gz, h;
            row_eval(r, dzl, gDa, gz, h);
            const double rcr = cR[r * WAVE];
            dsr = -rcr - gz;
            dlr = (rco_of(r) + cL[r * WAVE] * (rcr + gz)) / cS[r * WAVE];
        };
        auto max_step = [&]() __attribute__((always_inline)) {
            double am = 1e300;
            for (int r = 0; r < nrows; ++r) {
                double dsr, dlr;
                row_dir(r, dsr, dlr);
                if (dsr < 0) am = fmin(am, -cS[r * WAVE] / dsr);
                if (dlr < 0) am = fmin(am, -cL[r * WAVE] / dlr);
            }
            if (soc) { am = fmin(am, soc_step(sq, dsq)); am = fmin(am, soc_step(lq, dlq)); }
            return wave_min(am);
        };

        // ---- predictor (affine scaling)
        double rcq2[NQ];
        if (soc) {
            double d0 = 0.0;
#pragma unroll
            for (int j = 0; j < NQ; ++j) d0 += ltq[j] * ltq[j];
            rcq2[0] = -d0;
#pragma unroll
            for (int j = 1; j < NQ; ++j) rcq2[j] = -2.0 * ltq[0] * ltq[j];
        } else {
#pragma unroll
            for (int j = 0; j < NQ; ++j) rcq2[j] = 0.0;
        }
        newton(rcq2);
        if (a.trace && agent == a.trace_agent && it == 0 && act) {  // predictor direction dump
            double* dd = a.trace + 8 * a.trace_cap + (long long)t * 40;
#pragma unroll
            for (int i = 0; i < NZ; ++i) dd[i] = dzl[i];
            for (int g = 0; g < na && g < 17; ++g) dd[NZ + g] = gDa[g * WAVE];
            if (lane < NX) a.trace[8 * a.trace_cap + 64 * 40 + lane] = sdyi[lane];
        }
        const double aa = fmin(1.0, max_step());
        double gap_a = 0.0;
        for (int r = 0; r < nrows; ++r) {
            double dsr, dlr;
            row_dir(r, dsr, dlr);
            gap_a += (cS[r * WAVE] + aa * dsr) * (cL[r * WAVE] + aa * dlr);
            cP[r * WAVE] = dsr * dlr;
        }
        if (soc) {
#pragma unroll
            for (int j = 0; j < NQ; ++j) gap_a += (sq[j] + aa * dsq[j]) * (lq[j] + aa * dlq[j]);
        }
        gap_a = wave_sum(gap_a);
        const double mu_a = gap_a / fmax((double)deg, 1.0);
        const double sg = mu > 0 ? pow(fmax(mu_a, 0.0) / mu, 3.0) : 0.0;
        // ---- corrector
        corr = true;
        sgmu = sg * mu;
        if (soc) {
            double a1[NQ], b1[NQ];
#pragma unroll
            for (int i = 0; i < NQ; ++i) {
                double va = 0.0, vb = 0.0;
#pragma unroll
                for (int j = 0; j < NQ; ++j) { va += Wi[i * NQ + j] * dsq[j]; vb += W[i * NQ + j] * dlq[j]; }
                a1[i] = va; b1[i] = vb;
            }
            double d0 = 0.0;
#pragma unroll
            for (int j = 0; j < NQ; ++j) d0 += a1[j] * b1[j];
            rcq2[0] -= d0;
#pragma unroll
            for (int j = 1; j < NQ; ++j) rcq2[j] -= a1[0] * b1[j] + b1[0] * a1[j];
            rcq2[0] += sgmu;
        }
        newton(rcq2);
        const double al = fmin(1.0, 0.99 * max_step());
        {
            double chk = al;
#pragma unroll
            for (int i = 0; i < NZ; ++i) chk += 0.0 * dzl[i];
            chk = wave_sum(chk);  // NaN anywhere in the direction poisons the sum
            if (!(chk == chk) || !(al > 0.0)) {
                status = near ? SCVX_STATUS_MAX_ITER : SCVX_STATUS_NUMERICAL;
                fail_code = 4.0;
                break;
            }
        }
        if (a.trace && agent == a.trace_agent && lane == 0 && it < a.trace_cap) {
            double* tr_ = a.trace + 8 * it;
            tr_[0] = pres; tr_[1] = dres; tr_[2] = gap; tr_[3] = pobj; tr_[4] = aa; tr_[5] = al; tr_[6] = sg; tr_[7] = mu;
        }
        // ---- update
        for (int r = 0; r < nrows; ++r) {
            double dsr, dlr;
            row_dir(r, dsr, dlr);
            cS[r * WAVE] += al * dsr;
            cL[r * WAVE] += al * dlr;
        }
        if (act) {
#pragma unroll
            for (int i = 0; i < NZ; ++i) z[i] += al * dzl[i];
            for (int g = 0; g < na; ++g) gA[g * WAVE] += al * gDa[g * WAVE];
            if (soc) {
#pragma unroll
                for (int j = 0; j < NQ; ++j) { sq[j] += al * dsq[j]; lq[j] += al * dlq[j]; }
            }
            if (t < K - 1) {
#pragma unroll
                for (int i = 0; i < NX; ++i) sy[t][i] += al * sdy[t][i];
            }
        }
        if (lane < NX) { syi[lane] += al * sdyi[lane]; syf[lane] += al * sdyf[lane]; }
        __syncthreads();
    }

    // ------------------------------------------------------------------ outputs
    if (a.trace && agent == a.trace_agent && lane == 0) {
        double* dd = a.trace + 8 * a.trace_cap + 64 * 40 + 16;
        dd[0] = (double)cyc_factor; dd[1] = (double)cyc_solve; dd[2] = (double)(__builtin_amdgcn_s_memtime() - cyc_all0);
        for (int k = 0; k < 12; ++k) dd[3 + k] = sStamp[k];
        dd[15] = fail_code;
    }
    double pobj = 0.0;
    if (act) {
#pragma unroll
        for (int i = 0; i < NX; ++i) a.X[(agent * K + t) * NX + i] = z[i];
#pragma unroll
        for (int j = 0; j < NU; ++j) { a.U[(agent * K + t) * NU + j] = z[NX + j]; pobj += wu * z[NX + j] * z[NX + j]; }
        for (int g = 0; g < na; ++g) pobj += ((g < T.n_obs) ? T.w_obs : T.w_coll) * gA[g * WAVE];
        a.slack_coll[agent * K + t] = (T.j_max > 0 && na > 0) ? gA[T.n_obs * WAVE] : 0.0;
    }
    pobj = wave_sum(pobj);
    if (lane == 0) {
        a.obj[agent] = pobj;
        a.status[agent] = status;
        a.iters[agent] = it;
    }
}

}  // namespace scvx

using namespace scvx;

namespace {
double* g_trace = nullptr;
int g_trace_agent = 0, g_trace_cap = 0;

template <int NX, int NU>
int dispatch_model(const QPArgs& a, hipStream_t st) {
    hipLaunchKernelGGL((qp_ipm_kernel<NX, NU>), dim3(a.N), dim3(WAVE), 0, st, a);
    return check_launch("qp_ipm_kernel");
}

int qp_check(const scvx_qp_template* T, int N, int& rows, int& ngroups) {
    if (!T || N < 0) return set_error(SCVX_EINVAL, "qp: null template");
    if (T->K < 2 || T->K > WAVE) return set_error(SCVX_EUNSUPPORTED, "qp: K must be in [2, 64]");
    if (T->pos_dim < 1 || T->pos_dim > 3 || T->pos_dim > T->n_x) return set_error(SCVX_EINVAL, "qp: pos_dim");
    if (T->n_box < 0 || T->n_box > SCVX_MAX_BOX || T->n_obs < 0 || T->n_obs > SCVX_MAX_OBS || T->j_max < 0)
        return set_error(SCVX_EINVAL, "qp: box/obstacle/collision counts");
    for (int b = 0; b < T->n_box; ++b)
        if (T->box_idx[b] < 0 || T->box_idx[b] >= T->n_x) return set_error(SCVX_EINVAL, "qp: box index");
    if (T->max_iter < 1) return set_error(SCVX_EINVAL, "qp: max_iter");
    if (T->n_u > 4 || T->n_u < 1) return set_error(SCVX_EUNSUPPORTED, "qp: n_u must be in [1, 4]");
    qp_row_counts(*T, rows, ngroups);
    return SCVX_OK;
}
}  // namespace

// Diagnostics hook (not part of the solve contract): subsequent scvx_qp_solve_batched launches write
// 8 doubles per IPM iteration of agent `agent` into the device buffer (pres, dres, gap, pobj,
// alpha_aff, alpha, sigma, mu).  buf = NULL disables.
extern "C" int scvx_qp_set_trace(double* buf, int agent, int cap) {
    g_trace = buf; g_trace_agent = agent; g_trace_cap = buf ? cap : 0;
    return SCVX_OK;
}

extern "C" size_t scvx_qp_workspace_bytes(const scvx_qp_template* tpl, int N) {
    if (!tpl || N <= 0) return 0;
    return sizeof(double) * (size_t)N * (size_t)qp_ws_doubles_per_agent(*tpl, tpl->n_x, tpl->n_u);
}

extern "C" int scvx_qp_solve_batched(const scvx_qp_template* tpl, int N, const double* disc, const double* sigma,
                                     const double* Xref, const double* Uref, const double* x_init,
                                     const double* x_final, const double* tr, const double* coll_rows,
                                     const int32_t* coll_count, double* X, double* U, double* slack_coll,
                                     double* obj, int32_t* status, int32_t* iters, void* workspace,
                                     size_t workspace_bytes, void* stream) {
    int rows = 0, ngroups = 0;
    int rc = qp_check(tpl, N, rows, ngroups);
    if (rc != SCVX_OK) return rc;
    if (N == 0) return SCVX_OK;
    if (!disc || !sigma || !Xref || !Uref || !x_init || !tr || !X || !U || !slack_coll || !obj || !status || !iters)
        return set_error(SCVX_EINVAL, "qp: null buffer");
    if (tpl->has_final && !x_final) return set_error(SCVX_EINVAL, "qp: x_final required");
    if (tpl->j_max > 0 && (!coll_rows || !coll_count)) return set_error(SCVX_EINVAL, "qp: collision rows required");
    if (!workspace || workspace_bytes < scvx_qp_workspace_bytes(tpl, N)) return set_error(SCVX_EWORKSPACE, "qp: workspace too small");
    QPArgs a{};
    a.T = *tpl;
    a.N = N;
    a.disc = disc; a.sigma = sigma; a.Xref = Xref; a.Uref = Uref; a.x_init = x_init; a.x_final = x_final;
    a.tr = tr; a.coll_rows = coll_rows; a.coll_count = coll_count;
    a.X = X; a.U = U; a.slack_coll = slack_coll; a.obj = obj; a.status = status; a.iters = iters;
    a.ws = (double*)workspace;
    a.ws_agent = qp_ws_doubles_per_agent(*tpl, tpl->n_x, tpl->n_u);
    a.trace = g_trace; a.trace_agent = g_trace_agent; a.trace_cap = g_trace_cap;
    a.rows_max = rows;
    a.gmax = ngroups > 0 ? ngroups : 1;
    hipStream_t st = (hipStream_t)stream;
    const int m = tpl->model_id;
    if (m == SCVX_MODEL_DOUBLE_INTEGRATOR && tpl->n_x == 6 && tpl->n_u == 3) return dispatch_model<6, 3>(a, st);
    if (m == SCVX_MODEL_UNICYCLE && tpl->n_x == 3 && tpl->n_u == 2) return dispatch_model<3, 2>(a, st);
    if (m == SCVX_MODEL_SINGLE_INTEGRATOR && tpl->n_x == 3 && tpl->n_u == 3) return dispatch_model<3, 3>(a, st);
    if (m == SCVX_MODEL_QUADROTOR && tpl->n_x == 12 && tpl->n_u == 4) return dispatch_model<12, 4>(a, st);
    return set_error(SCVX_EUNSUPPORTED, "qp: model id / dimensions");
}
