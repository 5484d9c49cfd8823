// Batched trust-region QP/SOCP solve for the SCvx inner loop (MI355X / gfx950, float64).
//
// Replaces the per-agent CVXPY+Clarabel solve of Distributed_opt/dist_scvx_3d.py:51-111
// (x_traj_opt), batched over N agents; the problem is stated in include/scvx_hip.h.
//
// Algorithm: primal-dual interior point, Mehrotra predictor-corrector, Nesterov-Todd scaling for
// the per-node second-order cone ||u_t|| <= u_max, CVXOPT-style starting point.  Each Newton
// system is solved by a Riccati recursion over the K nodes in the FOH-transformed state
// xi_t = x_t - C_{t-1} u_t (x_{t+1} = A x_t + B u_t + C u_{t+1} + c  becomes
// xi_{t+1} = A xi_t + Bt u_t + c with Bt = B + A C_{t-1}); the terminal equality is handled by an
// n x n Schur complement M on its multiplier mu, accumulated in the factor sweep.  Soft-constraint
// slacks (obstacle slacks, the shared collision slack S_t of dist_scvx_3d.py:93-107) are
// eliminated per node.
//
// Mapping: one agent per 64-lane wavefront (= workgroup), lane t = node t.  The design follows
// the measured gfx950 latencies (tools/ubench/lat.hip: dependent LDS load ~60 cycles, FP64 FMA 6,
// a readlane-broadcast 6x6 chain step ~180, a global load under full-chip load ~2,500):
// nothing on a sequential chain touches global memory, and every lane-parallel phase issues its
// global loads as one batch.
//   * node phases  -- lane-parallel over the nodes.  The per-node state (z, y, slacks s and duals
//                     lambda of every inequality row, SOC pair, slack groups) lives in the
//                     agent workspace and is loaded as one batch at the start of each phase, so
//                     nothing node-sized stays in registers across the sweeps.  Rows have
//                     compile-time capacities (QPCfg: 2^m trust-region facets, NB boxes, NO
//                     obstacles, NC collision rows, their slack groups): every row loop is
//                     unrolled with the row kind resolved at compile time;
//   * factor sweep -- sequential over stages, element-parallel over lanes: 4 straight-line
//                     phases per stage, each lane's output element picked by a packed
//                     descriptor (no per-stage branching); stage packets are prefetched three
//                     stages ahead (register buffers) into a 2-slot LDS ring;
//   * solves       -- closed-loop form.  With Acl_t = A_t + Bt_t K_t (kept in LDS by the factor)
//                     the backward pass is the chain p_t = Acl_t' p_{t+1} + g_t and the forward
//                     pass the chain xi_{t+1} = Acl_t xi_t + f_t: g_t, f_t and every output off
//                     the chain (feed-forward k0, inputs, multipliers) are computed lane-parallel
//                     before/after the chain, and each chain step is one n-term dot product per
//                     lane with the previous vector broadcast by DPP row_newbcast (NX <= 16).
// Factor outputs other than Acl go to stage-minor workspace columns (ws[col * 64 + t]) that the
// lane-parallel passes read coalesced.
#pragma once
#ifndef __HIPCC_RTC__   // (this header is also compiled at run time for user models: csrc/subproblem_rtc.hip)
#include <hip/hip_runtime.h>

#include "common.hpp"
#endif
#include <type_traits>

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
    const int32_t* warm; // per agent: start from the state this workspace holds from the agent's last solve
    double* X;
    double* U;
    double* slack_coll;
    double* nu;          // virtual control [N][K-1][n] (w_nu > 0 classes)
    double* obj;
    int32_t* status;
    int32_t* iters;
    double* ws;          // workspace
    long long ws_agent;  // doubles per agent
    double* trace;       // optional per-iteration diagnostics of agent `trace_agent` (or nullptr)
    int trace_agent, trace_cap;
    const int32_t* order;  // optional dispatch order: workgroup b solves agent order[b] (nullptr: agent b)
};

// ---- sizes shared by host (workspace / LDS bytes) and device
constexpr int qp_dstr(int nx, int nu) { return nx * (nx + 2 * nu + 2); }
// stiff trust-region facets (the coupled classes, n <= 8, 2 <= m <= 4; see QPCfg::STF): the 2^m facet weights, their
// folded sum (diagonal and upper off-diagonals of sum_f D_f g_f g_f') and their maximum ride in the packet; at most
// m-1 of them stay explicit per stage
constexpr bool qp_stf(int nx, int nu, int nc) { return nx <= 8 && nu >= 2 && nu <= 4 && nc > 0; }
constexpr int qp_pm(int nx, int nu, int nc) { return qp_stf(nx, nu, nc) ? nu - 1 : 0; }
constexpr int qp_nfd(int nx, int nu, int nc) { return qp_stf(nx, nu, nc) ? (1 << nu) + 2 + nu * (nu - 1) / 2 : 0; }
constexpr int qp_pkt(int nx, int nu, int nv = 0, int nc = 0) {
    return 2 * nx * nx + 4 * nx * nu + nu * nu + nx + nv + qp_nfd(nx, nu, nc);
}
// global packet: n <= 8 compact (Q as its diagonal + the 3 off-diagonals of the position block, S, R upper
// packed, e, A, Bt (column-major), C_{t-1}, the virtual control's D) -- expanded to the LDS packet layout by the
// factor's prefetch through a per-lane gather table; n = 12 dense (the LDS layout itself, QPCfg::DPK)
constexpr int qp_gpk(int nx, int nu, int nv = 0, int nc = 0) {
    return nx > 8 ? qp_pkt(nx, nu, nv, nc)
                  : (nx + 3) + nx * nu + nu * (nu + 1) / 2 + nx + nx * nx + 2 * nx * nu + nv + qp_nfd(nx, nu, nc);
}
constexpr int qp_even(int x) { return (x + 1) & ~1; }
// workspace columns (K doubles each: one per node) of a capacity class
constexpr int qp_ncol(int nx, int nu, int nb, int ns, int ng, int nv = 0) {
    // disc^T | Bt | soft rows | groups | rd | r1a | cP | ub | node state | SOC | virtual control state |
    // warm-start state (row duals, initial / terminal multipliers)
    return qp_dstr(nx, nu) + nx * nu + 4 * ns + 4 * ng + (nx + nu) + ng + ((1 << nu) + 2 * nb + ns + ng) + nu +
           ((nx + nu) + nx + 2 * (nu + 1) + ng) + (3 * (nu + 1) + 1 + (nu + 1)) + 11 * nv +
           ((1 << nu) + 2 * nb + ns + ng) + 1 + (nx > 8 ? 2 * ((1 << nu) + 2 * nb + ns + ng) : 0);
}
// factor outputs per stage (stage-major block): K, kappa, LD, W2, P, Pi, u, Acl, [virtual control: G^-1 P,
// G^-1 Pi, G^-1, Acl~], [stiff facets: Gamma, Gamma_kappa, W, C^-1, facet indices], one junk slot (the global
// store of lanes without an output of their own)
constexpr int qp_fbs(int nx, int nu, int nv = 0, int nc = 0) {
    return 3 * nu * nx + nu * nu + 3 * nx * nx + nx + 4 * nv * nx +
           qp_pm(nx, nu, nc) * (2 * nx + nu + qp_pm(nx, nu, nc) + 1) + 1;
}
// per agent: columns [c][K], packets [K][GPK], factor blocks [K][FBS] -- only the K nodes: lanes >= K
// address past the end of the buffer (loads read 0, stores are dropped), so the agent's footprint is
// what its nodes touch (C3: 1024 agents x 199 KB stay inside the 256 MB Infinity Cache)
// n = 12 classes: the factor's per-lane phase descriptors, [repetition][lane] x 16 bytes (QPRepC + pad), after the
// factor blocks (agent-independent, rewritten at each sweep; see the factor sweep)
constexpr int qp_nrep(int nx, int nu) {
    return (2 * nx * nx + 2 * nx * nu + 2 * nx + 63) / 64 + (nx * nx + nu * nx + nu * nu + 63) / 64 + (4 * nx * nx + 63) / 64;
}
constexpr int qp_dtab(int nx, int nu) { return nx > 8 ? qp_nrep(nx, nu) * 64 * 2 : 0; }
constexpr long long qp_ws_doubles(int nx, int nu, int nb, int ns, int ng, int K, int nv = 0, int nc = 0) {
    return (long long)K * (qp_ncol(nx, nu, nb, ns, ng, nv) + qp_gpk(nx, nu, nv, nc) + qp_fbs(nx, nu, nv, nc)) +
           qp_dtab(nx, nu);
}
// LDS doubles of a class (QPCfg::lds_doubles, written out for the host of a runtime-compiled class, which
// has no QPCfg instantiation; QPCfg asserts that both agree)
constexpr int qp_lds_doubles(int nx, int nu, int nb, int no, int nc, int vc, int K) {
    const int nv = vc ? nx : 0;
    const int pkt = qp_pkt(nx, nu, nv, nc);
    const int f_sink = pkt + 5 * nx * nx + 5 * nx * nu + nu * nu;
    const int f_end = qp_even(f_sink + (nx > 8 ? nx : 8) + 4 * nv * nx);
    const int nr = (1 << nu) + 2 * nb + no + nc + no + (nc > 0 ? 1 : 0);
    const int l_var = qp_even(f_end + 2 * nx * nx + 8 * nx + 1 + 4) + 16 + (nx > 8 ? 0 : 2 * nr * 64);
    return l_var + K * nx + (K + 1) * nx + (nx <= 8 ? 8 * nx * nx : 0);
}
// byte offset of every access of a lane without a node (t >= K): beyond num_records of any workspace
constexpr int QP_OOB = 0x40000000;
// warm start: floor of every slack and dual of the previous iterate (scaled units; oracle/scvx_cpu.cpp)
constexpr double QP_WARM_ETA = 1e-3;
// ... except that a row's dual floor is min(QP_WARM_ETA, QP_WARM_KAPPA / s) at its recomputed slack s: a row far from
// active (box rows, obstacle rows away from the trajectory: s ~ 1..10) keeps a dual near its last, tiny value instead
// of 1e-3, so the start's complementarity s lambda is ~1e-5 there, not ~1e-2.  The warm solve starts ~100x closer
// to the end game: on the CPU twin over the bench's 25 steps, the slowest agent's IPM iterations summed over the
// timed steps fall 171 -> 132 (per-agent rule) and 240 -> 201 (global rule), seeds 2 and 3 alike
constexpr double QP_WARM_KAPPA = 1e-5;
// stiff trust-region facet: its barrier weight D = lambda / s above QP_STIFF x the largest diagonal entry of the rest
// of the stage's input Hessian Rhat (oracle/scvx_cpu.cpp STIFF_RATIO, the same rule)
constexpr double QP_STIFF = 1e6;

// a / b for the per-row barrier quantities (l / s, the rows' Newton terms): the hardware reciprocal, two Newton
// steps and a product (~1.5 ulp, six instructions) instead of the correctly rounded division sequence (eleven,
// with a longer dependent chain); these run once per row per phase on every node
__device__ __forceinline__ double qp_div(double a, double b) {
#ifdef QP_EXACT_DIV   // diagnostics build (tools/qp_div_accuracy.py): the correctly rounded division of round 4
    return a / b;
#endif
    double r = __builtin_amdgcn_rcp(b);
    r = fma(fma(-b, r, 1.0), r, r);
    r = fma(fma(-b, r, 1.0), r, r);
    return a * r;
}
// fraction-to-boundary of the end game (affine step >= 0.99).  In the warm-started Jacobi loop almost every
// solve is an end game from its first iteration: each step is a full Newton step up to this fraction, so
// the gap falls by 1 / (1 - QP_TAU_END) per iteration.  0.999 took the C3 bulk 5 iterations, 1 - 1e-5 takes
// it 3 (oracle/scvx_cpu.cpp, the same rule; 1 - 1e-6 lengthened the tail: measured on the twin over the
// bench's 25 steps)
constexpr double QP_TAU_END = 0.99999;
// chunked solve chains (NX <= 8): the K-1 transitions are cut into QP_NCH chunks, one per 8-lane group; a
// chunk holds at most QP_CLM transitions (K <= 64)
constexpr int QP_NCH = 8, QP_CLM = 8;

// VC_ = 1: the virtual-control class (scvx_qp_template.w_nu > 0): nu_t in every dynamics row, priced
// w_nu ||nu_t||_1 through its epigraph -e <= nu <= e.  nu is eliminated inside each Riccati stage
// (G = D + P_{t+1}, D = the node's nu curvature after e is eliminated), e and the 2 n rows per node
// live in workspace columns, not in the LDS row state.
template <int NX_, int NU_, int NB_, int NO_, int NC_, int VC_ = 0>
struct QPCfg {
    static constexpr int NX = NX_, NU = NU_, NB = NB_, NO = NO_, NC = NC_, VC = VC_;
    static constexpr int NV = VC_ ? NX_ : 0, NVA = NV > 0 ? NV : 1;
    static constexpr int NZ = NX + NU, NQ = NU + 1, NTR = 1 << NU;
    static constexpr int NS = NO + NC;                // soft halfspace rows
    static constexpr int NG = NO + (NC > 0 ? 1 : 0);  // slack groups (one per obstacle, one shared)
    static constexpr int R_BOX = NTR, R_OBS = NTR + 2 * NB, R_COL = R_OBS + NO, R_GRP = R_COL + NC;
    static constexpr int NR = R_GRP + NG;
    static constexpr int DSTR = qp_dstr(NX, NU);
    // factor packet [t][PKT]: node Hessian Q|S|R, e, then the constant A (column-major) | Bt
    // column-major | Bt row-major | C_{t-1} (column-major).  Every dot product of the factor
    // phases then reads two contiguous LDS vectors.
    // stiff trust-region facets (STF: the coupled classes, n <= 8 and 2 <= m <= 4): the node's R leaves the 2^m
    // facets' D g g' out; their weights D_f, their folded sum and max ride in the packet (P_FD) and factor phase 3
    // folds them back into Rhat, all but at most PM = m-1 stiff ones, which stay explicit stage unknowns (Woodbury;
    // see the factor).  The uncoupled classes (C3) fold the facets into R as before: no stiff facet has failed a
    // C3 solve, and the stage work costs ~13 % of an IPM iteration there (round 5 A/B).
    static constexpr bool STF = qp_stf(NX_, NU_, NC_);
    static constexpr int NFD = qp_nfd(NX_, NU_, NC_), PM = qp_pm(NX_, NU_, NC_), PMA = PM > 0 ? PM : 1;
    // packet: the facet weights | their folded sum (diagonal, upper off-diagonals) | their maximum
    static constexpr int NFO = NU_ * (NU_ - 1) / 2;
    static constexpr int P_Q = 0, P_S = P_Q + NX * NX, P_R = P_S + NX * NU, P_E = P_R + NU * NU,
                         P_A = P_E + NX, P_BT = P_A + NX * NX, P_BTR = P_BT + NX * NU, P_C = P_BTR + NX * NU,
                         P_D = P_C + NX * NU, P_FD = P_D + NV, PKT = P_FD + NFD;
    static_assert(PKT == qp_pkt(NX, NU, NV, NC), "packet size");
    // global packet (compact, n <= 8; qp_gpk): Q diagonal | Q position-block off-diagonals (0,1) (0,2) (1,2) |
    // S | R upper packed | e | A (column-major) | Bt (column-major) | C_{t-1} (column-major) | D
    static constexpr int G_QD = 0, G_QO = G_QD + NX, G_S = G_QO + 3, G_R = G_S + NX * NU,
                         G_E = G_R + NU * (NU + 1) / 2, G_A = G_E + NX, G_BT = G_A + NX * NX, G_C = G_BT + NX * NU,
                         G_D = G_C + NX * NU, G_FD = G_D + NV;
    // n = 12 (DPK): the global packet has the LDS layout element for element.  The compact form needs a per-lane
    // gather table of PFN offsets live across the factor sweep; at n = 12 the register allocator spilled it to
    // scratch, and every reload waited for the packet prefetches in flight.  The dense prefetch is one
    // contiguous load per 64 elements; Q's structural zeros are written once per solve (setup), with the
    // constant A | Bt | Bt row-major | C_{t-1}; the node phase writes Q's nonzeros (both triangles), S, R (both
    // halves), e, D.  (n <= 8 keeps the compact form: its 3-entry table costs nothing, the dense packet's extra
    // traffic does: C3 780 -> 742 SCvx-it/s, A/B round 4.)
    static constexpr bool DPK = NX > 8;
    static constexpr int GPK = DPK ? PKT : G_FD + NFD;
    static_assert(GPK == qp_gpk(NX, NU, NV, NC), "global packet size");
    static_assert(NX >= 3, "the position block is 3 x 3");
    // global packet element of LDS packet element e (-1: a structural zero)
    static constexpr int gsrc(int e) {
        if (DPK) return e;
        if (e < P_S) {
            const int i = e / NX, j = e % NX;
            if (i == j) return G_QD + i;
            if (i < 3 && j < 3) return G_QO + i + j - 1;  // (0,1) -> 0, (0,2) -> 1, (1,2) -> 2
            return -1;
        }
        if (e < P_R) return G_S + (e - P_S);
        if (e < P_E) {
            const int i = (e - P_R) / NU, j = (e - P_R) % NU, p = i < j ? i : j, q = i < j ? j : i;
            return G_R + p * NU - p * (p - 1) / 2 + (q - p);
        }
        if (e < P_A) return G_E + (e - P_E);
        if (e < P_BT) return G_A + (e - P_A);
        if (e < P_BTR) return G_BT + (e - P_BT);
        if (e < P_C) {
            const int i = (e - P_BTR) / NU, j = (e - P_BTR) % NU;
            return G_BT + j * NX + i;
        }
        if (e < P_D) return G_C + (e - P_C);
        if (e < P_FD) return G_D + (e - P_D);
        return G_FD + (e - P_FD);
    }
    // global packet index of the node-phase outputs e, D and of the constant blocks
    static constexpr int gE = DPK ? P_E : G_E, gD = DPK ? P_D : G_D, gS = DPK ? P_S : G_S, gA = DPK ? P_A : G_A,
                         gBT = DPK ? P_BT : G_BT, gC = DPK ? P_C : G_C, gFD = DPK ? P_FD : G_FD;
    static_assert(NX <= 16, "the solve chains broadcast within one 16-lane row");
    // factor outputs: stage-major blocks [t][FBS] (coalesced stores from the element-parallel
    // factor; each lane-parallel pass reads its own stage's block)
    static constexpr int B_K = 0;                  // K      NU x NX
    static constexpr int B_KAP = B_K + NU * NX;    // kappa  NU x NX
    static constexpr int B_LD = B_KAP + NU * NX;   // LDL' of Rhat: L[i][j] (i > j), 1/d_i on the diagonal
    static constexpr int B_W2 = B_LD + NU * NU;    // W2 = Bt' Pi_{t+1}  NU x NX
    static constexpr int B_P = B_W2 + NU * NX;     // P_t
    static constexpr int B_PI = B_P + NX * NX;     // Pi_t
    static constexpr int B_U = B_PI + NX * NX;     // P_{t+1} e_t
    static constexpr int B_ACL = B_U + NX;         // Acl_t = A_t + Bt_t K_t (row-major)
    // virtual control (VC): G^-1 P_{t+1}, G^-1 Pi_{t+1}, G^-1 (column-major), the chain matrix
    // Acl~ = G^-1 D Acl (row-major)
    static constexpr int B_YP = B_ACL + NX * NX, B_YPI = B_YP + NV * NX, B_GI = B_YPI + NV * NX,
                         B_ACL2 = B_GI + NV * NX;
    static constexpr int B_CH = NV > 0 ? B_ACL2 : B_ACL;  // what the solve chains read
    // stiff facets (STF): Gamma = -C^-1 G' R0^-1 Sh and Gamma_kappa = -C^-1 G' R0^-1 W2 (PM x NX, row-major: the
    // multiplier steps nu = Gamma xi + Gamma_kappa mu + gamma0), then W = R0^-1 G (NU x PM), C^-1 (PM x PM) and the
    // stiff facets' indices (PM, -1 = empty slot)
    static constexpr int B_GAM = B_ACL2 + NV * NX, B_GAK = B_GAM + PM * NX, B_WS = B_GAK + PM * NX,
                         B_CI = B_WS + NU * PM, B_SF = B_CI + PM * PM;
    static constexpr int NSMB = NU * PM + PM * PM + PM;   // W | C^-1 | indices: one small block
    static constexpr int B_JNK = B_SF + PM;  // junk slot (stores of lanes without an output)
    static constexpr int FBS = B_JNK + 1;
    static_assert(FBS == qp_fbs(NX, NU, NV, NC), "factor block");
    // stage-minor workspace columns
    static constexpr int C_DT = 0;                 // disc, transposed: A (col-major) | B | C | S | z
    static constexpr int C_BT = C_DT + DSTR;       // Bt_t (row-major)
    static constexpr int C_SOFT = C_BT + NX * NU;  // soft rows (g0, g1, g2, b)
    static constexpr int C_GRP = C_SOFT + 4 * NS;  // per group: Hpa/Haa (3), 1/Haa
    static constexpr int C_RD = C_GRP + 4 * NG;    // dual residual (x, u part)
    static constexpr int C_R1A = C_RD + NZ;        // group part of the current Newton rhs
    static constexpr int C_CP = C_R1A + NG;        // predictor products ds_a dl_a per row
    static constexpr int C_UB = C_CP + NR;         // reference input ubar_t
    // node state
    static constexpr int C_Z = C_UB + NU, C_Y = C_Z + NZ, C_SQ = C_Y + NX,
                         C_LQ = C_SQ + NQ, C_AV = C_LQ + NQ;
    // SOC scaling of the current iteration: w (NQ), eta, W lam (NQ), rc (NQ), rho (NQ)
    static constexpr int C_WV = C_AV + NG, C_ETA = C_WV + NQ, C_LTQ = C_ETA + 1, C_RCQ = C_LTQ + NQ,
                         C_RHO = C_RCQ + NQ;
    // virtual control state (lanes t < K-1): nu, e, slacks s1 s2 and duals l1 l2 of the rows nu - e <= 0,
    // -nu - e <= 0, the e part of the Newton rhs, the predictor products of the two rows, the dual residual
    // (nu, e parts)
    static constexpr int C_VN = C_RHO + NQ, C_VE = C_VN + NV, C_VS = C_VE + NV, C_VL = C_VS + 2 * NV,
                         C_VRE = C_VL + 2 * NV, C_VCP = C_VRE + NV, C_VRD = C_VCP + 2 * NV;
    // warm start: the row duals lambda_r at the last iterate (NR), and y_init (lanes 0..NX-1) / y_fin (lanes
    // NX..2NX-1) in one column (needs K >= 2 NX: the host checks)
    static constexpr int C_WL = C_VRD + 2 * NV, C_WY = C_WL + NR;
    // row slacks / duals: LDS [r][lane] for n <= 8; for the n = 12 classes workspace columns (their 49 rows
    // took 50 KB of LDS per agent, two waves per CU; in columns the class runs four)
    static constexpr bool ROWG = NX > 8;
    static constexpr int C_RS = C_WY + 1, C_RL = C_RS + (ROWG ? NR : 0);
    static constexpr int NCOL = C_RL + (ROWG ? NR : 0);
    static_assert(NCOL == qp_ncol(NX, NU, NB, NS, NG, NV), "column count");
    // LDS (doubles, compile-time offsets except the K-sized blocks at the end):
    // factor: the current stage's packet, P', Pi' (col-major), T1, T2 (col-major), W1, W2 (col-major), Qh,
    // Sh (col-major), Rh, [K | kappa] (col-major), sink
    static constexpr int F_RING = 0, F_PP = PKT, F_PIP = F_PP + NX * NX, F_T1 = F_PIP + NX * NX,
                         F_T2 = F_T1 + NX * NX, F_W1 = F_T2 + NX * NU, F_W2 = F_W1 + NX * NX,
                         F_QH = F_W2 + NU * NX, F_SH = F_QH + NX * NX, F_RH = F_SH + NU * NX,
                         F_KK = F_RH + NU * NU, F_SINK = F_KK + 2 * NU * NX,
                         // virtual control: G^-1 P, G^-1 Pi (column-major), Z = G^-1 D (row-major), Acl (column-major)
                         F_YP = F_SINK + (NX > 8 ? NX : 8), F_YPI = F_YP + NV * NX, F_Z = F_YPI + NV * NX,
                         F_ACLC = F_Z + NV * NX, F_END = qp_even(F_ACLC + NV * NX);
    static constexpr int L_M = F_END, L_PI0 = L_M + NX * NX, L_XE = L_PI0 + NX * NX, L_XI0 = L_XE + NX,
                         L_R2F = L_XI0 + NX, L_YI = L_R2F + NX, L_YF = L_YI + NX, L_DYI = L_YF + NX,
                         L_DYF = L_DYI + NX, L_PIV = L_DYF + NX, L_ONE = L_PIV + NX, L_FLAG = L_ONE + 1,
                         L_ST = qp_even(L_FLAG + 4), L_S = L_ST + 16, L_L = L_S + (NX > 8 ? 0 : NR * 64),
                         L_VAR = L_L + (NX > 8 ? 0 : NR * 64);
    // row slacks s / duals lambda [r][lane]; then K-sized: chain offsets g/f [K][NX], chain vectors [K+1][NX];
    // then (chunked solve chains, NX <= 8) the chunk transition matrices Phi_c [QP_NCH][NX][NX]
    static constexpr bool CHK = NX <= 8;
    static constexpr int lds_doubles(int K) { return L_VAR + K * NX + (K + 1) * NX + (CHK ? QP_NCH * NX * NX : 0); }
    static_assert(lds_doubles(50) == qp_lds_doubles(NX, NU, NB, NO, NC, VC, 50), "host LDS formula");
    static_assert(4 * NV <= WAVE, "virtual control: one Gauss-Jordan column per lane");
};

// packed phase descriptors (all operands are contiguous LDS vectors; the stage packet always sits at
// F_RING, so every offset is stage-invariant):
//   operand = LDS offset (15 bits)
//   output  = LDS offset | accumulate << 15 | (global column + 1) << 17
//   base    = LDS offset | kind << 16   (kind 0: none, 1: always, 2: last stage)
__host__ __device__ constexpr int qp_dpk(int off, int) { return off; }

// Agent workspace accessor: raw buffer loads/stores with the lane part of the address in one
// VGPR (voffset) and the column part as a (rematerialisable) SGPR constant (soffset), so no
// per-column 64-bit address is ever materialised in vector registers.
typedef unsigned int qp_u2 __attribute__((ext_vector_type(2)));
typedef unsigned int qp_u4 __attribute__((ext_vector_type(4)));
// Every memory op of the factor sweep is unconditional: lanes with nothing to store write to the
// junk slot of the stage block, and prefetch loads of padding / structurally zero packet elements
// read past the end of the workspace (0).  A load or store under a divergent branch makes the
// compiler's vmcnt accounting fall back to vmcnt(0), which drains the packet prefetches issued
// stages ahead (measured: most of the factor's per-stage time).
// solve-chain prefetch depth (stages of Acl / offsets held in registers ahead of the chain)
constexpr int QP_CPF = 4;
struct QPBuf {
    __amdgpu_buffer_rsrc_t rs;
#ifdef QP_BYTE_TRACE
    // diagnostics build (tools/qp_bytes_trace.py): workspace bytes this lane requested since the last region stamp
    // (lanes without a node address QP_OOB and move nothing); the stamps fold them into the trace buffer per region
    mutable double nby = 0.0;
    __device__ __forceinline__ void cnt(int voff, int soff, double b) const {
        nby += (voff < QP_OOB && soff < QP_OOB) ? b : 0.0;
    }
#else
    __device__ __forceinline__ void cnt(int, int, double) const {}
#endif
    __device__ __forceinline__ double ld(int voff, int soff) const {
        soff = __builtin_amdgcn_readfirstlane(soff);  // uniform by construction
        cnt(voff, soff, 8.0);
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0));
    }
    __device__ __forceinline__ void st(int voff, int soff, double v) const {
        soff = __builtin_amdgcn_readfirstlane(soff);
        cnt(voff, soff, 8.0);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(qp_u2, v), rs, voff, soff, 0);
    }
    __device__ __forceinline__ qp_u4 ld4(int voff, int soff) const {
        soff = __builtin_amdgcn_readfirstlane(soff);
        cnt(voff, soff, 16.0);
        return __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0);
    }
    __device__ __forceinline__ void st4(int voff, int soff, qp_u4 v) const {
        soff = __builtin_amdgcn_readfirstlane(soff);
        cnt(voff, soff, 16.0);
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, voff, soff, 0);
    }
};
// keep a value opaque to the optimiser (volatile: re-derived where it is used, never hoisted)
__device__ __forceinline__ int qp_opaque(int v) {
    asm volatile("" : "+v"(v));
    return v;
}
// 1.0 if a == b else 0.0, opaque to the optimiser: selecting an array element by a runtime
// index with this mask stays arithmetic (a compare/select chain is turned back into a
// dynamically indexed private array, i.e. scratch memory)
__device__ __forceinline__ double qp_mask(int a, int b) {
    int m = a == b ? 1 : 0;
    asm("" : "+v"(m));
    return (double)m;
}

// One lane's repetition of a factor phase, decoded once per sweep (the offsets are stage-invariant)
struct QPRep {
    int L, R, B, O, G;   // LDS operand / base / output offsets; byte voffset of the global store
    double b1, b2, acc;  // base multipliers (every stage, last stage only); 1 if the output accumulates
};
// lsink: LDS sink (outputs that go nowhere in LDS, and accumulating outputs, which live in registers
// during the sweep); jnk: the junk slot of the stage block
__device__ __forceinline__ QPRep qp_decode(const int (&d)[4], int one, int lsink, int jnk) {
    QPRep q;
    q.L = d[0] & 0x7FFF;
    q.R = d[1] & 0x7FFF;
    const int bk = d[3] >> 16;
    q.B = bk ? (d[3] & 0x7FFF) : one;
    q.b1 = bk == 1 ? 1.0 : 0.0;
    q.b2 = bk == 2 ? 1.0 : 0.0;
    const int O = d[2];
    const bool on = O >= 0, acc = on && ((O >> 15) & 1);
    q.O = (on && !acc) ? (O & 0x7FFF) : lsink;
    q.acc = acc ? 1.0 : 0.0;
    const int g = on ? (O >> 17) - 1 : -1;
    q.G = (g >= 0 ? g : jnk) * 8;
    return q;
}

template <int KK>
__device__ __forceinline__ double qp_dot(const double* lds, int L, int R) {
    const double* lp = lds + L;
    const double* rp = lds + R;
    double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
    for (int k = 0; k < KK; ++k) {
        if (k & 1) acc1 = fma(lp[k], rp[k], acc1); else acc0 = fma(lp[k], rp[k], acc0);
    }
    return acc0 + acc1;
}

// One element-parallel phase of the factor sweep: every lane evaluates its NREP repetitions
// (out = base + sum_k L[k] R[k]), writes each to its LDS slot and its global column, and adds the
// accumulating ones (M, xe: summed over the stages) into registers -- no LDS read-modify-write on the
// sweep's chain.
// (outputs [ALO, AHI) of the phase may accumulate: only the repetitions covering them keep a register sum)
template <int KK, int NREP, int ALO = 0, int AHI = WAVE * NREP>
__device__ __forceinline__ void qp_phase(double* lds, const QPRep (&d)[NREP], double blast, const QPBuf& wb, int fbo,
                                         double (&areg)[NREP]) {
    double val[NREP];
#pragma unroll
    for (int r = 0; r < NREP; ++r)
        val[r] = fma(lds[d[r].B], d[r].b1 + blast * d[r].b2, qp_dot<KK>(lds, d[r].L, d[r].R));
#pragma unroll
    for (int r = 0; r < NREP; ++r) {
        lds[d[r].O] = val[r];
        if (WAVE * r < AHI && WAVE * r + WAVE > ALO) areg[r] = fma(d[r].acc, val[r], areg[r]);
        wb.st(d[r].G, fbo, val[r]);
    }
}

// Compact repetition (n = 12 classes): the base / accumulate flags packed in F (bits 0-1: base kind 0 none,
// 1 every stage, 2 last stage; bit 2: accumulating output) instead of three doubles, and the accumulating
// outputs keep their LDS target in O (written every stage, overwritten by the register sum after the
// sweep; nothing reads V_M / V_XE during it).  20 repetitions x 6 instead of 11 registers at NX = 12.
// Packed in three registers (round 4: the six-int form held 120 registers across the n = 12 sweep, which
// spilled to scratch inside the stage loop): L | R << 16, B | O << 16, G | F << 16 (LDS offsets < 2^15
// doubles, the global byte offset within a stage block < 2^16).
struct QPRepC {
    int LR, BO, GF;
    __device__ __forceinline__ int L() const { return LR & 0xFFFF; }
    __device__ __forceinline__ int R() const { return LR >> 16; }
    __device__ __forceinline__ int B() const { return BO & 0xFFFF; }
    __device__ __forceinline__ int O() const { return BO >> 16; }
    __device__ __forceinline__ int G() const { return GF & 0xFFFF; }
    __device__ __forceinline__ int F() const { return GF >> 16; }
};
__device__ __forceinline__ QPRepC qp_decode_c(const int (&d)[4], int one, int lsink, int jnk) {
    QPRepC q;
    const int L = d[0] & 0x7FFF, R = d[1] & 0x7FFF;
    const int bk = d[3] >> 16;
    const int B = bk ? (d[3] & 0x7FFF) : one;
    const int O = d[2];
    const bool on = O >= 0, acc = on && ((O >> 15) & 1);
    const int Oo = on ? (O & 0x7FFF) : lsink;
    const int g = on ? (O >> 17) - 1 : -1;
    const int G = (g >= 0 ? g : jnk) * 8;
    const int F = bk | (acc ? 4 : 0);
    q.LR = L | (R << 16);
    q.BO = B | (Oo << 16);
    q.GF = G | (F << 16);
    return q;
}
// as qp_phase; outputs [ALO, AHI) of the phase may accumulate (only those repetitions keep a register sum)
template <int KK, int NREP, int ALO, int AHI>
__device__ __forceinline__ void qp_phase_c(double* lds, const QPRepC* d, double blast, const QPBuf& wb,
                                           int fbo, double (&areg)[NREP]) {
    const QPRepC* q = d;
    double val[NREP];
#pragma unroll
    for (int r = 0; r < NREP; ++r) {
        const int bk = q[r].F() & 3;
        const double bm = (bk == 1 ? 1.0 : 0.0) + blast * (bk == 2 ? 1.0 : 0.0);
        val[r] = fma(lds[q[r].B()], bm, qp_dot<KK>(lds, q[r].L(), q[r].R()));
    }
#pragma unroll
    for (int r = 0; r < NREP; ++r) {
        lds[q[r].O()] = val[r];
        if constexpr (true) {
            if (WAVE * r < AHI && WAVE * r + WAVE > ALO) areg[r] = fma((q[r].F() & 4) ? 1.0 : 0.0, val[r], areg[r]);
        }
        wb.st(q[r].G(), fbo, val[r]);
    }
}

template <class C>
__global__ __launch_bounds__(64) void qp_ipm_kernel(QPArgs a) {
    constexpr int NX = C::NX, NU = C::NU, NZ = C::NZ, NQ = C::NQ, NR = C::NR, NG = C::NG, NS = C::NS,
                  NO = C::NO, NC = C::NC, NB = C::NB, PKT = C::PKT, NV = C::NV, NVA = C::NVA;
    constexpr int NGA = NG > 0 ? NG : 1, NSA = NS > 0 ? NS : 1, NBA = NB > 0 ? NB : 1;
    // solve-chain prefetch depth: two stages for the n = 12 classes (4 x 12 held doubles would spill)
    constexpr int CPF = NX > 8 ? 2 : QP_CPF;
    extern __shared__ double lds[];
    const scvx_qp_template& T = a.T;
    const int K = T.K, lane = threadIdx.x, t = lane;
    // dispatch order: workgroups start in index order as slots free up, so when the agents outnumber the resident
    // waves (C4: 4096 agents, 1024 at a time) the host can deal the longest solves first (scvx_qp_solve_batched_ordered);
    // an entry outside [0, N) falls back to the workgroup's own index
    long long agent = blockIdx.x;
    if (a.order) {
        const int o = a.order[blockIdx.x];
        agent = (o >= 0 && o < a.N) ? o : (long long)blockIdx.x;
    }
    const bool act = t < K;
    const bool ineq = act && ((t < K - 1) || T.ineq_last);
    const bool fin = T.has_final != 0;
    const bool soc = ineq && T.has_soc;
    const bool has_coll = NC > 0 && T.j_max > 0;
    const int nobs = T.n_obs, nbox = T.n_box;
    const int ccount = (ineq && has_coll) ? min((int)a.coll_count[agent * K + t], min(T.j_max, NC)) : 0;
    const double trv = a.tr[agent];
    const double sig = a.sigma[agent];
    // objective scaling: the problem is solved with its objective divided by its largest weight
    // (osc = max(1, ||q||_inf), the slack-group weights, 1e4..1e6 here), so the multipliers are O(1);
    // the iterates then start better centred (C3: 17 -> 13 IPM iterations on average).  The minimiser is
    // unchanged; the reported objective and the gap test are in the caller's units.
    double qnorm = 0.0;  // ||q||_inf: the linear objective weights of the slack groups
    if (nobs > 0) qnorm = fmax(qnorm, T.w_obs);
    if (has_coll) qnorm = fmax(qnorm, T.w_coll);
    // soft terminal state (has_final = 0, w_final > 0): + w_final ||x_{K-1} - x_final||^2, linear term
    // -2 w_final x_final at node K-1 (a build-side option for nonlinear models, no reference row)
    const bool soft_fin = !fin && T.w_final > 0.0;
    if (soft_fin) {
        for (int i = 0; i < NX; ++i) qnorm = fmax(qnorm, 2.0 * T.w_final * fabs(a.x_final[agent * NX + i]));
    }
    // virtual control (VC classes): weight of the epigraph variables e; lanes t < K-1 carry nu_t
    if (NV > 0) qnorm = fmax(qnorm, T.w_nu);
    const bool vact = NV > 0 && act && t < K - 1;
    const bool warm = a.warm != nullptr && a.warm[agent] != 0;   // wave-uniform
    // proximal term w_prox ||x_t - xbar_t||^2 (every node): linear term -2 w_prox xbar_t
    const bool prox = T.w_prox > 0.0;
    if (prox) {
        double qp = 0.0;
        for (int i = 0; i < NX; ++i) qp = fmax(qp, act ? 2.0 * T.w_prox * fabs(a.Xref[(agent * K + (act ? t : 0)) * NX + i]) : 0.0);
        qnorm = fmax(qnorm, wave_max(qp));
    }
    const double osc = fmax(1.0, qnorm), iosc = 1.0 / osc;
    const double wnu = NV > 0 ? T.w_nu * iosc : 0.0;
    const double wpx = (prox && act) ? T.w_prox * iosc : 0.0;
    // the proximal term's constant w_prox sum ||xbar||^2 (scaled): the gap tests use the true objective
    double cpx = 0.0;
    if (prox) {
        double v = 0.0;
        for (int i = 0; i < NX; ++i) {
            const double xb = act ? a.Xref[(agent * K + t) * NX + i] : 0.0;
            v = fma(wpx * xb, xb, v);
        }
        cpx = wave_sum(v);
    }
    const double wu = ((t < K - 1) ? 1.0 : T.w_last) * iosc;
    const bool fixed_u = act && (t == K - 1) && T.fix_last_input;
    const bool tsoft = soft_fin && act && (t == K - 1);
    const double wfs = tsoft ? T.w_final * iosc : 0.0;
    const double* disc = a.disc + agent * (long long)(K - 1) * C::DSTR;
    double* ws = a.ws + agent * a.ws_agent;
    QPBuf wb;
    // num_records = the agent's workspace: the lanes without a node address QP_OOB (reads 0, stores dropped)
    wb.rs = __builtin_amdgcn_make_buffer_rsrc(ws, (short)0, (int)(a.ws_agent * 8), 0x00020000);
    const int colb = K * 8;      // bytes per workspace column (one double per node)
    const int vt = act ? t * 8 : QP_OOB;  // this lane's element of a stage-minor column
    const int PKB = C::NCOL * colb;       // byte offset of the packets [t][GPK]
    const int FBB = PKB + K * C::GPK * 8;  // byte offset of the factor output blocks [t][FBS]
    const int vpk = act ? t * C::GPK * 8 : QP_OOB;
    const int vfb = act ? t * C::FBS * 8 : QP_OOB;
    // Loads go through `vcur` / `vpcur`, this lane's offsets re-derived (opaquely) at the start of every
    // phase: a load in one phase is then never merged with the same load of an earlier phase, which
    // would keep the value live in registers across the sweeps in between.  The lane-parallel passes
    // read columns (one coalesced line set per load); a lane's packet / factor block is contiguous per
    // lane (64 lines per load), so those passes read them only where no column copy exists.
    int vcur = vt, vpcur = vpk;
    auto fresh = [&]() __attribute__((always_inline)) {
        vcur = qp_opaque(vt);
        vpcur = qp_opaque(vpk);
    };
    auto cld = [&](int c) __attribute__((always_inline)) -> double { return wb.ld(vcur, c * colb); };
    auto cst = [&](int c, double v) __attribute__((always_inline)) { wb.st(vt, c * colb, v); };
    // element g of this lane's (global) packet
    auto pld = [&](int g) __attribute__((always_inline)) -> double { return wb.ld(vpcur, PKB + g * 8); };
    // Batched loads: ldn issues the loads of n consecutive columns, hold pins values in registers.
    // Issue every load of a phase first and hold them before the first use, so the phase pays one
    // memory round trip (the scheduler otherwise serialises load -> wait -> use under pressure).
    auto ldn = [&](double* dst, int c0, int n) __attribute__((always_inline)) {
#pragma unroll
        for (int e = 0; e < n; ++e) dst[e] = cld(c0 + e);
    };
    // n consecutive elements of this lane's factor output block, from block offset b0
    auto ldb = [&](double* dst, int b0, int n) __attribute__((always_inline)) {
#pragma unroll
        for (int e = 0; e < n; ++e) dst[e] = wb.ld(vfb, FBB + (b0 + e) * 8);
    };
    // (n = 12 classes: not held -- their 144-element blocks would occupy the register file and spill;
    // the compiler then interleaves the loads with their uses instead)
    auto hold = [&](double* v, int n) __attribute__((always_inline)) {
        if constexpr (NX <= 8) {
#pragma unroll
            for (int e = 0; e < n; ++e) asm volatile("" : "+v"(v[e]));
        }
    };
    auto pst = [&](int e, double v) __attribute__((always_inline)) { wb.st(vpk, PKB + e * 8, v); };

    constexpr int V_M = C::L_M, V_PI0 = C::L_PI0, V_XE = C::L_XE, V_XI0 = C::L_XI0, V_R2F = C::L_R2F,
                  V_YI = C::L_YI, V_YF = C::L_YF, V_DYI = C::L_DYI, V_DYF = C::L_DYF, V_PIV = C::L_PIV,
                  V_ONE = C::L_ONE, V_FLAG = C::L_FLAG, V_ST = C::L_ST, V_S = C::L_S, V_L = C::L_L;
    // STF: 1 once a stage of the last factor sweep kept a stiff facet (the solve and the Newton passes skip the
    // stage-system terms otherwise: every stage's slots are empty then)
    constexpr int V_SANY = C::L_FLAG + 1;
    auto stf_any = [&]() __attribute__((always_inline)) -> bool {
        return __builtin_amdgcn_readfirstlane((int)(lds[V_SANY] != 0.0)) != 0;
    };
    const int V_G = C::L_VAR, V_CH = V_G + K * NX, V_PHI = V_CH + (K + 1) * NX;
    // chunked chains (C::CHK): transitions t = 0..K-2 in chunks of CL; lane = 8 ch + ce carries element ce of
    // chunk ch, whose transitions are [cs0, cs1)
    const int KS = K - 1, CL = (KS + QP_NCH - 1) / QP_NCH, NCH = (KS + CL - 1) / CL;
    // (a phase re-derives these from qp_opaque(lane) through chunk_coords(): the address arithmetic is then
    // rebuilt inside the phase, not hoisted out of the IPM loop and held -- or spilled -- across it)
    struct ChunkC { int ch, ce, cs0, cs1; bool act; };
    auto chunk_coords = [&]() __attribute__((always_inline)) -> ChunkC {
        ChunkC r;
        const int l = qp_opaque(lane);
        r.ch = l >> 3; r.ce = l & 7;
        r.cs0 = min(r.ch * CL, KS); r.cs1 = min(r.cs0 + CL, KS);
        r.act = r.ce < NX && r.cs0 < r.cs1;
        return r;
    };
    // region timers of the traced agent (diagnostics): cycles since the previous stamp -> V_ST[i]
    const bool stamp_on = a.trace && agent == a.trace_agent;
    long long tprev = 0;
    auto stamp = [&](int i) __attribute__((always_inline)) {
        if (stamp_on) {
            __builtin_amdgcn_s_waitcnt(0);  // attribute outstanding memory traffic to its region
            const long long now = __builtin_amdgcn_s_memtime();
            if (lane == 0 && i >= 0) lds[V_ST + i] += (double)(now - tprev);
            tprev = now;
#ifdef QP_BYTE_TRACE
            // the region's workspace bytes (every lane's) -> trace buffer after the cycle slots (host: 8 cap + 36)
            const double b = wave_sum(wb.nby);
            wb.nby = 0.0;
            if (lane == 0 && i >= 0) a.trace[8 * a.trace_cap + 20 + i] += b;
#endif
        }
    };

    // diagnostics build (-DQP_PHASE_TRACE): the factor's four phases per stage into V_ST[11..14], the virtual
    // control phases (5 of the previous stage, 0 of this one) and the packet issue into V_ST[15] (no memory drain)
    auto pstamp = [&](int i) __attribute__((always_inline)) {
#ifdef QP_PHASE_TRACE
        if (stamp_on) {
            const long long now = __builtin_amdgcn_s_memtime();
            if (lane == 0) lds[V_ST + i] += (double)(now - tprev);
            tprev = now;
        }
#else
        (void)i;
#endif
    };

    // ------------------------------------------------------------------ setup (once per solve)
    {
        double Cp[NX * NU];
#pragma unroll
        for (int e = 0; e < NX * NU; ++e)
            Cp[e] = (act && t > 0) ? disc[(long long)(t - 1) * C::DSTR + NX * NX + NX * NU + e] : 0.0;
        // transposed disc (zero for t >= K-1), Bt = B + A C_{t-1}, the constant part of the packets
        double Ad[NX * NX], Bd[NX * NU];
        const bool dyn = t < K - 1;
        for (int e = 0; e < C::DSTR; ++e) cst(C::C_DT + e, dyn ? disc[(long long)t * C::DSTR + e] : 0.0);
#pragma unroll
        for (int e = 0; e < NX * NX; ++e) Ad[e] = dyn ? disc[(long long)t * C::DSTR + e] : 0.0;
#pragma unroll
        for (int e = 0; e < NX * NU; ++e) Bd[e] = dyn ? disc[(long long)t * C::DSTR + NX * NX + e] : 0.0;
        if (act) {
#pragma unroll
            for (int i = 0; i < NX; ++i)
#pragma unroll
                for (int j = 0; j < NU; ++j) {
                    double v = Bd[j * NX + i];
#pragma unroll
                    for (int k = 0; k < NX; ++k) v = fma(Ad[k * NX + i], Cp[j * NX + k], v);
                    cst(C::C_BT + i * NU + j, v);
                    pst(C::gBT + j * NX + i, v);
                    if constexpr (C::DPK) pst(C::P_BTR + i * NU + j, v);
                }
#pragma unroll
            for (int e = 0; e < NX * NX; ++e) {
                pst(C::gA + e, Ad[e]);
                if constexpr (C::DPK) pst(C::P_Q + e, 0.0);
            }
#pragma unroll
            for (int e = 0; e < NX * NU; ++e) pst(C::gC + e, Cp[e]);
        }
        // soft rows: obstacle linearisations (single_integrator_model.py:113-126) from Xref, then
        // the caller's collision rows (dist_scvx_3d.py:93-107)
        const int pd = T.pos_dim;
        double xb[3] = {0, 0, 0};
        for (int i = 0; i < pd; ++i) xb[i] = act ? a.Xref[(agent * K + t) * NX + i] : 0.0;
#pragma unroll
        for (int o = 0; o < NO; ++o) {
            double d[3] = {0, 0, 0}, nr = 0.0, bo = 0.0;
            if (o < nobs) {
                bo = T.obs_radius[o];
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    d[i] = i < pd ? xb[i] - T.obs_center[o][i] : 0.0;
                    nr += d[i] * d[i];
                }
                nr = sqrt(nr) + 1e-6;
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    d[i] = d[i] / nr;
                    bo += i < pd ? d[i] * T.obs_center[o][i] : 0.0;
                }
            }
#pragma unroll
            for (int i = 0; i < 3; ++i) cst(C::C_SOFT + o * 4 + i, d[i]);
            cst(C::C_SOFT + o * 4 + 3, bo);
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            double g[4] = {0, 0, 0, 0};
            if (c < ccount) {
                const double* src = a.coll_rows + ((agent * K + t) * T.j_max + c) * (pd + 1);
                for (int i = 0; i < pd; ++i) g[i] = src[i];
                g[3] = src[pd];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) cst(C::C_SOFT + (NO + c) * 4 + i, g[i]);
        }
        // initial node state: z = (xbar, ubar), y = 0, slack groups 0
#pragma unroll
        for (int j = 0; j < NU; ++j) cst(C::C_UB + j, act ? a.Uref[(agent * K + t) * NU + j] : 0.0);
        if (warm) {   // the last solve's primal / dual state stays in place; its y_init / y_fin to LDS
            if (lane < 2 * NX) lds[V_YI + lane] = wb.ld(vt, C::C_WY * colb);   // (V_YF = V_YI + NX)
        } else {
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                cst(C::C_Z + i, act ? a.Xref[(agent * K + t) * NX + i] : 0.0);
                cst(C::C_Y + i, 0.0);
            }
#pragma unroll
            for (int j = 0; j < NU; ++j) cst(C::C_Z + NX + j, act ? a.Uref[(agent * K + t) * NU + j] : 0.0);
#pragma unroll
            for (int g = 0; g < NG; ++g) cst(C::C_AV + g, 0.0);
#pragma unroll
            for (int i = 0; i < NV; ++i) { cst(C::C_VN + i, 0.0); cst(C::C_VE + i, 0.0); }
            if (lane < NX) { lds[V_YI + lane] = 0.0; lds[V_YF + lane] = 0.0; }
        }
        if (lane == 0) lds[V_ONE] = 1.0;
        if (lane < 16) lds[V_ST + lane] = 0.0;
    }
    // C_{t-1} (column-major as disc) of this node, from the transposed disc of node t-1 (the lane below)
    auto load_cp = [&](double* Cp) __attribute__((always_inline)) {
#pragma unroll
        for (int e = 0; e < NX * NU; ++e) Cp[e] = wb.ld(vcur - 8, (C::C_DT + NX * NX + NX * NU + e) * colb);
        hold(Cp, NX * NU);
#pragma unroll
        for (int e = 0; e < NX * NU; ++e) Cp[e] = (t > 0) ? Cp[e] : 0.0;
    };

    // ------------------------------------------------------------------ factor sweep
    // Stage inputs (Q, S, R, e of the node phase; A, Bt, C_{t-1}) are in packet t; Acl goes to
    // LDS, the other outputs to the stage-minor columns, M (and its LU) / Pi_0 / xe to persistent
    // LDS.  false on a breakdown.
    constexpr int PFN = (PKT + WAVE - 1) / WAVE;
    auto factor = [&]() __attribute__((always_inline)) -> bool {
        // phase descriptors (rebuilt per call: nothing of them stays live outside the sweep)
        constexpr int E1 = 2 * NX * NX + 2 * NX * NU + 2 * NX, E2 = NX * NX + NU * NX + NU * NU, E4 = 4 * NX * NX;
        constexpr int R1 = (E1 + WAVE - 1) / WAVE, R2 = (E2 + WAVE - 1) / WAVE, R4 = (E4 + WAVE - 1) / WAVE;
        int d1[R1][4], d2[R2][4], d4[R4][4];
        {
            const int sink = C::F_SINK;
            const int ln = qp_opaque(lane);  // volatile: keeps the descriptors inside the IPM loop
#pragma unroll
            for (int rep = 0; rep < R1; ++rep) {
                int o = ln + rep * WAVE, L = 0, R = 0, O = -1, B = 0;
                if (o < NX * NX) {  // T1 = P' A  -> T1 column-major
                    const int i = o / NX, j = o % NX;
                    L = qp_dpk(C::F_PP + i * NX, 0); R = qp_dpk(C::P_A + j * NX, 1); O = C::F_T1 + j * NX + i;
                } else if ((o -= NX * NX) < NX * NU) {  // T2 = P' Bt -> column-major
                    const int i = o / NU, j = o % NU;
                    L = qp_dpk(C::F_PP + i * NX, 0); R = qp_dpk(C::P_BT + j * NX, 1); O = C::F_T2 + j * NX + i;
                } else if ((o -= NX * NU) < NX * NX) {  // W1 = A' Pi'   (I at the last stage)
                    const int i = o / NX, j = o % NX;
                    L = qp_dpk(C::P_A + i * NX, 1); R = qp_dpk(C::F_PIP + j * NX, 0); O = C::F_W1 + o;
                    B = (i == j) ? (V_ONE | (2 << 16)) : 0;
                } else if ((o -= NX * NX) < NU * NX) {  // W2 = Bt' Pi' -> column-major (C_{K-2}' at the last stage)
                    const int i = o / NX, j = o % NX;
                    L = qp_dpk(C::P_BT + i * NX, 1); R = qp_dpk(C::F_PIP + j * NX, 0);
                    O = (C::F_W2 + j * NU + i) | ((C::B_W2 + o + 1) << 17);
                    B = (C::P_C + i * NX + j) | (1 << 15) | (2 << 16);
                } else if ((o -= NU * NX) < NX) {  // u = P' e  (global only)
                    L = qp_dpk(C::F_PP + o * NX, 0); R = qp_dpk(C::P_E, 1); O = sink | ((C::B_U + o + 1) << 17);
                } else if ((o -= NX) < NX) {  // xe += Pi'' e
                    L = qp_dpk(C::F_PIP + o * NX, 0); R = qp_dpk(C::P_E, 1); O = (V_XE + o) | (1 << 15);
                }
                d1[rep][0] = L; d1[rep][1] = R; d1[rep][2] = O; d1[rep][3] = B;
            }
#pragma unroll
            for (int rep = 0; rep < R2; ++rep) {
                int o = ln + rep * WAVE, L = 0, R = 0, O = -1, B = 0;
                if (o < NX * NX) {  // Qh = Q + A' T1 (symmetric: (min, max) element for both halves)
                    const int i = o / NX, j = o % NX, p = i < j ? i : j, q = i < j ? j : i;
                    L = qp_dpk(C::P_A + p * NX, 1); R = qp_dpk(C::F_T1 + q * NX, 0); O = C::F_QH + o;
                    B = (C::P_Q + p * NX + q) | (1 << 15) | (1 << 16);
                } else if ((o -= NX * NX) < NU * NX) {  // Sh = S' + Bt' T1 -> column-major
                    const int i = o / NX, j = o % NX;
                    L = qp_dpk(C::P_BT + i * NX, 1); R = qp_dpk(C::F_T1 + j * NX, 0); O = C::F_SH + j * NU + i;
                    B = (C::P_S + j * NU + i) | (1 << 15) | (1 << 16);
                } else if ((o -= NU * NX) < NU * NU) {  // Rh = R + Bt' T2
                    const int i = o / NU, j = o % NU, p = i < j ? i : j, q = i < j ? j : i;
                    L = qp_dpk(C::P_BT + p * NX, 1); R = qp_dpk(C::F_T2 + q * NX, 0); O = C::F_RH + o;
                    B = (C::P_R + p * NU + q) | (1 << 15) | (1 << 16);
                }
                d2[rep][0] = L; d2[rep][1] = R; d2[rep][2] = O; d2[rep][3] = B;
            }
#pragma unroll
            for (int rep = 0; rep < R4; ++rep) {
                int o = ln + rep * WAVE, L = 0, R = 0, O = -1, B = 0;
                if (o < NX * NX) {  // P = Qh + Sh' K (symmetric)
                    const int i = o / NX, j = o % NX, p = i < j ? i : j, q = i < j ? j : i;
                    L = qp_dpk(C::F_SH + p * NU, 0); R = qp_dpk(C::F_KK + q * NU, 0);
                    O = (C::F_PP + o) | ((C::B_P + o + 1) << 17); B = (C::F_QH + p * NX + q) | (1 << 16);
                } else if ((o -= NX * NX) < NX * NX) {  // Pi = W1 + Sh' kappa -> Pi' column-major
                    const int i = o / NX, j = o % NX;
                    L = qp_dpk(C::F_SH + i * NU, 0); R = qp_dpk(C::F_KK + (NX + j) * NU, 0);
                    O = (C::F_PIP + j * NX + i) | ((C::B_PI + o + 1) << 17); B = (C::F_W1 + o) | (1 << 16);
                } else if ((o -= NX * NX) < NX * NX) {  // M += W2' kappa (symmetric)
                    const int i = o / NX, j = o % NX, p = i < j ? i : j, q = i < j ? j : i;
                    L = qp_dpk(C::F_W2 + p * NU, 0); R = qp_dpk(C::F_KK + (NX + q) * NU, 0); O = (V_M + o) | (1 << 15);
                } else if ((o -= NX * NX) < NX * NX) {  // Acl = A + Bt K  -> global (+ LDS column-major for VC)
                    const int i = o / NX, j = o % NX;
                    L = qp_dpk(C::P_BTR + i * NU, 1); R = qp_dpk(C::F_KK + j * NU, 0);
                    O = (C::NV > 0 ? C::F_ACLC + j * NX + i : sink) | ((C::B_ACL + o + 1) << 17);
                    B = (C::P_A + j * NX + i) | (1 << 15) | (1 << 16);
                }
                d4[rep][0] = L; d4[rep][1] = R; d4[rep][2] = O; d4[rep][3] = B;
            }
        }
        // decoded once per sweep; accumulating outputs (xe, M) are summed in registers.
        // n = 12 classes (CMP): the decoded repetitions (QPRepC, three words each) go to a per-agent table in the
        // workspace and every stage loads them back (one 16-byte load per repetition, issued ahead of the packet
        // prefetch).  Held in registers across the sweep they were spilled to scratch by the allocator (the
        // function-wide peak is elsewhere) and reloaded at each use behind a full vmcnt drain -- which also
        // drained the packet prefetches in flight: ~100 serialised memory round trips per stage.
        constexpr bool CMP = NX > 8;
        constexpr int RT = R1 + R2 + R4;
        static_assert(!CMP || RT == qp_nrep(NX, NU), "descriptor table size (qp_dtab, the host's workspace size)");
        const int DTB = FBB + K * C::FBS * 8;   // byte offset of the descriptor table [rep][lane] x 16 B
        QPRep q1[CMP ? 1 : R1], q2[CMP ? 1 : R2], q4[CMP ? 1 : R4];
        double a1[R1], a2[R2], a4[R4];
        // virtual control: the M contributions -Pi'' G^-1 Pi' of every stage (registers, like a4)
        constexpr int R0 = (NX * NX + WAVE - 1) / WAVE;
        double amv[R0];
#pragma unroll
        for (int r = 0; r < R0; ++r) amv[r] = 0.0;
        auto tab_st = [&](int r, const QPRepC& q) __attribute__((always_inline)) {
            qp_u4 w;
            w.x = (unsigned)q.LR; w.y = (unsigned)q.BO; w.z = (unsigned)q.GF; w.w = 0u;
            wb.st4(qp_opaque(lane) * 16, DTB + r * WAVE * 16, w);
        };
        auto tab_ld = [&](int r, int vo) __attribute__((always_inline)) -> QPRepC {
            const qp_u4 w = wb.ld4(vo, DTB + r * WAVE * 16);
            QPRepC q;
            q.LR = (int)w.x; q.BO = (int)w.y; q.GF = (int)w.z;
            return q;
        };
#pragma unroll
        for (int r = 0; r < R1; ++r) {
            if constexpr (CMP) tab_st(r, qp_decode_c(d1[r], V_ONE, C::F_SINK, C::B_JNK));
            else q1[r] = qp_decode(d1[r], V_ONE, C::F_SINK, C::B_JNK);
            a1[r] = 0.0;
        }
#pragma unroll
        for (int r = 0; r < R2; ++r) {
            if constexpr (CMP) tab_st(R1 + r, qp_decode_c(d2[r], V_ONE, C::F_SINK, C::B_JNK));
            else q2[r] = qp_decode(d2[r], V_ONE, C::F_SINK, C::B_JNK);
            a2[r] = 0.0;
        }
#pragma unroll
        for (int r = 0; r < R4; ++r) {
            if constexpr (CMP) tab_st(R1 + R2 + r, qp_decode_c(d4[r], V_ONE, C::F_SINK, C::B_JNK));
            else q4[r] = qp_decode(d4[r], V_ONE, C::F_SINK, C::B_JNK);
            a4[r] = 0.0;
        }
        for (int e = lane; e < NX * NX; e += WAVE) { lds[C::F_PP + e] = 0.0; lds[C::F_PIP + e] = 0.0; lds[V_M + e] = 0.0; }
        if (lane < NX) lds[V_XE + lane] = 0.0;
        if (lane == 0) { lds[V_FLAG] = 0.0; lds[V_SANY] = 0.0; }
        __syncthreads();  // the node phase wrote the packets (global) from other lanes
        // packets stream through one LDS slot (a stage's packet is overwritten by the next one after its
        // last read), loads issued 3 stages ahead (register buffers pf[0..2], so the stage loop is
        // unrolled by 3 to keep their indices static)
        // prefetch distance: 3 stages; 2 for the n = 12 classes (9 doubles per buffer, register pressure)
        constexpr int FPD = NX > 8 ? 2 : 3;
        double pf[FPD][PFN];
        // n <= 8: lane's global packet element per prefetch slot (structural zeros read past the end: 0);
        // n = 12 (dense packet): lane l loads elements l + 64 k (the padding lanes of the last slot read the next
        // packet / factor block and store to the sink) -- no table held across the sweep
        int pfo[C::DPK ? 1 : PFN];
        if constexpr (!C::DPK) {
#pragma unroll
            for (int k = 0; k < PFN; ++k) {
                const int e = qp_opaque(lane) + WAVE * k;
                const int g = e < PKT ? C::gsrc(e) : -1;  // padding lanes read 0 (stored to the sink)
                pfo[k] = g >= 0 ? g * 8 : QP_OOB;
            }
        }
        auto pf_load = [&](int ts, double* b) __attribute__((always_inline)) {
            if constexpr (C::DPK) {
                const int vo = qp_opaque(lane) * 8;
#pragma unroll
                for (int k = 0; k < PFN; ++k) b[k] = wb.ld(vo, PKB + (ts > 0 ? ts : 0) * C::GPK * 8 + k * WAVE * 8);
            } else {
#pragma unroll
                for (int k = 0; k < PFN; ++k) b[k] = wb.ld(pfo[k], PKB + (ts > 0 ? ts : 0) * C::GPK * 8);
            }
        };
        auto pf_store = [&](int ts, const double* b) __attribute__((always_inline)) {
            const int sl = NX > 8 ? qp_opaque(lane) : lane;
#pragma unroll
            for (int k = 0; k < PFN; ++k) {
                const int e = sl + WAVE * k;
                lds[e < PKT ? C::F_RING + e : C::F_SINK] = b[k];
            }
        };
        if constexpr (FPD == 3) {
            pf_load(K - 1, pf[0]);
            pf_load(K - 2, pf[1]);
            pf_load(K - 3, pf[2]);
            pf_store(K - 1, pf[0]);
            pf_load(K - 4, pf[0]);
        } else {
            pf_load(K - 1, pf[0]);
            pf_load(K - 2, pf[1]);
            pf_store(K - 1, pf[0]);
            pf_load(K - 3, pf[0]);
        }
        wsync();
        bool bad = false;
        // one stage; buffer `nb` receives stage ts-3 (issued now), buffer `cb` holds stage ts-1
        // (lastc: std::true_type for stage K-1, the only stage whose base terms / fixed last input differ -- a
        // compile-time flag, so the loop's stage copies carry no per-stage selects for them)
        auto stage = [&](auto lastc, int ts, double* nb, const double* cb) __attribute__((always_inline)) {
            constexpr bool last = decltype(lastc)::value;
            const double blast = last ? 1.0 : 0.0;
            const int fbo = FBB + ts * C::FBS * 8;  // byte offset of this stage's output block (uniform)
            // n = 12: the lane index re-derived per stage: lane-dependent addresses and masks are rebuilt in the
            // stage, not hoisted out of the IPM loop and held (spilled) across it (n <= 8: hoisted, in registers)
            const int sl = NX > 8 ? qp_opaque(lane) : lane;
            QPRepC qs[CMP ? RT : 1];
            if constexpr (CMP) {
                const int vo = qp_opaque(lane) * 16;
#pragma unroll
                for (int r = 0; r < RT; ++r) qs[r] = tab_ld(r, vo);
            }
            pf_load(ts - FPD, nb);  // unconditional: stage K-1 re-issues K-1-FPD, ts-FPD < 0 reads zeros
            // STF: the node's largest facet weight if it is a stiff candidate (assemble), else 0 -- read before the
            // phases, off phase 3's chain
            double dfmr = 0.0;
            if constexpr (C::STF) dfmr = lds[C::F_RING + C::P_FD + C::NTR + 1 + C::NFO];
            if constexpr (C::NV > 0) {
                // ---- phase 0 (virtual control nu_ts): G = diag(D) + P', then [G^-1 Pi' | G^-1 | G^-1 P'] by
                // Gauss-Jordan without pivoting (G is SPD): lane c < 4 NX owns column c of [G | Pi' | I | P'];
                // the pivot column is broadcast by readlane (no LDS round trip per pivot).  At the last stage
                // P' = Pi' = 0 and D = 1 (assemble), so nothing changes there.
                const int c = sl < 4 * NX ? sl : 0, blk = c / NX, cc = c - blk * NX;
                const int base = (blk == 1 ? C::F_PIP : C::F_PP) + cc * NX;   // P' symmetric: row = column
                const double keep = blk == 2 ? 0.0 : 1.0;
                const double dcc = lds[C::F_RING + C::P_D + cc];
                const double diag = (blk == 2 ? 1.0 : 0.0) + (blk == 0 ? dcc : 0.0);
                double col[NX];
#pragma unroll
                for (int i = 0; i < NX; ++i) col[i] = fma(keep, lds[base + i], qp_mask(i, cc) * diag);
#pragma unroll
                for (int k = 0; k < NX; ++k) {
                    double pv[NX];
#pragma unroll
                    for (int i = 0; i < NX; ++i) pv[i] = readlane_d(col[i], k);
                    bad |= !(pv[k] > 0.0);
                    const double rk = col[k] / pv[k];
#pragma unroll
                    for (int i = 0; i < NX; ++i) col[i] = (i == k) ? rk : fma(-pv[i], rk, col[i]);
                }
                // outputs: G^-1 Pi' -> F_YPI / B_YPI, Z = G^-1 D (row-major) -> F_Z, G^-1 -> B_GI,
                // G^-1 P' -> F_YP / B_YP (column-major)
                const bool own = sl >= NX && sl < 4 * NX;
                const int gcol = blk == 1 ? C::B_YPI : (blk == 2 ? C::B_GI : C::B_YP);
#pragma unroll
                for (int i = 0; i < NX; ++i) {
                    const int lo = !own ? C::F_SINK + i
                                        : (blk == 1 ? C::F_YPI + cc * NX + i
                                                    : (blk == 2 ? C::F_Z + i * NX + cc : C::F_YP + cc * NX + i));
                    lds[lo] = blk == 2 ? col[i] * dcc : col[i];
                    wb.st((own ? gcol + cc * NX + i : C::B_JNK) * 8, fbo, col[i]);
                }
                wsync();
                // P~ = D G^-1 P' (symmetrised) -> F_PP; M -= Pi'' G^-1 Pi' (registers)
#pragma unroll
                for (int r = 0; r < R0; ++r) {
                    const int o = sl + r * WAVE, oo = o < NX * NX ? o : 0, i = oo / NX, j = oo - i * NX;
                    const double pt = 0.5 * (lds[C::F_RING + C::P_D + i] * lds[C::F_YP + j * NX + i] +
                                             lds[C::F_RING + C::P_D + j] * lds[C::F_YP + i * NX + j]);
                    const double mv = qp_dot<NX>(lds, C::F_PIP + i * NX, C::F_YPI + j * NX);
                    amv[r] -= o < NX * NX ? mv : 0.0;
                    lds[o < NX * NX ? C::F_PP + o : C::F_SINK] = pt;
                }
                wsync();
                // Pi~ = D G^-1 Pi' -> F_PIP (column-major: element o = j NX + i is row i)
#pragma unroll
                for (int r = 0; r < R0; ++r) {
                    const int o = sl + r * WAVE, oo = o < NX * NX ? o : 0;
                    const double v = lds[C::F_RING + C::P_D + (oo % NX)] * lds[C::F_YPI + oo];
                    lds[o < NX * NX ? C::F_PIP + o : C::F_SINK] = v;
                }
                wsync();
            }
            pstamp(15);
            // ---- phase 1: T1 = P'A, T2 = P'Bt, W1 = A'Pi', W2 = Bt'Pi', u = P'e, xe += Pi''e
            if constexpr (CMP) qp_phase_c<NX, R1, E1 - NX, E1>(lds, qs, blast, wb, fbo, a1);
            else qp_phase<NX, R1, E1 - NX, E1>(lds, q1, blast, wb, fbo, a1);
            wsync();
            pstamp(11);
            // ---- phase 2: Qh = Q + A'T1, Sh = S' + Bt'T1, Rh = R + Bt'T2
            if constexpr (CMP) qp_phase_c<NX, R2, 0, 0>(lds, qs + R1, blast, wb, fbo, a2);
            else qp_phase<NX, R2, 0, 0>(lds, q2, blast, wb, fbo, a2);
            wsync();
            pstamp(12);
            // ---- phase 3: Rh = L D L' in registers (every lane); [K | kappa] = -Rh^-1 [Sh | W2]
            {
                const bool fx = last && T.fix_last_input;
                // the phase body is compiled twice for the stiff-facet classes: CAND for a candidate node (the facet
                // branch, the stage system) and the plain body for every other stage (the straight-line code of the
                // classes without facets), one scalar branch between them
                auto ph3 = [&](auto candc) __attribute__((always_inline)) {
                constexpr bool CAND = decltype(candc)::value;
                constexpr int PM = C::PM, PMA = C::PMA;
                double Lm[NU * NU], dinv[NU];
#pragma unroll
                for (int e = 0; e < NU * NU; ++e) Lm[e] = lds[C::F_RH + e];
                // stiff trust-region facets (STF): Rhat arrives without the facets.  Those whose weight exceeds
                // QP_STIFF x its largest diagonal stay explicit when there are at most m-1 of them and no two are
                // opposite (a face or an edge of the L1 ball: they leave a complement whose small curvature the fold
                // would lose); the others fold back.  m or more stiff ones (a vertex) make every direction of u stiff:
                // they fold too, the folded sum then loses nothing while the Woodbury form would cancel
                // (oracle/scvx_cpu.cpp, the same rule)
                int sfi[PMA];
                double sfd[PMA];
#pragma unroll
                for (int i = 0; i < PMA; ++i) { sfi[i] = -1; sfd[i] = 1.0; }
                bool stg = false;   // this stage keeps a stiff facet (uniform: a scalar branch)
                if constexpr (C::STF && CAND) {
                    constexpr int NTR = C::NTR, FS = C::F_RING + C::P_FD + NTR;
                    // a candidate node (assemble: its facets left out of R, dfm > 0); every lane reads the same packet
                    // words, and readfirstlane makes the branches scalar (not predicated)
                    {
                    double dnf = 0.0;
#pragma unroll
                    for (int j = 0; j < NU; ++j) dnf = fmax(dnf, fabs(Lm[j * NU + j]));
                    const double thr = QP_STIFF * dnf;
                    // common case: every facet folds (their sum, formed in the node phase)
                    {
                        int e = 0;
#pragma unroll
                        for (int i = 0; i < NU; ++i) {
                            Lm[i * NU + i] += lds[FS];
#pragma unroll
                            for (int j = i + 1; j < NU; ++j, ++e) {
                                const double o = lds[FS + 1 + e];
                                Lm[i * NU + j] += o;
                                Lm[j * NU + i] += o;
                            }
                        }
                    }
                    if (__builtin_amdgcn_readfirstlane((int)(dfmr > thr && !fx))) {   // rare: pick the stiff slots, fold only the others
                        double Df[NTR];
                        int cnt = 0;
#pragma unroll
                        for (int f = 0; f < NTR; ++f) {
                            Df[f] = lds[C::F_RING + C::P_FD + f];
                            const bool above = Df[f] > thr;
#pragma unroll
                            for (int i = 0; i < PM; ++i) {
                                sfi[i] = (above && cnt == i) ? f : sfi[i];
                                sfd[i] = (above && cnt == i) ? Df[f] : sfd[i];
                            }
                            cnt += above ? 1 : 0;
                        }
                        bool opp = false;
#pragma unroll
                        for (int i = 0; i < PM; ++i)
#pragma unroll
                            for (int k = i + 1; k < PM; ++k) opp |= sfi[i] >= 0 && sfi[k] >= 0 && (sfi[i] ^ sfi[k]) == NTR - 1;
                        const bool use = cnt <= PM && !opp;
#pragma unroll
                        for (int i = 0; i < PM; ++i) {
                            sfi[i] = use ? sfi[i] : -1;
                            sfd[i] = use ? sfd[i] : 1.0;
                        }
                        if (use) {   // Rhat + the non-stiff facets, one at a time (the twin's order)
#pragma unroll
                            for (int e = 0; e < NU * NU; ++e) Lm[e] = lds[C::F_RH + e];
#pragma unroll
                            for (int f = 0; f < NTR; ++f) {
                                bool st = false;
#pragma unroll
                                for (int i = 0; i < PM; ++i) st |= sfi[i] == f;
                                const double d = st ? 0.0 : Df[f];
#pragma unroll
                                for (int i = 0; i < NU; ++i)
#pragma unroll
                                    for (int j = 0; j < NU; ++j) Lm[i * NU + j] += (((f >> i) ^ (f >> j)) & 1) ? -d : d;
                            }
                        }
                        stg = __builtin_amdgcn_readfirstlane((int)use) != 0;
                        if (stg && sl == 0) lds[V_SANY] = 1.0;
                    }
                    }
                }
#ifdef QP_STF_DEBUG
                double Lm0[NU * NU];
#pragma unroll
                for (int e = 0; e < NU * NU; ++e) Lm0[e] = Lm[e];
#endif
                double dmax = 0.0;
#pragma unroll
                for (int j = 0; j < NU; ++j) dmax = fmax(dmax, fabs(Lm[j * NU + j]));
                // pivots that rounding pushed below 1e-13 max|diag| are clamped (Rh is a Schur
                // complement that loses definiteness at extreme barrier scalings); NaN is fatal
                const double dmin = 1e-13 * dmax + 1e-300;
                bool nan = dmax != dmax;
#pragma unroll
                for (int j = 0; j < NU; ++j) {
                    double d = Lm[j * NU + j];
#pragma unroll
                    for (int k = 0; k < j; ++k) d -= Lm[j * NU + k] * Lm[j * NU + k] * Lm[k * NU + k];
                    nan |= d != d;
                    d = d > dmin ? d : dmin;
                    Lm[j * NU + j] = d;
                    // 1/d: hardware reciprocal + two Newton steps (~1 ulp; the correctly rounded division is a
                    // ten-instruction sequence on this serial chain, three per stage)
                    double rq = __builtin_amdgcn_rcp(d);
                    rq = fma(fma(-d, rq, 1.0), rq, rq);
                    dinv[j] = fma(fma(-d, rq, 1.0), rq, rq);
#pragma unroll
                    for (int i = j + 1; i < NU; ++i) {
                        double v = Lm[i * NU + j];
#pragma unroll
                        for (int k = 0; k < j; ++k) v -= Lm[i * NU + k] * Lm[j * NU + k] * Lm[k * NU + k];
                        Lm[i * NU + j] = v * dinv[j];
                    }
                }
                bad |= nan;
                if (fx) {
#pragma unroll
                    for (int e = 0; e < NU * NU; ++e) Lm[e] = (e / NU == e % NU) ? 1.0 : 0.0;
#pragma unroll
                    for (int j = 0; j < NU; ++j) dinv[j] = 1.0;
                }
                // x <- R0^-1 x with R0 = L D L'
                auto ldl_solve = [&](double* x) __attribute__((always_inline)) {
#pragma unroll
                    for (int i = 0; i < NU; ++i) {
#pragma unroll
                        for (int k = 0; k < i; ++k) x[i] -= Lm[i * NU + k] * x[k];
                    }
#pragma unroll
                    for (int i = 0; i < NU; ++i) x[i] *= dinv[i];
#pragma unroll
                    for (int i = NU - 1; i >= 0; --i) {
#pragma unroll
                        for (int k = i + 1; k < NU; ++k) x[i] -= Lm[k * NU + i] * x[k];
                    }
                };
                // Woodbury pieces of the stiff facets (STF): Rhat^-1 = R0^-1 - W C^-1 W', W = R0^-1 G,
                // C = D^-1 + G'W; an empty slot has g = 0, so W = 0, C = 1 there and it changes nothing
                double Wm[NU * PMA], Ci[PMA * PMA];
#pragma unroll
                for (int e = 0; e < NU * PMA; ++e) Wm[e] = 0.0;
#pragma unroll
                for (int e = 0; e < PMA * PMA; ++e) Ci[e] = (e / PMA == e % PMA) ? 1.0 : 0.0;
                if (C::STF && CAND && stg) {
#pragma unroll
                    for (int i = 0; i < PM; ++i) {
                        double w[NU];
#pragma unroll
                        for (int j = 0; j < NU; ++j) w[j] = sfi[i] < 0 ? 0.0 : (((sfi[i] >> j) & 1) ? -1.0 : 1.0);
                        ldl_solve(w);
#pragma unroll
                        for (int j = 0; j < NU; ++j) Wm[j * PM + i] = w[j];
                    }
                    double Cm[PMA * PMA];
#pragma unroll
                    for (int i = 0; i < PM; ++i)
#pragma unroll
                        for (int k = 0; k < PM; ++k) {
                            double v = (i == k) ? (sfi[i] < 0 ? 1.0 : 1.0 / sfd[i]) : 0.0;
#pragma unroll
                            for (int j = 0; j < NU; ++j)
                                v += (sfi[i] < 0 ? 0.0 : (((sfi[i] >> j) & 1) ? -1.0 : 1.0)) * Wm[j * PM + k];
                            Cm[i * PM + k] = v;
                        }
                    // C^-1 by Gauss-Jordan without pivoting (C is symmetric positive definite in exact arithmetic); a
                    // pivot that is not positive and finite, or a non-finite entry of C^-1, fails the factor, as the
                    // twin's Cholesky of C does (oracle/scvx_cpu.cpp riccati_factor).  Written with __builtin_isfinite:
                    // with x = a * b, floating-point contraction turns x - x into fma(a, b, -x), the product's rounding
                    // error, so x - x == 0 flagged finite entries (round 6)
#ifdef QP_STF_DEBUG
                    double Cm0[PMA * PMA];
#pragma unroll
                    for (int e = 0; e < PM * PM; ++e) Cm0[e] = Cm[e];
#endif
#pragma unroll
                    for (int e = 0; e < PM * PM; ++e) Ci[e] = (e / PM == e % PM) ? 1.0 : 0.0;
#pragma unroll
                    for (int k = 0; k < PM; ++k) {
                        const double pv = Cm[k * PM + k];
                        bad |= !(pv > 0.0 && __builtin_isfinite(pv));   // as the twin's Cholesky of C
#ifdef QP_STF_DEBUG
                        if (sl == 0 && !(pv > 0.0 && __builtin_isfinite(pv))) {
                            printf("STF agent %lld stage %d pivot %d = %.6e | C %.6e %.6e %.6e %.6e | sfi %d %d sfd %.3e %.3e | "
                                   "W %.3e %.3e %.3e %.3e %.3e %.3e\n", agent, ts, k, pv, Cm0[0], Cm0[1], Cm0[2], Cm0[3],
                                   sfi[0], sfi[PMA > 1 ? 1 : 0], sfd[0], sfd[PMA > 1 ? 1 : 0], Wm[0], Wm[1], Wm[2],
                                   Wm[3 % (NU * PMA)], Wm[4 % (NU * PMA)], Wm[5 % (NU * PMA)]);
                            printf("STF agent %lld stage %d R0 (folded, before LDL) %.6e %.6e %.6e | %.6e %.6e %.6e | %.6e %.6e %.6e"
                                   " | Rhat %.6e %.6e %.6e %.6e %.6e %.6e %.6e %.6e %.6e | dinv %.6e %.6e %.6e | L %.6e %.6e %.6e\n",
                                   agent, ts, Lm0[0], Lm0[1 % (NU * NU)], Lm0[2 % (NU * NU)], Lm0[3 % (NU * NU)],
                                   Lm0[4 % (NU * NU)], Lm0[5 % (NU * NU)], Lm0[6 % (NU * NU)], Lm0[7 % (NU * NU)],
                                   Lm0[8 % (NU * NU)], lds[C::F_RH + 0], lds[C::F_RH + 1], lds[C::F_RH + 2],
                                   lds[C::F_RH + 3], lds[C::F_RH + 4 % (NU * NU)], lds[C::F_RH + 5 % (NU * NU)],
                                   lds[C::F_RH + 6 % (NU * NU)], lds[C::F_RH + 7 % (NU * NU)], lds[C::F_RH + 8 % (NU * NU)], dinv[0],
                                   dinv[1 % NU], dinv[2 % NU], Lm[3 % (NU * NU)], Lm[6 % (NU * NU)], Lm[7 % (NU * NU)]);
                            double Df8[8];
                            for (int f = 0; f < 8; ++f) Df8[f] = f < C::NTR ? lds[C::F_RING + C::P_FD + f] : 0.0;
                            printf("STF agent %lld stage %d facets D %.3e %.3e %.3e %.3e %.3e %.3e %.3e %.3e\n", agent, ts,
                                   Df8[0], Df8[1], Df8[2], Df8[3], Df8[4], Df8[5], Df8[6], Df8[7]);
                        }
#endif
                        const double rp = 1.0 / pv;
#pragma unroll
                        for (int j = 0; j < PM; ++j) { Cm[k * PM + j] *= rp; Ci[k * PM + j] *= rp; }
#pragma unroll
                        for (int i = 0; i < PM; ++i) {
                            if (i == k) continue;
                            const double f = Cm[i * PM + k];
#pragma unroll
                            for (int j = 0; j < PM; ++j) {
                                Cm[i * PM + j] = fma(-f, Cm[k * PM + j], Cm[i * PM + j]);
                                Ci[i * PM + j] = fma(-f, Ci[k * PM + j], Ci[i * PM + j]);
                            }
                        }
                    }
#pragma unroll
                    for (int e = 0; e < PM * PM; ++e) bad |= !__builtin_isfinite(Ci[e]);
#ifdef QP_STF_DEBUG
                    for (int e = 0; e < PM * PM; ++e)
                        if (sl == 0 && !__builtin_isfinite(Ci[e])) printf("STF agent %lld stage %d Ci[%d] = %.6e\n", agent, ts, e, Ci[e]);
#endif
                }
                {  // every lane runs the solve (lanes >= 2 NX on a copy of column 0, results to the sinks)
                    const bool kl = sl < 2 * NX;
                    const int c = kl ? sl : 0;
                    const int off = c < NX ? C::F_SH + c * NU : C::F_W2 + (c - NX) * NU;
                    double x[NU];
#pragma unroll
                    for (int i = 0; i < NU; ++i) x[i] = lds[off + i];
                    ldl_solve(x);
                    if constexpr (C::STF) {
                        // x -= W C^-1 G'x; the multiplier-step coefficients -C^-1 G'x -> Gamma / Gamma_kappa
                        double gx[PMA], zc[PMA];
#pragma unroll
                        for (int i = 0; i < PMA; ++i) zc[i] = 0.0;
                        if (CAND && stg) {
#pragma unroll
                        for (int i = 0; i < PM; ++i) {
                            double v = 0.0;
#pragma unroll
                            for (int j = 0; j < NU; ++j)
                                v += (sfi[i] < 0 ? 0.0 : (((sfi[i] >> j) & 1) ? -1.0 : 1.0)) * x[j];
                            gx[i] = v;
                        }
#pragma unroll
                        for (int i = 0; i < PM; ++i) {
                            double v = 0.0;
#pragma unroll
                            for (int k = 0; k < PM; ++k) v = fma(Ci[i * PM + k], gx[k], v);
                            zc[i] = v;
                        }
#pragma unroll
                        for (int j = 0; j < NU; ++j)
#pragma unroll
                            for (int i = 0; i < PM; ++i) x[j] = fma(-Wm[j * PM + i], zc[i], x[j]);
                        }
                        const int gb = c < NX ? C::B_GAM + c : C::B_GAK + c - NX;
#pragma unroll
                        for (int i = 0; i < PM; ++i) wb.st((kl ? gb + i * NX : C::B_JNK) * 8, fbo, fx ? 0.0 : -zc[i]);
                    }
                    const int g = c < NX ? C::B_K + c : C::B_KAP + c - NX;
#pragma unroll
                    for (int i = 0; i < NU; ++i) {
                        const double v = fx ? 0.0 : -x[i];
                        lds[kl ? C::F_KK + c * NU + i : C::F_SINK] = v;
                        wb.st((kl ? g + i * NX : C::B_JNK) * 8, fbo, v);
                    }
                }
                {   // lane e < NU^2 stores element e of [L | 1/d] (zero above the diagonal)
                    double v = 0.0;
#pragma unroll
                    for (int e = 0; e < NU * NU; ++e) {
                        const int ei = e / NU, ej = e % NU;
                        if (ei >= ej) v = (sl == e) ? (ei > ej ? Lm[e] : dinv[ei]) : v;
                    }
                    wb.st((sl < NU * NU ? C::B_LD + sl : C::B_JNK) * 8, fbo, v);
                }
                if constexpr (C::STF) {   // lane e < NSMB stores element e of W | C^-1 | stiff indices
                    double v = 0.0;
#pragma unroll
                    for (int e = 0; e < NU * PM; ++e) v = (sl == e) ? Wm[e] : v;
#pragma unroll
                    for (int e = 0; e < PM * PM; ++e) v = (sl == NU * PM + e) ? Ci[e] : v;
#pragma unroll
                    for (int e = 0; e < PM; ++e) v = (sl == NU * PM + PM * PM + e) ? (double)sfi[e] : v;
                    wb.st((sl < C::NSMB ? C::B_WS + sl : C::B_JNK) * 8, fbo, v);
                }
                };
                if constexpr (C::STF) {
                    if (__builtin_amdgcn_readfirstlane((int)(dfmr > 0.0))) ph3(std::true_type{});
                    else ph3(std::false_type{});
                } else {
                    ph3(std::false_type{});
                }
            }
            wsync();
            pstamp(13);
            // ---- phase 4: P = Qh + Sh'K, Pi = W1 + Sh'kappa, M += W2'kappa, Acl = A + Bt K
            if constexpr (CMP) qp_phase_c<NU, R4, 2 * NX * NX, 3 * NX * NX>(lds, qs + R1 + R2, blast, wb, fbo, a4);
            else qp_phase<NU, R4, 2 * NX * NX, 3 * NX * NX>(lds, q4, blast, wb, fbo, a4);
            if (ts > 0) pf_store(ts - 1, cb);
            wsync();
            pstamp(14);
            if constexpr (C::NV > 0) {
                // ---- phase 5 (virtual control): the chain matrix Acl~ = G^-1 D Acl -> global (row-major)
#pragma unroll
                for (int r = 0; r < R0; ++r) {
                    const int o = sl + r * WAVE, oo = o < NX * NX ? o : 0, i = oo / NX, j = oo - i * NX;
                    const double v = qp_dot<NX>(lds, C::F_Z + i * NX, C::F_ACLC + j * NX);
                    wb.st((o < NX * NX ? C::B_ACL2 + o : C::B_JNK) * 8, fbo, v);
                }
                wsync();
            }
        };
        // stage K-1's packet is in LDS, K-2 in pf[1], K-3 in pf[2], K-4 in pf[0]
        int ts = K - 1;
        if constexpr (FPD == 3) {
            stage(std::true_type{}, ts, pf[0], pf[1]);  // (its load of K-4 went out before the loop)
            --ts;
            while (ts >= 0) {
                stage(std::false_type{}, ts, pf[1], pf[2]);
                if (--ts < 0) break;
                stage(std::false_type{}, ts, pf[2], pf[0]);
                if (--ts < 0) break;
                stage(std::false_type{}, ts, pf[0], pf[1]);
                --ts;
            }
        } else {  // LDS: K-1, pf[1]: K-2, pf[0]: K-3 (in flight)
            stage(std::true_type{}, ts, pf[0], pf[1]);
            --ts;
            while (ts >= 0) {
                stage(std::false_type{}, ts, pf[1], pf[0]);
                if (--ts < 0) break;
                stage(std::false_type{}, ts, pf[0], pf[1]);
                --ts;
            }
        }
        if (bad) lds[V_FLAG] = 1.0;  // any lane (all agree)
        // the register-accumulated outputs (xe, M) to their LDS homes
        if constexpr (CMP) {
            const int vo = qp_opaque(lane) * 16;
#pragma unroll
            for (int r = 0; r < R1; ++r) {
                if (WAVE * r < E1 && WAVE * r + WAVE > E1 - NX) {
                    const QPRepC q = tab_ld(r, vo);
                    if (q.F() & 4) lds[q.O()] = a1[r];
                }
            }
#pragma unroll
            for (int r = 0; r < R4; ++r) {
                if (WAVE * r < 3 * NX * NX && WAVE * r + WAVE > 2 * NX * NX) {
                    const QPRepC q = tab_ld(R1 + R2 + r, vo);
                    if (q.F() & 4) lds[q.O()] = a4[r];
                }
            }
        } else {
#pragma unroll
            for (int r = 0; r < R1; ++r)
                if (d1[r][2] >= 0 && ((d1[r][2] >> 15) & 1)) lds[d1[r][2] & 0x7FFF] = a1[r];
#pragma unroll
            for (int r = 0; r < R4; ++r)
                if (d4[r][2] >= 0 && ((d4[r][2] >> 15) & 1)) lds[d4[r][2] & 0x7FFF] = a4[r];
        }
        wsync();
        if constexpr (C::NV > 0) {
#pragma unroll
            for (int r = 0; r < R0; ++r) {
                const int o = lane + r * WAVE;
                if (o < NX * NX) lds[V_M + o] += amv[r];
            }
            wsync();
        }
        // Pi_0 -> persistent; LU with partial pivoting of M (lane 0, registers)
        for (int e = lane; e < NX * NX; e += WAVE) lds[V_PI0 + e] = lds[C::F_PIP + (e % NX) * NX + e / NX];
        if constexpr (NX > 8) {
            // n = 12 classes: the same LU column-parallel (lane j < NX owns column j of M; pivot column k
            // broadcast by readlane) -- the lane-0 form holds NX x NX doubles in registers and spills.  Every
            // element sees the same operations in the same order as the lane-0 form below.
            if (fin) {
                const int j = lane < NX ? lane : 0;
                double col[NX];
#pragma unroll
                for (int i = 0; i < NX; ++i) col[i] = lds[V_M + i * NX + j];
#pragma unroll
                for (int k = 0; k < NX; ++k) {
                    double ck[NX];
#pragma unroll
                    for (int i = 0; i < NX; ++i) ck[i] = readlane_d(col[i], k);
                    int p = k;
                    double best = fabs(ck[k]);
#pragma unroll
                    for (int i = k + 1; i < NX; ++i) {
                        const double v = fabs(ck[i]);
                        if (v > best) { best = v; p = i; }
                    }
                    if (lane == 0) lds[V_PIV + k] = (double)p;
#pragma unroll
                    for (int i = k + 1; i < NX; ++i) {
                        const double m = qp_mask(i, p);
                        const double dlt = m * (col[i] - col[k]);
                        col[k] += dlt;
                        col[i] -= dlt;
                    }
#pragma unroll
                    for (int i = 0; i < NX; ++i) ck[i] = readlane_d(col[i], k);
                    const double d = ck[k];
                    if (lane == 0 && (d == 0.0 || d != d)) lds[V_FLAG] = 2.0;
                    const double inv = d != 0.0 ? 1.0 / d : 0.0;
#pragma unroll
                    for (int i = k + 1; i < NX; ++i) {
                        const double f = ck[i] * inv;
                        col[i] = (j == k) ? f : ((j > k) ? col[i] - f * col[k] : col[i]);
                    }
                }
                if (lane < NX)
#pragma unroll
                    for (int i = 0; i < NX; ++i) lds[V_M + i * NX + j] = col[i];
            }
        } else {
        if (fin && lane == 0) {
            double Mr[NX * NX];
#pragma unroll
            for (int e = 0; e < NX * NX; ++e) Mr[e] = lds[V_M + e];
#pragma unroll
            for (int k = 0; k < NX; ++k) {
                int p = k;
                double best = fabs(Mr[k * NX + k]);
#pragma unroll
                for (int i = k + 1; i < NX; ++i) {
                    const double v = fabs(Mr[i * NX + k]);
                    if (v > best) { best = v; p = i; }
                }
                lds[V_PIV + k] = (double)p;
#pragma unroll
                for (int i = k + 1; i < NX; ++i) {
                    const double m = qp_mask(i, p);
#pragma unroll
                    for (int j = 0; j < NX; ++j) {
                        const double dlt = m * (Mr[i * NX + j] - Mr[k * NX + j]);
                        Mr[k * NX + j] += dlt;
                        Mr[i * NX + j] -= dlt;
                    }
                }
                const double d = Mr[k * NX + k];
                if (d == 0.0 || d != d) lds[V_FLAG] = 2.0;
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
            for (int e = 0; e < NX * NX; ++e) lds[V_M + e] = Mr[e];
        }
        }
        wsync();
        if constexpr (C::CHK) {
            const ChunkC cc = chunk_coords();
            const int ch = cc.ch, ce = cc.ce, cs0 = cc.cs0, cs1 = cc.cs1;
            const bool cact = cc.act;
            // chunk transition matrices Phi_c = Acl_{s1-1} ... Acl_{s0} (the chain matrices B_CH of the chunk's
            // transitions, just stored by the sweep): lane (ch, ce) keeps row ce, Phi <- Acl_t Phi with the rows of
            // Phi broadcast inside the 8-lane group; the solve chains of this factor read them from LDS
            double ar[QP_CLM][NX], ph[NX];
#pragma unroll
            for (int j = 0; j < QP_CLM; ++j) {
                const int tj = cs0 + j;
                const int vo = (cact && j < CL && tj < cs1) ? (C::B_CH + ce * NX) * 8 + tj * C::FBS * 8 : QP_OOB;
#pragma unroll
                for (int k = 0; k < NX; ++k) ar[j][k] = wb.ld(vo + k * 8, FBB);
            }
#pragma unroll
            for (int c = 0; c < NX; ++c) ph[c] = (c == ce) ? 1.0 : 0.0;
#pragma unroll
            for (int j = 0; j < QP_CLM; ++j) {
                if (j < CL) {
                    double nw[NX];
#pragma unroll
                    for (int c = 0; c < NX; ++c) nw[c] = 0.0;
#pragma unroll
                    for (int k = 0; k < NX; ++k)
#pragma unroll
                        for (int c = 0; c < NX; ++c) nw[c] = fma(ar[j][k], oct_bcast_d(ph[c], k), nw[c]);
                    const bool ok = cs0 + j < cs1;
#pragma unroll
                    for (int c = 0; c < NX; ++c) ph[c] = ok ? nw[c] : ph[c];
                }
            }
#pragma unroll
            for (int c = 0; c < NX; ++c) lds[cact ? V_PHI + ch * NX * NX + ce * NX + c : C::F_SINK] = ph[c];
            wsync();
        }
        return lds[V_FLAG] == 0.0;
    };

    // ------------------------------------------------------------------ solve (one Newton rhs)
    // In: q (NX), r (NU), dv (NV: the linear term of nu_t, VC classes) of this node (registers), e (packet),
    // V_XI0 / V_R2F (LDS).
    // Out: dzo (NZ) = (dx_t, du_t), dyo (NX) = dy_t, dno (NV) = dnu_t of this lane; V_DYI / V_DYF (LDS) the
    // initial / terminal multiplier directions.  Assumes a __syncthreads() since the factor.
    // Virtual control: stage t sees P~ = D G^-1 P_{t+1} and p~ = p_{t+1} - (G^-1 P)'(p_{t+1} + d) in place of
    // P_{t+1}, p_{t+1} (oracle/scvx_cpu.cpp riccati_factor), the chains run on Acl~ = G^-1 D Acl, and
    // nu_t = xi_{t+1} - (A xi_t + Bt du_t + e_t) comes out of the forward chain.
    // rhs_s: rho of the stage's stiff facets (C::STF; 0 in empty slots), fnu: their multiplier steps (out)
    auto solve = [&](const double* q, const double* r, const double* dv, double* dzo, double* dyo, double* dno,
                     const double* rhs_s, double* fnu) __attribute__((always_inline)) {
        constexpr int PM = C::PM, PMA = C::PMA;
        double g0[PMA];   // nu's feed-forward part gamma0 = -C^-1 (G' R0^-1 rh + rho) (stiff facets)
#pragma unroll
        for (int i = 0; i < PMA; ++i) { g0[i] = 0.0; fnu[i] = 0.0; }
        // ---- backward pre-pass: g = q + K'r + Acl'(P~ e - (G^-1 P)'d) [- Gamma' rho: stiff facets]
        fresh();
        if (act) {
            double g[NX], u[NX];
            ldb(u, C::B_U, NX);
            if constexpr (NV > 0) {
                double Y[NX * NX];
                ldb(Y, C::B_YP, NX * NX);
                hold(u, NX);
                hold(Y, NX * NX);
#pragma unroll
                for (int j = 0; j < NX; ++j)
#pragma unroll
                    for (int i = 0; i < NX; ++i) u[j] = fma(-Y[j * NX + i], dv[i], u[j]);
            }
            double Kt[NU * NX], Ac[NX * NX];
            ldb(Kt, C::B_K, NU * NX);
            ldb(Ac, C::B_ACL, NX * NX);
            hold(Kt, NU * NX);
            hold(u, NX);
            hold(Ac, NX * NX);
#pragma unroll
            for (int i = 0; i < NX; ++i) g[i] = q[i];
            if constexpr (C::STF) {
                if (stf_any()) {
                    double Gm[PMA * NX];
                    ldb(Gm, C::B_GAM, PM * NX);
                    hold(Gm, PM * NX);
#pragma unroll
                    for (int i = 0; i < PM; ++i)
#pragma unroll
                        for (int j = 0; j < NX; ++j) g[j] = fma(-Gm[i * NX + j], rhs_s[i], g[j]);
                }
            }
#pragma unroll
            for (int i = 0; i < NU; ++i)
#pragma unroll
                for (int j = 0; j < NX; ++j) g[j] = fma(Kt[i * NX + j], r[i], g[j]);
            if (t < K - 1) {
#pragma unroll
                for (int i = 0; i < NX; ++i)
#pragma unroll
                    for (int j = 0; j < NX; ++j) g[j] = fma(Ac[i * NX + j], u[i], g[j]);
            }
#pragma unroll
            for (int i = 0; i < NX; ++i) lds[V_G + t * NX + i] = g[i];
        }
        wsync();
        stamp(4);
        if constexpr (C::CHK) {
            const ChunkC cc = chunk_coords();
            const int ch = cc.ch, ce = cc.ce, cs0 = cc.cs0, cs1 = cc.cs1;
            const bool cact = cc.act;
            // chunked: p_{s0} = Phi_c' p_{s1} + q_c per chunk (q_c the chunk's chain from p_{s1} = 0), so
            //   A  every chunk runs its own CL steps from 0 (the last chunk from p_{K-1} = g_{K-1}: exact),
            //   B  lanes < NX carry p across the chunk boundaries from the last chunk down (NCH - 1 steps,
            //      Phi_c' from LDS),
            //   C  every chunk re-runs its steps from its exact p_{s1}, storing p_t inside the chunk;
            // (CL + NCH - 1 + CL dependent steps instead of K - 1).  Lane (ch, ce) holds column ce of Acl_t for
            // its chunk's transitions t = cs1 - 1 - j in registers, loaded in one batch.
            double ac[QP_CLM][NX], gc[QP_CLM];
#pragma unroll
            for (int j = 0; j < QP_CLM; ++j) {
                const int tj = cs1 - 1 - j;
                const bool ok = cact && j < CL && tj >= cs0;
                const int vo = ok ? (C::B_CH + ce) * 8 + tj * C::FBS * 8 : QP_OOB;
#pragma unroll
                for (int k = 0; k < NX; ++k) ac[j][k] = wb.ld(vo + k * NX * 8, FBB);
                gc[j] = lds[V_G + (ok ? tj : 0) * NX + (ce < NX ? ce : 0)];
            }
            auto chainT = [&](double q, const double* a, double g) __attribute__((always_inline)) -> double {
                double v0 = g, v1 = 0.0;
#pragma unroll
                for (int k = 0; k < NX; ++k) {
                    const double qk = oct_bcast_d(q, k);
                    if (k & 1) v1 = fma(a[k], qk, v1); else v0 = fma(a[k], qk, v0);
                }
                return v0 + v1;
            };
            const double gK = lds[V_G + (K - 1) * NX + (ce < NX ? ce : 0)];
            if (lane < NX) lds[V_CH + (K - 1) * NX + lane] = gK;
            double q = (cs1 == KS) ? gK : 0.0;
#pragma unroll
            for (int j = 0; j < QP_CLM; ++j) {
                if (j < CL) {
                    const double qn = chainT(q, ac[j], gc[j]);
                    q = (cs1 - 1 - j >= cs0) ? qn : q;
                }
            }
            lds[cact ? V_CH + cs0 * NX + ce : C::F_SINK] = q;
            wsync();
            if (lane < NX) {
                double p = lds[V_CH + min((NCH - 1) * CL, KS) * NX + lane];
                for (int c = NCH - 2; c >= 0; --c) {
                    double v0 = lds[V_CH + c * CL * NX + lane], v1 = 0.0;
#pragma unroll
                    for (int k = 0; k < NX; ++k) {
                        const double pk = row_bcast_d(p, k);
                        const double f = lds[V_PHI + c * NX * NX + k * NX + lane];
                        if (k & 1) v1 = fma(f, pk, v1); else v0 = fma(f, pk, v0);
                    }
                    p = v0 + v1;
                    lds[V_CH + c * CL * NX + lane] = p;
                }
            }
            wsync();
            double p = lds[V_CH + (cact ? cs1 : 0) * NX + (ce < NX ? ce : 0)];
#pragma unroll
            for (int j = 0; j < QP_CLM; ++j) {
                if (j < CL) {
                    const int tj = cs1 - 1 - j;
                    const double pn = chainT(p, ac[j], gc[j]);
                    p = tj >= cs0 ? pn : p;
                    lds[(cact && tj > cs0) ? V_CH + tj * NX + ce : C::F_SINK] = p;
                }
            }
        } else {
            // ---- backward chain p_t = Acl_t' p_{t+1} + g_t (lane i: element i); p_{t+1} broadcast
            // from lanes 0..NX-1 by a DPP row broadcast (NX <= 16), the Acl column / g of the next stage read ahead
            if (lane < NX) {
                // lane i needs column i of Acl_t (stage block, B_CH + k*NX + i; Acl~ for VC)
                const int va = (C::B_CH + lane) * 8;
                auto ldA = [&](int ts, double* an, double& gn) __attribute__((always_inline)) {
                    const int tc = ts > 0 ? ts : 0;
    #pragma unroll
                    for (int k = 0; k < NX; ++k) an[k] = wb.ld(va + k * NX * 8, FBB + tc * C::FBS * 8);
                    gn = lds[V_G + tc * NX + lane];
                };
                auto chain = [&](double p, const double* ac, double g) __attribute__((always_inline)) -> double {
                    double v0 = g, v1 = 0.0;
    #pragma unroll
                    for (int k = 0; k < NX; ++k) {
                        const double pkv = row_bcast_d(p, k);
                        if (k & 1) v1 = fma(ac[k], pkv, v1); else v0 = fma(ac[k], pkv, v0);
                    }
                    return v0 + v1;
                };
                double p = lds[V_G + (K - 1) * NX + lane];
                lds[V_CH + (K - 1) * NX + lane] = p;
                // QP_CPF register buffers: operands loaded QP_CPF stages ahead (a global load under
                // full-chip load takes ~2,000 cycles; 8 stages measured no faster than 4 and spilled more)
                double ab[CPF][NX], gb[CPF];
    #pragma unroll
                for (int b = 0; b < CPF; ++b) ldA(K - 2 - b, ab[b], gb[b]);
                int ts = K - 2;
                auto step = [&](double* a, double& g) __attribute__((always_inline)) {
                    p = chain(p, a, g);
                    lds[V_CH + ts * NX + lane] = p;
                    ldA(ts - CPF, a, g);
                    --ts;
                };
                // groups of QP_CPF steps with no exit inside the loop body (a mid-body exit makes the
                // compiler's vmcnt tracking fall back to vmcnt(0) and drain the prefetches), then the
                // remaining steps continuing the buffer rotation
                while (ts >= CPF - 1) {
    #pragma unroll
                    for (int b = 0; b < CPF; ++b) step(ab[b], gb[b]);
                }
    #pragma unroll
                for (int b = 0; b < CPF - 1; ++b)
                    if (ts >= 0) step(ab[b], gb[b]);
            }
        }
        wsync();
        stamp(5);
        // ---- backward post-pass: k0 = -Rh^-1 (r + Bt'(P_{t+1} e + p_{t+1})), xacc = sum W2'k0
        fresh();
        double k0[NU], pv[NX], xa[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) { xa[i] = 0.0; pv[i] = 0.0; }
#pragma unroll
        for (int j = 0; j < NU; ++j) k0[j] = 0.0;
        if (act) {
            double uu[NX], Bt[NX * NU], Ld[NU * NU], W2[NU * NX];
            ldb(uu, C::B_U, NX);
            ldn(Bt, C::C_BT, NX * NU);
            ldb(Ld, C::B_LD, NU * NU);
            ldb(W2, C::B_W2, NU * NX);
            hold(uu, NX); hold(Bt, NX * NU); hold(Ld, NU * NU); hold(W2, NU * NX);
#pragma unroll
            for (int i = 0; i < NX; ++i) pv[i] = lds[V_CH + t * NX + i];
            double rh[NU];
#pragma unroll
            for (int j = 0; j < NU; ++j) rh[j] = r[j];
            if (t < K - 1) {
                double pn[NX];
#pragma unroll
                for (int i = 0; i < NX; ++i) pn[i] = lds[V_CH + (t + 1) * NX + i];
                if constexpr (NV > 0) {
                    // p~ = p - (G^-1 P)'(p + d);  xacc -= (G^-1 Pi)'(p + d)
                    double Y[NX * NX], w[NX];
#pragma unroll
                    for (int i = 0; i < NX; ++i) w[i] = pn[i] + dv[i];
                    ldb(Y, C::B_YP, NX * NX);
                    hold(Y, NX * NX);
#pragma unroll
                    for (int j = 0; j < NX; ++j)
#pragma unroll
                        for (int i = 0; i < NX; ++i) pn[j] = fma(-Y[j * NX + i], w[i], pn[j]);
                    ldb(Y, C::B_YPI, NX * NX);
                    hold(Y, NX * NX);
#pragma unroll
                    for (int j = 0; j < NX; ++j)
#pragma unroll
                        for (int i = 0; i < NX; ++i) xa[j] = fma(-Y[j * NX + i], w[i], xa[j]);
                }
#pragma unroll
                for (int i = 0; i < NX; ++i) {
                    const double h = uu[i] + pn[i];
#pragma unroll
                    for (int j = 0; j < NU; ++j) rh[j] = fma(Bt[i * NU + j], h, rh[j]);
                }
            }
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                double v = rh[i];
#pragma unroll
                for (int k = 0; k < i; ++k) v -= Ld[i * NU + k] * k0[k];
                k0[i] = v;
            }
#pragma unroll
            for (int i = 0; i < NU; ++i) k0[i] *= Ld[i * NU + i];
#pragma unroll
            for (int i = NU - 1; i >= 0; --i) {
                double v = k0[i];
#pragma unroll
                for (int k = i + 1; k < NU; ++k) v -= Ld[k * NU + i] * k0[k];
                k0[i] = v;
            }
            if constexpr (C::STF) if (stf_any()) {
                // a = R0^-1 rh (k0 here); gamma0 = -C^-1 (G'a + rho); k0 = -(a + W gamma0)
                double sm[C::NSMB];
                ldb(sm, C::B_WS, C::NSMB);
                hold(sm, C::NSMB);
                const double* Wm = sm;
                const double* Ci = sm + NU * PM;
                const double* sf = sm + NU * PM + PM * PM;
                double ga[PMA];
#pragma unroll
                for (int i = 0; i < PM; ++i) {
                    const int f = (int)sf[i];
                    double v = rhs_s[i];
#pragma unroll
                    for (int j = 0; j < NU; ++j) v += (f < 0 ? 0.0 : (((f >> j) & 1) ? -1.0 : 1.0)) * k0[j];
                    ga[i] = v;
                }
#pragma unroll
                for (int i = 0; i < PM; ++i) {
                    double v = 0.0;
#pragma unroll
                    for (int k = 0; k < PM; ++k) v = fma(-Ci[i * PM + k], ga[k], v);
                    g0[i] = fixed_u ? 0.0 : v;
                }
#pragma unroll
                for (int j = 0; j < NU; ++j)
#pragma unroll
                    for (int i = 0; i < PM; ++i) k0[j] = fma(Wm[j * PM + i], g0[i], k0[j]);
            }
#pragma unroll
            for (int i = 0; i < NU; ++i) k0[i] = fixed_u ? 0.0 : -k0[i];
#pragma unroll
            for (int i = 0; i < NU; ++i)
#pragma unroll
                for (int j = 0; j < NX; ++j) xa[j] = fma(W2[i * NX + j], k0[i], xa[j]);
        }
        // ---- terminal multiplier mu = M^-1 (r2f - xacc - xe - Pi_0' xi0)   (every lane)
        double mu[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            double v = lds[V_R2F + i] - wave_sum(xa[i]) - lds[V_XE + i];
#pragma unroll
            for (int k = 0; k < NX; ++k) v -= lds[V_PI0 + k * NX + i] * lds[V_XI0 + k];
            mu[i] = fin ? v : 0.0;
        }
        if (fin) {
#pragma unroll
            for (int k = 0; k < NX; ++k) {
                const int p = (int)lds[V_PIV + k];
#pragma unroll
                for (int i = k + 1; i < NX; ++i) {
                    const double dlt = qp_mask(i, p) * (mu[i] - mu[k]);
                    mu[k] += dlt;
                    mu[i] -= dlt;
                }
            }
#pragma unroll
            for (int k = 0; k < NX; ++k)
#pragma unroll
                for (int i = k + 1; i < NX; ++i) mu[i] -= lds[V_M + i * NX + k] * mu[k];
#pragma unroll
            for (int i = NX - 1; i >= 0; --i) {
                double v = mu[i];
#pragma unroll
                for (int j = i + 1; j < NX; ++j) v -= lds[V_M + i * NX + j] * mu[j];
                mu[i] = v / lds[V_M + i * NX + i];
            }
        }
        stamp(6);
        // ---- forward pre-pass: v0 = k0 + kappa mu, f = Bt v0 + e, pi = Pi_t mu
        fresh();
        double v0[NU], piv[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) piv[i] = 0.0;
#pragma unroll
        for (int j = 0; j < NU; ++j) v0[j] = k0[j];
        if (act) {
            double kap[NU * NX], Pi[NX * NX], Bt[NX * NU], ev[NX];
            ldb(kap, C::B_KAP, NU * NX);
            ldb(Pi, C::B_PI, NX * NX);
            ldn(Bt, C::C_BT, NX * NU);
#pragma unroll
            for (int i = 0; i < NX; ++i) ev[i] = pld(C::gE + i);
            hold(kap, NU * NX); hold(Pi, NX * NX); hold(Bt, NX * NU); hold(ev, NX);
#pragma unroll
            for (int i = 0; i < NU; ++i)
#pragma unroll
                for (int j = 0; j < NX; ++j) v0[i] = fma(kap[i * NX + j], mu[j], v0[i]);
#pragma unroll
            for (int i = 0; i < NX; ++i)
#pragma unroll
                for (int j = 0; j < NX; ++j) piv[i] = fma(Pi[i * NX + j], mu[j], piv[i]);
            if (t < K - 1) {
                double fv[NX];
#pragma unroll
                for (int i = 0; i < NX; ++i) {
                    double f = ev[i];
#pragma unroll
                    for (int j = 0; j < NU; ++j) f = fma(Bt[i * NU + j], v0[j], f);
                    fv[i] = f;
                }
                if constexpr (NV > 0) {
                    // f~ = G^-1 (D o f - p_{t+1} - d) - (G^-1 Pi) mu   (V_CH still holds the backward chain)
                    double Y[NX * NX], w[NX];
#pragma unroll
                    for (int i = 0; i < NX; ++i) w[i] = fma(pld(C::gD + i), fv[i], -lds[V_CH + (t + 1) * NX + i] - dv[i]);
                    ldb(Y, C::B_GI, NX * NX);
                    hold(Y, NX * NX);
#pragma unroll
                    for (int i = 0; i < NX; ++i) {
                        double v = 0.0;
#pragma unroll
                        for (int j = 0; j < NX; ++j) v = fma(Y[j * NX + i], w[j], v);
                        fv[i] = v;
                    }
                    ldb(Y, C::B_YPI, NX * NX);
                    hold(Y, NX * NX);
#pragma unroll
                    for (int i = 0; i < NX; ++i)
#pragma unroll
                        for (int j = 0; j < NX; ++j) fv[i] = fma(-Y[j * NX + i], mu[j], fv[i]);
                }
#pragma unroll
                for (int i = 0; i < NX; ++i) lds[V_G + t * NX + i] = fv[i];
            }
        }
        wsync();
        stamp(7);
        if constexpr (C::CHK) {
            const ChunkC cc = chunk_coords();
            const int ch = cc.ch, ce = cc.ce, cs0 = cc.cs0, cs1 = cc.cs1;
            const bool cact = cc.act;
            // chunked as the backward chain: x_{s1} = Phi_c x_{s0} + y_c per chunk;
            //   A  every chunk runs its CL steps from 0 (chunk 0 from xi_0: exact),
            //   B  lanes < NX carry x across the boundaries (NCH - 2 steps, Phi_c from LDS),
            //   C  every chunk re-runs from its exact x_{s0}, storing x_t inside the chunk (and x_{K-1}).
            // Lane (ch, ce) holds row ce of Acl_t, t = cs0 + j, in registers.
            double ar[QP_CLM][NX], fr[QP_CLM];
#pragma unroll
            for (int j = 0; j < QP_CLM; ++j) {
                const int tj = cs0 + j;
                const bool ok = cact && j < CL && tj < cs1;
                const int vo = ok ? (C::B_CH + ce * NX) * 8 + tj * C::FBS * 8 : QP_OOB;
#pragma unroll
                for (int k = 0; k < NX; ++k) ar[j][k] = wb.ld(vo + k * 8, FBB);
                fr[j] = lds[V_G + (ok ? tj : 0) * NX + (ce < NX ? ce : 0)];
            }
            auto chainF = [&](double x, const double* a, double f) __attribute__((always_inline)) -> double {
                double w0 = f, w1 = 0.0;
#pragma unroll
                for (int k = 0; k < NX; ++k) {
                    const double xk = oct_bcast_d(x, k);
                    if (k & 1) w1 = fma(a[k], xk, w1); else w0 = fma(a[k], xk, w0);
                }
                return w0 + w1;
            };
            const double x0 = lds[V_XI0 + (ce < NX ? ce : 0)];
            double x = (ch == 0) ? x0 : 0.0;
#pragma unroll
            for (int j = 0; j < QP_CLM; ++j) {
                if (j < CL) {
                    const double xn = chainF(x, ar[j], fr[j]);
                    x = (cs0 + j < cs1) ? xn : x;
                }
            }
            lds[cact ? V_CH + cs1 * NX + ce : C::F_SINK] = x;
            if (lane < NX) lds[V_CH + lane] = x0;
            wsync();
            if (lane < NX) {
                double xs = lds[V_CH + min(CL, KS) * NX + lane];
                for (int c = 1; c < NCH - 1; ++c) {
                    const int s1 = (c + 1) * CL;
                    double w0 = lds[V_CH + s1 * NX + lane], w1 = 0.0;
#pragma unroll
                    for (int k = 0; k < NX; ++k) {
                        const double xk = row_bcast_d(xs, k);
                        const double f = lds[V_PHI + c * NX * NX + lane * NX + k];
                        if (k & 1) w1 = fma(f, xk, w1); else w0 = fma(f, xk, w0);
                    }
                    xs = w0 + w1;
                    lds[V_CH + s1 * NX + lane] = xs;
                }
            }
            wsync();
            x = lds[V_CH + (cact ? cs0 : 0) * NX + (ce < NX ? ce : 0)];
#pragma unroll
            for (int j = 0; j < QP_CLM; ++j) {
                if (j < CL) {
                    const int tj = cs0 + j;
                    const double xn = chainF(x, ar[j], fr[j]);
                    const bool ok = tj < cs1;
                    x = ok ? xn : x;
                    lds[(cact && ok && (tj + 1 < cs1 || tj + 1 == KS)) ? V_CH + (tj + 1) * NX + ce : C::F_SINK] = x;
                }
            }
        } else {
            // ---- forward chain xi_{t+1} = Acl_t xi_t + f_t
            if (lane < NX) {
                // lane i needs row i of Acl_t (stage block, B_CH + i*NX + k; Acl~ for VC)
                const int va = (C::B_CH + lane * NX) * 8;
                auto ldA = [&](int ts, double* an, double& fn) __attribute__((always_inline)) {
                    const int tc = ts < K - 1 ? ts : K - 2;
    #pragma unroll
                    for (int k = 0; k < NX; ++k) an[k] = wb.ld(va + k * 8, FBB + tc * C::FBS * 8);
                    fn = lds[V_G + tc * NX + lane];
                };
                auto chain = [&](double x, const double* ac, double f) __attribute__((always_inline)) -> double {
                    double w0 = f, w1 = 0.0;
    #pragma unroll
                    for (int k = 0; k < NX; ++k) {
                        const double xk = row_bcast_d(x, k);
                        if (k & 1) w1 = fma(ac[k], xk, w1); else w0 = fma(ac[k], xk, w0);
                    }
                    return w0 + w1;
                };
                double x = lds[V_XI0 + lane];
                lds[V_CH + lane] = x;
                double ab[CPF][NX], fb[CPF];
    #pragma unroll
                for (int b = 0; b < CPF; ++b) ldA(b, ab[b], fb[b]);
                int ts = 0;
                auto step = [&](double* a, double& f) __attribute__((always_inline)) {
                    x = chain(x, a, f);
                    lds[V_CH + (ts + 1) * NX + lane] = x;
                    ldA(ts + CPF, a, f);
                    ++ts;
                };
                while (ts <= K - 1 - CPF) {  // CPF steps per trip, no exit inside (see the backward chain)
    #pragma unroll
                    for (int b = 0; b < CPF; ++b) step(ab[b], fb[b]);
                }
    #pragma unroll
                for (int b = 0; b < CPF - 1; ++b)
                    if (ts < K - 1) step(ab[b], fb[b]);
            }
        }
        wsync();
        stamp(8);
        // ---- forward post-pass: du = K xi + v0, dx = xi + C_{t-1} du, y_{t-1} = -(P xi + p + pi)
        fresh();
        double ym[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) ym[i] = 0.0;
#pragma unroll
        for (int i = 0; i < NZ; ++i) dzo[i] = 0.0;
#pragma unroll
        for (int i = 0; i < NV; ++i) dno[i] = 0.0;
        if (act) {
            double xi[NX], Cp[NX * NU], Kt[NU * NX], P[NX * NX];
            ldb(Kt, C::B_K, NU * NX);
            ldb(P, C::B_P, NX * NX);
            load_cp(Cp);
            hold(Kt, NU * NX); hold(P, NX * NX);
#pragma unroll
            for (int i = 0; i < NX; ++i) xi[i] = lds[V_CH + t * NX + i];
            double du[NU];
#pragma unroll
            for (int j = 0; j < NU; ++j) {
                double v = v0[j];
#pragma unroll
                for (int k = 0; k < NX; ++k) v = fma(Kt[j * NX + k], xi[k], v);
                du[j] = fixed_u ? 0.0 : v;
            }
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                double dx = xi[i];
#pragma unroll
                for (int j = 0; j < NU; ++j) dx = fma(Cp[j * NX + i], du[j], dx);
                dzo[i] = dx;
                double y = pv[i] + piv[i];
#pragma unroll
                for (int k = 0; k < NX; ++k) y = fma(P[i * NX + k], xi[k], y);
                ym[i] = -y;
            }
#pragma unroll
            for (int j = 0; j < NU; ++j) dzo[NX + j] = du[j];
            if constexpr (C::STF) if (stf_any()) {
                // the stiff facets' multiplier steps nu = Gamma xi + Gamma_kappa mu + gamma0 (no D (g'du - rho): the
                // product of a ~1e12 weight and a cancelling difference)
                double Gm[PMA * NX], Gk[PMA * NX];
                ldb(Gm, C::B_GAM, PM * NX);
                ldb(Gk, C::B_GAK, PM * NX);
                hold(Gm, PM * NX); hold(Gk, PM * NX);
#pragma unroll
                for (int i = 0; i < PM; ++i) {
                    double v = g0[i];
#pragma unroll
                    for (int k = 0; k < NX; ++k) v = fma(Gm[i * NX + k], xi[k], fma(Gk[i * NX + k], mu[k], v));
                    fnu[i] = v;
                }
            }
            if constexpr (NV > 0) {
                // dnu_t = xi_{t+1} - (A xi_t + Bt du_t + e_t)
                double Ad[NX * NX], Bt[NX * NU], ev[NX];
                ldn(Ad, C::C_DT, NX * NX);
                ldn(Bt, C::C_BT, NX * NU);
#pragma unroll
                for (int i = 0; i < NX; ++i) ev[i] = pld(C::gE + i);
                hold(Ad, NX * NX); hold(Bt, NX * NU); hold(ev, NX);
#pragma unroll
                for (int i = 0; i < NX; ++i) {
                    double v = lds[V_CH + (t + 1) * NX + i] - ev[i];
#pragma unroll
                    for (int k = 0; k < NX; ++k) v = fma(-Ad[k * NX + i], xi[k], v);
#pragma unroll
                    for (int j = 0; j < NU; ++j) v = fma(-Bt[i * NU + j], du[j], v);
                    dno[i] = (t < K - 1) ? v : 0.0;
                }
            }
        }
        // lane t computed y_{t-1}: lane t owns y_t (from lane t+1); lane 0's is the initial multiplier
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            const double nxt = __shfl_down(ym[i], 1, WAVE);
            dyo[i] = (t < K - 1) ? nxt : 0.0;
            if (lane == 0) { lds[V_DYI + i] = ym[i]; lds[V_DYF + i] = mu[i]; }
        }
        stamp(9);
    };

    // ------------------------------------------------------------------ node state (workspace)
    // Phase-local register copies: every node phase loads what it uses as one batch and stores
    // what it changes, so no node-sized state is live across the sweeps.
    // soft rows (g0, g1, g2, b) of this node: registers for up to 8 rows; above that (the 16- and 48-row classes,
    // whose node state would not fit the register file next to them) every use re-reads its workspace column
    // (an opaque offset per load: no load is merged with another and kept live across the phase)
    constexpr bool SGS = NS > 8;
    constexpr int NSR = SGS ? 1 : NSA;
    double z[NZ], y[NX], sq[NQ], lq[NQ], av[NGA], ub[NU], sg[NSR][3], sb[NSR];
    auto sgv = [&](int q, int i) __attribute__((always_inline)) -> double {
        if constexpr (SGS) return wb.ld(qp_opaque(vt), (C::C_SOFT + q * 4 + i) * colb);
        else return i < 3 ? sg[q][i] : sb[q];
    };
    // virtual control state of this node (VC classes, lanes t < K-1): nu, e, and per component the slacks /
    // duals of the rows nu - e <= 0 (index 2i) and -nu - e <= 0 (2i + 1)
    double vn[NVA], ve[NVA], vs[2 * NVA], vl[2 * NVA];
    // row slacks s_r and duals lambda_r of this node: LDS [r][lane]
    // (n = 12 classes: workspace columns C_RS / C_RL, C::ROWG)
    auto s_ = [&](int r) __attribute__((always_inline)) -> double {
        if constexpr (C::ROWG) return cld(C::C_RS + r);
        else return lds[V_S + r * WAVE + lane];
    };
    auto l_ = [&](int r) __attribute__((always_inline)) -> double {
        if constexpr (C::ROWG) return cld(C::C_RL + r);
        else return lds[V_L + r * WAVE + lane];
    };
    auto s_set = [&](int r, double v) __attribute__((always_inline)) {
        if constexpr (C::ROWG) cst(C::C_RS + r, v);
        else lds[V_S + r * WAVE + lane] = v;
    };
    auto l_set = [&](int r, double v) __attribute__((always_inline)) {
        if constexpr (C::ROWG) cst(C::C_RL + r, v);
        else lds[V_L + r * WAVE + lane] = v;
    };
    int bidx[NBA];
    auto issue_state = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < NZ; ++i) z[i] = cld(C::C_Z + i);
#pragma unroll
        for (int i = 0; i < NX; ++i) y[i] = cld(C::C_Y + i);
#pragma unroll
        for (int j = 0; j < NQ; ++j) { sq[j] = cld(C::C_SQ + j); lq[j] = cld(C::C_LQ + j); }
#pragma unroll
        for (int g = 0; g < NGA; ++g) av[g] = g < NG ? cld(C::C_AV + g) : 0.0;
#pragma unroll
        for (int j = 0; j < NU; ++j) ub[j] = cld(C::C_UB + j);
#pragma unroll
        for (int q = 0; q < (SGS ? 0 : NS); ++q) {
#pragma unroll
            for (int i = 0; i < 3; ++i) sg[q][i] = cld(C::C_SOFT + q * 4 + i);
            sb[q] = cld(C::C_SOFT + q * 4 + 3);
        }
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            vn[i] = cld(C::C_VN + i);
            ve[i] = cld(C::C_VE + i);
            vs[2 * i] = cld(C::C_VS + 2 * i); vs[2 * i + 1] = cld(C::C_VS + 2 * i + 1);
            vl[2 * i] = cld(C::C_VL + 2 * i); vl[2 * i + 1] = cld(C::C_VL + 2 * i + 1);
        }
    };
    auto hold_state = [&]() __attribute__((always_inline)) {
        hold(z, NZ); hold(y, NX); hold(sq, NQ); hold(lq, NQ); hold(av, NGA); hold(ub, NU);
        if (NV > 0) { hold(vn, NV); hold(ve, NV); hold(vs, 2 * NV); hold(vl, 2 * NV); }
#pragma unroll
        for (int q = 0; q < (SGS ? 0 : NS); ++q) { hold(sg[q], 3); hold(&sb[q], 1); }
#pragma unroll
        for (int b = 0; b < NB; ++b) bidx[b] = qp_opaque(T.box_idx[b]);
    };
    auto load_state = [&]() __attribute__((always_inline)) {
        fresh();
        issue_state();
        hold_state();
    };
    auto store_state = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < NZ; ++i) cst(C::C_Z + i, z[i]);
#pragma unroll
        for (int i = 0; i < NX; ++i) cst(C::C_Y + i, y[i]);
#pragma unroll
        for (int j = 0; j < NQ; ++j) { cst(C::C_SQ + j, sq[j]); cst(C::C_LQ + j, lq[j]); }
#pragma unroll
        for (int g = 0; g < NG; ++g) cst(C::C_AV + g, av[g]);
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            cst(C::C_VN + i, vn[i]);
            cst(C::C_VE + i, ve[i]);
            cst(C::C_VS + 2 * i, vs[2 * i]); cst(C::C_VS + 2 * i + 1, vs[2 * i + 1]);
            cst(C::C_VL + 2 * i, vl[2 * i]); cst(C::C_VL + 2 * i + 1, vl[2 * i + 1]);
        }
    };
    auto grp_on = [&](int g) __attribute__((always_inline)) -> bool { return ineq && (g < NO ? g < nobs : has_coll); };
    auto row_on = [&](int r) __attribute__((always_inline)) -> bool {
        if (r < C::R_BOX) return ineq;
        if (r < C::R_OBS) return ineq && ((r - C::R_BOX) >> 1) < nbox;
        if (r < C::R_COL) return ineq && (r - C::R_OBS) < nobs;
        if (r < C::R_GRP) return (r - C::R_COL) < ccount;
        return grp_on(r - C::R_GRP);
    };
    auto sel_x = [&](const double* zz, int idx) __attribute__((always_inline)) -> double {
        double v = 0.0;
#pragma unroll
        for (int i = 0; i < NX; ++i) v = fma(qp_mask(i, idx), zz[i], v);
        return v;
    };
    // G_r [z; a] and h_r of row r (static after unrolling)
    auto row_eval = [&](int r, const double* zz, const double* aa, double& gz, double& h) __attribute__((always_inline)) {
        if (r < C::R_BOX) {
            gz = 0.0; h = trv;
#pragma unroll
            for (int j = 0; j < NU; ++j) {
                const bool neg = (r >> j) & 1;
                gz += neg ? -zz[NX + j] : zz[NX + j];
                h += neg ? -ub[j] : ub[j];
            }
        } else if (r < C::R_OBS) {
            const int b = (r - C::R_BOX) >> 1, lo = (r - C::R_BOX) & 1;
            const double xi = sel_x(zz, bidx[b]);
            gz = lo ? -xi : xi; h = lo ? -T.box_lo[b] : T.box_hi[b];
        } else if (r < C::R_GRP) {
            const int q = r - C::R_OBS, g = q < NO ? q : NO;
            gz = -(sgv(q, 0) * zz[0] + sgv(q, 1) * zz[1] + sgv(q, 2) * zz[2]) - aa[g];
            h = -sgv(q, 3);
        } else {
            gz = -aa[r - C::R_GRP]; h = 0.0;
        }
    };
    // gzv += c G_r'|_z, gav += c G_r'|_a
    auto row_accT = [&](int r, double c, double* gzv, double* gav) __attribute__((always_inline)) {
        if (r < C::R_BOX) {
#pragma unroll
            for (int j = 0; j < NU; ++j) gzv[NX + j] += ((r >> j) & 1) ? -c : c;
        } else if (r < C::R_OBS) {
            const int b = (r - C::R_BOX) >> 1, lo = (r - C::R_BOX) & 1, idx = bidx[b];
#pragma unroll
            for (int i = 0; i < NX; ++i) gzv[i] = fma(qp_mask(i, idx), lo ? -c : c, gzv[i]);
        } else if (r < C::R_GRP) {
            const int q = r - C::R_OBS, g = q < NO ? q : NO;
#pragma unroll
            for (int i = 0; i < 3; ++i) gzv[i] -= c * sgv(q, i);
            gav[g] -= c;
        } else {
            gav[r - C::R_GRP] -= c;
        }
    };
    // gav += c G_r'|_a (group part only)
    auto row_accA = [&](int r, double c, double* gav) __attribute__((always_inline)) {
        if (r >= C::R_OBS && r < C::R_GRP) {
            const int q = r - C::R_OBS;
            gav[q < NO ? q : NO] -= c;
        } else if (r >= C::R_GRP) {
            gav[r - C::R_GRP] -= c;
        }
    };
    auto gweight = [&](int g) __attribute__((always_inline)) -> double { return (g < NO ? T.w_obs : T.w_coll) * iosc; };

    // Node Hessian (row scaling D_r = l/s or 1, SOC block Wi2uu) -> packet Q, S, R (xi/u
    // coordinates); group elimination factors -> columns C_GRP.  Also writes e = -rp.
    auto assemble = [&](bool unit, const double* Wi2uu, const double* rp) __attribute__((always_inline)) {
        double dbox[NX], Hpp[3][3], Huu[NU * NU], Dfc[C::STF ? C::NTR : 1];
#pragma unroll
        for (int i = 0; i < NX; ++i) dbox[i] = 2.0 * (wfs + wpx);
#pragma unroll
        for (int i = 0; i < 3; ++i) Hpp[i][0] = Hpp[i][1] = Hpp[i][2] = 0.0;
#pragma unroll
        for (int i = 0; i < NU; ++i)
#pragma unroll
            for (int j = 0; j < NU; ++j) Huu[i * NU + j] = (i == j ? 2.0 * wu : 0.0) + (soc ? Wi2uu[i * NU + j] : 0.0);
        double Haa[NGA], Hpa[NGA][3], D0[NGA];
#pragma unroll
        for (int g = 0; g < NGA; ++g) { Haa[g] = 0.0; D0[g] = 0.0; Hpa[g][0] = Hpa[g][1] = Hpa[g][2] = 0.0; }
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const double Dr = row_on(r) ? (unit ? 1.0 : qp_div(l_(r), s_(r))) : 0.0;
            if (r < C::R_BOX) {
                if constexpr (C::STF) {
                    Dfc[r] = Dr;   // folded below, all but the stiff ones
                } else {
#pragma unroll
                    for (int i = 0; i < NU; ++i)
#pragma unroll
                        for (int j = 0; j < NU; ++j) Huu[i * NU + j] += (((r >> i) ^ (r >> j)) & 1) ? -Dr : Dr;
                }
            } else if (r < C::R_OBS) {
                const int idx = bidx[(r - C::R_BOX) >> 1];
#pragma unroll
                for (int i = 0; i < NX; ++i) dbox[i] = fma(qp_mask(i, idx), Dr, dbox[i]);
            } else if (r < C::R_GRP) {
                const int q = r - C::R_OBS, g = q < NO ? q : NO;
                Haa[g] += Dr;
#pragma unroll
                for (int i = 0; i < 3; ++i) Hpa[g][i] += Dr * sgv(q, i);
            } else {
                Haa[r - C::R_GRP] += Dr;
                D0[r - C::R_GRP] = Dr;
            }
        }
        // slack groups eliminated: the position block gains H_pp - H_pa H_aa^-1 H_ap, written as the weighted
        // covariance sum_r D_r (sg_r - hp)(sg_r - hp)' + D_0 hp hp' (hp = H_pa / H_aa, D_0 the slack's sign row):
        // a sum of PSD terms.  The direct difference cancels once an active row's barrier weight dominates
        // (D1 D2 / (D1 + D2) computed as D1 - D1^2 / (D1 + D2)) and broke the factorisation of the C3 agents
        // whose obstacle slack is active at the optimum (oracle/scvx_cpu.cpp node_zz, the same form).
        double hp[NGA][3];
#pragma unroll
        for (int g = 0; g < NGA; ++g) {
            const double ih = (g < NG && grp_on(g)) ? qp_div(1.0, Haa[g]) : 0.0;
#pragma unroll
            for (int i = 0; i < 3; ++i) hp[g][i] = Hpa[g][i] * ih;
            if (g < NG) {
#pragma unroll
                for (int i = 0; i < 3; ++i) cst(C::C_GRP + g * 4 + i, hp[g][i]);
                cst(C::C_GRP + g * 4 + 3, ih);
            }
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) Hpp[i][j] = fma(D0[g] * hp[g][i], hp[g][j], Hpp[i][j]);
        }
#pragma unroll
        for (int r = C::R_OBS; r < C::R_GRP; ++r) {
            const double Dr = row_on(r) ? (unit ? 1.0 : qp_div(l_(r), s_(r))) : 0.0;
            const int q = r - C::R_OBS, g = q < NO ? q : NO;
            double c[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) c[i] = sgv(q, i) - hp[g][i];
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) Hpp[i][j] = fma(Dr * c[i], c[j], Hpp[i][j]);
        }
        if (!act) return;
        // virtual control: nu's curvature after its epigraph variable is eliminated, 4 D1 D2 / (D1 + D2)
        // (D = l/s of the rows nu - e <= 0, -nu - e <= 0; 2 at unit scaling); 1 at the last node (no nu)
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const double d1 = unit ? 1.0 : qp_div(vl[2 * i], vs[2 * i]), d2 = unit ? 1.0 : qp_div(vl[2 * i + 1], vs[2 * i + 1]);
            pst(C::gD + i, vact ? qp_div(4.0 * d1 * d2, d1 + d2) : 1.0);
        }
        double Q[NX * NX], Cp[NX * NU];
        load_cp(Cp);
#pragma unroll
        for (int i = 0; i < NX; ++i)
#pragma unroll
            for (int j = 0; j < NX; ++j) {
                double v = (i == j) ? dbox[i] : 0.0;
                if (i < 3 && j < 3) v += Hpp[i < 3 ? i : 0][j < 3 ? j : 0];
                Q[i * NX + j] = v;
                // global packet: the diagonal and the position block's off-diagonals (every other element is a
                // structural zero: written at setup in the dense form, absent from the compact one, which
                // keeps only the upper triangle)
                if constexpr (C::DPK) {
                    if (i == j || (i < 3 && j < 3)) pst(C::P_Q + i * NX + j, v);
                } else {
                    if (i == j) pst(C::G_QD + i, v);
                    else if (i < j && j < 3) pst(C::G_QO + i + j - 1, v);
                }
            }
        double Sx[NX * NU];
#pragma unroll
        for (int i = 0; i < NX; ++i)
#pragma unroll
            for (int j = 0; j < NU; ++j) {
                double v = 0.0;
#pragma unroll
                for (int k = 0; k < NX; ++k) v = fma(Q[i * NX + k], Cp[j * NX + k], v);
                Sx[i * NU + j] = v;
                pst(C::gS + i * NU + j, v);
            }
        double Ru[NU * NU];
#pragma unroll
        for (int i = 0; i < NU; ++i)
#pragma unroll
            for (int j = i; j < NU; ++j) {
                double v = Huu[i * NU + j];
#pragma unroll
                for (int k = 0; k < NX; ++k) v = fma(Cp[i * NX + k], Sx[k * NU + j], v);
                Ru[i * NU + j] = v;
            }
        if constexpr (C::STF) {
            // the facets' weights, their folded sum sum_f D_f g_f g_f' (the diagonal is sum_f D_f; off-diagonal (i, j) the
            // sum of D_f signed by the parity of facet bits i and j) and their max.  A facet can be stiff in its stage
            // (phase 3: above QP_STIFF x Rhat's largest diagonal) only if it is above QP_STIFF x R's (Rhat = R +
            // Bt'P Bt >= R): the other nodes (nearly all of them) fold their facets into R here and store dfm = 0, so
            // their stages run phase 3 without the facet branch
            double dsum = 0.0, dfm = 0.0, osum[C::NFO > 0 ? C::NFO : 1];
#pragma unroll
            for (int e = 0; e < C::NFO; ++e) osum[e] = 0.0;
#pragma unroll
            for (int f = 0; f < C::NTR; ++f) {
                pst(C::gFD + f, Dfc[f]);
                dsum += Dfc[f];
                dfm = fmax(dfm, Dfc[f]);
                int e = 0;
#pragma unroll
                for (int i = 0; i < NU; ++i)
#pragma unroll
                    for (int j = i + 1; j < NU; ++j, ++e) osum[e] += (((f >> i) ^ (f >> j)) & 1) ? -Dfc[f] : Dfc[f];
            }
            double rdm = 0.0;
#pragma unroll
            for (int i = 0; i < NU; ++i) rdm = fmax(rdm, fabs(Ru[i * NU + i]));
            const bool cand = dfm > QP_STIFF * rdm;
            {
                int e = 0;
#pragma unroll
                for (int i = 0; i < NU; ++i) {
                    Ru[i * NU + i] += cand ? 0.0 : dsum;
#pragma unroll
                    for (int j = i + 1; j < NU; ++j, ++e) Ru[i * NU + j] += cand ? 0.0 : osum[e];
                }
            }
            pst(C::gFD + C::NTR, cand ? dsum : 0.0);
#pragma unroll
            for (int e = 0; e < C::NFO; ++e) pst(C::gFD + C::NTR + 1 + e, cand ? osum[e] : 0.0);
            pst(C::gFD + C::NTR + 1 + C::NFO, cand ? dfm : 0.0);
        }
#pragma unroll
        for (int i = 0; i < NU; ++i)
#pragma unroll
            for (int j = i; j < NU; ++j) {  // upper triangle: packed by rows (compact), both halves (dense)
                const double v = Ru[i * NU + j];
                if constexpr (C::DPK) {
                    pst(C::P_R + i * NU + j, v);
                    if (j > i) pst(C::P_R + j * NU + i, v);
                } else {
                    pst(C::G_R + i * NU - i * (i - 1) / 2 + (j - i), v);
                }
            }
#pragma unroll
        for (int i = 0; i < NX; ++i) pst(C::gE + i, (t < K - 1) ? -rp[i] : 0.0);
    };
    // eliminate the group part of a Newton rhs (stores it for recover_aux): r1_p -= Hpa/Haa r1a;
    // returns the (xi, u) linear terms q, r of the node
    auto reduce_rhs = [&](double* r1, const double* r1a, double* q, double* r) __attribute__((always_inline)) {
        double grp[NGA * 4], Cp[NX * NU];
        ldn(grp, C::C_GRP, NG * 4);
        load_cp(Cp);
        hold(grp, NG * 4);
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            cst(C::C_R1A + g, r1a[g]);
#pragma unroll
            for (int i = 0; i < 3; ++i) r1[i] -= grp[g * 4 + i] * r1a[g];
        }
        if (fixed_u) {
#pragma unroll
            for (int j = 0; j < NU; ++j) r1[NX + j] = 0.0;
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) q[i] = -r1[i];
#pragma unroll
        for (int j = 0; j < NU; ++j) {
            double v = r1[NX + j];
#pragma unroll
            for (int k = 0; k < NX; ++k) v = fma(Cp[j * NX + k], r1[k], v);
            r[j] = fixed_u ? 0.0 : -v;
        }
    };
    // group directions: da_g = (r1a_g - Hpa_g' dp) / Haa_g
    auto recover_aux = [&](const double* dzl, double* da) __attribute__((always_inline)) {
        double grp[NGA * 4], r1a[NGA];
        ldn(grp, C::C_GRP, NG * 4);
        ldn(r1a, C::C_R1A, NG);
        hold(grp, NG * 4);
        hold(r1a, NG);
#pragma unroll
        for (int g = 0; g < NGA; ++g) da[g] = 0.0;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            double v = r1a[g] * grp[g * 4 + 3];
#pragma unroll
            for (int i = 0; i < 3; ++i) v -= grp[g * 4 + i] * dzl[i];
            da[g] = grp_on(g) ? v : 0.0;
        }
    };
    auto set_boundary = [&](const double* zz) __attribute__((always_inline)) {
        // lane 0 holds z_0, lane K-1 holds z_{K-1}
        if (t == 0) {
#pragma unroll
            for (int i = 0; i < NX; ++i) lds[V_XI0 + i] = a.x_init[agent * NX + i] - zz[i];
        }
        if (t == K - 1) {
#pragma unroll
            for (int i = 0; i < NX; ++i) lds[V_R2F + i] = fin ? a.x_final[agent * NX + i] - zz[i] : 0.0;
        }
    };
    // dynamics residual rp_t = x_{t+1} - A x_t - B u_t - C u_{t+1} - S sigma - z  (lane t < K-1)
    // (dt: this node's transposed disc row, batch-loaded by the caller)
    // (dt(e): element e of the row -- a register copy, or for n = 12 a load per use)
    auto dyn_residual = [&](const double* zz, auto dt, double* rp) __attribute__((always_inline)) {
        double zn[NZ];
#pragma unroll
        for (int i = 0; i < NZ; ++i) zn[i] = __shfl_down(zz[i], 1, WAVE);
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            double v = zn[i] - fma(dt(NX * NX + 2 * NX * NU + i), sig, dt(NX * NX + 2 * NX * NU + NX + i));
#pragma unroll
            for (int k = 0; k < NX; ++k) v -= dt(k * NX + i) * zz[k];
#pragma unroll
            for (int j = 0; j < NU; ++j)
                v -= dt(NX * NX + j * NX + i) * zz[NX + j] + dt(NX * NX + NX * NU + j * NX + i) * zn[NX + j];
            rp[i] = (t < K - 1) ? v : 0.0;
        }
    };
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
    // NT scaling W = eta [[w0, w1'], [w1, I + w1 w1'/(1 + w0)]], W^-1 the same with -w1, 1/eta
    auto w_apply = [&](const double* w, double eta, bool inv, const double* x, double* yv) __attribute__((always_inline)) {
        const double sgn = inv ? -1.0 : 1.0, sc = inv ? qp_div(1.0, eta) : eta;
        double d = 0.0;
#pragma unroll
        for (int j = 1; j < NQ; ++j) d += w[j] * x[j];
        d *= sgn;
        yv[0] = sc * (w[0] * x[0] + d);
        const double f = x[0] + qp_div(d, 1.0 + w[0]);
#pragma unroll
        for (int j = 1; j < NQ; ++j) yv[j] = sc * (x[j] + sgn * w[j] * f);
    };
    // SOC scaling of the iteration (columns C_WV..C_RHO)
    double wv[NQ], eta = 1.0, ltq[NQ], rcq[NQ];
    auto issue_soc = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < NQ; ++j) { wv[j] = cld(C::C_WV + j); ltq[j] = cld(C::C_LTQ + j); rcq[j] = cld(C::C_RCQ + j); }
        eta = cld(C::C_ETA);
    };
    auto hold_soc = [&]() __attribute__((always_inline)) { hold(wv, NQ); hold(ltq, NQ); hold(rcq, NQ); hold(&eta, 1); };
    auto load_soc = [&]() __attribute__((always_inline)) {
        fresh();
        issue_soc();
        hold_soc();
    };

    int status = SCVX_STATUS_MAX_ITER;
    int it = 0;
    double fail_code = 0.0;
    // ------------------------------------------------------------------ starting point
    if (warm) {
        // warm start (the Jacobi SCvx loop re-solves each agent's subproblem re-linearised at its own last
        // solution): z, y, the group and SOC duals and the row duals are the last iterate's; the slacks are
        // recomputed from this solve's rows at z; every slack and dual is floored at QP_WARM_ETA inside its
        // cone, a row's dual at min(QP_WARM_ETA, QP_WARM_KAPPA / s) (oracle/scvx_cpu.cpp warm_point does the same).
        // C3: 12.3 -> ~5 IPM iterations on average.
        load_state();
        double wl[NR];
        ldn(wl, C::C_WL, NR);
        hold(wl, NR);
        // the slack-relative dual floor, except in the classes with the stiff-facet stage system (the coupled double /
        // single integrators: there it lengthened the C4 tail; the twin the same)
        const bool kfl = !(C::STF && has_coll);
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            double gz, h;
            row_eval(r, z, av, gz, h);
            const bool on = row_on(r);
            const double sr = fmax(h - gz, QP_WARM_ETA);
            s_set(r, on ? sr : 1.0);
            l_set(r, on ? fmax(wl[r], kfl ? fmin(QP_WARM_ETA, QP_WARM_KAPPA / sr) : QP_WARM_ETA) : 0.0);
        }
        if (soc) {
            double nu2 = 0.0, nl2 = 0.0;
            sq[0] = T.u_max;
#pragma unroll
            for (int j = 0; j < NU; ++j) { sq[1 + j] = z[NX + j]; nu2 += z[NX + j] * z[NX + j]; nl2 += lq[1 + j] * lq[1 + j]; }
            sq[0] = fmax(sq[0], sqrt(nu2) + QP_WARM_ETA);
            lq[0] = fmax(lq[0], sqrt(nl2) + QP_WARM_ETA);
        } else {
#pragma unroll
            for (int j = 0; j < NQ; ++j) { sq[j] = 0.0; lq[j] = 0.0; }
        }
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            vs[2 * i] = vact ? fmax(ve[i] - vn[i], QP_WARM_ETA) : 1.0;
            vs[2 * i + 1] = vact ? fmax(ve[i] + vn[i], QP_WARM_ETA) : 1.0;
            vl[2 * i] = vact ? fmax(vl[2 * i], fmin(QP_WARM_ETA, QP_WARM_KAPPA / vs[2 * i])) : 0.0;
            vl[2 * i + 1] = vact ? fmax(vl[2 * i + 1], fmin(QP_WARM_ETA, QP_WARM_KAPPA / vs[2 * i + 1])) : 0.0;
        }
        store_state();
    } else {
    // minimiser of 1/2 z'Pz + q'z + 1/2 ||Gz - h||^2 s.t. Az = b from z_ref (aux = 0), unit scaling
    // (CVXOPT coneqp initialisation; oracle/qp_dense.py does the same on the dense form)
        fresh();
        constexpr bool DSTRM = NX > 8;   // n = 12: the 264-double disc row is read per use, not held
        double dt[DSTRM ? 1 : C::DSTR];
        issue_state();
        if constexpr (!DSTRM) ldn(dt, C::C_DT, C::DSTR);
        hold_state();
        if constexpr (!DSTRM) hold(dt, C::DSTR);
#pragma unroll
        for (int r = 0; r < NR; ++r) { s_set(r, 1.0); l_set(r, 0.0); }
        double Wu[NU * NU], rp[NX];
#pragma unroll
        for (int e = 0; e < NU * NU; ++e) Wu[e] = (e / NU == e % NU) ? 1.0 : 0.0;
        dyn_residual(z, [&](int e) __attribute__((always_inline)) -> double {
            if constexpr (DSTRM) return wb.ld(qp_opaque(vt), (C::C_DT + e) * colb);
            else return dt[e];
        }, rp);
        assemble(true, Wu, rp);
        double r1[NZ], r1a[NGA];
#pragma unroll
        for (int i = 0; i < NX; ++i) r1[i] = tsoft ? -2.0 * wfs * (z[i] - a.x_final[agent * NX + i]) : 0.0;
#pragma unroll
        for (int j = 0; j < NU; ++j) r1[NX + j] = -2.0 * wu * z[NX + j] - (soc ? z[NX + j] : 0.0);
#pragma unroll
        for (int g = 0; g < NGA; ++g) r1a[g] = -gweight(g);
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            double gz, h;
            row_eval(r, z, av, gz, h);
            if (row_on(r)) row_accT(r, -(gz - h), r1, r1a);
        }
        double q[NX], rr[NU];
        reduce_rhs(r1, r1a, q, rr);
        set_boundary(z);
        if (!factor()) { status = SCVX_STATUS_NUMERICAL; fail_code = 1.0; }
        __syncthreads();  // factor columns (global) -> lane-parallel solve passes
        double dz[NZ], dy[NX], da[NGA], dv0[NVA], dnv[NVA], rs0[C::PMA], fn0[C::PMA];
        // virtual control at unit scaling from nu = e = 0: nu's rhs is 0 (the two rows cancel), e's is -w_nu
#pragma unroll
        for (int i = 0; i < NVA; ++i) dv0[i] = 0.0;
        // (unit scaling: every facet folds, D = 1 is never stiff next to Rhat)
#pragma unroll
        for (int i = 0; i < C::PMA; ++i) rs0[i] = 0.0;
        solve(q, rr, dv0, dz, dy, dnv, rs0, fn0);
        recover_aux(dz, da);
        load_state();
#pragma unroll
        for (int i = 0; i < NZ; ++i) z[i] += act ? dz[i] : 0.0;
#pragma unroll
        for (int g = 0; g < NGA; ++g) av[g] += da[g];
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            vn[i] = vact ? dnv[i] : 0.0;
            ve[i] = vact ? -0.5 * wnu : 0.0;   // (r_e - b dnu) / a with a = 2, b = 0
        }
        double smin = 1e300, lmin = 1e300;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            double gz, h;
            row_eval(r, z, av, gz, h);
            const bool on = row_on(r);
            s_set(r, on ? h - gz : 1.0);
            l_set(r, on ? gz - h : 0.0);
            if (on) { smin = fmin(smin, h - gz); lmin = fmin(lmin, gz - h); }
        }
#pragma unroll
        for (int j = 0; j < NQ; ++j) { sq[j] = 0.0; lq[j] = 0.0; }
        if (soc) {
            double nu2 = 0.0;
            sq[0] = T.u_max; lq[0] = -T.u_max;
#pragma unroll
            for (int j = 0; j < NU; ++j) { sq[1 + j] = z[NX + j]; lq[1 + j] = -z[NX + j]; nu2 += z[NX + j] * z[NX + j]; }
            smin = fmin(smin, T.u_max - sqrt(nu2));
            lmin = fmin(lmin, -T.u_max - sqrt(nu2));
        }
#pragma unroll
        for (int i = 0; i < NV; ++i) {   // s = h - Gz, lambda = Gz - h of the rows nu - e <= 0, -nu - e <= 0
            vs[2 * i] = ve[i] - vn[i]; vl[2 * i] = vn[i] - ve[i];
            vs[2 * i + 1] = ve[i] + vn[i]; vl[2 * i + 1] = -vn[i] - ve[i];
            if (vact) {
                smin = fmin(smin, fmin(vs[2 * i], vs[2 * i + 1]));
                lmin = fmin(lmin, fmin(vl[2 * i], vl[2 * i + 1]));
            }
        }
        smin = wave_min(smin); lmin = wave_min(lmin);
        const double shs = fmax(0.0, 1.0 - smin), shl = fmax(0.0, 1.0 - lmin);
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            if (row_on(r)) { s_set(r, s_(r) + shs); l_set(r, l_(r) + shl); }
        }
        if (soc) { sq[0] += shs; lq[0] += shl; }
#pragma unroll
        for (int i = 0; i < 2 * NV; ++i) { vs[i] = vact ? vs[i] + shs : 1.0; vl[i] = vact ? vl[i] + shl : 0.0; }
        store_state();
    }
    double degl = 0.0;
#pragma unroll
    for (int r = 0; r < NR; ++r) degl += row_on(r) ? 1.0 : 0.0;
    degl += soc ? 1.0 : 0.0;
    degl += vact ? 2.0 * NV : 0.0;
    const double deg = fmax(wave_sum(degl), 1.0);
    const double tol = T.tol > 0 ? T.tol : 1e-9;

    // ------------------------------------------------------------------ IPM iterations
    const long long cyc_all0 = __builtin_amdgcn_s_memtime();
    double dres_best = 1e300, pres_best = 1e300;
    stamp(-1);
    // the residuals are evaluated once more after the last step: an iterate that reaches the
    // iteration cap is reported `optimal_inaccurate` only if it meets the reduced tolerances below,
    // otherwise `solver_error` (ECOS / Clarabel report a cap far from optimal as a failure too)
    for (it = 0; status != SCVX_STATUS_NUMERICAL; ++it) {
        // The disc row is consumed in two register chunks (A | S z, then B | C), so the whole row (DSTR
        // doubles) is never live next to the iterate: that peak made the C3 class spill.  The second
        // chunk's loads are issued once the first chunk is dead (one extra round trip per iteration).
        fresh();
        // n = 12 classes: A (NX^2 = 144 doubles) is not held in registers; it is read one column at a time
        // (below, once the multiplier terms of rd are in), in the same summation order
        constexpr bool ASTR = NX > 8;
        double Cpr[NX * NU], dA[ASTR ? 1 : NX * NX], dSz[2 * NX];
        issue_state();
        if constexpr (!ASTR) ldn(dA, C::C_DT, NX * NX);
        ldn(dSz, C::C_DT + NX * NX + 2 * NX * NU, 2 * NX);
        load_cp(Cpr);
        hold_state();
        if constexpr (!ASTR) hold(dA, NX * NX);
        hold(dSz, 2 * NX);
        double zn[NZ];
#pragma unroll
        for (int i = 0; i < NZ; ++i) zn[i] = __shfl_down(z[i], 1, WAVE);
        // rp_t = x_{t+1} - A x_t - B u_t - C u_{t+1} - S sigma - z (lane t < K-1), the dyn_residual order
        double rp[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            double v = zn[i] - fma(dSz[i], sig, dSz[NX + i]);
            if constexpr (!ASTR) {
#pragma unroll
                for (int k = 0; k < NX; ++k) v -= dA[k * NX + i] * z[k];
            }
            rp[i] = v;
        }
        // dual residual rd = Pz + q + A'y + G'lam (z and group parts)
        double rd[NZ], rda[NGA];
        // residual norms and Clarabel's normalisation of them (the solver dist_scvx_3d.py:110 calls):
        // primal ||r_p|| <= tol max(1, ||b|| + ||x|| + ||s||), dual ||r_d|| <= tol max(1, ||q|| + ||x|| + ||z||)
        // (inf-norms; b = every constant of the equality and inequality rows, x = primal variables,
        // s = slacks, z = every multiplier: rows, cone, dynamics, boundary conditions)
        double pres = 0.0, dres = 0.0, gap = 0.0, nb = 0.0, nxv = 0.0, nsl = 0.0, nzd = 0.0, pobj = 0.0;
        if (t < K - 1) {
#pragma unroll
            for (int i = 0; i < NX; ++i) nb = fmax(nb, fabs(fma(dSz[i], sig, dSz[NX + i])));
        }
        if (act) {
#pragma unroll
            for (int i = 0; i < NZ; ++i) nxv = fmax(nxv, fabs(z[i]));
#pragma unroll
            for (int g = 0; g < NG; ++g) nxv = fmax(nxv, grp_on(g) ? fabs(av[g]) : 0.0);
            if (t < K - 1) {
#pragma unroll
                for (int i = 0; i < NX; ++i) nzd = fmax(nzd, fabs(y[i]));
            }
        }
        if (lane < NX) nzd = fmax(nzd, fmax(fabs(lds[V_YI + lane]), fin ? fabs(lds[V_YF + lane]) : 0.0));
        if (t == 0) {
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                pres = fmax(pres, fabs(z[i] - a.x_init[agent * NX + i]));
                nb = fmax(nb, fabs(a.x_init[agent * NX + i]));
            }
        }
        if (act && t == K - 1 && fin) {
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                pres = fmax(pres, fabs(z[i] - a.x_final[agent * NX + i]));
                nb = fmax(nb, fabs(a.x_final[agent * NX + i]));
            }
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            rd[i] = tsoft ? 2.0 * wfs * (z[i] - a.x_final[agent * NX + i]) : 0.0;
            if (prox) rd[i] = fma(2.0 * wpx, z[i] - a.Xref[(agent * K + (act ? t : 0)) * NX + i], rd[i]);
        }
#pragma unroll
        for (int j = 0; j < NU; ++j) rd[NX + j] = 2.0 * wu * z[NX + j];
#pragma unroll
        for (int g = 0; g < NGA; ++g) rda[g] = gweight(g);
        {
            // dynamics and boundary multipliers first (y_{t-1} from lane t-1), so that the disc row and
            // C_{t-1} are dead before the row loop (register pressure of the residual phase)
            double ym[NX];
#pragma unroll
            for (int i = 0; i < NX; ++i) ym[i] = __shfl_up(y[i], 1, WAVE);
            if (act) {
                if (t == 0) {
#pragma unroll
                    for (int i = 0; i < NX; ++i) rd[i] += lds[V_YI + i];
                }
                if (t == K - 1 && fin) {
#pragma unroll
                    for (int i = 0; i < NX; ++i) rd[i] += lds[V_YF + i];
                }
                if (t >= 1) {
#pragma unroll
                    for (int i = 0; i < NX; ++i) rd[i] += ym[i];
#pragma unroll
                    for (int j = 0; j < NU; ++j)
#pragma unroll
                        for (int i = 0; i < NX; ++i) rd[NX + j] -= Cpr[j * NX + i] * ym[i];
                }
                if (t < K - 1 && !ASTR) {
#pragma unroll
                    for (int k = 0; k < NX; ++k)
#pragma unroll
                        for (int i = 0; i < NX; ++i) rd[k] -= dA[k * NX + i] * y[i];
                }
            }
            if constexpr (ASTR) {   // column k of A: rp -= A(:, k) x_k, rd_k -= A(:, k)' y (orders as above)
                const bool ay = act && t < K - 1;
#pragma unroll
                for (int k = 0; k < NX; ++k) {
                    double col[NX];
                    const int vo = qp_opaque(vt);
#pragma unroll
                    for (int i = 0; i < NX; ++i) col[i] = wb.ld(vo, (C::C_DT + k * NX + i) * colb);
#pragma unroll
                    for (int i = 0; i < NX; ++i) rp[i] -= col[i] * z[k];
#pragma unroll
                    for (int i = 0; i < NX; ++i) rd[k] -= ay ? col[i] * y[i] : 0.0;
                }
            }
        }
        {   // second chunk: B | C
            double dBC[2 * NX * NU];
            ldn(dBC, C::C_DT + NX * NX, 2 * NX * NU);
            hold(dBC, 2 * NX * NU);
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                double v = rp[i];
#pragma unroll
                for (int j = 0; j < NU; ++j) v -= dBC[j * NX + i] * z[NX + j] + dBC[NX * NU + j * NX + i] * zn[NX + j];
                rp[i] = (t < K - 1) ? v : 0.0;
            }
            if (act && t < K - 1) {
#pragma unroll
                for (int j = 0; j < NU; ++j)
#pragma unroll
                    for (int i = 0; i < NX; ++i) rd[NX + j] -= dBC[j * NX + i] * y[i];
            }
        }
#pragma unroll
        for (int i = 0; i < NV; ++i) rp[i] -= vact ? vn[i] : 0.0;   // + nu_t in the dynamics
#pragma unroll
        for (int i = 0; i < NX; ++i) pres = fmax(pres, fabs(rp[i]));
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            double gz, h;
            row_eval(r, z, av, gz, h);
            if (row_on(r)) {
                const double rcr = gz + s_(r) - h;
                pres = fmax(pres, fabs(rcr));
                nb = fmax(nb, fabs(h));
                nsl = fmax(nsl, s_(r));
                nzd = fmax(nzd, l_(r));
                gap += s_(r) * l_(r);
                row_accT(r, l_(r), rd, rda);
            }
        }
        if (soc) {
            rcq[0] = sq[0] - T.u_max;
#pragma unroll
            for (int j = 0; j < NU; ++j) { rcq[1 + j] = sq[1 + j] - z[NX + j]; rd[NX + j] -= lq[1 + j]; }
#pragma unroll
            for (int j = 0; j < NQ; ++j) {
                pres = fmax(pres, fabs(rcq[j]));
                gap += sq[j] * lq[j];
                nsl = fmax(nsl, fabs(sq[j]));
                nzd = fmax(nzd, fabs(lq[j]));
            }
            nb = fmax(nb, T.u_max);
        } else {
#pragma unroll
            for (int j = 0; j < NQ; ++j) rcq[j] = 0.0;
        }
        {
            if (act) {
                if (fixed_u) {
#pragma unroll
                    for (int j = 0; j < NU; ++j) rd[NX + j] = 0.0;
                }
#pragma unroll
                for (int i = 0; i < NZ; ++i) { dres = fmax(dres, fabs(rd[i])); cst(C::C_RD + i, rd[i]); }
                if (vact) {   // virtual control rows nu - e + s1 = 0, -nu - e + s2 = 0; rd = (-y + l1 - l2, w_nu - l1 - l2)
#pragma unroll
                    for (int i = 0; i < NV; ++i) {
                        const double rc1 = vn[i] - ve[i] + vs[2 * i], rc2 = -vn[i] - ve[i] + vs[2 * i + 1];
                        pres = fmax(pres, fmax(fabs(rc1), fabs(rc2)));
                        nsl = fmax(nsl, fmax(vs[2 * i], vs[2 * i + 1]));
                        nzd = fmax(nzd, fmax(vl[2 * i], vl[2 * i + 1]));
                        nxv = fmax(nxv, fmax(fabs(vn[i]), fabs(ve[i])));
                        gap += vs[2 * i] * vl[2 * i] + vs[2 * i + 1] * vl[2 * i + 1];
                        const double rdn = -y[i] + vl[2 * i] - vl[2 * i + 1], rde = wnu - vl[2 * i] - vl[2 * i + 1];
                        dres = fmax(dres, fmax(fabs(rdn), fabs(rde)));
                        cst(C::C_VRD + 2 * i, rdn);
                        cst(C::C_VRD + 2 * i + 1, rde);
                        pobj += wnu * ve[i];
                    }
                }
                if (prox) {   // w_prox ||x - xbar||^2 without its constant (as the soft terminal)
#pragma unroll
                    for (int i = 0; i < NX; ++i) pobj += wpx * z[i] * (z[i] - 2.0 * a.Xref[(agent * K + t) * NX + i]);
                }
#pragma unroll
                for (int g = 0; g < NG; ++g) {
                    if (grp_on(g)) { dres = fmax(dres, fabs(rda[g])); pobj += gweight(g) * av[g]; }
                }
#pragma unroll
                for (int j = 0; j < NU; ++j) pobj += wu * z[NX + j] * z[NX + j];
                if (tsoft) {  // the objective without its constant w_final ||x_final||^2 (Clarabel's)
#pragma unroll
                    for (int i = 0; i < NX; ++i) pobj += wfs * z[i] * (z[i] - 2.0 * a.x_final[agent * NX + i]);
                }
            }
        }
        pres = wave_max(pres); dres = wave_max(dres);
        nb = wave_max(nb); nxv = wave_max(nxv); nsl = wave_max(nsl); nzd = wave_max(nzd);
        gap = wave_sum(gap); pobj = wave_sum(pobj) + cpx;
        const double pnorm = fmax(1.0, nb + nxv + nsl), dnorm = fmax(iosc, (qnorm + nxv) * iosc + nzd);  // caller's units / osc
        const double mu = gap / deg;
        if (!isfinite(pres + dres + mu)) { status = SCVX_STATUS_NUMERICAL; fail_code = 3.0; break; }
        if (pres <= tol * pnorm && dres <= tol * dnorm && gap * osc <= tol * fmax(1.0, fabs(pobj * osc))) {
            status = SCVX_STATUS_OPTIMAL;
            break;
        }
        // reduced accuracy ("optimal_inaccurate"): what a numerical breakdown below leaves is still
        // usable if it meets the reduced tolerances of the reference's solvers (Clarabel / ECOS:
        // feasibility 1e-4, gap 5e-5 relative)
        const bool near = pres <= 1e-4 * pnorm && dres <= 1e-4 * dnorm && gap * osc <= 5e-5 * fmax(1.0, fabs(pobj * osc));
        if (it >= T.max_iter) {
            status = near ? SCVX_STATUS_MAX_ITER : SCVX_STATUS_NUMERICAL;
            fail_code = 5.0;
            break;
        }
        // insufficient progress (Clarabel's rule): a residual that jumps by 100x once the reduced
        // tolerances hold is the Newton system losing its accuracy at extreme barrier scalings;
        // stop at reduced accuracy instead of wandering on a corrupted direction
        if (near && (dres > fmax(100.0 * dres_best, tol * dnorm) || pres > fmax(100.0 * pres_best, tol * pnorm))) {
            status = SCVX_STATUS_MAX_ITER;
            fail_code = 7.0;
            break;
        }
        dres_best = fmin(dres_best, dres);
        pres_best = fmin(pres_best, pres);
        // diagnostics trace, residual part (written here so these values die before the direction phases)
        if (a.trace && agent == a.trace_agent && lane == 0 && it < a.trace_cap) {
            double* tr_ = a.trace + 8 * it;
            tr_[0] = pres; tr_[1] = dres; tr_[2] = gap; tr_[3] = pobj * osc; tr_[7] = mu;
        }
        // SOC Nesterov-Todd scaling (hyperbolic-rotation form, W lam = W^-1 s)
        double Wi2uu[NU * NU];
#pragma unroll
        for (int j = 0; j < NQ; ++j) { wv[j] = 0.0; ltq[j] = 0.0; }
        eta = 1.0;
#pragma unroll
        for (int e = 0; e < NU * NU; ++e) Wi2uu[e] = 0.0;
        if (soc) {
            double n1s = 0.0, n1z = 0.0;
#pragma unroll
            for (int j = 1; j < NQ; ++j) { n1s += sq[j] * sq[j]; n1z += lq[j] * lq[j]; }
            n1s = sqrt(n1s); n1z = sqrt(n1z);
            const double Js = fmax((sq[0] - n1s) * (sq[0] + n1s), 1e-300), Jz = fmax((lq[0] - n1z) * (lq[0] + n1z), 1e-300);
            const double ns = sqrt(Js), nz = sqrt(Jz);
            double sbv[NQ], zbv[NQ], dot = 0.0;
#pragma unroll
            for (int j = 0; j < NQ; ++j) { sbv[j] = qp_div(sq[j], ns); zbv[j] = qp_div(lq[j], nz); dot += sbv[j] * zbv[j]; }
            const double gam = sqrt((1.0 + dot) / 2.0);
#pragma unroll
            for (int j = 0; j < NQ; ++j) wv[j] = qp_div(sbv[j] + (j == 0 ? zbv[j] : -zbv[j]), 2.0 * gam);
            eta = sqrt(sqrt(qp_div(Js, Jz)));
            w_apply(wv, eta, false, lq, ltq);
            // (W^-2)_uu = rows/cols 1.. of W^-1 W^-1
            double Wi[NQ * NQ];
#pragma unroll
            for (int c = 0; c < NQ; ++c) {
                double ec[NQ], col[NQ];
#pragma unroll
                for (int j = 0; j < NQ; ++j) ec[j] = (j == c) ? 1.0 : 0.0;
                w_apply(wv, eta, true, ec, col);
#pragma unroll
                for (int j = 0; j < NQ; ++j) Wi[j * NQ + c] = col[j];
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
        }
#pragma unroll
        for (int j = 0; j < NQ; ++j) { cst(C::C_WV + j, wv[j]); cst(C::C_LTQ + j, ltq[j]); cst(C::C_RCQ + j, rcq[j]); }
        cst(C::C_ETA, eta);
        assemble(false, Wi2uu, rp);
        set_boundary(z);
        stamp(0);
        if (!factor()) { status = near ? SCVX_STATUS_MAX_ITER : SCVX_STATUS_NUMERICAL; fail_code = lds[V_FLAG]; break; }
        stamp(1);

        // complementarity rhs of row r: predictor -s l ; corrector -s l - ds_a dl_a + sigma mu
        double sgmu = 0.0;
        double dz[NZ], dy[NX], da[NGA], dsq[NQ], dlq[NQ], cpv[NR];
        double dnv[NVA], dne[NVA], vcpv[2 * NVA];   // virtual control directions, predictor products
        // stiff facets of this node's stage (C::STF): their indices (-1: empty slot) and multiplier steps
        double sfr[C::PMA], fnu[C::PMA];
#pragma unroll
        for (int i = 0; i < C::PMA; ++i) { sfr[i] = -1.0; fnu[i] = 0.0; }
        auto rco_of = [&](int r, bool corr) __attribute__((always_inline)) -> double {
            const double v = -s_(r) * l_(r);
            return corr ? v - cpv[r] + sgmu : v;
        };
        // virtual control rows of component i: complementarity rhs (rows 2i, 2i+1) and the directions
        auto vrco = [&](int r, bool corr) __attribute__((always_inline)) -> double {
            const double v = -vs[r] * vl[r];
            return corr ? v - vcpv[r] + sgmu : v;
        };
        auto vrow_dir = [&](int i, bool corr, double* dsr, double* dlr) __attribute__((always_inline)) {
            const double g1 = dnv[i] - dne[i], g2 = -dnv[i] - dne[i];
            const double rc1 = vn[i] - ve[i] + vs[2 * i], rc2 = -vn[i] - ve[i] + vs[2 * i + 1];
            dsr[0] = -rc1 - g1;
            dlr[0] = qp_div(vrco(2 * i, corr) + vl[2 * i] * (rc1 + g1), vs[2 * i]);
            dsr[1] = -rc2 - g2;
            dlr[1] = qp_div(vrco(2 * i + 1, corr) + vl[2 * i + 1] * (rc2 + g2), vs[2 * i + 1]);
        };
        // Newton direction for the complementarity rhs (rows: rco_of, SOC: rcq2); directions out
        auto newton = [&](bool corr, const double* rcq2) __attribute__((always_inline)) {
            double r1[NZ], r1a[NGA], rho[NQ];
            fresh();
            issue_state();
            issue_soc();
            ldn(r1, C::C_RD, NZ);
            if (corr) ldn(cpv, C::C_CP, NR);
            const bool sany = C::STF && stf_any();   // uniform: a stage of this factor kept a stiff facet
            if constexpr (C::STF) if (sany) ldb(sfr, C::B_SF, C::PM);
            hold_state();
            hold_soc();
            hold(r1, NZ);
            if (corr) hold(cpv, NR);
            if constexpr (C::STF) if (sany) hold(sfr, C::PM);
            double rhs_s[C::PMA];
#pragma unroll
            for (int i = 0; i < C::PMA; ++i) rhs_s[i] = 0.0;
#pragma unroll
            for (int i = 0; i < NZ; ++i) r1[i] = act ? -r1[i] : 0.0;
#pragma unroll
            for (int r = 0; r < NR; ++r) cpv[r] = corr ? cpv[r] : 0.0;
#pragma unroll
            for (int g = 0; g < NGA; ++g) r1a[g] = -gweight(g);
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                if (row_on(r)) {
                    double gz, h;
                    row_eval(r, z, av, gz, h);
                    const double rcr = gz + s_(r) - h;
                    row_accA(r, -l_(r), r1a);  // -rd, group part: -(w_g - sum lambda)
                    double c = -qp_div(rco_of(r, corr) + l_(r) * rcr, s_(r));
                    if constexpr (C::STF) {
                        if (r < C::R_BOX) {   // a stiff facet: its rho = -(rco / l + rc) goes to the stage system
                            const double rho_f = -(rco_of(r, corr) / l_(r) + rcr);
                            bool st = false;
#pragma unroll
                            for (int i = 0; i < C::PM; ++i) {
                                const bool m_ = sfr[i] == (double)r;
                                rhs_s[i] = m_ ? rho_f : rhs_s[i];
                                st |= m_;
                            }
                            c = st ? 0.0 : c;
                        }
                    }
                    row_accT(r, c, r1, r1a);
                }
            }
#pragma unroll
            for (int j = 0; j < NQ; ++j) rho[j] = 0.0;
            if (soc) {
                // rho = ltq o^-1 rcq2 ; u part of G'(W^-1 rho + W^-2 rcq) = -(...)[1:]
                double J = ltq[0] * ltq[0], r0 = ltq[0] * rcq2[0], w2[NQ], w3[NQ];
#pragma unroll
                for (int j = 1; j < NQ; ++j) { J -= ltq[j] * ltq[j]; r0 -= ltq[j] * rcq2[j]; }
                r0 = qp_div(r0, J);
                rho[0] = r0;
#pragma unroll
                for (int j = 1; j < NQ; ++j) rho[j] = qp_div(rcq2[j] - r0 * ltq[j], ltq[0]);
                w_apply(wv, eta, true, rcq, w2);
#pragma unroll
                for (int j = 0; j < NQ; ++j) w2[j] += rho[j];
                w_apply(wv, eta, true, w2, w3);
#pragma unroll
                for (int i = 0; i < NU; ++i) r1[NX + i] += w3[1 + i];
            }
#pragma unroll
            for (int j = 0; j < NQ; ++j) cst(C::C_RHO + j, rho[j]);
            double q[NX], rr[NU], dvl[NVA];
            reduce_rhs(r1, r1a, q, rr);
#pragma unroll
            for (int i = 0; i < NVA; ++i) dvl[i] = 0.0;
            if constexpr (NV > 0) {
                // rhs of (nu_i, e_i): -rd - sum_r G_r' (rco_r + l_r rc_r) / s_r, then e_i eliminated:
                // nu's linear term -(r_nu - b/a r_e), a = D1 + D2, b = D2 - D1 (r_e kept for the recovery)
                double vrd[2 * NV];
                ldn(vrd, C::C_VRD, 2 * NV);
                if (corr) ldn(vcpv, C::C_VCP, 2 * NV);
                hold(vrd, 2 * NV);
                if (corr) hold(vcpv, 2 * NV);
#pragma unroll
                for (int i = 0; i < NV; ++i) {
                    const double rc1 = vn[i] - ve[i] + vs[2 * i], rc2 = -vn[i] - ve[i] + vs[2 * i + 1];
                    const double c1 = -qp_div(vrco(2 * i, corr) + vl[2 * i] * rc1, vs[2 * i]);
                    const double c2 = -qp_div(vrco(2 * i + 1, corr) + vl[2 * i + 1] * rc2, vs[2 * i + 1]);
                    const double rn = -vrd[2 * i] + c1 - c2, re = -vrd[2 * i + 1] - c1 - c2;
                    const double d1 = qp_div(vl[2 * i], vs[2 * i]), d2 = qp_div(vl[2 * i + 1], vs[2 * i + 1]);
                    dvl[i] = vact ? -(rn - qp_div(d2 - d1, d1 + d2) * re) : 0.0;
                    cst(C::C_VRE + i, re);
                }
            }
            stamp(2);
            solve(q, rr, dvl, dz, dy, dnv, rhs_s, fnu);
            // post-solve: group and SOC directions (state reloaded: nothing crossed the sweeps)
            fresh();
            issue_state();
            issue_soc();
            if (corr) ldn(cpv, C::C_CP, NR);
            ldn(rho, C::C_RHO, NQ);
            hold_state();
            hold_soc();
            if (corr) hold(cpv, NR);
            hold(rho, NQ);
            recover_aux(dz, da);
            if constexpr (NV > 0) {   // de = (r_e - b dnu) / a
                double vre[NV];
                ldn(vre, C::C_VRE, NV);
                if (corr) ldn(vcpv, C::C_VCP, 2 * NV);
                hold(vre, NV);
                if (corr) hold(vcpv, 2 * NV);
#pragma unroll
                for (int i = 0; i < NV; ++i) {
                    const double d1 = qp_div(vl[2 * i], vs[2 * i]), d2 = qp_div(vl[2 * i + 1], vs[2 * i + 1]);
                    dne[i] = vact ? qp_div(vre[i] - (d2 - d1) * dnv[i], d1 + d2) : 0.0;
                    dnv[i] = vact ? dnv[i] : 0.0;
                }
#pragma unroll
                for (int r = 0; r < 2 * NV; ++r) vcpv[r] = corr ? vcpv[r] : 0.0;
            }
            if (soc) {
                double v2[NQ], w2[NQ];
                dsq[0] = -rcq[0];
                v2[0] = rcq[0];
#pragma unroll
                for (int j = 1; j < NQ; ++j) { dsq[j] = -rcq[j] + dz[NX + j - 1]; v2[j] = rcq[j] - dz[NX + j - 1]; }
                w_apply(wv, eta, true, v2, w2);
#pragma unroll
                for (int j = 0; j < NQ; ++j) w2[j] += rho[j];
                w_apply(wv, eta, true, w2, dlq);
            } else {
#pragma unroll
                for (int j = 0; j < NQ; ++j) { dsq[j] = 0.0; dlq[j] = 0.0; }
            }
#pragma unroll
            for (int r = 0; r < NR; ++r) cpv[r] = corr ? cpv[r] : 0.0;
        };
        // row directions ds = -rc - G d, dl = (rco + l (rc + G d)) / s
        auto row_dir = [&](int r, bool corr, double& dsr, double& dlr) __attribute__((always_inline)) {
            double gz, h, gd, h2;
            row_eval(r, z, av, gz, h);
            row_eval(r, dz, da, gd, h2);
            const double rcr = gz + s_(r) - h;
            dsr = -rcr - gd;
            dlr = qp_div(rco_of(r, corr) + l_(r) * (rcr + gd), s_(r));
            if constexpr (C::STF) {
                if (r < C::R_BOX) {   // a stiff facet's multiplier step comes from the stage system
#pragma unroll
                    for (int i = 0; i < C::PM; ++i) dlr = sfr[i] == (double)r ? fnu[i] : dlr;
                }
            }
        };
        // One pass over the rows for the step length: the ratio test without divisions (the best
        // candidate kept as a fraction bn / bd, bd > 0, compared by cross-multiplication; one division
        // at the end), the coefficients of the complementarity after a step a,
        //   sum (s + a ds)(l + a dl) = q0 + a q1 + a^2 q2   (predictor: mu_aff without another pass),
        // the predictor products ds dl the corrector needs (stored), and a NaN / Inf probe of every
        // live direction (0 * x poisons the sum).
        auto max_step = [&](bool corr, double* quad, double& probe) __attribute__((always_inline)) {
            double bn = 1e300, bd = 1.0, q0 = 0.0, q1 = 0.0, q2 = 0.0, pr = 0.0;
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                if (row_on(r)) {
                    double dsr, dlr;
                    row_dir(r, corr, dsr, dlr);
                    const double sr = s_(r), lr = l_(r);
                    const bool c1 = dsr < 0.0 && sr * bd < bn * -dsr;
                    bn = c1 ? sr : bn;
                    bd = c1 ? -dsr : bd;
                    const bool c2 = dlr < 0.0 && lr * bd < bn * -dlr;
                    bn = c2 ? lr : bn;
                    bd = c2 ? -dlr : bd;
                    q0 = fma(sr, lr, q0);
                    q1 += fma(sr, dlr, lr * dsr);
                    q2 = fma(dsr, dlr, q2);
                    pr += 0.0 * (dsr + dlr);
                    if (!corr) cst(C::C_CP + r, dsr * dlr);
                }
            }
            if constexpr (NV > 0) {
                if (vact) {
#pragma unroll
                    for (int i = 0; i < NV; ++i) {
                        double dsr[2], dlr[2];
                        vrow_dir(i, corr, dsr, dlr);
#pragma unroll
                        for (int k = 0; k < 2; ++k) {
                            const double sr = vs[2 * i + k], lr = vl[2 * i + k];
                            const bool c1 = dsr[k] < 0.0 && sr * bd < bn * -dsr[k];
                            bn = c1 ? sr : bn;
                            bd = c1 ? -dsr[k] : bd;
                            const bool c2 = dlr[k] < 0.0 && lr * bd < bn * -dlr[k];
                            bn = c2 ? lr : bn;
                            bd = c2 ? -dlr[k] : bd;
                            q0 = fma(sr, lr, q0);
                            q1 += fma(sr, dlr[k], lr * dsr[k]);
                            q2 = fma(dsr[k], dlr[k], q2);
                            pr += 0.0 * (dsr[k] + dlr[k]);
                            if (!corr) cst(C::C_VCP + 2 * i + k, dsr[k] * dlr[k]);
                        }
                    }
                }
            }
            double am = bn / bd;
            if (soc) {
                am = fmin(am, soc_step(sq, dsq));
                am = fmin(am, soc_step(lq, dlq));
#pragma unroll
                for (int j = 0; j < NQ; ++j) {
                    q0 = fma(sq[j], lq[j], q0);
                    q1 += fma(sq[j], dlq[j], lq[j] * dsq[j]);
                    q2 = fma(dsq[j], dlq[j], q2);
                    pr += 0.0 * (dsq[j] + dlq[j]);
                }
            }
#pragma unroll
            for (int i = 0; i < NZ; ++i) pr += 0.0 * dz[i];
            quad[0] = q0; quad[1] = q1; quad[2] = q2;
            probe = pr;
            return wave_min(am);
        };

        // ---- predictor (affine scaling)
        double rcq2[NQ];
        load_soc();
        {
            double ltq0[NQ];
#pragma unroll
            for (int j = 0; j < NQ; ++j) ltq0[j] = ltq[j];
            if (soc) {
                double d0 = 0.0;
#pragma unroll
                for (int j = 0; j < NQ; ++j) d0 += ltq0[j] * ltq0[j];
                rcq2[0] = -d0;
#pragma unroll
                for (int j = 1; j < NQ; ++j) rcq2[j] = -2.0 * ltq0[0] * ltq0[j];
            } else {
#pragma unroll
                for (int j = 0; j < NQ; ++j) rcq2[j] = 0.0;
            }
        }
        newton(false, rcq2);
        double quad[3], probe;
        const double aa = fmin(1.0, max_step(false, quad, probe));
        const double gap_a = wave_sum(fma(aa, fma(aa, quad[2], quad[1]), quad[0]));
        const double mu_a = gap_a / deg;
        // (the cube as products: pow() would keep its polynomial constants live across the IPM loop)
        const double sgr = mu > 0 ? fmax(mu_a, 0.0) / mu : 0.0;
        const double sgm = sgr * sgr * sgr;
        // ---- corrector
        sgmu = sgm * mu;
        if (soc) {
            double a1[NQ], b1[NQ];
            w_apply(wv, eta, true, dsq, a1);
            w_apply(wv, eta, false, dlq, b1);
            double d0 = 0.0;
#pragma unroll
            for (int j = 0; j < NQ; ++j) d0 += a1[j] * b1[j];
            rcq2[0] -= d0;
#pragma unroll
            for (int j = 1; j < NQ; ++j) rcq2[j] -= a1[0] * b1[j] + b1[0] * a1[j];
            rcq2[0] += sgmu;
        }
        stamp(3);
        newton(true, rcq2);
        // step fraction: 0.99, or QP_TAU_END once the affine predictor takes a (nearly) full step (the end
        // game, where the fraction alone caps the gap reduction per iteration at 1 / (1 - fraction))
        const double al = fmin(1.0, (aa >= 0.99 ? QP_TAU_END : 0.99) * max_step(true, quad, probe));
        stamp(3);
        {
            const double chk = wave_sum(al + probe);  // NaN / Inf anywhere in the direction poisons the sum
            if (!(chk == chk) || !(al > 0.0)) {
                status = near ? SCVX_STATUS_MAX_ITER : SCVX_STATUS_NUMERICAL;
                fail_code = 4.0;
                break;
            }
            // stall at reduced accuracy: once the barrier Hessians span ~1e12 the Newton direction loses
            // its dual accuracy and the step collapses; keep the current (reduced-tolerance) iterate
            // rather than stepping along a direction that can break the next factorization
            if (near && al < 1e-2) {
                status = SCVX_STATUS_MAX_ITER;
                fail_code = 6.0;
                break;
            }
        }
        if (a.trace && agent == a.trace_agent && lane == 0 && it < a.trace_cap) {
            double* tr_ = a.trace + 8 * it;
            tr_[4] = aa; tr_[5] = al; tr_[6] = sgm;
        }
        // ---- update
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            if (row_on(r)) {
                double dsr, dlr;
                row_dir(r, true, dsr, dlr);
                s_set(r, s_(r) + al * dsr);
                l_set(r, l_(r) + al * dlr);
            }
        }
        if constexpr (NV > 0) {
            if (vact) {
#pragma unroll
                for (int i = 0; i < NV; ++i) {
                    double dsr[2], dlr[2];
                    vrow_dir(i, true, dsr, dlr);
#pragma unroll
                    for (int k = 0; k < 2; ++k) { vs[2 * i + k] += al * dsr[k]; vl[2 * i + k] += al * dlr[k]; }
                    vn[i] += al * dnv[i];
                    ve[i] += al * dne[i];
                }
            }
        }
        if (act) {
#pragma unroll
            for (int i = 0; i < NZ; ++i) z[i] += al * dz[i];
#pragma unroll
            for (int g = 0; g < NGA; ++g) av[g] += al * da[g];
            if (soc) {
#pragma unroll
                for (int j = 0; j < NQ; ++j) { sq[j] += al * dsq[j]; lq[j] += al * dlq[j]; }
            }
#pragma unroll
            for (int i = 0; i < NX; ++i) y[i] += al * dy[i];
        }
        store_state();
        if (lane < NX) {
            lds[V_YI + lane] += al * lds[V_DYI + lane];
            lds[V_YF + lane] += al * lds[V_DYF + lane];
        }
        stamp(10);
    }

    // ------------------------------------------------------------------ outputs
    load_state();
    // the warm-start state of the next solve: row duals and the initial / terminal multipliers
#pragma unroll
    for (int r = 0; r < NR; ++r) cst(C::C_WL + r, l_(r));
    cst(C::C_WY, lane < 2 * NX ? lds[V_YI + lane] : 0.0);
    if (a.trace && agent == a.trace_agent && lane == 0) {
        double* dd = a.trace + 8 * a.trace_cap;
        dd[0] = 0.0; dd[1] = 0.0; dd[2] = (double)(__builtin_amdgcn_s_memtime() - cyc_all0);
        dd[3] = fail_code;
        for (int k = 0; k < 16; ++k) dd[4 + k] = lds[V_ST + k];
    }
    double pobj = 0.0;
    if (act) {
#pragma unroll
        for (int i = 0; i < NX; ++i) a.X[(agent * K + t) * NX + i] = z[i];
#pragma unroll
        for (int j = 0; j < NU; ++j) { a.U[(agent * K + t) * NU + j] = z[NX + j]; pobj += wu * z[NX + j] * z[NX + j]; }
#pragma unroll
        for (int g = 0; g < NG; ++g) pobj += grp_on(g) ? gweight(g) * av[g] : 0.0;
        if (tsoft) {
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                const double e = z[i] - a.x_final[agent * NX + i];
                pobj += wfs * e * e;
            }
        }
        if (prox) {   // w_prox ||x_t - xbar_t||^2 (with its constant: the objective in the caller's units)
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                const double e = z[i] - a.Xref[(agent * K + t) * NX + i];
                pobj += wpx * e * e;
            }
        }
        if (vact) {
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                pobj += wnu * ve[i];
                a.nu[(agent * (K - 1) + t) * NX + i] = vn[i];
            }
        }
        a.slack_coll[agent * K + t] = (has_coll && ineq) ? av[NG > 0 ? NG - 1 : 0] : 0.0;
    }
    pobj = wave_sum(pobj);
    if (lane == 0) {
        a.obj[agent] = pobj * osc;
        a.status[agent] = status;
        a.iters[agent] = it;
        if (a.trace && a.trace_agent < 0) a.trace[agent] = fail_code;  // diagnostics: every agent's exit code
    }
}

#ifndef __HIPCC_RTC__
// launch helpers (qp_capi.hip picks the instantiation)
template <class C>
int qp_launch(const QPArgs& a, hipStream_t st) {
    const size_t lds = sizeof(double) * (size_t)C::lds_doubles(a.T.K);
    if (lds > 65536) (void)hipFuncSetAttribute((const void*)qp_ipm_kernel<C>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(qp_ipm_kernel<C>, dim3(a.N), dim3(WAVE), lds, st, a);
    return check_launch("qp_ipm_kernel");
}
#endif

}  // namespace scvx
