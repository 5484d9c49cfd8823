// Row-capacity classes of the batched QP kernel (qp_ipm.hpp QPCfg<n, m, NB, NO, NC, VC>): the
// inequality-row state lives in registers, so every instantiation fixes how many box constraints
// (NB), obstacles (NO) and collision rows per node (NC) it can hold.  A solve runs on the first
// class of its model that fits the template; the per-model tables below are the instantiations
// compiled into libscvx_hip.so (qp_inst_*.hip).
#pragma once
#include "scvx_hip.h"

namespace scvx {

// flat (NB, NO, NC, VC) quadruples; VC = 1: the virtual-control classes (w_nu > 0)
#define SCVX_CAPS_DI 2, 0, 0, 0, 2, 8, 0, 0, 2, 0, 8, 0, 2, 0, 16, 0, 2, 8, 8, 0, 4, 16, 32, 0, 2, 8, 0, 1
#define SCVX_CAPS_UNICYCLE 2, 4, 0, 0, 2, 0, 8, 0, 4, 16, 32, 0
#define SCVX_CAPS_SI 4, 8, 0, 0, 4, 0, 8, 0, 4, 16, 32, 0
#define SCVX_CAPS_QUAD 4, 8, 8, 0, 4, 16, 32, 0, 4, 8, 8, 1, 4, 16, 32, 1
constexpr int QP_CAPS_W = 4;   // ints per class

// index of the first class in the flat table caps[0..4n) holding (n_box, n_obs, j_max) with the template's
// virtual-control setting, or -1
inline int qp_pick_caps(const int* caps, int n, const scvx_qp_template& T) {
    const int vc = T.w_nu > 0.0 ? 1 : 0;
    for (int i = 0; i < n; ++i) {
        const int* c = caps + QP_CAPS_W * i;
        if (T.n_box <= c[0] && T.n_obs <= c[1] && T.j_max <= c[2] && c[3] == vc) return i;
    }
    return -1;
}

}  // namespace scvx
