// Row-capacity classes of the batched QP kernel (qp_ipm.hpp QPCfg<n, m, NB, NO, NC>): the
// inequality-row state lives in registers, so every instantiation fixes how many box constraints
// (NB), obstacles (NO) and collision rows per node (NC) it can hold.  A solve runs on the first
// class of its model that fits the template; the per-model tables below are the instantiations
// compiled into libscvx_hip.so (qp_inst_*.hip).
#pragma once
#include "scvx_hip.h"

namespace scvx {

// flat (NB, NO, NC) triples
#define SCVX_CAPS_DI 2, 0, 0, 2, 8, 0, 2, 0, 8, 2, 0, 16, 2, 8, 8, 4, 16, 32
#define SCVX_CAPS_UNICYCLE 2, 4, 0, 2, 0, 8, 4, 16, 32
#define SCVX_CAPS_SI 4, 8, 0, 4, 0, 8, 4, 16, 32
#define SCVX_CAPS_QUAD 4, 8, 8, 4, 16, 32

// index of the first class in the flat table caps[0..3n) holding (n_box, n_obs, j_max), or -1
inline int qp_pick_caps(const int* caps, int n, const scvx_qp_template& T) {
    for (int i = 0; i < n; ++i)
        if (T.n_box <= caps[3 * i] && T.n_obs <= caps[3 * i + 1] && T.j_max <= caps[3 * i + 2]) return i;
    return -1;
}

}  // namespace scvx
