// Instantiation helper: one translation unit per model (parallel builds).
#pragma once
#include "qp_caps.hpp"
#include "qp_ipm.hpp"

namespace scvx {

// launch class `idx` of the table (compile-time list of QPCfg)
template <int NX, int NU, int IDX, int NB, int NO, int NC, int VC, int... REST>
struct QPDispatch {
    static int launch(int idx, const QPArgs& a, hipStream_t st) {
        if (idx == IDX) return qp_launch<QPCfg<NX, NU, NB, NO, NC, VC>>(a, st);
        return QPDispatch<NX, NU, IDX + 1, REST...>::launch(idx, a, st);
    }
};
template <int NX, int NU, int IDX, int NB, int NO, int NC, int VC>
struct QPDispatch<NX, NU, IDX, NB, NO, NC, VC> {
    static int launch(int idx, const QPArgs& a, hipStream_t st) {
        if (idx == IDX) return qp_launch<QPCfg<NX, NU, NB, NO, NC, VC>>(a, st);
        return set_error(SCVX_EUNSUPPORTED, "qp: no row-capacity class");
    }
};

}  // namespace scvx
