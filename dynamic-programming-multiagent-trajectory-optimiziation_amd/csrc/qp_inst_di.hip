// QP kernel instantiations for the di model (n=6, m=3); classes: qp_caps.hpp SCVX_CAPS_DI.
#include "qp_inst.hpp"

namespace scvx {

int qp_launch_di(int idx, const QPArgs& a, hipStream_t st) {
    return QPDispatch<6, 3, 0, SCVX_CAPS_DI>::launch(idx, a, st);
}

}  // namespace scvx
