// QP kernel instantiations for the si model (n=3, m=3); classes: qp_caps.hpp SCVX_CAPS_SI.
#include "qp_inst.hpp"

namespace scvx {

int qp_launch_si(int idx, const QPArgs& a, hipStream_t st) {
    return QPDispatch<3, 3, 0, SCVX_CAPS_SI>::launch(idx, a, st);
}

}  // namespace scvx
