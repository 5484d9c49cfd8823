// QP kernel instantiations for the unicycle model (n=3, m=2); classes: qp_caps.hpp SCVX_CAPS_UNICYCLE.
#include "qp_inst.hpp"

namespace scvx {

int qp_launch_unicycle(int idx, const QPArgs& a, hipStream_t st) {
    return QPDispatch<3, 2, 0, SCVX_CAPS_UNICYCLE>::launch(idx, a, st);
}

}  // namespace scvx
