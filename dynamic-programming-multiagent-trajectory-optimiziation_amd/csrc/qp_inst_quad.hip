// QP kernel instantiations for the quad model (n=12, m=4); classes: qp_caps.hpp SCVX_CAPS_QUAD.
#include "qp_inst.hpp"

namespace scvx {

int qp_launch_quad(int idx, const QPArgs& a, hipStream_t st) {
    return QPDispatch<12, 4, 0, SCVX_CAPS_QUAD>::launch(idx, a, st);
}

}  // namespace scvx
