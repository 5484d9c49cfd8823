// Launchers of the runtime-compiled subproblem kernels (csrc/subproblem_rtc.hip): templates with
// model_id = SCVX_MODEL_RUNTIME (user models; n_x, n_u from the template).
#pragma once
#include <hip/hip_runtime.h>

#include "qp_ipm.hpp"
#include "scp_kernel.hpp"

namespace scvx {
// Limits of the runtime-compiled classes, shared by the solve entry points (qp_check, scp_launch) and
// scvx_rtc_subproblem_compile, so a class that compiles is one that launches.  nullptr when the class is served.
// QP: the 3 x 3 position block (n_x >= 3), the solve chains' 16-lane broadcast and the virtual control's
// Gauss-Jordan over 4 n_x lanes (n_x <= 16), 2^n_u trust-region facets (n_u <= 4), j_max <= 32, and the class's
// LDS within 64 KiB at K (the compile entry, which has no K, checks the smallest K = 2).
inline const char* rtc_qp_class_error(int nx, int nu, int nb, int no, int nc, int vc, int K) {
    if (nx < 3 || nx > 16 || nu < 1 || nu > 4) return "qp: runtime model needs 3 <= n_x <= 16 and 1 <= n_u <= 4";
    if (nb < 0 || nb > SCVX_MAX_BOX || no < 0 || no > SCVX_MAX_OBS || nc < 0 || nc > 32 || vc < 0 || vc > 1)
        return "qp: runtime class needs n_box <= 4, n_obs <= 16, j_max <= 32";
    if (sizeof(double) * (size_t)qp_lds_doubles(nx, nu, nb, no, nc, vc, K) > 65536)
        return "qp: runtime class needs more than 64 KiB of LDS";
    return nullptr;
}
// SCP: the node vector z = [xi | g | game states | u | nu] within the kernel's 16 (n_x <= 8)
inline const char* rtc_scp_class_error(int nx, int nu, int ne) {
    if (nx < 1 || nx > 8 || nu < 1 || ne < 0 || 2 * nx + SCP_NG + ne + nu > 16)
        return "scp: runtime model needs 2 n_x + n_u + 4 (+ game states) <= 16";
    return nullptr;
}
// the QP kernel for class QPCfg<n_x, n_u, nb, no, nc, vc> (compiled at the first use)
int rtc_qp_launch(const QPArgs& a, int nb, int no, int nc, int vc, hipStream_t st);
// the SCP kernel scp_ipm_kernel<n_x, n_u, ne, nw>
int rtc_scp_launch(const SCPArgs& a, int ne, int nw, hipStream_t st);
}  // namespace scvx
