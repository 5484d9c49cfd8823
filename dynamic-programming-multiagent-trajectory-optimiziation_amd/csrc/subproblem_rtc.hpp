// Launchers of the runtime-compiled subproblem kernels (csrc/subproblem_rtc.hip): templates with
// model_id = SCVX_MODEL_RUNTIME (user models; n_x, n_u from the template).
#pragma once
#include <hip/hip_runtime.h>

#include "qp_ipm.hpp"
#include "scp_kernel.hpp"

namespace scvx {
// the QP kernel for class QPCfg<n_x, n_u, nb, no, nc, vc> (compiled at the first use)
int rtc_qp_launch(const QPArgs& a, int nb, int no, int nc, int vc, hipStream_t st);
// the SCP kernel scp_ipm_kernel<n_x, n_u, ne, nw>
int rtc_scp_launch(const SCPArgs& a, int ne, int nw, hipStream_t st);
}  // namespace scvx
