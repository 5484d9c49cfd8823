// C-ABI bookkeeping for libscvx_hip.so: version, thread-local last-error string.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#include "common.hpp"
#include "scvx_hip.h"

namespace scvx {
static thread_local char g_err[256] = "";

int set_error(int code, const char* msg) {
    std::snprintf(g_err, sizeof(g_err), "%s", msg);
    return code;
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        std::snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
        return SCVX_ELAUNCH;
    }
    return SCVX_OK;
}
}  // namespace scvx

extern "C" int scvx_version(void) { return SCVX_HIP_VERSION; }
extern "C" const char* scvx_last_error(void) { return scvx::g_err; }
