// Shared host-side helpers for the C-ABI: error codes never cross the ABI as exceptions.
#pragma once
#include <hip/hip_runtime.h>

#include "scvx_hip.h"

namespace scvx {
int set_error(int code, const char* msg);
int check_launch(const char* what);
}  // namespace scvx
