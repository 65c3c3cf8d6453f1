// ocn_internal.h -- shared internals of libocn_sw (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <initializer_list>
#include <string>

#include "../../include/ocn_sw.h"

// Rows of a block strip owned by one 64x4 workgroup (see sw_kernels.hip).
#ifndef OCN_ROWS
#define OCN_ROWS 32
#endif

// shared/constants.f90:23  FreeFallAcc = 9.8 (real(4))
#define OCN_FREE_FALL_ACC 9.8f

namespace ocn {

int set_error(int code, const std::string &msg);
int check_hip(hipError_t e, const char *what);
inline int check_launch() { return check_hip(hipGetLastError(), "kernel launch"); }

}  // namespace ocn
