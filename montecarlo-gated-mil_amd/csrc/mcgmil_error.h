// Error reporting shared by the library's translation units (mcgmil.hip, mcgmil_image.hip):
// the thread-local message behind mcgmil_last_error().
#pragma once
#include <hip/hip_runtime.h>

#include <string>

namespace mcgmil_detail {
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);
}  // namespace mcgmil_detail
