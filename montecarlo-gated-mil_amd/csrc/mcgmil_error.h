// Error reporting shared by the library's translation units (mcgmil.hip, mcgmil_image.hip):
// the thread-local message behind mcgmil_last_error().
#pragma once
#include <hip/hip_runtime.h>

#include <string>


namespace mcgmil_detail {
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);
// Raise kernel k's dynamic-LDS limit to 160 KiB on the CURRENT device, once per (kernel, device):
// MCGMIL_OK, or the hipFuncSetAttribute error through hip_fail (naming `what`).
int raise_lds_limit(const void* k, const char* what);
}  // namespace mcgmil_detail
