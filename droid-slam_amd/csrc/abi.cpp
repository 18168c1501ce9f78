// C-ABI support: error reporting and one-time device setup.
#include <hip/hip_runtime.h>

#include <string>

#include "common.hpp"

namespace droid {

static thread_local std::string g_last_error;

void set_last_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  set_last_error(msg);
  return code;
}

}  // namespace droid

extern "C" {

const char* droid_last_error(void) { return droid::g_last_error.c_str(); }

int droid_abi_version(void) { return 1; }

// How this library was built: bit 0 = the A/B build (make ab: the dropped
// kernel variants and the DROID_* experiment knobs), bit 1 = the profiling
// build (make prof: timeline stamps).  The product library returns 0.
int droid_build_info(void) {
#ifndef DROID_CONV_PROFILE
#define DROID_CONV_PROFILE 0
#endif
  return (DROID_AB ? 1 : 0) | (DROID_CONV_PROFILE ? 2 : 0);
}

// Number of visible HIP devices (0 on a GPU-less host); never launches work.
int droid_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

}  // extern "C"
