// Library-wide C-ABI entry points: error reporting, version, device query, exact round.
#include <string>

#include "egr_internal.h"

namespace egr {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

}  // namespace egr

extern "C" {

const char* egr_last_error(void) { return egr::g_last_error.c_str(); }

int egr_version(void) { return EGR_VERSION; }

int egr_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

double egr_py_round(double x, int32_t ndigits) {
  if (ndigits < 0 || ndigits > 15) return x;
  return egr::py_round(x, ndigits);
}

}  // extern "C"
