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

// Pinned host memory mapped into the device address space (the drop-in's zero-copy launches:
// a small batch's kernel reads its rows from, and writes its results to, host memory over
// PCIe, so a call costs one kernel launch and no DMA copies).  Coherent: the host sees the
// kernel's stores once the launch's completion event has fired.
int egr_host_alloc(int64_t bytes, void** host, void** dev) {
  if (bytes <= 0 || !host || !dev) return egr::fail(EGR_EINVAL, "egr_host_alloc: bad arguments");
  *host = *dev = nullptr;
  void* h = nullptr;
  EGR_HIP(hipHostMalloc(&h, (size_t)bytes, hipHostMallocMapped | hipHostMallocCoherent));
  void* d = nullptr;
  const hipError_t e = hipHostGetDevicePointer(&d, h, 0);
  if (e != hipSuccess) {
    (void)hipHostFree(h);
    return egr::fail(EGR_EDEVICE, std::string("hipHostGetDevicePointer: ") + hipGetErrorString(e));
  }
  *host = h;
  *dev = d;
  return EGR_OK;
}

int egr_host_free(void* host) {
  if (host) EGR_HIP(hipHostFree(host));
  return EGR_OK;
}

double egr_py_round(double x, int32_t ndigits) {
  if (ndigits < 0 || ndigits > 15) return x;
  return egr::py_round(x, ndigits);
}

}  // extern "C"
