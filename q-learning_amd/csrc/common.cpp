// libqlx common pieces: error reporting, version, device selection.
#include <hip/hip_runtime.h>

#include <string>

#include "qlx_internal.h"

namespace qlx {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int current_device_checked(int device) {
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count == 0)
    throw Error{QLX_E_HIP, std::string("no HIP device available: ") + hipGetErrorString(e)};
  if (device < 0 || device >= count) throw Error{QLX_E_INVALID, "device index out of range"};
  QLX_HIP(hipSetDevice(device));
  return device;
}

}  // namespace qlx

extern "C" {

const char* qlx_last_error(void) { return qlx::g_last_error.c_str(); }
int32_t qlx_version(void) { return 1; }

}  // extern "C"
