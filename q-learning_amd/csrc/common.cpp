// libqlx common pieces: error reporting, version, device selection.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>

#include <mutex>
#include <set>
#include <tuple>
#include "qlx_internal.h"

namespace qlx {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

void set_lds_limit(const void* kernel, size_t bytes) {
  static std::mutex mu;
  static std::set<std::tuple<int, const void*, size_t>> done;   // the attribute is set per device
  int dev = 0;
  QLX_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lock(mu);
  if (!done.insert({dev, kernel, bytes}).second) return;
  QLX_HIP(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
}

// QLX_DEBUG_SYNC=1: wait for the stream after each instrumented launch and name the launch in the error (fault
// localisation on the GPU box; off by default)
void debug_sync(hipStream_t s, const char* what) {
  static const bool on = [] {
    const char* v = std::getenv("QLX_DEBUG_SYNC");
    return v && v[0] == '1';
  }();
  if (!on) return;
  const hipError_t e = hipStreamSynchronize(s);
  if (e != hipSuccess) throw Error{QLX_E_HIP, std::string("after ") + what + ": " + hipGetErrorString(e)};
}

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
