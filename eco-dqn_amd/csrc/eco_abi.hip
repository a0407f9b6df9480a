// Error plumbing of the C ABI (eco_hip.h): thread-local last-error text.
#include "eco_common.h"

namespace eco {
static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(ECO_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
  return ECO_OK;
}
}  // namespace eco

extern "C" const char* eco_last_error(void) { return eco::g_last_error.c_str(); }
