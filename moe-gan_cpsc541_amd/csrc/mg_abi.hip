// Error plumbing and version of libmoegan_hip.
#include <string>

#include "mg_common.h"

static thread_local std::string g_last_error;

void mg_set_error(const std::string& msg) { g_last_error = msg; }

int mg_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_last_error = std::string(what) + ": " + hipGetErrorString(e);
    return MG_ERR_LAUNCH;
  }
  return MG_OK;
}

extern "C" const char* mg_last_error(void) { return g_last_error.c_str(); }
extern "C" int mg_version(void) { return 1; }
