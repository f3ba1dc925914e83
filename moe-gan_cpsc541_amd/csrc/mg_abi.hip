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

// Split-K slab workspace.  Growth frees the old block only after the device is idle, so an
// in-flight launch never reads freed memory; steady-state training never grows it (and a
// captured hipGraph keeps seeing the same pointer).
static void* g_ws = nullptr;
static size_t g_ws_bytes = 0;

void* mg_workspace(size_t bytes) {
  if (bytes <= g_ws_bytes) return g_ws;
  if (g_ws) {
    (void)hipDeviceSynchronize();
    (void)hipFree(g_ws);
  }
  size_t want = bytes + (bytes >> 2);
  if (hipMalloc(&g_ws, want) != hipSuccess) {
    g_ws = nullptr;
    g_ws_bytes = 0;
    return nullptr;
  }
  g_ws_bytes = want;
  return g_ws;
}

int g_mg_tune[MG_TUNE_COUNT] = {0};

extern "C" int mg_set_tuning(int key, int value) {
  if (key < 0 || key >= MG_TUNE_COUNT) return MG_ERR_ARG;
  g_mg_tune[key] = value;
  return MG_OK;
}

extern "C" const char* mg_last_error(void) { return g_last_error.c_str(); }
extern "C" int mg_version(void) { return 1; }
