// Error plumbing and version of libmoegan_hip.
#include <mutex>
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

// Split-K slab / partial-sum workspace, one block per stream (launches on different streams may run
// concurrently, launches on one stream are ordered, so per-stream reuse is race-free).  Growth frees the
// old block only after the device is idle, so an in-flight launch never reads freed memory; steady-state
// training never grows it (and a captured hipGraph keeps seeing the same pointers).
namespace {
struct WsEntry { hipStream_t stream; void* ptr; size_t bytes; };
constexpr int kMaxWsStreams = 128;  // torch hands out streams from a fixed pool (32 per priority)
WsEntry g_ws[kMaxWsStreams];
int g_ws_n = 0;
std::mutex g_ws_mu;
}  // namespace

void* mg_workspace(size_t bytes, hipStream_t stream) {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  WsEntry* e = nullptr;
  for (int i = 0; i < g_ws_n; ++i)
    if (g_ws[i].stream == stream) e = &g_ws[i];
  if (!e) {
    if (g_ws_n == kMaxWsStreams) return nullptr;
    e = &g_ws[g_ws_n++];
    *e = WsEntry{stream, nullptr, 0};
  }
  if (bytes <= e->bytes) return e->ptr;
  if (e->ptr) {
    (void)hipDeviceSynchronize();
    (void)hipFree(e->ptr);
  }
  size_t want = bytes + (bytes >> 2);
  if (hipMalloc(&e->ptr, want) != hipSuccess) {
    e->ptr = nullptr;
    e->bytes = 0;
    return nullptr;
  }
  e->bytes = want;
  return e->ptr;
}

int g_mg_tune[MG_TUNE_COUNT] = {0};

extern "C" int mg_set_tuning(int key, int value) {
  if (key < 0 || key >= MG_TUNE_COUNT) return MG_ERR_ARG;
  g_mg_tune[key] = value;
  return MG_OK;
}

extern "C" const char* mg_last_error(void) { return g_last_error.c_str(); }
extern "C" int mg_version(void) { return 1; }
