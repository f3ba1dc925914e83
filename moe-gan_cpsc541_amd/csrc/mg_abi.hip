// Error plumbing, scratch workspace, tuning switches and version of libmoegan_hip.
#include <atomic>
#include <mutex>
#include <vector>
#include <string>

#include "mg_common.h"

#ifndef MG_SRC_HASH
#define MG_SRC_HASH "unknown"
#endif

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

// Scratch for split-K slabs and reduction partials: one block per (device, stream).  Launches on one
// stream are ordered, so reusing the block across the calls enqueued on that stream is race-free, and
// launches on different streams or devices never share a block.  A block is either caller-owned
// (mg_set_workspace: the library never allocates or frees it; a request larger than it fails with
// MG_ERR_ARG) or library-owned (grown on demand: hipStreamSynchronize on that stream, hipFree, hipMalloc
// -- so grow it with mg_workspace_reserve before capturing a hipGraph; steady-state training never grows).
namespace {
struct WsEntry {
  int device;
  hipStream_t stream;
  void* ptr;
  size_t bytes;
  bool caller_owned;
};
constexpr int kMaxWsStreams = 256;  // torch hands out streams from a fixed pool (32 per priority per device)
WsEntry g_ws[kMaxWsStreams];
int g_ws_n = 0;
std::mutex g_ws_mu;

WsEntry* ws_entry(int dev, hipStream_t stream) {
  for (int i = 0; i < g_ws_n; ++i)
    if (g_ws[i].device == dev && g_ws[i].stream == stream) return &g_ws[i];
  if (g_ws_n == kMaxWsStreams) return nullptr;
  WsEntry* e = &g_ws[g_ws_n++];
  *e = WsEntry{dev, stream, nullptr, 0, false};
  return e;
}
}  // namespace

void* mg_workspace(size_t bytes, hipStream_t stream) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(g_ws_mu);
  WsEntry* e = ws_entry(dev, stream);
  if (!e) return nullptr;
  if (bytes <= e->bytes) return e->ptr;
  if (e->caller_owned) {
    mg_set_error("caller-provided workspace too small: " + std::to_string(bytes) + " bytes needed");
    return nullptr;
  }
  if (e->ptr) {
    (void)hipStreamSynchronize(stream);  // the only user of this block is `stream`
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

namespace {
struct CntEntry {
  int device;
  hipStream_t stream;
  int* ptr;
  int n;
};
std::vector<CntEntry> g_cnt;
std::mutex g_cnt_mu;
}  // namespace

int* mg_tile_counters(int n, hipStream_t stream) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(g_cnt_mu);
  for (auto& e : g_cnt)
    if (e.device == dev && e.stream == stream && e.n >= n) return e.ptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  const int want = std::max(n, 8192);
  int* p = nullptr;
  if (hipMalloc(reinterpret_cast<void**>(&p), (size_t)want * sizeof(int)) != hipSuccess) return nullptr;
  if (hipMemsetAsync(p, 0, (size_t)want * sizeof(int), stream) != hipSuccess) return nullptr;
  for (auto& e : g_cnt)
    if (e.device == dev && e.stream == stream) {  // a larger set replaces the old one (kept: in-flight launches)
      e.ptr = p;
      e.n = want;
      return p;
    }
  g_cnt.push_back(CntEntry{dev, stream, p, want});
  return p;
}

extern "C" int mg_set_workspace(void* ptr, size_t bytes, void* stream) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return MG_ERR_LAUNCH;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  std::lock_guard<std::mutex> lk(g_ws_mu);
  WsEntry* e = ws_entry(dev, st);
  MG_REQUIRE(e, "too many streams");
  if (e->ptr && !e->caller_owned) {
    (void)hipStreamSynchronize(st);
    (void)hipFree(e->ptr);
  }
  *e = ptr ? WsEntry{dev, st, ptr, bytes, true} : WsEntry{dev, st, nullptr, 0, false};
  return MG_OK;
}

extern "C" int mg_workspace_reserve(size_t bytes, void* stream) {
  if (!mg_workspace(bytes, reinterpret_cast<hipStream_t>(stream))) {
    if (g_last_error.empty()) mg_set_error("mg_workspace_reserve: allocation failed");
    return MG_ERR_LAUNCH;
  }
  return MG_OK;
}

extern "C" int64_t mg_workspace_bytes(void* stream) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  std::lock_guard<std::mutex> lk(g_ws_mu);
  for (int i = 0; i < g_ws_n; ++i)
    if (g_ws[i].device == dev && g_ws[i].stream == st) return (int64_t)g_ws[i].bytes;
  return 0;
}

std::atomic<int> g_mg_tune[MG_TUNE_COUNT];

extern "C" int mg_set_tuning(int key, int value) {
  if (key < 0 || key >= MG_TUNE_COUNT) {
    mg_set_error("mg_set_tuning: key out of range");
    return MG_ERR_ARG;
  }
  g_mg_tune[key].store(value, std::memory_order_relaxed);
  return MG_OK;
}

extern "C" const char* mg_last_error(void) { return g_last_error.c_str(); }
extern "C" int mg_version(void) { return 2; }
extern "C" const char* mg_source_hash(void) { return MG_SRC_HASH; }

// ---- measurement of one call inside a step (include/moegan_hip.h: mg_timer_event_* / mg_mark) ----
__global__ void k_roofline_mark_begin() {}
__global__ void k_roofline_mark_end() {}

extern "C" int mg_timer_event_create(void** event) {
  MG_REQUIRE(event != nullptr, "event must not be NULL");
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) {
    mg_set_error("mg_timer_event_create: hipEventCreateWithFlags failed");
    return MG_ERR_LAUNCH;
  }
  *event = reinterpret_cast<void*>(e);
  return MG_OK;
}

extern "C" int mg_timer_event_record(void* event, void* stream) {
  MG_REQUIRE(event != nullptr, "event must not be NULL");
  if (hipEventRecord(reinterpret_cast<hipEvent_t>(event), reinterpret_cast<hipStream_t>(stream)) != hipSuccess) {
    mg_set_error("mg_timer_event_record: hipEventRecord failed");
    return MG_ERR_LAUNCH;
  }
  return MG_OK;
}

extern "C" int mg_timer_event_elapsed(void* start, void* stop, float* ms) {
  MG_REQUIRE(start != nullptr && stop != nullptr && ms != nullptr, "events and ms must not be NULL");
  hipEvent_t s = reinterpret_cast<hipEvent_t>(start), e = reinterpret_cast<hipEvent_t>(stop);
  if (hipEventSynchronize(e) != hipSuccess || hipEventElapsedTime(ms, s, e) != hipSuccess) {
    mg_set_error("mg_timer_event_elapsed: hipEventSynchronize / hipEventElapsedTime failed");
    return MG_ERR_LAUNCH;
  }
  return MG_OK;
}

extern "C" int mg_timer_event_destroy(void* event) {
  if (event) (void)hipEventDestroy(reinterpret_cast<hipEvent_t>(event));
  return MG_OK;
}

extern "C" int mg_mark(int tag, void* stream) {
  MG_REQUIRE(tag == 0 || tag == 1, "tag must be 0 (begin) or 1 (end)");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (tag == 0) hipLaunchKernelGGL(k_roofline_mark_begin, dim3(1), dim3(64), 0, st);
  else hipLaunchKernelGGL(k_roofline_mark_end, dim3(1), dim3(64), 0, st);
  return mg_check_launch("mg_mark");
}
