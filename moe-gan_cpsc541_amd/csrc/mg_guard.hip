// Loss-level failure guards of train_aurora_gan as device-side flags (no host sync inside the step).
//
// The reference checks its losses on the host every batch (t2i_moe_gan.py:1315-1320, :1367-1376,
// :1396-1399).  Here the checks write bits of a per-step int32 flag word, and the optimizer kernels read
// that word (plus a per-accumulation-window word recording which parameter groups received a gradient)
// to decide whether they run -- so the step stays one captured hipGraph and the host reads the flags at
// most once per step, for logging.
#include "mg_common.h"

namespace {

// flags[0] |= bit if any of x[0..n) is NaN / Inf (one wave; n is a handful of loss scalars)
__global__ void k_finite_flag(const float* __restrict__ x, int n, int32_t bit, int32_t* __restrict__ flags) {
  bool bad = false;
  for (int i = threadIdx.x; i < n; i += 64) bad |= !isfinite(x[i]);
  if (__ballot(bad) != 0ull && threadIdx.x == 0) flags[0] |= bit;
}

// win &= ~reset_bits unless flags & keep_mask;  win |= set_bits unless flags & bad_mask
__global__ void k_flag_window(const int32_t* __restrict__ flags, int32_t reset_bits, int32_t keep_mask,
                              int32_t bad_mask, int32_t set_bits, int32_t* __restrict__ win) {
  if (threadIdx.x != 0) return;
  const int32_t f = flags[0];
  int32_t w = win[0];
  if ((f & keep_mask) == 0) w &= ~reset_bits;
  if ((f & bad_mask) == 0) w |= set_bits;
  win[0] = w;
}

// the loss checks and window updates of one phase in one launch (mg_guard_update): flags[0] |= bit[i] for every check
// whose scalars are not all finite, then the window updates in order on the updated flags (k_flag_window's rule)
__global__ void k_guard_update(mg_guard_desc d, int32_t* __restrict__ flags, int32_t* __restrict__ win) {
  int32_t add = 0;
  for (int c = 0; c < 4; ++c) {
    if (d.n[c] <= 0) continue;
    bool bad = false;
    for (int i = threadIdx.x; i < d.n[c]; i += 64) bad |= !isfinite(d.x[c][i]);
    if (__ballot(bad) != 0ull) add |= d.bit[c];
  }
  if (threadIdx.x != 0) return;
  const int32_t f = flags[0] | add;
  if (add) flags[0] = f;
  if (d.nwin > 0) {
    int32_t w = win[0];
    for (int j = 0; j < d.nwin && j < 2; ++j) {
      if ((f & d.keep_mask[j]) == 0) w &= ~d.reset_bits[j];
      if ((f & d.bad_mask[j]) == 0) w |= d.set_bits[j];
    }
    win[0] = w;
  }
}

MG_DEV bool gate_on(const int32_t* flags, int32_t mask) { return flags && (flags[0] & mask) != 0; }

// x[0 .. words) = 0 when (flags & mask) != 0 equals when_set (4-byte words, 16-B vectors where aligned)
__global__ __launch_bounds__(256) void k_zero_if(uint32_t* __restrict__ x, int64_t words,
                                                 const int32_t* __restrict__ flags, int32_t mask, int when_set) {
  if (gate_on(flags, mask) != (when_set != 0)) return;
  const int64_t nv = mg_al16(x) ? words / 4 : 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv; i += stride)
    reinterpret_cast<f32x4_t*>(x)[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  for (int64_t i = nv * 4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < words; i += stride) x[i] = 0u;
}

// acc += g unless flags & mask
__global__ __launch_bounds__(256) void k_gated_axpy(float* __restrict__ acc, const float* __restrict__ g, int64_t n,
                                                    const int32_t* __restrict__ flags, int32_t mask) {
  if (gate_on(flags, mask)) return;
  const int64_t nv = (mg_al16(acc) && mg_al16(g)) ? n / 4 : 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv; i += stride) {
    f32x4_t a = reinterpret_cast<const f32x4_t*>(acc)[i], b = reinterpret_cast<const f32x4_t*>(g)[i];
    reinterpret_cast<f32x4_t*>(acc)[i] = a + b;
  }
  for (int64_t i = nv * 4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) acc[i] += g[i];
}

// out = (flags & mask) ? src : 0
__global__ void k_select_if(const float* __restrict__ src, int n, const int32_t* __restrict__ flags, int32_t mask,
                            float* __restrict__ out) {
  const bool on = gate_on(flags, mask);
  for (int i = threadIdx.x; i < n; i += blockDim.x) out[i] = on ? src[i] : 0.f;
}

inline int nblk(int64_t n, int t = 256) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + t - 1) / t, 4096)); }

}  // namespace

extern "C" int mg_finite_flag(const float* x, int n, int32_t bit, int32_t* flags, void* stream) {
  MG_REQUIRE(x && flags && n >= 0, "null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n == 0) return MG_OK;
  hipLaunchKernelGGL(k_finite_flag, dim3(1), dim3(64), 0, st, x, n, bit, flags);
  return mg_check_launch("mg_finite_flag");
}

extern "C" int mg_flag_window(const int32_t* flags, int32_t reset_bits, int32_t keep_mask, int32_t bad_mask,
                              int32_t set_bits, int32_t* win, void* stream) {
  MG_REQUIRE(flags && win, "null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_flag_window, dim3(1), dim3(64), 0, st, flags, reset_bits, keep_mask, bad_mask, set_bits, win);
  return mg_check_launch("mg_flag_window");
}

extern "C" int mg_guard_update(const mg_guard_desc* d, int32_t* flags, int32_t* win, void* stream) {
  MG_REQUIRE(d && flags, "null pointer");
  MG_REQUIRE(d->nwin >= 0 && d->nwin <= 2 && (d->nwin == 0 || win), "0 <= nwin <= 2 (and a window word)");
  for (int c = 0; c < 4; ++c) MG_REQUIRE(d->n[c] <= 0 || d->x[c], "null check operand");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_guard_update, dim3(1), dim3(64), 0, st, *d, flags, win);
  return mg_check_launch("mg_guard_update");
}

extern "C" int mg_zero_if(void* x, int64_t bytes, const int32_t* flags, int32_t mask, int when_set, void* stream) {
  MG_REQUIRE(bytes % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 3) == 0, "4-byte words");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (bytes == 0) return MG_OK;
  const int64_t words = bytes / 4;
  hipLaunchKernelGGL(k_zero_if, dim3(nblk(words / 4 + 1)), dim3(256), 0, st, reinterpret_cast<uint32_t*>(x), words,
                     flags, mask, when_set);
  return mg_check_launch("mg_zero_if");
}

extern "C" int mg_gated_axpy(float* acc, const float* g, int64_t n, const int32_t* flags, int32_t mask, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n == 0) return MG_OK;
  hipLaunchKernelGGL(k_gated_axpy, dim3(nblk(n / 4 + 1)), dim3(256), 0, st, acc, g, n, flags, mask);
  return mg_check_launch("mg_gated_axpy");
}

extern "C" int mg_select_if(const float* src, int n, const int32_t* flags, int32_t mask, float* out, void* stream) {
  MG_REQUIRE(n >= 0 && n <= 4096, "n out of range");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n == 0) return MG_OK;
  hipLaunchKernelGGL(k_select_if, dim3(1), dim3(256), 0, st, src, n, flags, mask, out);
  return mg_check_launch("mg_select_if");
}
