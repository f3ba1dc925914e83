// Shared device/host helpers for libmoegan_hip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/moegan_hip.h"

typedef uint16_t bf16_t;  // raw bf16 storage (activations in bf16 mode)
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef unsigned short u16x8_t __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

#define MG_DEV __device__ __forceinline__

MG_DEV float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
MG_DEV bf16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (bf16_t)((u >> 16) | 0x40u);  // keep NaN a NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (bf16_t)(u >> 16);
}

// Element load/store as float regardless of storage type.
MG_DEV float ldf(const float* p, int64_t i) { return p[i]; }
MG_DEV float ldf(const bf16_t* p, int64_t i) { return bf2f(p[i]); }
MG_DEV void stf(float* p, int64_t i, float v) { p[i] = v; }
MG_DEV void stf(bf16_t* p, int64_t i, float v) { p[i] = f2bf(v); }

template <typename T> struct VecOf;  // 16-byte vectors
template <> struct VecOf<float> { static constexpr int N = 4; typedef f32x4_t type; };
template <> struct VecOf<bf16_t> { static constexpr int N = 8; typedef u16x8_t type; };

MG_DEV float lrelu(float x) { return x > 0.f ? x : 0.2f * x; }
MG_DEV float lrelu_grad(float y) { return y > 0.f ? 1.f : 0.2f; }
MG_DEV float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
MG_DEV float gelu_erf_grad(float x) {
  float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

MG_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
MG_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- error plumbing (C-ABI returns 0 / negative, message via mg_last_error) ----
void mg_set_error(const std::string& msg);
int mg_check_launch(const char* what);

#define MG_REQUIRE(cond, msg)                       \
  do {                                              \
    if (!(cond)) {                                  \
      mg_set_error(std::string(__func__) + ": " + (msg)); \
      return MG_ERR_ARG;                            \
    }                                               \
  } while (0)

static inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }
