// Modulated-convolution backward helpers (t2i_moe_gan.py:154-186).
//
// Forward (fused form, no per-sample weights are ever materialised):
//     s = modulation(w)            [B, Cin]
//     d[b,o] = rsqrt(sum_ci s^2 * wsq[o,ci] + 1e-8)        wsq = sum_taps W^2
//     y = d[b,o] * conv(x * s[b,ci], W)      (then optional LeakyReLU(0.2))
// Backward, with gy the gradient of y (pre-activation):
//     gyt = gy * d                     -> conv data / weight gradients
//     gdd[b,o] = -0.5 * d^2 * sum_pix gy * y       (= d(loss)/d(sum_ci s^2 wsq))
//     gxt = conv^T(gyt, W);  gx = gxt * s;  gs_x[b,ci] = sum_pix gxt * x
// The two kernels below produce gyt/gdd and gx/gs_x in one pass each.
#include "mg_common.h"

namespace {

// one block per (b, 256-channel slab); threads over channels, loop over the image's pixels
template <typename T, typename TG>
__global__ void k_bwd_out(const TG* __restrict__ gz, int64_t ld_gz, const T* __restrict__ z, int64_t ld_z,
                          const T* __restrict__ zsub, int64_t ld_zsub, const float* __restrict__ d, int HW, int Cout,
                          int act, T* __restrict__ gyt, int64_t ld_gyt, float* __restrict__ gdd) {
  int b = blockIdx.x;
  int o = blockIdx.y * blockDim.x + threadIdx.x;
  if (o >= Cout) return;
  float dd = d[(int64_t)b * Cout + o];
  float acc = 0.f;
  for (int p = 0; p < HW; ++p) {
    int64_t row = (int64_t)b * HW + p;
    float g = ldf(gz, row * ld_gz + o);
    float zz = ldf(z, row * ld_z + o);
    if (zsub) zz -= ldf(zsub, row * ld_zsub + o);  // output had a residual fused in
    float y = zz;
    if (act) {
      if (zz <= 0.f) {
        y = zz * 5.f;  // invert LeakyReLU(0.2)
        g *= 0.2f;
      }
    }
    acc += g * y;
    stf(gyt, row * ld_gyt + o, g * dd);
  }
  // sum_pix gy*y = d * sum_pix gy*ytilde ;  gdd = gd * (-0.5) d^3 with gd = sum gy*ytilde
  gdd[(int64_t)b * Cout + o] = -0.5f * dd * dd * acc;
}

template <typename TG, typename T, typename TO>
__global__ void k_bwd_in(const TG* __restrict__ gxt, int64_t ld_gxt, const T* __restrict__ x, int64_t ld_x,
                         const float* __restrict__ s, int HW, int Cin, TO* __restrict__ gx, int64_t ld_gx,
                         int accumulate, float* __restrict__ gs) {
  int b = blockIdx.x;
  int c = blockIdx.y * blockDim.x + threadIdx.x;
  if (c >= Cin) return;
  float sc = s[(int64_t)b * Cin + c];
  float acc = 0.f;
  for (int p = 0; p < HW; ++p) {
    int64_t row = (int64_t)b * HW + p;
    float g = ldf(gxt, row * ld_gxt + c);
    acc += g * ldf(x, row * ld_x + c);
    if (gx) {
      float v = g * sc;
      if (accumulate) v += ldf(gx, row * ld_gx + c);
      stf(gx, row * ld_gx + c, v);
    }
  }
  gs[(int64_t)b * Cin + c] += acc;
}

// out[b, c] (+)= sum_{p < HW} X[b*HW + p, c]   (per-image column sums)
template <typename T>
__global__ void k_segsum(const T* __restrict__ X, int64_t ld, int HW, int C, float* __restrict__ out) {
  int b = blockIdx.x;
  int c = blockIdx.y * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int p = 0; p < HW; ++p) s += ldf(X, ((int64_t)b * HW + p) * ld + c);
  out[(int64_t)b * C + c] += s;
}

}  // namespace

extern "C" int mg_segsum(int dtype, const void* X, int64_t ld, int B, int HW, int C, float* out, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 grid(B, cdiv(C, 256));
  int thr = std::min(256, ((C + 63) / 64) * 64);
  if (dtype == MG_F32) hipLaunchKernelGGL(k_segsum<float>, grid, dim3(thr), 0, st, (const float*)X, ld, HW, C, out);
  else hipLaunchKernelGGL(k_segsum<bf16_t>, grid, dim3(thr), 0, st, (const bf16_t*)X, ld, HW, C, out);
  return mg_check_launch("mg_segsum");
}

extern "C" int mg_modconv_bwd_out(int dtype, int gz_dtype, const void* gz, int64_t ld_gz, const void* z, int64_t ld_z,
                                  const void* zsub, int64_t ld_zsub, const float* d, int B, int HW, int Cout, int act,
                                  void* gyt, int64_t ld_gyt, float* gdd, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 grid(B, cdiv(Cout, 256));
  int thr = std::min(256, ((Cout + 63) / 64) * 64);
#define L_(T, TG) hipLaunchKernelGGL((k_bwd_out<T, TG>), grid, dim3(thr), 0, st, (const TG*)gz, ld_gz, (const T*)z, \
                                     ld_z, (const T*)zsub, ld_zsub, d, HW, Cout, act, (T*)gyt, ld_gyt, gdd)
  if (dtype == MG_F32) {
    if (gz_dtype == MG_F32) L_(float, float); else L_(float, bf16_t);
  } else {
    if (gz_dtype == MG_F32) L_(bf16_t, float); else L_(bf16_t, bf16_t);
  }
#undef L_
  return mg_check_launch("mg_modconv_bwd_out");
}

extern "C" int mg_modconv_bwd_in(int gxt_dtype, const void* gxt, int64_t ld_gxt, int dtype, const void* x,
                                 int64_t ld_x, const float* s, int B, int HW, int Cin, int gx_dtype, void* gx,
                                 int64_t ld_gx, int accumulate, float* gs, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 grid(B, cdiv(Cin, 256));
  int thr = std::min(256, ((Cin + 63) / 64) * 64);
#define L_(TG, T, TO) hipLaunchKernelGGL((k_bwd_in<TG, T, TO>), grid, dim3(thr), 0, st, (const TG*)gxt, ld_gxt, \
                                         (const T*)x, ld_x, s, HW, Cin, (TO*)gx, ld_gx, accumulate, gs)
  if (dtype == MG_F32) {
    if (gxt_dtype == MG_F32) {
      if (gx_dtype == MG_F32) L_(float, float, float); else L_(float, float, bf16_t);
    } else {
      if (gx_dtype == MG_F32) L_(bf16_t, float, float); else L_(bf16_t, float, bf16_t);
    }
  } else {
    if (gxt_dtype == MG_F32) {
      if (gx_dtype == MG_F32) L_(float, bf16_t, float); else L_(float, bf16_t, bf16_t);
    } else {
      if (gx_dtype == MG_F32) L_(bf16_t, bf16_t, float); else L_(bf16_t, bf16_t, bf16_t);
    }
  }
#undef L_
  return mg_check_launch("mg_modconv_bwd_in");
}
