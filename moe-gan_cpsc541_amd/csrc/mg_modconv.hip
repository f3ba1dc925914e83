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
#include <algorithm>

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
    if (act) {  // act 1: z = LeakyReLU(0.2)(y) (inverted here); act 2: z = y, the stored pre-activation
      if (zz <= 0.f) {
        if (act == 1) y = zz * 5.f;
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
                         const float* __restrict__ s, int64_t ld_s, int HW, int Cin, TO* __restrict__ gx,
                         int64_t ld_gx, int accumulate, float* __restrict__ gs) {
  int b = blockIdx.x;
  int c = blockIdx.y * blockDim.x + threadIdx.x;
  if (c >= Cin) return;
  float sc = s[(int64_t)b * ld_s + c];
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
  gs[(int64_t)b * ld_s + c] += acc;
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

// ---- vectorised forms: 8 channels per thread, pixels split over the block's rows, LDS reduction ----
// block = (C/8) x TY threads for one image b; requires C % 8 == 0, 16-B aligned rows.
template <typename T, typename TG>
__global__ __launch_bounds__(256) void k_bwd_out_v(const TG* __restrict__ gz, int64_t ld_gz, const T* __restrict__ z,
                                                   int64_t ld_z, const T* __restrict__ zsub, int64_t ld_zsub,
                                                   const float* __restrict__ d, int HW, int Cout, int act,
                                                   T* __restrict__ gyt, int64_t ld_gyt, float* __restrict__ gdd) {
  __shared__ __attribute__((aligned(16))) float red[256 * 8];
  const int b = blockIdx.x, tx = threadIdx.x, ty = threadIdx.y, TX = blockDim.x, TY = blockDim.y;
  const int o = (blockIdx.y * TX + tx) * 8;
  const bool live = o < Cout;
  float dd[8], acc[8], g[8], zz[8], t[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  if (live) ld8(d + (int64_t)b * Cout + o, dd);
  // two pixels per iteration with both loads in flight (one block per image: latency-bound otherwise)
  int p = ty;
  for (; live && p + TY < HW; p += 2 * TY) {
    const int64_t r0 = (int64_t)b * HW + p, r1 = r0 + TY;
    float g1[8], z1[8], t1[8];
    ld8(gz + r0 * ld_gz + o, g);
    ld8(gz + r1 * ld_gz + o, g1);
    ld8(z + r0 * ld_z + o, zz);
    ld8(z + r1 * ld_z + o, z1);
    if (zsub) {
      ld8(zsub + r0 * ld_zsub + o, t);
      ld8(zsub + r1 * ld_zsub + o, t1);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        zz[j] -= t[j];
        z1[j] -= t1[j];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float y = zz[j], y1 = z1[j];
      if (act && zz[j] <= 0.f) {
        if (act == 1) y = zz[j] * 5.f;
        g[j] *= 0.2f;
      }
      if (act && z1[j] <= 0.f) {
        if (act == 1) y1 = z1[j] * 5.f;
        g1[j] *= 0.2f;
      }
      acc[j] += g[j] * y;
      acc[j] += g1[j] * y1;
      t[j] = g[j] * dd[j];
      t1[j] = g1[j] * dd[j];
    }
    st8(gyt + r0 * ld_gyt + o, t);
    st8(gyt + r1 * ld_gyt + o, t1);
  }
  for (; live && p < HW; p += TY) {
    int64_t row = (int64_t)b * HW + p;
    ld8(gz + row * ld_gz + o, g);
    ld8(z + row * ld_z + o, zz);
    if (zsub) {
      ld8(zsub + row * ld_zsub + o, t);
#pragma unroll
      for (int j = 0; j < 8; ++j) zz[j] -= t[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float y = zz[j];
      if (act && zz[j] <= 0.f) {
        if (act == 1) y = zz[j] * 5.f;
        g[j] *= 0.2f;
      }
      acc[j] += g[j] * y;
      t[j] = g[j] * dd[j];
    }
    st8(gyt + row * ld_gyt + o, t);
  }
  const int tid = ty * TX + tx;
#pragma unroll
  for (int j = 0; j < 8; j += 4)  // (16-B LDS writes: the 4-B ones at a 32-B lane stride were 8-way bank conflicts)
    *reinterpret_cast<f32x4_t*>(&red[tid * 8 + j]) = f32x4_t{acc[j], acc[j + 1], acc[j + 2], acc[j + 3]};
  __syncthreads();
  if (ty == 0 && live) {
    for (int y = 1; y < TY; ++y)
#pragma unroll
      for (int j = 0; j < 8; j += 4) {
        const f32x4_t v = *reinterpret_cast<const f32x4_t*>(&red[(y * TX + tx) * 8 + j]);
        acc[j] += v[0];
        acc[j + 1] += v[1];
        acc[j + 2] += v[2];
        acc[j + 3] += v[3];
      }
#pragma unroll
    for (int j = 0; j < 8; ++j) gdd[(int64_t)b * Cout + o + j] = -0.5f * dd[j] * dd[j] * acc[j];
  }
}

template <typename TG, typename T, typename TO>
__global__ __launch_bounds__(256) void k_bwd_in_v(const TG* __restrict__ gxt, int64_t ld_gxt, const T* __restrict__ x,
                                                  int64_t ld_x, const float* __restrict__ s, int64_t ld_s, int HW, int Cin,
                                                  TO* __restrict__ gx, int64_t ld_gx, int accumulate,
                                                  float* __restrict__ gs) {
  __shared__ __attribute__((aligned(16))) float red[256 * 8];
  const int b = blockIdx.x, tx = threadIdx.x, ty = threadIdx.y, TX = blockDim.x, TY = blockDim.y;
  const int c = (blockIdx.y * TX + tx) * 8;
  const bool live = c < Cin;
  float sc[8], acc[8], g[8], xx[8], t[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  if (live) ld8(s + (int64_t)b * ld_s + c, sc);
  // pixels split over grid.z (more blocks in flight for few images x large maps)
  const int ppz = (HW + gridDim.z - 1) / gridDim.z, p1 = min(HW, ((int)blockIdx.z + 1) * ppz);
  // two pixels per iteration, all their loads issued before either is used (latency, not bandwidth, bounded
  // the one-pixel loop)
  int p = blockIdx.z * ppz + ty;
  for (; live && p + TY < p1; p += 2 * TY) {
    const int64_t r0 = (int64_t)b * HW + p, r1 = r0 + TY;
    float g1[8], x1[8], t1[8];
    ld8(gxt + r0 * ld_gxt + c, g);
    ld8(gxt + r1 * ld_gxt + c, g1);
    ld8(x + r0 * ld_x + c, xx);
    ld8(x + r1 * ld_x + c, x1);
    if (gx && accumulate) {
      ld8(gx + r0 * ld_gx + c, t);
      ld8(gx + r1 * ld_gx + c, t1);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += g[j] * xx[j];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += g1[j] * x1[j];
    if (gx) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        t[j] = g[j] * sc[j] + (accumulate ? t[j] : 0.f);
        t1[j] = g1[j] * sc[j] + (accumulate ? t1[j] : 0.f);
      }
      st8(gx + r0 * ld_gx + c, t);
      st8(gx + r1 * ld_gx + c, t1);
    }
  }
  for (; live && p < p1; p += TY) {
    int64_t row = (int64_t)b * HW + p;
    ld8(gxt + row * ld_gxt + c, g);
    ld8(x + row * ld_x + c, xx);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += g[j] * xx[j];
    if (gx) {
      if (accumulate) ld8(gx + row * ld_gx + c, t);
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = g[j] * sc[j] + (accumulate ? t[j] : 0.f);
      st8(gx + row * ld_gx + c, t);
    }
  }
  const int tid = ty * TX + tx;
#pragma unroll
  for (int j = 0; j < 8; j += 4)  // (16-B LDS writes: the 4-B ones at a 32-B lane stride were 8-way bank conflicts)
    *reinterpret_cast<f32x4_t*>(&red[tid * 8 + j]) = f32x4_t{acc[j], acc[j + 1], acc[j + 2], acc[j + 3]};
  __syncthreads();
  if (ty == 0 && live) {
    for (int y = 1; y < TY; ++y)
#pragma unroll
      for (int j = 0; j < 8; j += 4) {
        const f32x4_t v = *reinterpret_cast<const f32x4_t*>(&red[(y * TX + tx) * 8 + j]);
        acc[j] += v[0];
        acc[j + 1] += v[1];
        acc[j + 2] += v[2];
        acc[j + 3] += v[3];
      }
    if (gridDim.z > 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) atomicAdd(&gs[(int64_t)b * ld_s + c + j], acc[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) gs[(int64_t)b * ld_s + c + j] += acc[j];
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_segsum_v(const T* __restrict__ X, int64_t ld, int HW, int C,
                                                  float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float red[256 * 8];
  const int b = blockIdx.x, tx = threadIdx.x, ty = threadIdx.y, TX = blockDim.x, TY = blockDim.y;
  const int c = (blockIdx.y * TX + tx) * 8;
  const bool live = c < C;
  float acc[8], t[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  for (int p = ty; live && p < HW; p += TY) {
    ld8(X + ((int64_t)b * HW + p) * ld + c, t);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += t[j];
  }
  const int tid = ty * TX + tx;
#pragma unroll
  for (int j = 0; j < 8; j += 4)  // (16-B LDS writes: the 4-B ones at a 32-B lane stride were 8-way bank conflicts)
    *reinterpret_cast<f32x4_t*>(&red[tid * 8 + j]) = f32x4_t{acc[j], acc[j + 1], acc[j + 2], acc[j + 3]};
  __syncthreads();
  if (ty == 0 && live) {
    for (int y = 1; y < TY; ++y)
#pragma unroll
      for (int j = 0; j < 8; j += 4) {
        const f32x4_t v = *reinterpret_cast<const f32x4_t*>(&red[(y * TX + tx) * 8 + j]);
        acc[j] += v[0];
        acc[j + 1] += v[1];
        acc[j + 2] += v[2];
        acc[j + 3] += v[3];
      }
#pragma unroll
    for (int j = 0; j < 8; ++j) out[(int64_t)b * C + c + j] += acc[j];
  }
}

// xs[b, p, c] = x[b, p, c] * s[b, c]: the modulated-conv input, formed once per forward and shared by
// the forward conv and the weight gradient (instead of re-scaling every tap's operand in the GEMM loaders).
template <typename T>
__global__ __launch_bounds__(256) void k_scale_bc(const T* __restrict__ x, int64_t ldx, const float* __restrict__ s,
                                                  int64_t lds, int HW, int C, int64_t nvec, T* __restrict__ out,
                                                  int64_t ldo) {
  const int cv = C / 8;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    int64_t row = i / cv;
    int c = (int)(i - row * cv) * 8;
    int64_t b = row / HW;
    float v[8], sc[8];
    ld8(x + row * ldx + c, v);
    ld8(s + b * lds + c, sc);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= sc[j];
    st8(out + row * ldo + c, v);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_gather_rows(const T* __restrict__ src, int64_t lds, const int32_t* __restrict__ idx,
                                                     int idx_div, const float* __restrict__ rs, int n, int C,
                                                     T* __restrict__ out, int64_t ldo) {
  const int cv = C / 8;
  const int64_t total = (int64_t)n * cv;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    int r = (int)(i / cv);
    int c = (int)(i - (int64_t)r * cv) * 8;
    float v[8];
    ld8(src + (int64_t)(idx[r] / idx_div) * lds + c, v);
    if (rs) {
      float sc = rs[r];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= sc;
    }
    st8(out + (int64_t)r * ldo + c, v);
  }
}

// block shape for the vectorised per-image reductions: TX = channel vectors, TY = pixel lanes
inline void vshape(int C, dim3& grid, dim3& block, int B) {
  int cv = C / 8;
  int tx = cv < 256 ? cv : 256;
  int ty = 256 / tx;
  block = dim3(tx, ty);
  grid = dim3(B, cdiv(cv, tx));
}

}  // namespace

extern "C" int mg_scale_bc(int dtype, const void* x, int64_t ldx, const float* s, int64_t lds, int B, int HW, int C,
                           void* out, int64_t ldo, void* stream) {
  MG_REQUIRE(dtype == MG_F32 || dtype == MG_BF16, "bad dtype");
  MG_REQUIRE(C % 8 == 0 && ldx % 8 == 0 && ldo % 8 == 0 && lds % 4 == 0, "C and pitches must be multiples of 8");
  MG_REQUIRE(mg_al16(x) && mg_al16(out) && mg_al16(s), "x/out/s must be 16-byte aligned");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t nvec = (int64_t)B * HW * (C / 8);
  if (nvec == 0) return MG_OK;
  int blocks = (int)std::min<int64_t>(cdiv(nvec, 256), 4096);
  if (dtype == MG_F32)
    hipLaunchKernelGGL(k_scale_bc<float>, dim3(blocks), dim3(256), 0, st, (const float*)x, ldx, s, lds, HW, C, nvec,
                       (float*)out, ldo);
  else
    hipLaunchKernelGGL(k_scale_bc<bf16_t>, dim3(blocks), dim3(256), 0, st, (const bf16_t*)x, ldx, s, lds, HW, C, nvec,
                       (bf16_t*)out, ldo);
  return mg_check_launch("mg_scale_bc");
}

extern "C" int mg_gather_rows(int dtype, const void* src, int64_t lds, const int32_t* idx, int idx_div,
                              const float* rowscale, int n, int C, void* out, int64_t ldo, void* stream) {
  MG_REQUIRE(dtype == MG_F32 || dtype == MG_BF16, "bad dtype");
  MG_REQUIRE(C % 8 == 0 && lds % 8 == 0 && ldo % 8 == 0 && idx_div >= 1, "C and pitches must be multiples of 8");
  MG_REQUIRE(mg_al16(src) && mg_al16(out), "src/out must be 16-byte aligned");
  if (n == 0) return MG_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int blocks = (int)std::min<int64_t>(cdiv((int64_t)n * (C / 8), 256), 4096);
  if (dtype == MG_F32)
    hipLaunchKernelGGL(k_gather_rows<float>, dim3(blocks), dim3(256), 0, st, (const float*)src, lds, idx, idx_div,
                       rowscale, n, C, (float*)out, ldo);
  else
    hipLaunchKernelGGL(k_gather_rows<bf16_t>, dim3(blocks), dim3(256), 0, st, (const bf16_t*)src, lds, idx, idx_div,
                       rowscale, n, C, (bf16_t*)out, ldo);
  return mg_check_launch("mg_gather_rows");
}

extern "C" int mg_segsum(int dtype, const void* X, int64_t ld, int B, int HW, int C, float* out, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (C % 8 == 0 && ld % 8 == 0 && mg_al16(X) && mg_al16(out)) {
    dim3 g2, b2;
    vshape(C, g2, b2, B);
    if (dtype == MG_F32) hipLaunchKernelGGL(k_segsum_v<float>, g2, b2, 0, st, (const float*)X, ld, HW, C, out);
    else hipLaunchKernelGGL(k_segsum_v<bf16_t>, g2, b2, 0, st, (const bf16_t*)X, ld, HW, C, out);
    return mg_check_launch("mg_segsum");
  }
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
  dim3 blk(std::min(256, ((Cout + 63) / 64) * 64));
  bool vec = Cout % 8 == 0 && ld_gz % 8 == 0 && ld_z % 8 == 0 && ld_gyt % 8 == 0 && (!zsub || ld_zsub % 8 == 0) &&
             mg_al16(gz) && mg_al16(z) && mg_al16(gyt) && mg_al16(d) && (!zsub || mg_al16(zsub)) && mg_al16(gdd);
  if (vec) {
    vshape(Cout, grid, blk, B);
#define L_(T, TG) hipLaunchKernelGGL((k_bwd_out_v<T, TG>), grid, blk, 0, st, (const TG*)gz, ld_gz, (const T*)z, \
                                     ld_z, (const T*)zsub, ld_zsub, d, HW, Cout, act, (T*)gyt, ld_gyt, gdd)
    if (dtype == MG_F32) {
      if (gz_dtype == MG_F32) L_(float, float); else L_(float, bf16_t);
    } else {
      if (gz_dtype == MG_F32) L_(bf16_t, float); else L_(bf16_t, bf16_t);
    }
#undef L_
    return mg_check_launch("mg_modconv_bwd_out");
  }
  int thr = blk.x;
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
                                 int64_t ld_x, const float* s, int64_t ld_s, int B, int HW, int Cin, int gx_dtype,
                                 void* gx, int64_t ld_gx, int accumulate, float* gs, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 grid(B, cdiv(Cin, 256));
  dim3 blk(std::min(256, ((Cin + 63) / 64) * 64));
  bool vec = Cin % 8 == 0 && ld_gxt % 8 == 0 && ld_x % 8 == 0 && (!gx || ld_gx % 8 == 0) && ld_s % 4 == 0 &&
             mg_al16(gxt) && mg_al16(x) && mg_al16(s) && (!gx || mg_al16(gx)) && mg_al16(gs);
  int thr = blk.x;
  if (vec) {
    vshape(Cin, grid, blk, B);
    grid.z = std::max(1, std::min(cdiv(HW, (int)blk.y * 4), cdiv(1024, (int)(grid.x * grid.y))));
    if (mg_det()) grid.z = 1;  // deterministic mode: one writer per style-gradient element (no z-split atomics)
  }
#define L_(TG, T, TO)                                                                                              \
  do {                                                                                                             \
    if (vec)                                                                                                       \
      hipLaunchKernelGGL((k_bwd_in_v<TG, T, TO>), grid, blk, 0, st, (const TG*)gxt, ld_gxt, (const T*)x, ld_x, s, \
                         ld_s, HW, Cin, (TO*)gx, ld_gx, accumulate, gs);                                           \
    else                                                                                                           \
      hipLaunchKernelGGL((k_bwd_in<TG, T, TO>), grid, dim3(thr), 0, st, (const TG*)gxt, ld_gxt, \
                                         (const T*)x, ld_x, s, ld_s, HW, Cin, (TO*)gx, ld_gx, accumulate, gs); \
  } while (0)
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
