// Modulated Transformation Module warp (t2i_moe_gan.py:218-239) and the
// bilinear x2 upsample of GenerativeBlock (t2i_moe_gan.py:633, 657-658).  NHWC.
//
// Warp forward, one wave per output pixel:
//   off = conv3x3(o1, w2) + b2         (offset_net's second conv, 32 -> 2, fused)
//   grid = linspace grid + 0.05 * off, clamp(-1, 1)
//   out = grid_sample(x, grid, bilinear, zeros, align_corners=False)
// The sample coordinates and clamp masks are saved for the backward, which
// scatters dL/dx with fp32 atomics (256-B contiguous per wave instruction) and
// reduces dL/dgrid across the wave.
#include "mg_common.h"

namespace {

// torch.linspace(-1, 1, n)[i] (symmetric evaluation, as ATen does)
MG_DEV float linspace_pm1(int i, int n) {
  if (n == 1) return -1.f;
  float step = 2.f / (float)(n - 1);
  return (i < n / 2) ? (-1.f + step * (float)i) : (1.f - step * (float)(n - 1 - i));
}

template <typename T>
__global__ void k_warp_fwd(const T* __restrict__ x, const T* __restrict__ o1, const float* __restrict__ w2,
                           const float* __restrict__ b2, int B, int H, int W, int C, T* __restrict__ out,
                           float* __restrict__ samp) {
  int lane = threadIdx.x & 63;
  int64_t p = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (p >= (int64_t)B * H * W) return;
  int b = (int)(p / (H * W));
  int rem = (int)(p - (int64_t)b * H * W);
  int h = rem / W, w = rem - (rem / W) * W;
  // offset conv 32 -> 2 (3x3, pad 1): lanes split the 288 (tap, channel) products
  float s0 = 0.f, s1 = 0.f;
  for (int i = lane; i < 288; i += 64) {
    int tap = i >> 5, c = i & 31;
    int kh = tap / 3, kw = tap - kh * 3;
    int yy = h + kh - 1, xx = w + kw - 1;
    if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
      float v = ldf(o1, (((int64_t)b * H + yy) * W + xx) * 32 + c);
      s0 += v * w2[(0 * 32 + c) * 9 + tap];
      s1 += v * w2[(1 * 32 + c) * 9 + tap];
    }
  }
  s0 = wave_sum(s0) + b2[0];
  s1 = wave_sum(s1) + b2[1];
  float gx = linspace_pm1(w, W) + s0 * 0.05f;
  float gy = linspace_pm1(h, H) + s1 * 0.05f;
  float mx = (gx >= -1.f && gx <= 1.f) ? 1.f : 0.f;
  float my = (gy >= -1.f && gy <= 1.f) ? 1.f : 0.f;
  gx = fminf(fmaxf(gx, -1.f), 1.f);
  gy = fminf(fmaxf(gy, -1.f), 1.f);
  float ix = ((gx + 1.f) * W - 1.f) * 0.5f;
  float iy = ((gy + 1.f) * H - 1.f) * 0.5f;
  if (lane == 0) {
    samp[p * 4 + 0] = ix;
    samp[p * 4 + 1] = iy;
    samp[p * 4 + 2] = mx;
    samp[p * 4 + 3] = my;
  }
  int x0 = (int)floorf(ix), y0 = (int)floorf(iy);
  int x1 = x0 + 1, y1 = y0 + 1;
  float wnw = ((float)x1 - ix) * ((float)y1 - iy);
  float wne = (ix - (float)x0) * ((float)y1 - iy);
  float wsw = ((float)x1 - ix) * (iy - (float)y0);
  float wse = (ix - (float)x0) * (iy - (float)y0);
  bool vx0 = x0 >= 0 && x0 < W, vx1 = x1 >= 0 && x1 < W, vy0 = y0 >= 0 && y0 < H, vy1 = y1 >= 0 && y1 < H;
  const T* xb = x + (int64_t)b * H * W * C;
  for (int c = lane; c < C; c += 64) {
    float v = 0.f;
    if (vy0 && vx0) v += wnw * ldf(xb, ((int64_t)y0 * W + x0) * C + c);
    if (vy0 && vx1) v += wne * ldf(xb, ((int64_t)y0 * W + x1) * C + c);
    if (vy1 && vx0) v += wsw * ldf(xb, ((int64_t)y1 * W + x0) * C + c);
    if (vy1 && vx1) v += wse * ldf(xb, ((int64_t)y1 * W + x1) * C + c);
    stf(out, p * C + c, v);
  }
}

// Vectorised warp forward: one 16-B channel vector per thread, G = C / VEC threads per output pixel
// (contiguous lanes), 256 / G pixels per block.  The pixel's G threads split the 9 taps x 32 channels of
// the offset conv, reduce (s0, s1) with lane shuffles, then each gathers the 4 bilinear taps of its own
// channel vector with 16-B loads and stores 16 B.  Same math as k_warp_fwd.
template <typename T>
__global__ __launch_bounds__(256) void k_warp_fwd_v(const T* __restrict__ x, const T* __restrict__ o1,
                                                    const float* __restrict__ w2, const float* __restrict__ b2,
                                                    int B, int H, int W, int C, int lgG, T* __restrict__ out,
                                                    float* __restrict__ samp, const float* __restrict__ sc,
                                                    int64_t lds, T* __restrict__ xs) {
  constexpr int VEC = VecOf<T>::N;
  typedef typename VecOf<T>::type vec_t;
  constexpr int OV = 32 / VEC;  // offset-conv input vectors per tap
  // offset-conv weights as [v][NQ] float4s, v = tap * OV + c / VEC (one input vector), float4 k = (e = 2k, j = 0),
  // (2k, 1), (2k + 1, 0), (2k + 1, 1); chunk k of v stored at slot (k + v / 4) mod NQ, so the 16 distinct vectors a
  // lane group reads with one ds_read_b128 cover 64 distinct banks (the scalar [tap][c][j] reads were 8-way)
  constexpr int NQ = VEC / 2;
  __shared__ f32x4_t sw4[9 * OV * NQ];
  float* swf = reinterpret_cast<float*>(sw4);
  for (int i = threadIdx.x; i < 576; i += 256) {
    const int j = i / 288, c = (i / 9) % 32, tap = i % 9;
    const int v = tap * OV + c / VEC, e = c % VEC;
    swf[(v * NQ + (((e >> 1) + (v >> 2)) & (NQ - 1))) * 4 + (e & 1) * 2 + j] = w2[i];
  }
  __syncthreads();
  const int G = 1 << lgG;
  const int g = threadIdx.x & (G - 1);
  const int64_t p = (int64_t)blockIdx.x * (256 >> lgG) + (threadIdx.x >> lgG);
  const int64_t P = (int64_t)B * H * W;
  const bool live = p < P;
  const int64_t pp = live ? p : 0;
  const int b = (int)(pp / (H * W));
  const int rem = (int)(pp - (int64_t)b * H * W);
  const int h = rem / W, w = rem - (rem / W) * W;
  float s0 = 0.f, s1 = 0.f;
  for (int v = g; v < 9 * OV; v += G) {
    const int tap = v / OV, c0 = (v - tap * OV) * VEC;
    const int kh = tap / 3, kw = tap - kh * 3;
    const int yy = h + kh - 1, xx = w + kw - 1;
    if (live && yy >= 0 && yy < H && xx >= 0 && xx < W) {
      float t[VEC];
      const vec_t raw = *reinterpret_cast<const vec_t*>(o1 + (((int64_t)b * H + yy) * W + xx) * 32 + c0);
#pragma unroll
      for (int e = 0; e < VEC; ++e) t[e] = sizeof(T) == 2 ? bf2f((bf16_t)raw[e]) : (float)raw[e];
#pragma unroll
      for (int k = 0; k < NQ; ++k) {  // (the e order of the scalar form: bit-identical sums)
        const f32x4_t q = sw4[v * NQ + ((k + (v >> 2)) & (NQ - 1))];
        s0 += t[2 * k] * q[0];
        s1 += t[2 * k] * q[1];
        s0 += t[2 * k + 1] * q[2];
        s1 += t[2 * k + 1] * q[3];
      }
    }
  }
  for (int o = G >> 1; o > 0; o >>= 1) {
    s0 += __shfl_xor(s0, o, 64);
    s1 += __shfl_xor(s1, o, 64);
  }
  if (!live) return;
  s0 += b2[0];
  s1 += b2[1];
  float gx = linspace_pm1(w, W) + s0 * 0.05f;
  float gy = linspace_pm1(h, H) + s1 * 0.05f;
  const float mx = (gx >= -1.f && gx <= 1.f) ? 1.f : 0.f;
  const float my = (gy >= -1.f && gy <= 1.f) ? 1.f : 0.f;
  gx = fminf(fmaxf(gx, -1.f), 1.f);
  gy = fminf(fmaxf(gy, -1.f), 1.f);
  const float ix = ((gx + 1.f) * W - 1.f) * 0.5f;
  const float iy = ((gy + 1.f) * H - 1.f) * 0.5f;
  if (g == 0) *reinterpret_cast<f32x4_t*>(samp + p * 4) = f32x4_t{ix, iy, mx, my};
  const int x0 = (int)floorf(ix), y0 = (int)floorf(iy);
  const int x1 = x0 + 1, y1 = y0 + 1;
  const float wnw = ((float)x1 - ix) * ((float)y1 - iy);
  const float wne = (ix - (float)x0) * ((float)y1 - iy);
  const float wsw = ((float)x1 - ix) * (iy - (float)y0);
  const float wse = (ix - (float)x0) * (iy - (float)y0);
  const bool vx0 = x0 >= 0 && x0 < W, vx1 = x1 >= 0 && x1 < W, vy0 = y0 >= 0 && y0 < H, vy1 = y1 >= 0 && y1 < H;
  const T* xb = x + (int64_t)b * H * W * C;
  for (int c = g * VEC; c < C; c += G * VEC) {
    float acc[VEC], t[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) acc[e] = 0.f;
    auto tap = [&](bool ok, int yy, int xx, float wt) {
      if (!ok) return;
      const vec_t raw = *reinterpret_cast<const vec_t*>(xb + ((int64_t)yy * W + xx) * C + c);
#pragma unroll
      for (int e = 0; e < VEC; ++e) t[e] = sizeof(T) == 2 ? bf2f((bf16_t)raw[e]) : (float)raw[e];
#pragma unroll
      for (int e = 0; e < VEC; ++e) acc[e] += wt * t[e];
    };
    tap(vy0 && vx0, y0, x0, wnw);
    tap(vy0 && vx1, y0, x1, wne);
    tap(vy1 && vx0, y1, x0, wsw);
    tap(vy1 && vx1, y1, x1, wse);
    vec_t r;
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      if constexpr (sizeof(T) == 2) r[e] = f2bf(acc[e]);
      else r[e] = acc[e];
    }
    *reinterpret_cast<vec_t*>(out + p * C + c) = r;
    if (xs) {  // the next modulated conv's prescaled input, from the stored (rounded) value as mg_scale_bc does
      const float* sp = sc + (int64_t)b * lds + c;
      vec_t r2;
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const float v = (sizeof(T) == 2 ? bf2f((bf16_t)r[e]) : (float)r[e]) * sp[e];
        if constexpr (sizeof(T) == 2) r2[e] = f2bf(v);
        else r2[e] = v;
      }
      *reinterpret_cast<vec_t*>(xs + p * C + c) = r2;
    }
  }
}

template <typename T, typename TG>
__global__ void k_warp_bwd(const TG* __restrict__ gout, const T* __restrict__ x, const float* __restrict__ samp,
                           int B, int H, int W, int C, float* __restrict__ gx, float* __restrict__ goff) {
  int lane = threadIdx.x & 63;
  int64_t p = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (p >= (int64_t)B * H * W) return;
  int b = (int)(p / (H * W));
  float ix = samp[p * 4 + 0], iy = samp[p * 4 + 1], mx = samp[p * 4 + 2], my = samp[p * 4 + 3];
  int x0 = (int)floorf(ix), y0 = (int)floorf(iy);
  int x1 = x0 + 1, y1 = y0 + 1;
  float ax1 = (float)x1 - ix, ax0 = ix - (float)x0, ay1 = (float)y1 - iy, ay0 = iy - (float)y0;
  float wnw = ax1 * ay1, wne = ax0 * ay1, wsw = ax1 * ay0, wse = ax0 * ay0;
  bool vx0 = x0 >= 0 && x0 < W, vx1 = x1 >= 0 && x1 < W, vy0 = y0 >= 0 && y0 < H, vy1 = y1 >= 0 && y1 < H;
  const T* xb = x + (int64_t)b * H * W * C;
  float* gb = gx + (int64_t)b * H * W * C;
  float gix = 0.f, giy = 0.f;
  for (int c = lane; c < C; c += 64) {
    float g = ldf(gout, p * C + c);
    float vnw = 0.f, vne = 0.f, vsw = 0.f, vse = 0.f;
    if (vy0 && vx0) {
      int64_t o = ((int64_t)y0 * W + x0) * C + c;
      vnw = ldf(xb, o);
      atomicAdd(gb + o, wnw * g);
    }
    if (vy0 && vx1) {
      int64_t o = ((int64_t)y0 * W + x1) * C + c;
      vne = ldf(xb, o);
      atomicAdd(gb + o, wne * g);
    }
    if (vy1 && vx0) {
      int64_t o = ((int64_t)y1 * W + x0) * C + c;
      vsw = ldf(xb, o);
      atomicAdd(gb + o, wsw * g);
    }
    if (vy1 && vx1) {
      int64_t o = ((int64_t)y1 * W + x1) * C + c;
      vse = ldf(xb, o);
      atomicAdd(gb + o, wse * g);
    }
    // neighbour differences per channel before the channel sum (see k_mtm_bwd_img)
    gix += g * ((vne - vnw) * ay1 + (vse - vsw) * ay0);
    giy += g * ((vsw - vnw) * ax1 + (vse - vne) * ax0);
  }
  gix = wave_sum(gix);
  giy = wave_sum(giy);
  if (lane == 0) {
    goff[p * 2 + 0] = gix * (0.5f * W) * mx * 0.05f;
    goff[p * 2 + 1] = giy * (0.5f * H) * my * 0.05f;
  }
}

// Warp backward for images of at most 256 pixels: one block per (image, 64-channel chunk) owns that slice
// of dL/dx, so the bilinear scatter accumulates in LDS (ds_add_f32, lane = channel: conflict-free) and is
// added to gx once with plain stores -- instead of four global fp32 atomics per element.  dL/dgrid is
// reduced across the wave per pixel and added to goff (zeroed by the launcher) with one atomic per chunk.
template <typename T, typename TG>
__global__ __launch_bounds__(512) void k_warp_bwd_lds(const TG* __restrict__ gout, const T* __restrict__ x,
                                                      const float* __restrict__ samp, int B, int H, int W, int C,
                                                      float* __restrict__ gx, float* __restrict__ goff) {
  extern __shared__ float acc[];  // [H*W][64]
  const int b = blockIdx.x, c0 = blockIdx.y * 64;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int HW = H * W;
  for (int i = threadIdx.x; i < HW * 64; i += blockDim.x) acc[i] = 0.f;
  __syncthreads();
  const T* xb = x + (int64_t)b * HW * C + c0 + lane;
  for (int q = wv; q < HW; q += nw) {
    const int64_t p = (int64_t)b * HW + q;
    const f32x4_t sp = *reinterpret_cast<const f32x4_t*>(samp + p * 4);
    const float ix = sp[0], iy = sp[1], mx = sp[2], my = sp[3];
    const int x0 = (int)floorf(ix), y0 = (int)floorf(iy);
    const int x1 = x0 + 1, y1 = y0 + 1;
    const float ax1 = (float)x1 - ix, ax0 = ix - (float)x0, ay1 = (float)y1 - iy, ay0 = iy - (float)y0;
    const bool vx0 = x0 >= 0 && x0 < W, vx1 = x1 >= 0 && x1 < W, vy0 = y0 >= 0 && y0 < H, vy1 = y1 >= 0 && y1 < H;
    const float g = ldf(gout, p * C + c0 + lane);
    float vnw = 0.f, vne = 0.f, vsw = 0.f, vse = 0.f;
    if (vy0 && vx0) {
      const int o = y0 * W + x0;
      vnw = ldf(xb, (int64_t)o * C);
      atomicAdd(&acc[o * 64 + lane], ax1 * ay1 * g);
    }
    if (vy0 && vx1) {
      const int o = y0 * W + x1;
      vne = ldf(xb, (int64_t)o * C);
      atomicAdd(&acc[o * 64 + lane], ax0 * ay1 * g);
    }
    if (vy1 && vx0) {
      const int o = y1 * W + x0;
      vsw = ldf(xb, (int64_t)o * C);
      atomicAdd(&acc[o * 64 + lane], ax1 * ay0 * g);
    }
    if (vy1 && vx1) {
      const int o = y1 * W + x1;
      vse = ldf(xb, (int64_t)o * C);
      atomicAdd(&acc[o * 64 + lane], ax0 * ay0 * g);
    }
    float gix = g * ((vne - vnw) * ay1 + (vse - vsw) * ay0);  // neighbour differences first (see k_mtm_bwd_img)
    float giy = g * ((vsw - vnw) * ax1 + (vse - vne) * ax0);
    gix = wave_sum(gix);
    giy = wave_sum(giy);
    if (lane == 0) {
      atomicAdd(&goff[p * 2 + 0], gix * (0.5f * W) * mx * 0.05f);
      atomicAdd(&goff[p * 2 + 1], giy * (0.5f * H) * my * 0.05f);
    }
  }
  __syncthreads();
  float* gb = gx + (int64_t)b * HW * C + c0;
  for (int i = threadIdx.x; i < HW * 64; i += blockDim.x) {
    const int q = i >> 6, l = i & 63;
    gb[(int64_t)q * C + l] += acc[i];
  }
}

// offset_net second conv backward (32 -> 2, 3x3, pad 1) fused with the first conv's LeakyReLU:
//   g_a1[q, c] = lrelu'(o1[q,c]) * sum_{j,kh,kw} goff[q - (kh-1, kw-1), j] * w2[j, c, kh, kw]
//   gw2[j, c, kh, kw] += sum_q goff[q - (kh-1,kw-1), j] * o1[q, c];  gb2[j] += sum_p goff[p, j]
template <typename T>
__global__ void k_offset_head_bwd(const float* __restrict__ goff, const T* __restrict__ o1,
                                  const float* __restrict__ w2, int B, int H, int W, int ppb, T* __restrict__ ga1,
                                  float* __restrict__ gw2, float* __restrict__ gb2) {
  __shared__ float sw[576];
  __shared__ float red[576 + 2];
  for (int i = threadIdx.x; i < 576; i += blockDim.x) {
    sw[i] = w2[i];
    red[i] = 0.f;
  }
  if (threadIdx.x < 2) red[576 + threadIdx.x] = 0.f;
  __syncthreads();
  int c = threadIdx.x & 31, pl = threadIdx.x >> 5;  // 8 pixel lanes
  int64_t P = (int64_t)B * H * W;
  float accw[18];
#pragma unroll
  for (int i = 0; i < 18; ++i) accw[i] = 0.f;
  float accb0 = 0.f, accb1 = 0.f;
  for (int it = pl; it < ppb; it += 8) {
    int64_t q = (int64_t)blockIdx.x * ppb + it;
    if (q >= P) break;
    int b = (int)(q / (H * W));
    int rem = (int)(q - (int64_t)b * H * W);
    int h = rem / W, w = rem - (rem / W) * W;
    float ov = ldf(o1, q * 32 + c);
    float g = 0.f;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      int kh = tap / 3, kw = tap % 3;
      int yy = h - (kh - 1), xx = w - (kw - 1);  // output pixel p that reads q through this tap
      if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
        int64_t pp = ((int64_t)b * H + yy) * W + xx;
        float g0 = goff[pp * 2], g1 = goff[pp * 2 + 1];
        g += g0 * sw[c * 9 + tap] + g1 * sw[(32 + c) * 9 + tap];
        accw[tap] += g0 * ov;
        accw[9 + tap] += g1 * ov;
      }
    }
    stf(ga1, q * 32 + c, ov > 0.f ? g : 0.2f * g);
    if (c == 0) {
      accb0 += goff[q * 2];
      accb1 += goff[q * 2 + 1];
    }
  }
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    atomicAdd(&red[c * 9 + tap], accw[tap]);
    atomicAdd(&red[(32 + c) * 9 + tap], accw[9 + tap]);
  }
  if (c == 0) {
    atomicAdd(&red[576], accb0);
    atomicAdd(&red[577], accb1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 578; i += blockDim.x) {
    if (i < 576) atomicAdd(&gw2[i], red[i]);
    else atomicAdd(&gb2[i - 576], red[i]);
  }
}

// Offset-head backward for images of at most 256 pixels: a block owns 256 consecutive pixels (whole
// images), stages their goff in LDS (every in-image 3x3 neighbour is inside the block), and writes its
// (gw2, gb2) partial sums to a workspace row instead of same-address global atomics; k_offset_head_fin
// reduces the rows.  Same math as k_offset_head_bwd.
template <typename T>
__global__ __launch_bounds__(256) void k_offset_head_bwd_blk(const float* __restrict__ goff, const T* __restrict__ o1,
                                                             const float* __restrict__ w2, int B, int H, int W,
                                                             T* __restrict__ ga1, float* __restrict__ part) {
  __shared__ float sw[576];
  __shared__ float red[578];
  __shared__ float sg[256 * 2];
  const int64_t P = (int64_t)B * H * W;
  const int64_t q0 = (int64_t)blockIdx.x * 256;
  for (int i = threadIdx.x; i < 578; i += 256) {
    if (i < 576) sw[i] = w2[i];
    red[i] = 0.f;
  }
  for (int i = threadIdx.x; i < 512; i += 256) sg[i] = (q0 * 2 + i < P * 2) ? goff[q0 * 2 + i] : 0.f;
  __syncthreads();
  const int c = threadIdx.x & 31, pl = threadIdx.x >> 5;
  float accw[18];
#pragma unroll
  for (int i = 0; i < 18; ++i) accw[i] = 0.f;
  float accb0 = 0.f, accb1 = 0.f;
  for (int it = pl; it < 256; it += 8) {
    const int64_t q = q0 + it;
    if (q >= P) break;
    const int b = (int)(q / (H * W));
    const int rem = (int)(q - (int64_t)b * H * W);
    const int h = rem / W, w = rem - (rem / W) * W;
    const float ov = ldf(o1, q * 32 + c);
    float g = 0.f;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int kh = tap / 3, kw = tap % 3;
      const int yy = h - (kh - 1), xx = w - (kw - 1);  // output pixel that reads q through this tap
      if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
        const int lp = it + (yy - h) * W + (xx - w);  // same image: inside this block
        const float g0 = sg[lp * 2], g1 = sg[lp * 2 + 1];
        g += g0 * sw[c * 9 + tap] + g1 * sw[(32 + c) * 9 + tap];
        accw[tap] += g0 * ov;
        accw[9 + tap] += g1 * ov;
      }
    }
    stf(ga1, q * 32 + c, ov > 0.f ? g : 0.2f * g);
    if (c == 0) {
      accb0 += sg[it * 2];
      accb1 += sg[it * 2 + 1];
    }
  }
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    atomicAdd(&red[c * 9 + tap], accw[tap]);
    atomicAdd(&red[(32 + c) * 9 + tap], accw[9 + tap]);
  }
  if (c == 0) {
    atomicAdd(&red[576], accb0);
    atomicAdd(&red[577], accb1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 578; i += 256) part[(int64_t)blockIdx.x * 578 + i] = red[i];
}

__global__ __launch_bounds__(256) void k_offset_head_fin(const float* __restrict__ part, int nblk,
                                                         float* __restrict__ gw2, float* __restrict__ gb2) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= 578) return;
  float s = 0.f;
  for (int r = 0; r < nblk; ++r) s += part[(int64_t)r * 578 + i];
  if (i < 576) gw2[i] += s;
  else gb2[i - 576] += s;
}

// bilinear x2 source index (align_corners=False, scale 0.5): clamped at 0
MG_DEV void src_idx(int o, int in_size, int& i0, int& i1, float& l1) {
  float s = fmaxf(((float)o + 0.5f) * 0.5f - 0.5f, 0.f);
  i0 = (int)s;
  i1 = min(i0 + 1, in_size - 1);
  l1 = s - (float)i0;
}

template <typename T>
__global__ void k_up2_fwd(const T* __restrict__ x, int B, int H, int W, int C, T* __restrict__ out) {
  int OH = 2 * H, OW = 2 * W;
  int64_t n = (int64_t)B * OH * OW * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int c = (int)(i % C);
    int64_t pix = i / C;
    int ox = (int)(pix % OW);
    int oy = (int)((pix / OW) % OH);
    int b = (int)(pix / ((int64_t)OW * OH));
    int y0, y1, x0, x1;
    float ly, lx;
    src_idx(oy, H, y0, y1, ly);
    src_idx(ox, W, x0, x1, lx);
    const T* xb = x + (int64_t)b * H * W * C + c;
    float v = (1.f - ly) * ((1.f - lx) * ldf(xb, ((int64_t)y0 * W + x0) * C) + lx * ldf(xb, ((int64_t)y0 * W + x1) * C)) +
              ly * ((1.f - lx) * ldf(xb, ((int64_t)y1 * W + x0) * C) + lx * ldf(xb, ((int64_t)y1 * W + x1) * C));
    stf(out, i, v);
  }
}

// 8-channel vector forms (C % 8 == 0); same arithmetic order as the scalar kernels
// XS: also x * s for the block's 1x1 skip modulated conv (t2i_moe_gan.py:158-161, :615-616), s [B, C], formed from the
// stored (rounded) upsampled value as k_scale_bc would
template <typename T, bool XS = false>
__global__ __launch_bounds__(256) void k_up2_fwd_v(const T* __restrict__ x, int B, int H, int W, int C,
                                                   T* __restrict__ out, const float* __restrict__ sty = nullptr,
                                                   int64_t ld_sty = 0, T* __restrict__ xs = nullptr) {
  const int OH = 2 * H, OW = 2 * W, cv = C >> 3;
  const int n = B * OH * OW * cv;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    int c = (i % cv) * 8;
    int pix = i / cv;
    int ox = pix % OW, t = pix / OW, oy = t % OH, b = t / OH;
    int y0, y1, x0, x1;
    float ly, lx;
    src_idx(oy, H, y0, y1, ly);
    src_idx(ox, W, x0, x1, lx);
    const T* xb = x + (int64_t)b * H * W * C + c;
    float a[8], bb[8], cc[8], dd[8], v[8];
    ld8(xb + (y0 * W + x0) * C, a);
    ld8(xb + (y0 * W + x1) * C, bb);
    ld8(xb + (y1 * W + x0) * C, cc);
    ld8(xb + (y1 * W + x1) * C, dd);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      v[j] = (1.f - ly) * ((1.f - lx) * a[j] + lx * bb[j]) + ly * ((1.f - lx) * cc[j] + lx * dd[j]);
    st8(out + (int64_t)pix * C + c, v);
    if constexpr (XS) {
      float sc[8];
      ld8(sty + (int64_t)b * ld_sty + c, sc);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if constexpr (sizeof(T) == 2) v[j] = bf2f(f2bf(v[j]));
        v[j] *= sc[j];
      }
      st8(xs + (int64_t)pix * C + c, v);
    }
  }
}

template <typename TG, typename T>
__global__ __launch_bounds__(256) void k_up2_bwd_v(const TG* __restrict__ gout, int B, int H, int W, int C,
                                                   T* __restrict__ gx, int accumulate) {
  const int OH = 2 * H, OW = 2 * W, cv = C >> 3;
  const int n = B * H * W * cv;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    int c = (i % cv) * 8;
    int pix = i / cv;
    int ix = pix % W, t = pix / W, iy = t % H, b = t / H;
    float s[8], g[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] = 0.f;
    for (int oy = max(0, 2 * iy - 2); oy <= min(OH - 1, 2 * iy + 2); ++oy) {
      int y0, y1;
      float ly;
      src_idx(oy, H, y0, y1, ly);
      float wy = (y0 == iy ? 1.f - ly : 0.f) + (y1 == iy ? ly : 0.f);
      if (wy == 0.f) continue;
      for (int ox = max(0, 2 * ix - 2); ox <= min(OW - 1, 2 * ix + 2); ++ox) {
        int x0, x1;
        float lx;
        src_idx(ox, W, x0, x1, lx);
        float wx = (x0 == ix ? 1.f - lx : 0.f) + (x1 == ix ? lx : 0.f);
        if (wx == 0.f) continue;
        ld8(gout + (((int64_t)b * OH + oy) * OW + ox) * C + c, g);
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += wy * wx * g[j];
      }
    }
    T* dst = gx + (int64_t)pix * C + c;
    if (accumulate) {
      ld8(dst, g);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += g[j];
    }
    st8(dst, s);
  }
}

template <typename TG, typename T>
__global__ void k_up2_bwd(const TG* __restrict__ gout, int B, int H, int W, int C, T* __restrict__ gx,
                          int accumulate) {
  int OH = 2 * H, OW = 2 * W;
  int64_t n = (int64_t)B * H * W * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int c = (int)(i % C);
    int64_t pix = i / C;
    int ix = (int)(pix % W);
    int iy = (int)((pix / W) % H);
    int b = (int)(pix / ((int64_t)W * H));
    float s = 0.f;
    for (int oy = max(0, 2 * iy - 2); oy <= min(OH - 1, 2 * iy + 2); ++oy) {
      int y0, y1;
      float ly;
      src_idx(oy, H, y0, y1, ly);
      float wy = (y0 == iy ? 1.f - ly : 0.f) + (y1 == iy ? ly : 0.f);
      if (wy == 0.f) continue;
      for (int ox = max(0, 2 * ix - 2); ox <= min(OW - 1, 2 * ix + 2); ++ox) {
        int x0, x1;
        float lx;
        src_idx(ox, W, x0, x1, lx);
        float wx = (x0 == ix ? 1.f - lx : 0.f) + (x1 == ix ? lx : 0.f);
        if (wx == 0.f) continue;
        s += wy * wx * ldf(gout, (((int64_t)b * OH + oy) * OW + ox) * C + c);
      }
    }
    if (accumulate) s += ldf(gx, i);
    stf(gx, i, s);
  }
}

inline int nblk(int64_t n, int t = 256) { return (int)std::min<int64_t>((n + t - 1) / t, 65536); }


// Fused MTM backward for images of at most 1024 pixels, one 1024-thread block per image: grid_sample's data
// gradient as a GATHER instead of a scatter, then the offset head's backward from the image's dL/doffsets held
// in LDS (t2i_moe_gan.py:222-239 backward).
//  1. every output pixel p registers itself with the (up to 4) in-image source pixels q its bilinear sample
//     touches (LDS atomics give the slot), a block scan turns the counts into a CSR list per q;
//  2. items (pixel, 8-channel vector): gx[q] = sum over q's list of w(p->q) * gout[p]  (16-B loads, one plain
//     store: no fp32 atomics, no zero fill, optional accumulate into gx), and dL/dgrid of p = dot products of
//     gout[p] with x at its corners, reduced over the pixel's C/8 vector lanes with shuffles;
//  3. offset head (32 -> 2 conv, 3x3) backward fused with the first conv's LeakyReLU: ga1 for the image, and
//     the image's partial (gw2, gb2) row written to a workspace row (folded over images by a rows fold, mg_fold.hip).
template <typename T, typename TG, typename TX>
__global__ __launch_bounds__(1024) void k_mtm_bwd_img(const TG* __restrict__ gout, const T* __restrict__ x,
                                                      const float* __restrict__ samp, const T* __restrict__ o1,
                                                      const float* __restrict__ w2, int H, int W, int C, int lgV,
                                                      TX* __restrict__ gx, int accumulate, T* __restrict__ ga1,
                                                      float* __restrict__ part) {
  extern __shared__ float smem[];
  const int HW = H * W, tid = threadIdx.x, nt = blockDim.x;
  const int b = blockIdx.x;
  f32x4_t* sinf = reinterpret_cast<f32x4_t*>(smem);   // [HW] (ix, iy, mx, my)
  float* sgo = smem + 4 * HW;                          // [HW][2] dL/doffsets
  float* sw = sgo + 2 * HW;                            // [576] offset_net.2 weight
  float* red = sw + 576;                               // [578] (gw2, gb2) partials
  int* cnt = reinterpret_cast<int*>(red + 578);        // [HW + 1] counts -> CSR offsets
  int* slot = cnt + HW + 1;                            // [4 HW] slot of (p, corner) in q's list, -1 = none
  int* ent = slot + 4 * HW;                            // [4 HW] p * 4 + corner
  const int64_t row0 = (int64_t)b * HW;
  for (int i = tid; i <= HW; i += nt) cnt[i] = 0;
  for (int i = tid; i < 578; i += nt) {
    if (i < 576) sw[i] = w2[i];
    red[i] = 0.f;
  }
  __syncthreads();
  for (int p = tid; p < HW; p += nt) {
    const f32x4_t sp = *reinterpret_cast<const f32x4_t*>(samp + (row0 + p) * 4);
    sinf[p] = sp;
    const int x0 = (int)floorf(sp[0]), y0 = (int)floorf(sp[1]);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int xx = x0 + (k & 1), yy = y0 + (k >> 1);
      slot[p * 4 + k] = (xx >= 0 && xx < W && yy >= 0 && yy < H) ? atomicAdd(&cnt[yy * W + xx], 1) : -1;
    }
  }
  __syncthreads();
  if (tid < 64) {  // exclusive scan of cnt[0..HW) by wave 0, 64 entries per pass
    int carry = 0;
    for (int base = 0; base < HW; base += 64) {
      const int i = base + tid;
      const int v = i < HW ? cnt[i] : 0;
      int s = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(s, o, 64);
        if (tid >= o) s += t;
      }
      if (i < HW) cnt[i] = carry + s - v;
      carry += __shfl(s, 63, 64);
    }
    if (tid == 0) cnt[HW] = carry;
  }
  __syncthreads();
  for (int p = tid; p < HW; p += nt) {
    const f32x4_t sp = sinf[p];
    const int x0 = (int)floorf(sp[0]), y0 = (int)floorf(sp[1]);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int sl = slot[p * 4 + k];
      if (sl >= 0) ent[cnt[(y0 + (k >> 1)) * W + x0 + (k & 1)] + sl] = p * 4 + k;
    }
  }
  __syncthreads();
  // the LDS atomics above hand out list slots in arrival order: sort every list (a few entries) so the gather
  // below sums in a fixed order (bit-identical data gradients run to run)
  for (int q = tid; q < HW; q += nt) {
    const int e0 = cnt[q], e1 = cnt[q + 1];
    for (int i = e0 + 1; i < e1; ++i) {
      const int v = ent[i];
      int j = i - 1;
      while (j >= e0 && ent[j] > v) {
        ent[j + 1] = ent[j];
        --j;
      }
      ent[j + 1] = v;
    }
  }
  __syncthreads();
  const int V = 1 << lgV, items = HW << lgV;
  const TG* gb = gout + row0 * C;
  const T* xb = x + row0 * C;
  for (int base = 0; base < items; base += nt) {
    const int it = base + tid;
    const bool live = it < items;
    const int p = live ? it >> lgV : 0, c = (it & (V - 1)) * 8;
    float gix = 0.f, giy = 0.f, mx = 0.f, my = 0.f;
    if (live) {
      // Every global load of the item is issued before any is consumed (the first GQ list entries, p's own gout
      // row and its four corners): the list walk used to wait one load latency per entry, the kernel's bound
      // at one 1024-thread block per CU.  Entries past GQ (rare: > GQ samples landing on one pixel) follow.
      constexpr int GQ = 4;
      const int e0 = cnt[p], e1 = cnt[p + 1];
      Raw8<TG> gl[GQ];
      float wl[GQ];
#pragma unroll
      for (int i = 0; i < GQ; ++i) {
        if (e0 + i < e1) {
          const int en = ent[e0 + i], pe = en >> 2, k = en & 3;
          const f32x4_t sp = sinf[pe];
          const float fx0 = floorf(sp[0]), fy0 = floorf(sp[1]);
          const float ax = (k & 1) ? sp[0] - fx0 : (fx0 + 1.f) - sp[0];
          const float ay = (k >> 1) ? sp[1] - fy0 : (fy0 + 1.f) - sp[1];
          wl[i] = ax * ay;
          gl[i].load(gb + (int64_t)pe * C + c);
        }
      }
      const f32x4_t sp = sinf[p];
      mx = sp[2];
      my = sp[3];
      const int x0 = (int)floorf(sp[0]), y0 = (int)floorf(sp[1]);
      Raw8<TG> g;
      Raw8<T> xv[4];
      g.load(gb + (int64_t)p * C + c);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int xx = x0 + (k & 1), yy = y0 + (k >> 1);
        if (xx >= 0 && xx < W && yy >= 0 && yy < H) {
          xv[k].load(xb + (int64_t)(yy * W + xx) * C + c);
        } else {
          xv[k].zero();
        }
      }
      TX* gq = gx + (row0 + p) * C + c;
      Raw8<TX> o;
      if (accumulate) o.load(gq);
      // gather: q = p, summed in list order
      float acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
      for (int i = 0; i < GQ; ++i) {
        if (e0 + i < e1) {
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += wl[i] * gl[i][j];
        }
      }
      for (int e = e0 + GQ; e < e1; ++e) {
        const int en = ent[e], pe = en >> 2, k = en & 3;
        const f32x4_t se = sinf[pe];
        const float fx0 = floorf(se[0]), fy0 = floorf(se[1]);
        const float ax = (k & 1) ? se[0] - fx0 : (fx0 + 1.f) - se[0];
        const float ay = (k >> 1) ? se[1] - fy0 : (fy0 + 1.f) - se[1];
        const float wgt = ax * ay;
        float ge[8];
        ld8(gb + (int64_t)pe * C + c, ge);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += wgt * ge[j];
      }
      if (accumulate) {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += o[j];
      }
      st8(gq, acc);
      // dL/dgrid of p
      const float ax1 = (float)(x0 + 1) - sp[0], ax0 = sp[0] - (float)x0;
      const float ay1 = (float)(y0 + 1) - sp[1], ay0 = sp[1] - (float)y0;
      // dL/dgrid = sum_c g_c * (bilinear weight derivative . corner values): the corner values are differenced
      // per channel BEFORE the channel sum (as torch's grid_sampler backward does).  Summing each corner's dot
      // product first and differencing afterwards cancels two nearly equal sums -- neighbouring feature-map values
      // are close -- and measured ~1 % error on the offset heads' gradients in fp32 (tests/test_progressive_gpu.py).
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        gix += g[j] * ((xv[1][j] - xv[0][j]) * ay1 + (xv[3][j] - xv[2][j]) * ay0);
        giy += g[j] * ((xv[2][j] - xv[0][j]) * ax1 + (xv[3][j] - xv[1][j]) * ax0);
      }
    }
    for (int o = 1; o < V; o <<= 1) {
      gix += __shfl_xor(gix, o, 64);
      giy += __shfl_xor(giy, o, 64);
    }
    if (live && (it & (V - 1)) == 0) {
      sgo[p * 2 + 0] = gix * (0.5f * W) * mx * 0.05f;
      sgo[p * 2 + 1] = giy * (0.5f * H) * my * 0.05f;
    }
  }
  __syncthreads();
  // offset head backward: items (q, c), c = tid & 31 fixed per thread
  const int c = tid & 31;
  float accw[18];
#pragma unroll
  for (int i = 0; i < 18; ++i) accw[i] = 0.f;
  for (int it = tid; it < HW * 32; it += nt) {
    const int q = it >> 5;
    const int h = q / W, w = q - (q / W) * W;
    const float ov = ldf(o1, (row0 + q) * 32 + c);
    float g = 0.f;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int yy = h - (tap / 3 - 1), xx = w - (tap % 3 - 1);  // output pixel that reads q through this tap
      if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
        const int pp = yy * W + xx;
        const float g0 = sgo[pp * 2], g1 = sgo[pp * 2 + 1];
        g += g0 * sw[c * 9 + tap] + g1 * sw[(32 + c) * 9 + tap];
        accw[tap] += g0 * ov;
        accw[9 + tap] += g1 * ov;
      }
    }
    stf(ga1, (row0 + q) * 32 + c, ov > 0.f ? g : 0.2f * g);
  }
#pragma unroll
  for (int i = 0; i < 18; ++i) {
    accw[i] += __shfl_xor(accw[i], 32, 64);
  }
  // per-wave rows of the (gw2) partial, folded below in wave order: 16 waves hitting the same 576 LDS words
  // with atomics serialised ~300 atomic wave-instructions per block
  float* wpart = reinterpret_cast<float*>(ent + 4 * HW);  // [nt / 64][576]
  if ((tid & 63) < 32) {
    float* wr = wpart + (tid >> 6) * 576;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      wr[c * 9 + tap] = accw[tap];
      wr[(32 + c) * 9 + tap] = accw[9 + tap];
    }
  }
  __syncthreads();
  for (int i = tid; i < 576; i += nt) {
    float sacc = 0.f;
    for (int w = 0; w < (nt >> 6); ++w) sacc += wpart[w * 576 + i];
    red[i] = sacc;
  }
  if (tid < 64) {
    float s0 = 0.f, s1 = 0.f;
    for (int p = tid; p < HW; p += 64) {
      s0 += sgo[p * 2];
      s1 += sgo[p * 2 + 1];
    }
    s0 = wave_sum(s0);
    s1 = wave_sum(s1);
    if (tid == 0) {
      red[576] = s0;
      red[577] = s1;
    }
  }
  __syncthreads();
  for (int i = tid; i < 578; i += nt) part[(int64_t)b * 578 + i] = red[i];
}


}  // namespace

extern "C" int mg_warp_fwd(int dtype, const void* x, const void* o1, const float* w2, const float* b2, int B, int H,
                           int W, int C, void* out, float* samp, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t P = (int64_t)B * H * W;
  const int vec = dtype == MG_F32 ? 4 : 8;
  const int G = C / vec;
  if (C % vec == 0 && G <= 64 && (G & (G - 1)) == 0 && mg_al16(x) && mg_al16(o1) && mg_al16(out) && mg_al16(samp)) {
    int lgG = 0;
    while ((1 << lgG) < G) ++lgG;
    dim3 gv((unsigned)((P + (256 >> lgG) - 1) / (256 >> lgG)));
    if (dtype == MG_F32)
      hipLaunchKernelGGL(k_warp_fwd_v<float>, gv, dim3(256), 0, st, (const float*)x, (const float*)o1, w2, b2, B, H, W,
                         C, lgG, (float*)out, samp, (const float*)nullptr, (int64_t)0, (float*)nullptr);
    else
      hipLaunchKernelGGL(k_warp_fwd_v<bf16_t>, gv, dim3(256), 0, st, (const bf16_t*)x, (const bf16_t*)o1, w2, b2, B, H,
                         W, C, lgG, (bf16_t*)out, samp, (const float*)nullptr, (int64_t)0, (bf16_t*)nullptr);
    return mg_check_launch("mg_warp_fwd");
  }
  dim3 grid((unsigned)((P + 3) / 4));
  if (dtype == MG_F32)
    hipLaunchKernelGGL(k_warp_fwd<float>, grid, dim3(256), 0, st, (const float*)x, (const float*)o1, w2, b2, B, H, W, C, (float*)out, samp);
  else
    hipLaunchKernelGGL(k_warp_fwd<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)x, (const bf16_t*)o1, w2, b2, B, H, W, C, (bf16_t*)out, samp);
  return mg_check_launch("mg_warp_fwd");
}

extern "C" int mg_warp_fwd_scaled(int dtype, const void* x, const void* o1, const float* w2, const float* b2, int B,
                                  int H, int W, int C, const float* s, int64_t lds, void* out, void* out_scaled,
                                  float* samp, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t P = (int64_t)B * H * W;
  const int vec = dtype == MG_F32 ? 4 : 8;
  const int G = C / vec;
  if (C % vec == 0 && G <= 64 && (G & (G - 1)) == 0 && mg_al16(x) && mg_al16(o1) && mg_al16(out) && mg_al16(samp) &&
      mg_al16(s) && lds % 4 == 0 && mg_al16(out_scaled)) {
    int lgG = 0;
    while ((1 << lgG) < G) ++lgG;
    dim3 gv((unsigned)((P + (256 >> lgG) - 1) / (256 >> lgG)));
    if (dtype == MG_F32)
      hipLaunchKernelGGL(k_warp_fwd_v<float>, gv, dim3(256), 0, st, (const float*)x, (const float*)o1, w2, b2, B, H, W,
                         C, lgG, (float*)out, samp, s, lds, (float*)out_scaled);
    else
      hipLaunchKernelGGL(k_warp_fwd_v<bf16_t>, gv, dim3(256), 0, st, (const bf16_t*)x, (const bf16_t*)o1, w2, b2, B, H,
                         W, C, lgG, (bf16_t*)out, samp, s, lds, (bf16_t*)out_scaled);
    return mg_check_launch("mg_warp_fwd_scaled");
  }
  int rc = mg_warp_fwd(dtype, x, o1, w2, b2, B, H, W, C, out, samp, stream);
  if (rc != MG_OK) return rc;
  return mg_scale_bc(dtype, out, C, s, lds, B, H * W, C, out_scaled, C, stream);
}

extern "C" int mg_warp_bwd(int dtype, int gout_dtype, const void* gout, const void* x, const float* samp, int B, int H,
                           int W, int C, float* gx, float* goff, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t P = (int64_t)B * H * W;
  // measured slower than the atomic kernel at C2 (latency-bound per-pixel chain): opt-in via tuning key 8
  if (g_mg_tune[MG_TUNE_WARP_LDS] == 1 && C % 64 == 0 && H * W <= 256 && mg_al16(samp)) {
    if (hipMemsetAsync(goff, 0, (size_t)P * 2 * sizeof(float), st) != hipSuccess) return mg_check_launch("mg_warp_bwd");
    dim3 gl(B, C / 64);
    const size_t lds = (size_t)H * W * 64 * sizeof(float);
#define L_(T, TG) hipLaunchKernelGGL((k_warp_bwd_lds<T, TG>), gl, dim3(512), lds, st, (const TG*)gout, (const T*)x, samp, B, H, W, C, gx, goff)
    if (dtype == MG_F32) { if (gout_dtype == MG_F32) L_(float, float); else L_(float, bf16_t); }
    else { if (gout_dtype == MG_F32) L_(bf16_t, float); else L_(bf16_t, bf16_t); }
#undef L_
    return mg_check_launch("mg_warp_bwd");
  }
  dim3 grid((unsigned)((P + 3) / 4));
#define L_(T, TG) hipLaunchKernelGGL((k_warp_bwd<T, TG>), grid, dim3(256), 0, st, (const TG*)gout, (const T*)x, samp, B, H, W, C, gx, goff)
  if (dtype == MG_F32) { if (gout_dtype == MG_F32) L_(float, float); else L_(float, bf16_t); }
  else { if (gout_dtype == MG_F32) L_(bf16_t, float); else L_(bf16_t, bf16_t); }
#undef L_
  return mg_check_launch("mg_warp_bwd");
}

extern "C" int mg_mtm_bwd_fused(int dtype, int gout_dtype, const void* gout, const void* x, const float* samp,
                                const void* o1, const float* w2, int B, int H, int W, int C, int gx_dtype, void* gx,
                                int accumulate, void* ga1, float* gw2, float* gb2, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int HW = H * W;
  int lgV = 0;
  while ((8 << lgV) < C) ++lgV;
  MG_REQUIRE(B > 0 && HW > 0 && HW <= 1024 && C == (8 << lgV) && C <= 512, "needs H*W <= 1024 and C = 8 * 2^k <= 512");
  MG_REQUIRE(mg_al16(gout) && mg_al16(x) && mg_al16(samp) && mg_al16(gx), "16-B aligned gout / x / samp / gx");
  MG_REQUIRE(gx_dtype == dtype || gx_dtype == MG_F32, "gx dtype must be the activation dtype or fp32");
  bool deferred = false;
  float* part = mg_fold_partials((size_t)B * 578 * sizeof(float), st, &deferred);
  if (!part) {
    mg_set_error("mg_mtm_bwd_fused: workspace allocation failed");
    return MG_ERR_LAUNCH;
  }
  const size_t lds = (size_t)HW * 6 * sizeof(float) + (576 + 578) * sizeof(float) + (size_t)(9 * HW + 1) * sizeof(int) +
                     (size_t)16 * 576 * sizeof(float);  // + per-wave gw2 partial rows (16 waves of the 1024-thread block)
  MG_REQUIRE(lds <= 65536, "image too large for the per-image LDS lists");
#define L_(T, TG, TX) hipLaunchKernelGGL((k_mtm_bwd_img<T, TG, TX>), dim3(B), dim3(1024), lds, st, (const TG*)gout, \
    (const T*)x, samp, (const T*)o1, w2, H, W, C, lgV, (TX*)gx, accumulate, (T*)ga1, part)
  if (dtype == MG_F32) {
    if (gout_dtype == MG_F32) L_(float, float, float); else L_(float, bf16_t, float);
  } else if (gx_dtype == MG_F32) {
    if (gout_dtype == MG_F32) L_(bf16_t, float, float); else L_(bf16_t, bf16_t, float);
  } else {
    if (gout_dtype == MG_F32) L_(bf16_t, float, bf16_t); else L_(bf16_t, bf16_t, bf16_t);
  }
#undef L_
  mg_fold_rows_submit(mg_fold_rows{part, 578, B, 578, 576, gw2, gb2}, deferred, st);
  return mg_check_launch("mg_mtm_bwd_fused");
}

extern "C" int mg_offset_head_bwd(int dtype, const float* goff, const void* o1, const float* w2, int B, int H, int W,
                                  void* ga1, float* gw2, float* gb2, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t P = (int64_t)B * H * W;
  // block-partial variant: measured slower at C2 (few blocks at 4x4 / 8x8); opt-in via tuning key 8
  if (g_mg_tune[MG_TUNE_WARP_LDS] == 1 && H * W <= 256 && 256 % (H * W) == 0) {
    const int nb = (int)((P + 255) / 256);
    float* part = reinterpret_cast<float*>(mg_workspace((size_t)nb * 578 * sizeof(float), st));
    if (!part) {
      mg_set_error("mg_offset_head_bwd: workspace allocation failed");
      return MG_ERR_LAUNCH;
    }
    if (dtype == MG_F32)
      hipLaunchKernelGGL(k_offset_head_bwd_blk<float>, dim3(nb), dim3(256), 0, st, goff, (const float*)o1, w2, B, H, W,
                         (float*)ga1, part);
    else
      hipLaunchKernelGGL(k_offset_head_bwd_blk<bf16_t>, dim3(nb), dim3(256), 0, st, goff, (const bf16_t*)o1, w2, B, H,
                         W, (bf16_t*)ga1, part);
    hipLaunchKernelGGL(k_offset_head_fin, dim3(3), dim3(256), 0, st, part, nb, gw2, gb2);
    return mg_check_launch("mg_offset_head_bwd");
  }
  int ppb = 64;
  dim3 grid((unsigned)((P + ppb - 1) / ppb));
  if (dtype == MG_F32)
    hipLaunchKernelGGL(k_offset_head_bwd<float>, grid, dim3(256), 0, st, goff, (const float*)o1, w2, B, H, W, ppb, (float*)ga1, gw2, gb2);
  else
    hipLaunchKernelGGL(k_offset_head_bwd<bf16_t>, grid, dim3(256), 0, st, goff, (const bf16_t*)o1, w2, B, H, W, ppb, (bf16_t*)ga1, gw2, gb2);
  return mg_check_launch("mg_offset_head_bwd");
}

extern "C" int mg_upsample2x_fwd_scaled(int dtype, const void* x, int B, int H, int W, int C, void* out,
                                        const float* s, int64_t lds, void* xs, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t n = 4LL * B * H * W * C;
  MG_REQUIRE(C % 8 == 0 && lds % 4 == 0 && mg_al16(x) && mg_al16(out) && mg_al16(xs) && mg_al16(s),
             "mg_upsample2x_fwd_scaled: C a multiple of 8, 16-byte aligned operands");
  MG_REQUIRE(n / 8 < (1LL << 31), "mg_upsample2x_fwd_scaled: too many elements");
  if (n == 0) return MG_OK;
  const int blocks = nblk(n / 8);
  if (dtype == MG_F32)
    hipLaunchKernelGGL((k_up2_fwd_v<float, true>), dim3(blocks), dim3(256), 0, st, (const float*)x, B, H, W, C,
                       (float*)out, s, lds, (float*)xs);
  else
    hipLaunchKernelGGL((k_up2_fwd_v<bf16_t, true>), dim3(blocks), dim3(256), 0, st, (const bf16_t*)x, B, H, W, C,
                       (bf16_t*)out, s, lds, (bf16_t*)xs);
  return mg_check_launch("mg_upsample2x_fwd_scaled");
}

extern "C" int mg_upsample2x_fwd(int dtype, const void* x, int B, int H, int W, int C, void* out, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t n = 4LL * B * H * W * C;
  if (C % 8 == 0 && mg_al16(x) && mg_al16(out) && n / 8 < (1LL << 31)) {
    int blocks = nblk(n / 8);
    if (dtype == MG_F32)
      hipLaunchKernelGGL(k_up2_fwd_v<float>, dim3(blocks), dim3(256), 0, st, (const float*)x, B, H, W, C, (float*)out);
    else
      hipLaunchKernelGGL(k_up2_fwd_v<bf16_t>, dim3(blocks), dim3(256), 0, st, (const bf16_t*)x, B, H, W, C,
                         (bf16_t*)out);
    return mg_check_launch("mg_upsample2x_fwd");
  }
  if (dtype == MG_F32)
    hipLaunchKernelGGL(k_up2_fwd<float>, dim3(nblk(n)), dim3(256), 0, st, (const float*)x, B, H, W, C, (float*)out);
  else
    hipLaunchKernelGGL(k_up2_fwd<bf16_t>, dim3(nblk(n)), dim3(256), 0, st, (const bf16_t*)x, B, H, W, C, (bf16_t*)out);
  return mg_check_launch("mg_upsample2x_fwd");
}

extern "C" int mg_upsample2x_bwd(int gout_dtype, const void* gout, int B, int H, int W, int C, int gx_dtype, void* gx,
                                 int accumulate, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t n = (int64_t)B * H * W * C;
  if (C % 8 == 0 && mg_al16(gout) && mg_al16(gx) && n / 8 < (1LL << 31)) {
#define L_(TG, T) hipLaunchKernelGGL((k_up2_bwd_v<TG, T>), dim3(nblk(n / 8)), dim3(256), 0, st, (const TG*)gout, B, H, W, C, (T*)gx, accumulate)
    if (gout_dtype == MG_F32) { if (gx_dtype == MG_F32) L_(float, float); else L_(float, bf16_t); }
    else { if (gx_dtype == MG_F32) L_(bf16_t, float); else L_(bf16_t, bf16_t); }
#undef L_
    return mg_check_launch("mg_upsample2x_bwd");
  }
#define L_(TG, T) hipLaunchKernelGGL((k_up2_bwd<TG, T>), dim3(nblk(n)), dim3(256), 0, st, (const TG*)gout, B, H, W, C, (T*)gx, accumulate)
  if (gout_dtype == MG_F32) { if (gx_dtype == MG_F32) L_(float, float); else L_(float, bf16_t); }
  else { if (gx_dtype == MG_F32) L_(bf16_t, float); else L_(bf16_t, bf16_t); }
#undef L_
  return mg_check_launch("mg_upsample2x_bwd");
}
