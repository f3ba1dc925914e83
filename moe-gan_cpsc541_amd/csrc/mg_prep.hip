// Per-step weight preparation, casts, reductions and the flat AdamW of libmoegan_hip.
#include "mg_common.h"

namespace {

// wpack[o][(kh*KW+kw)*Cin + ci] = W[o][ci][kh][kw]; rows o >= Cout zero (padding)
template <typename T>
__global__ void k_pack_conv(const float* __restrict__ W, int Cout, int Cin, int KH, int KW, int rows,
                            T* __restrict__ out) {
  int64_t K = (int64_t)KH * KW * Cin;
  int64_t n = (int64_t)rows * K;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int o = (int)(i / K);
    int r = (int)(i - (int64_t)o * K);
    int tap = r / Cin, ci = r - tap * Cin;
    int kh = tap / KW, kw = tap - kh * KW;
    float v = o < Cout ? W[(((int64_t)o * Cin + ci) * KH + kh) * KW + kw] : 0.f;
    stf(out, i, v);
  }
}

// out[ci][(kh'*KW+kw')*Cout + o] = W[o][ci][KH-1-kh'][KW-1-kw']   (stride-1 data gradient)
template <typename T>
__global__ void k_pack_conv_flip(const float* __restrict__ W, int Cout, int Cin, int KH, int KW, int rows,
                                 T* __restrict__ out) {
  int64_t K = (int64_t)KH * KW * Cout;
  int64_t n = (int64_t)rows * K;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int ci = (int)(i / K);
    int r = (int)(i - (int64_t)ci * K);
    int tap = r / Cout, o = r - tap * Cout;
    int kh = KH - 1 - tap / KW, kw = KW - 1 - (tap % KW);
    float v = ci < Cin ? W[(((int64_t)o * Cin + ci) * KH + kh) * KW + kw] : 0.f;
    stf(out, i, v);
  }
}

// out[cls][ci][t*Cg + co] = W[co][ci][kh(py,ty)][kw(px,tx)]   (4x4 / stride-2 / pad-1 data gradient)
template <typename T>
__global__ void k_pack_dgrad_s2(const float* __restrict__ W, int Cg, int Cin, int rows, T* __restrict__ out) {
  int64_t K = 4LL * Cg;
  int64_t n = 4LL * rows * K;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int cls = (int)(i / ((int64_t)rows * K));
    int64_t r = i - (int64_t)cls * rows * K;
    int ci = (int)(r / K);
    int k = (int)(r - (int64_t)ci * K);
    int t = k / Cg, co = k - t * Cg;
    int ty = t >> 1, tx = t & 1, py = cls >> 1, px = cls & 1;
    int kh = py ? (ty ? 2 : 0) : (ty ? 3 : 1);
    int kw = px ? (tx ? 2 : 0) : (tx ? 3 : 1);
    float v = ci < Cin ? W[(((int64_t)co * Cin + ci) * 4 + kh) * 4 + kw] : 0.f;
    stf(out, i, v);
  }
}

// wsq[o][ci] = sum_taps W[o][ci][tap]^2   (rows o >= Cout zero)
__global__ void k_wsq(const float* __restrict__ W, int Cout, int Cin, int taps, int rows, float* __restrict__ out) {
  int64_t n = (int64_t)rows * Cin;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int o = (int)(i / Cin);
    float s = 0.f;
    if (o < Cout)
      for (int t = 0; t < taps; ++t) {
        float w = W[i * taps + t];
        s += w * w;
      }
    out[i] = s;
  }
}

// gW[o][ci][t] += 2 * W[o][ci][t] * gwsq[o][ci]
__global__ void k_wsq_bwd(const float* __restrict__ W, const float* __restrict__ gwsq, int Cout, int Cin, int taps,
                          float* __restrict__ gW) {
  int64_t n = (int64_t)Cout * Cin * taps;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    gW[i] += 2.f * W[i] * gwsq[i / taps];
}

template <typename TI, typename TO>
__global__ void k_cast(const TI* __restrict__ in, TO* __restrict__ out, int64_t n, float alpha, int square) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float v = ldf(in, i) * alpha;
    stf(out, i, square ? v * v : v);
  }
}

// strided 2-D copy/cast: out[r*ldo + c] (+)= alpha * in[r*ldi + c]
template <typename TI, typename TO>
__global__ void k_copy2d(const TI* __restrict__ in, int64_t ldi, TO* __restrict__ out, int64_t ldo, int R, int C,
                         float alpha, int accumulate) {
  int64_t n = (int64_t)R * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int r = (int)(i / C), c = (int)(i - (int64_t)r * C);
    float v = alpha * ldf(in, (int64_t)r * ldi + c);
    if (accumulate) v += ldf(out, (int64_t)r * ldo + c);
    stf(out, (int64_t)r * ldo + c, v);
  }
}

// out[c] (+)= sum_r X[r*ld + c]   (column sums; fp32 atomics across row splits)
template <typename T>
__global__ void k_colsum(const T* __restrict__ X, int64_t ld, int R, int C, int rows_per_block,
                         float* __restrict__ out) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  int r0 = blockIdx.y * rows_per_block, r1 = min(R, r0 + rows_per_block);
  float s = 0.f;
  for (int r = r0; r < r1; ++r) s += ldf(X, (int64_t)r * ld + c);
  atomicAdd(out + c, s);
}

// vectorised column sums: 8 columns per thread, rows split over TY lanes x grid.y, LDS reduction into
// one partial row per row-block (no same-address atomics), folded by k_colsum_fin.  C % 8 == 0.
template <typename T>
__global__ __launch_bounds__(256) void k_colsum_v(const T* __restrict__ X, int64_t ld, int R, int C,
                                                  int rows_per_block, float* __restrict__ part, int atomic_out) {
  __shared__ float red[256 * 8];
  const int tx = threadIdx.x, ty = threadIdx.y, TX = blockDim.x, TY = blockDim.y;
  const int c = (blockIdx.x * TX + tx) * 8;
  const bool live = c < C;
  const int r0 = blockIdx.y * rows_per_block, r1 = min(R, r0 + rows_per_block);
  float acc[8], t[8], t1[8], t2[8], t3[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  int r = r0 + ty;
  for (; live && r + 3 * TY < r1; r += 4 * TY) {  // four independent row loads in flight
    ld8(X + (int64_t)r * ld + c, t);
    ld8(X + (int64_t)(r + TY) * ld + c, t1);
    ld8(X + (int64_t)(r + 2 * TY) * ld + c, t2);
    ld8(X + (int64_t)(r + 3 * TY) * ld + c, t3);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += (t[j] + t1[j]) + (t2[j] + t3[j]);
  }
  for (; live && r < r1; r += TY) {
    ld8(X + (int64_t)r * ld + c, t);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += t[j];
  }
  const int tid = ty * TX + tx;
#pragma unroll
  for (int j = 0; j < 8; ++j) red[tid * 8 + j] = acc[j];
  __syncthreads();
  if (ty == 0 && live) {
    for (int y = 1; y < TY; ++y)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += red[(y * TX + tx) * 8 + j];
    if (atomic_out) {  // few row blocks: add straight into out (shallow same-address atomics, no fold launch)
#pragma unroll
      for (int j = 0; j < 8; ++j) atomicAdd(part + c + j, acc[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) part[(int64_t)blockIdx.y * C + c + j] = acc[j];
    }
  }
}

// block (64 columns x 16 partial lanes, 1024 threads); out[c] += sum_r part[r, c]
__global__ __launch_bounds__(1024) void k_colsum_fin(const float* __restrict__ part, int nparts, int C,
                                                     float* __restrict__ out) {
  __shared__ float red[16][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  float s0 = 0.f, s1 = 0.f;
  if (c < C) {
    int r = ty;
    for (; r + 16 < nparts; r += 32) {  // two independent loads in flight per lane
      s0 += part[(int64_t)r * C + c];
      s1 += part[(int64_t)(r + 16) * C + c];
    }
    if (r < nparts) s0 += part[(int64_t)r * C + c];
  }
  red[ty][tx] = s0 + s1;
  __syncthreads();
  if (ty == 0 && c < C) {
    float t = 0.f;
#pragma unroll
    for (int y = 0; y < 16; ++y) t += red[y][tx];
    out[c] += t;
  }
}

// weight norm: W[o] = g[o] * v[o] / ||v[o]||  (t2i_moe_gan.py:869-886, torch weight_norm dim=0)
MG_DEV void wn_fwd_row(const float* __restrict__ v, const float* __restrict__ g, int o, int K,
                       float* __restrict__ W, float* __restrict__ norm) {
  __shared__ float red[16];
  float s = 0.f;
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    float x = v[(int64_t)o * K + k];
    s += x * x;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
    red[0] = sqrtf(t);
  }
  __syncthreads();
  float n = red[0];
  if (threadIdx.x == 0) norm[o] = n;
  float sc = g[o] / n;
  for (int k = threadIdx.x; k < K; k += blockDim.x) W[(int64_t)o * K + k] = v[(int64_t)o * K + k] * sc;
}

__global__ void k_wn_fwd(const float* __restrict__ v, const float* __restrict__ g, int O, int K,
                         float* __restrict__ W, float* __restrict__ norm) {
  wn_fwd_row(v, g, blockIdx.x, K, W, norm);
}

// gg[o] += sum_k gW*v/n ; gv = (g/n) * (gW - (gg_o/n) * v)
MG_DEV void wn_bwd_row(const float* __restrict__ v, const float* __restrict__ g, const float* __restrict__ norm,
                       const float* __restrict__ gW, int o, int K, float* __restrict__ gv, float* __restrict__ gg) {
  __shared__ float red[16];
  float n = norm[o];
  float s = 0.f;
  for (int k = threadIdx.x; k < K; k += blockDim.x) s += gW[(int64_t)o * K + k] * v[(int64_t)o * K + k];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
    red[0] = t / n;
  }
  __syncthreads();
  float ggo = red[0];
  if (threadIdx.x == 0) gg[o] += ggo;
  float a = g[o] / n, b = ggo / n;
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    int64_t i = (int64_t)o * K + k;
    gv[i] += a * (gW[i] - b * v[i]);
  }
}

__global__ void k_wn_bwd(const float* __restrict__ v, const float* __restrict__ g, const float* __restrict__ norm,
                         const float* __restrict__ gW, int O, int K, float* __restrict__ gv, float* __restrict__ gg) {
  wn_bwd_row(v, g, norm, gW, blockIdx.x, K, gv, gg);
}

// several layers' weight norms (forward or backward) in one launch: block -> (descriptor, output row)
constexpr int kWnMax = 8;
struct WnArgs {
  mg_wn_desc d[kWnMax];
  int row_off[kWnMax + 1];
  int n, bwd;
};
__global__ void k_wn_batch(WnArgs a) {
  const int b = blockIdx.x;
  int p = 0;
  while (p + 1 < a.n && b >= a.row_off[p + 1]) ++p;
  const mg_wn_desc& q = a.d[p];
  const int o = b - a.row_off[p];
  if (a.bwd) wn_bwd_row(q.v, q.g, q.norm, q.gW, o, q.K, q.gv, q.gg);
  else wn_fwd_row(q.v, q.g, o, q.K, q.W, q.norm);
}

// sum of squares of n floats, accumulated into out[0] -- deterministically: <= 1024 blocks write one partial
// each, and k_sumsq_fin folds them in a fixed order (the clip coefficient then comes out bit-identical on
// every data-parallel rank that holds the same all-reduced gradient; float atomics would not).  Four
// independent 16-B loads per thread per iteration keep enough bytes in flight to run near HBM rate (one
// load per thread over 256 blocks measured 2.1 TB/s on the 39 M-float generator gradient).
__global__ __launch_bounds__(256) void k_sumsq(const float* __restrict__ x, int64_t n, float* __restrict__ part) {
  __shared__ float red[4];
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  const int64_t nv = mg_al16(x) ? n / 4 : 0;
  const f32x4_t* x4 = reinterpret_cast<const f32x4_t*>(x);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (; i + 3 * stride < nv; i += 4 * stride) {
    const f32x4_t a = x4[i], b = x4[i + stride], c = x4[i + 2 * stride], d = x4[i + 3 * stride];
    s0 += a[0] * a[0] + a[1] * a[1] + a[2] * a[2] + a[3] * a[3];
    s1 += b[0] * b[0] + b[1] * b[1] + b[2] * b[2] + b[3] * b[3];
    s2 += c[0] * c[0] + c[1] * c[1] + c[2] * c[2] + c[3] * c[3];
    s3 += d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3];
  }
  for (; i < nv; i += stride) {
    const f32x4_t a = x4[i];
    s0 += a[0] * a[0] + a[1] * a[1] + a[2] * a[2] + a[3] * a[3];
  }
  for (int64_t j = nv * 4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n; j += stride) {
    float v = x[j];
    s0 += v * v;
  }
  float s = wave_sum((s0 + s1) + (s2 + s3));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void k_sumsq_fin(const float* __restrict__ part, int nparts,
                                                   float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) s += part[i];  // fixed order per thread
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] += (red[0] + red[1]) + (red[2] + red[3]);
}

// mg_grad_norm_steps' second launch: the fixed-order fold of k_sumsq_fin written (not accumulated) to out[0], and the
// gated step counters of the optimizer launches that follow (k_opt_prologue's rule per counter)
__global__ __launch_bounds__(256) void k_sumsq_fin_steps(const float* __restrict__ part, int nparts, float* __restrict__ out,
                                                         int32_t* step0, int32_t run0, int32_t* step1, int32_t run1,
                                                         const int32_t* flags, int32_t skip_mask, const int32_t* win) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) s += part[i];  // fixed order per thread (k_sumsq_fin's)
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    out[0] = (red[0] + red[1]) + (red[2] + red[3]);
    const bool skip = flags && (flags[0] & skip_mask);
    if (step0 && !skip && !(win && run0 && !(win[0] & run0))) step0[0] += 1;
    if (step1 && !skip && !(win && run1 && !(win[0] & run1))) step1[0] += 1;
  }
}

// One AdamW element update (torch.optim.AdamW single-tensor math, t2i_moe_gan.py:1101-1102), with every
// multiply-add spelled out: all three AdamW kernels run the identical instruction sequence (bit-exact to
// each other whatever the surrounding code lets the compiler contract).
MG_DEV void adamw_elem(float gi, float& pi, float& mi, float& vi, float coef, float lr, float b1, float b2,
                       float eps, float wd, float step_size, float bc2_sqrt) {
#pragma clang fp contract(off)
  gi = gi * coef;
  pi = pi * (1.f - lr * wd);
  mi = mi + (gi - mi) * (1.f - b1);
  vi = vi * b2 + (1.f - b2) * gi * gi;
  const float denom = sqrtf(vi) / bc2_sqrt + eps;
  pi = pi - step_size * (mi / denom);
}

// torch.optim.AdamW (single-tensor semantics, t2i_moe_gan.py:1101-1102) fused with
// clip_grad_norm_ (t2i_moe_gan.py:1333-1337 / :1417-1421): coef = min(1, max_norm / (||g|| + 1e-6)).
__global__ void k_adamw(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                        float* __restrict__ v, int64_t n, float lr, float b1, float b2, float eps, float wd,
                        float bc1, float bc2_sqrt, const float* __restrict__ sumsq, float max_norm) {
  float coef = 1.f;
  if (sumsq) {
    float tn = sqrtf(sumsq[0]);
    coef = fminf(max_norm / (tn + 1e-6f), 1.f);
  }
  float step_size = lr / bc1;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float pi = p[i], mi = m[i], vi = v[i];
    adamw_elem(g[i], pi, mi, vi, coef, lr, b1, b2, eps, wd, step_size, bc2_sqrt);
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
  }
}

// Whether a gated optimizer launch runs (loss guards, mg_guard.hip): not when the step's flag word has a
// skip bit (a NaN/Inf discriminator loss skips the batch, t2i_moe_gan.py:1315-1320), and only when the
// accumulation-window word says the parameter group received a gradient (torch's AdamW skips a parameter
// whose .grad is None).  NULL words = always run.
MG_DEV bool opt_runs(const int32_t* flags, int32_t skip_mask, const int32_t* win, int32_t run_mask) {
  if (flags && (flags[0] & skip_mask)) return false;
  if (win && run_mask && !(win[0] & run_mask)) return false;
  return true;
}

__global__ void k_opt_prologue(float* __restrict__ sumsq, int32_t* __restrict__ step, const int32_t* flags,
                               int32_t skip_mask, const int32_t* win, int32_t run_mask) {
  if (threadIdx.x == 0) {
    if (sumsq) sumsq[0] = 0.f;
    if (step && opt_runs(flags, skip_mask, win, run_mask)) step[0] += 1;
  }
}

// k_adamw with the bias corrections derived on the device from the step counter
__global__ void k_adamw_dev(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, int64_t n, float lr, float b1, float b2, float eps, float wd,
                            const int32_t* __restrict__ step, const float* __restrict__ sumsq, float max_norm) {
  const float t = (float)step[0];
  const float bc1 = 1.f - powf(b1, t);
  const float bc2_sqrt = sqrtf(1.f - powf(b2, t));
  float coef = 1.f;
  if (sumsq) {
    float tn = sqrtf(sumsq[0]);
    coef = fminf(max_norm / (tn + 1e-6f), 1.f);
  }
  float step_size = lr / bc1;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float pi = p[i], mi = m[i], vi = v[i];
    adamw_elem(g[i], pi, mi, vi, coef, lr, b1, b2, eps, wd, step_size, bc2_sqrt);
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
  }
}

// AdamW + clip coefficient, 4 parameters per thread (16-B loads / stores), optionally also writing the
// bf16 compute shadow of the updated parameters (the next step's per-step cast, fused away).
template <bool NT>
MG_DEV f32x4_t ld4s(const f32x4_t* q) {
  if constexpr (NT) return __builtin_nontemporal_load(q);
  else return *q;
}
template <bool NT, typename V>
MG_DEV void st_s(V* q, V x) {
  if constexpr (NT) __builtin_nontemporal_store(x, q);
  else *q = x;
}

// NT: the optimizer state and gradients stream through non-temporal (cache-streaming) vector loads / stores:
// every byte is touched once per step, so keeping them out of L2 / MALL leaves those to the parameters' next users
template <bool NT>
__global__ __launch_bounds__(256) void k_adamw_dev_v(float* __restrict__ p, const float* __restrict__ g,
                                                     float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                     float lr, float b1, float b2, float eps, float wd,
                                                     const int32_t* __restrict__ step,
                                                     const float* __restrict__ sumsq, float max_norm,
                                                     bf16_t* __restrict__ shadow, const int32_t* flags,
                                                     int32_t skip_mask, const int32_t* win, int32_t run_mask) {
  if (!opt_runs(flags, skip_mask, win, run_mask)) return;
  const float t = (float)step[0];
  const float bc1 = 1.f - powf(b1, t);
  const float bc2_sqrt = sqrtf(1.f - powf(b2, t));
  float coef = 1.f;
  if (sumsq) {
    float tn = sqrtf(sumsq[0]);
    coef = fminf(max_norm / (tn + 1e-6f), 1.f);
  }
  const float step_size = lr / bc1;
  auto upd = [&](float gi, float& pi, float& mi, float& vi) {
    adamw_elem(gi, pi, mi, vi, coef, lr, b1, b2, eps, wd, step_size, bc2_sqrt);
  };
  const int64_t n4 = n >> 2;
  // two 4-parameter vectors per thread and iteration, all eight 16-B loads issued before the math (one vector per
  // iteration left one set of loads in flight per thread: ~4.2 TB/s on the C5 generator's 95 M parameters)
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  auto upd4 = [&](int64_t i, f32x4_t pv, f32x4_t gv, f32x4_t mv, f32x4_t vv) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float pj = pv[j], mj = mv[j], vj = vv[j];
      upd(gv[j], pj, mj, vj);
      pv[j] = pj;
      mv[j] = mj;
      vv[j] = vj;
    }
    st_s<NT>(reinterpret_cast<f32x4_t*>(p) + i, pv);
    st_s<NT>(reinterpret_cast<f32x4_t*>(m) + i, mv);
    st_s<NT>(reinterpret_cast<f32x4_t*>(v) + i, vv);
    if (shadow) {
      u16x4_t h;
#pragma unroll
      for (int j = 0; j < 4; ++j) h[j] = f2bf(pv[j]);
      reinterpret_cast<u16x4_t*>(shadow)[i] = h;
    }
  };
  const f32x4_t* p4 = reinterpret_cast<const f32x4_t*>(p);
  const f32x4_t* g4 = reinterpret_cast<const f32x4_t*>(g);
  const f32x4_t* m4 = reinterpret_cast<const f32x4_t*>(m);
  const f32x4_t* v4 = reinterpret_cast<const f32x4_t*>(v);
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (; i + stride < n4; i += 2 * stride) {
    const int64_t i2 = i + stride;
    const f32x4_t pa = ld4s<NT>(p4 + i), ga = ld4s<NT>(g4 + i), ma = ld4s<NT>(m4 + i), va = ld4s<NT>(v4 + i);
    const f32x4_t pb = ld4s<NT>(p4 + i2), gb = ld4s<NT>(g4 + i2), mb = ld4s<NT>(m4 + i2), vb = ld4s<NT>(v4 + i2);
    upd4(i, pa, ga, ma, va);
    upd4(i2, pb, gb, mb, vb);
  }
  if (i < n4) upd4(i, ld4s<NT>(p4 + i), ld4s<NT>(g4 + i), ld4s<NT>(m4 + i), ld4s<NT>(v4 + i));
  for (int64_t i = (n4 << 2) + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float pi = p[i], mi = m[i], vi = v[i];
    upd(g[i], pi, mi, vi);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
    if (shadow) shadow[i] = f2bf(pi);
  }
}

// generator constant [1, C, 4, 4] (NCHW) -> NHWC [B, 4, 4, C]
template <typename T>
__global__ void k_const_fwd(const float* __restrict__ cst, int C, int HW, int B, T* __restrict__ out) {
  int64_t n = (int64_t)B * HW * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int c = (int)(i % C);
    int p = (int)((i / C) % HW);
    stf(out, i, cst[(int64_t)c * HW + p]);
  }
}
// gconst[c][p] += sum_b g[b][p][c]
template <typename T>
__global__ void k_const_bwd(const T* __restrict__ g, int C, int HW, int B, int bchunk, float* __restrict__ gc) {
  // grid.y splits the batch (the [C, HW] map alone is too few threads to fill the chip); partial sums meet
  // in fp32 atomics
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= C * HW) return;
  int p = i / C, c = i - p * C;
  const int b0 = blockIdx.y * bchunk, b1 = min(B, b0 + bchunk);
  float s0 = 0.f, s1 = 0.f;
  int b = b0;
  for (; b + 1 < b1; b += 2) {
    s0 += ldf(g, ((int64_t)b * HW + p) * C + c);
    s1 += ldf(g, ((int64_t)(b + 1) * HW + p) * C + c);
  }
  if (b < b1) s0 += ldf(g, ((int64_t)b * HW + p) * C + c);
  atomicAdd(gc + (int64_t)c * HW + p, s0 + s1);
}

inline int nblk(int64_t n, int t = 256) { return (int)std::min<int64_t>((n + t - 1) / t, 65536); }

}  // namespace

#define DISPATCH_T(dtype, ...)                          \
  do {                                                  \
    if ((dtype) == MG_F32) {                            \
      typedef float T;                                  \
      __VA_ARGS__;                                      \
    } else {                                            \
      typedef bf16_t T;                                 \
      __VA_ARGS__;                                      \
    }                                                   \
  } while (0)

extern "C" int mg_pack_conv(int dtype, const float* W, int Cout, int Cin, int KH, int KW, int rows, void* out,
                            void* stream) {
  MG_REQUIRE(rows >= Cout, "rows < Cout");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t n = (int64_t)rows * KH * KW * Cin;
  DISPATCH_T(dtype, hipLaunchKernelGGL(k_pack_conv<T>, dim3(nblk(n)), dim3(256), 0, st, W, Cout, Cin, KH, KW, rows,
                                       reinterpret_cast<T*>(out)));
  return mg_check_launch("mg_pack_conv");
}

extern "C" int mg_pack_conv_flip(int dtype, const float* W, int Cout, int Cin, int KH, int KW, int rows, void* out,
                                 void* stream) {
  MG_REQUIRE(rows >= Cin, "rows < Cin");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t n = (int64_t)rows * KH * KW * Cout;
  DISPATCH_T(dtype, hipLaunchKernelGGL(k_pack_conv_flip<T>, dim3(nblk(n)), dim3(256), 0, st, W, Cout, Cin, KH, KW,
                                       rows, reinterpret_cast<T*>(out)));
  return mg_check_launch("mg_pack_conv_flip");
}

extern "C" int mg_pack_dgrad_s2(int dtype, const float* W, int Cg, int Cin, int rows, void* out, void* stream) {
  MG_REQUIRE(rows >= Cin, "rows < Cin");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t n = 16LL * rows * Cg;
  DISPATCH_T(dtype, hipLaunchKernelGGL(k_pack_dgrad_s2<T>, dim3(nblk(n)), dim3(256), 0, st, W, Cg, Cin, rows,
                                       reinterpret_cast<T*>(out)));
  return mg_check_launch("mg_pack_dgrad_s2");
}

extern "C" int mg_wsq(const float* W, int Cout, int Cin, int taps, int rows, float* out, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_wsq, dim3(nblk((int64_t)rows * Cin)), dim3(256), 0, st, W, Cout, Cin, taps, rows, out);
  return mg_check_launch("mg_wsq");
}

extern "C" int mg_wsq_bwd(const float* W, const float* gwsq, int Cout, int Cin, int taps, float* gW, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_wsq_bwd, dim3(nblk((int64_t)Cout * Cin * taps)), dim3(256), 0, st, W, gwsq, Cout, Cin, taps, gW);
  return mg_check_launch("mg_wsq_bwd");
}

extern "C" int mg_cast(int in_dtype, const void* in, int out_dtype, void* out, int64_t n, float alpha, int square,
                       void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n == 0) return MG_OK;
  if (in_dtype == MG_F32 && out_dtype == MG_F32)
    hipLaunchKernelGGL((k_cast<float, float>), dim3(nblk(n)), dim3(256), 0, st, (const float*)in, (float*)out, n, alpha, square);
  else if (in_dtype == MG_F32)
    hipLaunchKernelGGL((k_cast<float, bf16_t>), dim3(nblk(n)), dim3(256), 0, st, (const float*)in, (bf16_t*)out, n, alpha, square);
  else if (out_dtype == MG_F32)
    hipLaunchKernelGGL((k_cast<bf16_t, float>), dim3(nblk(n)), dim3(256), 0, st, (const bf16_t*)in, (float*)out, n, alpha, square);
  else
    hipLaunchKernelGGL((k_cast<bf16_t, bf16_t>), dim3(nblk(n)), dim3(256), 0, st, (const bf16_t*)in, (bf16_t*)out, n, alpha, square);
  return mg_check_launch("mg_cast");
}

extern "C" int mg_copy2d(int in_dtype, const void* in, int64_t ldi, int out_dtype, void* out, int64_t ldo, int R,
                         int C, float alpha, int accumulate, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t n = (int64_t)R * C;
  if (n == 0) return MG_OK;
  if (in_dtype == MG_F32 && out_dtype == MG_F32)
    hipLaunchKernelGGL((k_copy2d<float, float>), dim3(nblk(n)), dim3(256), 0, st, (const float*)in, ldi, (float*)out, ldo, R, C, alpha, accumulate);
  else if (in_dtype == MG_F32)
    hipLaunchKernelGGL((k_copy2d<float, bf16_t>), dim3(nblk(n)), dim3(256), 0, st, (const float*)in, ldi, (bf16_t*)out, ldo, R, C, alpha, accumulate);
  else if (out_dtype == MG_F32)
    hipLaunchKernelGGL((k_copy2d<bf16_t, float>), dim3(nblk(n)), dim3(256), 0, st, (const bf16_t*)in, ldi, (float*)out, ldo, R, C, alpha, accumulate);
  else
    hipLaunchKernelGGL((k_copy2d<bf16_t, bf16_t>), dim3(nblk(n)), dim3(256), 0, st, (const bf16_t*)in, ldi, (bf16_t*)out, ldo, R, C, alpha, accumulate);
  return mg_check_launch("mg_copy2d");
}

extern "C" int mg_colsum(int dtype, const void* X, int64_t ld, int R, int C, float* out, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (R == 0 || C == 0) return MG_OK;
  if (C % 8 == 0 && ld % 8 == 0 && mg_al16(X) && mg_al16(out)) {
    int cv = C / 8;
    int tx = std::min(cv, 32);
    int ty = 256 / tx;
    int cblk = cdiv(cv, tx);
    // ~1024 blocks in total (every CU busy), at least 8 rows per lane
    int rblk = std::max(1, std::min({cdiv(R, 8 * ty), 1024 / cblk, 256}));
    int rpb = cdiv(R, rblk);
    rblk = cdiv(R, rpb);
    dim3 grid(cblk, rblk);
    if (rblk <= 16 && (rblk == 1 || !mg_det())) {  // (deterministic mode: one writer per column, or the fold)
      DISPATCH_T(dtype, hipLaunchKernelGGL(k_colsum_v<T>, grid, dim3(tx, ty), 0, st, reinterpret_cast<const T*>(X),
                                           ld, R, C, rpb, out, 1));
      return mg_check_launch("mg_colsum");
    }
    float* part = reinterpret_cast<float*>(mg_workspace((size_t)rblk * C * sizeof(float), st));
    if (!part) {
      mg_set_error("mg_colsum: workspace allocation failed");
      return MG_ERR_LAUNCH;
    }
    DISPATCH_T(dtype, hipLaunchKernelGGL(k_colsum_v<T>, grid, dim3(tx, ty), 0, st, reinterpret_cast<const T*>(X), ld,
                                         R, C, rpb, part, 0));
    hipLaunchKernelGGL(k_colsum_fin, dim3(cdiv(C, 64)), dim3(1024), 0, st, part, rblk, C, out);
    return mg_check_launch("mg_colsum");
  }
  int rpb = mg_det() ? std::max(R, 1) : std::max(16, R / 256);  // deterministic: one row block, one add per column
  dim3 grid(cdiv(C, 256), cdiv(R, rpb));
  DISPATCH_T(dtype, hipLaunchKernelGGL(k_colsum<T>, grid, dim3(256), 0, st, reinterpret_cast<const T*>(X), ld, R, C,
                                       rpb, out));
  return mg_check_launch("mg_colsum");
}

extern "C" int mg_weight_norm_fwd(const float* v, const float* g, int O, int K, float* W, float* norm, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_wn_fwd, dim3(O), dim3(256), 0, st, v, g, O, K, W, norm);
  return mg_check_launch("mg_weight_norm_fwd");
}

extern "C" int mg_weight_norm_bwd(const float* v, const float* g, const float* norm, const float* gW, int O, int K,
                                  float* gv, float* gg, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_wn_bwd, dim3(O), dim3(256), 0, st, v, g, norm, gW, O, K, gv, gg);
  return mg_check_launch("mg_weight_norm_bwd");
}

extern "C" int mg_weight_norm_batch(int bwd, int n, const mg_wn_desc* descs, void* stream) {
  MG_REQUIRE(n >= 0 && (n == 0 || descs), "bad descriptor table");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int i0 = 0; i0 < n; i0 += kWnMax) {
    WnArgs a{};
    a.bwd = bwd ? 1 : 0;
    int rows = 0;
    for (int i = i0; i < n && i < i0 + kWnMax; ++i) {
      const mg_wn_desc& q = descs[i];
      MG_REQUIRE(q.O > 0 && q.K > 0 && q.v && q.g && q.norm, "bad weight-norm descriptor");
      MG_REQUIRE(bwd ? (q.gW && q.gv && q.gg) : (q.W != nullptr), "weight-norm descriptor misses an operand");
      a.d[a.n] = q;
      a.row_off[a.n++] = rows;
      rows += q.O;
    }
    a.row_off[a.n] = rows;
    hipLaunchKernelGGL(k_wn_batch, dim3(rows), dim3(256), 0, st, a);
    int rc = mg_check_launch("mg_weight_norm_batch");
    if (rc) return rc;
  }
  return MG_OK;
}

extern "C" int mg_sumsq(const float* x, int64_t n, float* out, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n == 0) return MG_OK;
  const int blocks = std::min(nblk(n / 16 + 1), 1024);
  float* part = reinterpret_cast<float*>(mg_workspace(1024 * sizeof(float), st));
  MG_REQUIRE(part, "no workspace");
  hipLaunchKernelGGL(k_sumsq, dim3(blocks), dim3(256), 0, st, x, n, part);
  hipLaunchKernelGGL(k_sumsq_fin, dim3(1), dim3(256), 0, st, part, blocks, out);
  return mg_check_launch("mg_sumsq");
}

extern "C" int mg_grad_norm_steps(const float* x, int64_t n, float* out, int32_t* step0, int32_t run_mask0, int32_t* step1,
                                  int32_t run_mask1, const int32_t* flags, int32_t skip_mask, const int32_t* win,
                                  void* stream) {
  MG_REQUIRE(x && out, "null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int blocks = n > 0 ? std::min(nblk(n / 16 + 1), 1024) : 0;
  float* part = reinterpret_cast<float*>(mg_workspace(1024 * sizeof(float), st));
  MG_REQUIRE(part, "no workspace");
  if (blocks > 0) hipLaunchKernelGGL(k_sumsq, dim3(blocks), dim3(256), 0, st, x, n, part);
  hipLaunchKernelGGL(k_sumsq_fin_steps, dim3(1), dim3(256), 0, st, part, blocks, out, step0, run_mask0, step1, run_mask1,
                     flags, skip_mask, win);
  return mg_check_launch("mg_grad_norm_steps");
}

extern "C" int mg_adamw(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
                        float eps, float weight_decay, int step, const float* sumsq, float max_norm, void* stream) {
  MG_REQUIRE(step >= 1, "step must be >= 1");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n == 0) return MG_OK;
  float bc1 = 1.f - powf(beta1, (float)step);
  float bc2 = 1.f - powf(beta2, (float)step);
  hipLaunchKernelGGL(k_adamw, dim3(std::min(nblk(n), 4096)), dim3(256), 0, st, p, g, m, v, n, lr, beta1, beta2, eps,
                     weight_decay, bc1, sqrtf(bc2), sumsq, max_norm);
  return mg_check_launch("mg_adamw");
}

extern "C" int mg_opt_prologue(float* sumsq, int32_t* step, const int32_t* flags, int32_t skip_mask,
                               const int32_t* win, int32_t run_mask, void* stream) {
  MG_REQUIRE(sumsq || step, "null pointers");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_opt_prologue, dim3(1), dim3(64), 0, st, sumsq, step, flags, skip_mask, win, run_mask);
  return mg_check_launch("mg_opt_prologue");
}

extern "C" int mg_adamw_dev(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                            float beta2, float eps, float weight_decay, const int32_t* step, const float* sumsq,
                            float max_norm, void* stream) {
  MG_REQUIRE(step, "null step counter");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n == 0) return MG_OK;
  hipLaunchKernelGGL(k_adamw_dev, dim3(std::min(nblk(n), 4096)), dim3(256), 0, st, p, g, m, v, n, lr, beta1, beta2,
                     eps, weight_decay, step, sumsq, max_norm);
  return mg_check_launch("mg_adamw_dev");
}

extern "C" int mg_adamw_dev_shadow(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                                   float beta2, float eps, float weight_decay, const int32_t* step,
                                   const float* sumsq, float max_norm, void* shadow_bf16, const int32_t* flags,
                                   int32_t skip_mask, const int32_t* win, int32_t run_mask, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n == 0) return MG_OK;
  MG_REQUIRE(mg_al16(p) && mg_al16(g) && mg_al16(m) && mg_al16(v) &&
             (!shadow_bf16 || (reinterpret_cast<uintptr_t>(shadow_bf16) & 7) == 0), "16-B aligned p/g/m/v, 8-B shadow");
  const dim3 grid(std::max<int64_t>(1, std::min<int64_t>(cdiv(n / 4 + 1, 256), 4096)));
  if (g_mg_tune[MG_TUNE_ADAMW_CACHED] == 1)
    hipLaunchKernelGGL(k_adamw_dev_v<false>, grid, dim3(256), 0, st, p, g, m, v, n, lr, beta1, beta2, eps,
                       weight_decay, step, sumsq, max_norm, reinterpret_cast<bf16_t*>(shadow_bf16), flags, skip_mask,
                       win, run_mask);
  else
    hipLaunchKernelGGL(k_adamw_dev_v<true>, grid, dim3(256), 0, st, p, g, m, v, n, lr, beta1, beta2, eps,
                       weight_decay, step, sumsq, max_norm, reinterpret_cast<bf16_t*>(shadow_bf16), flags, skip_mask,
                       win, run_mask);
  return mg_check_launch("mg_adamw_dev_shadow");
}

extern "C" int mg_const_fwd(int dtype, const float* cst, int C, int HW, int B, void* out, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t n = (int64_t)B * HW * C;
  DISPATCH_T(dtype, hipLaunchKernelGGL(k_const_fwd<T>, dim3(nblk(n)), dim3(256), 0, st, cst, C, HW, B,
                                       reinterpret_cast<T*>(out)));
  return mg_check_launch("mg_const_fwd");
}

extern "C" int mg_const_bwd(int dtype, const void* g, int C, int HW, int B, float* gc, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int bchunk = mg_det() ? std::max(B, 1) : std::max(8, cdiv(B, 16));  // deterministic: one add per element
  DISPATCH_T(dtype, hipLaunchKernelGGL(k_const_bwd<T>, dim3(cdiv(C * HW, 256), cdiv(B, bchunk)), dim3(256), 0, st,
                                       reinterpret_cast<const T*>(g), C, HW, B, bchunk, gc));
  return mg_check_launch("mg_const_bwd");
}
