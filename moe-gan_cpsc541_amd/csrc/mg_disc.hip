// Discriminator pieces not covered by the implicit-GEMM convs (t2i_moe_gan.py:858-907)
// and the GAN / R1 loss reductions of the training step (t2i_moe_gan.py:1276-1312, :1379-1382).
//
//  * conv_layers.0 (3 -> 128, 4x4 / s2 / p1) has K = 48: an explicit im2col
//    (K padded to the vector width) feeds the generic GEMM, forward and weight-grad.
//  * output_layer (384 -> 1, 4x4 valid) has N = 1: a bandwidth-bound direct
//    kernel.  Its 128 text channels are spatially constant, so their
//    contribution is a per-image scalar tb[b] computed by a GEMV on the host
//    side; the kernel below handles the 256 image channels.
//  * R1 needs the gradient of sum(out) w.r.t. the image: the head's part of it
//    is the same for every image (it only depends on W2), so it is built once
//    with a broadcast "gradient of ones".
#include "mg_common.h"

namespace {

// im2col for a 4x4 / stride-2 / pad-1 conv: row = output pixel, col = (kh*4+kw)*C + c, padded to Kp
template <typename TI, typename TO>
__global__ void k_im2col(const TI* __restrict__ x, int64_t sb, int64_t sh, int64_t sw, int64_t sc, int B, int H,
                         int W, int C, int Kp, TO* __restrict__ out) {
  // one thread per (output pixel, 8-column group): consecutive threads write one pixel's row contiguously
  // (16-B stores when bf16 and Kp % 8 == 0), and each thread's 8 gathers are independent loads
  const int OH = H / 2, OW = W / 2;
  const int G = (Kp + 7) >> 3;
  const int np = B * OH * OW;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= np * G) return;
  const int r = i / G, k0 = (i - r * G) * 8;
  const int ow = r % OW, oh = (r / OW) % OH, b = r / (OW * OH);
  const TI* xb = x + (int64_t)b * sb;
  TO* o = out + (int64_t)r * Kp;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = k0 + j;
    v[j] = 0.f;
    if (k < 16 * C) {
      const int tap = k / C, c = k - tap * C;
      const int ih = 2 * oh - 1 + (tap >> 2), iw = 2 * ow - 1 + (tap & 3);
      if (ih >= 0 && ih < H && iw >= 0 && iw < W) v[j] = ldf(xb, ih * sh + iw * sw + c * sc);
    }
  }
  if (sizeof(TO) == 2 && (Kp & 7) == 0 && mg_al16(out)) {
    st8(reinterpret_cast<bf16_t*>(o) + k0, v);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (k0 + j < Kp) stf(o, k0 + j, v[j]);
  }
}

// col2im of a 4x4 / stride-2 / pad-1 conv's data gradient (few input channels): Y[b, oy, ox, (kh*4+kw)*C + c] =
// sum_co g[b, oy, ox, co] W[co, c, kh, kw] (one small GEMM), summed here into out[b, y, x, c] over the <= 4
// (oy, ox, kh, kw) with y = 2 oy - 1 + kh, x = 2 ox - 1 + kw.  One thread per input pixel.
template <typename TI, typename TO>
__global__ void k_col2im_4x4s2(const TI* __restrict__ Y, int64_t ldy, int B, int OH, int OW, int C,
                               TO* __restrict__ out, int64_t ldo) {
  const int H = 2 * OH, W = 2 * OW;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * H * W) return;
  const int x = i % W, y = (i / W) % H, b = i / (W * H);
  // kh has the parity of y + 1: kh0 = (y + 1) & 1, the two candidates kh0 and kh0 + 2
  const int kh0 = (y + 1) & 1, kw0 = (x + 1) & 1;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int kh = kh0 + 2 * a, oy = (y + 1 - kh) >> 1;
    if (oy < 0 || oy >= OH) continue;
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2) {
      const int kw = kw0 + 2 * c2, ox = (x + 1 - kw) >> 1;
      if (ox < 0 || ox >= OW) continue;
      const TI* row = Y + ((int64_t)(b * OH + oy) * OW + ox) * ldy + (kh * 4 + kw) * C;
      for (int c = 0; c < C && c < 4; ++c) acc[c] += ldf(row, c);
    }
  }
  TO* o = out + (int64_t)i * ldo;
  for (int c = 0; c < C && c < 4; ++c) stf(o, c, acc[c]);
}

// head, image channels: out[b, o] = sum_{c<256, kh, kw} h1[b, oy+kh, ox+kw, c] * W2[c, kh, kw]
// one wave per output pixel; lanes over channels
template <typename T>
__global__ void k_head_fwd(const T* __restrict__ h1, const float* __restrict__ W2, int B, int Hf, int Cf,
                           float* __restrict__ out) {
  int Ho = Hf - 3;
  int64_t n = (int64_t)B * Ho * Ho;
  int lane = threadIdx.x & 63;
  int64_t o = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (o >= n) return;
  int b = (int)(o / (Ho * Ho));
  int rem = (int)(o - (int64_t)b * Ho * Ho);
  int oy = rem / Ho, ox = rem - (rem / Ho) * Ho;
  float s = 0.f;
  for (int tap = 0; tap < 16; ++tap) {
    int kh = tap >> 2, kw = tap & 3;
    const T* row = h1 + (((int64_t)b * Hf + oy + kh) * Hf + ox + kw) * Cf;
    for (int c = lane; c < Cf; c += 64) s += ldf(row, c) * W2[c * 16 + tap];
  }
  s = wave_sum(s);
  if (lane == 0) out[o] = s;
}

// Head as GEMMs: the 4x4 valid conv to one channel is P = h1 @ W2 ([pixels, 16 taps], an MFMA GEMM)
// followed by a shifted 16-tap sum, and its backward uses the tap-expanded gradient
//   G[b, y, x, tap] = g[b, y - kh, x - kw]   (0 outside the Ho x Ho map)
// so that g_a1 = G @ W2^T (epilogue: * lrelu') and dW2 = h1^T G are GEMMs as well.
template <typename TO>
__global__ __launch_bounds__(256) void k_head_gmat(const float* __restrict__ g, int64_t g_bstride, int B, int Hf,
                                                   TO* __restrict__ G) {
  const int Ho = Hf - 3;
  const int n = B * Hf * Hf;
  for (int p = blockIdx.x * 256 + threadIdx.x; p < n; p += gridDim.x * 256) {
    int x = p % Hf, t = p / Hf, y = t % Hf, b = t / Hf;
    const float* gb = g + (int64_t)b * g_bstride;
    float v[16];
#pragma unroll
    for (int kh = 0; kh < 4; ++kh)
#pragma unroll
      for (int kw = 0; kw < 4; ++kw) {
        int oy = y - kh, ox = x - kw;
        v[kh * 4 + kw] = ((unsigned)oy < (unsigned)Ho && (unsigned)ox < (unsigned)Ho) ? gb[oy * Ho + ox] : 0.f;
      }
    st8(G + (int64_t)p * 16, v);
    st8(G + (int64_t)p * 16 + 8, v + 8);
  }
}

__global__ __launch_bounds__(256) void k_head_sum(const float* __restrict__ P, int B, int Hf, float* __restrict__ out) {
  const int Ho = Hf - 3;
  const int n = B * Ho * Ho;
  for (int o = blockIdx.x * 256 + threadIdx.x; o < n; o += gridDim.x * 256) {
    int ox = o % Ho, t = o / Ho, oy = t % Ho, b = t / Ho;
    float s = 0.f;
#pragma unroll
    for (int kh = 0; kh < 4; ++kh)
#pragma unroll
      for (int kw = 0; kw < 4; ++kw) s += P[((int64_t)(b * Hf + oy + kh) * Hf + ox + kw) * 16 + kh * 4 + kw];
    out[o] = s;
  }
}

// head backward into the image features, fused with conv_layers.2's LeakyReLU:
//   g_a1[b, y, x, c] = lrelu'(a1[b,y,x,c]) * sum_{oy,ox} g[b, oy, ox] * W2[c, y-oy, x-ox]
// g_bstride = 0 broadcasts one gradient map to every image (R1: gradient of sum(out)).
template <typename T, typename TO>
__global__ void k_head_bwd_data(const float* __restrict__ g, int64_t g_bstride, const float* __restrict__ W2,
                                const T* __restrict__ a1, int B, int Hf, int Cf, TO* __restrict__ ga1) {
  int Ho = Hf - 3;
  int64_t n = (int64_t)B * Hf * Hf * Cf;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int c = (int)(i % Cf);
    int64_t pix = i / Cf;
    int x = (int)(pix % Hf), y = (int)((pix / Hf) % Hf), b = (int)(pix / ((int64_t)Hf * Hf));
    const float* gb = g + (int64_t)b * g_bstride;
    float s = 0.f;
    for (int kh = 0; kh < 4; ++kh) {
      int oy = y - kh;
      if (oy < 0 || oy >= Ho) continue;
      for (int kw = 0; kw < 4; ++kw) {
        int ox = x - kw;
        if (ox < 0 || ox >= Ho) continue;
        s += gb[oy * Ho + ox] * W2[c * 16 + kh * 4 + kw];
      }
    }
    if (a1) s *= lrelu_grad(ldf(a1, i));
    stf(ga1, i, s);
  }
}

// dW2[c, tap] += sum_b sum_o g[b, o] * h1[b, o + tap, c]   (block per image, thread per channel)
template <typename T>
__global__ void k_head_bwd_w(const float* __restrict__ g, int64_t g_bstride, const T* __restrict__ h1, int Hf,
                             int Cf, float* __restrict__ dW2, float* __restrict__ part) {
  int b = blockIdx.x;
  int c = threadIdx.x;
  if (c >= Cf) return;
  int Ho = Hf - 3;
  const float* gb = g + (int64_t)b * g_bstride;
  float acc[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) acc[t] = 0.f;
  for (int oy = 0; oy < Ho; ++oy)
    for (int ox = 0; ox < Ho; ++ox) {
      float gv = gb[oy * Ho + ox];
#pragma unroll
      for (int t = 0; t < 16; ++t)
        acc[t] += gv * ldf(h1, (((int64_t)b * Hf + oy + (t >> 2)) * Hf + ox + (t & 3)) * Cf + c);
    }
  if (part) {  // deterministic mode: the image's row, folded over images in order by the launcher
#pragma unroll
    for (int t = 0; t < 16; ++t) part[((int64_t)b * Cf + c) * 16 + t] = acc[t];
    return;
  }
#pragma unroll
  for (int t = 0; t < 16; ++t) atomicAdd(&dW2[c * 16 + t], acc[t]);
}

// D loss (t2i_moe_gan.py:940-949, :1309).  img_real = image part of the 64x64 real logits
// [B, No]; img_fake = image part of the 16x16 fake logits [B]; tb[b] = text part + bias of
// image b's caption.  real = img_real + tb[b]; mism = img_real + tb[perm[b]]; fake = img_fake + tb[b].
// out (zeroed by caller): [0] d_loss_gan, [1] mean softplus(-real), [2] mean softplus(fake), [3] mean softplus(mism)
// g_img_real / g_img_fake: d loss / d image-part logits; g_tb (zeroed): d loss / d tb.
__global__ void k_d_loss(const float* __restrict__ img, const float* __restrict__ img_fake,
                         const float* __restrict__ tb, const int* __restrict__ perm, int B, int No, int Nf,
                         float* __restrict__ out, float* __restrict__ g_img, float* __restrict__ g_fake,
                         float* __restrict__ g_tb, float* __restrict__ real_out, float* __restrict__ mism_out,
                         float* __restrict__ fake_out, float* __restrict__ part) {
  // part (deterministic mode): per block [out0, out1, out2, out3, g_tb self, g_tb perm] instead of the atomics
  // below, folded in block order by k_d_loss_fold
  __shared__ float red[4][16];
  int b = blockIdx.x;
  float sr = 0.f, sm = 0.f, gr = 0.f, gm = 0.f;
  float inv = 1.f / ((float)B * No);
  if (b > B) {
    // fake logits with Nf > 1 per image (progressive generator, images >= 32x32): one block per image
    int i = b - B - 1;
    float tf = tb[i], invf = 1.f / ((float)B * Nf), sf = 0.f, gs = 0.f;
    for (int o = threadIdx.x; o < Nf; o += blockDim.x) {
      int64_t e = (int64_t)i * Nf + o;
      float f = img_fake[e] + tf;
      if (fake_out) fake_out[e] = f;
      sf += (f > 20.f) ? f : log1pf(expf(f));
      float gf = 1.f / (1.f + expf(-f)) * invf;
      g_fake[e] = gf;
      gs += gf;
    }
    sf = wave_sum(sf); gs = wave_sum(gs);
    int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { red[0][w] = sf; red[1][w] = gs; }
    __syncthreads();
    if (threadIdx.x == 0) {
      float a = 0, c = 0;
      for (int k = 0; k < (int)(blockDim.x >> 6); ++k) { a += red[0][k]; c += red[1][k]; }
      if (part) {
        float* pr = part + (int64_t)b * 6;
        pr[0] = a * invf; pr[1] = 0.f; pr[2] = a * invf; pr[3] = 0.f; pr[4] = c; pr[5] = 0.f;
        return;
      }
      atomicAdd(&out[2], a * invf);
      atomicAdd(&out[0], a * invf);
      atomicAdd(&g_tb[i], c);
    }
    return;
  }
  if (b < B) {
    float tr = tb[b], tm = tb[perm[b]];
    for (int o = threadIdx.x; o < No; o += blockDim.x) {
      float base = img[(int64_t)b * No + o];
      float r = base + tr, m = base + tm;
      if (real_out) real_out[(int64_t)b * No + o] = r;
      if (mism_out) mism_out[(int64_t)b * No + o] = m;
      float spr = (-r > 20.f) ? -r : log1pf(expf(-r));  // softplus, torch threshold 20
      float spm = (m > 20.f) ? m : log1pf(expf(m));
      sr += spr;
      sm += spm;
      float dr = -1.f / (1.f + expf(r)) * inv;  // d softplus(-r)/dr = -sigmoid(-r)
      float dm = 1.f / (1.f + expf(-m)) * inv;
      g_img[(int64_t)b * No + o] = dr + dm;
      gr += dr;
      gm += dm;
    }
    sr = wave_sum(sr); sm = wave_sum(sm); gr = wave_sum(gr); gm = wave_sum(gm);
    int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { red[0][w] = sr; red[1][w] = sm; red[2][w] = gr; red[3][w] = gm; }
    __syncthreads();
    if (threadIdx.x == 0) {
      float a = 0, c = 0, d = 0, e = 0;
      for (int i = 0; i < (int)(blockDim.x >> 6); ++i) { a += red[0][i]; c += red[1][i]; d += red[2][i]; e += red[3][i]; }
      if (part) {
        float* pr = part + (int64_t)b * 6;
        pr[0] = (a + c) * inv; pr[1] = a * inv; pr[2] = 0.f; pr[3] = c * inv; pr[4] = d; pr[5] = e;
        return;
      }
      atomicAdd(&out[1], a * inv);
      atomicAdd(&out[3], c * inv);
      atomicAdd(&out[0], (a + c) * inv);
      atomicAdd(&g_tb[b], d);
      atomicAdd(&g_tb[perm[b]], e);
    }
  } else if (Nf == 1) {
    float sf = 0.f;
    for (int i = threadIdx.x; i < B; i += blockDim.x) {
      float f = img_fake[i] + tb[i];
      if (fake_out) fake_out[i] = f;
      sf += (f > 20.f) ? f : log1pf(expf(f));
      float gf = 1.f / (1.f + expf(-f)) / B;
      g_fake[i] = gf;
      if (!part) atomicAdd(&g_tb[i], gf);  // (deterministic mode: k_d_loss_fold reads g_fake)
    }
    sf = wave_sum(sf);
    if ((threadIdx.x & 63) == 0) red[0][threadIdx.x >> 6] = sf;
    __syncthreads();
    if (threadIdx.x == 0) {
      float a = 0;
      for (int i = 0; i < (int)(blockDim.x >> 6); ++i) a += red[0][i];
      if (part) {
        float* pr = part + (int64_t)b * 6;
        pr[0] = a / B; pr[1] = 0.f; pr[2] = a / B; pr[3] = 0.f; pr[4] = 0.f; pr[5] = 0.f;
        return;
      }
      atomicAdd(&out[2], a / B);
      atomicAdd(&out[0], a / B);
    }
  } else if (part && threadIdx.x == 0) {
    // Nf > 1: block B has no work (the fakes are blocks B+1..2B), but k_d_loss_fold sums every row
    float* pr = part + (int64_t)b * 6;
    pr[0] = 0.f; pr[1] = 0.f; pr[2] = 0.f; pr[3] = 0.f; pr[4] = 0.f; pr[5] = 0.f;
  }
}

// Deterministic mode: fold k_d_loss's block rows in block order.  out[k] += sum_blk part[blk][k]; g_tb[i] += own
// real-block term + the terms of the real blocks b with perm[b] == i + the fake term of image i.
__global__ __launch_bounds__(256) void k_d_loss_fold(const float* __restrict__ part, int nblk, const int* __restrict__ perm,
                                                     int B, int Nf, const float* __restrict__ g_fake,
                                                     float* __restrict__ out, float* __restrict__ g_tb) {
  if (threadIdx.x < 4) {
    float s = 0.f;
    for (int k = 0; k < nblk; ++k) s += part[(int64_t)k * 6 + threadIdx.x];
    out[threadIdx.x] += s;
  }
  for (int i = threadIdx.x; i < B; i += blockDim.x) {
    float s = part[(int64_t)i * 6 + 4];
    for (int b = 0; b < B; ++b)
      if (perm[b] == i) s += part[(int64_t)b * 6 + 5];
    s += Nf == 1 ? g_fake[i] : part[(int64_t)(B + 1 + i) * 6 + 4];
    g_tb[i] += s;
  }
}

// G adversarial loss softplus(-f).mean() (t2i_moe_gan.py:919) and its gradient
// Grid-stride over the B logits; with one block the block writes the mean, with several each block writes its
// partial sum and k_g_loss_fin folds them in block order (deterministic).  The progressive stages' multi-logit fakes
// (B x 841 at 128^2) would take 500 us in one block.
__global__ void k_g_loss(const float* __restrict__ fake, int B, float scale, float* __restrict__ out,
                         float* __restrict__ g, float* __restrict__ part) {
  __shared__ float red[16];
  float s = 0.f;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < B; i += gridDim.x * blockDim.x) {
    float f = fake[i];
    s += (-f > 20.f) ? -f : log1pf(expf(-f));
    g[i] = -1.f / (1.f + expf(f)) / B * scale;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) a += red[i];
    if (part) part[blockIdx.x] = a;
    else out[0] = a / B;
  }
}
__global__ void k_g_loss_fin(const float* __restrict__ part, int nb, int B, float* __restrict__ out) {
  float s = 0.f;
  for (int i = threadIdx.x; i < nb; i += 64) s += part[i];
  s = wave_sum(s);
  if (threadIdx.x == 0) out[0] = s / B;
}

// R1 (t2i_moe_gan.py:1285-1286): r1 = gamma/2 * mean_b ||g_b||^2; u = gamma/B * g  (d r1 / d g)
// One block per image: a single same-address atomic per image (a grid of per-chunk blocks serialised
// ~16k atomics on r1 at the memory side).
template <typename T, typename TU>
__global__ void k_r1(const T* __restrict__ g, int64_t per, int B, float gamma, float* __restrict__ r1,
                     TU* __restrict__ u, float* __restrict__ part) {
  __shared__ float red[16];
  int b = blockIdx.x;
  float s = 0.f;
  const T* gb = g + (int64_t)b * per;
  if ((per & 7) == 0 && mg_al16(gb) && (!u || mg_al16(u + (int64_t)b * per))) {
    float v[8];
    for (int64_t i = (int64_t)threadIdx.x * 8; i < per; i += (int64_t)blockDim.x * 8) {
      ld8(gb + i, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s += v[j] * v[j];
        v[j] *= gamma / B;
      }
      if (u) st8(u + (int64_t)b * per + i, v);
    }
  } else {
    for (int64_t i = threadIdx.x; i < per; i += blockDim.x) {
      float v = ldf(gb, i);
      s += v * v;
      if (u) stf(u, (int64_t)b * per + i, gamma / B * v);
    }
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) a += red[i];
    if (part) part[b] = a * gamma * 0.5f / B;  // deterministic mode: folded in image order
    else atomicAdd(r1, a * gamma * 0.5f / B);
  }
}

// out = a * lrelu'(m)  (elementwise; m = pre- or post-activation, same sign)
template <typename T, typename TM, typename TO>
__global__ void k_mask_mul(const T* __restrict__ a, const TM* __restrict__ m, int64_t n, TO* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    stf(out, i, ldf(a, i) * lrelu_grad(ldf(m, i)));
}

// text branch of the head (t2i_moe_gan.py:895-902): tb[b] = sum_c t[b,c] * w2sum[c] (+ bias)
//   g_tpre[b,c] = g_tb[b] * w2sum[c] * lrelu'(t[b,c]);  dW2[256+c, tap] += sum_b g_tb[b] * t[b,c]  (all 16 taps)
// block = 64 columns x 4 image lanes over a chunk of TB_CHUNK images; partial column sums folded in LDS,
// then one atomic per (column, tap) per block.
constexpr int TB_CHUNK = 32;
__global__ __launch_bounds__(256) void k_d_text_bwd(const float* __restrict__ g_tb, const float* __restrict__ t,
                                                    const float* __restrict__ w2sum, int B, int Ct, int cofs,
                                                    float* __restrict__ g_tpre, float* __restrict__ dW2,
                                                    float* __restrict__ part) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int b0 = blockIdx.y * TB_CHUNK, b1 = min(B, b0 + TB_CHUNK);
  float acc = 0.f;
  if (c < Ct) {
    const float ws = w2sum[c];
    for (int b = b0 + q; b < b1; b += 4) {
      float tv = t[(int64_t)b * Ct + c];
      float gb = g_tb[b];
      acc += gb * tv;
      g_tpre[(int64_t)b * Ct + c] = gb * ws * lrelu_grad(tv);
    }
  }
  red[q][cl] = acc;
  __syncthreads();
  if (q == 0 && c < Ct) {
    float s = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
    if (part) {  // deterministic mode: one row per image chunk, folded in chunk order into all 16 taps
      for (int tap = 0; tap < 16; ++tap) part[((int64_t)blockIdx.y * Ct + c) * 16 + tap] = s;
      return;
    }
    for (int tap = 0; tap < 16; ++tap) atomicAdd(&dW2[(int64_t)(cofs + c) * 16 + tap], s);
  }
}

inline int nblk(int64_t n, int t = 256) { return (int)std::min<int64_t>((n + t - 1) / t, 65536); }

}  // namespace

extern "C" int mg_d_text_bwd(const float* g_tb, const float* t, const float* w2sum, int B, int Ct, int cofs,
                             float* g_tpre, float* dW2, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int nch = cdiv(B, TB_CHUNK);
  float* part = nullptr;
  if (mg_det()) {
    part = reinterpret_cast<float*>(mg_workspace((size_t)nch * Ct * 16 * sizeof(float), st));
    if (!part) return MG_ERR_LAUNCH;
  }
  hipLaunchKernelGGL(k_d_text_bwd, dim3(cdiv(Ct, 64), nch), dim3(256), 0, st, g_tb, t, w2sum, B, Ct,
                     cofs, g_tpre, dW2, part);
  if (part) mg_det_fold_rows(part, nch, Ct * 16, Ct * 16, dW2 + (int64_t)cofs * 16, dW2 + (int64_t)cofs * 16, st);
  return mg_check_launch("mg_d_text_bwd");
}

extern "C" int mg_im2col_4x4s2(int in_dtype, const void* x, int64_t sb, int64_t sh, int64_t sw, int64_t sc, int B,
                               int H, int W, int C, int Kp, int out_dtype, void* out, void* stream) {
  MG_REQUIRE(Kp >= 16 * C, "Kp too small");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t nt = (int64_t)B * (H / 2) * (W / 2) * ((Kp + 7) / 8);
  MG_REQUIRE(nt < (1LL << 31), "too many pixels");
#define L_(TI, TO) hipLaunchKernelGGL((k_im2col<TI, TO>), dim3(cdiv(nt, 256)), dim3(256), 0, st, (const TI*)x, sb, sh, sw, sc, B, H, W, C, Kp, (TO*)out)
  if (in_dtype == MG_F32) { if (out_dtype == MG_F32) L_(float, float); else L_(float, bf16_t); }
  else { if (out_dtype == MG_F32) L_(bf16_t, float); else L_(bf16_t, bf16_t); }
#undef L_
  return mg_check_launch("mg_im2col_4x4s2");
}

extern "C" int mg_col2im_4x4s2(int in_dtype, const void* Y, int64_t ldy, int B, int OH, int OW, int C,
                               int out_dtype, void* out, int64_t ldo, void* stream) {
  MG_REQUIRE(C >= 1 && C <= 4, "1 <= C <= 4");
  MG_REQUIRE(ldy >= 16 * C && ldo >= C, "bad pitches");
  const int64_t n = (int64_t)B * 4 * OH * OW;
  MG_REQUIRE(n < (1LL << 31), "too many pixels");
  if (n == 0) return MG_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define L_(TI, TO) hipLaunchKernelGGL((k_col2im_4x4s2<TI, TO>), dim3(cdiv(n, 256)), dim3(256), 0, st, (const TI*)Y, ldy, B, OH, OW, C, (TO*)out, ldo)
  if (in_dtype == MG_F32) { if (out_dtype == MG_F32) L_(float, float); else L_(float, bf16_t); }
  else { if (out_dtype == MG_F32) L_(bf16_t, float); else L_(bf16_t, bf16_t); }
#undef L_
  return mg_check_launch("mg_col2im_4x4s2");
}

extern "C" int mg_disc_head_fwd(int dtype, const void* h1, const float* W2, int B, int Hf, int Cf, float* out,
                                void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t n = (int64_t)B * (Hf - 3) * (Hf - 3);
  dim3 grid((unsigned)((n + 3) / 4));
  if (dtype == MG_F32) hipLaunchKernelGGL(k_head_fwd<float>, grid, dim3(256), 0, st, (const float*)h1, W2, B, Hf, Cf, out);
  else hipLaunchKernelGGL(k_head_fwd<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)h1, W2, B, Hf, Cf, out);
  return mg_check_launch("mg_disc_head_fwd");
}

extern "C" int mg_disc_head_gmat(int out_dtype, const float* g, int64_t g_bstride, int B, int Hf, void* G,
                                 void* stream) {
  MG_REQUIRE(Hf >= 4, "Hf >= 4");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t n = (int64_t)B * Hf * Hf;
  if (n == 0) return MG_OK;
  if (out_dtype == MG_F32)
    hipLaunchKernelGGL(k_head_gmat<float>, dim3(nblk(n)), dim3(256), 0, st, g, g_bstride, B, Hf, (float*)G);
  else
    hipLaunchKernelGGL(k_head_gmat<bf16_t>, dim3(nblk(n)), dim3(256), 0, st, g, g_bstride, B, Hf, (bf16_t*)G);
  return mg_check_launch("mg_disc_head_gmat");
}

extern "C" int mg_disc_head_sum(const float* P, int B, int Hf, float* out, void* stream) {
  MG_REQUIRE(Hf >= 4, "Hf >= 4");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t n = (int64_t)B * (Hf - 3) * (Hf - 3);
  if (n == 0) return MG_OK;
  hipLaunchKernelGGL(k_head_sum, dim3(nblk(n)), dim3(256), 0, st, P, B, Hf, out);
  return mg_check_launch("mg_disc_head_sum");
}

extern "C" int mg_disc_head_bwd_data(int dtype, const float* g, int64_t g_bstride, const float* W2, const void* a1,
                                     int B, int Hf, int Cf, int out_dtype, void* ga1, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t n = (int64_t)B * Hf * Hf * Cf;
#define L_(T, TO) hipLaunchKernelGGL((k_head_bwd_data<T, TO>), dim3(nblk(n)), dim3(256), 0, st, g, g_bstride, W2, (const T*)a1, B, Hf, Cf, (TO*)ga1)
  if (dtype == MG_F32) { if (out_dtype == MG_F32) L_(float, float); else L_(float, bf16_t); }
  else { if (out_dtype == MG_F32) L_(bf16_t, float); else L_(bf16_t, bf16_t); }
#undef L_
  return mg_check_launch("mg_disc_head_bwd_data");
}

extern "C" int mg_disc_head_bwd_w(int dtype, const float* g, int64_t g_bstride, const void* h1, int B, int Hf, int Cf,
                                  float* dW2, void* stream) {
  MG_REQUIRE(Cf <= 1024, "Cf <= 1024");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int thr = ((Cf + 63) / 64) * 64;
  float* part = nullptr;
  if (mg_det()) {
    part = reinterpret_cast<float*>(mg_workspace((size_t)B * Cf * 16 * sizeof(float), st));
    if (!part) return MG_ERR_LAUNCH;
  }
  if (dtype == MG_F32) hipLaunchKernelGGL(k_head_bwd_w<float>, dim3(B), dim3(thr), 0, st, g, g_bstride, (const float*)h1, Hf, Cf, dW2, part);
  else hipLaunchKernelGGL(k_head_bwd_w<bf16_t>, dim3(B), dim3(thr), 0, st, g, g_bstride, (const bf16_t*)h1, Hf, Cf, dW2, part);
  if (part) mg_det_fold_rows(part, B, Cf * 16, Cf * 16, dW2, dW2, st);
  return mg_check_launch("mg_disc_head_bwd_w");
}

extern "C" int mg_d_loss(const float* img_real, const float* img_fake, const float* tb, const int32_t* perm, int B,
                         int No, int Nf, float* out, float* g_img, float* g_fake, float* g_tb, float* real_out,
                         float* mism_out, float* fake_out, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  MG_REQUIRE(B > 0 && No > 0 && Nf > 0, "mg_d_loss: B, No, Nf must be positive");
  // block B (one logit per fake, the reference's 16x16 fakes) or blocks B+1..2B (Nf logits per fake image)
  int grid = Nf == 1 ? B + 1 : 2 * B + 1;
  float* part = nullptr;
  if (mg_det()) {
    part = reinterpret_cast<float*>(mg_workspace((size_t)grid * 6 * sizeof(float), st));
    if (!part) return MG_ERR_LAUNCH;
  }
  hipLaunchKernelGGL(k_d_loss, dim3(grid), dim3(256), 0, st, img_real, img_fake, tb, perm, B, No, Nf, out, g_img,
                     g_fake, g_tb, real_out, mism_out, fake_out, part);
  if (part) hipLaunchKernelGGL(k_d_loss_fold, dim3(1), dim3(256), 0, st, part, grid, perm, B, Nf, g_fake, out, g_tb);
  return mg_check_launch("mg_d_loss");
}

extern "C" int mg_g_loss(const float* fake, int B, float scale, float* out, float* g, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int nb = std::min(256, std::max(1, B / 4096));
  float* part = nullptr;
  if (nb > 1) {
    part = reinterpret_cast<float*>(mg_workspace(nb * sizeof(float), st));
    MG_REQUIRE(part, "mg_g_loss: no workspace");
  }
  hipLaunchKernelGGL(k_g_loss, dim3(nb), dim3(256), 0, st, fake, B, scale, out, g, part);
  if (nb > 1) hipLaunchKernelGGL(k_g_loss_fin, dim3(1), dim3(64), 0, st, part, nb, B, out);
  return mg_check_launch("mg_g_loss");
}

extern "C" int mg_r1(int dtype, const void* g, int64_t per, int B, float gamma, float* r1, int u_dtype, void* u,
                     void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 grid(B);
  float* part = nullptr;
  if (mg_det()) {
    part = reinterpret_cast<float*>(mg_workspace((size_t)B * sizeof(float), st));
    if (!part) return MG_ERR_LAUNCH;
  }
#define L_(T, TU) hipLaunchKernelGGL((k_r1<T, TU>), grid, dim3(256), 0, st, (const T*)g, per, B, gamma, r1, (TU*)u, part)
  if (dtype == MG_F32) { if (u_dtype == MG_F32) L_(float, float); else L_(float, bf16_t); }
  else { if (u_dtype == MG_F32) L_(bf16_t, float); else L_(bf16_t, bf16_t); }
#undef L_
  if (part) hipLaunchKernelGGL(k_det_sum, dim3(1), dim3(256), 0, st, part, B, r1);
  return mg_check_launch("mg_r1");
}

extern "C" int mg_lrelu_mask_mul(int a_dtype, const void* a, int m_dtype, const void* m, int64_t n, int out_dtype,
                                 void* out, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define L_(T, TM, TO) hipLaunchKernelGGL((k_mask_mul<T, TM, TO>), dim3(nblk(n)), dim3(256), 0, st, (const T*)a, (const TM*)m, n, (TO*)out)
  if (a_dtype == MG_F32) {
    if (m_dtype == MG_F32) { if (out_dtype == MG_F32) L_(float, float, float); else L_(float, float, bf16_t); }
    else { if (out_dtype == MG_F32) L_(float, bf16_t, float); else L_(float, bf16_t, bf16_t); }
  } else {
    if (m_dtype == MG_F32) { if (out_dtype == MG_F32) L_(bf16_t, float, float); else L_(bf16_t, float, bf16_t); }
    else { if (out_dtype == MG_F32) L_(bf16_t, bf16_t, float); else L_(bf16_t, bf16_t, bf16_t); }
  }
#undef L_
  return mg_check_launch("mg_lrelu_mask_mul");
}
