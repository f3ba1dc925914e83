// The discriminator's first convolution, conv_layers.0 (3 -> 128, 4x4 / stride 2 / pad 1, t2i_moe_gan.py:874-880),
// as direct MFMA kernels for the bf16 step: forward (+ the R1 forward-mode pass), weight gradient and image
// gradient, without the [pixels x 48] im2col matrix and without the [pixels x 48] fp32 column-gradient matrix.
//
// The contraction is short (K = 16 taps x 3 channels = 48, padded to 64 for two v_mfma_f32_16x16x32_bf16 k-steps)
// and the channel count small, so every pass is bound by HBM bytes of the 128-channel activation (h0 / its
// gradient: 256 B per output pixel); the im2col + GEMM path moved ~1.4x those bytes and ran its single-K-step tiles
// latency-bound (27-50 us per pass at B=256, 64x64 images, vs ~9-13 us of HBM time).
//
//  * k_d0_fwd: one block per 128 consecutive output pixels.  The 128 x 48 patch tile is gathered straight from the
//    image (fp32 NCHW real images or the R1 pass's bf16 NHWC image) into an LDS KC image; W0 fragments come from
//    global memory (12 KiB, cache-resident).  Transposed MFMA products leave four consecutive channels of one
//    pixel per lane; the tile is staged through LDS and written as contiguous 16-B rows (the block's 128 pixels
//    are one 32 KiB run of h0).  Mode 0: + bias, LeakyReLU (h0).  Mode 1 (R1 forward-mode, :1282-1286):
//    * LeakyReLU'(h0) read from the same LDS staging buffer (m0 v0).  Same MFMA sequence over k as the GEMM path,
//    same fp32 epilogue, one bf16 rounding: bit-identical to im2col + mg_gemm.
//  * k_d0_wgrad: dW0[o][tap*3+c] += sum_p g[p][o] patch[p][tap*3+c].  Blocks stride over 128-pixel tiles; the
//    gradient tile [p][o] is stored as it arrives and the patch tile [p][k] likewise (MC images), both read with
//    the hardware transpose (ds_read_b64_tr_b16) so the reduction over pixels runs on MFMA.  The next tile's
//    global loads are issued before the current tile's products.  Per-block [128 x 48] partials are folded in
//    block order (deterministic in both modes).
//  * k_d0_dgrad: one block per image and band of RI input rows.  It loads the RI/2 + 2 gradient rows that band
//    needs into LDS, forms Y = g W0 ([pixels x 48], fp32, the same four MFMA k-steps as the GEMM path) into LDS
//    and sums every input pixel's <= 4 contributions in k_col2im_4x4s2's order: bit-identical to that path.
#include "mg_common.h"

namespace {

typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

constexpr int D0_T = 256;   // threads per block
constexpr int D0_BM = 128;  // output pixels per tile

// KC image [row][64] bf16: 16-B chunk (k / 8) of row r at chunk (k / 8) ^ (r & 7) -- conflict-free b128 reads
MG_DEV int kc64(int r, int k) { return r * 64 + ((((k >> 3) ^ (r & 7))) << 3) + (k & 7); }

// MC image [krow][ld] bf16 (columns contiguous), columns XOR-swizzled by 16 on odd k-octets
MG_DEV int mc_swz(int k) { return ((k >> 3) & 1) << 4; }
MG_DEV int mci(int k, int c, int ld) { return k * ld + (c ^ mc_swz(k)); }

// v_mfma_f32_16x16x32_bf16 operand from an MC image: lane (g = lane>>4, i = lane&15) gets column c0+i of k-rows
// kr0+8g .. kr0+8g+7 (two transposed 4-row reads)
MG_DEV bf16x8_t mc_frag(const bf16_t* img, int ld, int kr0, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int k = kr0 + 8 * g + q;
  auto base = (__attribute__((address_space(3))) char*)(img);
  const int col_lo = (c0 ^ mc_swz(k)) + 4 * p, col_hi = (c0 ^ mc_swz(k + 4)) + 4 * p;
  s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(base + ((int64_t)k * ld + col_lo) * 2));
  s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(base + ((int64_t)(k + 4) * ld + col_hi) * 2));
  u16x8_t r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return __builtin_bit_cast(bf16x8_t, r);
}

MG_DEV u16x8_t pack8(const float* v) {
  u16x8_t r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = f2bf(v[j]);
  return r;
}

// the 8 patch values k0 .. k0+7 (k = tap*3 + c, zero past 48 and outside the image) of output pixel p
template <typename TI>
MG_DEV u16x8_t patch8(const TI* __restrict__ x, int64_t sb, int64_t sh, int64_t sw, int64_t sc, int H, int W, int OH,
                      int OW, int P, int p, int k0) {
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = 0.f;
  if (p < P && k0 < 48) {
    const int ox = p % OW, oy = (p / OW) % OH, b = p / (OW * OH);
    const TI* xb = x + (int64_t)b * sb;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = k0 + j, tap = k / 3, c = k - tap * 3;
      const int ih = 2 * oy - 1 + (tap >> 2), iw = 2 * ox - 1 + (tap & 3);
      if (ih >= 0 && ih < H && iw >= 0 && iw < W) v[j] = ldf(xb, ih * sh + iw * sw + c * sc);
    }
  }
  return pack8(v);  // fp32 images: the same RNE rounding as mg_im2col_4x4s2's bf16 output
}

// W0 (packed [128][48] bf16, k = tap*3 + c) as the B operand of output channels o = 16 nf + (lane & 15), k-step ks
MG_DEV bf16x8_t w0_frag_rows(const bf16_t* __restrict__ w0, int nf, int ks, int lane) {
  const int o = 16 * nf + (lane & 15), k = 32 * ks + 8 * (lane >> 4);
  u16x8_t r = u16x8_t(0);
  if (k < 48) r = *reinterpret_cast<const u16x8_t*>(w0 + o * 48 + k);
  return __builtin_bit_cast(bf16x8_t, r);
}

constexpr int OS_LD = 136;  // output / aux staging pitch (bf16): 272-B rows, 16-B aligned

template <typename TI, int MODE>
__global__ __launch_bounds__(D0_T) void k_d0_fwd(const TI* __restrict__ x, int64_t sb, int64_t sh, int64_t sw,
                                                 int64_t sc, int H, int W, int P, const bf16_t* __restrict__ w0,
                                                 const float* __restrict__ bias, const bf16_t* __restrict__ aux,
                                                 bf16_t* __restrict__ out) {
  __shared__ bf16_t As[D0_BM * 64];
  __shared__ bf16_t Os[D0_BM * OS_LD];
  const int OH = H / 2, OW = W / 2;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int p0 = blockIdx.x * D0_BM;
  // patch tile -> LDS (rows past P are zeros); mode 1: the LeakyReLU' operand tile, coalesced 16-B runs
#pragma unroll
  for (int j = 0; j < D0_BM * 8 / D0_T; ++j) {
    const int i = tid + j * D0_T, r = i >> 3, ch = i & 7;
    *reinterpret_cast<u16x8_t*>(As + kc64(r, ch * 8)) = patch8(x, sb, sh, sw, sc, H, W, OH, OW, P, p0 + r, ch * 8);
  }
  if (MODE == 1) {
#pragma unroll
    for (int j = 0; j < D0_BM * 16 / D0_T; ++j) {
      const int i = tid + j * D0_T, r = i >> 4, c = (i & 15) * 8;
      if (p0 + r < P)
        *reinterpret_cast<u16x8_t*>(Os + r * OS_LD + c) =
            *reinterpret_cast<const u16x8_t*>(aux + (int64_t)(p0 + r) * 128 + c);
    }
  }
  bf16x8_t bw[8][2];
#pragma unroll
  for (int nf = 0; nf < 8; ++nf)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) bw[nf][ks] = w0_frag_rows(w0, nf, ks, lane);
  __syncthreads();
  // wave w: pixels 32w .. 32w+31 (two fragments) x all 128 channels
  f32x4_t acc[2][8];
#pragma unroll
  for (int mf = 0; mf < 2; ++mf)
#pragma unroll
    for (int nf = 0; nf < 8; ++nf) acc[mf][nf] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    bf16x8_t a[2];
#pragma unroll
    for (int mf = 0; mf < 2; ++mf)
      a[mf] = *reinterpret_cast<const bf16x8_t*>(As + kc64(32 * w + 16 * mf + (lane & 15), 32 * ks + 8 * (lane >> 4)));
#pragma unroll
    for (int mf = 0; mf < 2; ++mf)
#pragma unroll
      for (int nf = 0; nf < 8; ++nf)  // transposed: lane holds channels 16nf + 4(lane>>4) + j of one pixel
        acc[mf][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[nf][ks], a[mf], acc[mf][nf], 0, 0, 0);
  }
  // epilogue into the staging tile (mode 1 reads its LeakyReLU' operand from the same place first)
#pragma unroll
  for (int mf = 0; mf < 2; ++mf)
#pragma unroll
    for (int nf = 0; nf < 8; ++nf) {
      const int r = 32 * w + 16 * mf + (lane & 15), c = 16 * nf + 4 * (lane >> 4);
      bf16_t* s = Os + r * OS_LD + c;
      u16x4_t o;
      if (MODE == 0) {
        const f32x4_t bv = *reinterpret_cast<const f32x4_t*>(bias + c);
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = f2bf(lrelu(acc[mf][nf][j] + bv[j]));
      } else {
        const u16x4_t m = *reinterpret_cast<const u16x4_t*>(s);
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = f2bf(acc[mf][nf][j] * lrelu_grad(bf2f(m[j])));
      }
      *reinterpret_cast<u16x4_t*>(s) = o;
    }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < D0_BM * 16 / D0_T; ++j) {
    const int i = tid + j * D0_T, r = i >> 4, c = (i & 15) * 8;
    if (p0 + r < P)
      *reinterpret_cast<u16x8_t*>(out + (int64_t)(p0 + r) * 128 + c) =
          *reinterpret_cast<const u16x8_t*>(Os + r * OS_LD + c);
  }
}

constexpr int G_LD = 160;  // MC image pitches (bf16): odd multiples of 16 dwords
constexpr int X_LD = 96;

template <typename TI>
__global__ __launch_bounds__(D0_T) void k_d0_wgrad(const TI* __restrict__ x, int64_t sb, int64_t sh, int64_t sw,
                                                   int64_t sc, int H, int W, int P, const bf16_t* __restrict__ g,
                                                   float* __restrict__ part) {
  __shared__ bf16_t Gs[D0_BM * G_LD];
  __shared__ bf16_t Xs[D0_BM * X_LD];
  const int OH = H / 2, OW = W / 2;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ntiles = (P + D0_BM - 1) / D0_BM;
  constexpr int GV = D0_BM * 16 / D0_T, XV = D0_BM * 8 / D0_T;
  u16x8_t gr[GV], xr[XV];
  auto load = [&](int t) {
    const int p0 = t * D0_BM;
#pragma unroll
    for (int j = 0; j < GV; ++j) {
      const int i = tid + j * D0_T, r = i >> 4, c = (i & 15) * 8;
      gr[j] = (p0 + r < P) ? *reinterpret_cast<const u16x8_t*>(g + (int64_t)(p0 + r) * 128 + c) : u16x8_t(0);
    }
#pragma unroll
    for (int j = 0; j < XV; ++j) {
      const int i = tid + j * D0_T, r = i >> 3, ch = i & 7;
      xr[j] = patch8(x, sb, sh, sw, sc, H, W, OH, OW, P, p0 + r, ch * 8);
    }
  };
  // wave w: output channels 32w .. 32w+31 (two fragments) x k 0..63 (four fragments)
  f32x4_t acc[2][4];
#pragma unroll
  for (int mf = 0; mf < 2; ++mf)
#pragma unroll
    for (int nf = 0; nf < 4; ++nf) acc[mf][nf] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  int t = blockIdx.x;
  if (t < ntiles) load(t);
  for (; t < ntiles; t += gridDim.x) {
    __syncthreads();  // the previous tile's fragment reads are done
#pragma unroll
    for (int j = 0; j < GV; ++j) {
      const int i = tid + j * D0_T, r = i >> 4, c = (i & 15) * 8;
      *reinterpret_cast<u16x8_t*>(Gs + mci(r, c, G_LD)) = gr[j];
    }
#pragma unroll
    for (int j = 0; j < XV; ++j) {
      const int i = tid + j * D0_T, r = i >> 3, ch = i & 7;
      *reinterpret_cast<u16x8_t*>(Xs + mci(r, ch * 8, X_LD)) = xr[j];
    }
    __syncthreads();
    if (t + gridDim.x < ntiles) load(t + gridDim.x);  // next tile's loads overlap this tile's products
#pragma unroll
    for (int ks = 0; ks < D0_BM / 32; ++ks) {
      bf16x8_t a[2], b[4];
#pragma unroll
      for (int mf = 0; mf < 2; ++mf) a[mf] = mc_frag(Gs, G_LD, 32 * ks, 32 * w + 16 * mf, lane);
#pragma unroll
      for (int nf = 0; nf < 4; ++nf) b[nf] = mc_frag(Xs, X_LD, 32 * ks, 16 * nf, lane);
#pragma unroll
      for (int mf = 0; mf < 2; ++mf)
#pragma unroll
        for (int nf = 0; nf < 4; ++nf)
          acc[mf][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mf], b[nf], acc[mf][nf], 0, 0, 0);
    }
  }
  // this block's partial: acc[mf][nf][j] = dW[o = 32w + 16mf + 4(lane>>4) + j][k = 16nf + (lane&15)], k < 48
  float* pb = part + (int64_t)blockIdx.x * (128 * 48);
#pragma unroll
  for (int mf = 0; mf < 2; ++mf)
#pragma unroll
    for (int nf = 0; nf < 3; ++nf)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int o = 32 * w + 16 * mf + 4 * (lane >> 4) + j, k = 16 * nf + (lane & 15);
        pb[o * 48 + k] = acc[mf][nf][j];
      }
}

// image gradient: one block per (image, band of RI input rows)
template <typename TO, int RI, int OWMAX>
__global__ __launch_bounds__(D0_T) void k_d0_dgrad(const bf16_t* __restrict__ g, int OH, int OW,
                                                   const bf16_t* __restrict__ w0, TO* __restrict__ out, int64_t ldo) {
  constexpr int NR = RI / 2 + 2;       // gradient rows a band needs
  constexpr int NPX = NR * OWMAX;      // pixels staged (<= 16 fragments of 16)
  constexpr int GBYTES = NPX * 128 * 2, YBYTES = NPX * 48 * 4;
  __shared__ __attribute__((aligned(16))) char smem[GBYTES > YBYTES ? GBYTES : YBYTES];
  bf16_t* Gs = reinterpret_cast<bf16_t*>(smem);  // KC image, 128 channels = two 64-wide k blocks
  float* Ys = reinterpret_cast<float*>(smem);
  const int H = 2 * OH, W = 2 * OW;
  const int bands = H / RI;
  const int b = blockIdx.x / bands, y0 = (blockIdx.x - b * bands) * RI;
  const int oyA = y0 / 2 - 1;  // staged row i holds gradient row oyA + i (rows outside [0, OH) read as zeros)
  const int npx = NR * OW;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < npx * 16; i += D0_T) {
    const int r = i >> 4, c = (i & 15) * 8;
    const int oy = oyA + r / OW, ox = r % OW;
    u16x8_t v = u16x8_t(0);
    if (oy >= 0 && oy < OH) v = *reinterpret_cast<const u16x8_t*>(g + ((int64_t)(b * OH + oy) * OW + ox) * 128 + c);
    *reinterpret_cast<u16x8_t*>(Gs + (c >> 6) * (NPX * 64) + kc64(r, c & 63)) = v;
  }
  // W0 as B with k = input channel o of the gradient: column n = (tap, c) of k-step ks (o = 32 ks + 8(lane>>4) + j)
  bf16x8_t bw[3][4];
#pragma unroll
  for (int nf = 0; nf < 3; ++nf)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int n = 16 * nf + (lane & 15), o = 32 * ks + 8 * (lane >> 4);
      u16x8_t r;
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = w0[(o + j) * 48 + n];
      bw[nf][ks] = __builtin_bit_cast(bf16x8_t, r);
    }
  __syncthreads();
  constexpr int MF = NPX / 16;
  constexpr int MFW = (MF + 3) / 4;  // fragments per wave
  f32x4_t acc[MFW][3];
#pragma unroll
  for (int m = 0; m < MFW; ++m)
#pragma unroll
    for (int nf = 0; nf < 3; ++nf) acc[m][nf] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int m = 0; m < MFW; ++m) {
    const int mf = w + 4 * m;
    if (mf * 16 >= npx) break;  // wave-uniform
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int k = 32 * ks + 8 * (lane >> 4);
      const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(Gs + (k >> 6) * (NPX * 64) + kc64(16 * mf + (lane & 15), k & 63));
#pragma unroll
      for (int nf = 0; nf < 3; ++nf) acc[m][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[nf][ks], acc[m][nf], 0, 0, 0);
    }
  }
  __syncthreads();  // every fragment read of the gradient image is done: Y overwrites it
#pragma unroll
  for (int m = 0; m < MFW; ++m) {
    const int mf = w + 4 * m;
    if (mf * 16 >= npx) break;
#pragma unroll
    for (int nf = 0; nf < 3; ++nf)
#pragma unroll
      for (int j = 0; j < 4; ++j) Ys[(16 * mf + 4 * (lane >> 4) + j) * 48 + 16 * nf + (lane & 15)] = acc[m][nf][j];
  }
  __syncthreads();
  // col2im from LDS, k_col2im_4x4s2's order: kh = kh0, kh0 + 2; kw = kw0, kw0 + 2
  for (int i = tid; i < RI * W; i += D0_T) {
    const int y = y0 + i / W, xq = i % W;
    const int kh0 = (y + 1) & 1, kw0 = (xq + 1) & 1;
    float s[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int kh = kh0 + 2 * a, oy = (y + 1 - kh) >> 1;
      if (oy < 0 || oy >= OH) continue;
#pragma unroll
      for (int c2 = 0; c2 < 2; ++c2) {
        const int kw = kw0 + 2 * c2, ox = (xq + 1 - kw) >> 1;
        if (ox < 0 || ox >= OW) continue;
        const float* row = Ys + ((oy - oyA) * OW + ox) * 48 + (kh * 4 + kw) * 3;
#pragma unroll
        for (int c = 0; c < 3; ++c) s[c] += row[c];
      }
    }
    TO* o = out + ((int64_t)(b * H + y) * W + xq) * ldo;
#pragma unroll
    for (int c = 0; c < 3; ++c) stf(o, c, s[c]);
  }
}

}  // namespace

extern "C" int mg_d0_fwd(int in_dtype, const void* x, int64_t sb, int64_t sh, int64_t sw, int64_t sc, int B, int H,
                         int W, const void* w0p, const float* bias, const void* aux, void* out, void* stream) {
  MG_REQUIRE(in_dtype == MG_F32 || in_dtype == MG_BF16, "in_dtype must be MG_F32 or MG_BF16");
  MG_REQUIRE(B > 0 && H >= 2 && W >= 2 && H % 2 == 0 && W % 2 == 0, "even image sides");
  MG_REQUIRE(aux != nullptr || bias != nullptr, "bias (mode 0) or aux (mode 1)");
  MG_REQUIRE(mg_al16(w0p) && mg_al16(out) && mg_al16(bias) && mg_al16(aux), "16-byte aligned W0 / out / bias / aux");
  const int64_t P = (int64_t)B * (H / 2) * (W / 2);
  MG_REQUIRE(P * 128 < (1ll << 31), "output too large");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int grid = cdiv(P, D0_BM);
  const bf16_t* w = reinterpret_cast<const bf16_t*>(w0p);
  const bf16_t* a = reinterpret_cast<const bf16_t*>(aux);
  bf16_t* o = reinterpret_cast<bf16_t*>(out);
#define L_(TI, MODE) hipLaunchKernelGGL((k_d0_fwd<TI, MODE>), dim3(grid), dim3(D0_T), 0, st, (const TI*)x, sb, sh, sw, sc, H, W, (int)P, w, bias, a, o)
  if (in_dtype == MG_F32) { if (aux) L_(float, 1); else L_(float, 0); }
  else { if (aux) L_(bf16_t, 1); else L_(bf16_t, 0); }
#undef L_
  return mg_check_launch("mg_d0_fwd");
}

extern "C" int mg_d0_wgrad(int in_dtype, const void* x, int64_t sb, int64_t sh, int64_t sw, int64_t sc, int B, int H,
                           int W, const void* g, float* dw, void* stream) {
  MG_REQUIRE(in_dtype == MG_F32 || in_dtype == MG_BF16, "in_dtype must be MG_F32 or MG_BF16");
  MG_REQUIRE(B > 0 && H >= 2 && W >= 2 && H % 2 == 0 && W % 2 == 0, "even image sides");
  MG_REQUIRE(mg_al16(g), "16-byte aligned gradient");
  const int64_t P = (int64_t)B * (H / 2) * (W / 2);
  MG_REQUIRE(P * 128 < (1ll << 31), "gradient too large");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int ntiles = cdiv(P, D0_BM);
  // ~4 tiles per block at B=256 64x64 (2048 tiles): enough blocks to cover the chip twice, few partial rows
  const int grid = std::min(ntiles, 512);
  float* part = reinterpret_cast<float*>(mg_workspace((size_t)grid * 128 * 48 * sizeof(float), st));
  if (!part) return MG_ERR_ARG;
#define L_(TI) hipLaunchKernelGGL((k_d0_wgrad<TI>), dim3(grid), dim3(D0_T), 0, st, (const TI*)x, sb, sh, sw, sc, H, W, (int)P, (const bf16_t*)g, part)
  if (in_dtype == MG_F32) L_(float);
  else L_(bf16_t);
#undef L_
  mg_det_fold_rows(part, grid, 128 * 48, 128 * 48, dw, nullptr, st);
  return mg_check_launch("mg_d0_wgrad");
}

extern "C" int mg_d0_dgrad(const void* g, int B, int OH, int OW, const void* w0p, int out_dtype, void* out,
                           int64_t ldo, void* stream) {
  MG_REQUIRE(out_dtype == MG_F32 || out_dtype == MG_BF16, "out_dtype must be MG_F32 or MG_BF16");
  MG_REQUIRE(B > 0 && OW >= 1 && OW <= 64 && OH >= 1, "1 <= OW <= 64");
  MG_REQUIRE(ldo >= 3, "ldo >= 3");
  MG_REQUIRE(mg_al16(g), "16-byte aligned gradient");
  const int H = 2 * OH;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bf16_t* gp = reinterpret_cast<const bf16_t*>(g);
  const bf16_t* w = reinterpret_cast<const bf16_t*>(w0p);
#define L_(TO, RI, OWM) hipLaunchKernelGGL((k_d0_dgrad<TO, RI, OWM>), dim3(B * (H / RI)), dim3(D0_T), 0, st, gp, OH, OW, w, (TO*)out, ldo)
  if (OW <= 32 && H % 8 == 0) {
    if (out_dtype == MG_F32) L_(float, 8, 32); else L_(bf16_t, 8, 32);
  } else if (H % 4 == 0) {
    if (out_dtype == MG_F32) L_(float, 4, 64); else L_(bf16_t, 4, 64);
  } else {
    MG_REQUIRE(false, "image height must be a multiple of 4");
  }
#undef L_
  return mg_check_launch("mg_d0_dgrad");
}
