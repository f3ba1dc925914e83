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
//    * LeakyReLU'(h0) read from the same LDS staging buffer (m0 v0).  (The patch comes from input rows staged in LDS
//    with coalesced loads; the output tile is staged through LDS for 16-B row stores.  Measured at B=256, 64x64:
//    real 29 us vs 52 us for im2col + GEMM, R1 pass 34 vs 53 us.)  Same MFMA sequence over k as the GEMM path,
//    same fp32 epilogue, one bf16 rounding: bit-identical to im2col + mg_gemm.
//  * k_d0_wgrad: dW0[o][tap*3+c] += sum_p g[p][o] patch[p][tap*3+c].  Blocks stride over 128-pixel tiles; the
//    gradient tile [p][o] is stored as it arrives and the patch tile [p][k] likewise (MC images), both read with
//    the hardware transpose (ds_read_b64_tr_b16) so the reduction over pixels runs on MFMA.  The next tile's
//    global loads are issued before the current tile's products.  Per-block [128 x 48] partials are folded in
//    block order (deterministic in both modes).
//  * k_d0_dgrad: one block per image and band of RI input rows.  It loads the RI/2 + 2 gradient rows that band
//    needs into LDS, forms Y = g W0 ([pixels x 48], fp32, the same four MFMA k-steps as the GEMM path) into LDS
//    and sums every input pixel's <= 4 contributions in k_col2im_4x4s2's order: bit-identical to that path.
#include <algorithm>

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

// ---- input staging.  A 128-pixel tile is NRO = 128 / OW whole output rows; output row j of the tile reads input
// rows 2 oy - 1 .. 2 oy + 2, staged as Xs[j][kh][1 + iw][c] (bf16, channels padded to 4 = 8 B per pixel, columns
// -1 and W zero).  Loads are coalesced runs of the image; the patch is then assembled from LDS. ----
template <int NRO> struct Rows {
  static constexpr int OW = D0_BM / NRO, W = 2 * OW, PITCH = (W + 2) * 4;  // bf16 per staged input row
  static constexpr int ELEMS = NRO * 4 * PITCH;
  // staging items per thread (fp32 planar: 4-pixel vectors of one channel; bf16 interleaved: one pixel)
  static constexpr int NV_PL = (NRO * 4 * 3 * (W / 4) + D0_T - 1) / D0_T;
  static constexpr int NV_IL = (NRO * 4 * W + D0_T - 1) / D0_T;
};

// Staged values in registers (prefetchable): PLANAR (fp32 NCHW, sw = 1) or interleaved (bf16 NHWC, sc = 1, sw = ld)
template <typename TI, int NRO> struct StageRegs;
template <int NRO> struct StageRegs<float, NRO> { f32x4_t v[Rows<NRO>::NV_PL]; };
template <int NRO> struct StageRegs<bf16_t, NRO> { u16x4_t v[Rows<NRO>::NV_IL]; };

template <int NRO>
MG_DEV bool row_of(int item_row, int R0, int OH, int H, int& b, int& ih) {  // staged row (j, kh) -> image row
  const int j = item_row >> 2, kh = item_row & 3;
  const int R = R0 + j;
  b = R / OH;
  const int oy = R - b * OH;
  ih = 2 * oy - 1 + kh;
  return ih >= 0 && ih < H;
}

template <int NRO>
MG_DEV void stage_load(const float* __restrict__ x, int64_t sb, int64_t sh, int64_t sc, int H, int OH, int R0, int Rend,
                       StageRegs<float, NRO>& r, int tid) {
  using RW = Rows<NRO>;
#pragma unroll
  for (int i = 0; i < RW::NV_PL; ++i) {
    const int it = tid + i * D0_T;
    const int v = it % (RW::W / 4), rc = it / (RW::W / 4), c = rc % 3, row = rc / 3;
    r.v[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    int b, ih;
    if (row < NRO * 4 && R0 + (row >> 2) < Rend && row_of<NRO>(row, R0, OH, H, b, ih))
      r.v[i] = *reinterpret_cast<const f32x4_t*>(x + (int64_t)b * sb + ih * sh + c * sc + 4 * v);
  }
}
template <int NRO>
MG_DEV void stage_load(const bf16_t* __restrict__ x, int64_t sb, int64_t sh, int64_t sw, int H, int OH, int R0, int Rend,
                       StageRegs<bf16_t, NRO>& r, int tid) {
  using RW = Rows<NRO>;
#pragma unroll
  for (int i = 0; i < RW::NV_IL; ++i) {
    const int it = tid + i * D0_T;
    const int iw = it % RW::W, row = it / RW::W;
    r.v[i] = u16x4_t(0);
    int b, ih;
    if (row < NRO * 4 && R0 + (row >> 2) < Rend && row_of<NRO>(row, R0, OH, H, b, ih))
      r.v[i] = *reinterpret_cast<const u16x4_t*>(x + (int64_t)b * sb + ih * sh + iw * sw);
  }
}
template <int NRO>
MG_DEV void stage_store(const StageRegs<float, NRO>& r, bf16_t* Xs, int tid) {
  using RW = Rows<NRO>;
#pragma unroll
  for (int i = 0; i < RW::NV_PL; ++i) {
    const int it = tid + i * D0_T;
    const int v = it % (RW::W / 4), rc = it / (RW::W / 4), c = rc % 3, row = rc / 3;
    if (row < NRO * 4) {
      bf16_t* d = Xs + row * RW::PITCH + (1 + 4 * v) * 4 + c;
#pragma unroll
      for (int e = 0; e < 4; ++e) d[4 * e] = f2bf(r.v[i][e]);  // the same RNE rounding as mg_im2col_4x4s2
    }
  }
  // zero pads: columns -1 and W and the fourth channel of every pixel
  for (int it = tid; it < NRO * 4 * (RW::W + 2); it += D0_T) {
    const int col = it % (RW::W + 2), row = it / (RW::W + 2);
    if (col == 0 || col == RW::W + 1) *reinterpret_cast<u16x4_t*>(Xs + row * RW::PITCH + col * 4) = u16x4_t(0);
    else Xs[row * RW::PITCH + col * 4 + 3] = 0;
  }
}
template <int NRO>
MG_DEV void stage_store(const StageRegs<bf16_t, NRO>& r, bf16_t* Xs, int tid) {
  using RW = Rows<NRO>;
#pragma unroll
  for (int i = 0; i < RW::NV_IL; ++i) {
    const int it = tid + i * D0_T;
    const int iw = it % RW::W, row = it / RW::W;
    if (row < NRO * 4) {
      u16x4_t v = r.v[i];
      v[3] = 0;
      *reinterpret_cast<u16x4_t*>(Xs + row * RW::PITCH + (1 + iw) * 4) = v;
    }
  }
  for (int it = tid; it < NRO * 4 * 2; it += D0_T) {
    const int row = it >> 1, col = (it & 1) ? RW::W + 1 : 0;
    *reinterpret_cast<u16x4_t*>(Xs + row * RW::PITCH + col * 4) = u16x4_t(0);
  }
}

// the patch chunks of tile pixel r from the staged rows: thread (r = tid >> 1, half = tid & 1) assembles the 24
// values k = 24 half .. 24 half + 23 (kernel rows kh = 2 half, 2 half + 1; k = (kh*4 + kw)*3 + c) as chunks 3 half
// .. 3 half + 2, and zeroes chunk 6 + half.  ``put(r, chunk, value)`` stores one 16-B chunk.
template <int NRO, class Put>
MG_DEV void build_patch(const bf16_t* Xs, int tid, Put put) {
  using RW = Rows<NRO>;
  const int r = tid >> 1, half = tid & 1;
  const int j = r / RW::OW, ox = r - j * RW::OW;
  bf16_t v[24];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int kh = 2 * half + a;
    const bf16_t* row = Xs + (j * 4 + kh) * RW::PITCH + (2 * ox) * 4;  // column 2 ox - 1, staged at index 2 ox
#pragma unroll
    for (int kw = 0; kw < 4; ++kw) {
      const u16x4_t px = *reinterpret_cast<const u16x4_t*>(row + kw * 4);
#pragma unroll
      for (int c = 0; c < 3; ++c) v[a * 12 + kw * 3 + c] = px[c];
    }
  }
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    u16x8_t ch;
#pragma unroll
    for (int e = 0; e < 8; ++e) ch[e] = v[q * 8 + e];
    put(r, 3 * half + q, ch);
  }
  put(r, 6 + half, u16x8_t(0));
}

constexpr int OS_LD = 136;  // (STAGE) output / aux staging pitch (bf16): 272-B rows, 16-B aligned

template <typename TI, int MODE, int NRO, bool STAGE>
__global__ __launch_bounds__(D0_T) void k_d0_fwd(const TI* __restrict__ x, int64_t sb, int64_t sh, int64_t sw,
                                                 int64_t sc, int H, int P, const bf16_t* __restrict__ w0,
                                                 const float* __restrict__ bias, const bf16_t* __restrict__ aux,
                                                 bf16_t* __restrict__ out) {
  using RW = Rows<NRO>;
  constexpr int AS_BYTES = D0_BM * 64 * 2, OS_BYTES = STAGE ? D0_BM * OS_LD * 2 : 0;
  __shared__ __attribute__((aligned(16))) char smem_a[AS_BYTES > OS_BYTES ? AS_BYTES : OS_BYTES];
  bf16_t* As = reinterpret_cast<bf16_t*>(smem_a);
  bf16_t* Os = reinterpret_cast<bf16_t*>(smem_a);  // (STAGE) the patch image is dead once the products are done
  __shared__ __attribute__((aligned(16))) bf16_t Xs[RW::ELEMS];
  const int OH = H / 2;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int p0 = blockIdx.x * D0_BM;
  {
    StageRegs<TI, NRO> st;
    if constexpr (sizeof(TI) == 4) stage_load<NRO>(x, sb, sh, sc, H, OH, p0 / RW::OW, P / RW::OW, st, tid);
    else stage_load<NRO>(x, sb, sh, sw, H, OH, p0 / RW::OW, P / RW::OW, st, tid);
    stage_store<NRO>(st, Xs, tid);
  }
  __syncthreads();
  build_patch<NRO>(Xs, tid, [&](int r, int chunk, u16x8_t v) {
    *reinterpret_cast<u16x8_t*>(As + kc64(r, chunk * 8)) = v;
  });
  __syncthreads();
  // wave w: pixels 32w .. 32w+31 (two fragments) x all 128 channels; transposed products leave channels
  // 16nf + 4(lane>>4) + j of pixel 32w + 16mf + (lane&15) in acc[mf][nf][j]
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
    for (int nf = 0; nf < 8; ++nf) {
      const bf16x8_t bw = w0_frag_rows(w0, nf, ks, lane);
#pragma unroll
      for (int mf = 0; mf < 2; ++mf)
        acc[mf][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw, a[mf], acc[mf][nf], 0, 0, 0);
    }
  }
  if constexpr (STAGE) {
    // epilogue through LDS: the block's 128 pixels are one contiguous 32 KiB run of the output, written (and, mode
    // 1, the LeakyReLU' operand read) as 16-B vectors by consecutive lanes
    __syncthreads();  // every wave is done reading the patch image
    if (MODE == 1) {
#pragma unroll
      for (int j = 0; j < D0_BM * 16 / D0_T; ++j) {
        const int i = tid + j * D0_T, r = i >> 4, c = (i & 15) * 8;
        if (p0 + r < P)
          *reinterpret_cast<u16x8_t*>(Os + r * OS_LD + c) =
              *reinterpret_cast<const u16x8_t*>(aux + (int64_t)(p0 + r) * 128 + c);
      }
      __syncthreads();
    }
#pragma unroll
    for (int mf = 0; mf < 2; ++mf)
#pragma unroll
      for (int nf = 0; nf < 8; ++nf) {
        const int r = 32 * w + 16 * mf + (lane & 15), c = 16 * nf + 4 * (lane >> 4);
        bf16_t* sp = Os + r * OS_LD + c;
        u16x4_t ov;
        if (MODE == 0) {
          const f32x4_t bv = *reinterpret_cast<const f32x4_t*>(bias + c);
#pragma unroll
          for (int j = 0; j < 4; ++j) ov[j] = f2bf(lrelu(acc[mf][nf][j] + bv[j]));
        } else {
          const u16x4_t m = *reinterpret_cast<const u16x4_t*>(sp);
#pragma unroll
          for (int j = 0; j < 4; ++j) ov[j] = f2bf(acc[mf][nf][j] * lrelu_grad(bf2f(m[j])));
        }
        *reinterpret_cast<u16x4_t*>(sp) = ov;
      }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < D0_BM * 16 / D0_T; ++j) {
      const int i = tid + j * D0_T, r = i >> 4, c = (i & 15) * 8;
      if (p0 + r < P)
        *reinterpret_cast<u16x8_t*>(out + (int64_t)(p0 + r) * 128 + c) =
            *reinterpret_cast<const u16x8_t*>(Os + r * OS_LD + c);
    }
    return;
  }
  // epilogue straight from the accumulators: 8-B runs of 4 channels (a pixel's 256-B row is completed by the
  // wave's other lanes / fragments, and L2 merges the pieces before they reach HBM)
#pragma unroll
  for (int mf = 0; mf < 2; ++mf) {
    const int r = 32 * w + 16 * mf + (lane & 15);
    if (p0 + r >= P) continue;
#pragma unroll
    for (int nf = 0; nf < 8; ++nf) {
      const int c = 16 * nf + 4 * (lane >> 4);
      const int64_t o = (int64_t)(p0 + r) * 128 + c;
      u16x4_t ov;
      if (MODE == 0) {
        const f32x4_t bv = *reinterpret_cast<const f32x4_t*>(bias + c);
#pragma unroll
        for (int j = 0; j < 4; ++j) ov[j] = f2bf(lrelu(acc[mf][nf][j] + bv[j]));
      } else {
        const u16x4_t m = *reinterpret_cast<const u16x4_t*>(aux + o);
#pragma unroll
        for (int j = 0; j < 4; ++j) ov[j] = f2bf(acc[mf][nf][j] * lrelu_grad(bf2f(m[j])));
      }
      *reinterpret_cast<u16x4_t*>(out + o) = ov;
    }
  }
}

constexpr int G_LD = 160;  // MC image pitches (bf16): odd multiples of 16 dwords
constexpr int X_LD = 96;

template <typename TI, int NRO>
__global__ __launch_bounds__(D0_T) void k_d0_wgrad(const TI* __restrict__ x, int64_t sb, int64_t sh, int64_t sw,
                                                   int64_t sc, int H, int P, const bf16_t* __restrict__ g,
                                                   float* __restrict__ part) {
  using RW = Rows<NRO>;
  __shared__ bf16_t Gs[D0_BM * G_LD];
  __shared__ bf16_t Xp[D0_BM * X_LD];
  __shared__ __attribute__((aligned(16))) bf16_t Xs[RW::ELEMS];
  const int OH = H / 2;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ntiles = (P + D0_BM - 1) / D0_BM;
  constexpr int GV = D0_BM * 16 / D0_T;
  u16x8_t gr[GV];
  StageRegs<TI, NRO> st;
  auto load = [&](int t) {
    const int p0 = t * D0_BM;
#pragma unroll
    for (int j = 0; j < GV; ++j) {
      const int i = tid + j * D0_T, r = i >> 4, c = (i & 15) * 8;
      gr[j] = (p0 + r < P) ? *reinterpret_cast<const u16x8_t*>(g + (int64_t)(p0 + r) * 128 + c) : u16x8_t(0);
    }
    if constexpr (sizeof(TI) == 4) stage_load<NRO>(x, sb, sh, sc, H, OH, p0 / RW::OW, P / RW::OW, st, tid);
    else stage_load<NRO>(x, sb, sh, sw, H, OH, p0 / RW::OW, P / RW::OW, st, tid);
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
    stage_store<NRO>(st, Xs, tid);
    __syncthreads();
    build_patch<NRO>(Xs, tid, [&](int r, int chunk, u16x8_t v) {
      *reinterpret_cast<u16x8_t*>(Xp + mci(r, chunk * 8, X_LD)) = v;
    });
    if (t + gridDim.x < ntiles) load(t + gridDim.x);  // next tile's loads overlap this tile's products
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < D0_BM / 32; ++ks) {
      bf16x8_t a[2], b[4];
#pragma unroll
      for (int mf = 0; mf < 2; ++mf) a[mf] = mc_frag(Gs, G_LD, 32 * ks, 32 * w + 16 * mf, lane);
#pragma unroll
      for (int nf = 0; nf < 4; ++nf) b[nf] = mc_frag(Xp, X_LD, 32 * ks, 16 * nf, lane);
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

// first level of the partial fold: tmp[y][i] = sum of rows y*rpg .. (y+1)*rpg - 1 of part (fixed order)
__global__ __launch_bounds__(256) void k_fold_cols(const float* __restrict__ part, int nrows, int ncols, int rpg,
                                                   float* __restrict__ tmp, int accumulate) {
  const int i = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
  if (i >= ncols) return;
  const int r0 = y * rpg, r1 = min(nrows, r0 + rpg);
  float s = 0.f;
  int r = r0;
  for (; r + 8 <= r1; r += 8) {  // eight loads in flight, summed in row order
    float v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = part[(int64_t)(r + q) * ncols + i];
#pragma unroll
    for (int q = 0; q < 8; ++q) s += v[q];
  }
  for (; r < r1; ++r) s += part[(int64_t)r * ncols + i];
  if (accumulate) tmp[(int64_t)y * ncols + i] += s;
  else tmp[(int64_t)y * ncols + i] = s;
}

// image gradient: one block per (image, band of RI input rows)
// VEC: ldo is the vector width (4 fp32 / 8 bf16) and the pixel's padding channels are written as 0
template <typename TO, int RI, int OWMAX, bool VEC>
__global__ __launch_bounds__(D0_T) void k_d0_dgrad(const bf16_t* __restrict__ g, int OH, int OW,
                                                   const bf16_t* __restrict__ w0, TO* __restrict__ out, int64_t ldo) {
  constexpr int NR = RI / 2 + 2;       // gradient rows a band needs
  constexpr int NPX = NR * OWMAX;      // pixels staged (<= 16 fragments of 16)
  constexpr int W_LD = 96;
  constexpr int WBYTES = 128 * W_LD * 2, YBYTES = NPX * 48 * 4;
  __shared__ __attribute__((aligned(16))) char smem[WBYTES > YBYTES ? WBYTES : YBYTES];
  bf16_t* Ws = reinterpret_cast<bf16_t*>(smem);
  float* Ys = reinterpret_cast<float*>(smem);
  const int H = 2 * OH, W = 2 * OW;
  const int bands = H / RI;
  const int b = blockIdx.x / bands, y0 = (blockIdx.x - b * bands) * RI;
  const int oyA = y0 / 2 - 1;  // Y row i holds gradient row oyA + i (rows outside [0, OH) give zeros)
  const int npx = NR * OW;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr int MF = NPX / 16;
  constexpr int MFW = (MF + 3) / 4;  // fragments per wave
  // A fragments (pixel rows, k = gradient channel) straight from global memory: 16-B runs of 8 channels
  bf16x8_t a[MFW][4];
#pragma unroll
  for (int m = 0; m < MFW; ++m) {
    const int px = 16 * (w + 4 * m) + (lane & 15);
    const int oy = oyA + px / OW, ox = px % OW;
    const bool ok = px < npx && oy >= 0 && oy < OH;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      u16x8_t v = u16x8_t(0);
      if (ok) v = *reinterpret_cast<const u16x8_t*>(g + ((int64_t)(b * OH + oy) * OW + ox) * 128 + 32 * ks + 8 * (lane >> 4));
      a[m][ks] = __builtin_bit_cast(bf16x8_t, v);
    }
  }
  // W0 as the B operand (k = gradient channel o, column n = (tap, c)): staged as an MC image [o][n] (the buffer is
  // free until Y is written) and read into registers with the transpose read
  for (int i = tid; i < 128 * 8; i += D0_T) {
    const int o = i >> 3, ch = i & 7;
    u16x8_t v = u16x8_t(0);
    if (ch < 6) v = *reinterpret_cast<const u16x8_t*>(w0 + o * 48 + ch * 8);
    *reinterpret_cast<u16x8_t*>(Ws + mci(o, ch * 8, W_LD)) = v;
  }
  __syncthreads();
  bf16x8_t bw[3][4];
#pragma unroll
  for (int nf = 0; nf < 3; ++nf)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) bw[nf][ks] = mc_frag(Ws, W_LD, 32 * ks, 16 * nf, lane);
  __syncthreads();  // the W0 image is in registers: the buffer takes Y
  f32x4_t acc[MFW][3];
#pragma unroll
  for (int m = 0; m < MFW; ++m)
#pragma unroll
    for (int nf = 0; nf < 3; ++nf) acc[m][nf] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int m = 0; m < MFW; ++m) {
    if ((w + 4 * m) * 16 >= npx) break;  // wave-uniform
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int nf = 0; nf < 3; ++nf) acc[m][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m][ks], bw[nf][ks], acc[m][nf], 0, 0, 0);
#pragma unroll
    for (int nf = 0; nf < 3; ++nf)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        Ys[(16 * (w + 4 * m) + 4 * (lane >> 4) + j) * 48 + 16 * nf + (lane & 15)] = acc[m][nf][j];
  }
  __syncthreads();
  // col2im from LDS, k_col2im_4x4s2's order: kh = kh0, kh0 + 2; kw = kw0, kw0 + 2
  for (int i = tid; i < RI * W; i += D0_T) {
    const int y = y0 + i / W, xq = i % W;
    const int kh0 = (y + 1) & 1, kw0 = (xq + 1) & 1;
    float s[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int a2 = 0; a2 < 2; ++a2) {
      const int kh = kh0 + 2 * a2, oy = (y + 1 - kh) >> 1;
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
    if (VEC) {  // the pixel's whole channel run in one store: channels 3 .. ldo-1 become 0
      if constexpr (sizeof(TO) == 4) {
        *reinterpret_cast<f32x4_t*>(o) = f32x4_t{s[0], s[1], s[2], 0.f};
      } else {
        u16x8_t v = u16x8_t(0);
        v[0] = f2bf(s[0]); v[1] = f2bf(s[1]); v[2] = f2bf(s[2]);
        *reinterpret_cast<u16x8_t*>(o) = v;
      }
    } else {
#pragma unroll
      for (int c = 0; c < 3; ++c) stf(o, c, s[c]);
    }
  }
}

}  // namespace

// staging layout check shared by the forward and the weight gradient: fp32 planar (NCHW, sw = 1) or bf16
// interleaved (NHWC, sc = 1, pixel pitch sw >= 4, 8-B aligned pixels); OW a power of two in [4, 64]
static int d0_layout(int in_dtype, const void* x, int64_t sb, int64_t sh, int64_t sw, int64_t sc, int H, int W) {
  const int OW = W / 2;
  MG_REQUIRE(OW >= 4 && OW <= 64 && (OW & (OW - 1)) == 0, "W / 2 must be a power of two in [4, 64]");
  MG_REQUIRE(H >= 2 && H % 2 == 0, "even image height");
  if (in_dtype == MG_F32) {
    MG_REQUIRE(sw == 1 && sh % 4 == 0 && sc % 4 == 0 && sb % 4 == 0 && mg_al16(x),
               "fp32 images: planar rows (NCHW: sw = 1, 16-B aligned rows)");
  } else {
    MG_REQUIRE(in_dtype == MG_BF16, "in_dtype must be MG_F32 or MG_BF16");
    MG_REQUIRE(sc == 1 && sw >= 4 && sw % 4 == 0 && sh % 4 == 0 && sb % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 7) == 0,
               "bf16 images: interleaved channels (NHWC: sc = 1, pixel pitch a multiple of 4)");
  }
  return MG_OK;
}

#define D0_NRO_SWITCH(OW, MACRO)         \
  switch (OW) {                          \
    case 4: MACRO(32); break;            \
    case 8: MACRO(16); break;            \
    case 16: MACRO(8); break;            \
    case 32: MACRO(4); break;            \
    default: MACRO(2); break;            \
  }

extern "C" int mg_d0_fwd(int in_dtype, const void* x, int64_t sb, int64_t sh, int64_t sw, int64_t sc, int B, int H,
                         int W, const void* w0p, const float* bias, const void* aux, void* out, void* stream) {
  MG_REQUIRE(B > 0, "B > 0");
  if (int rc = d0_layout(in_dtype, x, sb, sh, sw, sc, H, W)) return rc;
  MG_REQUIRE(aux != nullptr || bias != nullptr, "bias (mode 0) or aux (mode 1)");
  MG_REQUIRE(mg_al16(w0p) && mg_al16(out) && mg_al16(bias) && mg_al16(aux), "16-byte aligned W0 / out / bias / aux");
  const int64_t P = (int64_t)B * (H / 2) * (W / 2);
  MG_REQUIRE(P * 128 < (1ll << 31), "output too large");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int grid = cdiv(P, D0_BM);
  const bf16_t* w = reinterpret_cast<const bf16_t*>(w0p);
  const bf16_t* a = reinterpret_cast<const bf16_t*>(aux);
  bf16_t* o = reinterpret_cast<bf16_t*>(out);
  const bool stage = g_mg_tune[MG_TUNE_D0_STORE] != 1;  // LDS-staged rows: 29.1 vs 32.8 us (real), 33.9 vs 37.2 (R1)
#define L_(TI, MODE, NRO)                                                                                              \
  do {                                                                                                                 \
    if (stage) hipLaunchKernelGGL((k_d0_fwd<TI, MODE, NRO, true>), dim3(grid), dim3(D0_T), 0, st, (const TI*)x, sb, sh, sw, sc, H, (int)P, w, bias, a, o); \
    else hipLaunchKernelGGL((k_d0_fwd<TI, MODE, NRO, false>), dim3(grid), dim3(D0_T), 0, st, (const TI*)x, sb, sh, sw, sc, H, (int)P, w, bias, a, o); \
  } while (0)
#define F32_0(NRO) L_(float, 0, NRO)
#define F32_1(NRO) L_(float, 1, NRO)
#define BF_0(NRO) L_(bf16_t, 0, NRO)
#define BF_1(NRO) L_(bf16_t, 1, NRO)
  if (in_dtype == MG_F32) {
    if (aux) { D0_NRO_SWITCH(W / 2, F32_1) } else { D0_NRO_SWITCH(W / 2, F32_0) }
  } else {
    if (aux) { D0_NRO_SWITCH(W / 2, BF_1) } else { D0_NRO_SWITCH(W / 2, BF_0) }
  }
#undef F32_0
#undef F32_1
#undef BF_0
#undef BF_1
#undef L_
  return mg_check_launch("mg_d0_fwd");
}

extern "C" int mg_d0_wgrad(int in_dtype, const void* x, int64_t sb, int64_t sh, int64_t sw, int64_t sc, int B, int H,
                           int W, const void* g, float* dw, void* stream) {
  MG_REQUIRE(B > 0, "B > 0");
  if (int rc = d0_layout(in_dtype, x, sb, sh, sw, sc, H, W)) return rc;
  MG_REQUIRE(mg_al16(g), "16-byte aligned gradient");
  const int64_t P = (int64_t)B * (H / 2) * (W / 2);
  MG_REQUIRE(P * 128 < (1ll << 31), "gradient too large");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int ntiles = cdiv(P, D0_BM);
  // two blocks per CU (73 KB of LDS each), ~4 tiles per block at B=256 64x64 (2048 tiles)
  const int grid = std::min(ntiles, 512);
  const int ncols = 128 * 48, groups = std::min(grid, 32), rpg = cdiv(grid, groups);
  float* part = reinterpret_cast<float*>(mg_workspace((size_t)(grid + groups) * ncols * sizeof(float), st));
  if (!part) return MG_ERR_ARG;
  float* tmp = part + (size_t)grid * ncols;
#define L_(TI, NRO) hipLaunchKernelGGL((k_d0_wgrad<TI, NRO>), dim3(grid), dim3(D0_T), 0, st, (const TI*)x, sb, sh, sw, sc, H, (int)P, (const bf16_t*)g, part)
#define F32_(NRO) L_(float, NRO)
#define BF_(NRO) L_(bf16_t, NRO)
  if (in_dtype == MG_F32) { D0_NRO_SWITCH(W / 2, F32_) } else { D0_NRO_SWITCH(W / 2, BF_) }
#undef F32_
#undef BF_
#undef L_
  // fixed-order fold of the block partials: groups of rpg rows, then the groups
  hipLaunchKernelGGL(k_fold_cols, dim3(cdiv(ncols, 256), groups), dim3(256), 0, st, part, grid, ncols, rpg, tmp, 0);
  hipLaunchKernelGGL(k_fold_cols, dim3(cdiv(ncols, 256), 1), dim3(256), 0, st, tmp, groups, ncols, groups, dw, 1);
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
  const bool vec = (out_dtype == MG_F32 ? ldo == 4 : ldo == 8) && mg_al16(out);
#define L_(TO, RI, OWM)                                                                                                \
  do {                                                                                                                 \
    if (vec) hipLaunchKernelGGL((k_d0_dgrad<TO, RI, OWM, true>), dim3(B * (H / RI)), dim3(D0_T), 0, st, gp, OH, OW, w, (TO*)out, ldo); \
    else hipLaunchKernelGGL((k_d0_dgrad<TO, RI, OWM, false>), dim3(B * (H / RI)), dim3(D0_T), 0, st, gp, OH, OW, w, (TO*)out, ldo); \
  } while (0)
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

// ---------------------------------------------------------------------------------------------------------------
// Discriminator head, image channels (output_layer.0: 4x4 valid conv 256 -> 1, t2i_moe_gan.py:901-907), bf16 step.
//  * k_dhead_fwd: one block per image: P[px][tap] = h1[px] . W2[:, tap] on MFMA (A rows straight from HBM, the
//    [16 x 256] tap-major weight as B), P in LDS, out[oy][ox] = sum_tap P[(oy+kh, ox+kw)][tap] in k_head_sum's order.
//    Replaces the [pixels x 16] fp32 GEMM output + the separate shifted sum (fp32 summation-order agreement).
//  * k_dhead_bwd: one block per image: g_a1[px][c] = LeakyReLU'(h1[px][c]) * sum_tap G[px][tap] W2[c][tap] with the
//    tap-expanded gradient G[px][tap] = g[y-kh][x-kw] formed in registers from the image's logit gradients (no
//    [pixels x 16] matrix), the K = 16 product on one MFMA per 16 x 16 block: bit-identical to mg_disc_head_gmat +
//    mg_gemm with the LeakyReLU' epilogue.
namespace {

__global__ __launch_bounds__(256) void k_dhead_fwd(const bf16_t* __restrict__ h1, const bf16_t* __restrict__ w2t,
                                                   int Hf, float* __restrict__ out) {
  extern __shared__ float Ps[];  // [Hf*Hf][16]
  const int b = blockIdx.x, npx = Hf * Hf, Ho = Hf - 3;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  bf16x8_t bw[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
    bw[ks] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u16x8_t*>(w2t + (lane & 15) * 256 + 32 * ks + 8 * (lane >> 4)));
  const bf16_t* hb = h1 + (int64_t)b * npx * 256;
  for (int mf = w; mf * 16 < npx; mf += 4) {
    bf16x8_t a[8];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
      a[ks] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u16x8_t*>(hb + (int64_t)(16 * mf + (lane & 15)) * 256 + 32 * ks + 8 * (lane >> 4)));
    f32x4_t acc = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ks], bw[ks], acc, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) Ps[(16 * mf + 4 * (lane >> 4) + j) * 16 + (lane & 15)] = acc[j];
  }
  __syncthreads();
  for (int o = tid; o < Ho * Ho; o += 256) {
    const int oy = o / Ho, ox = o - oy * Ho;
    float s = 0.f;
#pragma unroll
    for (int kh = 0; kh < 4; ++kh)
#pragma unroll
      for (int kw = 0; kw < 4; ++kw) s += Ps[((oy + kh) * Hf + ox + kw) * 16 + kh * 4 + kw];
    out[(int64_t)b * Ho * Ho + o] = s;
  }
}

__global__ __launch_bounds__(256) void k_dhead_bwd(const float* __restrict__ g, int64_t g_bstride,
                                                   const bf16_t* __restrict__ h1, const bf16_t* __restrict__ w2c,
                                                   int Hf, bf16_t* __restrict__ ga1) {
  __shared__ float gs[32 * 32];
  const int b = blockIdx.x, npx = Hf * Hf, Ho = Hf - 3;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float* gb = g + (int64_t)b * g_bstride;
  for (int i = tid; i < Ho * Ho; i += 256) gs[i] = gb[i];
  // W2 rows (channel c = 16 nf + (lane&15)) over the 16 taps; k 16..31 of the 32-wide step are zero
  bf16x8_t wf[16];
#pragma unroll
  for (int nf = 0; nf < 16; ++nf) {
    u16x8_t v = u16x8_t(0);
    if ((lane >> 4) < 2) v = *reinterpret_cast<const u16x8_t*>(w2c + (16 * nf + (lane & 15)) * 16 + 8 * (lane >> 4));
    wf[nf] = __builtin_bit_cast(bf16x8_t, v);
  }
  __syncthreads();
  const bf16_t* hb = h1 + (int64_t)b * npx * 256;
  bf16_t* ob = ga1 + (int64_t)b * npx * 256;
  for (int mf = w; mf * 16 < npx; mf += 4) {
    // G column of pixel px = 16 mf + (lane&15): taps 8(lane>>4) .. +7 (bf16, as mg_disc_head_gmat stores it)
    const int px = 16 * mf + (lane & 15), y = px / Hf, x = px - (px / Hf) * Hf;
    u16x8_t gv = u16x8_t(0);
    if ((lane >> 4) < 2) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int tap = 8 * (lane >> 4) + j, oy = y - (tap >> 2), ox = x - (tap & 3);
        const float v = ((unsigned)oy < (unsigned)Ho && (unsigned)ox < (unsigned)Ho) ? gs[oy * Ho + ox] : 0.f;
        gv[j] = f2bf(v);
      }
    }
    const bf16x8_t gf = __builtin_bit_cast(bf16x8_t, gv);
#pragma unroll 4
    for (int nf = 0; nf < 16; ++nf) {
      // transposed product: lane holds channels 16 nf + 4(lane>>4) + j of pixel px
      const f32x4_t acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[nf], gf, f32x4_t{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      const int c = 16 * nf + 4 * (lane >> 4);
      const u16x4_t m = *reinterpret_cast<const u16x4_t*>(hb + (int64_t)px * 256 + c);
      u16x4_t o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = f2bf(acc[j] * lrelu_grad(bf2f(m[j])));
      *reinterpret_cast<u16x4_t*>(ob + (int64_t)px * 256 + c) = o;
    }
  }
}

}  // namespace

extern "C" int mg_d_head_fwd(const void* h1, const void* w2t, int B, int Hf, float* out, void* stream) {
  MG_REQUIRE(B > 0 && Hf >= 4 && Hf <= 32 && (Hf * Hf) % 16 == 0, "4 <= Hf <= 32, Hf^2 a multiple of 16");
  MG_REQUIRE(mg_al16(h1) && mg_al16(w2t), "16-byte aligned h1 / W2");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_dhead_fwd, dim3(B), dim3(256), (size_t)Hf * Hf * 16 * sizeof(float), st,
                     reinterpret_cast<const bf16_t*>(h1), reinterpret_cast<const bf16_t*>(w2t), Hf, out);
  return mg_check_launch("mg_d_head_fwd");
}

extern "C" int mg_d_head_bwd(const float* g, int64_t g_bstride, const void* h1, const void* w2c, int B, int Hf,
                             void* ga1, void* stream) {
  MG_REQUIRE(B > 0 && Hf >= 4 && Hf <= 32 && (Hf * Hf) % 16 == 0, "4 <= Hf <= 32, Hf^2 a multiple of 16");
  MG_REQUIRE(mg_al16(h1) && mg_al16(w2c) && mg_al16(ga1), "16-byte aligned h1 / W2 / g_a1");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_dhead_bwd, dim3(B), dim3(256), 0, st, g, g_bstride, reinterpret_cast<const bf16_t*>(h1),
                     reinterpret_cast<const bf16_t*>(w2c), Hf, reinterpret_cast<bf16_t*>(ga1));
  return mg_check_launch("mg_d_head_bwd");
}
