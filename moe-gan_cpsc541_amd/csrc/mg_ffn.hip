// Fused expert FFN forward of the sparse MoE (t2i_moe_gan.py:257-263, :444-491): for each 128-row tile of one
// expert's dispatched tokens, Y = GELU(X W1^T + b1) W2^T + b2 with the hidden activation kept on chip.
//
// The hidden dimension (Hd = 4C) is walked in 64-unit chunks: GEMM1 (X tile [128 x C] from LDS, resident for the
// whole block, times the chunk's W1 rows, issued as W1 . X^T so each lane's accumulator holds four consecutive
// hidden units of one row) -> + b1 (one 16-B load) and GELU in registers (the pre-activation / GELU output go to
// HBM as 8-B runs straight from the accumulator layout, only when the backward needs them) -> bf16 GELU output to
// LDS (8-B stores) -> GEMM2 accumulates the chunk's contribution into the [128 x C] output held in registers.
// The kernel is VALU-issue bound (GELU ~70 cycles per element vs 16 per 16x16x32 MFMA); a register prefetch of
// the next chunk's weights measured slower (113 -> 121 us), so the other block on the CU covers those loads.
// LDS is 80 KiB at C = 128, so two blocks (16 waves) share a CU and hide each other's barriers.  The unfused path
// (two grouped GEMMs) writes and re-reads the [rows x 4C] hidden activation; here a no-grad forward moves only X
// in and Y out.
//
// Arithmetic matches the grouped-GEMM path bit for bit: the same v_mfma_f32_16x16x32_bf16 sequence over k, the
// same fp32 bias add and fast GELU (mg_common.h gelu_fast) before the bf16 rounding of the hidden activation.
//
// 512 threads = 8 waves (4 along rows x 2 along columns); bf16 only; C in {128, 256}.
#include "mg_common.h"

namespace {

constexpr int FT = 512;   // threads
constexpr int FBM = 128;  // rows per tile
constexpr int FHC = 64;   // hidden units per chunk

// KC image of a [ROWS][K] bf16 operand stored as 64-wide k blocks; the 16-B chunk (k / 8) of row r sits at
// chunk (k / 8) ^ (r & 7) of its 128-B row, so a fragment read (16 rows x 16 B) is conflict-free.
template <int ROWS> MG_DEV int kci(int r, int k) {
  return ((k >> 6) * ROWS + r) * 64 + ((((k >> 3) & 7) ^ (r & 7)) << 3) + (k & 7);
}

MG_DEV bf16x8_t frag(const bf16_t* img, int i) { return *reinterpret_cast<const bf16x8_t*>(img + i); }

template <int C>
struct FfnSmem {
  bf16_t xs[FBM * C];    // X tile (then the bf16 output tile)
  bf16_t w1[FHC * C];    // chunk of W1 rows, KC image (B of GEMM1)
  bf16_t hs[FBM * FHC];  // GELU(hidden) chunk, KC image (A of GEMM2)
  bf16_t w2[C * FHC];    // chunk of W2 columns, KC image (B of GEMM2)
};

template <int C>
__global__ __launch_bounds__(FT) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_moe_ffn_fwd(const bf16_t* __restrict__ X, int64_t ldx,
                                                    const int* __restrict__ idx, int idx_div, int ngroups,
                                                    const int* __restrict__ row_off, const int* __restrict__ tile_off,
                                                    int Hd, const bf16_t* __restrict__ W1, const float* __restrict__ b1,
                                                    const bf16_t* __restrict__ W2, const float* __restrict__ b2,
                                                    bf16_t* __restrict__ Pre, bf16_t* __restrict__ Hid,
                                                    bf16_t* __restrict__ Y) {
  __shared__ FfnSmem<C> sm;
  const int t = blockIdx.x;
  int g = -1;
  for (int i = 0; i < ngroups; ++i)
    if (t >= tile_off[i] && t < tile_off[i + 1]) {
      g = i;
      break;
    }
  if (g < 0) return;  // past the last tile (the grid is an upper bound)
  const int r0 = row_off[g] + (t - tile_off[g]) * FBM, rend = row_off[g + 1];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  const bf16_t* W1g = W1 + (int64_t)g * Hd * C;
  const bf16_t* W2g = W2 + (int64_t)g * C * Hd;
  const float* b1g = b1 + (int64_t)g * Hd;
  bf16_t* preb = Pre ? Pre + (int64_t)r0 * Hd : nullptr;
  bf16_t* hidb = Hid ? Hid + (int64_t)r0 * Hd : nullptr;

  // ---- X tile -> LDS (rows past the group read as zeros) ----
  constexpr int XV = FBM * C / 8 / FT;
#pragma unroll
  for (int j = 0; j < XV; ++j) {
    const int v = tid + j * FT, r = v / (C / 8), k = (v % (C / 8)) * 8;
    const int gr = r0 + r;
    u16x8_t val = u16x8_t(0);
    if (gr < rend) {
      const int src = idx ? idx[gr] / idx_div : gr;
      val = *reinterpret_cast<const u16x8_t*>(X + (int64_t)src * ldx + k);
    }
    *reinterpret_cast<u16x8_t*>(sm.xs + kci<FBM>(r, k)) = val;
  }

  // ---- weight chunk staging: W1 rows [h0, h0+64) x C, W2 [C] x columns [h0, h0+64) ----
  constexpr int WV = FHC * C / 8 / FT;
  u16x8_t w1r[WV], w2r[WV];
  auto load_w = [&](int h0) {
#pragma unroll
    for (int j = 0; j < WV; ++j) {
      const int v = tid + j * FT;
      const int hh = v / (C / 8), k1 = (v % (C / 8)) * 8;
      w1r[j] = *reinterpret_cast<const u16x8_t*>(W1g + (int64_t)(h0 + hh) * C + k1);
      const int c = v / (FHC / 8), k2 = (v % (FHC / 8)) * 8;
      w2r[j] = *reinterpret_cast<const u16x8_t*>(W2g + (int64_t)c * Hd + h0 + k2);
    }
  };
  auto store_w = [&]() {
#pragma unroll
    for (int j = 0; j < WV; ++j) {
      const int v = tid + j * FT;
      const int hh = v / (C / 8), k1 = (v % (C / 8)) * 8;
      *reinterpret_cast<u16x8_t*>(sm.w1 + kci<FHC>(hh, k1)) = w1r[j];
      const int c = v / (FHC / 8), k2 = (v % (FHC / 8)) * 8;
      *reinterpret_cast<u16x8_t*>(sm.w2 + kci<C>(c, k2)) = w2r[j];
    }
  };

  constexpr int FN2 = C / 32;  // GEMM2 column fragments per wave (C / 2 columns)
  f32x4_t acc2[2][FN2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < FN2; ++b) acc2[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int h0 = 0; h0 < Hd; h0 += FHC) {
    // (no register prefetch: at 128 VGPRs it would spill; the other block on the CU covers this load)
    load_w(h0);
    __syncthreads();  // the previous chunk's GEMM2 is done with w2 and hs
    store_w();
    __syncthreads();
    // ---- GEMM1: hidden[128 x 64] = X[128 x C] . W1c[64 x C]^T; wave (wm, wn): rows wm*32, cols wn*32 ----
    f32x4_t acc1[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) acc1[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
    for (int k0 = 0; k0 < C; k0 += 32) {
      bf16x8_t a[2], b[2];
#pragma unroll
      for (int fm = 0; fm < 2; ++fm) a[fm] = frag(sm.xs, kci<FBM>(wm * 32 + fm * 16 + fr, k0 + fk));
#pragma unroll
      for (int fn = 0; fn < 2; ++fn) b[fn] = frag(sm.w1, kci<FHC>(wn * 32 + fn * 16 + fr, k0 + fk));
#pragma unroll
      for (int fm = 0; fm < 2; ++fm)
#pragma unroll
        for (int fn = 0; fn < 2; ++fn)  // transposed product: lane holds 4 consecutive hidden units of one row
          acc1[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[fn], a[fm], acc1[fm][fn], 0, 0, 0);
    }
    // ---- + b1, pre-activation / GELU out (when saved), bf16 GELU -> hs.  The previous chunk's GEMM2 finished
    // reading hs before the barriers at the top of this chunk.  acc1[fm][fn][j] = hidden unit
    // wn*32 + fn*16 + 4*(lane>>4) + j of row wm*32 + fm*16 + (lane&15): four consecutive hidden units per lane, so
    // the bias is one 16-B load and every store (LDS image, saved tensors) is one 8-B run. ----
    // 32-bit element offsets from the tile's first row (128 rows x Hd fit easily)
    const int nrows = rend - r0;
#pragma unroll
    for (int fm = 0; fm < 2; ++fm)
#pragma unroll
      for (int fn = 0; fn < 2; ++fn) {
        const int row = wm * 32 + fm * 16 + fr;
        const int col = wn * 32 + fn * 16 + 4 * (lane >> 4);
        const f32x4_t bias = *reinterpret_cast<const f32x4_t*>(b1g + h0 + col);
        u16x4_t pv, gv;
#pragma unroll
        for (int j = 0; j < 4; j += 2) {  // element pairs on packed fp32 (mg_common.h gelu_fast2)
          const float v0 = acc1[fm][fn][j] + bias[j], v1 = acc1[fm][fn][j + 1] + bias[j + 1];
          const f32x2_t y = gelu_fast2(f32x2_t{v0, v1});
          pv[j] = __builtin_bit_cast(unsigned short, f2bf(v0));
          pv[j + 1] = __builtin_bit_cast(unsigned short, f2bf(v1));
          gv[j] = __builtin_bit_cast(unsigned short, f2bf(y.x));
          gv[j + 1] = __builtin_bit_cast(unsigned short, f2bf(y.y));
        }
        if (row < nrows) {
          const int o = row * Hd + h0 + col;
          if (Pre) *reinterpret_cast<u16x4_t*>(preb + o) = pv;
          if (Hid) *reinterpret_cast<u16x4_t*>(hidb + o) = gv;
        }
        *reinterpret_cast<u16x4_t*>(sm.hs + kci<FBM>(row, col)) = gv;
      }
    __syncthreads();
    // ---- GEMM2: out[128 x C] += hs[128 x 64] . W2c[C x 64]^T; wave (wm, wn): rows wm*32, cols wn*C/2 ----
#pragma unroll
    for (int k0 = 0; k0 < FHC; k0 += 32) {
      bf16x8_t a[2];
#pragma unroll
      for (int fm = 0; fm < 2; ++fm) a[fm] = frag(sm.hs, kci<FBM>(wm * 32 + fm * 16 + fr, k0 + fk));
#pragma unroll
      for (int fn = 0; fn < FN2; ++fn) {
        const bf16x8_t b = frag(sm.w2, kci<C>(wn * (C / 2) + fn * 16 + fr, k0 + fk));
#pragma unroll
        for (int fm = 0; fm < 2; ++fm)
          acc2[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[fm], b, acc2[fm][fn], 0, 0, 0);
      }
    }
  }
  // ---- epilogue: + b2, bf16, staged through LDS (the X tile is dead) for 16-B row stores ----
  __syncthreads();
  const float* b2g = b2 + (int64_t)g * C;
#pragma unroll
  for (int fm = 0; fm < 2; ++fm)
#pragma unroll
    for (int fn = 0; fn < FN2; ++fn) {
      const int col = wn * (C / 2) + fn * 16 + fr;
      const float bias = b2g[col];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = wm * 32 + fm * 16 + 4 * (lane >> 4) + j;
        sm.xs[row * C + col] = f2bf(acc2[fm][fn][j] + bias);
      }
    }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < XV; ++j) {
    const int v = tid + j * FT, r = v / (C / 8), k = (v % (C / 8)) * 8;
    const int gr = r0 + r;
    if (gr < rend) *reinterpret_cast<u16x8_t*>(Y + (int64_t)gr * C + k) = *reinterpret_cast<const u16x8_t*>(sm.xs + r * C + k);
  }
}

// ---------------------------------------------------------------------------------------------------------------
// Fused expert FFN backward, first half (t2i_moe_gan.py:257-263 backward): per 128-row tile of one expert's
// dispatched rows, walking the hidden dimension in 64-unit chunks,
//   GEMM1  gH = gG W2_e[:, chunk]        (K = C; W2 chunk staged as an MC image [c][h], transposed reads)
//          gP = gH * GELU'(Pre)          (the same fp32 product and bf16 rounding as mg_gemm_grouped's epilogue)
//          gP -> HBM (the weight gradient of W1 reads it), -> LDS (A of GEMM2), column sums -> gb1 partial row
//   GEMM2  gX += gP_chunk W1_e[chunk, :] (K = 64 per chunk, the [128 x C] accumulator in registers)
// so gP is written once and never re-read for gX or gb1 (the unfused path wrote gP, read it for gX, for the bias
// column sums and for gW1).  GEMM1 / GEMM2 run the MFMA sequence of the two grouped GEMMs they replace, in the
// same k order: gP and gX are bit-identical to that path; gb1 sums the rows in a fixed order (per-tile partial
// rows folded per expert in tile order).  LDS at C = 128: gG tile 32 KiB + W2 chunk 24 + W1 chunk 20 + gP chunk 16 =
// 92 KiB (padded MC pitches, below), one block per CU.  bf16, C = 128 (256 opt-in).
// MC image pitches: an odd multiple of 16 dwords, so the transposed fragment reads (k-rows kr0 + q and kr0 + 8 + q,
// q = 0..3, per lane half) hit 8 distinct bank octets -- the unpadded pitches (64 and 128 bf16: 32 and 64 dwords) put
// k-rows q and q + 2 (W2) / all four q (W1) on one octet, 2- and 4-way conflicts.  C = 256 keeps W1 unpadded
// (the padded images would exceed the 160 KiB of LDS).
template <int C, int FH> struct BwdPitch {
  static constexpr int W2 = FH + 32;
  static constexpr int W1 = C == 128 ? C + 32 : C;
};
template <int C, int FH>
struct FfnBwdSmem {
  bf16_t gs[FBM * C];               // gG tile, KC image (A of GEMM1); the bf16 gX tile at the end
  bf16_t w2[C * BwdPitch<C, FH>::W2];   // W2_e[:, chunk] as an MC image [c][h] (k-rows c); column sums reuse it
  bf16_t w1[FH * BwdPitch<C, FH>::W1]; // W1_e[chunk, :] as an MC image [h][c] (k-rows h)
  bf16_t hs[FBM * FH];              // gP chunk, KC image (A of GEMM2)
};

typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;
MG_DEV int mswz(int k) { return ((k >> 3) & 1) << 4; }
MG_DEV int mci(int k, int c, int ld) { return k * ld + (c ^ mswz(k)); }
// lane (g = lane>>4, i = lane&15) gets column c0+i of k-rows kr0+8g .. kr0+8g+7
MG_DEV bf16x8_t mc_frag(const bf16_t* img, int ld, int kr0, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int k = kr0 + 8 * g + q;
  auto base = (__attribute__((address_space(3))) char*)(img);
  const int col = (c0 ^ mswz(k)) + 4 * p;
  s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(base + (k * ld + col) * 2));
  s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(base + ((k + 4) * ld + col) * 2));
  u16x8_t r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return __builtin_bit_cast(bf16x8_t, r);
}

// GELU'(x) and GELU(x) from one erf evaluation: the operation sequences of gelu_fast_grad2 and gelu_fast2
// (mg_common.h), so both results are bit-identical to those functions -- the GELU output is what the weight gradient
// of W2 otherwise forms on load from the pre-activation (mg_gemm.h vgelu)
MG_DEV f32x2_t gelu_fast_both2(f32x2_t x, f32x2_t& y) {
  f32x2_t g;
  const f32x2_t e = gelu_erf_core(x, g);
  const f32x2_t hx = x * gsplat<f32x2_t>(0.5f);
  y = gfma(hx, e, hx);
  return gfma(x * gsplat<f32x2_t>(0.3989422804014327f), g, gfma(gsplat<f32x2_t>(0.5f), e, gsplat<f32x2_t>(0.5f)));
}

template <int C, int FH>
__device__ __forceinline__ void ffn_bwd_body(
    const bf16_t* __restrict__ gG, const bf16_t* __restrict__ Pre, int ngroups, const int* __restrict__ row_off,
    const int* __restrict__ tile_off, int Hd, const bf16_t* __restrict__ W1, const bf16_t* __restrict__ W2,
    bf16_t* __restrict__ gP, bf16_t* __restrict__ gX, float* __restrict__ part, float* __restrict__ part2,
    bf16_t* __restrict__ hid) {
  __shared__ FfnBwdSmem<C, FH> sm;
  const int t = blockIdx.x;
  int g = -1;
  for (int i = 0; i < ngroups; ++i)
    if (t >= tile_off[i] && t < tile_off[i + 1]) {
      g = i;
      break;
    }
  if (g < 0) return;  // past the last tile (the grid is an upper bound)
  const int r0 = row_off[g] + (t - tile_off[g]) * FBM, rend = row_off[g + 1];
  const int nrows = rend - r0;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  const bf16_t* W1g = W1 + (int64_t)g * Hd * C;
  const bf16_t* W2g = W2 + (int64_t)g * C * Hd;
  const bf16_t* preb = Pre + (int64_t)r0 * Hd;
  bf16_t* gpb = gP + (int64_t)r0 * Hd;
  bf16_t* hidb = hid ? hid + (int64_t)r0 * Hd : nullptr;
  float* partb = part + (int64_t)t * Hd;

  // ---- gG tile -> LDS (rows past the group read as zeros) ----
  constexpr int XV = FBM * C / 8 / FT;
#pragma unroll
  for (int j = 0; j < XV; ++j) {
    const int v = tid + j * FT, r = v / (C / 8), k = (v % (C / 8)) * 8;
    u16x8_t val = u16x8_t(0);
    if (r < nrows) val = *reinterpret_cast<const u16x8_t*>(gG + (int64_t)(r0 + r) * C + k);
    *reinterpret_cast<u16x8_t*>(sm.gs + kci<FBM>(r, k)) = val;
  }
  constexpr int WV = FH * C / 8 / FT;
  constexpr int FN1 = FH / 32;  // GEMM1 hidden-unit fragments per wave (FH / 2 units)
  constexpr int FN2 = C / 32;  // GEMM2 column fragments per wave (C / 2 columns)
  f32x4_t acc2[2][FN2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < FN2; ++b) acc2[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // register ring (distance one chunk): the next chunk's weights are loaded right after this chunk's are stored to
  // LDS, and its GELU' operand right after this chunk's epilogue used it, so both latencies overlap the products
  u16x8_t w1r[WV], w2r[WV];
  u16x4_t pre_r[2][FN1];
  auto load_w = [&](int h0) {
#pragma unroll
    for (int j = 0; j < WV; ++j) {
      const int v = tid + j * FT;
      const int c = v / (FH / 8), q = (v % (FH / 8)) * 8;   // W2_e[c][h0 + q .. +8]
      w2r[j] = *reinterpret_cast<const u16x8_t*>(W2g + (int64_t)c * Hd + h0 + q);
      const int hh = v / (C / 8), c1 = (v % (C / 8)) * 8;     // W1_e[h0 + hh][c1 .. +8]
      w1r[j] = *reinterpret_cast<const u16x8_t*>(W1g + (int64_t)(h0 + hh) * C + c1);
    }
  };
  auto load_pre = [&](int h0) {
#pragma unroll
    for (int fm = 0; fm < 2; ++fm)
#pragma unroll
      for (int fn = 0; fn < FN1; ++fn) {
        const int row = wm * 32 + fm * 16 + fr;
        const int col = wn * (FH / 2) + fn * 16 + 4 * (lane >> 4);
        pre_r[fm][fn] = row < nrows ? *reinterpret_cast<const u16x4_t*>(preb + (int64_t)row * Hd + h0 + col) : u16x4_t(0);
      }
  };
  load_w(0);
  load_pre(0);
  for (int h0 = 0; h0 < Hd; h0 += FH) {
    __syncthreads();  // the previous chunk's GEMM2 / column sums are done with w1, w2 and hs
#pragma unroll
    for (int j = 0; j < WV; ++j) {
      const int v = tid + j * FT;
      const int c = v / (FH / 8), q = (v % (FH / 8)) * 8;
      *reinterpret_cast<u16x8_t*>(sm.w2 + mci(c, q, BwdPitch<C, FH>::W2)) = w2r[j];
      const int hh = v / (C / 8), c1 = (v % (C / 8)) * 8;
      *reinterpret_cast<u16x8_t*>(sm.w1 + mci(hh, c1, BwdPitch<C, FH>::W1)) = w1r[j];
    }
    __syncthreads();
    if (h0 + FH < Hd) load_w(h0 + FH);
    // ---- GEMM1: gH[128 x FH] = gG[128 x C] . W2c[C x FH]; wave (wm, wn): rows wm*32, hidden units wn*FH/2 ----
    f32x4_t acc1[2][FN1];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < FN1; ++b) acc1[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int k0 = 0; k0 < C; k0 += 32) {
      bf16x8_t a[2], b[FN1];
#pragma unroll
      for (int fm = 0; fm < 2; ++fm) a[fm] = frag(sm.gs, kci<FBM>(wm * 32 + fm * 16 + fr, k0 + fk));
#pragma unroll
      for (int fn = 0; fn < FN1; ++fn) b[fn] = mc_frag(sm.w2, BwdPitch<C, FH>::W2, k0, wn * (FH / 2) + fn * 16, lane);
#pragma unroll
      for (int fm = 0; fm < 2; ++fm)
#pragma unroll
        for (int fn = 0; fn < FN1; ++fn)  // transposed product: lane holds 4 consecutive hidden units of one row
          acc1[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[fn], a[fm], acc1[fm][fn], 0, 0, 0);
    }
    // ---- gP = gH * GELU'(Pre): HBM (8-B runs) and the LDS image for GEMM2 ----
#pragma unroll
    for (int fm = 0; fm < 2; ++fm)
#pragma unroll
      for (int fn = 0; fn < FN1; ++fn) {
        const int row = wm * 32 + fm * 16 + fr;
        const int col = wn * (FH / 2) + fn * 16 + 4 * (lane >> 4);
        const u16x4_t pv = pre_r[fm][fn];
        u16x4_t gv, hv;
#pragma unroll
        for (int j = 0; j < 4; j += 2) {  // element pairs on packed fp32 (mg_common.h gelu_fast_grad2)
          f32x2_t y;
          const f32x2_t d = gelu_fast_both2(f32x2_t{bf2f(pv[j]), bf2f(pv[j + 1])}, y);
          gv[j] = __builtin_bit_cast(unsigned short, f2bf(acc1[fm][fn][j] * d.x));
          gv[j + 1] = __builtin_bit_cast(unsigned short, f2bf(acc1[fm][fn][j + 1] * d.y));
          hv[j] = __builtin_bit_cast(unsigned short, f2bf(y.x));
          hv[j + 1] = __builtin_bit_cast(unsigned short, f2bf(y.y));
        }
        if (row < nrows) {
          *reinterpret_cast<u16x4_t*>(gpb + (int64_t)row * Hd + h0 + col) = gv;
          if (hidb) *reinterpret_cast<u16x4_t*>(hidb + (int64_t)row * Hd + h0 + col) = hv;
        }
        *reinterpret_cast<u16x4_t*>(sm.hs + kci<FBM>(row, col)) = gv;  // rows past the group: gG = 0, so gP = 0
      }
    if (h0 + FH < Hd) load_pre(h0 + FH);
    __syncthreads();  // hs complete; every GEMM1 read of w2 done
    // column sums of the bf16 gP chunk (what the weight gradient reads): 8 row groups of 16 per column, in order,
    // into the free w2 buffer
    float* red = reinterpret_cast<float*>(sm.w2);  // [8 row groups][FH columns]
    for (int col = tid & 63; col < FH; col += 64) {
      const int rg = tid >> 6;
      float cs = 0.f;
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) cs += bf2f(sm.hs[kci<FBM>(rg * 16 + rr, col)]);
      red[rg * FH + col] = cs;
    }
    // ---- GEMM2: gX[128 x C] += hs[128 x FH] . W1c[FH x C]; wave (wm, wn): rows wm*32, cols wn*C/2 ----
#pragma unroll 1
    for (int k0 = 0; k0 < FH; k0 += 32) {
      bf16x8_t a[2];
#pragma unroll
      for (int fm = 0; fm < 2; ++fm) a[fm] = frag(sm.hs, kci<FBM>(wm * 32 + fm * 16 + fr, k0 + fk));
#pragma unroll
      for (int fn = 0; fn < FN2; ++fn) {
        const bf16x8_t b = mc_frag(sm.w1, BwdPitch<C, FH>::W1, k0, wn * (C / 2) + fn * 16, lane);
#pragma unroll
        for (int fm = 0; fm < 2; ++fm)
          acc2[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[fm], b, acc2[fm][fn], 0, 0, 0);
      }
    }
    __syncthreads();  // red complete
    if (tid < FH) {
      float cs = 0.f;
#pragma unroll
      for (int rg = 0; rg < FT / 64; ++rg) cs += red[rg * FH + tid];
      partb[h0 + tid] = cs;
    }
  }
  __syncthreads();  // every read of hs / w1 / w2 by the last chunk is done
  // ---- layer-2 bias gradient (gb2 = column sums of gG over the expert's rows): this tile's partial row from the
  // gG tile still in LDS -- FT / C row groups per column in order, then the groups in order (fixed order) ----
  if (part2) {
    constexpr int RG = FT / C;  // row groups
    float* red2 = reinterpret_cast<float*>(sm.hs);  // [RG][C] (hs is free)
    const int col = tid % C, rg = tid / C;
    float cs = 0.f;
    for (int rr = rg * (FBM / RG); rr < (rg + 1) * (FBM / RG); ++rr) cs += bf2f(sm.gs[kci<FBM>(rr, col)]);
    red2[rg * C + col] = cs;
    __syncthreads();
    if (tid < C) {
      float t2 = 0.f;
#pragma unroll
      for (int g2 = 0; g2 < RG; ++g2) t2 += red2[g2 * C + tid];
      part2[(int64_t)t * C + tid] = t2;
    }
    __syncthreads();  // the gG tile's reads are done before the gX tile overwrites it
  }
  // ---- epilogue: gX tile, bf16, staged through LDS (the gG tile is dead) for 16-B row stores ----
#pragma unroll
  for (int fm = 0; fm < 2; ++fm)
#pragma unroll
    for (int fn = 0; fn < FN2; ++fn) {
      const int col = wn * (C / 2) + fn * 16 + fr;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = wm * 32 + fm * 16 + 4 * (lane >> 4) + j;
        sm.gs[row * C + col] = f2bf(acc2[fm][fn][j]);
      }
    }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < XV; ++j) {
    const int v = tid + j * FT, r = v / (C / 8), k = (v % (C / 8)) * 8;
    if (r < nrows) *reinterpret_cast<u16x8_t*>(gX + (int64_t)(r0 + r) * C + k) = *reinterpret_cast<const u16x8_t*>(sm.gs + r * C + k);
  }
}

// the 256-VGPR form (one block per CU) is the default: 174 vs 220 us at the C2 step's shapes for the 128-VGPR form,
// profiles/round4_ffn_bwd_probe.txt, which the padded images (92 KiB) no longer fit twice per CU anyway
template <int C>
__global__ __launch_bounds__(FT) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_moe_ffn_bwd(
    const bf16_t* __restrict__ gG, const bf16_t* __restrict__ Pre, int ngroups, const int* __restrict__ row_off,
    const int* __restrict__ tile_off, int Hd, const bf16_t* __restrict__ W1, const bf16_t* __restrict__ W2,
    bf16_t* __restrict__ gP, bf16_t* __restrict__ gX, float* __restrict__ part, float* __restrict__ part2,
    bf16_t* __restrict__ hid) {
  ffn_bwd_body<C, 64>(gG, Pre, ngroups, row_off, tile_off, Hd, W1, W2, gP, gX, part, part2, hid);
}
template <int C, int FH>
__global__ __launch_bounds__(FT) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_moe_ffn_bwd_w2(
    const bf16_t* __restrict__ gG, const bf16_t* __restrict__ Pre, int ngroups, const int* __restrict__ row_off,
    const int* __restrict__ tile_off, int Hd, const bf16_t* __restrict__ W1, const bf16_t* __restrict__ W2,
    bf16_t* __restrict__ gP, bf16_t* __restrict__ gX, float* __restrict__ part, float* __restrict__ part2,
    bf16_t* __restrict__ hid) {
  ffn_bwd_body<C, FH>(gG, Pre, ngroups, row_off, tile_off, Hd, W1, W2, gP, gX, part, part2, hid);
}

// gb1[g][h] += sum over the tiles of group g (tile order) of part[tile][h]: 64 columns x 4 tile lanes per block,
// eight loads in flight per lane, the four lane sums folded in lane order
__global__ __launch_bounds__(256) void k_ffn_bias_fold(const float* __restrict__ part, const int* __restrict__ tile_off,
                                                       int Hd, float* __restrict__ gb1) {
  __shared__ float red[4][64];
  const int h = blockIdx.x * 64 + (threadIdx.x & 63), ty = threadIdx.x >> 6, g = blockIdx.y;
  const int t0 = tile_off[g], t1 = tile_off[g + 1];
  float s = 0.f;
  if (h < Hd) {
    int t = t0 + ty;
    for (; t + 28 < t1; t += 32) {
      float v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = part[(int64_t)(t + 4 * q) * Hd + h];
#pragma unroll
      for (int q = 0; q < 8; ++q) s += v[q];
    }
    for (; t < t1; t += 4) s += part[(int64_t)t * Hd + h];
  }
  red[ty][threadIdx.x & 63] = s;
  __syncthreads();
  if (ty == 0 && h < Hd) gb1[(int64_t)g * Hd + h] += ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
}

}  // namespace

extern "C" int mg_moe_ffn_fwd(int dtype, int total_rows, int C, int Hd, int ngroups, const int32_t* row_off, const int32_t* tile_off,
                              int max_tiles, const void* X, int64_t ldx, const int32_t* x_idx, int x_idx_div,
                              const void* W1, const float* b1, const void* W2, const float* b2, void* pre, void* hid,
                              void* Y, void* stream) {
  MG_REQUIRE(dtype == MG_BF16, "bf16 only");
  MG_REQUIRE(C == 128 || C == 256, "C must be 128 or 256");
  MG_REQUIRE(Hd > 0 && Hd % FHC == 0, "Hd must be a multiple of 64");
  MG_REQUIRE(ngroups >= 1 && ngroups <= 64, "1 <= ngroups <= 64");
  MG_REQUIRE(ldx % 8 == 0 && mg_al16(X) && mg_al16(W1) && mg_al16(W2) && mg_al16(Y) && mg_al16(pre) && mg_al16(hid) &&
                 mg_al16(b1),
             "operands (and b1) must be 16-byte aligned, ldx a multiple of 8");
  MG_REQUIRE(x_idx_div >= 1, "x_idx_div >= 1");
  MG_REQUIRE(total_rows >= 0 && max_tiles >= (total_rows + FBM - 1) / FBM, "max_tiles below the row tiles");
  if (max_tiles <= 0 || total_rows == 0) return MG_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define L_(CC)                                                                                                       \
  hipLaunchKernelGGL(k_moe_ffn_fwd<CC>, dim3(max_tiles), dim3(FT), 0, st, reinterpret_cast<const bf16_t*>(X), ldx, \
                     x_idx, x_idx_div, ngroups, row_off, tile_off, Hd, reinterpret_cast<const bf16_t*>(W1), b1,      \
                     reinterpret_cast<const bf16_t*>(W2), b2, reinterpret_cast<bf16_t*>(pre),                        \
                     reinterpret_cast<bf16_t*>(hid), reinterpret_cast<bf16_t*>(Y))
  if (C == 128) L_(128);
  else L_(256);
#undef L_
  return mg_check_launch("mg_moe_ffn_fwd");
}

extern "C" int mg_moe_ffn_bwd(int dtype, int total_rows, int C, int Hd, int ngroups, const int32_t* row_off,
                              const int32_t* tile_off, int max_tiles, const void* gG, const void* pre, const void* W1,
                              const void* W2, void* gP, void* gX, void* hid, float* gb1, float* gb2, void* stream) {
  MG_REQUIRE(dtype == MG_BF16, "bf16 only");
  MG_REQUIRE(C == 128 || C == 256, "C must be 128 or 256");
  MG_REQUIRE(Hd > 0 && Hd % 128 == 0, "Hd must be a multiple of 128");
  MG_REQUIRE(!hid || mg_al16(hid), "hid must be 16-byte aligned");
  MG_REQUIRE(ngroups >= 1 && ngroups <= 64, "1 <= ngroups <= 64");
  MG_REQUIRE(mg_al16(gG) && mg_al16(pre) && mg_al16(W1) && mg_al16(W2) && mg_al16(gP) && mg_al16(gX),
             "operands must be 16-byte aligned");
  MG_REQUIRE(total_rows >= 0 && max_tiles >= (total_rows + FBM - 1) / FBM, "max_tiles below the row tiles");
  if (max_tiles <= 0 || total_rows == 0) return MG_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  float* part = reinterpret_cast<float*>(mg_workspace((size_t)max_tiles * (Hd + C) * sizeof(float), st));
  if (!part) return MG_ERR_ARG;
  float* part2 = gb2 ? part + (size_t)max_tiles * Hd : nullptr;
  // one block per CU either way (92 / 160 KiB of LDS at C = 128 / 256): the 256-VGPR form unless A/B-tuned
  const bool one_block = C == 256 || g_mg_tune[MG_TUNE_FFN_BWD_OCC] != 2;
#define L_(K, ...)                                                                                                   \
  hipLaunchKernelGGL((K<__VA_ARGS__>), dim3(max_tiles), dim3(FT), 0, st, reinterpret_cast<const bf16_t*>(gG),       \
                     reinterpret_cast<const bf16_t*>(pre), ngroups, row_off, tile_off, Hd,                            \
                     reinterpret_cast<const bf16_t*>(W1), reinterpret_cast<const bf16_t*>(W2),                        \
                     reinterpret_cast<bf16_t*>(gP), reinterpret_cast<bf16_t*>(gX), part, part2,                  \
                     reinterpret_cast<bf16_t*>(hid))
  // C = 128: 128-unit hidden chunks by default (half the chunk barriers, twice the MFMA work between them; 144 KiB of
  // LDS); tuning slot MG_TUNE_FFN_BWD_OCC = 3 keeps the 64-unit chunks of rounds 4-5 (A/B)
  if (C == 256) L_(k_moe_ffn_bwd_w2, 256, 64);
  else if (!one_block) L_(k_moe_ffn_bwd, 128);
  else if (g_mg_tune[MG_TUNE_FFN_BWD_OCC] == 3) L_(k_moe_ffn_bwd_w2, 128, 64);
  else L_(k_moe_ffn_bwd_w2, 128, 128);
#undef L_
  if (gb1) hipLaunchKernelGGL(k_ffn_bias_fold, dim3(cdiv(Hd, 64), ngroups), dim3(256), 0, st, part, tile_off, Hd, gb1);
  if (gb2) hipLaunchKernelGGL(k_ffn_bias_fold, dim3(cdiv(C, 64), ngroups), dim3(256), 0, st, part2, tile_off, C, gb2);
  return mg_check_launch("mg_moe_ffn_bwd");
}
