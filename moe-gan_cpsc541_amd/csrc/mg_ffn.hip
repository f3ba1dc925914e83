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
        for (int j = 0; j < 4; ++j) {
          const float v = acc1[fm][fn][j] + bias[j];
          pv[j] = __builtin_bit_cast(unsigned short, f2bf(v));
          gv[j] = __builtin_bit_cast(unsigned short, f2bf(gelu_fast(v)));
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
