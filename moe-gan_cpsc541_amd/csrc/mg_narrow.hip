// Direct 3x3 / stride-1 / pad-1 convolutions with a 32-channel side on the small maps (4x4 .. 16x16): the MTM offset
// heads of the generator (offset_net.0, Cin -> 32 + LeakyReLU, t2i_moe_gan.py:199-216) and their backward --
// the data gradient (a 32 -> Cin conv with the flipped kernel, accumulated into the block's input gradient) and
// the weight gradient.
//
// The implicit-GEMM path re-reads every input pixel once per tap (9x the activation through L2, 128 x 32 tiles or
// short 288-deep K loops), which left these at 20-49 us per call at B=256 against 4-8 us of HBM bytes.  Here a
// block stages a 128-pixel tile of the input WITH its halo (one zero-padded ring per image segment) in LDS once per
// channel chunk and forms all nine taps from it:
//
//  * k_conv3_direct<S, CC, CT>: out[p][o] = sum_tap sum_c x[p + tap][c] W[o][tap*Cin + c] for one 128-pixel tile
//    and CT output channels; the input chunk [positions][CC] and the weight slice [CT][9 x CC] both in LDS (16-B
//    fragment reads, pitches chosen so 8 consecutive lanes hit 8 distinct bank quads), the next chunk's global
//    loads in registers while the current one multiplies.  Transposed products leave 4 consecutive output channels
//    of one pixel per lane; the tile is staged through LDS and finished by the GEMM library's 8-column epilogue
//    (bias, activation, accumulate, bf16 / fp32 output).  Small maps (few tiles) split the input channels over
//    blockIdx.z into fp32 slabs folded in split order by splitk_reduce_kernel (deterministic).
//      - forward of the offset head: CC = 64, CT = 32 (the whole Cout);
//      - its data gradient: Cin = 32 (one chunk, K = 288), CT = 64 output channels per block.
//  * k_wgrad3_direct<S>: dW[o][tap*Cin + c] = sum_p g[p][o] x[p + tap][c] over a block's run of tiles for a
//    32-channel chunk: the gradient tile [pixels][32] and the halo'd input tile are MC images (pixel rows) read with
//    the hardware transpose, so the reduction over pixels runs on MFMA; per-block partials are folded by the conv
//    library's slab fold (mg_fold.hip) into the reference [Cout][Cin][3][3] layout (fixed order, deterministic).
#include <algorithm>

#include "mg_gemm.h"
#include "mg_host.h"

using namespace mg;

namespace {

typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

constexpr int NT = 256;  // threads per block
constexpr int TP = 128;  // pixels per tile

// 128-pixel tiles of S x S maps: one image band of TP / S rows (S >= 16) or TP / S^2 whole images.  Staged
// positions: per image segment (SEGROWS + 2) rows of S + 2 columns (the zero ring of the padding).
template <int S, int TPX = TP> struct Geo {
  static constexpr int HW = S * S;
  static constexpr int SEGROWS = HW >= TPX ? TPX / S : S;
  static constexpr int NSEG = HW >= TPX ? 1 : TPX / HW;
  static constexpr int PW = S + 2;
  static constexpr int SEGPOS = (SEGROWS + 2) * PW;
  static constexpr int NPOS = NSEG * SEGPOS;
  // staged position of tile pixel p
  static MG_DEV int pos(int p) {
    const int seg = p / (SEGROWS * S), r = (p / S) % SEGROWS, c = p % S;
    return seg * SEGPOS + (r + 1) * PW + c + 1;
  }
  // staged position -> (image offset, row, column) of the source pixel; false outside the image (zero ring)
  static MG_DEV bool src(int pos, int img0, int h0, int B, int& b, int& h, int& w) {
    const int seg = pos / SEGPOS, rem = pos - seg * SEGPOS;
    b = img0 + seg;
    h = h0 + rem / PW - 1;
    w = rem % PW - 1;
    return b < B && (unsigned)h < (unsigned)S && (unsigned)w < (unsigned)S;
  }
  static MG_DEV int tap_off(int tap) { return (tap / 3 - 1) * PW + (tap % 3 - 1); }
};

// WPX: pixel fragments (16 pixels) per wave -- 2 (128-pixel tiles) or 4 (256-pixel tiles: each weight fragment read
// from LDS serves four pixel fragments instead of two)
template <int S, int CC, int CT, typename TO, bool PART, int WPX = 2>
__global__ __launch_bounds__(NT) void k_conv3_direct(const bf16_t* __restrict__ x, int B, int Cin, int chunks,
                                                     const bf16_t* __restrict__ w, int Cout, Epi<TO> ep,
                                                     float* __restrict__ part, int P) {
  constexpr int TP = 64 * WPX;  // pixels per tile (4 waves)
  using G = Geo<S, TP>;
  constexpr int XP = CC + 8, WPI = 9 * CC + 8;  // LDS pitches (bf16): 8 consecutive rows -> 8 distinct bank quads
  constexpr int XV = CC / 8, NXI = (G::NPOS * XV + NT - 1) / NT, NWI = (CT * 9 * XV + NT - 1) / NT;
  constexpr int WO = CT / 16;
  constexpr int LDS_IN = (G::NPOS * XP + CT * WPI) * 2, LDS_EPI = TP * (CT + 4) * 4;
  __shared__ __attribute__((aligned(16))) char smem[LDS_IN > LDS_EPI ? LDS_IN : LDS_EPI];
  bf16_t* xs = reinterpret_cast<bf16_t*>(smem);
  bf16_t* wsm = xs + G::NPOS * XP;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // XCD-aware tile order: the blocks one XCD receives (bid % 8) take consecutive tiles (shared halo rows in its L2)
  const int ntiles = gridDim.x;
  int t = blockIdx.x;
  if ((ntiles & 7) == 0) t = (t & 7) * (ntiles >> 3) + (t >> 3);
  const int o0 = blockIdx.y * CT;
  const int c_beg = blockIdx.z * chunks * CC;
  const int m0 = t * TP, img0 = m0 / G::HW, h0 = (m0 % G::HW) / S;
  u16x8_t xr[NXI], wr[NWI];
  auto load = [&](int c0) {
#pragma unroll
    for (int i = 0; i < NXI; ++i) {
      const int it = tid + i * NT;
      xr[i] = u16x8_t(0);
      int b, h, ww;
      if (it < G::NPOS * XV && G::src(it / XV, img0, h0, B, b, h, ww))
        xr[i] = *reinterpret_cast<const u16x8_t*>(x + ((int64_t)(b * S + h) * S + ww) * Cin + c0 + 8 * (it % XV));
    }
#pragma unroll
    for (int i = 0; i < NWI; ++i) {
      const int it = tid + i * NT;
      wr[i] = u16x8_t(0);
      if (it < CT * 9 * XV) {
        const int o = it / (9 * XV), rem = it % (9 * XV), tap = rem / XV, v = rem % XV;
        if (o0 + o < Cout)
          wr[i] = *reinterpret_cast<const u16x8_t*>(w + (int64_t)(o0 + o) * 9 * Cin + tap * Cin + c0 + 8 * v);
      }
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int i = 0; i < NXI; ++i) {
      const int it = tid + i * NT;
      if (it < G::NPOS * XV) *reinterpret_cast<u16x8_t*>(xs + (it / XV) * XP + 8 * (it % XV)) = xr[i];
    }
#pragma unroll
    for (int i = 0; i < NWI; ++i) {
      const int it = tid + i * NT;
      if (it < CT * 9 * XV) {
        const int o = it / (9 * XV), rem = it % (9 * XV);
        *reinterpret_cast<u16x8_t*>(wsm + o * WPI + rem * 8) = wr[i];  // rem * 8 = tap * CC + 8 v
      }
    }
  };
  // wave wid: pixels 16 WPX wid .. (WPX fragments) x the CT channels; transposed products leave channels
  // o0 + 16 of + 4 (lane>>4) + j of pixel 16 WPX wid + 16 mf + (lane&15) in acc[mf][of][j]
  int pb[WPX];
#pragma unroll
  for (int mf = 0; mf < WPX; ++mf) pb[mf] = G::pos(16 * WPX * wid + 16 * mf + (lane & 15)) * XP + 8 * (lane >> 4);
  const int wb = (lane & 15) * WPI + 8 * (lane >> 4);
  f32x4_t acc[WPX][WO];
#pragma unroll
  for (int mf = 0; mf < WPX; ++mf)
#pragma unroll
    for (int of = 0; of < WO; ++of) acc[mf][of] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  load(c_beg);
  for (int ch = 0; ch < chunks; ++ch) {
    if (ch) __syncthreads();  // every wave is done reading the previous chunk
    stash();
    __syncthreads();
    if (ch + 1 < chunks) load(c_beg + (ch + 1) * CC);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int toff = G::tap_off(tap) * XP;
#pragma unroll
      for (int ks = 0; ks < CC / 32; ++ks) {
        bf16x8_t a[WO], b[WPX];
#pragma unroll
        for (int mf = 0; mf < WPX; ++mf) b[mf] = *reinterpret_cast<const bf16x8_t*>(xs + pb[mf] + toff + 32 * ks);
#pragma unroll
        for (int of = 0; of < WO; ++of)
          a[of] = *reinterpret_cast<const bf16x8_t*>(wsm + of * 16 * WPI + wb + tap * CC + 32 * ks);
#pragma unroll
        for (int mf = 0; mf < WPX; ++mf)
#pragma unroll
          for (int of = 0; of < WO; ++of)
            acc[mf][of] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[of], b[mf], acc[mf][of], 0, 0, 0);
      }
    }
  }
  __syncthreads();
  float* stg = reinterpret_cast<float*>(smem);  // [TP][CT + 4] fp32
#pragma unroll
  for (int mf = 0; mf < WPX; ++mf)
#pragma unroll
    for (int of = 0; of < WO; ++of)
      *reinterpret_cast<f32x4_t*>(stg + (16 * WPX * wid + 16 * mf + (lane & 15)) * (CT + 4) + 16 * of +
                                  4 * (lane >> 4)) = acc[mf][of];
  __syncthreads();
  for (int it = tid; it < TP * CT / 8; it += NT) {
    const int px = it / (CT / 8), oc = 8 * (it % (CT / 8)), m = m0 + px;
    if (m >= P || o0 + oc >= Cout) continue;
    float v[8];
    const float* s = stg + px * (CT + 4) + oc;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = s[j];
    if constexpr (PART) {
      float* d = part + ((int64_t)blockIdx.z * P + m) * Cout + o0 + oc;
      *reinterpret_cast<f32x4_t*>(d) = f32x4_t{v[0], v[1], v[2], v[3]};
      *reinterpret_cast<f32x4_t*>(d + 4) = f32x4_t{v[4], v[5], v[6], v[7]};
    } else {
      ep.vec8(m, o0 + oc, v);
    }
  }
}

// ---- weight gradient: dW[o][tap*Cin + c] (32 output channels o) over a run of tiles, one 32-channel chunk ----
constexpr int WG_CC = 32;

// MC images with k = pixel rows: column c of row r at r * 32 + (c ^ swizzle(r)).  The transposed fragment read
// takes rows k, k+1, k+2, k+3 (g = 0 half) and the rows 8 pixels on (g = 1) in one cycle; the swizzle flips
// 16 columns between those two row sets.  For the gradient tile rows are pixels (8 apart); for the staged input
// rows are positions, and 8 pixels on is D positions on (S = 16: 8, S = 8: the next image row, 10; S = 4: two
// image rows on, 12).
template <int S> MG_DEV int xswz(int pos) {
  constexpr int D = S >= 16 ? 8 : (8 / S) * (S + 2);
  return ((pos / D) & 1) << 4;
}
MG_DEV int gswz(int px) { return ((px >> 3) & 1) << 4; }

MG_DEV bf16x8_t tr_frag(const bf16_t* img, int row_lo, int sw_lo, int row_hi, int sw_hi, int c0, int lane) {
  auto base = (__attribute__((address_space(3))) char*)(img);
  const int p = lane & 3;
  s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4_t*)(base + (row_lo * WG_CC + ((c0 ^ sw_lo) + 4 * p)) * 2));
  s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4_t*)(base + (row_hi * WG_CC + ((c0 ^ sw_hi) + 4 * p)) * 2));
  u16x8_t r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return __builtin_bit_cast(bf16x8_t, r);
}

template <int S>
__global__ __launch_bounds__(NT) void k_wgrad3_direct(const bf16_t* __restrict__ g, int64_t ldg,
                                                      const bf16_t* __restrict__ x, int B, int Cin, int ngroups,
                                                      int tpg, int ntiles, float* __restrict__ part) {
  using G = Geo<S>;
  constexpr int XV = WG_CC / 8, NXI = (G::NPOS * XV + NT - 1) / NT, NGI = TP * 4 / NT;
  __shared__ __attribute__((aligned(16))) bf16_t xs[G::NPOS * WG_CC];
  __shared__ __attribute__((aligned(16))) bf16_t gs[TP * WG_CC];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // block -> (pixel group, channel chunk): the blocks one XCD receives (bid % 8) run one group's chunks together
  // (the gradient tile re-read per chunk stays in that XCD's L2)
  const int chunks = Cin / WG_CC;
  const int bid = blockIdx.x, xcd = bid & 7, j = bid >> 3;
  const int grp = (j / chunks) * 8 + xcd, chunk = j % chunks;
  if (grp >= ngroups) return;
  const int c0 = chunk * WG_CC;
  const int t_beg = grp * tpg, t_end = std::min(ntiles, t_beg + tpg);
  const int P = B * G::HW;
  u16x8_t xr[NXI], gr[NGI];
  auto load = [&](int t) {
    const int m0 = t * TP, img0 = m0 / G::HW, h0 = (m0 % G::HW) / S;
#pragma unroll
    for (int i = 0; i < NXI; ++i) {
      const int it = tid + i * NT;
      xr[i] = u16x8_t(0);
      int b, h, ww;
      if (it < G::NPOS * XV && G::src(it / XV, img0, h0, B, b, h, ww))
        xr[i] = *reinterpret_cast<const u16x8_t*>(x + ((int64_t)(b * S + h) * S + ww) * Cin + c0 + 8 * (it % XV));
    }
#pragma unroll
    for (int i = 0; i < NGI; ++i) {
      const int it = tid + i * NT, px = it >> 2, m = m0 + px;
      gr[i] = m < P ? *reinterpret_cast<const u16x8_t*>(g + (int64_t)m * ldg + 8 * (it & 3)) : u16x8_t(0);
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int i = 0; i < NXI; ++i) {
      const int it = tid + i * NT;
      if (it < G::NPOS * XV) {
        const int pos = it / XV;
        *reinterpret_cast<u16x8_t*>(xs + pos * WG_CC + ((8 * (it % XV)) ^ xswz<S>(pos))) = xr[i];
      }
    }
#pragma unroll
    for (int i = 0; i < NGI; ++i) {
      const int it = tid + i * NT, px = it >> 2;
      *reinterpret_cast<u16x8_t*>(gs + px * WG_CC + ((8 * (it & 3)) ^ gswz(px))) = gr[i];
    }
  };
  // wave wid: output channels 16 (wid >> 1) .. +15 (the gradient's columns) x input channels c0 + 16 (wid & 1) ..
  // +15, all nine taps: acc[tap][j] = dW[o = 16 (wid>>1) + 4 (lane>>4) + j][tap][c = c0 + 16 (wid&1) + (lane&15)]
  const int of = wid >> 1, cf = wid & 1;
  const int gq = lane >> 4, q = (lane >> 2) & 3;
  f32x4_t acc[9];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) acc[tap] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  if (t_beg < t_end) load(t_beg);
  for (int t = t_beg; t < t_end; ++t) {
    if (t > t_beg) __syncthreads();
    stash();
    __syncthreads();
    if (t + 1 < t_end) load(t + 1);
#pragma unroll
    for (int ks = 0; ks < TP / 32; ++ks) {
      const int plo = 32 * ks + 8 * gq + q, phi = plo + 4;  // this lane's k-rows (pixels)
      const bf16x8_t a = tr_frag(gs, plo, gswz(plo), phi, gswz(phi), 16 * of, lane);
      const int qlo = G::pos(plo), qhi = G::pos(phi);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int rlo = qlo + G::tap_off(tap), rhi = qhi + G::tap_off(tap);
        const bf16x8_t b = tr_frag(xs, rlo, xswz<S>(rlo), rhi, xswz<S>(rhi), 16 * cf, lane);
        acc[tap] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[tap], 0, 0, 0);
      }
    }
  }
  // partial slab [grp][32][9 Cin] (the slab fold's layout, mg_fold.hip: column tap * Cin + c)
  const int N = 9 * Cin;
  float* dst = part + (int64_t)grp * 32 * N + c0 + 16 * cf + (lane & 15);
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) dst[(int64_t)(16 * of + 4 * gq + jj) * N + tap * Cin] = acc[tap][jj];
}

template <int S, int CC, int CT, typename TO, int WPX = 2>
bool launch_conv(const void* x, int B, int Cin, const void* wpack, int Cout, const mg_epilogue* e, void* y,
                 int64_t ldy, hipStream_t st) {
  const int P = B * S * S, tiles = cdiv(P, 64 * WPX), nch = Cin / CC;
  auto ep = make_epi<TO>(y, ldy, e);
  ep.vec_ok = ep.host_vec_ok() ? 1 : 0;
  if (!ep.vec_ok) return false;
  // few tiles (8x8, 4x4 maps): split the channel chunks over blockIdx.z so ~512 blocks stream the input
  const int tb = g_mg_tune[MG_TUNE_NARROW_BLOCKS], target = tb > 0 ? tb : 512;
  int splits = 1;
  while (splits < nch && (int64_t)tiles * cdiv(Cout, CT) * splits < target && nch % (2 * splits) == 0) splits *= 2;
  const bf16_t* xb = reinterpret_cast<const bf16_t*>(x);
  const bf16_t* wb = reinterpret_cast<const bf16_t*>(wpack);
  const dim3 grid(tiles, cdiv(Cout, CT), splits);
  if (splits == 1) {
    hipLaunchKernelGGL((k_conv3_direct<S, CC, CT, TO, false, WPX>), grid, dim3(NT), 0, st, xb, B, Cin, nch, wb, Cout,
                       ep, nullptr, P);
    return true;
  }
  float* ws = reinterpret_cast<float*>(mg_workspace((size_t)splits * P * Cout * sizeof(float), st));
  if (!ws) return false;
  hipLaunchKernelGGL((k_conv3_direct<S, CC, CT, TO, true, WPX>), grid, dim3(NT), 0, st, xb, B, Cin, nch / splits,
                     wb, Cout, ep, ws, P);
  const int blocks = (int)std::min<int64_t>(cdiv((int64_t)P * Cout, 256 * 8), 2048);
  hipLaunchKernelGGL((splitk_reduce_kernel<Epi<TO>>), dim3(blocks), dim3(256), 0, st, ws, splits, P, Cout, ep);
  return true;
}

template <typename TO>
bool conv_dispatch(const void* x, int B, int S, int Cin, const void* wpack, int Cout, const mg_epilogue* e, void* y,
                   int64_t ldy, hipStream_t st) {
  if (Cout == 32) {  // the offset head: Cin -> 32
    if (g_mg_tune[MG_TUNE_NARROW_WPX] == 4) {  // A/B: 256-pixel tiles, four pixel fragments per wave
      switch (S) {
        case 16: return launch_conv<16, 64, 32, TO, 4>(x, B, Cin, wpack, Cout, e, y, ldy, st);
        case 8: return launch_conv<8, 64, 32, TO, 4>(x, B, Cin, wpack, Cout, e, y, ldy, st);
        case 4: return launch_conv<4, 64, 32, TO, 4>(x, B, Cin, wpack, Cout, e, y, ldy, st);
      }
      return false;
    }
    switch (S) {
      case 16: return launch_conv<16, 64, 32, TO>(x, B, Cin, wpack, Cout, e, y, ldy, st);
      case 8: return launch_conv<8, 64, 32, TO>(x, B, Cin, wpack, Cout, e, y, ldy, st);
      case 4: return launch_conv<4, 64, 32, TO>(x, B, Cin, wpack, Cout, e, y, ldy, st);
    }
    return false;
  }
  switch (S) {  // its data gradient: 32 -> Cin
    case 16: return launch_conv<16, 32, 64, TO>(x, B, Cin, wpack, Cout, e, y, ldy, st);
    case 8: return launch_conv<8, 32, 64, TO>(x, B, Cin, wpack, Cout, e, y, ldy, st);
    case 4: return launch_conv<4, 32, 64, TO>(x, B, Cin, wpack, Cout, e, y, ldy, st);
  }
  return false;
}

}  // namespace

bool mg_conv3_direct_ok(int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad, bool wgrad) {
  // A/B: 1 every form through the implicit GEMM; 2 / 3 / 4 only the forward / data-gradient / weight-gradient form
  const int off = g_mg_tune[MG_TUNE_NARROW];
  if (off == 1 || (wgrad && off == 4) || (!wgrad && off == (Cin == 32 ? 3 : 2))) return false;
  if (KH != 3 || KW != 3 || stride != 1 || pad != 1 || H != W || (H != 4 && H != 8 && H != 16)) return false;
  // the data-gradient form over 16x16 maps into >= 256 channels is output-bound (a read-modify-write of the whole
  // gradient) and the implicit GEMM streams that faster (31 vs 34 us at B=256, profiles/round4_narrow_probe.txt)
  if (Cin == 32 && H >= 16 && Cout >= 256) return false;
  return (Cout == 32 && Cin % 64 == 0) || (Cin == 32 && Cout % 64 == 0);
}

bool mg_conv3_direct(const void* x, int B, int H, int Cin, const void* wpack, int Cout, const mg_epilogue* e, void* y,
                     int64_t ldy, int y_dtype, hipStream_t st) {
  if (e && (e->atomic || e->remap_taps > 0 || e->a_idx || e->a_rowscale || e->a_gelu)) return false;
  if (y_dtype == MG_F32) return conv_dispatch<float>(x, B, H, Cin, wpack, Cout, e, y, ldy, st);
  return conv_dispatch<bf16_t>(x, B, H, Cin, wpack, Cout, e, y, ldy, st);
}

// partial slabs [ngroups][32][9 Cin] for the slab fold (mg_fold.hip); false when not handled (shape / workspace)
bool mg_wgrad3_direct(const void* gy, int64_t ldg, const void* x, int B, int H, int Cin, float** ws_out, int* splits,
                      bool* deferred, hipStream_t st) {
  if (ldg % 8 || Cin % WG_CC) return false;
  const int P = B * H * H, ntiles = cdiv(P, TP), chunks = Cin / WG_CC;
  // ~256 blocks (one per CU; each streams its tiles with the next one's loads in flight), >= 4 tiles per group
  const int tb = g_mg_tune[MG_TUNE_NARROW_BLOCKS], target = tb > 0 ? tb : 256;
  int ngroups = std::max(1, std::min(ntiles / 2, target / chunks));
  ngroups = (ngroups + 7) / 8 * 8;  // whole XCD rounds (groups past the last tile exit at once)
  const int tpg = cdiv(ntiles, ngroups);
  float* ws = mg_fold_partials((size_t)ngroups * 32 * 9 * Cin * sizeof(float), st, deferred);
  if (!ws) return false;
  const bf16_t* gb = reinterpret_cast<const bf16_t*>(gy);
  const bf16_t* xb = reinterpret_cast<const bf16_t*>(x);
  const dim3 grid(ngroups * chunks);
  switch (H) {
    case 16: hipLaunchKernelGGL(k_wgrad3_direct<16>, grid, dim3(NT), 0, st, gb, ldg, xb, B, Cin, ngroups, tpg, ntiles, ws); break;
    case 8: hipLaunchKernelGGL(k_wgrad3_direct<8>, grid, dim3(NT), 0, st, gb, ldg, xb, B, Cin, ngroups, tpg, ntiles, ws); break;
    case 4: hipLaunchKernelGGL(k_wgrad3_direct<4>, grid, dim3(NT), 0, st, gb, ldg, xb, B, Cin, ngroups, tpg, ntiles, ws); break;
    default: return false;
  }
  *ws_out = ws;
  *splits = ngroups;
  return true;
}
