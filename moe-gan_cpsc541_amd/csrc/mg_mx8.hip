// MX-fp8 implicit convolution for gfx950 (BASELINE config C5: "fp8 MFMA conv path").
//
// y = epilogue( conv(x, W) ) with both operands in OCP e4m3 carrying one E8M0 scale per 32 consecutive
// reduction elements (the OCP MX block format), multiplied by v_mfma_scale_f32_16x16x128_f8f6f4 -- twice
// the bf16 MFMA rate per clock, fp32 accumulation.  The non-scaled fp8 MFMA (16x16x32) runs at the bf16
// rate on gfx950, so the block-scaled form is the one that buys throughput.
//
//  * Activations are quantized once per use by mg_quant_mx8 of the NHWC rows ([B*H*W][Cin] -> e4m3 +
//    [B*H*W][Cin/32] scales): a 32-element block is 32 channels of one input pixel, and since Cin % 128 == 0
//    a 128-wide K step lies inside one tap, so the implicit-conv loader fetches the step's 4 scale bytes of
//    a pixel with one dword load at (element offset / 32).  Quantizing inside the conv's loader instead
//    (measured first) was 1.7x SLOWER than bf16: the ~60 VALU per 8 elements, repeated for all 9 taps and
//    every column tile, outweigh the MFMA time of a K step 4:1.
//  * Weights are quantized once per optimizer step by mg_quant_mx8 (packed [Cout][kh][kw][Cin] rows).
//  * Scale choice: e = ceil(log2(amax / 448)), so every scaled element is <= 448 (e4m3's largest finite
//    value) and nothing saturates; v_cvt_pk_fp8_f32 rounds to nearest even.
//
// Register layout of the scaled MFMA (pinned on the GPU with exact data, tools/fp8_probe.hip): lane group
// q = lane >> 4 holds k in [16q, 16q+16) in bytes 0..15 and [64+16q, 64+16q+16) in bytes 16..31 of its 8
// VGPRs (row / column = lane & 15), and supplies the scale of the 32-k block q.  With a 128-B LDS row per
// operand row that is 16-B chunks q and q+4 -- the same swizzled KC image (chunk c stored at c ^ (row & 7))
// the bf16 core uses, so fragment reads and stores are conflict-free.
#include "mg_gemm.h"
#include "mg_host.h"

namespace mg {
namespace {

typedef int i32x8_t __attribute__((ext_vector_type(8)));
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

constexpr int MXK = 128;  // K step (fp8 elements = bytes per LDS row)

// E8M0 exponent for a block with maximum |x| = amax: 2^(e-127) >= amax / 448, smallest such power of two.
// All-zero blocks get e = 1 (any scale works); a NaN maximum yields a NaN block (the loss guards see it).
MG_DEV int mx_exp(float amax) {
  if (!(amax > 0.f)) return amax == 0.f ? 1 : 255;  // 255 = E8M0 NaN
  int ex;
  const float m = frexpf(amax * (1.f / 448.f), &ex);  // amax / 448 = m * 2^ex, m in [0.5, 1)
  const int e = (m == 0.5f ? ex - 1 : ex) + 127;
  return e < 1 ? 1 : (e > 254 ? 254 : e);
}
// 2^(127 - e): the factor that maps the block into e4m3 range (exact power of two)
MG_DEV float mx_inv(int e) { return __uint_as_float((uint32_t)(254 - e) << 23); }

// 8 bf16 -> 8 e4m3 bytes scaled by inv (v_cvt_pk_fp8_f32: OCP e4m3, RNE, saturating)
MG_DEV u32x2_t mx_pack8(const u16x8_t v, float inv) {
  u32x2_t r;
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(v[0]) * inv, bf2f(v[1]) * inv, 0, false);
  r[0] = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(bf2f(v[2]) * inv, bf2f(v[3]) * inv, w, true);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(v[4]) * inv, bf2f(v[5]) * inv, 0, false);
  r[1] = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(bf2f(v[6]) * inv, bf2f(v[7]) * inv, w, true);
  return r;
}
MG_DEV float amax8(const u16x8_t v) {
  float a = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) a = fmaxf(a, fabsf(bf2f(v[j])));
  // NaN must survive the max (fmaxf drops it): flag it explicitly
#pragma unroll
  for (int j = 0; j < 8; ++j) a = bf2f(v[j]) != bf2f(v[j]) ? __builtin_nanf("") : a;
  return a;
}
// maximum over the 4 lanes of an aligned lane quad (NaN-propagating)
MG_DEV float quad_max(float a) {
#pragma unroll
  for (int o = 1; o < 4; o <<= 1) {
    const float b = __shfl_xor(a, o, 64);
    a = (a != a || b != b) ? __builtin_nanf("") : fmaxf(a, b);
  }
  return a;
}

// swizzled 128-B row image: 16-B chunk c of row r at chunk c ^ (r & 7)
MG_DEV int mx_off(int r, int chunk) { return r * MXK + ((chunk ^ (r & 7)) << 4); }

template <int BM, int BN, class EP>
__global__ __launch_bounds__(256) void k_mx8_conv(LdKCConv<uint8_t> A, const uint8_t* __restrict__ xsc,
                                                  const uint8_t* __restrict__ wq, const uint8_t* __restrict__ wsc,
                                                  EP ep, int M, int N, int K) {
  constexpr int WM = BM / 2, WN = BN / 2, FM = WM / 16, FN = WN / 16;
  constexpr int A_VPT = BM * (MXK / 16) / 256;  // 16-B fp8 vectors per thread per K step
  constexpr int B_VPT = BN * (MXK / 16) / 256;
  static_assert(A_VPT >= 1 && B_VPT >= 1, "tile too small");
  constexpr int A_BYTES = BM * MXK, B_BYTES = BN * MXK;
  constexpr int EPI_BYTES = 4 * 16 * (WN + 4) * 4;
  constexpr int TILE_BYTES = A_BYTES + B_BYTES + 4 * (BM + BN);
  __shared__ __attribute__((aligned(16))) uint8_t smem[TILE_BYTES > EPI_BYTES ? TILE_BYTES : EPI_BYTES];
  uint8_t* const As = smem;
  uint8_t* const Bs = smem + A_BYTES;
  uint32_t* const SA = reinterpret_cast<uint32_t*>(smem + A_BYTES + B_BYTES);  // [BM] 4 scale bytes of the step
  uint32_t* const SB = SA + BM;                                                 // [BN]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int KB = K >> 5;  // scale bytes per weight row

  // per-thread load slots: vector v -> (row v / 8, 16-B chunk v % 8); the thread holding chunk 0 of a row
  // also fetches the row's 4 scale bytes of the step
  typename LdKCConv<uint8_t>::Slot as_[A_VPT];
  int a_r[A_VPT], a_c[A_VPT];
#pragma unroll
  for (int i = 0; i < A_VPT; ++i) {
    const int v = tid + i * 256;
    a_r[i] = v >> 3;
    a_c[i] = v & 7;
    const int r = m0 + a_r[i];
    as_[i] = A.slot(r, a_c[i] * 16, r < M);
  }
  uint32_t b_off[B_VPT];
  int b_r[B_VPT], b_c[B_VPT];
#pragma unroll
  for (int i = 0; i < B_VPT; ++i) {
    const int v = tid + i * 256;
    b_r[i] = v >> 3;
    b_c[i] = v & 7;
    const int n = n0 + b_r[i];
    b_off[i] = n < N ? (uint32_t)((int64_t)n * K + b_c[i] * 16) : MG_OOB;
  }
  const bool sb_thr = tid < BN;
  const uint32_t sb_off = (sb_thr && n0 + tid < N) ? (uint32_t)((int64_t)(n0 + tid) * KB) : MG_OOB;
  const rsrc_t rA = A.rsrc(), rSA = make_rsrc(xsc), rB = make_rsrc(wq), rSB = make_rsrc(wsc);

  u32x4_t ra[A_VPT], rb[B_VPT];
  uint32_t rsa[A_VPT], rsb = 0;
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_VPT; ++i) {
      uint32_t o, so;
      A.template offs<false, MXK>(as_[i], k0, K, o, so);
      ra[i] = bload<u32x4_t>(rA, o, so);
      // the pixel's scale bytes: element offset / 32 (chunk 0 of the row, k0 % 128 == 0); keeps the OOB bit
      if (a_c[i] == 0) rsa[i] = __builtin_amdgcn_raw_buffer_load_b32(rSA, ((o & 0x7fffffffu) >> 5) | (o & MG_OOB), 0, 0);
    }
#pragma unroll
    for (int i = 0; i < B_VPT; ++i) rb[i] = bload<u32x4_t>(rB, b_off[i], (uint32_t)k0);
    if (sb_thr) rsb = __builtin_amdgcn_raw_buffer_load_b32(rSB, sb_off, (uint32_t)(k0 >> 5), 0);
  };
  auto sstore = [&]() {
#pragma unroll
    for (int i = 0; i < A_VPT; ++i) {
      *reinterpret_cast<u32x4_t*>(As + mx_off(a_r[i], a_c[i])) = ra[i];
      if (a_c[i] == 0) SA[a_r[i]] = rsa[i];
    }
#pragma unroll
    for (int i = 0; i < B_VPT; ++i) *reinterpret_cast<u32x4_t*>(Bs + mx_off(b_r[i], b_c[i])) = rb[i];
    if (sb_thr) SB[tid] = rsb;
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  auto compute = [&]() {
    i32x8_t af[FM];
    int sa[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int r = wm * WM + i * 16 + fr;
      const u32x4_t lo = *reinterpret_cast<const u32x4_t*>(As + mx_off(r, fq));
      const u32x4_t hi = *reinterpret_cast<const u32x4_t*>(As + mx_off(r, fq + 4));
      af[i] = i32x8_t{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
      sa[i] = (int)((SA[r] >> (8 * fq)) & 255u);
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int c = wn * WN + j * 16 + fr;
      const u32x4_t lo = *reinterpret_cast<const u32x4_t*>(Bs + mx_off(c, fq));
      const u32x4_t hi = *reinterpret_cast<const u32x4_t*>(Bs + mx_off(c, fq + 4));
      const i32x8_t bf = {(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
      const int sb = (int)((SB[c] >> (8 * fq)) & 255u);
#pragma unroll
      for (int i = 0; i < FM; ++i)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bf, acc[i][j], 0, 0, 0, sa[i], 0, sb);
    }
  };

  // one LDS buffer, one register stage: store, barrier, prefetch the next step, multiply
  gload(0);
  for (int k0 = 0; k0 < K; k0 += MXK) {
    __syncthreads();
    sstore();
    __syncthreads();
    if (k0 + MXK < K) gload(k0 + MXK);
    compute();
  }
  epi_tile<BM, BN>(acc, smem, ep, m0, n0, M, N, 0);
}

// weights / standalone: rows of K bf16 (row pitch ldx) -> e4m3 [rows][K] + E8M0 [rows][K / 32].  One thread per
// 8 elements, a lane quad per 32-element block (the same arithmetic as the conv kernel's on-load quantizer).
__global__ __launch_bounds__(256) void k_quant_mx8(const bf16_t* __restrict__ x, int64_t ldx, int64_t rows, int K,
                                                   uint8_t* __restrict__ q, uint8_t* __restrict__ sc) {
  const int kv = K >> 3;
  const int64_t nvec = rows * kv;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t - (threadIdx.x & 3) < nvec; t += (int64_t)gridDim.x * 256) {
    // whole quads stay in the loop together (K % 32 == 0, so a quad never straddles rows)
    const bool ok = t < nvec;
    const int64_t r = ok ? t / kv : 0;
    const int c = ok ? (int)(t - r * kv) : 0;
    const u16x8_t v = ok ? *reinterpret_cast<const u16x8_t*>(x + r * ldx + c * 8) : u16x8_t(0);
    const int e = mx_exp(quad_max(amax8(v)));
    const u32x2_t p = mx_pack8(v, mx_inv(e));
    if (ok) {
      *reinterpret_cast<u32x2_t*>(q + r * K + c * 8) = p;
      if ((c & 3) == 0) sc[r * (K >> 5) + (c >> 2)] = (uint8_t)e;
    }
  }
}

// several weight quantizations in one launch (the per-step MX-fp8 copies of every packed 3x3 weight and its flipped
// data-gradient form): blockIdx.y = descriptor, the same per-vector arithmetic as k_quant_mx8
struct QuantBatch {
  const bf16_t* x[MG_QUANT_BATCH_MAX];
  int64_t ldx[MG_QUANT_BATCH_MAX];
  int64_t rows[MG_QUANT_BATCH_MAX];
  int K[MG_QUANT_BATCH_MAX];
  uint8_t* q[MG_QUANT_BATCH_MAX];
  uint8_t* sc[MG_QUANT_BATCH_MAX];
};
__global__ __launch_bounds__(256) void k_quant_mx8_batch(QuantBatch b) {
  const int d = blockIdx.y, K = b.K[d], kv = K >> 3;
  const int64_t nvec = b.rows[d] * kv;
  const bf16_t* x = b.x[d];
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t - (threadIdx.x & 3) < nvec; t += (int64_t)gridDim.x * 256) {
    const bool ok = t < nvec;
    const int64_t r = ok ? t / kv : 0;
    const int c = ok ? (int)(t - r * kv) : 0;
    const u16x8_t v = ok ? *reinterpret_cast<const u16x8_t*>(x + r * b.ldx[d] + c * 8) : u16x8_t(0);
    const int e = mx_exp(quad_max(amax8(v)));
    const u32x2_t p = mx_pack8(v, mx_inv(e));
    if (ok) {
      *reinterpret_cast<u32x2_t*>(b.q[d] + r * K + c * 8) = p;
      if ((c & 3) == 0) b.sc[d][r * (K >> 5) + (c >> 2)] = (uint8_t)e;
    }
  }
}

template <int BM, int BN, typename TO>
void run_mx8(const void* x, const void* xsc, int B, int H, int W, int Cin, const void* wq, const void* wsc, int Cout,
             int KH, int KW, int stride, int pad, void* y, int64_t ldy, const mg_epilogue* e, hipStream_t st) {
  const int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  const int M = B * OH * OW, K = KH * KW * Cin;
  LdKCConv<uint8_t> la{reinterpret_cast<const uint8_t*>(x), H, W, Cin, ilog2(Cin), ilog2(OW), ilog2(OH * OW), M,
                      KW, stride, pad, K, nullptr, kwinv(KW)};
  Epi<TO> ep = make_epi<TO>(y, ldy, e);
  ep.vec_ok = ep.host_vec_ok() ? 1 : 0;
  hipLaunchKernelGGL((k_mx8_conv<BM, BN, Epi<TO>>), dim3(cdiv(M, BM), cdiv(Cout, BN)), dim3(256), 0, st, la,
                     reinterpret_cast<const uint8_t*>(xsc), reinterpret_cast<const uint8_t*>(wq), reinterpret_cast<const uint8_t*>(wsc), ep, M, Cout, K);
}

template <typename TO>
void run_mx8_tiles(const void* x, const void* xsc, int B, int H, int W, int Cin, const void* wq, const void* wsc, int Cout, int KH,
                   int KW, int stride, int pad, void* y, int64_t ldy, const mg_epilogue* e, hipStream_t st) {
  const int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  const int64_t M = (int64_t)B * OH * OW;
  const int tile = g_mg_tune[MG_TUNE_CONV_TILE];
  if (tile == 128 || (tile == 0 && cdiv(M, 128) * (int64_t)cdiv(Cout, 128) >= 240))
    run_mx8<128, 128, TO>(x, xsc, B, H, W, Cin, wq, wsc, Cout, KH, KW, stride, pad, y, ldy, e, st);
  else
    run_mx8<64, 64, TO>(x, xsc, B, H, W, Cin, wq, wsc, Cout, KH, KW, stride, pad, y, ldy, e, st);
}

}  // namespace
}  // namespace mg

using namespace mg;

extern "C" int mg_quant_mx8(const void* x, int64_t ldx, int64_t rows, int K, void* q, void* scale, void* stream) {
  MG_REQUIRE(K > 0 && K % 32 == 0, "K must be a positive multiple of 32");
  MG_REQUIRE(ldx >= K && ldx % 8 == 0, "ldx must be >= K and a multiple of 8");
  MG_REQUIRE(rows >= 0, "rows must be >= 0");
  MG_REQUIRE(mg_al16(x) && (reinterpret_cast<uintptr_t>(q) & 7) == 0, "x must be 16-B and q 8-B aligned");
  if (rows == 0) return MG_OK;
  const int64_t nvec = rows * (K / 8);
  const int blocks = (int)std::min<int64_t>(cdiv(nvec, 256), 8192);
  hipLaunchKernelGGL(k_quant_mx8, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<const bf16_t*>(x), ldx, rows, K, reinterpret_cast<uint8_t*>(q),
                     reinterpret_cast<uint8_t*>(scale));
  return mg_check_launch("mg_quant_mx8");
}

extern "C" int mg_quant_mx8_batch(int n, const mg_quant_desc* d, void* stream) {
  MG_REQUIRE(n >= 0, "n must be >= 0");
  for (int i0 = 0; i0 < n; i0 += MG_QUANT_BATCH_MAX) {
    const int cnt = std::min(MG_QUANT_BATCH_MAX, n - i0);
    QuantBatch b{};
    int64_t most = 0;
    for (int j = 0; j < cnt; ++j) {
      const mg_quant_desc& q = d[i0 + j];
      MG_REQUIRE(q.K > 0 && q.K % 32 == 0 && q.ldx >= q.K && q.ldx % 8 == 0 && q.rows >= 0,
                 "mg_quant_mx8_batch: K a positive multiple of 32, ldx >= K and a multiple of 8");
      MG_REQUIRE(mg_al16(q.x) && (reinterpret_cast<uintptr_t>(q.q) & 7) == 0, "x must be 16-B and q 8-B aligned");
      b.x[j] = reinterpret_cast<const bf16_t*>(q.x);
      b.ldx[j] = q.ldx;
      b.rows[j] = q.rows;
      b.K[j] = q.K;
      b.q[j] = reinterpret_cast<uint8_t*>(q.q);
      b.sc[j] = reinterpret_cast<uint8_t*>(q.scale);
      most = std::max<int64_t>(most, q.rows * (q.K / 8));
    }
    if (most == 0) continue;
    const int blocks = (int)std::min<int64_t>(cdiv(most, 256), 2048);
    hipLaunchKernelGGL(k_quant_mx8_batch, dim3(blocks, cnt), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), b);
  }
  return mg_check_launch("mg_quant_mx8_batch");
}

extern "C" int mg_conv2d_fwd_mx8(const void* x, const void* xscale, int B, int H, int W, int Cin, const void* wq, const void* wscale,
                                 int Cout, int KH, int KW, int stride, int pad, void* y, int64_t ldy, int y_dtype,
                                 const mg_epilogue* ep, void* stream) {
  MG_REQUIRE(Cin >= MXK && Cin % MXK == 0 && (Cin & (Cin - 1)) == 0,
             "Cin must be a power of two >= 128 (a 128-wide K step inside one tap)");
  MG_REQUIRE(KH * KW <= 32, "at most 32 taps");
  const int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  MG_REQUIRE(OH > 0 && OW > 0 && !(H & (H - 1)) && !(W & (W - 1)) && !(OH & (OH - 1)) && !(OW & (OW - 1)),
             "spatial sizes must be powers of two");
  MG_REQUIRE(y_dtype == MG_F32 || y_dtype == MG_BF16, "bad y_dtype");
  MG_REQUIRE(!(ep && ep->atomic), "atomic epilogue not supported");
  MG_REQUIRE(mg_al16(x) && mg_al16(wq), "x / wq must be 16-byte aligned");
  MG_REQUIRE((reinterpret_cast<uintptr_t>(wscale) & 3) == 0 && (reinterpret_cast<uintptr_t>(xscale) & 3) == 0,
             "xscale / wscale must be 4-byte aligned");
  MG_REQUIRE(ldy >= Cout, "ldy must be >= Cout");
  MG_REQUIRE((int64_t)B * H * W * Cin < (1ll << 31) && (int64_t)Cout * KH * KW * Cin < (1ll << 31) &&
                 (int64_t)B * OH * OW * ldy * (y_dtype == MG_F32 ? 4 : 2) < (1ll << 31),
             "an operand exceeds 2 GiB (32-bit buffer offsets)");
  if (B == 0) return MG_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (y_dtype == MG_F32) run_mx8_tiles<float>(x, xscale, B, H, W, Cin, wq, wscale, Cout, KH, KW, stride, pad, y, ldy, ep, st);
  else run_mx8_tiles<bf16_t>(x, xscale, B, H, W, Cin, wq, wscale, Cout, KH, KW, stride, pad, y, ldy, ep, st);
  return mg_check_launch("mg_conv2d_fwd_mx8");
}
