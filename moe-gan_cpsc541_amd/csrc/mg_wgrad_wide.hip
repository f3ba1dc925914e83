// Weight gradients of the step's linear layers as "wide" split-K GEMMs: C[M][N] += alpha * sum_k A[k][m] B[k][n]
// with A = the output gradient [K tokens x M] and B = the layer input [K x N], both bf16 and row-major (M / N
// contiguous), K = tokens (4096 .. 65536) and M x N small (the self-attention in/out projections and 1x1 skips,
// t2i_moe_gan.py:545-556 backward: 128 x 128 .. 1536 x 512).
//
// The generic GEMM runs these as 64 x 64 tiles split over K into ~512 blocks with fp32 atomics: every A column strip
// is re-read N / 64 times and every B strip M / 64 times (4-8x the operand bytes), and the 2-8 M atomic adds run at
// the chip's ~1.3 TB/s atomic rate (MI355X_MICROARCH.md) -- 20-40 us per call for 8-67 MB of operands.  Here a block
// owns a 128 x 128 or 256 x 256 output tile (all of M x N for most shapes) for one K chunk: the operands are read
// once or twice, K is split so that ~256 blocks stream them, and the per-block fp32 partial tiles are folded in a
// fixed order by two passes (deterministic in both library modes).
//
// Block: 512 threads = 8 waves as 2 (M) x 4 (N), wave tile (BM/2) x (BN/4) of 16x16 fragments; k-steps of 32 rows
// staged as MC images (rows stored as they arrive, 16-B coalesced) in a double-buffered LDS ring, one barrier per
// k-step, the next step's global loads in registers while the current one multiplies; fragments by the hardware
// transpose read (ds_read_b64_tr_b16).
#include <algorithm>

#include "mg_common.h"

namespace {

typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

constexpr int WT = 512;  // threads
constexpr int WBK = 32;  // k rows per step

MG_DEV int swz(int k) { return ((k >> 3) & 1) << 4; }

MG_DEV bf16x8_t mc_frag(const bf16_t* img, int ld, int kr0, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int k = kr0 + 8 * g + q;
  auto base = (__attribute__((address_space(3))) char*)(img);
  const int col = (c0 ^ swz(k)) + 4 * p;
  s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(base + (k * ld + col) * 2));
  s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(base + ((k + 4) * ld + col) * 2));
  u16x8_t r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return __builtin_bit_cast(bf16x8_t, r);
}

template <int BM, int BN>
__global__ __launch_bounds__(WT) void k_wgrad_wide(const bf16_t* __restrict__ A, int64_t lda,
                                                   const bf16_t* __restrict__ B, int64_t ldb, int M, int N, int K,
                                                   int kchunk, float* __restrict__ part) {
  constexpr int LDA = BM + 32, LDB = BN + 32;  // pitches: odd multiples of 16 dwords
  constexpr int AV = WBK * BM / 8 / WT, BV = WBK * BN / 8 / WT;  // 16-B loads per thread per k-step
  constexpr int WM = BM / 2, WN = BN / 4, FM = WM / 16, FN = WN / 16;
  static_assert(AV >= 1 && BV >= 1, "tile too small for the block");
  __shared__ bf16_t As[2][WBK * LDA];
  __shared__ bf16_t Bs[2][WBK * LDB];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int k_lo = blockIdx.z * kchunk, k_hi = std::min(K, k_lo + kchunk);
  u16x8_t ar[AV], br[BV];
  auto load = [&](int k0) {
#pragma unroll
    for (int j = 0; j < AV; ++j) {
      const int i = tid + j * WT, r = i / (BM / 8), c = (i % (BM / 8)) * 8;
      ar[j] = (k0 + r < k_hi && m0 + c < M) ? *reinterpret_cast<const u16x8_t*>(A + (int64_t)(k0 + r) * lda + m0 + c)
                                            : u16x8_t(0);
    }
#pragma unroll
    for (int j = 0; j < BV; ++j) {
      const int i = tid + j * WT, r = i / (BN / 8), c = (i % (BN / 8)) * 8;
      br[j] = (k0 + r < k_hi && n0 + c < N) ? *reinterpret_cast<const u16x8_t*>(B + (int64_t)(k0 + r) * ldb + n0 + c)
                                            : u16x8_t(0);
    }
  };
  f32x4_t acc[FM][FN];
#pragma unroll
  for (int a = 0; a < FM; ++a)
#pragma unroll
    for (int b = 0; b < FN; ++b) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  load(k_lo);
  int buf = 0;
  for (int k0 = k_lo; k0 < k_hi; k0 += WBK) {
#pragma unroll
    for (int j = 0; j < AV; ++j) {
      const int i = tid + j * WT, r = i / (BM / 8), c = (i % (BM / 8)) * 8;
      *reinterpret_cast<u16x8_t*>(&As[buf][r * LDA + (c ^ swz(r))]) = ar[j];
    }
#pragma unroll
    for (int j = 0; j < BV; ++j) {
      const int i = tid + j * WT, r = i / (BN / 8), c = (i % (BN / 8)) * 8;
      *reinterpret_cast<u16x8_t*>(&Bs[buf][r * LDB + (c ^ swz(r))]) = br[j];
    }
    __syncthreads();  // (the other buffer was last read before the previous barrier)
    if (k0 + WBK < k_hi) load(k0 + WBK);
    bf16x8_t b[FN];
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) b[fn] = mc_frag(Bs[buf], LDB, 0, wn * WN + 16 * fn, lane);
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
      const bf16x8_t a = mc_frag(As[buf], LDA, 0, wm * WM + 16 * fm, lane);
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[fn], acc[fm][fn], 0, 0, 0);
    }
    buf ^= 1;
  }
  // this block's partial tile: acc[fm][fn][j] = C[m0 + wm*WM + 16fm + 4(lane>>4) + j][n0 + wn*WN + 16fn + (lane&15)]
  float* pb = part + (int64_t)blockIdx.z * M * N;
#pragma unroll
  for (int fm = 0; fm < FM; ++fm)
#pragma unroll
    for (int fn = 0; fn < FN; ++fn)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + wm * WM + 16 * fm + 4 * (lane >> 4) + j, n = n0 + wn * WN + 16 * fn + (lane & 15);
        if (m < M && n < N) pb[(int64_t)m * N + n] = acc[fm][fn][j];
      }
}

// fold level 1: tmp[grp][i] = sum of part[s][i] for s in the group's split range (ascending); level 2 (final):
// C[m][n] += alpha * sum of tmp[grp][i] (ascending)
__global__ __launch_bounds__(256) void k_wide_fold(const float* __restrict__ part, int nsplit, int64_t MN, int per,
                                                   float* __restrict__ tmp) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= MN) return;
  const int s0 = blockIdx.y * per, s1 = std::min(nsplit, s0 + per);
  float s = 0.f;
  int r = s0;
  for (; r + 8 <= s1; r += 8) {
    float v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = part[(int64_t)(r + q) * MN + i];
#pragma unroll
    for (int q = 0; q < 8; ++q) s += v[q];
  }
  for (; r < s1; ++r) s += part[(int64_t)r * MN + i];
  tmp[(int64_t)blockIdx.y * MN + i] = s;
}
__global__ __launch_bounds__(256) void k_wide_final(const float* __restrict__ tmp, int ngrp, int M, int N, float alpha,
                                                    float* __restrict__ C, int64_t ldc) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x, MN = (int64_t)M * N;
  if (i >= MN) return;
  float s = 0.f;
  for (int g = 0; g < ngrp; ++g) s += tmp[(int64_t)g * MN + i];
  const int64_t m = i / N, n = i - m * N;
  // an atomic add keeps mg_gemm's atomic-epilogue contract (concurrent writers into one gradient buffer, e.g. from
  // the main and the side stream, accumulate); with one writer it is the same single fp32 addition as C += alpha s
  atomicAdd(C + m * ldc + n, alpha * s);
}

}  // namespace

// Called by mg_gemm for bf16, a_kc = b_kc = 0 (both operands [K][*] row-major), an fp32 C accumulated through a
// plain atomic epilogue (alpha only), large K and small M x N.  Returns true when it handled the call.
bool mg_wgrad_wide(int M, int N, int K, const void* A, int64_t lda, const void* B, int64_t ldb, float* C, int64_t ldc,
                   float alpha, hipStream_t st) {
  if (g_mg_tune[MG_TUNE_WIDE_WGRAD] == 1) return false;  // A/B: the generic split-K GEMM
  if (K < 2048 || M % 8 || N % 8 || (int64_t)M * N > 1024 * 1024) return false;
  // measured (profiles/round4_wgrad_wide_probe.txt): a win only when K is long against the tile edges -- the
  // (384|128) x 128 x 65536 projections, 1.2-1.3x; at K = 4096-16384 the partial-tile folds cost more than the
  // generic GEMM's re-reads save, and a 16-wide N leaves the MFMA tile mostly empty (2: every eligible shape, tests)
  if (g_mg_tune[MG_TUNE_WIDE_WGRAD] != 2 && ((int64_t)K < 64 * (int64_t)(M + N) || M < 64 || N < 64)) return false;
  const bool big = M >= 256 && N >= 256;
  const int BM = big ? 256 : 128, BN = big ? 256 : 128;
  const int64_t tiles = (int64_t)cdiv(M, BM) * cdiv(N, BN), MN = (int64_t)M * N;
  // ~256 blocks, >= 512 rows of K each
  int splits = (int)std::max<int64_t>(1, std::min<int64_t>(256 / tiles, K / 512));
  int kchunk = (K + splits - 1) / splits;
  kchunk = (kchunk + WBK - 1) / WBK * WBK;
  splits = (K + kchunk - 1) / kchunk;
  const int per = 16, ngrp = (splits + per - 1) / per;
  float* part = reinterpret_cast<float*>(mg_workspace((size_t)(splits + ngrp) * MN * sizeof(float), st));
  if (!part) return false;
  float* tmp = part + (size_t)splits * MN;
  const dim3 grid(cdiv(M, BM), cdiv(N, BN), splits);
  const bf16_t* a = reinterpret_cast<const bf16_t*>(A);
  const bf16_t* b = reinterpret_cast<const bf16_t*>(B);
  if (big) hipLaunchKernelGGL((k_wgrad_wide<256, 256>), grid, dim3(WT), 0, st, a, lda, b, ldb, M, N, K, kchunk, part);
  else hipLaunchKernelGGL((k_wgrad_wide<128, 128>), grid, dim3(WT), 0, st, a, lda, b, ldb, M, N, K, kchunk, part);
  hipLaunchKernelGGL(k_wide_fold, dim3(cdiv(MN, 256), ngrp), dim3(256), 0, st, part, splits, MN, per, tmp);
  hipLaunchKernelGGL(k_wide_final, dim3(cdiv(MN, 256)), dim3(256), 0, st, tmp, ngrp, M, N, alpha, C, ldc);
  return true;
}
