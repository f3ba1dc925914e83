// Long-reduction weight gradients: C[M][N] += alpha * sum_k A[k][m] B[k][n] with A = the output gradient [K x M] and
// B = the layer input [K x N], both bf16 and row-major (M / N contiguous), K = tokens / pixels (16384 .. 65536) and
// M x N small: the self-attention in / out projections (t2i_moe_gan.py:545-556 backward, 128 x 128 .. 768 x 256)
// and the 1x1 convolutions (ConvolutionBlock.skip_proj / AttentionBlock.proj_in / proj_out, :574, :615-616: Cout x Cin
// over B*H*W pixels).
//
// The generic GEMM runs these as 64 x 64 tiles split over K with fp32 atomics: every A strip is re-read N / 64 times
// and every B strip M / 64 times, and each block walks its K chunk with one step of loads in flight, so a step costs a
// full HBM round trip (~1-2 us) against ~50 ns of MFMA work -- 20-40 us per call for 8-67 MB of operands.  Here a
// block owns a 128 x 128 or 256 x 256 output tile (all of M x N for most shapes) for one K chunk, so the operands are
// read once or twice, and streams its chunk through an 8-stage LDS-DMA ring (buffer_load ... lds) with six 16 KiB K
// steps in flight while one is multiplied.  The per-block fp32 partial tiles are folded in a fixed order
// (deterministic in both library modes) by the gradient-fold rows pass (mg_fold.hip, deferred to the backward's flush
// inside a step), or by two passes of their own for a scaled / strided C.
//
// Block: 512 threads = 8 waves as 2 (M) x 4 (N), wave tile (BM/2) x (BN/4) of 16x16 fragments, read from the
// row-major ("MC") LDS images by the hardware transpose read (ds_read_b64_tr_b16).  Rows past the split's chunk and
// columns past M / N take an out-of-range offset (the hardware writes zeros): no branches in the loop.
#include <algorithm>

#include "mg_gemm.h"

namespace {
using mg::dma16;
using mg::dma_desc;
using mg::i32x4_t;
using mg::MG_OOB;

typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

constexpr int WT = 512;  // threads

// LDS image of one K step: [BK rows][BM cols] bf16 per operand, unpadded (each LDS-DMA wave-instruction fills 1 KiB
// = 1024 / (2 BM) consecutive rows in lane order), 16-B chunk c of row k stored at chunk c ^ swz(k): the eight rows
// k = 8g + q (g = 0, 1; q < 4) that one 32-lane half of a ds_read_b64_tr_b16 touches land on distinct 32-B bank pairs.
MG_DEV int swz(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 1; }

// the LDS-DMAs are asm statements (mg_gemm.h dma16): hipcc treats the ds_read_b64_tr_b16 intrinsic as aliasing any
// in-flight LDS-DMA and would drain every DMA (vmcnt(0)) before each step's fragment reads
MG_DEV bf16x8_t mc_frag(const bf16_t* img, int cols, int kbase, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int k = kbase + 8 * g + q;
  auto base = (__attribute__((address_space(3))) char*)(img);
  const int ch = (c0 >> 3) + (p >> 1), sub = (p & 1) * 8;  // 16-B chunk of column c0 + 4p, byte offset in it
  s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4_t*)(base + k * cols * 2 + ((ch ^ swz(k)) << 4) + sub));
  s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4_t*)(base + (k + 4) * cols * 2 + ((ch ^ swz(k + 4)) << 4) + sub));
  u16x8_t r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return __builtin_bit_cast(bf16x8_t, r);
}

// NB LDS stages, NB - 2 K steps of LDS-DMA in flight while one is multiplied: step t + NB - 2 is issued into the stage
// step t - 2 read (every wave finished reading it before the barrier of step t - 1), a counted vmcnt retires this
// wave's DMA of step t, and one raw barrier per step publishes it (the pipeline rules of cdna_hip_programming.md
// "Pipelining across barriers": all LDS in one array, no __syncthreads while a DMA is in flight).  Steps past the
// split's rows read zeros (out-of-range offsets), so every step issues the same DMA count.
template <int BM, int BN, int BK, int NB>
__global__ __launch_bounds__(WT) void k_wgrad_wide(const bf16_t* __restrict__ A, int64_t lda,
                                                   const bf16_t* __restrict__ B, int64_t ldb, int M, int N, int K,
                                                   int kchunk, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) bf16_t dsm[];
  constexpr int AE = BK * BM, STAGE = BK * (BM + BN);
  constexpr int ARI = 512 / BM, BRI = 512 / BN;  // rows per 1-KiB DMA instruction
  constexpr int AI = BK / ARI / 8, BI = BK / BRI / 8;  // DMA instructions per wave per step
  constexpr int PER = AI + BI;
  constexpr int WM = BM / 2, WN = BN / 4, FM = WM / 16, FN = WN / 16;
  static_assert(AI >= 1 && BI >= 1 && NB >= 3, "tile / stage shape");
  static_assert((NB - 2) * PER < 64, "vmcnt range");
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int k_lo = blockIdx.z * kchunk, k_hi = std::min(K, k_lo + kchunk);
  const i32x4_t ra = dma_desc(A), rb = dma_desc(B);
  // instruction i of wave w fills rows (8i + w) * RI ..; lane L: row + L / (cols / 8), physical chunk L % (cols / 8)
  int a_r[AI], b_r[BI];
  uint32_t a_off[AI], b_off[BI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int r = (8 * i + wid) * ARI + lane / (BM / 8), c = m0 + 8 * ((lane % (BM / 8)) ^ swz(r));
    a_r[i] = r;
    a_off[i] = c < M ? (uint32_t)(((int64_t)(k_lo + r) * lda + c) * 2) : MG_OOB;
  }
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int r = (8 * i + wid) * BRI + lane / (BN / 8), c = n0 + 8 * ((lane % (BN / 8)) ^ swz(r));
    b_r[i] = r;
    b_off[i] = c < N ? (uint32_t)(((int64_t)(k_lo + r) * ldb + c) * 2) : MG_OOB;
  }
  auto issue = [&](int t) {
    const int k0 = t * BK;
    bf16_t* st = dsm + (t % NB) * STAGE;
    const uint32_t sa = (uint32_t)((int64_t)k0 * lda * 2), sb = (uint32_t)((int64_t)k0 * ldb * 2);
#pragma unroll
    for (int i = 0; i < AI; ++i)
      dma16(ra, k_lo + k0 + a_r[i] < k_hi ? a_off[i] : MG_OOB, sa, st + (8 * i + wid) * 512);
#pragma unroll
    for (int i = 0; i < BI; ++i)
      dma16(rb, k_lo + k0 + b_r[i] < k_hi ? b_off[i] : MG_OOB, sb, st + AE + (8 * i + wid) * 512);
  };
  f32x4_t acc[FM][FN];
#pragma unroll
  for (int a = 0; a < FM; ++a)
#pragma unroll
    for (int b = 0; b < FN; ++b) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int nsteps = std::max(0, (k_hi - k_lo + BK - 1) / BK);
#pragma unroll
  for (int p = 0; p < NB - 2; ++p) issue(p);
  for (int t = 0; t < nsteps; ++t) {
    issue(t + NB - 2);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NB - 2) * PER) : "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const bf16_t* as = dsm + (t % NB) * STAGE;
    const bf16_t* bs = as + AE;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8_t b[FN];
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) b[fn] = mc_frag(bs, BN, kk, wn * WN + 16 * fn, lane);
#pragma unroll
      for (int fm = 0; fm < FM; ++fm) {
        const bf16x8_t a = mc_frag(as, BM, kk, wm * WM + 16 * fm, lane);
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
          acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[fn], acc[fm][fn], 0, 0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the zero-row DMAs past the last step land before the block ends
  // this block's partial tile, staged through the (now idle) LDS as [BM][BN] fp32 and stored in natural order as
  // 16-B row runs: part[split][m][n] (row pitch N), what the gradient-fold rows pass reads
  float* pb = part + (int64_t)blockIdx.z * M * N;
  if constexpr (BM * BN * 4 <= NB * STAGE * 2) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    float* tile = reinterpret_cast<float*>(dsm);
#pragma unroll
    for (int fm = 0; fm < FM; ++fm)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          tile[(wm * WM + 16 * fm + 4 * (lane >> 4) + j) * BN + wn * WN + 16 * fn + (lane & 15)] = acc[fm][fn][j];
    __syncthreads();
    for (int v = tid; v < BM * BN / 4; v += WT) {
      const int r = v / (BN / 4), c = (v % (BN / 4)) * 4, m = m0 + r, n = n0 + c;
      if (m < M && n < N)
        *reinterpret_cast<f32x4_t*>(pb + (int64_t)m * N + n) = *reinterpret_cast<const f32x4_t*>(tile + r * BN + c);
    }
  } else {  // (256^2 tiles: 256 KiB of partial tile, more than the LDS ring -- straight from the accumulators)
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
}

// immediate fold (a scaled or strided C): level 1 tmp[grp][i] = sum of part[s][i] over the group's splits
// (ascending), level 2 C[m][n] += alpha * sum of tmp[grp][i] (ascending); i = m * N + n
__global__ __launch_bounds__(256) void k_wide_fold(const float* __restrict__ part, int nsplit, int64_t MN, int per,
                                                   float* __restrict__ tmp) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= MN) return;
  const int s0 = blockIdx.y * per, s1 = std::min(nsplit, s0 + per);
  f32x4_t s = {0.f, 0.f, 0.f, 0.f};
  int r = s0;
  for (; r + 8 <= s1; r += 8) {
    f32x4_t v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = *reinterpret_cast<const f32x4_t*>(part + (int64_t)(r + q) * MN + i);
#pragma unroll
    for (int q = 0; q < 8; ++q) s += v[q];
  }
  for (; r < s1; ++r) s += *reinterpret_cast<const f32x4_t*>(part + (int64_t)r * MN + i);
  *reinterpret_cast<f32x4_t*>(tmp + (int64_t)blockIdx.y * MN + i) = s;
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

template <int BM, int BN, int BK, int NB>
void launch_wide(dim3 grid, hipStream_t st, const bf16_t* a, int64_t lda, const bf16_t* b, int64_t ldb, int M, int N,
                 int K, int kchunk, float* part) {
  constexpr int bytes = NB * BK * (BM + BN) * 2;
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&k_wgrad_wide<BM, BN, BK, NB>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL((k_wgrad_wide<BM, BN, BK, NB>), grid, dim3(WT), bytes, st, a, lda, b, ldb, M, N, K, kchunk, part);
}

}  // namespace

// Called by mg_gemm for bf16, a_kc = b_kc = 0 (both operands [K][*] row-major), an fp32 C accumulated through a
// plain atomic epilogue (alpha only), and by mg_conv2d_wgrad for 1x1 / stride-1 convolutions.  Returns true when it
// handled the call.
bool mg_wgrad_wide(int M, int N, int K, const void* A, int64_t lda, const void* B, int64_t ldb, float* C, int64_t ldc,
                   float alpha, hipStream_t st) {
  const int mode = g_mg_tune[MG_TUNE_WIDE_WGRAD];
  if (mode == 1) return false;  // A/B: the generic split-K GEMM
  if (K < 2048 || M % 8 || N % 8 || (int64_t)M * N > 1024 * 1024) return false;
  // a win when K is long against the tile edges (profiles/round6_wgrad_wide_probe.txt); a 16-wide N leaves the MFMA
  // tile mostly empty (2: every eligible shape, tests)
  if (mode < 2 && ((int64_t)K < 32 * (int64_t)(M + N) || M < 64 || N < 64)) return false;
  // 128^2 tiles, K steps of 32 rows in 8 LDS stages of 16 KiB (six steps = 96 KiB in flight per block: the HBM
  // latency under load is ~2 us against ~0.1 us of MFMA work per step); 256^2 tiles (operands read once, only two
  // 32 KiB steps in flight within the LDS) on request (mode 4)
  const bool big = M >= 256 && N >= 256 && mode == 4;
  const int BM = big ? 256 : 128, BN = BM, BK = 32;
  const int64_t tiles = (int64_t)cdiv(M, BM) * cdiv(N, BN);
  // ~target blocks (tuning slot MG_TUNE_WIDE_BLOCKS, default 256), >= 8 K steps each, <= 128 splits: the folds read
  // every split's partial tile (measured, profiles/round6_wgrad_wide_probe.txt: 128 x 128 x 65536 in 128 splits
  // 18.8 us with its folds, in 256 splits 23.6 us)
  const int target = g_mg_tune[MG_TUNE_WIDE_BLOCKS] > 0 ? (int)g_mg_tune[MG_TUNE_WIDE_BLOCKS] : 256;
  int splits = (int)std::max<int64_t>(
      1, std::min<int64_t>({std::max<int64_t>(1, target / tiles), (int64_t)K / (8 * BK), (int64_t)128}));
  const int kchunk = cdiv(cdiv(K, splits), BK) * BK;
  splits = cdiv(K, kchunk);
  const int64_t MN = (int64_t)M * N;
  const bf16_t* a = reinterpret_cast<const bf16_t*>(A);
  const bf16_t* b = reinterpret_cast<const bf16_t*>(B);
  const dim3 grid(cdiv(M, BM), cdiv(N, BN), splits);
  // an unscaled, dense C (every weight gradient of the step): the partial tiles go through the gradient-fold rows
  // pass -- deferred to the backward's flush inside a step (one launch for every fold of the phase), immediate
  // otherwise; same fixed split order either way
  if (alpha == 1.f && ldc == N) {
    bool deferred = false;
    float* part = mg_fold_partials((size_t)splits * MN * sizeof(float), st, &deferred);
    if (!part) return false;
    if (big) launch_wide<256, 256, 32, 4>(grid, st, a, lda, b, ldb, M, N, K, kchunk, part);
    else launch_wide<128, 128, 32, 8>(grid, st, a, lda, b, ldb, M, N, K, kchunk, part);
    mg_fold_rows_submit(mg_fold_rows{part, MN, (int32_t)splits, (int32_t)MN, (int32_t)MN, C, nullptr}, deferred, st);
    return true;
  }
  const int per = 16, ngrp = (splits + per - 1) / per;
  float* part = reinterpret_cast<float*>(mg_workspace((size_t)(splits + ngrp) * MN * sizeof(float), st));
  if (!part) return false;
  float* tmp = part + (size_t)splits * MN;
  if (big) launch_wide<256, 256, 32, 4>(grid, st, a, lda, b, ldb, M, N, K, kchunk, part);
  else launch_wide<128, 128, 32, 8>(grid, st, a, lda, b, ldb, M, N, K, kchunk, part);
  hipLaunchKernelGGL(k_wide_fold, dim3(cdiv(MN, 1024), ngrp), dim3(256), 0, st, part, splits, MN, per, tmp);
  hipLaunchKernelGGL(k_wide_final, dim3(cdiv(MN, 256)), dim3(256), 0, st, tmp, ngrp, M, N, alpha, C, ldc);
  return true;
}
