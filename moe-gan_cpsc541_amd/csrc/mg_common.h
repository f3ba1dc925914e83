// Shared device/host helpers for libmoegan_hip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <string>

#include "../../include/moegan_hip.h"

typedef uint16_t bf16_t;  // raw bf16 storage (activations in bf16 mode)
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef unsigned short u16x8_t __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

#define MG_DEV __device__ __forceinline__

MG_DEV float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
MG_DEV bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }  // v_cvt_pk_bf16_f32 (RNE)

// Element load/store as float regardless of storage type.
MG_DEV float ldf(const float* p, int64_t i) { return p[i]; }
MG_DEV float ldf(const bf16_t* p, int64_t i) { return bf2f(p[i]); }
MG_DEV void stf(float* p, int64_t i, float v) { p[i] = v; }
MG_DEV void stf(bf16_t* p, int64_t i, float v) { p[i] = f2bf(v); }

template <typename T> struct VecOf;  // 16-byte vectors
template <> struct VecOf<float> { static constexpr int N = 4; typedef f32x4_t type; };
template <> struct VecOf<bf16_t> { static constexpr int N = 8; typedef u16x8_t type; };
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
template <> struct VecOf<uint8_t> { static constexpr int N = 16; typedef u32x4_t type; };  // e4m3 bytes

// 8 consecutive elements <-> float[8] (16-B aligned bf16, or 2 x 16-B fp32)
MG_DEV void ld8(const float* p, float* t) {
  f32x4_t a = *reinterpret_cast<const f32x4_t*>(p), b = *reinterpret_cast<const f32x4_t*>(p + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) { t[j] = a[j]; t[j + 4] = b[j]; }
}
MG_DEV void ld8(const bf16_t* p, float* t) {
  u16x8_t a = *reinterpret_cast<const u16x8_t*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) t[j] = bf2f(a[j]);
}
// 8 consecutive elements held in their storage format until used (bf16: 4 VGPRs rather than 8 floats)
template <typename T> struct Raw8;
template <> struct Raw8<float> {
  f32x4_t a, b;
  MG_DEV void load(const float* p) {
    a = *reinterpret_cast<const f32x4_t*>(p);
    b = *reinterpret_cast<const f32x4_t*>(p + 4);
  }
  MG_DEV void zero() { a = b = f32x4_t{0.f, 0.f, 0.f, 0.f}; }
  MG_DEV float operator[](int j) const { return j < 4 ? a[j] : b[j - 4]; }
};
template <> struct Raw8<bf16_t> {
  u16x8_t a;
  MG_DEV void load(const bf16_t* p) { a = *reinterpret_cast<const u16x8_t*>(p); }
  MG_DEV void zero() { a = u16x8_t{0, 0, 0, 0, 0, 0, 0, 0}; }
  MG_DEV float operator[](int j) const { return bf2f(a[j]); }
};

MG_DEV void st8(float* p, const float* v) {
  *reinterpret_cast<f32x4_t*>(p) = f32x4_t{v[0], v[1], v[2], v[3]};
  *reinterpret_cast<f32x4_t*>(p + 4) = f32x4_t{v[4], v[5], v[6], v[7]};
}
MG_DEV void st8(bf16_t* p, const float* v) {
  u16x8_t r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = f2bf(v[j]);
  *reinterpret_cast<u16x8_t*>(p) = r;
}
__host__ __device__ inline bool mg_al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// torch.clamp semantics: NaN passes through (fminf/fmaxf alone would map NaN to a bound, hiding the
// non-finite values the training loop's guards must see, t2i_moe_gan.py:1315, :1396)
MG_DEV float clampf(float x, float lo, float hi) { return x != x ? x : fminf(fmaxf(x, lo), hi); }

MG_DEV float lrelu(float x) { return x > 0.f ? x : 0.2f * x; }
MG_DEV float lrelu_grad(float y) { return y > 0.f ? 1.f : 0.2f; }
MG_DEV float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
MG_DEV float gelu_erf_grad(float x) {
  float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}
// bf16-output forms: erf by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below the 2^-9 bf16
// rounding of the result) -- one reciprocal, one exp and five FMAs instead of the piecewise erff; the
// GELU gradient reuses that exp(-x^2/2) for the Gaussian density.  One explicit operation sequence (every FMA
// spelled out, so no contraction choice differs between forms) instantiated for a scalar and for a pair: the pair
// form runs its multiplies and FMAs as packed-fp32 instructions (v_pk_fma_f32 / v_pk_mul_f32, two elements per
// instruction; rcp / exp stay per element) and gives the same bits per element.  The fused expert kernels spend
// most of their VALU issue here (the backward's GELU' per hidden unit was ~30 instructions per element).
typedef float f32x2_t __attribute__((ext_vector_type(2)));
MG_DEV float gfma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
MG_DEV f32x2_t gfma(f32x2_t a, f32x2_t b, f32x2_t c) { return __builtin_elementwise_fma(a, b, c); }
MG_DEV float gabs(float a) { return __builtin_fabsf(a); }
MG_DEV f32x2_t gabs(f32x2_t a) { return __builtin_elementwise_abs(a); }
MG_DEV float gcopysign(float a, float b) { return __builtin_copysignf(a, b); }
MG_DEV f32x2_t gcopysign(f32x2_t a, f32x2_t b) { return __builtin_elementwise_copysign(a, b); }
MG_DEV float grcp(float a) { return __builtin_amdgcn_rcpf(a); }
MG_DEV f32x2_t grcp(f32x2_t a) { return f32x2_t{__builtin_amdgcn_rcpf(a.x), __builtin_amdgcn_rcpf(a.y)}; }
MG_DEV float gexp(float a) { return __expf(a); }
MG_DEV f32x2_t gexp(f32x2_t a) { return f32x2_t{__expf(a.x), __expf(a.y)}; }
template <typename V> MG_DEV V gsplat(float c) { return V(c); }
// (t, g) of the erf approximation: t = 1 / (1 + p a), g = exp(-a^2), a = |x| / sqrt 2; returns erf(|x| / sqrt 2)
// with the sign of x
template <typename V> MG_DEV V gelu_erf_core(V x, V& g) {
  const V a = gabs(x) * gsplat<V>(0.70710678118654752f);
  const V t = grcp(gfma(gsplat<V>(0.3275911f), a, gsplat<V>(1.f)));
  g = gexp(-(a * a));  // exp(-x^2 / 2)
  V q = gfma(t, gsplat<V>(1.061405429f), gsplat<V>(-1.453152027f));
  q = gfma(t, q, gsplat<V>(1.421413741f));
  q = gfma(t, q, gsplat<V>(-0.284496736f));
  q = gfma(t, q, gsplat<V>(0.254829592f));
  const V p = t * q;
  return gcopysign(gfma(-p, g, gsplat<V>(1.f)), x);
}
template <typename V> MG_DEV V gelu_fast_t(V x) {
  V g;
  const V e = gelu_erf_core(x, g);
  const V hx = x * gsplat<V>(0.5f);
  return gfma(hx, e, hx);  // 0.5 x (1 + e)
}
template <typename V> MG_DEV V gelu_fast_grad_t(V x) {
  V g;
  const V e = gelu_erf_core(x, g);
  // 0.5 (1 + e) + x phi(x), phi(x) = exp(-x^2 / 2) / sqrt(2 pi)
  return gfma(x * gsplat<V>(0.3989422804014327f), g, gfma(gsplat<V>(0.5f), e, gsplat<V>(0.5f)));
}
MG_DEV float gelu_fast(float x) { return gelu_fast_t<float>(x); }
MG_DEV float gelu_fast_grad(float x) { return gelu_fast_grad_t<float>(x); }
MG_DEV f32x2_t gelu_fast2(f32x2_t x) { return gelu_fast_t<f32x2_t>(x); }
MG_DEV f32x2_t gelu_fast_grad2(f32x2_t x) { return gelu_fast_grad_t<f32x2_t>(x); }

MG_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
MG_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- error plumbing (C-ABI returns 0 / negative, message via mg_last_error) ----
void mg_set_error(const std::string& msg);
int mg_check_launch(const char* what);
// Tuning overrides (0 = automatic), set through mg_set_tuning for A/B measurements.
enum { MG_TUNE_WGRAD_TILE = 0, MG_TUNE_GWGRAD_TILE = 1, MG_TUNE_CONV_TILE = 2, MG_TUNE_GEMM_TILE = 3,
       MG_TUNE_WGRAD_SPLITS = 4, MG_TUNE_NO_SLABS = 5, MG_TUNE_XCD = 6 /* 0 auto (= all), 1 all, 2 split-K, 3 none */, MG_TUNE_WGRAD_MODE = 7,
       MG_TUNE_WARP_LDS = 8, MG_TUNE_SHORTK = 9, MG_TUNE_ATOMIC_BLOCKS = 10, MG_TUNE_DETERMINISTIC = 11,
       MG_TUNE_S1_OFF = 12,  // 1: weight gradients of stride-1 convs through the generic LdMCConv (A/B)
       MG_TUNE_D0_STORE = 13,  // mg_d0_fwd output path: 0 automatic, 1 straight from the accumulators, 2 LDS-staged rows
       MG_TUNE_FFN_BWD_OCC = 14,  // mg_moe_ffn_bwd: 0 automatic (one block per CU, 256 VGPRs, 128-unit chunks), 2 two blocks (128 VGPRs), 3 64-unit chunks
       MG_TUNE_WIDE_WGRAD = 15,   // 1: long-reduction weight gradients through the generic split-K GEMM (A/B), 2: mg_wgrad_wide.hip on every eligible shape, 3: the same (128^2 tiles), 4: 256^2 tiles where M, N >= 256
       MG_TUNE_NARROW = 16,  // the 32-channel 3x3 convs (offset heads) through the implicit GEMM: 1 all, 2 fwd, 3 dgrad, 4 wgrad
       MG_TUNE_NARROW_BLOCKS = 17,  // mg_narrow.hip grid target (blocks): 0 automatic
       MG_TUNE_DISPATCH3 = 18,  // 1: mg_moe_dispatch as count / scan / scatter (A/B; default count + scatter-scan)
       MG_TUNE_NARROW_WPX = 19,  // 4: offset-head forward on 256-pixel tiles (four pixel fragments per wave; A/B)
       MG_TUNE_GWGRAD_BLOCKS = 20,  // mg_gemm_grouped_wgrad split target (blocks of 128^2 tiles): 0 automatic (512)
       MG_TUNE_BATCH_SPLIT = 21,  // mg_gemm_batch split-K slabs, > 1: on, that block target (A/B; 0 / 1 off: neutral in the step)
       MG_TUNE_GROUPED_SHORTK = 22,  // grouped expert GEMMs with K <= this on 64^2 tiles (0: 512, -1: never)
       MG_TUNE_SPLITK_FUSED = 23,    // 1: split-K slabs reduced inside the launch (measured slower at C2: off)
       MG_TUNE_ROUTER_TEAM = 24,     // A/B bitmask, lane-FMA forms instead of the MFMA / team ones: 1 router
                                     // logits, 2 router backward (thread per token), 4 token gradient
       MG_TUNE_ADAMW_CACHED = 25,    // 1: AdamW streams through the caches (A/B; default non-temporal loads / stores)
       MG_TUNE_ATOMIC_MINK = 26,     // atomic split-K GEMMs: the least K per split (0: automatic)
       MG_TUNE_WIDE_BLOCKS = 27,     // mg_wgrad_wide.hip grid target (blocks): 0 automatic (256)
       MG_TUNE_WGRAD_SLAB_BLOCKS = 28,  // conv weight-gradient slab split target (blocks): 0 automatic (1024)
       MG_TUNE_COUNT = 29 };
extern std::atomic<int> g_mg_tune[MG_TUNE_COUNT];
// Deterministic mode (mg_set_tuning(MG_TUNE_DETERMINISTIC, 1)): every reduction that crosses workgroups runs in
// a fixed order -- per-block partial rows in the stream's workspace folded by one pass, or one writer per
// output element -- instead of fp32 atomics, so a step is bit-reproducible run to run (slower).
inline bool mg_det() { return g_mg_tune[MG_TUNE_DETERMINISTIC].load(std::memory_order_relaxed) != 0; }
// Device scratch, one block per (device, stream): caller-owned (mg_set_workspace) or library-owned
// (grown on demand, never shrunk).  NULL when it cannot be provided (mg_last_error says why).
void* mg_workspace(size_t bytes, hipStream_t stream);
// per-stream zeroed int counters for in-launch split-K reductions (mg_gemm.h gemm_splitk_fused_kernel): at least n,
// allocated and zeroed outside stream capture only (NULL otherwise: the caller takes the two-launch form)
int* mg_tile_counters(int n, hipStream_t stream);
// Gradient folds (mg_fold.hip).  A producer of fold partials asks mg_fold_alloc first: non-NULL = the stream defers
// its folds (mg_fold_defer) and the partials live in the deferral arena until the flush, so the fold is recorded
// (deferred = true); NULL = take mg_workspace and fold now.  Both paths run the same fold kernels.
void* mg_fold_alloc(size_t bytes, hipStream_t stream);
int mg_fold_rows_submit(const mg_fold_rows& r, bool deferred, hipStream_t stream);
int mg_fold_wgrad_submit(const mg_fold_wgrad& r, bool deferred, hipStream_t stream);
// partials buffer for a fold: the deferral arena when the stream defers, else the stream's workspace
inline float* mg_fold_partials(size_t bytes, hipStream_t st, bool* deferred) {
  void* p = mg_fold_alloc(bytes, st);
  *deferred = p != nullptr;
  return reinterpret_cast<float*>(p ? p : mg_workspace(bytes, st));
}

// Fixed-order fold of partial rows (deterministic mode): out_a[i] += sum_r part[r * ncols + i] for i < na,
// out_b[i - na] += ... for na <= i < ncols (64 columns x 16 row lanes per block, rows folded in lane order).
namespace {
__global__ __launch_bounds__(1024) void k_det_fold_rows(const float* __restrict__ part, int nrows, int ncols, int na,
                                                        float* __restrict__ out_a, float* __restrict__ out_b) {
  __shared__ float red[16][64];
  const int cx = threadIdx.x & 63, ry = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + cx;
  float s = 0.f;
  if (i < ncols)
    for (int r = ry; r < nrows; r += 16) s += part[(int64_t)r * ncols + i];
  red[ry][cx] = s;
  __syncthreads();
  if (ry == 0 && i < ncols) {
    float t = 0.f;
#pragma unroll
    for (int y = 0; y < 16; ++y) t += red[y][cx];
    if (i < na) out_a[i] += t;
    else out_b[i - na] += t;
  }
}
// out[0] += sum of part[0 .. n) in a fixed order (one block)
__global__ __launch_bounds__(256) void k_det_sum(const float* __restrict__ part, int n, float* __restrict__ out) {
  __shared__ float ws[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += part[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] += (ws[0] + ws[1]) + (ws[2] + ws[3]);
}
}  // namespace
static inline void mg_det_fold_rows(const float* part, int nrows, int ncols, int na, float* out_a, float* out_b,
                             hipStream_t st) {
  hipLaunchKernelGGL(k_det_fold_rows, dim3((ncols + 63) / 64), dim3(1024), 0, st, part, nrows, ncols, na, out_a, out_b);
}

#define MG_REQUIRE(cond, msg)                       \
  do {                                              \
    if (!(cond)) {                                  \
      mg_set_error(std::string(__func__) + ": " + (msg)); \
      return MG_ERR_ARG;                            \
    }                                               \
  } while (0)

static inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// mg_narrow.hip: direct 3x3 / s1 / p1 convs with a 32-channel side on 4x4 .. 16x16 maps (bf16 NHWC operands)
bool mg_conv3_direct_ok(int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad, bool wgrad);
bool mg_conv3_direct(const void* x, int B, int H, int Cin, const void* wpack, int Cout, const mg_epilogue* e, void* y,
                     int64_t ldy, int y_dtype, hipStream_t st);
bool mg_wgrad3_direct(const void* gy, int64_t ldg, const void* x, int B, int H, int Cin, float** ws_out, int* splits,
                      bool* deferred,
                      hipStream_t st);

// mg_wgrad_wide.hip: wide split-K weight gradients (bf16 [K][M] x [K][N] -> fp32 C +=), true when handled
bool mg_wgrad_wide(int M, int N, int K, const void* A, int64_t lda, const void* B, int64_t ldb, float* C, int64_t ldc,
                   float alpha, hipStream_t st);
