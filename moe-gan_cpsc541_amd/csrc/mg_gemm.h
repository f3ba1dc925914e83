// MFMA GEMM core for libmoegan_hip (gfx950).
//
// C[m, n] = sum_k A[m, k] * B[k, n], tiles staged through LDS with both
// operands stored k-contiguous ([rows][BK+pad]) so every lane reads its MFMA
// fragment with one 16-byte ds_read.  When two LDS stages fit (bf16), the K loop
// is double-buffered with two register stages: step t+3 is loaded while step t
// is multiplied, one barrier per K step.  256 threads = 4 waves in a 2x2
// arrangement; each wave owns a (BM/2)x(BN/2) sub-tile of 16x16 fragments.
//
//   T = bf16_t : v_mfma_f32_16x16x32_bf16 (fp32 accumulate)
//   T = float  : v_mfma_f32_16x16x4_f32   (exact fp32, the parity mode)
//
// Operand access is delegated to loader structs so one kernel body serves
// plain / transposed operands, implicit NHWC convolutions, the parity-class
// split of a stride-2 data gradient, per-group weights for expert batches and
// (XF instantiations only) row gathers, GELU-on-load and modulation scales.
// Loads are raw buffer loads with hardware zero-fill for out-of-range slots;
// see the Loaders section.
//
// Grouping (expert batches) is resolved per block from device-side offset
// tables, so no host synchronisation is needed to size the launch.
#pragma once
#include <type_traits>

#include "mg_common.h"

namespace mg {


constexpr int NTHREADS = 256;
// K-loop pipeline (build-time): tiles of at most MG_DB_MAX_TILE outputs double-buffer LDS (one barrier
// per K step) when two stages fit 64 KiB; MG_NSTAGE register stages in that mode.
#ifndef MG_DB_MAX_TILE
#define MG_DB_MAX_TILE 0  // measured: double buffering lost to the occupancy it costs (v0-v3 A/B)
#endif
#ifndef MG_NSTAGE
#define MG_NSTAGE 1
#endif
// LDS-DMA (buffer_load ... lds) staging for bf16 KC x KC tiles
// epilogue staging synchronised per block (1) or per wave (0: each wave owns its staging band)
#ifndef MG_EPI_BLOCK_SYNC
#define MG_EPI_BLOCK_SYNC 0
#endif
// single LDS buffer with two register stages (prefetch distance two K steps) for tiles of at most
// MG_SB2_MAX_TILE outputs
#ifndef MG_SB2_MAX_TILE
#define MG_SB2_MAX_TILE 0
#endif
// raise the wave priority over the K step's MFMA phase (A/B switch; MI355X_MICROARCH.md: static priority)
#ifndef MG_EPI_PREFETCH
#define MG_EPI_PREFETCH 1
#endif
#ifndef MG_SETPRIO
#define MG_SETPRIO 1  // measured: step 9.273 -> 9.245 ms, 4096^3 953 -> 1066 TF/s, D conv1 751 -> 815 TF/s
#endif
#ifndef MG_GLDS
#define MG_GLDS 0  // measured: on par with register staging at C2 (gemm 4096^3 +9%, expert GEMMs -20%)
#endif
// LDS-DMA staging for the implicit-conv forward / data-gradient tiles of at most 64 x 64 outputs only (the latency-
// bound 3x3 modulated convs on 4x4 / 8x8 / 16x16 maps: their per-step VGPR -> LDS stores are the register path's
// cost; measured round 6 with MG_GLDS on everything: conv8 41.4 -> 35.7 us, conv4 47.7 -> 42.9 us, while the
// expert GEMMs lost, so the switch is per loader)
#ifndef MG_GLDS_CONV
#define MG_GLDS_CONV 1
#endif
// LDS-DMA staging for 64 x 64 tiles whose operands are both k-major ("MC": weight gradients, C = A^T B over pixels
// / tokens): unpadded LDS images swizzled on the source side, the DMAs as asm statements (hipcc treats the
// ds_read_b64_tr_b16 intrinsic as aliasing any in-flight LDS-DMA and would wait vmcnt(0) before every fragment read)
#ifndef MG_GLDS_MC
#define MG_GLDS_MC 1
#endif
// LDS stages of the LDS-DMA pipeline: the loads of step t + STAGES - 1 are in flight while step t is multiplied.
// 3 runs one barrier per step (step t + 2 issued after step t's barrier); measured slower on every 64^2 conv tile
// (conv 3x3 at 8^2 35.7 -> 43.4 us, the 16^2 weight gradient 46.9 -> 61.6 us, step 8.10 -> 8.29 ms, same box): the
// third 16 KiB stage costs more resident blocks than the deeper prefetch and the saved barrier give back
#ifndef MG_GLDS_STAGES
#define MG_GLDS_STAGES 2
#endif

template <typename T> struct Frag;
template <> struct Frag<bf16_t> { static constexpr int PAD = 8; };
template <> struct Frag<float> { static constexpr int PAD = 4; };

template <typename T> MG_DEV typename VecOf<T>::type vzero() { return typename VecOf<T>::type(0); }

// scale a vector by per-element fp32 factors (modulation / gate), returning storage type
MG_DEV f32x4_t vscale(f32x4_t v, const float* s) { return f32x4_t{v[0] * s[0], v[1] * s[1], v[2] * s[2], v[3] * s[3]}; }
MG_DEV u16x8_t vscale(u16x8_t v, const float* s) {
  u16x8_t r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = f2bf(bf2f(v[j]) * s[j]);
  return r;
}
MG_DEV f32x4_t vscale1(f32x4_t v, float s) { return v * s; }
MG_DEV u16x8_t vscale1(u16x8_t v, float s) {
  u16x8_t r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = f2bf(bf2f(v[j]) * s);
  return r;
}
MG_DEV f32x4_t vgelu(f32x4_t v) { return f32x4_t{gelu_erf(v[0]), gelu_erf(v[1]), gelu_erf(v[2]), gelu_erf(v[3])}; }
// bf16 operands: the epilogues' fast erf form (|erf error| <= 1.5e-7, far below the bf16 rounding of the result;
// the piecewise erff is ~3x the instructions in a loader that runs per K step)
MG_DEV u16x8_t vgelu(u16x8_t v) {
  u16x8_t r;
#pragma unroll
  for (int j = 0; j < 8; j += 2) {  // element pairs on packed fp32
    const f32x2_t y = gelu_fast2(f32x2_t{bf2f(v[j]), bf2f(v[j + 1])});
    r[j] = f2bf(y.x);
    r[j + 1] = f2bf(y.y);
  }
  return r;
}

// ---------------------------------------------------------------------------
// Loaders
// ---------------------------------------------------------------------------
// Every operand vector is fetched by a raw buffer load through a wave-uniform descriptor covering
// [0, 2^31) bytes.  A slot that must read zeros (row past M, padding tap, K tail) is given the
// out-of-range offset MG_OOB and the hardware returns 0: no exec-mask branches, no selects on the
// loaded data.  Per-slot state (byte offset of the slot's row / column, valid-tap masks) is computed
// once before the K loop, so a K step costs at most a few VALU per vector (0 for plain operands,
// whose K advance rides in the scalar offset).
//
// XF = the operand needs a transform (row gather, GELU-on-load, row / channel scale).  Transforms
// are applied by fix() when the staged registers are written to LDS -- after the MFMAs of the
// step -- so they never wait on a load that is still in flight.  The fast instantiations (XF =
// false) carry none of that code.
//
//   KC loader (reduction index contiguous): Slot slot(int row, int kofs, bool ok)
//   MC loader (output index contiguous):   Slot slot(int col0, int kofs, bool ok)
//   both:  template <bool TAIL, int TBK> vec load(rsrc, const Slot&, int k0, int kend)
//          void fix(const Slot&, int k0, vec&)      (XF only)
// Offsets are 32-bit: every operand tensor must be < 2 GiB (checked on the host).

constexpr uint32_t MG_OOB = 0x80000000u;
typedef __amdgpu_buffer_rsrc_t rsrc_t;
MG_DEV rsrc_t make_rsrc(const void* p) {
  // the base is wave-uniform (kernel argument / block-derived); readfirstlane makes that provable so the
  // compiler keeps the descriptor in SGPRs (no waterfall loops around the loads)
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0, 0x7fffffff,
                                           0x00020000);
}
template <typename V> MG_DEV V bload(rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
// LDS-DMA form (buffer_load_dwordx4 ... lds): the wave's 64 x 16 B land contiguously at the wave-uniform
// LDS address `lds` (lane order); out-of-range offsets write zeros.
MG_DEV void bload_lds(rsrc_t r, uint32_t voff, uint32_t soff, void* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}
// The same DMA as an asm statement, for the MC images (see MG_GLDS_MC): raw descriptor words (as make_rsrc), M0 saved
// and restored inside the statement; s_nop 4 covers a descriptor / soffset SGPR just written by v_readfirstlane,
// s_nop 0 the M0 write before the DMA (cdna_hip_programming.md §5.7).  Waited for by the kernel's counted vmcnt.
typedef int i32x4_t __attribute__((ext_vector_type(4)));
MG_DEV i32x4_t dma_desc(const void* p) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  return i32x4_t{(int)__builtin_amdgcn_readfirstlane((uint32_t)a), (int)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)),
                 0x7fffffff, 0x00020000};
}
MG_DEV void dma16(const i32x4_t& d, uint32_t voff, uint32_t soff, const void* lds) {
  const uint32_t m = __builtin_amdgcn_readfirstlane(
      (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const void*)lds));
  unsigned keep;
  asm volatile(
      "s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(d), "s"(m), "s"(__builtin_amdgcn_readfirstlane(soff))
      : "memory");
}
template <class L, class = void> struct has_gldsmc : std::false_type {};
template <class L> struct has_gldsmc<L, std::void_t<decltype(L::kGldsMC)>> : std::integral_constant<bool, L::kGldsMC> {};

// KC loaders define offs<TAIL, TBK>(slot, k0, kend, voff, soff); load / glds derive from it.
#define MG_KC_LOADS                                                                                           \
  template <bool TAIL, int TBK> MG_DEV vec_t load(rsrc_t r, const Slot& s, int k0, int kend) const {          \
    uint32_t o, so;                                                                                           \
    offs<TAIL, TBK>(s, k0, kend, o, so);                                                                      \
    return bload<vec_t>(r, o, so);                                                                            \
  }                                                                                                           \
  template <bool TAIL, int TBK> MG_DEV void glds(rsrc_t r, const Slot& s, int k0, int kend, void* lds) const { \
    uint32_t o, so;                                                                                           \
    offs<TAIL, TBK>(s, k0, kend, o, so);                                                                      \
    bload_lds(r, o, so, lds);                                                                                 \
  }

// KC, plain rows with optional row gather / per-row scale / GELU-on-load (XF).
//   row r -> source row (idx ? idx[r] / idx_div : r); value *= rs[r] if rs
template <typename T, bool XF = false>
struct LdKC {
  typedef typename VecOf<T>::type vec_t;
  const T* p; int64_t ld; int rows; int K;
  const int* idx; int idx_div;   // gather: source row = idx[r] / idx_div
  const float* rs;               // optional per-row scale (indexed by r)
  int gelu;                      // apply GELU to loaded values
  struct Slot { uint32_t off; int kofs; float s; };
  MG_DEV void set_group(int) {}
  MG_DEV rsrc_t rsrc() const { return make_rsrc(p); }
  MG_DEV Slot slot(int r, int kofs, bool ok) const {
    Slot s{MG_OOB, kofs, 1.f};
    if (ok && r < rows) {
      int src = r;
      if constexpr (XF) {
        if (idx) src = idx[r] / idx_div;
        if (rs) s.s = rs[r];
      }
      s.off = (uint32_t)(((int64_t)src * ld + kofs) * (int64_t)sizeof(T));
    }
    return s;
  }
  static constexpr bool kGlds = !XF;  // no transform: may stage by LDS-DMA
  static constexpr bool kConv = false;  // implicit-convolution A loader (LdKCConv)
  template <bool TAIL, int TBK> MG_DEV void offs(const Slot& s, int k0, int kend, uint32_t& off, uint32_t& soff) const {
    off = s.off;
    if constexpr (TAIL) off = (k0 + s.kofs < kend) ? off : MG_OOB;
    soff = (uint32_t)k0 * (uint32_t)sizeof(T);
  }
  MG_KC_LOADS
  MG_DEV void fix(const Slot& s, int, vec_t& v) const {
    if constexpr (XF) {
      if (gelu) v = vgelu(v);
      if (rs) v = vscale1(v, s.s);
    }
  }
};

// KC, implicit NHWC convolution: row = output pixel (b, oh, ow), k = tap*Cin + ci.
// Requires Cin % VEC == 0 (one tap per vector) and power-of-two OH/OW/Cin; KH*KW <= 32.
// The slot keeps the byte offset of its pixel's tap (0, 0) and a bit mask of the taps that fall
// inside the image.  SC = false (Cin >= TBK): a K step lies inside one tap, so the tap and its offset
// are wave-uniform scalars and a vector costs 4 VALU; SC = true (small Cin): per-lane tap.
template <typename T, bool XF = false, bool SC = false>
struct LdKCConv {
  typedef typename VecOf<T>::type vec_t;
  const T* x; int H, W, Cin, lgCin, lgOW, lgOHW, M;
  int KW, stride, pad, K;
  const float* scale;  // optional [B, Cin] per-sample input-channel scale (modulation), XF only
  int kwinv;           // (tap * kwinv) >> 16 == tap / KW for every tap of the kernel
  struct Slot { int32_t base; uint32_t mask; int kofs; int b; };
  MG_DEV void set_group(int) {}
  MG_DEV rsrc_t rsrc() const { return make_rsrc(x); }
  MG_DEV Slot slot(int r, int kofs, bool ok) const {
    Slot s{0, 0u, kofs, 0};
    if (!ok || r >= M) return s;
    s.b = r >> lgOHW;
    const int rem = r & ((1 << lgOHW) - 1);
    const int oh = rem >> lgOW, ow = rem & ((1 << lgOW) - 1);
    const int ih0 = oh * stride - pad, iw0 = ow * stride - pad;
    s.base = (((s.b * H + ih0) * W + iw0) << lgCin) * (int)sizeof(T);
    const int KH = (K >> lgCin) / KW;
    uint32_t m = 0;
    for (int kh = 0; kh < KH; ++kh)
      for (int kw = 0; kw < KW; ++kw)
        if ((unsigned)(ih0 + kh) < (unsigned)H && (unsigned)(iw0 + kw) < (unsigned)W) m |= 1u << (kh * KW + kw);
    s.mask = m;
    return s;
  }
  static constexpr bool kGlds = !XF;
  static constexpr bool kConv = true;
  template <bool TAIL, int TBK> MG_DEV void offs(const Slot& s, int k0, int kend, uint32_t& off, uint32_t& soff) const {
    const int k = k0 + s.kofs;
    const int kk = SC ? k : k0;  // SC = false: k0 is a multiple of TBK <= Cin, the step stays inside tap k0 / Cin
    const int tap = kk >> lgCin;
    const int kh = (tap * kwinv) >> 16, kw = tap - kh * KW;
    const int tapoff = (((kh * W + kw) << lgCin) + (kk & (Cin - 1))) * (int)sizeof(T);
    // invalid tap -> bit 31 set (out of range); arithmetic, not a select, so no branch is formed
    off = (uint32_t)(s.base + tapoff + (SC ? 0 : s.kofs * (int)sizeof(T))) | ((~s.mask >> tap) << 31);
    if constexpr (TAIL) off = k < kend ? off : MG_OOB;
    soff = 0;
  }
  MG_KC_LOADS
  MG_DEV void fix(const Slot& s, int k0, vec_t& v) const {
    if constexpr (XF) {
      if (scale) v = vscale(v, scale + (int64_t)s.b * Cin + ((k0 + s.kofs) & (Cin - 1)));
    }
  }
};

// MC, plain: element (k, c) at p[k*ld + c]; optional row gather on k, per-k scale, GELU-on-load (XF).
template <typename T, bool XF = false>
struct LdMC {
  typedef typename VecOf<T>::type vec_t;
  const T* p; int64_t ld; int cols; int K;
  const int* idx; int idx_div; const float* rs; int gelu;
  struct Slot { uint32_t off; int kofs; bool ok; };
  static constexpr bool kGlds = false;
  MG_DEV void set_group(int) {}
  MG_DEV rsrc_t rsrc() const { return make_rsrc(p); }
  MG_DEV Slot slot(int c0, int kofs, bool ok) const {
    Slot s{MG_OOB, kofs, ok && c0 < cols};
    if (s.ok) s.off = XF ? (uint32_t)(c0 * (int)sizeof(T)) : (uint32_t)(((int64_t)kofs * ld + c0) * (int64_t)sizeof(T));
    return s;
  }
  template <bool TAIL, int TBK> MG_DEV vec_t load(rsrc_t r, const Slot& s, int k0, int kend) const {
    if constexpr (XF) {
      const int k = k0 + s.kofs;
      const bool ok = s.ok && (!TAIL || k < kend);
      const int src = ok ? (idx ? idx[k] / idx_div : k) : 0;
      return bload<vec_t>(r, ok ? (uint32_t)((int64_t)src * ld * (int64_t)sizeof(T)) + s.off : MG_OOB, 0);
    } else {
      uint32_t off = s.off;
      if constexpr (TAIL) off = (k0 + s.kofs < kend) ? off : MG_OOB;
      return bload<vec_t>(r, off, (uint32_t)((int64_t)k0 * ld * (int64_t)sizeof(T)));
    }
  }
  MG_DEV void fix(const Slot& s, int k0, vec_t& v) const {
    if constexpr (XF) {
      const int k = k0 + s.kofs;
      if (k >= K) return;
      if (gelu) v = vgelu(v);
      if (rs) v = vscale1(v, rs[k]);
    }
  }
  static constexpr bool kGldsMC = !XF;
  MG_DEV i32x4_t desc() const { return dma_desc(p); }
  template <bool TAIL, int TBK> MG_DEV void gldsmc(const i32x4_t& d, const Slot& s, int k0, int kend, void* lds) const {
    uint32_t off = s.off;
    if constexpr (TAIL) off = (k0 + s.kofs < kend) ? off : MG_OOB;
    dma16(d, off, (uint32_t)((int64_t)k0 * ld * (int64_t)sizeof(T)), lds);
  }
};

// MC, implicit conv columns for weight gradients: element (k = output pixel, c = tap*Cin + ci).
template <typename T, bool XF = false>
struct LdMCConv {
  typedef typename VecOf<T>::type vec_t;
  const T* x; int H, W, Cin, lgCin, lgOW, lgOHW, K;  // K = number of output pixels
  int KW, stride, pad, cols;
  const float* scale;  // XF only
  struct Slot { int dh, dw, ci, kofs; uint32_t bad; };
  static constexpr bool kGlds = false;
  MG_DEV void set_group(int) {}
  MG_DEV rsrc_t rsrc() const { return make_rsrc(x); }
  MG_DEV Slot slot(int c0, int kofs, bool ok) const {
    Slot s;
    s.bad = (ok && c0 < cols) ? 0u : 1u;
    const int tap = c0 >> lgCin;
    s.ci = c0 & (Cin - 1);
    const int kh = tap / KW;
    s.dh = kh - pad;
    s.dw = tap - kh * KW - pad;
    s.kofs = kofs;
    return s;
  }
  template <bool TAIL, int TBK> MG_DEV vec_t load(rsrc_t r, const Slot& s, int k0, int kend) const {
    const int k = k0 + s.kofs;
    const int b = k >> lgOHW;
    const int oh = (k >> lgOW) & ((1 << (lgOHW - lgOW)) - 1), ow = k & ((1 << lgOW) - 1);
    const int ih = oh * stride + s.dh, iw = ow * stride + s.dw;
    const uint32_t bad = (uint32_t)((unsigned)ih >= (unsigned)H) | (uint32_t)((unsigned)iw >= (unsigned)W) | s.bad;
    uint32_t off = ((uint32_t)((((b * H + ih) * W + iw) << lgCin) + s.ci) * (uint32_t)sizeof(T)) | (bad << 31);
    if constexpr (TAIL) off = k < kend ? off : MG_OOB;
    return bload<vec_t>(r, off, 0);
  }
  MG_DEV void fix(const Slot& s, int k0, vec_t& v) const {
    if constexpr (XF) {
      const int k = k0 + s.kofs;
      if (scale && k < K) v = vscale(v, scale + (int64_t)(k >> lgOHW) * Cin + s.ci);
    }
  }
};

// MC conv columns for the weight gradient of a stride-1 "same" convolution (H = OH, W = OW) with OW <= TBK and
// OH <= 32: the input pixel of output pixel p through tap (dh, dw) is p + dh*W + dw, so the slot keeps that byte
// offset minus the step's (k0 * Cin) part, the column's validity (ow = kofs mod OW is the same every step, because
// k0 is a multiple of TBK and so of OW) and a 32-bit mask of the output rows whose tap row lies inside the image.
// A K step then costs an add / and / shift for the row test and one add + select for the offset (the generic
// LdMCConv decodes b, oh, ow and rebuilds the address per vector).
template <typename T>
struct LdMCConvS1 {
  typedef typename VecOf<T>::type vec_t;
  const T* x; int lgCin, lgOW, OH, W, KW, pad, K, cols;
  struct Slot { int32_t voff; uint32_t bad_rows; int kr; int kofs; };
  static constexpr bool kGlds = false;
  MG_DEV void set_group(int) {}
  MG_DEV rsrc_t rsrc() const { return make_rsrc(x); }
  MG_DEV Slot slot(int c0, int kofs, bool ok) const {
    const int Cin = 1 << lgCin;
    const int tap = c0 >> lgCin, ci = c0 & (Cin - 1);
    const int kh = tap / KW, dh = kh - pad, dw = tap - kh * KW - pad;
    const int ow = kofs & ((1 << lgOW) - 1);
    Slot s;
    s.kofs = kofs;
    s.kr = kofs >> lgOW;
    s.voff = (((kofs + dh * W + dw) << lgCin) + ci) * (int)sizeof(T);
    uint32_t bad = 0u;
    for (int oh = 0; oh < OH; ++oh)
      if ((unsigned)(oh + dh) >= (unsigned)OH) bad |= 1u << oh;
    if (!ok || c0 >= cols || (unsigned)(ow + dw) >= (unsigned)W) bad = 0xffffffffu;
    s.bad_rows = bad;
    return s;
  }
  template <bool TAIL, int TBK> MG_DEV vec_t load(rsrc_t r, const Slot& s, int k0, int kend) const {
    const int oh = ((k0 >> lgOW) + s.kr) & (OH - 1);
    bool bad = (s.bad_rows >> oh) & 1u;
    if constexpr (TAIL) bad = bad || (k0 + s.kofs >= kend);
    const uint32_t off = bad ? MG_OOB : (uint32_t)(s.voff + (k0 << lgCin) * (int)sizeof(T));
    return bload<vec_t>(r, off, 0);
  }
  MG_DEV void fix(const Slot&, int, vec_t&) const {}
  static constexpr bool kGldsMC = true;
  MG_DEV i32x4_t desc() const { return dma_desc(x); }
  template <bool TAIL, int TBK> MG_DEV void gldsmc(const i32x4_t& d, const Slot& s, int k0, int kend, void* lds) const {
    const int oh = ((k0 >> lgOW) + s.kr) & (OH - 1);
    bool bad = (s.bad_rows >> oh) & 1u;
    if constexpr (TAIL) bad = bad || (k0 + s.kofs >= kend);
    dma16(d, bad ? MG_OOB : (uint32_t)(s.voff + (k0 << lgCin) * (int)sizeof(T)), 0u, lds);
  }
};

// KC, data gradient of a 4x4 / stride-2 / pad-1 convolution ("transposed conv"),
// split into the 4 output-parity classes (py, px).  Row r (class-major) =
// (class, b, i, j) -> input-grid pixel (b, 2i+py, 2j+px); k = t*Cg + co with
// t = ty*2 + tx the 2x2 taps of that class reading g[b, i+dy, j+dx, co].
template <typename T, bool XF = false, bool SC = false>
struct LdKCConvT {
  typedef typename VecOf<T>::type vec_t;
  const T* g; int OH, OW, Cg, lgCg, lgOW, lgOHW, Mc, K;
  int cls;
  struct Slot { int32_t base; uint32_t mask; int kofs; };
  MG_DEV void set_group(int c) { cls = c; }
  MG_DEV rsrc_t rsrc() const { return make_rsrc(g); }
  MG_DEV static int dy_of(int py, int ty) { return py ? (ty ? 0 : 1) : (ty ? -1 : 0); }
  MG_DEV Slot slot(int r, int kofs, bool ok) const {
    Slot s{0, 0u, kofs};
    if (!ok) return s;
    const int rem = r - cls * Mc;
    const int b = rem >> lgOHW;
    const int i = (rem >> lgOW) & ((1 << (lgOHW - lgOW)) - 1), j = rem & ((1 << lgOW) - 1);
    s.base = (((b * OH + i) * OW + j) << lgCg) * (int)sizeof(T);
    const int py = cls >> 1, px = cls & 1;
    uint32_t m = 0;
    for (int t = 0; t < 4; ++t) {
      const int oh = i + dy_of(py, t >> 1), ow = j + dy_of(px, t & 1);
      if ((unsigned)oh < (unsigned)OH && (unsigned)ow < (unsigned)OW) m |= 1u << t;
    }
    s.mask = m;
    return s;
  }
  static constexpr bool kGlds = !XF;
  static constexpr bool kConv = true;  // (64^2 tiles stage it by LDS-DMA)
  template <bool TAIL, int TBK> MG_DEV void offs(const Slot& s, int k0, int kend, uint32_t& off, uint32_t& soff) const {
    const int k = k0 + s.kofs;
    const int kk = SC ? k : k0;  // SC = false: the step stays inside tap k0 / Cg (wave-uniform)
    const int t = kk >> lgCg;
    const int dy = dy_of(cls >> 1, t >> 1), dx = dy_of(cls & 1, t & 1);
    const int tapoff = (((dy * OW + dx) << lgCg) + (kk & (Cg - 1))) * (int)sizeof(T);
    off = (uint32_t)(s.base + tapoff + (SC ? 0 : s.kofs * (int)sizeof(T))) | ((~s.mask >> t) << 31);
    if constexpr (TAIL) off = k < kend ? off : MG_OOB;
    soff = 0;
  }
  MG_KC_LOADS
  MG_DEV void fix(const Slot&, int, vec_t&) const {}
};

// Grouped B operand: KC rows of a per-group weight (base + g*gstride).
template <typename T, bool XF = false>
struct LdKCGroupW {
  typedef typename VecOf<T>::type vec_t;
  const T* p0; int64_t ld; int rows; int K; int64_t gstride;
  const T* p;
  struct Slot { uint32_t off; int kofs; };
  MG_DEV void set_group(int g) { p = p0 + (int64_t)g * gstride; }
  MG_DEV rsrc_t rsrc() const { return make_rsrc(p); }
  MG_DEV Slot slot(int r, int kofs, bool ok) const {
    return Slot{(ok && r < rows) ? (uint32_t)(((int64_t)r * ld + kofs) * (int64_t)sizeof(T)) : MG_OOB, kofs};
  }
  static constexpr bool kGlds = !XF;
  static constexpr bool kConv = false;
  template <bool TAIL, int TBK> MG_DEV void offs(const Slot& s, int k0, int kend, uint32_t& off, uint32_t& soff) const {
    off = s.off;
    if constexpr (TAIL) off = (k0 + s.kofs < kend) ? off : MG_OOB;
    soff = (uint32_t)k0 * (uint32_t)sizeof(T);
  }
  MG_KC_LOADS
  MG_DEV void fix(const Slot&, int, vec_t&) const {}
};
template <typename T, bool XF = false>
struct LdMCGroupW {
  typedef typename VecOf<T>::type vec_t;
  const T* p0; int64_t ld; int cols; int K; int64_t gstride;
  const T* p;
  struct Slot { uint32_t off; int kofs; };
  static constexpr bool kGlds = false;
  MG_DEV void set_group(int g) { p = p0 + (int64_t)g * gstride; }
  MG_DEV rsrc_t rsrc() const { return make_rsrc(p); }
  MG_DEV Slot slot(int c0, int kofs, bool ok) const {
    return Slot{(ok && c0 < cols) ? (uint32_t)(((int64_t)kofs * ld + c0) * (int64_t)sizeof(T)) : MG_OOB, kofs};
  }
  template <bool TAIL, int TBK> MG_DEV vec_t load(rsrc_t r, const Slot& s, int k0, int kend) const {
    uint32_t off = s.off;
    if constexpr (TAIL) off = (k0 + s.kofs < kend) ? off : MG_OOB;
    return bload<vec_t>(r, off, (uint32_t)((int64_t)k0 * ld * (int64_t)sizeof(T)));
  }
  MG_DEV void fix(const Slot&, int, vec_t&) const {}
};

// ---------------------------------------------------------------------------
// Epilogue
// ---------------------------------------------------------------------------
enum { ACT_NONE = 0, ACT_LRELU = 1, ACT_GELU = 2, ACT_MUL_GELU_GRAD = 3, ACT_MUL_LRELU_GRAD = 4, ACT_RSQRT_EPS = 5,
       ACT_QUICK_GELU = 6 };

// QuickGELU x * sigmoid(1.702 x) (the CLIP image tower's MLP activation)
MG_DEV float quick_gelu(float x) { return x / (1.f + __expf(-1.702f * x)); }

template <typename TO>
struct Epi {
  TO* C; int64_t ldc; int64_t gstride_c;  // per-group output offset
  float alpha;
  const float* bias; int64_t gstride_bias;  // bias[n] (+ g*gstride_bias)
  const float* scale; int scale_shift; int64_t scale_ld;  // v *= scale[(m >> shift)*ld + n]
  const float* rowscale;                      // v *= rowscale[m]
  int act; const TO* aux; int64_t ld_aux;     // aux for *_GRAD acts
  const TO* resid; int64_t ld_res;
  int accumulate;  // C += v (non-atomic)
  int atomic;      // fp32 atomic add (split-K / scatter)
  int remap_lgcin, remap_taps;  // weight-grad layout remap when remap_taps > 0
  const float* addvec; int add_shift; int64_t add_ld;  // v += addvec[(m >> add_shift)*add_ld + n]
  int rm_mode, rm_Mc, rm_lgOW, rm_lgOHW;  // rm_mode 1: stride-2 transposed-conv class rows -> NHWC rows
  TO* Cpre; int64_t ldc_pre;  // optional: store the pre-activation value too (row m, column n)
  int64_t zstride;  // split-K partial slabs: output offset zi * zstride (raw partial epilogue)
  int zi;           // this block's split index (set by gemm_kernel: blockIdx.z, or its XCD-ordered remap)
  int vec_ok;       // host-checked: 8-column vector path legal (alignment / pitches, no remap, no atomics)
  int g;
  MG_DEV void set_group(int gg) { g = gg; }
  MG_DEV int remap_row(int m) const {  // class-major (py,px,b,i,j) -> NHWC row (b, 2i+py, 2j+px)
    int cls = m / rm_Mc, rem = m - cls * rm_Mc;
    int b = rem >> rm_lgOHW, i = (rem >> rm_lgOW) & ((1 << (rm_lgOHW - rm_lgOW)) - 1), j = rem & ((1 << rm_lgOW) - 1);
    int OW2 = 2 << rm_lgOW, OH2 = 2 << (rm_lgOHW - rm_lgOW);
    return (b * OH2 + 2 * i + (cls >> 1)) * OW2 + 2 * j + (cls & 1);
  }
  // host side: decide whether the 8-column vector epilogue may be used
  bool host_vec_ok() const {
    auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    if (atomic || remap_taps > 0) return false;
    if (!al(C) || ldc % 8 || gstride_c % 8 || zstride % 8) return false;
    if (bias && (!al(bias) || gstride_bias % 4)) return false;
    if (scale && (!al(scale) || scale_ld % 4)) return false;
    if (aux && (act == ACT_MUL_GELU_GRAD || act == ACT_MUL_LRELU_GRAD) && (!al(aux) || ld_aux % 8)) return false;
    if (resid && (!al(resid) || ld_res % 8)) return false;
    if (Cpre && (!al(Cpre) || ldc_pre % 8)) return false;
    if (addvec && (!al(addvec) || add_ld % 4)) return false;
    return true;
  }
  // The one row-streamed epilogue operand -- the *_GRAD aux, else the residual -- is loaded for a whole tile
  // before the epilogue's band loop (epi_tile): its HBM latency then overlaps the accumulator staging instead of
  // stalling every 16-row band (expert gP GEMM, 131072 x 512 x 128 with GELU': 141 -> 120 us measured).
  typedef typename VecOf<TO>::type ovec_t;
  static constexpr int OV = 8 / VecOf<TO>::N;  // 16-B vectors per 8 columns: 1 (bf16), 2 (fp32)
  struct Pf { ovec_t v[OV]; };
  MG_DEV int pf_kind() const {
    return (aux && (act == ACT_MUL_GELU_GRAD || act == ACT_MUL_LRELU_GRAD)) ? 1 : (resid ? 2 : 0);
  }
  MG_DEV void pf_load(int m, int n, Pf& p) const {
    if (rm_mode == 1) m = remap_row(m);
    const TO* src = pf_kind() == 1 ? aux + (int64_t)m * ld_aux + n : resid + (int64_t)m * ld_res + n;
#pragma unroll
    for (int j = 0; j < OV; ++j) p.v[j] = *reinterpret_cast<const ovec_t*>(src + j * VecOf<TO>::N);
  }
  MG_DEV static void pf_unpack(const Pf& p, float* t) {
#pragma unroll
    for (int j = 0; j < OV; ++j)
#pragma unroll
      for (int i = 0; i < VecOf<TO>::N; ++i) {
        if constexpr (sizeof(TO) == 2) t[j * VecOf<TO>::N + i] = bf2f(p.v[j][i]);
        else t[j * VecOf<TO>::N + i] = p.v[j][i];
      }
  }
  // 8 consecutive columns n..n+7 (all < N), only when vec_ok; pf = the prefetched pf_kind() operand
  __attribute__((always_inline)) MG_DEV void vec8(int m, int n, float* v, const Pf* pf = nullptr) const {
    if (rm_mode == 1) m = remap_row(m);
    float t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= alpha;
    if (scale) {
      ld8(scale + (int64_t)(m >> scale_shift) * scale_ld + n, t);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= t[j];
    }
    if (bias) {
      ld8(bias + (int64_t)g * gstride_bias + n, t);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += t[j];
    }
    if (Cpre) st8(Cpre + (int64_t)m * ldc_pre + n, v);
    if (act == ACT_LRELU) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = lrelu(v[j]);
    } else if (act == ACT_GELU) {
      if constexpr (sizeof(TO) == 2) {
#pragma unroll
        for (int j = 0; j < 8; j += 2) {  // element pairs on packed fp32
          const f32x2_t y = gelu_fast2(f32x2_t{v[j], v[j + 1]});
          v[j] = y.x;
          v[j + 1] = y.y;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = gelu_erf(v[j]);
      }
    } else if (act == ACT_MUL_GELU_GRAD) {
      if (pf) pf_unpack(*pf, t);
      else ld8(aux + (int64_t)m * ld_aux + n, t);
      if constexpr (sizeof(TO) == 2) {
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const f32x2_t d = gelu_fast_grad2(f32x2_t{t[j], t[j + 1]});
          v[j] *= d.x;
          v[j + 1] *= d.y;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= gelu_erf_grad(t[j]);
      }
    } else if (act == ACT_MUL_LRELU_GRAD) {
      if (pf) pf_unpack(*pf, t);
      else ld8(aux + (int64_t)m * ld_aux + n, t);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= lrelu_grad(t[j]);
    } else if (act == ACT_RSQRT_EPS) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = rsqrtf(v[j] + 1e-8f);
    } else if (act == ACT_QUICK_GELU) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = quick_gelu(v[j]);
    }
    if (rowscale) {
      float r = rowscale[m];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= r;
    }
    if (addvec) {
      ld8(addvec + (int64_t)(m >> add_shift) * add_ld + n, t);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += t[j];
    }
    if (resid) {
      if (pf && pf_kind() == 2) pf_unpack(*pf, t);
      else ld8(resid + (int64_t)m * ld_res + n, t);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += t[j];
    }
    TO* c = C + (int64_t)g * gstride_c + (int64_t)m * ldc + n + (int64_t)zi * zstride;
    if (accumulate) {
      ld8(c, t);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += t[j];
    }
    st8(c, v);
  }
  MG_DEV void operator()(int m, int n, float v) const {
    if (rm_mode == 1) m = remap_row(m);  // all row lookups use the NHWC row
    v *= alpha;
    if (scale) v *= scale[(int64_t)(m >> scale_shift) * scale_ld + n];
    if (bias) v += bias[(int64_t)g * gstride_bias + n];
    if (Cpre) stf(Cpre, (int64_t)m * ldc_pre + n, v);
    if (act == ACT_LRELU) v = lrelu(v);
    else if (act == ACT_GELU) v = sizeof(TO) == 2 ? gelu_fast(v) : gelu_erf(v);
    else if (act == ACT_MUL_GELU_GRAD) {
      const float x = ldf(aux, (int64_t)m * ld_aux + n);
      v *= sizeof(TO) == 2 ? gelu_fast_grad(x) : gelu_erf_grad(x);
    }
    else if (act == ACT_MUL_LRELU_GRAD) v *= lrelu_grad(ldf(aux, (int64_t)m * ld_aux + n));
    else if (act == ACT_RSQRT_EPS) v = rsqrtf(v + 1e-8f);
    else if (act == ACT_QUICK_GELU) v = quick_gelu(v);
    if (rowscale) v *= rowscale[m];
    if (addvec) v += addvec[(int64_t)(m >> add_shift) * add_ld + n];
    if (resid) v += ldf(resid, (int64_t)m * ld_res + n);
    int64_t nn = n;
    if (remap_taps > 0) nn = (int64_t)(n & ((1 << remap_lgcin) - 1)) * remap_taps + (n >> remap_lgcin);
    int64_t idx = (int64_t)g * gstride_c + (int64_t)m * ldc + nn + (int64_t)zi * zstride;
    if (atomic) {
      atomicAdd(reinterpret_cast<float*>(C) + idx, v);
    } else {
      if (accumulate) v += ldf(C, idx);
      stf(C, idx, v);
    }
  }
};

// grouping descriptor (device tables)
struct Grouping {
  int mode;              // 0 none, 1 grouped-M (rows), 2 grouped-K (reduction rows)
  int ngroups;
  const int* row_off;    // [ngroups+1] row (mode 1) / reduction (mode 2) offsets
  const int* tile_off;   // mode 1: [ngroups+1] prefix of ceil(rows_g / BM)
  int rows_per_group;    // mode 3: ngroups equal groups of this many rows (no tables)
  int swz;               // mode 0: XCD-aware tile order (1: every launch, 2: split-K launches only)
  int sub_shift;         // mode 1: the tables count tiles of (BM << sub_shift) rows; block x = table tile << sub_shift
                         // + sub-tile (64-row tiles over the dispatch's 128-row tile table)
};

// ---------------------------------------------------------------------------
// Kernel
// ---------------------------------------------------------------------------
// LDS images.  KC operand: [rows][BK + PADK] (k contiguous), fragments read with ds_read_b128 (bf16)
// or ds_read_b32 (fp32).  MC operand: [BK][rows + PADM] (rows contiguous, stored straight from the
// coalesced global vectors) and, for bf16, read with two ds_read_b64_tr_b16 per fragment (the hardware
// transpose delivers 4 k-rows of one column per lane).  The MC row pitch is an odd multiple of 16
// dwords and columns are XOR-swizzled by 16 elements on odd k-octets, so both halves of a wave's
// transposed read (k-rows 8g..8g+3 for lane groups g = 0, 1) hit 8 distinct bank octets.
template <typename T> struct Tile;
template <> struct Tile<bf16_t> { static constexpr int BK = 64, PADK = 0, PADM = 32; };
template <> struct Tile<float> { static constexpr int BK = 32, PADK = 4, PADM = 16; };

// K step of a GEMM instantiation: X3 (fp32 operands multiplied as split bf16, hi*hi + hi*lo + lo*hi) stages its
// tiles as bf16 images, so it takes the bf16 step
// MG_BK_SMALL: the K step of bf16 tiles of at most 64 x 64 outputs (A/B build switch; 64 = the common step).  A
// 128-deep step doubles the bytes each of those latency-bound blocks keeps in flight per barrier.
#ifndef MG_BK_SMALL
#define MG_BK_SMALL 64
#endif
// MG_X3_BK: the K step of the split-bf16 fp32 tiles (64 x 64 only; the small-M prefix / demodulation GEMMs are
// serial chains of K steps on few tiles, so a deeper step halves their chain; 64 = the bf16 step)
#ifndef MG_X3_BK
#define MG_X3_BK 64
#endif
template <typename T, bool X3, int BM = 128, int BN = 128> constexpr int tile_bk() {
  return X3 ? (BM * BN <= 64 * 64 ? MG_X3_BK : Tile<bf16_t>::BK)
            : (sizeof(T) == 2 && BM * BN <= 64 * 64) ? MG_BK_SMALL : Tile<T>::BK;
}
// the largest K step any bf16 tile uses (the implicit-conv loaders' "one tap per K step" test needs Cin >= it)
template <typename T> constexpr int max_tile_bk() { return tile_bk<T, false, 64, 64>() > Tile<T>::BK ? tile_bk<T, false, 64, 64>() : Tile<T>::BK; }

template <typename T> MG_DEV constexpr int mc_swz(int k) { return sizeof(T) == 2 ? ((k >> 3) & 1) << 4 : 0; }
// KC image element offset of (row r, k) for bf16: 16-B chunk (k / 8) stored at chunk (k / 8) ^ (r & 7)
// of an unpadded 128-B row -- conflict-free ds_read_b128 fragment reads and ds_write_b128 stores.
template <typename T> MG_DEV constexpr int kc_off(int r, int k, int ldk) {
  // (a 256-B row -- a 128-deep step -- swizzles its 16 chunks by row & 15: rows 256 B apart share their banks)
  return sizeof(T) == 2 ? r * ldk + ((((k >> 3) ^ (r & ((ldk >> 3) - 1) & 15))) << 3) + (k & 7) : r * ldk + k;
}

typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

// A/B fragment of v_mfma_f32_16x16x32_bf16 from an MC image: lane (g = lane>>4, i = lane&15) gets
// column c0+i of k-rows kr0+8g .. kr0+8g+7.
MG_DEV bf16x8_t mc_frag_bf16(const bf16_t* img, int ld, int kr0, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int k = kr0 + 8 * g + q;
  const int col = (c0 ^ mc_swz<bf16_t>(k)) + 4 * p;
  auto base = (__attribute__((address_space(3))) char*)(img);
  s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(base + ((int64_t)k * ld + col) * 2));
  s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(base + ((int64_t)(k + 4) * ld + col) * 2));
  u16x8_t r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return __builtin_bit_cast(bf16x8_t, r);
}

// MG_GLDS_MC images (64 columns = 128-B rows, unpadded): 16-B chunk c of k-row k stored at chunk c ^ swz64(k).  Rows
// alternate 32-bank halves; the four same-parity rows of one 32-lane half of a transposed read (k = 8g + q) get
// distinct chunk pairs.
// 128 columns (256-B rows, every row on the same banks): the eight rows of a 32-lane half get distinct chunk pairs
// of the 16.
MG_DEV constexpr int swz64(int k) { return (((k >> 1) & 1) | (((k >> 3) & 1) << 1)) << 1; }
MG_DEV constexpr int swz128(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 1; }
template <int COLS> MG_DEV constexpr int swzmc(int k) { return COLS == 64 ? swz64(k) : swz128(k); }
template <int COLS>
MG_DEV bf16x8_t mc_frag_glds(const bf16_t* img, int kr0, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int k = kr0 + 8 * g + q;
  const int ch = (c0 >> 3) + (p >> 1), sub = (p & 1) * 8;
  auto base = (__attribute__((address_space(3))) char*)(img);
  s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4_t*)(base + k * (COLS * 2) + ((ch ^ swzmc<COLS>(k)) << 4) + sub));
  s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4_t*)(base + (k + 4) * (COLS * 2) + ((ch ^ swzmc<COLS>(k + 4)) << 4) + sub));
  u16x8_t r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return __builtin_bit_cast(bf16x8_t, r);
}

// Epilogue of one output tile: stage one 16-row band of each wave's accumulators through LDS (`smem`, at
// least 4 * 16 * (BN/2 + 4) floats), then a plain (non-unrolled) loop applies the fused epilogue with
// consecutive lanes on consecutive columns.  Static indexing keeps acc in registers; the loop keeps the
// inlined epilogue code small.  Waves are arranged 2x2, each owning a (BM/2)x(BN/2) block of 16x16 fragments
// in the MFMA C/D layout (dtype-independent on gfx950).
template <int BM, int BN, class EP, bool PF = false>
MG_DEV void epi_tile(const f32x4_t (&acc)[BM / 32][BN / 32], void* smem, const EP& ep, int m0, int n0, int Mloc,
                     int N, int mrow_base) {
  constexpr int WM = BM / 2, WN = BN / 2, FM = WM / 16, FN = WN / 16;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int fr = lane & 15, fq = lane >> 4;
  constexpr int CSP = WN + 4;  // staging pitch in floats (16-B aligned rows)
  float* cs = reinterpret_cast<float*>(smem) + wid * 16 * CSP;
  // vector path with a streamed operand: every band's loads issued up front (NE 8-column groups per lane)
  // (only where the prefetched tile fits in 32 VGPRs: 64x64 / 128x32 tiles, 128x128 bf16 -- wider tiles spill)
  constexpr int NE = (2 * WN + 63) / 64;
  // PF: instantiated for the expert GEMMs only (turned on for every tile it cost the step 0.18 ms: code size /
  // register allocation of the other kernels); bf16 operands only (fp32 ones spilled)
  constexpr bool kPf = PF && MG_EPI_PREFETCH && EP::OV == 1 && FM * NE * 4 <= 32;
  const bool pfp = kPf && ep.vec_ok && ep.pf_kind() != 0;
  typename EP::Pf pf[kPf ? FM : 1][kPf ? NE : 1];
  if constexpr (kPf) if (pfp) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int t = 0; t < NE; ++t) {
        const int e = lane + 64 * t;
        const int rr = e / (WN / 8), cc = (e - rr * (WN / 8)) * 8;
        const int m = m0 + wm * WM + i * 16 + rr, n = n0 + wn * WN + cc;
        if (e < 2 * WN && m < Mloc && n + 8 <= N) ep.pf_load(mrow_base + m, n, pf[i][t]);
      }
  }
  // each wave stages through its own LDS band: one block barrier retires the K loop's reads of the
  // tiles, after that a wave only orders its own LDS writes and reads (wave-scope fence)
  __syncthreads();
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    if (MG_EPI_BLOCK_SYNC) __syncthreads();
    else { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); __builtin_amdgcn_wave_barrier(); }
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) cs[(fq * 4 + r) * CSP + j * 16 + fr] = acc[i][j][r];
    if (MG_EPI_BLOCK_SYNC) __syncthreads();
    else { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); __builtin_amdgcn_wave_barrier(); }
    const int mb = m0 + wm * WM + i * 16, nb = n0 + wn * WN;
    if (kPf && pfp) {
#pragma unroll
      for (int t = 0; t < (kPf ? NE : 0); ++t) {
        const int e = lane + 64 * t;
        const int rr = e / (WN / 8), cc = (e - rr * (WN / 8)) * 8;
        const int m = mb + rr, n = nb + cc;
        if (e >= 2 * WN || m >= Mloc) continue;
        const float* src = cs + rr * CSP + cc;
        if (n + 8 <= N) {
          float v[8];
          f32x4_t a = *reinterpret_cast<const f32x4_t*>(src), b = *reinterpret_cast<const f32x4_t*>(src + 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[j + 4] = b[j]; }
          ep.vec8(mrow_base + m, n, v, &pf[kPf ? i : 0][kPf ? t : 0]);
        } else {
          for (int j = 0; j < 8 && n + j < N; ++j) ep(mrow_base + m, n + j, src[j]);
        }
      }
    } else if (ep.vec_ok) {
      // 8 consecutive columns per lane: vector loads of the epilogue operands, one 16-B store (bf16)
#pragma unroll 1
      for (int e = lane; e < 2 * WN; e += 64) {
        int rr = e / (WN / 8), cc = (e - (e / (WN / 8)) * (WN / 8)) * 8;
        int m = mb + rr, n = nb + cc;
        if (m >= Mloc) continue;
        const float* src = cs + rr * CSP + cc;
        if (n + 8 <= N) {
          float v[8];
          f32x4_t a = *reinterpret_cast<const f32x4_t*>(src), b = *reinterpret_cast<const f32x4_t*>(src + 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[j + 4] = b[j]; }
          ep.vec8(mrow_base + m, n, v);
        } else {
          for (int j = 0; j < 8 && n + j < N; ++j) ep(mrow_base + m, n + j, src[j]);
        }
      }
    } else {
#pragma unroll 1
      for (int e = lane; e < 16 * WN; e += 64) {
        int rr = e / WN, cc = e - (e / WN) * WN;
        int m = mb + rr, n = nb + cc;
        if (m < Mloc && n < N) ep(mrow_base + m, n, cs[rr * CSP + cc]);
      }
    }
  }
}

// One output tile: C[m0.., n0..] of rows [mrow_base, mrow_base + Mloc) over k in [kbeg, kend).
template <typename T, int BM, int BN, bool A_KC, bool B_KC, class AL, class BL, class EP, bool X3 = false,
          bool PF = false>
MG_DEV void gemm_tile(const AL& A, const BL& B, const EP& ep, int m0, int n0, int Mloc, int N, int kbeg, int kend,
                      int mrow_base) {
  static_assert(!X3 || std::is_same<T, float>::value, "split-bf16 staging takes fp32 operands");
  constexpr int VEC = VecOf<T>::N;
  typedef typename VecOf<T>::type vec_t;
  // LT: element type of the LDS images (X3: bf16 hi / lo images of the fp32 operands, bf16 tile geometry)
  typedef typename std::conditional<X3, bf16_t, T>::type LT;
  constexpr int TBK = tile_bk<T, X3, BM, BN>();
  constexpr int LDK = TBK + Tile<LT>::PADK;
  // LDS-DMA staging of two MC operands (MG_GLDS_MC): unpadded, source-swizzled images
  constexpr bool GMC = [] {
    if constexpr (!A_KC && !B_KC)
      return MG_GLDS_MC && !X3 && sizeof(T) == 2 && BM == BN && (BM == 64 || BM == 128) && TBK == 64 &&
             has_gldsmc<AL>::value && has_gldsmc<BL>::value;
    else return false;
  }();
  constexpr int PADMC = GMC ? 0 : Tile<LT>::PADM;
  constexpr int LDA = A_KC ? LDK : BM + PADMC;
  constexpr int LDB = B_KC ? LDK : BN + PADMC;
  constexpr int A_ELEMS = A_KC ? BM * LDK : TBK * LDA;
  constexpr int B_ELEMS = B_KC ? BN * LDK : TBK * LDB;
  constexpr int WM = BM / 2, WN = BN / 2, FM = WM / 16, FN = WN / 16;
  // per-thread vector counts
  constexpr int A_VPT = BM * TBK / VEC / NTHREADS;
  constexpr int B_VPT = BN * TBK / VEC / NTHREADS;
  static_assert(A_VPT >= 1 && B_VPT >= 1, "tile too small for 256 threads");
  // LDS: NBUF stages of (A tile, B tile), reused by the epilogue to stage accumulators.  Double
  // buffering (with a second register stage) when two stages fit the 64 KiB static limit.
  // X3: (A_hi, A_lo, B_hi, B_lo) images in one stage
  constexpr int STAGE = (X3 ? 2 : 1) * (A_ELEMS + B_ELEMS);
  // LDS-DMA staging (bf16, both operands k-contiguous without transforms): two LDS stages, no registers
  constexpr bool GLDS_SEL = [] {
    if constexpr (A_KC && B_KC) return MG_GLDS || (MG_GLDS_CONV && AL::kConv && BM * BN <= 64 * 64);
    else return false;
  }();
  constexpr int GSTAGES = MG_GLDS ? 2 : MG_GLDS_STAGES;
  constexpr bool GLDS = [] {
    if constexpr (A_KC && B_KC)
      return GLDS_SEL && !X3 && sizeof(T) == 2 && AL::kGlds && BL::kGlds && GSTAGES * STAGE * (int)sizeof(T) <= 65536;
    else return GMC;
  }();
  constexpr int NBUF = GLDS ? (GSTAGES * STAGE * (int)sizeof(LT) <= 65536 ? GSTAGES : 2)
                            : ((!X3 && 2 * STAGE * (int)sizeof(T) <= 65536 && BM * BN <= MG_DB_MAX_TILE) ? 2 : 1);
  constexpr bool SB2 = NBUF == 1 && !X3 && BM * BN <= MG_SB2_MAX_TILE;
  constexpr int NS = NBUF == 2 ? MG_NSTAGE : (SB2 ? 2 : 1);
  __shared__ __attribute__((aligned(16))) LT smem[NBUF * STAGE];
  static_assert(4 * 16 * (WN + 4) * 4 <= (int)sizeof(LT) * STAGE, "epilogue staging does not fit");

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  // in grouped-M mode the A loader / epilogue see absolute rows; clamp via Mloc
  const int mlimit = mrow_base + Mloc;

  // ---- per-thread load slots ----
  typename AL::Slot as_[A_VPT];
  typename BL::Slot bs_[B_VPT];
  int a_r[A_VPT], a_k[A_VPT], b_r[B_VPT], b_k[B_VPT];
  // GLDS: wave-instruction i of wave w fills LDS rows (4i + w) * 8 .. +8 (1 KiB, lane order); lane L takes
  // row +(L >> 3) and stores physical chunk L & 7, so it loads logical chunk (L & 7) ^ (row & 7) (the swizzle
  // moves to the source address; fragment reads use kc_off unchanged).
#pragma unroll
  for (int i = 0; i < A_VPT; ++i) {
    int v = tid + i * NTHREADS;
    // GMC: wave-instruction i of wave w fills the 1 KiB of k-rows (4i + w) * R .. + R of the [TBK][BM] image (R = 8 /
    // 4 rows of 64 / 128 columns); lane L takes k-row + L / (BM / 8), physical 16-B chunk L % (BM / 8), so it loads
    // column chunk (L % (BM / 8)) ^ swzmc(k-row)
    if constexpr (GMC) {
      a_k[i] = (i * 4 + wid) * (64 / (BM / 8)) + lane / (BM / 8);
      a_r[i] = 8 * ((lane % (BM / 8)) ^ swzmc<BM>(a_k[i]));
    }
    else if constexpr (GLDS) { a_r[i] = (i * 4 + wid) * 8 + (lane >> 3); a_k[i] = 8 * ((lane & 7) ^ ((lane >> 3) & 7)); }
    else if constexpr (A_KC) { a_r[i] = v / (TBK / VEC); a_k[i] = (v % (TBK / VEC)) * VEC; }
    else { a_k[i] = v / (BM / VEC); a_r[i] = (v % (BM / VEC)) * VEC; }
    const int r = mrow_base + m0 + a_r[i];
    as_[i] = A.slot(r, a_k[i], r < mlimit);
  }
#pragma unroll
  for (int i = 0; i < B_VPT; ++i) {
    int v = tid + i * NTHREADS;
    if constexpr (GMC) {
      b_k[i] = (i * 4 + wid) * (64 / (BN / 8)) + lane / (BN / 8);
      b_r[i] = 8 * ((lane % (BN / 8)) ^ swzmc<BN>(b_k[i]));
    }
    else if constexpr (GLDS) { b_r[i] = (i * 4 + wid) * 8 + (lane >> 3); b_k[i] = 8 * ((lane & 7) ^ ((lane >> 3) & 7)); }
    else if constexpr (B_KC) { b_r[i] = v / (TBK / VEC); b_k[i] = (v % (TBK / VEC)) * VEC; }
    else { b_k[i] = v / (BN / VEC); b_r[i] = (v % (BN / VEC)) * VEC; }
    bs_[i] = B.slot(n0 + b_r[i], b_k[i], true);
  }
  const rsrc_t rA = A.rsrc(), rB = B.rsrc();
  i32x4_t dA{}, dB{};  // (GMC: raw descriptors for the asm DMAs)
  if constexpr (GMC) {
    dA = A.desc();
    dB = B.desc();
  }

  // NS register stages: the loads of K step t + NS are issued while step t is multiplied
  vec_t ra[NS][A_VPT], rb[NS][B_VPT];
  // issue the buffer loads of K step k0 into register stage R (TAIL: the step reaches past kend)
  auto gload = [&](auto R, int k0, auto tail) {
    constexpr int r = decltype(R)::value;
    constexpr bool TL = decltype(tail)::value;
#pragma unroll
    for (int i = 0; i < A_VPT; ++i) ra[r][i] = A.template load<TL, TBK>(rA, as_[i], k0, kend);
#pragma unroll
    for (int i = 0; i < B_VPT; ++i) rb[r][i] = B.template load<TL, TBK>(rB, bs_[i], k0, kend);
  };
  auto gload_any = [&](auto R, int k0) {
    if (k0 + TBK <= kend) gload(R, k0, std::false_type{});
    else gload(R, k0, std::true_type{});
  };
  // register stage R (K step k0) -> LDS buffer (As, Bs)
  auto sstore = [&](auto R, int k0, LT* As, LT* Bs) {
    constexpr int r = decltype(R)::value;
    if constexpr (X3) {
      // fp32 vector -> bf16 hi = rn(v), lo = rn(v - hi); the 4 elements land as 8-byte runs in the hi and lo
      // images (KC: half a 16-B chunk of the swizzled row; MC: 4 columns, the 16-column swizzle keeps them whole)
      auto split_store = [&](const f32x4_t& v, LT* hi_img, LT* lo_img, int off) {
        typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
        u16x4 h, l;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          h[j] = f2bf(v[j]);
          l[j] = f2bf(v[j] - bf2f(h[j]));
        }
        *reinterpret_cast<u16x4*>(&hi_img[off]) = h;
        *reinterpret_cast<u16x4*>(&lo_img[off]) = l;
      };
#pragma unroll
      for (int i = 0; i < A_VPT; ++i) {
        vec_t v = ra[r][i];
        A.fix(as_[i], k0, v);
        const int off = A_KC ? kc_off<LT>(a_r[i], a_k[i], LDK) : a_k[i] * LDA + (a_r[i] ^ mc_swz<LT>(a_k[i]));
        split_store(v, As, As + A_ELEMS, off);
      }
#pragma unroll
      for (int i = 0; i < B_VPT; ++i) {
        vec_t v = rb[r][i];
        B.fix(bs_[i], k0, v);
        const int off = B_KC ? kc_off<LT>(b_r[i], b_k[i], LDK) : b_k[i] * LDB + (b_r[i] ^ mc_swz<LT>(b_k[i]));
        split_store(v, Bs, Bs + B_ELEMS, off);
      }
      return;
    } else {
#pragma unroll
    for (int i = 0; i < A_VPT; ++i) {
      vec_t v = ra[r][i];
      A.fix(as_[i], k0, v);
      if constexpr (A_KC) *reinterpret_cast<vec_t*>(&As[kc_off<T>(a_r[i], a_k[i], LDK)]) = v;
      else *reinterpret_cast<vec_t*>(&As[a_k[i] * LDA + (a_r[i] ^ mc_swz<T>(a_k[i]))]) = v;
    }
#pragma unroll
    for (int i = 0; i < B_VPT; ++i) {
      vec_t v = rb[r][i];
      B.fix(bs_[i], k0, v);
      if constexpr (B_KC) *reinterpret_cast<vec_t*>(&Bs[kc_off<T>(b_r[i], b_k[i], LDK)]) = v;
      else *reinterpret_cast<vec_t*>(&Bs[b_k[i] * LDB + (b_r[i] ^ mc_swz<T>(b_k[i]))]) = v;
    }
    }
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  // one K step of MFMAs from the LDS buffer (As, Bs)
  auto compute = [&](const LT* As, const LT* Bs) {
    if constexpr (X3) {
      // three bf16 products per fragment pair: hi*hi + hi*lo + lo*hi (the lo*lo term is below fp32 rounding of
      // the sum); images: As = A_hi, As + A_ELEMS = A_lo, Bs = B_hi, Bs + B_ELEMS = B_lo
      auto frag = [&](const LT* img, int ld, bool kc, int row0, int kk) {
        if (kc) return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u16x8_t*>(&img[kc_off<LT>(row0 + fr, kk * 32 + fq * 8, ld)]));
        return mc_frag_bf16(img, ld, kk * 32, row0, lane);
      };
#pragma unroll
      for (int kk = 0; kk < TBK / 32; ++kk) {
        bf16x8_t ah[FM], al[FM], bh[FN], bl[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          ah[i] = frag(As, LDA, A_KC, wm * WM + i * 16, kk);
          al[i] = frag(As + A_ELEMS, LDA, A_KC, wm * WM + i * 16, kk);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          bh[j] = frag(Bs, LDB, B_KC, wn * WN + j * 16, kk);
          bl[j] = frag(Bs + B_ELEMS, LDB, B_KC, wn * WN + j * 16, kk);
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
          }
      }
    } else if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int kk = 0; kk < TBK / 32; ++kk) {
        bf16x8_t af[FM], bfv[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          if constexpr (A_KC)
            af[i] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u16x8_t*>(&As[kc_off<T>(wm * WM + i * 16 + fr, kk * 32 + fq * 8, LDK)]));
          else if constexpr (GMC)
            af[i] = mc_frag_glds<BM>(As, kk * 32, wm * WM + i * 16, lane);
          else
            af[i] = mc_frag_bf16(As, LDA, kk * 32, wm * WM + i * 16, lane);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          if constexpr (B_KC)
            bfv[j] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u16x8_t*>(&Bs[kc_off<T>(wn * WN + j * 16 + fr, kk * 32 + fq * 8, LDK)]));
          else if constexpr (GMC)
            bfv[j] = mc_frag_glds<BN>(Bs, kk * 32, wn * WN + j * 16, lane);
          else
            bfv[j] = mc_frag_bf16(Bs, LDB, kk * 32, wn * WN + j * 16, lane);
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfv[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < TBK / 4; ++kk) {
        float af[FM], bfv[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
          af[i] = A_KC ? As[(wm * WM + i * 16 + fr) * LDK + kk * 4 + fq] : As[(kk * 4 + fq) * LDA + wm * WM + i * 16 + fr];
#pragma unroll
        for (int j = 0; j < FN; ++j)
          bfv[j] = B_KC ? Bs[(wn * WN + j * 16 + fr) * LDK + kk * 4 + fq] : Bs[(kk * 4 + fq) * LDB + wn * WN + j * 16 + fr];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfv[j], acc[i][j], 0, 0, 0);
      }
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;

  if constexpr (GLDS) {
    // LDS-DMA, two stages: step t+1's loads are issued before step t is multiplied; a counted vmcnt
    // retires only step t's (issued earlier), a raw barrier publishes them, and a second barrier keeps
    // step t+2's DMA from overwriting the buffer while another wave still reads it.
    static_assert((NBUF - 1) * (A_VPT + B_VPT) < 64, "vmcnt range");
    static_assert(NBUF == 2 || NBUF == 3, "LDS-DMA pipeline: 2 or 3 stages");
    auto issue = [&](int k0, LT* buf) {
      if constexpr (GMC) {
        if (k0 + TBK <= kend) {
#pragma unroll
          for (int i = 0; i < A_VPT; ++i) A.template gldsmc<false, TBK>(dA, as_[i], k0, kend, buf + (i * 4 + wid) * 512);
#pragma unroll
          for (int i = 0; i < B_VPT; ++i)
            B.template gldsmc<false, TBK>(dB, bs_[i], k0, kend, buf + A_ELEMS + (i * 4 + wid) * 512);
        } else {
#pragma unroll
          for (int i = 0; i < A_VPT; ++i) A.template gldsmc<true, TBK>(dA, as_[i], k0, kend, buf + (i * 4 + wid) * 512);
#pragma unroll
          for (int i = 0; i < B_VPT; ++i)
            B.template gldsmc<true, TBK>(dB, bs_[i], k0, kend, buf + A_ELEMS + (i * 4 + wid) * 512);
        }
        return;
      } else if (k0 + TBK <= kend) {
#pragma unroll
        for (int i = 0; i < A_VPT; ++i) A.template glds<false, TBK>(rA, as_[i], k0, kend, buf + (i * 4 + wid) * 8 * LDK);
#pragma unroll
        for (int i = 0; i < B_VPT; ++i)
          B.template glds<false, TBK>(rB, bs_[i], k0, kend, buf + A_ELEMS + (i * 4 + wid) * 8 * LDK);
      } else {
#pragma unroll
        for (int i = 0; i < A_VPT; ++i) A.template glds<true, TBK>(rA, as_[i], k0, kend, buf + (i * 4 + wid) * 8 * LDK);
#pragma unroll
        for (int i = 0; i < B_VPT; ++i)
          B.template glds<true, TBK>(rB, bs_[i], k0, kend, buf + A_ELEMS + (i * 4 + wid) * 8 * LDK);
      }
    };
    const int nsteps = kend > kbeg ? (kend - kbeg + TBK - 1) / TBK : 0;
    constexpr int PER = A_VPT + B_VPT;  // DMA instructions per step
    if constexpr (NBUF == 3) {
      // three stages, ONE barrier per step: step t + 2 is issued after the barrier of step t, into the stage step
      // t - 1 read (every wave finished step t - 1 before arriving at that barrier); before it, a counted vmcnt
      // retires this wave's DMA of step t (step t + 1's may stay in flight)
      if (nsteps > 0) issue(kbeg, smem);
      if (nsteps > 1) issue(kbeg + TBK, smem + STAGE);
      for (int t = 0; t < nsteps; ++t) {
        LT* cur = smem + (t % 3) * STAGE;
        if (t + 1 < nsteps) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of step t - 1 have landed (WAR)
        __builtin_amdgcn_s_barrier();
        if (t + 2 < nsteps) issue(kbeg + (t + 2) * TBK, smem + ((t + 2) % 3) * STAGE);
        compute(cur, cur + A_ELEMS);
      }
    } else {
    // two stages: step t + 1 is in flight while step t is multiplied
#pragma unroll
    for (int p = 0; p < NBUF - 1; ++p)
      if (p < nsteps) issue(kbeg + p * TBK, smem + p * STAGE);
    for (int t = 0; t < nsteps; ++t) {
      LT* cur = smem + (t % NBUF) * STAGE;
      const int ahead = t + NBUF - 1;
      if (ahead < nsteps) {
        issue(kbeg + ahead * TBK, smem + (ahead % NBUF) * STAGE);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NBUF - 1) * PER) : "memory");
      } else if (NBUF > 2 && nsteps - 1 - t == 1) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      compute(cur, cur + A_ELEMS);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of cur have landed (WAR)
      __builtin_amdgcn_s_barrier();
    }
    }
  } else if constexpr (NBUF == 2) {
    // Two LDS buffers, one barrier per K step.  Step t multiplies LDS[t & 1], then writes the register
    // stage holding step t+1 into LDS[(t+1) & 1] (last read by step t-1, whose closing barrier freed it)
    // and refills that stage with step t+1+NS.
    if (kbeg < kend) {
      gload_any(I0{}, kbeg);
      if constexpr (NS == 2)
        if (kbeg + TBK < kend) gload_any(I1{}, kbeg + TBK);
      sstore(I0{}, kbeg, smem, smem + A_ELEMS);
      if (kbeg + NS * TBK < kend) gload_any(I0{}, kbeg + NS * TBK);
      __syncthreads();
    }
    // one multiply per loop body (so the accumulators keep their registers); with two register stages
    // the parity of the stage being written back is a uniform branch between two static-index copies
    const int nsteps = kend > kbeg ? (kend - kbeg + TBK - 1) / TBK : 0;
    for (int t = 0; t < nsteps; ++t) {
      const int k0 = kbeg + t * TBK;
      const LT* cur = smem + (t & 1) * STAGE;
      compute(cur, cur + A_ELEMS);
      const int kn = k0 + TBK;
      if (kn < kend) {
        LT* nxt = smem + ((t + 1) & 1) * STAGE;
        if (NS == 1 || (t & 1)) {
          sstore(I0{}, kn, nxt, nxt + A_ELEMS);
          if (kn + NS * TBK < kend) gload_any(I0{}, kn + NS * TBK);
        } else if constexpr (NS == 2) {
          sstore(I1{}, kn, nxt, nxt + A_ELEMS);
          if (kn + NS * TBK < kend) gload_any(I1{}, kn + NS * TBK);
        }
      }
      __syncthreads();
    }
  } else if constexpr (SB2) {
    // one LDS buffer, two register stages: the loads of step t+2 are issued right after step t's registers went
    // to LDS, so two multiplies (not one) cover each load's latency.  Straight-line body over two K steps with
    // tail-safe loads throughout (past kend they read zeros), so no branch splits the load stream and the
    // compiler's vmcnt waits count only the older stage.
    LT* const As = smem;
    LT* const Bs = smem + (X3 ? 2 : 1) * A_ELEMS;
    using TT = std::true_type;
    // scheduling barriers pin the issue order (stage 0 before stage 1, each reload before its multiply) so on
    // both paths into the loop head stage 0 is the older stage and its wait is vmcnt(#stage-1 loads), not 0
    gload(I0{}, kbeg, TT{});
    __builtin_amdgcn_sched_barrier(0);
    gload(I1{}, kbeg + TBK, TT{});
    __builtin_amdgcn_sched_barrier(0);
    // whole pairs of K steps in the loop (one exit: the waits at its head see one load order), an odd last
    // step after it
    int k0 = kbeg;
    for (; k0 + TBK < kend; k0 += 2 * TBK) {
      __syncthreads();
      sstore(I0{}, k0, As, Bs);
      __syncthreads();
      gload(I0{}, k0 + 2 * TBK, TT{});
      __builtin_amdgcn_sched_barrier(0);
      compute(As, Bs);
      __syncthreads();
      sstore(I1{}, k0 + TBK, As, Bs);
      __syncthreads();
      gload(I1{}, k0 + 3 * TBK, TT{});
      __builtin_amdgcn_sched_barrier(0);
      compute(As, Bs);
    }
    if (k0 < kend) {
      __syncthreads();
      sstore(I0{}, k0, As, Bs);
      __syncthreads();
      compute(As, Bs);
    }
  } else {
    // one LDS buffer, one register stage: store, barrier, prefetch the next step, multiply
    LT* const As = smem;
    LT* const Bs = smem + (X3 ? 2 : 1) * A_ELEMS;
    if (kbeg < kend) gload_any(I0{}, kbeg);
    for (int k0 = kbeg; k0 < kend; k0 += TBK) {
      __syncthreads();
      sstore(I0{}, k0, As, Bs);
      __syncthreads();
      if (k0 + TBK < kend) gload_any(I0{}, k0 + TBK);
      if (MG_SETPRIO) __builtin_amdgcn_s_setprio(1);  // the multiply phase first in the SIMD's issue arbitration
      compute(As, Bs);
      if (MG_SETPRIO) __builtin_amdgcn_s_setprio(0);
    }
  }

  epi_tile<BM, BN, EP, PF>(acc, smem, ep, m0, n0, Mloc, N, mrow_base);
}


// TAG only names the instantiation (1 = MoE expert GEMMs) so profiles can attribute its dispatches.
template <typename T, int BM, int BN, bool A_KC, bool B_KC, class AL, class BL, class EP, int TAG = 0, bool X3 = false>
__global__ __launch_bounds__(NTHREADS) void gemm_kernel(AL A, BL B, EP ep, int M, int N, int K, int kchunk, Grouping grp) {
  constexpr int TBK = tile_bk<T, X3, BM, BN>();
  // ---- resolve tile / group ----
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (((grp.mode == 0 || grp.mode == 1) && grp.swz && (grp.swz == 1 || gridDim.z > 1)) || (grp.mode == 2 && grp.swz)) {
    // XCD-aware tile order: workgroups are dispatched round-robin over the 8 XCDs by linear id, so blocks that
    // share an XCD (linear id % 8) take a contiguous run of (split, m-tile, n-tile) work items, n fastest --
    // all tiles of one K split (which read the same operand rows: a split-K weight gradient re-reads its
    // operands once per output tile) and neighbouring m-tiles then meet in the same L2.
    const int gx = gridDim.x, gy = gridDim.y, gxy = gx * gy, nb = gxy * gridDim.z;
    const int bid = bx + by * gx + bz * gxy;
    const int xcd = bid & 7, q = nb >> 3, r = nb & 7;
    const int w = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    bz = w / gxy;
    const int rem = w - bz * gxy;
    bx = rem / gy;
    by = rem - bx * gy;
  }
  int m0 = bx * BM, n0 = by * BN;
  ep.zi = bz;
  int mrow_base = 0;  // global row offset of this group (mode 1)
  int Mloc = M;
  int kbeg = bz * kchunk, kend = min(K, kbeg + kchunk);
  int g = 0;
  if (grp.mode == 1) {
    int t = bx >> grp.sub_shift;
    g = -1;
    for (int i = 0; i < grp.ngroups; ++i)
      if (t >= grp.tile_off[i] && t < grp.tile_off[i + 1]) { g = i; break; }
    if (g < 0) return;
    mrow_base = grp.row_off[g];
    Mloc = grp.row_off[g + 1] - mrow_base;
    m0 = (t - grp.tile_off[g]) * (BM << grp.sub_shift) + (bx & ((1 << grp.sub_shift) - 1)) * BM;
    if (m0 >= Mloc) return;  // a sub-tile past the group's last row
  } else if (grp.mode == 3) {
    int tpg = (grp.rows_per_group + BM - 1) / BM;
    g = blockIdx.x / tpg;
    if (g >= grp.ngroups) return;
    mrow_base = g * grp.rows_per_group;
    Mloc = grp.rows_per_group;
    m0 = (blockIdx.x - g * tpg) * BM;
  } else if (grp.mode == 2) {
    int splits = gridDim.z / grp.ngroups;
    g = bz / splits;  // (bz: the XCD-ordered z index, so the tiles of one group's K split share an XCD's L2)
    int s = bz - g * splits;
    int r0 = grp.row_off[g], r1 = grp.row_off[g + 1];
    int per = ((r1 - r0 + splits - 1) / splits + TBK - 1) / TBK * TBK;
    kbeg = r0 + s * per;
    kend = min(r1, kbeg + per);
    ep.zi = s;  // split-K partial slabs: slab s of group g (zstride = one slab of every group)
    if (kbeg >= kend) {
      if (ep.zstride == 0) return;  // accumulating epilogue: nothing to add
      kend = kbeg;                  // a slab is written whole: an empty split stores its zeros
    }
  }
  A.set_group(g);
  B.set_group(g);
  ep.set_group(g);
  gemm_tile<T, BM, BN, A_KC, B_KC, AL, BL, EP, X3, TAG == 1>(A, B, ep, m0, n0, Mloc, N, kbeg, kend, mrow_base);
}

// ---------------------------------------------------------------------------
// Batched independent small GEMMs: up to MG_BATCH_MAX problems of one dtype / orientation per launch,
// described in the kernel arguments; block -> (problem, tile) through a tile prefix.
// ---------------------------------------------------------------------------
constexpr int MG_BATCH_MAX = 8;
template <typename TO, class AL, class BL>
struct BatchArgs {
  AL a[MG_BATCH_MAX];
  BL b[MG_BATCH_MAX];
  Epi<TO> e[MG_BATCH_MAX];
  int M[MG_BATCH_MAX], N[MG_BATCH_MAX], K[MG_BATCH_MAX], tiles_n[MG_BATCH_MAX], tile_off[MG_BATCH_MAX + 1];
  int n;
  // split-K slabs (SPLIT launches, grid.y = the split count): problem p's split s covers K rows
  // [s * kchunk[p], +kchunk[p]) and writes its raw fp32 partial to ws + ws_off[p] + s * M[p] * N[p]
  int kchunk[MG_BATCH_MAX];
  int64_t ws_off[MG_BATCH_MAX];
  float* ws;
};

template <typename T, bool A_KC, bool B_KC, class AL, class BL, typename TO, bool X3 = false, bool SPLIT = false>
__global__ __launch_bounds__(NTHREADS) void gemm_batch_kernel(BatchArgs<TO, AL, BL> args) {
  const int t = blockIdx.x;
  int p = 0;
  while (p + 1 < args.n && t >= args.tile_off[p + 1]) ++p;
  const int lt = t - args.tile_off[p];
  const int tm = lt / args.tiles_n[p], tn = lt - tm * args.tiles_n[p];
  if constexpr (SPLIT) {
    const int s = blockIdx.y, kbeg = s * args.kchunk[p], M = args.M[p], N = args.N[p];
    if (kbeg >= args.K[p]) return;  // this problem has fewer splits (shorter K)
    Epi<float> slab{};
    slab.C = args.ws + args.ws_off[p];
    slab.ldc = N;
    slab.alpha = 1.f;
    slab.zstride = (int64_t)M * N;
    slab.zi = s;
    slab.vec_ok = (N & 7) == 0;
    gemm_tile<T, 64, 64, A_KC, B_KC, AL, BL, Epi<float>, X3>(args.a[p], args.b[p], slab, tm * 64, tn * 64, M, N, kbeg,
                                                             min(args.K[p], kbeg + args.kchunk[p]), 0);
  } else {
    gemm_tile<T, 64, 64, A_KC, B_KC, AL, BL, Epi<TO>, X3>(args.a[p], args.b[p], args.e[p], tm * 64, tn * 64,
                                                            args.M[p], args.N[p], 0, args.K[p], 0);
  }
}

// ---------------------------------------------------------------------------
// Split-K with the reduction in the same launch.  Every K-split block writes its fp32 slab as before; then it
// publishes (every wave drains its stores, barrier, one lane: agent-scope release, drain, relaxed agent-scope
// ticket on the tile's counter) and the block that draws the last ticket resets the counter, acquires at agent
// scope and reduces the tile's slabs in split order through the real epilogue -- the reduction kernel's order,
// so the outputs are bit-identical to the two-launch form (cdna_hip_programming.md, "In-launch split-K
// reduction").  Counters live per stream (mg_tile_counters), zeroed once at allocation and by every last arriver.
// ---------------------------------------------------------------------------
template <int BM, int BN, class EP>
MG_DEV void splitk_tile_fixup(const float* __restrict__ ws, int splits, int M, int N, const EP& ep, int m0, int n0,
                              int* cnt) {
  __shared__ int last_flag;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int is_last = old == splits - 1;
    if (is_last) {
      __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    last_flag = is_last;
  }
  __syncthreads();
  if (!last_flag) return;
  const int64_t MN = (int64_t)M * N;
  for (int e = threadIdx.x; e < BM * BN / 8; e += NTHREADS) {
    const int r = e / (BN / 8), c = (e - r * (BN / 8)) * 8;
    const int m = m0 + r, n = n0 + c;
    if (m >= M || n >= N) continue;
    const float* p = ws + (int64_t)m * N + n;
    if (ep.vec_ok && (N & 7) == 0) {
      float v[8], t[8];
      ld8(p, v);
#pragma unroll 4
      for (int sp = 1; sp < splits; ++sp) {
        ld8(p + sp * MN, t);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += t[j];
      }
      ep.vec8(m, n, v);
    } else {
      for (int j = 0; j < 8 && n + j < N; ++j) {
        float v = 0.f;
        for (int sp = 0; sp < splits; ++sp) v += p[sp * MN + j];
        ep(m, n + j, v);
      }
    }
  }
}

template <typename T, int BM, int BN, bool A_KC, bool B_KC, class AL, class BL, typename TO, bool X3 = false>
__global__ __launch_bounds__(NTHREADS) void gemm_splitk_fused_kernel(AL A, BL B, Epi<float> slab, Epi<TO> ep, int M,
                                                                      int N, int K, int kchunk, int* cnt) {
  const int s = blockIdx.z;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  slab.zi = s;
  const int kbeg = s * kchunk, kend = min(K, kbeg + kchunk);
  gemm_tile<T, BM, BN, A_KC, B_KC, AL, BL, Epi<float>, X3>(A, B, slab, m0, n0, M, N, kbeg, kend, 0);
  splitk_tile_fixup<BM, BN>(slab.C, gridDim.z, M, N, ep, m0, n0, cnt + blockIdx.x * gridDim.y + blockIdx.y);
}

// launch helper: picks the grid; grouped-M launches an upper bound of tiles.
template <typename T, int BM, int BN, bool A_KC, bool B_KC, int TAG = 0, bool X3 = false, class AL, class BL, class EP>
inline void launch_gemm(const AL& A, const BL& B, const EP& ep, int M, int N, int K, int splits, Grouping grp,
                        int max_tiles_m, hipStream_t st) {
  constexpr int TBK = tile_bk<T, X3, BM, BN>();
  int kchunk = K;
  if (grp.mode != 2 && splits > 1) kchunk = ((K + splits - 1) / splits + TBK - 1) / TBK * TBK;
  if (grp.mode != 2) splits = (K + kchunk - 1) / kchunk;
  if (splits < 1) splits = 1;
  int gx = grp.mode == 1 ? max_tiles_m << grp.sub_shift : grp.mode == 3 ? cdiv(grp.rows_per_group, BM) * grp.ngroups : cdiv(M, BM);
  int gz = grp.mode == 2 ? splits * grp.ngroups : splits;
  dim3 grid(gx, cdiv(N, BN), gz);
  EP e2 = ep;
  e2.vec_ok = e2.host_vec_ok() ? 1 : 0;
  // XCD-aware order (gemm_kernel): tuning slot MG_TUNE_XCD 0 (default) / 1 every launch (dense or grouped), 2 split-K
  // launches only, 3 none.  Round 4 measured it neutral-to-worse in isolation (profiles/round4_xcd_probe.txt); in
  // the round-5 step it is a steady win: C2 8.51 / 8.51 -> 8.39 / 8.39 ms, C5 11.21 -> 11.02 ms (same-box A/B,
  // tools/gpu.sh tune=6=0 / tune=6=1), so on by default.
  const int xcd = g_mg_tune[MG_TUNE_XCD];
  if (grp.mode == 0 || grp.mode == 1) grp.swz = xcd == 0 ? 1 : xcd == 3 ? 0 : xcd;
  // grouped weight gradients (mode 2): on by default (slot value 3 turns it off).  Their (group, K split) slices
  // are read by every output tile of the slice; in dispatch order those tiles land on different XCDs, and the
  // PMC passes showed the narrow operand fetched once per tile (a 16x16 block's gW1 read 270 MB for 168 MB of
  // operands)
  if (grp.mode == 2) grp.swz = xcd == 3 ? 0 : 1;
  hipLaunchKernelGGL((gemm_kernel<T, BM, BN, A_KC, B_KC, AL, BL, EP, TAG, X3>), grid, dim3(NTHREADS), 0, st, A, B, e2, M, N,
                     K, kchunk, grp);
}

// split-K slab reduction: C = epilogue(sum_s ws[s]) for a [M, N] tile set (ws row pitch N), over blocks
// blk of nblk.  Slabs are added in split order (fixed, whatever the grid); their loads are issued four at a
// time so the (small, latency-bound) reduction waits about once per four slabs, not once per slab.
template <class EP>
MG_DEV void splitk_reduce_body(const float* __restrict__ ws, int splits, int M, int N, const EP& ep, int blk, int nblk) {
  const int64_t MN = (int64_t)M * N;
  if (ep.vec_ok && (N & 7) == 0) {  // 8 columns per thread: 16-B slab loads, the vector epilogue
    const int64_t n8 = MN >> 3;
    for (int64_t q = (int64_t)blk * 256 + threadIdx.x; q < n8; q += (int64_t)nblk * 256) {
      const int64_t i = q << 3;
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, t[4][8];
      if (splits > 0) ld8(ws + i, v);
      int s = 1;
      for (; s + 4 <= splits; s += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) ld8(ws + (s + u) * MN + i, t[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] += t[u][j];
      }
      for (; s < splits; ++s) {
        ld8(ws + s * MN + i, t[0]);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += t[0][j];
      }
      const int m = (int)(i / N), n = (int)(i - (int64_t)m * N);
      ep.vec8(m, n, v);
    }
    return;
  }
  for (int64_t i = (int64_t)blk * 256 + threadIdx.x; i < MN; i += (int64_t)nblk * 256) {
    float v = 0.f, t[4];
    int s = 0;
    for (; s + 4 <= splits; s += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) t[u] = ws[(s + u) * MN + i];
#pragma unroll
      for (int u = 0; u < 4; ++u) v += t[u];
    }
    for (; s < splits; ++s) v += ws[s * MN + i];
    int m = (int)(i / N), n = (int)(i - (int64_t)(i / N) * N);
    ep(m, n, v);
  }
}

template <class EP>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, int splits, int M, int N,
                                                            EP ep) {
  splitk_reduce_body(ws, splits, M, N, ep, blockIdx.x, gridDim.x);
}

// the batched GEMMs' slab reductions: blocks [blk_off[p], blk_off[p + 1]) reduce problem p's splits[p] slabs
template <typename TO>
struct BatchReduceArgs {
  Epi<TO> e[MG_BATCH_MAX];
  int64_t ws_off[MG_BATCH_MAX];
  int M[MG_BATCH_MAX], N[MG_BATCH_MAX], splits[MG_BATCH_MAX], blk_off[MG_BATCH_MAX + 1];
  int n;
  const float* ws;
};

template <typename TO>
__global__ __launch_bounds__(256) void batch_reduce_kernel(BatchReduceArgs<TO> r) {
  const int t = blockIdx.x;
  int p = 0;
  while (p + 1 < r.n && t >= r.blk_off[p + 1]) ++p;
  splitk_reduce_body(r.ws + r.ws_off[p], r.splits[p], r.M[p], r.N[p], r.e[p], t - r.blk_off[p],
                     r.blk_off[p + 1] - r.blk_off[p]);
}

}  // namespace mg
