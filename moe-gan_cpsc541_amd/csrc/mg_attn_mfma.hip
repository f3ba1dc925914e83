// Self-attention of the AttentionBlock on MFMA (bf16 operands, fp32 accumulate), gfx950.
//
// nn.MultiheadAttention, 8 heads (t2i_moe_gan.py:533-551) at this model's sizes: L = 16 / 64 / 256
// tokens per image, head dim D = 64 / 32 / 16.  One wave owns a 16-row tile (queries in the forward
// and the dQ pass, keys in the dK/dV pass) of one (image, head) "unit"; a unit's Q, K, V (and dO)
// live in LDS for the whole block.
//
// Products contracted over D (S = Q K^T, dP = dO V^T) use the MFMA with both operands read as rows
// (16x16x16 for D = 16, 16x16x32 otherwise).  Products contracted over tokens (O = P V, dQ = dS K,
// dV = P^T dO, dK = dS^T Q) take their A operand straight from the accumulator registers of the first
// product: computing the first product "swapped" (S^T when the second contracts over keys for a
// query-owner wave, S when it contracts over queries for a key-owner wave) leaves lane l holding the
// 8 tokens {4g..4g+3} U {16+4g..16+4g+3} (g = l >> 4) of a 32-token chunk for row l & 15 -- a
// permuted k order, matched on the B side by two ds_read_b64_tr_b16 of token rows 4g.. and 16+4g..
// No softmax state crosses lanes except two xor-shuffles per row statistic.
//
// Softmax is exact two-pass (all scores of a row tile stay in registers: L/4 floats per lane).
#include <algorithm>

#include "mg_common.h"

namespace {

typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

template <int D> struct Pitch;  // LDS row pitch (bf16): rows 0..7 of a tr-read half hit distinct bank octets
template <> struct Pitch<16> { static constexpr int P = 16; };  // + the chunk swizzle below
template <> struct Pitch<32> { static constexpr int P = 48; };
template <> struct Pitch<64> { static constexpr int P = 80; };

template <int D> struct Frag;
template <> struct Frag<16> { s16x4_t a; };
template <> struct Frag<32> { bf16x8_t a; };
template <> struct Frag<64> { bf16x8_t a, b; };

// D = 16 images (32-B rows, four 8-B chunks): chunk j of row r is stored at chunk j ^ swz16(r).  A row-operand read
// (ds_read_b64, lanes 0-31 = rows 0..15 x chunks 0, 1) then puts rows r and r + 8 on different bank quads (unswizzled
// they share one: the measured 40-61 % bank-conflict share of these kernels), and a transposed read (rows 4g+q of one
// 8-row half x chunks 0..3) still hits 8 distinct bank octets per lane group.
MG_DEV constexpr int swz16(int r) { return ((r >> 3) & 1) << 1; }
template <int D> MG_DEV constexpr int col_off(int r, int c) {  // element offset of column c (a multiple of 4) in row r
  return D == 16 ? ((((c >> 2) ^ swz16(r))) << 2) + (c & 3) : c;
}

// row-operand fragment of a [rows][D] LDS image: row r, d-chunk of lane group g
template <int D> MG_DEV Frag<D> ldfrag(const bf16_t* img, int r, int g);
template <> MG_DEV Frag<16> ldfrag<16>(const bf16_t* img, int r, int g) {
  return Frag<16>{*reinterpret_cast<const s16x4_t*>(img + r * Pitch<16>::P + col_off<16>(r, 4 * g))};
}
template <> MG_DEV Frag<32> ldfrag<32>(const bf16_t* img, int r, int g) {
  return Frag<32>{__builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u16x8_t*>(img + r * Pitch<32>::P + 8 * g))};
}
template <> MG_DEV Frag<64> ldfrag<64>(const bf16_t* img, int r, int g) {
  const bf16_t* p = img + r * Pitch<64>::P;
  return Frag<64>{__builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u16x8_t*>(p + 8 * g)),
                  __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u16x8_t*>(p + 32 + 8 * g))};
}

// C[m][n] = sum_d X[m][d] Y[n][d]  (lane: m = 4g + reg, n = lane & 15)
MG_DEV f32x4_t mfma_d(const Frag<16>& x, const Frag<16>& y) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(x.a, y.a, f32x4_t{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
}
MG_DEV f32x4_t mfma_d(const Frag<32>& x, const Frag<32>& y) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(x.a, y.a, f32x4_t{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
}
MG_DEV f32x4_t mfma_d(const Frag<64>& x, const Frag<64>& y) {
  f32x4_t c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x.a, y.a, f32x4_t{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(x.b, y.b, c, 0, 0, 0);
}

// acc[m][n] += sum_{k in 32-token chunk} A[m][k] Y[k][n]: A from registers (permuted k order), Y an LDS
// image [tokens][pitch], rows chunk0 + {4g..4g+3, 16+4g..16+4g+3}, columns c0..c0+15.
template <int D>
MG_DEV f32x4_t mfma_tok(bf16x8_t a, const bf16_t* img, int pitch, int chunk0, int c0, int lane, f32x4_t acc) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  auto base = (__attribute__((address_space(3))) char*)(img);
  const int r0 = chunk0 + 4 * g + q;
  s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4_t*)(base + (r0 * pitch + col_off<D>(r0, c0 + 4 * p)) * 2));
  s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4_t*)(base + ((r0 + 16) * pitch + col_off<D>(r0 + 16, c0 + 4 * p)) * 2));
  u16x8_t b;
  b[0] = lo[0]; b[1] = lo[1]; b[2] = lo[2]; b[3] = lo[3];
  b[4] = hi[0]; b[5] = hi[1]; b[6] = hi[2]; b[7] = hi[3];
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8_t, b), acc, 0, 0, 0);
}

MG_DEV bf16x8_t pack8(const f32x4_t& lo, const f32x4_t& hi) {
  u16x8_t r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = f2bf(lo[j]);
    r[j + 4] = f2bf(hi[j]);
  }
  return __builtin_bit_cast(bf16x8_t, r);
}

MG_DEV float max16x4(float v) {  // across the 4 lane groups holding one column
  v = fmaxf(v, __shfl_xor(v, 16, 64));
  return fmaxf(v, __shfl_xor(v, 32, 64));
}
MG_DEV float sum16x4(float v) {
  v += __shfl_xor(v, 16, 64);
  return v + __shfl_xor(v, 32, 64);
}

// stage rows [0, L) of a [L][D] head slice (row pitch ld in elements, column offset col) into an LDS
// image with pitch P; rows [L, Lp) are zero-filled.  Threads of the unit cooperate (n_thr, t0).
template <int D>
MG_DEV void stage(bf16_t* img, const bf16_t* src, int64_t ld, int L, int Lp, int t, int n_thr) {
  constexpr int P = Pitch<D>::P, CV = D / 8;
  for (int e = t; e < Lp * CV; e += n_thr) {
    int r = e / CV, c = (e - r * CV) * 8;
    u16x8_t v = u16x8_t(0);
    if (r < L) v = *reinterpret_cast<const u16x8_t*>(src + r * ld + c);
    *reinterpret_cast<u16x8_t*>(img + r * P + col_off<D>(r, c)) = v;  // (the swizzle keeps 16-B pairs whole)
  }
}

// Block -> (image, head) unit.  A head's q / k / v / out columns are D * 2 bytes of each token row (32 B at the 16x16
// block's D = 16), so the heads of one image share every 128-B line.  Blocks are dispatched round-robin over the 8
// XCDs (blockIdx % 8), each with its own L2: with unit = blockIdx every XCD held one head of every image and fetched
// each line for its 32 B (4x the algorithmic bytes; profiles/family_traffic.json round 6: 1.15 GB per step for the
// attention family).  With one unit per block and B % 8 == 0, XCD x runs all heads of images x, x + 8, ...
template <int U>
MG_DEV int attn_block_unit(int bid, int B, int heads) {
  if (U != 1 || (B & 7)) return bid;
  const int x = bid & 7, s = bid >> 3;
  return ((s / heads) * 8 + x) * heads + s % heads;
}

// ---------------------------------------------------------------------------
// forward: O = softmax(Q K^T / sqrt(D)) V, lse per query
// ---------------------------------------------------------------------------
// LT: token tile length (a multiple of 16); the sequence length L <= LT is a runtime argument (L = LT for the
// generator's blocks; CLIP's 50 tokens run on the 64-token tiles with rows >= L masked on load and store)
// MASK: L < max(LT, 32) (key / query slots past L masked); false for the generator's blocks (L == LT >= 32), whose softmax runs
// without the per-score compare / select.  Scores are exponentiated as exp2(s * scale * log2 e - max), one fma and one
// v_exp per score, and the 1 / sum normalisation is applied to the P V output rather than to every probability.
template <int D, int LT, int U, bool MASK>  // U units (image, head) per block, WPU waves per unit
__global__ __launch_bounds__(256) void k_attn_fwd_mfma(const bf16_t* __restrict__ qkv, int B, int L, int C, int heads,
                                                       bf16_t* __restrict__ out, float* __restrict__ lse) {
  constexpr int P = Pitch<D>::P;
  constexpr int Lp = LT < 32 ? 32 : LT;
  constexpr int WPU = LT / 16 < 4 ? LT / 16 : 4;
  constexpr int NKB = Lp / 16;
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, fr = lane & 15;
  const int ul = wave / WPU, wu = wave % WPU;
  const int unit = attn_block_unit<U>(blockIdx.x, B, heads) * U + ul;
  const bool live = unit < B * heads;
  const int b = live ? unit / heads : 0, h = live ? unit - (unit / heads) * heads : 0;
  bf16_t* Ks = smem + ul * 2 * Lp * P;
  bf16_t* Vs = Ks + Lp * P;
  const int64_t ld = 3LL * C;
  const bf16_t* base = qkv + (int64_t)b * L * ld + h * D;
  if (live) {
    stage<D>(Ks, base + C, ld, L, Lp, wu * 64 + lane, WPU * 64);
    stage<D>(Vs, base + 2 * C, ld, L, Lp, wu * 64 + lane, WPU * 64);
  }
  __syncthreads();
  if (!live) return;
  const float scale = rsqrtf((float)D);
  for (int t = wu; t < LT / 16; t += WPU) {
    // Q fragment straight from HBM (rows t*16 + fr; rows past L read as the clamped last row, never stored)
    Frag<D> qf;
    {
      const bf16_t* qr = base + (int64_t)min(t * 16 + fr, L - 1) * ld;
      if constexpr (D == 16) qf.a = *reinterpret_cast<const s16x4_t*>(qr + 4 * g);
      else if constexpr (D == 32) qf.a = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u16x8_t*>(qr + 8 * g));
      else {
        qf.a = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u16x8_t*>(qr + 8 * g));
        qf.b = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u16x8_t*>(qr + 32 + 8 * g));
      }
    }
    // pass 1: S^T blocks (lane: key kb*16 + 4g + r, query t*16 + fr), raw scores; row max
    f32x4_t s[NKB];
    float m = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
      s[kb] = mfma_d(ldfrag<D>(Ks, kb * 16 + fr, g), qf);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if constexpr (MASK)
          if (kb * 16 + 4 * g + r >= L) s[kb][r] = -INFINITY;
        m = fmaxf(m, s[kb][r]);
      }
    }
    m = max16x4(m);
    // p = exp(scale * (s - m)) = exp2(s * k2 - m * k2)
    const float k2 = scale * 1.4426950408889634f, mk = m * k2;
    float l = 0.f;
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float p = __builtin_amdgcn_exp2f(fmaf(s[kb][r], k2, -mk));  // (a masked -inf score gives 0)
        s[kb][r] = p;
        l += p;
      }
    l = sum16x4(l);
    // pass 2: O = P V / l  (lane: query t*16 + 4g + r, d = db*16 + fr); the unnormalised probabilities (max 1)
    // are the bf16 MFMA operand, the row's 1 / l scales the output
    f32x4_t o[D / 16];
#pragma unroll
    for (int db = 0; db < D / 16; ++db) o[db] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NKB / 2; ++c) {
      bf16x8_t pa = pack8(s[2 * c], s[2 * c + 1]);
#pragma unroll
      for (int db = 0; db < D / 16; ++db) o[db] = mfma_tok<D>(pa, Vs, P, 32 * c, db * 16, lane, o[db]);
    }
    // o[db][r] belongs to query t*16 + 4g + r, whose 1 / l lives in lane (4g + r) of every lane group
    float inv_r[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) inv_r[r] = 1.f / __shfl(l, 4 * g + r, 64);
#pragma unroll
    for (int db = 0; db < D / 16; ++db)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (!MASK || t * 16 + 4 * g + r < L)
          out[((int64_t)b * L + t * 16 + 4 * g + r) * C + h * D + db * 16 + fr] = f2bf(o[db][r] * inv_r[r]);
    if (g == 0 && (!MASK || t * 16 + fr < L)) lse[((int64_t)b * heads + h) * L + t * 16 + fr] = m * scale + __logf(l);
  }
}

// ---------------------------------------------------------------------------
// backward: dQ (query-owner waves), then dK, dV (key-owner waves)
// ---------------------------------------------------------------------------
template <int D, int L, int U>
__global__ __launch_bounds__(256) void k_attn_bwd_mfma(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ out,
                                                       const bf16_t* __restrict__ gout, const float* __restrict__ lse,
                                                       int B, int C, int heads, bf16_t* __restrict__ gqkv) {
  constexpr int P = Pitch<D>::P;
  constexpr int Lp = L < 32 ? 32 : L;
  constexpr int WPU = L / 16 < 4 ? L / 16 : 4;
  constexpr int NB = Lp / 16;
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, fr = lane & 15;
  const int ul = wave / WPU, wu = wave % WPU;
  const int unit = attn_block_unit<U>(blockIdx.x, B, heads) * U + ul;
  const bool live = unit < B * heads;
  const int b = live ? unit / heads : 0, h = live ? unit - (unit / heads) * heads : 0;
  bf16_t* Qs = smem + ul * (4 * Lp * P + 4 * Lp);  // 4 images + 2 float vectors (as 4*Lp bf16 slots)
  bf16_t* Ks = Qs + Lp * P;
  bf16_t* Vs = Ks + Lp * P;
  bf16_t* Gs = Vs + Lp * P;  // dO
  float* Ls = reinterpret_cast<float*>(Gs + Lp * P);
  float* Ds = Ls + Lp;
  const int64_t ld = 3LL * C;
  const bf16_t* base = qkv + (int64_t)b * L * ld + h * D;
  const int tu = wu * 64 + lane, nu = WPU * 64;
  if (live) {
    stage<D>(Qs, base, ld, L, Lp, tu, nu);
    stage<D>(Ks, base + C, ld, L, Lp, tu, nu);
    stage<D>(Vs, base + 2 * C, ld, L, Lp, tu, nu);
    stage<D>(Gs, gout + (int64_t)b * L * C + h * D, C, L, Lp, tu, nu);
    for (int i = tu; i < Lp; i += nu) {
      float dsum = 0.f, lv = 0.f;
      if (i < L) {
        const int64_t row = ((int64_t)b * L + i) * C + h * D;
#pragma unroll
        for (int c = 0; c < D; c += 8) {
          float o8[8], g8[8];
          ld8(out + row + c, o8);
          ld8(gout + row + c, g8);
#pragma unroll
          for (int j = 0; j < 8; ++j) dsum += o8[j] * g8[j];
        }
        lv = lse[((int64_t)b * heads + h) * L + i] * 1.4426950408889634f;  // log2 units: p = exp2(s k2 - lv)
      }
      Ls[i] = lv;
      Ds[i] = dsum;
    }
  }
  __syncthreads();
  if (!live) return;
  const float scale = rsqrtf((float)D), k2 = scale * 1.4426950408889634f;
  constexpr bool MASKK = Lp != L;  // token slots past L exist only when L < 32
  bf16_t* grow = gqkv + (int64_t)b * L * ld + h * D;
  // ---- pass A: dQ = scale * dS K for query tiles
  for (int t = wu; t < L / 16; t += WPU) {
    Frag<D> qf = ldfrag<D>(Qs, t * 16 + fr, g), gf = ldfrag<D>(Gs, t * 16 + fr, g);
    const float li = Ls[t * 16 + fr], di = Ds[t * 16 + fr];  // this lane's query column
    f32x4_t dq[D / 16];
#pragma unroll
    for (int db = 0; db < D / 16; ++db) dq[db] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
    for (int c = 0; c < NB / 2; ++c) {
      f32x4_t ds[2];
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) {
        const int kb = 2 * c + jb;
        f32x4_t st = mfma_d(ldfrag<D>(Ks, kb * 16 + fr, g), qf);   // S^T[key][query]
        f32x4_t dpt = mfma_d(ldfrag<D>(Vs, kb * 16 + fr, g), gf);  // dP^T[key][query]
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float p = __builtin_amdgcn_exp2f(fmaf(st[r], k2, -li));
          if constexpr (MASKK)
            if (kb * 16 + 4 * g + r >= L) p = 0.f;
          ds[jb][r] = p * (dpt[r] - di);
        }
      }
      bf16x8_t a = pack8(ds[0], ds[1]);
#pragma unroll
      for (int db = 0; db < D / 16; ++db) dq[db] = mfma_tok<D>(a, Ks, P, 32 * c, db * 16, lane, dq[db]);
    }
#pragma unroll
    for (int db = 0; db < D / 16; ++db)
#pragma unroll
      for (int r = 0; r < 4; ++r) grow[(int64_t)(t * 16 + 4 * g + r) * ld + db * 16 + fr] = f2bf(dq[db][r] * scale);
  }
  // ---- pass B: dV = P^T dO, dK = scale * dS^T Q for key tiles
  for (int t = wu; t < L / 16; t += WPU) {
    Frag<D> kf = ldfrag<D>(Ks, t * 16 + fr, g), vf = ldfrag<D>(Vs, t * 16 + fr, g);
    f32x4_t dk[D / 16], dv[D / 16];
#pragma unroll
    for (int db = 0; db < D / 16; ++db) dk[db] = dv[db] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
    for (int c = 0; c < NB / 2; ++c) {
      f32x4_t pp[2], ds[2];
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) {
        const int qb = 2 * c + jb;
        f32x4_t sv = mfma_d(ldfrag<D>(Qs, qb * 16 + fr, g), kf);   // S[query][key]
        f32x4_t dp = mfma_d(ldfrag<D>(Gs, qb * 16 + fr, g), vf);   // dP[query][key]
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qi = qb * 16 + 4 * g + r;
          float p = __builtin_amdgcn_exp2f(fmaf(sv[r], k2, -Ls[qi]));
          if constexpr (MASKK)
            if (qi >= L) p = 0.f;
          pp[jb][r] = p;
          ds[jb][r] = p * (dp[r] - Ds[qi]);
        }
      }
      bf16x8_t ap = pack8(pp[0], pp[1]), ad = pack8(ds[0], ds[1]);
#pragma unroll
      for (int db = 0; db < D / 16; ++db) {
        dv[db] = mfma_tok<D>(ap, Gs, P, 32 * c, db * 16, lane, dv[db]);
        dk[db] = mfma_tok<D>(ad, Qs, P, 32 * c, db * 16, lane, dk[db]);
      }
    }
#pragma unroll
    for (int db = 0; db < D / 16; ++db)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t o = (int64_t)(t * 16 + 4 * g + r) * ld + db * 16 + fr;
        grow[o + C] = f2bf(dk[db][r] * scale);
        grow[o + 2 * C] = f2bf(dv[db][r]);
      }
  }
}

// units per block: fill 4 waves, but keep the block's LDS within 64 KiB
template <int D, int L>
constexpr int units_fwd() {
  constexpr int WPU = L / 16 < 4 ? L / 16 : 4, Lp = L < 32 ? 32 : L;
  int u = 4 / WPU;
  while (u > 1 && (size_t)u * 2 * Lp * Pitch<D>::P * 2 > 65536) u /= 2;
  return u;
}
template <int D, int L>
constexpr int units_bwd() {
  constexpr int WPU = L / 16 < 4 ? L / 16 : 4, Lp = L < 32 ? 32 : L;
  int u = 4 / WPU;
  while (u > 1 && (size_t)u * (4 * Lp * Pitch<D>::P + 4 * Lp) * 2 > 65536) u /= 2;
  return u;
}

template <int D, int LT>
int launch_fwd(const bf16_t* qkv, int B, int C, int heads, bf16_t* out, float* lse, hipStream_t st, int L = LT) {
  constexpr int P = Pitch<D>::P, Lp = LT < 32 ? 32 : LT, WPU = LT / 16 < 4 ? LT / 16 : 4, U = units_fwd<D, LT>();
  size_t sm = (size_t)U * 2 * Lp * P * sizeof(bf16_t);
  if (L == Lp)  // (LT = 16 tiles pad the keys to 32 slots: masked)
    hipLaunchKernelGGL((k_attn_fwd_mfma<D, LT, U, false>), dim3(cdiv(B * heads, U)), dim3(64 * U * WPU), sm, st, qkv, B,
                       L, C, heads, out, lse);
  else
    hipLaunchKernelGGL((k_attn_fwd_mfma<D, LT, U, true>), dim3(cdiv(B * heads, U)), dim3(64 * U * WPU), sm, st, qkv, B,
                       L, C, heads, out, lse);
  return mg_check_launch("mg_attn_fwd (mfma)");
}
template <int D, int L>
int launch_bwd(const bf16_t* qkv, const bf16_t* out, const bf16_t* gout, const float* lse, int B, int C, int heads,
               bf16_t* gqkv, hipStream_t st) {
  constexpr int P = Pitch<D>::P, Lp = L < 32 ? 32 : L, WPU = L / 16 < 4 ? L / 16 : 4, U = units_bwd<D, L>();
  size_t sm = (size_t)U * (4 * Lp * P + 4 * Lp) * sizeof(bf16_t);
  hipLaunchKernelGGL((k_attn_bwd_mfma<D, L, U>), dim3(cdiv(B * heads, U)), dim3(64 * U * WPU), sm, st, qkv, out, gout,
                     lse, B, C, heads, gqkv);
  return mg_check_launch("mg_attn_bwd (mfma)");
}

}  // namespace

// bf16 MFMA attention for the model's (L, D) pairs; returns 1 when the shape is not covered (caller
// falls back to the scalar kernels of mg_attn.hip), else an MG status.
int mg_attn_fwd_mfma(const void* qkv, int B, int L, int C, int heads, void* out, float* lse, hipStream_t st) {
  const int D = C / heads;
  auto q = reinterpret_cast<const bf16_t*>(qkv);
  auto o = reinterpret_cast<bf16_t*>(out);
  if (!mg_al16(qkv) || !mg_al16(out) || C % 8) return 1;
  if (D == 64 && L == 16) return launch_fwd<64, 16>(q, B, C, heads, o, lse, st);
  if (D == 32 && L == 64) return launch_fwd<32, 64>(q, B, C, heads, o, lse, st);
  if (D == 16 && L == 256) return launch_fwd<16, 256>(q, B, C, heads, o, lse, st);
  if (D == 64 && L == 64) return launch_fwd<64, 64>(q, B, C, heads, o, lse, st);
  if (D == 32 && L == 16) return launch_fwd<32, 16>(q, B, C, heads, o, lse, st);
  if (D == 16 && L == 64) return launch_fwd<16, 64>(q, B, C, heads, o, lse, st);
  if (D == 64 && L > 32 && L < 64) return launch_fwd<64, 64>(q, B, C, heads, o, lse, st, L);  // CLIP ViT-B/32: 50
  return 1;
}

int mg_attn_bwd_mfma(const void* qkv, const void* out, const void* gout, const float* lse, int B, int L, int C,
                     int heads, void* gqkv, hipStream_t st) {
  const int D = C / heads;
  auto q = reinterpret_cast<const bf16_t*>(qkv);
  auto o = reinterpret_cast<const bf16_t*>(out);
  auto g = reinterpret_cast<const bf16_t*>(gout);
  auto gq = reinterpret_cast<bf16_t*>(gqkv);
  if (!mg_al16(qkv) || !mg_al16(out) || !mg_al16(gout) || !mg_al16(gqkv) || C % 8) return 1;
  if (D == 64 && L == 16) return launch_bwd<64, 16>(q, o, g, lse, B, C, heads, gq, st);
  if (D == 32 && L == 64) return launch_bwd<32, 64>(q, o, g, lse, B, C, heads, gq, st);
  if (D == 16 && L == 256) return launch_bwd<16, 256>(q, o, g, lse, B, C, heads, gq, st);
  if (D == 64 && L == 64) return launch_bwd<64, 64>(q, o, g, lse, B, C, heads, gq, st);
  if (D == 32 && L == 16) return launch_bwd<32, 16>(q, o, g, lse, B, C, heads, gq, st);
  if (D == 16 && L == 64) return launch_bwd<16, 64>(q, o, g, lse, B, C, heads, gq, st);
  return 1;
}
