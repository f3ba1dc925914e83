// LayerNorm and self-attention kernels of the AttentionBlock (t2i_moe_gan.py:493-576).
//
// Token layout: rows = B*L tokens (L = H*W per image), C channels.
// Self-attention (nn.MultiheadAttention, 8 heads, batch_first) works on the
// packed projection qkv [rows, 3C] (q | k | v, head h at columns h*d..h*d+d).
// At this model's sizes (L <= 256, d = C/8 <= 64) one workgroup holds one
// (image, head) pair entirely in LDS; each thread owns a query row (forward,
// backward dQ) or a key row (backward dK/dV).  The cross-attention has a
// single key, so its softmax is identically 1 and it is computed as a per-image
// vector by plain GEMMs in the host engine (no kernel here).
#include "mg_common.h"

namespace {

template <typename T, int NPL>  // NPL = C/64 elements per lane
__global__ void k_ln_fwd(const T* __restrict__ x, int64_t ldx, int R, const float* __restrict__ gamma,
                         const float* __restrict__ beta, float eps, T* __restrict__ y, int64_t ldy,
                         float* __restrict__ mean, float* __restrict__ rstd, int act) {
  int lane = threadIdx.x & 63;
  int r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= R) return;
  constexpr int C = NPL * 64;
  float v[NPL];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    v[i] = ldf(x, (int64_t)r * ldx + lane + 64 * i);
    s += v[i];
  }
  float mu = wave_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    float t = v[i] - mu;
    q += t * t;
  }
  float rs = rsqrtf(wave_sum(q) / C + eps);
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    int c = lane + 64 * i;
    float o = (v[i] - mu) * rs * gamma[c] + beta[c];
    stf(y, (int64_t)r * ldy + c, act ? lrelu(o) : o);
  }
  if (lane == 0) {
    mean[r] = mu;
    rstd[r] = rs;
  }
}

template <typename T, typename TG, int NPL>
__global__ void k_ln_bwd(const TG* __restrict__ gy, int64_t ldg, const T* __restrict__ x, int64_t ldx, int R,
                         const float* __restrict__ mean, const float* __restrict__ rstd,
                         const float* __restrict__ gamma, T* __restrict__ gx, int64_t ldgx, int accumulate,
                         float* __restrict__ ggamma, float* __restrict__ gbeta, int rows_per_wave,
                         float* __restrict__ part) {
  int lane = threadIdx.x & 63;
  constexpr int C = NPL * 64;
  float pg[NPL], pb[NPL];
#pragma unroll
  for (int i = 0; i < NPL; ++i) pg[i] = pb[i] = 0.f;
  int wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  for (int rr = 0; rr < rows_per_wave; ++rr) {
    int r = wave * rows_per_wave + rr;
    if (r >= R) break;
    float mu = mean[r], rs = rstd[r];
    float xh[NPL], gh[NPL];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      int c = lane + 64 * i;
      float g = ldf(gy, (int64_t)r * ldg + c);
      xh[i] = (ldf(x, (int64_t)r * ldx + c) - mu) * rs;
      gh[i] = g * gamma[c];
      pg[i] += g * xh[i];
      pb[i] += g;
      s1 += gh[i];
      s2 += gh[i] * xh[i];
    }
    s1 = wave_sum(s1) / C;
    s2 = wave_sum(s2) / C;
    if (gx) {
#pragma unroll
      for (int i = 0; i < NPL; ++i) {
        int c = lane + 64 * i;
        float v = rs * (gh[i] - s1 - xh[i] * s2);
        if (accumulate) v += ldf(gx, (int64_t)r * ldgx + c);
        stf(gx, (int64_t)r * ldgx + c, v);
      }
    }
  }
  if (ggamma && part) {  // deterministic mode: the wave's partial row, folded in wave order by the launcher
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      part[(int64_t)wave * 2 * C + lane + 64 * i] = pg[i];
      part[(int64_t)wave * 2 * C + C + lane + 64 * i] = pb[i];
    }
  } else if (ggamma) {
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      atomicAdd(ggamma + lane + 64 * i, pg[i]);
      atomicAdd(gbeta + lane + 64 * i, pb[i]);
    }
  }
}

// ---------------------------------------------------------------------------
// self-attention forward: block = (image b, head h); thread i = query row i
// ---------------------------------------------------------------------------
template <typename T, int D>
__global__ void k_attn_fwd(const T* __restrict__ qkv, int L, int C, int heads, T* __restrict__ out,
                           float* __restrict__ lse) {
  extern __shared__ float sm[];
  float* Ks = sm;
  float* Vs = sm + L * D;
  int b = blockIdx.x / heads, h = blockIdx.x - (blockIdx.x / heads) * heads;
  const int64_t ld = 3LL * C;
  const T* base = qkv + (int64_t)b * L * ld;
  for (int e = threadIdx.x; e < L * D; e += blockDim.x) {
    int j = e / D, c = e - j * D;
    Ks[e] = ldf(base, (int64_t)j * ld + C + h * D + c);
    Vs[e] = ldf(base, (int64_t)j * ld + 2 * C + h * D + c);
  }
  __syncthreads();
  int i = threadIdx.x;
  if (i >= L) return;
  const float scale = rsqrtf((float)D);
  float q[D], acc[D];
#pragma unroll
  for (int c = 0; c < D; ++c) {
    q[c] = ldf(base, (int64_t)i * ld + h * D + c) * scale;
    acc[c] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  for (int j = 0; j < L; ++j) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < D; ++c) s += q[c] * Ks[j * D + c];
    float mn = fmaxf(m, s);
    float corr = __expf(m - mn);
    float p = __expf(s - mn);
    l = l * corr + p;
#pragma unroll
    for (int c = 0; c < D; ++c) acc[c] = acc[c] * corr + p * Vs[j * D + c];
    m = mn;
  }
  float inv = 1.f / l;
  int64_t orow = ((int64_t)b * L + i) * C + h * D;
#pragma unroll
  for (int c = 0; c < D; ++c) stf(out, orow + c, acc[c] * inv);
  lse[((int64_t)b * heads + h) * L + i] = m + __logf(l);
}

// backward: pass A (thread = query row): dQ; pass B (thread = key row): dK, dV.
// LDS holds K,V during pass A and Q,dO during pass B (2*L*D floats + 2*L).
template <typename T, typename TG, int D>
__global__ void k_attn_bwd(const T* __restrict__ qkv, const T* __restrict__ out, const TG* __restrict__ gout,
                           const float* __restrict__ lse, int L, int C, int heads, T* __restrict__ gqkv) {
  extern __shared__ float sm[];
  float* S0 = sm;
  float* S1 = S0 + L * D;
  float* Ls = S1 + L * D;  // lse
  float* Ds = Ls + L;      // delta_i = dO_i . O_i
  int b = blockIdx.x / heads, h = blockIdx.x - (blockIdx.x / heads) * heads;
  const int64_t ld = 3LL * C;
  const T* base = qkv + (int64_t)b * L * ld;
  const float scale = rsqrtf((float)D);
  for (int e = threadIdx.x; e < L * D; e += blockDim.x) {
    int j = e / D, c = e - j * D;
    S0[e] = ldf(base, (int64_t)j * ld + C + h * D + c);      // K
    S1[e] = ldf(base, (int64_t)j * ld + 2 * C + h * D + c);  // V
  }
  int t = threadIdx.x;
  float q[D], g[D];
  int64_t grow = ((int64_t)b * L + t) * C + h * D;
  if (t < L) {
    float dsum = 0.f;
#pragma unroll
    for (int c = 0; c < D; ++c) {
      q[c] = ldf(base, (int64_t)t * ld + h * D + c) * scale;
      g[c] = ldf(gout, grow + c);
      dsum += g[c] * ldf(out, grow + c);
    }
    Ds[t] = dsum;
    Ls[t] = lse[((int64_t)b * heads + h) * L + t];
  }
  __syncthreads();
  int64_t row = ((int64_t)b * L + t) * ld + h * D;
  if (t < L) {
    float dq[D];
#pragma unroll
    for (int c = 0; c < D; ++c) dq[c] = 0.f;
    float li = Ls[t], di = Ds[t];
    for (int j = 0; j < L; ++j) {
      float s = 0.f, dp = 0.f;
#pragma unroll
      for (int c = 0; c < D; ++c) {
        s += q[c] * S0[j * D + c];
        dp += g[c] * S1[j * D + c];
      }
      float ds = __expf(s - li) * (dp - di);
#pragma unroll
      for (int c = 0; c < D; ++c) dq[c] += ds * S0[j * D + c];
    }
#pragma unroll
    for (int c = 0; c < D; ++c) stf(gqkv, row + c, dq[c] * scale);
  }
  __syncthreads();
  if (t < L) {
#pragma unroll
    for (int c = 0; c < D; ++c) {
      S0[t * D + c] = q[c];  // Q (scaled)
      S1[t * D + c] = g[c];  // dO
    }
  }
  __syncthreads();
  if (t < L) {
    float k[D], v[D], dk[D], dv[D];
#pragma unroll
    for (int c = 0; c < D; ++c) {
      k[c] = ldf(base, (int64_t)t * ld + C + h * D + c);
      v[c] = ldf(base, (int64_t)t * ld + 2 * C + h * D + c);
      dk[c] = dv[c] = 0.f;
    }
    for (int i = 0; i < L; ++i) {
      float s = 0.f, dp = 0.f;
#pragma unroll
      for (int c = 0; c < D; ++c) {
        s += S0[i * D + c] * k[c];
        dp += S1[i * D + c] * v[c];
      }
      float p = __expf(s - Ls[i]);
      float ds = p * (dp - Ds[i]);
#pragma unroll
      for (int c = 0; c < D; ++c) {
        dv[c] += p * S1[i * D + c];
        dk[c] += ds * S0[i * D + c];  // S0 carries the 1/sqrt(D) scale
      }
    }
#pragma unroll
    for (int c = 0; c < D; ++c) {
      stf(gqkv, row + C + c, dk[c]);
      stf(gqkv, row + 2 * C + c, dv[c]);
    }
  }
}

// ---- vectorised LayerNorm: LPR = C/8 lanes per row, each lane 8 consecutive channels (16-B loads);
// a wave covers 64/LPR rows at once.  Row statistics are reduced over the row's LPR lanes.
template <int LPR>
MG_DEV float row_sum(float v) {
#pragma unroll
  for (int o = 1; o < LPR; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T, int LPR>
__global__ __launch_bounds__(256) void k_ln_fwd_v(const T* __restrict__ x, int64_t ldx, int R,
                                                  const float* __restrict__ gamma, const float* __restrict__ beta,
                                                  float eps, T* __restrict__ y, int64_t ldy, float* __restrict__ mean,
                                                  float* __restrict__ rstd, int act) {
  constexpr int C = LPR * 8, RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, sl = lane / LPR, c = (lane % LPR) * 8;
  float ga[8], be[8];
  ld8(gamma + c, ga);
  ld8(beta + c, be);
  const int nwaves = gridDim.x * (blockDim.x >> 6);
  for (int r0 = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * RPW; r0 < R; r0 += nwaves * RPW) {
    const int r = r0 + sl;
    const bool ok = r < R;
    float v[8];
    if (ok) ld8(x + (int64_t)r * ldx + c, v);
    else
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = 0.f;
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j];
    const float mu = row_sum<LPR>(s) / C;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) q += (v[j] - mu) * (v[j] - mu);
    const float rs = rsqrtf(row_sum<LPR>(q) / C + eps);
    if (ok) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o[j] = (v[j] - mu) * rs * ga[j] + be[j];
        if (act) o[j] = lrelu(o[j]);
      }
      st8(y + (int64_t)r * ldy + c, o);
      if (lane % LPR == 0) {
        mean[r] = mu;
        rstd[r] = rs;
      }
    }
  }
}

// backward: each wave walks ROWS_PER_WAVE rows (RPW at a time); gamma/beta gradients are accumulated per lane
// (fixed channels), folded over the wave's row slots and the block's waves in LDS into one partial row per block
// (part; the host folds the rows), or one atomic per channel and block when part is null.
template <typename T, typename TG, int LPR>
__global__ __launch_bounds__(256) void k_ln_bwd_v(const TG* __restrict__ gy, int64_t ldg, const T* __restrict__ x,
                                                  int64_t ldx, int R, const float* __restrict__ mean,
                                                  const float* __restrict__ rstd, const float* __restrict__ gamma,
                                                  T* __restrict__ gx, int64_t ldgx, int accumulate,
                                                  float* __restrict__ ggamma, float* __restrict__ gbeta,
                                                  int rows_per_wave, float* __restrict__ part) {
  constexpr int C = LPR * 8, RPW = 64 / LPR;
  __shared__ float red[2][4][C];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, sl = lane / LPR, c = (lane % LPR) * 8;
  float ga[8], pg[8], pb[8];
  ld8(gamma + c, ga);
#pragma unroll
  for (int j = 0; j < 8; ++j) pg[j] = pb[j] = 0.f;
  const int w = blockIdx.x * (blockDim.x >> 6) + wv;
  const int rbeg = w * rows_per_wave, rend = min(R, rbeg + rows_per_wave);
  // two row slots per lane group per iteration, both rows' loads issued before either is used (one wave per
  // SIMD walked its rows load-to-use serially: ~30 us for 65536 rows of 128)
  for (int r0 = rbeg; r0 < rend; r0 += 2 * RPW) {
    float g[2][8], xh[2][8], o[2][8], mu[2], rs[2];
    bool ok[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = r0 + u * RPW + sl;
      ok[u] = r < rend;
      mu[u] = rs[u] = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) g[u][j] = xh[u][j] = o[u][j] = 0.f;
      if (ok[u]) {
        mu[u] = mean[r];
        rs[u] = rstd[r];
        ld8(gy + (int64_t)r * ldg + c, g[u]);
        ld8(x + (int64_t)r * ldx + c, xh[u]);
        if (gx && accumulate) ld8(gx + (int64_t)r * ldgx + c, o[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = r0 + u * RPW + sl;
      float gh[8], s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        xh[u][j] = (xh[u][j] - mu[u]) * rs[u];
        gh[j] = g[u][j] * ga[j];
        pg[j] += g[u][j] * xh[u][j];
        pb[j] += g[u][j];
        s1 += gh[j];
        s2 += gh[j] * xh[u][j];
      }
      s1 = row_sum<LPR>(s1) / C;  // every lane of a row group takes part (row validity is uniform in it)
      s2 = row_sum<LPR>(s2) / C;
      if (gx && ok[u]) {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[u][j] = rs[u] * (gh[j] - s1 - xh[u][j] * s2) + (accumulate ? o[u][j] : 0.f);
        st8(gx + (int64_t)r * ldgx + c, o[u]);
      }
    }
  }
  if (!ggamma) return;
  // fold the wave's row slots (lanes l, l+LPR, ...) then the block's waves
#pragma unroll
  for (int j = 0; j < 8; ++j) {
#pragma unroll
    for (int o = LPR; o < 64; o <<= 1) {
      pg[j] += __shfl_xor(pg[j], o, 64);
      pb[j] += __shfl_xor(pb[j], o, 64);
    }
  }
  if (sl == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[0][wv][c + j] = pg[j];
      red[1][wv][c + j] = pb[j];
    }
  }
  __syncthreads();
  const int nw = blockDim.x >> 6;
  for (int i = threadIdx.x; i < 2 * C; i += blockDim.x) {
    const int k = i / C, cc = i - k * C;
    float s = 0.f;
    for (int q = 0; q < nw; ++q) s += red[k][q][cc];
    if (part) part[(int64_t)blockIdx.x * 2 * C + i] = s;  // deterministic mode: folded in block order
    else atomicAdd((k ? gbeta : ggamma) + cc, s);
  }
}

}  // namespace

extern "C" int mg_layernorm_fwd(int dtype, const void* x, int64_t ldx, int R, int C, const float* gamma,
                                const float* beta, float eps, void* y, int64_t ldy, float* mean, float* rstd, int act,
                                void* stream) {
  // 128 / 256 / 512: the generator's widths; 768: the CLIP image tower (forward only, clip_vit.py)
  MG_REQUIRE(C == 128 || C == 256 || C == 512 || C == 768, "C must be 128, 256, 512 or 768");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (R == 0) return MG_OK;
  if (C <= 512 && ldx % 8 == 0 && ldy % 8 == 0 && mg_al16(x) && mg_al16(y) && mg_al16(gamma) && mg_al16(beta)) {
    const int lpr = C / 8, rpw = 64 / lpr;
    dim3 g2(std::min(cdiv(R, 4 * rpw), 2048)), b2(256);
#define LV_(T, P) hipLaunchKernelGGL((k_ln_fwd_v<T, P>), g2, b2, 0, st, (const T*)x, ldx, R, gamma, beta, eps, (T*)y, ldy, mean, rstd, act)
    if (dtype == MG_F32) {
      if (C == 128) LV_(float, 16); else if (C == 256) LV_(float, 32); else LV_(float, 64);
    } else {
      if (C == 128) LV_(bf16_t, 16); else if (C == 256) LV_(bf16_t, 32); else LV_(bf16_t, 64);
    }
#undef LV_
    return mg_check_launch("mg_layernorm_fwd");
  }
  dim3 grid(cdiv(R, 4)), blk(256);
#define L_(T, N) hipLaunchKernelGGL((k_ln_fwd<T, N>), grid, blk, 0, st, (const T*)x, ldx, R, gamma, beta, eps, (T*)y, ldy, mean, rstd, act)
  if (dtype == MG_F32) {
    if (C == 128) L_(float, 2); else if (C == 256) L_(float, 4); else if (C == 512) L_(float, 8); else L_(float, 12);
  } else {
    if (C == 128) L_(bf16_t, 2); else if (C == 256) L_(bf16_t, 4); else if (C == 512) L_(bf16_t, 8); else L_(bf16_t, 12);
  }
#undef L_
  return mg_check_launch("mg_layernorm_fwd");
}

extern "C" int mg_layernorm_bwd(int dtype, int gy_dtype, const void* gy, int64_t ldg, const void* x, int64_t ldx,
                                int R, int C, const float* mean, const float* rstd, const float* gamma, void* gx,
                                int64_t ldgx, int accumulate, float* ggamma, float* gbeta, void* stream) {
  MG_REQUIRE(C == 128 || C == 256 || C == 512, "C must be 128, 256 or 512");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (R == 0) return MG_OK;
  if (ldg % 8 == 0 && ldx % 8 == 0 && (!gx || ldgx % 8 == 0) && mg_al16(gy) && mg_al16(x) && (!gx || mg_al16(gx)) &&
      mg_al16(gamma)) {
    // two iterations of two row slots per wave (16 rows at C = 128, 4 at C = 512): 1024 - 4096 waves, ~4 per SIMD
    // to hide the row loads.  Round 5 ran ~1024 waves (one per SIMD, 8 - 64 serial rows each: 16 - 28 us per call)
    // because every block added its gamma / beta sums into the same 2C addresses with atomics; now each block
    // writes one partial row [2C] and a fixed-order rows fold (mg_fold.hip, deferred to the backward's flush inside
    // a step) adds them, in both library modes
    const int lpr = C / 8, rw = 64 / lpr;
    const int rows = 4 * rw;
    dim3 g2(cdiv(cdiv(R, rows), 4)), b2(256);
    float* part = nullptr;
    bool deferred = false;
    if (ggamma) {
      part = mg_fold_partials((size_t)g2.x * 2 * C * sizeof(float), st, &deferred);
      if (!part) return MG_ERR_LAUNCH;
    }
#define LV_(T, TG, P) hipLaunchKernelGGL((k_ln_bwd_v<T, TG, P>), g2, b2, 0, st, (const TG*)gy, ldg, (const T*)x, ldx, R, \
                                         mean, rstd, gamma, (T*)gx, ldgx, accumulate, ggamma, gbeta, rows, part)
#define LVC_(T, TG) if (C == 128) LV_(T, TG, 16); else if (C == 256) LV_(T, TG, 32); else LV_(T, TG, 64)
    if (dtype == MG_F32) {
      if (gy_dtype == MG_F32) { LVC_(float, float); } else { LVC_(float, bf16_t); }
    } else {
      if (gy_dtype == MG_F32) { LVC_(bf16_t, float); } else { LVC_(bf16_t, bf16_t); }
    }
#undef LVC_
#undef LV_
    if (part) mg_fold_rows_submit(mg_fold_rows{part, 2 * C, (int32_t)g2.x, 2 * C, C, ggamma, gbeta}, deferred, st);
    return mg_check_launch("mg_layernorm_bwd");
  }
  int rpw = std::max(1, std::min(64, R / 1024));
  dim3 grid(cdiv(cdiv(R, rpw), 4)), blk(256);
  float* part = nullptr;
  if (ggamma && mg_det()) {
    part = reinterpret_cast<float*>(mg_workspace((size_t)grid.x * 4 * 2 * C * sizeof(float), st));
    if (!part) return MG_ERR_LAUNCH;
    (void)hipMemsetAsync(part, 0, (size_t)grid.x * 4 * 2 * C * sizeof(float), st);  // waves past R leave their row
  }
#define L_(T, TG, N) hipLaunchKernelGGL((k_ln_bwd<T, TG, N>), grid, blk, 0, st, (const TG*)gy, ldg, (const T*)x, ldx, R, \
                                        mean, rstd, gamma, (T*)gx, ldgx, accumulate, ggamma, gbeta, rpw, part)
#define LC_(T, TG) if (C == 128) L_(T, TG, 2); else if (C == 256) L_(T, TG, 4); else L_(T, TG, 8)
  if (dtype == MG_F32) {
    if (gy_dtype == MG_F32) { LC_(float, float); } else { LC_(float, bf16_t); }
  } else {
    if (gy_dtype == MG_F32) { LC_(bf16_t, float); } else { LC_(bf16_t, bf16_t); }
  }
#undef LC_
#undef L_
  if (part) mg_det_fold_rows(part, (int)grid.x * 4, 2 * C, C, ggamma, gbeta, st);
  return mg_check_launch("mg_layernorm_bwd");
}

int mg_attn_fwd_mfma(const void* qkv, int B, int L, int C, int heads, void* out, float* lse, hipStream_t st);
int mg_attn_bwd_mfma(const void* qkv, const void* out, const void* gout, const float* lse, int B, int L, int C,
                     int heads, void* gqkv, hipStream_t st);

extern "C" int mg_attn_fwd(int dtype, const void* qkv, int B, int L, int C, int heads, void* out, float* lse,
                           void* stream) {
  int D = C / heads;
  MG_REQUIRE(D == 16 || D == 32 || D == 64, "head dim must be 16, 32 or 64");
  MG_REQUIRE(L <= 1024, "at most 1024 tokens per image");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == MG_BF16 && B > 0) {  // MFMA path for the model's shapes (exact fp32 parity mode stays scalar)
    int rc = mg_attn_fwd_mfma(qkv, B, L, C, heads, out, lse, st);
    if (rc != 1) return rc;
  }
  int thr = std::max(64, ((L + 63) / 64) * 64);
  size_t sm = 2 * (size_t)L * D * sizeof(float);
#define L_(T, DD) hipLaunchKernelGGL((k_attn_fwd<T, DD>), dim3(B * heads), dim3(thr), sm, st, (const T*)qkv, L, C, heads, (T*)out, lse)
  if (dtype == MG_F32) {
    if (D == 16) L_(float, 16); else if (D == 32) L_(float, 32); else L_(float, 64);
  } else {
    if (D == 16) L_(bf16_t, 16); else if (D == 32) L_(bf16_t, 32); else L_(bf16_t, 64);
  }
#undef L_
  return mg_check_launch("mg_attn_fwd");
}

extern "C" int mg_attn_bwd(int dtype, int gout_dtype, const void* qkv, const void* out, const void* gout,
                           const float* lse, int B, int L, int C, int heads, void* gqkv, void* stream) {
  int D = C / heads;
  MG_REQUIRE(D == 16 || D == 32 || D == 64, "head dim must be 16, 32 or 64");
  MG_REQUIRE(L <= 1024, "at most 1024 tokens per image");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == MG_BF16 && gout_dtype == MG_BF16 && B > 0) {
    int rc = mg_attn_bwd_mfma(qkv, out, gout, lse, B, L, C, heads, gqkv, st);
    if (rc != 1) return rc;
  }
  int thr = std::max(64, ((L + 63) / 64) * 64);
  size_t sm = (2 * (size_t)L * D + 2 * (size_t)L) * sizeof(float);
#define L_(T, TG, DD) hipLaunchKernelGGL((k_attn_bwd<T, TG, DD>), dim3(B * heads), dim3(thr), sm, st, (const T*)qkv, \
                                         (const T*)out, (const TG*)gout, lse, L, C, heads, (T*)gqkv)
#define LD_(T, TG) if (D == 16) L_(T, TG, 16); else if (D == 32) L_(T, TG, 32); else L_(T, TG, 64)
  if (dtype == MG_F32) {
    if (gout_dtype == MG_F32) { LD_(float, float); } else { LD_(float, bf16_t); }
  } else {
    if (gout_dtype == MG_F32) { LD_(bf16_t, float); } else { LD_(bf16_t, bf16_t); }
  }
#undef LD_
#undef L_
  return mg_check_launch("mg_attn_bwd");
}

// ---------------------------------------------------------------------------
// CLIP image-tower input (CLIPLoss.forward, t2i_moe_gan.py:90-94, then the ViT's conv1 patchify): clamp to
// [-1, 1], bilinear resize R x R -> res x res (align_corners=False, PyTorch's source-index rule: src =
// max(0, (dst + 0.5) * R / res - 0.5), neighbour clamped at the edge), and write the unfolded patch rows
// [B * (res/patch)^2, 3 * patch * patch] in (c, kh, kw) order, bf16 -- straight from the generator's NHWC
// (channel-padded) image.  16-B stores of 8 consecutive kw.
// ---------------------------------------------------------------------------
namespace {
// one block per patch row (b, gy, gx): the clamped source window of the patch (at most 2 + P * R / res pixels a
// side, R <= res) is staged in LDS once, then thread (c, kh, 8-wide kw segment) interpolates from LDS
template <typename T, int P>
__global__ void k_clip_patches(const T* __restrict__ img, int R, int ld, int res, bf16_t* __restrict__ out) {
  constexpr int WMAX = P + 2;
  __shared__ float win[3][WMAX][WMAX];
  const int g = res / P;
  const int prow = blockIdx.x, gx = prow % g, gy = (prow / g) % g, b = prow / (g * g);
  const int t = threadIdx.x, sg = t % (P / 8), kh = (t / (P / 8)) % P, c = t / (P * P / 8);
  const float scale = (float)R / (float)res;
  auto src = [&](int d) { return fmaxf(scale * (d + 0.5f) - 0.5f, 0.f); };
  const int ya = (int)src(gy * P), xa = (int)src(gx * P);  // window origin (source indices are monotone)
  const int yb = min((int)src(gy * P + P - 1) + 1, R - 1), xb = min((int)src(gx * P + P - 1) + 1, R - 1);
  const int wh = yb - ya + 1, ww = xb - xa + 1;
  for (int e = t; e < wh * ww; e += blockDim.x) {
    const int yy = e / ww, xx = e - yy * ww;
    const T* px = img + (((int64_t)b * R + ya + yy) * R + xa + xx) * ld;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) win[ch][yy][xx] = fminf(fmaxf(ldf(px, ch), -1.f), 1.f);
  }
  __syncthreads();
  const int y = gy * P + kh;
  const float sy = src(y);
  const int y0 = (int)sy, y1 = y0 + (y0 < R - 1 ? 1 : 0);
  const float ly1 = sy - y0, ly0 = 1.f - ly1;
  const float* w0 = &win[c][y0 - ya][0];
  const float* w1 = &win[c][y1 - ya][0];
  u16x8_t o;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int x = gx * P + sg * 8 + j;
    const float sx = src(x);
    const int x0 = (int)sx, x1 = x0 + (x0 < R - 1 ? 1 : 0);
    const float lx1 = sx - x0, lx0 = 1.f - lx1;
    const float v00 = w0[x0 - xa], v01 = w0[x1 - xa], v10 = w1[x0 - xa], v11 = w1[x1 - xa];
    o[j] = f2bf(ly0 * (lx0 * v00 + lx1 * v01) + ly1 * (lx0 * v10 + lx1 * v11));
  }
  *reinterpret_cast<u16x8_t*>(out + (int64_t)prow * (3 * P * P) + (c * P + kh) * P + sg * 8) = o;
}
}  // namespace

extern "C" int mg_clip_patches(int dtype, const void* img, int B, int R, int ld, int res, int patch, void* out,
                               void* stream) {
  MG_REQUIRE(dtype == MG_F32 || dtype == MG_BF16, "bad dtype");
  MG_REQUIRE(patch == 32, "patch must be 32 (ViT-B/32)");
  MG_REQUIRE(B >= 0 && R >= 1 && R <= res && ld >= 3 && res % patch == 0, "bad clip patch geometry (R <= res)");
  MG_REQUIRE(mg_al16(out), "out must be 16-byte aligned");
  MG_REQUIRE((int64_t)B * (res / patch) * (res / patch) < (1LL << 31) && (int64_t)R * ld < (1LL << 31),
             "too many patches");
  if (B == 0) return MG_OK;
  const int rows = B * (res / patch) * (res / patch);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == MG_F32)
    hipLaunchKernelGGL((k_clip_patches<float, 32>), dim3(rows), dim3(3 * 32 * 32 / 8), 0, st, (const float*)img, R, ld,
                       res, (bf16_t*)out);
  else
    hipLaunchKernelGGL((k_clip_patches<bf16_t, 32>), dim3(rows), dim3(3 * 32 * 32 / 8), 0, st, (const bf16_t*)img, R,
                       ld, res, (bf16_t*)out);
  return mg_check_launch("mg_clip_patches");
}
