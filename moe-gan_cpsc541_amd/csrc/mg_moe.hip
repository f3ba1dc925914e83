// Bayesian router + mixture-of-experts dispatch/combine (t2i_moe_gan.py:265-491).
//
// The router's weight-uncertainty projections are sampled once per forward
// (explicit epsilon, :302-333), then re-associated:
//     logits_raw = [x @ Wf | w @ Wt] @ Wc = x @ (Wf @ Wc[:128]) + (w @ Wt) @ Wc[128:]
// so the per-token work is a C x E product (E experts) instead of C x 128 + 256 x E,
// and the text half is a per-image [B, E] vector (the text rows repeat per image, :456).
// Per token: temperature scale + clamp (:375-381), softmax, clamp, renormalise
// (:384-389), then top-k selection with lowest-index tie-break (:393 / :473).
// k == E reproduces the reference's dense soft training combine (:465-470);
// k == 1 with eval weights reproduces the hard top-1 eval dispatch (:471-483).
// Dispatch builds per-expert position lists deterministically (token order),
// consumed by the grouped expert GEMMs (mg_gemm_grouped) without host syncs.
#include "mg_common.h"

namespace {

MG_DEV float softplusf(float x) { return log1pf(expf(x)); }
MG_DEV float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }

__global__ void k_reparam(const float* __restrict__ mu, const float* __restrict__ rho, const float* __restrict__ eps,
                          int64_t n, float* __restrict__ W) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float m = clampf(mu[i], -10.f, 10.f);
    float r = clampf(rho[i], -8.f, 4.f);
    float sg = clampf(softplusf(r), 1e-6f, 10.f);
    float e = clampf(eps[i], -2.f, 2.f);
    W[i] = m + sg * e;
  }
}

MG_DEV float teff_of(const float* temp, float anneal) { return fminf(fmaxf(temp[0] * anneal, 0.5f), 5.f); }

constexpr int RTEAM = 8;  // lanes per token in the router's softmax / top-k

// Softmax / top-k of one token spread over its team of RTEAM lanes: lane tl owns experts tl, tl + 8, ... and
// holds their raw logits x . Wfc in araw[]; the team reduces max / sums / arg-max with shuffles, so probs and
// zlog leave as 32-byte runs per token instead of one lane's scalar stores (the team-serial epilogue ran at
// ~9 % of HBM).  Every lane of the wave calls it (shuffles); ok = false for a team past the last token.
template <int E>
MG_DEV void router_token(const float* araw, bool ok, int t, int tl, int lgHW, const float* __restrict__ Lt,
                         const float* __restrict__ temp, float anneal, int k, int eval_mode,
                         float* __restrict__ probs, float* __restrict__ zlog, int* __restrict__ topi,
                         float* __restrict__ gate) {
  constexpr int TEAM = RTEAM;
  constexpr int NE = E >= TEAM ? E / TEAM : 1;
  const int b = (ok ? t : 0) >> lgHW;
  const float te = teff_of(temp, anneal);
  float z[NE], p[NE];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < NE; ++j) {
    const int e = tl + TEAM * j;
    const bool own = e < E;
    z[j] = own && ok ? (araw[j] + Lt[(int64_t)b * E + e]) / te : 0.f;
    p[j] = own ? clampf(z[j], -20.f, 20.f) : -INFINITY;
    mx = fmaxf(mx, p[j]);
  }
  mx = fmaxf(mx, __shfl_xor(mx, 1, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 2, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 4, 64));
  float sm = 0.f;
#pragma unroll
  for (int j = 0; j < NE; ++j) {
    p[j] = tl + TEAM * j < E ? expf(p[j] - mx) : 0.f;
    sm += p[j];
  }
  sm += __shfl_xor(sm, 1, 64);
  sm += __shfl_xor(sm, 2, 64);
  sm += __shfl_xor(sm, 4, 64);
  float s2 = 0.f;
#pragma unroll
  for (int j = 0; j < NE; ++j) {
    p[j] = tl + TEAM * j < E ? clampf(p[j] / sm, 1e-6f, 1.f) : 0.f;
    s2 += p[j];
  }
  s2 += __shfl_xor(s2, 1, 64);
  s2 += __shfl_xor(s2, 2, 64);
  s2 += __shfl_xor(s2, 4, 64);
#pragma unroll
  for (int j = 0; j < NE; ++j) p[j] = p[j] / s2;
  // top-k, lowest index first among equals: team arg-max k times (rounds unrolled over E so every lane keeps
  // the picks it will store in registers: pick r goes to lane r % TEAM)
  constexpr int NK = (E + TEAM - 1) / TEAM;
  unsigned used = 0u;  // bit j: this lane's j-th expert taken
  float gsum = 0.f, mg[NK];
  int g0 = 0, mt[NK];
#pragma unroll
  for (int j = 0; j < NK; ++j) {
    mg[j] = 0.f;
    mt[j] = 0;
  }
#pragma unroll
  for (int r = 0; r < E; ++r) {
    if (r < k) {
      float bv = -INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int j = 0; j < NE; ++j) {
        const int e = tl + TEAM * j;
        const float pv = p[j] == p[j] ? p[j] : -INFINITY;  // NaN ranks lowest: the pick is always an expert
        if (e < E && !((used >> j) & 1u) && (pv > bv || (pv == bv && e < bi))) {
          bv = pv;
          bi = e;
        }
      }
#pragma unroll
      for (int o = 1; o < TEAM; o <<= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ov > bv || (ov == bv && oi < bi)) {
          bv = ov;
          bi = oi;
        }
      }
      if (bi < E && (bi & (TEAM - 1)) == tl) used |= 1u << (bi / TEAM);
      if (r == 0) g0 = bi;
      if ((r & (TEAM - 1)) == tl) {
        mt[r / TEAM] = bi < E ? bi : 0;
        mg[r / TEAM] = bv;
      }
      gsum += bv;
    }
  }
  if (ok) {
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      const int e = tl + TEAM * j;
      if (e < E) {
        zlog[(int64_t)t * E + e] = z[j];
        probs[(int64_t)t * E + e] = eval_mode ? (e == g0 ? 1.f : 0.f) : p[j];
      }
    }
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      const int r = tl + TEAM * j;
      if (r < k) {
        topi[(int64_t)t * k + r] = mt[j];
        gate[(int64_t)t * k + r] = eval_mode ? 1.f : (k == E ? mg[j] : mg[j] / gsum);
      }
    }
  }
}

// TEAM lanes per token; block = 256 threads = 256/TEAM tokens
template <typename T, int E>
__global__ void k_router_fwd(const T* __restrict__ tok, int64_t ld, int Tn, int C, const float* __restrict__ Wfc,
                             const float* __restrict__ Lt, int lgHW, const float* __restrict__ temp, float anneal,
                             int k, int eval_mode, float* __restrict__ probs, float* __restrict__ zlog,
                             int* __restrict__ topi, float* __restrict__ gate) {
  constexpr int TEAM = RTEAM;
  constexpr int VEC = VecOf<T>::N;
  // Wfc [C][E] in LDS with element e of row c at (e + c / VEC) mod E: the 8 lanes of a team read rows
  // VEC apart, which the rotation puts on distinct banks
  extern __shared__ float wsm[];
  for (int i = threadIdx.x; i < C * E; i += blockDim.x) {
    const int c = i / E, e = i - c * E;
    wsm[c * E + ((e + c / VEC) & (E - 1))] = Wfc[i];
  }
  __syncthreads();
  int team = threadIdx.x / TEAM, tl = threadIdx.x % TEAM;
  // grid-stride over tokens: each block stages Wfc once for many tokens
  for (int t = blockIdx.x * (blockDim.x / TEAM) + team; t - team < Tn; t += gridDim.x * (blockDim.x / TEAM)) {
  bool ok = t < Tn;
  float acc[E];
#pragma unroll
  for (int e = 0; e < E; ++e) acc[e] = 0.f;
  if (ok) {
    for (int c0 = tl * VEC; c0 < C; c0 += TEAM * VEC) {
      auto v = *reinterpret_cast<const typename VecOf<T>::type*>(tok + (int64_t)t * ld + c0);
      const int rot = c0 / VEC;
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        float x;
        if constexpr (sizeof(T) == 4) x = v[j]; else x = bf2f(v[j]);
        const float* wr = wsm + (c0 + j) * E;
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] += x * wr[(e + rot) & (E - 1)];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    acc[e] += __shfl_xor(acc[e], 1, 64);
    acc[e] += __shfl_xor(acc[e], 2, 64);
    acc[e] += __shfl_xor(acc[e], 4, 64);
  }
  constexpr int NE = E >= TEAM ? E / TEAM : 1;
  float araw[NE];
#pragma unroll
  for (int j = 0; j < NE; ++j) {
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < E; ++q)
      if (q == tl + TEAM * j) v = acc[q];
    araw[j] = v;
  }
  router_token<E>(araw, ok, t, tl, lgHW, Lt, temp, anneal, k, eval_mode, probs, zlog, topi, gate);
  }  // token loop
}

// Router logits on the matrix cores (bf16 tokens, E >= 8, C = 128 / 256 / 384 / 512): z[T x E] = tok . Wfc with
// v_mfma_f32_16x16x32_bf16, Wfc split into bf16 hi + lo halves (w = hi + lo + O(2^-18 |w|), below the fp32
// rounding of a C-term sum; tokens are bf16 already).  A block takes nt 16-token tiles; its 4 waves split the
// channels in quarters, each holding its quarter of Wfc as B fragments in registers (read straight from L2, no
// LDS staging) and loading every A fragment it needs up front, so a block is one load latency, a few MFMAs,
// one LDS fold of the 4 partial tiles (fixed wave order) and the team softmax / top-k.  The lane-FMA team kernel
// above spends one FMA plus one LDS read per token-channel-expert and, at few tokens per layer, is latency bound
// (C5: 40 / 33 / 53 us at 4096 / 16384 / 65536 tokens).
constexpr int RNT = 4;  // most 16-token tiles per block: NT = 4 / NKS (the A fragments a lane holds)
template <int E, int NKS>
__global__ __launch_bounds__(256) void k_router_fwd_mfma(const bf16_t* __restrict__ tok, int64_t ld, int Tn, int C,
                                                         int nt, const float* __restrict__ Wfc,
                                                         const float* __restrict__ Lt, int lgHW,
                                                         const float* __restrict__ temp, float anneal, int k,
                                                         int eval_mode, float* __restrict__ probs,
                                                         float* __restrict__ zlog, int* __restrict__ topi,
                                                         float* __restrict__ gate) {
  constexpr int EP = E < 16 ? 16 : E;  // experts padded to the 16-column MFMA tile
  constexpr int NH = EP / 16;
  constexpr int ZP = EP + 1;
  constexpr int NT = RNT / NKS;
  constexpr int ZW = NT * 16 * ZP;  // one wave's partial logits
  __shared__ float zpart[4 * ZW];   // [wave][token of the block][expert]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int fr = lane & 15, fq = lane >> 4;
  const int tb0 = blockIdx.x * nt * 16;
  const int c0 = wave * (NKS * 32) + fq * 8;  // this wave's channel quarter (C = 128 NKS)
  // A fragments, all loaded up front; rows past the last token re-read it
  bf16x8_t af[NT][NKS];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int st = 0; st < NKS; ++st) {
      const int64_t row = min(tb0 + j * 16 + fr, Tn - 1);
      af[j][st] = __builtin_bit_cast(bf16x8_t, j < nt ? *reinterpret_cast<const u16x8_t*>(tok + row * ld + c0 + st * 32)
                                                      : u16x8_t{0, 0, 0, 0, 0, 0, 0, 0});
    }
  // B fragments of the quarter: expert h * 16 + fr, channels c0 + 32 st .. + 8, as bf16 hi / lo
  bf16x8_t bh[NKS][NH], bl[NKS][NH];
#pragma unroll
  for (int st = 0; st < NKS; ++st)
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const int e = h * 16 + fr;
      float w[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) w[q] = e < E ? Wfc[(int64_t)(c0 + st * 32 + q) * E + e] : 0.f;
      u16x8_t hv, lv;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        hv[q] = f2bf(w[q]);
        lv[q] = f2bf(w[q] - bf2f(hv[q]));
      }
      bh[st][h] = __builtin_bit_cast(bf16x8_t, hv);
      bl[st][h] = __builtin_bit_cast(bf16x8_t, lv);
    }
  float* zw = zpart + wave * ZW;
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    if (j < nt) {  // block-uniform
      f32x4_t acc[NH];
#pragma unroll
      for (int h = 0; h < NH; ++h) acc[h] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < NKS; ++st)
#pragma unroll
        for (int h = 0; h < NH; ++h) {
          acc[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[j][st], bl[st][h], acc[h], 0, 0, 0);
          acc[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[j][st], bh[st][h], acc[h], 0, 0, 0);
        }
      // D[token fq*4 + r][expert h*16 + fr]
#pragma unroll
      for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) zw[(j * 16 + fq * 4 + r) * ZP + h * 16 + fr] = acc[h][r];
    }
  }
  __syncthreads();
  // teams of 8 lanes, 32 tokens per pass (a pass's active teams fill whole waves: nt * 16 is a multiple of 16);
  // the four channel quarters fold in wave order
  const int team = threadIdx.x / RTEAM, tl = threadIdx.x % RTEAM;
  constexpr int NE = E / RTEAM;
  for (int row = team; row < nt * 16; row += 256 / RTEAM) {
    const int t = tb0 + row;
    float araw[NE];
#pragma unroll
    for (int q = 0; q < NE; ++q) {
      const int o = row * ZP + tl + RTEAM * q;
      araw[q] = ((zpart[o] + zpart[ZW + o]) + zpart[2 * ZW + o]) + zpart[3 * ZW + o];
    }
    router_token<E>(araw, t < Tn, t, tl, lgHW, Lt, temp, anneal, k, eval_mode, probs, zlog, topi, gate);
  }
}

// ---- dispatch: deterministic per-expert position lists ----
constexpr int DCH = 1024;  // assignments per block (C2 16x16 layer: 128 blocks)
__global__ void k_disp_count(const int* __restrict__ topi, int n, int E, int* __restrict__ blk_counts) {
  extern __shared__ int cnt[];
  for (int e = threadIdx.x; e < E; e += blockDim.x) cnt[e] = 0;
  __syncthreads();
  int a0 = blockIdx.x * DCH, a1 = min(n, a0 + DCH);
  for (int a = a0 + threadIdx.x; a < a1; a += blockDim.x) atomicAdd(&cnt[topi[a]], 1);
  __syncthreads();
  for (int e = threadIdx.x; e < E; e += blockDim.x) blk_counts[blockIdx.x * E + e] = cnt[e];
}

__global__ void k_disp_scan(int* __restrict__ blk_counts, int nblk, int E, int bm, int* __restrict__ row_off,
                            int* __restrict__ tile_off) {
  // single block; thread e scans expert e over blocks (in place -> block bases relative to expert start)
  __shared__ int tot[1024];
  int e = threadIdx.x;
  if (e < E) {
    int s = 0;
    for (int b = 0; b < nblk; ++b) {
      int c = blk_counts[b * E + e];
      blk_counts[b * E + e] = s;
      s += c;
    }
    tot[e] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int r = 0, tl = 0;
    for (int i = 0; i < E; ++i) {
      row_off[i] = r;
      tile_off[i] = tl;
      r += tot[i];
      tl += (tot[i] + bm - 1) / bm;
    }
    row_off[E] = r;
    tile_off[E] = tl;
  }
}

// Parallel form of k_disp_scan for nblk * E <= 16384: the block counts are staged in LDS, 1024 / E lanes per expert
// sum contiguous runs of blocks, the E expert threads scan those run sums, and every lane writes its run's
// exclusive bases back (same values as the serial scan).
__global__ __launch_bounds__(1024) void k_disp_scan_par(int* __restrict__ blk_counts, int nblk, int E, int bm,
                                                        int* __restrict__ row_off, int* __restrict__ tile_off) {
  extern __shared__ int sm[];  // [nblk * E] counts | [1024] run sums | [32] expert totals
  const int n = nblk * E, tid = threadIdx.x;
  int* run = sm + n;
  int* tot = run + 1024;
  for (int i = tid; i < n; i += 1024) sm[i] = blk_counts[i];
  __syncthreads();
  const int P = 1024 / E, e = tid % E, part = tid / E;
  const int chunk = (nblk + P - 1) / P, b0 = part * chunk, b1 = min(nblk, b0 + chunk);
  int s = 0;
  for (int b = b0; b < b1; ++b) s += sm[b * E + e];
  run[part * E + e] = s;
  __syncthreads();
  if (tid < E) {
    int acc = 0;
    for (int q = 0; q < P; ++q) {
      const int c = run[q * E + tid];
      run[q * E + tid] = acc;
      acc += c;
    }
    tot[tid] = acc;
  }
  __syncthreads();
  int base = run[part * E + e];
  for (int b = b0; b < b1; ++b) {
    const int c = sm[b * E + e];
    blk_counts[b * E + e] = base;
    base += c;
  }
  if (tid == 0) {
    int r = 0, tl = 0;
    for (int i = 0; i < E; ++i) {
      row_off[i] = r;
      tile_off[i] = tl;
      r += tot[i];
      tl += (tot[i] + bm - 1) / bm;
    }
    row_off[E] = r;
    tile_off[E] = tl;
  }
}

// Positions of a block's DCH assignments in the expert-sorted order, in assignment order within each expert (the
// same order as a serial pass).  The block walks its chunk in DCH / 256 rounds of 256 consecutive assignments (one
// per thread); per round and expert, a wave ballot gives the wave's count (popcount) and each lane's rank among
// the wave's lanes of that expert (mbcnt) -- a few instructions per expert, no per-thread E-wide scans.  One
// thread per expert then turns the (round, wave) counts into exclusive bases in assignment order.
template <int E>
__global__ __launch_bounds__(256) void k_disp_scatter(const int* __restrict__ topi, const float* __restrict__ gate,
                                                      int n, const int* __restrict__ blk_base,
                                                      const int* __restrict__ row_off, int* __restrict__ perm,
                                                      int* __restrict__ pos_of, float* __restrict__ gate_pos) {
  constexpr int R = DCH / 256;
  __shared__ int wc[R * 4][E];  // count of expert e in (round r, wave w); then its exclusive base
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int a0 = blockIdx.x * DCH;
  // every round's assignment into registers first (independent loads in flight)
  int ex_r[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int a = a0 + r * 256 + (int)threadIdx.x;
    ex_r[r] = a < n ? topi[a] : -1;
  }
  int rk[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    int rank = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const uint64_t m = __ballot(ex_r[r] == e);
      if (ex_r[r] == e)
        rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (lane == 0) wc[r * 4 + wid][e] = __popcll(m);
    }
    rk[r] = rank;
  }
  __syncthreads();
  if ((int)threadIdx.x < E) {  // (round, wave) order = assignment order
    const int e = threadIdx.x;
    int base = row_off[e] + blk_base[blockIdx.x * E + e];
    for (int q = 0; q < R * 4; ++q) {
      const int c = wc[q][e];
      wc[q][e] = base;
      base += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int a = a0 + r * 256 + (int)threadIdx.x;
    const int ex = ex_r[r];
    if (a < n && (unsigned)ex < (unsigned)E) {
      const int pos = wc[r * 4 + wid][ex] + rk[r];
      perm[pos] = a;
      pos_of[a] = pos;
      gate_pos[pos] = gate[a];
    }
  }
}

// k_disp_scatter with the block-count scan folded in (one launch less per dispatch, ~5 us): every block sums the
// per-block counts of the blocks before it (its bases) and of all blocks (the expert totals -> row offsets) from
// blk_counts, which k_disp_count left in L2; block 0 also writes row_off / tile_off.  Same positions as the
// three-kernel form (exclusive prefixes in block order, integer sums).
template <int E>
__global__ __launch_bounds__(256) void k_disp_scatter_scan(const int* __restrict__ topi, const float* __restrict__ gate,
                                                           int n, int nblk, int bm, const int* __restrict__ blk_counts,
                                                           int* __restrict__ row_off, int* __restrict__ tile_off,
                                                           int* __restrict__ perm, int* __restrict__ pos_of,
                                                           float* __restrict__ gate_pos) {
  constexpr int R = DCH / 256, P = 256 / E;
  __shared__ int wc[R * 4][E];
  __shared__ int red_pre[256], red_tot[256];
  __shared__ int tot_sh[E];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int a0 = blockIdx.x * DCH;
  int ex_r[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int a = a0 + r * 256 + tid;
    ex_r[r] = a < n ? topi[a] : -1;
  }
  {  // thread (q, e): the counts of expert e in blocks q, q + P, ... (before this block, and in all)
    const int e = tid % E, q = tid / E;
    int pre = 0, tot = 0;
    for (int bb = q; bb < nblk; bb += P) {
      const int c = blk_counts[bb * E + e];
      tot += c;
      pre += bb < (int)blockIdx.x ? c : 0;
    }
    red_pre[tid] = pre;
    red_tot[tid] = tot;
  }
  int rk[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    int rank = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const uint64_t m = __ballot(ex_r[r] == e);
      if (ex_r[r] == e)
        rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (lane == 0) wc[r * 4 + wid][e] = __popcll(m);
    }
    rk[r] = rank;
  }
  __syncthreads();
  if (tid < E) {
    int t = 0;
    for (int q = 0; q < P; ++q) t += red_tot[q * E + tid];
    tot_sh[tid] = t;
  }
  __syncthreads();
  if (tid < E) {  // (round, wave) order = assignment order
    const int e = tid;
    int base = 0;
    for (int e2 = 0; e2 < e; ++e2) base += tot_sh[e2];
    for (int q = 0; q < P; ++q) base += red_pre[q * E + e];
    for (int q = 0; q < R * 4; ++q) {
      const int c = wc[q][e];
      wc[q][e] = base;
      base += c;
    }
  }
  if (blockIdx.x == 0 && tid == 0) {
    int r = 0, tl = 0;
    for (int i = 0; i < E; ++i) {
      row_off[i] = r;
      tile_off[i] = tl;
      r += tot_sh[i];
      tl += (tot_sh[i] + bm - 1) / bm;
    }
    row_off[E] = r;
    tile_off[E] = tl;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int a = a0 + r * 256 + tid;
    const int ex = ex_r[r];
    if (a < n && (unsigned)ex < (unsigned)E) {
      const int pos = wc[r * 4 + wid][ex] + rk[r];
      perm[pos] = a;
      pos_of[a] = pos;
      gate_pos[pos] = gate[a];
    }
  }
}

// out[t] = resid[t] + sum_j gate[t,j] * Y[pos_of[t*k+j]]
template <typename T>
__global__ void k_combine(const T* __restrict__ Y, int64_t ldy, const int* __restrict__ pos_of,
                          const float* __restrict__ gate, int Tn, int k, int C, const T* __restrict__ resid,
                          int64_t ldr, T* __restrict__ out, int64_t ldo) {
  int64_t n = (int64_t)Tn * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int t = (int)(i / C), c = (int)(i - (int64_t)t * C);
    float s = 0.f;
    for (int j = 0; j < k; ++j) {
      int a = t * k + j;
      s += gate[a] * ldf(Y, (int64_t)pos_of[a] * ldy + c);
    }
    if (resid) s = ldf(resid, (int64_t)t * ldr + c) + s;
    stf(out, (int64_t)t * ldo + c, s);
  }
}

// 8-channel vector form of k_combine (same arithmetic order).  XS: also the next modulated conv's input x * s
// (t2i_moe_gan.py:158-161, AttentionBlock.proj_out), s [B, C] one style row per image of HW tokens, from the
// stored (rounded) out -- the bytes k_scale_bc would write, without re-reading out
template <typename T, bool XS = false>
__global__ __launch_bounds__(256) void k_combine_v(const T* __restrict__ Y, int64_t ldy, const int* __restrict__ pos_of,
                                                   const float* __restrict__ gate, int Tn, int k, int C,
                                                   const T* __restrict__ resid, int64_t ldr, T* __restrict__ out,
                                                   int64_t ldo, const float* __restrict__ sty = nullptr,
                                                   int64_t ld_sty = 0, int lg_hw = 0, T* __restrict__ xs = nullptr,
                                                   int64_t ldxs = 0) {
  const int cv = C >> 3;
  const int n = Tn * cv;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int t = i / cv, c = (i - t * cv) * 8;
    float s[8], y[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) s[q] = 0.f;
    for (int j = 0; j < k; ++j) {
      const int a = t * k + j;
      const float g = gate[a];
      ld8(Y + (int64_t)pos_of[a] * ldy + c, y);
#pragma unroll
      for (int q = 0; q < 8; ++q) s[q] += g * y[q];
    }
    if (resid) {
      ld8(resid + (int64_t)t * ldr + c, y);
#pragma unroll
      for (int q = 0; q < 8; ++q) s[q] = y[q] + s[q];
    }
    st8(out + (int64_t)t * ldo + c, s);
    if constexpr (XS) {
      float r[8];
      if constexpr (sizeof(T) == 2) {  // the product of the stored bf16 value, as k_scale_bc forms it
#pragma unroll
        for (int q = 0; q < 8; ++q) r[q] = bf2f(f2bf(s[q]));
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) r[q] = s[q];
      }
      ld8(sty + (int64_t)(t >> lg_hw) * ld_sty + c, y);
#pragma unroll
      for (int q = 0; q < 8; ++q) r[q] *= y[q];
      st8(xs + (int64_t)t * ldxs + c, r);
    }
  }
}

// 8-channel vector form of k_token_grad; Wfc [C, E] staged in LDS (dynamic, C * E floats), the token's
// g_raw row read as 16-B vectors
template <typename T, typename TO, int E>
__global__ __launch_bounds__(256) void k_token_grad_v(const T* __restrict__ gX, int64_t ldx,
                                                      const int* __restrict__ pos_of, int Tn, int k, int C,
                                                      const float* __restrict__ g_raw, const float* __restrict__ Wfc,
                                                      TO* __restrict__ out, int64_t ldo) {
  extern __shared__ float sW[];  // [E][C]: a lane's 8 channels are contiguous (16-B reads, no bank conflicts)
  // staged in destination order (consecutive lanes, consecutive words: the source-order loop put a lane group's
  // stores C words apart, one bank: 8-way conflicts); the strided global reads hit L2
  for (int j = threadIdx.x; j < C * E; j += 256) sW[j] = Wfc[(j % C) * E + j / C];
  __syncthreads();
  const int cv = C >> 3;
  const int n = Tn * cv;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int t = i / cv, c = (i - t * cv) * 8;
    float s[8], v[8], gr[E];
#pragma unroll
    for (int q = 0; q < 8; ++q) s[q] = 0.f;
#pragma unroll
    for (int e = 0; e < E; e += 4) {
      const f32x4_t g4 = *reinterpret_cast<const f32x4_t*>(g_raw + (int64_t)t * E + e);
      gr[e] = g4[0]; gr[e + 1] = g4[1]; gr[e + 2] = g4[2]; gr[e + 3] = g4[3];
    }
    if (gX)
      for (int j = 0; j < k; ++j) {
        ld8(gX + (int64_t)pos_of[t * k + j] * ldx + c, v);
#pragma unroll
        for (int q = 0; q < 8; ++q) s[q] += v[q];
      }
    // a lane's two 16-B weight reads, 32 B apart across lanes, put lanes l and l + 8 of a ds_read_b128 lane group on
    // one bank quad; lanes with bit 3 set read their second half first (both halves land, order only)
    const int hsw = (threadIdx.x >> 3) & 1;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const f32x4_t wa = *reinterpret_cast<const f32x4_t*>(sW + e * C + c + 4 * hsw);
      const f32x4_t wb = *reinterpret_cast<const f32x4_t*>(sW + e * C + c + 4 - 4 * hsw);
      const f32x4_t w0 = hsw ? wb : wa, w1 = hsw ? wa : wb;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        s[q] += gr[e] * w0[q];
        s[q + 4] += gr[e] * w1[q];
      }
    }
    st8(out + (int64_t)t * ldo + c, s);
  }
}

// Token gradient with the router term on the matrix cores: out[t] = sum_j gX[pos_of[t*k+j]] + g_raw[t] . Wfc^T.
// The [16 x E] . [E x C] products run as v_mfma_f32_16x16x32_bf16 with both fp32 operands split into bf16 hi + lo
// (three products, lo * lo dropped: relative error ~2^-16 per term); experts past E (E = 8, 16) are zero k-rows.
// A block takes nt 16-token tiles; wave w owns output channels [16 NB w, 16 NB (w + 1)) and holds their Wfc
// fragments in registers (straight from L2, no staging); the product tile goes through LDS ([16 nt][C + 4] fp32)
// to a coalesced pass that adds the k gathered expert-output gradients and stores 16-B vectors.  The lane-FMA
// kernel above spends 2 LDS reads + 8 FMAs per token-8-channel-expert and staged C x E floats per block
// (C5: 48 - 57 us per call against ~4 - 18 us of HBM traffic).
template <typename T, typename TO, int E, int NB>
__global__ __launch_bounds__(256) void k_token_grad_mfma(const T* __restrict__ gX, int64_t ldx,
                                                         const int* __restrict__ pos_of, int Tn, int k, int nt,
                                                         const float* __restrict__ g_raw,
                                                         const float* __restrict__ Wfc, TO* __restrict__ out,
                                                         int64_t ldo) {
  constexpr int C = 64 * NB;
  constexpr int CP = C + 4;
  extern __shared__ __align__(16) float gtile[];  // [nt * 16][CP]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int fr = lane & 15, fq = lane >> 4;
  const bool kin = fq * 8 < E;  // this lane's 8 k-rows (experts) exist
  const int tb0 = blockIdx.x * nt * 16;
  auto split = [](const float* w, bf16x8_t& hi, bf16x8_t& lo) {
    u16x8_t hv, lv;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      hv[q] = f2bf(w[q]);
      lv[q] = f2bf(w[q] - bf2f(hv[q]));
    }
    hi = __builtin_bit_cast(bf16x8_t, hv);
    lo = __builtin_bit_cast(bf16x8_t, lv);
  };
  // B fragments: Wfc^T[e][c] for channel c = 16 (NB w + b) + fr, experts fq*8 .. +8 (a Wfc row run)
  bf16x8_t bh[NB], bl[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int c = (wave * NB + b) * 16 + fr;
    float w[8];
    if (kin) {
      const f32x4_t w0 = *reinterpret_cast<const f32x4_t*>(Wfc + (int64_t)c * E + fq * 8);
      const f32x4_t w1 = *reinterpret_cast<const f32x4_t*>(Wfc + (int64_t)c * E + fq * 8 + 4);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        w[q] = w0[q];
        w[q + 4] = w1[q];
      }
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) w[q] = 0.f;
    }
    split(w, bh[b], bl[b]);
  }
  for (int j = 0; j < nt; ++j) {
    const int64_t row = min(tb0 + j * 16 + fr, Tn - 1);  // rows past the last token: never stored
    float a[8];
    if (kin) {
      const f32x4_t a0 = *reinterpret_cast<const f32x4_t*>(g_raw + row * E + fq * 8);
      const f32x4_t a1 = *reinterpret_cast<const f32x4_t*>(g_raw + row * E + fq * 8 + 4);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        a[q] = a0[q];
        a[q + 4] = a1[q];
      }
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) a[q] = 0.f;
    }
    bf16x8_t ah, al;
    split(a, ah, al);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      f32x4_t acc = f32x4_t{0.f, 0.f, 0.f, 0.f};
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[b], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[b], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[b], acc, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) gtile[(j * 16 + fq * 4 + r) * CP + (wave * NB + b) * 16 + fr] = acc[r];
    }
  }
  __syncthreads();
  constexpr int CV = C / 8;
  const int n = nt * 16 * CV;
  for (int i = threadIdx.x; i < n; i += 256) {
    const int r = i / CV, c = (i - r * CV) * 8, t = tb0 + r;
    if (t >= Tn) continue;
    float sv[8], v[8];
    const f32x4_t s0 = *reinterpret_cast<const f32x4_t*>(gtile + r * CP + c);
    const f32x4_t s1 = *reinterpret_cast<const f32x4_t*>(gtile + r * CP + c + 4);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      sv[q] = s0[q];
      sv[q + 4] = s1[q];
    }
    if (gX)
      for (int j = 0; j < k; ++j) {
        ld8(gX + (int64_t)pos_of[t * k + j] * ldx + c, v);
#pragma unroll
        for (int q = 0; q < 8; ++q) sv[q] += v[q];
      }
    st8(out + (int64_t)t * ldo + c, sv);
  }
}

// g_gate[a] = <gout[t], Y[pos_of[a]]>, one wave per assignment
template <typename T, typename TG>
__global__ void k_gate_grad(const TG* __restrict__ gout, int64_t ldg, const T* __restrict__ Y, int64_t ldy,
                            const int* __restrict__ pos_of, int n, int k, int C, float* __restrict__ g_gate) {
  // 8 lanes per assignment with 16-B vectors (one wave per assignment issued 2-byte loads and spent most of
  // its time launching: 131072 waves for the 16x16 block)
  const int a = blockIdx.x * (blockDim.x >> 3) + (threadIdx.x >> 3), tl = threadIdx.x & 7;
  const bool ok = a < n;
  float s = 0.f;
  if (ok) {
    const int t = a / k;
    const int64_t pr = (int64_t)pos_of[a] * ldy, pg = (int64_t)t * ldg;
    for (int c = tl * 8; c < C; c += 64) {
      float g[8], y[8];
      ld8(gout + pg + c, g);
      ld8(Y + pr + c, y);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += g[j] * y[j];
    }
  }
  s += __shfl_xor(s, 1, 64);
  s += __shfl_xor(s, 2, 64);
  s += __shfl_xor(s, 4, 64);
  if (ok && tl == 0) g_gate[a] = s;
}

// per-token router backward: (g_gate, balance coefficients) -> g_raw [T, E], the per-image sums gsum [B, E] and
// one temperature-gradient partial per block (tpart; a rows fold, mg_fold.hip, adds them to the parameter gradient).
// Every reduction runs in a fixed order (segmented butterflies inside a wave, waves of one image folded in wave
// order, block partials folded by one block), so the results are bit-identical run to run: the image's tokens are
// contiguous, an image of HW <= 64 tokens lies inside one wave and one of 128 / 256 tokens inside one block.
template <int E>
__global__ __launch_bounds__(256) void k_router_bwd(const float* __restrict__ probs, const float* __restrict__ zlog,
                             const int* __restrict__ topi, const float* __restrict__ gate,
                             const float* __restrict__ g_gate, const float* __restrict__ g_probs,
                             const float* __restrict__ g_logits,
                             const float* __restrict__ coef, int Tn, int k, int lgHW, const float* __restrict__ temp,
                             float anneal, float* __restrict__ g_raw, float* __restrict__ gsum,
                             float* __restrict__ tpart) {
  __shared__ float red[4 * E];
  __shared__ float tred[4];
  const int t0 = blockIdx.x * blockDim.x;
  const int t = t0 + threadIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float te = teff_of(temp, anneal);
  float gt_part = 0.f;
  float grv[E];
#pragma unroll
  for (int e = 0; e < E; ++e) grv[e] = 0.f;
  if (t < Tn) {
    float p[E], gp[E], z[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      p[e] = probs[(int64_t)t * E + e];
      z[e] = zlog[(int64_t)t * E + e];
      gp[e] = (coef ? coef[e] : 0.f) + (g_probs ? g_probs[(int64_t)t * E + e] : 0.f);
    }
    if (g_gate) {
      if (k == E) {
        for (int j = 0; j < k; ++j) {
          int ex = topi[(int64_t)t * k + j];
#pragma unroll
          for (int e = 0; e < E; ++e)
            if (e == ex) gp[e] += g_gate[(int64_t)t * k + j];
        }
      } else {
        float S = 0.f, dot = 0.f;
        for (int j = 0; j < k; ++j) {
          int ex = topi[(int64_t)t * k + j];
#pragma unroll
          for (int e = 0; e < E; ++e)
            if (e == ex) S += p[e];
          dot += g_gate[(int64_t)t * k + j] * gate[(int64_t)t * k + j];
        }
        for (int j = 0; j < k; ++j) {
          int ex = topi[(int64_t)t * k + j];
          float v = (g_gate[(int64_t)t * k + j] - dot) / S;
#pragma unroll
          for (int e = 0; e < E; ++e)
            if (e == ex) gp[e] += v;
        }
      }
    }
    // recompute softmax s and clamped q
    float l[E], s[E], q[E];
    float mx = -INFINITY;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      l[e] = fminf(fmaxf(z[e], -20.f), 20.f);
      mx = fmaxf(mx, l[e]);
    }
    float den = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      s[e] = expf(l[e] - mx);
      den += s[e];
    }
    float Sq = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      s[e] /= den;
      q[e] = fminf(fmaxf(s[e], 1e-6f), 1.f);
      Sq += q[e];
    }
    // p = q / Sq
    float d1 = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) d1 += gp[e] * (q[e] / Sq);
    float gs_[E];
    float d2 = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      float gq = (gp[e] - d1) / Sq;
      gs_[e] = (s[e] >= 1e-6f && s[e] <= 1.f) ? gq : 0.f;
      d2 += gs_[e] * s[e];
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
      float gl = s[e] * (gs_[e] - d2);
      if (g_logits) gl += g_logits[(int64_t)t * E + e];  // the router's second output, logits (:378-381)
      gl = (z[e] >= -20.f && z[e] <= 20.f) ? gl : 0.f;
      gt_part += -gl * z[e] / te;
      grv[e] = gl / te;
      g_raw[(int64_t)t * E + e] = grv[e];
    }
  }
  // per-image sums: butterfly over the image's lanes (all of the wave when the image spans waves)
  const int seg = lgHW >= 6 ? 64 : (1 << lgHW);
#pragma unroll
  for (int e = 0; e < E; ++e)
    for (int o = 1; o < seg; o <<= 1) grv[e] += __shfl_xor(grv[e], o, 64);
  if (lgHW <= 6) {
    if ((lane & (seg - 1)) == 0 && t < Tn) {
#pragma unroll
      for (int e = 0; e < E; ++e) gsum[(int64_t)(t >> lgHW) * E + e] = grv[e];
    }
  } else if (lane == 0) {
#pragma unroll
    for (int e = 0; e < E; ++e) red[wave * E + e] = grv[e];
  }
  gt_part = wave_sum(gt_part);
  if (lane == 0) tred[wave] = gt_part;
  __syncthreads();
  if (lgHW > 6) {  // 128 / 256 tokens per image: 2 / 4 waves of this block, folded in wave order
    const int wpi = 1 << (lgHW - 6);
    const int nimg = (min(Tn, t0 + (int)blockDim.x) - t0 + (1 << lgHW) - 1) >> lgHW;
    for (int i = threadIdx.x; i < nimg * E; i += blockDim.x) {
      const int bl = i / E, e = i - bl * E;
      float v = 0.f;
      for (int w = bl * wpi; w < bl * wpi + wpi; ++w) v += red[w * E + e];
      gsum[(int64_t)((t0 >> lgHW) + bl) * E + e] = v;
    }
  }
  if (threadIdx.x == 0 && tpart) {
    float tt = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) tt += tred[i];
    float raw = temp[0] * anneal;
    tpart[blockIdx.x] = (raw >= 0.5f && raw <= 5.f) ? tt * anneal : 0.f;
  }
}


MG_DEV float team_sum(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  return v;
}

// Team form of k_router_bwd (E >= 8, the same math): RTEAM lanes per token, lane tl owning experts tl, tl + 8, ...,
// the per-token reductions over experts as team butterflies.  A block of NT teams (32 / 64 / 128: one team per
// token up to 128-token images) covers TB = max(NT, HW) consecutive tokens, each team TB / NT of them in turn, so
// every image lies inside one block;
// per-image sums and the block's temperature partial fold the team partials in team order (fixed order:
// bit-identical run to run).  The thread-per-token kernel ran 16 blocks for the 4096 tokens of a 4x4 layer and
// read each token's rows as scattered 4-B loads (C5: 39 us per call); here a wave reads 8 tokens' rows whole.
template <int E, int NT>
__global__ __launch_bounds__(NT * RTEAM) void k_router_bwd_team(const float* __restrict__ probs,
                                                         const float* __restrict__ zlog, const int* __restrict__ topi,
                                                         const float* __restrict__ gate,
                                                         const float* __restrict__ g_gate,
                                                         const float* __restrict__ g_probs,
                                                         const float* __restrict__ g_logits,
                                                         const float* __restrict__ coef, int Tn, int k, int lgHW,
                                                         const float* __restrict__ temp, float anneal,
                                                         float* __restrict__ g_raw, float* __restrict__ gsum,
                                                         float* __restrict__ tpart) {
  constexpr int NE = E / RTEAM;  // NT: teams per block
  __shared__ float red[NT * E];
  __shared__ float tred[NT];
  const int team = threadIdx.x / RTEAM, tl = threadIdx.x % RTEAM;
  const int HW = 1 << lgHW;
  const int TB = HW > NT ? HW : NT;
  const int t0 = blockIdx.x * TB;
  const float te = teff_of(temp, anneal);
  float acc[NE];
#pragma unroll
  for (int j = 0; j < NE; ++j) acc[j] = 0.f;
  float gt_part = 0.f;
  for (int tt = team; tt < TB; tt += NT) {
    const int t = t0 + tt;
    const bool ok = t < Tn;  // team-uniform; a dead team computes on zeros (the shuffles stay wave-wide)
    const int64_t r = (int64_t)(ok ? t : 0) * E;
    float p[NE], gp[NE], z[NE];
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      const int e = tl + RTEAM * j;
      p[j] = probs[r + e];
      z[j] = zlog[r + e];
      gp[j] = (coef ? coef[e] : 0.f) + (g_probs ? g_probs[r + e] : 0.f);
    }
    if (g_gate) {
      const int64_t rk = (int64_t)(ok ? t : 0) * k;
      if (k == E) {
        for (int i = 0; i < k; ++i) {
          const int ex = topi[rk + i];
          const float gg = g_gate[rk + i];
#pragma unroll
          for (int j = 0; j < NE; ++j)
            if (tl + RTEAM * j == ex) gp[j] += gg;
        }
      } else {
        float S = 0.f, dot = 0.f;
        for (int i = 0; i < k; ++i) {
          const int ex = topi[rk + i];
#pragma unroll
          for (int j = 0; j < NE; ++j)
            if (tl + RTEAM * j == ex) S += p[j];
          dot += g_gate[rk + i] * gate[rk + i];
        }
        S = team_sum(S);
        for (int i = 0; i < k; ++i) {
          const int ex = topi[rk + i];
          const float v = (g_gate[rk + i] - dot) / S;
#pragma unroll
          for (int j = 0; j < NE; ++j)
            if (tl + RTEAM * j == ex) gp[j] += v;
        }
      }
    }
    // recompute softmax s and clamped q
    float l[NE], sv[NE], q[NE];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      l[j] = fminf(fmaxf(z[j], -20.f), 20.f);
      mx = fmaxf(mx, l[j]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 1, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 2, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 4, 64));
    float den = 0.f;
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      sv[j] = expf(l[j] - mx);
      den += sv[j];
    }
    den = team_sum(den);
    float Sq = 0.f;
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      sv[j] /= den;
      q[j] = fminf(fmaxf(sv[j], 1e-6f), 1.f);
      Sq += q[j];
    }
    Sq = team_sum(Sq);
    float d1 = 0.f;  // p = q / Sq
#pragma unroll
    for (int j = 0; j < NE; ++j) d1 += gp[j] * (q[j] / Sq);
    d1 = team_sum(d1);
    float gs_[NE], d2 = 0.f;
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      const float gq = (gp[j] - d1) / Sq;
      gs_[j] = (sv[j] >= 1e-6f && sv[j] <= 1.f) ? gq : 0.f;
      d2 += gs_[j] * sv[j];
    }
    d2 = team_sum(d2);
    if (ok) {
#pragma unroll
      for (int j = 0; j < NE; ++j) {
        const int e = tl + RTEAM * j;
        float gl = sv[j] * (gs_[j] - d2);
        if (g_logits) gl += g_logits[r + e];  // the router's second output, logits (:378-381)
        gl = (z[j] >= -20.f && z[j] <= 20.f) ? gl : 0.f;
        gt_part += -gl * z[j] / te;
        acc[j] += gl / te;
        g_raw[r + e] = gl / te;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NE; ++j) red[team * E + tl + RTEAM * j] = acc[j];
  gt_part = team_sum(gt_part);
  if (tl == 0) tred[team] = gt_part;
  __syncthreads();
  // per-image sums over the image's teams, in team order
  const int nimg = TB >> lgHW;
  const int tpi = HW < NT ? HW : NT;  // teams per image
  for (int i = threadIdx.x; i < nimg * E; i += NT * RTEAM) {
    const int bl = i / E, e = i - bl * E;
    if (t0 + bl * HW < Tn) {
      float v = 0.f;
      for (int w = bl * tpi; w < bl * tpi + tpi; ++w) v += red[w * E + e];
      gsum[(int64_t)((t0 >> lgHW) + bl) * E + e] = v;
    }
  }
  if (threadIdx.x == 0 && tpart) {
    float tt = 0.f;
    for (int i = 0; i < NT; ++i) tt += tred[i];
    const float raw = temp[0] * anneal;
    tpart[blockIdx.x] = (raw >= 0.5f && raw <= 5.f) ? tt * anneal : 0.f;
  }
}

// g_tok[t, c] = sum_j gX[pos_of[t*k+j], c] + sum_e g_raw[t, e] * Wfc[c, e]
template <typename T, typename TO>
__global__ void k_token_grad(const T* __restrict__ gX, int64_t ldx, const int* __restrict__ pos_of, int Tn, int k,
                             int C, const float* __restrict__ g_raw, const float* __restrict__ Wfc, int E,
                             TO* __restrict__ out, int64_t ldo) {
  int64_t n = (int64_t)Tn * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int t = (int)(i / C), c = (int)(i - (int64_t)t * C);
    float s = 0.f;
    if (gX)
      for (int j = 0; j < k; ++j) s += ldf(gX, (int64_t)pos_of[t * k + j] * ldx + c);
    for (int e = 0; e < E; ++e) s += g_raw[(int64_t)t * E + e] * Wfc[(int64_t)c * E + e];
    stf(out, (int64_t)t * ldo + c, s);
  }
}

// G1[c, e] += sum_t tok[t, c] * g_raw[t, e]
template <typename T, int E>
__global__ void k_router_feat_grad(const T* __restrict__ tok, int64_t ld, int Tn, int C,
                                   const float* __restrict__ g_raw, int chunk, float* __restrict__ G1,
                                   float* __restrict__ part) {
  __shared__ float gr[64 * E];
  int c = threadIdx.x;
  int t0 = blockIdx.x * chunk, t1 = min(Tn, t0 + chunk);
  float acc[E];
#pragma unroll
  for (int e = 0; e < E; ++e) acc[e] = 0.f;
  for (int tb = t0; tb < t1; tb += 64) {
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * E; i += blockDim.x) {
      int tt = tb + i / E;
      gr[i] = tt < t1 ? g_raw[(int64_t)tb * E + i] : 0.f;
    }
    __syncthreads();
    if (c < C) {
      int te = min(64, t1 - tb);
      for (int j = 0; j < te; ++j) {
        float x = ldf(tok, (int64_t)(tb + j) * ld + c);
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] += x * gr[j * E + e];
      }
    }
  }
  if (c < C) {
    if (part) {  // per-block partial row (no same-address atomics); a rows fold (mg_fold.hip) sums them
#pragma unroll
      for (int e = 0; e < E; ++e) part[(int64_t)blockIdx.x * C * E + (int64_t)c * E + e] = acc[e];
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) atomicAdd(&G1[(int64_t)c * E + e], acc[e]);
    }
  }
}

// LDS floats of k_router_feat_grad_v's in-block fold of R partial rows (CV * E values per channel lane, TX lanes
// padded to TX + 1), and the most it may use (65 KiB: the C = 512 / 32-expert blocks; the launch raises the
// dynamic-LDS limit past 64 KiB)
__host__ __device__ inline int64_t rfg_fold_floats(int R, int cve, int TX) { return (int64_t)R * cve * (TX + 1); }
constexpr int64_t kRfgFoldMax = 16640;

// Vector form: a block is TX = C / CV channel lanes (CV channels each, 16-B loads for CV = 8 bf16) x TY = 256 / TX
// token lanes walking its token chunk; the token lanes of a wave fold with shuffles and each wave-row group
// writes one partial row [C * E] (folded by a rows fold, mg_fold.hip).  The thread-per-channel form issued 2-byte loads
// one token at a time (35 us for 65536 tokens x 128 channels).
template <typename T, int E, int CV>
__global__ __launch_bounds__(256) void k_router_feat_grad_v(const T* __restrict__ tok, int64_t ld, int Tn, int C,
                                                            const float* __restrict__ g_raw, int chunk,
                                                            float* __restrict__ part) {
  // channel group blockIdx.y of gridDim.y: channels [cb, cb + Cb)
  const int Cb = C / gridDim.y, cb = blockIdx.y * Cb;
  const int TX = Cb / CV, TY = 256 / TX;
  const int tx = threadIdx.x % TX, ty = threadIdx.x / TX;
  const int c = cb + tx * CV;
  const int t0 = blockIdx.x * chunk, t1 = min(Tn, t0 + chunk);
  float acc[CV][E];
#pragma unroll
  for (int j = 0; j < CV; ++j)
#pragma unroll
    for (int e = 0; e < E; ++e) acc[j][e] = 0.f;
  // four tokens' loads in flight per lane (the accumulation order per lane is unchanged)
#pragma unroll 4
  for (int t = t0 + ty; t < t1; t += TY) {
    float x[CV];
    if constexpr (CV == 8) {
      ld8(tok + (int64_t)t * ld + c, x);
    } else {
#pragma unroll
      for (int j = 0; j < CV; ++j) x[j] = ldf(tok, (int64_t)t * ld + c + j);
    }
    float gv[E];  // the token's E raw-logit gradients as 16-B loads (rows are 16-B aligned: E % 4 == 0)
#pragma unroll
    for (int e = 0; e < E; e += 4) {
      const f32x4_t q = *reinterpret_cast<const f32x4_t*>(g_raw + (int64_t)t * E + e);
      gv[e] = q[0];
      gv[e + 1] = q[1];
      gv[e + 2] = q[2];
      gv[e + 3] = q[3];
    }
#pragma unroll
    for (int e = 0; e < E; ++e)
#pragma unroll
      for (int j = 0; j < CV; ++j) acc[j][e] += x[j] * gv[e];
  }
  const int tyw = TX < 64 ? 64 / TX : 1;  // token lanes per wave
  for (int o = TX; o < 64; o <<= 1)
#pragma unroll
    for (int j = 0; j < CV; ++j)
#pragma unroll
      for (int e = 0; e < E; ++e) acc[j][e] += __shfl_xor(acc[j][e], o, 64);
  const int R = TY / tyw;  // partial rows of this block (one per wave-row group)
  if (R > 1 && rfg_fold_floats(R, CV * E, TX) <= kRfgFoldMax) {  // fold them in LDS (fixed order): one row per block
    // red[r][j * E + e][tx], rows of TX + 1 words: a lane's CV * E values used to be consecutive words (lanes CV * E
    // words apart: every lane on one bank, 77 % bank-conflict cycles); now the lanes of one store are consecutive
    // words and the fold's reads (consecutive (j, e) of one channel lane) are TX + 1 (odd) words apart
    extern __shared__ float red[];  // R * CV * E * (TX + 1) floats (dynamic; host: rfg_fold_floats)
    const int TXP = TX + 1;
    if (ty % tyw == 0) {
#pragma unroll
      for (int j = 0; j < CV; ++j)
#pragma unroll
        for (int e = 0; e < E; ++e) red[((ty / tyw) * CV * E + j * E + e) * TXP + tx] = acc[j][e];
    }
    __syncthreads();
    float* pr = part + (int64_t)blockIdx.x * C * E + (int64_t)cb * E;  // (this group's channel slice of the row)
    for (int i = threadIdx.x; i < Cb * E; i += 256) {
      const int li = i / (CV * E), je = i - li * (CV * E);  // element (c - cb) * E + e = (li * CV + j) * E + e
      float v = 0.f;
      for (int r = 0; r < R; ++r) v += red[(r * CV * E + je) * TXP + li];
      pr[i] = v;
    }
    return;
  }
  if (ty % tyw == 0) {
    float* pr = part + ((int64_t)blockIdx.x * R + ty / tyw) * C * E + (int64_t)c * E;
#pragma unroll
    for (int j = 0; j < CV; ++j)
#pragma unroll
      for (int e = 0; e < E; ++e) pr[j * E + e] = acc[j][e];
  }
}


// out[g][n] += sum_{r in group g} X[src(r)][n] * rs[r]  (grouped bias gradients)
template <typename T>
__global__ void k_grouped_colsum(const T* __restrict__ X, int64_t ld, const int* __restrict__ idx, int idx_div,
                                 const float* __restrict__ rs, const int* __restrict__ row_off, int G, int N,
                                 int rows_per_block, float* __restrict__ out) {
  int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  int total = row_off[G];
  int r0 = blockIdx.y * rows_per_block, r1 = min(total, r0 + rows_per_block);
  if (r0 >= r1) return;
  int g = 0;
  while (g < G && row_off[g + 1] <= r0) ++g;
  float s = 0.f;
  for (int r = r0; r < r1; ++r) {
    while (r >= row_off[g + 1]) {
      atomicAdd(&out[(int64_t)g * N + n], s);
      s = 0.f;
      ++g;
    }
    int src = idx ? idx[r] / idx_div : r;
    float v = ldf(X, (int64_t)src * ld + n);
    s += rs ? v * rs[r] : v;
  }
  atomicAdd(&out[(int64_t)g * N + n], s);
}

// 8-column vector form: block = TX column vectors x TY row lanes over one chunk of rows.  A thread flushes its
// running sum to global memory only when its rows cross a group boundary (rare: E boundaries in total); the
// sums for the chunk's last group are folded over the row lanes in LDS and added once per column.
template <typename T, int NT>
__global__ __launch_bounds__(NT) void k_grouped_colsum_v(const T* __restrict__ X, int64_t ld,
                                                         const int* __restrict__ idx, int idx_div,
                                                         const float* __restrict__ rs, const int* __restrict__ row_off,
                                                         int G, int N, int rows_per_block, float* __restrict__ out) {
  __shared__ float red[NT * 8];
  __shared__ int ro[65];  // row_off staged once: the group searches below are LDS reads, not chains of dependent
                          // global loads (8 of them cost ~8 us before the first row was read)
  const int tx = threadIdx.x, ty = threadIdx.y, TX = blockDim.x, TY = blockDim.y;
  const int n = (blockIdx.x * TX + tx) * 8;
  {
    const int t = ty * TX + tx;
    if (t <= G) ro[t] = row_off[t];
  }
  __syncthreads();
  const int total = ro[G];
  const int r0 = blockIdx.y * rows_per_block, r1 = min(total, r0 + rows_per_block);
  if (r0 >= r1) return;
  int glast = 0;
  while (glast < G && ro[glast + 1] <= r1 - 1) ++glast;
  float s[8], v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  int g = -1, gend = -1;
  const bool live = n < N;
  int r = r0 + ty;
  while (live && r < r1) {
    if (r >= gend) {
      if (g >= 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          atomicAdd(&out[(int64_t)g * N + n + j], s[j]);
          s[j] = 0.f;
        }
      }
      g = 0;
      while (g < G && ro[g + 1] <= r) ++g;
      gend = ro[g + 1];
    }
    if (!idx && !rs && r + 3 * TY < min(gend, r1)) {  // four rows of one group: independent loads in flight
      float v1[8], v2[8], v3[8];
      ld8(X + (int64_t)r * ld + n, v);
      ld8(X + (int64_t)(r + TY) * ld + n, v1);
      ld8(X + (int64_t)(r + 2 * TY) * ld + n, v2);
      ld8(X + (int64_t)(r + 3 * TY) * ld + n, v3);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += (v[j] + v1[j]) + (v2[j] + v3[j]);
      r += 4 * TY;
      continue;
    }
    const int src = idx ? idx[r] / idx_div : r;
    ld8(X + (int64_t)src * ld + n, v);
    const float sc = rs ? rs[r] : 1.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] += rs ? v[j] * sc : v[j];
    r += TY;
  }
  if (live && g >= 0 && g != glast) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      atomicAdd(&out[(int64_t)g * N + n + j], s[j]);
      s[j] = 0.f;
    }
  }
  const int tid = ty * TX + tx;
#pragma unroll
  for (int j = 0; j < 8; ++j) red[tid * 8 + j] = s[j];
  __syncthreads();
  if (ty == 0 && live) {
    for (int y = 1; y < TY; ++y)
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += red[(y * TX + tx) * 8 + j];
#pragma unroll
    for (int j = 0; j < 8; ++j) atomicAdd(&out[(int64_t)glast * N + n + j], s[j]);
  }
}

// Deterministic mode: per (row chunk, group) partial rows part[(chunk * G + g) * N + n], the row lanes of a
// block folded in LDS in lane order; k_grouped_colsum_fold then adds, per (group, column), the partials of the
// chunks that group's rows touch, in chunk order.
template <typename T>
__global__ __launch_bounds__(256) void k_grouped_colsum_part(const T* __restrict__ X, int64_t ld,
                                                             const int* __restrict__ idx, int idx_div,
                                                             const float* __restrict__ rs,
                                                             const int* __restrict__ row_off, int G, int N, int rpb,
                                                             float* __restrict__ part) {
  __shared__ float red[256 * 8];
  __shared__ int ro[65];  // row_off staged once (see k_grouped_colsum_v)
  const int tx = threadIdx.x, ty = threadIdx.y, TX = blockDim.x, TY = blockDim.y;
  const int n = (blockIdx.x * TX + tx) * 8;
  const bool live = n < N;
  {
    const int t = ty * TX + tx;
    if (t <= G) ro[t] = row_off[t];
  }
  __syncthreads();
  const int total = ro[G];
  const int r0 = blockIdx.y * rpb, r1 = min(total, r0 + rpb);
  for (int g = 0; g < G; ++g) {
    const int gs = max(r0, ro[g]), ge = min(r1, ro[g + 1]);
    if (gs >= ge) continue;  // block-uniform
    float s[8], v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] = 0.f;
    if (live) {
      for (int r = gs + ty; r < ge; r += TY) {
        const int src = idx ? idx[r] / idx_div : r;
        ld8(X + (int64_t)src * ld + n, v);
        const float sc = rs ? rs[r] : 1.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += v[j] * sc;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) red[(ty * TX + tx) * 8 + j] = s[j];
    __syncthreads();
    if (ty == 0 && live) {
      for (int y = 1; y < TY; ++y)
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += red[(y * TX + tx) * 8 + j];
#pragma unroll
      for (int j = 0; j < 8; ++j) part[((int64_t)blockIdx.y * G + g) * N + n + j] = s[j];
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void k_grouped_colsum_fold(const float* __restrict__ part,
                                                             const int* __restrict__ row_off, int G, int N, int rpb,
                                                             float* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= G * N) return;
  const int g = i / N, n = i - g * N;
  const int lo = row_off[g], hi = row_off[g + 1];
  if (lo >= hi) return;
  float s = 0.f;
  for (int c = lo / rpb; c <= (hi - 1) / rpb; ++c) s += part[((int64_t)c * G + g) * N + n];
  out[i] += s;
}

// KL of one router, two passes: per-block partial sums over the three (mu, rho) pairs, then one block
// folds the partials and applies the reference's nan/inf/clamp rules.
// 0.5 sum(sigma^2 + mu^2 - 1 - log sigma^2) over one router's three (mu, rho) pairs, one partial per block of a
// grid-stride split into nparts blocks
MG_DEV void router_kl_part_block(const float* __restrict__ mf, const float* __restrict__ rf, int nf,
                                 const float* __restrict__ mt, const float* __restrict__ rt, int nt,
                                 const float* __restrict__ mc, const float* __restrict__ rc, int nc, int part_i,
                                 int nparts, float* __restrict__ part) {
  __shared__ float red[4];
  const int64_t n = (int64_t)nf + nt + nc;
  float ps = 0.f;
  for (int64_t i = (int64_t)part_i * 256 + threadIdx.x; i < n; i += (int64_t)nparts * 256) {
    float m, r;
    if (i < nf) { m = mf[i]; r = rf[i]; }
    else if (i < nf + nt) { m = mt[i - nf]; r = rt[i - nf]; }
    else { m = mc[i - nf - nt]; r = rc[i - nf - nt]; }
    float sg = softplusf(r);
    float lv = 2.f * logf(sg);
    ps += expf(lv) + m * m - 1.f - lv;
  }
  ps = wave_sum(ps);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ps;
  __syncthreads();
  if (threadIdx.x == 0) part[part_i] = 0.5f * (red[0] + red[1] + red[2] + red[3]);
}

__global__ __launch_bounds__(256) void k_router_kl_part(const float* __restrict__ mf, const float* __restrict__ rf,
                                                        int nf, const float* __restrict__ mt,
                                                        const float* __restrict__ rt, int nt,
                                                        const float* __restrict__ mc, const float* __restrict__ rc,
                                                        int nc, float* __restrict__ part) {
  router_kl_part_block(mf, rf, nf, mt, rt, nt, mc, rc, nc, blockIdx.x, gridDim.x, part);
}

// several routers: blockIdx.y = record, each with its own number of partials (the single-router split, so the
// terms are bit-identical to mg_router_kl's); partials of record j at part + 256 j
constexpr int KL_MAX_RECS = 8;
struct KlBatch {
  mg_kl_rec r[KL_MAX_RECS];
  int nparts[KL_MAX_RECS];
};
__global__ __launch_bounds__(256) void k_router_kl_part_batch(KlBatch b, float* __restrict__ part) {
  const int j = blockIdx.y;
  const mg_kl_rec& r = b.r[j];
  if ((int)blockIdx.x >= b.nparts[j]) return;  // block-uniform
  router_kl_part_block(r.mu_f, r.rho_f, r.nf, r.mu_t, r.rho_t, r.nt, r.mu_c, r.rho_c, r.nc, blockIdx.x, b.nparts[j],
                       part + 256 * j);
}
MG_DEV void router_kl_fin_wave(const float* __restrict__ part, int nparts, float* __restrict__ out) {
  float s = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 64) s += part[i];
  s = wave_sum(s);
  if (threadIdx.x == 0) {
    float v = s;
    float pass = 1.f;
    if (isnan(v)) { v = 0.f; pass = 0.f; }
    else if (isinf(v)) { v = v > 0 ? 200.f : 0.f; pass = 0.f; }
    if (v > 120.f) { v = 120.f; pass = 0.f; }
    if (v < 0.f) { v = 0.f; pass = 0.f; }
    out[0] = v;
    out[1] = pass;
  }
}
__global__ void k_router_kl_fin(const float* __restrict__ part, int nparts, float* __restrict__ out) {
  router_kl_fin_wave(part, nparts, out);
}
__global__ void k_router_kl_fin_batch(KlBatch b, const float* __restrict__ part, float* __restrict__ out) {
  router_kl_fin_wave(part + 256 * blockIdx.x, b.nparts[blockIdx.x], out + 2 * blockIdx.x);
}

// KL of one router (t2i_moe_gan.py:405-423): out[0] = clamp(nan_to_num(sum), 0, 120), out[1] = grad-pass flag
__global__ void k_router_kl(const float* __restrict__ mf, const float* __restrict__ rf, int nf,
                            const float* __restrict__ mt, const float* __restrict__ rt, int nt,
                            const float* __restrict__ mc, const float* __restrict__ rc, int nc,
                            float* __restrict__ out) {
  __shared__ float red[16];
  float s = 0.f;
  for (int part = 0; part < 3; ++part) {
    const float* m = part == 0 ? mf : part == 1 ? mt : mc;
    const float* r = part == 0 ? rf : part == 1 ? rt : rc;
    int n = part == 0 ? nf : part == 1 ? nt : nc;
    float ps = 0.f;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      float sg = softplusf(r[i]);
      float lv = 2.f * logf(sg);
      ps += expf(lv) + m[i] * m[i] - 1.f - lv;
    }
    ps = wave_sum(ps);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ps;
    __syncthreads();
    if (threadIdx.x == 0) {
      float tt = 0.f;
      for (int i = 0; i < (int)(blockDim.x >> 6); ++i) tt += red[i];
      s += 0.5f * tt;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    float v = s;
    float pass = 1.f;
    if (isnan(v)) { v = 0.f; pass = 0.f; }
    else if (isinf(v)) { v = v > 0 ? 200.f : 0.f; pass = 0.f; }
    if (v > 120.f) { v = 120.f; pass = 0.f; }
    if (v < 0.f) { v = 0.f; pass = 0.f; }
    out[0] = v;
    out[1] = pass;
  }
}

// gmu += gW*[|mu|<=10] + c*mu ; grho += gW*clamp(eps)*dsigma/drho + c*sig(rho)*(sigma - 1/sigma)
// (flags & mask: the generator loss was replaced by 0, t2i_moe_gan.py:1396-1399 -- only the KL term remains)
__global__ void k_router_param_bwd(const float* __restrict__ mu, const float* __restrict__ rho,
                                   const float* __restrict__ eps, const float* __restrict__ gW, int64_t n,
                                   const float* __restrict__ klc, float* __restrict__ gmu, float* __restrict__ grho,
                                   const int32_t* __restrict__ flags, int32_t mask) {
  float c = klc ? klc[0] : 0.f;
  if (flags && (flags[0] & mask)) gW = nullptr;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float m = mu[i], r = rho[i];
    float gm = c * m, gr = 0.f;
    float sp = softplusf(r);
    float sgm = sigmoidf_(r);
    gr += c * sgm * (sp - 1.f / sp);
    if (gW) {
      float g = gW[i];
      if (m >= -10.f && m <= 10.f) gm += g;
      float rcl = fminf(fmaxf(r, -8.f), 4.f);
      float spc = softplusf(rcl);
      if (r >= -8.f && r <= 4.f && spc >= 1e-6f && spc <= 10.f) gr += g * fminf(fmaxf(eps[i], -2.f), 2.f) * sigmoidf_(rcl);
    }
    gmu[i] += gm;
    grho[i] += gr;
  }
}

// every router parameter tensor of a backward in one launch: blocks [blk_off[d], blk_off[d + 1]) run descriptor d
// with k_router_param_bwd's per-element arithmetic (the same results; the per-tensor launches were ~5 us each of
// pure launch latency, 9 per step at C2)
constexpr int MG_RPB_MAX = 32;
struct RpbBatch {
  mg_router_param_desc d[MG_RPB_MAX];
  int blk_off[MG_RPB_MAX + 1];
  int n;
};
__global__ __launch_bounds__(256) void k_router_param_bwd_batch(RpbBatch b, const int32_t* __restrict__ flags,
                                                                 int32_t mask) {
  int di = 0;
  while (di + 1 < b.n && (int)blockIdx.x >= b.blk_off[di + 1]) ++di;
  const mg_router_param_desc& q = b.d[di];
  const int nb = b.blk_off[di + 1] - b.blk_off[di], bi = blockIdx.x - b.blk_off[di];
  const float c = q.kl_coef ? q.kl_coef[0] : 0.f;
  const float* gW = (flags && (flags[0] & mask)) ? nullptr : q.gW;
  for (int64_t i = bi * (int64_t)blockDim.x + threadIdx.x; i < q.n; i += (int64_t)nb * blockDim.x) {
    float m = q.mu[i], r = q.rho[i];
    float gm = c * m, gr = 0.f;
    float sp = softplusf(r);
    float sgm = sigmoidf_(r);
    gr += c * sgm * (sp - 1.f / sp);
    if (gW) {
      float g = gW[i];
      if (m >= -10.f && m <= 10.f) gm += g;
      float rcl = fminf(fmaxf(r, -8.f), 4.f);
      float spc = softplusf(rcl);
      if (r >= -8.f && r <= 4.f && spc >= 1e-6f && spc <= 10.f) gr += g * fminf(fmaxf(q.eps[i], -2.f), 2.f) * sigmoidf_(rcl);
    }
    q.gmu[i] += gm;
    q.grho[i] += gr;
  }
}

// balance loss (t2i_moe_gan.py:951-1000) from the global per-expert prob sums:
// out[0] = loss; coef[e] = d loss / d probs[t, e] (* grad_scale)
// one lane per expert (E <= 64), mean / variance as wave butterflies (fixed order); the serial single-lane form
// walked its E loads one round trip at a time (C5: 18 us for 32 experts)
__global__ void k_balance(const float* __restrict__ load, int E, float T, float weight, float grad_scale,
                          float* __restrict__ out, float* __restrict__ coef) {
  const int e = threadIdx.x;
  const bool own = e < E;
  const float frac = own ? (load[e] + 1e-6f) / T : 0.f;
  const float mean = wave_sum(frac) / E;
  const float dv = own ? frac - mean : 0.f;
  const float var = wave_sum(dv * dv);
  const float sd = sqrtf(var / (E - 1));
  const float den = mean + 1e-6f;
  const float cv = sd / den;
  const float raw = E * cv;
  const float L = isnan(raw) ? 0.f : fminf(fmaxf(raw, 0.f), 10.f);
  if (e == 0) out[0] = weight * L;
  const bool pass = !isnan(raw) && raw >= 0.f && raw <= 10.f;
  if (own) {
    float dcv = 0.f;
    if (pass && sd > 0.f) {
      const float dsd = dv / ((E - 1) * sd);
      dcv = (dsd * den - sd / E) / (den * den);
    }
    coef[e] = pass ? weight * E * dcv / T * grad_scale : 0.f;
  }
}

// generator KL (t2i_moe_gan.py:846, :1367-1376, :1402-1404): total = sum of the routers' clamped KLs;
// the step clamps total at 50 (zero gradient above).  coef[r] = eff_w * [total <= 50] * pass_r
__global__ void k_kl_coefs(const float* __restrict__ kl2, int R, float eff_w, float* __restrict__ coef,
                           float* __restrict__ total) {
  if (threadIdx.x != 0) return;
  float t = 0.f;
  for (int r = 0; r < R; ++r) t += kl2[2 * r];
  // kl > 50 -> clamp (no gradient); NaN / Inf -> the constant 0 (no gradient), :1369-1376
  const bool finite = isfinite(t);
  const bool live = finite && t <= 50.f;
  for (int r = 0; r < R; ++r) coef[r] = live ? eff_w * kl2[2 * r + 1] : 0.f;
  total[0] = live ? t : (finite ? 50.f : 0.f);
}

inline int nblk(int64_t n, int t = 256) { return (int)std::min<int64_t>((n + t - 1) / t, 65536); }

}  // namespace

extern "C" int mg_kl_coefs(const float* kl2, int R, float eff_w, float* coef, float* total, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_kl_coefs, dim3(1), dim3(64), 0, st, kl2, R, eff_w, coef, total);
  return mg_check_launch("mg_kl_coefs");
}

extern "C" int mg_router_reparam(const float* mu, const float* rho, const float* eps, int64_t n, float* W,
                                 void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_reparam, dim3(nblk(n)), dim3(256), 0, st, mu, rho, eps, n, W);
  return mg_check_launch("mg_router_reparam");
}

extern "C" int mg_router_fwd(int dtype, const void* tok, int64_t ld, int T, int C, const float* Wfc, const float* Lt,
                             int E, int k, int HW, const float* temperature, float anneal, int eval_mode,
                             float* probs, float* zlog, int32_t* topi, float* gate, void* stream) {
  MG_REQUIRE(E == 4 || E == 8 || E == 16 || E == 32, "E must be 4, 8, 16 or 32");
  MG_REQUIRE(k >= 1 && k <= E, "bad k");
  MG_REQUIRE((HW & (HW - 1)) == 0, "HW must be a power of two");
  const int vec = dtype == MG_F32 ? 4 : 8;
  MG_REQUIRE(C % (vec * 8) == 0 && ld % vec == 0, "C must be a multiple of 8 vectors");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int lg = 0;
  while ((1 << lg) < HW) ++lg;
  if (T <= 0) return 0;
  if (dtype != MG_F32 && E >= 8 && C % 128 == 0 && C <= 512 && ld % 8 == 0 && mg_al16(tok) &&
      (g_mg_tune[MG_TUNE_ROUTER_TEAM] & 1) == 0) {
    // tiles per block: up to 4 / (C / 128) (the A fragments a lane holds) once there are >= 1024 blocks' worth
    const int ntile = cdiv(T, 16);
    const int nks = C / 128;
    const int nt = std::max(1, std::min(RNT / nks, ntile / 1024));
    dim3 gm(cdiv(ntile, nt));
#define L_(EE, NK) hipLaunchKernelGGL((k_router_fwd_mfma<EE, NK>), gm, dim3(256), 0, st, (const bf16_t*)tok, ld, T, C, \
                                      nt, Wfc, Lt, lg, temperature, anneal, k, eval_mode, probs, zlog, topi, gate)
#define LK_(EE) if (nks == 1) L_(EE, 1); else if (nks == 2) L_(EE, 2); else if (nks == 3) L_(EE, 3); else L_(EE, 4)
    if (E == 8) { LK_(8); } else if (E == 16) { LK_(16); } else { LK_(32); }
#undef LK_
#undef L_
    return mg_check_launch("mg_router_fwd");
  }
  dim3 grid(std::min(cdiv(T, 32), 1024));
  size_t sm = (size_t)C * E * sizeof(float);
#define L_(TT, EE) hipLaunchKernelGGL((k_router_fwd<TT, EE>), grid, dim3(256), sm, st, (const TT*)tok, ld, T, C, Wfc, Lt, lg, \
                                      temperature, anneal, k, eval_mode, probs, zlog, topi, gate)
#define LE_(TT) if (E == 4) L_(TT, 4); else if (E == 8) L_(TT, 8); else if (E == 16) L_(TT, 16); else L_(TT, 32)
  if (dtype == MG_F32) { LE_(float); } else { LE_(bf16_t); }
#undef LE_
#undef L_
  return mg_check_launch("mg_router_fwd");
}

extern "C" int mg_moe_dispatch(const int32_t* topi, const float* gate, int T, int k, int E, int bm, int32_t* ws,
                               int32_t* row_off, int32_t* tile_off, int32_t* perm, int32_t* pos_of, float* gate_pos,
                               void* stream) {
  MG_REQUIRE(E == 4 || E == 8 || E == 16 || E == 32, "E must be 4, 8, 16 or 32");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int n = T * k;
  int nb = cdiv(n, DCH);
  MG_REQUIRE(nb <= 65535, "too many assignments");
  hipLaunchKernelGGL(k_disp_count, dim3(nb), dim3(256), E * sizeof(int), st, topi, n, E, ws);
  if (g_mg_tune[MG_TUNE_DISPATCH3] != 1) {  // the scan folded into the scatter (A/B: 1 = three kernels)
#define L_(EE) hipLaunchKernelGGL((k_disp_scatter_scan<EE>), dim3(nb), dim3(256), 0, st, topi, gate, n, nb, bm, ws, \
                                  row_off, tile_off, perm, pos_of, gate_pos)
    if (E == 4) L_(4); else if (E == 8) L_(8); else if (E == 16) L_(16); else L_(32);
#undef L_
    return mg_check_launch("mg_moe_dispatch");
  }
  // gfx950 assumption: at the 16384-count cutoff the parallel scan takes (16384 + 1056) * 4 B = 69.7 KB of dynamic
  // LDS, over the 64 KB of older parts but within the 160 KB a gfx950 workgroup may use
  if ((int64_t)nb * E <= 16384)
    hipLaunchKernelGGL(k_disp_scan_par, dim3(1), dim3(1024), (size_t)(nb * E + 1024 + 32) * sizeof(int), st, ws, nb, E,
                       bm, row_off, tile_off);
  else
    hipLaunchKernelGGL(k_disp_scan, dim3(1), dim3(64), 0, st, ws, nb, E, bm, row_off, tile_off);
#define L_(EE) hipLaunchKernelGGL((k_disp_scatter<EE>), dim3(nb), dim3(256), 0, st, topi, gate, n, ws, row_off, perm, pos_of, gate_pos)
  if (E == 4) L_(4); else if (E == 8) L_(8); else if (E == 16) L_(16); else L_(32);
#undef L_
  return mg_check_launch("mg_moe_dispatch");
}

extern "C" int mg_moe_combine(int dtype, const void* Y, int64_t ldy, const int32_t* pos_of, const float* gate, int T,
                              int k, int C, const void* resid, int64_t ldr, void* out, int64_t ldo, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t n = (int64_t)T * C;
  if (C % 8 == 0 && ldy % 8 == 0 && ldo % 8 == 0 && (!resid || ldr % 8 == 0) && mg_al16(Y) && mg_al16(out) &&
      (!resid || mg_al16(resid)) && n / 8 < (1LL << 31)) {
    int blocks = nblk(n / 8);
    if (dtype == MG_F32)
      hipLaunchKernelGGL(k_combine_v<float>, dim3(blocks), dim3(256), 0, st, (const float*)Y, ldy, pos_of, gate, T, k,
                         C, (const float*)resid, ldr, (float*)out, ldo);
    else
      hipLaunchKernelGGL(k_combine_v<bf16_t>, dim3(blocks), dim3(256), 0, st, (const bf16_t*)Y, ldy, pos_of, gate, T,
                         k, C, (const bf16_t*)resid, ldr, (bf16_t*)out, ldo);
    return mg_check_launch("mg_moe_combine");
  }
  if (dtype == MG_F32)
    hipLaunchKernelGGL(k_combine<float>, dim3(nblk(n)), dim3(256), 0, st, (const float*)Y, ldy, pos_of, gate, T, k, C,
                       (const float*)resid, ldr, (float*)out, ldo);
  else
    hipLaunchKernelGGL(k_combine<bf16_t>, dim3(nblk(n)), dim3(256), 0, st, (const bf16_t*)Y, ldy, pos_of, gate, T, k,
                       C, (const bf16_t*)resid, ldr, (bf16_t*)out, ldo);
  return mg_check_launch("mg_moe_combine");
}

extern "C" int mg_moe_combine_scaled(int dtype, const void* Y, int64_t ldy, const int32_t* pos_of, const float* gate,
                                     int T, int k, int C, const void* resid, int64_t ldr, void* out, int64_t ldo,
                                     const float* s, int64_t lds, int HW, void* xs, int64_t ldxs, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t n = (int64_t)T * C;
  MG_REQUIRE(C % 8 == 0 && ldy % 8 == 0 && ldo % 8 == 0 && ldxs % 8 == 0 && lds % 4 == 0 && (!resid || ldr % 8 == 0),
             "mg_moe_combine_scaled: C and pitches multiples of 8 (style pitch of 4)");
  MG_REQUIRE(mg_al16(Y) && mg_al16(out) && mg_al16(xs) && mg_al16(s) && (!resid || mg_al16(resid)),
             "mg_moe_combine_scaled: 16-byte aligned operands");
  MG_REQUIRE(HW > 0 && (HW & (HW - 1)) == 0 && T % HW == 0, "mg_moe_combine_scaled: HW a power of two dividing T");
  MG_REQUIRE(n / 8 < (1LL << 31), "mg_moe_combine_scaled: too many elements");
  if (n == 0) return MG_OK;
  int lg = 0;
  while ((1 << lg) < HW) ++lg;
  const int blocks = nblk(n / 8);
  if (dtype == MG_F32)
    hipLaunchKernelGGL((k_combine_v<float, true>), dim3(blocks), dim3(256), 0, st, (const float*)Y, ldy, pos_of, gate, T,
                       k, C, (const float*)resid, ldr, (float*)out, ldo, s, lds, lg, (float*)xs, ldxs);
  else
    hipLaunchKernelGGL((k_combine_v<bf16_t, true>), dim3(blocks), dim3(256), 0, st, (const bf16_t*)Y, ldy, pos_of, gate,
                       T, k, C, (const bf16_t*)resid, ldr, (bf16_t*)out, ldo, s, lds, lg, (bf16_t*)xs, ldxs);
  return mg_check_launch("mg_moe_combine_scaled");
}

extern "C" int mg_moe_gate_grad(int dtype, int gout_dtype, const void* gout, int64_t ldg, const void* Y, int64_t ldy,
                                const int32_t* pos_of, int T, int k, int C, float* g_gate, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int n = T * k;
  MG_REQUIRE(C % 8 == 0 && ldg % 8 == 0 && ldy % 8 == 0 && mg_al16(gout) && mg_al16(Y),
             "mg_moe_gate_grad: C and row pitches multiples of 8, 16-B aligned rows");
  dim3 grid(cdiv(n, 32));  // 32 assignments (8 lanes each) per block
#define L_(TT, TG) hipLaunchKernelGGL((k_gate_grad<TT, TG>), grid, dim3(256), 0, st, (const TG*)gout, ldg, (const TT*)Y, ldy, pos_of, n, k, C, g_gate)
  if (dtype == MG_F32) { if (gout_dtype == MG_F32) L_(float, float); else L_(float, bf16_t); }
  else { if (gout_dtype == MG_F32) L_(bf16_t, float); else L_(bf16_t, bf16_t); }
#undef L_
  return mg_check_launch("mg_moe_gate_grad");
}

extern "C" int mg_router_bwd(const float* probs, const float* zlog, const int32_t* topi, const float* gate,
                             const float* g_gate, const float* g_probs, const float* g_logits, const float* coef, int T,
                             int E, int k, int HW,
                             const float* temperature, float anneal, float* g_raw, float* gsum, float* g_temp,
                             void* stream) {
  MG_REQUIRE(E == 4 || E == 8 || E == 16 || E == 32, "E must be 4, 8, 16 or 32");
  MG_REQUIRE(HW >= 1 && HW <= 256 && (HW & (HW - 1)) == 0, "HW must be a power of two <= 256");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int lg = 0;
  while ((1 << lg) < HW) ++lg;
  const bool team = E >= 8 && (g_mg_tune[MG_TUNE_ROUTER_TEAM] & 2) == 0;
  const int nteam = HW >= 128 ? 128 : HW >= 64 ? 64 : 32;  // teams per block
  dim3 grid(team ? cdiv(T, std::max(HW, nteam)) : cdiv(T, 256));
  float* tpart = nullptr;
  bool deferred = false;
  if (g_temp) {
    tpart = mg_fold_partials((size_t)grid.x * sizeof(float), st, &deferred);
    if (!tpart) return MG_ERR_LAUNCH;
  }
#define L_(KN, TH) hipLaunchKernelGGL(KN, grid, dim3(TH), 0, st, probs, zlog, topi, gate, g_gate, g_probs, g_logits, coef, T, k, lg, \
                                      temperature, anneal, g_raw, gsum, tpart)
#define LT_(EE) if (nteam == 32) L_((k_router_bwd_team<EE, 32>), 256); else if (nteam == 64) L_((k_router_bwd_team<EE, 64>), 512); \
                else L_((k_router_bwd_team<EE, 128>), 1024)
  if (team) {
    if (E == 8) { LT_(8); } else if (E == 16) { LT_(16); } else { LT_(32); }
  } else {
    if (E == 4) L_(k_router_bwd<4>, 256); else if (E == 8) L_(k_router_bwd<8>, 256); else if (E == 16) L_(k_router_bwd<16>, 256); else L_(k_router_bwd<32>, 256);
  }
#undef LT_
#undef L_
  // the temperature partials (one per block) as a one-column rows fold
  if (g_temp) mg_fold_rows_submit(mg_fold_rows{tpart, 1, (int)grid.x, 1, 1, g_temp, nullptr}, deferred, st);
  return mg_check_launch("mg_router_bwd");
}

extern "C" int mg_moe_token_grad(int dtype, const void* gX, int64_t ldx, const int32_t* pos_of, int T, int k, int C,
                                 const float* g_raw, const float* Wfc, int E, int out_dtype, void* out, int64_t ldo,
                                 void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t n = (int64_t)T * C;
  if (T <= 0) return 0;
  if ((C == 128 || C == 256 || C == 512) && (E == 8 || E == 16 || E == 32) && (!gX || (ldx % 8 == 0 && mg_al16(gX))) &&
      ldo % 8 == 0 && mg_al16(out) && mg_al16(g_raw) && mg_al16(Wfc) && (g_mg_tune[MG_TUNE_ROUTER_TEAM] & 4) == 0) {
    // tiles per block: the product tile [16 nt][C + 4] fp32 within ~33 KiB, once there are >= 1024 blocks' worth
    const int ntile = cdiv(T, 16);
    const int nt = std::max(1, std::min(512 / C, ntile / 1024));
    const size_t lds = (size_t)nt * 16 * (C + 4) * sizeof(float);
    dim3 gm(cdiv(ntile, nt));
#define LM_(TT, TO, EE, NB) hipLaunchKernelGGL((k_token_grad_mfma<TT, TO, EE, NB>), gm, dim3(256), lds, st, (const TT*)gX, \
                                            ldx, pos_of, T, k, nt, g_raw, Wfc, (TO*)out, ldo)
#define LMC_(TT, TO, EE) if (C == 128) LM_(TT, TO, EE, 2); else if (C == 256) LM_(TT, TO, EE, 4); else LM_(TT, TO, EE, 8)
#define LME_(TT, TO) if (E == 8) { LMC_(TT, TO, 8); } else if (E == 16) { LMC_(TT, TO, 16); } else { LMC_(TT, TO, 32); }
    if (dtype == MG_F32) { if (out_dtype == MG_F32) { LME_(float, float); } else { LME_(float, bf16_t); } }
    else { if (out_dtype == MG_F32) { LME_(bf16_t, float); } else { LME_(bf16_t, bf16_t); } }
#undef LME_
#undef LMC_
#undef LM_
    return mg_check_launch("mg_moe_token_grad");
  }
  if (C % 8 == 0 && (!gX || (ldx % 8 == 0 && mg_al16(gX))) && ldo % 8 == 0 && mg_al16(out) && n / 8 < (1LL << 31) &&
      (E == 4 || E == 8 || E == 16 || E == 32) && mg_al16(g_raw) && (size_t)C * E * 4 <= 65536) {
    const size_t lds = (size_t)C * E * sizeof(float);
    // grid sized to fill the chip once (each block stages Wfc), grid-stride over the rest
    const int blocks = (int)std::min<int64_t>(nblk(n / 8), 2048);
#define LV_(TT, TO, EE) hipLaunchKernelGGL((k_token_grad_v<TT, TO, EE>), dim3(blocks), dim3(256), lds, st, (const TT*)gX, ldx, pos_of, T, k, C, g_raw, Wfc, (TO*)out, ldo)
#define LVE_(TT, TO) if (E == 4) LV_(TT, TO, 4); else if (E == 8) LV_(TT, TO, 8); else if (E == 16) LV_(TT, TO, 16); else LV_(TT, TO, 32)
    if (dtype == MG_F32) { if (out_dtype == MG_F32) { LVE_(float, float); } else { LVE_(float, bf16_t); } }
    else { if (out_dtype == MG_F32) { LVE_(bf16_t, float); } else { LVE_(bf16_t, bf16_t); } }
#undef LVE_
#undef LV_
    return mg_check_launch("mg_moe_token_grad");
  }
#define L_(TT, TO) hipLaunchKernelGGL((k_token_grad<TT, TO>), dim3(nblk(n)), dim3(256), 0, st, (const TT*)gX, ldx, pos_of, T, k, C, g_raw, Wfc, E, (TO*)out, ldo)
  if (dtype == MG_F32) { if (out_dtype == MG_F32) L_(float, float); else L_(float, bf16_t); }
  else { if (out_dtype == MG_F32) L_(bf16_t, float); else L_(bf16_t, bf16_t); }
#undef L_
  return mg_check_launch("mg_moe_token_grad");
}

extern "C" int mg_router_feat_grad(int dtype, const void* tok, int64_t ld, int T, int C, const float* g_raw, int E,
                                   float* G1, void* stream) {
  MG_REQUIRE(E == 4 || E == 8 || E == 16 || E == 32, "E must be 4, 8, 16 or 32");
  MG_REQUIRE(C <= 512, "C <= 512");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int CV = E <= 8 ? 8 : (E == 16 ? 4 : 2);
  if (C % CV == 0 && C / CV <= 256 && (256 % (C / CV)) == 0 && ld % 8 == 0 && mg_al16(tok) && mg_al16(g_raw) &&
      T > 0) {
    // channel groups (grid y) of at most 64 lanes x CV channels: at 32 experts (CV = 2) a 512-channel block was 256
    // channel lanes x ONE token lane walking its whole chunk serially (120 us for the 4x4 block's 4096 tokens at C5)
    const int Cb = std::min(C, 64 * CV), CG = C / Cb;
    const int TX = Cb / CV, TY = 256 / TX, R = TY / (TX < 64 ? 64 / TX : 1);
    const int rows_per_block = (R > 1 && rfg_fold_floats(R, CV * E, TX) <= kRfgFoldMax) ? 1 : R;  // in-block LDS fold
    // ~1024 blocks with at most 4 M floats of partial rows (at 32 experts the old 256-block / 1 M-float budget
    // left 64 blocks walking 1024 tokens each: 175 us for the 16x16 block's 65536 tokens at C5)
    int chunk = std::max(TY, (T / 1024 + TY - 1) / TY * TY);
    // and >= 2E tokens per block, so the partial rows (C x E fp32 per block) stay within the token bytes read
    // (C x 2 per token): at the 4x4 block (T = 4096, C = 512) 4-token chunks wrote 16 MB of partials for 4 MB of tokens
    chunk = std::max(chunk, (2 * E + TY - 1) / TY * TY);
    const int64_t row = (int64_t)rows_per_block * C * E;
    const int64_t min_chunk = ((int64_t)T * row / (4 << 20) + TY - 1) / TY * TY;
    if (min_chunk > chunk) chunk = (int)min_chunk;
    const int nb = cdiv(T, chunk);
    bool deferred = false;
    float* part = mg_fold_partials((size_t)nb * rows_per_block * C * E * sizeof(float), st, &deferred);
    MG_REQUIRE(part != nullptr, "mg_router_feat_grad: no workspace");
    const size_t smem = rows_per_block == 1 ? (size_t)rfg_fold_floats(R, CV * E, TX) * sizeof(float) : 0;
#define LV_(TT, EE, CC)                                                                                              \
  do {                                                                                                              \
    if (smem > 65536)                                                                                               \
      MG_REQUIRE(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_router_feat_grad_v<TT, EE, CC>),              \
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem) == hipSuccess,          \
                 "mg_router_feat_grad: dynamic LDS limit");                                                         \
    hipLaunchKernelGGL((k_router_feat_grad_v<TT, EE, CC>), dim3(nb, CG), dim3(256), smem, st, (const TT*)tok, ld, T, \
                       C, g_raw, chunk, part);                                                                      \
  } while (0)
#define LVE_(TT) if (E == 4) LV_(TT, 4, 8); else if (E == 8) LV_(TT, 8, 8); else if (E == 16) LV_(TT, 16, 4); \
                 else LV_(TT, 32, 2)
    if (dtype == MG_F32) { LVE_(float); } else { LVE_(bf16_t); }
#undef LVE_
#undef LV_
    // the partial rows' fold (mg_fold.hip; the G1 consumers, the router-parameter GEMMs, run after the flush)
    mg_fold_rows_submit(mg_fold_rows{part, C * E, nb * rows_per_block, C * E, C * E, G1, nullptr}, deferred, st);
    return mg_check_launch("mg_router_feat_grad");
  }
  // ~512 blocks (a 64-token step per LDS refill); per-block partial rows folded by a rows fold (mg_fold.hip)
  int chunk = std::max(64, std::min(256, (T / 512) / 64 * 64));
  dim3 grid(cdiv(T, chunk));
  int thr = ((C + 63) / 64) * 64;
  bool deferred = false;
  float* part = mg_fold_partials((size_t)grid.x * C * E * sizeof(float), st, &deferred);
#define L_(TT, EE) hipLaunchKernelGGL((k_router_feat_grad<TT, EE>), grid, dim3(thr), 0, st, (const TT*)tok, ld, T, C, g_raw, chunk, G1, part)
#define LE_(TT) if (E == 4) L_(TT, 4); else if (E == 8) L_(TT, 8); else if (E == 16) L_(TT, 16); else L_(TT, 32)
  if (dtype == MG_F32) { LE_(float); } else { LE_(bf16_t); }
#undef LE_
#undef L_
  if (part) mg_fold_rows_submit(mg_fold_rows{part, C * E, (int)grid.x, C * E, C * E, G1, nullptr}, deferred, st);
  return mg_check_launch("mg_router_feat_grad");
}

extern "C" int mg_grouped_colsum(int dtype, const void* X, int64_t ld, const int32_t* idx, int idx_div, const float* rs,
                                 const int32_t* row_off, int G, int N, int max_rows, float* out, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (mg_det() && N % 8 == 0 && ld % 8 == 0 && mg_al16(X) && max_rows > 0) {  // deterministic mode
    const int cv = N / 8, tx = std::min(cv, 32), ty = 256 / tx;
    const int cblk = cdiv(cv, tx);
    const int rpb = std::max(64, cdiv(max_rows, std::max(1, 256 / cblk)));
    const int nch = cdiv(max_rows, rpb);
    float* part = reinterpret_cast<float*>(mg_workspace((size_t)nch * G * N * sizeof(float), st));
    if (!part) return MG_ERR_LAUNCH;
    dim3 grid(cblk, nch), blk(tx, ty);
    if (dtype == MG_F32)
      hipLaunchKernelGGL(k_grouped_colsum_part<float>, grid, blk, 0, st, (const float*)X, ld, idx,
                         idx_div > 0 ? idx_div : 1, rs, row_off, G, N, rpb, part);
    else
      hipLaunchKernelGGL(k_grouped_colsum_part<bf16_t>, grid, blk, 0, st, (const bf16_t*)X, ld, idx,
                         idx_div > 0 ? idx_div : 1, rs, row_off, G, N, rpb, part);
    hipLaunchKernelGGL(k_grouped_colsum_fold, dim3(cdiv((int64_t)G * N, 256)), dim3(256), 0, st, part, row_off, G, N,
                       rpb, out);
    return mg_check_launch("mg_grouped_colsum (deterministic)");
  }
  if (N % 8 == 0 && ld % 8 == 0 && mg_al16(X) && max_rows > 0) {
    // 1024-thread blocks, ~256 of them (one per CU, 64 KiB of loads in flight each): a quarter of the
    // same-address atomics of 1024 small blocks, at least 8 rows per row lane
    const int cv = N / 8, tx = std::min(cv, 64), ty = 1024 / tx;
    const int cblk = cdiv(cv, tx);
    int rpb = std::max(8 * ty, cdiv(max_rows, std::max(1, 256 / cblk)));
    dim3 grid(cblk, cdiv(max_rows, rpb)), blk(tx, ty);
    if (dtype == MG_F32)
      hipLaunchKernelGGL((k_grouped_colsum_v<float, 1024>), grid, blk, 0, st, (const float*)X, ld, idx,
                         idx_div > 0 ? idx_div : 1, rs, row_off, G, N, rpb, out);
    else
      hipLaunchKernelGGL((k_grouped_colsum_v<bf16_t, 1024>), grid, blk, 0, st, (const bf16_t*)X, ld, idx,
                         idx_div > 0 ? idx_div : 1, rs, row_off, G, N, rpb, out);
    return mg_check_launch("mg_grouped_colsum");
  }
  int rpb = std::max(64, max_rows / 512);
  dim3 grid(cdiv(N, 256), cdiv(max_rows, rpb));
  if (dtype == MG_F32)
    hipLaunchKernelGGL(k_grouped_colsum<float>, grid, dim3(256), 0, st, (const float*)X, ld, idx, idx_div > 0 ? idx_div : 1, rs, row_off, G, N, rpb, out);
  else
    hipLaunchKernelGGL(k_grouped_colsum<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)X, ld, idx, idx_div > 0 ? idx_div : 1, rs, row_off, G, N, rpb, out);
  return mg_check_launch("mg_grouped_colsum");
}

extern "C" int mg_router_kl(const float* mu_f, const float* rho_f, int nf, const float* mu_t, const float* rho_t,
                            int nt, const float* mu_c, const float* rho_c, int nc, float* out, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t n = (int64_t)nf + nt + nc;
  // up to 256 partials (~2 elements per thread: a longer grid-stride loop is one load round trip per element)
  // in this stream's workspace block (reuse is ordered by the stream)
  int nparts = (int)std::min<int64_t>(256, std::max<int64_t>(1, cdiv(n, 512)));
  float* s_part = reinterpret_cast<float*>(mg_workspace(256 * sizeof(float), st));
  MG_REQUIRE(s_part, "no workspace");
  hipLaunchKernelGGL(k_router_kl_part, dim3(nparts), dim3(256), 0, st, mu_f, rho_f, nf, mu_t, rho_t, nt, mu_c, rho_c,
                     nc, s_part);
  hipLaunchKernelGGL(k_router_kl_fin, dim3(1), dim3(64), 0, st, s_part, nparts, out);
  return mg_check_launch("mg_router_kl");
}

extern "C" int mg_router_kl_batch(int n, const mg_kl_rec* recs, float* out, void* stream) {
  MG_REQUIRE(n >= 1 && n <= KL_MAX_RECS && recs && out, "mg_router_kl_batch: 1..8 records");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  KlBatch b{};
  int maxp = 1;
  for (int j = 0; j < n; ++j) {
    b.r[j] = recs[j];
    const int64_t m = (int64_t)recs[j].nf + recs[j].nt + recs[j].nc;
    b.nparts[j] = (int)std::min<int64_t>(256, std::max<int64_t>(1, cdiv(m, 512)));  // as mg_router_kl
    maxp = std::max(maxp, b.nparts[j]);
  }
  float* s_part = reinterpret_cast<float*>(mg_workspace((size_t)256 * n * sizeof(float), st));
  MG_REQUIRE(s_part, "no workspace");
  hipLaunchKernelGGL(k_router_kl_part_batch, dim3(maxp, n), dim3(256), 0, st, b, s_part);
  hipLaunchKernelGGL(k_router_kl_fin_batch, dim3(n), dim3(64), 0, st, b, s_part, out);
  return mg_check_launch("mg_router_kl_batch");
}

extern "C" int mg_router_param_bwd(const float* mu, const float* rho, const float* eps, const float* gW, int64_t n,
                                   const float* kl_coef, float* gmu, float* grho, const int32_t* flags, int32_t mask,
                                   void* stream) {
  MG_REQUIRE(!gW || eps, "eps required with gW");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_router_param_bwd, dim3(nblk(n)), dim3(256), 0, st, mu, rho, eps, gW, n, kl_coef, gmu, grho,
                     flags, mask);
  return mg_check_launch("mg_router_param_bwd");
}

extern "C" int mg_router_param_bwd_batch(int n, const mg_router_param_desc* descs, const int32_t* flags, int32_t mask,
                                         void* stream) {
  MG_REQUIRE(n >= 0 && n <= MG_RPB_MAX, "0 <= n <= 32 descriptors");
  if (n == 0) return MG_OK;
  RpbBatch b{};
  b.n = n;
  b.blk_off[0] = 0;
  for (int i = 0; i < n; ++i) {
    MG_REQUIRE(!descs[i].gW || descs[i].eps, "eps required with gW");
    MG_REQUIRE(descs[i].n >= 0, "n >= 0");
    b.d[i] = descs[i];
    b.blk_off[i + 1] = b.blk_off[i] + std::max(1, nblk(descs[i].n));
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_router_param_bwd_batch, dim3(b.blk_off[n]), dim3(256), 0, st, b, flags, mask);
  return mg_check_launch("mg_router_param_bwd_batch");
}

extern "C" int mg_balance(const float* load, int E, float T, float weight, float grad_scale, float* out, float* coef,
                          void* stream) {
  MG_REQUIRE(E >= 2 && E <= 64, "E out of range");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_balance, dim3(1), dim3(64), 0, st, load, E, T, weight, grad_scale, out, coef);
  return mg_check_launch("mg_balance");
}
