// Multi-tensor launches of libmoegan_hip: the per-step weight preparation of every layer (conv weight packing,
// demodulation sums, router reparameterisation) and the bias-gradient column sums of a whole backward, each
// as ONE launch over a descriptor table passed by value in the kernel arguments (no device-side table, so a
// captured hipGraph replays it as is).  Same element maps as the single-tensor kernels of mg_prep.hip /
// mg_moe.hip, which stay the reference implementations the tests compare against.
#include "mg_common.h"

namespace {

constexpr int kMaxDesc = 32;
constexpr int kPrepThreads = 256, kPrepIlp = 4;

struct PrepArgs {
  mg_prep_desc d[kMaxDesc];
  int block_off[kMaxDesc + 1];
  int n;
};

MG_DEV float softplusf_b(float x) { return log1pf(expf(x)); }

template <typename T>
MG_DEV void prep_elem(const mg_prep_desc& q, int64_t i) {
  switch (q.kind) {
    case MG_PREP_PACK: {  // item (o, ci): wpack[o][t*Cin + ci] = W[o][ci][t] for every tap t; rows >= Cout zero
      const int ii = (int)i, taps = q.KH * q.KW;
      const int o = ii / q.Cin, ci = ii - o * q.Cin;
      T* out = reinterpret_cast<T*>(q.out) + (int64_t)o * taps * q.Cin + ci;
      const float* w = q.W + (int64_t)ii * taps;
      for (int t = 0; t < taps; ++t) stf(out, (int64_t)t * q.Cin, o < q.Cout ? w[t] : 0.f);
      break;
    }
    case MG_PREP_PACK_FLIP: {  // item (ci, o): out[ci][t'*Cout + o] = W[o][ci][taps-1-t'] (kernel flipped)
      const int ii = (int)i, taps = q.KH * q.KW;
      const int ci = ii / q.Cout, o = ii - ci * q.Cout;
      T* out = reinterpret_cast<T*>(q.out) + (int64_t)ci * taps * q.Cout + o;
      const float* w = q.W + ((int64_t)o * q.Cin + ci) * taps;
      for (int t = 0; t < taps; ++t) stf(out, (int64_t)t * q.Cout, ci < q.Cin ? w[taps - 1 - t] : 0.f);
      break;
    }
    case MG_PREP_PACK_DGRAD_S2: {  // out[cls][ci][t*Cg + co] = W[co][ci][kh(py,ty)][kw(px,tx)]  (Cout = Cg)
      const int K = 4 * q.Cout, ii = (int)i;
      const int cls = ii / (q.rows * K);
      const int r = ii - cls * q.rows * K;
      const int ci = r / K;
      const int k = r - ci * K;
      const int t = k / q.Cout, co = k - t * q.Cout;
      const int ty = t >> 1, tx = t & 1, py = cls >> 1, px = cls & 1;
      const int kh = py ? (ty ? 2 : 0) : (ty ? 3 : 1);
      const int kw = px ? (tx ? 2 : 0) : (tx ? 3 : 1);
      float v = ci < q.Cin ? q.W[(((int64_t)co * q.Cin + ci) * 4 + kh) * 4 + kw] : 0.f;
      stf(reinterpret_cast<T*>(q.out), i, v);
      break;
    }
    case MG_PREP_WSQ: {  // wsq[o][ci] = sum_taps W[o][ci][tap]^2 (fp32 out; rows >= Cout zero)
      const int taps = q.KH * q.KW;
      const int o = (int)i / q.Cin;
      float s = 0.f;
      if (o < q.Cout)
        for (int t = 0; t < taps; ++t) {
          const float w = q.W[i * taps + t];
          s += w * w;
        }
      reinterpret_cast<float*>(q.out)[i] = s;
      break;
    }
    case MG_PREP_WSQ_BWD: {  // gW[o][ci][t] += 2 W[o][ci][t] gwsq[o][ci]   (aux = gwsq)
      const int taps = q.KH * q.KW;
      float* g = reinterpret_cast<float*>(q.out);
      g[i] += 2.f * q.W[i] * q.aux[(int)i / taps];
      break;
    }
    case MG_PREP_REPARAM: {  // W = clamp(mu) + clamp(softplus(clamp(rho))) * clamp(eps)  (aux = rho, aux2 = eps)
      const float m = clampf(q.W[i], -10.f, 10.f);
      const float r = clampf(q.aux[i], -8.f, 4.f);
      const float sg = clampf(softplusf_b(r), 1e-6f, 10.f);
      const float e = clampf(q.aux2[i], -2.f, 2.f);
      reinterpret_cast<float*>(q.out)[i] = m + sg * e;
      break;
    }
    default:
      break;
  }
}

// Flipped pack through an LDS tile: (16 input channels x 32 output channels x taps) per block.  The item form
// read W[o][ci][*] with o varying across lanes (a stride of Cin * taps floats: every lane its own cache line);
// here each output channel's 16 x taps floats are read as one contiguous run and the flipped rows are written
// 32 output channels (64 B of bf16) at a time.
constexpr int kFlipTC = 16, kFlipTO = 32, kFlipMaxTaps = 9;
__host__ __device__ inline bool flip_tiled(const mg_prep_desc& q) { return q.kind == MG_PREP_PACK_FLIP && q.KH * q.KW <= kFlipMaxTaps; }

template <typename T>
MG_DEV void flip_tile(const mg_prep_desc& q, int lb) {
  __shared__ float sm[kFlipTC][kFlipMaxTaps][kFlipTO + 1];
  const int taps = q.KH * q.KW;
  const int nto = (q.Cout + kFlipTO - 1) / kFlipTO;
  const int ci0 = (lb / nto) * kFlipTC, o0 = (lb % nto) * kFlipTO;
  const int run = kFlipTC * taps;  // contiguous floats of W[o][ci0 ..][*]
  for (int e = threadIdx.x; e < kFlipTO * run; e += kPrepThreads) {
    const int oo = e / run, r = e - oo * run;
    const int cc = r / taps, t = r - cc * taps;
    const int o = o0 + oo, ci = ci0 + cc;
    sm[cc][t][oo] = (o < q.Cout && ci < q.Cin) ? q.W[((int64_t)o * q.Cin + ci) * taps + t] : 0.f;
  }
  __syncthreads();
  T* out = reinterpret_cast<T*>(q.out);
  for (int e = threadIdx.x; e < kFlipTC * taps * kFlipTO; e += kPrepThreads) {
    const int oo = e % kFlipTO, r = e / kFlipTO;
    const int cc = r / taps, tt = r - cc * taps;  // tt = flipped tap position in the output
    const int o = o0 + oo, ci = ci0 + cc;
    if (o < q.Cout && ci < q.rows) stf(out, ((int64_t)ci * taps + tt) * q.Cout + o, sm[cc][taps - 1 - tt][oo]);
  }
}

template <typename T>
__global__ __launch_bounds__(kPrepThreads) void k_prep_batch(PrepArgs a) {
  const int b = blockIdx.x;
  int p = 0;
  while (p + 1 < a.n && b >= a.block_off[p + 1]) ++p;
  const mg_prep_desc& q = a.d[p];
  if (flip_tiled(q)) {
    flip_tile<T>(q, b - a.block_off[p]);
    return;
  }
  const int64_t base = (int64_t)(b - a.block_off[p]) * kPrepThreads * kPrepIlp + threadIdx.x;
#pragma unroll
  for (int j = 0; j < kPrepIlp; ++j) {
    const int64_t i = base + (int64_t)j * kPrepThreads;
    if (i < q.n) prep_elem<T>(q, i);
  }
}

int64_t prep_count(const mg_prep_desc& q) {
  switch (q.kind) {
    case MG_PREP_PACK: return (int64_t)q.rows * q.Cin;       // one item per (row, input channel)
    case MG_PREP_PACK_FLIP: return (int64_t)q.rows * q.Cout;  // one item per (input channel, output channel)
    case MG_PREP_PACK_DGRAD_S2: return 16LL * q.rows * q.Cout;
    case MG_PREP_WSQ: return (int64_t)q.rows * q.Cin;
    case MG_PREP_WSQ_BWD: return (int64_t)q.Cout * q.Cin * q.KH * q.KW;
    case MG_PREP_REPARAM: return q.n;
    default: return -1;
  }
}

// ---- column sums ----
// A block covers CL*8 columns (8 per lane, CL column lanes, CL = min(32, ceil(C/8)) rounded up to a power of two)
// and rpb rows, split over RL = 256/CL row lanes, so narrow gradients (C = 32: 4 column lanes, 64 row lanes)
// keep every lane busy; the RL partial rows fold through LDS and one fp32 atomic per column.
struct ColsumArgs {
  mg_colsum_desc d[kMaxDesc];
  int rpb[kMaxDesc];        // rows per block
  int lcl[kMaxDesc];        // log2 of the column lanes
  int col_blocks[kMaxDesc];
  int block_off[kMaxDesc + 1];
  int n;
};

template <typename T>
MG_DEV void colsum_block(const mg_colsum_desc& q, int rpb, int lcl, int cb, int rb) {
  __shared__ float red[4096];  // RL * 8 * (CL + PAD) <= 2048 + 32 * 64
  const int CL = 1 << lcl, RL = 256 >> lcl;
  const int tx = threadIdx.x & (CL - 1), ty = threadIdx.x >> lcl;
  const T* X = reinterpret_cast<const T*>(q.X);
  const int r0 = rb * rpb, r1 = min(q.R, r0 + rpb);
  const int c = cb * CL * 8 + tx * 8;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  const bool vec = (q.C % 8 == 0) && (q.ld % 8 == 0) && mg_al16(q.X);
  if (c < q.C) {
    if (vec) {
      float t0[8], t1[8], t2[8], t3[8];
      int r = r0 + ty;
      for (; r + 3 * RL < r1; r += 4 * RL) {  // four independent row loads in flight
        ld8(X + (int64_t)r * q.ld + c, t0);
        ld8(X + (int64_t)(r + RL) * q.ld + c, t1);
        ld8(X + (int64_t)(r + 2 * RL) * q.ld + c, t2);
        ld8(X + (int64_t)(r + 3 * RL) * q.ld + c, t3);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += (t0[j] + t1[j]) + (t2[j] + t3[j]);
      }
      for (; r < r1; r += RL) {
        ld8(X + (int64_t)r * q.ld + c, t0);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += t0[j];
      }
    } else {
      for (int r = r0 + ty; r < r1; r += RL)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (c + j < q.C) acc[j] += ldf(X, (int64_t)r * q.ld + c + j);
    }
  }
  // red[ty][j][tx] (column tx * 8 + j), j rows padded by 4 words: a lane group's stores of one j are consecutive
  // words, and fold thread col (consecutive columns, so the atomics below stay coalesced) reads word
  // j * (CL + 4) + tx -- 4j + tx distinct mod 32 over 32 consecutive columns, conflict-free both ways (the plain
  // [ty][col] layout put the stores 8 words apart: 8-way)
  const int PAD = CL >= 4 ? 4 : 0, pitch = 8 * (CL + PAD);
#pragma unroll
  for (int j = 0; j < 8; ++j) red[ty * pitch + j * (CL + PAD) + tx] = acc[j];
  __syncthreads();
  const int cols = CL * 8;
  for (int col = threadIdx.x; col < cols; col += 256) {
    const int gc = cb * cols + col;
    if (gc < q.C) {
      float s = 0.f;
      const int w = (col & 7) * (CL + PAD) + (col >> 3);
      for (int y = 0; y < RL; ++y) s += red[y * pitch + w];
      atomicAdd(q.out + gc, s);
    }
  }
}

__global__ __launch_bounds__(256) void k_colsum_batch(ColsumArgs a) {
  const int b = blockIdx.x;
  int p = 0;
  while (p + 1 < a.n && b >= a.block_off[p + 1]) ++p;
  const mg_colsum_desc& q = a.d[p];
  const int lb = b - a.block_off[p];
  const int cb = lb % a.col_blocks[p], rb = lb / a.col_blocks[p];
  if (q.dtype == MG_BF16)
    colsum_block<bf16_t>(q, a.rpb[p], a.lcl[p], cb, rb);
  else
    colsum_block<float>(q, a.rpb[p], a.lcl[p], cb, rb);
}

}  // namespace

extern "C" int mg_prep_batch(int dtype, int n, const mg_prep_desc* descs, void* stream) {
  MG_REQUIRE(dtype == MG_F32 || dtype == MG_BF16, "bad dtype");
  MG_REQUIRE(n >= 0 && (n == 0 || descs), "bad descriptor table");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int i0 = 0; i0 < n; i0 += kMaxDesc) {
    PrepArgs a{};
    a.n = 0;
    int blocks = 0;
    for (int i = i0; i < n && i < i0 + kMaxDesc; ++i) {
      mg_prep_desc q = descs[i];
      const int64_t cnt = prep_count(q);
      MG_REQUIRE(cnt >= 0, "unknown prep kind");
      MG_REQUIRE(q.W && q.out, "null operand");
      MG_REQUIRE(q.kind != MG_PREP_WSQ_BWD || q.aux, "wsq_bwd needs gwsq (aux)");
      MG_REQUIRE(q.kind != MG_PREP_REPARAM || (q.aux && q.aux2), "reparam needs rho (aux) and eps (aux2)");
      MG_REQUIRE(q.kind == MG_PREP_PACK_DGRAD_S2 || q.kind == MG_PREP_REPARAM || (q.KH > 0 && q.KW > 0),
                 "bad kernel size");
      MG_REQUIRE(cnt < (1LL << 31) / 2, "descriptor too large");
      q.n = cnt;
      if (cnt == 0) continue;
      a.d[a.n] = q;
      a.block_off[a.n] = blocks;
      blocks += flip_tiled(q) ? ((q.rows + kFlipTC - 1) / kFlipTC) * ((q.Cout + kFlipTO - 1) / kFlipTO)
                              : (int)((cnt + kPrepThreads * kPrepIlp - 1) / (kPrepThreads * kPrepIlp));
      ++a.n;
    }
    a.block_off[a.n] = blocks;
    if (a.n == 0) continue;
    if (dtype == MG_BF16)
      hipLaunchKernelGGL(k_prep_batch<bf16_t>, dim3(blocks), dim3(kPrepThreads), 0, st, a);
    else
      hipLaunchKernelGGL(k_prep_batch<float>, dim3(blocks), dim3(kPrepThreads), 0, st, a);
    int rc = mg_check_launch("mg_prep_batch");
    if (rc) return rc;
  }
  return MG_OK;
}

extern "C" int mg_colsum_batch(int n, const mg_colsum_desc* descs, void* stream) {
  MG_REQUIRE(n >= 0 && (n == 0 || descs), "bad descriptor table");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (mg_det()) {  // deterministic mode: each sum by mg_colsum's fixed-order fold, one after the other
    for (int i = 0; i < n; ++i) {
      const mg_colsum_desc& q = descs[i];
      int rc = mg_colsum(q.dtype, q.X, q.ld, q.R, q.C, q.out, stream);
      if (rc) return rc;
    }
    return MG_OK;
  }
  for (int i0 = 0; i0 < n; i0 += kMaxDesc) {
    ColsumArgs a{};
    a.n = 0;
    int blocks = 0;
    for (int i = i0; i < n && i < i0 + kMaxDesc; ++i) {
      const mg_colsum_desc& q = descs[i];
      MG_REQUIRE(q.dtype == MG_F32 || q.dtype == MG_BF16, "bad dtype");
      MG_REQUIRE(q.R >= 0 && q.C >= 0 && q.ld >= q.C, "bad shape");
      MG_REQUIRE(q.R == 0 || q.C == 0 || (q.X && q.out), "null operand");
      if (q.R == 0 || q.C == 0) continue;
      int lcl = 0;
      while ((1 << lcl) < 32 && (1 << lcl) * 8 < q.C) ++lcl;
      const int cols = 8 << lcl, rl = 256 >> lcl;
      const int cbk = (q.C + cols - 1) / cols;
      // ~32K elements per block, a multiple of the row lanes
      int rpb = std::max(rl, 32768 / cols);
      rpb = (rpb + rl - 1) / rl * rl;
      const int rbk = (q.R + rpb - 1) / rpb;
      a.d[a.n] = q;
      a.rpb[a.n] = rpb;
      a.lcl[a.n] = lcl;
      a.col_blocks[a.n] = cbk;
      a.block_off[a.n] = blocks;
      blocks += cbk * rbk;
      ++a.n;
    }
    a.block_off[a.n] = blocks;
    if (a.n == 0) continue;
    hipLaunchKernelGGL(k_colsum_batch, dim3(blocks), dim3(256), 0, st, a);
    int rc = mg_check_launch("mg_colsum_batch");
    if (rc) return rc;
  }
  return MG_OK;
}
