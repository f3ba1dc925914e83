// Gradient folds: the second pass of every two-pass gradient reduction (split-K weight-gradient slabs, per-image
// and per-block partial rows), immediate or deferred to one batched launch per backward.
//
// The weight gradients of the step are produced in two passes so that no two workgroups add into the same
// address: the first pass writes partial slabs / rows, the fold sums them in a fixed order into the parameter
// gradient.  Every fold was its own launch (~5-8 us of mostly launch latency each; ~30 per C2 step: the conv
// weight-gradient slabs, the MTM offset-head rows, the router feature and temperature rows).  Nothing reads those
// gradients before the optimizer (or, for the router feature rows, before the batched router-parameter GEMMs at
// the end of the backward), so with deferral on (mg_fold_defer) a producer writes its partials into a per-stream
// arena that is not reused until mg_fold_flush, records the fold, and the flush runs all recorded folds as one
// launch per fold kind.  Immediate folds run through the same kernels with one record, so a gradient is
// bit-identical whether its fold was deferred or not.
//
// Kinds:
//   rows: out[i] += sum_r src[r * stride + i] for i < ncols (i >= na: out_b[i - na]); 16 row lanes per column,
//         lanes in order (the order of the per-producer fold kernels it replaced)
//   wgrad: gw[o][ci][tap] += sum_s ws[s][o][tap * Cin + ci] (split-K slabs of a conv weight gradient folded into the
//         reference [Cout][Cin][KH][KW] layout, four slabs in flight, fixed order)
#include <mutex>
#include <vector>

#include "mg_common.h"

namespace {

constexpr int kFoldMax = 40;  // records per launch (kernel arguments stay below 4 KiB)

// A launch's records; blk_off: each record's first block (a chained record has no blocks of its own: the blocks of
// its chain head run it after the head, next[] linking the chain in submission order, -1 ending it)
template <typename R>
struct Batch {
  R r[kFoldMax];
  int blk_off[kFoldMax + 1];
  int next[kFoldMax];
  int n;
};
using RowsBatch = Batch<mg_fold_rows>;
using WgradBatch = Batch<mg_fold_wgrad>;

MG_DEV int find_rec(const int* blk_off, int n) {
  int d = 0;
  while (d + 1 < n && (int)blockIdx.x >= blk_off[d + 1]) ++d;
  return d;
}

// a record folds 4-column vectors (16-B loads) when its columns, pitch, pointers and split point allow
__host__ __device__ inline bool rows_vec(const mg_fold_rows& q) {
  return (q.ncols % 4) == 0 && (q.stride % 4) == 0 && (q.na % 4) == 0 && mg_al16(q.src) && mg_al16(q.out_a) &&
         (q.na >= q.ncols || mg_al16(q.out_b));
}

// Two block shapes, chosen per record:
//   thin (nrows <= 16: the split-K slabs of the grouped expert weight gradients, a few rows of up to millions of
//        columns): 1024 column lanes, each summing its rows in order -- one 16-B load per row, every lane busy;
//   wide (more rows: the per-image / per-block partial rows): 64 column lanes x 16 row lanes, lane y summing rows
//        y, y + 16, ..., then the 16 lanes in order.
// For nrows <= 16 both orders are the same sequential sum 0 + row 0 + row 1 + ... (the wide form only adds zeros
// after it), so a record folds bit-identically whichever shape it gets.  A lane owns 4 consecutive columns in
// vector records.
__host__ __device__ inline bool rows_thin(const mg_fold_rows& q) { return q.nrows <= 16; }

MG_DEV void fold_rows_block(const mg_fold_rows& q, int blk, f32x4_t (*red)[64]) {
  const bool vec = rows_vec(q);
  const int w = vec ? 4 : 1;
  if (rows_thin(q)) {
    const int i = (blk * 1024 + threadIdx.x) * w;
    if (i >= q.ncols) return;
    float* o = i < q.na ? q.out_a + i : q.out_b + (i - q.na);
    if (vec) {
      f32x4_t v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (r < q.nrows) v[r] = *reinterpret_cast<const f32x4_t*>(q.src + (int64_t)r * q.stride + i);
      f32x4_t t = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (r < q.nrows) t += v[r];
      *reinterpret_cast<f32x4_t*>(o) += t;
    } else {
      float t = 0.f;
      for (int r = 0; r < q.nrows; ++r) t += q.src[(int64_t)r * q.stride + i];
      o[0] += t;
    }
    return;
  }
  const int cx = threadIdx.x & 63, ry = threadIdx.x >> 6;
  const int i = (blk * 64 + cx) * w;
  f32x4_t s = f32x4_t{0.f, 0.f, 0.f, 0.f};
  if (i < q.ncols) {
    if (vec) {
      for (int r = ry; r < q.nrows; r += 16) s += *reinterpret_cast<const f32x4_t*>(q.src + (int64_t)r * q.stride + i);
    } else {
      for (int r = ry; r < q.nrows; r += 16) s[0] += q.src[(int64_t)r * q.stride + i];
    }
  }
  red[ry][cx] = s;
  __syncthreads();
  if (ry == 0 && i < q.ncols) {
    f32x4_t t = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int y = 0; y < 16; ++y) t += red[y][cx];
    float* o = i < q.na ? q.out_a + i : q.out_b + (i - q.na);
    if (vec) *reinterpret_cast<f32x4_t*>(o) += t;
    else o[0] += t[0];
  }
  __syncthreads();  // (red is reused by the next record of the chain)
}

__global__ __launch_bounds__(1024) void k_fold_rows_batch(RowsBatch b) {
  __shared__ f32x4_t red[16][64];
  int d = find_rec(b.blk_off, b.n);
  const int blk = blockIdx.x - b.blk_off[d];
  for (; d >= 0; d = b.next[d]) fold_rows_block(b.r[d], blk, red);
}

inline int rows_blocks(const mg_fold_rows& q) {
  return std::max(1, cdiv(q.ncols, (rows_thin(q) ? 1024 : 64) * (rows_vec(q) ? 4 : 1)));
}

// block (o, chunk of CC input channels) of one record.  Its taps x CC values are nv 16-B vectors; the 256 threads
// split as G = 256 / nv split groups (G = 1 when nv >= 128) x nv vectors, group g summing slabs g, g + G, ... in
// order (eight loads in flight), then the groups folded in order through LDS -- every thread busy even for the
// narrow chunks (CC = 8 or 16: nv = 18 or 36) whose single-group form left 7 of 8 threads idle behind serial
// split loads.  The chunk is written in the reference [Cout][Cin][taps] order.
MG_DEV void fold_wgrad_block(const mg_fold_wgrad& q, int lb, f32x4_t* lds4) {
  const int Cin = 1 << q.lgCin, N = q.taps << q.lgCin, CC = 1 << q.lgCC;
  const int64_t MN = (int64_t)q.Cout * N;
  const int nch = Cin >> q.lgCC;
  const int o = lb / nch, c0 = (lb - o * nch) << q.lgCC;
  const float* src = q.ws + (int64_t)o * N + c0;
  const int nv = (q.taps << q.lgCC) >> 2;  // 16-B vectors of this block
  const int G = nv >= 128 ? 1 : min(256 / nv, q.splits);
  const int SP = (CC >> 2) + 1;  // seg row pitch in vectors (+1: the transposed reads below walk taps, not banks)
  f32x4_t* seg4 = lds4 + (G > 1 ? G * nv : 0);
  const int gi = threadIdx.x / nv;
  for (int v = threadIdx.x - gi * nv; gi < G && v < nv; v += (G > 1 ? nv : 256)) {
    const int tap = (4 * v) >> q.lgCC, ci = (4 * v) & (CC - 1);
    const float* p = src + ((int64_t)tap << q.lgCin) + ci;
    // slabs gi, gi + G, ... eight loads in flight (past the last slab: zeros), summed as a fixed tree
    f32x4_t acc = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int s = gi; s < q.splits; s += 8 * G) {
      f32x4_t a[8];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        a[k] = s + k * G < q.splits ? *reinterpret_cast<const f32x4_t*>(p + (int64_t)(s + k * G) * MN)
                                    : f32x4_t{0.f, 0.f, 0.f, 0.f};
      acc += ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    }
    if (G > 1) lds4[gi * nv + v] = acc;
    else seg4[tap * SP + (ci >> 2)] = acc;
    if (G > 1) break;
  }
  if (G > 1) {
    __syncthreads();
    for (int v = threadIdx.x; v < nv; v += 256) {
      f32x4_t t = lds4[v];
      for (int g = 1; g < G; ++g) t += lds4[g * nv + v];
      seg4[((4 * v) >> q.lgCC) * SP + (((4 * v) & (CC - 1)) >> 2)] = t;
    }
  }
  __syncthreads();
  const float* seg = reinterpret_cast<const float*>(seg4);
  float* dst = q.gw + ((int64_t)o * Cin + c0) * q.taps;
  for (int j = threadIdx.x; j < (q.taps << q.lgCC); j += 256) {  // j = ci_local * taps + tap (reference order)
    const int ci = j / q.taps, tap = j - ci * q.taps;
    dst[j] += seg[tap * 4 * SP + ci];
  }
  __syncthreads();  // (the LDS is reused by the next record of the chain)
}

__global__ __launch_bounds__(256) void k_fold_wgrad_batch(WgradBatch b) {
  extern __shared__ f32x4_t lds4[];  // [G][nv] group partials, then [nv] folded (seg)
  int d = find_rec(b.blk_off, b.n);
  const int lb = blockIdx.x - b.blk_off[d];
  for (; d >= 0; d = b.next[d]) fold_wgrad_block(b.r[d], lb, lds4);
}

inline int wgrad_groups(const mg_fold_wgrad& q) {
  const int nv = (q.taps << q.lgCC) >> 2;
  return nv >= 128 ? 1 : std::min(256 / nv, q.splits);
}
inline size_t wgrad_lds(const mg_fold_wgrad& q) {
  const int nv = (q.taps << q.lgCC) >> 2, G = wgrad_groups(q);
  return (size_t)((G > 1 ? G * nv : 0) + nv + q.taps) * 16;
}

inline int wgrad_blocks(const mg_fold_wgrad& q) { return q.Cout * ((1 << q.lgCin) >> q.lgCC); }

// Records of one launch run concurrently and add with plain read-modify-writes, so two records whose outputs
// overlap (the real, fake and R1 weight gradients of one discriminator conv) must not share a launch: each record
// goes to level 1 + the highest level of an earlier record it overlaps, and the levels launch in order -- every
// output still receives its folds in submission order (bit-identical to immediate folds).
struct Span {
  uintptr_t lo, hi;
};
inline bool overlap(const Span& a, const Span& b) { return a.lo < b.hi && b.lo < a.hi; }
inline void spans(const mg_fold_rows& q, Span* s, int* ns) {
  *ns = 0;
  const int na = std::min(q.na, q.ncols);
  if (na > 0) s[(*ns)++] = Span{(uintptr_t)q.out_a, (uintptr_t)(q.out_a + na)};
  if (q.ncols > na) s[(*ns)++] = Span{(uintptr_t)q.out_b, (uintptr_t)(q.out_b + (q.ncols - na))};
}
inline void spans(const mg_fold_wgrad& q, Span* s, int* ns) {
  *ns = 1;
  s[0] = Span{(uintptr_t)q.gw, (uintptr_t)(q.gw + (int64_t)q.Cout * (q.taps << q.lgCin))};
}
// records with the same output and block mapping chain (one launch folds them in order, block by block); other
// overlapping outputs take levels
inline bool same_target(const mg_fold_rows& a, const mg_fold_rows& b) {
  return a.out_a == b.out_a && a.out_b == b.out_b && a.ncols == b.ncols && a.na == b.na && rows_vec(a) == rows_vec(b) &&
         rows_thin(a) == rows_thin(b);
}
inline bool same_target(const mg_fold_wgrad& a, const mg_fold_wgrad& b) {
  return a.gw == b.gw && a.Cout == b.Cout && a.lgCin == b.lgCin && a.taps == b.taps && a.lgCC == b.lgCC;
}
inline int nblocks(const mg_fold_rows& q) { return rows_blocks(q); }
inline int nblocks(const mg_fold_wgrad& q) { return wgrad_blocks(q); }
inline size_t lds_bytes(const mg_fold_rows&) { return 0; }
inline size_t lds_bytes(const mg_fold_wgrad& q) { return wgrad_lds(q); }
constexpr int kChainMax = 8;

template <typename R>
void launch_folds(const R* recs, int n, hipStream_t st, void (*kern)(Batch<R>), int threads) {
  // chains: head[i] = the first earlier record with the same target (or i), at most kChainMax per chain
  std::vector<int> head(n), len(n, 0);
  for (int i = 0; i < n; ++i) {
    head[i] = i;
    for (int j = 0; j < i; ++j)
      if (head[j] == j && len[j] < kChainMax && same_target(recs[j], recs[i])) {
        head[i] = j;
        break;
      }
    ++len[head[i]];
  }
  // levels of the chain heads
  std::vector<int> lev(n, 0);
  std::vector<Span> sp(2 * n);
  std::vector<int> ns(n);
  int nlev = 0;
  for (int i = 0; i < n; ++i) {
    spans(recs[i], &sp[2 * i], &ns[i]);
    if (head[i] != i) continue;
    for (int j = 0; j < i; ++j) {
      if (head[j] != j) continue;
      for (int a = 0; a < ns[i]; ++a)
        for (int c = 0; c < ns[j]; ++c)
          if (overlap(sp[2 * i + a], sp[2 * j + c])) lev[i] = std::max(lev[i], lev[j] + 1);
    }
    nlev = std::max(nlev, lev[i] + 1);
  }
  for (int l = 0; l < nlev; ++l) {
    Batch<R> b{};
    size_t lds = 0;
    auto launch = [&]() {
      if (b.n > 0) hipLaunchKernelGGL(kern, dim3(b.blk_off[b.n]), dim3(threads), lds, st, b);
      b = Batch<R>{};
      lds = 0;
    };
    for (int i = 0; i < n; ++i) {
      if (head[i] != i || lev[i] != l) continue;
      if (b.n + len[i] > kFoldMax) launch();
      int prev = -1;
      for (int k = i; k < n; ++k) {  // the chain, in submission order
        if (head[k] != i) continue;
        const int slot = b.n++;
        b.r[slot] = recs[k];
        b.next[slot] = -1;
        b.blk_off[slot + 1] = b.blk_off[slot] + (prev < 0 ? nblocks(recs[k]) : 0);
        if (prev >= 0) b.next[prev] = slot;
        prev = slot;
        lds = std::max(lds, lds_bytes(recs[k]));
      }
    }
    launch();
  }
}

void launch_rows(const mg_fold_rows* recs, int n, hipStream_t st) {
  launch_folds(recs, n, st, k_fold_rows_batch, 1024);
}

void launch_wgrad(const mg_fold_wgrad* recs, int n, hipStream_t st) {
  launch_folds(recs, n, st, k_fold_wgrad_batch, 256);
}

// ---- per-stream deferral state: pending records and the partials arena ----
struct Chunk {
  char* p;
  size_t bytes;
};
struct Defer {
  int device;
  hipStream_t stream;
  bool on;
  std::vector<mg_fold_rows> rows;
  std::vector<mg_fold_wgrad> wgrad;
  std::vector<Chunk> chunks;
  size_t ci, used;  // current chunk, bytes used in it
};
std::mutex g_fold_mu;
std::vector<Defer> g_defer;
// device bytes one stream's partials arena may hold (C2 step: ~0.3 GB on the capture stream)
constexpr size_t kFoldArenaCap = (size_t)2 << 30;

Defer* defer_entry(hipStream_t st, bool create) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  for (auto& d : g_defer)
    if (d.device == dev && d.stream == st) return &d;
  if (!create) return nullptr;
  g_defer.push_back(Defer{dev, st, false, {}, {}, {}, 0, 0});
  return &g_defer.back();
}

}  // namespace

void* mg_fold_alloc(size_t bytes, hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_fold_mu);
  Defer* d = defer_entry(st, false);
  if (!d || !d->on) return nullptr;
  bytes = (bytes + 255) & ~(size_t)255;
  while (d->ci < d->chunks.size() && d->used + bytes > d->chunks[d->ci].bytes) {
    ++d->ci;
    d->used = 0;
  }
  if (d->ci == d->chunks.size()) {
    // a new chunk: only outside stream capture (the eager warm-up of a captured step sizes the arena, and the
    // capture then replays the same allocation sequence); under capture the caller folds immediately instead
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    // capped per stream: past the cap the producer folds immediately (same kernels, bit-identical gradients)
    size_t held = 0;
    for (const Chunk& c : d->chunks) held += c.bytes;
    const size_t chunk = std::max(bytes, (size_t)64 << 20);
    if (held + chunk > kFoldArenaCap) return nullptr;
    Chunk c{nullptr, chunk};
    if (hipMalloc(reinterpret_cast<void**>(&c.p), c.bytes) != hipSuccess) return nullptr;
    d->chunks.push_back(c);
    d->used = 0;
  }
  void* p = d->chunks[d->ci].p + d->used;
  d->used += bytes;
  return p;
}

int mg_fold_rows_submit(const mg_fold_rows& r, bool deferred, hipStream_t st) {
  if (deferred) {
    std::lock_guard<std::mutex> lk(g_fold_mu);
    Defer* d = defer_entry(st, false);
    if (d && d->on) {
      d->rows.push_back(r);
      return MG_OK;
    }
  }
  launch_rows(&r, 1, st);
  return MG_OK;
}

int mg_fold_wgrad_submit(const mg_fold_wgrad& r, bool deferred, hipStream_t st) {
  if (deferred) {
    std::lock_guard<std::mutex> lk(g_fold_mu);
    Defer* d = defer_entry(st, false);
    if (d && d->on) {
      d->wgrad.push_back(r);
      return MG_OK;
    }
  }
  launch_wgrad(&r, 1, st);
  return MG_OK;
}

extern "C" int mg_fold_flush(void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  std::vector<mg_fold_rows> rows;
  std::vector<mg_fold_wgrad> wg;
  {
    std::lock_guard<std::mutex> lk(g_fold_mu);
    Defer* d = defer_entry(st, false);
    if (!d) return MG_OK;
    rows.swap(d->rows);
    wg.swap(d->wgrad);
    d->ci = 0;  // the arena is reused from the start by the next backward
    d->used = 0;
  }
  if (!wg.empty()) launch_wgrad(wg.data(), (int)wg.size(), st);
  if (!rows.empty()) launch_rows(rows.data(), (int)rows.size(), st);
  return mg_check_launch("mg_fold_flush");
}

extern "C" int mg_fold_defer(int on, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (!on) {
    const int rc = mg_fold_flush(stream);
    std::lock_guard<std::mutex> lk(g_fold_mu);
    Defer* d = defer_entry(st, false);
    if (d) d->on = false;
    return rc;
  }
  std::lock_guard<std::mutex> lk(g_fold_mu);
  Defer* d = defer_entry(st, true);
  MG_REQUIRE(d, "no device");
  MG_REQUIRE(d->rows.empty() && d->wgrad.empty(), "mg_fold_defer: folds pending (flush first)");
  d->on = true;
  return MG_OK;
}

extern "C" int mg_fold_release(void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  std::vector<Chunk> chunks;
  {
    std::lock_guard<std::mutex> lk(g_fold_mu);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return MG_OK;
    for (size_t i = 0; i < g_defer.size(); ++i) {
      Defer& d = g_defer[i];
      if (d.device != dev || d.stream != st) continue;
      MG_REQUIRE(!d.on && d.rows.empty() && d.wgrad.empty(), "mg_fold_release: the stream still defers folds");
      chunks.swap(d.chunks);
      g_defer.erase(g_defer.begin() + i);
      break;
    }
  }
  if (!chunks.empty()) {
    // the partials may still be read by folds enqueued on the stream
    if (hipStreamSynchronize(st) != hipSuccess) {
      mg_set_error("mg_fold_release: hipStreamSynchronize failed");
      return MG_ERR_LAUNCH;
    }
    for (const Chunk& c : chunks) (void)hipFree(c.p);
  }
  return MG_OK;
}

extern "C" int64_t mg_fold_arena_bytes(void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  std::lock_guard<std::mutex> lk(g_fold_mu);
  Defer* d = defer_entry(st, false);
  if (!d) return 0;
  int64_t held = 0;
  for (const Chunk& c : d->chunks) held += (int64_t)c.bytes;
  return held;
}

extern "C" int mg_fold_rows_batch(int n, const mg_fold_rows* recs, void* stream) {
  MG_REQUIRE(n >= 0 && recs, "bad records");
  for (int i = 0; i < n; ++i)
    MG_REQUIRE(recs[i].src && recs[i].out_a && (recs[i].na >= recs[i].ncols || recs[i].out_b) && recs[i].ncols >= 0 &&
                   recs[i].nrows >= 0,
               "bad fold record");
  if (n > 0) launch_rows(recs, n, reinterpret_cast<hipStream_t>(stream));
  return mg_check_launch("mg_fold_rows_batch");
}

extern "C" int mg_fold_rows_queue(int n, const mg_fold_rows* recs, void* stream) {
  MG_REQUIRE(n >= 0 && (n == 0 || recs), "bad records");
  for (int i = 0; i < n; ++i)
    MG_REQUIRE(recs[i].src && recs[i].out_a && (recs[i].na >= recs[i].ncols || recs[i].out_b) && recs[i].ncols >= 0 &&
                   recs[i].nrows >= 0,
               "bad fold record");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  {
    std::lock_guard<std::mutex> lk(g_fold_mu);
    Defer* d = defer_entry(st, false);
    if (d && d->on) {
      d->rows.insert(d->rows.end(), recs, recs + n);
      return MG_OK;
    }
  }
  if (n > 0) launch_rows(recs, n, st);
  return mg_check_launch("mg_fold_rows_queue");
}
