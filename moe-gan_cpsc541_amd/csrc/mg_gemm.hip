// GEMM / implicit-conv entry points of libmoegan_hip.
#include <algorithm>
#include <string>
#include <type_traits>

#include "mg_gemm.h"
#include "mg_host.h"

using namespace mg;

namespace {


constexpr Grouping kNoGroup{0, 1, nullptr, nullptr, 0};
// plain (ungrouped) launch with the tuned XCD tile order (MG_TUNE_XCD), for the direct split-K slab launches
inline Grouping xcd_group() {  // XCD-aware block order (gemm_kernel): on unless tuning slot MG_TUNE_XCD says otherwise
  Grouping g = kNoGroup;
  const int x = g_mg_tune[MG_TUNE_XCD];
  g.swz = x == 0 ? 1 : x == 3 ? 0 : x;
  return g;
}

inline bool a_xf(const mg_epilogue* e) { return e && (e->a_idx || e->a_rowscale || e->a_gelu); }

template <typename T, typename TO, int BM, int BN, bool AK, bool BKc, bool XF, bool X3 = false>
void run_plain(int M, int N, int K, const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc,
               const mg_epilogue* e, int splits, hipStream_t st) {
  auto ep = make_epi<TO>(C, ldc, e);
  const int32_t* aidx = e ? e->a_idx : nullptr;
  int adiv = (e && e->a_idx_div > 0) ? e->a_idx_div : 1;
  const float* ars = e ? e->a_rowscale : nullptr;
  int agelu = e ? e->a_gelu : 0;
  if constexpr (AK) {
    LdKC<T, XF> la{reinterpret_cast<const T*>(A), lda, M, K, aidx, adiv, ars, agelu};
    if constexpr (BKc) {
      LdKC<T> lb{reinterpret_cast<const T*>(B), ldb, N, K, nullptr, 1, nullptr, 0};
      launch_gemm<T, BM, BN, true, true, 0, X3>(la, lb, ep, M, N, K, splits, kNoGroup, 0, st);
    } else {
      LdMC<T> lb{reinterpret_cast<const T*>(B), ldb, N, K, nullptr, 1, nullptr, 0};
      launch_gemm<T, BM, BN, true, false, 0, X3>(la, lb, ep, M, N, K, splits, kNoGroup, 0, st);
    }
  } else {
    LdMC<T, XF> la{reinterpret_cast<const T*>(A), lda, M, K, aidx, adiv, ars, agelu};
    if constexpr (BKc) {
      LdKC<T> lb{reinterpret_cast<const T*>(B), ldb, N, K, nullptr, 1, nullptr, 0};
      launch_gemm<T, BM, BN, false, true, 0, X3>(la, lb, ep, M, N, K, splits, kNoGroup, 0, st);
    } else {
      LdMC<T> lb{reinterpret_cast<const T*>(B), ldb, N, K, nullptr, 1, nullptr, 0};
      launch_gemm<T, BM, BN, false, false, 0, X3>(la, lb, ep, M, N, K, splits, kNoGroup, 0, st);
    }
  }
}

template <typename T, typename TO, int BM, int BN, bool XF = false, bool X3 = false>
void run_plain_orient(int a_kc, int b_kc, int M, int N, int K, const void* A, int64_t lda, const void* B,
                      int64_t ldb, void* C, int64_t ldc, const mg_epilogue* e, int splits, hipStream_t st) {
  if (a_kc && b_kc) run_plain<T, TO, BM, BN, true, true, XF, X3>(M, N, K, A, lda, B, ldb, C, ldc, e, splits, st);
  else if (a_kc) run_plain<T, TO, BM, BN, true, false, XF, X3>(M, N, K, A, lda, B, ldb, C, ldc, e, splits, st);
  else if (b_kc) run_plain<T, TO, BM, BN, false, true, XF, X3>(M, N, K, A, lda, B, ldb, C, ldc, e, splits, st);
  else run_plain<T, TO, BM, BN, false, false, XF, X3>(M, N, K, A, lda, B, ldb, C, ldc, e, splits, st);
}

template <typename T, typename TO, bool X3 = false>
void run_plain_tiles(int a_kc, int b_kc, int M, int N, int K, const void* A, int64_t lda, const void* B,
                     int64_t ldb, void* C, int64_t ldc, const mg_epilogue* e, int splits, hipStream_t st) {
  if constexpr (X3) {  // split-bf16 fp32 GEMMs (small-M prefix / demodulation products): 64x64 tiles only
    if (a_xf(e)) run_plain_orient<T, TO, 64, 64, true, true>(a_kc, b_kc, M, N, K, A, lda, B, ldb, C, ldc, e, splits, st);
    else run_plain_orient<T, TO, 64, 64, false, true>(a_kc, b_kc, M, N, K, A, lda, B, ldb, C, ldc, e, splits, st);
    return;
  }
  if (a_xf(e)) {  // loader transforms: generic 64x64 instantiation
    run_plain_orient<T, TO, 64, 64, true>(a_kc, b_kc, M, N, K, A, lda, B, ldb, C, ldc, e, splits, st);
    return;
  }
  const int tile = g_mg_tune[MG_TUNE_GEMM_TILE];
  // one K step (K <= BK: the D head GEMMs, K = 16 / 48): 64^2 tiles keep more blocks in flight (9.46 -> 9.44 ms per
  // step, A/B MG_TUNE_SHORTK = 2 restores the size rule below)
  if (tile == 0 && K <= Tile<T>::BK && g_mg_tune[MG_TUNE_SHORTK] != 2) {
    run_plain_orient<T, TO, 64, 64>(a_kc, b_kc, M, N, K, A, lda, B, ldb, C, ldc, e, splits, st);
    return;
  }
  // short K over many rows (the token projections, K = 128 / 256 at 16K-64K rows): each tile's K loop is one or two
  // steps, so it is bound by load latency and more, smaller tiles keep more bytes in flight (measured at the C2
  // shapes: 65536 x 256 x 128 26.5 -> 15.7 us, 65536 x 384 x 128 28.5 -> 22.5 us on 64^2;
  // profiles/round4_shortk_probe.txt)
  if (tile == 0 && K <= 256 && M >= 16384) {
    run_plain_orient<T, TO, 64, 64>(a_kc, b_kc, M, N, K, A, lda, B, ldb, C, ldc, e, splits, st);
    return;
  }
  if constexpr (sizeof(T) == 2) {
    // 128 x 256 when N fills it and the grid covers the chip (measured: 4096^3 bf16 816 -> 920 TF/s;
    // the step's few-tile projections stay on 128^2 / 64^2)
    if (tile == 257 || (tile == 0 && N % 256 == 0 && (int64_t)cdiv(M, 128) * (N / 256) * splits >= 480)) {
      run_plain_orient<T, TO, 128, 256>(a_kc, b_kc, M, N, K, A, lda, B, ldb, C, ldc, e, splits, st);
      return;
    }
  }
  if (tile == 128 || (tile == 0 && (int64_t)cdiv(M, 128) * cdiv(N, 128) * splits >= 480))
    run_plain_orient<T, TO, 128, 128>(a_kc, b_kc, M, N, K, A, lda, B, ldb, C, ldc, e, splits, st);
  else
    run_plain_orient<T, TO, 64, 64>(a_kc, b_kc, M, N, K, A, lda, B, ldb, C, ldc, e, splits, st);
}

// Few-tile GEMMs (styles, mapping, router/attention projections at small M) are latency-bound: a
// 64x64 grid of ~32 blocks walks K serially.  Split K over ~256 blocks into fp32 slabs and apply
// the real epilogue in a reduction pass.  Returns false when the shape does not qualify.
// ``want_splits`` > 0 (deterministic mode, an atomic split-K epilogue): exactly that many slabs, any tile count;
// the reduction pass then adds each output element once.
template <typename T, typename TO, bool X3 = false>
bool run_splitk_slabs(int a_kc, int b_kc, int M, int N, int K, const void* A, int64_t lda, const void* B,
                      int64_t ldb, void* C, int64_t ldc, const mg_epilogue* e, hipStream_t st, int want_splits = 0) {
  constexpr int TBK = tile_bk<T, X3, 64, 64>();
  int64_t tiles = (int64_t)cdiv(M, 64) * cdiv(N, 64);
  if (a_xf(e)) return false;
  int splits;
  if (want_splits > 0) {
    splits = std::max(1, std::min(want_splits, cdiv(K, TBK)));
  } else {
    if (tiles >= 96 || K < 4 * TBK) return false;
    splits = (int)std::min<int64_t>(256 / tiles, K / (2 * TBK));
  }
  if (splits < 2) return false;
  int kchunk = ((K + splits - 1) / splits + TBK - 1) / TBK * TBK;
  splits = (K + kchunk - 1) / kchunk;
  const int64_t MN = (int64_t)M * N;
  float* ws = reinterpret_cast<float*>(mg_workspace((size_t)splits * MN * sizeof(float), st));
  if (!ws) return false;
  mg_epilogue raw{};
  raw.alpha = 1.f;
  Epi<float> slab = make_epi<float>(ws, N, &raw);
  slab.zstride = MN;
  slab.vec_ok = slab.host_vec_ok() ? 1 : 0;
  auto ep = make_epi<TO>(C, ldc, e);
  ep.vec_ok = ep.host_vec_ok() ? 1 : 0;
  // the reduction inside the launch (last-arriving split of each tile; A/B slot MG_TUNE_SPLITK_FUSED): measured at
  // C2 no faster on the few-tile GEMMs (the agent-scope release / acquire cost what the second launch did) and
  // 30-70 % slower on the many-tile conv slabs (every block's release writes back its XCD's dirty L2 lines)
  int* cnt = g_mg_tune[MG_TUNE_SPLITK_FUSED] == 1 ? mg_tile_counters((int)tiles, st) : nullptr;
  auto go = [&](auto la, auto lb, auto akc, auto bkc) {
    dim3 grid(cdiv(M, 64), cdiv(N, 64), splits);
    if (cnt)
      hipLaunchKernelGGL((gemm_splitk_fused_kernel<T, 64, 64, decltype(akc)::value, decltype(bkc)::value,
                                                  decltype(la), decltype(lb), TO, X3>),
                         grid, dim3(NTHREADS), 0, st, la, lb, slab, ep, M, N, K, kchunk, cnt);
    else
      hipLaunchKernelGGL((gemm_kernel<T, 64, 64, decltype(akc)::value, decltype(bkc)::value, decltype(la),
                                      decltype(lb), Epi<float>, 0, X3>),
                         grid, dim3(NTHREADS), 0, st, la, lb, slab, M, N, K, kchunk, xcd_group());
  };
  const T* Ap = reinterpret_cast<const T*>(A);
  const T* Bp = reinterpret_cast<const T*>(B);
  using TT = std::true_type;
  using FF = std::false_type;
  if (a_kc) {
    LdKC<T> la{Ap, lda, M, K, nullptr, 1, nullptr, 0};
    if (b_kc) go(la, LdKC<T>{Bp, ldb, N, K, nullptr, 1, nullptr, 0}, TT{}, TT{});
    else go(la, LdMC<T>{Bp, ldb, N, K, nullptr, 1, nullptr, 0}, TT{}, FF{});
  } else {
    LdMC<T> la{Ap, lda, M, K, nullptr, 1, nullptr, 0};
    if (b_kc) go(la, LdKC<T>{Bp, ldb, N, K, nullptr, 1, nullptr, 0}, FF{}, TT{});
    else go(la, LdMC<T>{Bp, ldb, N, K, nullptr, 1, nullptr, 0}, FF{}, FF{});
  }
  if (cnt) return true;
  int blocks = (int)std::min<int64_t>(cdiv(MN, 256), 2048);
  hipLaunchKernelGGL((splitk_reduce_kernel<Epi<TO>>), dim3(blocks), dim3(256), 0, st, ws, splits, M, N, ep);
  return true;
}

}  // namespace

extern "C" int mg_gemm(int dtype, int M, int N, int K, const void* A, int64_t lda, int a_kc, const void* B,
                       int64_t ldb, int b_kc, void* C, int64_t ldc, int c_dtype, const mg_epilogue* ep, int splits,
                       void* stream) {
  MG_REQUIRE(dtype == MG_F32 || dtype == MG_BF16 || dtype == MG_F32X3, "bad dtype");
  MG_REQUIRE(M >= 0 && N >= 0 && K >= 0, "negative size");
  if (M == 0 || N == 0) return MG_OK;
  const bool x3 = dtype == MG_F32X3;
  if (x3) dtype = MG_F32;  // fp32 storage; the MFMA products run on split bf16
  const int vec = dtype == MG_F32 ? 4 : 8;
  MG_REQUIRE(aligned16(A) && aligned16(B), "A/B must be 16-byte aligned");
  MG_REQUIRE(lda % vec == 0 && ldb % vec == 0, "lda/ldb must be multiples of the 16-byte vector");
  MG_REQUIRE(a_kc ? (K % vec == 0) : (M % vec == 0), "A vector dim must be a multiple of the 16-byte vector");
  MG_REQUIRE(b_kc ? (K % vec == 0) : (N % vec == 0), "B vector dim must be a multiple of the 16-byte vector");
  MG_REQUIRE(under2g((a_kc ? (int64_t)M : K) * lda, dtype) && under2g((b_kc ? (int64_t)N : K) * ldb, dtype) &&
                 under2g((int64_t)M * ldc, c_dtype),
             "an operand exceeds 2 GiB (32-bit buffer offsets)");
  if (splits < 1 && dtype == MG_BF16 && !x3 && !a_kc && !b_kc && c_dtype == MG_F32 && ep && ep->atomic &&
      !ep->bias && !ep->scale && !ep->rowscale && !ep->act && !ep->aux && !ep->resid && !ep->accumulate &&
      !ep->remap_taps && !ep->a_idx && !ep->a_rowscale && !ep->a_gelu && !ep->addvec && !ep->out_pre &&
      mg_wgrad_wide(M, N, K, A, lda, B, ldb, reinterpret_cast<float*>(C), ldc, ep->alpha,
                    reinterpret_cast<hipStream_t>(stream)))
    return mg_check_launch("mg_gemm (wide weight gradient)");
  if (splits < 1) {  // auto split-K (atomic fp32 epilogues only): ~512 blocks, >= 256 of K per split
    if (ep && ep->atomic) {
      int64_t tiles = (int64_t)cdiv(M, 64) * cdiv(N, 64);
      const int target = g_mg_tune[MG_TUNE_ATOMIC_BLOCKS] > 0 ? (int)g_mg_tune[MG_TUNE_ATOMIC_BLOCKS] : 512;
      int64_t want = std::max<int64_t>(1, target / std::max<int64_t>(tiles, 1));
      // the least K per split: 256 (one bf16 128-deep step pair), or the tuned value (A/B: a few-tile fp32 weight
      // gradient at K = B = 256 rows otherwise walks its 4 K steps serially on 64 blocks)
      const int mink = g_mg_tune[MG_TUNE_ATOMIC_MINK] > 0 ? (int)g_mg_tune[MG_TUNE_ATOMIC_MINK] : 256;
      splits = (int)std::max<int64_t>(1, std::min<int64_t>(want, K / mink));
    } else {
      splits = 1;
    }
  }
  MG_REQUIRE(splits == 1 || (ep && ep->atomic && c_dtype == MG_F32), "split-K requires an atomic fp32 epilogue");
  MG_REQUIRE(!(ep && ep->atomic) || c_dtype == MG_F32, "atomic epilogue requires fp32 C");
  if (K == 0) splits = 1;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (splits > 1 && mg_det()) {  // deterministic mode: fp32 slabs + one fixed-order reduction, not atomics
    bool done;
    if (x3)
      done = run_splitk_slabs<float, float, true>(a_kc, b_kc, M, N, K, A, lda, B, ldb, C, ldc, ep, st, splits);
    else if (dtype == MG_F32)
      done = run_splitk_slabs<float, float>(a_kc, b_kc, M, N, K, A, lda, B, ldb, C, ldc, ep, st, splits);
    else
      done = run_splitk_slabs<bf16_t, float>(a_kc, b_kc, M, N, K, A, lda, B, ldb, C, ldc, ep, st, splits);
    if (done) return mg_check_launch("mg_gemm (deterministic split-K slabs)");
    splits = 1;
  }
  if (splits == 1 && !(ep && ep->atomic) && !g_mg_tune[MG_TUNE_NO_SLABS]) {
    bool done;
    if (x3)
      done = c_dtype == MG_F32 ? run_splitk_slabs<float, float, true>(a_kc, b_kc, M, N, K, A, lda, B, ldb, C, ldc, ep, st)
                               : run_splitk_slabs<float, bf16_t, true>(a_kc, b_kc, M, N, K, A, lda, B, ldb, C, ldc, ep, st);
    else if (dtype == MG_F32)
      done = c_dtype == MG_F32 ? run_splitk_slabs<float, float>(a_kc, b_kc, M, N, K, A, lda, B, ldb, C, ldc, ep, st)
                               : run_splitk_slabs<float, bf16_t>(a_kc, b_kc, M, N, K, A, lda, B, ldb, C, ldc, ep, st);
    else
      done = c_dtype == MG_F32 ? run_splitk_slabs<bf16_t, float>(a_kc, b_kc, M, N, K, A, lda, B, ldb, C, ldc, ep, st)
                               : run_splitk_slabs<bf16_t, bf16_t>(a_kc, b_kc, M, N, K, A, lda, B, ldb, C, ldc, ep, st);
    if (done) return mg_check_launch("mg_gemm (split-K slabs)");
  }
  if (x3) {
    if (c_dtype == MG_F32) run_plain_tiles<float, float, true>(a_kc, b_kc, M, N, K, A, lda, B, ldb, C, ldc, ep, splits, st);
    else run_plain_tiles<float, bf16_t, true>(a_kc, b_kc, M, N, K, A, lda, B, ldb, C, ldc, ep, splits, st);
  } else if (dtype == MG_F32) {
    if (c_dtype == MG_F32) run_plain_tiles<float, float>(a_kc, b_kc, M, N, K, A, lda, B, ldb, C, ldc, ep, splits, st);
    else run_plain_tiles<float, bf16_t>(a_kc, b_kc, M, N, K, A, lda, B, ldb, C, ldc, ep, splits, st);
  } else {
    if (c_dtype == MG_F32) run_plain_tiles<bf16_t, float>(a_kc, b_kc, M, N, K, A, lda, B, ldb, C, ldc, ep, splits, st);
    else run_plain_tiles<bf16_t, bf16_t>(a_kc, b_kc, M, N, K, A, lda, B, ldb, C, ldc, ep, splits, st);
  }
  return mg_check_launch("mg_gemm");
}

// ---------------------------------------------------------------------------
// batched small GEMMs
// ---------------------------------------------------------------------------
namespace {
template <typename T, typename TO, bool AK, bool BKc, bool X3 = false>
int run_batch(int n, const mg_gemm_desc* d, hipStream_t st) {
  using AL = typename std::conditional<AK, LdKC<T>, LdMC<T>>::type;
  using BL = typename std::conditional<BKc, LdKC<T>, LdMC<T>>::type;
  for (int i0 = 0; i0 < n; i0 += MG_BATCH_MAX) {
    BatchArgs<TO, AL, BL> args;
    static_assert(sizeof(args) <= 4096 && sizeof(BatchReduceArgs<TO>) <= 4096, "kernel arguments over 4 KB");
    int cnt = std::min(MG_BATCH_MAX, n - i0), tiles = 0, used = 0;
    for (int j = 0; j < cnt; ++j) {
      const mg_gemm_desc& q = d[i0 + j];
      if (q.M == 0 || q.N == 0) continue;
      const mg_epilogue* e = q.ep;
      const T* Ap = reinterpret_cast<const T*>(q.A);
      const T* Bp = reinterpret_cast<const T*>(q.B);
      args.a[used] = AL{Ap, q.lda, q.M, q.K, nullptr, 1, nullptr, 0};
      args.b[used] = BL{Bp, q.ldb, q.N, q.K, nullptr, 1, nullptr, 0};
      args.e[used] = make_epi<TO>(q.C, q.ldc, e);
      args.e[used].vec_ok = args.e[used].host_vec_ok() ? 1 : 0;
      args.M[used] = q.M;
      args.N[used] = q.N;
      args.K[used] = q.K;
      args.tiles_n[used] = cdiv(q.N, 64);
      args.tile_off[used] = tiles;
      tiles += cdiv(q.M, 64) * cdiv(q.N, 64);
      ++used;
    }
    if (!used) continue;
    args.tile_off[used] = tiles;
    args.n = used;
    // Few-tile batches (router / cross-attention value-chain products at M = batch) walk K serially in ~100
    // blocks.  Opt-in (tuning slot 21 = block target): split K into fp32 slabs, then one batched reduction applies
    // each real epilogue.  The batched GEMMs halve (12.9 -> 7.1 us average) but the reduction launches cost what
    // that saves: 8.844 / 8.826 ms per step with / without at 512 blocks (same box, three rounds), so off.
    constexpr int TBK = tile_bk<T, X3, 64, 64>();
    const int bs = g_mg_tune[MG_TUNE_BATCH_SPLIT];
    int S = 1;
    if (bs > 1) {
      const int target = bs;
      int maxK = 0;
      for (int j = 0; j < used; ++j) maxK = std::max(maxK, args.K[j]);
      if (2 * tiles <= target) S = std::min(target / tiles, maxK / (2 * TBK));
    }
    if (S >= 2) {
      BatchReduceArgs<TO> r;
      int64_t off = 0;
      int blks = 0;
      for (int j = 0; j < used; ++j) {
        const int K = args.K[j], kc = K > 0 ? cdiv(cdiv(K, S), TBK) * TBK : TBK;
        const int64_t MN = (int64_t)args.M[j] * args.N[j];
        args.kchunk[j] = kc;
        args.ws_off[j] = r.ws_off[j] = off;
        r.e[j] = args.e[j];
        r.M[j] = args.M[j];
        r.N[j] = args.N[j];
        r.splits[j] = K > 0 ? cdiv(K, kc) : 0;
        r.blk_off[j] = blks;
        off += (r.splits[j] * MN + 7) / 8 * 8;  // 32-B aligned slabs
        blks += (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(MN, args.N[j] % 8 == 0 ? 2048 : 256), 256));
      }
      r.blk_off[used] = blks;
      r.n = used;
      float* ws = reinterpret_cast<float*>(mg_workspace((size_t)std::max<int64_t>(off, 8) * sizeof(float), st));
      if (ws) {
        args.ws = ws;
        r.ws = ws;
        hipLaunchKernelGGL((gemm_batch_kernel<T, AK, BKc, AL, BL, TO, X3, true>), dim3(tiles, S), dim3(NTHREADS), 0, st,
                           args);
        hipLaunchKernelGGL((batch_reduce_kernel<TO>), dim3(blks), dim3(256), 0, st, r);
        continue;
      }
    }
    hipLaunchKernelGGL((gemm_batch_kernel<T, AK, BKc, AL, BL, TO, X3>), dim3(tiles), dim3(NTHREADS), 0, st, args);
  }
  return mg_check_launch("mg_gemm_batch");
}
}  // namespace

extern "C" int mg_gemm_batch(int dtype, int a_kc, int b_kc, int c_dtype, int n, const mg_gemm_desc* d,
                             void* stream) {
  MG_REQUIRE(dtype == MG_F32 || dtype == MG_BF16 || dtype == MG_F32X3, "bad dtype");
  const int vec = dtype == MG_BF16 ? 8 : 4;
  const int mdt = dtype == MG_F32X3 ? MG_F32 : dtype;  // storage dtype
  for (int i = 0; i < n; ++i) {
    const mg_gemm_desc& q = d[i];
    MG_REQUIRE(q.M >= 0 && q.N >= 0 && q.K >= 0, "negative size");
    MG_REQUIRE(aligned16(q.A) && aligned16(q.B), "A/B must be 16-byte aligned");
    MG_REQUIRE(q.lda % vec == 0 && q.ldb % vec == 0, "lda/ldb must be multiples of the 16-byte vector");
    MG_REQUIRE(a_kc ? (q.K % vec == 0) : (q.M % vec == 0), "A vector dim must be a multiple of the vector");
    MG_REQUIRE(b_kc ? (q.K % vec == 0) : (q.N % vec == 0), "B vector dim must be a multiple of the vector");
    MG_REQUIRE(!(q.ep && q.ep->atomic) || c_dtype == MG_F32, "atomic epilogue requires fp32 C");
    MG_REQUIRE(!a_xf(q.ep), "A loader transforms (a_idx / a_rowscale / a_gelu) are not supported by mg_gemm_batch");
    MG_REQUIRE(under2g((a_kc ? (int64_t)q.M : q.K) * q.lda, mdt) &&
                   under2g((b_kc ? (int64_t)q.N : q.K) * q.ldb, mdt) && under2g((int64_t)q.M * q.ldc, c_dtype),
               "an operand exceeds 2 GiB (32-bit buffer offsets)");
  }
  if (n <= 0) return MG_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (mg_det() && n > 1) {  // deterministic mode: descriptors may accumulate into one output -> one launch each
    bool atomic = false;
    for (int i = 0; i < n; ++i) atomic = atomic || (d[i].ep && d[i].ep->atomic);
    if (atomic) {
      for (int i = 0; i < n; ++i) {
        int rc = mg_gemm_batch(dtype, a_kc, b_kc, c_dtype, 1, d + i, stream);
        if (rc) return rc;
      }
      return MG_OK;
    }
  }
#define B_(T, TO, ...)                                                                                          \
  (a_kc ? (b_kc ? run_batch<T, TO, true, true, ##__VA_ARGS__>(n, d, st) : run_batch<T, TO, true, false, ##__VA_ARGS__>(n, d, st)) \
        : (b_kc ? run_batch<T, TO, false, true, ##__VA_ARGS__>(n, d, st) : run_batch<T, TO, false, false, ##__VA_ARGS__>(n, d, st)))
  if (dtype == MG_F32) return c_dtype == MG_F32 ? B_(float, float) : B_(float, bf16_t);
  if (dtype == MG_F32X3) return c_dtype == MG_F32 ? B_(float, float, true) : B_(float, bf16_t, true);
  return c_dtype == MG_F32 ? B_(bf16_t, float) : B_(bf16_t, bf16_t);
#undef B_
}

// ---------------------------------------------------------------------------
// implicit-GEMM convolution
// ---------------------------------------------------------------------------
namespace {
template <typename T, typename TO, int BM, int BN, bool XF = false, bool SC = false>
void run_conv(const void* x, int B, int H, int W, int Cin, const void* wpack, int Cout, int KH, int KW, int stride,
              int pad, const float* sc, void* y, int64_t ldy, const mg_epilogue* e, hipStream_t st) {
  int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  int M = B * OH * OW, K = KH * KW * Cin;
  LdKCConv<T, XF, SC> la{reinterpret_cast<const T*>(x), H, W, Cin, ilog2(Cin), ilog2(OW), ilog2(OH * OW), M,
                         KW, stride, pad, K, sc, kwinv(KW)};
  LdKC<T> lb{reinterpret_cast<const T*>(wpack), K, Cout, K, nullptr, 1, nullptr, 0};
  auto ep = make_epi<TO>(y, ldy, e);
  launch_gemm<T, BM, BN, true, true>(la, lb, ep, M, Cout, K, 1, kNoGroup, 0, st);
}
// Implicit conv with few output tiles for its K (the MTM offset heads, Cout = 32, K = 9*Cin up to 4608; the 4x4
// 512 -> 512 convs, 512 tiles of 72 K steps) walks K serially in too few blocks to hide load latency: split K into
// fp32 slabs over ~1024 blocks of >= 8 K steps each and apply the epilogue in the reduction.  Narrow outputs
// (Cout <= 32) use 128 x 32 tiles (no MFMA columns wasted).
template <typename T, typename TO, bool SC, int BM, int BN>
bool conv_slabs_t(const void* x, int B, int H, int W, int Cin, const void* wpack, int Cout, int KH, int KW,
                  int stride, int pad, const float* sc, void* y, int64_t ldy, const mg_epilogue* e, hipStream_t st) {
  constexpr int TBK = tile_bk<T, false, BM, BN>();
  int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  int M = B * OH * OW, K = KH * KW * Cin;
  int64_t tiles = (int64_t)cdiv(M, BM) * cdiv(Cout, BN);
  const int ksteps = K / TBK;
  if (tiles >= 1024 || ksteps < 16 || (e && e->atomic) || sc || g_mg_tune[MG_TUNE_NO_SLABS]) return false;
  int splits = (int)std::min<int64_t>(cdiv(1024, tiles), ksteps / 8);
  if (splits < 2) return false;
  int kchunk = ((K + splits - 1) / splits + TBK - 1) / TBK * TBK;
  splits = (K + kchunk - 1) / kchunk;
  const int64_t MN = (int64_t)M * Cout;
  float* ws = reinterpret_cast<float*>(mg_workspace((size_t)splits * MN * sizeof(float), st));
  if (!ws) return false;
  mg_epilogue raw{};
  raw.alpha = 1.f;
  Epi<float> slab = make_epi<float>(ws, Cout, &raw);
  slab.zstride = MN;
  slab.vec_ok = slab.host_vec_ok() ? 1 : 0;
  LdKCConv<T, false, SC> la{reinterpret_cast<const T*>(x), H, W, Cin, ilog2(Cin), ilog2(OW), ilog2(OH * OW), M,
                            KW, stride, pad, K, sc, kwinv(KW)};
  LdKC<T> lb{reinterpret_cast<const T*>(wpack), K, Cout, K, nullptr, 1, nullptr, 0};
  dim3 grid(cdiv(M, BM), cdiv(Cout, BN), splits);
  auto ep = make_epi<TO>(y, ldy, e);
  ep.vec_ok = ep.host_vec_ok() ? 1 : 0;
  int* cnt = g_mg_tune[MG_TUNE_SPLITK_FUSED] == 1 ? mg_tile_counters((int)tiles, st) : nullptr;
  if (cnt) {  // the reduction inside the launch (gemm_splitk_fused_kernel; A/B only, see run_splitk_slabs)
    hipLaunchKernelGGL((gemm_splitk_fused_kernel<T, BM, BN, true, true, LdKCConv<T, false, SC>, LdKC<T>, TO>), grid,
                       dim3(NTHREADS), 0, st, la, lb, slab, ep, M, Cout, K, kchunk, cnt);
    return true;
  }
  hipLaunchKernelGGL((gemm_kernel<T, BM, BN, true, true, LdKCConv<T, false, SC>, LdKC<T>, Epi<float>>), grid,
                     dim3(NTHREADS), 0, st, la, lb, slab, M, Cout, K, kchunk, xcd_group());
  int blocks = (int)std::min<int64_t>(cdiv(MN, 256), 2048);
  hipLaunchKernelGGL((splitk_reduce_kernel<Epi<TO>>), dim3(blocks), dim3(256), 0, st, ws, splits, M, Cout, ep);
  return true;
}

template <typename T, typename TO, bool SC>
bool conv_slabs(const void* x, int B, int H, int W, int Cin, const void* wpack, int Cout, int KH, int KW, int stride,
                int pad, const float* sc, void* y, int64_t ldy, const mg_epilogue* e, hipStream_t st) {
  if constexpr (sizeof(T) == 2) {
    if (Cout <= 32)
      return conv_slabs_t<T, TO, SC, 128, 32>(x, B, H, W, Cin, wpack, Cout, KH, KW, stride, pad, sc, y, ldy, e, st);
  }
  return conv_slabs_t<T, TO, SC, 64, 64>(x, B, H, W, Cin, wpack, Cout, KH, KW, stride, pad, sc, y, ldy, e, st);
}

template <typename T, typename TO>
void run_conv_tiles(const void* x, int B, int H, int W, int Cin, const void* wpack, int Cout, int KH, int KW,
                    int stride, int pad, const float* sc, void* y, int64_t ldy, const mg_epilogue* e,
                    hipStream_t st) {
  if constexpr (sizeof(T) == 2) {  // 32-channel 3x3 convs on small maps (offset heads): direct, halo tiles in LDS
    if (!sc && mg_conv3_direct_ok(H, W, Cin, Cout, KH, KW, stride, pad, false) &&
        mg_conv3_direct(x, B, H, Cin, wpack, Cout, e, y, ldy, std::is_same<TO, float>::value ? MG_F32 : MG_BF16, st))
      return;
  }
  const bool small_c = Cin < max_tile_bk<T>();  // a K step spans several taps: per-lane tap decode
  if (small_c ? conv_slabs<T, TO, true>(x, B, H, W, Cin, wpack, Cout, KH, KW, stride, pad, sc, y, ldy, e, st)
              : conv_slabs<T, TO, false>(x, B, H, W, Cin, wpack, Cout, KH, KW, stride, pad, sc, y, ldy, e, st))
    return;
  const int tile = g_mg_tune[MG_TUNE_CONV_TILE];
  if constexpr (sizeof(T) == 2) {
    // modulation-scaled loads on 128^2 tiles when the grid still covers the chip (measured at B=256: the
    // 16x16 modulated 3x3 conv, 128 -> 128 channels, 58 -> 47 us; the 8x8 one stays on 64^2)
    if (sc && !small_c && (tile == 128 || (tile == 0 && cdiv(B * ((H + 2 * pad - KH) / stride + 1) *
                                                                  ((W + 2 * pad - KW) / stride + 1), 128) *
                                                             (int64_t)cdiv(Cout, 128) >= 480))) {
      run_conv<T, TO, 128, 128, true, true>(x, B, H, W, Cin, wpack, Cout, KH, KW, stride, pad, sc, y, ldy, e, st);
      return;
    }
    if (sc && !small_c && tile == 257) {
      run_conv<T, TO, 128, 256, true, true>(x, B, H, W, Cin, wpack, Cout, KH, KW, stride, pad, sc, y, ldy, e, st);
      return;
    }
  }
  if (sc || small_c) {  // modulation scale on load / small Cin: generic 64x64 instantiations
    if (sc) run_conv<T, TO, 64, 64, true, true>(x, B, H, W, Cin, wpack, Cout, KH, KW, stride, pad, sc, y, ldy, e, st);
    else run_conv<T, TO, 64, 64, false, true>(x, B, H, W, Cin, wpack, Cout, KH, KW, stride, pad, sc, y, ldy, e, st);
    return;
  }
  int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  int64_t M = (int64_t)B * OH * OW;
  if constexpr (sizeof(T) == 2) {
    // 8-fragment wave tiles (128 x 64 / 64 x 128 per wave): 25 % fewer LDS bytes per MFMA.  128 x 256 by
    // default when Cout fills it and the grid still covers the chip (measured at B=256: the
    // discriminator's 4x4/s2 conv, N = 256, 100 -> 92 us; one column tile also reads the input once)
    // narrow outputs (the MTM offset heads, Cout = 32) over many pixels: 128 x 32 tiles, no MFMA columns wasted
    if (tile == 0 && Cout <= 32 && M >= 32768) {
      run_conv<T, TO, 128, 32>(x, B, H, W, Cin, wpack, Cout, KH, KW, stride, pad, sc, y, ldy, e, st);
      return;
    }
    if (tile == 257 || (tile == 0 && Cout % 256 == 0 && cdiv(M, 128) * (int64_t)(Cout / 256) >= 480 &&
                        !(KH * KW * Cin <= 256 && M >= 16384))) {
      run_conv<T, TO, 128, 256>(x, B, H, W, Cin, wpack, Cout, KH, KW, stride, pad, sc, y, ldy, e, st);
      return;
    }
    if (tile == 256) {
      run_conv<T, TO, 256, 128>(x, B, H, W, Cin, wpack, Cout, KH, KW, stride, pad, sc, y, ldy, e, st);
      return;
    }
  }
  // 1x1 convs over many pixels (K = Cin <= 256): latency-bound single-step tiles, as the short-K GEMMs above
  const bool short_k = KH * KW * Cin <= 256 && M >= 16384;
  if (tile == 128 || (tile == 0 && !short_k && cdiv(M, 128) * (int64_t)cdiv(Cout, 128) >= 480 && Cout > 64))
    run_conv<T, TO, 128, 128>(x, B, H, W, Cin, wpack, Cout, KH, KW, stride, pad, sc, y, ldy, e, st);
  else
    run_conv<T, TO, 64, 64>(x, B, H, W, Cin, wpack, Cout, KH, KW, stride, pad, sc, y, ldy, e, st);
}
}  // namespace

extern "C" int mg_conv2d_fwd(int dtype, const void* x, int B, int H, int W, int Cin, const void* wpack, int Cout,
                             int KH, int KW, int stride, int pad, const float* in_scale, void* y, int64_t ldy,
                             int y_dtype, const mg_epilogue* ep, void* stream) {
  MG_REQUIRE(dtype == MG_F32 || dtype == MG_BF16, "bad dtype");
  MG_REQUIRE(Cin >= 8 && pow2(Cin), "Cin must be a power of two >= 8");
  int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  MG_REQUIRE(pow2(H) && pow2(W) && pow2(OH) && pow2(OW), "spatial sizes must be powers of two");
  MG_REQUIRE(aligned16(x) && aligned16(wpack), "x/wpack must be 16-byte aligned");
  MG_REQUIRE(!(ep && ep->atomic) || y_dtype == MG_F32, "atomic epilogue requires fp32 output");
  MG_REQUIRE(under2g((int64_t)B * H * W * Cin, dtype) && under2g((int64_t)Cout * KH * KW * Cin, dtype) &&
                 under2g((int64_t)B * OH * OW * ldy, y_dtype),
             "an operand exceeds 2 GiB (32-bit buffer offsets)");
  if (B == 0) return MG_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == MG_F32) {
    if (y_dtype == MG_F32) run_conv_tiles<float, float>(x, B, H, W, Cin, wpack, Cout, KH, KW, stride, pad, in_scale, y, ldy, ep, st);
    else run_conv_tiles<float, bf16_t>(x, B, H, W, Cin, wpack, Cout, KH, KW, stride, pad, in_scale, y, ldy, ep, st);
  } else {
    if (y_dtype == MG_F32) run_conv_tiles<bf16_t, float>(x, B, H, W, Cin, wpack, Cout, KH, KW, stride, pad, in_scale, y, ldy, ep, st);
    else run_conv_tiles<bf16_t, bf16_t>(x, B, H, W, Cin, wpack, Cout, KH, KW, stride, pad, in_scale, y, ldy, ep, st);
  }
  return mg_check_launch("mg_conv2d_fwd");
}

namespace {
template <typename T, int BM, int BN, bool XF = false>
void run_wgrad(const void* gy, int64_t ldg, const void* x, int B, int H, int W, int Cin, const float* sc, int Cout,
               int KH, int KW, int stride, int pad, float* gw, int splits, hipStream_t st) {
  int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  int P = B * OH * OW, N = KH * KW * Cin;
  LdMC<T> la{reinterpret_cast<const T*>(gy), ldg, Cout, P, nullptr, 1, nullptr, 0};
  LdMCConv<T, XF> lb{reinterpret_cast<const T*>(x), H, W, Cin, ilog2(Cin), ilog2(OW), ilog2(OH * OW), P,
                     KW, stride, pad, N, sc};
  mg_epilogue e{};
  e.alpha = 1.f;
  e.atomic = 1;
  e.remap_lgcin = ilog2(Cin);
  e.remap_taps = KH * KW;
  auto ep = make_epi<float>(gw, N, &e);
  launch_gemm<T, BM, BN, false, false>(la, lb, ep, Cout, N, P, splits, kNoGroup, 0, st);
}

// Weight gradient with split-K into fp32 slabs written by the 8-column vector epilogue (coalesced, no atomics),
// then the slab fold into the reference layout (mg_fold.hip: immediate, or deferred to the backward's flush).  Returns false when the workspace cannot be had (caller falls back to atomics).
// stride-1 "same" convolution whose weight gradient can use the cheap-address column loader (LdMCConvS1)
inline bool wgrad_s1(int H, int W, int KH, int KW, int stride, int pad, int tbk) {
  return stride == 1 && KH == KW && 2 * pad == KH - 1 && W <= tbk && H <= 32 && pow2(H) && pow2(W);
}

template <typename T, int BM, int BN, bool XF = false>
bool run_wgrad_slabs(const void* gy, int64_t ldg, const void* x, int B, int H, int W, int Cin, const float* sc,
                     int Cout, int KH, int KW, int stride, int pad, float* gw, int splits, hipStream_t st) {
  constexpr int TBK = tile_bk<T, false, BM, BN>();
  int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  int P = B * OH * OW, N = KH * KW * Cin;
  int kchunk = ((P + splits - 1) / splits + TBK - 1) / TBK * TBK;
  splits = (P + kchunk - 1) / kchunk;
  const int64_t MN = (int64_t)Cout * N;
  bool deferred = false;
  float* ws = mg_fold_partials((size_t)splits * MN * sizeof(float), st, &deferred);
  if (!ws) return false;
  LdMC<T> la{reinterpret_cast<const T*>(gy), ldg, Cout, P, nullptr, 1, nullptr, 0};
  LdMCConv<T, XF> lb{reinterpret_cast<const T*>(x), H, W, Cin, ilog2(Cin), ilog2(OW), ilog2(OH * OW), P,
                     KW, stride, pad, N, sc};
  mg_epilogue raw{};
  raw.alpha = 1.f;
  Epi<float> slab = make_epi<float>(ws, N, &raw);
  slab.zstride = MN;
  slab.vec_ok = slab.host_vec_ok() ? 1 : 0;
  dim3 grid(cdiv(Cout, BM), cdiv(N, BN), splits);
  if (!XF && !g_mg_tune[MG_TUNE_S1_OFF] && wgrad_s1(H, W, KH, KW, stride, pad, TBK)) {
    LdMCConvS1<T> lb1{reinterpret_cast<const T*>(x), ilog2(Cin), ilog2(OW), OH, W, KW, pad, P, N};
    hipLaunchKernelGGL((gemm_kernel<T, BM, BN, false, false, LdMC<T>, LdMCConvS1<T>, Epi<float>>), grid,
                       dim3(NTHREADS), 0, st, la, lb1, slab, Cout, N, P, kchunk, xcd_group());
  } else {
    hipLaunchKernelGGL((gemm_kernel<T, BM, BN, false, false, LdMC<T>, LdMCConv<T, XF>, Epi<float>>), grid,
                       dim3(NTHREADS), 0, st, la, lb, slab, Cout, N, P, kchunk, xcd_group());
  }
  // (Cout x Cin / CC) blocks: enough to spread the slab reads over the chip, >= 8 channels per segment
  int lgCC = ilog2(Cin);
  while (lgCC > 3 && (int64_t)Cout * (Cin >> lgCC) < 1024) --lgCC;
  mg_fold_wgrad_submit(mg_fold_wgrad{ws, splits, Cout, ilog2(Cin), KH * KW, lgCC, gw}, deferred, st);
  return true;
}
}  // namespace

extern "C" int mg_conv2d_wgrad(int dtype, const void* gy, int64_t ldg, const void* x, int B, int H, int W, int Cin,
                               const float* in_scale, int Cout, int KH, int KW, int stride, int pad, float* gw,
                               int splits, void* stream) {
  MG_REQUIRE(dtype == MG_F32 || dtype == MG_BF16, "bad dtype");
  const int vec = dtype == MG_F32 ? 4 : 8;
  int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  MG_REQUIRE(pow2(Cin) && Cin >= vec, "Cin must be a power of two >= vector width");
  MG_REQUIRE(pow2(OH) && pow2(OW), "output spatial sizes must be powers of two");
  MG_REQUIRE(Cout % vec == 0 && ldg % vec == 0, "Cout / ldg must be multiples of the vector width");
  MG_REQUIRE(under2g((int64_t)B * H * W * Cin, dtype) && under2g((int64_t)B * OH * OW * ldg, dtype),
             "an operand exceeds 2 GiB (32-bit buffer offsets)");
  MG_REQUIRE(aligned16(gy) && aligned16(x), "gy/x must be 16-byte aligned");
  if (B == 0) return MG_OK;
  const int64_t P = (int64_t)B * OH * OW;
  const int N = KH * KW * Cin;
  // 128^2 tiles (half the operand traffic per flop) when both output dims fill them; split K so the grid
  // covers the chip about twice (occupancy-2 kernels) without cutting a split below 1024 pixels
  const int tile = g_mg_tune[MG_TUNE_WGRAD_TILE];
  // 128^2 tiles pay off on long per-split reductions (measured at B=256: the discriminator's 4x4/s2 conv
  // weight gradient, Cout 256 x 2048 over 65536 pixels, 137 -> 106 us; the generator's modulated convs
  // stay faster on 64^2 tiles)
  const bool big = dtype == MG_BF16 && Cout >= 128 && N >= 128 &&
                   (tile == 128 || (tile == 0 && Cout >= 256 && N >= 1024 && P >= 32768));
  const int64_t tiles = big ? (int64_t)cdiv(Cout, 128) * cdiv(N, 128) : (int64_t)cdiv(Cout, 64) * cdiv(N, 64);
  const bool slabs = g_mg_tune[MG_TUNE_WGRAD_MODE] == 0;
  if (splits < 1 && g_mg_tune[MG_TUNE_WGRAD_SPLITS] > 0) splits = g_mg_tune[MG_TUNE_WGRAD_SPLITS];
  if (splits < 1) {
    // atomics: measured sweet spot ~576 blocks, >= 2048 pixels per split (the remapped fp32 atomics are
    // scattered, so few splits); slabs: ~2048 blocks, >= 1024 pixels and <= 16 slabs (measured at B=256:
    // D conv1 / modconv 8x8 / modconv 16x16 weight gradients 1.36x / 1.2x / 1.6x over ~512 blocks)
    const int sb = g_mg_tune[MG_TUNE_WGRAD_SLAB_BLOCKS];
    // (slabs, 64^2 tiles: 1024 blocks since round 6 -- same step time as 2048, half the slab bytes the deferred fold
    // reads: same box 8.056 / 8.047 ms at 2048 / 1024, 8.161 at 512; tuning slot MG_TUNE_WGRAD_SLAB_BLOCKS)
    const int64_t want = slabs ? (sb > 0 ? sb : 1024) : (big ? 288 : 576);
    int64_t t = std::max<int64_t>(tiles, 1);
    // few 64^2 tiles: up to 32 slabs (modconv 16x16 wgrad 65 -> 58 us); a handful (to_rgb, Cout 3 -> 8 rows):
    // up to 128, so the reduction over B*H*W pixels still spreads over >= 128 blocks
    const int64_t cap = (!big && tiles < 8) ? 128 : (!big && tiles < 64) ? 32 : 16;
    splits = (int)std::max<int64_t>(1, std::min<int64_t>((want + t / 2) / t, slabs ? std::min<int64_t>(cap, P / 1024)
                                                                                      : P / 2048));
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // 1x1 / stride-1 convolutions: gw[Cout][Cin] += gy^T x over the B*H*W pixels, the long-reduction kernel of the
  // linear-layer weight gradients (mg_wgrad_wide.hip; it declines shapes it does not win on)
  if (dtype == MG_BF16 && !in_scale && KH == 1 && KW == 1 && stride == 1 && pad == 0 &&
      mg_wgrad_wide(Cout, Cin, (int)P, gy, ldg, x, Cin, gw, Cin, 1.f, st))
    return mg_check_launch("mg_conv2d_wgrad (1x1, long reduction)");
  if (dtype == MG_BF16 && !in_scale && Cout == 32 && Cin >= 32 && mg_conv3_direct_ok(H, W, Cin, Cout, KH, KW, stride, pad, true)) {
    float* ws = nullptr;
    int ng = 0;
    bool deferred = false;
    if (mg_wgrad3_direct(gy, ldg, x, B, H, Cin, &ws, &ng, &deferred, st)) {
      const int lgCC = 3;  // 32 x Cin / 8 fold blocks
      mg_fold_wgrad_submit(mg_fold_wgrad{ws, ng, Cout, ilog2(Cin), 9, lgCC, gw}, deferred, st);
      return mg_check_launch("mg_conv2d_wgrad (direct 3x3, 32 channels)");
    }
  }
  if (dtype == MG_BF16 && slabs && in_scale && tile == 128 && Cout >= 128 && N >= 128 &&
      run_wgrad_slabs<bf16_t, 128, 128, true>(gy, ldg, x, B, H, W, Cin, in_scale, Cout, KH, KW, stride, pad, gw,
                                               splits, st))
    return mg_check_launch("mg_conv2d_wgrad (scaled, 128)");
  if (dtype == MG_BF16 && slabs && !in_scale && (tile == 256 || tile == 257)) {
    bool ok = tile == 256 ? run_wgrad_slabs<bf16_t, 256, 128>(gy, ldg, x, B, H, W, Cin, in_scale, Cout, KH, KW, stride,
                                                              pad, gw, splits, st)
                          : run_wgrad_slabs<bf16_t, 128, 256>(gy, ldg, x, B, H, W, Cin, in_scale, Cout, KH, KW, stride,
                                                              pad, gw, splits, st);
    if (ok) return mg_check_launch("mg_conv2d_wgrad (slabs, wide)");
  }
  if (in_scale) {  // modulation scale on load: generic 64x64 instantiation (slabs, atomics if no workspace)
    bool ok = dtype == MG_BF16 ? run_wgrad_slabs<bf16_t, 64, 64, true>(gy, ldg, x, B, H, W, Cin, in_scale, Cout, KH, KW,
                                                                       stride, pad, gw, splits, st)
                               : run_wgrad_slabs<float, 64, 64, true>(gy, ldg, x, B, H, W, Cin, in_scale, Cout, KH, KW,
                                                                      stride, pad, gw, splits, st);
    if (!ok) {
      if (dtype == MG_BF16) run_wgrad<bf16_t, 64, 64, true>(gy, ldg, x, B, H, W, Cin, in_scale, Cout, KH, KW, stride, pad, gw, splits, st);
      else run_wgrad<float, 64, 64, true>(gy, ldg, x, B, H, W, Cin, in_scale, Cout, KH, KW, stride, pad, gw, splits, st);
    }
    return mg_check_launch("mg_conv2d_wgrad (scaled)");
  }
  if (slabs && dtype == MG_BF16) {
    bool ok = big ? run_wgrad_slabs<bf16_t, 128, 128>(gy, ldg, x, B, H, W, Cin, in_scale, Cout, KH, KW, stride, pad,
                                                       gw, splits, st)
                  : run_wgrad_slabs<bf16_t, 64, 64>(gy, ldg, x, B, H, W, Cin, in_scale, Cout, KH, KW, stride, pad, gw,
                                                     splits, st);
    if (ok) return mg_check_launch("mg_conv2d_wgrad (slabs)");
  } else if (slabs) {
    if (run_wgrad_slabs<float, 64, 64>(gy, ldg, x, B, H, W, Cin, in_scale, Cout, KH, KW, stride, pad, gw, splits, st))
      return mg_check_launch("mg_conv2d_wgrad (slabs)");
  }
  if (dtype == MG_F32) run_wgrad<float, 64, 64>(gy, ldg, x, B, H, W, Cin, in_scale, Cout, KH, KW, stride, pad, gw, splits, st);
  else if (big) run_wgrad<bf16_t, 128, 128>(gy, ldg, x, B, H, W, Cin, in_scale, Cout, KH, KW, stride, pad, gw, splits, st);
  else run_wgrad<bf16_t, 64, 64>(gy, ldg, x, B, H, W, Cin, in_scale, Cout, KH, KW, stride, pad, gw, splits, st);
  return mg_check_launch("mg_conv2d_wgrad");
}

// ---------------------------------------------------------------------------
// grouped (per-expert) GEMMs
// ---------------------------------------------------------------------------
namespace {
template <typename T, typename TO, bool BKc, bool XF>
void run_grouped(int total_rows, int N, int K, int ngroups, const int32_t* row_off, const int32_t* tile_off,
                 int max_tiles, const void* A, int64_t lda, const void* B, int64_t ldb, int64_t b_gstride, void* C,
                 int64_t ldc, const mg_epilogue* e, hipStream_t st) {
  auto ep = make_epi<TO>(C, ldc, e);
  ep.gstride_bias = N;
  const int32_t* aidx = e ? e->a_idx : nullptr;
  int adiv = (e && e->a_idx_div > 0) ? e->a_idx_div : 1;
  LdKC<T, XF> la{reinterpret_cast<const T*>(A), lda, total_rows, K, aidx, adiv, e ? e->a_rowscale : nullptr,
                 e ? e->a_gelu : 0};
  Grouping grp{1, ngroups, row_off, tile_off, 0};
  if constexpr (sizeof(T) == 2) {
    // 64 x 64 tiles over the 128-row tile table (two sub-tiles per table tile) for short-K expert GEMMs (layer 1,
    // K = C; the backward's gG x W2, K = C): load-latency-bound on 128^2 tiles like the dense short-K projections.
    // Measured at B = 256, E = 8 top-2 (tools/expert_probe.py, profiles/round5_expert_probe.txt): layer 1 with the
    // bias + GELU + saved pre-activation epilogue 72.8 -> 55.7 us (8x8 block, K = 256), 56.5 -> 46.6 us (4x4, K = 512),
    // 114 -> 93 us (16x16, K = 128); layer 2 (K = 4C) is no faster, so it keeps 128^2.  A/B: tuning slot
    // MG_TUNE_GROUPED_SHORTK (0 automatic: K <= 512, -1 never, > 0 that threshold), MG_TUNE_GEMM_TILE = 64 forces.
    const int tl0 = g_mg_tune[MG_TUNE_GEMM_TILE], sk = g_mg_tune[MG_TUNE_GROUPED_SHORTK];
    if (tl0 == 64 || (tl0 == 0 && sk >= 0 && K <= (sk > 0 ? sk : 512))) {
      grp.sub_shift = 1;
      if constexpr (BKc) {
        LdKCGroupW<T> lb{reinterpret_cast<const T*>(B), ldb, N, K, b_gstride, nullptr};
        launch_gemm<T, 64, 64, true, true, 1>(la, lb, ep, total_rows, N, K, 1, grp, max_tiles, st);
      } else {
        LdMCGroupW<T> lb{reinterpret_cast<const T*>(B), ldb, N, K, b_gstride, nullptr};
        launch_gemm<T, 64, 64, true, false, 1>(la, lb, ep, total_rows, N, K, 1, grp, max_tiles, st);
      }
      return;
    }
    // 128 x 256 tiles (same 128-row tile prefix, half the column tiles): by default for one 256-wide column tile
    // over a long K (the 8x8 block's expert layer 2, 32768 x 256 x 1024: 44 -> 39 us; wider N measured slower,
    // profiles/round4_grouped_probe.txt)
    const int tl = g_mg_tune[MG_TUNE_GEMM_TILE];
    if ((tl == 257 && N >= 256) || (tl == 0 && N == 256 && K >= 1024)) {
      if constexpr (BKc) {
        LdKCGroupW<T> lb{reinterpret_cast<const T*>(B), ldb, N, K, b_gstride, nullptr};
        launch_gemm<T, 128, 256, true, true, 1>(la, lb, ep, total_rows, N, K, 1, grp, max_tiles, st);
      } else {
        LdMCGroupW<T> lb{reinterpret_cast<const T*>(B), ldb, N, K, b_gstride, nullptr};
        launch_gemm<T, 128, 256, true, false, 1>(la, lb, ep, total_rows, N, K, 1, grp, max_tiles, st);
      }
      return;
    }
  }
  if constexpr (BKc) {
    LdKCGroupW<T> lb{reinterpret_cast<const T*>(B), ldb, N, K, b_gstride, nullptr};
    launch_gemm<T, 128, 128, true, true, 1>(la, lb, ep, total_rows, N, K, 1, grp, max_tiles, st);
  } else {
    LdMCGroupW<T> lb{reinterpret_cast<const T*>(B), ldb, N, K, b_gstride, nullptr};
    launch_gemm<T, 128, 128, true, false, 1>(la, lb, ep, total_rows, N, K, 1, grp, max_tiles, st);
  }
}

template <typename T, bool XF>
void run_grouped_wgrad(int M, int N, int ngroups, const int32_t* row_off, int total_rows, const void* A, int64_t lda,
                       const void* B, int64_t ldb, const int32_t* b_idx, int b_idx_div, int b_gelu, float* C,
                       int splits, const mg_epilogue* e, hipStream_t st) {
  LdMC<T, XF> la{reinterpret_cast<const T*>(A), lda, M, total_rows, e ? e->a_idx : nullptr,
             (e && e->a_idx_div > 0) ? e->a_idx_div : 1, e ? e->a_rowscale : nullptr, e ? e->a_gelu : 0};
  LdMC<T, XF> lb{reinterpret_cast<const T*>(B), ldb, N, total_rows, b_idx, b_idx_div > 0 ? b_idx_div : 1, nullptr,
             b_gelu};
  mg_epilogue ee{};
  ee.alpha = e ? e->alpha : 1.f;
  const int64_t MN = (int64_t)M * N, GMN = MN * ngroups;
  // where the K splits meet: fp32 atomics into C; or, when this stream defers its gradient folds (mg_fold.hip),
  // plain stores of per-split partial slabs [splits][ngroups][M][N] folded later in split order (no atomic traffic:
  // the ~8 M fp32 atomics per expert weight gradient were a quarter of its time at the C2 shapes, and the fold joins
  // the backward's one batched flush); one split: a single writer per element, read-modify-write
  bool deferred = false;
  float* slabs = nullptr;
  if (splits > 1 && ee.alpha == 1.f && GMN < (1ll << 31)) {
    slabs = reinterpret_cast<float*>(mg_fold_alloc((size_t)splits * GMN * sizeof(float), st));
    deferred = slabs != nullptr;
  }
  if (!slabs) {  // (slabs: plain stores of every element, the fold adds them into C)
    if (splits > 1) ee.atomic = 1;
    else ee.accumulate = 1;
  }
  auto ep = make_epi<float>(slabs ? slabs : C, N, &ee);
  ep.gstride_c = MN;
  if (slabs) ep.zstride = GMN;
  Grouping grp{2, ngroups, row_off, nullptr, 0};
  if (sizeof(T) == 2 && M >= 128 && N >= 128 && g_mg_tune[MG_TUNE_GWGRAD_TILE] != 64)
    launch_gemm<T, 128, 128, false, false, 1>(la, lb, ep, M, N, total_rows, splits, grp, 0, st);
  else
    launch_gemm<T, 64, 64, false, false, 1>(la, lb, ep, M, N, total_rows, splits, grp, 0, st);
  if (slabs)  // C[g][m][n] += alpha * sum_s slab[s][g][m][n]
    mg_fold_rows_submit(mg_fold_rows{slabs, GMN, splits, (int32_t)GMN, (int32_t)GMN, C, nullptr}, deferred, st);
}
}  // namespace

extern "C" int mg_gemm_grouped(int dtype, int total_rows, int N, int K, int ngroups, const int32_t* row_off,
                               const int32_t* tile_off, int max_tiles, const void* A, int64_t lda, const void* B,
                               int64_t ldb, int b_kc, int64_t b_gstride, void* C, int64_t ldc, int c_dtype,
                               const mg_epilogue* ep, void* stream) {
  MG_REQUIRE(dtype == MG_F32 || dtype == MG_BF16, "bad dtype");
  const int vec = dtype == MG_F32 ? 4 : 8;
  MG_REQUIRE(K % vec == 0 && lda % vec == 0 && ldb % vec == 0, "K/lda/ldb must be multiples of the vector width");
  MG_REQUIRE(b_kc || N % vec == 0, "N must be a multiple of the vector width for b_kc=0");
  MG_REQUIRE(under2g((int64_t)total_rows * lda, dtype) && under2g((int64_t)ngroups * b_gstride, dtype) &&
                 under2g((int64_t)total_rows * ldc, c_dtype),
             "an operand exceeds 2 GiB (32-bit buffer offsets)");
  MG_REQUIRE(aligned16(A) && aligned16(B), "A/B must be 16-byte aligned");
  if (max_tiles <= 0 || N == 0) return MG_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define MG_GRP4(T, TO, X)                                                                                       \
  (b_kc ? run_grouped<T, TO, true, X>(total_rows, N, K, ngroups, row_off, tile_off, max_tiles, A, lda, B, ldb,  \
                                      b_gstride, C, ldc, ep, st)                                                 \
        : run_grouped<T, TO, false, X>(total_rows, N, K, ngroups, row_off, tile_off, max_tiles, A, lda, B, ldb, \
                                       b_gstride, C, ldc, ep, st))
#define MG_GRP(T, TO) (a_xf(ep) ? MG_GRP4(T, TO, true) : MG_GRP4(T, TO, false))
  if (dtype == MG_F32) {
    if (c_dtype == MG_F32) MG_GRP(float, float); else MG_GRP(float, bf16_t);
  } else {
    if (c_dtype == MG_F32) MG_GRP(bf16_t, float); else MG_GRP(bf16_t, bf16_t);
  }
#undef MG_GRP
#undef MG_GRP4
  return mg_check_launch("mg_gemm_grouped");
}

extern "C" int mg_gemm_grouped_wgrad(int dtype, int M, int N, int ngroups, const int32_t* row_off, int total_rows,
                                     const void* A, int64_t lda, const void* B, int64_t ldb, const int32_t* b_idx,
                                     int b_idx_div, int b_gelu, float* C, int splits, const mg_epilogue* ep,
                                     void* stream) {
  MG_REQUIRE(dtype == MG_F32 || dtype == MG_BF16, "bad dtype");
  const int vec = dtype == MG_F32 ? 4 : 8;
  MG_REQUIRE(M % vec == 0 && N % vec == 0 && lda % vec == 0 && ldb % vec == 0, "M/N/lda/ldb must be vector multiples");
  MG_REQUIRE(under2g((int64_t)total_rows * lda, dtype) && under2g((int64_t)total_rows * ldb, dtype),
             "an operand exceeds 2 GiB (32-bit buffer offsets)");
  MG_REQUIRE(aligned16(A) && aligned16(B), "A/B must be 16-byte aligned");
  if (splits < 1) {
    const bool big = dtype == MG_BF16 && M >= 128 && N >= 128 && g_mg_tune[MG_TUNE_GWGRAD_TILE] != 64;
    int tiles = big ? cdiv(M, 128) * cdiv(N, 128) * ngroups : cdiv(M, 64) * cdiv(N, 64) * ngroups;
    int rows_per_group = std::max(1, total_rows / std::max(1, ngroups));
    // ~512 blocks of 128^2 tiles.  Isolated with uniform routing, ~256 (fewer splits, fewer fp32 atomic adds) ran the
    // C2 expert shapes 15-20 % faster (profiles/round4_gwgrad_probe.txt), but in the step -- skewed expert loads, the
    // largest expert's chunks set the tail -- it measured 8.86 -> 8.93 ms on one box (tools/gpu_gw_ab.sh), so the
    // target stays 512 (A/B: tuning slot MG_TUNE_GWGRAD_BLOCKS)
    const int tb = g_mg_tune[MG_TUNE_GWGRAD_BLOCKS], target = big ? (tb > 0 ? tb : 512) : 1024;
    splits = std::max(1, std::min({64, cdiv(target, std::max(1, tiles)), std::max(1, rows_per_group / 1024)}));
  }
  if (mg_det()) splits = 1;  // deterministic mode: one writer (one atomic add) per element and group
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bool xf = a_xf(ep) || b_idx || b_gelu;
#define MG_GW(T, X) run_grouped_wgrad<T, X>(M, N, ngroups, row_off, total_rows, A, lda, B, ldb, b_idx, b_idx_div, b_gelu, C, splits, ep, st)
  if (dtype == MG_F32) { if (xf) MG_GW(float, true); else MG_GW(float, false); }
  else { if (xf) MG_GW(bf16_t, true); else MG_GW(bf16_t, false); }
#undef MG_GW
  return mg_check_launch("mg_gemm_grouped_wgrad");
}

// ---------------------------------------------------------------------------
// data gradient of a 4x4 / stride-2 / pad-1 conv (discriminator convs, R1 path)
// ---------------------------------------------------------------------------
namespace {
template <typename T, typename TO, bool SC>
void run_dgrad_s2(const void* g, int B, int OH, int OW, int Cg, const void* wcls, int Cin, void* out, int64_t ldo,
                  const mg_epilogue* e, hipStream_t st) {
  int Mc = B * OH * OW;
  LdKCConvT<T, false, SC> la{reinterpret_cast<const T*>(g), OH, OW, Cg, ilog2(Cg), ilog2(OW), ilog2(OH * OW), Mc, 4 * Cg, 0};
  LdKCGroupW<T> lb{reinterpret_cast<const T*>(wcls), 4 * Cg, Cin, 4 * Cg, (int64_t)Cin * 4 * Cg, nullptr};
  auto ep = make_epi<TO>(out, ldo, e);
  ep.rm_mode = 1;
  ep.rm_Mc = Mc;
  ep.rm_lgOW = ilog2(OW);
  ep.rm_lgOHW = ilog2(OH * OW);
  Grouping grp{3, 4, nullptr, nullptr, Mc};
  // 128^2 tiles when they fill the chip; the 8x8 -> 4x4 discriminator conv (4 x 4096 rows x 128) had 128 of them,
  // 16 serial K steps each on half the CUs: 64^2 tiles (512, LDS-DMA staged: LdKCConvT::kConv)
  if (Cin >= 128 && !SC && (int64_t)cdiv(4 * Mc, 128) * cdiv(Cin, 128) >= 256)
    launch_gemm<T, 128, 128, true, true>(la, lb, ep, 4 * Mc, Cin, 4 * Cg, 1, grp, 0, st);
  else if (sizeof(T) == 2 && Cin <= 32 && !SC)  // image gradient (Cin = 3): 128 x 32 tiles waste 8x, not 16x, MFMA work
    launch_gemm<T, 128, 32, true, true>(la, lb, ep, 4 * Mc, Cin, 4 * Cg, 1, grp, 0, st);
  else
    launch_gemm<T, 64, 64, true, true>(la, lb, ep, 4 * Mc, Cin, 4 * Cg, 1, grp, 0, st);
}
}  // namespace

extern "C" int mg_conv2d_dgrad_s2(int dtype, const void* g, int B, int OH, int OW, int Cg, const void* wcls, int Cin,
                                  void* out, int64_t ldo, int out_dtype, const mg_epilogue* ep, void* stream) {
  MG_REQUIRE(dtype == MG_F32 || dtype == MG_BF16, "bad dtype");
  MG_REQUIRE(pow2(Cg) && Cg >= 8, "Cg must be a power of two >= 8");
  MG_REQUIRE(pow2(OH) && pow2(OW), "OH, OW must be powers of two");
  MG_REQUIRE(aligned16(g) && aligned16(wcls), "g/wcls must be 16-byte aligned");
  MG_REQUIRE(under2g((int64_t)B * OH * OW * Cg, dtype) && under2g((int64_t)B * 4 * OH * OW * ldo, out_dtype),
             "an operand exceeds 2 GiB (32-bit buffer offsets)");
  MG_REQUIRE(!(ep && ep->atomic) || out_dtype == MG_F32, "atomic epilogue requires fp32 output");
  if (B == 0) return MG_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == MG_F32) {
    if (out_dtype == MG_F32) (Cg < max_tile_bk<float>() ? run_dgrad_s2<float, float, true>(g, B, OH, OW, Cg, wcls, Cin, out, ldo, ep, st) : run_dgrad_s2<float, float, false>(g, B, OH, OW, Cg, wcls, Cin, out, ldo, ep, st));
    else (Cg < max_tile_bk<float>() ? run_dgrad_s2<float, bf16_t, true>(g, B, OH, OW, Cg, wcls, Cin, out, ldo, ep, st) : run_dgrad_s2<float, bf16_t, false>(g, B, OH, OW, Cg, wcls, Cin, out, ldo, ep, st));
  } else {
    if (out_dtype == MG_F32) (Cg < max_tile_bk<bf16_t>() ? run_dgrad_s2<bf16_t, float, true>(g, B, OH, OW, Cg, wcls, Cin, out, ldo, ep, st) : run_dgrad_s2<bf16_t, float, false>(g, B, OH, OW, Cg, wcls, Cin, out, ldo, ep, st));
    else (Cg < max_tile_bk<bf16_t>() ? run_dgrad_s2<bf16_t, bf16_t, true>(g, B, OH, OW, Cg, wcls, Cin, out, ldo, ep, st) : run_dgrad_s2<bf16_t, bf16_t, false>(g, B, OH, OW, Cg, wcls, Cin, out, ldo, ep, st));
  }
  return mg_check_launch("mg_conv2d_dgrad_s2");
}
