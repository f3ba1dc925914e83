/* libmoegan_hip -- C ABI of the MI355X-native MoE-GAN training-step kernels.
 *
 * The reference (moegan/t2i_moe_gan.py) has no FFI: its hot path is a stack of
 * PyTorch modules.  This header is the boundary those modules' math is moved
 * behind; the drop-in Python modules (moe-gan_cpsc541_amd/t2i_moe_gan.py) bind
 * it with ctypes.  Each entry cites the reference code it replaces.
 *
 * Conventions
 *  - Plain pointers + sizes, no framework types.  The caller owns every input
 *    and output buffer (device memory).
 *  - Scratch: split-K slabs and reduction partials live in one workspace block
 *    per (device, stream).  By default the library owns it and grows it on
 *    demand (hipStreamSynchronize on that stream, hipFree, hipMalloc), so size
 *    it with mg_workspace_reserve() before capturing a hipGraph.  A caller that
 *    wants the library never to allocate registers its own block with
 *    mg_set_workspace(); a call needing more than that block then fails with
 *    MG_ERR_ARG instead of allocating.  No entry point synchronises otherwise.
 *  - Activations are NHWC ("token") layout: [B, H, W, C] == [B*H*W, C] rows.
 *  - dtype: MG_F32 (exact fp32 parity mode) or MG_BF16 (bf16 storage, fp32
 *    accumulate).  Weight gradients and all reductions are fp32.
 *  - Operands of the GEMM/convolution entry points are read through 32-bit
 *    buffer offsets: each must be smaller than 2 GiB (checked, MG_ERR_ARG).
 *  - Every call is enqueued on `stream` (a hipStream_t; NULL = default).
 *  - Return 0 on success or a negative MG_ERR_*; mg_last_error() gives the
 *    thread-local message.
 *  - Thread safety: entry points may be called concurrently from several
 *    threads.  Process-wide state is limited to the workspace table (mutex
 *    guarded) and the mg_set_tuning switches (atomic; meant for A/B runs).
 */
#ifndef MOEGAN_HIP_H
#define MOEGAN_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MG_OK 0
#define MG_ERR_ARG (-1)
#define MG_ERR_LAUNCH (-2)

#define MG_F32 0
#define MG_BF16 1
/* mg_gemm / mg_gemm_batch only: fp32 operands and accumulation, the MFMA products taken as split bf16
   (hi * hi + hi * lo + lo * hi with hi = bf16(x), lo = bf16(x - hi)): ~2^-16 relative per product instead of the
   exact-fp32 MFMA's 2^-24, at the bf16 MFMA rate.  The bf16 mode's fp32 GEMMs (mapping, text projection, styles,
   demodulation, router / cross-attention vectors) use it; the fp32 parity mode keeps MG_F32. */
#define MG_F32X3 2

/* epilogue activation codes */
#define MG_ACT_NONE 0
#define MG_ACT_LRELU 1          /* LeakyReLU(0.2)  (t2i_moe_gan.py:216, :685) */
#define MG_ACT_GELU 2           /* exact-erf GELU  (t2i_moe_gan.py:258) */
#define MG_ACT_MUL_GELU_GRAD 3  /* v *= GELU'(aux[m,n]) */
#define MG_ACT_MUL_LRELU_GRAD 4 /* v *= LReLU'(aux[m,n]) */
#define MG_ACT_RSQRT_EPS 5      /* v = rsqrt(v + 1e-8)  (demodulation, t2i_moe_gan.py:165) */
#define MG_ACT_QUICK_GELU 6     /* v * sigmoid(1.702 v)  (CLIP ViT MLP, forward-only CLIP loss :66-119) */

/* Fused GEMM epilogue / prologue options (all pointers optional = NULL).
 *   v = alpha * acc
 *   v *= scale[(m >> scale_shift) * scale_ld + n]       (demodulation d[b, o])
 *   v += bias[n];  v = act(v);  v *= rowscale[m];  v += resid[m * ld_res + n]
 *   C[m, n] (+)= v   (accumulate: read-modify-write; atomic: fp32 atomic add)
 *   remap_taps > 0 : column n = tap*Cin + ci is stored at ci*taps + tap
 *                    (conv weight-gradient in the reference [Cout][Cin][kh][kw] layout)
 *   a_idx: A row gather (row r reads source row a_idx[r] / a_idx_div),
 *   a_rowscale: A row scale, a_gelu: GELU applied to A as it is loaded. */
typedef struct mg_epilogue {
  float alpha;
  const float* bias;
  const float* scale;
  int32_t scale_shift;
  int64_t scale_ld;
  const float* rowscale;
  int32_t act;
  const void* aux;
  int64_t ld_aux;
  const void* resid;
  int64_t ld_res;
  int32_t accumulate;
  int32_t atomic;
  int32_t remap_lgcin;
  int32_t remap_taps;
  const int32_t* a_idx;
  int32_t a_idx_div;
  const float* a_rowscale;
  int32_t a_gelu;
  const float* addvec; /* v += addvec[(m >> add_shift) * add_ld + n] (per-image broadcast add) */
  int32_t add_shift;
  int64_t add_ld;
  void* out_pre;       /* optional second output: the value before the activation (same dtype as C) */
  int64_t ld_pre;
} mg_epilogue;

const char* mg_last_error(void);
int mg_version(void);
/* sha256 prefix of the sources this library was built from (csrc/srchash.py): lets a caller prove the
   binary it loaded matches the sources it ships with. */
const char* mg_source_hash(void);

/* Workspace control (see Conventions).  mg_set_workspace: use the caller-owned block [ptr, ptr+bytes) for
   `stream` on the current device (ptr = NULL returns the stream to a library-owned block).
   mg_workspace_reserve: grow this stream's library-owned block to at least `bytes` now.
   mg_workspace_bytes: current size of this stream's block (0 = none yet). */
int mg_set_workspace(void* ptr, size_t bytes, void* stream);
int mg_workspace_reserve(size_t bytes, void* stream);
int64_t mg_workspace_bytes(void* stream);
/* Tuning override for measurements (key: 0 conv-wgrad tile, 1 grouped-wgrad tile, 2 conv tile,
   3 gemm tile [64 | 128], 4 conv-wgrad splits, 5 disable split-K slabs, 6 enable the XCD-aware tile
   order; value 0 = automatic). */
int mg_set_tuning(int key, int value);

/* Measurement of one call inside a training step (bench.py's roofline kernel; no reference
   counterpart: the reference times nothing below the Python loop, t2i_moe_gan.py:1262-1421).
   mg_timer_event_create: a timing event WITHOUT the system-scope release / acquire fence of a default HIP event
   (hipEventDisableSystemFence): a default event's L2 writeback + invalidate was measured to add ~18 % to the
   bracketed kernel's time; *event receives the handle.  mg_timer_event_record: record on `stream`.
   mg_timer_event_elapsed: waits for `stop`, *ms = stop - start.  mg_mark: one empty single-wave kernel,
   k_roofline_mark_begin (tag 0) or k_roofline_mark_end (tag 1), so a rocprofv3 kernel trace / PMC pass of the same
   run can find the dispatches the bracketed call made (tools/roofline_kernel.py). */
int mg_timer_event_create(void** event);
int mg_timer_event_record(void* event, void* stream);
int mg_timer_event_elapsed(void* start, void* stop, float* ms);
int mg_timer_event_destroy(void* event);
int mg_mark(int tag, void* stream);

/* One problem of a batched GEMM launch (mg_gemm_batch): C[M,N] = epilogue(op(A) @ op(B)). */
typedef struct mg_gemm_desc {
  int32_t M, N, K;
  const void* A;
  int64_t lda;
  const void* B;
  int64_t ldb;
  void* C;
  int64_t ldc;
  const mg_epilogue* ep; /* may be NULL */
} mg_gemm_desc;

/* Generic MFMA GEMM: C[M,N] = epilogue(op(A)[M,K] @ op(B)[K,N]).
 *   a_kc = 1 : A[m*lda + k]     a_kc = 0 : A[k*lda + m]
 *   b_kc = 1 : B[n*ldb + k]     b_kc = 0 : B[k*ldb + n]
 *   (nn.Linear forward is a_kc=1, b_kc=1 with B = weight [out, in].)
 * Replaces the torch.matmul / F.linear calls of the hot path
 * (t2i_moe_gan.py:158, :257-260, :364-371, :682-698, :510).
 * c_dtype selects the output storage (MG_F32 / MG_BF16); splits > 1 splits K
 * (requires ep->atomic and an fp32 C). */
int mg_gemm(int dtype, int M, int N, int K, const void* A, int64_t lda, int a_kc, const void* B, int64_t ldb,
            int b_kc, void* C, int64_t ldc, int c_dtype, const mg_epilogue* ep, int splits, void* stream);

/* n independent GEMMs of one dtype / orientation / output dtype in as few launches as possible
   (8 problems per launch, 64x64 tiles, no split-K): the per-layer small GEMMs of the generator (the
   demodulation coefficients of every modulated conv, router / cross-attention projections). */
int mg_gemm_batch(int dtype, int a_kc, int b_kc, int c_dtype, int n, const mg_gemm_desc* descs, void* stream);

/* Implicit-GEMM NHWC convolution (square kernel KHxKW, stride, pad):
 *   y[b,oh,ow,o] = epilogue( sum_{kh,kw,ci} x[b,ih,iw,ci] * in_scale[b,ci] * wpack[o][(kh*KW+kw)*Cin+ci] )
 * in_scale (optional, fp32 [B,Cin]) fuses the modulated-conv style (t2i_moe_gan.py:158-161).
 * Cin must be a multiple of 32; H, W, OH, OW, Cin powers of two.
 * Used for ModulatedConv forward (:169-180), its data gradient (flipped wpack),
 * offset_net (:209-213) and the discriminator convs (:874-887). */
int mg_conv2d_fwd(int dtype, const void* x, int B, int H, int W, int Cin, const void* wpack, int Cout, int KH,
                  int KW, int stride, int pad, const float* in_scale, void* y, int64_t ldy, int y_dtype,
                  const mg_epilogue* ep, void* stream);

/* MX-fp8 form of mg_conv2d_fwd (BASELINE config C5, "fp8 MFMA conv path"; same math as :169-180):
 *   y[b,oh,ow,o] = epilogue( sum_{kh,kw,ci} Q(x)[b,ih,iw,ci] * Q(W)[o][(kh*KW+kw)*Cin+ci] )
 * Q = OCP MX quantization: e4m3 elements with one E8M0 scale per 32 consecutive channels, multiplied by
 * v_mfma_scale_f32_16x16x128_f8f6f4 (fp32 accumulation).  x / xscale = mg_quant_mx8 of the NHWC
 * activation rows ([B*H*W][Cin] e4m3, [B*H*W][Cin/32] E8M0); wq / wscale = mg_quant_mx8 of the packed
 * [Cout][KH*KW*Cin] bf16 weights.  Cin a power of two >= 128; in_scale is not supported (quantize x * s).
 * Replaces the 3x3 modulated-conv forward and data-gradient GEMMs under fp8 (engine_g.mc_fwd / mc_bwd). */
int mg_conv2d_fwd_mx8(const void* x, const void* xscale, int B, int H, int W, int Cin, const void* wq,
                      const void* wscale, int Cout, int KH, int KW, int stride, int pad, void* y, int64_t ldy, int y_dtype, const mg_epilogue* ep,
                      void* stream);

/* MX-fp8 quantization of bf16 rows: x [rows][K] (pitch ldx) -> q [rows][K] e4m3 bytes and
 * scale [rows][K/32] E8M0 bytes; per 32-element block e = ceil(log2(amax / 448)) + 127 (nothing saturates),
 * round-to-nearest-even.  K % 32 == 0.  Used per optimizer step for the fp8 conv weights. */
int mg_quant_mx8(const void* x, int64_t ldx, int64_t rows, int K, void* q, void* scale, void* stream);
/* Several mg_quant_mx8 quantizations in one launch (the per-step MX-fp8 copies of the packed 3x3 weights and their
   flipped data-gradient forms); each descriptor as mg_quant_mx8's arguments, at most MG_QUANT_BATCH_MAX per launch
   (more are split into launches). */
#define MG_QUANT_BATCH_MAX 32
typedef struct mg_quant_desc {
  const void* x;
  int64_t ldx;
  int64_t rows;
  int32_t K;
  void* q;
  void* scale;
} mg_quant_desc;
int mg_quant_mx8_batch(int n, const mg_quant_desc* d, void* stream);

/* Weight gradient of the convolution above, accumulated (fp32 atomics) into
 * gw in the reference layout [Cout][Cin][KH][KW]:
 *   gw[o,ci,kh,kw] += sum_{b,oh,ow} gy[b,oh,ow,o] * x[b,ih,iw,ci] * in_scale[b,ci] */
int mg_conv2d_wgrad(int dtype, const void* gy, int64_t ldg, const void* x, int B, int H, int W, int Cin,
                    const float* in_scale, int Cout, int KH, int KW, int stride, int pad, float* gw, int splits,
                    void* stream);

/* Data gradient of a 4x4 / stride-2 / pad-1 convolution (the discriminator's
 * conv_layers, t2i_moe_gan.py:876,880), as four output-parity implicit GEMMs:
 *   out[b, ih, iw, ci] = epilogue( sum_{co,kh,kw} g[b, oh, ow, co] * W[co, ci, kh, kw] ),  ih = 2*oh - 1 + kh
 * g: [B, OH, OW, Cg] NHWC; out: [B, 2*OH, 2*OW, ldo]; wcls = mg_pack_dgrad_s2() of W.
 * Used for the ordinary D backward and for the R1 gradient / double-backward (:1282). */
int mg_conv2d_dgrad_s2(int dtype, const void* g, int B, int OH, int OW, int Cg, const void* wcls, int Cin,
                       void* out, int64_t ldo, int out_dtype, const mg_epilogue* ep, void* stream);

/* Grouped (per-expert) GEMM, grouped over output rows:
 *   for each group g: rows [row_off[g], row_off[g+1]) of C =
 *       epilogue(A_rows @ B_g^T-or-B_g)  with B_g = B + g * b_gstride
 * tile_off[g] = sum_{g'<g} ceil(rows_g' / 128)  (device tables: no host sync).
 * max_tiles = an upper bound of tile_off[ngroups].  bias stride per group = N. */
int mg_gemm_grouped(int dtype, int total_rows, int N, int K, int ngroups, const int32_t* row_off,
                    const int32_t* tile_off, int max_tiles, const void* A, int64_t lda, const void* B,
                    int64_t ldb, int b_kc, int64_t b_gstride, void* C, int64_t ldc, int c_dtype,
                    const mg_epilogue* ep, void* stream);

/* Grouped weight gradient (grouped over the reduction rows):
 *   for each g: C_g[M,N] += sum_{r in [row_off[g], row_off[g+1])} A[r, m] * B[r, n]
 * A and B are row-major [rows, M] / [rows, N] (with optional gathers/scales of
 * the epilogue struct applied to A: a_idx, a_rowscale, a_gelu; b_idx/b_gelu
 * below for B).  C fp32, accumulated atomically; C_g = C + g * M * N. */
int mg_gemm_grouped_wgrad(int dtype, int M, int N, int ngroups, const int32_t* row_off, int total_rows,
                          const void* A, int64_t lda, const void* B, int64_t ldb, const int32_t* b_idx,
                          int b_idx_div, int b_gelu, float* C, int splits, const mg_epilogue* ep, void* stream);

/* Fused expert FFN forward (t2i_moe_gan.py:257-263 for every expert of a SparseMoE at once): for the rows of
   group g (row_off / tile_off as mg_moe_dispatch builds them with bm = 128),
     Y[r] = GELU(X[r] W1[g]^T + b1[g]) W2[g]^T + b2[g]
   with W1 [G][Hd][C], W2 [G][C][Hd] (bf16), b1 [G][Hd], b2 [G][C] (fp32), Y [rows][C].  The hidden activation
   stays on chip; pre (the pre-activation) and hid (the GELU output) [rows][Hd] are written only when non-NULL
   (the backward's saved tensors); total_rows = row_off[G].  X row r is X[x_idx[r] / x_idx_div] when x_idx is given (the dispatch gather),
   else X[r].  Same arithmetic as mg_gemm_grouped with the GELU / bias epilogues.  bf16, C in {128, 256},
   Hd % 64 == 0; grid = max_tiles blocks. */
int mg_moe_ffn_fwd(int dtype, int total_rows, int C, int Hd, int ngroups, const int32_t* row_off, const int32_t* tile_off, int max_tiles, const void* X, int64_t ldx, const int32_t* x_idx, int x_idx_div, const void* W1, const float* b1, const void* W2, const float* b2, void* pre, void* hid, void* Y, void* stream);

/* Fused expert FFN backward, first half (t2i_moe_gan.py:257-263 backward, per dispatch group g): for the rows r of
   each group, gP[r] = (gG[r] W2_g) * GELU'(pre[r]) ([total_rows, Hd] bf16, written for the weight gradient of W1),
   gX[r] = gP[r] W1_g ([total_rows, C] bf16), and gb1[g] (fp32 [ngroups, Hd], accumulated; NULL skips it) +=
   sum over the group's rows of gP (the bf16 values), folded in a fixed order.  gP and gX are bit-identical to
   mg_gemm_grouped (gG x W2 with the GELU' epilogue, then gP x W1).  bf16, C = 128 or 256 (256: 144 KiB of LDS,
   one block per CU, gfx950), Hd % 128 == 0; gb2 (fp32 [ngroups, C], accumulated; NULL skips it) += the column
   sums of gG over the group's rows (the layer-2 bias gradient, from the gG tile the pass holds in LDS, per-tile
   partial rows folded in tile order); W1 [G, Hd, C],
   W2 [G, C, Hd]; grid = max_tiles blocks of 128 rows.  hid (optional, bf16 [total_rows, Hd]): GELU(pre) as the
   weight gradient of W2 reads it, from the same erf evaluation as GELU'(pre). */
int mg_moe_ffn_bwd(int dtype, int total_rows, int C, int Hd, int ngroups, const int32_t* row_off, const int32_t* tile_off, int max_tiles, const void* gG, const void* pre, const void* W1, const void* W2, void* gP, void* gX, void* hid, float* gb1, float* gb2, void* stream);

/* ---- op-level entry points ---- */

/* CLIP image-tower input (CLIPLoss.forward t2i_moe_gan.py:90-94 + the ViT conv1 patchify): clamp [-1,1], bilinear
   R->res (align_corners=False) from NHWC [B,R,R,ld] (channels 0..2), unfolded patch rows [B*(res/patch)^2, 3*patch*patch] bf16. */
int mg_clip_patches(int dtype, const void* img, int B, int R, int ld, int res, int patch, void* out, void* stream);

/* LayerNorm over C (128/256/512) per row (+ optional LeakyReLU), saving mean/rstd. t2i_moe_gan.py:505-507, :684. */
int mg_layernorm_fwd(int dtype, const void* x, int64_t ldx, int R, int C, const float* gamma, const float* beta, float eps, void* y, int64_t ldy, float* mean, float* rstd, int act, void* stream);

/* LayerNorm backward (gx (+)=, ggamma/gbeta += via atomics). */
int mg_layernorm_bwd(int dtype, int gy_dtype, const void* gy, int64_t ldg, const void* x, int64_t ldx, int R, int C, const float* mean, const float* rstd, const float* gamma, void* gx, int64_t ldgx, int accumulate, float* ggamma, float* gbeta, void* stream);

/* Self-attention core for nn.MultiheadAttention (8 heads) on packed qkv [B*L, 3C]; saves logsumexp. t2i_moe_gan.py:513, :546. */
int mg_attn_fwd(int dtype, const void* qkv, int B, int L, int C, int heads, void* out, float* lse, void* stream);

/* Self-attention backward -> gqkv [B*L, 3C]. */
int mg_attn_bwd(int dtype, int gout_dtype, const void* qkv, const void* out, const void* gout, const float* lse, int B, int L, int C, int heads, void* gqkv, void* stream);

/* Head text-branch backward: g_tpre, dW2 text rows (all taps). */
int mg_d_text_bwd(const float* g_tb, const float* t, const float* w2sum, int B, int Ct, int cofs, float* g_tpre, float* dW2, void* stream);

/* im2col for the discriminator's first conv (3->128, 4x4/s2/p1), any input strides, K padded to Kp. */
int mg_im2col_4x4s2(int in_dtype, const void* x, int64_t sb, int64_t sh, int64_t sw, int64_t sc, int B, int H, int W, int C, int Kp, int out_dtype, void* out, void* stream);

/* Data gradient of a 4x4 / stride-2 / pad-1 conv with few (C <= 4) input channels, second half: Y [B*OH*OW, ldy]
   = g @ wpack (wpack as mg_pack_conv, [Cg][16*C]) holds every (tap, channel) contribution of an output pixel;
   out[b, y, x, c] (pitch ldo, written for c < C) = sum over the <= 4 (oy, ox, kh, kw) with y = 2oy-1+kh,
   x = 2ox-1+kw of Y[b, oy, ox, (kh*4+kw)*C + c].  Replaces the padded-channel mg_conv2d_dgrad_s2 for the
   discriminator's first conv (image gradient of R1, t2i_moe_gan.py:1281-1286, and the G phase). */
int mg_col2im_4x4s2(int in_dtype, const void* Y, int64_t ldy, int B, int OH, int OW, int C, int out_dtype, void* out, int64_t ldo, void* stream);

/* The discriminator's first conv (conv_layers.0: 3 -> 128, 4x4 / s2 / p1, t2i_moe_gan.py:874-880) as direct MFMA
   kernels for the bf16 step (replace mg_im2col_4x4s2 + mg_gemm and the dgrad GEMM + mg_col2im_4x4s2 there).
   w0p: the packed bf16 weight [128][48] (k = tap*3 + c); x: image (MG_F32 or MG_BF16) with element strides
   sb / sh / sw / sc, B x H x W, 3 channels read; out / aux / g: NHWC bf16 [B, H/2, W/2, 128].
   mg_d0_fwd: aux == NULL -> out = LeakyReLU(conv(x) + bias) (h0, :880); aux != NULL -> out = conv(x) *
   LeakyReLU'(aux) (the R1 double backward's forward-mode pass through the layer, :1282-1286).
   mg_d0_wgrad: dw [128][48] fp32 (GEMM layout) += sum over output pixels of g[p][o] * patch[p][tap*3+c]; fixed
   order (per-block partials in the stream's workspace, folded in block order).
   mg_d0_dgrad: out[b, y, x, c] (pitch ldo, c < 3; MG_F32 or MG_BF16) = d/d x of sum g * conv(x): the image
   gradient (R1 :1282, the G phase :1379-1382); OW <= 64, H a multiple of 4.  When ldo is one 16-B vector
   (4 fp32 / 8 bf16) the padding channels 3 .. ldo-1 are written as 0, otherwise they are left untouched.
   The forward and the weight gradient take fp32 planar images (NCHW, sw = 1) or bf16 interleaved ones (NHWC,
   sc = 1, pixel pitch sw a multiple of 4); W / 2 a power of two in [4, 64]. */
int mg_d0_fwd(int in_dtype, const void* x, int64_t sb, int64_t sh, int64_t sw, int64_t sc, int B, int H, int W, const void* w0p, const float* bias, const void* aux, void* out, void* stream);
int mg_d0_wgrad(int in_dtype, const void* x, int64_t sb, int64_t sh, int64_t sw, int64_t sc, int B, int H, int W, const void* g, float* dw, void* stream);
int mg_d0_dgrad(const void* g, int B, int OH, int OW, const void* w0p, int out_dtype, void* out, int64_t ldo, void* stream);

/* Discriminator head, image channels, bf16 step (output_layer.0, t2i_moe_gan.py:901-907): mg_d_head_fwd: out[b, oy*Ho
   + ox] (fp32, Ho = Hf - 3) = sum_{c, kh, kw} h1[b, oy+kh, ox+kw, c] W2[c, kh*4+kw] with w2t the bf16 [16 taps][256]
   weight (mg_gemm + mg_disc_head_sum up to fp32 summation order).  mg_d_head_bwd: g_a1[b, y, x, c] (bf16) = LeakyReLU'(h1[b,
   y, x, c]) * sum_tap g[b, y-kh, x-kw] W2[c, tap] with w2c the bf16 [256][16 taps] weight and g [B, Ho*Ho] fp32
   (image stride g_bstride; 0 broadcasts one map, the R1 pass) -- bit-identical to mg_disc_head_gmat + mg_gemm with
   the LeakyReLU' epilogue.  h1 / g_a1: NHWC [B, Hf, Hf, 256]; 4 <= Hf <= 32. */
int mg_d_head_fwd(const void* h1, const void* w2t, int B, int Hf, float* out, void* stream);
int mg_d_head_bwd(const float* g, int64_t g_bstride, const void* h1, const void* w2c, int B, int Hf, void* ga1, void* stream);

/* Discriminator output_layer, image channels: out[b,o] = sum h1[b,o+tap,c] W2[c,tap] (t2i_moe_gan.py:885-907). */
int mg_disc_head_fwd(int dtype, const void* h1, const float* W2, int B, int Hf, int Cf, float* out, void* stream);

/* Discriminator head as GEMMs (t2i_moe_gan.py:901-907, output_layer: 4x4 valid conv to 1 channel):
   mg_disc_head_gmat: tap-expanded gradient G[b,y,x,tap] = g[b, y-kh, x-kw] ([B*Hf*Hf, 16]; g_bstride 0
   broadcasts one map, the R1 path); mg_disc_head_sum: out[b,oy,ox] = sum_tap P[b, oy+kh, ox+kw, tap]
   for P = h1 @ W2 ([B*Hf*Hf, 16] fp32). */
int mg_disc_head_gmat(int out_dtype, const float* g, int64_t g_bstride, int B, int Hf, void* G, void* stream);
int mg_disc_head_sum(const float* P, int B, int Hf, float* out, void* stream);

/* Head backward into features, fused with LeakyReLU' of a1 (g_bstride = 0 broadcasts: R1). */
int mg_disc_head_bwd_data(int dtype, const float* g, int64_t g_bstride, const float* W2, const void* a1, int B, int Hf, int Cf, int out_dtype, void* ga1, void* stream);

/* Head weight gradient (image channels) dW2[c,tap] += sum_b,o g h1. */
int mg_disc_head_bwd_w(int dtype, const float* g, int64_t g_bstride, const void* h1, int B, int Hf, int Cf, float* dW2, void* stream);

/* Discriminator loss (t2i_moe_gan.py:940-949) for real (No patch logits per image), fake (Nf per image: 1 for the
   reference's 16x16 fakes, (R/4-3)^2 for the progressive extension's RxR fakes) and mismatched-text logits + gradients. */
int mg_d_loss(const float* img_real, const float* img_fake, const float* tb, const int32_t* perm, int B, int No, int Nf, float* out, float* g_img, float* g_fake, float* g_tb, float* real_out, float* mism_out, float* fake_out, void* stream);

/* Generator adversarial loss softplus(-f).mean() and its gradient (t2i_moe_gan.py:917-924). */
int mg_g_loss(const float* fake, int B, float scale, float* out, float* g, void* stream);

/* R1 penalty (t2i_moe_gan.py:1285-1286): r1 += gamma/2 mean_b ||g_b||^2; u = gamma/B g. */
int mg_r1(int dtype, const void* g, int64_t per, int B, float gamma, float* r1, int u_dtype, void* u, void* stream);

/* out = a * LeakyReLU'(m). */
int mg_lrelu_mask_mul(int a_dtype, const void* a, int m_dtype, const void* m, int64_t n, int out_dtype, void* out, void* stream);

/* out[b,c] += sum_{p<HW} X[b*HW+p, c]  (per-image sums: cross-attention vector gradient). */
int mg_segsum(int dtype, const void* X, int64_t ld, int B, int HW, int C, float* out, void* stream);

/* ModulatedConv backward, output side: gyt = gy*d (gy = gz * lrelu'), gdd = -0.5 d^2 sum_pix gy*y; z may carry a fused residual (zsub).
   act: 0 none, 1 = z is LeakyReLU(0.2)(y) (inverted), 2 = z is the pre-activation y itself (stored by the forward's
   out_pre epilogue when a residual is fused: its sign is exact).  t2i_moe_gan.py:154-186. */
int mg_modconv_bwd_out(int dtype, int gz_dtype, const void* gz, int64_t ld_gz, const void* z, int64_t ld_z, const void* zsub, int64_t ld_zsub, const float* d, int B, int HW, int Cout, int act, void* gyt, int64_t ld_gyt, float* gdd, void* stream);

/* Row gather: out[r, :C] = src[idx[r] / idx_div, :C] * (rowscale ? rowscale[r] : 1)  (MoE dispatch
   order, t2i_moe_gan.py:430-445: tokens routed to expert e, k copies per token).  C % 8 == 0. */
int mg_gather_rows(int dtype, const void* src, int64_t lds, const int32_t* idx, int idx_div, const float* rowscale, int n, int C, void* out, int64_t ldo, void* stream);

/* Modulated-conv input xs[b,p,c] = x[b,p,c] * s[b,c] (x rows [B*HW, ldx], C % 8 == 0); replaces the
   per-tap operand scaling of the fused modulated conv (t2i_moe_gan.py:167-171, x * style). */
int mg_scale_bc(int dtype, const void* x, int64_t ldx, const float* s, int64_t lds, int B, int HW, int C, void* out, int64_t ldo, void* stream);

/* ModulatedConv backward, input side: gx (+)= gxt*s, gs[b,ci] += sum_pix gxt*x (s and gs rows of pitch ld_s:
   column slices of the batched style matrix). */
int mg_modconv_bwd_in(int gxt_dtype, const void* gxt, int64_t ld_gxt, int dtype, const void* x, int64_t ld_x, const float* s, int64_t ld_s, int B, int HW, int Cin, int gx_dtype, void* gx, int64_t ld_gx, int accumulate, float* gs, void* stream);

/* Generator KL total and per-router gradient coefficients (total clamped at 50, t2i_moe_gan.py:1369-1370). */
int mg_kl_coefs(const float* kl2, int R, float eff_w, float* coef, float* total, void* stream);

/* BayesianRouter.reparameterize with explicit epsilon (t2i_moe_gan.py:302-333). */
int mg_router_reparam(const float* mu, const float* rho, const float* eps, int64_t n, float* W, void* stream);

/* BayesianRouter.forward on tokens (t2i_moe_gan.py:335-402): logits = tok@Wfc + Lt[b], temperature/clamp/softmax/clamp/renorm, top-k (lowest index on ties), gate weights (renormalised for k<E, probs for k==E, 1 in eval). zlog = scaled pre-clamp logits. */
int mg_router_fwd(int dtype, const void* tok, int64_t ld, int T, int C, const float* Wfc, const float* Lt, int E, int k, int HW, const float* temperature, float anneal, int eval_mode, float* probs, float* zlog, int32_t* topi, float* gate, void* stream);

/* Deterministic per-expert position lists (token order): row_off/tile_off (BM=bm), perm[pos]=assignment, pos_of[assignment]=pos, gate_pos. ws: int32 [ceil(T*k/1024)*E]. */
int mg_moe_dispatch(const int32_t* topi, const float* gate, int T, int k, int E, int bm, int32_t* ws, int32_t* row_off, int32_t* tile_off, int32_t* perm, int32_t* pos_of, float* gate_pos, void* stream);

/* out[t] = resid[t] + sum_j gate[t,j] Y[pos_of[t*k+j]]  (SparseMoE combine + AttentionBlock residual, t2i_moe_gan.py:465-470, :571). */
int mg_moe_combine(int dtype, const void* Y, int64_t ldy, const int32_t* pos_of, const float* gate, int T, int k, int C, const void* resid, int64_t ldr, void* out, int64_t ldo, void* stream);
/* mg_moe_combine plus the AttentionBlock's proj_out modulated-conv input (t2i_moe_gan.py:158-161, :574): also
   xs[t] = bf16(out[t]) * s[t / HW] (s: [T / HW, C] fp32, one style row per image; HW a power of two), the bytes
   mg_scale_bc would form from the stored out. */
int mg_moe_combine_scaled(int dtype, const void* Y, int64_t ldy, const int32_t* pos_of, const float* gate, int T, int k, int C, const void* resid, int64_t ldr, void* out, int64_t ldo, const float* s, int64_t lds, int HW, void* xs, int64_t ldxs, void* stream);

/* g_gate[t*k+j] = <gout[t], Y[pos_of[t*k+j]]>. */
int mg_moe_gate_grad(int dtype, int gout_dtype, const void* gout, int64_t ldg, const void* Y, int64_t ldy, const int32_t* pos_of, int T, int k, int C, float* g_gate, void* stream);

/* Router backward per token -> g_raw [T,E], per-image sums gsum [B,E] (written), temperature grad (+=; per-block
   partials in the stream's workspace, folded in a fixed order: bit-identical run to run).  HW (tokens per image) a
   power of two <= 256.  Upstream gradients (each optional): g_gate (combine weights), g_probs + coef[e]
   (probabilities), g_logits (the clamped logits, the router's second output).  Reference :374-389. */
int mg_router_bwd(const float* probs, const float* zlog, const int32_t* topi, const float* gate, const float* g_gate, const float* g_probs, const float* g_logits, const float* coef, int T, int E, int k, int HW, const float* temperature, float anneal, float* g_raw, float* gsum, float* g_temp, void* stream);

/* g_tok[t] = sum_j gX[pos_of[t*k+j]] + sum_e g_raw[t,e] Wfc[:,e]. */
int mg_moe_token_grad(int dtype, const void* gX, int64_t ldx, const int32_t* pos_of, int T, int k, int C, const float* g_raw, const float* Wfc, int E, int out_dtype, void* out, int64_t ldo, void* stream);

/* G1[c,e] += sum_t tok[t,c] g_raw[t,e]. */
int mg_router_feat_grad(int dtype, const void* tok, int64_t ld, int T, int C, const float* g_raw, int E, float* G1, void* stream);

/* out[g][n] += sum_{r in group g} X[idx(r)][n] * rs[r]  (per-expert bias gradients). */
int mg_grouped_colsum(int dtype, const void* X, int64_t ld, const int32_t* idx, int idx_div, const float* rs, const int32_t* row_off, int G, int N, int max_rows, float* out, void* stream);

/* BayesianRouter.kl_divergence (t2i_moe_gan.py:405-423): out[0] = clamped KL, out[1] = gradient-pass flag. */
int mg_router_kl(const float* mu_f, const float* rho_f, int nf, const float* mu_t, const float* rho_t, int nt, const float* mu_c, const float* rho_c, int nc, float* out, void* stream);
/* The KL terms of up to 8 routers in two launches (the generator's per-block routers at the start of its forward;
   replaces one mg_router_kl pair per block, t2i_moe_gan.py:405-423): out[2 j] = KL of record j, out[2 j + 1] = its
   pass flag, bit-identical to mg_router_kl on the same record. */
typedef struct {
  const float* mu_f; const float* rho_f; const float* mu_t; const float* rho_t; const float* mu_c; const float* rho_c;
  int32_t nf; int32_t nt; int32_t nc; int32_t pad;
} mg_kl_rec;
int mg_router_kl_batch(int n, const mg_kl_rec* recs, float* out, void* stream);

/* Router parameter gradients: reparameterisation chain (gW, NULL = none) + KL term (coefficient *kl_coef).
   flags[0] & mask (optional): drop the gW chain -- a non-finite generator loss was replaced by 0 and only the
   KL term keeps a gradient (t2i_moe_gan.py:1396-1404). */
int mg_router_param_bwd(const float* mu, const float* rho, const float* eps, const float* gW, int64_t n, const float* kl_coef, float* gmu, float* grho, const int32_t* flags, int32_t mask, void* stream);

/* Every router parameter tensor of a backward in one launch (at most 32 descriptors): for each descriptor the
   arithmetic of mg_router_param_bwd (same results), one shared guard word (flags & mask drops every gW chain). */
typedef struct mg_router_param_desc {
  const float* mu;
  const float* rho;
  const float* eps;
  const float* gW;
  const float* kl_coef;
  float* gmu;
  float* grho;
  int64_t n;
} mg_router_param_desc;
int mg_router_param_bwd_batch(int n, const mg_router_param_desc* descs, const int32_t* flags, int32_t mask, void* stream);

/* moe_balance_loss from global per-expert prob sums (t2i_moe_gan.py:951-1000): out[0] = loss, coef[e] = d loss/d probs[t,e] * grad_scale. */
int mg_balance(const float* load, int E, float T, float weight, float grad_scale, float* out, float* coef, void* stream);

/* MTM offset head (conv 32->2) + linspace grid + clamp + bilinear grid_sample (zeros, align_corners=False), t2i_moe_gan.py:222-239. samp [P,4] saved. */
int mg_warp_fwd(int dtype, const void* x, const void* o1, const float* w2, const float* b2, int B, int H, int W, int C, void* out, float* samp, void* stream);
/* mg_warp_fwd that also writes out_scaled[b,..,c] = out[b,..,c] * s[b*lds + c] in the same pass: the following
 * modulated conv's prescaled input (t2i_moe_gan.py:158-161, as mg_scale_bc). s fp32. */
int mg_warp_fwd_scaled(int dtype, const void* x, const void* o1, const float* w2, const float* b2, int B, int H, int W, int C, const float* s, int64_t lds, void* out, void* out_scaled, float* samp, void* stream);

/* grid_sample backward: gx (fp32, +=, atomics) and goff [P,2] = d loss / d offsets. */
int mg_warp_bwd(int dtype, int gout_dtype, const void* gout, const void* x, const float* samp, int B, int H, int W, int C, float* gx, float* goff, void* stream);

/* Fused MTM backward for images of at most 1024 pixels (t2i_moe_gan.py:222-239 backward; replaces mg_warp_bwd +
   mg_offset_head_bwd there): grid_sample data gradient by gather into gx (dtype gx_dtype, = or += when accumulate;
   no atomics), dL/doffsets per pixel, and the offset head backward: ga1, gw2 +=, gb2 +=.  C = 8 * 2^k <= 512. */
int mg_mtm_bwd_fused(int dtype, int gout_dtype, const void* gout, const void* x, const float* samp, const void* o1, const float* w2, int B, int H, int W, int C, int gx_dtype, void* gx, int accumulate, void* ga1, float* gw2, float* gb2, void* stream);

/* offset_net second conv backward fused with the first conv's LeakyReLU: ga1, gw2 +=, gb2 +=. */
int mg_offset_head_bwd(int dtype, const float* goff, const void* o1, const float* w2, int B, int H, int W, void* ga1, float* gw2, float* gb2, void* stream);

/* nn.Upsample(scale_factor=2, bilinear, align_corners=False), NHWC (t2i_moe_gan.py:633). */
int mg_upsample2x_fwd(int dtype, const void* x, int B, int H, int W, int C, void* out, void* stream);
/* mg_upsample2x_fwd plus the ConvolutionBlock's skip_proj modulated-conv input (:615-616, :158-161): also
   xs = bf16(out) * s[b] (s: [B, C] fp32 style rows, pitch lds), what mg_scale_bc would form from out. */
int mg_upsample2x_fwd_scaled(int dtype, const void* x, int B, int H, int W, int C, void* out, const float* s, int64_t lds, void* xs, void* stream);

/* bilinear x2 backward (gather form, deterministic). */
int mg_upsample2x_bwd(int gout_dtype, const void* gout, int B, int H, int W, int C, int gx_dtype, void* gx, int accumulate, void* stream);

/* Per-step weight packing (fp32 master -> compute dtype): wpack[o][(kh*KW+kw)*Cin+ci] = W[o][ci][kh][kw]; rows >= Cout zero-padded. */
int mg_pack_conv(int dtype, const float* W, int Cout, int Cin, int KH, int KW, int rows, void* out, void* stream);

/* Flipped/transposed pack for the stride-1 data gradient: out[ci][(kh*KW+kw)*Cout+o] = W[o][ci][KH-1-kh][KW-1-kw]. */
int mg_pack_conv_flip(int dtype, const float* W, int Cout, int Cin, int KH, int KW, int rows, void* out, void* stream);

/* Per-parity-class pack for mg_conv2d_dgrad_s2: out[cls][ci][t*Cg+co]. */
int mg_pack_dgrad_s2(int dtype, const float* W, int Cg, int Cin, int rows, void* out, void* stream);

/* wsq[o][ci] = sum_taps W[o][ci][tap]^2 (demodulation, t2i_moe_gan.py:165). */
int mg_wsq(const float* W, int Cout, int Cin, int taps, int rows, float* out, void* stream);

/* gW[o][ci][t] += 2 W[o][ci][t] gwsq[o][ci]  (demodulation backward). */
int mg_wsq_bwd(const float* W, const float* gwsq, int Cout, int Cin, int taps, float* gW, void* stream);

/* Multi-tensor weight preparation: every descriptor's element map in ONE launch (tables of more than 32
   descriptors take one launch per 32).  Kinds and fields (W = fp32 source; out in the launch dtype for the
   packs, fp32 otherwise):
     MG_PREP_PACK          = mg_pack_conv       (Cout, Cin, KH, KW, rows)
     MG_PREP_PACK_FLIP     = mg_pack_conv_flip  (Cout, Cin, KH, KW, rows)
     MG_PREP_PACK_DGRAD_S2 = mg_pack_dgrad_s2   (Cout = Cg, Cin, rows)
     MG_PREP_WSQ           = mg_wsq             (Cout, Cin, KH*KW = taps, rows)
     MG_PREP_WSQ_BWD       = mg_wsq_bwd         (Cout, Cin, KH*KW = taps; aux = gwsq; out = gW, +=)
     MG_PREP_REPARAM       = mg_router_reparam  (W = mu, aux = rho, aux2 = eps, n; out = W)
   n is derived from the shape fields except for MG_PREP_REPARAM. */
#define MG_PREP_PACK 1
#define MG_PREP_PACK_FLIP 2
#define MG_PREP_PACK_DGRAD_S2 3
#define MG_PREP_WSQ 4
#define MG_PREP_WSQ_BWD 5
#define MG_PREP_REPARAM 6
typedef struct mg_prep_desc {
  int32_t kind;
  int32_t Cout, Cin, KH, KW, rows;
  int64_t n;
  const float* W;
  const float* aux;
  const float* aux2;
  void* out;
} mg_prep_desc;
int mg_prep_batch(int dtype, int n, const mg_prep_desc* descs, void* stream);

/* Gradient folds: the second pass of the two-pass gradient reductions (split-K weight-gradient slabs, per-image /
   per-block partial rows), normally one launch each right after its producer.  mg_fold_defer(1, stream): from now
   on the producers on `stream` (conv weight gradients with split-K slabs, the direct offset-head weight gradient,
   the fused MTM backward's offset-head rows, the router feature / temperature rows) keep their partials in a
   per-stream arena that is not reused before the flush and record their folds; mg_fold_flush(stream) runs every
   recorded fold in one launch per kind and recycles the arena; mg_fold_defer(0, stream) flushes and stops.  The
   gradients are only final after the flush.  Deferred and immediate folds run the same kernels (bit-identical).
   The arena grows outside stream capture only (a captured step replays the allocation sequence of its eager warm-up;
   under capture a producer that finds no room folds immediately). */
typedef struct mg_fold_rows {
  const float* src; /* nrows partial rows, row r at src + r * stride */
  int64_t stride;
  int32_t nrows, ncols, na; /* out_a[i] += sum_r src[r * stride + i] for i < na, out_b[i - na] for na <= i < ncols */
  float* out_a;
  float* out_b;
} mg_fold_rows;
typedef struct mg_fold_wgrad {
  const float* ws; /* splits slabs [splits][Cout][taps * Cin] (tap-major columns) */
  int32_t splits, Cout, lgCin, taps, lgCC; /* Cin = 1 << lgCin; blocks of CC = 1 << lgCC input channels */
  float* gw;       /* [Cout][Cin][taps] (reference layout), accumulated */
} mg_fold_wgrad;
int mg_fold_defer(int on, void* stream);
int mg_fold_flush(void* stream);
/* The arena: capped at 2 GiB per stream (a producer that finds no room folds immediately).  mg_fold_release frees a
   stream's arena (after a stream synchronize; the stream must not be deferring); mg_fold_arena_bytes: bytes held. */
int mg_fold_release(void* stream);
int64_t mg_fold_arena_bytes(void* stream);
/* the rows-fold kernel on caller records (tests / tools) */
int mg_fold_rows_batch(int n, const mg_fold_rows* recs, void* stream);
/* caller records as folds of the stream: queued behind its pending folds when it defers them (they run after
   every deferred weight-gradient fold of the flush, so a record may read one's output), else run now */
int mg_fold_rows_queue(int n, const mg_fold_rows* recs, void* stream);

/* Multi-tensor column sums (bias gradients of a whole backward in one launch): out[c] += sum_r X[r*ld+c]
   for every descriptor; fp32 atomics across row blocks (at most 32 descriptors per launch). */
typedef struct mg_colsum_desc {
  int32_t dtype, R, C;
  int64_t ld;
  const void* X;
  float* out;
} mg_colsum_desc;
int mg_colsum_batch(int n, const mg_colsum_desc* descs, void* stream);

/* out = (alpha*in)[^2 if square] with dtype conversion. */
int mg_cast(int in_dtype, const void* in, int out_dtype, void* out, int64_t n, float alpha, int square, void* stream);

/* strided 2-D copy/cast: out[r*ldo+c] (+)= alpha*in[r*ldi+c]. */
int mg_copy2d(int in_dtype, const void* in, int64_t ldi, int out_dtype, void* out, int64_t ldo, int R, int C, float alpha, int accumulate, void* stream);

/* out[c] += sum_r X[r*ld+c]  (bias gradients). */
int mg_colsum(int dtype, const void* X, int64_t ld, int R, int C, float* out, void* stream);

/* weight_norm (dim 0): W = g v / ||v||  (t2i_moe_gan.py:869-886). */
int mg_weight_norm_fwd(const float* v, const float* g, int O, int K, float* W, float* norm, void* stream);

/* weight_norm backward: gg += sum gW v/||v||, gv += (g/||v||)(gW - gg_o v/||v||). */
int mg_weight_norm_bwd(const float* v, const float* g, const float* norm, const float* gW, int O, int K, float* gv, float* gg, void* stream);

/* Batched weight_norm of several layers in one launch (the discriminator's four, t2i_moe_gan.py:869-886): per
   descriptor, bwd = 0 computes W and norm from (v, g) as mg_weight_norm_fwd; bwd = 1 accumulates gv and gg from
   (v, g, norm, gW) as mg_weight_norm_bwd.  One block per output row; at most 8 descriptors per launch. */
typedef struct mg_wn_desc {
  int32_t O, K;
  const float* v;
  const float* g;
  float* norm;     /* fwd: out; bwd: in */
  float* W;        /* fwd: out */
  const float* gW; /* bwd: in */
  float* gv;       /* bwd: +=  */
  float* gg;       /* bwd: +=  */
} mg_wn_desc;
int mg_weight_norm_batch(int bwd, int n, const mg_wn_desc* descs, void* stream);

/* out[0] += sum x^2 (clip_grad_norm_ total norm, t2i_moe_gan.py:1336/1420); deterministic (fixed-order fold). */
int mg_sumsq(const float* x, int64_t n, float* out, void* stream);

/* torch.optim.AdamW step over a flat fp32 range fused with clip_grad_norm_ (coef from *sumsq, max_norm); t2i_moe_gan.py:1101-1102. */
int mg_adamw(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2, float eps, float weight_decay, int step, const float* sumsq, float max_norm, void* stream);

/* Optimizer prologue for graph-replayable steps: sumsq[0] = 0 (if sumsq), step[0] += 1 (if step and the gate
   below passes; the AdamW step counter lives on the device so a captured hipGraph advances it on every replay:
   torch's state['step']).
   Gate (loss guards, mg_finite_flag / mg_flag_window): the update is skipped when flags[0] & skip_mask, and
   when run_mask != 0 and !(win[0] & run_mask); flags = NULL: always run. */
int mg_opt_prologue(float* sumsq, int32_t* step, const int32_t* flags, int32_t skip_mask, const int32_t* win,
                    int32_t run_mask, void* stream);

/* clip_grad_norm_'s sum of squares and the AdamW step counters of one parameter store in two launches instead of
   mg_opt_prologue + mg_sumsq + one mg_opt_prologue per optimizer launch: out[0] = sum of x[0..n)^2 (written, the fixed
   fold order of mg_sumsq), then step0[0] += 1 and step1[0] += 1 (NULL = none) each under mg_opt_prologue's gate --
   not when flags[0] & skip_mask, and only when win[0] & run_mask (run_mask 0 or win NULL: always). */
int mg_grad_norm_steps(const float* x, int64_t n, float* out, int32_t* step0, int32_t run_mask0, int32_t* step1, int32_t run_mask1, const int32_t* flags, int32_t skip_mask, const int32_t* win, void* stream);

/* mg_adamw with the step count read from device memory (*step >= 1); bias corrections on the device. */
int mg_adamw_dev(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2, float eps, float weight_decay, const int32_t* step, const float* sumsq, float max_norm, void* stream);
/* Same update (t2i_moe_gan.py:1333-1421), 16-B vectors, and (shadow_bf16 != NULL) the bf16 compute copy of the
   updated parameters written in the same pass (replaces the next step's fp32 -> bf16 parameter cast). */
int mg_adamw_dev_shadow(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2, float eps, float weight_decay, const int32_t* step, const float* sumsq, float max_norm, void* shadow_bf16, const int32_t* flags, int32_t skip_mask, const int32_t* win, int32_t run_mask, void* stream);

/* ---- loss guards (t2i_moe_gan.py:1315-1320 NaN/Inf d_loss -> skip the batch; :1367-1376 NaN KL -> 0;
   :1396-1399 NaN/Inf g_loss -> 0) as device-side flags, read by the gated optimizer calls above ---- */
#define MG_FLAG_D_BAD 1  /* discriminator loss (GAN + R1) non-finite: the whole batch is skipped */
#define MG_FLAG_G_BAD 2  /* generator loss (GAN + CLIP + balance) non-finite: replaced by 0 (KL term kept) */
#define MG_WIN_D 1       /* accumulation window: the discriminator received a gradient */
#define MG_WIN_G_MAIN 2  /* ... the generator's non-KL parameters received a gradient */
#define MG_WIN_G_KL 4    /* ... the routers' KL parameters (mu / rho) received a gradient */
/* flags[0] |= bit if any of x[0..n) is NaN or Inf. */
int mg_finite_flag(const float* x, int n, int32_t bit, int32_t* flags, void* stream);
/* Window word update: win[0] &= ~reset_bits unless flags[0] & keep_mask (a skipped batch does not reach the
   reference's zero_grad, t2i_moe_gan.py:1353); then win[0] |= set_bits unless flags[0] & bad_mask. */
int mg_flag_window(const int32_t* flags, int32_t reset_bits, int32_t keep_mask, int32_t bad_mask, int32_t set_bits, int32_t* win, void* stream);

/* One phase's loss checks and window updates in one launch (mg_finite_flag x n + mg_flag_window x nwin): for each
   check c with n[c] > 0, flags[0] |= bit[c] if any of x[c][0 .. n[c]) is NaN / Inf; then the nwin (<= 2) window
   updates in order, each with mg_flag_window's rule on the updated flags. */
typedef struct mg_guard_desc {
  const float* x[4];
  int32_t n[4];
  int32_t bit[4];
  int32_t nwin;
  int32_t reset_bits[2];
  int32_t keep_mask[2];
  int32_t bad_mask[2];
  int32_t set_bits[2];
} mg_guard_desc;
int mg_guard_update(const mg_guard_desc* d, int32_t* flags, int32_t* win, void* stream);
/* x[0..bytes) = 0 when ((flags[0] & mask) != 0) == (when_set != 0). */
int mg_zero_if(void* x, int64_t bytes, const int32_t* flags, int32_t mask, int when_set, void* stream);
/* acc[i] += g[i] unless flags[0] & mask (gradient accumulation of a batch that may be skipped). */
int mg_gated_axpy(float* acc, const float* g, int64_t n, const int32_t* flags, int32_t mask, void* stream);
/* out[i] = (flags[0] & mask) ? src[i] : 0  (n <= 4096). */
int mg_select_if(const float* src, int n, const int32_t* flags, int32_t mask, float* out, void* stream);
/* A step's random inputs in one launch (csrc/mg_rng.hip): eps_a[0..na) and eps_b[0..nb) ~ N(0, 1) (the router noise
   of the two generator forwards, t2i_moe_gan.py:302-333) and perm = a uniformly random permutation of 0..B-1 (the
   mismatched captions, :1278; B <= 4096).  Counter-based: the draws depend only on the two seeds. */
int mg_step_inputs(float* eps_a, int64_t na, float* eps_b, int64_t nb, int32_t* perm, int B, uint64_t seed_eps,
                   uint64_t seed_perm, void* stream);

/* generator constant [1,C,4,4] -> NHWC [B,4,4,C] (t2i_moe_gan.py:815). */
int mg_const_fwd(int dtype, const float* cst, int C, int HW, int B, void* out, void* stream);

/* gconst[c][p] += sum_b g[b][p][c]. */
int mg_const_bwd(int dtype, const void* g, int C, int HW, int B, float* gc, void* stream);

#ifdef __cplusplus
}
#endif
#endif
