/* libmoegan_hip -- C ABI of the MI355X-native MoE-GAN training-step kernels.
 *
 * The reference (moegan/t2i_moe_gan.py) has no FFI: its hot path is a stack of
 * PyTorch modules.  This header is the boundary those modules' math is moved
 * behind; the drop-in Python modules (moe-gan_cpsc541_amd/t2i_moe_gan.py) bind
 * it with ctypes.  Each entry cites the reference code it replaces.
 *
 * Conventions
 *  - Plain pointers + sizes, no framework types.  The caller owns every buffer
 *    (device memory) and the library never allocates, frees or synchronises.
 *  - Activations are NHWC ("token") layout: [B, H, W, C] == [B*H*W, C] rows.
 *  - dtype: MG_F32 (exact fp32 parity mode) or MG_BF16 (bf16 storage, fp32
 *    accumulate).  Weight gradients and all reductions are fp32.
 *  - Every call is enqueued on `stream` (a hipStream_t; NULL = default).
 *  - Return 0 on success or a negative MG_ERR_*; mg_last_error() gives the
 *    thread-local message.  Thread-safe / reentrant (no global state).
 */
#ifndef MOEGAN_HIP_H
#define MOEGAN_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MG_OK 0
#define MG_ERR_ARG (-1)
#define MG_ERR_LAUNCH (-2)

#define MG_F32 0
#define MG_BF16 1

/* epilogue activation codes */
#define MG_ACT_NONE 0
#define MG_ACT_LRELU 1          /* LeakyReLU(0.2)  (t2i_moe_gan.py:216, :685) */
#define MG_ACT_GELU 2           /* exact-erf GELU  (t2i_moe_gan.py:258) */
#define MG_ACT_MUL_GELU_GRAD 3  /* v *= GELU'(aux[m,n]) */
#define MG_ACT_MUL_LRELU_GRAD 4 /* v *= LReLU'(aux[m,n]) */
#define MG_ACT_RSQRT_EPS 5      /* v = rsqrt(v + 1e-8)  (demodulation, t2i_moe_gan.py:165) */

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
} mg_epilogue;

const char* mg_last_error(void);
int mg_version(void);

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

/* Implicit-GEMM NHWC convolution (square kernel KHxKW, stride, pad):
 *   y[b,oh,ow,o] = epilogue( sum_{kh,kw,ci} x[b,ih,iw,ci] * in_scale[b,ci] * wpack[o][(kh*KW+kw)*Cin+ci] )
 * in_scale (optional, fp32 [B,Cin]) fuses the modulated-conv style (t2i_moe_gan.py:158-161).
 * Cin must be a multiple of 32; H, W, OH, OW, Cin powers of two.
 * Used for ModulatedConv forward (:169-180), its data gradient (flipped wpack),
 * offset_net (:209-213) and the discriminator convs (:874-887). */
int mg_conv2d_fwd(int dtype, const void* x, int B, int H, int W, int Cin, const void* wpack, int Cout, int KH,
                  int KW, int stride, int pad, const float* in_scale, void* y, int64_t ldy, int y_dtype,
                  const mg_epilogue* ep, void* stream);

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

#ifdef __cplusplus
}
#endif
#endif
