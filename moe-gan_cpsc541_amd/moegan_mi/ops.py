"""Thin Python wrappers over the C ABI (tensor plumbing only; all math is in HIP).

Every function enqueues on torch's current stream and returns its output
tensor(s).  Shapes follow include/moegan_hip.h: activations are NHWC/token
rows, weights are in the reference layout unless a ``pack`` says otherwise.
"""
import ctypes
import math

import os

import torch

from . import _lib as L

call, ptr, dt, S = L.call, L.ptr, L.dt, L.stream
E = L.epilogue


TUNE_DETERMINISTIC = 11  # mg_common.h MG_TUNE_DETERMINISTIC


def set_deterministic(on=True):
    """Deterministic mode of the library: every cross-workgroup reduction of the step in a fixed
    order (partial rows + one fold, or one writer per element) instead of fp32 atomics, so two identically
    initialised steps give bit-identical results; slower.  Process-wide, like torch's own switch."""
    call("mg_set_tuning", TUNE_DETERMINISTIC, 1 if on else 0)


def _ld(t):
    return t.stride(0) if t.dim() > 1 else t.shape[0]


# Optional live kernel timer (bench.py): when set, launches whose (kind, dims) satisfy
# TIMER.want(kind, dims) are bracketed by HIP events on the current stream while TIMER.active.
# Under graph capture such a launch becomes an eager segment (graphs.eager), so the events
# still bracket exactly that kernel on every replay.
TIMER = None


class KernelTimer:
    def __init__(self, want, active=True):
        self.want = want
        self.active = active
        self.events = []  # (kind, dims, start, end)

    def record(self, kind, dims, fn):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        r = fn()
        e.record()
        self.events.append((kind, dims, s, e))
        return r

    def results(self):
        torch.cuda.synchronize()
        return [(k, d, s.elapsed_time(e)) for k, d, s, e in self.events]


def _timed_run(kind, dims, fn):
    t = TIMER
    if t is None or not t.active:
        return fn()
    return t.record(kind, dims, fn)


def _timed(kind, dims, fn):
    if TIMER is None or not TIMER.want(kind, dims):
        return fn()
    from . import graphs
    return graphs.eager(lambda: _timed_run(kind, dims, fn))


# ---------------------------------------------------------------------------
# Per-step pool of zero-initialised scratch (accumulation targets of atomics / accumulating epilogues):
# TrainStep.step zeroes the used prefix of ONE buffer per step instead of one fill launch per buffer.
# Outside an active step (module API, tests) zeros() is plain torch.zeros.
# ---------------------------------------------------------------------------
class ZeroArena:
    ALIGN = 256

    def __init__(self):
        self.buf = None
        self.off = 0
        self.need = 0
        self.active = False

    def begin(self, device):
        if self.need > 0 and (self.buf is None or self.buf.numel() < self.need or self.buf.device != device):
            self.buf = torch.empty(self.need, device=device, dtype=torch.uint8)
        if self.buf is not None:
            self.buf[:min(self.need, self.buf.numel())].zero_()
        self.off = 0
        self.active = True

    def end(self):
        self.need = max(self.need, self.off)
        self.active = False

    def zeros(self, shape, dtype, device):
        n = math.prod(shape) * torch.empty((), dtype=dtype).element_size()
        a = (n + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        o = self.off
        if self.active:
            self.off += a
        if (not self.active or self.buf is None or o + a > self.buf.numel() or o + a > self.need
                or self.buf.device != torch.device(device)):
            return torch.zeros(shape, device=device, dtype=dtype)
        return self.buf[o:o + n].view(dtype).view(shape)


ARENA = ZeroArena()


def fold_defer(on):
    """Defer (True) the gradient folds of the library's two-pass reductions issued on the current stream until
    fold_flush(), or flush and stop deferring (False) -- mg_fold_defer."""
    call("mg_fold_defer", int(bool(on)), S())
    if not on:
        _FOLD_KEEP.clear()


class _FoldRows(ctypes.Structure):
    """Mirror of ``mg_fold_rows``."""
    _fields_ = [("src", ctypes.c_void_p), ("stride", ctypes.c_int64), ("nrows", ctypes.c_int32),
                ("ncols", ctypes.c_int32), ("na", ctypes.c_int32), ("out_a", ctypes.c_void_p), ("out_b", ctypes.c_void_p)]


_FOLD_KEEP = []  # tensors a queued fold reads or writes: held until the flush (the caching allocator must not
# hand their memory to later work while the fold is still pending)


def fold_add(pairs):
    """dst += src (fp32, contiguous, same size) for every (src, dst) pair as folds of the current stream: queued
    behind its deferred folds inside a training step (so src may be a deferred fold's output), else run now."""
    _FOLD_KEEP.extend(t for pair in pairs for t in pair)
    recs = (_FoldRows * len(pairs))()
    for i, (src, dst) in enumerate(pairs):
        assert src.dtype == dst.dtype == torch.float32 and src.is_contiguous() and dst.is_contiguous()
        assert src.numel() == dst.numel() < 2 ** 31
        recs[i] = _FoldRows(src.data_ptr(), src.numel(), 1, src.numel(), src.numel(), dst.data_ptr(), None)
    call("mg_fold_rows_queue", len(pairs), ctypes.addressof(recs), S())


def fold_release(stream=None):
    """Free the gradient-fold partials arena of ``stream`` (default: the current stream) -- mg_fold_release.  The
    arena is kept across steps on purpose (a captured step replays its allocations); release it when the stream's
    training ends (TrainStep.release)."""
    st = L.ctypes.c_void_p(stream.cuda_stream) if stream is not None else S()
    call("mg_fold_release", st)


def fold_arena_bytes(stream=None):
    """Device bytes held by the gradient-fold arena of ``stream`` (memory accounting; mg_fold_arena_bytes)."""
    st = L.ctypes.c_void_p(stream.cuda_stream) if stream is not None else S()
    return int(L.lib().mg_fold_arena_bytes(st))


def fold_flush():
    """Run every deferred gradient fold of the current stream (one launch per fold kind; mg_fold_flush)."""
    call("mg_fold_flush", S())
    _FOLD_KEEP.clear()


def zeros(*shape, device, dtype=torch.float32):
    return ARENA.zeros(tuple(shape), dtype, device)


def ilog2(v):
    r = int(math.log2(v))
    assert 1 << r == v, v
    return r


# ---------------------------------------------------------------------------
# GEMM family
# ---------------------------------------------------------------------------
MG_F32X3 = 2  # include/moegan_hip.h: fp32 operands, split-bf16 MFMA products
_F32X3 = [False]


def set_f32x3(on):
    """fp32-operand GEMMs (mg_gemm / mg_gemm_batch) as split-bf16 products (MG_F32X3) while ``on``: the bf16
    training step's fp32 prefix / demodulation / router-vector GEMMs (TrainStep.step sets it for the step's
    duration); the fp32 parity mode keeps exact-fp32 MFMA.  Returns the previous setting."""
    prev = _F32X3[0]
    _F32X3[0] = bool(on)
    return prev


def _gdt(A):
    d = dt(A)
    return MG_F32X3 if (d == L.MG_F32 and _F32X3[0]) else d


def gemm(A, B, M, N, K, *, a_kc=True, b_kc=True, out=None, out_dtype=None, lda=None, ldb=None, ldc=None,
         ep=None, splits=1):
    """C[M,N] = epilogue(op(A) @ op(B)) (mg_gemm)."""
    if out is None:
        out = torch.empty(M, N, device=A.device, dtype=out_dtype or A.dtype)
    call("mg_gemm", _gdt(A), M, N, K, ptr(A), lda if lda is not None else _ld(A), int(a_kc), ptr(B),
         ldb if ldb is not None else _ld(B), int(b_kc), ptr(out), ldc if ldc is not None else _ld(out),
         dt(out), ep, splits, S())
    return out


def gemm_batch(problems, *, a_kc=True, b_kc=True):
    """Independent GEMMs in few launches (mg_gemm_batch).  problems: list of dicts with keys
    A, B, M, N, K, out (preallocated) and optional ep, lda, ldb, ldc.  All share dtype/orientation."""
    n = len(problems)
    if n == 0:
        return
    arr = (L.GemmDesc * n)()
    keep = []
    for i, q in enumerate(problems):
        A, B, out = q["A"], q["B"], q["out"]
        ep = q.get("ep")
        keep.append(ep)
        arr[i] = L.GemmDesc(q["M"], q["N"], q["K"], ptr(A), q.get("lda", _ld(A)), ptr(B), q.get("ldb", _ld(B)),
                            ptr(out), q.get("ldc", _ld(out)), ctypes.pointer(ep) if ep is not None else None)
    call("mg_gemm_batch", _gdt(problems[0]["A"]), int(a_kc), int(b_kc), dt(problems[0]["out"]), n, arr, S())


def linear(x, W, bias=None, act=0, out=None, out_dtype=None, **epk):
    """y = act(x @ W^T + bias), x [M,K], W [N,K]."""
    M, K = x.shape
    N = W.shape[0]
    return gemm(x, W, M, N, K, out=out, out_dtype=out_dtype, ep=E(bias=bias, act=act, **epk))


def linear_dgrad(g, W, out=None, accumulate=0, out_dtype=None, lrelu_out=None):
    """gx = g @ W for g [M,N], W [N,K] -> [M,K]; ``lrelu_out`` (the leaky-ReLU output y of the layer below, same
    dtype and shape as gx): gx *= lrelu'(y) in the epilogue."""
    M, N = g.shape
    K = W.shape[1]
    if lrelu_out is not None:
        odt = out_dtype or g.dtype
        assert lrelu_out.dtype == odt and tuple(lrelu_out.shape) == (M, K) and lrelu_out.stride(1) == 1
        ep = E(accumulate=accumulate, act=L.ACT_MUL_LRELU_GRAD, aux=lrelu_out, ld_aux=lrelu_out.stride(0))
    else:
        ep = E(accumulate=accumulate)
    return gemm(g, W, M, K, N, b_kc=False, out=out, out_dtype=out_dtype, ep=ep)


def linear_wgrad(g, x, gW, alpha=1.0):
    """gW [N,K] (fp32) += g^T x for g [M,N], x [M,K]."""
    M, N = g.shape
    K = x.shape[1]
    return gemm(g, x, N, K, M, a_kc=False, b_kc=False, out=gW, ldc=gW.stride(0),
                ep=E(alpha=alpha, atomic=1), splits=0)


def conv2d(x, wpack, Cout, KH, KW, stride=1, pad=0, in_scale=None, out=None, out_dtype=None, ep=None, ldy=None,
           tag=None):
    """NHWC implicit-GEMM conv (mg_conv2d_fwd): x [B,H,W,Cin] -> [B,OH,OW,Cout].  ``tag`` names the call site
    for the live kernel timer (kind "conv2d:<tag>")."""
    B, H, W, Cin = x.shape
    OH = (H + 2 * pad - KH) // stride + 1
    OW = (W + 2 * pad - KW) // stride + 1
    if out is None:
        out = torch.empty(B, OH, OW, ldy or Cout, device=x.device, dtype=out_dtype or x.dtype)
    _timed("conv2d" if tag is None else "conv2d:" + tag, (B * OH * OW, Cout, KH * KW * Cin),
           lambda: call("mg_conv2d_fwd", dt(x), ptr(x), B, H, W, Cin, ptr(wpack), Cout, KH, KW, stride, pad,
                        ptr(in_scale), ptr(out), ldy or out.shape[-1], dt(out), ep, S()))
    return out


def quant_mx8(x, K=None):
    """MX-fp8 quantization of bf16 rows (mg_quant_mx8): x [rows, K] -> (q uint8 e4m3 [rows, K], scale uint8
    E8M0 [rows, K/32])."""
    x2 = x.reshape(-1, x.shape[-1]) if K is None else x.reshape(-1, K)
    rows, K = x2.shape
    q = torch.empty(rows, K, device=x.device, dtype=torch.uint8)
    sc = torch.empty(rows, K // 32, device=x.device, dtype=torch.uint8)
    call("mg_quant_mx8", ptr(x2), x2.stride(0), rows, K, ptr(q), ptr(sc), S())
    return q, sc


def quant_mx8_batch(xs):
    """quant_mx8 of several bf16 [rows, K] matrices in one launch (mg_quant_mx8_batch): [(q, scale)] per input."""
    out = []
    arr = (L.QuantDesc * max(1, len(xs)))()
    for i, x in enumerate(xs):
        rows, K = x.shape
        q = torch.empty(rows, K, device=x.device, dtype=torch.uint8)
        sc = torch.empty(rows, K // 32, device=x.device, dtype=torch.uint8)
        arr[i] = L.QuantDesc(ptr(x), x.stride(0), rows, K, ptr(q), ptr(sc))
        out.append((q, sc))
    if xs:
        call("mg_quant_mx8_batch", len(xs), arr, S())
    return out


def conv2d_mx8(xq, xsc, wq, wsc, Cout, KH, KW, stride=1, pad=0, out=None, out_dtype=torch.bfloat16, ep=None,
               ldy=None, tag=None):
    """MX-fp8 NHWC implicit-GEMM conv (mg_conv2d_fwd_mx8): xq [B,H,W,Cin] e4m3 / xsc [B*H*W, Cin/32] and
    wq / wsc from quant_mx8 (activation rows, packed [Cout, KH*KW*Cin] weights)."""
    B, H, W, Cin = xq.shape
    x = xq
    OH = (H + 2 * pad - KH) // stride + 1
    OW = (W + 2 * pad - KW) // stride + 1
    if out is None:
        out = torch.empty(B, OH, OW, ldy or Cout, device=x.device, dtype=out_dtype)
    _timed("conv2d_mx8" if tag is None else "conv2d_mx8:" + tag, (B * OH * OW, Cout, KH * KW * Cin),
           lambda: call("mg_conv2d_fwd_mx8", ptr(x), ptr(xsc), B, H, W, Cin, ptr(wq), ptr(wsc), Cout, KH, KW, stride, pad,
                        ptr(out), ldy or out.shape[-1], dt(out), ep, S()))
    return out


def conv2d_wgrad(gy, x, Cout, KH, KW, stride, pad, gw, in_scale=None, ldg=None, splits=0):
    """gw [Cout,Cin,KH,KW] fp32 += weight gradient (mg_conv2d_wgrad)."""
    B, H, W, Cin = x.shape
    call("mg_conv2d_wgrad", dt(x), ptr(gy), ldg or gy.shape[-1], ptr(x), B, H, W, Cin, ptr(in_scale), Cout, KH, KW,
         stride, pad, ptr(gw), splits, S())
    return gw


def dgrad_s2(g, wcls, Cin, out, ep=None):
    """4x4/s2/p1 conv data gradient: g [B,OH,OW,Cg] -> out [B,2OH,2OW,ldo]."""
    B, OH, OW, Cg = g.shape
    call("mg_conv2d_dgrad_s2", dt(g), ptr(g), B, OH, OW, Cg, ptr(wcls), Cin, ptr(out), out.shape[-1], dt(out), ep,
         S())
    return out


def dgrad_s2_small(g, wpack, Cin, out):
    """4x4/s2/p1 conv data gradient for few input channels (Cin <= 4): Y = g @ wpack ([Cg, 16*Cin] pack_conv
    layout; fp32), then mg_col2im_4x4s2 into out [B, 2OH, 2OW, ldo] (channels < Cin written)."""
    B, OH, OW, Cg = g.shape
    Y = gemm(g.view(-1, Cg), wpack, B * OH * OW, 16 * Cin, Cg, b_kc=False, out_dtype=torch.float32)
    call("mg_col2im_4x4s2", L.MG_F32, ptr(Y), 16 * Cin, B, OH, OW, Cin, dt(out), ptr(out), out.shape[-1], S())
    return out


def gemm_grouped(A, B, row_off, tile_off, max_tiles, N, K, *, b_kc=True, b_gstride, out, ep=None, lda=None,
                 ldb=None, ldc=None):
    _timed("gemm_grouped", (out.shape[0], N, K),
           lambda: call("mg_gemm_grouped", dt(A), out.shape[0], N, K, row_off.shape[0] - 1, ptr(row_off),
                        ptr(tile_off), max_tiles, ptr(A), lda or _ld(A), ptr(B), ldb or B.shape[-1], int(b_kc),
                        b_gstride, ptr(out), ldc or _ld(out), dt(out), ep, S()))
    return out


# the fused forward's GELU output is stored for the layer-2 weight gradient (1) or recomputed there from the
# pre-activation by the GEMM loader (0, default).  Measured at the C2 16x16 block (profiles/round5_expert_probe*.txt):
# the saved forward 133 -> 90 us without the [rows x 4C] GELU-output write, the weight gradient 74 -> 80 us with
# GELU on load.
FFN_SAVE_HID = os.environ.get("MOEGAN_FFN_HID", "0") == "1"


def ffn_fusable(dtype, C):
    """The fused expert FFN is used where it measured faster than the two grouped GEMMs: bf16, C = 128
    (B=256, E=8 top-2: 145 -> 116 us no-grad, 170 -> 144 us saved).  C = 256 stays on the grouped GEMMs
    (its [128 x 256] output tile leaves one block per CU: 115 -> 175 us)."""
    return dtype == torch.bfloat16 and C == 128


def moe_ffn_fwd(X, W1, b1, W2, b2, row_off, tile_off, max_tiles, Y, *, pre=None, hid=None, x_idx=None,
                x_idx_div=1):
    """Fused expert FFN (mg_moe_ffn_fwd): Y = GELU(X W1_g^T + b1_g) W2_g^T + b2_g per dispatch group."""
    G, Hd, C = W1.shape
    call("mg_moe_ffn_fwd", L.MG_BF16, Y.shape[0], C, Hd, G, ptr(row_off), ptr(tile_off), max_tiles, ptr(X), _ld(X), ptr(x_idx),
         x_idx_div, ptr(W1), ptr(b1), ptr(W2), ptr(b2), ptr(pre), ptr(hid), ptr(Y), S())
    return Y


def moe_ffn_bwd(gG, Pre, W1, W2, row_off, tile_off, max_tiles, gP, gX, gb1=None, gb2=None, hid=None):
    """Fused expert FFN backward (mg_moe_ffn_bwd): gP = (gG W2_g) * GELU'(Pre), gX = gP W1_g, gb1 += colsum(gP),
    gb2 += colsum(gG) (per group); optionally hid = GELU(Pre) (bf16, what the W2 weight gradient reads)."""
    G, Hd, C = W1.shape
    _timed("moe_ffn_bwd", (gG.shape[0], C, Hd),
           lambda: call("mg_moe_ffn_bwd", L.MG_BF16, gG.shape[0], C, Hd, G, ptr(row_off), ptr(tile_off), max_tiles,
                        ptr(gG), ptr(Pre), ptr(W1), ptr(W2), ptr(gP), ptr(gX), ptr(hid), ptr(gb1), ptr(gb2), S()))
    return gP, gX


def ffn_bwd_fusable(dtype, C):
    """The fused expert backward (gP and gX in one pass over the rows, gb1 from the same pass): bf16, C = 128
    (C = 256 with MOEGAN_FFN_BWD_FUSED256=1: built and tested, not yet measured faster)."""
    if dtype != torch.bfloat16 or os.environ.get("MOEGAN_FFN_BWD_FUSED", "1") != "1":
        return False
    return C == 128 or (C == 256 and os.environ.get("MOEGAN_FFN_BWD_FUSED256", "0") == "1")


def gemm_grouped_wgrad(A, B, row_off, total_rows, M, N, out, *, b_idx=None, b_idx_div=1, b_gelu=0, ep=None,
                       lda=None, ldb=None, splits=0):
    """out[g] (fp32 [G,M,N]) += sum over rows of group g of A[r,:]^T B[r,:]."""
    call("mg_gemm_grouped_wgrad", dt(A), M, N, row_off.shape[0] - 1, ptr(row_off), total_rows, ptr(A),
         lda or _ld(A), ptr(B), ldb or _ld(B), ptr(b_idx), b_idx_div, b_gelu, ptr(out), splits, ep, S())
    return out


# ---------------------------------------------------------------------------
# prep / elementwise / reductions
# ---------------------------------------------------------------------------
def pack_conv(W, dtype, rows=None, flip=False):
    Cout, Cin, KH, KW = W.shape
    if flip:
        rows = rows or Cin
        out = torch.empty(rows, KH * KW * Cout, device=W.device, dtype=dtype)
        call("mg_pack_conv_flip", dt(out), ptr(W), Cout, Cin, KH, KW, rows, ptr(out), S())
    else:
        rows = rows or Cout
        out = torch.empty(rows, KH * KW * Cin, device=W.device, dtype=dtype)
        call("mg_pack_conv", dt(out), ptr(W), Cout, Cin, KH, KW, rows, ptr(out), S())
    return out


def pack_dgrad_s2(W, dtype, rows=None):
    Cg, Cin = W.shape[:2]
    rows = rows or Cin
    out = torch.empty(4, rows, 4 * Cg, device=W.device, dtype=dtype)
    call("mg_pack_dgrad_s2", dt(out), ptr(W), Cg, Cin, rows, ptr(out), S())
    return out


def wsq(W, rows=None):
    Cout, Cin = W.shape[:2]
    taps = W[0, 0].numel()
    rows = rows or Cout
    out = torch.empty(rows, Cin, device=W.device, dtype=torch.float32)
    call("mg_wsq", ptr(W), Cout, Cin, taps, rows, ptr(out), S())
    return out


class PrepBatch:
    """Weight-preparation jobs (packs, demodulation sums and their backward, router reparameterisation)
    collected and launched as one mg_prep_batch call; the outputs are allocated when a job is added."""

    def __init__(self, dtype):
        self.dtype = dtype
        self.descs, self.keep = [], []

    def _add(self, kind, W, out, Cout=0, Cin=0, KH=0, KW=0, rows=0, n=0, aux=None, aux2=None):
        assert W.is_contiguous() and out.is_contiguous()
        self.descs.append(L.PrepDesc(kind, Cout, Cin, KH, KW, rows, n, W.data_ptr(),
                                     None if aux is None else aux.data_ptr(),
                                     None if aux2 is None else aux2.data_ptr(), out.data_ptr()))
        self.keep += [W, out, aux, aux2]
        return out

    def pack(self, W, rows=None, flip=False):
        Cout, Cin, KH, KW = W.shape
        if flip:
            rows = rows or Cin
            out = torch.empty(rows, KH * KW * Cout, device=W.device, dtype=self.dtype)
            return self._add(L.PREP_PACK_FLIP, W, out, Cout, Cin, KH, KW, rows)
        rows = rows or Cout
        out = torch.empty(rows, KH * KW * Cin, device=W.device, dtype=self.dtype)
        return self._add(L.PREP_PACK, W, out, Cout, Cin, KH, KW, rows)

    def pack_dgrad_s2(self, W, rows=None):
        Cg, Cin = W.shape[:2]
        rows = rows or Cin
        out = torch.empty(4, rows, 4 * Cg, device=W.device, dtype=self.dtype)
        return self._add(L.PREP_PACK_DGRAD_S2, W, out, Cg, Cin, 4, 4, rows)

    def wsq(self, W, rows=None):
        Cout, Cin = W.shape[:2]
        taps = W[0, 0].numel()
        rows = rows or Cout
        out = torch.empty(rows, Cin, device=W.device, dtype=torch.float32)
        return self._add(L.PREP_WSQ, W, out, Cout, Cin, taps, 1, rows)

    def wsq_bwd(self, W, gwsq, gW):
        Cout, Cin = W.shape[:2]
        assert gwsq.is_contiguous()
        return self._add(L.PREP_WSQ_BWD, W, gW, Cout, Cin, W[0, 0].numel(), 1, aux=gwsq)

    def reparam(self, mu, rho, eps):
        W = torch.empty_like(mu)
        return self._add(L.PREP_REPARAM, mu, W, n=mu.numel(), aux=rho, aux2=eps)

    def run(self):
        if self.descs:
            n = len(self.descs)
            arr = (L.PrepDesc * n)(*self.descs)
            call("mg_prep_batch", L.MG_BF16 if self.dtype == torch.bfloat16 else L.MG_F32, n, arr, S())
        self.descs, self.keep = [], []


def wsq_bwd(W, gwsq, gW):
    Cout, Cin = W.shape[:2]
    call("mg_wsq_bwd", ptr(W), ptr(gwsq), Cout, Cin, W[0, 0].numel(), ptr(gW), S())


def cast(x, dtype=None, out=None, alpha=1.0, square=0):
    if out is None:
        out = torch.empty(x.shape, device=x.device, dtype=dtype or x.dtype)
    call("mg_cast", dt(x), ptr(x), dt(out), ptr(out), x.numel(), alpha, square, S())
    return out


def copy2d(x, out, R, C, alpha=1.0, accumulate=0, ldi=None, ldo=None):
    call("mg_copy2d", dt(x), ptr(x), ldi or _ld(x), dt(out), ptr(out), ldo or _ld(out), R, C, alpha, accumulate, S())
    return out


class ColsumQueue:
    """Bias-gradient column sums deferred to one mg_colsum_batch launch.  Only active inside a training step
    (TrainStep sets ``active`` and flushes before the gradients are read); everywhere else ``colsum(...,
    defer=True)`` runs at once.  A deferred source must not be written again before the flush."""

    def __init__(self):
        self.active = False
        self.items = []  # (ColsumDesc, X, out)

    def add(self, X, out, R, C, ld):
        self.items.append((L.ColsumDesc(dt(X), R, C, ld, X.data_ptr(), out.data_ptr()), X, out))

    def flush(self):
        if not self.items:
            return
        n = len(self.items)
        arr = (L.ColsumDesc * n)(*[d for d, _, _ in self.items])
        call("mg_colsum_batch", n, arr, S())
        self.items = []


COLSUMS = ColsumQueue()


def colsum(X, out, R=None, C=None, ld=None, defer=False):
    """out += column sums of X (mg_colsum); ``defer`` queues it on COLSUMS while a step is running."""
    R = R if R is not None else X.shape[0]
    C = C if C is not None else X.shape[-1]
    ld = ld or X.shape[-1]
    if defer and COLSUMS.active:
        COLSUMS.add(X, out, R, C, ld)
        return out
    call("mg_colsum", dt(X), ptr(X), ld, R, C, ptr(out), S())
    return out


def segsum(X, B, HW, C, out, ld=None):
    call("mg_segsum", dt(X), ptr(X), ld or C, B, HW, C, ptr(out), S())
    return out


def weight_norm_fwd(v, g):
    O = v.shape[0]
    K = v[0].numel()
    W = torch.empty_like(v)
    norm = torch.empty(O, device=v.device, dtype=torch.float32)
    call("mg_weight_norm_fwd", ptr(v), ptr(g), O, K, ptr(W), ptr(norm), S())
    return W, norm


def weight_norm_bwd(v, g, norm, gW, gv, gg):
    O = v.shape[0]
    call("mg_weight_norm_bwd", ptr(v), ptr(g), ptr(norm), ptr(gW), O, v[0].numel(), ptr(gv), ptr(gg), S())


def weight_norm_fwd_batch(layers):
    """[(v, g)] -> [(W, norm)] for every layer in one launch (mg_weight_norm_batch)."""
    outs, descs = [], []
    for v, g in layers:
        O, K = v.shape[0], v[0].numel()
        W = torch.empty_like(v)
        norm = torch.empty(O, device=v.device, dtype=torch.float32)
        outs.append((W, norm))
        descs.append(L.WnDesc(O, K, ptr(v), ptr(g), ptr(norm), ptr(W), None, None, None))
    arr = (L.WnDesc * len(descs))(*descs)
    call("mg_weight_norm_batch", 0, len(descs), arr, S())
    return outs


def weight_norm_bwd_batch(layers):
    """[(v, g, norm, gW, gv, gg)]: gv, gg accumulate every layer's weight-norm backward in one launch."""
    descs = [L.WnDesc(v.shape[0], v[0].numel(), ptr(v), ptr(g), ptr(norm), None, ptr(gW), ptr(gv), ptr(gg))
             for v, g, norm, gW, gv, gg in layers]
    arr = (L.WnDesc * len(descs))(*descs)
    call("mg_weight_norm_batch", 1, len(descs), arr, S())


def sumsq(x, out):
    call("mg_sumsq", ptr(x), x.numel(), ptr(out), S())
    return out


def adamw(p, g, m, v, lr, beta1, beta2, eps, wd, step, sumsq_buf=None, max_norm=0.0):
    call("mg_adamw", ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), lr, beta1, beta2, eps, wd, step, ptr(sumsq_buf),
         max_norm, S())


def opt_prologue(sumsq_buf, step_dev, gate=None):
    """sumsq_buf[0] = 0 (if given); step_dev[0] += 1 (device-side AdamW step counter, graph-replayable) unless
    the gate ``(flags, skip_mask, win, run_mask)`` says the optimizer does not run this step."""
    fl, skip, win, run = gate if gate is not None else (None, 0, None, 0)
    call("mg_opt_prologue", ptr(sumsq_buf), ptr(step_dev), ptr(fl), skip, ptr(win), run, S())


def adamw_dev(p, g, m, v, lr, beta1, beta2, eps, wd, step_dev, sumsq_buf=None, max_norm=0.0, shadow=None,
              gate=None):
    """AdamW with the device step counter and clip coefficient; ``shadow`` (bf16, same length) also receives the
    updated parameters (mg_adamw_dev_shadow); ``gate`` as in opt_prologue."""
    fl, skip, win, run = gate if gate is not None else (None, 0, None, 0)
    call("mg_adamw_dev_shadow", ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), lr, beta1, beta2, eps, wd, ptr(step_dev),
         ptr(sumsq_buf), max_norm, ptr(shadow), ptr(fl), skip, ptr(win), run, S())


# ---------------------------------------------------------------------------
# loss guards (mg_guard.hip): device flag words, no host sync
# ---------------------------------------------------------------------------
FLAG_D_BAD, FLAG_G_BAD = 1, 2
WIN_D, WIN_G_MAIN, WIN_G_KL = 1, 2, 4


def finite_flag(x, bit, flags):
    call("mg_finite_flag", ptr(x), x.numel(), bit, ptr(flags), S())


def flag_window(flags, win, *, reset_bits=0, keep_mask=0, bad_mask=0, set_bits=0):
    """win &= ~reset_bits unless flags & keep_mask; win |= set_bits unless flags & bad_mask."""
    call("mg_flag_window", ptr(flags), reset_bits, keep_mask, bad_mask, set_bits, ptr(win), S())


def guard_update(flags, win=None, checks=(), windows=()):
    """One launch (mg_guard_update) for a phase's loss checks -- ``checks``: (tensor, bit), flags |= bit when the
    tensor is not all finite -- and then its window updates -- ``windows``: dicts of flag_window's keyword
    arguments, applied in order on the updated flags."""
    assert len(checks) <= 4 and len(windows) <= 2
    d = L.GuardDesc()
    for i, (t, bit) in enumerate(checks):
        d.x[i], d.n[i], d.bit[i] = t.data_ptr(), t.numel(), bit
    d.nwin = len(windows)
    for j, w in enumerate(windows):
        d.reset_bits[j], d.keep_mask[j] = w.get("reset_bits", 0), w.get("keep_mask", 0)
        d.bad_mask[j], d.set_bits[j] = w.get("bad_mask", 0), w.get("set_bits", 0)
    call("mg_guard_update", ctypes.byref(d), ptr(flags), ptr(win), S())


def grad_norm_steps(x, out, steps=(), flags=None, skip_mask=0, win=None):
    """out[0] = sum of x^2 (mg_grad_norm_steps, written) and, for each (step counter, run mask) in ``steps`` (at
    most two), the counter advanced under opt_prologue's gate."""
    assert len(steps) <= 2
    st = list(steps) + [(None, 0)] * (2 - len(steps))
    call("mg_grad_norm_steps", ptr(x), x.numel(), ptr(out), ptr(st[0][0]), st[0][1], ptr(st[1][0]), st[1][1],
         ptr(flags), skip_mask, ptr(win), S())


def zero_if(x, flags, mask, when_set=True):
    """x = 0 when (flags & mask) != 0 equals ``when_set``."""
    call("mg_zero_if", ptr(x), x.numel() * x.element_size(), ptr(flags), mask, int(bool(when_set)), S())


def step_inputs(eps_a, eps_b, perm, seed_eps, seed_perm):
    """eps_a, eps_b (fp32) ~ N(0, 1) and perm (int32 [B]) a random permutation, one launch (mg_step_inputs)."""
    call("mg_step_inputs", ptr(eps_a), eps_a.numel(), ptr(eps_b), eps_b.numel(), ptr(perm), perm.numel(),
         ctypes.c_uint64(seed_eps & (2 ** 64 - 1)), ctypes.c_uint64(seed_perm & (2 ** 64 - 1)), S())


def gated_axpy(acc, g, flags, mask):
    call("mg_gated_axpy", ptr(acc), ptr(g), acc.numel(), ptr(flags), mask, S())


def select_if(src, flags, mask, out=None):
    out = torch.empty_like(src) if out is None else out
    call("mg_select_if", ptr(src), src.numel(), ptr(flags), mask, ptr(out), S())
    return out


def const_fwd(cst, B, dtype):
    C, HW = cst.shape[1], cst.shape[2] * cst.shape[3]
    out = torch.empty(B, cst.shape[2], cst.shape[3], C, device=cst.device, dtype=dtype)
    call("mg_const_fwd", dt(out), ptr(cst), C, HW, B, ptr(out), S())
    return out


def const_bwd(g, gcst):
    B, H, W, C = g.shape
    call("mg_const_bwd", dt(g), ptr(g), C, H * W, B, ptr(gcst), S())


# ---------------------------------------------------------------------------
# modulated conv helpers
# ---------------------------------------------------------------------------
def modconv_bwd_out(gz, z, d, B, HW, Cout, act, gyt, gdd, zsub=None, ld_gz=None, ld_z=None, ld_gyt=None):
    call("mg_modconv_bwd_out", dt(z), dt(gz), ptr(gz), ld_gz or gz.shape[-1], ptr(z), ld_z or z.shape[-1],
         ptr(zsub), zsub.shape[-1] if zsub is not None else 0, ptr(d), B, HW, Cout, act, ptr(gyt),
         ld_gyt or gyt.shape[-1], ptr(gdd), S())


def gather_rows(src, idx, idx_div=1, rowscale=None, out=None):
    """out[r] = src[idx[r] // idx_div] * rowscale[r] (mg_gather_rows)."""
    n, C = idx.shape[0], src.shape[-1]
    if out is None:
        out = torch.empty(n, C, device=src.device, dtype=src.dtype)
    call("mg_gather_rows", dt(src), ptr(src), _ld(src), ptr(idx), idx_div, ptr(rowscale), n, C, ptr(out), _ld(out), S())
    return out


def scale_bc(x, s, out=None):
    """xs[b, ..., c] = x[b, ..., c] * s[b, c] for NHWC x [B, H, W, C] (mg_scale_bc)."""
    B, C = x.shape[0], x.shape[-1]
    HW = x.numel() // (B * C)
    if out is None:
        out = torch.empty_like(x)
    call("mg_scale_bc", dt(x), ptr(x), C, ptr(s), s.stride(0), B, HW, C, ptr(out), C, S())
    return out


def modconv_bwd_in(gxt, x, s, B, HW, Cin, gx, gs, accumulate=0):
    """gx (+)= gxt * s; gs += sum_pix gxt * x.  s / gs may be column slices sharing one row pitch."""
    assert s.stride(0) == gs.stride(0) and s.stride(-1) == 1 and gs.stride(-1) == 1
    call("mg_modconv_bwd_in", dt(gxt), ptr(gxt), gxt.shape[-1], dt(x), ptr(x), x.shape[-1], ptr(s), s.stride(0), B, HW,
         Cin, dt(gx) if gx is not None else 0, ptr(gx), gx.shape[-1] if gx is not None else 0, accumulate, ptr(gs),
         S())


# ---------------------------------------------------------------------------
# norm / attention
# ---------------------------------------------------------------------------
def layernorm_fwd(x, gamma, beta, eps=1e-5, act=0, out=None):
    R, C = x.shape[0], x.shape[-1]
    out = torch.empty_like(x) if out is None else out
    mean = torch.empty(R, device=x.device, dtype=torch.float32)
    rstd = torch.empty(R, device=x.device, dtype=torch.float32)
    call("mg_layernorm_fwd", dt(x), ptr(x), x.shape[-1], R, C, ptr(gamma), ptr(beta), eps, ptr(out), out.shape[-1],
         ptr(mean), ptr(rstd), act, S())
    return out, mean, rstd


def layernorm_bwd(gy, x, mean, rstd, gamma, gx, ggamma, gbeta, accumulate=0):
    R, C = x.shape[0], x.shape[-1]
    call("mg_layernorm_bwd", dt(x), dt(gy), ptr(gy), gy.shape[-1], ptr(x), x.shape[-1], R, C, ptr(mean), ptr(rstd),
         ptr(gamma), ptr(gx), gx.shape[-1] if gx is not None else 0, accumulate, ptr(ggamma), ptr(gbeta), S())


def attn_fwd(qkv, B, L, C, heads=8):
    out = torch.empty(B * L, C, device=qkv.device, dtype=qkv.dtype)
    lse = torch.empty(B, heads, L, device=qkv.device, dtype=torch.float32)
    call("mg_attn_fwd", dt(qkv), ptr(qkv), B, L, C, heads, ptr(out), ptr(lse), S())
    return out, lse


def attn_bwd(qkv, out, gout, lse, B, L, C, heads=8):
    gqkv = torch.empty_like(qkv)
    call("mg_attn_bwd", dt(qkv), dt(gout), ptr(qkv), ptr(out), ptr(gout), ptr(lse), B, L, C, heads, ptr(gqkv), S())
    return gqkv


# ---------------------------------------------------------------------------
# router / MoE
# ---------------------------------------------------------------------------
def reparam(mu, rho, eps):
    W = torch.empty_like(mu)
    call("mg_router_reparam", ptr(mu), ptr(rho), ptr(eps), mu.numel(), ptr(W), S())
    return W


def router_fwd(tok, Wfc, Lt, E_, k, HW, temperature, anneal, eval_mode=0):
    T, C = tok.shape
    dev = tok.device
    probs = torch.empty(T, E_, device=dev, dtype=torch.float32)
    zlog = torch.empty(T, E_, device=dev, dtype=torch.float32)
    topi = torch.empty(T, k, device=dev, dtype=torch.int32)
    gate = torch.empty(T, k, device=dev, dtype=torch.float32)
    call("mg_router_fwd", dt(tok), ptr(tok), tok.shape[-1], T, C, ptr(Wfc), ptr(Lt), E_, k, HW, ptr(temperature),
         anneal, eval_mode, ptr(probs), ptr(zlog), ptr(topi), ptr(gate), S())
    return probs, zlog, topi, gate


def moe_dispatch(topi, gate, E_, bm=128):
    T, k = topi.shape
    dev = topi.device
    n = T * k
    ws = torch.empty(((n + 1023) // 1024) * E_, device=dev, dtype=torch.int32)  # per-chunk counts (mg_moe.hip DCH)
    row_off = torch.empty(E_ + 1, device=dev, dtype=torch.int32)
    tile_off = torch.empty(E_ + 1, device=dev, dtype=torch.int32)
    perm = torch.empty(n, device=dev, dtype=torch.int32)
    pos_of = torch.empty(n, device=dev, dtype=torch.int32)
    gate_pos = torch.empty(n, device=dev, dtype=torch.float32)
    call("mg_moe_dispatch", ptr(topi), ptr(gate), T, k, E_, bm, ptr(ws), ptr(row_off), ptr(tile_off), ptr(perm),
         ptr(pos_of), ptr(gate_pos), S())
    return row_off, tile_off, perm, pos_of, gate_pos


def moe_combine(Y, pos_of, gate, resid, out, style=None, HW=None):
    """out = resid + the gated expert rows (mg_moe_combine).  ``style`` [B, C] fp32 (a row view with unit column
    stride) and ``HW`` (tokens per image): also return xs = out * style[image] for the modulated conv that reads out
    (mg_moe_combine_scaled; replaces an mg_scale_bc pass)."""
    T, k = gate.shape
    C = out.shape[-1]
    if style is None:
        call("mg_moe_combine", dt(Y), ptr(Y), Y.shape[-1], ptr(pos_of), ptr(gate), T, k, C, ptr(resid),
             resid.shape[-1] if resid is not None else 0, ptr(out), out.shape[-1], S())
        return out
    assert style.stride(1) == 1 and style.dtype == torch.float32
    xs = torch.empty_like(out)
    call("mg_moe_combine_scaled", dt(Y), ptr(Y), Y.shape[-1], ptr(pos_of), ptr(gate), T, k, C, ptr(resid),
         resid.shape[-1] if resid is not None else 0, ptr(out), out.shape[-1], ptr(style), style.stride(0), HW,
         ptr(xs), xs.shape[-1], S())
    return out, xs


def moe_gate_grad(gout, Y, pos_of, T, k):
    g = torch.empty(T, k, device=Y.device, dtype=torch.float32)
    call("mg_moe_gate_grad", dt(Y), dt(gout), ptr(gout), gout.shape[-1], ptr(Y), Y.shape[-1], ptr(pos_of), T, k,
         Y.shape[-1], ptr(g), S())
    return g


def router_bwd(probs, zlog, topi, gate, g_gate, g_probs, coef, HW, temperature, anneal, g_temp, B, g_logits=None):
    T, E_ = probs.shape
    k = topi.shape[1]
    g_raw = torch.empty(T, E_, device=probs.device, dtype=torch.float32)
    gsum = zeros(B, E_, device=probs.device)
    call("mg_router_bwd", ptr(probs), ptr(zlog), ptr(topi), ptr(gate), ptr(g_gate), ptr(g_probs), ptr(g_logits),
         ptr(coef), T, E_, k, HW, ptr(temperature), anneal, ptr(g_raw), ptr(gsum), ptr(g_temp), S())
    return g_raw, gsum


def moe_token_grad(gX, pos_of, g_raw, Wfc, out, k):
    T, C = out.shape
    E_ = g_raw.shape[1]
    call("mg_moe_token_grad", dt(gX) if gX is not None else dt(out), ptr(gX), gX.shape[-1] if gX is not None else 0,
         ptr(pos_of), T, k, C, ptr(g_raw), ptr(Wfc), E_, dt(out), ptr(out), out.shape[-1], S())
    return out


def router_feat_grad(tok, g_raw, G1):
    T, C = tok.shape
    call("mg_router_feat_grad", dt(tok), ptr(tok), tok.shape[-1], T, C, ptr(g_raw), g_raw.shape[1], ptr(G1), S())
    return G1


def grouped_colsum(X, row_off, N, max_rows, out, idx=None, idx_div=1, rs=None):
    call("mg_grouped_colsum", dt(X), ptr(X), X.shape[-1], ptr(idx), idx_div, ptr(rs), ptr(row_off),
         row_off.shape[0] - 1, N, max_rows, ptr(out), S())
    return out


def router_kl(mf, rf, mt, rt, mc, rc, out):
    call("mg_router_kl", ptr(mf), ptr(rf), mf.numel(), ptr(mt), ptr(rt), mt.numel(), ptr(mc), ptr(rc), mc.numel(),
         ptr(out), S())
    return out


class _KlRec(ctypes.Structure):
    """Mirror of ``mg_kl_rec``."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("mu_f", "rho_f", "mu_t", "rho_t", "mu_c", "rho_c")] + \
               [(n, ctypes.c_int32) for n in ("nf", "nt", "nc", "pad")]


def router_kl_batch(routers, out):
    """KL terms of several routers in two launches: routers = [(mf, rf, mt, rt, mc, rc), ...], out [n, 2]
    (row j as router_kl's out for router j, bit-identical)."""
    for j0 in range(0, len(routers), 8):  # at most 8 records per call
        group = routers[j0:j0 + 8]
        recs = (_KlRec * len(group))()
        for j, (mf, rf, mt, rt, mc, rc) in enumerate(group):
            recs[j] = _KlRec(ptr(mf), ptr(rf), ptr(mt), ptr(rt), ptr(mc), ptr(rc), mf.numel(), mt.numel(), mc.numel(),
                             0)
        call("mg_router_kl_batch", len(group), ctypes.addressof(recs), ptr(out[j0:]), S())
    return out


def kl_coefs(kl2, R, eff_w, coef, total):
    call("mg_kl_coefs", ptr(kl2), R, eff_w, ptr(coef), ptr(total), S())


def router_param_bwd(mu, rho, eps, gW, kl_coef, gmu, grho, flags=None, mask=0):
    call("mg_router_param_bwd", ptr(mu), ptr(rho), ptr(eps), ptr(gW), mu.numel(), ptr(kl_coef), ptr(gmu),
         ptr(grho), ptr(flags), mask, S())


def router_param_bwd_batch(items, flags=None, mask=0):
    """Every router parameter gradient of a backward in one launch (mg_router_param_bwd_batch).  items: tuples
    (mu, rho, eps, gW, kl_coef, gmu, grho) as router_param_bwd takes them."""
    for i in range(0, len(items), 32):
        part = items[i:i + 32]
        arr = (L.RouterParamDesc * len(part))()
        for j, (mu, rho, eps, gW, klc, gmu, grho) in enumerate(part):
            arr[j] = L.RouterParamDesc(ptr(mu), ptr(rho), ptr(eps), ptr(gW), ptr(klc), ptr(gmu), ptr(grho), mu.numel())
        call("mg_router_param_bwd_batch", len(part), arr, ptr(flags), mask, S())


def balance(load, E_, T, weight, grad_scale, out, coef):
    call("mg_balance", ptr(load), E_, float(T), weight, grad_scale, ptr(out), ptr(coef), S())


# ---------------------------------------------------------------------------
# MTM warp / upsample
# ---------------------------------------------------------------------------
def warp_fwd(x, o1, w2, b2, s=None):
    """MTM warp (mg_warp_fwd).  With ``s`` [B, C] (fp32, row stride s.stride(0)) also returns the warped map
    scaled per (image, channel) -- the next modulated conv's input -- from the same pass (mg_warp_fwd_scaled):
    (out, samp) or (out, samp, out_scaled)."""
    B, H, W, C = x.shape
    out = torch.empty_like(x)
    samp = torch.empty(B * H * W, 4, device=x.device, dtype=torch.float32)
    if s is None:
        call("mg_warp_fwd", dt(x), ptr(x), ptr(o1), ptr(w2), ptr(b2), B, H, W, C, ptr(out), ptr(samp), S())
        return out, samp
    xs = torch.empty_like(x)
    call("mg_warp_fwd_scaled", dt(x), ptr(x), ptr(o1), ptr(w2), ptr(b2), B, H, W, C, ptr(s), s.stride(0), ptr(out),
         ptr(xs), ptr(samp), S())
    return out, samp, xs


def warp_bwd(gout, x, samp, gx32, goff):
    B, H, W, C = x.shape
    call("mg_warp_bwd", dt(x), dt(gout), ptr(gout), ptr(x), ptr(samp), B, H, W, C, ptr(gx32), ptr(goff), S())


def mtm_bwd_fused(gout, x, samp, o1, w2, gx, ga1, gw2, gb2, accumulate=0):
    """Per-image fused MTM backward (mg_mtm_bwd_fused): gather-form grid_sample data gradient into gx
    (= or +=, gx's dtype), dL/doffsets in LDS, offset head backward -> ga1, gw2 +=, gb2 +=."""
    B, H, W, C = x.shape
    call("mg_mtm_bwd_fused", dt(x), dt(gout), ptr(gout), ptr(x), ptr(samp), ptr(o1), ptr(w2), B, H, W, C, dt(gx),
         ptr(gx), accumulate, ptr(ga1), ptr(gw2), ptr(gb2), S())


def mtm_bwd_fusable(x):
    B, H, W, C = x.shape
    return (H * W <= 512 and C % 8 == 0 and C <= 512 and (C // 8) & (C // 8 - 1) == 0 and x.is_contiguous()
            and os.environ.get("MOEGAN_MTM_FUSED", "1") != "0")


def offset_head_bwd(goff, o1, w2, ga1, gw2, gb2):
    B, H, W, _ = o1.shape
    call("mg_offset_head_bwd", dt(o1), ptr(goff), ptr(o1), ptr(w2), B, H, W, ptr(ga1), ptr(gw2), ptr(gb2), S())


def upsample2x(x, style=None):
    """nn.Upsample(2, bilinear) NHWC (mg_upsample2x_fwd).  ``style`` [B, C] fp32 (unit column stride): also return
    xs = out * style[b] for the 1x1 skip modulated conv that reads out (mg_upsample2x_fwd_scaled)."""
    B, H, W, C = x.shape
    out = torch.empty(B, 2 * H, 2 * W, C, device=x.device, dtype=x.dtype)
    if style is None:
        call("mg_upsample2x_fwd", dt(x), ptr(x), B, H, W, C, ptr(out), S())
        return out
    assert style.stride(1) == 1 and style.dtype == torch.float32
    xs = torch.empty_like(out)
    call("mg_upsample2x_fwd_scaled", dt(x), ptr(x), B, H, W, C, ptr(out), ptr(style), style.stride(0), ptr(xs), S())
    return out, xs


def upsample2x_bwd(gout, gx, accumulate=0):
    B, H, W, C = gx.shape
    call("mg_upsample2x_bwd", dt(gout), ptr(gout), B, H, W, C, dt(gx), ptr(gx), accumulate, S())
    return gx


# ---------------------------------------------------------------------------
# discriminator / losses
# ---------------------------------------------------------------------------
def d0_fwd(x, strides, B, H, W, w0p, bias=None, aux=None):
    """Discriminator conv_layers.0 (3 -> 128, 4x4/s2/p1) direct (bf16): h0 = LeakyReLU(conv(x) + bias), or with
    ``aux`` = h0 the R1 forward-mode pass conv(x) * LeakyReLU'(h0).  x: image with element strides ``strides``."""
    out = torch.empty(B, H // 2, W // 2, 128, device=x.device, dtype=torch.bfloat16)
    sb, sh, sw, sc = strides
    call("mg_d0_fwd", dt(x), ptr(x), sb, sh, sw, sc, B, H, W, ptr(w0p), ptr(bias), ptr(aux), ptr(out), S())
    return out


def d0_wgrad(x, strides, B, H, W, g, dw):
    """dw [128, 48] fp32 (GEMM layout) += weight gradient of conv_layers.0 for output gradient g [B, H/2, W/2, 128]."""
    sb, sh, sw, sc = strides
    call("mg_d0_wgrad", dt(x), ptr(x), sb, sh, sw, sc, B, H, W, ptr(g), ptr(dw), S())
    return dw


def d0_dgrad(g, w0p, out):
    """Image gradient of conv_layers.0: g [B, OH, OW, 128] bf16 -> out [B, 2OH, 2OW, ldo] (channels < 3)."""
    B, OH, OW, _ = g.shape
    call("mg_d0_dgrad", ptr(g), B, OH, OW, ptr(w0p), dt(out), ptr(out), out.shape[-1], S())
    return out


def im2col_4x4s2(x, strides, B, H, W, C, Kp, dtype):
    out = torch.empty(B * (H // 2) * (W // 2), Kp, device=x.device, dtype=dtype)
    sb, sh, sw, sc = strides
    call("mg_im2col_4x4s2", dt(x), ptr(x), sb, sh, sw, sc, B, H, W, C, Kp, dt(out), ptr(out), S())
    return out


def disc_head_fwd(h1, W2img):
    B, Hf, _, Cf = h1.shape
    out = torch.empty(B, (Hf - 3) * (Hf - 3), device=h1.device, dtype=torch.float32)
    call("mg_disc_head_fwd", dt(h1), ptr(h1), ptr(W2img), B, Hf, Cf, ptr(out), S())
    return out


def d_head_fwd(h1, w2t, B, Hf):
    """Head image part (mg_d_head_fwd, bf16): out [B, (Hf-3)^2] fp32."""
    Ho = Hf - 3
    out = torch.empty(B, Ho * Ho, device=h1.device)
    call("mg_d_head_fwd", ptr(h1), ptr(w2t), B, Hf, ptr(out), S())
    return out


def d_head_bwd(g, g_bstride, h1, w2c, B, Hf, out):
    """g_a1 = LeakyReLU'(h1) * (G W2img^T) with the tap-expanded G formed in the kernel (mg_d_head_bwd, bf16)."""
    call("mg_d_head_bwd", ptr(g), g_bstride, ptr(h1), ptr(w2c), B, Hf, ptr(out), S())
    return out


def disc_head_gmat(g, g_bstride, B, Hf, dtype):
    """Tap-expanded head gradient G [B*Hf*Hf, 16] (mg_disc_head_gmat)."""
    G = torch.empty(B * Hf * Hf, 16, device=g.device, dtype=dtype)
    call("mg_disc_head_gmat", L.MG_F32 if dtype == torch.float32 else L.MG_BF16, ptr(g), g_bstride, B, Hf, ptr(G),
         S())
    return G


def disc_head_sum(P, B, Hf):
    """out[b, oy*Ho + ox] = sum_tap P[b, oy+kh, ox+kw, tap] (mg_disc_head_sum)."""
    Ho = Hf - 3
    out = torch.empty(B, Ho * Ho, device=P.device)
    call("mg_disc_head_sum", ptr(P), B, Hf, ptr(out), S())
    return out


def disc_head_bwd_data(g, g_bstride, W2img, a1, out):
    B, Hf, _, Cf = out.shape
    call("mg_disc_head_bwd_data", dt(a1), ptr(g), g_bstride, ptr(W2img), ptr(a1), B, Hf, Cf, dt(out), ptr(out), S())
    return out


def disc_head_bwd_w(g, g_bstride, h1, dW2):
    B, Hf, _, Cf = h1.shape
    call("mg_disc_head_bwd_w", dt(h1), ptr(g), g_bstride, ptr(h1), B, Hf, Cf, ptr(dW2), S())


def d_text_bwd(g_tb, t, w2sum, cofs, g_tpre, dW2):
    B, Ct = t.shape
    call("mg_d_text_bwd", ptr(g_tb), ptr(t), ptr(w2sum), B, Ct, cofs, ptr(g_tpre), ptr(dW2), S())


def d_loss(img_real, img_fake, tb, perm, out, g_img, g_fake, g_tb, real_out=None, mism_out=None, fake_out=None):
    B, No = img_real.shape
    Nf = img_fake.numel() // B
    call("mg_d_loss", ptr(img_real), ptr(img_fake), ptr(tb), ptr(perm), B, No, Nf, ptr(out), ptr(g_img), ptr(g_fake),
         ptr(g_tb), ptr(real_out), ptr(mism_out), ptr(fake_out), S())


def clip_patches(img, res=224, patch=32):
    """Generator image NHWC [B, R, R, ld] (channels 0..2) -> CLIP ViT patch rows [B*(res/patch)^2, 3*patch*patch] bf16:
    clamp, bilinear resize to res, unfold (mg_clip_patches)."""
    B, R, R2, ld = img.shape
    assert R == R2 and img.is_contiguous()
    g = res // patch
    out = torch.empty(B * g * g, 3 * patch * patch, device=img.device, dtype=torch.bfloat16)
    call("mg_clip_patches", dt(img), ptr(img), B, R, ld, res, patch, ptr(out), S())
    return out


def g_loss(fake, out, g, scale=1.0):
    call("mg_g_loss", ptr(fake), fake.shape[0], scale, ptr(out), ptr(g), S())


def r1(g, B, gamma, r1_out, u):
    per = g.numel() // B
    call("mg_r1", dt(g), ptr(g), per, B, gamma, ptr(r1_out), dt(u) if u is not None else 0, ptr(u), S())


def lrelu_mask_mul(a, m, out):
    call("mg_lrelu_mask_mul", dt(a), ptr(a), dt(m), ptr(m), a.numel(), dt(out), ptr(out), S())
    return out
