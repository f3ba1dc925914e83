"""Thin Python wrappers over the C ABI (tensor plumbing only; all math is in HIP)."""
import math

import torch

from . import _lib as L


def _ld(t):
    return t.stride(0) if t.dim() > 1 else t.shape[0]


def gemm(A, B, M, N, K, *, a_kc=True, b_kc=True, out=None, out_dtype=None, lda=None, ldb=None, ldc=None,
         ep=None, splits=1):
    """C[M,N] = epilogue(op(A) @ op(B)).  See mg_gemm in include/moegan_hip.h."""
    if out is None:
        out = torch.empty(M, N, device=A.device, dtype=out_dtype or A.dtype)
    L.call("mg_gemm", L.dt(A), M, N, K, L.ptr(A), lda if lda is not None else _ld(A), int(a_kc), L.ptr(B),
           ldb if ldb is not None else _ld(B), int(b_kc), L.ptr(out), ldc if ldc is not None else _ld(out),
           L.dt(out), ep, splits, L.stream())
    return out


def linear(x, W, bias=None, act=0, out=None, **epk):
    """y = act(x @ W^T + bias) for x [M,K], W [N,K] (nn.Linear semantics)."""
    M, K = x.shape
    N = W.shape[0]
    ep = L.epilogue(bias=bias, act=act, **epk)
    return gemm(x, W, M, N, K, out=out, ep=ep)


def conv2d(x, wpack, Cout, KH, KW, stride=1, pad=0, in_scale=None, out=None, out_dtype=None, ep=None, ldy=None):
    """NHWC implicit-GEMM conv: x [B,H,W,Cin] -> y [B,OH,OW,Cout] (see mg_conv2d_fwd)."""
    B, H, W, Cin = x.shape
    OH = (H + 2 * pad - KH) // stride + 1
    OW = (W + 2 * pad - KW) // stride + 1
    if out is None:
        out = torch.empty(B, OH, OW, ldy or Cout, device=x.device, dtype=out_dtype or x.dtype)
    L.call("mg_conv2d_fwd", L.dt(x), L.ptr(x), B, H, W, Cin, L.ptr(wpack), Cout, KH, KW, stride, pad,
           L.ptr(in_scale), L.ptr(out), ldy or out.shape[-1], L.dt(out), ep, L.stream())
    return out


def conv2d_wgrad(gy, x, Cout, KH, KW, stride, pad, gw, in_scale=None, ldg=None, splits=0):
    """gw [Cout,Cin,KH,KW] (fp32) += weight gradient (see mg_conv2d_wgrad)."""
    B, H, W, Cin = x.shape
    L.call("mg_conv2d_wgrad", L.dt(x), L.ptr(gy), ldg or gy.shape[-1], L.ptr(x), B, H, W, Cin, L.ptr(in_scale),
           Cout, KH, KW, stride, pad, L.ptr(gw), splits, L.stream())
    return gw


def gemm_grouped(A, B, row_off, tile_off, max_tiles, N, K, *, b_kc=True, b_gstride, out, ep=None, lda=None,
                 ldb=None, ldc=None):
    total_rows = out.shape[0]
    L.call("mg_gemm_grouped", L.dt(A), total_rows, N, K, row_off.shape[0] - 1, L.ptr(row_off), L.ptr(tile_off),
           max_tiles, L.ptr(A), lda or _ld(A), L.ptr(B), ldb or B.shape[-1], int(b_kc), b_gstride, L.ptr(out),
           ldc or _ld(out), L.dt(out), ep, L.stream())
    return out


def gemm_grouped_wgrad(A, B, row_off, total_rows, M, N, out, *, b_idx=None, b_idx_div=1, b_gelu=0, ep=None,
                       lda=None, ldb=None, splits=0):
    """out[g] (fp32 [G,M,N]) += sum over rows of group g of A[r,:]^T B[r,:] (see mg_gemm_grouped_wgrad)."""
    L.call("mg_gemm_grouped_wgrad", L.dt(A), M, N, row_off.shape[0] - 1, L.ptr(row_off), total_rows, L.ptr(A),
           lda or _ld(A), L.ptr(B), ldb or _ld(B), L.ptr(b_idx), b_idx_div, b_gelu, L.ptr(out), splits, ep,
           L.stream())
    return out


def ilog2(v):
    return int(math.log2(v))
