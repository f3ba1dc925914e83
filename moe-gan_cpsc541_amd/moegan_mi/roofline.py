"""Per-family roofline attribution of the training step (bench.py).

Every C-ABI call of one eager step is observed through ``_lib.HOOK``: its algorithmic work is computed from
the call's own shape arguments (FLOPs for the MFMA families, bytes for the HBM-bound ones: each operand
read once, each output written once -- the SURVEY.md §8(d) formulas) and the call is bracketed by HIP events
on the stream it is enqueued on.  A family's achieved rate is its total work over its total event time.

A call's event time includes every kernel that entry point launches (e.g. ``mg_conv2d_wgrad`` = GEMM +
``k_wgrad_fold`` / split-K reduce), so the wgrad family carries its fold.  ``KERNELS`` maps the rocprofv3
kernel names to the same families so the PMC traffic of a ``--pmc`` pass (tools/family_traffic.py) can be
attributed per family too.
"""
import re

import torch

from . import _lib as L

ELT = {0: 4, 1: 2, 2: 4}  # MG_F32, MG_BF16, MG_F32X3 (fp32 storage)
MX8_PEAK_TFLOPS = 5000.0  # dense MX-fp8 MFMA peak (MI355X_MICROARCH.md: 2x the bf16 rate per clock)

# family -> (bound, entry points)
FAMILIES = {
    "conv_fwd": ("mfma", ("mg_conv2d_fwd",)),
    "conv_fwd_mx8": ("mfma8", ("mg_conv2d_fwd_mx8",)),  # MX-fp8 (C5): priced against the fp8 MFMA peak
    "conv_dgrad_s2": ("mfma", ("mg_conv2d_dgrad_s2",)),
    "conv_wgrad+fold": ("mfma", ("mg_conv2d_wgrad",)),
    "expert_gemm": ("mfma", ("mg_gemm_grouped", "mg_gemm_grouped_wgrad", "mg_moe_ffn_fwd", "mg_moe_ffn_bwd")),
    "gemm": ("mfma", ("mg_gemm", "mg_gemm_batch")),
    "attention": ("mfma", ("mg_attn_fwd", "mg_attn_bwd")),
    "router_fwd": ("hbm", ("mg_router_fwd",)),
    "dispatch_combine": ("hbm", ("mg_gather_rows", "mg_moe_combine")),
    "warp_fwd": ("hbm", ("mg_warp_fwd", "mg_warp_fwd_scaled")),
    "mtm_bwd": ("hbm", ("mg_mtm_bwd_fused",)),
    "modconv_bwd_io": ("hbm", ("mg_modconv_bwd_in", "mg_modconv_bwd_out", "mg_scale_bc")),
    "r1": ("hbm", ("mg_r1",)),
    "sumsq": ("hbm", ("mg_sumsq", "mg_grad_norm_steps")),
    "adamw": ("hbm", ("mg_adamw_dev", "mg_adamw_dev_shadow", "mg_adamw")),
    "bias_colsum": ("hbm", ("mg_colsum", "mg_grouped_colsum", "mg_colsum_batch", "mg_segsum", "mg_const_bwd")),
    "weight_prep": ("hbm", ("mg_pack_conv", "mg_pack_conv_flip", "mg_pack_dgrad_s2", "mg_wsq", "mg_wsq_bwd",
                            "mg_router_reparam", "mg_weight_norm_fwd", "mg_weight_norm_bwd", "mg_weight_norm_batch",
                            "mg_quant_mx8",
                            "mg_prep_batch")),
    "layernorm": ("hbm", ("mg_layernorm_fwd", "mg_layernorm_bwd")),
    "router_aux": ("hbm", ("mg_router_bwd", "mg_moe_gate_grad", "mg_moe_token_grad", "mg_router_feat_grad",
                           "mg_router_param_bwd", "mg_router_param_bwd_batch", "mg_moe_dispatch", "mg_router_kl",
                           "mg_router_kl_batch")),
    "im2col_col2im": ("hbm", ("mg_im2col_4x4s2", "mg_col2im_4x4s2")),
    # deferred second passes of the two-pass gradient reductions (mg_fold.hip), one batched launch per kind
    "grad_fold": ("hbm", ("mg_fold_flush", "mg_fold_rows_batch", "mg_fold_rows_queue", "mg_fold_defer")),
    "d_conv0": ("hbm", ("mg_d0_fwd", "mg_d0_wgrad", "mg_d0_dgrad")),
    "elementwise": ("hbm", ("mg_cast", "mg_copy2d", "mg_lrelu_mask_mul", "mg_upsample2x_fwd", "mg_upsample2x_bwd",
                            "mg_const_fwd", "mg_gated_axpy", "mg_select_if", "mg_zero_if", "mg_clip_patches")),
    "disc_head": ("hbm", ("mg_disc_head_fwd", "mg_disc_head_gmat", "mg_disc_head_sum", "mg_disc_head_bwd_data",
                          "mg_d_head_fwd", "mg_d_head_bwd",
                          "mg_disc_head_bwd_w", "mg_d_text_bwd")),
    "mtm_bwd_unfused": ("hbm", ("mg_warp_bwd", "mg_offset_head_bwd")),
    # scalar losses, guard words, optimizer prologue: a few hundred bytes each, launch-latency bound
    "losses_flags": ("hbm", ("mg_d_loss", "mg_g_loss", "mg_finite_flag", "mg_flag_window", "mg_kl_coefs", "mg_balance",
                             "mg_opt_prologue", "mg_guard_update")),
}
_FAMILY_OF = {e: f for f, (_, es) in FAMILIES.items() for e in es}

# rocprofv3 kernel name (regex, first match wins) -> family, for PMC attribution
KERNELS = [
    (r"k_fold_wgrad_batch|k_fold_rows_batch", "grad_fold"),
    (r"k_wgrad_fold|splitk_reduce_kernel<mg::Epi<float>|k_wgrad3_direct", "conv_wgrad+fold"),
    (r"k_conv3_direct", "conv_fwd"),
    (r"k_mx8_conv", "conv_fwd_mx8"),
    # TAG = 1 instantiations (mg_gemm.h: "..., TAG, X3>("), fused FFN
    (r"gemm_kernel<.*, 1(, (true|false))?>\(|k_moe_ffn_fwd|k_moe_ffn_bwd|k_ffn_bias_fold", "expert_gemm"),
    (r"gemm_kernel<[^>]*LdKCConvT", "conv_dgrad_s2"),
    (r"gemm_kernel<.*LdMCConv", "conv_wgrad+fold"),
    (r"gemm_kernel<.*LdKCConv", "conv_fwd"),
    (r"gemm_kernel<|gemm_batch_kernel<|splitk_reduce_kernel", "gemm"),
    (r"k_attn_", "attention"),
    (r"k_router_fwd", "router_fwd"),
    (r"k_gather_rows|k_combine", "dispatch_combine"),
    (r"k_warp_fwd", "warp_fwd"),
    (r"k_mtm_bwd", "mtm_bwd"),
    (r"k_bwd_in|k_bwd_out|k_scale_bc", "modconv_bwd_io"),
    (r"k_r1", "r1"),
    (r"k_sumsq", "sumsq"),
    (r"k_adamw", "adamw"),
    (r"k_colsum|k_grouped_colsum|k_segsum|k_const_bwd", "bias_colsum"),
    (r"k_pack_|k_wsq|k_reparam|k_wn_|k_quant_mx8|k_prep_batch", "weight_prep"),
    (r"k_ln_|k_layernorm", "layernorm"),
    (r"k_router_bwd|k_fold_partials|k_gate_grad|k_token_grad|k_router_feat_grad|k_feat_grad_fin|k_router_param_bwd|"
     r"k_disp_|k_router_kl", "router_aux"),
    (r"k_im2col|k_col2im", "im2col_col2im"),
    (r"k_d0_|k_fold_cols", "d_conv0"),
    (r"k_wgrad_wide|k_wide_fold|k_wide_final", "gemm"),
    (r"k_cast|k_copy2d|k_mask_mul|k_up2|k_const_fwd|k_gated_axpy|k_select_if|k_zero_if|k_clip_patches",
     "elementwise"),
    (r"k_head_|k_d_text|k_dhead_", "disc_head"),
    (r"k_warp_bwd|k_offset_head", "mtm_bwd_unfused"),
    (r"k_d_loss|k_g_loss|k_finite_flag|k_flag_window|k_guard_update|k_kl_coefs|k_balance|k_opt_prologue",
     "losses_flags"),
]


def kernel_family(kernel_name):
    for pat, fam in KERNELS:
        if re.search(pat, kernel_name):
            return fam
    return "other"


def _conv_out(H, W, KH, KW, s, p):
    return (H + 2 * p - KH) // s + 1, (W + 2 * p - KW) // s + 1


def work(name, a):
    """Algorithmic work of one call: FLOPs (MFMA families) or bytes (HBM families); None = not modelled."""
    if name in ("mg_conv2d_fwd", "mg_conv2d_wgrad", "mg_conv2d_fwd_mx8"):
        OH, OW = _conv_out(a["H"], a["W"], a["KH"], a["KW"], a["stride"], a["pad"])
        return 2.0 * a["B"] * OH * OW * a["Cout"] * a["KH"] * a["KW"] * a["Cin"]
    if name == "mg_conv2d_dgrad_s2":  # 4x4 stride-2 transpose: every input pixel takes 4 of the 16 taps
        return 2.0 * a["B"] * (2 * a["OH"]) * (2 * a["OW"]) * a["Cin"] * a["Cg"] * 4
    if name == "mg_gemm":
        return 2.0 * a["M"] * a["N"] * a["K"]
    if name == "mg_gemm_batch":
        d = a["descs"]
        return sum(2.0 * d[i].M * d[i].N * d[i].K for i in range(a["n"]))
    if name == "mg_gemm_grouped":
        return 2.0 * a["total_rows"] * a["N"] * a["K"]
    if name == "mg_gemm_grouped_wgrad":
        return 2.0 * a["M"] * a["N"] * a["total_rows"]
    if name == "mg_moe_ffn_fwd":  # two GEMMs per routed row
        return 4.0 * a["total_rows"] * a["C"] * a["Hd"]
    if name == "mg_moe_ffn_bwd":  # gH = gG W2 and gX = gP W1 per routed row
        return 4.0 * a["total_rows"] * a["C"] * a["Hd"]
    if name == "mg_attn_fwd":  # S = QK^T, O = PV
        return 4.0 * a["B"] * a["L"] * a["L"] * a["C"]
    if name == "mg_attn_bwd":  # dV, dP, dQ, dK (the S recompute is not algorithmic work)
        return 8.0 * a["B"] * a["L"] * a["L"] * a["C"]
    if name == "mg_router_fwd":
        T, C, E, k = a["T"], a["C"], a["E"], a["k"]
        return T * C * ELT[a["dtype"]] + E * C * 4 + T * E * 8 + T * k * 8
    if name == "mg_gather_rows":
        return 2.0 * a["n"] * a["C"] * ELT[a["dtype"]]
    if name == "mg_moe_combine":
        e = ELT[a["dtype"]]
        return (a["T"] * a["k"] + 2 * a["T"]) * a["C"] * e
    if name in ("mg_warp_fwd", "mg_warp_fwd_scaled"):
        P, C, e = a["B"] * a["H"] * a["W"], a["C"], ELT[a["dtype"]]
        outs = 2 if name == "mg_warp_fwd_scaled" else 1
        return P * (C * e * (1 + outs) + 32 * e + 16)
    if name == "mg_mtm_bwd_fused":
        P, C, e = a["B"] * a["H"] * a["W"], a["C"], ELT[a["dtype"]]
        gx = C * ELT[a["gx_dtype"]] * (2 if a["accumulate"] else 1)
        return P * (C * ELT[a["gout_dtype"]] + C * e + 16 + 32 * e * 2 + gx)
    if name == "mg_scale_bc":
        return 2.0 * a["B"] * a["HW"] * a["C"] * ELT[a["dtype"]]
    if name == "mg_modconv_bwd_in":
        n = a["B"] * a["HW"] * a["Cin"]
        gx = ELT[a["gx_dtype"]] * (2 if a["accumulate"] else 1)
        return n * (ELT[a["gxt_dtype"]] + ELT[a["dtype"]] + gx)
    if name == "mg_modconv_bwd_out":
        n = a["B"] * a["HW"] * a["Cout"]
        e = ELT[a["dtype"]]
        return n * (ELT[a["gz_dtype"]] + e + (e if a["zsub"] else 0) + e)
    if name == "mg_r1":
        return a["B"] * a["per"] * (ELT[a["dtype"]] + ELT[a["u_dtype"]])
    if name == "mg_sumsq":
        return 4.0 * a["n"]
    if name in ("mg_adamw_dev", "mg_adamw"):
        return 28.0 * a["n"]
    if name == "mg_adamw_dev_shadow":
        return (28.0 + (2 if a["shadow_bf16"] else 0)) * a["n"]
    if name in ("mg_pack_conv", "mg_pack_conv_flip"):
        K = a["KH"] * a["KW"]
        return a["Cout"] * a["Cin"] * K * 4 + (a["rows"] * a["Cin"] if name == "mg_pack_conv" else
                                                a["rows"] * a["Cout"]) * K * ELT[a["dtype"]]
    if name == "mg_pack_dgrad_s2":
        return a["Cg"] * a["Cin"] * 16 * 4 + 16 * a["rows"] * a["Cg"] * ELT[a["dtype"]]
    if name == "mg_wsq":
        return a["Cout"] * a["Cin"] * a["taps"] * 4 + a["rows"] * a["Cin"] * 4
    if name == "mg_wsq_bwd":
        return a["Cout"] * a["Cin"] * (a["taps"] * 12 + 4)
    if name == "mg_router_reparam":
        return 16.0 * a["n"]
    if name == "mg_weight_norm_fwd":
        return 8.0 * a["O"] * a["K"]
    if name == "mg_weight_norm_bwd":
        return 16.0 * a["O"] * a["K"]
    if name == "mg_weight_norm_batch":  # per descriptor, the single-layer formulas above
        d = a["descs"]
        return sum((16.0 if a["bwd"] else 8.0) * d[i].O * d[i].K for i in range(a["n"]))
    if name == "mg_colsum":
        return a["R"] * a["C"] * ELT[a["dtype"]] + a["C"] * 8
    if name == "mg_grouped_colsum":  # max_rows = the routed rows (T * k) the engine passes; rs: one fp32 per row
        return a["max_rows"] * (a["N"] * ELT[a["dtype"]] + (4 if a["rs"] else 0) + 4) + a["G"] * a["N"] * 8
    if name == "mg_colsum_batch":
        d = a["descs"]
        return sum(d[i].R * d[i].C * ELT[d[i].dtype] + d[i].C * 8 for i in range(a["n"]))
    if name == "mg_segsum":
        return a["B"] * a["HW"] * a["C"] * ELT[a["dtype"]] + a["B"] * a["C"] * 8
    if name == "mg_const_bwd":
        return a["B"] * a["HW"] * a["C"] * ELT[a["dtype"]] + a["HW"] * a["C"] * 8
    if name == "mg_const_fwd":
        return a["HW"] * a["C"] * 4 + a["B"] * a["HW"] * a["C"] * ELT[a["dtype"]]
    if name == "mg_prep_batch":  # per descriptor, the formulas of the single-tensor entry points
        d, tot = a["descs"], 0.0
        for i in range(a["n"]):
            q = d[i]
            kk = q.KH * q.KW
            if q.kind == 1:
                tot += q.Cout * q.Cin * kk * 4 + q.rows * q.Cin * kk * ELT[a["dtype"]]
            elif q.kind == 2:
                tot += q.Cout * q.Cin * kk * 4 + q.rows * q.Cout * kk * ELT[a["dtype"]]
            elif q.kind == 3:
                tot += q.Cout * q.Cin * 16 * 4 + 16 * q.rows * q.Cout * ELT[a["dtype"]]
            elif q.kind == 4:
                tot += q.Cout * q.Cin * kk * 4 + q.rows * q.Cin * 4
            elif q.kind == 5:
                tot += q.Cout * q.Cin * (kk * 12 + 4)
            elif q.kind == 6:
                tot += 16.0 * q.n
        return tot
    if name == "mg_layernorm_fwd":
        e = ELT[a["dtype"]]
        return a["R"] * a["C"] * 2 * e + a["R"] * 8 + a["C"] * 8
    if name == "mg_layernorm_bwd":
        gx = ELT[a["dtype"]] * (2 if a["accumulate"] else 1)
        return a["R"] * (a["C"] * (ELT[a["gy_dtype"]] + ELT[a["dtype"]] + gx) + 8) + a["C"] * 16
    if name == "mg_router_bwd":
        T, E, k = a["T"], a["E"], a["k"]
        return T * E * 12 + T * k * 12 + (T * E * 4 if a["g_probs"] else 0) + (T * E * 4 if a["g_logits"] else 0)
    if name == "mg_moe_gate_grad":  # every routed row of Y and its token's gradient row once
        T, k, C = a["T"], a["k"], a["C"]
        return T * k * (C * ELT[a["dtype"]] + 8) + T * C * ELT[a["gout_dtype"]]
    if name == "mg_moe_token_grad":
        T, k, C, E = a["T"], a["k"], a["C"], a["E"]
        gx = T * k * (C * ELT[a["dtype"]] + 4) if a["gX"] else 0
        return gx + T * E * 4 + C * E * 4 + T * C * ELT[a["out_dtype"]]
    if name == "mg_router_feat_grad":
        return a["T"] * (a["C"] * ELT[a["dtype"]] + a["E"] * 4) + a["C"] * a["E"] * 8
    if name == "mg_router_param_bwd":  # mu, rho, eps, gW read; gmu, grho read-modify-write
        return 32.0 * a["n"]
    if name == "mg_moe_dispatch":  # topi + gate in; row_off / perm / pos_of / gate_pos out
        return a["T"] * a["k"] * 20.0
    if name == "mg_router_kl":
        return 8.0 * (a["nf"] + a["nt"] + a["nc"])
    if name == "mg_im2col_4x4s2":
        B, H, W = a["B"], a["H"], a["W"]
        return B * H * W * a["C"] * ELT[a["in_dtype"]] + B * (H // 2) * (W // 2) * a["Kp"] * ELT[a["out_dtype"]]
    if name == "mg_col2im_4x4s2":
        B, OH, OW, C = a["B"], a["OH"], a["OW"], a["C"]
        return B * OH * OW * 16 * C * ELT[a["in_dtype"]] + B * 4 * OH * OW * C * ELT[a["out_dtype"]]
    if name in ("mg_d0_fwd", "mg_d0_wgrad"):  # image read + the 128-channel bf16 map (out / aux / gradient)
        B, H, W = a["B"], a["H"], a["W"]
        maps = 1 + (1 if name == "mg_d0_fwd" and a["aux"] else 0)
        return B * H * W * 3 * ELT[a["in_dtype"]] + maps * B * (H // 2) * (W // 2) * 128 * 2
    if name == "mg_d0_dgrad":
        B, OH, OW = a["B"], a["OH"], a["OW"]
        return B * OH * OW * 128 * 2 + B * 4 * OH * OW * 3 * ELT[a["out_dtype"]]
    if name == "mg_d_head_fwd":  # h1 read, logits written
        return a["B"] * a["Hf"] ** 2 * 256 * 2 + a["B"] * (a["Hf"] - 3) ** 2 * 4
    if name == "mg_d_head_bwd":  # h1 (LeakyReLU' operand) read, g_a1 written
        return 2 * a["B"] * a["Hf"] ** 2 * 256 * 2
    if name == "mg_cast":
        return a["n"] * (ELT[a["in_dtype"]] + ELT[a["out_dtype"]])
    if name == "mg_copy2d":
        return a["R"] * a["C"] * (ELT[a["in_dtype"]] + ELT[a["out_dtype"]] * (2 if a["accumulate"] else 1))
    if name == "mg_lrelu_mask_mul":
        return a["n"] * (ELT[a["a_dtype"]] + ELT[a["m_dtype"]] + ELT[a["out_dtype"]])
    if name == "mg_upsample2x_fwd":
        return a["B"] * a["H"] * a["W"] * a["C"] * ELT[a["dtype"]] * 5
    if name == "mg_upsample2x_bwd":
        n = a["B"] * a["H"] * a["W"] * a["C"]
        return n * 4 * ELT[a["gout_dtype"]] + n * ELT[a["gx_dtype"]] * (2 if a["accumulate"] else 1)
    if name == "mg_gated_axpy":
        return 12.0 * a["n"]
    if name == "mg_select_if":
        return 8.0 * a["n"]
    if name == "mg_zero_if":
        return float(a["bytes"])
    if name == "mg_clip_patches":  # the 3 image channels in, bf16 patch rows out
        B, R, res = a["B"], a["R"], a["res"]
        return B * R * R * 3 * ELT[a["dtype"]] + B * res * res * 3 * 2
    if name == "mg_disc_head_fwd":
        return a["B"] * a["Hf"] * a["Hf"] * a["Cf"] * ELT[a["dtype"]] + a["B"] * (a["Hf"] - 3) ** 2 * 4
    if name == "mg_disc_head_gmat":
        return a["B"] * (a["Hf"] - 3) ** 2 * 4 + a["B"] * a["Hf"] * a["Hf"] * 16 * ELT[a["out_dtype"]]
    if name == "mg_disc_head_sum":
        return a["B"] * a["Hf"] * a["Hf"] * 16 * 4 + a["B"] * (a["Hf"] - 3) ** 2 * 4
    if name == "mg_disc_head_bwd_data":
        n = a["B"] * a["Hf"] * a["Hf"] * a["Cf"]
        return n * (ELT[a["dtype"]] + ELT[a["out_dtype"]]) + a["B"] * (a["Hf"] - 3) ** 2 * 4
    if name == "mg_disc_head_bwd_w":
        return a["B"] * a["Hf"] * a["Hf"] * a["Cf"] * ELT[a["dtype"]] + a["B"] * (a["Hf"] - 3) ** 2 * 4
    if name == "mg_d_text_bwd":
        return a["B"] * a["Ct"] * 12.0
    if name == "mg_warp_bwd":
        P, C = a["B"] * a["H"] * a["W"], a["C"]
        return P * (C * (ELT[a["gout_dtype"]] + ELT[a["dtype"]] + 8) + 16 + 8)
    if name == "mg_offset_head_bwd":
        P = a["B"] * a["H"] * a["W"]
        return P * (8 + 32 * ELT[a["dtype"]] * 2)
    if name == "mg_d_loss":
        B = a["B"]
        return B * (a["No"] * 2 + a["Nf"]) * 8.0 + B * 8
    if name == "mg_g_loss":
        return a["B"] * 8.0
    if name == "mg_finite_flag":
        return 4.0 * a["n"]
    if name == "mg_kl_coefs":
        return 8.0 * a["R"]
    if name == "mg_balance":
        return 8.0 * a["E"]
    if name in ("mg_flag_window", "mg_opt_prologue", "mg_guard_update"):
        return 16.0
    if name == "mg_grad_norm_steps":
        return 4.0 * a["n"]
    if name == "mg_router_param_bwd_batch":
        d = a["descs"]
        return sum(32.0 * d[i].n for i in range(a["n"]))
    if name == "mg_quant_mx8":  # bf16 in, e4m3 + one E8M0 byte per 32 out
        return a["rows"] * a["K"] * (2 + 1 + 1 / 32)
    return None


def alg_bytes(name, a):
    """Compulsory HBM bytes of one MFMA-family call (each operand read once, each output written once); None where
    not modelled.  Beside work(): an MFMA call's roofline is FLOPs, its traffic is judged against these bytes."""
    if name == "mg_conv2d_fwd":
        OH, OW = _conv_out(a["H"], a["W"], a["KH"], a["KW"], a["stride"], a["pad"])
        e = ELT[a["dtype"]]
        return (a["B"] * a["H"] * a["W"] * a["Cin"] * e + a["Cout"] * a["KH"] * a["KW"] * a["Cin"] * e +
                a["B"] * OH * OW * a["Cout"] * ELT[a["y_dtype"]])
    if name == "mg_conv2d_wgrad":
        OH, OW = _conv_out(a["H"], a["W"], a["KH"], a["KW"], a["stride"], a["pad"])
        e = ELT[a["dtype"]]
        return (a["B"] * OH * OW * a["Cout"] * e + a["B"] * a["H"] * a["W"] * a["Cin"] * e +
                a["Cout"] * a["Cin"] * a["KH"] * a["KW"] * 4)
    if name == "mg_gemm":
        e = ELT[a["dtype"]]
        return (a["M"] * a["K"] + a["K"] * a["N"]) * e + a["M"] * a["N"] * ELT[a["c_dtype"]]
    if name == "mg_gemm_grouped":
        e = ELT[a["dtype"]]
        return (a["total_rows"] * a["K"] + a["ngroups"] * a["N"] * a["K"]) * e + a["total_rows"] * a["N"] * ELT[a["c_dtype"]]
    if name == "mg_moe_ffn_bwd":  # gG and gX (C), pre and gP (Hd) per routed row, bf16
        return a["total_rows"] * (2 * a["C"] + 2 * a["Hd"]) * 2
    if name == "mg_moe_ffn_fwd":
        return a["total_rows"] * 2 * a["C"] * 2
    return None


class Attribution:
    """Install with ``with Attribution() as at: run_step()``; then ``at.summary(steps=1)``.

    The eager step is host-bound (Python enqueues each call), so events around a call would also time the
    host's launch latency.  ``__enter__`` therefore first parks the stream on a spin kernel of ``lead_ms``
    (longer than the host needs to enqueue the whole step): the calls then run back to back behind it and each
    event pair brackets only its own kernels.  ``host_bound`` reports whether the GPU caught up with the host
    anyway (the lead was too short), which would inflate the small families."""

    def __init__(self, lead_ms=150.0, keep_args=False):
        self.calls = []  # (entry point, family, work, start event, end event)
        self.sigs = []  # _lib.scalar_signature of each call
        self.keep_args = keep_args
        self.args = []  # scalar arguments per call (keep_args)
        self.lead_ms = lead_ms
        self.host_bound = None

    def _hook(self, name, args, run):
        names = L.ARGNAMES.get(name)
        a = {}
        if names:
            for n, v in zip(names, args):
                a[n] = v.value if hasattr(v, "value") and not isinstance(v, L.ctypes.Array) else v
        try:
            w = work(name, a)
        except (KeyError, TypeError, AttributeError):
            w = None
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        rc = run()
        e.record()
        self.calls.append((name, _FAMILY_OF.get(name, "other"), w, s, e))
        self.sigs.append(L.scalar_signature(name, args))
        if self.keep_args:
            self.args.append({k: v for k, v in a.items() if isinstance(v, (int, float))})
        return rc

    def __enter__(self):
        assert L.HOOK is None, "nested attribution"
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        torch.cuda._sleep(2_000_000)
        e.record()
        e.synchronize()
        cyc_per_ms = 2_000_000 / max(s.elapsed_time(e), 1e-3)
        torch.cuda._sleep(int(self.lead_ms * cyc_per_ms))
        L.HOOK = self._hook
        return self

    def __exit__(self, *exc):
        L.HOOK = None
        if self.calls:
            self.host_bound = bool(self.calls[0][3].query())  # first call already ran: the GPU caught up

    def top_calls(self, family=None, n=30):
        """The n slowest calls (of one family), with their scalar shape arguments (needs keep_args)."""
        torch.cuda.synchronize()
        rows = []
        for i, (name, f, w, s, e) in enumerate(self.calls):
            if family is None or f == family:
                ms = s.elapsed_time(e)
                rows.append((ms, name, w, self.args[i] if self.keep_args else {}))
        return sorted(rows, key=lambda r: -r[0])[:n]

    def largest_call(self, family, steps=1):
        """The call signature of ``family`` with the most event time per launch (the family's largest kernel):
        dict(signature, entry, launches_per_step, ms_per_launch, work_per_launch, args {name: value})."""
        torch.cuda.synchronize()
        groups = {}
        for i, (name, f, w, s, e) in enumerate(self.calls):
            if f != family:
                continue
            g = groups.setdefault(self.sigs[i], {"ms": 0.0, "n": 0, "work": w, "i": i})
            g["ms"] += s.elapsed_time(e)
            g["n"] += 1
        if not groups:
            return None
        # the largest kernel: the most time per launch (its share per step is reported beside it); a per-step
        # total would let a cheap call repeated many times win, and flip between near-equal totals run to run
        sig, g = max(groups.items(), key=lambda kv: (kv[1]["ms"] / kv[1]["n"], kv[1]["ms"]))
        name = sig[0]
        types = L._SIGS[name][1]
        scal = [n for n, t in zip(L.ARGNAMES[name], types) if t in (L._i32, L._i64, L._f32)]
        args = dict(zip(scal, sig[1]))
        try:
            nbytes = alg_bytes(name, args)
        except KeyError:
            nbytes = None
        return {"signature": sig, "entry": name, "launches_per_step": g["n"] / steps, "ms_per_launch": g["ms"] / g["n"],
                "work_per_launch": g["work"], "bytes_per_launch": nbytes, "args": args}

    def summary(self, steps=1, peak_tflops=2500.0, peak_gbs=8000.0):
        torch.cuda.synchronize()
        if self.host_bound:
            import warnings
            warnings.warn("roofline attribution: the GPU caught up with the host; small families are inflated")
        fam = {}
        for name, f, w, s, e in self.calls:
            r = fam.setdefault(f, {"calls": 0, "ms": 0.0, "work": 0.0, "entry_points": set()})
            r["calls"] += 1
            r["ms"] += s.elapsed_time(e)
            r["work"] += w or 0.0
            r["entry_points"].add(name)
        out = []
        for f, r in sorted(fam.items(), key=lambda kv: -kv[1]["ms"]):
            bound = FAMILIES[f][0] if f in FAMILIES else None
            ms = r["ms"] / steps
            rec = {"family": f, "bound": bound, "launches_per_step": r["calls"] / steps, "ms_per_step": round(ms, 4)}
            if bound in ("mfma", "mfma8"):
                pk = MX8_PEAK_TFLOPS if bound == "mfma8" else peak_tflops
                tf = r["work"] / steps / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
                rec.update({"bound": "mfma", "gflop_per_step": round(r["work"] / steps / 1e9, 3),
                            "achieved": round(tf, 1), "unit": "TFLOP/s", "peak": pk, "frac": round(tf / pk, 4)})
            elif bound == "hbm":
                gbs = r["work"] / steps / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
                rec.update({"mb_per_step": round(r["work"] / steps / 1e6, 3), "achieved": round(gbs, 1),
                            "unit": "GB/s", "peak": peak_gbs, "frac": round(gbs / peak_gbs, 4)})
            else:
                rec["entry_points"] = sorted(r["entry_points"])[:12]
            out.append(rec)
        return out
