"""Time the GEMM-core launches that dominate the C2 training step, in one process.

  python tools/gemm_probe.py [--iters 20] [--only NAME,...]

Shapes are the bench workload's (B=256, bf16, E=8 top-2); each line prints the median launch
time and the algorithmic TFLOP/s.  Used to A/B GEMM-core changes with a single GPU call.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "moe-gan_cpsc541_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--variants", default="", help="';'-separated tuning sets, e.g. '0=64;0=128'")
    a = ap.parse_args()
    from moegan_mi import _lib as L
    from moegan_mi import ops
    dev = "cuda"
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)

    def rn(*s, dt=torch.float32, sc=1.0):
        return (torch.randn(*s, device=dev, generator=g) * sc).to(dt)

    B = 256
    cases = []
    # D conv_layers.2 forward (roofline kernel)
    h0 = rn(B, 32, 32, 128, dt=bf)
    w1 = ops.pack_conv(rn(256, 128, 4, 4, sc=0.02), bf)
    cases.append(("d_conv1_fwd", 2.0 * B * 256 * 256 * 2048,
                  lambda: ops.conv2d(h0, w1, 256, 4, 4, 2, 1, ep=ops.E(act=L.ACT_LRELU))))
    # modulated 3x3 convs (gen_block_16 / gen_block_8 MTM)
    x16 = rn(B, 16, 16, 128, dt=bf)
    s16 = rn(B, 128) + 1
    w16 = ops.pack_conv(rn(128, 128, 3, 3, sc=0.03), bf)
    cases.append(("modconv16_fwd", 2.0 * B * 256 * 128 * 1152,
                  lambda: ops.conv2d(x16, w16, 128, 3, 3, 1, 1, in_scale=s16)))
    x8 = rn(B, 8, 8, 256, dt=bf)
    s8 = rn(B, 256) + 1
    w8 = ops.pack_conv(rn(256, 256, 3, 3, sc=0.02), bf)
    cases.append(("modconv8_fwd", 2.0 * B * 64 * 256 * 2304, lambda: ops.conv2d(x8, w8, 256, 3, 3, 1, 1, in_scale=s8)))
    # plain (prescaled-input) 3x3 convs at 8x8 and 4x4
    x8p = rn(B, 8, 8, 256, dt=bf)
    cases.append(("conv8_fwd", 2.0 * B * 64 * 256 * 2304, lambda: ops.conv2d(x8p, w8, 256, 3, 3, 1, 1)))
    x4p = rn(B, 4, 4, 512, dt=bf)
    w4 = ops.pack_conv(rn(512, 512, 3, 3, sc=0.02), bf)
    cases.append(("conv4_fwd", 2.0 * B * 16 * 512 * 4608, lambda: ops.conv2d(x4p, w4, 512, 3, 3, 1, 1)))
    x16p = rn(B, 16, 16, 128, dt=bf)
    cases.append(("conv16_fwd", 2.0 * B * 256 * 128 * 1152, lambda: ops.conv2d(x16p, w16, 128, 3, 3, 1, 1)))
    woff = ops.pack_conv(rn(32, 128, 3, 3, sc=0.03), bf)
    cases.append(("offset_head16_fwd", 2.0 * B * 256 * 32 * 1152,
                  lambda: ops.conv2d(x16p, woff, 32, 3, 3, 1, 1, ep=ops.E(act=L.ACT_LRELU))))
    # weight gradients
    gy16 = rn(B * 256, 128, dt=bf)
    gw16 = torch.zeros(128, 128, 3, 3, device=dev)
    cases.append(("modconv16_wgrad", 2.0 * B * 256 * 128 * 1152,
                  lambda: ops.conv2d_wgrad(gy16, x16, 128, 3, 3, 1, 1, gw16)))
    gy8 = rn(B * 64, 256, dt=bf)
    x8b = rn(B, 8, 8, 512, dt=bf)
    gw8 = torch.zeros(256, 512, 3, 3, device=dev)
    cases.append(("modconv8_wgrad", 2.0 * B * 64 * 256 * 4608,
                  lambda: ops.conv2d_wgrad(gy8, x8b, 256, 3, 3, 1, 1, gw8)))
    gy1 = rn(B, 16, 16, 256, dt=bf)
    gw1 = torch.zeros(256, 128, 4, 4, device=dev)
    cases.append(("d_conv1_wgrad", 2.0 * B * 256 * 256 * 2048,
                  lambda: ops.conv2d_wgrad(gy1, h0, 256, 4, 4, 2, 1, gw1)))
    # 1x1 conv weight gradients (attention-block / skip projections): M x N small, K = B*H*W pixels
    for tag, (H_, ci, co) in {"w1x1_16_128": (16, 128, 128), "w1x1_16_256": (16, 256, 128), "w1x1_8_256": (8, 256, 256),
                              "w1x1_4_512": (4, 512, 512), "w1x1_16_8": (16, 128, 8)}.items():
        gyq = rn(B * H_ * H_, co, dt=bf)
        xq = rn(B, H_, H_, ci, dt=bf)
        gwq = torch.zeros(co, ci, 1, 1, device=dev)
        cases.append((tag, 2.0 * B * H_ * H_ * co * ci,
                      lambda gyq=gyq, xq=xq, gwq=gwq, co=co: ops.conv2d_wgrad(gyq, xq, co, 1, 1, 1, 0, gwq)))
    gl = rn(B * 256, 512, dt=bf)
    xl = rn(B * 256, 128, dt=bf)
    gwl = torch.zeros(512, 128, device=dev)
    cases.append(("linear_wgrad_bf16", 2.0 * B * 256 * 512 * 128, lambda: ops.linear_wgrad(gl, xl, gwl)))
    # grouped expert GEMM (8 experts x 16384 rows, 128 -> 512, GELU)
    E_, rows = 8, 16384
    Ae = rn(E_ * rows, 128, dt=bf)
    We = rn(E_ * 512, 128, dt=bf, sc=0.05)
    row_off = torch.arange(0, E_ + 1, device=dev, dtype=torch.int32) * rows
    tile_off = torch.arange(0, E_ + 1, device=dev, dtype=torch.int32) * (rows // 128)
    oute = torch.empty(E_ * rows, 512, device=dev, dtype=bf)
    be = rn(E_, 512)
    cases.append(("expert_fc1", 2.0 * E_ * rows * 512 * 128,
                  lambda: ops.gemm_grouped(Ae, We, row_off, tile_off, E_ * rows // 128, 512, 128, b_gstride=512 * 128,
                                           out=oute, ep=ops.E(act=L.ACT_GELU))))
    # expert layer-2 data gradient with GELU' (the backward's gP GEMM, B = W2 [C, Hd] N-contiguous)
    W2e = rn(E_ * 128, 512, dt=bf, sc=0.05)
    gGe = rn(E_ * rows, 128, dt=bf)
    Pre_e = rn(E_ * rows, 512, dt=bf)
    gPe = torch.empty(E_ * rows, 512, device=dev, dtype=bf)
    cases.append(("expert_gP", 2.0 * E_ * rows * 512 * 128,
                  lambda: ops.gemm_grouped(gGe, W2e, row_off, tile_off, E_ * rows // 128 + E_, 512, 128, b_kc=False,
                                           b_gstride=128 * 512, out=gPe, ldb=512,
                                           ep=ops.E(act=L.ACT_MUL_GELU_GRAD, aux=Pre_e, ld_aux=512))))
    cases.append(("expert_gP_noaux", 2.0 * E_ * rows * 512 * 128,
                  lambda: ops.gemm_grouped(gGe, W2e, row_off, tile_off, E_ * rows // 128 + E_, 512, 128, b_kc=False,
                                           b_gstride=128 * 512, out=gPe, ldb=512)))
    # expert layer-1 data gradient gX = gP W1 (K = 512)
    W1e = rn(E_ * 512, 128, dt=bf, sc=0.05)
    gXe = torch.empty(E_ * rows, 128, device=dev, dtype=bf)
    cases.append(("expert_gX", 2.0 * E_ * rows * 512 * 128,
                  lambda: ops.gemm_grouped(gPe, W1e, row_off, tile_off, E_ * rows // 128 + E_, 128, 512, b_kc=False,
                                           b_gstride=512 * 128, out=gXe, ldb=128)))
    # D conv0 at 64x64 (K = 48 im2col columns)
    cols0 = rn(B * 1024, 48, dt=bf)
    W0 = rn(128, 48, dt=bf, sc=0.1)
    b0 = rn(128)
    cases.append(("d_conv0_fwd", 2.0 * B * 1024 * 128 * 48,
                  lambda: ops.linear(cols0, W0, bias=b0, act=L.ACT_LRELU)))
    ga0 = rn(B * 1024, 128, dt=bf)
    dW0 = torch.zeros(128, 48, device=dev)
    cases.append(("d_conv0_wgrad", 2.0 * B * 1024 * 128 * 48,
                  lambda: ops.gemm(ga0, cols0, 128, 48, B * 1024, a_kc=False, b_kc=False, out=dW0,
                                   ep=ops.E(atomic=1), splits=0)))
    cases.append(("d_conv0_dgrad", 2.0 * B * 1024 * 128 * 48,
                  lambda: ops.gemm(ga0, W0, B * 1024, 48, 128, b_kc=False, out_dtype=torch.float32)))
    # fused expert FFN (fc1 + GELU + fc2 on chip), no-grad and saved forms
    We1 = rn(E_, 512, 128, dt=bf, sc=0.08)
    We2 = rn(E_, 128, 512, dt=bf, sc=0.04)
    be1, be2 = rn(E_ * 512), rn(E_ * 128)
    Yf = torch.empty(E_ * rows, 128, device=dev, dtype=bf)
    Pf = torch.empty(E_ * rows, 512, device=dev, dtype=bf)
    Hf = torch.empty(E_ * rows, 512, device=dev, dtype=bf)
    mt = E_ * rows // 128 + E_
    cases.append(("ffn128_nosave", 4.0 * E_ * rows * 512 * 128,
                  lambda: ops.moe_ffn_fwd(Ae, We1, be1, We2, be2, row_off, tile_off, mt, Yf)))
    cases.append(("ffn128_save", 4.0 * E_ * rows * 512 * 128,
                  lambda: ops.moe_ffn_fwd(Ae, We1, be1, We2, be2, row_off, tile_off, mt, Yf, pre=Pf, hid=Hf)))
    # expert weight gradient (grouped over rows, plain operands)
    gG = rn(E_ * rows, 128, dt=bf)
    Hid = rn(E_ * rows, 512, dt=bf)
    gWe = torch.zeros(E_, 128, 512, device=dev)
    cases.append(("expert_wgrad", 2.0 * E_ * rows * 512 * 128,
                  lambda: ops.gemm_grouped_wgrad(gG, Hid, row_off, E_ * rows, 128, 512, gWe)))
    # discriminator head / R1 LReLU' products (one K step, bf16 in / out, streamed aux)
    Gh = rn(B * 256, 16, dt=bf)
    W2i = rn(256, 16, dt=bf, sc=0.2)
    h1a = rn(B * 256, 256, dt=bf)
    cases.append(("d_head_ga1", 2.0 * B * 256 * 256 * 16,
                  lambda: ops.gemm(Gh, W2i, B * 256, 256, 16, out_dtype=torch.bfloat16,
                                   ep=ops.E(act=L.ACT_MUL_LRELU_GRAD, aux=h1a, ld_aux=256))))
    h0a = rn(B * 1024, 128, dt=bf)
    cases.append(("d_r1_m0v0", 2.0 * B * 1024 * 128 * 48,
                  lambda: ops.gemm(cols0, W0, B * 1024, 128, 48, out_dtype=torch.bfloat16,
                                   ep=ops.E(act=L.ACT_MUL_LRELU_GRAD, aux=h0a, ld_aux=128))))
    # calibration: square bf16 GEMM
    Ab = rn(4096, 4096, dt=bf)
    Bb = rn(4096, 4096, dt=bf)
    cases.append(("gemm4096_bf16", 2.0 * 4096 ** 3, lambda: ops.gemm(Ab, Bb, 4096, 4096, 4096)))
    # plain bf16 linear (attention proj / qkv shape)
    xq = rn(B * 256, 128, dt=bf)
    wq = rn(384, 128, dt=bf, sc=0.05)
    cases.append(("qkv_linear_bf16", 2.0 * B * 256 * 384 * 128, lambda: ops.linear(xq, wq)))
    # small fp32 GEMMs (styles, mapping)
    w = rn(B, 512)
    Wm = rn(512, 512, sc=0.04)
    bm = rn(512)
    cases.append(("style_fp32", 2.0 * B * 512 * 512, lambda: ops.linear(w, Wm, bias=bm)))
    gs = rn(B, 512)
    gwm = torch.zeros(512, 512, device=dev)
    cases.append(("style_wgrad_fp32", 2.0 * B * 512 * 512, lambda: ops.linear_wgrad(gs, w, gwm)))
    cases.append(("style_dgrad_fp32", 2.0 * B * 512 * 512, lambda: ops.linear_dgrad(gs, Wm)))
    # hipBLASLt (torch.matmul) on the plain-GEMM equivalents of the conv shapes: the library ceiling
    for tag, (M, N, K) in {"conv8": (B * 64, 256, 2304), "conv4": (B * 16, 512, 4608),
                           "conv16": (B * 256, 128, 1152), "dconv1": (B * 256, 256, 2048),
                           "fc1": (8 * 16384, 512, 128), "sq4096": (4096, 4096, 4096)}.items():
        At, Bt = rn(M, K, dt=bf), rn(N, K, dt=bf)
        cases.append((f"torch_{tag}", 2.0 * M * N * K, lambda At=At, Bt=Bt: torch.matmul(At, Bt.t())))

    only = set(a.only.split(",")) if a.only else None
    variants = [("", {})]
    if a.variants:
        variants = []
        for v in a.variants.split(";"):
            kv = dict(tuple(int(t) for t in x.split("=")) for x in v.split(",") if x)
            variants.append((v, kv))
    todo = [(n + (f"[{vn}]" if vn else ""), f, fn, kv) for n, f, fn in cases for vn, kv in variants
            if not only or n in only]
    for name, flop, fn, kv in todo:
        for k in range(16):
            L.call("mg_set_tuning", k, 0)
        for k, v in kv.items():
            L.call("mg_set_tuning", k, v)
        for _ in range(3):
            fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.iters)]
        for s, e in ev:
            s.record()
            fn()
            e.record()
        torch.cuda.synchronize()
        ms = sorted(s.elapsed_time(e) for s, e in ev)
        med = ms[len(ms) // 2]
        print(f"{name:20s} {med * 1e3:9.1f} us  {flop / med / 1e9:8.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
