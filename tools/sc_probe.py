import sys, torch
sys.path.insert(0, "moe-gan_cpsc541_amd")
from moegan_mi import ops
from moegan_mi.engine_g import GeneratorEngine
torch.manual_seed(0)
for dt in (torch.float32, torch.bfloat16):
    for (B, H, Cin, Cout, k) in ((2, 32, 128, 128, 3), (2, 64, 128, 64, 3), (2, 64, 64, 8, 1), (3, 32, 128, 8, 1)):
        x = torch.randn(B, H, H, Cin, device="cuda").to(dt)
        s = torch.randn(B, Cin, device="cuda") * 0.5 + 1
        W = torch.randn(Cout, Cin, k, k, device="cuda") * 0.05
        # pack like the engine: [Cout, k*k*Cin] (tap-major, ci fastest)
        wp = W.permute(0, 2, 3, 1).reshape(Cout, -1).contiguous().to(dt)
        y1 = ops.conv2d(x, wp, Cout, k, k, 1, k // 2, in_scale=s, out_dtype=torch.float32)
        y2 = ops.conv2d(ops.scale_bc(x, s), wp, Cout, k, k, 1, k // 2, out_dtype=torch.float32)
        gy = torch.randn(B, H, H, Cout, device="cuda").to(dt)
        g1 = torch.zeros(Cout, Cin, k, k, device="cuda"); g2 = torch.zeros_like(g1)
        ops.conv2d_wgrad(gy, x, Cout, k, k, 1, k // 2, g1, in_scale=s)
        ops.conv2d_wgrad(gy, ops.scale_bc(x, s), Cout, k, k, 1, k // 2, g2)
        torch.cuda.synchronize()
        r = lambda a, b: float((a - b).norm() / b.norm())
        print(dt, (B, H, Cin, Cout, k), "fwd rel", r(y1, y2), "wgrad rel", r(g1, g2))
