"""ResNet-50 3x3 conv shapes: implicit-GEMM MFMA kernel vs MIOpen (channels-last), fwd + dgrad."""
import sys
import time

import torch

sys.path.insert(0, '.')
from paddle_ray_amd.ops import fused as K  # noqa: E402


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / it * 1e3


B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
shapes = [(56, 64, 64, 1), (56, 128, 128, 2), (28, 128, 128, 1), (28, 256, 256, 2), (14, 256, 256, 1),
          (14, 512, 512, 2), (7, 512, 512, 1)]
tot = {'ours_f': 0, 'mi_f': 0, 'ours_d': 0, 'mi_d': 0}
for hw, cin, cout, s in shapes:
    x = torch.randn(B, hw, hw, cin, device='cuda', dtype=torch.bfloat16)
    w = (torch.randn(cout, cin, 3, 3, device='cuda') * 0.05).to(torch.bfloat16)
    wk = w.permute(0, 2, 3, 1).reshape(cout, 9 * cin).contiguous()
    xc = x.permute(0, 3, 1, 2)
    wc = w.contiguous(memory_format=torch.channels_last)
    y = K._conv_lds(x, wk, None, 3, 3, s, 1)
    yr = torch.nn.functional.conv2d(xc, wc, None, s, 1)
    err = (y.float() - yr.permute(0, 2, 3, 1).float()).abs().max().item()
    f_o = t(lambda: K._conv_lds(x, wk, None, 3, 3, s, 1))
    f_m = t(lambda: torch.nn.functional.conv2d(xc, wc, None, s, 1))
    fl = 2 * y.numel() * cin * 9
    line = f"hw{hw} {cin}->{cout} s{s}: fwd ours {f_o:.3f} ms ({fl / f_o / 1e9:.0f} TF/s) miopen {f_m:.3f} ms err {err:.3f}"
    tot['ours_f'] += f_o
    tot['mi_f'] += f_m
    if s == 1:
        dy = torch.randn_like(y)
        wf = w.flip(2, 3).permute(1, 2, 3, 0).reshape(cin, 9 * cout).contiguous()
        dyc = dy.permute(0, 3, 1, 2)
        d_o = t(lambda: K._conv_lds(dy, wf, None, 3, 3, 1, 1))
        d_m = t(lambda: torch.ops.aten.convolution_backward(dyc, xc, wc, None, [1, 1], [1, 1], [1, 1], False,
                                                            [0, 0], 1, [True, False, False]))
        dx = K._conv_lds(dy, wf, None, 3, 3, 1, 1)
        dxr = torch.ops.aten.convolution_backward(dyc, xc, wc, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                                  [True, False, False])[0]
        derr = (dx.float() - dxr.permute(0, 2, 3, 1).float()).abs().max().item()
        line += f" | dgrad ours {d_o:.3f} miopen {d_m:.3f} err {derr:.3f}"
        tot['ours_d'] += d_o
        tot['mi_d'] += d_m
    print(line, flush=True)
print({k: round(v, 3) for k, v in tot.items()}, flush=True)

# weight gradient: in-tree implicit GEMM vs MIOpen
tw = {'ours': 0.0, 'miopen': 0.0}
for hw, cin, cout, s in shapes:
    x = torch.randn(B, hw, hw, cin, device='cuda', dtype=torch.bfloat16)
    w = (torch.randn(cout, cin, 3, 3, device='cuda') * 0.05).to(torch.bfloat16)
    ho = (hw + 2 - 3) // s + 1
    dy = torch.randn(B, ho, ho, cout, device='cuda', dtype=torch.bfloat16)
    xc, dyc = x.permute(0, 3, 1, 2), dy.permute(0, 3, 1, 2)
    wc = w.contiguous(memory_format=torch.channels_last)
    mi = lambda: torch.ops.aten.convolution_backward(dyc, xc, wc, None, [s, s], [1, 1], [1, 1], False,  # noqa
                                                     [0, 0], 1, [False, True, False])
    ou = lambda: K._conv_wgrad_lds(dy, x, 3, 3, s, 1)  # noqa
    ref = mi()[1].float()
    got = ou().permute(0, 3, 1, 2).float()
    err = (got - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
    t_o, t_m = t(ou), t(mi)
    tw['ours'] += t_o
    tw['miopen'] += t_m
    print(f"wgrad hw{hw} {cin}->{cout} s{s}: ours {t_o:.3f} ms miopen {t_m:.3f} ms rel err {err:.4f}", flush=True)
print({k: round(v, 3) for k, v in tw.items()}, flush=True)
