"""ResNet-50 (bs 256) 3x3 weight-gradient shapes: the in-tree implicit-GEMM wgrad vs MIOpen's
(aten convolution_backward on the channels-last tensors), device-synchronised means."""
import sys
import time

import torch

sys.path.insert(0, '.')
from paddle_ray_amd.ops import fused as K  # noqa: E402

SHAPES = [  # n, h, w, cin, cout, stride
    (256, 56, 56, 64, 64, 1), (256, 28, 28, 128, 128, 1), (256, 56, 56, 128, 128, 2),
    (256, 14, 14, 256, 256, 1), (256, 7, 7, 512, 512, 1)]


def t(fn, it=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / it * 1e6


print('| n h w cin cout s | ours us | MIOpen us | ratio | rel err |')
print('|---|---|---|---|---|')
for n, h, w_, cin, cout, s in SHAPES:
    x = torch.randn(n, h, w_, cin, device='cuda', dtype=torch.bfloat16)
    ho, wo = (h + 2 - 3) // s + 1, (w_ + 2 - 3) // s + 1
    dy = torch.randn(n, ho, wo, cout, device='cuda', dtype=torch.bfloat16)
    wt = torch.randn(cout, cin, 3, 3, device='cuda', dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    ours = lambda: K._conv_wgrad_lds(dy, x, 3, 3, s, 1)  # noqa: E731
    lib = lambda: torch.ops.aten.convolution_backward(  # noqa: E731
        dy.permute(0, 3, 1, 2), x.permute(0, 3, 1, 2), wt, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1,
        [False, True, False])[1]
    a = ours().permute(0, 3, 1, 2).float()
    b = lib().float()
    err = ((a - b).abs().max() / b.abs().max()).item()
    to, tl = t(ours), t(lib)
    print(f'| {n} {h} {w_} {cin} {cout} {s} | {to:.1f} | {tl:.1f} | {tl / to:.2f} | {err:.1e} |', flush=True)
