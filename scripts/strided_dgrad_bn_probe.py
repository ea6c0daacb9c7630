"""ResNet-50 strided 3x3 dgrads feeding a BatchNorm+ReLU backward: (four sub-pixel phase convs
with the kBnG epilogue + BN finalize/apply) vs (MIOpen dgrad + the 3-kernel BN backward).
Interleaved timing in one process."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_ray_amd.ops import fused as F  # noqa: E402


def timeit(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


print("| H in | C | phases+kBnG+parts us | MIOpen+BN us | err |\n|---|---|---|---|---|")
for h, c in [(56, 128), (28, 256), (14, 512)]:
    torch.manual_seed(0)
    n = 256
    x2 = (torch.randn(n * h * h, c, device='cuda') + 0.2).bfloat16()
    s_ = torch.rand(c, device='cuda') + 0.5
    b_ = torch.randn(c, device='cuda') * 0.1
    a, mean, invstd, mask = F._bn_fwd_hip(x2, None, s_, b_, None, None, True, 0.9, 1e-5, True)
    w = (torch.randn(c, c, 3, 3, device='cuda') * 0.03).to(torch.bfloat16)
    dy = torch.randn(n, h // 2, h // 2, c, device='cuda', dtype=torch.bfloat16)
    xs = (n, h, h, c)
    rec = F._BnHandoff(x2, mask, mean)

    def ours():
        g = F._conv_dgrad_s2(dy, w, xs, rec)
        part = rec.part
        rec.g = rec.part = None
        return F._bn_bwd_parts_hip(g.view(-1, c), x2, s_, mean, invstd, part)[0]

    def lib():
        gx = torch.ops.aten.convolution_backward(
            dy.permute(0, 3, 1, 2), a.view(xs).permute(0, 3, 1, 2), w, None, [2, 2], [1, 1], [1, 1], False,
            [0, 0], 1, [True, False, False])[0]
        g = gx.permute(0, 2, 3, 1).contiguous().view(-1, c)
        return F._bn_bwd_hip(g, None, mask, x2, s_, mean, invstd, True, False)[0]
    r0, r1 = ours().float(), lib().float()
    err = (r0 - r1).abs().max().item() / r1.abs().max().item()
    ts = [[], []]
    for _ in range(5):
        ts[0].append(timeit(ours))
        ts[1].append(timeit(lib))
    print(f"| {h} | {c} | {statistics.median(ts[0]):.1f} | {statistics.median(ts[1]):.1f} | {err:.1e} |", flush=True)
