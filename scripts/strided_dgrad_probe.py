"""ResNet-50 (bs 256) strided 3x3 dgrads: the four sub-pixel phase convs on the in-tree kernel
vs MIOpen's convolution_backward (NHWC). Interleaved timing in one process."""
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


print("| H in | C | phases us | MIOpen us | err |\n|---|---|---|---|---|")
for h, c in [(56, 128), (28, 256), (14, 512)]:
    torch.manual_seed(0)
    x = torch.randn(256, h, h, c, device='cuda', dtype=torch.bfloat16)
    w = (torch.randn(c, c, 3, 3, device='cuda') * 0.03).to(torch.bfloat16)
    dy = torch.randn(256, h // 2, h // 2, c, device='cuda', dtype=torch.bfloat16)
    ours = lambda: F._conv_dgrad_s2(dy, w, x.shape)  # noqa: E731
    lib = lambda: torch.ops.aten.convolution_backward(  # noqa: E731
        dy.permute(0, 3, 1, 2), x.permute(0, 3, 1, 2), w, None, [2, 2], [1, 1], [1, 1], False, [0, 0], 1,
        [True, False, False])[0]
    a, b = ours().float(), lib().permute(0, 2, 3, 1).float()
    err = (a - b).abs().max().item() / b.abs().max().item()
    ts = [[], []]
    for _ in range(5):
        ts[0].append(timeit(ours))
        ts[1].append(timeit(lib))
    print(f"| {h} | {c} | {statistics.median(ts[0]):.1f} | {statistics.median(ts[1]):.1f} | {err:.1e} |", flush=True)
