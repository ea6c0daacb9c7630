"""GPT-1.3B weight-gradient GEMMs (xᵀ·dy, K = 16384 tokens) written with beta = 1 (accumulate
into the zeroed gradient slab) vs beta = 0 (overwrite): the cost of the C read."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_ray_amd.ops import fused as F  # noqa: E402

T = 16384


def timeit(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


g = torch.Generator(device='cuda').manual_seed(0)
r = lambda *s: ((torch.rand(*s, device='cuda', generator=g) * 2 - 1) * 0.5).to(torch.bfloat16)  # noqa
tot = [0.0, 0.0]
for name, M, N in (('qkv.wgrad', 2048, 6144), ('out.wgrad', 2048, 2048), ('fc1.wgrad', 2048, 8192),
                   ('fc2.wgrad', 8192, 2048)):
    x, dy = r(T, M), r(T, N)
    c = torch.zeros(M, N, device='cuda', dtype=torch.bfloat16)
    f0 = lambda: F.gemm(F.GEMM_TN, x, dy, out=c, beta=0)  # noqa
    f1 = lambda: F.gemm(F.GEMM_TN, x, dy, out=c, beta=1)  # noqa
    f0(), f1()
    ts = [[], []]
    for _ in range(7):
        ts[0].append(timeit(f0))
        ts[1].append(timeit(f1))
    m = [statistics.median(t) for t in ts]
    tot[0] += m[0]
    tot[1] += m[1]
    print(f"| {name} | {M} | {N} | beta0 {m[0]:.1f} us | beta1 {m[1]:.1f} us | +{m[1] - m[0]:.1f} |", flush=True)
print(f"per layer: beta0 {tot[0]:.1f} us, beta1 {tot[1]:.1f} us; x24 = {(tot[1] - tot[0]) * 24 / 1e3:.2f} ms/step")
