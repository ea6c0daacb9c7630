"""Plain x·W GEMMs of the GPT-1.3B step (qkv / out / fc2 forward, LM-head logits dgrad shape):
per-tile W8T kernel (default policy) vs the persistent kernel with 8 / 4 waves, interleaved
medians, fp32-reference error.   python scripts/r6_fwd_policy_probe.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_ray_amd.ops import fused as F, _native  # noqa: E402

T = 16384


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    L = _native.lib()
    F._GEMM_MODE = 'mfma'
    g = torch.Generator(device='cuda').manual_seed(0)
    r = lambda *s: ((torch.rand(*s, device='cuda', generator=g) * 2 - 1) * 0.5).to(torch.bfloat16)  # noqa
    cases = [('qkv.fwd', T, 6144, 2048), ('out.fwd', T, 2048, 2048), ('fc2.fwd', T, 2048, 8192),
             ('fc1.fwd', T, 8192, 2048)]
    masks = [('tile', 0), ('pts8', 1), ('pts4', 1 | 32)]
    print('| GEMM | ' + ' | '.join(f'{n} us' for n, _ in masks) + ' | hipBLASLt us | err |')
    print('|---|' + '---|' * (len(masks) + 2))
    for name, M, N, K in cases:
        a, b = r(M, K), r(K, N)
        c = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
        fns = []
        for _, mk in masks:
            def f(mk=mk):
                L.gemm_set_pts(mk)
                F._gemm_hip(0, a, b, out=c)
            fns.append(f)
        fns.append(lambda: torch.mm(a, b))
        ref = a.float() @ b.float()
        errs = []
        for f in fns[:-1]:
            c.zero_()
            f()
            errs.append(((c.float() - ref).abs().max() / ref.abs().max()).item())
        del ref
        ts = [[] for _ in fns]
        for _ in range(7):
            for i, f in enumerate(fns):
                ts[i].append(timeit(f, 10))
        L.gemm_set_pts(0)
        m = [statistics.median(t) for t in ts]
        print(f"| {name} {M}x{N}x{K} | " + ' | '.join(f'{x:.1f}' for x in m) + f" | {max(errs):.1e} |", flush=True)


if __name__ == '__main__':
    main()
