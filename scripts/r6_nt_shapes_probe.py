"""dy·Wᵀ (NT) GEMMs of the BERT-base and GPT-1.3B steps: in-tree per-tile W4T kernel, persistent
W4 kernel and hipBLASLt, interleaved medians + fp32-reference error.
python scripts/r6_nt_shapes_probe.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_ray_amd.ops import fused as F, _native  # noqa: E402


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
    cases = [('bert.qkv.dgrad', 16384, 768, 2304), ('bert.fc1.dgrad', 16384, 768, 3072),
             ('bert.out.dgrad', 16384, 768, 768), ('bert.fc2.dgrad', 16384, 3072, 768),
             ('gpt.out.dgrad', 16384, 2048, 2048), ('gpt.qkv.dgrad', 16384, 2048, 6144)]
    print('| GEMM | tile W4T us | persistent W4 us | hipBLASLt us | best in-tree / hipBLASLt | err |')
    print('|---|---|---|---|---|---|')
    for name, M, N, K in cases:
        a, b = r(M, K), r(N, K)
        c = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)

        def tile():
            L.gemm_set_pts(0)
            F._gemm_hip(1, a, b, out=c)

        def pts():
            L.gemm_set_pts(2)
            F._gemm_hip(1, a, b, out=c)
            L.gemm_set_pts(0)
        fns = [tile, pts, lambda: torch.mm(a, b.t())]
        ref = a.float() @ b.float().t()
        errs = []
        for f in fns[:2]:
            c.zero_()
            f()
            errs.append(((c.float() - ref).abs().max() / ref.abs().max()).item())
        del ref
        ts = [[] for _ in fns]
        for _ in range(7):
            for i, f in enumerate(fns):
                ts[i].append(timeit(f, 10))
        m = [statistics.median(t) for t in ts]
        print(f"| {name} {M}x{N}x{K} | {m[0]:.1f} | {m[1]:.1f} | {m[2]:.1f} | {min(m[0], m[1]) / m[2]:.3f} | "
              f"{max(errs):.1e} |", flush=True)


if __name__ == '__main__':
    main()
