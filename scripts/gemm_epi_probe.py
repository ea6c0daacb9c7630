"""Where the persistent dy·Wᵀ kernel's epilogue time goes (fc2 dgrad shape by default): plain,
beta=1 (C read), multiply-by-z without / with the column sums, dGELU (tanh) with column sums, vs
hipBLASLt. Interleaved timing in one process.

    python scripts/gemm_epi_probe.py [M N K]
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_ray_amd.ops import fused as F, _native  # noqa: E402

M, N, Kd = (int(x) for x in sys.argv[1:4]) if len(sys.argv) >= 4 else (16384, 8192, 2048)


def timeit(fn, iters=10):
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
    r = lambda *s: (torch.rand(*s, device='cuda', generator=g) * 2 - 1).to(torch.bfloat16)  # noqa: E731
    dy, w, z = r(M, Kd), r(N, Kd), r(M, N)
    c = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)

    def pts(fn):
        def f():
            L.gemm_set_pts(2)
            fn()
            L.gemm_set_pts(0)
        return f
    fns = [
        ('hipBLASLt', lambda: torch.mm(dy, w.t())),
        ('PTS plain', pts(lambda: F._gemm_hip(1, dy, w, out=c))),
        ('PTS beta=1', pts(lambda: F._gemm_hip(1, dy, w, out=c, beta=1))),
        ('PTS *z', pts(lambda: F._gemm_hip(1, dy, w, out=c, z=z, epi='mulz'))),
        ('PTS *z + colsum', pts(lambda: F._gemm_hip(1, dy, w, out=c, z=z, epi='mulz', want_colsum=True))),
        ('PTS dgelu + colsum', pts(lambda: F._gemm_hip(1, dy, w, out=c, z=z, epi='dgelu_tanh', want_colsum=True))),
        ('TS plain', lambda: F._gemm_hip(1, dy, w, out=c)),
    ]
    for _, f in fns:
        f()
    torch.cuda.synchronize()
    ts = [[] for _ in fns]
    for _ in range(7):
        for i, (_, f) in enumerate(fns):
            ts[i].append(timeit(f))
    print(f"M={M} N={N} K={Kd}\n| variant | us |\n|---|---|")
    for (name, _), t in zip(fns, ts):
        print(f"| {name} | {statistics.median(t):.1f} |", flush=True)


if __name__ == '__main__':
    main()
