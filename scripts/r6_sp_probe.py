"""Persistent W4 GEMM refill spacing (PRA_PTS_VAR, read once per process) on the GPT shapes:
interleaved medians vs hipBLASLt.   PRA_PTS_VAR=n python scripts/r6_sp_probe.py"""
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
    sp = (os.environ.get("PRA_PTS_VAR", "0") + "/buf" + os.environ.get("PRA_PTS_BUF", "0")
          + "/stg" + os.environ.get("PRA_PTS_STG", "0"))
    g = torch.Generator(device='cuda').manual_seed(0)
    r = lambda *s: ((torch.rand(*s, device='cuda', generator=g) * 2 - 1) * 0.5).to(torch.bfloat16)  # noqa
    cases = [('fc1.fwd', 0, T, 8192, 2048), ('fc2.dgrad', 1, T, 8192, 2048), ('qkv.dgrad', 1, T, 2048, 6144),
             ('out.dgrad', 1, T, 2048, 2048), ('fc1.dgrad', 1, T, 2048, 8192)]
    for name, lay, M, N, K in cases:
        a = r(M, K)
        b = r(K, N) if lay == 0 else r(N, K)
        c = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)

        def ours():
            L.gemm_set_pts(2 if lay == 1 else (1 | 32))
            F._gemm_hip(lay, a, b, out=c)
            L.gemm_set_pts(0)

        def blas():
            torch.mm(a, b) if lay == 0 else torch.mm(a, b.t())
        ours()
        ref = a.float() @ (b.float() if lay == 0 else b.float().t())
        err = ((c.float() - ref).abs().max() / ref.abs().max()).item()
        del ref
        ts = [[], []]
        for _ in range(7):
            ts[0].append(timeit(ours, 10))
            ts[1].append(timeit(blas, 10))
        m = [statistics.median(t) for t in ts]
        pf = 2.0 * M * N * K / (m[0] * 1e-6) / 1e15
        print(f"| SP={sp} | {name} | {m[0]:.1f} | {m[1]:.1f} | {m[0] / m[1]:.3f} | {pf:.3f} | {err:.1e} |", flush=True)


if __name__ == '__main__':
    main()
