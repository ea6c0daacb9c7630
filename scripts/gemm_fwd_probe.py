"""x·W (forward layout) GEMMs of the GPT-1.3B step: per-tile TS kernel (default) vs the persistent
kernel at 4 waves (PTS4: pra_gemm_set_pts(1 | 32)) and at 8 waves (PTS8: pra_gemm_set_pts(1)) vs
hipBLASLt; plain and with the fc1 bias+GELU(+gelu') epilogue. Interleaved timing.

    python scripts/gemm_fwd_probe.py
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_ray_amd.ops import fused as F, _native  # noqa: E402

T = 16384
SHAPES = [('qkv.fwd', T, 6144, 2048), ('out.fwd', T, 2048, 2048), ('fc1.fwd', T, 8192, 2048),
          ('fc2.fwd', T, 2048, 8192), ('head.dgrad', T, 2048, 50304)]


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
    cfgs = [('TS', 0), ('PTS4', 1 | 32), ('PTS8', 1)]
    print("| GEMM | M | N | K | " + " | ".join(f"{c} us" for c, _ in cfgs) + " | hipBLASLt us | err PTS4 |")
    print("|---|---|---|---|" + "---|" * (len(cfgs) + 2), flush=True)
    for name, M, N, K in SHAPES + [('fc1.fwd+gelu_d', T, 8192, 2048)]:
        a, b = r(M, K), r(K, N)
        c = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
        epi = name.endswith('gelu_d')
        bias = r(N) if epi else None
        z = torch.empty_like(c) if epi else None

        def mk(mask):
            def f():
                L.gemm_set_pts(mask)
                F._gemm_hip(0, a, b, out=c, bias=bias, z=z, epi='gelu_tanh_d' if epi else None)
                L.gemm_set_pts(0)
            return f
        fns = [mk(m) for _, m in cfgs] + [lambda: torch.mm(a, b)]
        mk(1 | 32)()
        ref = a.float() @ b.float()
        if epi:
            ref = torch.nn.functional.gelu(ref + bias.float(), approximate='tanh')
        err = ((c.float() - ref).abs().max() / ref.abs().max()).item()
        for f in fns:
            f()
        torch.cuda.synchronize()
        it = 3 if M * N * K > 1e12 else 10
        ts = [[] for _ in fns]
        for _ in range(5):
            for i, f in enumerate(fns):
                ts[i].append(timeit(f, it))
        m = [statistics.median(t) for t in ts]
        print(f"| {name} | {M} | {N} | {K} | " + " | ".join(f"{x:.1f}" for x in m) + f" | {err:.1e} |", flush=True)


if __name__ == '__main__':
    main()
