"""GPT-1.3B MLP GEMMs with their fused epilogues vs the plain kernels and hipBLASLt (interleaved
timing, medians of 5 rounds), plus the long-K dy·Wᵀ dgrads on the in-tree persistent kernel.

    python scripts/r6_gemm_probe.py
"""
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
    rows = []
    # (name, layout, M, N, K, epi)
    cases = [('fc1.fwd', 0, T, 8192, 2048, None), ('fc1.fwd+gelu_tanh_d', 0, T, 8192, 2048, 'gelu_tanh_d'),
             ('fc2.dgrad', 1, T, 8192, 2048, None), ('fc2.dgrad*z', 1, T, 8192, 2048, 'mulz'),
             ('qkv.dgrad', 1, T, 2048, 6144, None), ('out.dgrad', 1, T, 2048, 2048, None),
             ('fc1.dgrad', 1, T, 2048, 8192, None), ('head.fwd', 1, T, 50304, 2048, None)]
    print("| GEMM | M | N | K | in-tree PTS4 us | hipBLASLt us | PF/s in-tree | rel err |")
    print("|---|---|---|---|---|---|---|---|", flush=True)
    for name, lay, M, N, K, epi in cases:
        a = r(M, K)
        b = r(K, N) if lay == 0 else r(N, K)
        c = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
        z = r(M, N) if epi == 'mulz' else (torch.empty_like(c) if epi else None)
        bias = r(N) if epi == 'gelu_tanh_d' else None

        def ours():
            F._gemm_hip(lay, a, b, out=c, bias=bias, z=z, epi=epi)

        def ours_persist():
            L.gemm_set_pts(1 << lay if lay == 1 else (1 | 32))
            F._gemm_hip(lay, a, b, out=c, bias=bias, z=z, epi=epi)
            L.gemm_set_pts(0)

        def blas():
            if lay == 0:
                torch.mm(a, b)
            else:
                torch.mm(a, b.t())
        fn = ours_persist if epi is None else ours
        fn()
        bf = b.float() if lay == 0 else b.float().t()
        ref = a.float() @ bf
        if epi == 'gelu_tanh_d':
            ref = torch.nn.functional.gelu(ref + bias.float(), approximate='tanh')
        elif epi == 'mulz':
            ref = ref * z.float()
        err = ((c.float() - ref).abs().max() / ref.abs().max()).item()
        del ref, bf
        it = 3 if M * N * K > 1e12 else 10
        ts = [[], []]
        for _ in range(5):
            ts[0].append(timeit(fn, it))
            ts[1].append(timeit(blas, it))
        m = [statistics.median(t) for t in ts]
        pf = 2.0 * M * N * K / (m[0] * 1e-6) / 1e15
        print(f"| {name} | {M} | {N} | {K} | {m[0]:.1f} | {m[1]:.1f} | {pf:.3f} | {err:.1e} |", flush=True)
        rows.append((name, m))


if __name__ == '__main__':
    main()
