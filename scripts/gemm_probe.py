"""GEMM layout / library probe for the GPT-3 1.3B shapes (M = 16 x 1024 tokens).

Prints achieved TFLOP/s per (shape, layout, library) so the model can pick the fastest
weight layout and decide whether TunableOp tuning pays. Usage (on the GPU box):
  python scripts/gemm_probe.py [--lib hipblaslt|rocblas] [--tunable]
"""
import argparse
import json
import os
import sys
import time

ap = argparse.ArgumentParser()
ap.add_argument('--lib', default='hipblaslt')
ap.add_argument('--tunable', action='store_true')
ap.add_argument('--iters', type=int, default=20)
args = ap.parse_args()
if args.tunable:
    os.environ['PYTORCH_TUNABLEOP_ENABLED'] = '1'
    os.environ['PYTORCH_TUNABLEOP_TUNING'] = '1'
    os.environ.setdefault('PYTORCH_TUNABLEOP_FILENAME', 'gpurun_out/tunableop_results.csv')
import torch  # noqa: E402

torch.backends.cuda.preferred_blas_library(args.lib)
dev = 'cuda'
M = 16384
shapes = {'qkv': (2048, 6144), 'out': (2048, 2048), 'fc1': (2048, 8192), 'fc2': (8192, 2048),
          'logits': (2048, 50304)}


def bench(fn, flops):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.iters):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / args.iters
    return flops / dt / 1e12, dt * 1e6


res = []
for name, (K, N) in shapes.items():
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    w_kn = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
    w_nk = w_kn.t().contiguous()
    f = 2 * M * N * K
    cases = {
        'fwd x@W[K,N]': lambda: x @ w_kn,
        'fwd x@W[N,K]^T': lambda: x @ w_nk.t(),
        'dX dy@W[K,N]^T': lambda: dy @ w_kn.t(),
        'dX dy@W[N,K]': lambda: dy @ w_nk,
        'dW[K,N] x^T@dy': lambda: x.t() @ dy,
        'dW[N,K] dy^T@x': lambda: dy.t() @ x,
    }
    for cname, fn in cases.items():
        tf, us = bench(fn, f)
        res.append({'gemm': name, 'case': cname, 'tflops': round(tf, 1), 'us': round(us, 1)})
        print(f'{name:7s} {cname:18s} {tf:8.1f} TF/s {us:9.1f} us', flush=True)
    del x, dy, w_kn, w_nk
print(json.dumps({'lib': args.lib, 'tunable': args.tunable, 'results': res}))
