"""Run the HIP flash-attention fwd+bwd on one shape N times (for rocprofv3 counter passes)
and print TF/s per kernel from CUDA events.

usage: python -m scripts.fa_one [B H S D causal iters]"""
import sys
import time

import torch


def main():
    a = sys.argv[1:]
    B, H, S, D = (int(x) for x in (a[:4] if len(a) >= 4 else (16, 16, 1024, 128)))
    causal = bool(int(a[4])) if len(a) > 4 else True
    iters = int(a[5]) if len(a) > 5 else 10
    from paddle_ray_amd.ops import fused as K
    from paddle_ray_amd.ops import registry as R
    g = torch.Generator(device='cuda').manual_seed(0)
    q, k, v = (torch.randn(B, S, H, D, device='cuda', dtype=torch.bfloat16, generator=g)
               for _ in range(3))
    do = torch.randn(B, S, H, D, device='cuda', dtype=torch.bfloat16, generator=g)
    scale = D ** -0.5
    o, lse = R.dispatch('flash_attn_fwd', q, q, k, v, causal, scale)
    R.dispatch('flash_attn_bwd', q, do, q, k, v, o, lse, causal, scale)
    torch.cuda.synchronize()
    f_fwd = 4 * B * H * S * S * D / (2 if causal else 1)
    for name, fn, fl in (('fwd', lambda: R.dispatch('flash_attn_fwd', q, q, k, v, causal, scale), f_fwd),
                         ('bwd', lambda: R.dispatch('flash_attn_bwd', q, do, q, k, v, o, lse, causal, scale),
                          2.5 * f_fwd)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / iters
        print(f"{name}: {dt * 1e6:.1f} us  {fl / dt / 1e12:.1f} TF/s (B{B} H{H} S{S} D{D} causal={causal})",
              flush=True)
        # the same calls replayed from one captured HIP graph: GPU time without host launch gaps
        graph = torch.cuda.CUDAGraph()
        fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(graph):
            for _ in range(iters):
                fn()
        graph.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        graph.replay()
        torch.cuda.synchronize()
        dg = (time.perf_counter() - t0) / iters
        print(f"{name} (graph replay): {dg * 1e6:.1f} us  {fl / dg / 1e12:.1f} TF/s", flush=True)


if __name__ == '__main__':
    main()
