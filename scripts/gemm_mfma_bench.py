"""MFMA gemm_bias_act (gemm.hip) vs hipBLASLt matmul + separate bias/GELU pass on the GPT-3 1.3B
layer shapes (tokens = 16 x 1024). Prints one line per shape; used for profiles/r1_gemm_mfma."""
import sys
import os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_ray_amd.ops import fused as F  # noqa: E402


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


M = 16384
for (K, N, act) in [(2048, 6144, None), (2048, 8192, 'gelu'), (8192, 2048, None), (2048, 2048, None),
                    (4096, 4096, None), (8192, 8192, None)]:
    x = torch.randn(M, K, device='cuda', dtype=torch.bfloat16)
    w = torch.randn(K, N, device='cuda', dtype=torch.bfloat16) / K ** 0.5
    b = torch.randn(N, device='cuda', dtype=torch.bfloat16)
    a = F._ACT[act]
    t_mfma = timeit(lambda: F._gba_hip(x, w, b, a, False))
    if act:
        t_lib = timeit(lambda: F.bias_gelu(x @ w, b, False))
    else:
        t_lib = timeit(lambda: torch.addmm(b, x, w))
    fl = 2 * M * N * K
    print(f"M={M} K={K} N={N} act={act}: mfma {t_mfma:8.1f} us ({fl / t_mfma / 1e9:6.3f} PF/s)   "
          f"hipBLASLt+epilogue {t_lib:8.1f} us ({fl / t_lib / 1e9:6.3f} PF/s)", flush=True)
