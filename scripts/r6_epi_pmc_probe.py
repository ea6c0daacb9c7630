"""fc1 forward 16384 x 8192 x 2048 on the persistent W4 kernel, plain vs the fused bias + tanh-GELU
+ gelu' epilogue (5 calls each): run under rocprofv3 --pmc to compare per-dispatch VALU / MFMA work.
python scripts/r6_epi_pmc_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_ray_amd.ops import fused as F, _native  # noqa: E402

L = _native.lib()
F._GEMM_MODE = 'mfma'
g = torch.Generator(device='cuda').manual_seed(0)
r = lambda *s: ((torch.rand(*s, device='cuda', generator=g) * 2 - 1) * 0.5).to(torch.bfloat16)  # noqa
M, N, K = 16384, 8192, 2048
a, b, bias = r(M, K), r(K, N), r(N)
c = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
z = torch.empty_like(c)
L.gemm_set_pts(1 | 32)
for _ in range(5):
    F._gemm_hip(0, a, b, out=c)
for _ in range(5):
    F._gemm_hip(0, a, b, out=c, bias=bias, z=z, epi='gelu_tanh_d')
torch.cuda.synchronize()
L.gemm_set_pts(0)
print('ok')
