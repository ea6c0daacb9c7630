"""Persistent GEMM tile order under co-resident load: the fused MLP GEMMs (x·W + bias + GELU with
GELU', dy·Wᵀ · Z) and a long-K dy·Wᵀ, alone and with 32 workgroups of a spinning load on a side
stream (the RCCL channels of overlapped communication). PRA_PTS_DYN=0|1 (read once)."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_ray_amd.ops import fused as F, _native  # noqa: E402

T = 16384
L = _native.lib()
F._GEMM_MODE = 'mfma'
dyn = os.environ.get('PRA_PTS_DYN', '1')
g = torch.Generator(device='cuda').manual_seed(0)
r = lambda *s: ((torch.rand(*s, device='cuda', generator=g) * 2 - 1) * 0.5).to(torch.bfloat16)  # noqa
sink = torch.zeros(256, device='cuda')
side = torch.cuda.Stream()


def timeit(fn, iters, hog):
    torch.cuda.synchronize()
    if hog:
        with torch.cuda.stream(side):
            L.spin_hog(hog, int(2.2e9 * 0.02), sink.data_ptr(), side.cuda_stream)   # ~20 ms of load
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


cases = [('fc1.fwd+gelu_d', 0, T, 8192, 2048, 'gelu_tanh_d'), ('fc2.dgrad*z', 1, T, 8192, 2048, 'mulz'),
         ('qkv.dgrad', 1, T, 2048, 6144, None)]
for name, lay, M, N, K, epi in cases:
    a = r(M, K)
    b = r(K, N) if lay == 0 else r(N, K)
    c = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
    z = r(M, N) if epi == 'mulz' else (torch.empty_like(c) if epi else None)
    bias = r(N) if epi == 'gelu_tanh_d' else None

    def fn():
        if epi is None:
            L.gemm_set_pts(2)
        F._gemm_hip(lay, a, b, out=c, bias=bias, z=z, epi=epi)
        if epi is None:
            L.gemm_set_pts(0)
    fn()
    ref = a.float() @ (b.float() if lay == 0 else b.float().t())
    if epi == 'gelu_tanh_d':
        ref = torch.nn.functional.gelu(ref + bias.float(), approximate='tanh')
    elif epi == 'mulz':
        ref = ref * z.float()
    err = ((c.float() - ref).abs().max() / ref.abs().max()).item()
    del ref
    ts = [[], []]
    for _ in range(5):
        ts[0].append(timeit(fn, 8, 0))
        ts[1].append(timeit(fn, 8, 32))
    m = [statistics.median(t) for t in ts]
    print(f"| DYN={dyn} | {name} | alone {m[0]:.1f} us | 32-WG load {m[1]:.1f} us | x{m[1] / m[0]:.2f} | err {err:.1e} |",
          flush=True)
