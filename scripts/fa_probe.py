"""Flash-attention kernel probe: times the HIP fwd / bwd kernels on the GPT-3 1.3B
attention shape (B 16, S 1024, H 16, D 128, causal, packed qkv) and checks them against
the fp32 reference. Run under rocprofv3 for per-kernel times / counters."""
import argparse
import math
import sys
import time

import torch

sys.path.insert(0, '.')
from paddle_ray_amd.ops import fused as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--B', type=int, default=16)
ap.add_argument('--S', type=int, default=1024)
ap.add_argument('--H', type=int, default=16)
ap.add_argument('--D', type=int, default=128)
ap.add_argument('--iters', type=int, default=20)
ap.add_argument('--causal', type=int, default=1)
ap.add_argument('--check', type=int, default=1)
a = ap.parse_args()
torch.manual_seed(0)
B, S, H, D = a.B, a.S, a.H, a.D
qkv = torch.randn(B, S, 3, H, D, device='cuda', dtype=torch.bfloat16)
q, k, v = qkv.unbind(2)
scale = 1 / math.sqrt(D)
causal = bool(a.causal)
o, lse = K._fa_fwd_hip(q, k, v, causal, scale)
do = torch.randn_like(o)
dqkv = torch.empty_like(qkv)
dq, dk, dv = dqkv.unbind(2)


def t(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / a.iters


frac = 0.5 if causal else 1.0
f_fwd = 4 * B * H * S * S * D * frac
tf = t(lambda: K._fa_fwd_hip(q, k, v, causal, scale))
tb = t(lambda: K._fa_bwd_hip(do, q, k, v, o, lse, causal, scale, dq, dk, dv))
print(f'fwd {tf*1e6:8.1f} us {f_fwd/tf/1e12:7.1f} TF/s | bwd {tb*1e6:8.1f} us '
      f'{2.5*f_fwd/tb/1e12:7.1f} TF/s (5 GEMMs)', flush=True)
if a.check:
    bs = 2
    qf, kf, vf = (x[:bs].float().requires_grad_() for x in (q, k, v))
    ref_o, _ = K._fa_fwd_ref(qf, kf, vf, causal, scale)
    ref_o.backward(do[:bs].float())
    e = lambda x, y: ((x.float() - y).abs().max() / y.abs().max()).item()  # noqa: E731
    print(f'rel err o {e(o[:bs], ref_o):.2e} dq {e(dq[:bs], qf.grad):.2e} '
          f'dk {e(dk[:bs], kf.grad):.2e} dv {e(dv[:bs], vf.grad):.2e}', flush=True)
