"""Flash-attention probe for the BERT-base shape (B 32, S 512, H 12, D 64, non-causal): times
the plain kernels, the extended kernels without extras, with dropout, and with an additive
padding mask, forward and backward (graph-free, device-synchronised means)."""
import argparse
import math
import sys
import time

import torch

sys.path.insert(0, '.')
from paddle_ray_amd.ops import fused as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--B', type=int, default=32)
ap.add_argument('--S', type=int, default=512)
ap.add_argument('--H', type=int, default=12)
ap.add_argument('--D', type=int, default=64)
ap.add_argument('--causal', type=int, default=0)
ap.add_argument('--iters', type=int, default=20)
a = ap.parse_args()
torch.manual_seed(0)
B, S, H, D = a.B, a.S, a.H, a.D
causal = bool(a.causal)
qkv = torch.randn(B, S, 3, H, D, device='cuda', dtype=torch.bfloat16)
q, k, v = (t.detach().requires_grad_() for t in qkv.unbind(2))
scale = 1 / math.sqrt(D)
frac = 0.5 if causal else 1.0
f_fwd = 4 * B * H * S * S * D * frac


def t(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / a.iters


def report(name, fwd, bwd):
    tf = t(fwd)
    tb = t(bwd)
    print(f'{name:18s} fwd {tf*1e6:8.1f} us {f_fwd/tf/1e12:7.1f} TF/s | bwd {tb*1e6:8.1f} us '
          f'{2.5*f_fwd/tb/1e12:7.1f} TF/s', flush=True)


o, lse = K._fa_fwd_hip(q.detach(), k.detach(), v.detach(), causal, scale)
do = torch.randn_like(o)
report('plain', lambda: K._fa_fwd_hip(q.detach(), k.detach(), v.detach(), causal, scale),
       lambda: K._fa_bwd_hip(do, q.detach(), k.detach(), v.detach(), o, lse, causal, scale))
mask = torch.zeros(B, 1, 1, S, device='cuda', dtype=torch.bfloat16)
mask[:, :, :, S - S // 8:] = float('-inf')
for name, kw in (('ext', {}), ('ext+dropout0.1', {'dropout': 0.1}), ('ext+mask', {'attn_mask': mask}),
                 ('ext+mask+dropout', {'attn_mask': mask, 'dropout': 0.1})):
    kw = dict(kw)
    if name == 'ext':
        # force the extended kernels with no extras (dropout 0, no mask)
        fn = lambda: K.FlashAttnExtFn.apply(q, k, v, None, None, None, S, S, causal, scale, 0.0, 0, 0)  # noqa
    else:
        fn = lambda kw=kw: K.flash_attention_ext(q, k, v, causal=causal, **kw)  # noqa
    out = fn()
    report(name, fn, lambda: torch.autograd.grad(out, (q, k, v), do, retain_graph=True))
