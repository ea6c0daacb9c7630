"""Compare the in-tree flash-attention kernels with PyTorch's SDPA backends on the GPT-3
1.3B attention shape (timing reference only; the framework always runs its own kernels)."""
import math
import sys
import time

import torch

sys.path.insert(0, '.')
from paddle_ray_amd.ops import fused as K  # noqa: E402

B, S, H, D = 16, 1024, 16, 128
torch.manual_seed(0)
qkv = torch.randn(B, S, 3, H, D, device='cuda', dtype=torch.bfloat16)
q, k, v = qkv.unbind(2)
scale = 1 / math.sqrt(D)
f_fwd = 4 * B * H * S * S * D * 0.5


def t(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


o, lse = K._fa_fwd_hip(q, k, v, True, scale)
do = torch.randn_like(o)
dqkv = torch.empty_like(qkv)
dq, dk, dv = dqkv.unbind(2)
tf = t(lambda: K._fa_fwd_hip(q, k, v, True, scale))
tb = t(lambda: K._fa_bwd_hip(do, q, k, v, o, lse, True, scale, dq, dk, dv))
print(f'pra   fwd {tf*1e6:7.1f} us ({f_fwd/tf/1e12:6.1f} TF/s)  bwd {tb*1e6:7.1f} us '
      f'({2.5*f_fwd/tb/1e12:6.1f} TF/s)', flush=True)
qt, kt, vt = (x.transpose(1, 2).contiguous().requires_grad_() for x in (q, k, v))
dot = do.transpose(1, 2).contiguous()
from torch.nn.attention import SDPBackend, sdpa_kernel  # noqa: E402
for name, be in [('flash', SDPBackend.FLASH_ATTENTION), ('efficient', SDPBackend.EFFICIENT_ATTENTION)]:
    try:
        with sdpa_kernel(be):
            fw = lambda: torch.nn.functional.scaled_dot_product_attention(qt, kt, vt, is_causal=True)  # noqa
            tf2 = t(fw)
            out = fw()

            def fb():
                qt.grad = kt.grad = vt.grad = None
                torch.nn.functional.scaled_dot_product_attention(qt, kt, vt, is_causal=True).backward(dot)
            tfb = t(fb)
        print(f'{name:9s} fwd {tf2*1e6:7.1f} us ({f_fwd/tf2/1e12:6.1f} TF/s)  bwd~ {(tfb-tf2)*1e6:7.1f} us '
              f'({2.5*f_fwd/(tfb-tf2)/1e12:6.1f} TF/s)', flush=True)
    except Exception as e:  # noqa: BLE001
        print(name, 'unavailable:', str(e)[:200], flush=True)
