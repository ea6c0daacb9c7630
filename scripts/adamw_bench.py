"""Multi-tensor AdamW kernel on a GPT-3 1.3B-sized parameter set (bf16 params + grads, fp32
master/m/v: 28 B per parameter per step). Prints kernel time and achieved HBM bandwidth."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_ray_amd.ops.fused import MultiTensorAdamW  # noqa: E402

sizes = [50304 * 2048] + [2048 * 6144, 2048 * 2048, 2048 * 8192, 8192 * 2048] * 24 + [2048 * 3] * 100
dev = 'cuda'
ps = [torch.randn(n, device=dev).to(torch.bfloat16) for n in sizes]
gs = [torch.randn(n, device=dev).to(torch.bfloat16) for n in sizes]
ms = [torch.zeros(n, device=dev) for n in sizes]
vs = [torch.zeros(n, device=dev) for n in sizes]
masters = [p.float() for p in ps]
opt = MultiTensorAdamW(ps, lambda: gs, ms, vs, masters, [0.01] * len(sizes), [1.0] * len(sizes))
for i in range(3):
    opt.step(1e-4, 0.9, 0.95, 1e-8, i + 1)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
it = 10
s.record()
for i in range(it):
    opt.step(1e-4, 0.9, 0.95, 1e-8, i + 4)
e.record()
torch.cuda.synchronize()
ms_ = s.elapsed_time(e) / it
n = sum(sizes)
print(f"params {n / 1e9:.3f} B: {ms_:.3f} ms/step, {28 * n / ms_ / 1e9:.2f} TB/s", flush=True)
