"""AdamW (multi-precision, bf16 params + grads, fp32 master / moments) over GPT-1.3B-sized
parameters: ms per step.   PRA_ADAMW_X2={0,1} python scripts/r6_adamw_ab.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import paddle_ray_amd as paddle  # noqa: E402

paddle.set_device('gpu:0')
shapes = [(50304, 2048)] + [(2048, 6144), (6144,), (2048, 2048), (2048,), (2048, 8192), (8192,), (8192, 2048),
                            (2048,), (2048,), (2048,), (2048,), (2048,)] * 24
ps = []
for s in shapes:
    p = paddle.create_parameter(list(s), 'bfloat16')
    p._t.grad = torch.randn(s, device='cuda', dtype=torch.bfloat16) * 1e-3
    ps.append(p)
n = sum(p._t.numel() for p in ps)
opt = paddle.optimizer.AdamW(1e-4, parameters=ps, multi_precision=True,
                             grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
for _ in range(3):
    opt.step()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts = []
for _ in range(5):
    s.record()
    for _ in range(5):
        opt.step()
    e.record()
    torch.cuda.synchronize()
    ts.append(s.elapsed_time(e) / 5)
ts.sort()
print(f"X2={os.environ.get('PRA_ADAMW_X2', '1')} params={n / 1e9:.3f}B adamw step median {ts[2]:.3f} ms "
      f"({30 * n / (ts[2] * 1e-3) / 1e12:.2f} TB/s at 30 B/param)", flush=True)
