"""Debug: host seed draws of the GPU TransformerEncoderLayer forward, and the extended flash
kernel vs its fp32 reference at a 62-bit seed (the size _dropout_seed draws)."""
import sys

import numpy as np
import torch

sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import paddle_ray_amd as paddle  # noqa: E402
from paddle_ray_amd.ops import fused as K  # noqa: E402

calls = []
orig = K._dropout_seed


def spy():
    v = orig()
    calls.append(v)
    return v


K._dropout_seed = spy
torch.manual_seed(0)
B, S, H, D = 2, 128, 4, 64
q, k, v = (torch.randn(B, S, H, D) for _ in range(3))
m = torch.zeros(B, 1, 1, S)
m[1, ..., 100:] = -1e9
for sd in (12345, 3119511124627235423, (1 << 31) + 7, (1 << 40) + 3):
    og = K.flash_attention_ext(*(t.cuda().bfloat16() for t in (q, k, v)), attn_mask=m.cuda().bfloat16(), dropout=0.2,
                               seed=sd)
    orf, _ = K._fa_ext_ref_dense(q, k, v, False, 1 / 8.0, m, 0.2, sd, 0)
    print(f"seed {sd}: max err {(og.float().cpu() - orf).abs().max().item():.4f}", flush=True)
paddle.seed(21)
layer = paddle.nn.TransformerEncoderLayer(256, 4, 512, dropout=0.0, attn_dropout=0.2)
layer.train()
layer.to(device='gpu', dtype='bfloat16')
x = paddle.randn([B, S, 256])
mk = np.zeros((B, 1, 1, S), 'float32')
mk[1, ..., 100:] = -1e9
xg = paddle.to_tensor(x.numpy(), place='gpu').astype('bfloat16')
mg = paddle.to_tensor(mk, place='gpu').astype('bfloat16')
paddle.seed(77)
y = layer(xg, mg)
print("GPU forward draws:", calls, flush=True)
paddle.seed(77)
print("expected first draws:", [int(torch.randint(0, 2 ** 62, (1,)).item()) for _ in range(2)])
