"""Debug: flash_attention_ext on the device vs its fp32 host reference at the MHA test's shapes,
then nn.TransformerEncoderLayer GPU bf16 vs host fp32 with and without attention dropout."""
import copy
import sys

import numpy as np
import torch

sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import paddle_ray_amd as paddle  # noqa: E402
from paddle_ray_amd.ops import fused as K  # noqa: E402

torch.manual_seed(0)
B, S, H, D = 2, 128, 4, 64
q, k, v = (torch.randn(B, S, H, D) for _ in range(3))
m = torch.zeros(B, 1, 1, S)
m[1, ..., 100:] = -1e9
for p in (0.0, 0.2):
    og = K.flash_attention_ext(*(t.cuda().bfloat16() for t in (q, k, v)), attn_mask=m.cuda().bfloat16(), dropout=p,
                               seed=12345)
    orf, _ = K._fa_ext_ref_dense(q, k, v, False, 1 / 8.0, m, p, 12345, 0)
    print(f"ext p={p}: max err {(og.float().cpu() - orf).abs().max().item():.4f} (ref max {orf.abs().max().item():.3f})")
for drop in (0.0, 0.2):
    paddle.seed(21)
    layer = paddle.nn.TransformerEncoderLayer(256, 4, 512, dropout=0.0, attn_dropout=drop)
    layer.train()
    ref = copy.deepcopy(layer)
    layer.to(device='gpu', dtype='bfloat16')
    x = paddle.randn([B, S, 256])
    mk = np.zeros((B, 1, 1, S), 'float32')
    mk[1, ..., 100:] = -1e9
    paddle.seed(77)
    y = layer(paddle.to_tensor(x.numpy(), place='gpu').astype('bfloat16'),
              paddle.to_tensor(mk, place='gpu').astype('bfloat16'))
    s1 = torch.randint(0, 2 ** 62, (1,)).item()
    paddle.seed(77)
    yr = ref(paddle.to_tensor(x.numpy()), paddle.to_tensor(mk))
    s2 = torch.randint(0, 2 ** 62, (1,)).item()
    print(f"layer attn_dropout={drop}: max err {np.abs(y.astype('float32').numpy() - yr.numpy()).max():.4f} "
          f"(ref max {np.abs(yr.numpy()).max():.3f}); next host draws equal: {s1 == s2}")
