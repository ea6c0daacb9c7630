"""Debug: capture the flash_attention_ext call inside the GPU TransformerEncoderLayer and compare
it with the fp32 reference at the same seed; then per-batch layer errors vs the host copy."""
import copy
import sys

import numpy as np
import torch

sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import paddle_ray_amd as paddle  # noqa: E402
from paddle_ray_amd.ops import fused as K  # noqa: E402
from paddle_ray_amd.nn.layer import transformer as TR  # noqa: E402

cap = []
orig_ext = K.flash_attention_ext
orig_rng = K._fa_next_rng


def rng(seed=None, numel=1):
    r = orig_rng(seed, numel)
    cap.append(('rng', r))
    return r


def ext(q, k, v, causal=False, scale=None, attn_mask=None, dropout=0.0, seed=None):
    o = orig_ext(q, k, v, causal, scale, attn_mask, dropout, seed)
    cap.append(('ext', q.detach().clone(), k.detach().clone(), v.detach().clone(),
                None if attn_mask is None else attn_mask.detach().clone(), dropout, o.detach().clone(),
                q.stride(), attn_mask.stride() if attn_mask is not None else None))
    return o


K._fa_next_rng = rng
K.flash_attention_ext = ext
B, S = 2, 128
paddle.seed(21)
layer = paddle.nn.TransformerEncoderLayer(256, 4, 512, dropout=0.0, attn_dropout=0.2)
layer.train()
ref = copy.deepcopy(layer)
layer.to(device='gpu', dtype='bfloat16')
x = paddle.randn([B, S, 256])
mk = np.zeros((B, 1, 1, S), 'float32')
mk[1, ..., 100:] = -1e9
xg = paddle.to_tensor(x.numpy(), place='gpu').astype('bfloat16')
mg = paddle.to_tensor(mk, place='gpu').astype('bfloat16')
paddle.seed(77)
y = layer(xg, mg)
gpu_cap = list(cap)
cap.clear()
paddle.seed(77)
yr = ref(paddle.to_tensor(x.numpy()), paddle.to_tensor(mk))
cpu_cap = list(cap)
print("gpu rng:", [c[1] for c in gpu_cap if c[0] == 'rng'], "cpu rng:", [c[1] for c in cpu_cap if c[0] == 'rng'])
ge = [c for c in gpu_cap if c[0] == 'ext'][0]
ce = [c for c in cpu_cap if c[0] == 'ext'][0]
print("gpu q stride", ge[7], "mask stride", ge[8], "mask dtype", ge[4].dtype, "cpu q stride", ce[7])
sd = [c[1] for c in gpu_cap if c[0] == 'rng'][0][0]
orf, _ = K._fa_ext_ref_dense(ge[1].float().cpu(), ge[2].float().cpu(), ge[3].float().cpu(), False, 1 / 8.0,
                             ge[4].float().cpu(), ge[5], sd, 0)
print("captured gpu call vs ref at its seed: max err", (ge[6].float().cpu() - orf).abs().max().item())
print("gpu ext out vs cpu ext out: max err", (ge[6].float().cpu() - ce[6]).abs().max().item(),
      "inputs q err", (ge[1].float().cpu() - ce[1]).abs().max().item())
d = np.abs(y.astype('float32').numpy() - yr.numpy())
print("layer per-batch max err", d.reshape(B, -1).max(1))
