"""Which torch-profiler CPU events carry the device kernels of natively launched HIP kernels?"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import paddle_ray_amd as paddle  # noqa: E402
from paddle_ray_amd.models import gpt_config, GPTForPretraining  # noqa: E402

paddle.set_device('gpu:0')
paddle.set_default_dtype('bfloat16')
model = GPTForPretraining(gpt_config('gpt3-tiny'))
paddle.set_default_dtype('float32')
opt = paddle.optimizer.AdamW(1e-3, parameters=model.parameters(), multi_precision=True)
ids = paddle.randint(0, 1024, [4, 129])


def step():
    loss = model(ids[:, :-1], ids[:, 1:])
    loss.backward()
    with torch.profiler.record_function('OPT_RANGE'):
        opt.step()
    opt.clear_grad()


step()
torch.cuda.synchronize()
with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]) as p:
    step()
    torch.cuda.synchronize()
evs = p.events()
cnt = collections.Counter()
for e in evs:
    if getattr(e, 'kernels', None) and e.device_type != torch.autograd.DeviceType.CUDA:
        cnt[(e.name, bool(e.name.startswith('aten::')))] += 1
for k, v in cnt.most_common(20):
    print('withkernels', v, k)
for e in evs:
    if e.name == 'OPT_RANGE':
        print('OPT_RANGE device_time_total', e.device_time_total, 'children', [c.name for c in e.cpu_children][:10])
adam = [e for e in evs if 'adamw' in e.name.lower()]
for e in adam[:5]:
    print('adam event', e.name, e.device_type, getattr(e, 'device_time_total', None))
names = collections.Counter(e.name for e in evs if e.device_type != torch.autograd.DeviceType.CUDA and not e.name.startswith('aten::'))
print('non-aten cpu names', names.most_common(15))
