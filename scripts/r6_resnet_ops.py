"""Which aten ops launch the at::native elementwise kernels in the ResNet-50 training step."""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import paddle_ray_amd as paddle  # noqa: E402
from paddle_ray_amd.vision.models import resnet50  # noqa: E402

paddle.set_device('gpu:0')
model = paddle.amp.decorate(resnet50(data_format='NHWC'), level='O2', dtype='bfloat16')
opt = paddle.optimizer.Momentum(0.1, 0.9, parameters=model.parameters(), weight_decay=1e-4, multi_precision=True)
x = paddle.Tensor(torch.randn(256, 224, 224, 3, device='cuda', dtype=torch.bfloat16))
y = paddle.Tensor(torch.randint(0, 1000, (256,), device='cuda'))
ce = paddle.nn.CrossEntropyLoss()


def step():
    loss = ce(model(x), y)
    loss.backward()
    opt.step()
    opt.clear_grad()


for _ in range(3):
    step()
torch.cuda.synchronize()
with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA],
                            record_shapes=True) as p:
    step()
    torch.cuda.synchronize()
cnt = collections.Counter()
for e in p.events():
    if e.device_type == torch.autograd.DeviceType.CUDA:
        continue
    for k in (getattr(e, 'kernels', None) or []):
        if 'at::native' in k.name:
            par = e
            chain = []
            while par is not None and len(chain) < 4:
                chain.append(par.name)
                par = par.cpu_parent
            cnt[(k.name.split('<')[0][-50:] + '|' + k.name.split('at::native::')[-1][:60], ' <- '.join(chain),
                 str(e.input_shapes)[:80])] += 1
for k, v in cnt.most_common(40):
    print(v, k)
