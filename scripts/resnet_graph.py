"""ResNet-50 NHWC bf16 training step: eager vs jit.to_static HIP-graph capture (forward and
backward replayed as two graphs). Same init and data; prints both losses and step times."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, '.')
import paddle_ray_amd as paddle  # noqa: E402
from paddle_ray_amd.vision.models import resnet50  # noqa: E402


def run(graph, steps, warm, bs):
    paddle.seed(0)
    model = resnet50(data_format='NHWC')
    model = paddle.amp.decorate(model, level='O2', dtype='bfloat16')
    if graph:
        st = paddle.static.BuildStrategy()
        st.use_hip_graph = True
        model = paddle.jit.to_static(model, build_strategy=st)
    opt = paddle.optimizer.Momentum(0.1, 0.9, parameters=model.parameters(), weight_decay=1e-4,
                                    multi_precision=True)
    g = torch.Generator(device='cuda').manual_seed(1)
    x = paddle.Tensor(torch.randn(bs, 224, 224, 3, device='cuda', dtype=torch.bfloat16, generator=g))
    y = paddle.Tensor(torch.randint(0, 1000, (bs,), device='cuda', generator=g))
    ce = paddle.nn.CrossEntropyLoss()
    losses = []

    def step():
        loss = ce(model(x), y)
        loss.backward()
        opt.step()
        opt.clear_grad()
        return loss

    for _ in range(warm):
        losses.append(float(step()))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    losses.append(float(loss))
    return losses, dt


if __name__ == '__main__':
    paddle.set_device('gpu')
    bs = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    le, te = run(False, 10, 4, bs)
    print(f"eager: {te * 1e3:.2f} ms/step {bs / te:.0f} img/s losses {le}", flush=True)
    lg, tg = run(True, 10, 4, bs)
    print(f"graph: {tg * 1e3:.2f} ms/step {bs / tg:.0f} img/s losses {lg}", flush=True)
