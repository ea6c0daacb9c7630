"""Which op breaks the HIP-graph training capture of the NHWC ResNet-50 step (prints the
capture status / failure reason of jit.to_static)."""
import os
import sys
import traceback

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import paddle_ray_amd as paddle  # noqa: E402
from paddle_ray_amd.vision.models import resnet50  # noqa: E402

bs = int(sys.argv[1]) if len(sys.argv) > 1 else 16
paddle.set_device('gpu:0')
model = resnet50(data_format='NHWC')
model = paddle.amp.decorate(model, level='O2', dtype='bfloat16')
st = paddle.static.BuildStrategy()
st.use_hip_graph = True
model = paddle.jit.to_static(model, build_strategy=st)
x = paddle.Tensor(torch.randn(bs, 224, 224, 3, device='cuda', dtype=torch.bfloat16))
y = paddle.Tensor(torch.randint(0, 1000, (bs,), device='cuda'))
ce = paddle.nn.CrossEntropyLoss()
sf = model.forward
orig = sf._capture


def cap(key, build):
    try:
        g = build()
        sf._graphs[key] = g
        return g
    except Exception:
        traceback.print_exc()
        raise
sf._capture = cap
try:
    loss = ce(model(x), y)
    loss.backward()
    torch.cuda.synchronize()
    print("status", sf.graph_status(), "loss", float(loss))
except Exception:
    traceback.print_exc()
