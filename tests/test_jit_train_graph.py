"""to_static training capture: forward + backward of a layer replayed as two HIP graphs
(build_strategy.use_hip_graph) trains exactly like eager execution."""
import numpy as np
import pytest

import paddle_ray_amd as paddle
import paddle_ray_amd.nn as nn
import paddle_ray_amd.nn.functional as F


class _Net(nn.Layer):
    def __init__(self):
        super().__init__()
        self.l1 = nn.Linear(64, 128)
        self.ln = nn.LayerNorm(128)
        self.l2 = nn.Linear(128, 10)

    def forward(self, x):
        return self.l2(F.gelu(self.ln(self.l1(x))))


def _run(use_graph, steps=6):
    paddle.seed(0)
    net = _Net()
    if use_graph:
        bs = paddle.static.BuildStrategy()
        bs.use_hip_graph = True
        net = paddle.jit.to_static(net, build_strategy=bs)
    opt = paddle.optimizer.AdamW(1e-2, parameters=net.parameters())
    rs = np.random.RandomState(0)
    xs = rs.randn(32, 64).astype('float32')
    ys = rs.randint(0, 10, (32,)).astype('int64')
    losses = []
    for _ in range(steps):
        x, y = paddle.to_tensor(xs), paddle.to_tensor(ys)  # fresh tensors each step
        loss = F.cross_entropy(net(x), y)
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
    return losses, net


@pytest.mark.gpu
def test_to_static_training_graph_matches_eager():
    paddle.set_device('gpu')
    eager, _ = _run(False)
    graph, net = _run(True)
    np.testing.assert_allclose(graph, eager, rtol=2e-4, atol=2e-5)
    assert graph[-1] < graph[0]
    sf = net.forward
    assert len(sf._graphs) == 1 and next(iter(sf._graphs))[0] == 'train'
