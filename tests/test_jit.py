"""paddle.jit: to_static keeps eager semantics, program export, save/load round trip
(parity: test/dygraph_to_static/test_save_load.py, test_jit_save_load.py)."""
import numpy as np
import pytest

import paddle_ray_amd as paddle
import paddle_ray_amd.nn as nn
import paddle_ray_amd.nn.functional as F
from paddle_ray_amd.static import InputSpec


class Net(nn.Layer):
    def __init__(self):
        super().__init__()
        self.conv = nn.Conv2D(3, 8, 3, padding=1)
        self.bn = nn.BatchNorm2D(8)
        self.fc = nn.Linear(8 * 4 * 4, 10)
        self.drop = nn.Dropout(0.5)

    def forward(self, x):
        h = F.relu(self.bn(self.conv(x)))
        h = F.adaptive_avg_pool2d(h, 4)
        return F.softmax(self.fc(self.drop(paddle.flatten(h, 1))), -1)


def test_to_static_eager_semantics_and_training():
    paddle.seed(0)
    net = Net()
    st = paddle.jit.to_static(net)
    x = paddle.randn([2, 3, 8, 8])
    out = st(x)
    assert out.shape == [2, 10]
    out.sum().backward()
    assert net.fc.weight.grad is not None


def test_to_static_decorator_on_method():
    class M(nn.Layer):
        def __init__(self):
            super().__init__()
            self.l = nn.Linear(4, 4)

        @paddle.jit.to_static(input_spec=[InputSpec([None, 4], 'float32')])
        def forward(self, x):
            return self.l(x) * 2
    m = M()
    x = paddle.randn([3, 4])
    np.testing.assert_allclose(m(x).numpy(), (m.l(x) * 2).numpy(), rtol=1e-6)
    prog = m.forward.main_program
    assert len(prog.global_block().ops) >= 2


def test_jit_save_load_roundtrip(tmp_path):
    paddle.seed(1)
    net = Net()
    net.eval()
    x = paddle.randn([4, 3, 8, 8])
    ref = net(x).numpy()
    path = str(tmp_path / 'net' / 'inference')
    paddle.jit.save(net, path, input_spec=[InputSpec([None, 3, 8, 8], 'float32', 'img')])
    loaded = paddle.jit.load(path)
    np.testing.assert_allclose(loaded(x).numpy(), ref, rtol=1e-5, atol=1e-6)
    # fine-tune the translated layer
    opt = paddle.optimizer.SGD(0.1, parameters=loaded.parameters())
    loss = loaded(x).sum()
    loss.backward()
    opt.step()
    assert len(loaded.parameters()) == len(net.parameters())


def test_static_function_plain_fn():
    @paddle.jit.to_static
    def f(a, b):
        return paddle.matmul(a, b) + 1
    a, b = paddle.randn([2, 3]), paddle.randn([3, 2])
    np.testing.assert_allclose(f(a, b).numpy(), (paddle.matmul(a, b) + 1).numpy(), rtol=1e-6)
    prog, feeds, fetches = f.get_concrete_program(InputSpec([2, 3]), InputSpec([3, 2]))
    assert fetches[0].shape == [2, 2]


@pytest.mark.gpu
def test_to_static_hip_graph_replay():
    paddle.set_device('gpu')
    paddle.seed(0)
    net = Net()
    net.eval()
    st = paddle.jit.to_static(Net())
    st.set_state_dict(net.state_dict())
    st.eval()
    with paddle.no_grad():
        for bs in (2, 4, 2):
            x = paddle.randn([bs, 3, 8, 8])
            np.testing.assert_allclose(st(x).numpy(), net(x).numpy(), rtol=1e-4, atol=1e-5)
    assert len(st.forward._graphs) == 2


def test_inference_predictor(tmp_path):
    from paddle_ray_amd import inference
    paddle.seed(2)
    net = Net()
    net.eval()
    path = str(tmp_path / 'm')
    paddle.jit.save(net, path, input_spec=[InputSpec([None, 3, 8, 8], 'float32', 'img')])
    cfg = inference.Config(path + '.pdmodel', path + '.pdiparams')
    pred = inference.create_predictor(cfg)
    assert pred.get_input_names() == ['img']
    x = np.random.RandomState(0).rand(2, 3, 8, 8).astype('float32')
    pred.get_input_handle('img').copy_from_cpu(x)
    pred.run()
    out = pred.get_output_handle(pred.get_output_names()[0]).copy_to_cpu()
    np.testing.assert_allclose(out, net(paddle.to_tensor(x)).numpy(), rtol=1e-5, atol=1e-6)
