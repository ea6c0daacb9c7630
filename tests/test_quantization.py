"""paddle.quantization / paddle.nn.quant (parity: test/quantization/test_qat.py,
test_ptq.py, test_imperative_qat.py, test_imperative_ptq.py, test_fake_quantize_op.py)."""
import numpy as np
import pytest
import torch

import paddle_ray_amd as paddle
from paddle_ray_amd import nn
from paddle_ray_amd.ops import quant as Q
from paddle_ray_amd.quantization import (QAT, PTQ, QuantConfig, ImperativeQuantAware,
                                         ImperativePTQ, PTQConfig, KLQuantizer,
                                         HistQuantizer, AbsmaxQuantizer,
                                         PerChannelAbsmaxQuantizer, fuse_layers)
from paddle_ray_amd.quantization.quanters import FakeQuanterWithAbsMaxObserver
from paddle_ray_amd.quantization.observers import AbsmaxObserver
from paddle_ray_amd.quantization.imperative import cal_kl_threshold


def test_fake_quant_dequant_matches_formula():
    x = torch.randn(64, 32)
    s = x.abs().max()
    y = Q.fake_quant_dequant(x, s, bits=8)
    ref = torch.clamp(torch.round(x / s * 127), -128, 127) * s / 127
    torch.testing.assert_close(y, ref)
    assert (y - x).abs().max() <= s / 127 / 2 + 1e-6


def test_channel_wise_and_ste():
    x = torch.randn(8, 16, requires_grad=True)
    s = Q.absmax(x, axis=0)
    y = Q.fake_quant_dequant(x, s, 4, axis=0)
    y.sum().backward()
    assert torch.equal(x.grad, torch.ones_like(x))
    ref = torch.clamp(torch.round(x.detach() / s[:, None] * 7), -8, 7) * s[:, None] / 7
    torch.testing.assert_close(y.detach(), ref)


def test_fp8_e4m3_simulation():
    x = torch.randn(256)
    y = Q.fake_quant_dequant(x, x.abs().max(), fp8=True)
    rel = ((y - x).abs() / x.abs().clamp_min(1e-3)).max()
    assert rel < 0.07  # 3 mantissa bits


def test_quantize_dequantize_linear_roundtrip():
    x = torch.randn(100)
    s = x.abs().max()
    q = Q.quantize_linear(x, s)
    assert q.abs().max() <= 128
    torch.testing.assert_close(Q.dequantize_linear(q, s), Q.fake_quant_dequant(x, s))


def test_moving_average_scale():
    st, acc = torch.ones(1), torch.ones(1)
    s = Q.moving_average_update(st, acc, torch.tensor(3.0), 0.9)
    assert abs(float(s) - (0.9 + 3.0) / (0.9 + 1)) < 1e-6


class _Net(nn.Layer):
    def __init__(self):
        super().__init__()
        self.conv = nn.Conv2D(1, 4, 3, padding=1)
        self.relu = nn.ReLU()
        self.pool = nn.AdaptiveAvgPool2D(1)
        self.fc = nn.Linear(4, 3)

    def forward(self, x):
        h = self.pool(self.relu(self.conv(x)))
        return self.fc(paddle.flatten(h, 1))


def _data(n=32):
    paddle.seed(0)
    x = paddle.randn([n, 1, 6, 6])
    y = paddle.to_tensor(np.random.RandomState(0).randint(0, 3, (n,)))
    return x, y


def _train(model, steps=30):
    x, y = _data()
    opt = paddle.optimizer.Adam(learning_rate=0.05, parameters=model.parameters())
    losses = []
    for _ in range(steps):
        loss = nn.functional.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
    return losses


def test_qat_config_api_trains_and_converts():
    paddle.seed(1)
    model = _Net()
    q = FakeQuanterWithAbsMaxObserver(moving_rate=0.9)
    qat = QAT(QuantConfig(activation=q, weight=q))
    qm = qat.quantize(model)
    assert type(qm.fc).__name__ == 'QuantedLinear'
    assert type(qm.conv).__name__ == 'QuantedConv2D'
    losses = _train(qm)
    assert losses[-1] < losses[0]
    qm.eval()
    x, _ = _data(4)
    out_fake = qm(x).numpy()
    conv = qat.convert(qm)
    np.testing.assert_allclose(conv(x).numpy(), out_fake, rtol=1e-4, atol=1e-4)


def test_qat_requires_training_mode():
    m = _Net()
    m.eval()
    q = FakeQuanterWithAbsMaxObserver()
    with pytest.raises(RuntimeError):
        QAT(QuantConfig(activation=q, weight=q)).quantize(m)


def test_ptq_observers():
    model = _Net()
    model.eval()
    ptq = PTQ(QuantConfig(activation=AbsmaxObserver(), weight=AbsmaxObserver()))
    qm = ptq.quantize(model)
    x, _ = _data(8)
    ref = model(x).numpy()
    out = qm(x).numpy()
    assert np.abs(out - ref).max() < 0.1 * (np.abs(ref).max() + 1e-3)
    conv = ptq.convert(qm)
    assert conv(x).shape == [8, 3]


def test_imperative_qat(tmp_path):
    paddle.seed(2)
    model = _Net()
    iqa = ImperativeQuantAware(weight_quantize_type='channel_wise_abs_max')
    iqa.quantize(model)
    assert type(model.conv._layer).__name__ == 'QuantizedConv2D'
    assert type(model.fc._layer).__name__ == 'QuantizedLinear'
    losses = _train(model)
    assert losses[-1] < losses[0]
    iqa.save_quantized_model(model, str(tmp_path / 'qat'))
    import json
    scales = json.load(open(str(tmp_path / 'qat.quant.json')))['scales']
    assert any('_fake_quant_weight' in k for k in scales)


def test_imperative_qat_skip_quant():
    model = _Net()
    model.fc.skip_quant = True
    ImperativeQuantAware().quantize(model)
    assert type(model.fc).__name__ == 'Linear'


@pytest.mark.parametrize('act_q', [AbsmaxQuantizer, KLQuantizer, HistQuantizer])
def test_imperative_ptq(tmp_path, act_q):
    model = _Net()
    model.eval()
    ptq = ImperativePTQ(PTQConfig(act_q(), PerChannelAbsmaxQuantizer()))
    qm = ptq.quantize(model)
    x, _ = _data(16)
    ref = model(x).numpy()
    for i in range(4):
        qm(x[i * 4:(i + 1) * 4])
    qm = ptq.save_quantized_model(qm, str(tmp_path / 'ptq'))
    assert type(qm.fc).__name__ == 'QuantizedLinear'
    th = qm._ptq_thresholds
    assert th['fc']['in_threshold'][0] > 0 and len(th['conv']['weight_threshold'][0]) == 4
    out = qm(x).numpy()
    assert np.abs(out - ref).max() < 0.15 * (np.abs(ref).max() + 1e-3)


def test_kl_threshold_clips_outliers():
    rs = np.random.RandomState(0)
    data = np.abs(np.concatenate([rs.randn(100000), [9.0]]))
    hist, edges = np.histogram(data, bins=1024, range=(0, data.max()))
    t = cal_kl_threshold(hist, edges[1] - edges[0], 8)
    assert 4.4 < t < 8.9


def test_fuse_conv_bn_matches_eval():
    paddle.seed(3)
    m = nn.Sequential(nn.Conv2D(2, 4, 3), nn.BatchNorm2D(4))
    m.train()
    m(paddle.randn([8, 2, 5, 5]))  # populate running stats
    m.eval()
    x = paddle.randn([2, 2, 5, 5])
    ref = m(x).numpy()
    f = fuse_layers(m, [['0', '1']])
    np.testing.assert_allclose(f(x).numpy(), ref, rtol=1e-4, atol=1e-4)
    assert type(f[1]).__name__ == 'Identity'


def test_nn_quant_layers():
    from paddle_ray_amd.nn import quant as NQ
    x = paddle.randn([4, 8])
    fq = NQ.FakeQuantAbsMax(quant_bits=8)
    np.testing.assert_allclose(fq(x).numpy(), x.numpy(), atol=float(x.abs().max()) / 127)
    ma = NQ.FakeQuantMovingAverageAbsMax()
    ma.train()
    ma(x)
    assert float(ma._scale) > 0
    stub = NQ.QuantStub()
    assert stub(x).shape == [4, 8]
