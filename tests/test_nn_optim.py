"""nn.Layer / functional / autograd / optimizers / AMP / checkpoint (CPU)."""
import os

import numpy as np
import pytest
import torch

import paddle_ray_amd as paddle
import paddle_ray_amd.nn as nn
import paddle_ray_amd.nn.functional as F


def A(x):
    return x.numpy()


def test_layer_params_and_state_dict(tmp_path):
    class Net(nn.Layer):
        def __init__(self):
            super().__init__()
            self.fc1 = nn.Linear(4, 8)
            self.bn = nn.BatchNorm1D(8)
            self.fc2 = nn.Linear(8, 2, bias_attr=False)

        def forward(self, x):
            return self.fc2(F.relu(self.bn(self.fc1(x))))

    net = Net()
    names = [n for n, _ in net.named_parameters()]
    assert names == ['fc1.weight', 'fc1.bias', 'bn.weight', 'bn.bias', 'fc2.weight']
    assert net.fc1.weight.shape == [4, 8]  # paddle [in, out] layout
    sd = net.state_dict()
    assert 'bn._mean' in sd and 'bn._variance' in sd
    paddle.save(sd, str(tmp_path / 'm.pdparams'))
    net2 = Net()
    missing, unexpected = net2.set_state_dict(paddle.load(str(tmp_path / 'm.pdparams')))
    assert not missing and not unexpected
    x = paddle.randn([3, 4])
    net.eval()
    net2.eval()
    np.testing.assert_allclose(A(net(x)), A(net2(x)), rtol=1e-6)
    assert len(net.sublayers()) == 3
    net.train()
    assert net.bn.training


def test_linear_matches_numpy_and_grad():
    lin = nn.Linear(3, 2)
    x = paddle.to_tensor(np.random.rand(5, 3).astype('float32'), stop_gradient=False)
    y = lin(x)
    np.testing.assert_allclose(A(y), A(x) @ A(lin.weight) + A(lin.bias), rtol=1e-5)
    y.sum().backward()
    np.testing.assert_allclose(A(lin.weight.grad), A(x).sum(0)[:, None].repeat(2, 1), rtol=1e-5)
    np.testing.assert_allclose(A(x.grad), A(lin.weight).sum(1)[None].repeat(5, 0), rtol=1e-5)
    lin.clear_gradients()
    assert float(lin.weight.grad.abs().sum()) == 0


def test_functional_ops_vs_torch():
    a = torch.randn(4, 10)
    x = paddle.to_tensor(a.numpy())
    np.testing.assert_allclose(A(F.softmax(x)), torch.softmax(a, -1).numpy(), rtol=1e-5)
    np.testing.assert_allclose(A(F.gelu(x)), torch.nn.functional.gelu(a).numpy(), rtol=1e-5,
                               atol=1e-6)
    np.testing.assert_allclose(A(F.gelu(x, approximate=True)),
                               torch.nn.functional.gelu(a, approximate='tanh').numpy(), rtol=1e-5,
                               atol=1e-6)
    w, b = paddle.ones([10]), paddle.zeros([10])
    np.testing.assert_allclose(A(F.layer_norm(x, 10, w, b)),
                               torch.nn.functional.layer_norm(a, (10,)).numpy(), rtol=1e-4,
                               atol=1e-5)
    lab = torch.randint(0, 10, (4,))
    ce = F.cross_entropy(x, paddle.to_tensor(lab.numpy()))
    np.testing.assert_allclose(float(ce), float(torch.nn.functional.cross_entropy(a, lab)),
                               rtol=1e-5)
    ce2 = F.cross_entropy(x, paddle.to_tensor(lab.numpy()[:, None]))
    np.testing.assert_allclose(float(ce2), float(ce), rtol=1e-6)
    sce = F.softmax_with_cross_entropy(x, paddle.to_tensor(lab.numpy()[:, None]))
    assert sce.shape == [4, 1]
    img = paddle.randn([2, 3, 8, 8])
    assert F.conv2d(img, paddle.randn([5, 3, 3, 3]), padding=1).shape == [2, 5, 8, 8]
    assert F.max_pool2d(img, 2).shape == [2, 3, 4, 4]
    assert F.adaptive_avg_pool2d(img, 1).shape == [2, 3, 1, 1]
    assert F.interpolate(img, scale_factor=2).shape == [2, 3, 16, 16]
    assert F.pad(img, [1, 1, 2, 2]).shape == [2, 3, 12, 10]
    assert F.one_hot(paddle.to_tensor([0, 2]), 3).shape == [2, 3]
    d = F.dropout(paddle.ones([1000]), 0.5, training=True)
    assert 300 < float((d == 0).sum()) < 700


def test_rms_norm_and_ln_grad():
    x = paddle.randn([6, 16])
    x.stop_gradient = False
    ln = nn.LayerNorm(16)
    y = ln(x)
    y.sum().backward()
    xt = torch.tensor(x.numpy(), requires_grad=True)
    torch.nn.functional.layer_norm(xt, (16,)).sum().backward()
    np.testing.assert_allclose(A(x.grad), xt.grad.numpy(), atol=1e-5)
    r = nn.RMSNorm(16)
    assert r(x).shape == [6, 16]


def test_conv_bn_pool_layers():
    m = nn.Sequential(nn.Conv2D(3, 8, 3, padding=1), nn.BatchNorm2D(8), nn.ReLU(),
                      nn.MaxPool2D(2), nn.Flatten(), nn.Linear(8 * 4 * 4, 10))
    y = m(paddle.randn([2, 3, 8, 8]))
    assert y.shape == [2, 10]
    y.mean().backward()
    assert m[0].weight.grad is not None
    nhwc = nn.Conv2D(3, 4, 3, padding=1, data_format='NHWC')
    assert nhwc(paddle.randn([1, 8, 8, 3])).shape == [1, 8, 8, 4]


def test_rnn_layers():
    lstm = nn.LSTM(8, 16, num_layers=2, direction='bidirect')
    y, (h, c) = lstm(paddle.randn([4, 5, 8]))
    assert y.shape == [4, 5, 32] and h.shape == [4, 4, 16]
    gru = nn.GRU(8, 16)
    y, h = gru(paddle.randn([2, 3, 8]))
    assert y.shape == [2, 3, 16]
    cell = nn.LSTMCell(8, 16)
    rnn = nn.RNN(cell)
    y, (h, c) = rnn(paddle.randn([2, 3, 8]))
    assert y.shape == [2, 3, 16]


def test_transformer_layers():
    enc = nn.TransformerEncoder(nn.TransformerEncoderLayer(32, 4, 64, dropout=0.0), 2)
    x = paddle.randn([2, 5, 32])
    assert enc(x).shape == [2, 5, 32]
    mha = nn.MultiHeadAttention(32, 4)
    mask = paddle.zeros([2, 4, 5, 5])
    assert mha(x, x, x, mask).shape == [2, 5, 32]
    t = nn.Transformer(32, 4, 1, 1, 64, dropout=0.0)
    assert t(x, paddle.randn([2, 3, 32])).shape == [2, 3, 32]


def test_autograd_grad_and_pylayer():
    x = paddle.to_tensor([2.0, 3.0], stop_gradient=False)
    y = (x * x).sum()
    (g,) = paddle.grad(y, x, create_graph=True)
    np.testing.assert_allclose(A(g), [4., 6.])

    class Cube(paddle.autograd.PyLayer):
        @staticmethod
        def forward(ctx, t):
            ctx.save_for_backward(t)
            return t ** 3

        @staticmethod
        def backward(ctx, dy):
            (t,) = ctx.saved_tensor()
            return dy * 3 * t ** 2

    z = paddle.to_tensor([1.0, 2.0], stop_gradient=False)
    Cube.apply(z).sum().backward()
    np.testing.assert_allclose(A(z.grad), [3., 12.])
    with paddle.no_grad():
        w = z * 2
    assert w.stop_gradient


@pytest.mark.parametrize('opt_name', ['SGD', 'Momentum', 'Adam', 'AdamW', 'Adagrad', 'RMSProp',
                                      'Adamax', 'Adadelta', 'Lamb'])
def test_optimizers_reduce_loss(opt_name):
    paddle.seed(0)
    net = nn.Linear(4, 1)
    x = paddle.randn([32, 4])
    y = paddle.matmul(x, paddle.to_tensor([[1.], [-2.], [3.], [0.5]]))
    kw = dict(parameters=net.parameters())
    if opt_name == 'Adadelta':
        kw['epsilon'] = 1e-2  # adadelta's step size is sqrt(eps)-driven early on
    lr = {'SGD': 0.1, 'Momentum': 0.05, 'Adagrad': 0.5, 'RMSProp': 0.05, 'Adadelta': 1.0}.get(
        opt_name, 0.05)
    opt = getattr(paddle.optimizer, opt_name)(learning_rate=lr, **kw)
    losses = []
    for _ in range(60):
        loss = F.mse_loss(net(x), y)
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
    assert losses[-1] < losses[0] * 0.5, (opt_name, losses[0], losses[-1])


def test_adamw_matches_torch():
    paddle.seed(1)
    w0 = np.random.rand(5, 3).astype('float32')
    p = paddle.create_parameter([5, 3], 'float32',
                                default_initializer=paddle.nn.initializer.Assign(w0))
    opt = paddle.optimizer.AdamW(0.01, parameters=[p], weight_decay=0.1)
    tp = torch.nn.Parameter(torch.tensor(w0))
    topt = torch.optim.AdamW([tp], lr=0.01, weight_decay=0.1)
    for i in range(5):
        g = np.random.rand(5, 3).astype('float32')
        p.grad = paddle.to_tensor(g)
        opt.step()
        tp.grad = torch.tensor(g)
        topt.step()
    np.testing.assert_allclose(A(p), tp.detach().numpy(), rtol=1e-5, atol=1e-6)


def test_grad_clip_global_norm():
    p = paddle.create_parameter([4], 'float32')
    p.grad = paddle.to_tensor([3., 4., 0., 0.])
    opt = paddle.optimizer.SGD(1.0, parameters=[p], grad_clip=nn.ClipGradByGlobalNorm(1.0))
    before = p.numpy().copy()
    opt.step()
    np.testing.assert_allclose(before - p.numpy(), [0.6, 0.8, 0, 0], rtol=1e-5)


def test_optimizer_state_dict_roundtrip(tmp_path):
    net = nn.Linear(3, 3)
    sched = paddle.optimizer.lr.StepDecay(0.1, 2)
    opt = paddle.optimizer.Adam(sched, parameters=net.parameters())
    net(paddle.randn([2, 3])).sum().backward()
    opt.step()
    sched.step()
    paddle.save(opt.state_dict(), str(tmp_path / 'o.pdopt'))
    opt2 = paddle.optimizer.Adam(paddle.optimizer.lr.StepDecay(0.1, 2),
                                 parameters=net.parameters())
    opt2.set_state_dict(paddle.load(str(tmp_path / 'o.pdopt')))
    k = f'{net.weight.name}_moment1_0'
    np.testing.assert_allclose(opt2._accumulators['moment1'][net.weight.name].numpy(),
                               opt._accumulators['moment1'][net.weight.name].numpy())
    assert opt2._learning_rate.last_epoch == 1


def test_lr_schedulers():
    s = paddle.optimizer.lr.LinearWarmup(0.1, 5, 0.0, 0.1)
    vals = []
    for _ in range(7):
        vals.append(s())
        s.step()
    assert vals[0] == 0.0 and abs(vals[5] - 0.1) < 1e-9
    c = paddle.optimizer.lr.CosineAnnealingDecay(1.0, 10)
    for _ in range(10):
        c.step()
    assert c() < 0.05
    p = paddle.optimizer.lr.PiecewiseDecay([2, 4], [1.0, 0.5, 0.1])
    out = []
    for _ in range(5):
        out.append(p())
        p.step()
    assert out == [1.0, 1.0, 0.5, 0.5, 0.1]
    r = paddle.optimizer.lr.ReduceOnPlateau(1.0, patience=1)
    for m in [1, 1, 1, 1]:
        r.step(m)
    assert r() < 1.0
    oc = paddle.optimizer.lr.OneCycleLR(1.0, 10)
    assert oc() < 1.0


def test_amp_autocast_and_scaler():
    net = nn.Linear(4, 4)
    opt = paddle.optimizer.SGD(0.1, parameters=net.parameters())
    scaler = paddle.amp.GradScaler(init_loss_scaling=1024)
    with paddle.amp.auto_cast(dtype='bfloat16'):
        loss = net(paddle.randn([2, 4])).mean()
    scaled = scaler.scale(loss)
    scaled.backward()
    scaler.step(opt)
    scaler.update()
    assert scaler.get_loss_scaling() == 1024
    m2 = paddle.amp.decorate(nn.Linear(4, 4), level='O2', dtype='bfloat16')
    assert m2.weight.dtype == paddle.bfloat16


def test_initializers():
    w = paddle.create_parameter([100, 100], 'float32',
                                default_initializer=nn.initializer.Normal(0, 0.02))
    assert abs(float(w.std()) - 0.02) < 0.002
    c = paddle.create_parameter([3], 'float32', default_initializer=nn.initializer.Constant(2.))
    np.testing.assert_allclose(c.numpy(), [2, 2, 2])
    k = paddle.create_parameter([64, 32, 3, 3], 'float32',
                                default_initializer=nn.initializer.KaimingNormal())
    assert abs(float(k.std()) - np.sqrt(2 / (32 * 9))) < 0.01


def test_save_load_nested_and_bf16(tmp_path):
    obj = {'a': paddle.to_tensor([1., 2.]).astype('bfloat16'), 'b': [paddle.ones([2]), 3],
           'c': {'d': np.arange(3)}}
    paddle.save(obj, str(tmp_path / 'x.pd'))
    back = paddle.load(str(tmp_path / 'x.pd'))
    assert back['a'].dtype == paddle.bfloat16
    np.testing.assert_allclose(back['a'].numpy(), [1., 2.])
    assert back['b'][1] == 3
    r = paddle.load(str(tmp_path / 'x.pd'), return_numpy=True)
    assert isinstance(r['b'][0], np.ndarray)


def test_safe_loader_refuses_code(tmp_path):
    import pickle

    class Evil:
        def __reduce__(self):
            return (os.system, ('echo pwned',))
    with open(tmp_path / 'evil.pdparams', 'wb') as f:
        pickle.dump({'x': Evil()}, f)
    with pytest.raises(pickle.UnpicklingError):
        paddle.load(str(tmp_path / 'evil.pdparams'))


def test_linear_fused_wgrad_accumulation_matches():
    """LinearFn accumulates dW into an existing .grad (beta=1 GEMM) and fires hooks."""
    import torch
    from paddle_ray_amd.ops import fused as K
    torch.manual_seed(0)
    x = torch.randn(6, 5, 4, requires_grad=True)
    w = torch.randn(4, 3, requires_grad=True)
    b = torch.randn(3, requires_grad=True)
    fired = []
    w.register_post_accumulate_grad_hook(lambda t: fired.append(1))
    w.grad = torch.full_like(w, 0.5)  # pre-existing grad (flat buffer / micro-batch accum)
    K.linear(x, w, b).square().sum().backward()
    xr, wr, br = (t.detach().clone().requires_grad_() for t in (x, w, b))
    (xr @ wr + br).square().sum().backward()
    torch.testing.assert_close(w.grad, wr.grad + 0.5)
    torch.testing.assert_close(x.grad, xr.grad)
    torch.testing.assert_close(b.grad, br.grad)
    assert fired == [1]


def test_fused_bn_add_act_matches_composition():
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn.functional as F
    paddle.seed(0)
    bn = paddle.nn.BatchNorm2D(16, data_format='NHWC')
    bn2 = paddle.nn.BatchNorm2D(16, data_format='NHWC')
    bn2.set_state_dict(bn.state_dict())
    x = paddle.randn([4, 5, 5, 16])
    z = paddle.randn([4, 5, 5, 16])
    x.stop_gradient = False
    y1 = F.fused_bn_add_act(x, z, bn._mean, bn._variance, bn.weight, bn.bias, True, 0.9, 1e-5,
                            'relu', 'NHWC')
    y2 = F.relu(bn2(x) + z)
    np.testing.assert_allclose(y1.numpy(), y2.numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(bn._mean.numpy(), bn2._mean.numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(bn._variance.numpy(), bn2._variance.numpy(), rtol=1e-5, atol=1e-6)
    g1 = paddle.grad(y1.sum(), [x])[0]
    g2 = paddle.grad(y2.sum(), [x])[0]
    np.testing.assert_allclose(g1.numpy(), g2.numpy(), rtol=1e-4, atol=1e-5)
