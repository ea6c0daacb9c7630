"""incubate.operators.ResNetUnit / resnet_unit / unzip (reference: python/paddle/fluid/tests/
unittests/ir/test_fuse_resnet_unit.py compares the fused unit against conv2d + batch_norm
(+ add) + relu; unzip's expected output is the reference docstring example,
incubate/operators/unzip.py:40-62)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as TF

import paddle_ray_amd as paddle
from paddle_ray_amd.framework.core import _u
from paddle_ray_amd.incubate.operators import ResNetUnit, unzip


def _ref(unit, x, z, training=True):
    """fp32 PyTorch reference of the same unit (NHWC filters -> OIHW)."""
    nchw = unit._data_format == 'NCHW'

    def conv_bn(inp, f, s, b, m, v, stride):
        f = _u(f).float()
        if not nchw:
            f = f.permute(0, 3, 1, 2)
            inp = inp.permute(0, 3, 1, 2)
        c = TF.conv2d(inp.float(), f, None, stride, unit._padding)
        rm, rv = _u(m).clone().reshape(-1), _u(v).clone().reshape(-1)
        y = TF.batch_norm(c, rm, rv, _u(s).float().reshape(-1), _u(b).float().reshape(-1),
                          training, 1 - unit._momentum, unit._eps)
        return y, rm, rv

    y, rm, rv = conv_bn(x, unit.filter_x, unit.scale_x, unit.bias_x, unit.mean_x, unit.var_x,
                        unit._stride)
    if unit._has_shortcut:
        yz, _, _ = conv_bn(z, unit.filter_z, unit.scale_z, unit.bias_z, unit.mean_z, unit.var_z,
                           unit._stride_z)
        y = y + yz
    elif unit._fuse_add:
        zz = z.float() if nchw else z.float().permute(0, 3, 1, 2)
        y = y + zz
    y = torch.relu(y)
    if not nchw:
        y = y.permute(0, 2, 3, 1)
    return y, rm, rv


@pytest.mark.parametrize('cfg', [
    dict(k=3, stride=1, fmt='NHWC'),
    dict(k=3, stride=2, fmt='NHWC', shortcut=True),
    dict(k=1, stride=1, fmt='NHWC', add=True),
    dict(k=3, stride=1, fmt='NCHW', add=True),
])
def test_resnet_unit_matches_conv_bn_relu(cfg):
    torch.manual_seed(0)
    cin, cout, hw = 8, 16, 6
    unit = ResNetUnit(cin, cout, cfg['k'], stride=cfg['stride'], data_format=cfg['fmt'],
                      fuse_add=cfg.get('add', False), has_shortcut=cfg.get('shortcut', False),
                      num_channels_z=cin, stride_z=cfg['stride'])
    shape = [2, cin, hw, hw] if cfg['fmt'] == 'NCHW' else [2, hw, hw, cin]
    x = torch.randn(shape)
    if cfg.get('shortcut'):
        z = torch.randn(shape)
    elif cfg.get('add'):
        ho = hw // cfg['stride']
        z = torch.randn([2, cout, ho, ho] if cfg['fmt'] == 'NCHW' else [2, ho, ho, cout])
    else:
        z = None
    ref, rm, rv = _ref(unit, x, z)
    xt = paddle.to_tensor(x.numpy(), stop_gradient=False)
    y = unit(xt, paddle.to_tensor(z.numpy()) if z is not None else None)
    np.testing.assert_allclose(y.numpy(), ref.detach().numpy(), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(unit.mean_x.numpy().ravel(), rm.numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(unit.var_x.numpy().ravel(), rv.numpy(), rtol=1e-5, atol=1e-6)
    y.sum().backward()
    assert list(unit.filter_x.grad.shape) == list(unit.filter_x.shape)
    assert unit.mean_x.grad is None


def test_resnet_unit_eval_uses_running_stats():
    unit = ResNetUnit(8, 8, 3, is_test=True)
    unit.mean_x.set_value(np.full([1, 1, 1, 8], 0.5, np.float32))
    x = paddle.randn([1, 4, 4, 8])
    before = unit.mean_x.numpy().copy()
    y = unit(x)
    ref, _, _ = _ref(unit, _u(x), None, training=False)
    np.testing.assert_allclose(y.numpy(), ref.detach().numpy(), rtol=1e-4, atol=1e-4)
    np.testing.assert_array_equal(unit.mean_x.numpy(), before)


def test_resnet_unit_errors():
    with pytest.raises(ValueError):
        ResNetUnit(8, 8, 3, data_format='NDHWC')
    u = ResNetUnit(8, 8, 3, fuse_add=True)
    with pytest.raises(ValueError):
        u(paddle.randn([1, 4, 4, 8]))


def test_unzip_reference_example():
    x = paddle.to_tensor(np.array([[1, 2, 3, 4], [10, 20, 30, 40], [100, 200, 300, 400]]))
    lod = paddle.to_tensor(np.array([0, 4, 4, 8, 8, 8, 8, 12, 12, 12, 12]))
    out = unzip(x, lod).numpy()
    exp = np.zeros((10, 4), np.int64)
    exp[0], exp[2], exp[6] = [1, 2, 3, 4], [10, 20, 30, 40], [100, 200, 300, 400]
    np.testing.assert_array_equal(out, exp)


@pytest.mark.gpu
def test_resnet_unit_gpu_bf16_native():
    """bf16 AMP, NHWC, Cin/Cout % 64 == 0: conv on the in-tree implicit-GEMM kernel, BN (+ add
    + ReLU) on bn.hip with fp32 scale/shift/statistics."""
    from paddle_ray_amd.ops import registry as R
    torch.manual_seed(1)
    paddle.set_device('gpu')
    unit = ResNetUnit(64, 128, 3, has_shortcut=True, num_channels_z=64)
    x = torch.randn(4, 16, 16, 64, device='cuda')
    ref, rm, _ = _ref(unit, x.bfloat16().float(), x.bfloat16().float())
    R.reset_stats()
    with paddle.amp.auto_cast(dtype='bfloat16'):
        y = unit(paddle.to_tensor(x), paddle.to_tensor(x))
    torch.cuda.synchronize()
    assert _u(y).dtype == torch.bfloat16
    err = (_u(y).float() - ref).abs().max().item()
    assert err < 0.08, err
    np.testing.assert_allclose(unit.mean_x.numpy().ravel(), rm.cpu().numpy(), rtol=2e-2, atol=2e-3)
    st = R.stats()
    assert st.get(('batch_norm_fwd', 'hip'), 0) >= 2, st
    y.astype('float32').sum().backward()
    assert _u(unit.filter_x.grad).isfinite().all()
    assert _u(unit.scale_z.grad).isfinite().all()


def _static_net(fuse, train):
    from paddle_ray_amd.incubate.passes import fuse_resnet_unit_pass
    paddle.seed(3)
    prog, sp = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(prog, sp):
        x = paddle.static.data('x', [2, 8, 8, 8])
        conv = paddle.nn.Conv2D(8, 16, 1, bias_attr=False, data_format='NHWC')
        bn = paddle.nn.BatchNorm(16, act='relu', data_layout='NHWC')
        out = bn(conv(x))  # relu(bn(conv)): the reference's one-input pattern
        c2 = paddle.nn.Conv2D(16, 16, 3, padding=1, bias_attr=False, data_format='NHWC')
        b2 = paddle.nn.BatchNorm(16, data_layout='NHWC')
        c3 = paddle.nn.Conv2D(8, 16, 1, bias_attr=False, data_format='NHWC')
        b3 = paddle.nn.BatchNorm(16, data_layout='NHWC')
        # relu(bn(conv(out)) + bn(conv(x))): the two-input (shortcut) pattern
        out2 = paddle.nn.functional.relu(b2(c2(out)) + b3(c3(x)))
        c4 = paddle.nn.Conv2D(16, 16, 3, padding=1, bias_attr=False, data_format='NHWC')
        b4 = paddle.nn.BatchNorm(16, data_layout='NHWC')
        out3 = paddle.nn.functional.relu(b4(c4(out2)) + out2)  # fuse_add pattern
        if fuse:
            fuse_resnet_unit_pass(prog)
        loss = paddle.mean(out3)
        if train:
            paddle.optimizer.SGD(0.1).minimize(loss)
    exe = paddle.static.Executor()
    exe.run(sp)
    feed = {'x': np.random.RandomState(0).randn(2, 8, 8, 8).astype('float32')}
    res = [exe.run(prog, feed=feed, fetch_list=[loss, out3]) for _ in range(3)]
    return res, prog


@pytest.mark.parametrize('train', [False, True])
def test_fuse_resnet_unit_pass(train):
    paddle.enable_static()
    try:
        ref, p0 = _static_net(False, train)
        got, p1 = _static_net(True, train)
    finally:
        paddle.disable_static()
    assert p1._fused_resnet_units == 3
    types = [o.type.split(':')[-1] for o in p1.global_block().ops if o.role == 'forward']
    assert 'batch_norm' not in types and 'relu' not in types, types
    for (l0, o0), (l1, o1) in zip(ref, got):
        np.testing.assert_allclose(l1, l0, rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(o1, o0, rtol=1e-4, atol=1e-5)
