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


# -- graph replay semantics, capture fallback, dy2static control flow ---------------------------
@pytest.mark.gpu
def test_hip_graph_replay_outputs_are_fresh():
    """y1 = f(x1); y2 = f(x2) must keep y1 (replay rewrites the graph's static buffers)."""
    paddle.set_device('gpu')
    lin = paddle.nn.Linear(8, 8)
    lin.eval()
    f = paddle.jit.to_static(lin)
    with paddle.no_grad():
        x1, x2 = paddle.randn([4, 8]), paddle.randn([4, 8])
        y1 = f(x1)
        y1_ref = y1.numpy().copy()
        y2 = f(x2)
        y3 = f(x1)
    assert list(f.forward.graph_status().values()) == ['graph']
    np.testing.assert_allclose(y1.numpy(), y1_ref)
    np.testing.assert_allclose(y2.numpy(), lin(x2).numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(y3.numpy(), y1_ref, rtol=1e-6)
    assert y1._t.data_ptr() != y2._t.data_ptr()


@pytest.mark.gpu
def test_hip_graph_capture_failure_falls_back_to_eager():
    """A data-dependent host read cannot be captured: the call runs eagerly, correctly."""
    paddle.set_device('gpu')

    @paddle.jit.to_static
    def f(x):
        if x.mean() > 0:   # host read of a device value
            return x * 2
        return x - 1

    with paddle.no_grad():
        p, n = paddle.ones([4]), -paddle.ones([4])
        np.testing.assert_allclose(f(p).numpy(), 2 * np.ones(4))
        np.testing.assert_allclose(f(n).numpy(), -2 * np.ones(4))
        np.testing.assert_allclose(f(p).numpy(), 2 * np.ones(4))
    st = list(f.graph_status().values())
    assert len(st) == 1 and st[0].startswith('eager'), st


class _Branchy(paddle.nn.Layer):
    def __init__(self):
        super().__init__()
        self.l = paddle.nn.Linear(4, 4)

    def forward(self, x):
        y = self.l(x)
        if y.mean() > 0 and y.max() > 1:
            z = y * 2.0
        else:
            z = y - 10.0
        i = paddle.zeros([1])
        while i < y.abs().max():   # trip count depends on the input
            z = z + 1.0
            i = i + 1
        if z.sum() > 1e9:
            return z * 0
        return z


def test_dy2static_if_while_both_branches_after_save_load(tmp_path):
    """`if` / `while` on tensor values: eager and jit.save/load agree for BOTH branches (the
    saved program holds conditional_block / while sub-blocks decided by the fed values)."""
    paddle.seed(0)
    net = _Branchy()
    net.l.weight.set_value(np.eye(4, dtype='float32'))
    net.l.bias.set_value(np.zeros(4, 'float32'))
    pos = paddle.to_tensor(np.full((2, 4), 5.0, 'float32'))
    neg = paddle.to_tensor(np.full((2, 4), -5.0, 'float32'))
    e_pos, e_neg = net(pos).numpy(), net(neg).numpy()
    np.testing.assert_allclose(e_pos, np.full((2, 4), 15.0))
    np.testing.assert_allclose(e_neg, np.full((2, 4), -10.0))
    path = str(tmp_path / 'branchy')
    paddle.jit.save(net, path, input_spec=[InputSpec([None, 4], 'float32')])
    from paddle_ray_amd.static import program_desc as PD
    desc = PD.decode('ProgramDesc', open(path + '.pdmodel', 'rb').read())
    types = [o['type'] for b in desc['blocks'] for o in b.get('ops', [])]
    assert any('conditional_block_op' in t for t in types) and any('while_op' in t for t in types)
    assert len(desc['blocks']) >= 3  # block 0 + the if-branches + the while body
    assert all(b['parent_idx'] == (-1 if b['idx'] == 0 else b['parent_idx']) for b in desc['blocks'])
    ld = paddle.jit.load(path)
    np.testing.assert_allclose(ld(pos).numpy(), e_pos, rtol=1e-6)
    np.testing.assert_allclose(ld(neg).numpy(), e_neg, rtol=1e-6)
    two = paddle.to_tensor(np.full((2, 4), 2.0, 'float32'))  # 2 trips instead of 5
    np.testing.assert_allclose(ld(two).numpy(), net(two).numpy(), rtol=1e-6)


def test_dy2static_converter_units():
    from paddle_ray_amd.jit.dy2static import convert_function

    def g(x, n):
        acc = 0
        k = 0
        while k < n:
            acc = acc + x
            k = k + 1
        if acc > 10 or n == 0:
            out = acc
        else:
            out = -acc
        return out
    cg = convert_function(g)
    assert getattr(cg, '_pra_converted', False)
    for x, n in ((3, 5), (1, 2), (4, 0)):
        assert cg(x, n) == g(x, n)


_DY2S_GLOBAL_HITS = 0


class _PlainParent(paddle.nn.Layer):
    def __init__(self):
        super().__init__()
        self.l = paddle.nn.Linear(4, 4)

    def forward(self, x):
        return self.l(x) + 1.0


class _BranchyChild(_PlainParent):
    """Converted forward with zero-argument super(), a private (mangled) attribute and a
    ``global`` write: the twin must keep the class cell, the owner's mangling and the real
    module globals."""

    def __init__(self):
        super().__init__()
        self.__scale = 3.0

    def forward(self, x):
        global _DY2S_GLOBAL_HITS
        _DY2S_GLOBAL_HITS += 1
        if x.mean() > 0:
            x = x * self.__scale
        else:
            x = x - 1.0
        return super().forward(x)


def test_dy2static_super_private_global(tmp_path):
    from paddle_ray_amd.jit.dy2static import convert_function
    paddle.seed(0)
    net = _BranchyChild()
    net.l.weight.set_value(np.eye(4, dtype='float32'))
    net.l.bias.set_value(np.zeros(4, 'float32'))
    pos = paddle.to_tensor(np.full((2, 4), 1.0, 'float32'))
    f = convert_function(net.forward)
    assert getattr(f, '_pra_converted', False)
    before = _DY2S_GLOBAL_HITS
    np.testing.assert_allclose(f(pos).numpy(), net(pos).numpy())
    assert _DY2S_GLOBAL_HITS == before + 2  # the twin wrote the module's real global
    path = str(tmp_path / 'child')
    paddle.jit.save(net, path, input_spec=[InputSpec([None, 4], 'float32')])
    ld = paddle.jit.load(path)
    neg = paddle.to_tensor(np.full((2, 4), -1.0, 'float32'))
    for x in (pos, neg):
        np.testing.assert_allclose(ld(x).numpy(), net(x).numpy(), rtol=1e-6)


def test_dy2static_nonlocal_closure():
    from paddle_ray_amd.jit.dy2static import convert_function
    calls = [0]
    k = 2.0

    def g(x):
        nonlocal k
        calls[0] += 1
        if x.sum() > 0:
            y = x * k
        else:
            y = x
        k = k + 1.0
        return y

    cg = convert_function(g)
    assert getattr(cg, '_pra_converted', False)
    out = cg(paddle.ones([2]))
    np.testing.assert_allclose(out.numpy(), [2.0, 2.0])
    assert k == 3.0 and calls[0] == 1  # the nonlocal write reached the real cell


class _MLPNorm(paddle.nn.Layer):
    def __init__(self):
        super().__init__()
        self.l1 = paddle.nn.Linear(16, 32)
        self.ln = paddle.nn.LayerNorm(32)
        self.l2 = paddle.nn.Linear(32, 4)

    def forward(self, x):
        return self.l2(paddle.nn.functional.gelu(self.ln(self.l1(x))))


def test_convert_to_mixed_precision_and_predictor_pool(tmp_path):
    """inference.convert_to_mixed_precision (wrapper.py): bf16 parameters except those of
    black-listed op types, O2 replay, fp32 I/O kept; PredictorPool hands out independent
    predictors (reference: paddle.inference.PredictorPool)."""
    from paddle_ray_amd import inference
    from paddle_ray_amd.static import program_desc as PD
    paddle.seed(3)
    net = _MLPNorm()
    net.eval()
    path = str(tmp_path / 'm')
    paddle.jit.save(net, path, input_spec=[InputSpec([None, 16], 'float32', 'x')])
    ops = [od['type'] for od in PD.decode('ProgramDesc', open(path + '.pdmodel', 'rb').read())['blocks'][0]['ops']]
    ln_type = next(t for t in ops if 'layer_norm' in t)
    mixed = str(tmp_path / 'mixed' / 'm')
    inference.convert_to_mixed_precision(path + '.pdmodel', path + '.pdiparams', mixed + '.pdmodel',
                                         mixed + '.pdiparams', inference.PrecisionType.Bfloat16,
                                         inference.PlaceType.GPU, keep_io_types=True, black_list={ln_type})
    params = paddle.load(mixed + '.pdiparams')
    dts = {k: v.dtype for k, v in params.items()}
    assert any('bfloat16' in str(d) for d in dts.values())
    ln_names = [k for k in params if params[k].shape == [32] and 'bfloat16' not in str(params[k].dtype)]
    assert len(ln_names) >= 2          # the LayerNorm's scale and shift stay fp32
    x = np.random.RandomState(1).rand(5, 16).astype('float32')
    ref = net(paddle.to_tensor(x)).numpy()
    pool = inference.PredictorPool(inference.Config(mixed + '.pdmodel', mixed + '.pdiparams'), 2)
    assert len(pool) == 2 and pool.retrive(0) is not pool.retrive(1)
    outs = []
    for i in range(2):
        p = pool.retrive(i)
        p.get_input_handle('x').copy_from_cpu(x)
        p.run()
        outs.append(p.get_output_handle(p.get_output_names()[0]).copy_to_cpu())
    assert outs[0].dtype == np.float32
    np.testing.assert_allclose(outs[0], outs[1])
    np.testing.assert_allclose(outs[0], ref, rtol=5e-2, atol=5e-2)
    assert not np.array_equal(outs[0], ref)       # really ran in bf16
    with pytest.raises(ValueError):
        inference.convert_to_mixed_precision(path + '.pdmodel', path + '.pdiparams', mixed + '2.pdmodel',
                                             mixed + '2.pdiparams', inference.PrecisionType.Int8,
                                             inference.PlaceType.GPU)
