"""Static-graph IR: per-op grad OpDescs from append_backward, allowlisted .pdmodel loading,
static AMP (decorate) training parity with dygraph, HIP-graph capture of a training program.

Parity: python/paddle/fluid/backward.py:1826 (append_backward emits grad ops),
framework.proto OpDesc (op types resolved through the op registry),
python/paddle/static/amp/decorator.py (OptimizerWithMixedPrecision)."""
import json

import numpy as np
import pytest

import paddle_ray_amd as paddle
import paddle_ray_amd.nn as nn
import paddle_ray_amd.nn.functional as F
from paddle_ray_amd import static


@pytest.fixture
def static_mode():
    paddle.enable_static()
    yield
    paddle.disable_static()


def test_append_backward_emits_grad_ops_and_sums(static_mode):
    paddle.seed(0)
    main = static.Program()
    with static.program_guard(main):
        x = static.data('x', [None, 4], 'float32')
        lin = nn.Linear(4, 4)
        h = lin(x)
        h2 = lin(F.relu(h))           # the same parameters feed two ops -> sum ops
        loss = paddle.mean(h2 * h)    # h feeds two ops -> sum op
        pg = static.append_backward(loss)
    ops = main.global_block().ops
    types = [op.type for op in ops]
    assert 'backward' not in types
    assert sum(t.endswith('_grad') for t in types) >= 4, types
    assert types.count('sum') >= 3, types       # h, weight, bias
    assert 'fill_grad_seed' in types
    assert all(op.role in ('forward', 'backward') for op in ops)
    exe = static.Executor()
    xv = np.random.RandomState(0).randn(3, 4).astype('float32')
    fetched = exe.run(main, feed={'x': xv}, fetch_list=[loss] + [g for _, g in pg])
    paddle.disable_static()
    xt = paddle.to_tensor(xv)
    hh = lin(xt)
    ref = paddle.mean(lin(F.relu(hh)) * hh)
    ref.backward()
    paddle.enable_static()
    np.testing.assert_allclose(fetched[0], ref.numpy(), rtol=1e-5)
    by_name = {p.name: g for (p, _), g in zip(pg, fetched[1:])}
    np.testing.assert_allclose(by_name[lin.weight.name], lin.weight.grad.numpy(), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(by_name[lin.bias.name], lin.bias.grad.numpy(), rtol=1e-4, atol=1e-6)


def test_gradients_wrt_data_and_target_grads(static_mode):
    main = static.Program()
    with static.program_guard(main):
        x = static.data('x', [3], 'float32')
        x.stop_gradient = False
        y = paddle.exp(x) * x
        gx, = static.gradients([y], [x], target_gradients=None)
    xv = np.array([0.5, 1.0, -1.0], 'float32')
    r, = static.Executor().run(main, feed={'x': xv}, fetch_list=[gx])
    np.testing.assert_allclose(r, np.exp(xv) * (1 + xv), rtol=1e-5)


def test_tampered_pdmodel_refused(static_mode, tmp_path):
    main = static.Program()
    with static.program_guard(main):
        x = static.data('x', [None, 4], 'float32')
        y = F.relu(static.nn.fc(x, 3))
    exe = static.Executor()
    path = str(tmp_path / 'm')
    static.save_inference_model(path, [x], [y], exe, program=main)
    from paddle_ray_amd.static import program_desc as PD
    raw = open(path + '.pdmodel', 'rb').read()
    desc = PD.decode('ProgramDesc', raw)
    ops = desc['blocks'][0]['ops']
    assert ops[0]['type'] == 'feed' and ops[-1]['type'] == 'fetch'
    prog, _, fetch = static.load_inference_model(path, exe)  # the untampered model loads
    k = next(i for i, o in enumerate(ops) if o['type'] not in ('feed', 'fetch'))
    for evil in ('os:system', 'posix:system', 'subprocess:check_output', 'builtins:eval'):
        bad = [dict(o) for o in ops]
        call = PD.dumps_call({'args': ['touch ' + str(tmp_path / 'pwned')], 'kwargs': {}})
        bad[k] = dict(bad[k], type=evil, attrs=[{'name': '__pra_call__', 'type': 2, 's': call}])
        d2 = dict(desc, blocks=[dict(desc['blocks'][0], ops=bad)] + desc['blocks'][1:])
        open(path + '.pdmodel', 'wb').write(PD.encode('ProgramDesc', d2))
        with pytest.raises(ValueError, match='not a registered'):
            static.load_inference_model(path, exe)
        # the legacy JSON op list is refused the same way
        open(path + '.pdmodel', 'wb').write(json.dumps(
            {'version': 2, 'feeds': [], 'fetches': [], 'vars': {}, 'params': [],
             'ops': [{'type': evil, 'args': ['touch x'], 'kwargs': {}, 'in': [], 'out': []}]}).encode())
        with pytest.raises(ValueError, match='not a registered'):
            static.load_inference_model(path, exe)
    assert not (tmp_path / 'pwned').exists()


def _bert_batch(rs, B=2, S=16):
    ids = rs.randint(5, 64, (B, S))
    labels = np.full((B, S), -1)
    pos = rs.rand(B, S) < 0.3
    labels[pos] = ids[pos]
    ids[pos] = 3
    return ids.astype('int64'), labels.astype('int64'), rs.randint(0, 2, (B,)).astype('int64')


def _bert_static_vs_dygraph(cfg_name, steps, device=None, **overrides):
    from paddle_ray_amd.models import bert_config, BertForPretraining
    cfg = bert_config(cfg_name, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0,
                      **overrides)
    rs = np.random.RandomState(0)
    batches = [_bert_batch(rs) for _ in range(steps)]
    # dygraph reference
    paddle.disable_static()
    paddle.seed(7)
    m = BertForPretraining(cfg)
    sd = {k: v.numpy().copy() for k, v in m.state_dict().items()}
    opt = paddle.optimizer.AdamW(1e-3, parameters=m.parameters())
    ref = []
    for ids, lab, nsp in batches:
        with paddle.amp.auto_cast(dtype='bfloat16'):
            loss = m(paddle.to_tensor(ids), labels=paddle.to_tensor(lab),
                     next_sentence_label=paddle.to_tensor(nsp))
        loss.backward()
        opt.step()
        opt.clear_grad()
        ref.append(float(loss))
    # static program: same init, AMP through static.amp.decorate
    paddle.seed(7)
    m2 = BertForPretraining(cfg)
    m2.set_state_dict(sd)
    paddle.enable_static()
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        ids_v = static.data('ids', [None, 16], 'int64')
        lab_v = static.data('lab', [None, 16], 'int64')
        nsp_v = static.data('nsp', [None], 'int64')
        loss_v = m2(ids_v, labels=lab_v, next_sentence_label=nsp_v)
        opt2 = static.amp.decorate(paddle.optimizer.AdamW(1e-3, parameters=m2.parameters()),
                                   use_bf16=True)
        opt2.minimize(loss_v)
    assert any(op.type.endswith('_grad') for op in main.global_block().ops)
    exe = static.Executor()
    exe.run(startup)
    got = [float(exe.run(main, feed={'ids': i, 'lab': l, 'nsp': n}, fetch_list=[loss_v])[0])
           for i, l, n in batches]
    return ref, got


def test_bert_static_amp_matches_dygraph_tiny(static_mode):
    ref, got = _bert_static_vs_dygraph('bert-tiny', 5)
    np.testing.assert_allclose(got, ref, rtol=2e-3, atol=2e-3)
    assert got[-1] < got[0]


@pytest.mark.gpu
def test_bert_base_static_amp_matches_dygraph_gpu():
    paddle.set_device('gpu')
    try:
        paddle.enable_static()
        ref, got = _bert_static_vs_dygraph('bert-base-uncased', 5)
    finally:
        paddle.disable_static()
    np.testing.assert_allclose(got, ref, rtol=1e-2, atol=1e-2)


@pytest.mark.gpu
def test_training_program_hip_graph_capture():
    """Forward + grad ops of a training program replay as one captured HIP graph; the
    optimizer step runs after it. Same losses as the op-by-op replay."""
    paddle.set_device('gpu')
    paddle.enable_static()
    try:
        def build(seed):
            paddle.seed(seed)
            main, startup = static.Program(), static.Program()
            with static.program_guard(main, startup):
                x = static.data('x', [8, 16], 'float32')
                y = static.data('y', [8, 1], 'int64')
                h = F.gelu(static.nn.fc(x, 32))
                loss = F.cross_entropy(static.nn.fc(h, 4), y)
                paddle.optimizer.Adam(0.01).minimize(loss)
            return main, startup, loss
        rs = np.random.RandomState(0)
        xv = rs.randn(8, 16).astype('float32')
        yv = rs.randint(0, 4, (8, 1)).astype('int64')
        exe = static.Executor()
        m1, s1, l1 = build(3)
        exe.run(s1)
        eager = [float(exe.run(m1, feed={'x': xv, 'y': yv}, fetch_list=[l1])[0]) for _ in range(6)]
        m2, s2, l2 = build(3)
        exe.run(s2)
        cp = static.CompiledProgram(m2)
        cp._build_strategy.use_hip_graph = True
        graph = [float(exe.run(cp, feed={'x': xv, 'y': yv}, fetch_list=[l2])[0]) for _ in range(6)]
        assert len(m2._graph_cache) == 1
        np.testing.assert_allclose(graph, eager, rtol=1e-4, atol=1e-5)
        assert graph[-1] < graph[0]
    finally:
        paddle.disable_static()
