"""Static graph mode: Program recording, Executor replay (native scheduler), minimize,
inference model save/load (parity: test/legacy_test/test_executor_*, test_program.py,
test_inference_model_io.py)."""
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


def test_native_scheduler_matches_python():
    from paddle_ray_amd.native import build_plan, build_plan_py, runtime
    ins = [[0], [1], [1, 2], [0], [3]]
    outs = [[1], [2], [3], [4], []]
    a = build_plan(ins, outs, [3], [])
    b = build_plan_py(ins, outs, [3], [])
    assert [list(x) if not isinstance(x, int) else x for x in a[0]] == list(b[0])
    assert 3 in a[3]  # op producing var 4 is dead
    assert runtime() is not None, "native runtime extension must be built"


def test_static_mlp_matches_dygraph(static_mode):
    paddle.seed(1)
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        x = static.data('x', [None, 8], 'float32')
        lin1 = nn.Linear(8, 16)
        lin2 = nn.Linear(16, 4)
        h = F.relu(lin1(x))
        y = lin2(h)
        out = paddle.mean(y * 2.0 + 1.0, axis=-1)
    assert out.shape == [-1]
    exe = static.Executor()
    exe.run(startup)
    xv = np.random.RandomState(0).randn(5, 8).astype('float32')
    r, = exe.run(main, feed={'x': xv}, fetch_list=[out])
    paddle.disable_static()
    ref = paddle.mean(lin2(F.relu(lin1(paddle.to_tensor(xv)))) * 2.0 + 1.0, axis=-1).numpy()
    paddle.enable_static()
    np.testing.assert_allclose(r, ref, rtol=1e-5, atol=1e-6)
    # different batch size reuses the same program
    r2, = exe.run(main, feed={'x': xv[:3]}, fetch_list=[out])
    np.testing.assert_allclose(r2, ref[:3], rtol=1e-5, atol=1e-6)


def test_static_minimize_trains(static_mode):
    paddle.seed(2)
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        x = static.data('x', [None, 4], 'float32')
        lbl = static.data('y', [None, 1], 'int64')
        logits = static.nn.fc(x, 3)
        loss = F.cross_entropy(logits, lbl)
        opt = paddle.optimizer.Adam(0.05)
        opt.minimize(loss)
    exe = static.Executor()
    exe.run(startup)
    rs = np.random.RandomState(0)
    xv = rs.randn(32, 4).astype('float32')
    yv = (xv[:, :1] > 0).astype('int64') + (xv[:, 1:2] > 0).astype('int64')
    losses = [float(exe.run(main, feed={'x': xv, 'y': yv}, fetch_list=[loss])[0])
              for _ in range(40)]
    assert losses[-1] < losses[0] * 0.6, losses
    test_prog = main.clone(for_test=True)
    assert not any(op.type in ('backward', 'optimize') for op in test_prog.global_block().ops)


def test_append_backward_grad_fetch(static_mode):
    main = static.Program()
    with static.program_guard(main):
        x = static.data('x', [2, 3], 'float32')
        w = static.create_parameter([3, 1], 'float32')
        y = paddle.sum(paddle.matmul(x, w))
        pg = static.append_backward(y)
    exe = static.Executor()
    xv = np.ones([2, 3], 'float32')
    (p, g), = [(p, g) for p, g in pg if p is w]
    _, gv = exe.run(main, feed={'x': xv}, fetch_list=[y, g])
    np.testing.assert_allclose(gv, np.full([3, 1], 2.0), rtol=1e-6)


def test_gradients_op(static_mode):
    main = static.Program()
    with static.program_guard(main):
        x = static.data('x', [4], 'float32')
        x.stop_gradient = False
        y = paddle.sum(x * x)
        gx, = static.gradients([y], [x])
    exe = static.Executor()
    xv = np.arange(4, dtype='float32')
    r, = exe.run(main, feed={'x': xv}, fetch_list=[gx])
    np.testing.assert_allclose(r, 2 * xv)


def test_getitem_operators_and_methods(static_mode):
    main = static.Program()
    with static.program_guard(main):
        x = static.data('x', [None, 6], 'float32')
        y = (1.0 - x[:, 1:4]).reshape([-1, 3, 1]).transpose([0, 2, 1])
        z = paddle.concat([y, y * y], axis=1)
    assert z.shape == [-1, 2, 3]
    exe = static.Executor()
    xv = np.random.rand(2, 6).astype('float32')
    r, = exe.run(main, feed={'x': xv}, fetch_list=[z])
    yy = (1.0 - xv[:, 1:4]).reshape(-1, 1, 3)
    np.testing.assert_allclose(r, np.concatenate([yy, yy * yy], 1), rtol=1e-6)


def test_layer_fallback_recorded_as_one_op(static_mode):
    """Layers whose forward uses raw tensors are recorded as a single layer op."""
    class Raw(nn.Layer):
        def forward(self, x):
            from paddle_ray_amd.framework.core import Tensor, _u
            return Tensor(_u(x).flip(-1) * 3)
    main = static.Program()
    with static.program_guard(main):
        x = static.data('x', [None, 3], 'float32')
        y = Raw()(x) + 1
    assert any(op.type == 'layer:Raw' for op in main.global_block().ops)
    r, = static.Executor().run(main, feed={'x': np.array([[1, 2, 3]], 'float32')},
                               fetch_list=[y])
    np.testing.assert_allclose(r, [[10, 7, 4]])


def test_dead_code_pruned(static_mode):
    main = static.Program()
    with static.program_guard(main):
        x = static.data('x', [3], 'float32')
        a = x + 1
        b = paddle.exp(x)  # not fetched
    exe = static.Executor()
    r, = exe.run(main, feed={'x': np.zeros(3, 'float32')}, fetch_list=[a])
    np.testing.assert_allclose(r, np.ones(3))
    _, _, _, pruned = __import__('paddle_ray_amd.native', fromlist=['x']).build_plan(
        [op.in_vids for op in main.global_block().ops],
        [op.out_vids for op in main.global_block().ops], [a.vid], [])
    assert list(pruned) == [1]


def test_save_load_inference_model(static_mode, tmp_path):
    paddle.seed(3)
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        x = static.data('img', [None, 1, 8, 8], 'float32')
        c = static.nn.conv2d(x, 4, 3, padding=1, act='relu')
        bn = static.nn.batch_norm(c, is_test=True)
        p = F.max_pool2d(bn, 2)
        out = F.softmax(static.nn.fc(p.flatten(1), 5))
    exe = static.Executor()
    exe.run(startup)
    xv = np.random.RandomState(1).rand(2, 1, 8, 8).astype('float32')
    test_prog = main.clone(for_test=True)
    ref, = exe.run(test_prog, feed={'img': xv}, fetch_list=[out])
    path = str(tmp_path / 'inf' / 'model')
    static.save_inference_model(path, [x], [out], exe, program=test_prog)
    prog, feed_names, fetch_targets = static.load_inference_model(path, exe)
    assert feed_names == ['img']
    r, = exe.run(prog, feed={'img': xv}, fetch_list=fetch_targets)
    np.testing.assert_allclose(r, ref, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_executor_hip_graph_replay():
    paddle.set_device('gpu')
    paddle.enable_static()
    try:
        main = static.Program()
        with static.program_guard(main):
            x = static.data('x', [None, 16], 'float32')
            y = F.gelu(static.nn.fc(x, 32)) * 3.0
        cp = static.CompiledProgram(main)
        cp._build_strategy.use_hip_graph = True
        exe = static.Executor()
        xv = np.random.rand(4, 16).astype('float32')
        a, = exe.run(main, feed={'x': xv}, fetch_list=[y])
        b, = exe.run(cp, feed={'x': xv}, fetch_list=[y])
        c, = exe.run(cp, feed={'x': xv * 2}, fetch_list=[y])
        d, = exe.run(main, feed={'x': xv * 2}, fetch_list=[y])
        np.testing.assert_allclose(a, b, rtol=1e-5)
        np.testing.assert_allclose(c, d, rtol=1e-5)
        assert len(main._graph_cache) == 1
    finally:
        paddle.disable_static()


def test_static_bert_direct_grad_ops_match_eager():
    """BERT pretraining recorded op by op: the fused linear / flash-attention / add+dropout+LN /
    MLP / softmax-CE ops carry DIRECT grad ops (Function.backward on the saved context, no _vjp
    autograd replay), and one SGD step through the Executor equals the eager step."""
    import numpy as np
    import collections
    import paddle_ray_amd as paddle
    from paddle_ray_amd import static
    from paddle_ray_amd.models import bert_config, BertForPretraining
    cfg = bert_config('bert-tiny', hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    bs, S, P = 2, 16, 3
    rs = np.random.RandomState(0)
    ids = rs.randint(5, cfg.vocab_size, (bs, S))
    ids[1, 12:] = cfg.pad_token_id  # padded keys: the static program always builds the mask
    pos = np.stack([np.sort(rs.choice(12, P, replace=False)) + i * S for i in range(bs)]).reshape(-1)
    lab = ids.reshape(-1)[pos].copy()
    nsp = rs.randint(0, 2, (bs,))

    def build():
        paddle.seed(1)
        return BertForPretraining(cfg)
    m_e = build()
    opt_e = paddle.optimizer.SGD(0.1, parameters=m_e.parameters())
    loss_e = m_e(paddle.to_tensor(ids), masked_positions=paddle.to_tensor(pos), labels=paddle.to_tensor(lab),
                 next_sentence_label=paddle.to_tensor(nsp))
    loss_e.backward()
    opt_e.step()
    m_s = build()
    paddle.enable_static()
    try:
        main_p, startup = static.Program(), static.Program()
        with static.program_guard(main_p, startup):
            iv = static.data('ids', [bs, S], 'int64')
            pv = static.data('pos', [bs * P], 'int64')
            lv = static.data('lab', [bs * P], 'int64')
            nv = static.data('nsp', [bs], 'int64')
            loss_v = m_s(iv, masked_positions=pv, labels=lv, next_sentence_label=nv)
            paddle.optimizer.SGD(0.1, parameters=m_s.parameters()).minimize(loss_v)
        types = collections.Counter((op.role, op.type, op.fn.__name__) for op in main_p.global_block().ops)
        for t in ('fused_linear', 'fused_flash_qkv', 'fused_add_dropout_ln', 'fused_mlp_gelu',
                  'fused_softmax_ce', 'fused_linear_nt', 'fused_bias_gelu'):
            assert types[('backward', t + '_grad', '_fn_grad')] >= 1, t
            assert not any(k[1] == t + '_grad' and k[2] != '_fn_grad' for k in types), t
        # gradient-sum fusion: the residual stream's second partial gradient is folded into the
        # Linear / MLP dgrad (beta=1 GEMM) instead of a separate `sum` op
        ops = main_p.global_block().ops
        folded = [op for op in ops if op.type in ('fused_linear_grad', 'fused_mlp_gelu_grad') and 'acc' in op.kwargs]
        assert len(folded) >= 2 * cfg.num_hidden_layers, len(folded)
        exe = static.Executor()
        exe.run(startup)
        out = exe.run(main_p, feed={'ids': ids, 'pos': pos, 'lab': lab, 'nsp': nsp}, fetch_list=[loss_v])
    finally:
        paddle.disable_static()
    np.testing.assert_allclose(float(out[0]), float(loss_e), rtol=1e-5)
    for (n, pe), ps in zip(m_e.named_parameters(), m_s.parameters()):
        np.testing.assert_allclose(ps.numpy(), pe.numpy(), rtol=1e-4, atol=1e-6, err_msg=n)
