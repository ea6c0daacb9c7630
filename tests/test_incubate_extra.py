"""incubate extras: ASP n:m sparsity, memory_efficient_attention + attn_bias, identity_loss,
graph_khop_sampler, auto_checkpoint, multiprocessing reductions (parity:
test/asp/test_asp_*.py, test/legacy_test/test_memory_efficient_attention.py,
test_identity_loss_op.py, test_graph_khop_sampler.py, test_auto_checkpoint*.py,
test_paddle_multiprocessing.py)."""
import multiprocessing as _mp

import numpy as np
import pytest
import torch

import paddle_ray_amd as paddle
from paddle_ray_amd import nn
from paddle_ray_amd.incubate import asp
from paddle_ray_amd.incubate.nn import attn_bias as AB
from paddle_ray_amd.incubate.nn import memory_efficient_attention


def test_asp_masks():
    x = np.array([[0, 1, 3, 0], [1, 0, 0, 1]])
    assert asp.check_mask_1d(x, 2, 4) and not asp.check_mask_1d(np.array([[0, 1, 5, 4]]), 2, 4)
    m = np.random.RandomState(0).randn(8, 12)
    k1, kg, kb = (f(m, 2, 4) for f in (asp.get_mask_1d, asp.get_mask_2d_greedy,
                                       asp.get_mask_2d_best))
    assert asp.check_mask_1d(k1 * m, 2, 4)
    assert asp.check_mask_2d(kg * m, 2, 4) and asp.check_mask_2d(kb * m, 2, 4)
    assert (np.abs(m) * kb).sum() >= (np.abs(m) * kg).sum() - 1e-9
    assert asp.calculate_density(k1) == 0.5
    w4 = np.random.RandomState(1).randn(3, 3, 8, 6)
    mk = asp.create_mask(w4, asp.MaskAlgo.MASK_1D)
    assert mk.shape == w4.shape and asp.check_sparsity(mk * w4, asp.CheckMethod.CHECK_1D)


def test_asp_prune_and_train():
    paddle.seed(0)
    model = nn.Sequential(nn.Linear(16, 32), nn.ReLU(), nn.Linear(32, 4))
    asp.set_excluded_layers(['2.weight'])
    try:
        masks = asp.prune_model(model, 2, 4)
    finally:
        asp.reset_excluded_layers()
    assert list(masks) == ['0.weight']
    opt = asp.decorate(paddle.optimizer.Adam(0.01, parameters=model.parameters()))
    x = paddle.randn([8, 16])
    for _ in range(3):
        model(x).mean().backward()
        opt.step()
        opt.clear_grad()
    w = model[0].weight.numpy()
    assert asp.check_sparsity(w.T, n=2, m=4) and abs(asp.calculate_density(w) - 0.5) < 1e-6
    assert asp.calculate_density(model[2].weight.numpy()) == 1.0


def _ref_attn(q, k, v, bias, scale):
    s = torch.einsum('bmhk,bnhk->bhmn', q.double(), k.double()) * scale
    if bias is not None:
        s = s + bias.double()
    return torch.einsum('bhmn,bnhk->bmhk', torch.softmax(s, -1), v.double())


def test_memory_efficient_attention_biases():
    torch.manual_seed(0)
    q, k, v = (torch.randn(1, 10, 2, 8) for _ in range(3))
    scale = 8 ** -0.5
    out = memory_efficient_attention(paddle.Tensor(q), paddle.Tensor(k), paddle.Tensor(v))
    np.testing.assert_allclose(out.numpy(), _ref_attn(q, k, v, None, scale).numpy(), atol=1e-5)
    causal = AB.LowerTriangularMask()
    out = memory_efficient_attention(paddle.Tensor(q), paddle.Tensor(k), paddle.Tensor(v), causal)
    m = torch.full((10, 10), float('-inf')).triu(1)
    np.testing.assert_allclose(out.numpy(), _ref_attn(q, k, v, m, scale).numpy(), atol=1e-5)
    bd = AB.BlockDiagonalMask.from_seqlens([4, 6])
    dense = bd.materialize([1, 2, 10, 10]).numpy()
    assert dense[0, 0, 0, 5] == -np.inf and dense[0, 0, 5, 5] == 0
    out = memory_efficient_attention(paddle.Tensor(q), paddle.Tensor(k), paddle.Tensor(v), bd)
    ref = torch.cat([_ref_attn(q[:, :4], k[:, :4], v[:, :4], None, scale),
                     _ref_attn(q[:, 4:], k[:, 4:], v[:, 4:], None, scale)], 1)
    np.testing.assert_allclose(out.numpy(), ref.numpy(), atol=1e-5)
    bdc = bd.make_causal()
    assert bdc.materialize([10, 10]).numpy()[1, 2] == -np.inf
    parts = bd.split(paddle.Tensor(q))
    assert [p.shape[1] for p in parts] == [4, 6]
    pad = AB.BlockDiagonalCausalWithOffsetPaddedKeysMask.from_seqlens([1, 1], 4, [2, 3])
    mm = pad.materialize([2, 8]).numpy()
    assert (mm[0, :2] == 0).all() and mm[0, 2] == -np.inf and (mm[1, 4:7] == 0).all()
    bias = torch.randn(1, 2, 10, 10)
    out = memory_efficient_attention(paddle.Tensor(q), paddle.Tensor(k), paddle.Tensor(v),
                                     paddle.Tensor(bias), scale=0.3)
    np.testing.assert_allclose(out.numpy(), _ref_attn(q, k, v, bias, 0.3).numpy(), atol=1e-5)


def test_identity_loss_and_khop():
    x = paddle.to_tensor([1.0, 2.0, 3.0])
    assert float(paddle.incubate.identity_loss(x, 'mean')) == 2.0
    assert float(paddle.incubate.identity_loss(x, 0)) == 6.0
    assert paddle.incubate.identity_loss(x, 'none').shape == [3]
    # CSC graph: node v's neighbors are row[colptr[v]:colptr[v+1]]
    row = paddle.to_tensor(np.array([1, 2, 0, 3, 0, 4, 1, 0], np.int64))
    colptr = paddle.to_tensor(np.array([0, 2, 4, 6, 7, 8], np.int64))
    src, dst, idx, rn = paddle.incubate.graph_khop_sampler(row, colptr,
                                                           paddle.to_tensor(np.array([0])),
                                                           [2, 2])
    nodes = idx.numpy()
    assert nodes[0] == 0 and rn.numpy().tolist() == [0]
    assert src.shape == dst.shape and int(src.numpy().max()) < len(nodes)


def test_auto_checkpoint_resume(tmp_path, monkeypatch):
    from paddle_ray_amd.incubate.checkpoint import auto_checkpoint as ac
    monkeypatch.setenv('PADDLE_JOB_ID', 'job1')
    monkeypatch.setenv('PADDLE_CHECKPOINT_PATH', str(tmp_path))
    lin = nn.Linear(2, 2)
    ac.register('model', lin)
    try:
        seen = []
        for ep in ac.train_epoch_range(5, save_checkpoint_inter=0):
            seen.append(ep)
            with torch.no_grad():
                lin.weight._t.fill_(float(ep))
            if ep == 2:
                break  # "crash" after epoch 2's work, before it is recorded
        assert seen == [0, 1, 2]
        lin.weight._t.data.zero_()
        resumed = list(ac.train_epoch_range(5, save_checkpoint_inter=0))
        assert resumed == [2, 3, 4]
        assert float(lin.weight.numpy()[0, 0]) == 1.0  # restored from the epoch-1 checkpoint
        assert list(ac.train_epoch_range(5, save_checkpoint_inter=0)) == []
    finally:
        ac.unregister()


def _child(qin, qout):
    t = qin.get(timeout=30)
    t._t.add_(1.0)
    qout.put('done')


def test_multiprocessing_shares_cpu_tensors():
    mp = paddle.incubate.multiprocessing
    t = paddle.zeros([4])
    ctx = _mp.get_context('fork')
    qin, qout = ctx.Queue(), ctx.Queue()
    p = ctx.Process(target=_child, args=(qin, qout), daemon=True)
    p.start()
    try:
        qin.put(t)
        assert qout.get(timeout=30) == 'done'
    finally:
        p.join(10)
        if p.is_alive():
            p.kill()
    assert mp is not None and float(t.numpy().sum()) == 4.0


def test_fused_linear_activation_cpu():
    import paddle_ray_amd as paddle
    from paddle_ray_amd.incubate.nn import functional as IF
    x = paddle.randn([3, 5, 16])
    w = paddle.randn([16, 24])
    b = paddle.randn([24])
    for act in (None, 'gelu', 'relu'):
        y = IF.fused_linear_activation(x, w, b, activation=act)
        z = x._t @ w._t + b._t
        ref = {None: z, 'gelu': torch.nn.functional.gelu(z), 'relu': torch.relu(z)}[act]
        assert torch.allclose(y._t, ref, atol=1e-5)
    y = IF.fused_linear_activation(x, paddle.Tensor(w._t.t().contiguous()), b, trans_y=True, activation='relu')
    assert torch.allclose(y._t, torch.relu(x._t @ w._t + b._t), atol=1e-5)
