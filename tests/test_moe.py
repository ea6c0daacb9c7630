"""MoE layer (gates, capacity, expert-parallel all_to_all) vs a dense per-token reference,
single-process and on 2 gloo ranks (parity: reference test_moe_api / collective
global_scatter/global_gather tests)."""
import numpy as np
import pytest
import torch

import paddle_ray_amd as paddle
from paddle_ray_amd import nn
from paddle_ray_amd.distributed.models.moe import utils as U
from paddle_ray_amd.incubate.distributed.models.moe import MoELayer, NaiveGate

from dist_utils import run_ranks  # noqa: E402


class Expert(nn.Layer):
    def __init__(self, d, h):
        super().__init__()
        self.a = nn.Linear(d, h)
        self.b = nn.Linear(h, d)

    def forward(self, x):
        return self.b(paddle.nn.functional.gelu(self.a(x)))


def _dense_ref(x, gate, experts, top_k):
    """out[t] = sum_k val[t,k] * expert_{idx[t,k]}(x[t])."""
    t = x._t.reshape(-1, x.shape[-1])
    g = gate.gate(paddle.Tensor(t))._t
    val, idx = torch.topk(g, top_k, dim=-1, sorted=False)
    out = torch.zeros_like(t)
    for i in range(t.shape[0]):
        for k in range(top_k):
            e = int(idx[i, k])
            out[i] += val[i, k] * experts[e](paddle.Tensor(t[i:i + 1]))._t[0]
    return out.reshape(x.shape)


def test_routing_utils():
    idx = paddle.to_tensor(np.array([[0, 2], [2, 1], [2, -1], [0, 2]], dtype=np.int64))
    cnt = U._number_count(idx, 4).numpy()
    assert cnt.tolist() == [2, 1, 4, 0]
    pos = U._assign_pos(idx, paddle.to_tensor(np.cumsum(cnt))).numpy()
    assert pos.tolist() == [0, 6, 3, 1, 2, 4, 7]
    # expert 2 capacity 2: keeps its first two routes (flat order), drops the rest
    pruned = U._prune_gate_by_capacity(idx, paddle.to_tensor(np.array([2, 1, 2, 0])), 4, 1)
    assert pruned.numpy().tolist() == [[0, 2], [2, 1], [-1, -1], [0, -1]]
    lim = U._limit_by_capacity(paddle.to_tensor(np.array([3, 1, 2, 5])),
                               paddle.to_tensor(np.array([4, 4])), 2).numpy()
    assert lim.tolist() == [3, 1, 1, 3]
    rr = U._random_routing(paddle.to_tensor(np.array([[0, 1], [1, 0]])),
                           paddle.to_tensor(np.array([[0.9, 0.1], [0.9, 0.6]], np.float32)),
                           paddle.to_tensor(np.array([0.5, 0.5], np.float32))).numpy()
    assert rr.tolist() == [[0, -1], [1, 0]]


def test_moe_layer_matches_dense():
    paddle.seed(3)
    d = 16
    experts = nn.LayerList([Expert(d, 32) for _ in range(4)])
    gate = NaiveGate(d, 4, 1, topk=2)
    moe = MoELayer(d, experts, gate=gate)
    x = paddle.randn([2, 6, d])
    x.stop_gradient = False
    y = moe(x)
    ref = _dense_ref(x, gate, experts, 2)
    np.testing.assert_allclose(y.numpy(), ref.detach().numpy(), rtol=1e-4, atol=1e-5)
    gx = paddle.grad(y.sum(), [x])[0].numpy()
    xr = x.detach()
    xr.stop_gradient = False
    gr = paddle.grad(paddle.Tensor(_dense_ref(xr, gate, experts, 2)).sum(), [xr])[0].numpy()
    np.testing.assert_allclose(gx, gr, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize('kind', ['gshard', 'switch'])
def test_moe_gates_train(kind):
    paddle.seed(0)
    d = 8
    experts = nn.LayerList([Expert(d, 16) for _ in range(4)])
    moe = MoELayer(d, experts, gate={'type': kind, 'top_k': 2 if kind == 'gshard' else 1})
    opt = paddle.optimizer.Adam(1e-2, parameters=moe.parameters())
    x = paddle.randn([4, 8, d])
    tgt = paddle.randn([4, 8, d])
    losses = []
    for _ in range(15):
        out = moe(x)
        loss = ((out - tgt) ** 2).mean() + 0.01 * moe.gate.get_loss()
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
    assert losses[-1] < losses[0]


def _ep_worker(rank, world):
    import paddle_ray_amd as paddle
    from paddle_ray_amd import nn
    from paddle_ray_amd.incubate.distributed.models.moe import MoELayer, NaiveGate
    paddle.seed(7)
    d, ne = 16, 2
    all_experts = [Expert(d, 24) for _ in range(ne * world)]   # identical on every rank
    gate = NaiveGate(d, ne, world, topk=2)                       # 4 global experts
    paddle.seed(100 + rank)
    x = paddle.randn([2, 5, d])                                  # different tokens per rank
    x.stop_gradient = False
    group = paddle.distributed.new_group(list(range(world)))
    local = nn.LayerList(all_experts[rank * ne:(rank + 1) * ne])
    moe = MoELayer(d, local, gate=gate, moe_group=group)
    y = moe(x)
    gx = paddle.grad(y.sum(), [x])[0]
    ref = _dense_ref(x, gate, all_experts, 2)
    return y.numpy(), ref.detach().numpy(), gx.numpy()


def test_moe_expert_parallel_gloo(tmp_path):
    res = run_ranks(_ep_worker, 2, tmp_path)
    for y, ref, gx in res:
        np.testing.assert_allclose(y, ref, rtol=1e-4, atol=1e-5)
        assert np.isfinite(gx).all() and np.abs(gx).sum() > 0


def _scatter_worker(rank, world):
    import paddle_ray_amd as paddle
    from paddle_ray_amd.distributed.utils import global_scatter, global_gather
    ne = 2
    # rank r sends (r + 1) rows to every global expert g, values encode (src, g)
    lc = [rank + 1] * (ne * world)
    rows = []
    for g in range(ne * world):
        rows += [[rank * 100 + g]] * (rank + 1)
    x = paddle.to_tensor(np.array(rows, dtype=np.float32))
    gc = [w + 1 for w in range(world) for _ in range(ne)]
    y = global_scatter(x, lc, gc)
    back = global_gather(y, lc, gc)
    return y.numpy().ravel().tolist(), back.numpy().ravel().tolist(), x.numpy().ravel().tolist()


def test_global_scatter_gather_gloo(tmp_path):
    res = run_ranks(_scatter_worker, 2, tmp_path)
    for rank, (y, back, x) in enumerate(res):
        exp = []
        for e in range(2):             # expert-major, source worker inner
            g = rank * 2 + e
            for w in range(2):
                exp += [w * 100 + g] * (w + 1)
        assert y == exp
        assert back == x


# ---------------------------------------------------------------- incubate optimizers
def _quad_model():
    paddle.seed(1)
    return nn.Linear(4, 1)


def _loss(m, x, y):
    return ((m(x) - y) ** 2).mean()


def test_lookahead_and_model_average():
    from paddle_ray_amd.incubate import LookAhead, ModelAverage
    m = _quad_model()
    x, y = paddle.randn([32, 4]), paddle.randn([32, 1])
    inner = paddle.optimizer.SGD(0.1, parameters=m.parameters())
    la = LookAhead(inner, alpha=0.5, k=3)
    ma = ModelAverage(0.5, parameters=m.parameters(), min_average_window=2,
                      max_average_window=4)
    w_hist = []
    first = None
    for i in range(6):
        loss = _loss(m, x, y)
        first = first if first is not None else float(loss)
        loss.backward()
        la.step()
        ma.step()
        la.clear_grad()
        w_hist.append(m.weight.numpy().copy())
    assert float(_loss(m, x, y)) < first
    w = m.weight.numpy().copy()
    with ma.apply():
        avg = m.weight.numpy().copy()
        assert not np.allclose(avg, w)
    np.testing.assert_allclose(m.weight.numpy(), w)


def test_lbfgs_and_functional_minimizers():
    from paddle_ray_amd.incubate.optimizer import LBFGS
    from paddle_ray_amd.incubate.optimizer.functional import minimize_bfgs, minimize_lbfgs
    m = _quad_model()
    x, y = paddle.randn([64, 4]), paddle.randn([64, 1])
    opt = LBFGS(1.0, max_iter=50, line_search_fn='strong_wolfe', parameters=m.parameters())

    def closure():
        opt.clear_grad()
        loss = _loss(m, x, y)
        loss.backward()
        return loss
    l0 = float(_loss(m, x, y))
    opt.step(closure)
    # least squares optimum
    X = np.concatenate([x.numpy(), np.ones((64, 1), np.float32)], 1)
    sol, *_ = np.linalg.lstsq(X, y.numpy(), rcond=None)
    best = float(((X @ sol - y.numpy()) ** 2).mean())
    assert float(_loss(m, x, y)) <= best + 1e-4 < l0

    A = paddle.to_tensor(np.diag([1.0, 4.0, 9.0]).astype(np.float32))
    f = lambda v: (paddle.matmul(paddle.matmul(v.unsqueeze(0), A), v.unsqueeze(1)).sum()
                   - v.sum())
    x0 = paddle.to_tensor(np.zeros(3, np.float32))
    for fn in (minimize_bfgs, minimize_lbfgs):
        out = fn(f, x0)
        assert bool(out[0].numpy())
        np.testing.assert_allclose(out[2].numpy(), [0.5, 0.125, 1 / 18], rtol=1e-3, atol=1e-4)


def test_distributed_fused_lamb_single():
    from paddle_ray_amd.incubate import DistributedFusedLamb
    m = _quad_model()
    x, y = paddle.randn([32, 4]), paddle.randn([32, 1])
    opt = DistributedFusedLamb(0.05, parameters=m.parameters(),
                               grad_clip=nn.ClipGradByGlobalNorm(1.0),
                               gradient_accumulation_steps=2)
    l0 = float(_loss(m, x, y))
    for _ in range(20):
        _loss(m, x, y).backward()
        opt.step()
        opt.clear_grad()
    assert float(_loss(m, x, y)) < l0


def test_autotune_set_config_cpu():
    from paddle_ray_amd.incubate import autotune
    cfg = autotune.set_config({'kernel': {'enable': True, 'tuning_range': [1, 3]},
                               'layout': {'enable': False}})
    assert cfg['kernel']['tuning_range'] == [1, 3]
    assert paddle.get_flags('FLAGS_cudnn_exhaustive_search')['FLAGS_cudnn_exhaustive_search']
    autotune.set_config({'kernel': {'enable': False}})
    assert not paddle.get_flags('FLAGS_cudnn_exhaustive_search')['FLAGS_cudnn_exhaustive_search']
