"""Multi-process CPU (gloo) tests: collectives, DataParallel, sharding 1/2/3, TP, PP parity.

Reference strategy: python/paddle/fluid/tests/unittests/test_dist_base.py trains the
same model single-process and multi-process and compares losses/params.
"""
import numpy as np
import pytest

from dist_utils import run_ranks

pytestmark = pytest.mark.timeout(300) if hasattr(pytest.mark, 'timeout') else []


# ---------------------------------------------------------------------------------------------
def _collectives(rank, world):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.distributed as dist
    out = {}
    t = paddle.to_tensor([float(rank + 1)] * 4)
    dist.all_reduce(t)
    out['all_reduce'] = t.numpy()
    lst = []
    dist.all_gather(lst, paddle.to_tensor([rank]))
    out['all_gather'] = [x.numpy() for x in lst]
    b = paddle.to_tensor([rank * 10.])
    dist.broadcast(b, src=1)
    out['broadcast'] = b.numpy()
    rs = paddle.zeros([2])
    dist.reduce_scatter(rs, [paddle.to_tensor([1., 2.]) * (rank + 1),
                             paddle.to_tensor([3., 4.]) * (rank + 1)])
    out['reduce_scatter'] = rs.numpy()
    objs = []
    dist.all_gather_object(objs, {'r': rank})
    out['objs'] = objs
    o = []
    dist.alltoall([paddle.to_tensor([rank * 2.]), paddle.to_tensor([rank * 2. + 1])], o)
    out['alltoall'] = [x.numpy() for x in o]
    if rank == 0:
        dist.send(paddle.to_tensor([42.]), dst=1)
    else:
        r = paddle.zeros([1])
        dist.recv(r, src=0)
        out['recv'] = r.numpy()
    g = dist.new_group([0, 1])
    t2 = paddle.to_tensor([1.])
    dist.all_reduce(t2, group=g)
    out['group'] = t2.numpy()
    return out


def test_collectives(tmp_path):
    res = run_ranks(_collectives, 2, tmp_path)
    for r in res:
        np.testing.assert_allclose(r['all_reduce'], [3.] * 4)
        assert [int(x[0]) for x in r['all_gather']] == [0, 1]
        np.testing.assert_allclose(r['broadcast'], [10.])
        assert r['objs'] == [{'r': 0}, {'r': 1}]
        np.testing.assert_allclose(r['group'], [2.])
    np.testing.assert_allclose(res[0]['reduce_scatter'], [3., 6.])
    np.testing.assert_allclose(res[1]['reduce_scatter'], [9., 12.])
    np.testing.assert_allclose([x[0] for x in res[0]['alltoall']], [0., 2.])
    np.testing.assert_allclose([x[0] for x in res[1]['alltoall']], [1., 3.])
    np.testing.assert_allclose(res[1]['recv'], [42.])


# ---------------------------------------------------------------------------------------------
def _make_mlp(seed=0):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn as nn
    paddle.seed(seed)
    return nn.Sequential(nn.Linear(8, 32), nn.GELU(), nn.Linear(32, 32), nn.Tanh(),
                         nn.Linear(32, 4))


def _data(n=16, seed=1):
    rng = np.random.RandomState(seed)
    return rng.rand(n, 8).astype('float32'), rng.rand(n, 4).astype('float32')


def _train(model, opt, xs, ys, steps=4, wrap_step=None):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn.functional as F
    losses = []
    for _ in range(steps):
        loss = F.mse_loss(model(paddle.to_tensor(xs)), paddle.to_tensor(ys))
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
    return losses


def _single_reference(steps=4, clip=False, opt='adamw'):
    import paddle_ray_amd as paddle
    m = _make_mlp()
    kw = dict(parameters=m.parameters())
    if clip:
        kw['grad_clip'] = paddle.nn.ClipGradByGlobalNorm(0.5)
    o = paddle.optimizer.AdamW(0.01, weight_decay=0.01, **kw) if opt == 'adamw' else \
        paddle.optimizer.Momentum(0.05, 0.9, **kw)
    xs, ys = _data()
    _train(m, o, xs, ys, steps)
    return [p.numpy() for p in m.parameters()]


def _dp_worker(rank, world):
    import paddle_ray_amd as paddle
    m = _make_mlp()
    dp = paddle.DataParallel(m, comm_buffer_size=1)
    o = paddle.optimizer.AdamW(0.01, parameters=m.parameters(), weight_decay=0.01)
    xs, ys = _data()
    n = len(xs) // world
    _train(dp, o, xs[rank * n:(rank + 1) * n], ys[rank * n:(rank + 1) * n])
    return [p.numpy() for p in m.parameters()]


def test_data_parallel_matches_single(tmp_path):
    ref = _single_reference()
    res = run_ranks(_dp_worker, 2, tmp_path)
    for r in res:
        for a, b in zip(r, ref):
            np.testing.assert_allclose(a, b, rtol=2e-4, atol=2e-5)


def _sharding_worker(rank, world, level, clip, opt):
    import paddle_ray_amd as paddle
    from paddle_ray_amd.distributed.sharding import group_sharded_parallel
    m = _make_mlp()
    kw = dict(parameters=m.parameters())
    if clip:
        kw['grad_clip'] = paddle.nn.ClipGradByGlobalNorm(0.5)
    o = paddle.optimizer.AdamW(0.01, weight_decay=0.01, **kw) if opt == 'adamw' else \
        paddle.optimizer.Momentum(0.05, 0.9, **kw)
    sm, so, _ = group_sharded_parallel(m, o, level, bucket_mb=0)  # tiny buckets: many units
    xs, ys = _data()
    n = len(xs) // world
    _train(sm, so, xs[rank * n:(rank + 1) * n], ys[rank * n:(rank + 1) * n])
    sm.state_dict()  # forces the stage-3 gather
    return [p.numpy() for p in m.parameters()]


@pytest.mark.parametrize('level', ['os', 'os_g', 'p_g_os'])
def test_sharding_matches_single(tmp_path, level):
    ref = _single_reference(clip=True)
    res = run_ranks(_sharding_worker, 2, tmp_path, (level, True, 'adamw'))
    for r in res:
        for a, b in zip(r, ref):
            np.testing.assert_allclose(a, b, rtol=2e-4, atol=2e-5)


def test_sharding_momentum(tmp_path):
    ref = _single_reference(opt='momentum')
    res = run_ranks(_sharding_worker, 2, tmp_path, ('p_g_os', False, 'momentum'))
    for a, b in zip(res[0], ref):
        np.testing.assert_allclose(a, b, rtol=2e-4, atol=2e-5)


# ---------------------------------------------------------------------------------------------
def _tp_worker(rank, world):
    import paddle_ray_amd as paddle
    from paddle_ray_amd.distributed import fleet
    from paddle_ray_amd.models import gpt_config, GPTForPretraining
    st = fleet.DistributedStrategy()
    st.hybrid_configs = {'dp_degree': 1, 'mp_degree': 2, 'pp_degree': 1}
    fleet.init(is_collective=True, strategy=st)
    paddle.seed(0)
    cfg = gpt_config('gpt3-tiny', mp_degree=2, hidden_dropout=0.0, num_layers=2)
    model = GPTForPretraining(cfg)
    ids = paddle.to_tensor(np.random.RandomState(0).randint(0, 1024, (2, 17)))
    loss = model(ids[:, :-1], ids[:, 1:])
    loss.backward()
    # gather TP shards of the first qkv weight to compare with the single-process model
    w = model.gpt.layers[0].attn.qkv_proj.weight
    return {'loss': float(loss), 'w_shape': w.shape,
            'emb_grad_norm': float(model.gpt.embeddings.word_embeddings.weight.grad.norm())}


def test_tensor_parallel_gpt(tmp_path):
    res = run_ranks(_tp_worker, 2, tmp_path)
    assert res[0]['w_shape'] == [128, 192]  # 3*128 / 2 columns per rank
    assert abs(res[0]['loss'] - res[1]['loss']) < 1e-5
    assert 5.5 < res[0]['loss'] < 8.0  # ~ln(1024) at init


def _tp_parity_worker(rank, world):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn.functional as F
    from paddle_ray_amd.distributed import fleet
    from paddle_ray_amd.parallel.tensor_parallel import ColumnParallelLinear, RowParallelLinear
    st = fleet.DistributedStrategy()
    st.hybrid_configs = {'dp_degree': 1, 'mp_degree': 2, 'pp_degree': 1}
    fleet.init(is_collective=True, strategy=st)
    rng = np.random.RandomState(0)
    w1, w2 = rng.rand(8, 16).astype('float32'), rng.rand(16, 8).astype('float32')
    col = ColumnParallelLinear(8, 16, has_bias=False, gather_output=False)
    row = RowParallelLinear(16, 8, has_bias=False, input_is_parallel=True)
    col.weight.set_value(w1[:, rank * 8:(rank + 1) * 8])
    row.weight.set_value(w2[rank * 8:(rank + 1) * 8])
    x = paddle.to_tensor(rng.rand(4, 8).astype('float32'), stop_gradient=False)
    y = row(F.relu(col(x)))
    y.sum().backward()
    return {'y': y.numpy(), 'xg': x.grad.numpy()}


def test_tensor_parallel_linear_parity(tmp_path):
    import torch
    res = run_ranks(_tp_parity_worker, 2, tmp_path)
    rng = np.random.RandomState(0)
    w1, w2 = rng.rand(8, 16).astype('float32'), rng.rand(16, 8).astype('float32')
    x = torch.tensor(rng.rand(4, 8).astype('float32'), requires_grad=True)
    y = torch.relu(x @ torch.tensor(w1)) @ torch.tensor(w2)
    y.sum().backward()
    for r in res:
        np.testing.assert_allclose(r['y'], y.detach().numpy(), rtol=1e-5)
        np.testing.assert_allclose(r['xg'], x.grad.numpy(), rtol=1e-5)


# ---------------------------------------------------------------------------------------------
def _pp_worker(rank, world):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn as nn
    import paddle_ray_amd.nn.functional as F
    from paddle_ray_amd.distributed import fleet
    from paddle_ray_amd.distributed.fleet.meta_parallel import LayerDesc, PipelineLayer
    st = fleet.DistributedStrategy()
    st.hybrid_configs = {'dp_degree': 1, 'mp_degree': 1, 'pp_degree': 2}
    st.pipeline_configs = {'micro_batch_size': 2, 'accumulate_steps': 4}
    fleet.init(is_collective=True, strategy=st)
    paddle.seed(0)
    descs = [LayerDesc(nn.Linear, 8, 16), LayerDesc(nn.Tanh), LayerDesc(nn.Linear, 16, 16),
             LayerDesc(nn.Tanh), LayerDesc(nn.Linear, 16, 4)]
    # build ALL layers identically on every rank (same RNG stream), keep the local stage
    pl = PipelineLayer(descs, num_stages=2, loss_fn=lambda o, y: F.mse_loss(o, y))
    # copy weights from the full single-process model built with the same seed
    paddle.seed(0)
    full = [d.build_layer() for d in descs]
    lo = pl.segment_parts[pl._stage_id]
    for i, l in enumerate(pl.run_function):
        l.set_state_dict(full[lo + i].state_dict())
    model = fleet.distributed_model(pl)
    opt = paddle.optimizer.SGD(0.1, parameters=pl.parameters())
    xs, ys = _data(8)
    losses = []
    for _ in range(3):
        losses.append(float(model.train_batch([paddle.to_tensor(xs), paddle.to_tensor(ys)], opt)))
    return {'losses': losses, 'nparams': len(pl.parameters())}


def test_pipeline_parallel_1f1b(tmp_path):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn as nn
    import paddle_ray_amd.nn.functional as F
    res = run_ranks(_pp_worker, 2, tmp_path)
    # single-process reference: same layers, same micro-batching (mean of micro losses)
    paddle.seed(0)
    layers = [nn.Linear(8, 16), nn.Tanh(), nn.Linear(16, 16), nn.Tanh(), nn.Linear(16, 4)]
    seq = nn.Sequential(*layers)
    opt = paddle.optimizer.SGD(0.1, parameters=seq.parameters())
    xs, ys = _data(8)
    ref = []
    for _ in range(3):
        tot = 0.
        for i in range(4):
            l = F.mse_loss(seq(paddle.to_tensor(xs[2 * i:2 * i + 2])),
                           paddle.to_tensor(ys[2 * i:2 * i + 2])) / 4
            l.backward()
            tot += float(l)
        opt.step()
        opt.clear_grad()
        ref.append(tot)
    np.testing.assert_allclose(res[0]['losses'], ref, rtol=1e-4)
    np.testing.assert_allclose(res[1]['losses'], ref, rtol=1e-4)


# ---------------------------------------------------------------------------------------------
def _watchdog_worker(rank, world):
    import time
    import paddle_ray_amd as paddle
    import paddle_ray_amd.distributed as dist
    from paddle_ray_amd.distributed import watchdog
    wd = watchdog.get_watchdog()
    wd.timeout_s, wd.poll_s = 0.5, 0.1
    hb = watchdog.Heartbeat(interval=0.2).start()
    time.sleep(0.3)
    alive = hb.dead_ranks(stale_s=5.0)
    if rank == 1:
        time.sleep(2.0)  # straggler: rank 0's all_reduce stays in flight
    t = paddle.to_tensor([1.0])
    dist.all_reduce(t)
    hb.stop()
    return {'reports': list(wd.reports), 'dead': alive, 'sum': float(t)}


def test_comm_watchdog_and_heartbeat(tmp_path):
    res = run_ranks(_watchdog_worker, 2, tmp_path)
    assert res[0]['sum'] == 2.0 and res[1]['sum'] == 2.0
    assert any("all_reduce" in m for m in res[0]['reports']), res[0]['reports']
    assert not res[1]['reports']
    assert res[0]['dead'] == [] and res[1]['dead'] == []
