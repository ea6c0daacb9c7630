"""Static-mode auto parallel: annotate a serial program, complete, partition per rank
(parity: reference test/auto_parallel/test_completion.py, test_partitioner.py,
test_dist_*_reshard). The partitioned programs must compute the serial loss and, after one
optimizer step, hold exactly the slices of the serially updated parameters."""
import numpy as np
import pytest

from dist_utils import run_ranks

pytestmark = pytest.mark.timeout(300) if hasattr(pytest.mark, 'timeout') else []

B, H, F_, C = 8, 6, 8, 4


def _build(specs, mesh):
    """Serial MLP + cross-entropy, annotated with `specs` (None = leave replicated)."""
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn as nn
    import paddle_ray_amd.nn.functional as F
    from paddle_ray_amd import static
    from paddle_ray_amd.distributed import auto_parallel as ap
    paddle.seed(7)
    main = static.Program()
    with static.program_guard(main):
        x = static.data('x', [B, H], 'float32')
        y = static.data('y', [B, 1], 'int64')
        l1, l2 = nn.Linear(H, F_), nn.Linear(F_, C)
        for t, key in ((x, 'x'), (y, 'y'), (l1.weight, 'w1'), (l1.bias, 'b1'), (l2.weight, 'w2')):
            if specs.get(key) is not None:
                ap.shard_tensor(t, mesh, specs[key])
        h = F.gelu(l1(x))
        loss = F.cross_entropy(l2(h), y)
    return main, x, y, h, loss, (l1.weight, l1.bias, l2.weight, l2.bias)


def _data():
    rs = np.random.RandomState(3)
    return rs.randn(B, H).astype('float32'), rs.randint(0, C, (B, 1)).astype('int64')


def _slice(a, mapping, mesh_shape, coord):
    for i, d in enumerate(mapping):
        if d >= 0:
            n = a.shape[i] // mesh_shape[d]
            a = np.take(a, range(coord[d] * n, (coord[d] + 1) * n), axis=i)
    return a


def _run(rank, world, mesh_ids, names, specs):
    import paddle_ray_amd as paddle
    from paddle_ray_amd import static
    from paddle_ray_amd.distributed import auto_parallel as ap
    paddle.enable_static()
    mesh = ap.ProcessMesh(mesh_ids, names)
    main, x, y, h, loss, params = _build(specs, mesh)
    dist, vmap, part = ap.parallelize(main)
    local = [part.local_param(p) for p in params]
    with static.program_guard(dist):
        paddle.optimizer.SGD(0.5, parameters=local).minimize(vmap[loss])
    with static.program_guard(main):
        paddle.optimizer.SGD(0.5, parameters=list(params)).minimize(loss)
    exe = static.Executor()
    xv, yv = _data()
    ref_loss, = exe.run(main, feed={'x': xv, 'y': yv}, fetch_list=[loss])
    d_loss, = exe.run(dist, feed={'x': xv, 'y': yv}, fetch_list=[vmap[loss]])
    coord = mesh.coord()
    errs = []
    for p, lp in zip(params, local):
        want = _slice(p.numpy(), part.ctx.get(p), mesh.shape, coord)
        got = lp.numpy()
        assert got.shape == want.shape, (got.shape, want.shape)
        errs.append(float(np.abs(got - want).max()))
    mapping = {'h': part.ctx.get(h), 'w2': part.ctx.get(params[2])}
    comm = [op.type for op in dist.global_block().ops
            if op.role == 'forward' and op.type.startswith('ap_')]
    ops = [op.type for op in dist.global_block().ops]
    paddle.disable_static()
    return {'ref': float(ref_loss), 'loss': float(d_loss), 'errs': errs, 'map': mapping,
            'comm': comm, 'ops': ops, 'shapes': [list(lp.shape) for lp in local]}


def test_completion_rules_single_process():
    import paddle_ray_amd as paddle
    from paddle_ray_amd.distributed import auto_parallel as ap
    paddle.enable_static()
    try:
        mesh = ap.ProcessMesh([[0, 1], [2, 3]], ['dp', 'mp'])
        main, x, y, h, loss, (w1, b1, w2, b2) = _build(
            {'x': ['dp', None], 'w1': [None, 'mp'], 'b1': ['mp'], 'w2': ['mp', None]}, mesh)
        ctx = ap.DistributedContext(main)
        ap.Completer(ctx).complete_forward_annotation()
        assert ctx.shard_spec(h) == ['dp', 'mp']          # batch from x, column from w1
        assert ctx.get(loss) == []
        plans = {op.type.rsplit(':', 1)[-1]: (req, outs, partial) for op, req, outs, partial in ctx.plans}
        req, outs, partial = plans['cross_entropy']
        assert outs == [[]] and partial == {0: 'avg'}      # mean over the dp-split batch
        lin2 = [p for p in ctx.plans if p[0].type.endswith(':linear')][1]
        assert lin2[2] == [[0, -1]] and lin2[3] == {1: 'sum'}   # row-parallel: partial over mp
    finally:
        paddle.disable_static()


@pytest.mark.parametrize('kind', ['tp', 'dp'])
def test_partitioned_step_matches_serial_2ranks(tmp_path, kind):
    specs = {'tp': {'w1': [None, 'x'], 'b1': ['x'], 'w2': ['x', None]},
             'dp': {'x': ['x', None], 'y': ['x', None]}}[kind]
    res = run_ranks(_run, 2, tmp_path, args=([0, 1], ['x'], specs))
    for o in res:
        assert abs(o['loss'] - o['ref']) < 1e-5, o
        assert max(o['errs']) < 1e-5, o
    if kind == 'tp':
        assert res[0]['shapes'][0] == [H, F_ // 2] and res[0]['shapes'][2] == [F_ // 2, C]
        # Megatron MLP on a data input (no grad): one forward all-reduce after the
        # row-parallel matmul and nothing else
        assert res[0]['comm'] == ['ap_allreduce'], res[0]['comm']
        assert res[0]['map']['h'] == [-1, 0]
    else:
        assert res[0]['shapes'][0] == [H, F_]
        # replicated parameters: no per-parameter identity / backward all-reduce op; their
        # gradients go through the bucketed async all-reduce inserted at minimize
        assert set(res[0]['comm']) == {'ap_slice', 'ap_allreduce'}, res[0]['comm']
        assert 'c_allreduce_coalesced' in res[0]['ops']


def test_partitioned_step_hybrid_2x2(tmp_path):
    specs = {'x': ['dp', None], 'y': ['dp', None], 'w1': [None, 'mp'], 'b1': ['mp'],
             'w2': ['mp', None]}
    res = run_ranks(_run, 4, tmp_path, args=([[0, 1], [2, 3]], ['dp', 'mp'], specs))
    for o in res:
        assert abs(o['loss'] - o['ref']) < 1e-5, o
        assert max(o['errs']) < 1e-5, o
        assert o['map']['h'] == [0, 1]


def _run_reshard(rank, world):
    """Column-parallel layer on an activation, then a softmax that needs the whole row:
    the partitioner inserts identity (bwd all-reduce) on the activation and an all-gather
    before the softmax."""
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn as nn
    import paddle_ray_amd.nn.functional as F
    from paddle_ray_amd import static
    from paddle_ray_amd.distributed import auto_parallel as ap
    paddle.enable_static()
    paddle.seed(11)
    mesh = ap.ProcessMesh([0, 1], ['mp'])
    main = static.Program()
    with static.program_guard(main):
        x = static.data('x', [B, H], 'float32')
        l0, l1, l2 = nn.Linear(H, H), nn.Linear(H, F_), nn.Linear(F_, C)
        ap.shard_tensor(l1.weight, mesh, [None, 'mp'])
        s = F.softmax(l1(F.relu(l0(x))), axis=-1)
        loss = paddle.mean(paddle.sum(l2(s) * l2(s), axis=-1))
    params = [l0.weight, l0.bias, l1.weight, l1.bias, l2.weight, l2.bias]
    dist, vmap, part = ap.parallelize(main)
    local = [part.local_param(p) for p in params]
    with static.program_guard(dist):
        paddle.optimizer.SGD(0.5, parameters=local).minimize(vmap[loss])
    with static.program_guard(main):
        paddle.optimizer.SGD(0.5, parameters=params).minimize(loss)
    exe = static.Executor()
    xv = _data()[0]
    ref, = exe.run(main, feed={'x': xv}, fetch_list=[loss])
    got, = exe.run(dist, feed={'x': xv}, fetch_list=[vmap[loss]])
    errs = [float(np.abs(lp.numpy() - _slice(p.numpy(), part.ctx.get(p), mesh.shape, mesh.coord())).max())
            for p, lp in zip(params, local)]
    comm = [op.type for op in dist.global_block().ops
            if op.role == 'forward' and op.type.startswith('ap_')]
    paddle.disable_static()
    return {'ref': float(ref), 'loss': float(got), 'errs': errs, 'comm': comm}


def test_partitioner_reshard_before_softmax(tmp_path):
    for o in run_ranks(_run_reshard, 2, tmp_path):
        assert abs(o['loss'] - o['ref']) < 1e-5, o
        assert max(o['errs']) < 1e-5, o
        assert o['comm'] == ['ap_identity', 'ap_gather'], o['comm']


def _run_embed(rank, world):
    """Hidden-split embedding table -> scalar scale (keeps the split) -> row-parallel linear:
    one all-reduce in the forward, and one SGD step equals the serial step."""
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn as nn
    import paddle_ray_amd.nn.functional as F
    from paddle_ray_amd import static
    from paddle_ray_amd.distributed import auto_parallel as ap
    paddle.enable_static()
    paddle.seed(5)
    mesh = ap.ProcessMesh([0, 1], ['mp'])
    V, S_ = 32, 6
    main = static.Program()
    with static.program_guard(main):
        ids = static.data('ids', [B, S_], 'int64')
        lbl = static.data('lbl', [B, S_, 1], 'int64')
        emb, head = nn.Embedding(V, H), nn.Linear(H, C)
        ap.shard_tensor(emb.weight, mesh, [None, 'mp'])
        ap.shard_tensor(head.weight, mesh, ['mp', None])
        loss = F.cross_entropy(head(emb(ids) * 0.5), lbl)
    params = [emb.weight, head.weight, head.bias]
    dist, vmap, part = ap.parallelize(main)
    local = [part.local_param(p) for p in params]
    with static.program_guard(dist):
        paddle.optimizer.SGD(0.5, parameters=local).minimize(vmap[loss])
    with static.program_guard(main):
        paddle.optimizer.SGD(0.5, parameters=params).minimize(loss)
    rs = np.random.RandomState(9)
    feed = {'ids': rs.randint(0, V, (B, S_)).astype('int64'), 'lbl': rs.randint(0, C, (B, S_, 1)).astype('int64')}
    exe = static.Executor()
    ref, = exe.run(main, feed=feed, fetch_list=[loss])
    got, = exe.run(dist, feed=feed, fetch_list=[vmap[loss]])
    errs = [float(np.abs(lp.numpy() - _slice(p.numpy(), part.ctx.get(p), mesh.shape, mesh.coord())).max())
            for p, lp in zip(params, local)]
    comm = [op.type for op in dist.global_block().ops if op.role == 'forward' and op.type.startswith('ap_')]
    paddle.disable_static()
    return {'ref': float(ref), 'loss': float(got), 'errs': errs, 'comm': comm}


def test_partitioner_hidden_split_embedding(tmp_path):
    for o in run_ranks(_run_embed, 2, tmp_path):
        assert abs(o['loss'] - o['ref']) < 1e-5, o
        assert max(o['errs']) < 1e-5, o
        assert o['comm'] == ['ap_allreduce'], o['comm']


def _engine_static(rank, world, annotate, ckpt=None):
    """auto_parallel.Engine on a static program: the model is built in static mode (shard_tensor
    annotates its weights), prepare() completes + partitions, fit() trains."""
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn as nn
    import paddle_ray_amd.nn.functional as F
    from paddle_ray_amd.distributed import auto_parallel as ap
    from paddle_ray_amd.static import InputSpec
    from paddle_ray_amd.io import Dataset
    paddle.enable_static()
    paddle.seed(3)
    mesh = ap.ProcessMesh([0, 1], ['mp'])

    class MLP(nn.Layer):
        def __init__(self):
            super().__init__()
            self.l1, self.l2 = nn.Linear(H, F_), nn.Linear(F_, C)
            if annotate:
                ap.shard_tensor(self.l1.weight, mesh, [None, 'mp'])
                ap.shard_tensor(self.l1.bias, mesh, ['mp'])
                ap.shard_tensor(self.l2.weight, mesh, ['mp', None])

        def forward(self, x):
            return self.l2(F.relu(self.l1(x)))

    class DS(Dataset):
        def __init__(self):
            rs = np.random.RandomState(0)
            self.x = rs.randn(32, H).astype('float32')
            self.y = rs.randint(0, C, (32, 1)).astype('int64')

        def __getitem__(self, i):
            return self.x[i], self.y[i]

        def __len__(self):
            return 32

    specs = ([InputSpec([B, H], 'float32', 'x')], [InputSpec([B, 1], 'int64', 'y')])
    model = MLP()
    opt = paddle.optimizer.Momentum(0.2, momentum=0.9, parameters=model.parameters())
    eng = ap.Engine(model, nn.CrossEntropyLoss(), opt)
    eng.prepare(*specs)
    hist = eng.fit(DS(), batch_size=B, epochs=2, verbose=0)
    ev = eng.evaluate(DS(), batch_size=B, verbose=0)
    shapes = [list(p.shape) for p in eng.local_parameters()]
    out = {'loss': hist['loss'], 'eval': ev['loss'], 'shapes': shapes}
    if ckpt is not None:
        # save after fit (gathered full tensors), predict through the partitioned program, then
        # a fresh engine (other init) loads the checkpoint: same predictions, same next step
        pred = eng.predict(DS(), batch_size=B)
        eng.save(ckpt)
        more = eng.fit(DS(), batch_size=B, epochs=1, steps_per_epoch=2, verbose=0)['loss']
        paddle.seed(99)
        with paddle.utils.unique_name.guard():   # a fresh process's parameter names (.pdopt keys)
            model2 = MLP()
        opt2 = paddle.optimizer.Momentum(0.2, momentum=0.9, parameters=model2.parameters())
        eng2 = ap.Engine(model2, nn.CrossEntropyLoss(), opt2)
        eng2.prepare(*specs)
        eng2.load(ckpt)
        pred2 = eng2.predict(DS(), batch_size=B)
        more2 = eng2.fit(DS(), batch_size=B, epochs=1, steps_per_epoch=2, verbose=0)['loss']
        from paddle_ray_amd.framework.io import load
        saved = {k: v.numpy() for k, v in load(ckpt + '.pdparams').items()}
        out.update(pred=[p[0] for p in pred], pred2=[p[0] for p in pred2], more=more, more2=more2,
                   saved=saved)
    paddle.disable_static()
    return out


def test_engine_static_partitioned_matches_serial(tmp_path):
    (tmp_path / 'ref').mkdir()
    (tmp_path / 'tp').mkdir()
    ref = run_ranks(_engine_static, 2, tmp_path / 'ref', (False,))[0]
    res = run_ranks(_engine_static, 2, tmp_path / 'tp', (True,))
    assert res[0]['shapes'][0] == [H, F_ // 2] and res[0]['shapes'][2] == [F_ // 2, C]
    for o in res:
        np.testing.assert_allclose(o['loss'], ref['loss'], rtol=1e-5, atol=1e-6)
        assert abs(o['eval'] - ref['eval']) < 1e-5
    assert ref['loss'][-1] < ref['loss'][0]


def test_engine_static_save_load_predict(tmp_path):
    """the static Engine saves the TRAINED shards (gathered to full tensors, same
    file as an unpartitioned run), load() puts a checkpoint back into the shards, predict()
    runs the partitioned program."""
    (tmp_path / 'ref').mkdir()
    (tmp_path / 'tp').mkdir()
    ref = run_ranks(_engine_static, 2, tmp_path / 'ref', (False, str(tmp_path / 'ref' / 'ck')))[0]
    res = run_ranks(_engine_static, 2, tmp_path / 'tp', (True, str(tmp_path / 'tp' / 'ck')))
    for k, v in ref['saved'].items():
        np.testing.assert_allclose(res[0]['saved'][k], v, rtol=1e-5, atol=1e-6)
    for o in res + [ref]:
        for a, b in zip(o['pred'], o['pred2']):
            np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(o['more'], o['more2'], rtol=1e-5, atol=1e-6)
    for a, b in zip(res[0]['pred'], ref['pred']):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-5)


def _run_dp_trace(rank, world, bucket_mb):
    """Data-parallel partitioned step under CommTrace: the gradient all-reduces."""
    import paddle_ray_amd as paddle
    from paddle_ray_amd import static
    from paddle_ray_amd.distributed import auto_parallel as ap
    from paddle_ray_amd.distributed.comm_trace import CommTrace
    paddle.enable_static()
    mesh = ap.ProcessMesh(list(range(world)), ['dp'])
    main, x, y, h, loss, params = _build({'x': ['dp', None], 'y': ['dp', None]}, mesh)
    dist, vmap, part = ap.parallelize(main)
    dist.__dict__['_ap_bucket_mb'] = bucket_mb
    local = [part.local_param(p) for p in params]
    with static.program_guard(dist):
        paddle.optimizer.SGD(0.5, parameters=local).minimize(vmap[loss])
    with static.program_guard(main):
        paddle.optimizer.SGD(0.5, parameters=list(params)).minimize(loss)
    exe = static.Executor()
    xv, yv = _data()
    exe.run(main, feed={'x': xv, 'y': yv}, fetch_list=[loss])
    with CommTrace() as tr:
        exe.run(dist, feed={'x': xv, 'y': yv}, fetch_list=[vmap[loss]])
    ars = [(r.bytes, r.async_op, tuple(r.ranks)) for r in tr.ops('all_reduce')]
    ops = [op.type for op in dist.global_block().ops]
    errs = [float(np.abs(lp.numpy() - p.numpy()).max()) for p, lp in zip(params, local)]
    paddle.disable_static()
    return {'ars': ars, 'ops': ops, 'errs': errs,
            'pbytes': [int(np.prod(p.shape)) * 4 for p in local]}


@pytest.mark.parametrize('bucket_mb,nb', [(32, 1), (1e-6, 4)])
def test_auto_parallel_dp_bucketed_grad_allreduce(tmp_path, bucket_mb, nb):
    """world 4, pure data parallel: the replicated parameters' gradients are all-reduced in
    `nb` flat buckets (async, issued from inside the backward), not one synchronous all-reduce
    per parameter; the partitioned step still matches the serial one."""
    res = run_ranks(_run_dp_trace, 4, tmp_path, args=(bucket_mb,))
    for o in res:
        assert max(o['errs']) < 1e-5, o
        grad_ars = [a for a in o['ars'] if a[1]]          # the async (gradient) all-reduces
        assert len(grad_ars) == nb, o['ars']
        assert sum(a[0] for a in grad_ars) == sum(o['pbytes'])
        assert all(a[2] == (0, 1, 2, 3) for a in grad_ars)
        ops = o['ops']
        ar = [i for i, t in enumerate(ops) if t == 'c_allreduce_coalesced']
        grads = [i for i, t in enumerate(ops) if t.endswith('_grad') or t == 'grad']
        assert len(ar) == nb and ops.count('ap_identity') == 0
        if nb > 1:
            assert ar[0] < grads[-1], ops           # the first bucket leaves before the backward ends
