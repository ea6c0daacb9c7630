"""ZeRO-3 parameter release, fleet hybrid sharding and distributed AMP (gloo, CPU).

Parity targets: group_sharded_stage3.py (_release_param / _allgather_buffer / backward
re-gather), fleet/model.py ShardingParallel + hybrid_parallel_optimizer.py sharding reduce,
hybrid_parallel_gradscaler.py found_inf MAX all-reduce."""
import numpy as np
import pytest

from dist_utils import run_ranks


def _deep_mlp(seed=0, n=6, width=16):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn as nn
    paddle.seed(seed)
    layers = [nn.Linear(8, width), nn.GELU()]
    for _ in range(n - 2):
        layers += [nn.Linear(width, width), nn.Tanh()]
    layers += [nn.Linear(width, 4)]
    return nn.Sequential(*layers)


def _data(n=16, seed=1):
    rng = np.random.RandomState(seed)
    return rng.rand(n, 8).astype('float32'), rng.rand(n, 4).astype('float32')


def _opt(paddle, params, clip=True):
    kw = dict(parameters=params)
    if clip:
        kw['grad_clip'] = paddle.nn.ClipGradByGlobalNorm(0.5)
    return paddle.optimizer.AdamW(0.01, weight_decay=0.01, **kw)


def _single_mlp(steps=4):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn.functional as F
    m = _deep_mlp()
    o = _opt(paddle, m.parameters())
    xs, ys = _data()
    for _ in range(steps):
        loss = F.mse_loss(m(paddle.to_tensor(xs)), paddle.to_tensor(ys))
        loss.backward()
        o.step()
        o.clear_grad()
    return [p.numpy() for p in m.parameters()]


def _zero3_worker(rank, world, steps=4):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn.functional as F
    from paddle_ray_amd.distributed.sharding import group_sharded_parallel
    m = _deep_mlp()
    o = _opt(paddle, m.parameters())
    sm, so, _ = group_sharded_parallel(m, o, 'p_g_os', segment_size=0, bucket_mb=1)
    st = sm._state
    unit_gids = [gi for u in st.unit_meta for gi in u.gids]
    xs, ys = _data()
    n = len(xs) // world
    xs, ys = xs[rank * n:(rank + 1) * n], ys[rank * n:(rank + 1) * n]
    freed_after_fwd, freed_after_step = [], []
    for _ in range(steps):
        out = sm(paddle.to_tensor(xs))
        freed_after_fwd.append(all(st.groups[gi].param_buf.untyped_storage().nbytes() == 0
                                   for gi in unit_gids))
        loss = F.mse_loss(out, paddle.to_tensor(ys))
        loss.backward()
        so.step()
        so.clear_grad()
        freed_after_step.append(all(st.groups[gi].resident_bytes() == 0 for gi in unit_gids))
    sd = sm.state_dict()
    return {'params': [sd[k].numpy() for k in sd], 'n_units': len(st.unit_meta),
            'freed_fwd': freed_after_fwd, 'freed_step': freed_after_step,
            'peak': st.peak_resident_bytes, 'full': st.full_bytes()}


def test_zero3_releases_params_and_matches_single(tmp_path):
    ref = _single_mlp()
    res = run_ranks(_zero3_worker, 2, tmp_path)
    for r in res:
        assert r['n_units'] == 6
        assert all(r['freed_fwd']) and all(r['freed_step'])
        # only ~2 units (current + prefetched) are ever gathered at once
        assert r['peak'] < 0.6 * r['full'], (r['peak'], r['full'])
        for a, b in zip(r['params'], ref):
            np.testing.assert_allclose(a, b, rtol=2e-4, atol=2e-5)


def _gpt_cfg(recompute):
    from paddle_ray_amd.models import gpt_config
    return gpt_config('gpt3-tiny', num_layers=3, hidden_dropout=0.0, recompute=recompute)


def _gpt_batch():
    return np.random.RandomState(3).randint(0, 1024, (4, 17))


def _gpt_single(recompute, steps=3):
    import paddle_ray_amd as paddle
    from paddle_ray_amd.models import GPTForPretraining
    paddle.seed(0)
    m = GPTForPretraining(_gpt_cfg(recompute))
    o = _opt(paddle, m.parameters())
    ids = paddle.to_tensor(_gpt_batch())
    losses = []
    for _ in range(steps):
        loss = m(ids[:, :-1], ids[:, 1:])
        loss.backward()
        o.step()
        o.clear_grad()
        losses.append(float(loss))
    return losses, {k: v.numpy() for k, v in m.state_dict().items()}


def _gpt_zero3_worker(rank, world, recompute, steps=3):
    import paddle_ray_amd as paddle
    from paddle_ray_amd.models import GPTForPretraining
    from paddle_ray_amd.distributed.sharding import group_sharded_parallel
    paddle.seed(0)
    m = GPTForPretraining(_gpt_cfg(recompute))
    o = _opt(paddle, m.parameters())
    sm, so, _ = group_sharded_parallel(m, o, 'p_g_os', segment_size=4096, bucket_mb=1)
    ids = paddle.to_tensor(_gpt_batch()[rank * 2:(rank + 1) * 2])
    losses = []
    for _ in range(steps):
        loss = sm(ids[:, :-1], ids[:, 1:])
        loss.backward()
        so.step()
        so.clear_grad()
        t = paddle.to_tensor([float(loss)])
        paddle.distributed.all_reduce(t)
        losses.append(float(t) / world)
    sd = sm.state_dict()
    return losses, {k: v.numpy() for k, v in sd.items()}, len(sm._state.unit_meta)


@pytest.mark.parametrize('recompute', [False, True])
def test_zero3_gpt_blocks_match_single(tmp_path, recompute):
    ref_losses, ref_sd = _gpt_single(recompute)
    res = run_ranks(_gpt_zero3_worker, 2, tmp_path, (recompute,))
    for losses, sd, n_units in res:
        assert n_units == 3  # one unit per transformer block
        np.testing.assert_allclose(losses, ref_losses, rtol=1e-4, atol=1e-5)
        for k, v in ref_sd.items():
            np.testing.assert_allclose(sd[k], v, rtol=5e-4, atol=5e-5, err_msg=k)


# -- fleet hybrid sharding -------------------------------------------------------------------
def _fleet_worker(rank, world, hybrid):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn.functional as F
    from paddle_ray_amd.distributed import fleet
    st = fleet.DistributedStrategy()
    st.hybrid_configs = hybrid
    fleet.init(is_collective=True, strategy=st)
    hcg = fleet.get_hybrid_communicate_group()
    m = _deep_mlp()
    o = _opt(paddle, m.parameters())
    m = fleet.distributed_model(m)
    o = fleet.distributed_optimizer(o)
    xs, ys = _data()
    n = len(xs) // world
    xs, ys = xs[rank * n:(rank + 1) * n], ys[rank * n:(rank + 1) * n]
    for _ in range(4):
        loss = F.mse_loss(m(paddle.to_tensor(xs)), paddle.to_tensor(ys))
        loss.backward()
        o.step()
        o.clear_grad()
    sd = m.state_dict()
    return {'params': [sd[k].numpy() for k in sd], 'sh': hcg.get_sharding_parallel_world_size(),
            'dp': hcg.get_data_parallel_world_size()}


@pytest.mark.parametrize('world,hybrid', [
    (2, {'sharding_degree': 2, 'dp_degree': 1}),
    (4, {'sharding_degree': 2, 'dp_degree': 2}),
])
def test_fleet_sharding_matches_single(tmp_path, world, hybrid):
    ref = _single_mlp()
    res = run_ranks(_fleet_worker, world, tmp_path, (hybrid,))
    for r in res:
        assert r['sh'] == 2 and r['dp'] == hybrid['dp_degree']
        for a, b in zip(r['params'], ref):
            np.testing.assert_allclose(a, b, rtol=2e-4, atol=2e-5)


# -- distributed AMP -------------------------------------------------------------------------
def _amp_worker(rank, world):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn.functional as F
    from paddle_ray_amd.distributed.sharding import group_sharded_parallel
    m = _deep_mlp()
    o = paddle.optimizer.SGD(0.1, parameters=m.parameters())
    scaler = paddle.amp.GradScaler(init_loss_scaling=1024.0)
    sm, so, scaler = group_sharded_parallel(m, o, 'os_g', scaler=scaler, segment_size=0)
    xs, ys = _data()
    n = len(xs) // world
    xs, ys = xs[rank * n:(rank + 1) * n], ys[rank * n:(rank + 1) * n]
    before = [p.numpy().copy() for p in m.parameters()]
    found, scales = [], []
    for step in range(3):
        x = xs.copy()
        if step == 1 and rank == 1:
            x[0, 0] = np.inf  # only rank 1 overflows
        loss = F.mse_loss(sm(paddle.to_tensor(x)), paddle.to_tensor(ys))
        scaler.scale(loss).backward()
        snap = [p.numpy().copy() for p in m.parameters()]
        scaler.step(so)
        found.append(scaler._found_inf)
        changed = any(not np.array_equal(a, p.numpy()) for a, p in zip(snap, m.parameters()))
        scaler.update()
        scales.append(scaler.get_loss_scaling())
        so.clear_grad()
        found[-1] = (found[-1], changed)
    return {'found': found, 'scales': scales,
            'moved': any(not np.array_equal(a, p.numpy()) for a, p in zip(before, m.parameters()))}


def test_sharded_grad_scaler_skips_together(tmp_path):
    res = run_ranks(_amp_worker, 2, tmp_path)
    for r in res:
        # step 1: rank 1 saw inf -> BOTH ranks report found_inf and skip the update
        assert [f for f, _ in r['found']] == [False, True, False], r
        assert [c for _, c in r['found']] == [True, False, True], r
        assert r['scales'][1] == r['scales'][0] * 0.5
    assert res[0]['scales'] == res[1]['scales']


def test_amp_custom_lists_cpu():
    import torch
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn.functional as F
    x = paddle.to_tensor(np.random.rand(4, 8).astype('float32'))
    w = paddle.to_tensor(np.random.rand(8, 3).astype('float32'))
    with paddle.amp.auto_cast(custom_white_list={'softmax'}, dtype='bfloat16'):
        assert F.softmax(x).dtype == paddle.bfloat16
    with paddle.amp.auto_cast(custom_black_list={'matmul'}, dtype='bfloat16'):
        assert paddle.matmul(x, w).dtype == paddle.float32
        assert paddle.matmul(x, w)._t.dtype == torch.float32
    with pytest.raises(ValueError):
        with paddle.amp.auto_cast(custom_white_list={'a'}, custom_black_list={'a'}):
            pass


# -- sharding over any inner optimizer (dygraph_sharding_optimizer.py:29-212) -------------------
_GENERIC = {
    'Lamb': lambda paddle, ps: paddle.optimizer.Lamb(0.01, lamb_weight_decay=0.01, parameters=ps,
                                                    grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5)),
    'Adagrad': lambda paddle, ps: paddle.optimizer.Adagrad(0.05, parameters=ps, initial_accumulator_value=0.1),
    'RMSProp': lambda paddle, ps: paddle.optimizer.RMSProp(0.01, momentum=0.5, centered=True, parameters=ps),
    'Adamax': lambda paddle, ps: paddle.optimizer.Adamax(0.01, parameters=ps, weight_decay=0.01),
    'Adadelta': lambda paddle, ps: paddle.optimizer.Adadelta(0.5, parameters=ps),
}


def _generic_single(name, steps=3):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn.functional as F
    m = _deep_mlp()
    o = _GENERIC[name](paddle, m.parameters())
    xs, ys = _data()
    for _ in range(steps):
        loss = F.mse_loss(m(paddle.to_tensor(xs)), paddle.to_tensor(ys))
        loss.backward()
        o.step()
        o.clear_grad()
    return [p.numpy() for p in m.parameters()], _by_index(m, o.state_dict())


def _by_index(m, sd):
    """optimizer state keyed by (parameter position, accumulator) (names differ per process)"""
    names = {p.name: i for i, p in enumerate(m.parameters())}
    out = {}
    for k, v in sd.items():
        if not hasattr(v, 'numpy'):
            continue
        for n, i in names.items():
            if k.startswith(n + '_'):
                out[f'{i}:{k[len(n) + 1:]}'] = v.numpy()
    return out


def _generic_worker(rank, world, name, level, steps=3):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn.functional as F
    from paddle_ray_amd.distributed.sharding import group_sharded_parallel
    m = _deep_mlp()
    o = _GENERIC[name](paddle, m.parameters())
    sm, so, _ = group_sharded_parallel(m, o, level, segment_size=0, bucket_mb=1)
    xs, ys = _data()
    for _ in range(steps):
        # the full batch on every rank: the sharded gradient average equals the single-process one
        loss = F.mse_loss(sm(paddle.to_tensor(xs)), paddle.to_tensor(ys))
        loss.backward()
        so.step()
        so.clear_grad()
    sd = sm.state_dict()
    osd = so.state_dict()
    return {'params': [sd[k].numpy() for k in sd],
            'opt': _by_index(m, osd)}


@pytest.mark.parametrize('name', sorted(_GENERIC))
@pytest.mark.parametrize('level', ['os_g', 'p_g_os'])
def test_sharding_wraps_any_inner_optimizer(tmp_path, name, level):
    ref, ref_opt = _generic_single(name)
    res = run_ranks(_generic_worker, 2, tmp_path, (name, level))
    for r in res:
        for a, b in zip(r['params'], ref):
            np.testing.assert_allclose(a, b, rtol=2e-5, atol=2e-6)
        # the gathered optimizer state uses the plain optimizer's per-parameter keys and values
        assert set(ref_opt) <= set(r['opt']), sorted(set(ref_opt) - set(r['opt']))
        for k, v in ref_opt.items():
            np.testing.assert_allclose(r['opt'][k], v, rtol=2e-5, atol=2e-6)


def _clip_opt(paddle, params, kind):
    clip = paddle.nn.ClipGradByValue(0.05) if kind == 'value' else paddle.nn.ClipGradByNorm(0.1)
    return paddle.optimizer.AdamW(0.01, weight_decay=0.01, parameters=params, grad_clip=clip)


def _clip_single(kind, steps=3):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn.functional as F
    m = _deep_mlp()
    o = _clip_opt(paddle, m.parameters(), kind)
    xs, ys = _data()
    for _ in range(steps):
        F.mse_loss(m(paddle.to_tensor(xs)), paddle.to_tensor(ys)).backward()
        o.step()
        o.clear_grad()
    return [p.numpy() for p in m.parameters()]


def _clip_worker(rank, world, kind, level, steps=3):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn.functional as F
    from paddle_ray_amd.distributed.sharding import group_sharded_parallel
    m = _deep_mlp()
    o = _clip_opt(paddle, m.parameters(), kind)
    sm, so, _ = group_sharded_parallel(m, o, level, segment_size=0, bucket_mb=1)
    xs, ys = _data()
    n = len(xs) // world
    xs, ys = xs[rank * n:(rank + 1) * n], ys[rank * n:(rank + 1) * n]
    for _ in range(steps):
        F.mse_loss(sm(paddle.to_tensor(xs)), paddle.to_tensor(ys)).backward()
        so.step()
        so.clear_grad()
    sd = sm.state_dict()
    return [sd[k].numpy() for k in sd]


@pytest.mark.parametrize('kind', ['value', 'norm'])
@pytest.mark.parametrize('level', ['os', 'os_g', 'p_g_os'])
def test_sharding_clip_by_value_and_norm(tmp_path, kind, level):
    """ClipGradByValue (element-wise on each rank's shard pieces) and ClipGradByNorm (per
    parameter: squared norms of a parameter's pieces summed across ranks) under sharding give
    the single-process result; the 6-layer MLP's parameters straddle the 2 ranks' shards."""
    ref = _clip_single(kind)
    for r in run_ranks(_clip_worker, 2, tmp_path, (kind, level)):
        for a, b in zip(r, ref):
            np.testing.assert_allclose(a, b, rtol=2e-4, atol=2e-5)
