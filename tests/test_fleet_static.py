"""Static-graph Fleet collective training (reference: fleet.py:1216 `minimize` -> meta-optimizer
chain; meta_optimizers/raw_program_optimizer.py, gradient_merge_optimizer.py,
sharding_optimizer.py (stage 1), lamb_optimizer.py, lars_optimizer.py, localsgd_optimizer.py).

Each rank feeds DIFFERENT data; after training, the parameters must be bit-equal across ranks
and match the serial program trained on the concatenated batch."""
import numpy as np
import pytest

from dist_utils import run_ranks

pytestmark = pytest.mark.timeout(300) if hasattr(pytest.mark, 'timeout') else []

B, H, F_, C = 4, 6, 8, 3


def _data(world, steps, micro=1):
    rs = np.random.RandomState(11)
    xs = rs.randn(steps, micro, world, B, H).astype('float32')
    ys = rs.randint(0, C, (steps, micro, world, B, 1)).astype('int64')
    return xs, ys


def _program(opt_name):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn as nn
    import paddle_ray_amd.nn.functional as F
    from paddle_ray_amd import static
    paddle.seed(5)
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        x = static.data('x', [B, H], 'float32')
        y = static.data('y', [B, 1], 'int64')
        l1, l2 = nn.Linear(H, F_), nn.Linear(F_, C)
        loss = F.cross_entropy(l2(F.gelu(l1(x))), y)
    params = [l1.weight, l1.bias, l2.weight, l2.bias]
    if opt_name == 'sgd':
        opt = paddle.optimizer.SGD(0.3, parameters=params)
    elif opt_name == 'momentum':
        opt = paddle.optimizer.Momentum(0.1, momentum=0.9, parameters=params)
    else:
        opt = paddle.optimizer.Adam(0.05, parameters=params)
    return main, startup, loss, params, opt


def _train_fleet(rank, world, opt_name, strategy_kw, steps, micro):
    import paddle_ray_amd as paddle
    from paddle_ray_amd import static
    from paddle_ray_amd.distributed import fleet
    paddle.enable_static()
    main, startup, loss, params, opt = _program(opt_name)
    st = fleet.DistributedStrategy()
    for k, v in strategy_kw.items():
        setattr(st, k, v)
    fleet.init(is_collective=True, strategy=st)
    with static.program_guard(main, startup):
        dopt = fleet.distributed_optimizer(opt, strategy=st)
        dopt.minimize(loss)
    exe = static.Executor()
    exe.run(startup)
    xs, ys = _data(world, steps, micro)
    losses = []
    for s in range(steps):
        for m in range(micro):
            out = exe.run(main, feed={'x': xs[s, m, rank], 'y': ys[s, m, rank]}, fetch_list=[loss])
            losses.append(float(out[0]))
    state = main.__dict__.get('_fleet_state')
    info = {'buckets': [len(b) for b in state.buckets] if state is not None else None,
            'ops': [op.type for op in main.global_block().ops]}
    res = [p.numpy().copy() for p in params], losses, info, type(dopt._inner_opt).__name__
    paddle.disable_static()
    return res


def _train_serial(opt_name, world, steps, micro, lamb=False):
    """The reference result: one process, the concatenation of every rank's micro-batches."""
    import paddle_ray_amd as paddle
    from paddle_ray_amd import static
    paddle.enable_static()
    paddle.seed(5)
    import paddle_ray_amd.nn as nn
    import paddle_ray_amd.nn.functional as F
    main, startup = static.Program(), static.Program()
    n = world * micro
    with static.program_guard(main, startup):
        x = static.data('x', [n * B, H], 'float32')
        y = static.data('y', [n * B, 1], 'int64')
        l1, l2 = nn.Linear(H, F_), nn.Linear(F_, C)
        loss = F.cross_entropy(l2(F.gelu(l1(x))), y)
        params = [l1.weight, l1.bias, l2.weight, l2.bias]
        if lamb:
            opt = paddle.optimizer.Lamb(0.05, lamb_weight_decay=0.01, parameters=params)
        elif opt_name == 'sgd':
            opt = paddle.optimizer.SGD(0.3, parameters=params)
        elif opt_name == 'momentum':
            opt = paddle.optimizer.Momentum(0.1, momentum=0.9, parameters=params)
        else:
            opt = paddle.optimizer.Adam(0.05, parameters=params)
        opt.minimize(loss)
    exe = static.Executor()
    exe.run(startup)
    xs, ys = _data(world, steps, micro)
    for s in range(steps):
        exe.run(main, feed={'x': xs[s].reshape(n * B, H), 'y': ys[s].reshape(n * B, 1)},
                fetch_list=[loss])
    res = [p.numpy().copy() for p in params]
    paddle.disable_static()
    return res


def _check(results, ref, tol=2e-5):
    w0 = results[0][0]
    for r in results[1:]:
        for a, b in zip(w0, r[0]):
            assert np.array_equal(a, b), "ranks diverged"
    for a, b in zip(w0, ref):
        np.testing.assert_allclose(a, b, rtol=tol, atol=tol)


@pytest.mark.parametrize('world', [2, 4])
def test_static_fleet_dp_matches_serial(tmp_path, world):
    res = run_ranks(_train_fleet, world, tmp_path, args=('sgd', {}, 3, 1))
    _check(res, _train_serial('sgd', world, 3, 1))
    info = res[0][2]
    assert 'c_allreduce_coalesced' in info['ops'] and 'c_sync_comm_stream' in info['ops']
    # the bucket op sits inside the backward (before the last grad op), not after it
    ops = info['ops']
    first_ar = ops.index('c_allreduce_coalesced')
    last_grad = max(i for i, t in enumerate(ops) if t.endswith('_grad') or t == 'grad')
    # one bucket holds all four gradients: its all-reduce is issued right behind the grad op
    # that produces the bucket's last gradient, ahead of the join and the optimizer
    assert first_ar == last_grad + 1, ops
    assert first_ar < ops.index('c_sync_comm_stream') < ops.index('fleet_optimize')
    assert sum(info['buckets']) == 4


def test_static_fleet_dp_small_buckets_overlap(tmp_path):
    """fuse_grad_size_in_MB tiny: one bucket per gradient, issued in gradient-production order,
    each right after its producer (inside the backward)."""
    res = run_ranks(_train_fleet, 2, tmp_path, args=('adam', {'fuse_grad_size_in_MB': 1e-6}, 2, 1))
    _check(res, _train_serial('adam', 2, 2, 1))
    info = res[0][2]
    ops = info['ops']
    assert info['buckets'] == [1, 1, 1, 1]
    ar = [i for i, t in enumerate(ops) if t == 'c_allreduce_coalesced']
    grads = [i for i, t in enumerate(ops) if t.endswith('_grad') or t == 'grad']
    assert ar[0] < grads[-1], (ops,)   # communication starts before the backward ends


def test_static_fleet_gradient_merge(tmp_path):
    kw = {'gradient_merge': True, 'gradient_merge_configs': {'k_steps': 2, 'avg': True}}
    res = run_ranks(_train_fleet, 2, tmp_path, args=('sgd', kw, 2, 2))
    _check(res, _train_serial('sgd', 2, 2, 2))


def test_static_fleet_sharding_stage1(tmp_path):
    kw = {'sharding': True, 'sharding_configs': {'stage': 1},
          'hybrid_configs': {'sharding_degree': 2, 'dp_degree': 1}}
    res = run_ranks(_train_fleet, 2, tmp_path, args=('adam', kw, 3, 1))
    _check(res, _train_serial('adam', 2, 3, 1), tol=5e-5)


def test_static_fleet_lamb_swap(tmp_path):
    res = run_ranks(_train_fleet, 2, tmp_path, args=('adam', {'lamb': True}, 2, 1))
    assert res[0][3] == 'Lamb'
    _check(res, _train_serial('adam', 2, 2, 1, lamb=True), tol=5e-5)


def test_static_fleet_localsgd(tmp_path):
    # k_steps = 1 with SGD: averaging the parameters after every local step equals averaging
    # the gradients
    kw = {'localsgd': True, 'localsgd_configs': {'k_steps': 1, 'begin_step': 1}}
    res = run_ranks(_train_fleet, 2, tmp_path, args=('sgd', kw, 3, 1))
    _check(res, _train_serial('sgd', 2, 3, 1))
    assert 'c_allreduce_coalesced' not in res[0][2]['ops']


def _localsgd_steps(rank, world, begin, k, steps):
    import paddle_ray_amd as paddle
    from paddle_ray_amd import static
    from paddle_ray_amd.distributed import fleet
    paddle.enable_static()
    main, startup, loss, params, opt = _program('sgd')
    st = fleet.DistributedStrategy()
    st.localsgd = True
    st.localsgd_configs = {'k_steps': k, 'begin_step': begin}
    fleet.init(is_collective=True, strategy=st)
    with static.program_guard(main, startup):
        fleet.distributed_optimizer(opt, strategy=st).minimize(loss)
    exe = static.Executor()
    xs, ys = _data(world, steps)
    snaps = []
    for s in range(steps):
        exe.run(main, feed={'x': xs[s, 0, rank], 'y': ys[s, 0, rank]}, fetch_list=[loss])
        snaps.append([p.numpy().copy() for p in params])
    paddle.disable_static()
    return snaps


def test_static_fleet_localsgd_begin_step(tmp_path):
    """Before begin_step every step averages (the ranks never drift during warm-up); after it,
    averaging happens k_steps after the previous one (steps 1..3, then 5)."""
    res = run_ranks(_localsgd_steps, 2, tmp_path, args=(3, 2, 5))
    same = [all(np.array_equal(a, b) for a, b in zip(res[0][s], res[1][s])) for s in range(5)]
    assert same == [True, True, True, False, True], same


def _sharding_amp_clip(rank, world, sharding):
    import paddle_ray_amd as paddle
    from paddle_ray_amd import static
    from paddle_ray_amd.distributed import fleet
    paddle.enable_static()
    main, startup, loss, params, _ = _program('adam')
    opt = paddle.optimizer.Adam(0.05, parameters=params,
                                grad_clip=paddle.nn.ClipGradByGlobalNorm(0.05))
    st = fleet.DistributedStrategy()
    st.amp = True
    st.amp_configs = {'init_loss_scaling': 1024.0, 'use_dynamic_loss_scaling': True}
    if sharding:
        st.sharding = True
        st.sharding_configs = {'stage': 1}
        st.hybrid_configs = {'sharding_degree': 2, 'dp_degree': 1}
    fleet.init(is_collective=True, strategy=st)
    with static.program_guard(main, startup):
        fleet.distributed_optimizer(opt, strategy=st).minimize(loss)
    exe = static.Executor()
    xs, ys = _data(world, 3)
    for s in range(3):
        exe.run(main, feed={'x': xs[s, 0, rank], 'y': ys[s, 0, rank]}, fetch_list=[loss])
    out = [p.numpy().copy() for p in params]
    paddle.disable_static()
    return out


def test_static_fleet_sharding_amp_clip_matches_dp(tmp_path):
    """Sharding stage 1 + AMP loss scaling + global-norm clip: the owner-only update must see
    the same unscaled gradients, clip coefficient and found_inf as plain data parallel."""
    (tmp_path / 'sh').mkdir()
    (tmp_path / 'dp').mkdir()
    sh = run_ranks(_sharding_amp_clip, 2, tmp_path / 'sh', args=(True,))
    dp = run_ranks(_sharding_amp_clip, 2, tmp_path / 'dp', args=(False,))
    for a, b in zip(sh[0], sh[1]):
        assert np.array_equal(a, b)
    for a, b in zip(sh[0], dp[0]):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)


def _lars_momentum(rank, world):
    import paddle_ray_amd as paddle
    from paddle_ray_amd.distributed import fleet
    st = fleet.DistributedStrategy()
    st.lars = True
    st.lars_configs = {'lars_coeff': 0.01, 'lars_weight_decay': 0.0}
    fleet.init(is_collective=True, strategy=st)
    lin = paddle.nn.Linear(4, 3)
    opt = fleet.distributed_optimizer(paddle.optimizer.Momentum(0.1, parameters=lin.parameters()))
    name = type(opt._inner_opt).__name__
    st2 = fleet.DistributedStrategy()
    st2.dgc = True
    try:
        fleet.distributed_optimizer(paddle.optimizer.Momentum(0.1, parameters=lin.parameters()), strategy=st2)
        dgc = 'accepted'
    except NotImplementedError:
        dgc = 'raised'
    return name, dgc


def test_fleet_lars_swap_and_dgc_rejected(tmp_path):
    res = run_ranks(_lars_momentum, 2, tmp_path)
    assert res[0] == ('LarsMomentum', 'raised')


def test_lars_momentum_update_rule():
    """LarsMomentum against the reference equations (fluid/optimizer.py LarsMomentumOptimizer)."""
    import paddle_ray_amd as paddle
    import torch
    paddle.seed(0)
    p = paddle.create_parameter([5, 3], 'float32')
    w0 = p.numpy().copy()
    g = np.random.RandomState(0).randn(5, 3).astype('float32')
    opt = paddle.optimizer.LarsMomentum(0.1, momentum=0.9, lars_coeff=0.01, lars_weight_decay=0.001,
                                        parameters=[p])
    v = np.zeros_like(w0)
    w = w0.copy()
    for _ in range(2):
        p._t.grad = torch.from_numpy(g.copy())
        opt.step()
        pn, gn = np.linalg.norm(w), np.linalg.norm(g)
        llr = 0.1 * 0.01 * pn / (gn + 0.001 * pn)
        v = 0.9 * v + llr * (g + 0.001 * w)
        w = w - v
    np.testing.assert_allclose(p.numpy(), w, rtol=1e-5, atol=1e-6)
