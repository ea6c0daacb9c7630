"""Static-graph forward recomputation (reference: python/paddle/fluid/backward.py:907
`_append_backward_ops_with_checkpoints_`, fluid/optimizer.py:6447 RecomputeOptimizer,
fleet/meta_optimizers/recompute_optimizer.py:97).

A GPT-tiny-shaped stack of pre-LN residual MLP blocks with dropout is built twice from the same
seed: once plain, once with the block outputs as checkpoints. The gradients must be BIT-identical
(the recomputed dropout masks repeat: RNG restore), the op list must carry the re-emitted
segments, and the executor's peak live bytes must drop."""
import numpy as np
import pytest

from dist_utils import run_ranks

B, S, H, L = 4, 16, 32, 4


def _build(checkpointed, opt_kind=None, drop=0.1):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn as nn
    import paddle_ray_amd.nn.functional as F
    from paddle_ray_amd import static
    paddle.seed(7)
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        x = static.data('x', [B, S, H], 'float32')
        h = x
        ckpts, params = [], []
        for _ in range(L):
            ln, l1, l2 = nn.LayerNorm(H), nn.Linear(H, 4 * H), nn.Linear(4 * H, H)
            params += [ln.weight, ln.bias, l1.weight, l1.bias, l2.weight, l2.bias]
            h = h + F.dropout(l2(F.gelu(l1(ln(h)))), p=drop, training=True)
            ckpts.append(h)
        loss = (h * h).mean()
        if opt_kind is None:
            pg = static.append_backward(loss, checkpoints=ckpts[:-1] if checkpointed else None)
            return main, loss, pg
        opt = paddle.optimizer.SGD(0.1, parameters=params)
        if checkpointed:
            opt = static.RecomputeOptimizer(opt)
            opt._set_checkpoints(ckpts[:-1])
        opt.minimize(loss)
    return main, loss, params


def _run_grads(checkpointed):
    import paddle_ray_amd as paddle
    from paddle_ray_amd import static
    paddle.enable_static()
    try:
        main, loss, pg = _build(checkpointed)
        exe = static.Executor()
        exe.enable_memory_trace()
        xv = np.random.RandomState(3).randn(B, S, H).astype('float32')
        paddle.seed(11)
        out = exe.run(main, feed={'x': xv}, fetch_list=[loss] + [g for _, g in pg])
        roles = [op.role for op in main.global_block().ops]
        types = [op.type for op in main.global_block().ops]
        return out, exe.peak_live_bytes, roles, types
    finally:
        paddle.disable_static()


def test_static_recompute_bit_identical_grads_and_less_memory():
    ref, peak_ref, roles_ref, _ = _run_grads(False)
    got, peak_rc, roles, types = _run_grads(True)
    assert 'recompute' not in roles_ref
    # three checkpoints -> the head segment plus the segments between consecutive checkpoints
    assert roles.count('recompute') > 0
    assert types.count('recompute_rng_save') == types.count('recompute_rng_swap') == \
        types.count('recompute_rng_restore') >= 2
    # every re-emitted op comes after the forward (it runs inside the backward)
    first_bwd = roles.index('backward')
    assert all(i > first_bwd for i, r in enumerate(roles) if r == 'recompute')
    assert len(ref) == len(got)
    for a, b in zip(ref, got):
        assert np.array_equal(a, b), "recomputed gradients differ"
    assert peak_rc < peak_ref * 0.85, (peak_rc, peak_ref)


def test_recompute_optimizer_trains_like_plain():
    import paddle_ray_amd as paddle
    from paddle_ray_amd import static
    res = {}
    for ck in (False, True):
        paddle.enable_static()
        try:
            main, loss, params = _build(ck, opt_kind='sgd')
            exe = static.Executor()
            xv = np.random.RandomState(4).randn(B, S, H).astype('float32')
            paddle.seed(1)
            losses = [float(exe.run(main, feed={'x': xv}, fetch_list=[loss])[0]) for _ in range(3)]
            res[ck] = (losses, [p.numpy().copy() for p in params])
        finally:
            paddle.disable_static()
    assert res[False][0] == res[True][0]
    for a, b in zip(res[False][1], res[True][1]):
        assert np.array_equal(a, b)
    assert res[True][0][-1] < res[True][0][0]


def test_recompute_optimizer_rejects_dygraph_and_missing_checkpoints():
    import paddle_ray_amd as paddle
    from paddle_ray_amd import static
    with pytest.raises(Exception):
        static.RecomputeOptimizer(paddle.optimizer.SGD(0.1, parameters=[paddle.create_parameter([2], 'float32')]))
    paddle.enable_static()
    try:
        main, startup = static.Program(), static.Program()
        with static.program_guard(main, startup):
            x = static.data('x', [2, 3], 'float32')
            lin = paddle.nn.Linear(3, 2)
            loss = lin(x).mean()
            opt = static.RecomputeOptimizer(paddle.optimizer.SGD(0.1, parameters=lin.parameters()))
            with pytest.raises(ValueError):
                opt.minimize(loss)
            with pytest.raises(TypeError):
                opt._set_checkpoints(3)
    finally:
        paddle.disable_static()


def test_device_guard_multi_device_minimize_raises():
    import paddle_ray_amd as paddle
    from paddle_ray_amd import static
    paddle.enable_static()
    try:
        main, startup = static.Program(), static.Program()
        with static.program_guard(main, startup):
            x = static.data('x', [2, 3], 'float32')
            with static.device_guard('gpu:0'):
                a = paddle.nn.Linear(3, 3)(x)
            with static.device_guard('gpu:1'):
                loss = paddle.nn.Linear(3, 1)(a).mean()
            assert main.global_block().ops[-1].attrs.get('device') == 'gpu:1'
            with pytest.raises(NotImplementedError):
                paddle.optimizer.SGD(0.1).minimize(loss)
        # one device (or cpu + gpu placement hints) is fine
        main2, startup2 = static.Program(), static.Program()
        with static.program_guard(main2, startup2):
            x = static.data('x', [2, 3], 'float32')
            with static.device_guard('gpu'):
                loss = paddle.nn.Linear(3, 1)(x).mean()
            paddle.optimizer.SGD(0.1).minimize(loss)
    finally:
        paddle.disable_static()


# -- static fleet: strategy.recompute works, strategy.pipeline raises -------------------------------
def _fleet_recompute(rank, world, recompute):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn as nn
    import paddle_ray_amd.nn.functional as F
    from paddle_ray_amd import static
    from paddle_ray_amd.distributed import fleet
    paddle.enable_static()
    paddle.seed(5)
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        x = static.data('x', [4, 8], 'float32')
        l1, l2, l3 = nn.Linear(8, 16), nn.Linear(16, 16), nn.Linear(16, 1)
        h1 = F.gelu(l1(x))
        h1.name = 'ck_h1'
        h2 = F.gelu(l2(h1))
        h2.name = 'ck_h2'
        loss = (l3(h2) ** 2).mean()
        params = [l1.weight, l1.bias, l2.weight, l2.bias, l3.weight, l3.bias]
        st = fleet.DistributedStrategy()
        st.recompute = recompute
        st.recompute_configs = {'checkpoints': ['ck_h1', 'ck_h2']}
        fleet.init(is_collective=True, strategy=st)
        fleet.distributed_optimizer(paddle.optimizer.SGD(0.2, parameters=params), strategy=st).minimize(loss)
    exe = static.Executor()
    rs = np.random.RandomState(2)
    for _ in range(3):
        xv = rs.randn(world, 4, 8).astype('float32')[rank]
        exe.run(main, feed={'x': xv}, fetch_list=[loss])
    roles = [op.role for op in main.global_block().ops]
    out = [p.numpy().copy() for p in params], roles.count('recompute')
    # strategy.pipeline on a program without a device_guard stage split (1 stage, 2 ranks) is
    # rejected, not ignored (the pipeline itself: tests/test_static_pipeline.py)
    main2, startup2 = static.Program(), static.Program()
    with static.program_guard(main2, startup2):
        x = static.data('x', [4, 8], 'float32')
        lin = nn.Linear(8, 1)
        loss2 = lin(x).mean()
        st2 = fleet.DistributedStrategy()
        st2.pipeline = True
        try:
            fleet.distributed_optimizer(paddle.optimizer.SGD(0.1, parameters=lin.parameters()),
                                        strategy=st2).minimize(loss2)
            pipe = 'accepted'
        except ValueError as e:
            pipe = 'raised' if 'stages' in str(e) else str(e)
    paddle.disable_static()
    return out, pipe


def test_static_fleet_recompute_matches_plain_and_pipeline_raises(tmp_path):
    (tmp_path / 'rc').mkdir()
    (tmp_path / 'plain').mkdir()
    res_rc = run_ranks(_fleet_recompute, 2, tmp_path / 'rc', args=(True,))
    res_plain = run_ranks(_fleet_recompute, 2, tmp_path / 'plain', args=(False,))
    (w_rc, n_rc), pipe = res_rc[0]
    (w_pl, n_pl), _ = res_plain[0]
    assert n_rc > 0 and n_pl == 0
    assert pipe == 'raised'
    for a, b in zip(w_rc, res_rc[1][0][0]):
        assert np.array_equal(a, b)
    for a, b in zip(w_rc, w_pl):
        assert np.array_equal(a, b)
