"""Static-graph pipeline parallelism (reference: fluid/optimizer.py PipelineOptimizer, fleet
pipeline_optimizer.py; test/collective/fleet/pipeline_mnist*.py style: a pipelined run must
train like the single-process run of the same program). gloo ranks on CPU."""
import numpy as np
import pytest

from dist_utils import run_ranks

B, H, F_, C = 8, 6, 16, 4


def _program(guard, clip=None, skip=False, three=False):
    """x -> [gpu:0] Linear -> tanh -> [gpu:1] Linear -> gelu (-> [gpu:2] Linear) -> CE loss."""
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn as nn
    import paddle_ray_amd.nn.functional as F
    from paddle_ray_amd import static
    import contextlib
    paddle.seed(11)
    g = static.device_guard if guard else (lambda d: contextlib.nullcontext())
    main = static.Program()
    with static.program_guard(main):
        x = static.data('x', [-1, H], 'float32')
        y = static.data('y', [-1, 1], 'int64')
        with g('gpu:0'):
            l1 = nn.Linear(H, F_)
            h0 = paddle.tanh(l1(x))
        with g('gpu:1'):
            l2 = nn.Linear(F_, F_ if three else C)
            z1 = l2(h0)
            h1 = F.gelu(z1)
            if skip:
                h1 = h1 + h0[:, :h1.shape[1]] * 0.5        # a skip edge 0 -> 1 used twice
        params = [l1.weight, l1.bias, l2.weight, l2.bias]
        if three:
            with g('gpu:2'):
                l3 = nn.Linear(F_, C)
                h1 = l3(h1) + 0.1 * paddle.sum(h0, axis=1, keepdim=True)   # skip edge 0 -> 2
            params += [l3.weight, l3.bias]
        loss = F.cross_entropy(h1, y)            # unguarded: follows its inputs' stage
    main.__dict__['_test_vars'] = {'h0': h0, 'z1': z1}
    return main, loss, params


def _data(steps, bs):
    rs = np.random.RandomState(5)
    return [{'x': rs.randn(bs, H).astype('float32'), 'y': rs.randint(0, C, (bs, 1)).astype('int64')}
            for _ in range(steps)]


def _serial(clip, skip, three, opt_name='momentum'):
    import paddle_ray_amd as paddle
    from paddle_ray_amd import static
    paddle.enable_static()
    main, loss, params = _program(False, clip, skip, three)
    with static.program_guard(main):
        _opt(opt_name, clip).minimize(loss)
    exe = static.Executor()
    losses = [float(exe.run(main, feed=f, fetch_list=[loss])[0]) for f in _data(3, B)]
    out = [p.numpy() for p in params]
    paddle.disable_static()
    return losses, out


def _opt(name, clip):
    import paddle_ray_amd as paddle
    c = paddle.nn.ClipGradByGlobalNorm(clip) if clip else None
    if name == 'adam':
        return paddle.optimizer.AdamW(0.01, grad_clip=c)
    return paddle.optimizer.Momentum(0.3, momentum=0.9, grad_clip=c)


def _pipe(rank, world, n_micro, schedule, clip, skip, three, use_fleet, opt_name, dp=1, recompute=False,
          shard=False):
    import paddle_ray_amd as paddle
    from paddle_ray_amd import static
    paddle.enable_static()
    main, loss, params = _program(True, clip, skip, three)
    with static.program_guard(main):
        if use_fleet:
            from paddle_ray_amd.distributed import fleet
            st = fleet.DistributedStrategy()
            st.pipeline = True
            st.pipeline_configs = {'accumulate_steps': n_micro, 'micro_batch_size': B // n_micro,
                                   'schedule_mode': schedule}
            st.hybrid_configs = {'dp_degree': dp, 'mp_degree': 1, 'pp_degree': world // dp}
            if shard:
                st.sharding = True
                st.sharding_configs = {'stage': 1}
            if recompute:
                st.recompute = True
                st.recompute_configs = {'checkpoints': [v.name for v in main._test_vars.values()]}
            fleet.init(is_collective=True, strategy=st)
            fleet.distributed_optimizer(_opt(opt_name, clip)).minimize(loss)
        else:
            inner = _opt(opt_name, clip)
            if recompute:
                inner = static.RecomputeOptimizer(inner)
                inner._set_checkpoints(list(main._test_vars.values()))
            static.PipelineOptimizer(inner, num_microbatches=n_micro, schedule_mode=schedule).minimize(loss)
    exe = static.Executor()
    losses = [float(exe.run(main, feed=f, fetch_list=[loss])[0]) for f in _data(3, B)]
    pipe = main._pipeline
    mine = {p.name for p in pipe.params}
    out = {i: p.numpy() for i, p in enumerate(params) if p.name in mine}
    n_ops = (len(pipe.fwd_ops), len(pipe.bwd_ops))
    n_rc = sum(op.role == 'recompute' for op in pipe.bwd_ops)
    n_states = len(getattr(pipe.opt, '_accumulators', {}).get('moment1', {}))
    n_params = len(pipe.params)
    paddle.disable_static()
    return {'losses': losses, 'params': out, 'stage': pipe.stage, 'ops': n_ops,
            'sends': len(pipe.fsend) + len(pipe.bsend), 'recompute_ops': n_rc,
            'dropped': len(pipe.drop_after_fwd), 'n_states': n_states, 'n_params': n_params}


@pytest.mark.parametrize('n_micro,schedule,use_fleet', [(1, 'F-then-B', False), (4, 'F-then-B', False),
                                                        (4, '1F1B', True), (2, '1F1B', False)])
def test_static_pipeline_matches_serial_2stages(tmp_path, n_micro, schedule, use_fleet):
    ref_losses, ref = _serial(None, False, False)
    res = run_ranks(_pipe, 2, tmp_path, args=(n_micro, schedule, None, False, False, use_fleet, 'momentum'))
    got = {}
    for o in res:
        np.testing.assert_allclose(o['losses'], ref_losses, rtol=1e-5, atol=1e-6)
        got.update(o['params'])
        assert o['ops'][0] > 0 and o['ops'][1] > 0 and o['sends'] >= 1
    assert sorted(got) == [0, 1, 2, 3]
    for i, p in got.items():
        np.testing.assert_allclose(p, ref[i], rtol=1e-5, atol=1e-6)
    assert ref_losses[-1] < ref_losses[0]


@pytest.mark.parametrize('use_fleet,schedule', [(False, '1F1B'), (True, 'F-then-B')])
def test_static_pipeline_with_recompute(tmp_path, use_fleet, schedule):
    """Pipeline + recompute (RecomputeOptimizer inside PipelineOptimizer, or fleet strategy.pipeline
    + strategy.recompute): each stage re-runs its segment in the backward and matches the serial
    run; the segments' intermediates are dropped per micro-batch."""
    ref_losses, ref = _serial(None, False, False)
    res = run_ranks(_pipe, 2, tmp_path, args=(4, schedule, None, False, False, use_fleet, 'momentum', 1, True))
    got = {}
    for o in res:
        np.testing.assert_allclose(o['losses'], ref_losses, rtol=1e-5, atol=1e-6)
        got.update(o['params'])
        assert o['recompute_ops'] > 0, o
    assert sum(o['dropped'] for o in res) > 0
    for i, p in got.items():
        np.testing.assert_allclose(p, ref[i], rtol=1e-5, atol=1e-6)


def _pipe_gm(rank, world, k):
    import paddle_ray_amd as paddle
    from paddle_ray_amd import static
    from paddle_ray_amd.distributed import fleet
    paddle.enable_static()
    main, loss, params = _program(True)
    with static.program_guard(main):
        st = fleet.DistributedStrategy()
        st.pipeline = True
        st.pipeline_configs = {'accumulate_steps': 2, 'micro_batch_size': B // 2, 'schedule_mode': '1F1B'}
        st.gradient_merge = True
        st.gradient_merge_configs = {'k_steps': k, 'avg': True}
        st.hybrid_configs = {'dp_degree': 1, 'mp_degree': 1, 'pp_degree': world}
        fleet.init(is_collective=True, strategy=st)
        fleet.distributed_optimizer(_opt('momentum', None)).minimize(loss)
    exe = static.Executor()
    losses = [float(exe.run(main, feed=f, fetch_list=[loss])[0]) for f in _data(2 * k, B)]
    mine = {p.name for p in main._pipeline.params}
    out = {i: p.numpy() for i, p in enumerate(params) if p.name in mine}
    paddle.disable_static()
    return {'losses': losses, 'params': out}


def test_static_pipeline_with_gradient_merge(tmp_path):
    """strategy.pipeline + gradient_merge (k = 2, avg): two pipeline runs, one optimizer step --
    the serial program stepping once per concatenated pair of batches."""
    import paddle_ray_amd as paddle
    from paddle_ray_amd import static
    k = 2
    data = _data(2 * k, B)
    paddle.enable_static()
    main, loss, params = _program(False)
    with static.program_guard(main):
        _opt('momentum', None).minimize(loss)
    exe = static.Executor()
    ref_losses = []
    for j in range(2):
        pair = data[j * k:(j + 1) * k]
        feed = {n: np.concatenate([f[n] for f in pair]) for n in ('x', 'y')}
        ref_losses.append(float(exe.run(main, feed=feed, fetch_list=[loss])[0]))
    ref = [p.numpy() for p in params]
    paddle.disable_static()
    res = run_ranks(_pipe_gm, 2, tmp_path, args=(k,))
    got = {}
    for o in res:
        pl = np.asarray(o['losses']).reshape(2, k).mean(1)
        np.testing.assert_allclose(pl, ref_losses, rtol=1e-5, atol=1e-6)
        got.update(o['params'])
    assert sorted(got) == [0, 1, 2, 3]
    for i, p in got.items():
        np.testing.assert_allclose(p, ref[i], rtol=1e-5, atol=1e-6)


def _pipe_lars(rank, world):
    import paddle_ray_amd as paddle
    from paddle_ray_amd import static
    from paddle_ray_amd.distributed import fleet
    paddle.enable_static()
    main, loss, params = _program(True)
    with static.program_guard(main):
        st = fleet.DistributedStrategy()
        st.pipeline = True
        st.pipeline_configs = {'accumulate_steps': 2, 'micro_batch_size': B // 2, 'schedule_mode': '1F1B'}
        st.lars = True
        st.lars_configs = {'lars_coeff': 0.01, 'lars_weight_decay': 0.001}
        st.hybrid_configs = {'dp_degree': 1, 'mp_degree': 1, 'pp_degree': world}
        fleet.init(is_collective=True, strategy=st)
        fleet.distributed_optimizer(_opt('momentum', None)).minimize(loss)
    exe = static.Executor()
    losses = [float(exe.run(main, feed=f, fetch_list=[loss])[0]) for f in _data(3, B)]
    pipe = main._pipeline
    mine = {p.name for p in pipe.params}
    out = {i: p.numpy() for i, p in enumerate(params) if p.name in mine}
    kind = type(pipe.opt).__name__
    paddle.disable_static()
    return {'losses': losses, 'params': out, 'opt': kind}


def test_static_pipeline_with_lars_swap(tmp_path):
    """strategy.lars under the pipeline: every stage steps LarsMomentum (per-parameter trust
    ratios on its own parameters), as the serial program minimized with LarsMomentum."""
    import paddle_ray_amd as paddle
    from paddle_ray_amd import static
    paddle.enable_static()
    main, loss, params = _program(False)
    with static.program_guard(main):
        paddle.optimizer.LarsMomentum(0.3, momentum=0.9, lars_coeff=0.01, lars_weight_decay=0.001).minimize(loss)
    exe = static.Executor()
    ref_losses = [float(exe.run(main, feed=f, fetch_list=[loss])[0]) for f in _data(3, B)]
    ref = [p.numpy() for p in params]
    paddle.disable_static()
    res = run_ranks(_pipe_lars, 2, tmp_path)
    got = {}
    for o in res:
        assert o['opt'] == 'LarsMomentum'
        np.testing.assert_allclose(o['losses'], ref_losses, rtol=1e-5, atol=1e-6)
        got.update(o['params'])
    for i, p in got.items():
        np.testing.assert_allclose(p, ref[i], rtol=1e-5, atol=1e-6)


def test_static_pipeline_with_data_parallel_2x2(tmp_path):
    """fleet hybrid dp 2 x pp 2: each stage's gradients are averaged over its data-parallel
    replica (same batch on both replicas here: the serial run is the reference)."""
    ref_losses, ref = _serial(0.05, False, False)
    res = run_ranks(_pipe, 4, tmp_path, args=(2, '1F1B', 0.05, False, False, True, 'momentum', 2))
    for o in res:
        np.testing.assert_allclose(o['losses'], ref_losses, rtol=1e-5, atol=1e-6)
        for i, p in o['params'].items():
            np.testing.assert_allclose(p, ref[i], rtol=1e-5, atol=1e-6)
    assert sorted({o['stage'] for o in res}) == [0, 1]


def test_static_pipeline_with_sharding_2x2(tmp_path):
    """pp 2 x dp 2 with sharding stage 1 inside each stage: a replica steps only the parameters it
    owns (AdamW states 1/2 per replica), the global-norm clip still sees every gradient, the owners
    broadcast the updates."""
    ref_losses, ref = _serial(0.05, False, False, 'adam')
    res = run_ranks(_pipe, 4, tmp_path, args=(2, '1F1B', 0.05, False, False, True, 'adam', 2, False, True))
    for o in res:
        np.testing.assert_allclose(o['losses'], ref_losses, rtol=1e-5, atol=1e-6)
        for i, p in o['params'].items():
            np.testing.assert_allclose(p, ref[i], rtol=1e-4, atol=1e-6)
    assert sorted({o['stage'] for o in res}) == [0, 1]
    for stage in (0, 1):
        reps = [o for o in res if o['stage'] == stage]
        assert sum(o['n_states'] for o in reps) == reps[0]['n_params']
        assert all(0 < o['n_states'] < o['n_params'] for o in reps)


def _pipe_local(rank, world, localsgd):
    import paddle_ray_amd as paddle
    from paddle_ray_amd import static
    from paddle_ray_amd.distributed import fleet
    paddle.enable_static()
    main, loss, params = _program(True)
    with static.program_guard(main):
        st = fleet.DistributedStrategy()
        st.pipeline = True
        st.pipeline_configs = {'accumulate_steps': 2, 'micro_batch_size': B // 2, 'schedule_mode': '1F1B'}
        st.hybrid_configs = {'dp_degree': 2, 'mp_degree': 1, 'pp_degree': 2}
        if localsgd:
            st.localsgd = True
            st.localsgd_configs = {'k_steps': 1, 'begin_step': 1}
        fleet.init(is_collective=True, strategy=st)
        fleet.distributed_optimizer(paddle.optimizer.SGD(0.3)).minimize(loss)
    dp_rank = fleet.get_hybrid_communicate_group().get_data_parallel_rank()
    exe = static.Executor()
    data = _data(6, B)[dp_rank::2]          # a different batch on each data-parallel replica
    for f in data:
        exe.run(main, feed=f, fetch_list=[loss])
    pipe = main._pipeline
    mine = {p.name for p in pipe.params}
    out = {i: p.numpy() for i, p in enumerate(params) if p.name in mine}
    paddle.disable_static()
    return {'params': out, 'stage': pipe.stage}


def test_static_pipeline_with_localsgd_2x2(tmp_path):
    """pp 2 x dp 2 with localsgd (k_steps 1): replicas step on their own batches and average the
    parameters, which for SGD equals the data-parallel gradient all-reduce."""
    (tmp_path / 'a').mkdir()
    (tmp_path / 'b').mkdir()
    loc = run_ranks(_pipe_local, 4, tmp_path / 'a', args=(True,))
    ref = run_ranks(_pipe_local, 4, tmp_path / 'b', args=(False,))
    for o, r in zip(loc, ref):
        assert o['stage'] == r['stage']
        for i, p in o['params'].items():
            np.testing.assert_allclose(p, r['params'][i], rtol=1e-5, atol=1e-6)


def test_static_pipeline_skip_edges_clip_adam_3stages(tmp_path):
    """Three stages with activations used on two later stages (skip edges) and gradients summed
    across stages, AdamW, a global-norm clip over all stages."""
    ref_losses, ref = _serial(0.05, True, True, 'adam')
    res = run_ranks(_pipe, 3, tmp_path, args=(4, '1F1B', 0.05, True, True, False, 'adam'))
    got = {}
    for o in res:
        np.testing.assert_allclose(o['losses'], ref_losses, rtol=1e-5, atol=1e-6)
        got.update(o['params'])
    assert sorted(got) == list(range(6))
    for i, p in got.items():
        np.testing.assert_allclose(p, ref[i], rtol=1e-4, atol=1e-6)


def _bad(rank, world, what):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn as nn
    from paddle_ray_amd import static
    paddle.enable_static()
    main = static.Program()
    err = None
    with static.program_guard(main):
        x = static.data('x', [-1, H], 'float32')
        lin = nn.Linear(H, H)
        with static.device_guard('gpu:0'):
            h = lin(x)
        with static.device_guard('gpu:1'):
            out = lin(h) if what == 'shared' else h * 2.0
        loss = paddle.mean(out)
        try:
            static.PipelineOptimizer(paddle.optimizer.SGD(0.1), 2).minimize(loss)
        except (NotImplementedError, ValueError) as e:
            err = type(e).__name__
    paddle.disable_static()
    return err


def test_static_pipeline_rejects_shared_params(tmp_path):
    res = run_ranks(_bad, 2, tmp_path, args=('shared',))
    assert res == ['NotImplementedError', 'NotImplementedError']


def test_plain_minimize_still_raises_for_multi_device():
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn as nn
    from paddle_ray_amd import static
    paddle.enable_static()
    try:
        main = static.Program()
        with static.program_guard(main):
            x = static.data('x', [-1, H], 'float32')
            with static.device_guard('gpu:0'):
                h = nn.Linear(H, H)(x)
            with static.device_guard('gpu:1'):
                loss = paddle.mean(nn.Linear(H, H)(h))
            with pytest.raises(NotImplementedError):
                paddle.optimizer.SGD(0.1).minimize(loss)
    finally:
        paddle.disable_static()
