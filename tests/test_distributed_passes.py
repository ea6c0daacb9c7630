"""paddle.distributed.passes (reference tests: test/distributed_passes/test_white_lists.py,
check_pass_conflict_example.py, test_auto_parallel_{amp,fp16,recompute,gradient_merge,sharding}
_pass.py, test_dist_fuse_gemm_epilogue_pass.py, test_dist_fuse_*: a program trained with the
pass must train like the one without it). CPU; the partitioned cases run on gloo ranks."""
import numpy as np
import pytest

from dist_utils import run_ranks

B, H, F_, C = 8, 6, 8, 4


@pytest.fixture
def static_mode():
    import paddle_ray_amd as paddle
    paddle.enable_static()
    yield
    paddle.disable_static()


def _ffn_program(passes=(), after=False, p=0.0, opt_fn=None, seed=0, recompute_ck=False):
    """x -> Linear -> gelu -> Linear -> dropout -> +x -> LayerNorm -> mse."""
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn as nn
    import paddle_ray_amd.nn.functional as F
    from paddle_ray_amd import static
    paddle.seed(seed)
    main = static.Program()
    with static.program_guard(main):
        x = static.data('x', [4, 8], 'float32')
        y = static.data('y', [4, 8], 'float32')
        l1, l2, ln = nn.Linear(8, 16), nn.Linear(16, 8), nn.LayerNorm(8)
        h = F.gelu(l1(x))
        z = ln(x + F.dropout(l2(h), p))
        loss = paddle.mean((z - y) ** 2)
        opt = opt_fn() if opt_fn else paddle.optimizer.SGD(0.1)
        ps = [pp(h) if callable(pp) else pp for pp in passes]
        if not after:
            for pp in ps:
                pp.apply([main], [None])
        opt.minimize(loss)
        if after:
            for pp in ps:
                pp.apply([main], [None])
    return main, loss, [l1.weight, l1.bias, l2.weight, l2.bias, ln.weight, ln.bias]


def _feeds(n=3, rows=4):
    rs = np.random.RandomState(0)
    return [{'x': rs.randn(rows, 8).astype('float32'), 'y': rs.randn(rows, 8).astype('float32')}
            for _ in range(n)]


def _train(main, loss, feeds):
    from paddle_ray_amd import static
    exe = static.Executor()
    return [float(exe.run(main, feed=f, fetch_list=[loss])[0]) for f in feeds]


def _fwd_types(main):
    return [op.type.rsplit(':', 1)[-1] for op in main.global_block().ops if op.role == 'forward']


# -- registry / manager ---------------------------------------------------------------------------
def test_registry_and_conflict_resolution():
    from paddle_ray_amd.distributed.passes import new_pass, PassManager, PassContext
    from paddle_ray_amd.distributed.passes.pass_base import registered_passes
    for n in ('auto_parallel_amp', 'auto_parallel_fp16', 'auto_parallel_recompute',
              'auto_parallel_gradient_merge_pass', 'auto_parallel_sharding', 'auto_parallel_grad_clip',
              'auto_parallel_data_parallel_optimization', 'fuse_all_reduce', 'fuse_gemm_epilogue',
              'fused_feedforward', 'fuse_elewise_add_act', 'fuse_optimizer'):
        assert n in registered_passes()
    with pytest.raises(AssertionError):
        new_pass('no_such_pass')
    p = new_pass('fuse_all_reduce', {'max_memory_size': 1 << 20})
    assert p.get_attr('max_memory_size') == 1 << 20 and p.name == 'fuse_all_reduce'
    # a fusion pass given first is moved behind the communication pass (check_pass_conflict_example)
    pm = PassManager([new_pass('fuse_elewise_add_act'), new_pass('fuse_all_reduce', {'max_memory_size': 1})])
    assert pm.names == ['fuse_all_reduce', 'fuse_elewise_add_act']
    # fusion passes in canonical order, a second pass of one type dropped
    pm = PassManager([new_pass('fuse_optimizer'), new_pass('fuse_gemm_epilogue'),
                      new_pass('fused_feedforward'), new_pass('fuse_gemm_epilogue')])
    assert pm.names == ['fused_feedforward', 'fuse_gemm_epilogue', 'fuse_optimizer']
    # a pass whose attributes are invalid is dropped (_check_self)
    pm = PassManager([new_pass('auto_parallel_amp', {'dtype': 'int8'}), new_pass('fuse_all_reduce')])
    assert pm.names == []       # fuse_all_reduce without max_memory_size fails _check_self too
    # without auto_solve_conflict the list stays as given
    pm = PassManager([new_pass('fuse_elewise_add_act'), new_pass('fuse_all_reduce')], auto_solve_conflict=False)
    assert pm.names == ['fuse_elewise_add_act', 'fuse_all_reduce']
    # passes already applied in the context constrain the next manager
    ctx = PassContext()
    ctx._add_pass(new_pass('fuse_gemm_epilogue'))
    pm = PassManager([new_pass('fuse_all_reduce', {'max_memory_size': 1}), new_pass('fuse_optimizer')], ctx)
    assert pm.names == ['fuse_optimizer']
    ctx.set_attr('k', 1)
    assert ctx.get_attr('k') == 1 and ctx.get_attr('missing', 5) == 5


# -- fusion ----------------------------------------------------------------------------------------
@pytest.mark.parametrize('after', [False, True])
@pytest.mark.parametrize('name,want', [
    ('fused_feedforward', ['fused_mlp_gelu', 'fused_add_dropout_ln']),
    ('fuse_gemm_epilogue', ['fused_mlp_gelu', 'add', 'dropout', 'add', 'layer_norm']),
])
def test_fusion_pass_trains_like_unfused(static_mode, name, want, after):
    from paddle_ray_amd.distributed.passes import new_pass
    feeds = _feeds(1) * 3
    m0, l0, _ = _ffn_program()
    ref = _train(m0, l0, feeds)
    m1, l1, _ = _ffn_program([new_pass(name)], after=after)
    assert _fwd_types(m1)[:len(want)] == want, _fwd_types(m1)
    np.testing.assert_allclose(_train(m1, l1, feeds), ref, rtol=1e-5, atol=1e-6)
    assert ref[-1] < ref[0]


def test_fuse_gemm_epilogue_linear_gelu_and_plain(static_mode):
    """linear -> gelu (no second linear) and a lone linear: fused_linear + fused_bias_gelu."""
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn as nn
    import paddle_ray_amd.nn.functional as F
    from paddle_ray_amd import static
    from paddle_ray_amd.distributed.passes import new_pass

    def build(fuse):
        paddle.seed(1)
        main = static.Program()
        with static.program_guard(main):
            x = static.data('x', [4, 8], 'float32')
            y = static.data('y', [4, 8], 'float32')
            la, lb = nn.Linear(8, 8), nn.Linear(8, 8)
            loss = paddle.mean((F.gelu(la(x), approximate=True) + lb(x) - y) ** 2)
            if fuse:
                new_pass('fuse_gemm_epilogue').apply([main], [None])
            paddle.optimizer.SGD(0.1).minimize(loss)
        return main, loss
    feeds = _feeds()
    m0, l0 = build(False)
    m1, l1 = build(True)
    assert _fwd_types(m1)[:3] == ['fused_linear', 'fused_bias_gelu', 'fused_linear'], _fwd_types(m1)
    np.testing.assert_allclose(_train(m1, l1, feeds), _train(m0, l0, feeds), rtol=1e-5, atol=1e-6)


def test_fuse_elewise_add_act(static_mode):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn.functional as F
    from paddle_ray_amd import static
    from paddle_ray_amd.distributed.passes import new_pass

    def build(fuse):
        paddle.seed(2)
        main = static.Program()
        with static.program_guard(main):
            x = static.data('x', [4, 8], 'float32')
            y = static.data('y', [4, 8], 'float32')
            b = static.create_parameter([8], 'float32')
            w = static.create_parameter([8, 8], 'float32')
            loss = paddle.mean((F.gelu(paddle.matmul(x, w) + b) - y) ** 2)
            ctx = new_pass('fuse_elewise_add_act').apply([main], [None]) if fuse else None
            paddle.optimizer.SGD(0.1).minimize(loss)
        return main, loss, ctx
    feeds = _feeds()
    m0, l0, _ = build(False)
    m1, l1, ctx = build(True)
    assert 'fused_bias_gelu' in _fwd_types(m1) and 'gelu' not in _fwd_types(m1)
    assert ctx.get_attr('fuse_elewise_add_act_count') == 1
    np.testing.assert_allclose(_train(m1, l1, feeds), _train(m0, l0, feeds), rtol=1e-5, atol=1e-6)


def test_fuse_optimizer_marks_multi_tensor_optimizers(static_mode):
    import paddle_ray_amd as paddle
    from paddle_ray_amd.distributed.passes import new_pass
    m, _, _ = _ffn_program(opt_fn=lambda: paddle.optimizer.Momentum(0.1, momentum=0.9))
    ctx = new_pass('fuse_optimizer').apply([m], [None])
    assert ctx.get_attr('fuse_optimizer_count') == 1
    assert next(op for op in m.global_block().ops if op.role == 'optimize').attrs['fused_optimizer']
    m, _, _ = _ffn_program()
    ctx = new_pass('fuse_optimizer').apply([m], [None])
    assert ctx.get_attr('fuse_optimizer_count') == 0 and ctx.get_attr('fuse_optimizer_unfused') == ['SGD']


# -- amp -------------------------------------------------------------------------------------------
def test_amp_pass_bf16_matches_static_decorate(static_mode):
    import paddle_ray_amd as paddle
    from paddle_ray_amd.distributed.passes import new_pass
    from paddle_ray_amd.static import amp as samp
    feeds = _feeds()
    m0, l0, _ = _ffn_program(opt_fn=lambda: samp.decorate(paddle.optimizer.SGD(0.1), use_bf16=True))
    ref = _train(m0, l0, feeds)
    for after in (False, True):
        m1, l1, _ = _ffn_program([new_pass('auto_parallel_amp', {'dtype': 'bfloat16'})], after=after)
        fw = [op for op in m1.global_block().ops if op.role == 'forward']
        assert all(str(op.attrs['amp']['dtype']) == 'torch.bfloat16' for op in fw)
        grads = [op for op in m1.global_block().ops if op.role == 'backward' and 'fwd' in op.attrs]
        assert grads and all('amp' in op.attrs for op in grads)
        np.testing.assert_allclose(_train(m1, l1, feeds), ref, rtol=0, atol=0)


def test_amp_pass_fp16_installs_loss_scaling(static_mode):
    from paddle_ray_amd.distributed.passes import new_pass
    from paddle_ray_amd.static.amp import _ScaleRef
    for after in (False, True):
        m, _, _ = _ffn_program([new_pass('auto_parallel_fp16', {
            'dtype': 'float16', 'init_loss_scaling': 1024.0, 'use_dynamic_loss_scaling': True})], after=after)
        ops = m.global_block().ops
        seed = next(op for op in ops if op.type == 'fill_grad_seed')
        assert isinstance(seed.args[1], _ScaleRef) and float(seed.args[1]) == 1024.0
        opt_op = next(op for op in ops if op.role == 'optimize')
        assert opt_op.kwargs['scaler'] is not None
        assert all(op.attrs['amp']['level'] == 'O2' for op in ops if op.role == 'forward')
    with pytest.raises(NotImplementedError):
        _ffn_program([new_pass('auto_parallel_fp16', {'dtype': 'float16', 'use_optimizer_fp16': True})])


# -- recompute -------------------------------------------------------------------------------------
@pytest.mark.parametrize('after', [False, True])
def test_recompute_pass_checkpoints_bit_identical(static_mode, after):
    from paddle_ray_amd.distributed.passes import new_pass
    feeds = _feeds(4)
    m0, l0, p0 = _ffn_program(p=0.3)
    ref = _train(m0, l0, feeds)
    m1, l1, p1 = _ffn_program([lambda h: new_pass('auto_parallel_recompute', {'checkpoints': [h]})],
                              after=after, p=0.3)
    assert any(op.role == 'recompute' for op in m1.global_block().ops)
    assert _train(m1, l1, feeds) == ref              # dropout masks replayed bit for bit
    for a, b in zip(p0, p1):
        np.testing.assert_array_equal(a.numpy(), b.numpy())


def test_recompute_pass_annotated_regions(static_mode):
    """auto_parallel.recompute(...) regions recorded in a static program become the segments;
    no_recompute_segments keeps the chosen ones."""
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn as nn
    import paddle_ray_amd.nn.functional as F
    from paddle_ray_amd import static
    from paddle_ray_amd.distributed import auto_parallel as ap
    from paddle_ray_amd.distributed.passes import new_pass

    def build(mode):
        paddle.seed(3)
        main = static.Program()
        with static.program_guard(main):
            x = static.data('x', [4, 8], 'float32')
            y = static.data('y', [4, 8], 'float32')
            blocks = [nn.Sequential(nn.Linear(8, 8), nn.GELU(), nn.Linear(8, 8)) for _ in range(2)]
            h = x
            for blk in blocks:
                h = F.dropout((ap.recompute(blk) if mode else blk)(h), 0.2) + h
            loss = paddle.mean((h - y) ** 2)
            if mode == 'all':
                new_pass('auto_parallel_recompute').apply([main], [None])
            elif mode == 'skip0':
                new_pass('auto_parallel_recompute', {'no_recompute_segments': [0]}).apply([main], [None])
            paddle.optimizer.SGD(0.1).minimize(loss)
        return main, loss
    feeds = _feeds(3)
    m0, l0 = build(None)
    ref = _train(m0, l0, feeds)
    for mode, nseg in (('all', 2), ('skip0', 1)):
        m, l = build(mode)
        swaps = [op for op in m.global_block().ops if op.type == 'recompute_rng_swap']
        assert len(swaps) == nseg, mode
        assert _train(m, l, feeds) == ref
    with pytest.raises(ValueError):
        _ffn_program([new_pass('auto_parallel_recompute')])      # nothing to recompute


# -- gradient merge ----------------------------------------------------------------------------------
@pytest.mark.parametrize('after', [False, True])
def test_gradient_merge_pass_equals_big_batch(static_mode, after):
    """k_steps=2, avg: 4 runs on half batches == 2 runs on the concatenated batches."""
    import paddle_ray_amd as paddle
    from paddle_ray_amd.distributed.passes import new_pass
    halves = _feeds(4, rows=4)
    full = [{k: np.concatenate([halves[2 * i][k], halves[2 * i + 1][k]]) for k in ('x', 'y')}
            for i in range(2)]

    def build(passes, rows):
        import paddle_ray_amd.nn as nn
        from paddle_ray_amd import static
        paddle.seed(4)
        main = static.Program()
        with static.program_guard(main):
            x = static.data('x', [rows, 8], 'float32')
            y = static.data('y', [rows, 8], 'float32')
            lin = nn.Linear(8, 8)
            loss = paddle.mean((paddle.tanh(lin(x)) - y) ** 2)
            opt = paddle.optimizer.Momentum(0.2, momentum=0.9)
            if not after:
                for p in passes:
                    p.apply([main], [None])
            opt.minimize(loss)
            if after:
                for p in passes:
                    p.apply([main], [None])
        return main, loss, lin
    m0, l0, lin0 = build([], 8)
    _train(m0, l0, full)
    m1, l1, lin1 = build([new_pass('auto_parallel_gradient_merge_pass', {'k_steps': 2, 'avg': True})], 4)
    w_before = lin1.weight.numpy().copy()
    from paddle_ray_amd import static
    exe = static.Executor()
    exe.run(m1, feed=halves[0], fetch_list=[l1])
    np.testing.assert_array_equal(lin1.weight.numpy(), w_before)     # mid-window: no step
    for f in halves[1:]:
        exe.run(m1, feed=f, fetch_list=[l1])
    np.testing.assert_allclose(lin1.weight.numpy(), lin0.weight.numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(lin1.bias.numpy(), lin0.bias.numpy(), rtol=1e-5, atol=1e-6)


def test_sharding_pass_rejects_stage_2_and_3(static_mode):
    from paddle_ray_amd.distributed.passes import new_pass
    for st in (2, 3):
        with pytest.raises(NotImplementedError):
            _ffn_program([new_pass('auto_parallel_sharding', {'stage': st})])


def test_rebuild_restores_optimizer_and_composes(static_mode):
    """Passes applied one after another on a minimized program: each rebuild starts from the
    forward (no duplicated grad / optimize ops)."""
    from paddle_ray_amd.distributed.passes import new_pass
    m, loss, _ = _ffn_program()
    n_ops = len(m.global_block().ops)
    n_vars = len(m.global_block().vars)
    for p in (new_pass('auto_parallel_amp', {'dtype': 'bfloat16'}), new_pass('fuse_gemm_epilogue'),
              new_pass('auto_parallel_gradient_merge_pass', {'k_steps': 2})):
        p.apply([m], [None])
    ops = m.global_block().ops
    assert sum(op.role == 'optimize' for op in ops) == 1
    assert sum(op.type == 'fill_grad_seed' for op in ops) == 1
    assert len(ops) < n_ops + 8 and len(m.global_block().vars) < n_vars + 12
    assert ops[-1].type == 'fleet_optimize' and m._fleet_state.k_steps == 2
    _train(m, loss, _feeds(2))


# -- partitioned programs on gloo ranks -----------------------------------------------------------------
def _build_serial(specs, mesh, clip=None):
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
    return main, h, loss, (l1.weight, l1.bias, l2.weight, l2.bias)


def _slice(a, mapping, mesh_shape, coord):
    for i, d in enumerate(mapping):
        if d >= 0:
            n = a.shape[i] // mesh_shape[d]
            a = np.take(a, range(coord[d] * n, (coord[d] + 1) * n), axis=i)
    return a


def _run_passes(rank, world, mesh_ids, names, specs, names_on, clip_norm, dp_axis):
    import paddle_ray_amd as paddle
    from paddle_ray_amd import static
    from paddle_ray_amd.distributed import auto_parallel as ap
    from paddle_ray_amd.distributed.passes import new_pass, PassManager
    paddle.enable_static()
    mesh = ap.ProcessMesh(mesh_ids, names)
    main, h, loss, params = _build_serial(specs, mesh)
    dist, vmap, part = ap.parallelize(main)
    local = [part.local_param(p) for p in params]

    def mk(ps):
        clip = paddle.nn.ClipGradByGlobalNorm(clip_norm) if clip_norm else None
        return paddle.optimizer.Momentum(0.5, momentum=0.9, parameters=ps, grad_clip=clip)

    def passes(is_dist, hv):
        out = [new_pass('auto_parallel_recompute', {'checkpoints': [hv]}),
               new_pass('auto_parallel_gradient_merge_pass', {'k_steps': 2, 'avg': True})]
        if is_dist and 'sharding' in names_on:
            g = mesh.axis_group(dp_axis) if dp_axis is not None else None
            out.append(new_pass('auto_parallel_sharding', {'stage': 1, 'group': g}))
        if is_dist and 'clip' in names_on:
            out.append(new_pass('auto_parallel_grad_clip'))
        if is_dist and 'bucket' in names_on:
            out.append(new_pass('fuse_all_reduce', {'max_memory_size': 64}))
        return out
    with static.program_guard(dist):
        mk([p for p in local]).minimize(vmap[loss])
    PassManager(passes(True, vmap[h])).apply([dist], [None])        # after minimize: rebuild
    with static.program_guard(main):
        for p in passes(False, h):
            p.apply([main], [None])
        mk(list(params)).minimize(loss)
    exe = static.Executor()
    rs = np.random.RandomState(3)
    feeds = [{'x': rs.randn(B, H).astype('float32'), 'y': rs.randint(0, C, (B, 1)).astype('int64')}
             for _ in range(4)]
    ref, got = [], []
    for f in feeds:
        ref.append(float(exe.run(main, feed=f, fetch_list=[loss])[0]))
        got.append(float(exe.run(dist, feed=f, fetch_list=[vmap[loss]])[0]))
    coord = mesh.coord()
    errs = [float(np.abs(lp.numpy() - _slice(p.numpy(), part.ctx.get(p), mesh.shape, coord)).max())
            for p, lp in zip(params, local)]
    ops = [op.type for op in dist.global_block().ops]
    st = dist._fleet_state
    owned = None if st.shard is None else sorted(st.shard.owner.items())
    paddle.disable_static()
    return {'ref': ref, 'loss': got, 'errs': errs, 'ops': ops, 'owned': owned,
            'moved': float(np.abs(params[0].numpy()).sum())}


def test_partitioned_dp_sharding_gradient_merge_recompute(tmp_path):
    specs = {'x': ['x', None], 'y': ['x', None]}
    res = run_ranks(_run_passes, 2, tmp_path, args=([0, 1], ['x'], specs, ('sharding', 'bucket'), None, 0))
    for o in res:
        np.testing.assert_allclose(o['loss'], o['ref'], rtol=1e-5, atol=1e-6)
        assert max(o['errs']) < 1e-5, o['errs']
        assert o['ops'].count('c_allreduce_coalesced') > 1      # 64-byte buckets
        assert 'recompute_rng_swap' in o['ops']
    # stage 1: every parameter has one owner, both ranks own something
    assert res[0]['owned'] == res[1]['owned'] and len({r for _, r in res[0]['owned']}) == 2


@pytest.mark.parametrize('with_pass', [True, False])
def test_partitioned_tp_global_norm_clip(tmp_path, with_pass):
    """Tensor-parallel weights: without the grad-clip pass each rank clips by its shard's norm
    (diverges from serial); with it the clip sees the whole model's norm."""
    specs = {'w1': [None, 'x'], 'b1': ['x'], 'w2': ['x', None]}
    on = ('clip',) if with_pass else ()
    res = run_ranks(_run_passes, 2, tmp_path, args=([0, 1], ['x'], specs, on, 0.05, None))
    errs = max(max(o['errs']) for o in res)
    if with_pass:
        assert errs < 1e-5, errs
        for o in res:
            np.testing.assert_allclose(o['loss'], o['ref'], rtol=1e-5, atol=1e-6)
    else:
        assert errs > 1e-4, errs


def test_partitioned_hybrid_sharding_and_clip_4ranks(tmp_path):
    specs = {'x': ['dp', None], 'y': ['dp', None], 'w1': [None, 'mp'], 'b1': ['mp'], 'w2': ['mp', None]}
    res = run_ranks(_run_passes, 4, tmp_path,
                    args=([[0, 1], [2, 3]], ['dp', 'mp'], specs, ('sharding', 'clip'), 0.05, 0))
    for o in res:
        np.testing.assert_allclose(o['loss'], o['ref'], rtol=1e-5, atol=1e-6)
        assert max(o['errs']) < 1e-5, o['errs']


def _engine_strategy(rank, world, annotate):
    """Static auto_parallel.Engine with strategy.recompute (auto_parallel.recompute region),
    gradient_merge and a global-norm clip: the Engine applies them as passes."""
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
            return self.l2(F.dropout(ap.recompute(lambda t: F.relu(self.l1(t)))(x), 0.0))

    class DS(Dataset):
        def __init__(self):
            rs = np.random.RandomState(0)
            self.x = rs.randn(32, H).astype('float32')
            self.y = rs.randint(0, C, (32, 1)).astype('int64')

        def __getitem__(self, i):
            return self.x[i], self.y[i]

        def __len__(self):
            return 32

    st = ap.Strategy()
    st.recompute.enable = True
    st.gradient_merge.enable = True
    st.gradient_merge.k_steps = 2
    model = MLP()
    opt = paddle.optimizer.Momentum(0.2, momentum=0.9, parameters=model.parameters(),
                                    grad_clip=paddle.nn.ClipGradByGlobalNorm(0.05))
    eng = ap.Engine(model, nn.CrossEntropyLoss(), opt, strategy=st)
    eng.prepare([InputSpec([B, H], 'float32', 'x')], [InputSpec([B, 1], 'int64', 'y')])
    hist = eng.fit(DS(), batch_size=B, epochs=2, verbose=0)
    prog = eng._dist['program']
    ops = [op.type for op in prog.global_block().ops]
    names = eng._pass_context and [p.name for p in eng._pass_context.passes]
    paddle.disable_static()
    return {'loss': hist['loss'], 'ops': ops, 'passes': names, 'k': prog._fleet_state.k_steps}


def test_engine_static_strategy_passes(tmp_path):
    (tmp_path / 'ref').mkdir()
    (tmp_path / 'tp').mkdir()
    ref = run_ranks(_engine_strategy, 2, tmp_path / 'ref', (False,))[0]
    res = run_ranks(_engine_strategy, 2, tmp_path / 'tp', (True,))
    for o in res:
        np.testing.assert_allclose(o['loss'], ref['loss'], rtol=1e-5, atol=1e-6)
        assert o['passes'] == ['auto_parallel_recompute', 'auto_parallel_gradient_merge_pass',
                               'auto_parallel_grad_clip'], o['passes']
        assert 'recompute_rng_swap' in o['ops'] and o['k'] == 2


@pytest.mark.gpu
def test_fused_feedforward_pass_on_gpu_bf16():
    """On the MI355X the fused ops run the in-tree HIP kernels (MLP GEMM epilogues, add +
    dropout + LayerNorm): the fused bf16 program trains like the unfused one."""
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn as nn
    import paddle_ray_amd.nn.functional as F
    from paddle_ray_amd import static
    from paddle_ray_amd.distributed.passes import new_pass
    paddle.set_device('gpu:0')
    paddle.enable_static()
    try:
        def build(fuse):
            paddle.seed(5)
            paddle.set_default_dtype('bfloat16')
            main = static.Program()
            with static.program_guard(main):
                x = static.data('x', [256, 512], 'bfloat16')
                l1, l2, ln = nn.Linear(512, 2048), nn.Linear(2048, 512), nn.LayerNorm(512)
                z = ln(x + F.dropout(l2(F.gelu(l1(x), approximate=True)), 0.0))
                loss = paddle.mean(z.astype('float32') ** 2)
                if fuse:
                    new_pass('fused_feedforward').apply([main], [None])
                paddle.optimizer.AdamW(1e-3, multi_precision=True).minimize(loss)
            paddle.set_default_dtype('float32')
            return main, loss
        xv = np.random.RandomState(0).randn(256, 512).astype('float32')
        feed = {'x': xv}      # cast to the bf16 data var and moved to the device by the Executor
        out = []
        for fuse in (False, True):
            m, l = build(fuse)
            exe = static.Executor()
            out.append([float(exe.run(m, feed=feed, fetch_list=[l])[0]) for _ in range(4)])
            if fuse:
                assert _fwd_types(m)[:2] == ['fused_mlp_gelu', 'fused_add_dropout_ln']
        np.testing.assert_allclose(out[1], out[0], rtol=2e-2, atol=2e-3)
        assert out[1][-1] < out[1][0]
    finally:
        paddle.disable_static()
