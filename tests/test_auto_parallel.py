"""paddle.distributed.auto_parallel: ProcessMesh, shard_tensor/reshard/shard_op, Strategy, Engine.

Reference strategy: python/paddle/fluid/tests/unittests/auto_parallel/ (test_process_mesh.py,
test_interface.py, engine_api.py trains an MLP through Engine.fit/evaluate/predict). Multi-rank
cases run on gloo (CPU) ranks; Engine DP is checked for parameter parity with single-process
full-batch training.
"""
import numpy as np
import pytest

from dist_utils import run_ranks

pytestmark = pytest.mark.timeout(300) if hasattr(pytest.mark, 'timeout') else []


def test_process_mesh_and_strategy():
    from paddle_ray_amd.distributed import auto_parallel as auto
    m = auto.ProcessMesh([[0, 1, 2], [3, 4, 5]], dim_names=['dp', 'mp'])
    assert m.shape == [2, 3] and m.ndim == 2 and m.process_ids == list(range(6))
    assert m.get_dim_size('mp') == 3 and m.coord(4) == [1, 1] and m.coord(9) is None
    assert m[1].process_ids == [3, 4, 5] and m[1].dim_names == ['mp']
    assert m == auto.ProcessMesh(shape=[2, 3], process_ids=list(range(6)), dim_names=['dp', 'mp'])
    with m:
        assert auto.get_current_process_mesh() is m
    assert auto.get_current_process_mesh() is None
    with pytest.raises(AssertionError):
        auto.ProcessMesh([0, 0])
    s = auto.Strategy({'gradient_merge': {'enable': True, 'k_steps': 4}})
    assert s.gradient_merge.k_steps == 4 and s.amp.enable is False
    s.amp.enable = True
    assert s.to_dict()['amp']['enable'] is True
    with pytest.raises(AttributeError):
        s.amp.bogus = 1
    with pytest.raises(ValueError):
        auto.Strategy({'nope': 1})


def _mesh2x2(rank, world):
    import torch
    import paddle_ray_amd as paddle
    from paddle_ray_amd.distributed import auto_parallel as auto
    mesh = auto.ProcessMesh([[0, 1], [2, 3]], dim_names=['x', 'y'])
    full = torch.arange(48, dtype=torch.float32).reshape(6, 8)
    out = {}
    a = auto.shard_tensor(paddle.Tensor(full.clone()), mesh, ['x', 'y'])
    out['xy'] = a.numpy()
    b = auto.reshard(a, mesh, ['y', None])       # gathers both axes, re-splits rows over y
    out['y_none'] = b.numpy()
    out['global'] = auto.to_global(b).numpy()
    # gradient flows back through the gather to the local shard
    w = paddle.Tensor(full.clone())
    w.stop_gradient = False
    s = auto.shard_tensor(w, mesh, [None, 'x'])
    g = auto.to_global(s)
    (g._t * g._t).sum().backward()
    out['grad'] = w._t.grad.numpy()   # the shard is a view of w: its gradient lands in w's local columns
    # shard_op: replicated inputs in, output annotated as sharded over x
    f = auto.shard_op(lambda u: u * 2, mesh, in_shard_specs=[None], out_shard_specs=[['x', None]])
    r = f(paddle.Tensor(full.clone()))
    out['op'] = r.numpy()
    out['op_attr'] = auto.dist_attr(r).dims_mapping
    return out


def test_shard_reshard_2x2(tmp_path):
    res = run_ranks(_mesh2x2, 4, tmp_path)
    full = np.arange(48, dtype=np.float32).reshape(6, 8)
    coords = {0: (0, 0), 1: (0, 1), 2: (1, 0), 3: (1, 1)}
    for r, o in enumerate(res):
        cx, cy = coords[r]
        np.testing.assert_array_equal(o['xy'], full[3 * cx:3 * cx + 3, 4 * cy:4 * cy + 4])
        np.testing.assert_array_equal(o['y_none'], full[3 * cy:3 * cy + 3])
        np.testing.assert_array_equal(o['global'], full)
        np.testing.assert_array_equal(o['op'], 2 * full[3 * cx:3 * cx + 3])
        assert o['op_attr'] == [0, -1]
        want = np.zeros_like(full)
        want[:, 4 * cx:4 * cx + 4] = 2 * full[:, 4 * cx:4 * cx + 4]
        np.testing.assert_allclose(o['grad'], want)


def _engine(rank, world):
    import torch
    import paddle_ray_amd as paddle
    from paddle_ray_amd.distributed import auto_parallel as auto
    from paddle_ray_amd.io import TensorDataset

    def make():
        paddle.seed(7)
        return paddle.nn.Sequential(paddle.nn.Linear(8, 16), paddle.nn.Tanh(), paddle.nn.Linear(16, 1))
    g = torch.Generator().manual_seed(3)
    X = torch.randn(32, 8, generator=g)
    Y = torch.randn(32, 1, generator=g)
    ds = TensorDataset([paddle.Tensor(X), paddle.Tensor(Y)])
    model = make()
    opt = paddle.optimizer.SGD(0.1, parameters=model.parameters())
    eng = auto.Engine(model, paddle.nn.MSELoss(), opt,
                      strategy=auto.Strategy({'gradient_merge': {'enable': True, 'k_steps': 2}}))
    hist = eng.fit(ds, batch_size=4, epochs=2, verbose=0)    # 4 steps/epoch/rank, step every 2
    ev = eng.evaluate(ds, batch_size=8, verbose=0)
    pred = eng.predict(ds, test_sample_split=1, batch_size=8)
    # single-process reference: global batch 8 = both ranks' 4-sample batches, merged over 2 steps
    ref = make()
    ropt = paddle.optimizer.SGD(0.1, parameters=ref.parameters())
    lossf = paddle.nn.MSELoss()
    for _ in range(2):
        for s in range(4):
            idx = [i for r in range(world) for i in range(16 * r + 4 * s, 16 * r + 4 * s + 4)]
            l = lossf(ref(paddle.Tensor(X[idx])), paddle.Tensor(Y[idx])) / 2
            l.backward()
            if s % 2 == 1:
                ropt.step()
                ropt.clear_grad()
    diff = max(float((p._t - q._t).abs().max()) for p, q in zip(model.parameters(), ref.parameters()))
    return {'diff': diff, 'n': len(hist['loss']), 'eval': ev['loss'], 'pred': len(pred)}


def test_engine_dp_parity(tmp_path):
    res = run_ranks(_engine, 2, tmp_path)
    for o in res:
        assert o['n'] == 8 and o['pred'] == 2
        assert o['diff'] < 1e-5, o
        assert np.isfinite(o['eval'])
