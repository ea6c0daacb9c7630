"""Checkpoint byte-format parity with the reference (python/paddle/framework/io.py:54-70
_build_saved_state_dict, :293 reduce_varbase, io_utils.py _unpack_saved_dict /
_pack_loaded_dict) and sharded-checkpoint resume at a different world size."""
import pickle

import numpy as np
import torch

import paddle_ray_amd as paddle
from dist_utils import run_ranks


def test_saved_layout_matches_reference(tmp_path):
    paddle.seed(0)
    lin = paddle.nn.Linear(4, 3)
    sd = lin.state_dict()
    sd['bf'] = paddle.Tensor(torch.randn(5).to(torch.bfloat16))
    sd['bf'].name = 'bf_param'
    sd['nested'] = {'t': lin.weight, 'n': 7}
    path = str(tmp_path / 'm.pdparams')
    paddle.save(sd, path)
    raw = pickle.load(open(path, 'rb'))  # our own file: a plain unpickle is safe here
    table = raw['StructuredToParameterName@@']
    assert table['weight'] == lin.weight.name and table['bias'] == lin.bias.name
    assert isinstance(raw['weight'], np.ndarray) and raw['weight'].dtype == np.float32
    assert raw['bf'].dtype == np.uint16  # bf16 as its bit pattern, like the reference
    name, arr = raw['nested']['t']        # nested tensors: the reduce_varbase (name, ndarray)
    assert name == lin.weight.name and np.array_equal(arr, lin.weight.numpy())
    back = paddle.load(path)
    assert 'StructuredToParameterName@@' not in back
    assert back['weight'].name == lin.weight.name
    assert back['bf'].dtype == paddle.bfloat16
    np.testing.assert_array_equal(back['bf'].astype('float32').numpy(), sd['bf'].astype('float32').numpy())
    np.testing.assert_array_equal(back['nested']['t'].numpy(), lin.weight.numpy())
    kept = paddle.load(path, keep_name_table=True)
    assert kept['StructuredToParameterName@@']['bias'] == lin.bias.name
    assert isinstance(paddle.load(path, return_numpy=True)['weight'], np.ndarray)


def test_loads_reference_layout_with_big_param_slices(tmp_path):
    """A file laid out exactly as the reference writes it with pickle protocol 2: a param
    split into 'key@@.i' slices under 'UnpackBigParamInfor@@', a bf16 uint16 array, the name
    table, and an optimizer-style nested LR_Scheduler dict."""
    w = np.arange(12, dtype=np.float32).reshape(3, 4)
    bf = np.array([0x3f80, 0x4000, 0xbf80], dtype=np.uint16)  # 1.0, 2.0, -1.0 in bf16
    ref_layout = {
        'w@@.0': w.flatten()[:5], 'w@@.1': w.flatten()[5:10], 'w@@.2': w.flatten()[10:],
        'UnpackBigParamInfor@@': {'w': {'OriginShape': (3, 4), 'slices': ['w@@.0', 'w@@.1', 'w@@.2']}},
        'b': bf,
        'LR_Scheduler': {'last_epoch': 3, 'last_lr': 0.5},
        'StructuredToParameterName@@': {'w': 'linear_7.w_0', 'b': 'linear_7.b_0'},
    }
    path = str(tmp_path / 'ref.pdparams')
    with open(path, 'wb') as f:
        pickle.dump(ref_layout, f, protocol=2)
    out = paddle.load(path)
    np.testing.assert_array_equal(out['w'].numpy(), w)
    assert out['w'].name == 'linear_7.w_0'
    assert out['b'].dtype == paddle.bfloat16
    np.testing.assert_array_equal(out['b'].astype('float32').numpy(), [1.0, 2.0, -1.0])
    assert out['LR_Scheduler'] == {'last_epoch': 3, 'last_lr': 0.5}


def test_protocol2_splits_big_params(tmp_path):
    t = paddle.to_tensor(np.random.RandomState(0).rand(10, 7).astype('float32'))
    path = str(tmp_path / 'big.pdparams')
    paddle.save({'big': t}, path, protocol=2, _max_slice_bytes=64)
    raw = pickle.load(open(path, 'rb'))
    assert 'UnpackBigParamInfor@@' in raw and 'big' not in raw
    assert len(raw['UnpackBigParamInfor@@']['big']['slices']) == 5  # 70 floats, 16 per slice
    np.testing.assert_array_equal(paddle.load(path)['big'].numpy(), t.numpy())


def test_checkpoint_refuses_code():
    import io
    import os

    class Evil:
        def __reduce__(self):
            return (os.system, ('true',))
    buf = io.BytesIO()
    pickle.dump({'x': Evil()}, buf)
    buf.seek(0)
    try:
        paddle.load(buf)
    except pickle.UnpicklingError:
        pass
    else:
        raise AssertionError("a checkpoint naming os.system must not load")


def _mlp():
    """Same parameter names in every process (optimizer state is keyed by parameter name,
    as in the reference): build under a fresh unique-name scope."""
    import paddle_ray_amd.nn as nn
    from paddle_ray_amd.utils import unique_name
    paddle.seed(0)
    with unique_name.guard():
        return nn.Sequential(nn.Linear(8, 32), nn.GELU(), nn.Linear(32, 4))


def _data(n=16):
    rs = np.random.RandomState(1)
    return rs.rand(n, 8).astype('float32'), rs.rand(n, 4).astype('float32')


def _train(model, opt, xs, ys, steps):
    import paddle_ray_amd.nn.functional as F
    for _ in range(steps):
        loss = F.mse_loss(model(paddle.to_tensor(xs)), paddle.to_tensor(ys))
        loss.backward()
        opt.step()
        opt.clear_grad()


def _sharded_save_worker(rank, world, out):
    from paddle_ray_amd.distributed.sharding import group_sharded_parallel, \
        save_group_sharded_model
    m = _mlp()
    o = paddle.optimizer.AdamW(0.01, parameters=m.parameters(), weight_decay=0.01)
    sm, so, _ = group_sharded_parallel(m, o, 'os_g', segment_size=0, bucket_mb=0)
    xs, ys = _data()
    n = len(xs) // world
    _train(sm, so, xs[rank * n:(rank + 1) * n], ys[rank * n:(rank + 1) * n], 2)
    save_group_sharded_model(sm, out, so)
    return True


def test_sharded_checkpoint_resumes_at_world_size_1(tmp_path):
    out = str(tmp_path / 'ckpt')
    run_ranks(_sharded_save_worker, 2, tmp_path, (out,))
    # resume in ONE process with the plain optimizer, then 2 more steps
    m = _mlp()
    o = paddle.optimizer.AdamW(0.01, parameters=m.parameters(), weight_decay=0.01)
    m.set_state_dict(paddle.load(out + '/model.pdparams'))
    o.set_state_dict(paddle.load(out + '/model.pdopt'))
    xs, ys = _data()
    _train(m, o, xs, ys, 2)
    # continuous single-process reference: 4 steps
    r = _mlp()
    ro = paddle.optimizer.AdamW(0.01, parameters=r.parameters(), weight_decay=0.01)
    _train(r, ro, xs, ys, 4)
    for a, b in zip(m.parameters(), r.parameters()):
        np.testing.assert_allclose(a.numpy(), b.numpy(), rtol=2e-4, atol=2e-5)


def test_adam_beta_pow_reference_convention():
    """beta{1,2}_pow_acc follow the reference (adamw.py:343-348): beta**(t+1) after t updates,
    and a file without '@step' resumes at step t."""
    import paddle_ray_amd as paddle
    lin = paddle.nn.Linear(3, 2)
    opt = paddle.optimizer.AdamW(0.1, beta1=0.8, beta2=0.9, parameters=lin.parameters())
    for _ in range(3):
        lin(paddle.ones([2, 3])).sum().backward()
        opt.step()
        opt.clear_grad()
    sd = opt.state_dict()
    key = [k for k in sd if k.endswith('_beta1_pow_acc_0')][0]
    np.testing.assert_allclose(float(sd[key]), 0.8 ** 4, rtol=1e-6)
    k2 = key.replace('beta1', 'beta2')
    np.testing.assert_allclose(float(sd[k2]), 0.9 ** 4, rtol=1e-6)
    sd.pop('@step')
    opt2 = paddle.optimizer.AdamW(0.1, beta1=0.8, beta2=0.9, parameters=lin.parameters())
    opt2.set_state_dict(sd)
    assert opt2._step_count == 3
