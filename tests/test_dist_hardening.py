"""Multi-GPU hardening, rehearsed on gloo/CPU: ZeRO-3 gradient accumulation across several
backward passes, the two-communicator ZeRO-3 schedule (all-gathers on a twin process group),
the resident (no backward re-gather) mode, the bench rank supervisor and the launcher's
device binding."""
import os
import subprocess
import sys
import time

import numpy as np
import pytest

from dist_utils import run_ranks
from test_sharding_zero3 import _deep_mlp, _data, _opt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _single_accum(k=3, steps=2):
    """One optimizer step per k micro-batches, single process (loss summed over micro-batches)."""
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn.functional as F
    m = _deep_mlp()
    o = _opt(paddle, m.parameters())
    xs, ys = _data(n=24)
    for _ in range(steps):
        for i in range(k):
            # rank r of 2 sees rows [r*12:(r+1)*12]; micro-batch i is 4 rows of each rank's part
            rows = np.concatenate([np.arange(r * 12 + 4 * i, r * 12 + 4 * i + 4) for r in range(2)])
            loss = F.mse_loss(m(paddle.to_tensor(xs[rows])), paddle.to_tensor(ys[rows]))
            loss.backward()
        o.step()
        o.clear_grad()
    return [p.numpy() for p in m.parameters()]


def _zero3_accum_worker(rank, world, release, k=3, steps=2):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn.functional as F
    from paddle_ray_amd.distributed.sharding import group_sharded_parallel
    m = _deep_mlp()
    o = _opt(paddle, m.parameters())
    sm, so, _ = group_sharded_parallel(m, o, 'p_g_os', segment_size=0, bucket_mb=1,
                                       release_after_forward=release)
    st = sm._state
    xs, ys = _data(n=24)
    regathers = 0
    for _ in range(steps):
        for i in range(k):
            rows = np.arange(rank * 12 + 4 * i, rank * 12 + 4 * i + 4)
            out = sm(paddle.to_tensor(xs[rows]))
            loss = F.mse_loss(out, paddle.to_tensor(ys[rows]))
            n_before = len(st.gather_works)
            loss.backward()
            regathers += n_before
        so.step()
        so.clear_grad()
    sd = sm.state_dict()
    return {'params': [sd[kk].numpy() for kk in sd], 'release': st.release_after_forward,
            'twin': st.ag_pg is not st.pg, 'n_units': len(st.unit_meta)}


@pytest.mark.parametrize('release', [True, False])
def test_zero3_accumulates_over_backward_passes(tmp_path, release):
    """k backward passes + one step under stage 3 == one step on the summed loss (the
    reduce-scatter of passes 2..k is added into the owned shard, not overwritten)."""
    ref = _single_accum()
    res = run_ranks(_zero3_accum_worker, 2, tmp_path, (release,))
    for r in res:
        assert r['release'] == release and r['twin'] and r['n_units'] == 6
        for a, b in zip(r['params'], ref):
            # the single process averages each micro-batch over 8 rows; the 2 ranks average over
            # 4 rows each and the reduce-scatter averages the ranks: the same gradient
            np.testing.assert_allclose(a, b, rtol=3e-4, atol=3e-5)


def _twin_worker(rank, world):
    import torch
    from paddle_ray_amd.distributed import collective as C
    groups = [C.new_group([0, 1]), C.new_group([2, 3])]
    mine = groups[rank // 2]
    tw = C.twin_group(mine)
    t = torch.tensor([float(rank)])
    torch.distributed.all_reduce(t, group=tw.process_group)
    return tw.ranks, float(t), tw.process_group is not mine.process_group


def test_twin_group_has_same_ranks(tmp_path):
    res = run_ranks(_twin_worker, 4, tmp_path)
    assert res[0] == ([0, 1], 1.0, True) and res[3] == ([2, 3], 5.0, True)


def test_bench_supervisor_stops_siblings_on_failure():
    sys.path.insert(0, ROOT)
    import bench
    procs = [subprocess.Popen([sys.executable, '-c', 'import time; time.sleep(60)']),
             subprocess.Popen([sys.executable, '-c', 'import sys, time; time.sleep(0.5); sys.exit(3)']),
             subprocess.Popen([sys.executable, '-c', 'import time; time.sleep(60)'])]
    t0 = time.monotonic()
    rc = bench._supervise(procs, limit_s=120, grace_s=5)
    assert rc == 3
    assert time.monotonic() - t0 < 20
    assert all(p.poll() is not None for p in procs)


def test_bench_supervisor_wall_clock_limit():
    sys.path.insert(0, ROOT)
    import bench
    procs = [subprocess.Popen([sys.executable, '-c', 'import time; time.sleep(60)']) for _ in range(2)]
    t0 = time.monotonic()
    rc = bench._supervise(procs, limit_s=1.0, grace_s=5)
    assert rc == 124 and time.monotonic() - t0 < 15
    assert all(p.poll() is not None for p in procs)


def test_spawn_join_terminates_siblings():
    import importlib
    import multiprocessing as mp
    S = importlib.import_module('paddle_ray_amd.distributed.spawn')
    ctx = mp.get_context('spawn')
    ps = [ctx.Process(target=time.sleep, args=(60,)), ctx.Process(target=sys.exit, args=(2,))]
    for p in ps:
        p.start()
    t0 = time.monotonic()
    with pytest.raises(RuntimeError):
        S.MultiprocessContext(ps).join()
    assert time.monotonic() - t0 < 30
    assert all(p.exitcode is not None for p in ps)


def test_launcher_device_binding(monkeypatch):
    import torch
    from paddle_ray_amd.distributed import collective as C
    monkeypatch.setattr(torch.cuda, 'device_count', lambda: 8)
    monkeypatch.setenv('LOCAL_RANK', '1')
    monkeypatch.setenv('FLAGS_selected_gpus', '5')
    assert C._bound_device() == 5
    assert C.ParallelEnv().device_id == 5
    monkeypatch.setenv('FLAGS_selected_gpus', '4,5')
    assert C.ParallelEnv().device_id == 4
    monkeypatch.delenv('FLAGS_selected_gpus')
    assert C._bound_device() == 1


def _gm_worker(rank, world, k=2, steps=2):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn.functional as F
    from paddle_ray_amd.distributed import fleet
    st = fleet.DistributedStrategy()
    st.hybrid_configs = {'dp_degree': 2}
    st.gradient_merge = True
    st.gradient_merge_configs = {'k_steps': k, 'avg': True}
    fleet.init(is_collective=True, strategy=st)
    m = _deep_mlp()
    o = paddle.optimizer.SGD(0.1, parameters=m.parameters())
    dm = fleet.distributed_model(m)
    o = fleet.distributed_optimizer(o)
    xs, ys = _data(n=16)
    for s in range(steps * k):
        rows = np.arange(rank * 8 + 4 * (s % k), rank * 8 + 4 * (s % k) + 4)
        loss = F.mse_loss(dm(paddle.to_tensor(xs[rows])), paddle.to_tensor(ys[rows]))
        loss.backward()
        o.step()
        o.clear_grad()
    sd = fleet.state_dict()
    red = dm._reducer if hasattr(dm, '_reducer') else dm._layers._reducer
    return {'params': [p.numpy() for p in m.parameters()], 'finalized': red.finalize_count,
            'keys': sorted(sd), 'n_model': len(sd['model'])}


def _gm_single(k=2, steps=2):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn.functional as F
    m = _deep_mlp()
    o = paddle.optimizer.SGD(0.1, parameters=m.parameters())
    xs, ys = _data(n=16)
    for _ in range(steps):
        for i in range(k):
            rows = np.concatenate([np.arange(r * 8 + 4 * i, r * 8 + 4 * i + 4) for r in range(2)])
            (F.mse_loss(m(paddle.to_tensor(xs[rows])), paddle.to_tensor(ys[rows])) / k).backward()
        o.step()
        o.clear_grad()
    return [p.numpy() for p in m.parameters()]


def test_gradient_merge_all_reduces_once_per_window(tmp_path):
    ref = _gm_single()
    res = run_ranks(_gm_worker, 2, tmp_path)
    for r in res:
        assert r['finalized'] == 2  # 2 windows of k=2 backward passes: 2 reductions, not 4
        assert r['keys'] == ['model', 'optimizer'] and r['n_model'] > 0
        for a, b in zip(r['params'], ref):
            np.testing.assert_allclose(a, b, rtol=2e-4, atol=2e-5)
