"""The collective watchdog sees the hot-path reducers: a DataParallel gradient bucket whose
all-reduce stalls (one rank late into backward) is reported with its bucket name while the
other rank waits in it, and training then completes normally.

Parity: process_group_nccl.cc per-task timeout watchdog (reported op + rank)."""
import time

import numpy as np

from dist_utils import run_ranks


def _stall_worker(rank, world):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn as nn
    import paddle_ray_amd.distributed as dist
    from paddle_ray_amd.distributed import watchdog
    dist.init_parallel_env()
    wd = watchdog.get_watchdog()
    wd.timeout_s, wd.poll_s = 0.5, 0.05
    seen = []
    wd.on_timeout = lambda name, el: seen.append(name)
    paddle.seed(0)
    model = paddle.DataParallel(nn.Sequential(nn.Linear(8, 16), nn.ReLU(), nn.Linear(16, 2)))
    opt = paddle.optimizer.SGD(0.1, parameters=model.parameters())
    x = paddle.to_tensor(np.random.RandomState(rank).rand(4, 8).astype('float32'))
    loss = model(x).sum()
    if rank == 1:
        time.sleep(2.5)      # rank 1 stalls: rank 0's bucket all-reduce cannot complete
    loss.backward()
    opt.step()
    opt.clear_grad()
    w = model.parameters()[0].numpy()
    return {'seen': seen, 'w': w, 'inflight': wd.in_flight()}


def test_watchdog_reports_stalled_dp_bucket(tmp_path):
    res = run_ranks(_stall_worker, 2, tmp_path)
    assert any(n.startswith('dp_bucket.') for n in res[0]['seen']), res[0]['seen']
    assert not res[1]['seen'], res[1]['seen']          # the late rank never waited long
    np.testing.assert_allclose(res[0]['w'], res[1]['w'])  # the step still completed in sync
    assert res[0]['inflight'] == [] and res[1]['inflight'] == []
