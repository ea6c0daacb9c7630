"""RCCL (torch.distributed 'nccl' on ROCm) on the real device: a fresh single-rank process
initialises the default group through paddle.distributed.init_parallel_env (backend auto ->
RCCL on a GPU), runs the collectives the DP / sharding / TP paths use on bf16 and fp32 GPU
tensors, then trains a tiny GPT under sharding stage 3 and DataParallel for two steps.

One GPU per box here, so world size 1 (RCCL refuses two ranks on one device); the multi-rank
schedules are covered over gloo by test_distributed.py / test_sharding_zero3.py."""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = textwrap.dedent("""
    import torch, torch.distributed as dist
    import paddle_ray_amd as paddle
    from paddle_ray_amd.distributed import collective as C
    C.init_parallel_env()
    assert dist.get_backend() == 'nccl', dist.get_backend()
    dev = torch.device('cuda', torch.cuda.current_device())
    for dt in (torch.bfloat16, torch.float32):
        x = torch.arange(4096, device=dev, dtype=dt)
        t = paddle.Tensor(x.clone())
        C.all_reduce(t)
        assert torch.equal(t._t, x)
        out = torch.empty(4096, device=dev, dtype=dt)
        dist.all_gather_into_tensor(out, x, async_op=True).wait()
        assert torch.equal(out, x)
        rs = torch.empty(4096, device=dev, dtype=dt)
        dist.reduce_scatter_tensor(rs, x, async_op=True).wait()
        assert torch.equal(rs, x)
        b = paddle.Tensor(x.clone())
        C.broadcast(b, 0)
        assert torch.equal(b._t, x)
    from paddle_ray_amd.models import gpt_config, GPTForPretraining
    from paddle_ray_amd.distributed.sharding import group_sharded_parallel
    losses = {}
    for mode in ('sharding3', 'dp'):
        paddle.seed(7)
        paddle.set_default_dtype('bfloat16')
        model = GPTForPretraining(gpt_config('gpt3-tiny'))
        paddle.set_default_dtype('float32')
        opt = paddle.optimizer.AdamW(1e-3, parameters=model.parameters(), multi_precision=True)
        if mode == 'sharding3':
            model, opt, _ = group_sharded_parallel(model, opt, 'p_g_os')
        else:
            model = paddle.DataParallel(model)
        g = torch.Generator(device=dev).manual_seed(0)
        ids = paddle.Tensor(torch.randint(0, 1024, (2, 65), device=dev, generator=g))
        ls = []
        for _ in range(2):
            loss = model(ids[:, :-1], ids[:, 1:])
            loss.backward()
            opt.step()
            opt.clear_grad()
            ls.append(float(loss))
        losses[mode] = ls
    torch.cuda.synchronize()
    assert abs(losses['sharding3'][0] - losses['dp'][0]) < 1e-3, losses
    assert abs(losses['sharding3'][1] - losses['dp'][1]) < 5e-2, losses
    dist.destroy_process_group()
    print('rccl ok', losses)
""")


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_rccl_single_rank_collectives_and_training():
    env = dict(os.environ, RANK='0', LOCAL_RANK='0', WORLD_SIZE='1', MASTER_ADDR='127.0.0.1',
               MASTER_PORT=str(_free_port()), PYTHONPATH=ROOT + os.pathsep + os.environ.get('PYTHONPATH', ''),
               HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get('HSA_ENABLE_IPC_MODE_LEGACY', '0'))
    env.pop('PRA_DIST_BACKEND', None)
    r = subprocess.run([sys.executable, '-c', SCRIPT], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert 'rccl ok' in r.stdout, r.stdout[-2000:]
