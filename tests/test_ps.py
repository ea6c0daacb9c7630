"""Parameter-server mode (distributed/ps over distributed.rpc): server-side update rules against
torch, and a 2-server / 2-trainer job training a sparse embedding + dense head (role environment
of the reference's PaddleCloudRoleMaker)."""
import os
import socket

import numpy as np
import torch
import torch.multiprocessing as mp

from paddle_ray_amd.distributed import ps


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_server_rules_match_torch():
    w0 = np.random.default_rng(0).standard_normal(5).astype(np.float32)
    g = np.random.default_rng(1).standard_normal(5).astype(np.float32)
    ps._srv_create_dense('t_sgd', w0, {'kind': 'sgd', 'lr': 0.1})
    ps._srv_push_dense({'t_sgd': g})
    np.testing.assert_allclose(ps._srv_pull_dense(['t_sgd'])[0], w0 - 0.1 * g, rtol=1e-6)
    ps._srv_create_dense('t_adam', w0, {'kind': 'adam', 'lr': 0.05})
    p = torch.nn.Parameter(torch.from_numpy(w0.copy()))
    opt = torch.optim.Adam([p], lr=0.05, eps=1e-8)
    for k in range(3):
        ps._srv_push_dense({'t_adam': g * (k + 1)})
        p.grad = torch.from_numpy(g * (k + 1))
        opt.step()
    np.testing.assert_allclose(ps._srv_pull_dense(['t_adam'])[0], p.detach().numpy(), rtol=1e-5, atol=1e-6)
    # sparse rows: created on first touch, deterministic per (seed, id)
    ps._srv_create_sparse('t_emb', 4, {'kind': 'sgd', 'lr': 1.0}, 0.1, 7)
    a = ps._srv_pull_sparse('t_emb', [3, 9])
    np.testing.assert_array_equal(a, ps._srv_pull_sparse('t_emb', [3, 9]))
    ps._srv_push_sparse('t_emb', [9], np.ones((1, 4), np.float32))
    np.testing.assert_allclose(ps._srv_pull_sparse('t_emb', [9])[0], a[1] - 1.0, rtol=1e-6)
    assert ps._srv_sparse_size('t_emb') == 2


def _proc(role, idx, eps, q):
    os.environ.update({'TRAINING_ROLE': role, 'PADDLE_PSERVERS_IP_PORT_LIST': ','.join(eps),
                       'PADDLE_TRAINERS_NUM': '2'})
    from paddle_ray_amd.distributed import fleet
    if role == 'PSERVER':
        os.environ['POD_IP'], os.environ['PADDLE_PORT'] = eps[idx].split(':')
    else:
        os.environ['PADDLE_TRAINER_ID'] = str(idx)
    fleet.init(is_collective=False)          # the reference's PS-mode entry points
    if fleet.is_server():
        assert fleet.server_num() == 2 and fleet.server_index() == idx
        fleet.init_server()
        fleet.run_server()
        q.put((role, idx, None))
        return
    assert fleet.worker_num() == 2 and fleet.worker_index() == idx and fleet.is_first_worker() == (idx == 0)
    fleet.init_worker()
    torch.manual_seed(0)
    emb = ps.SparseEmbedding('emb', 8, optimizer='sgd', lr=0.5, init_std=0.1)
    head = torch.nn.Linear(8, 1)
    opt = ps.DistributedOptimizer(head.parameters(), optimizer='adam', lr=0.05)
    g = torch.Generator().manual_seed(100 + idx)
    losses = []
    for step in range(40):
        ids = torch.randint(0, 50, (32, 3), generator=g)
        y = (ids % 2 == 0).float().mean(1, keepdim=True)
        loss = torch.nn.functional.mse_loss(head(emb(ids).mean(1)), y)
        opt.clear_grad()
        loss.backward()
        opt.step()
        losses.append(float(loss))
    n_rows = ps.sparse_table_size('emb')
    fleet.stop_worker()
    q.put((role, idx, (losses, n_rows)))


def test_ps_two_servers_two_trainers():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    eps = ['127.0.0.1:%d' % _port(), '127.0.0.1:%d' % _port()]
    procs = [ctx.Process(target=_proc, args=('PSERVER', i, eps, q)) for i in range(2)]
    procs += [ctx.Process(target=_proc, args=('TRAINER', i, eps, q)) for i in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    tr = {i: r for role, i, r in res if role == 'TRAINER'}
    for i in range(2):
        losses, n_rows = tr[i]
        assert np.mean(losses[-8:]) < 0.5 * np.mean(losses[:4]), losses
        assert n_rows == 50          # every id in [0, 50) touched, rows split over both servers
