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


# -- sync mode and persistence (the_one_ps.py:1340,1459,1644,1730; fleet.py:695,934) ------------------
def _env(role, idx, eps, n_tr):
    os.environ.update({'TRAINING_ROLE': role, 'PADDLE_PSERVERS_IP_PORT_LIST': ','.join(eps),
                       'PADDLE_TRAINERS_NUM': str(n_tr)})
    if role == 'PSERVER':
        os.environ['POD_IP'], os.environ['PADDLE_PORT'] = eps[idx].split(':')
    else:
        os.environ['PADDLE_TRAINER_ID'] = str(idx)


def _batches(idx, steps):
    g = torch.Generator().manual_seed(500 + idx)
    out = []
    for _ in range(steps):
        ids = torch.randint(0, 20, (8, 3), generator=g)
        y = torch.randn(8, 1, generator=g)
        out.append((ids, y))
    return out


def _sync_proc(role, idx, eps, q):
    _env(role, idx, eps, 2)
    from paddle_ray_amd.distributed import fleet
    st = fleet.DistributedStrategy()
    st.a_sync = False
    fleet.init(is_collective=False, strategy=st)
    if fleet.is_server():
        fleet.init_server()
        fleet.run_server()
        q.put((role, idx, None))
        return
    fleet.init_worker()
    torch.manual_seed(0)
    emb = ps.SparseEmbedding('semb', 4, optimizer='sgd', lr=0.3, init_std=0.5, seed=3)
    head = torch.nn.Linear(4, 1)
    opt = ps.DistributedOptimizer(head.parameters(), optimizer='sgd', lr=0.2)
    assert emb.mode == 'sync' and opt.mode == 'sync'
    for ids, y in _batches(idx, 5):
        loss = torch.nn.functional.mse_loss(head(emb(ids).mean(1)), y)
        opt.clear_grad()
        loss.backward()
        opt.step()
    rows = ps.pull_sparse('semb', list(range(20)), min_version=5, all_servers=True).numpy()
    w = [p.detach().numpy().copy() for p in head.parameters()]
    fleet.stop_worker()
    q.put((role, idx, (rows, w)))


def _run_job(target, n_srv, n_tr, extra=()):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    eps = ['127.0.0.1:%d' % _port() for _ in range(n_srv)]
    procs = [ctx.Process(target=target, args=('PSERVER', i, eps, q) + tuple(extra)) for i in range(n_srv)]
    procs += [ctx.Process(target=target, args=('TRAINER', i, eps, q) + tuple(extra)) for i in range(n_tr)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return {i: r for role, i, r in res if role == 'TRAINER'}


def test_ps_sync_mode_matches_serial_sgd():
    """a_sync=False: each step's pushes of both trainers are merged (mean) before one update ->
    identical to serial SGD on the union of the two trainers' batches."""
    tr = _run_job(_sync_proc, 2, 2)
    # the serial reference: same initial rows (deterministic per (seed, id)) and head
    table = np.stack([(np.random.default_rng([3, i]).standard_normal(4) * 0.5).astype(np.float32)
                      for i in range(20)])
    torch.manual_seed(0)
    head = torch.nn.Linear(4, 1)
    emb = torch.nn.Parameter(torch.from_numpy(table.copy()))
    opt = torch.optim.SGD([{'params': head.parameters(), 'lr': 0.2}, {'params': [emb], 'lr': 0.3}])
    b0, b1 = _batches(0, 5), _batches(1, 5)
    for (i0, y0), (i1, y1) in zip(b0, b1):
        l0 = torch.nn.functional.mse_loss(head(emb[i0].mean(1)), y0)
        l1 = torch.nn.functional.mse_loss(head(emb[i1].mean(1)), y1)
        opt.zero_grad()
        ((l0 + l1) / 2).backward()
        opt.step()
    for t in (0, 1):
        rows, w = tr[t]
        np.testing.assert_allclose(rows, emb.detach().numpy(), rtol=1e-5, atol=1e-6)
        for a, b in zip(w, head.parameters()):
            np.testing.assert_allclose(a, b.detach().numpy(), rtol=1e-5, atol=1e-6)


def _persist_proc(role, idx, eps, q, dirname, phase):
    _env(role, idx, eps, 1)
    from paddle_ray_amd.distributed import fleet
    fleet.init(is_collective=False)
    if fleet.is_server():
        fleet.init_server(dirname if phase == 2 else None)
        fleet.run_server()
        q.put((role, idx, None))
        return
    fleet.init_worker()
    torch.manual_seed(1)
    emb = ps.SparseEmbedding('pemb', 6, optimizer='adam', lr=0.05, init_std=0.2, seed=9)
    head = torch.nn.Linear(6, 2)
    opt = ps.DistributedOptimizer(head.parameters(), optimizer='adam', lr=0.05)
    g = torch.Generator().manual_seed(42)

    def step(ids):
        loss = head(emb(ids).mean(1)).pow(2).mean()
        opt.clear_grad()
        loss.backward()
        opt.step()
    ids_last = torch.randint(0, 30, (16, 4), generator=torch.Generator().manual_seed(7))
    if phase == 1:
        for _ in range(6):
            step(torch.randint(0, 30, (16, 4), generator=g))
        inv = fleet.save_persistables(None, dirname)
        before = ps.pull_sparse('pemb', list(range(30))).numpy()
    else:
        inv = None
        before = ps.pull_sparse('pemb', list(range(30))).numpy()
    size = ps.sparse_table_size('pemb')
    w_before = [p.detach().numpy().copy() for p in head.parameters()]
    step(ids_last)          # one more identical Adam step: needs the restored moments to agree
    after = ps.pull_sparse('pemb', list(range(30))).numpy()
    w_after = [p.detach().numpy().copy() for p in head.parameters()]
    fleet.stop_worker()
    q.put((role, idx, (before, w_before, after, w_after, size, inv)))


def test_ps_save_restart_resume(tmp_path):
    """save_persistables from a 2-server job, restart with 3 servers + init_server(dirname): the
    tables (rows re-partitioned by id % 3) and the Adam state resume exactly."""
    d = str(tmp_path / 'ckpt')
    t1 = _run_job(_persist_proc, 2, 1, (d, 1))[0]
    assert os.path.exists(os.path.join(d, 'sparse', 'pemb', 'part-0-of-2.npz'))
    assert os.path.exists(os.path.join(d, 'sparse', 'pemb', 'part-1-of-2.npz'))
    t2 = _run_job(_persist_proc, 3, 1, (d, 2))[0]
    b1, wb1, a1, wa1, n1, inv = t1
    b2, wb2, a2, wa2, n2, _ = t2
    assert len(inv) == 2 and sum(v['pemb'] for v in (i['sparse'] for i in inv)) == n1
    np.testing.assert_array_equal(b1, b2)          # every row restored bit for bit
    assert n2 >= n1
    for x, y in zip(wb1, wb2):
        np.testing.assert_array_equal(x, y)
    np.testing.assert_allclose(a1, a2, rtol=1e-6, atol=1e-7)    # Adam moments restored
    for x, y in zip(wa1, wa2):
        np.testing.assert_allclose(x, y, rtol=1e-6, atol=1e-7)
