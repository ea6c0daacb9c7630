"""Per-step collective schedule at world 8 (gloo, CPU ranks), recorded with
``distributed.comm_trace.CommTrace``: which op, how many bytes, on which communicator, and in what
order relative to the compute that depends on it. A schedule that is correct here issues the same
RCCL calls on the 8-GPU node (the framework code path is identical; only the backend differs).

* GPT-tiny, sharding stage 3 (parity: group_sharded_stage3.py `_allgather_buffer` prefetch /
  `_register_backward_hooks` reduce): every unit's all-gather is issued one unit AHEAD of the
  unit's compute (forward and, with release-after-forward, the backward re-gather), on the twin
  all-gather communicator, with bytes = the unit's flat parameters; the gradient reduce-scatters
  run on the main sharding communicator during the backward.
* ERNIE-tiny TP2 x PP4 (parity: pp_utils/p2p_communication.py:180-295 partial send/recv,
  pipeline_parallel.py 1F1B): stage-boundary activations / gradients move as 1/mp slices to the
  same-mp-rank peer of the next / previous stage and are all-gathered over the mp pair; the 1F1B
  order of sends and receives per stage; tensor-parallel all-reduces on the mp communicator.
"""
import dataclasses

import numpy as np

from dist_utils import run_ranks


def _gpt_zero3_worker(rank, world, resident):
    import paddle_ray_amd as paddle
    from paddle_ray_amd.models import gpt_config, GPTForPretraining
    from paddle_ray_amd.distributed.sharding import group_sharded_parallel
    from paddle_ray_amd.distributed.comm_trace import CommTrace
    paddle.seed(0)
    cfg = gpt_config('gpt3-tiny', num_layers=4, hidden_dropout=0.0)
    model = GPTForPretraining(cfg)
    opt = paddle.optimizer.AdamW(1e-3, parameters=model.parameters())
    sm, so, _ = group_sharded_parallel(model, opt, 'p_g_os', segment_size=0,
                                       release_after_forward=not resident)
    st = sm._state
    rs = np.random.RandomState(rank)
    ids = paddle.to_tensor(rs.randint(0, cfg.vocab_size, (2, 33)).astype('int64'))

    def step(tr=None):
        loss = sm(ids[:, :-1], ids[:, 1:])
        tr and tr.mark('fwd_end')
        loss.backward()
        tr and tr.mark('bwd_end')
        so.step()
        tr and tr.mark('opt_end')
        so.clear_grad()
    step()
    with CommTrace() as tr:
        tr.hook_layers({f'u{u.index}': u.layer for u in st.unit_meta})
        step(tr)
    import torch.distributed as dist
    unit_bytes = [sum(st.groups[gi].numel * st.groups[gi].param_buf.element_size() for gi in u.gids)
                  for u in st.unit_meta]
    grad_bytes = [sum(st.groups[gi].numel * st.groups[gi].grad_buf.element_size() for gi in u.gids)
                  for u in st.unit_meta]
    return {'records': [dataclasses.asdict(r) for r in tr.records], 'unit_bytes': unit_bytes,
            'grad_bytes': grad_bytes, 'ag_comm': str(st.ag_pg.group_name),
            'main_comm': str((st.pg or dist.group.WORLD).group_name), 'n_units': len(st.unit_meta)}


def _idx(recs, label):
    return next(r['seq'] for r in recs if r['kind'] == 'mark' and r['op'] == label)


def _check_zero3(res, resident):
    for rank, r in enumerate(res):
        recs, n = r['records'], r['n_units']
        assert n == 4
        ags = [x for x in recs if x['op'] == 'all_gather_into_tensor']
        rss = [x for x in recs if x['op'] == 'reduce_scatter_tensor']
        for a in ags:  # async, all 8 ranks, input = output / world
            assert a['ranks'] == tuple(range(8)) and a['async_op'] and a['bytes'] * 8 == a['out_bytes']
        fwd_end, bwd_end = _idx(recs, 'fwd_end'), _idx(recs, 'bwd_end')
        # the step opens with the root (resident) parameters' gather on the main communicator,
        # after the previous update made them stale
        assert ags[0]['comm'] == r['main_comm'] and ags[0]['seq'] < _idx(recs, 'fwd:u0')
        unit_ags = [a for a in ags if a['comm'] == r['ag_comm']]
        assert len(unit_ags) == len(ags) - 1  # every unit gather rides the twin communicator
        fwd_ags = [a for a in unit_ags if a['seq'] < fwd_end]
        # forward: units 0..3 in order, unit k+1's gather ISSUED before unit k's compute starts
        assert [a['out_bytes'] for a in fwd_ags] == r['unit_bytes'], (rank, fwd_ags)
        for k in range(n):
            assert fwd_ags[k]['seq'] < _idx(recs, f'fwd:u{max(k - 1, 0)}'), (rank, k)
        bwd_ags = [a for a in unit_ags if fwd_end < a['seq'] < bwd_end]
        if resident:
            assert not bwd_ags  # gathered units stay resident from forward to backward
        else:
            # backward re-gather, last unit first; unit k-1 issued before unit k's backward starts
            assert [a['out_bytes'] for a in bwd_ags] == r['unit_bytes'][::-1], (rank, bwd_ags)
            for k in range(n - 1, 0, -1):
                assert bwd_ags[n - k]['seq'] < _idx(recs, f'bwd:u{k}'), (rank, k)
        assert not [a for a in ags if a['seq'] > bwd_end]  # nothing gathered by the update
        # gradient reduce-scatters: main communicator, input = the full gradient, output = 1/8;
        # one per unit, each issued right after its unit's backward (before the next unit's
        # backward starts), then the root's
        assert all(x['comm'] == r['main_comm'] and x['bytes'] == 8 * x['out_bytes'] for x in rss)
        unit_rs = [x for x in rss if x['bytes'] in r['grad_bytes']]
        assert len(unit_rs) == n and len(rss) == n + 1
        assert all(fwd_end < x['seq'] < bwd_end for x in rss)
        for k in range(n - 1, 0, -1):
            rs_k = unit_rs[n - 1 - k]
            assert _idx(recs, f'bwd:u{k}') < rs_k['seq'] < _idx(recs, f'bwd:u{k - 1}'), (rank, k)
    # every rank issues the same ops with the same bytes
    tot = {tuple((x['op'], x['bytes'], x['comm']) for x in r['records'] if x['kind'] == 'comm') for r in res}
    assert len(tot) == 1


def test_gpt_zero3_schedule_world8_release(tmp_path):
    _check_zero3(run_ranks(_gpt_zero3_worker, 8, tmp_path, (False,)), resident=False)


def test_gpt_zero3_schedule_world8_resident(tmp_path):
    _check_zero3(run_ranks(_gpt_zero3_worker, 8, tmp_path, (True,)), resident=True)


def _ernie_tp_pp_worker(rank, world, mp, pp, partial, steps=1, trace=True):
    import paddle_ray_amd as paddle
    from paddle_ray_amd.distributed import fleet
    from paddle_ray_amd.distributed.comm_trace import CommTrace
    from paddle_ray_amd.models import bert_config, ernie_pipe
    st = fleet.DistributedStrategy()
    st.hybrid_configs = {'dp_degree': 1, 'mp_degree': mp, 'pp_degree': pp}
    M = 4
    st.pipeline_configs = {'micro_batch_size': 2, 'accumulate_steps': M, 'enable_partial_send_recv': partial}
    fleet.init(is_collective=True, strategy=st)
    hcg = fleet.get_hybrid_communicate_group()
    paddle.seed(0)
    cfg = bert_config('bert-tiny', mp_degree=mp, hidden_dropout_prob=0.0,
                      attention_probs_dropout_prob=0.0, num_hidden_layers=max(2, pp))
    pl = ernie_pipe(cfg)
    model = fleet.distributed_model(pl)
    opt = fleet.distributed_optimizer(paddle.optimizer.AdamW(3e-3, parameters=pl.parameters()))
    rs = np.random.RandomState(0)
    ids = rs.randint(5, 64, (2 * M, 16))
    data = [paddle.to_tensor(ids), paddle.to_tensor(ids.copy())]
    losses = [float(model.train_batch(data, opt))]
    p2p = model._p2p
    b0 = p2p.bytes_sent
    recs = []
    for _ in range(steps):
        if trace:
            with CommTrace() as tr:
                losses.append(float(model.train_batch(data, opt)))
            recs = [dataclasses.asdict(r) for r in tr.records]
        else:
            losses.append(float(model.train_batch(data, opt)))
    import torch.distributed as dist
    return {'losses': losses, 'records': recs, 'stage': hcg.get_stage_id(),
            'mp_rank': hcg.get_model_parallel_rank(), 'p2p_bytes': p2p.bytes_sent - b0,
            'mp_ranks': tuple(hcg.get_model_parallel_group().ranks),
            'mp_comm': str(hcg.get_model_parallel_group().process_group.group_name),
            'pipe_ranks': tuple(hcg.get_pipe_parallel_group().ranks), 'hidden': cfg.hidden_size}


def test_ernie_tp2_pp4_schedule_world8(tmp_path):
    res = run_ranks(_ernie_tp_pp_worker, 8, tmp_path, (2, 4, True))
    M, mb, S = 4, 2, 16
    for r in res:
        recs, s, nst = r['records'], r['stage'], 4
        act = mb * S * r['hidden'] * 4           # one micro-batch's hidden state, fp32
        sends = [x for x in recs if x['op'] == 'isend' and x['bytes'] >= act // 4]
        recvs = [x for x in recs if x['op'] == 'irecv' and x['out_bytes'] >= act // 4]
        nxt = r['pipe_ranks'][s + 1] if s + 1 < nst else None
        prv = r['pipe_ranks'][s - 1] if s > 0 else None
        # every boundary transfer is a 1/mp slice to / from the same-mp-rank neighbour stage
        for x in sends + recvs:
            assert x['peer'] in (nxt, prv) and len(x['ranks']) == 2, x
        fwd_sends = [x for x in sends if x['peer'] == nxt]
        bwd_sends = [x for x in sends if x['peer'] == prv]
        assert len(fwd_sends) == (M if s < nst - 1 else 0)
        assert len(bwd_sends) == (M if s > 0 else 0)
        assert all(x['bytes'] == act // 2 for x in fwd_sends + bwd_sends), (s, fwd_sends[:1], act)
        # each partial receive is completed by an all-gather over the mp pair (full activation)
        for x in recvs:
            assert x['out_bytes'] == act // 2
            ag = next(y for y in recs[x['seq'] + 1:] if y['op'] == 'all_gather_into_tensor')
            assert ag['ranks'] == r['mp_ranks'] and ag['comm'] == r['mp_comm'] and ag['out_bytes'] == act
        # 1F1B order on the boundary: stage s sends forward activations in warmup
        # min(M, nst - s - 1), then alternates send-act / send-grad
        order = ['F' if x['peer'] == nxt else 'B' for x in sends]
        warm = min(M, nst - s - 1)
        if 0 < s < nst - 1:
            assert order[:warm] == ['F'] * warm, (s, order)
            assert order.count('F') == M and order.count('B') == M
        # tensor parallel: the mp all-reduces ride the mp communicator only
        ars = [x for x in recs if x['op'] == 'all_reduce' and x['comm'] == r['mp_comm']]
        assert ars and all(x['ranks'] == r['mp_ranks'] for x in ars)


def test_partial_send_recv_loss_parity_and_bytes(tmp_path):
    """TP2 x PP2 (4 ranks): partial send/recv on and off give the same losses; the on run moves
    half the point-to-point bytes per rank."""
    (tmp_path / 'on').mkdir()
    (tmp_path / 'off').mkdir()
    on = run_ranks(_ernie_tp_pp_worker, 4, tmp_path / 'on', (2, 2, True, 3, False))
    off = run_ranks(_ernie_tp_pp_worker, 4, tmp_path / 'off', (2, 2, False, 3, False))
    for a, b in zip(on, off):
        np.testing.assert_allclose(a['losses'], b['losses'], rtol=1e-6, atol=1e-7)
        if b['p2p_bytes']:
            assert a['p2p_bytes'] * 2 == b['p2p_bytes'], (a['p2p_bytes'], b['p2p_bytes'])
