"""Pipeline parallel completeness (gloo, CPU): tied embedding across stages
(SharedLayerDesc weight broadcast + gradient all-reduce), tuple activations between stages,
the interleaved (virtual-stage) schedule, and dp x pp with bucketed DP all-reduce — each
checked against a single-process run of the same model and micro-batching.

Parity: pp_layers.py:485 _synchronize_shared_weights, :498 allreduce_shared_weight_gradients,
pipeline_parallel.py:461 PipelineParallelWithInterleave."""
import numpy as np
import pytest

from dist_utils import run_ranks

V, H = 32, 16


def _layers():
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn as nn
    from paddle_ray_amd.framework.core import Tensor, _u

    class Split(nn.Layer):      # emits a TUPLE activation
        def __init__(self):
            super().__init__()
            self.lin = nn.Linear(H, H)

        def forward(self, x):
            h = self.lin(x)
            return h, paddle.tanh(h) * 0.5

    class Join(nn.Layer):       # consumes the tuple
        def __init__(self):
            super().__init__()
            self.lin = nn.Linear(H, H)

        def forward(self, xs):
            a, b = xs
            return self.lin(a + b)

    class Mid(nn.Layer):
        def __init__(self):
            super().__init__()
            self.lin = nn.Linear(H, H)

        def forward(self, x):
            return paddle.tanh(self.lin(x))

    def head(emb, x):
        return paddle.matmul(x, emb.weight, transpose_y=True)

    return Split, Join, Mid, head


def _loss(logits, labels):
    import paddle_ray_amd.nn.functional as F
    return F.cross_entropy(logits.reshape([-1, V]), labels.reshape([-1]))


def _descs():
    import paddle_ray_amd.nn as nn
    from paddle_ray_amd.parallel.pipeline import LayerDesc, SharedLayerDesc
    Split, Join, Mid, head = _layers()
    # pp=2 cuts after Split (a tuple crosses the stage boundary); with 2 virtual stages the
    # chunks are [embed, Mid] [Mid, Split] | [Join] [Mid, head] and the tuple crosses the ring
    return [SharedLayerDesc('embed', nn.Embedding, None, 'weight', V, H),
            LayerDesc(Mid), LayerDesc(Mid), LayerDesc(Split), LayerDesc(Join), LayerDesc(Mid),
            SharedLayerDesc('embed', nn.Embedding, head, 'weight', V, H)]


def _build_full(seed=0):
    """Reference layers built in desc order (the shared embedding once)."""
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn as nn
    paddle.seed(seed)
    Split, Join, Mid, head = _layers()
    emb = nn.Embedding(V, H)
    body = [Mid(), Mid(), Split(), Join(), Mid()]
    return emb, body, head


def _data(n=16, seed=3):
    rs = np.random.RandomState(seed)
    return rs.randint(0, V, (n, 6)).astype('int64'), rs.randint(0, V, (n, 6)).astype('int64')


def _single(steps, n_micro, mbs, data_slices=1):
    import paddle_ray_amd as paddle
    emb, body, head = _build_full()
    params = emb.parameters() + [p for l in body for p in l.parameters()]
    opt = paddle.optimizer.SGD(0.2, parameters=params)
    xs, ys = _data(n_micro * mbs * data_slices)
    losses = []
    for _ in range(steps):
        tot = 0.0
        nm = n_micro * data_slices
        for i in range(nm):
            x = emb(paddle.to_tensor(xs[i * mbs:(i + 1) * mbs]))
            for l in body:
                x = l(x)
            loss = _loss(head(emb, x), paddle.to_tensor(ys[i * mbs:(i + 1) * mbs])) / nm
            loss.backward()
            tot += float(loss)
        opt.step()
        opt.clear_grad()
        losses.append(tot * data_slices)
    return losses, emb.weight.numpy()


def _pp_worker(rank, world, pp, dp, virtual, steps=3, n_micro=4, mbs=2):
    import paddle_ray_amd as paddle
    from paddle_ray_amd.distributed import fleet
    from paddle_ray_amd.parallel.pipeline import PipelineLayer
    st = fleet.DistributedStrategy()
    st.hybrid_configs = {'dp_degree': dp, 'mp_degree': 1, 'pp_degree': pp}
    st.pipeline_configs = {'micro_batch_size': mbs, 'accumulate_steps': n_micro}
    fleet.init(is_collective=True, strategy=st)
    hcg = fleet.get_hybrid_communicate_group()
    paddle.seed(100 + rank)  # different random init per rank: the shared weight is broadcast
    pl = PipelineLayer(_descs(), loss_fn=_loss, num_virtual_pipeline_stages=virtual)
    emb, body, head = _build_full()
    full = [emb] + body + [emb]
    nst = pp * virtual
    for v in range(virtual):
        part = v * pp + hcg.get_stage_id()
        lo, hi = pl.segment_parts[part], pl.segment_parts[part + 1]
        for i in range(lo, hi):
            d = pl._layers_desc[i]
            if hasattr(d, 'layer_name'):
                continue
            pl._chunks[v][i - lo].set_state_dict(full[i].state_dict())
    if 'embed' in pl.shared_layers and hcg.get_stage_id() == 0:
        pl.shared_layers['embed'].set_state_dict(emb.state_dict())
    pl._synchronize_shared_weights()  # re-broadcast the reference init from the first owner
    model = fleet.distributed_model(pl)
    opt = paddle.optimizer.SGD(0.2, parameters=pl.parameters())
    xs, ys = _data(n_micro * mbs * dp)
    d = hcg.get_data_parallel_rank()
    n = n_micro * mbs
    losses = []
    for _ in range(steps):
        losses.append(float(model.train_batch(
            [paddle.to_tensor(xs[d * n:(d + 1) * n]), paddle.to_tensor(ys[d * n:(d + 1) * n])], opt)))
    embw = pl.shared_layers['embed'].weight.numpy() if 'embed' in pl.shared_layers else None
    return {'losses': losses, 'emb': embw, 'stage': hcg.get_stage_id(), 'dp': d, 'nst': nst,
            'peak': model.peak_live_units}


def test_pp2_tied_embedding_and_tuple_acts(tmp_path):
    ref, ref_emb = _single(3, 4, 2)
    res = run_ranks(_pp_worker, 2, tmp_path, (2, 1, 1))
    for r in res:
        np.testing.assert_allclose(r['losses'], ref, rtol=1e-4, atol=1e-6)
        # both stages hold the tied embedding; their copies stayed identical and correct
        np.testing.assert_allclose(r['emb'], ref_emb, rtol=1e-4, atol=1e-6)


def test_pp2_interleaved_virtual_stages(tmp_path):
    ref, ref_emb = _single(3, 4, 2)
    res = run_ranks(_pp_worker, 2, tmp_path, (2, 1, 2))
    for r in res:
        assert r['nst'] == 4
        np.testing.assert_allclose(r['losses'], ref, rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(r['emb'], ref_emb, rtol=1e-4, atol=1e-6)


def test_dp2_pp2_bucketed_dp(tmp_path):
    ref, ref_emb = _single(3, 4, 2, data_slices=2)
    res = run_ranks(_pp_worker, 4, tmp_path, (2, 2, 1))
    for r in res:
        # each dp replica reports the mean loss of its own half of the batch
        assert len(r['losses']) == 3
        np.testing.assert_allclose(r['emb'], ref_emb, rtol=1e-4, atol=1e-6)


def _ernie_tied_worker(rank, world):
    import paddle_ray_amd as paddle
    from paddle_ray_amd.distributed import fleet
    from paddle_ray_amd.models import bert_config, ernie_pipe
    st = fleet.DistributedStrategy()
    st.hybrid_configs = {'dp_degree': 1, 'mp_degree': 1, 'pp_degree': 2}
    st.pipeline_configs = {'micro_batch_size': 2, 'accumulate_steps': 2}
    fleet.init(is_collective=True, strategy=st)
    paddle.seed(rank)  # different init per stage: the shared embedding must be broadcast
    cfg = bert_config('bert-tiny', hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0,
                      num_hidden_layers=2)
    pl = ernie_pipe(cfg, tie_word_embeddings=True)
    model = fleet.distributed_model(pl)
    opt = paddle.optimizer.AdamW(3e-3, parameters=pl.parameters())
    rs = np.random.RandomState(0)
    ids = rs.randint(5, 64, (4, 16))
    losses = [float(model.train_batch([paddle.to_tensor(ids), paddle.to_tensor(ids.copy())], opt))
              for _ in range(6)]
    return {'losses': losses, 'emb': pl.shared_layers['embed'].word_embeddings.weight.numpy()}


def test_ernie_pipe_tied_embeddings(tmp_path):
    res = run_ranks(_ernie_tied_worker, 2, tmp_path)
    np.testing.assert_allclose(res[0]['emb'], res[1]['emb'], rtol=1e-6, atol=1e-7)
    assert res[0]['losses'][-1] < res[0]['losses'][0]


# -- interleaved 1F1B schedule, bounded activations, pp x sharding ----------------------------
def test_interleaved_order_is_a_valid_1f1b():
    from paddle_ray_amd.parallel.pipeline import interleaved_order
    for nst, V, M in [(2, 2, 4), (2, 2, 8), (4, 2, 8), (4, 3, 12), (2, 3, 2)]:
        for st in range(nst):
            warmup, seq = interleaved_order(M, nst, V, st)
            fw = [k for op, k in seq if op == 'F']
            bw = [k for op, k in seq if op == 'B']
            assert fw == list(range(M * V)) and bw == list(range(M * V))
            live, peak = 0, 0
            for op, _ in seq:
                live += 1 if op == 'F' else -1
                peak = max(peak, live)
            # live activations are bounded by the startup depth, not by M
            assert peak == min(warmup + 1, M * V) if M != nst else peak == M * V
            if M > nst:
                assert peak <= (nst - st - 1) * 2 + (V - 1) * nst + 1


def _pp_peak_worker(rank, world, n_micro):
    r = _pp_worker(rank, world, 2, 1, 2, steps=1, n_micro=n_micro)
    return r


def test_interleaved_peak_live_units_independent_of_microbatches(tmp_path):
    import paddle_ray_amd  # noqa: F401
    peaks = {}
    for n_micro in (4, 8):
        (tmp_path / str(n_micro)).mkdir()
        res = run_ranks(_pp_peak_worker, 2, tmp_path / str(n_micro), (n_micro,))
        peaks[n_micro] = [r['peak'] for r in sorted(res, key=lambda r: r['stage'])]
        ref, _ = _single(1, n_micro, 2)
        for r in res:
            np.testing.assert_allclose(r['losses'], ref, rtol=1e-4, atol=1e-6)
    # stage 0 (deepest startup): (2-0-1)*2 + (2-1)*2 + 1 = 5 live units; stage 1: 3
    assert peaks[4] == peaks[8] == [5, 3], peaks
    assert all(p <= 2 * 2 + 2 for p in peaks[8])  # far below V * M = 16


def _pp_sharding_worker(rank, world, steps=3, n_micro=4, mbs=2):
    import paddle_ray_amd as paddle
    from paddle_ray_amd.distributed import fleet
    from paddle_ray_amd.parallel.pipeline import PipelineLayer
    st = fleet.DistributedStrategy()
    st.hybrid_configs = {'dp_degree': 1, 'mp_degree': 1, 'pp_degree': 2, 'sharding_degree': 2}
    st.sharding_configs = {'stage': 1}
    st.pipeline_configs = {'micro_batch_size': mbs, 'accumulate_steps': n_micro}
    fleet.init(is_collective=True, strategy=st)
    hcg = fleet.get_hybrid_communicate_group()
    paddle.seed(100 + rank)
    pl = PipelineLayer(_descs(), loss_fn=_loss)
    emb, body, head = _build_full()
    full = [emb] + body + [emb]
    part = hcg.get_stage_id()
    lo, hi = pl.segment_parts[part], pl.segment_parts[part + 1]
    for i in range(lo, hi):
        if not hasattr(pl._layers_desc[i], 'layer_name'):
            pl._chunks[0][i - lo].set_state_dict(full[i].state_dict())
    if hcg.get_stage_id() == 0:
        pl.shared_layers['embed'].set_state_dict(emb.state_dict())
    pl._synchronize_shared_weights()
    opt = paddle.optimizer.AdamW(0.05, parameters=pl.parameters(), weight_decay=0.01,
                                 grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
    model = fleet.distributed_model(pl)
    opt = fleet.distributed_optimizer(opt)
    xs, ys = _data(n_micro * mbs * 2)
    d = hcg.get_sharding_parallel_rank()
    n = n_micro * mbs
    for _ in range(steps):
        model.train_batch([paddle.to_tensor(xs[d * n:(d + 1) * n]),
                           paddle.to_tensor(ys[d * n:(d + 1) * n])], opt)
    params = {}
    for v, fns in enumerate(pl._chunks):
        for i, f in enumerate(fns):
            idx = pl.segment_parts[part] + i
            if hasattr(f, 'parameters') and not hasattr(pl._layers_desc[idx], 'layer_name'):
                params[idx] = [p.numpy() for p in f.parameters()]
    return {'stage': hcg.get_stage_id(), 'sh': hcg.get_sharding_parallel_world_size(),
            'emb': pl.shared_layers['embed'].weight.numpy(), 'params': params,
            'sharded': type(opt).__name__}


def _single_adamw(steps=3, n_micro=4, mbs=2, slices=2):
    import paddle_ray_amd as paddle
    emb, body, head = _build_full()
    params = emb.parameters() + [p for l in body for p in l.parameters()]
    opt = paddle.optimizer.AdamW(0.05, parameters=params, weight_decay=0.01,
                                 grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
    xs, ys = _data(n_micro * mbs * slices)
    nm = n_micro * slices
    for _ in range(steps):
        for i in range(nm):
            x = emb(paddle.to_tensor(xs[i * mbs:(i + 1) * mbs]))
            for l in body:
                x = l(x)
            (_loss(head(emb, x), paddle.to_tensor(ys[i * mbs:(i + 1) * mbs])) / nm).backward()
        opt.step()
        opt.clear_grad()
    full = [emb] + body + [emb]
    return emb.weight.numpy(), {i: [p.numpy() for p in full[i].parameters()] for i in range(1, 6)}


def test_pp2_sharding2_matches_single(tmp_path):
    """pipeline x sharding stage 1 on 4 ranks: AdamW + global-norm clip with optimizer state
    sharded inside each stage reproduces the single-process parameters."""
    ref_emb, ref = _single_adamw()
    res = run_ranks(_pp_sharding_worker, 4, tmp_path)
    for r in res:
        assert r['sh'] == 2 and r['sharded'] == 'ShardedOptimizer'
        np.testing.assert_allclose(r['emb'], ref_emb, rtol=2e-4, atol=2e-5)
        for idx, ps in r['params'].items():
            for a, b in zip(ps, ref[idx]):
                np.testing.assert_allclose(a, b, rtol=2e-4, atol=2e-5, err_msg=str(idx))
