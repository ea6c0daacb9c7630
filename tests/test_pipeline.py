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
    return {'losses': losses, 'emb': embw, 'stage': hcg.get_stage_id(), 'dp': d, 'nst': nst}


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
