"""BERT / ERNIE encoders (parity: python/paddle/fluid/tests/unittests/prim/model/bert.py):
pretraining loss decreases, fused == unfused layer, padding-mask path, heads, and an
ERNIE TP x PP hybrid (mp 2 x pp 2 on 4 gloo ranks)."""
import numpy as np

import paddle_ray_amd as paddle
from paddle_ray_amd.models import (bert_config, BertForPretraining, BertModel,
                                   BertForSequenceClassification, BertForQuestionAnswering,
                                   ernie_config, ErnieModel)
from dist_utils import run_ranks


def _batch(rs, B=4, S=16, V=1024):
    ids = rs.randint(5, 64, (B, S))
    labels = np.full((B, S), -1)
    pos = rs.rand(B, S) < 0.3
    labels[pos] = ids[pos]
    ids[pos] = 3  # [MASK]
    return (paddle.to_tensor(ids), paddle.to_tensor(labels),
            paddle.to_tensor(rs.randint(0, 2, (B,))))


def test_bert_pretraining_trains():
    paddle.seed(0)
    m = BertForPretraining(bert_config('bert-tiny', hidden_dropout_prob=0.0,
                                       attention_probs_dropout_prob=0.0))
    opt = paddle.optimizer.AdamW(2e-3, parameters=m.parameters())
    rs = np.random.RandomState(0)
    ids, labels, nsp = _batch(rs)
    losses = []
    for _ in range(25):
        loss = m(ids, labels=labels, next_sentence_label=nsp)
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
    assert losses[-1] < losses[0] - 1.0, losses


def test_bert_fused_layer_matches_unfused():
    paddle.seed(1)
    m = BertModel(bert_config('bert-tiny', hidden_dropout_prob=0.0,
                              attention_probs_dropout_prob=0.0))
    m.eval()
    ids = paddle.randint(1, 1000, [2, 12])
    a = m(ids)[0].numpy()
    for layer in m.encoder:
        layer.fused = False
    b = m(ids)[0].numpy()
    np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5)


def test_bert_padding_mask_ignores_pad_tokens():
    paddle.seed(2)
    m = BertModel(bert_config('bert-tiny', hidden_dropout_prob=0.0,
                              attention_probs_dropout_prob=0.0))
    m.eval()
    ids = np.random.RandomState(1).randint(5, 500, (1, 10))
    padded = np.concatenate([ids, np.zeros((1, 6), dtype=ids.dtype)], 1)
    a = m(paddle.to_tensor(ids))[0].numpy()
    b = m(paddle.to_tensor(padded))[0].numpy()[:, :10]
    np.testing.assert_allclose(a, b, rtol=1e-3, atol=1e-4)


def test_bert_heads_and_ernie():
    paddle.seed(3)
    cfg = bert_config('bert-tiny')
    ids = paddle.randint(1, 1000, [2, 8])
    assert BertForSequenceClassification(cfg, num_classes=3)(ids).shape == [2, 3]
    s, e = BertForQuestionAnswering(cfg)(ids)
    assert s.shape == [2, 8] and e.shape == [2, 8]
    ecfg = ernie_config('ernie-3.0-medium-zh', vocab_size=1000, num_hidden_layers=1,
                        hidden_size=64, num_attention_heads=2, intermediate_size=128)
    seq, pooled = ErnieModel(ecfg)(ids, task_type_ids=paddle.zeros([2, 8], 'int64'))
    assert seq.shape == [2, 8, 64] and pooled.shape == [2, 64]


def _ernie_hybrid_worker(rank, world):
    import paddle_ray_amd as paddle
    from paddle_ray_amd.distributed import fleet
    from paddle_ray_amd.models import bert_config, ernie_pipe
    st = fleet.DistributedStrategy()
    st.hybrid_configs = {'dp_degree': 1, 'mp_degree': 2, 'pp_degree': 2}
    st.pipeline_configs = {'micro_batch_size': 2, 'accumulate_steps': 2}
    fleet.init(is_collective=True, strategy=st)
    paddle.seed(0)
    cfg = bert_config('bert-tiny', mp_degree=2, hidden_dropout_prob=0.0,
                      attention_probs_dropout_prob=0.0, num_hidden_layers=2)
    pl = ernie_pipe(cfg)
    model = fleet.distributed_model(pl)
    opt = fleet.distributed_optimizer(paddle.optimizer.AdamW(3e-3, parameters=pl.parameters()))
    rs = np.random.RandomState(0)
    ids = rs.randint(5, 64, (4, 16))
    labels = ids.copy()
    losses = [float(model.train_batch([paddle.to_tensor(ids), paddle.to_tensor(labels)], opt))
              for _ in range(8)]
    return {'losses': losses}


def test_ernie_tp_pp_hybrid(tmp_path):
    res = run_ranks(_ernie_hybrid_worker, 4, tmp_path)
    last = [r['losses'] for r in res]
    # the last pipeline stage (ranks of pp stage 1) reports the loss; it must go down
    ls = max(last, key=lambda l: l[0])
    assert ls[-1] < ls[0], ls
