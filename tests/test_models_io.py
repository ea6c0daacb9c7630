"""Model zoo, DataLoader, hapi.Model, metric, profiler (CPU)."""
import os

import numpy as np
import pytest

import paddle_ray_amd as paddle
import paddle_ray_amd.nn as nn
import paddle_ray_amd.nn.functional as F
from paddle_ray_amd.io import DataLoader, TensorDataset, Dataset, BatchSampler, \
    DistributedBatchSampler


def test_gpt_tiny_trains():
    from paddle_ray_amd.models import gpt_config, GPTForPretraining
    paddle.seed(0)
    m = GPTForPretraining(gpt_config('gpt3-tiny', hidden_dropout=0.0))
    opt = paddle.optimizer.AdamW(3e-3, parameters=m.parameters())
    ids = paddle.randint(0, 64, [4, 33])  # small vocab subset -> learnable
    losses = []
    for _ in range(30):
        loss = m(ids[:, :-1], ids[:, 1:])
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
    assert losses[-1] < losses[0] - 1.0, losses


def test_gpt_fused_matches_unfused():
    """Fused residual/LN block path == plain per-op reference path (same weights)."""
    from paddle_ray_amd.models import gpt_config, GPTForPretraining
    paddle.seed(0)
    m = GPTForPretraining(gpt_config('gpt3-tiny', hidden_dropout=0.0))
    ids = paddle.randint(0, 1024, [2, 17])
    fused = float(m(ids[:, :-1], ids[:, 1:]))
    for blk in m.gpt.layers:
        blk.fused = False
    plain = float(m(ids[:, :-1], ids[:, 1:]))
    assert abs(fused - plain) < 1e-4


def test_gpt_recompute_same_grads():
    from paddle_ray_amd.models import gpt_config, GPTForPretraining
    paddle.seed(0)
    m = GPTForPretraining(gpt_config('gpt3-tiny', hidden_dropout=0.1))
    ids = paddle.randint(0, 1024, [2, 17])
    paddle.seed(5)
    m(ids[:, :-1], ids[:, 1:]).backward()
    g1 = m.gpt.layers[0].mlp.fc1.weight.grad.numpy().copy()
    m.clear_gradients()
    m.cfg.recompute = True
    m.gpt.cfg.recompute = True
    paddle.seed(5)
    m(ids[:, :-1], ids[:, 1:]).backward()
    g2 = m.gpt.layers[0].mlp.fc1.weight.grad.numpy()
    np.testing.assert_allclose(g1, g2, rtol=1e-4, atol=1e-6)


def test_vision_models_forward():
    from paddle_ray_amd.vision.models import LeNet, resnet18, resnet50, mobilenet_v2, vgg11
    assert LeNet()(paddle.randn([2, 1, 28, 28])).shape == [2, 10]
    assert resnet18(num_classes=7)(paddle.randn([1, 3, 64, 64])).shape == [1, 7]
    r = resnet50(num_classes=5, data_format='NHWC')
    out = r(paddle.randn([1, 64, 64, 3]))
    assert out.shape == [1, 5]
    assert mobilenet_v2(num_classes=3)(paddle.randn([2, 3, 64, 64])).shape == [2, 3]
    assert sum(p.size for p in resnet50().parameters()) == 25557032


def test_dataloader_batching_and_workers():
    xs = np.arange(20, dtype='float32').reshape(10, 2)
    ys = np.arange(10, dtype='int64')
    ds = TensorDataset([xs, ys])
    dl = DataLoader(ds, batch_size=4, shuffle=False, drop_last=False)
    batches = list(dl)
    assert len(batches) == 3 and len(dl) == 3
    assert batches[0][0].shape == [4, 2]
    np.testing.assert_allclose(batches[-1][1].numpy(), [8, 9])
    dl2 = DataLoader(ds, batch_size=5, num_workers=2)
    assert sum(b[0].shape[0] for b in dl2) == 10
    bs = BatchSampler(ds, batch_size=3, drop_last=True)
    assert len(list(bs)) == 3
    d0 = list(DistributedBatchSampler(ds, 2, num_replicas=2, rank=0))
    d1 = list(DistributedBatchSampler(ds, 2, num_replicas=2, rank=1))
    assert not set(sum(d0, [])) & set(sum(d1, []))


def test_hapi_model_fit_lenet(tmp_path):
    from paddle_ray_amd.vision.datasets import MNIST
    from paddle_ray_amd.vision.models import LeNet
    paddle.seed(0)

    class Small(Dataset):
        def __init__(self):
            self.base = MNIST(mode='test')

        def __len__(self):
            return 64

        def __getitem__(self, i):
            return self.base[i]
    model = paddle.Model(LeNet())
    opt = paddle.optimizer.Adam(1e-3, parameters=model.parameters())
    model.prepare(opt, nn.CrossEntropyLoss(), paddle.metric.Accuracy())
    model.fit(Small(), batch_size=16, epochs=2, verbose=0)
    res = model.evaluate(Small(), batch_size=16, verbose=0)
    assert 'loss' in res and 'acc' in res
    model.save(str(tmp_path / 'lenet'))
    assert os.path.exists(str(tmp_path / 'lenet.pdparams'))
    assert os.path.exists(str(tmp_path / 'lenet.pdopt'))
    model.load(str(tmp_path / 'lenet'))
    preds = model.predict(Small(), batch_size=32, stack_outputs=True)
    assert preds[0].shape == (64, 10)
    info = paddle.summary(LeNet(), (1, 1, 28, 28))
    assert info['total_params'] == 61610


def test_metrics():
    acc = paddle.metric.Accuracy(topk=(1, 2))
    pred = paddle.to_tensor([[0.1, 0.9, 0.0], [0.8, 0.1, 0.1]])
    lab = paddle.to_tensor([[1], [1]])
    acc.update(acc.compute(pred, lab))
    a1, a2 = acc.accumulate()
    assert a1 == 0.5 and a2 == 1.0
    p = paddle.metric.Precision()
    p.update(np.array([1, 1, 0]), np.array([1, 0, 0]))
    assert p.accumulate() == 0.5
    auc = paddle.metric.Auc()
    auc.update(np.array([[0.1, 0.9], [0.8, 0.2]]), np.array([1, 0]))
    assert auc.accumulate() == 1.0


def test_profiler_record_event(tmp_path):
    import paddle_ray_amd.profiler as profiler
    prof = profiler.Profiler(targets=[profiler.ProfilerTarget.CPU])
    prof.start()
    for _ in range(3):
        with profiler.RecordEvent('my_op'):
            paddle.matmul(paddle.randn([8, 8]), paddle.randn([8, 8]))
        prof.step()
    prof.stop()
    out = prof.summary()
    assert 'my_op' in out
    prof.export(str(tmp_path / 'trace.json'))
    assert os.path.exists(str(tmp_path / 'trace.json'))


def test_incubate_fused_layers():
    from paddle_ray_amd.incubate.nn import FusedMultiHeadAttention, FusedFeedForward, \
        FusedLinear, FusedBiasDropoutResidualLayerNorm
    x = paddle.randn([2, 5, 32])
    attn = FusedMultiHeadAttention(32, 4, dropout_rate=0.0, attn_dropout_rate=0.0)
    assert attn(x).shape == [2, 5, 32]
    ffn = FusedFeedForward(32, 64, dropout_rate=0.0, activation='gelu')
    assert ffn(x).shape == [2, 5, 32]
    assert FusedLinear(32, 8)(x).shape == [2, 5, 8]
    ln = FusedBiasDropoutResidualLayerNorm(32, dropout_rate=0.0)
    assert ln(x, x).shape == [2, 5, 32]
