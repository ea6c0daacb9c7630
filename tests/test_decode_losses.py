"""Decoding APIs and the sequence losses the round-1 build lacked.

* rnnt_loss: the reference's own fixtures (python/paddle/fluid/tests/unittests/
  test_warprnnt_op.py: per-sample losses, and the log-prob gradient mapped through
  log-softmax) plus the docstring example of python/paddle/nn/functional/loss.py:1857.
* hsigmoid_loss: against an independent per-sample loop of the hierarchical-sigmoid
  definition (default and custom trees), gradients by float64 gradcheck.
* BeamSearchDecoder + dynamic_decode: beam 1 equals greedy decoding; a beam wide enough to
  keep every prefix finds the exhaustive best sequence.
"""
import itertools
import math

import numpy as np
import torch

import paddle_ray_amd as paddle
import paddle_ray_amd.nn as nn
import paddle_ray_amd.nn.functional as F

_ACTS = np.array([
    [[[-1.40493705, -0.68276381, -1.38870219], [-1.25243963, -1.03148021, -1.02802034],
      [-1.19624572, -0.93786934, -1.18347801]],
     [[-1.03417513, -0.84465814, -1.53815849], [-0.96884241, -1.01432347, -1.35545407],
      [-0.82076925, -1.10135010, -1.48067081]],
     [[-1.43828803, -1.16579869, -0.79630424], [-1.38401855, -0.83654478, -1.15129927],
      [-1.05188255, -1.29604414, -0.97522265]],
     [[-1.34330978, -0.86678589, -1.14344457], [-0.72518815, -1.32106859, -1.39063758],
      [-1.09984781, -1.00059987, -1.20590993]]],
    [[[-1.02221057, -1.47617485, -0.88748174], [-1.18362952, -0.78488945, -1.43689575],
      [-1.00784739, -1.28566450, -1.02574476]],
     [[-1.02589709, -1.13153743, -1.14260096], [-1.09942215, -1.12238913, -1.07459704],
      [-1.09359647, -0.89829379, -1.35585602]],
     [[-1.07782876, -0.84361953, -1.47178440], [-1.23424792, -1.00248783, -1.07299990],
      [-0.96521771, -1.19895815, -1.14698912]],
     [[-1.50722446, -1.15380039, -0.76994115], [-1.19125975, -0.89919308, -1.24041594],
      [-0.91301359, -1.19665577, -1.21576258]]]], dtype=np.float64)
# gradient of the loss w.r.t. the log-probs, sample 0 (reference fixture set_gradient)
_G0 = np.array([
    [[-0.43222645, -0.56777355, 0.0], [-0.3656501, 0.0, -0.20212345], [-0.20212345, 0.0, 0.0]],
    [[-0.16521672, -0.26700973, 0.0], [-0.39436539, 0.0, -0.23829444], [-0.44041789, 0.0, 0.0]],
    [[-0.05212979, -0.11308693, 0.0], [-0.18313787, 0.0, -0.32431445], [-0.76473234, 0.0, 0.0]],
    [[0.0, -0.05212979, 0.0], [0.0, 0.0, -0.23526766], [-1.0, 0.0, 0.0]]])


def test_rnnt_loss_reference_fixture():
    acts = np.concatenate([_ACTS, _ACTS[1:]], 0)  # samples 1 and 2 of the fixture are equal
    labels = np.array([[1, 2], [1, 1], [1, 1]], np.int32)
    x = paddle.to_tensor(acts, stop_gradient=False)
    loss = F.rnnt_loss(x, paddle.to_tensor(labels), paddle.to_tensor(np.array([4, 4, 4], np.int32)),
                       paddle.to_tensor(np.array([2, 2, 2], np.int32)), blank=0,
                       fastemit_lambda=0.0, reduction='none')
    np.testing.assert_allclose(loss.numpy(), [4.2806528590890736, 3.9384369822503591,
                                              3.9384369822503591], rtol=1e-7)
    loss.sum().backward()
    # acts are already log-softmax'd: d/dlogits = g - softmax * sum(g) per (t, u) row
    g0 = _G0 - np.exp(acts[0]) * _G0.sum(-1, keepdims=True)
    np.testing.assert_allclose(x.grad.numpy()[0], g0, rtol=1e-5, atol=1e-7)


def test_rnnt_loss_docstring_example_and_layer():
    acts = np.array([[[[0.1, 0.6, 0.1, 0.1, 0.1], [0.1, 0.1, 0.6, 0.1, 0.1],
                       [0.1, 0.1, 0.2, 0.8, 0.1]],
                      [[0.1, 0.6, 0.1, 0.1, 0.1], [0.1, 0.1, 0.2, 0.1, 0.1],
                       [0.7, 0.1, 0.2, 0.1, 0.1]]]])
    args = (paddle.to_tensor(acts), paddle.to_tensor(np.array([[1, 2]], np.int32)),
            paddle.to_tensor(np.array([2], np.int32)), paddle.to_tensor(np.array([2], np.int32)))
    out = F.rnnt_loss(*args, reduction='sum', fastemit_lambda=0.0, blank=0)
    np.testing.assert_allclose(float(out), 4.49566677, rtol=1e-7)
    lay = nn.RNNTLoss(blank=0, fastemit_lambda=0.0, reduction='mean')
    np.testing.assert_allclose(float(lay(*args)), 4.49566677, rtol=1e-7)


def test_rnnt_fastemit_keeps_value_scales_emission_grad():
    rs = np.random.RandomState(0)
    acts = rs.randn(2, 5, 4, 6)
    lab = rs.randint(1, 6, (2, 3)).astype(np.int32)
    args = lambda x: (x, paddle.to_tensor(lab), paddle.to_tensor(np.array([5, 4], np.int32)),  # noqa
                      paddle.to_tensor(np.array([3, 2], np.int32)))
    x0 = paddle.to_tensor(acts, stop_gradient=False)
    x1 = paddle.to_tensor(acts, stop_gradient=False)
    l0 = F.rnnt_loss(*args(x0), fastemit_lambda=0.0)
    l1 = F.rnnt_loss(*args(x1), fastemit_lambda=0.5)
    np.testing.assert_allclose(float(l0), float(l1), rtol=1e-12)
    l0.backward()
    l1.backward()
    assert not np.allclose(x0.grad.numpy(), x1.grad.numpy())


def _hs_loop(x, w, b, label, num_classes, table=None, code=None):
    out = np.zeros((x.shape[0], 1))
    L = (num_classes - 1).bit_length()
    for i in range(x.shape[0]):
        if table is None:
            c = int(label[i]) + num_classes
            path = [((c >> (j + 1)) - 1, (c >> j) & 1) for j in range(c.bit_length() - 1)]
            pad = L - len(path)
        else:
            path = []
            for n, bt in zip(table[i], code[i]):
                if n < 0:
                    break
                path.append((int(n), int(bt)))
            pad = len(table[i]) - len(path)
        s = pad * math.log(2.0)  # padded slots count softplus(0), like the reference kernel
        for n, bt in path:
            pre = float(np.clip(x[i] @ w[n] + (b[n, 0] if b is not None else 0.0), -40, 40))
            s += math.log1p(math.exp(pre)) - bt * pre
        out[i, 0] = s
    return out


def test_hsigmoid_default_and_custom_tree():
    rs = np.random.RandomState(3)
    N, D, C = 7, 5, 6
    x = rs.randn(N, D)
    w = rs.randn(C - 1, D)
    b = rs.randn(C - 1, 1)
    lab = rs.randint(0, C, (N, 1))
    got = F.hsigmoid_loss(paddle.to_tensor(x), paddle.to_tensor(lab), C, paddle.to_tensor(w),
                          paddle.to_tensor(b))
    np.testing.assert_allclose(got.numpy(), _hs_loop(x, w, b, lab[:, 0], C), rtol=1e-10)
    table = np.array([[0, 1, -1], [0, 2, 3], [1, -1, -1], [0, 1, 4], [2, 3, -1], [4, -1, -1],
                      [0, 3, 1]])
    code = rs.randint(0, 2, table.shape)
    got = F.hsigmoid_loss(paddle.to_tensor(x), paddle.to_tensor(lab), C, paddle.to_tensor(w),
                          paddle.to_tensor(b), paddle.to_tensor(table), paddle.to_tensor(code))
    np.testing.assert_allclose(got.numpy(), _hs_loop(x, w, b, None, C, table, code), rtol=1e-10)

    def f(xt, wt, bt):
        return F.hsigmoid_loss(paddle.Tensor(xt), paddle.Tensor(torch.from_numpy(lab)), C,
                               paddle.Tensor(wt), paddle.Tensor(bt))._t
    ins = tuple(torch.from_numpy(a).requires_grad_(True) for a in (x, w, b))
    assert torch.autograd.gradcheck(f, ins)
    layer = nn.HSigmoidLoss(D, C)
    assert layer.weight.shape == [C - 1, D] and layer.bias.shape == [C - 1, 1]
    assert layer(paddle.to_tensor(x.astype('float32')), paddle.to_tensor(lab)).shape == [N, 1]


def _decoder_parts(V=5, H=8):
    paddle.seed(2)
    emb = nn.Embedding(V, H)
    cell = nn.GRUCell(H, H)
    out = nn.Linear(H, V)
    return emb, cell, out


def _greedy(emb, cell, out, h0, start, end, steps):
    h = h0
    tok = paddle.to_tensor(np.full((h0.shape[0],), start, 'int64'))
    ids, done = [], np.zeros(h0.shape[0], bool)
    for _ in range(steps):
        o, h = cell(emb(tok), h)
        nxt = out(o).numpy().argmax(-1)
        nxt = np.where(done, end, nxt)
        ids.append(nxt)
        done |= nxt == end
        tok = paddle.to_tensor(nxt.astype('int64'))
        if done.all():
            break
    return np.stack(ids, 1)


def test_beam_search_beam1_is_greedy():
    emb, cell, out = _decoder_parts()
    h0 = paddle.to_tensor(np.random.RandomState(0).randn(3, 8).astype('float32'))
    dec = nn.BeamSearchDecoder(cell, start_token=0, end_token=1, beam_size=1,
                               embedding_fn=emb, output_fn=out)
    ids, states, lens = nn.dynamic_decode(dec, inits=h0, max_step_num=5, return_length=True)
    assert ids.shape[0] == 3 and ids.shape[2] == 1
    greedy = _greedy(emb, cell, out, h0, 0, 1, ids.shape[1])
    np.testing.assert_array_equal(ids.numpy()[:, :, 0], greedy)


def test_beam_search_wide_beam_is_exhaustive():
    V, T = 4, 3
    emb, cell, out = _decoder_parts(V)
    h0 = paddle.to_tensor(np.random.RandomState(1).randn(2, 8).astype('float32'))
    end = 3
    dec = nn.BeamSearchDecoder(cell, start_token=0, end_token=end, beam_size=V ** (T - 1),
                               embedding_fn=emb, output_fn=out)
    ids, states = nn.dynamic_decode(dec, inits=h0, max_step_num=T - 1)
    assert ids.shape[1] == T
    best_beam = states.log_probs.numpy().argmax(-1)

    def score(b, seq):
        h = paddle.to_tensor(h0.numpy()[b:b + 1])
        tok, s = 0, 0.0
        for t in seq:
            o, h = cell(emb(paddle.to_tensor(np.array([tok], 'int64'))), h)
            lp = torch.log_softmax(out(o)._t.double(), -1)[0]
            s += float(lp[t].detach())
            if t == end:
                break
            tok = t
        return s
    for b in range(2):
        brute = max(itertools.product(range(V), repeat=T), key=lambda seq: score(b, seq))
        got = ids.numpy()[b, :, best_beam[b]]
        # compare up to the first end token (later tokens of a finished beam are padding)
        cut = lambda s: list(s[:list(s).index(end) + 1]) if end in list(s) else list(s)  # noqa
        assert cut(got) == cut(brute), (got, brute)
        np.testing.assert_allclose(states.log_probs.numpy()[b].max(), score(b, brute), rtol=1e-4)
