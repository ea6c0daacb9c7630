"""BatchNorm+ReLU backward reductions taken in the epilogue of the consumer convolution's dgrad
(ops.fused._BnHandoff, gemm_core.h kBnG): the conv dgrad writes the ReLU-masked gradient g and the
per-tile sums of g and g * (x - mean); the BN backward runs finalize + apply only. Parity: the
reference's fused_bn_activation / batch_norm_grad kernels (fluid/operators/fused/
fused_bn_activation_op.cu) compute the same dx, dscale, dbias from a separate reduction.

Checked against the unfused in-tree path on the same bf16 data and against fp32 autograd."""
import pytest
import torch

from paddle_ray_amd.ops import fused as K


def test_handoff_take_requires_same_unmodified_buffer():
    x2 = torch.zeros(16, 8)
    rec = K._BnHandoff(x2, torch.zeros(16, dtype=torch.uint8), torch.zeros(8))
    g = torch.randn(16, 8)
    part = torch.zeros(2, 1, 8)
    rec.g, rec.part, rec.gver = g, part, g._version
    assert rec.take(g) is part and rec.used == 1
    rec.g, rec.part, rec.gver = g, part, g._version
    assert rec.take(g.clone()) is None            # a different buffer (autograd summed a 2nd grad)
    rec.g, rec.part, rec.gver = g, part, g._version
    g.add_(1.0)                                   # accumulated in place: version moved
    assert rec.take(g) is None
    assert rec.part is None and rec.g is None     # always cleared


def _chain(x, s, b, w, kind, extra_use):
    rm, rv = torch.zeros(x.shape[-1], device=x.device), torch.ones(x.shape[-1], device=x.device)
    a = K.batch_norm_act(x, None, s, b, rm, rv, True, 0.9, 1e-5, True)
    if kind == '3x3':
        y = K.conv_kxk_nhwc(a, w, None, 1, 1)
    elif kind == '3x3s2':   # strided dgrad: four sub-pixel phase convs, each with the kBnG epilogue
        y = K.conv_kxk_nhwc(a, w, None, 2, 1)
    elif kind == '3x3_stats':
        co = w.shape[0]
        assert K.conv_bn_stats_ok(a, w, 1, 1, torch.zeros(co, device=x.device), True)
        y = K.conv_bn_act_nhwc(a, w, 1, 1, torch.ones(co, device=x.device), torch.zeros(co, device=x.device),
                               torch.zeros(co, device=x.device), torch.ones(co, device=x.device), True, 0.9,
                               1e-5, None, True)
    else:
        y = K.conv1x1_nhwc(a, w)
    if extra_use:
        y = y.float().sum() + (a.float() * 0.5).sum()
    return a, y


CASES = [('3x3', 64, 64), ('3x3', 128, 128), ('3x3', 256, 64), ('3x3_stats', 64, 128),
         ('3x3s2', 64, 64), ('3x3s2', 128, 256),
         ('1x1', 64, 256), ('1x1', 128, 512), ('1x1', 256, 256)]


@pytest.mark.gpu
@pytest.mark.parametrize('case', CASES)
@pytest.mark.parametrize('extra_use', [False, True])
def test_bn_dgrad_fused_matches(case, extra_use, monkeypatch):
    kind, c, cout = case
    monkeypatch.setattr(K, '_BN_DGRAD_SPLIT', True)   # cover the W8 (C > 128) tile too
    monkeypatch.setattr(K, '_STRIDED_DGRAD', True)    # (off by default: MIOpen measured faster)
    torch.manual_seed(0)
    dev = 'cuda'
    n, hw = 4, 12
    x = (torch.randn(n, hw, hw, c, device=dev) * 1.5 + 0.3).bfloat16()
    kk = 3 if kind.startswith('3x3') else 1
    w = (torch.randn(cout, c, kk, kk, device=dev) * (2.0 / (kk * kk * c)) ** 0.5).bfloat16()
    s = torch.rand(c, device=dev) + 0.5
    b = torch.randn(c, device=dev) * 0.1
    st = 2 if kind == '3x3s2' else 1
    g = torch.randn(n, hw // st, hw // st, cout, device=dev).bfloat16()

    def run(fuse):
        monkeypatch.setattr(K, '_BN_DGRAD_FUSE', fuse)
        xs, ws = x.clone().requires_grad_(), w.clone().requires_grad_()
        ss, bs = s.clone().requires_grad_(), b.clone().requires_grad_()
        a, y = _chain(xs, ss, bs, ws, kind, extra_use)
        if extra_use:
            y.backward()
        else:
            y.backward(g)
        rec = getattr(a, '_pra_bn', None)
        return xs.grad, ws.grad, ss.grad, bs.grad, (rec.used if rec is not None else None)

    fused = run(True)
    plain = run(False)
    torch.cuda.synchronize()
    # the handoff engaged exactly when the conv is the BN output's only consumer
    assert fused[4] == (0 if extra_use else 1), fused[4]
    assert plain[4] is None
    for got, want in zip(fused[:4], plain[:4]):
        err = (got.float() - want.float()).abs().max().item() / (want.float().abs().max().item() + 1e-6)
        assert err < 0.02, err
    if kind == '3x3_stats':
        return   # (a second BN follows the conv there: the unfused in-tree path is the reference)
    # fp32 autograd reference of the same chain
    xf, wf = x.float().requires_grad_(), w.float().requires_grad_()
    sf, bf = s.clone().requires_grad_(), b.clone().requires_grad_()
    xn = xf.permute(0, 3, 1, 2)
    a = torch.relu(torch.nn.functional.batch_norm(xn, None, None, sf, bf, True, 0.1, 1e-5))
    y = torch.nn.functional.conv2d(a, wf, None, st, kk // 2).permute(0, 2, 3, 1)
    if extra_use:
        (y.sum() + (a * 0.5).sum()).backward()
    else:
        y.backward(g.float())
    for got, want in zip(fused[:4], (xf.grad, wf.grad, sf.grad, bf.grad)):
        err = (got.float() - want).abs().max().item() / (want.abs().max().item() + 1e-6)
        assert err < 0.05, err
