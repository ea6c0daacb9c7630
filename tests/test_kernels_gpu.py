"""Numerics of every gfx950 HIP kernel vs a PyTorch fp32 reference of the same op."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from paddle_ray_amd.ops import fused as F  # noqa: E402
from paddle_ray_amd.ops import registry as R  # noqa: E402
from paddle_ray_amd.ops import _native  # noqa: E402

DEV = 'cuda'


def test_native_loaded():
    assert _native.available(), _native.load_error()


def _tol(dt):
    return {torch.float32: 2e-5, torch.float16: 2e-3, torch.bfloat16: 2e-2}[dt]


@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize('cols', [2048, 1000, 768, 8192])
def test_layer_norm(dt, cols):
    torch.manual_seed(0)
    x = torch.randn(37, cols, device=DEV, dtype=dt, requires_grad=True)
    w = torch.randn(cols, device=DEV, dtype=dt, requires_grad=True)
    b = torch.randn(cols, device=DEV, dtype=dt, requires_grad=True)
    y = F.layer_norm(x, w, b, 1e-5)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = torch.nn.functional.layer_norm(xr, (cols,), wr, br, 1e-5)
    yr.backward(dy.float())
    tol = _tol(dt)
    assert torch.allclose(y.float(), yr, atol=tol * 4, rtol=tol)
    assert torch.allclose(x.grad.float(), xr.grad, atol=tol * 8, rtol=tol * 4)
    assert torch.allclose(w.grad.float(), wr.grad, atol=tol * 40, rtol=tol * 4)
    assert torch.allclose(b.grad.float(), br.grad, atol=tol * 40, rtol=tol * 4)


@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
def test_rms_norm(dt):
    x = torch.randn(64, 4096, device=DEV, dtype=dt, requires_grad=True)
    w = torch.randn(4096, device=DEV, dtype=dt, requires_grad=True)
    y = F.rms_norm(x, w, 1e-6)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, wr = (t.detach().float().requires_grad_() for t in (x, w))
    yr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6) * wr
    yr.backward(dy.float())
    tol = _tol(dt)
    assert torch.allclose(y.float(), yr, atol=tol * 4, rtol=tol)
    assert torch.allclose(x.grad.float(), xr.grad, atol=tol * 8, rtol=tol * 4)
    assert torch.allclose(w.grad.float(), wr.grad, atol=tol * 40, rtol=tol * 4)


@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('cols', [1024, 50304, 333])
def test_softmax(dt, cols):
    x = torch.randn(19, cols, device=DEV, dtype=dt, requires_grad=True)
    y = F.softmax_lastdim(x)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_()
    yr = torch.softmax(xr, -1)
    yr.backward(dy.float())
    tol = _tol(dt)
    assert torch.allclose(y.float(), yr, atol=tol, rtol=tol)
    assert torch.allclose(x.grad.float(), xr.grad, atol=tol, rtol=tol * 4)


@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('V', [50304, 1001])
def test_softmax_ce(dt, V):
    N = 67
    x = (torch.randn(N, V, device=DEV) * 3).to(dt).requires_grad_()
    lab = torch.randint(0, V, (N,), device=DEV)
    lab[3] = -100
    loss = F.softmax_cross_entropy(x, lab, -100)
    g = torch.rand(N, device=DEV)
    loss.backward(g)
    xr = x.detach().float().requires_grad_()
    lr = torch.nn.functional.cross_entropy(xr, lab, ignore_index=-100, reduction='none')
    lr.backward(g)
    assert torch.allclose(loss, lr, atol=1e-3, rtol=1e-4)
    tol = _tol(dt)
    assert torch.allclose(x.grad.float(), xr.grad, atol=tol * 0.1, rtol=tol * 4)


@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('approx', [True, False])
@pytest.mark.parametrize('rows,cols', [(33, 8192), (1000, 2048)])
def test_bias_gelu(dt, approx, rows, cols):
    x = torch.randn(rows, cols, device=DEV, dtype=dt, requires_grad=True)
    b = torch.randn(cols, device=DEV, dtype=dt, requires_grad=True)
    y = F.bias_gelu(x, b, approx)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, br = (t.detach().float().requires_grad_() for t in (x, b))
    yr = torch.nn.functional.gelu(xr + br, approximate='tanh' if approx else 'none')
    yr.backward(dy.float())
    tol = _tol(dt)
    assert torch.allclose(y.float(), yr, atol=tol, rtol=tol)
    assert torch.allclose(x.grad.float(), xr.grad, atol=tol * 2, rtol=tol * 2)
    assert torch.allclose(b.grad.float(), br.grad, atol=tol * 40 * max(1, rows // 100),
                          rtol=tol * 4)


def _attn_ref(q, k, v, causal, scale):
    qf, kf, vf = (t.float().permute(0, 2, 1, 3) for t in (q, k, v))
    s = qf @ kf.transpose(-1, -2) * scale
    if causal:
        Sq, Sk = s.shape[-2:]
        m = torch.ones(Sq, Sk, dtype=torch.bool, device=s.device).triu(Sk - Sq + 1)
        s = s.masked_fill(m, float('-inf'))
    return (torch.softmax(s, -1) @ vf).permute(0, 2, 1, 3)


@pytest.mark.parametrize('dt', [torch.bfloat16, torch.float16])
@pytest.mark.parametrize('D', [64, 128])
@pytest.mark.parametrize('causal', [True, False])
@pytest.mark.parametrize('S', [256, 200])
def test_flash_attention(dt, D, causal, S):
    torch.manual_seed(1)
    B, H = 2, 3
    qkv = torch.randn(B, S, 3, H, D, device=DEV, dtype=dt)
    q, k, v = qkv.unbind(2)  # strided views, like the GPT fused projection
    q, k, v = (t.detach().requires_grad_() for t in (q, k, v))
    scale = 1.0 / math.sqrt(D)
    o = F.flash_attention(q, k, v, causal=causal, scale=scale)
    do = torch.randn_like(o)
    o.backward(do)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf = _attn_ref(qr, kr, vr, causal, scale)
    orf.backward(do.float())
    tol = 2e-2 if dt == torch.bfloat16 else 4e-3
    assert (o.float() - orf).abs().max().item() < tol * 2, (o.float() - orf).abs().max()
    for g, gr in ((q.grad, qr.grad), (k.grad, kr.grad), (v.grad, vr.grad)):
        err = (g.float() - gr).abs().max().item()
        assert err < tol * 4 * max(1.0, gr.abs().max().item()), err


@pytest.mark.parametrize('causal', [True, False])
@pytest.mark.parametrize('Sq,Sk', [(130, 300), (300, 130), (64, 1024), (520, 520)])
def test_flash_attention_cross_lengths(causal, Sq, Sk):
    """Sq != Sk (bottom-right aligned causal mask) and lengths around the 64-row tiles: the
    masked/unmasked tile split of every kernel must agree with the reference."""
    torch.manual_seed(2)
    B, H, D = 2, 2, 128
    q = torch.randn(B, Sq, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, Sk, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, Sk, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    scale = 1.0 / math.sqrt(D)
    o = F.flash_attention(q, k, v, causal=causal, scale=scale)
    do = torch.randn_like(o)
    o.backward(do)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    # reference with rows that see no key (causal, Sq > Sk) defined as zero output / zero grad
    qf, kf, vf = (t.permute(0, 2, 1, 3) for t in (qr, kr, vr))
    sc = qf @ kf.transpose(-1, -2) * scale
    if causal:
        m = torch.ones(Sq, Sk, dtype=torch.bool, device=DEV).triu(Sk - Sq + 1)
        sc = sc.masked_fill(m, float('-inf'))
    dead = torch.isinf(sc).all(-1, keepdim=True)
    pr = torch.softmax(sc.masked_fill(dead, 0.0), -1) * (~dead)
    orf = (pr @ vf).permute(0, 2, 1, 3)
    orf.backward(do.float())
    assert (o.float() - orf).abs().max().item() < 4e-2
    for g, gr in ((q.grad, qr.grad), (k.grad, kr.grad), (v.grad, vr.grad)):
        err = (g.float() - gr).abs().max().item()
        assert err < 8e-2 * max(1.0, gr.abs().max().item()), err


def test_flash_attention_spike_rows():
    """A spiked key forces the online-softmax rescale path (CDNA guide rule 26)."""
    B, S, H, D = 1, 256, 2, 128
    q = torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16)
    k[:, 200] *= 30
    o = F.flash_attention(q, k, v, causal=True)
    ref = _attn_ref(q, k, v, True, 1 / math.sqrt(D))
    assert (o.float() - ref).abs().max().item() < 5e-2


@pytest.mark.parametrize('master', [True, False])
def test_adamw_multi_tensor(master):
    torch.manual_seed(0)
    shapes = [(1000,), (70000,), (3, 5)]
    pdt = torch.bfloat16 if master else torch.float32
    ps = [torch.randn(s, device=DEV).to(pdt) for s in shapes]
    gs = [torch.randn(s, device=DEV).to(pdt) for s in shapes]
    ms = [torch.zeros(s, device=DEV) for s in shapes]
    vs = [torch.zeros(s, device=DEV) for s in shapes]
    mas = [p.float().clone() for p in ps] if master else [None] * 3
    wds, lrm = [0.1, 0.0, 0.01], [1.0, 0.5, 1.0]
    ref_p = [p.clone() for p in ps]
    ref_m = [m.clone() for m in ms]
    ref_v = [v.clone() for v in vs]
    ref_ma = [m.clone() for m in mas] if master else [None] * 3
    mt = F.MultiTensorAdamW(ps, lambda: gs, ms, vs, mas, wds, lrm)
    for step in (1, 2, 3):
        mt.step(1e-2, 0.9, 0.999, 1e-8, step, grad_scale=0.5)
        F.adamw_ref(ref_p, gs, ref_m, ref_v, ref_ma, 1e-2, 0.9, 0.999, 1e-8, wds, lrm, step, 0.5)
    torch.cuda.synchronize()
    for a, b in zip(ps, ref_p):
        assert torch.allclose(a.float(), b.float(), atol=1e-2 if master else 1e-5)
    for a, b in zip(ms, ref_m):
        assert torch.allclose(a, b, atol=1e-5)
    if master:
        for a, b in zip(mas, ref_ma):
            assert torch.allclose(a, b, atol=1e-5)


def test_sumsq():
    ts = [torch.randn(1000, device=DEV), torch.randn(77, 3, device=DEV).bfloat16()]
    got = F.global_l2_norm_sq(ts)
    ref = sum((t.float() ** 2).sum() for t in ts)
    assert torch.allclose(got, ref, rtol=1e-4)


def test_registry_uses_hip():
    R.reset_stats()
    x = torch.randn(4, 64, device=DEV)
    F.layer_norm(x, None, None, 1e-5)
    assert R.stats().get(('layer_norm_fwd', 'hip'), 0) == 1


@pytest.mark.parametrize('p', [0.0, 0.1])
@pytest.mark.parametrize('cols', [2048, 1024, 776])
def test_add_dropout_layer_norm(p, cols):
    torch.manual_seed(0)
    dt = torch.bfloat16
    x = torch.randn(67, cols, device=DEV, dtype=dt, requires_grad=True)
    h = torch.randn(67, cols, device=DEV, dtype=dt, requires_grad=True)
    hb = torch.randn(cols, device=DEV, dtype=dt, requires_grad=True)
    w = torch.randn(cols, device=DEV, dtype=dt, requires_grad=True)
    b = torch.randn(cols, device=DEV, dtype=dt, requires_grad=True)
    torch.manual_seed(5)
    r, y = F.add_dropout_layer_norm(x, h, hb, w, b, p, 1e-5)
    gr, gy = torch.randn_like(r), torch.randn_like(y)
    (r.float() * gr.float()).sum().add((y.float() * gy.float()).sum()).backward()
    # reference with the SAME counter-hash mask
    torch.manual_seed(5)
    seed = F._dropout_seed() if p > 0 else 0
    xr, hr, hbr, wr, br = (t.detach().float().requires_grad_() for t in (x, h, hb, w, b))
    t = hr + hbr
    if p > 0:
        keep = F._hash_keep_ref(t.numel(), p, seed, DEV).view(t.shape)
        t = torch.where(keep, t / (1 - p), torch.zeros_like(t))
    rr = xr + t
    yr = torch.nn.functional.layer_norm(rr, (cols,), wr, br, 1e-5)
    (rr * gr.float()).sum().add((yr * gy.float()).sum()).backward()
    assert torch.allclose(r.float(), rr, atol=5e-2, rtol=2e-2)
    assert torch.allclose(y.float(), yr, atol=1e-1, rtol=5e-2)
    for a, bb, tol in ((x.grad, xr.grad, 0.15), (h.grad, hr.grad, 0.15), (w.grad, wr.grad, 2.0),
                       (b.grad, br.grad, 2.0), (hb.grad, hbr.grad, 2.0)):
        assert (a.float() - bb).abs().max().item() < tol * max(1, bb.abs().max().item() * 0.05), \
            (a.float() - bb).abs().max()


def test_dropout_rate():
    x = torch.zeros(256, 2048, device=DEV, dtype=torch.bfloat16)
    h = torch.ones(256, 2048, device=DEV, dtype=torch.bfloat16)
    r, _ = F.add_dropout_layer_norm(x, h, None, None, None, 0.1, 1e-5)
    frac = (r == 0).float().mean().item()
    assert abs(frac - 0.1) < 0.005, frac


@pytest.mark.parametrize('D', [64, 128])
def test_flash_attention_qkvpacked(D):
    torch.manual_seed(3)
    B, S, H = 2, 192, 4
    qkv = torch.randn(B, S, 3, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = F.flash_attention_qkvpacked(qkv, causal=True)
    do = torch.randn_like(o)
    o.backward(do)
    ref = qkv.detach().float().requires_grad_()
    q, k, v = ref.unbind(2)
    orf = _attn_ref(q, k, v, True, 1 / math.sqrt(D))
    orf.backward(do.float())
    assert (o.float() - orf).abs().max().item() < 4e-2
    err = (qkv.grad.float() - ref.grad).abs().max().item()
    assert err < 8e-2 * max(1.0, ref.grad.abs().max().item()), err


def _bn_ref(x, z, w, b, relu, eps):
    xf = x.float()
    mean = xf.mean(0)
    var = xf.var(0, unbiased=False)
    y = (xf - mean) * torch.rsqrt(var + eps) * w + b
    if z is not None:
        y = y + z.float()
    return torch.relu(y) if relu else y, mean, var


@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('M,C', [(4096, 64), (3 * 7 * 7, 2048), (1000, 256), (50, 24)])
@pytest.mark.parametrize('relu,res', [(False, False), (True, False), (True, True)])
def test_batch_norm_act(dt, M, C, relu, res):
    torch.manual_seed(0)
    x = (torch.randn(M, C, device=DEV) * 2 + 3).to(dt).requires_grad_()
    z = torch.randn(M, C, device=DEV, dtype=dt, requires_grad=True) if res else None
    w = torch.rand(C, device=DEV, requires_grad=True)
    b = torch.randn(C, device=DEV, requires_grad=True)
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    R.reset_stats()
    y = F.batch_norm_act(x, z, w, b, rm, rv, True, 0.9, 1e-5, relu)
    if C % 8 == 0:
        assert R.stats().get(('batch_norm_fwd', 'hip'), 0) == 1
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_()
    zr = z.detach().float().requires_grad_() if res else None
    wr, br = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    yr, mean, var = _bn_ref(xr, zr, wr, br, relu, 1e-5)
    yr.backward(dy.float())
    tol = _tol(dt)
    assert torch.allclose(y.float(), yr, atol=tol * 4, rtol=tol)
    assert torch.allclose(rm, 0.1 * mean, atol=1e-4, rtol=1e-4)
    assert torch.allclose(rv, 0.9 + 0.1 * var * M / (M - 1), atol=1e-4, rtol=1e-4)
    assert torch.allclose(x.grad.float(), xr.grad, atol=tol * 8, rtol=tol * 4)
    assert torch.allclose(w.grad, wr.grad, atol=tol * 40 * math.sqrt(M) / 8, rtol=tol * 4)
    assert torch.allclose(b.grad, br.grad, atol=tol * 40 * math.sqrt(M) / 8, rtol=tol * 4)
    if res:
        assert torch.allclose(z.grad.float(), zr.grad, atol=tol * 4, rtol=tol)


def test_batch_norm_infer():
    C = 128
    x = torch.randn(300, C, device=DEV, dtype=torch.bfloat16)
    w, b = torch.rand(C, device=DEV), torch.randn(C, device=DEV)
    rm, rv = torch.randn(C, device=DEV), torch.rand(C, device=DEV) + 0.5
    y = F.batch_norm_act(x, None, w, b, rm, rv, False, 0.9, 1e-5, True)
    yr = torch.relu((x.float() - rm) * torch.rsqrt(rv + 1e-5) * w + b)
    assert torch.allclose(y.float(), yr, atol=0.05, rtol=0.02)


def test_resnet_block_uses_fused_bn():
    import paddle_ray_amd as paddle
    from paddle_ray_amd.vision.models import resnet50
    paddle.set_device('gpu:0')
    m = resnet50(data_format='NHWC', num_classes=10)
    m = paddle.amp.decorate(m, level='O2', dtype='bfloat16')
    x = paddle.Tensor(torch.randn(4, 64, 64, 3, device=DEV, dtype=torch.bfloat16))
    R.reset_stats()
    out = m(x)
    out.sum().backward()
    st = R.stats()
    # (backward: the reduce-in-the-conv-dgrad path counts as 'hip_parts', ops/fused.py _BnHandoff)
    nb = st.get(('batch_norm_bwd', 'hip'), 0) + st.get(('batch_norm_bwd', 'hip_parts'), 0)
    assert st.get(('batch_norm_fwd', 'hip'), 0) == 53 and nb == 53, st
    assert st.get(('batch_norm_bwd', 'hip_parts'), 0) > 0, st


@pytest.mark.parametrize('stride', [1, 2])
def test_conv1x1_gemm_path(stride, monkeypatch):
    import paddle_ray_amd as paddle
    import paddle_ray_amd.nn.functional as PF
    monkeypatch.setattr(PF, '_CONV1X1_GEMM', True)
    x = torch.randn(4, 14, 14, 64, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = torch.randn(128, 64, 1, 1, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = PF.conv2d(paddle.Tensor(x), paddle.Tensor(w), stride=stride, data_format='NHWC')._t
    yr = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.float(), stride=stride)
    yr = yr.permute(0, 2, 3, 1)
    assert y.shape == yr.shape
    assert torch.allclose(y.float(), yr, atol=0.1, rtol=0.02)
    dy = torch.randn_like(y)
    gx, gw = torch.autograd.grad(y, [x, w], dy)
    gxr, gwr = torch.autograd.grad(yr, [x, w], dy.float())
    assert torch.allclose(gx.float(), gxr.float(), atol=0.1, rtol=0.02)
    assert torch.allclose(gw.float(), gwr.float(), atol=0.5, rtol=0.02)


@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('D', [2048, 64, 1000])
def test_embedding_fwd_bwd(dt, D):
    torch.manual_seed(0)
    V = 300
    ids = torch.randint(0, V, (6, 50), device=DEV)
    ids[0, :10] = 7          # a long run of one id
    ids[1, 0] = 5            # padding row
    w = torch.randn(V, D, device=DEV, dtype=dt, requires_grad=True)
    R.reset_stats()
    out = F.embedding(ids, w, 5)
    if D % 8 == 0:
        assert R.stats().get(('embedding_fwd', 'hip'), 0) == 1
    keep = (ids != 5).unsqueeze(-1)
    ref = torch.nn.functional.embedding(ids, w.detach().float()) * keep
    assert torch.equal(out.float(), ref)
    dy = torch.randn_like(out)
    out.backward(dy)
    gref = torch.zeros(V, D, device=DEV)
    gref.index_add_(0, ids.reshape(-1), (dy.float() * keep).reshape(-1, D))
    tol = _tol(dt) * 10
    assert torch.allclose(w.grad.float(), gref, atol=tol, rtol=tol)
    # second backward accumulates into the existing grad in place
    out2 = F.embedding(ids, w, 5)
    with torch.no_grad():
        g0 = w.grad.clone()
    out2.backward(dy)
    assert torch.allclose(w.grad.float(), g0.float() + gref, atol=2 * tol, rtol=tol)


@pytest.mark.parametrize('dt', [torch.float32, torch.bfloat16])
def test_embedding_bwd_long_runs_segmented(dt):
    """Runs much longer than a 32-row segment (token types, positions: one id over the whole
    batch) are split over many waves and recombined; runs crossing block boundaries, runs that
    start mid-block and the padding id all meet the index_add reference."""
    torch.manual_seed(1)
    V, D = 40, 768
    ids = torch.cat([torch.zeros(5000, dtype=torch.long), torch.full((33,), 3), torch.full((1,), 4),
                     torch.randint(0, V, (700,)), torch.full((64,), 9), torch.full((95,), 5)]).to(DEV)
    ids = ids[torch.randperm(ids.numel(), device=DEV)].view(71, 83)
    w = torch.randn(V, D, device=DEV, dtype=dt, requires_grad=True)
    out = F.embedding(ids, w, 5)
    dy = torch.randn_like(out)
    out.backward(dy)
    keep = (ids != 5).unsqueeze(-1)
    gref = torch.zeros(V, D, device=DEV)
    gref.index_add_(0, ids.reshape(-1), (dy.float() * keep).reshape(-1, D))
    tol = _tol(dt) * 10
    assert torch.allclose(w.grad.float(), gref, atol=tol * 8, rtol=tol)


def test_embedding_out_of_range_reads_zero():
    w = torch.randn(10, 16, device=DEV)
    ids = torch.tensor([[0, 9, 10, -1, 1000]], device=DEV)
    out = F.embedding(ids, w, None)
    assert torch.equal(out[0, 2:], torch.zeros(3, 16, device=DEV))
    assert torch.equal(out[0, :2], w[[0, 9]])


def test_memory_efficient_attention_block_diagonal_gpu():
    """Packed variable-length sequences run ONE varlen HIP flash launch (causal and not)."""
    import paddle_ray_amd as paddle
    from paddle_ray_amd.incubate.nn import attn_bias as AB, memory_efficient_attention
    torch.manual_seed(0)
    lens = [64, 128, 40]
    q, k, v = (torch.randn(1, sum(lens), 4, 128, device=DEV, dtype=torch.bfloat16)
               for _ in range(3))
    for bias in (AB.BlockDiagonalMask.from_seqlens(lens),
                 AB.BlockDiagonalMask.from_seqlens(lens).make_causal()):
        R.reset_stats()
        out = memory_efficient_attention(paddle.Tensor(q), paddle.Tensor(k), paddle.Tensor(v),
                                         bias)._t
        assert R.stats().get(('flash_attn_varlen', 'hip'), 0) == 1
        dense = bias.materialize([1, 4, sum(lens), sum(lens)])._t.to(DEV)
        s = torch.einsum('bmhk,bnhk->bhmn', q.float(), k.float()) / math.sqrt(128) + dense
        ref = torch.einsum('bhmn,bnhk->bmhk', torch.softmax(s, -1), v.float())
        assert (out.float() - ref).abs().max().item() < 2e-2


@pytest.mark.parametrize('causal', [True, False])
@pytest.mark.parametrize('Sq,Sk,D', [(1024, 1024, 128), (300, 130, 128), (130, 300, 64), (520, 520, 64)])
def test_flash_attention_dq_paths_agree(causal, Sq, Sk, D, monkeypatch):
    """dQ from the stored dS^T (default) vs the recomputing dQ sweep: both against an fp32
    reference and against each other. dV must be identical between the paths (dK differs by
    the delta = rowsum(dO*O) summation order: preprocess kernel vs inside the dQ sweep)."""
    from paddle_ray_amd.ops import fused as K
    torch.manual_seed(5)
    B, H = 2, 4
    q = torch.randn(B, Sq, H, D, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(B, Sk, H, D, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(B, Sk, H, D, device=DEV, dtype=torch.bfloat16)
    scale = 1.0 / math.sqrt(D)
    o, lse = K._fa_fwd_hip(q, k, v, causal, scale)
    do = torch.randn_like(o)
    grads = {}
    for path in ('ds', 'sweep'):
        monkeypatch.setattr(K, '_FA_DQ', path)
        grads[path] = K._fa_bwd_hip(do, q, k, v, o, lse, causal, scale)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    qf, kf, vf = (t.permute(0, 2, 1, 3) for t in (qr, kr, vr))
    sc = qf @ kf.transpose(-1, -2) * scale
    if causal:
        m = torch.ones(Sq, Sk, dtype=torch.bool, device=DEV).triu(Sk - Sq + 1)
        sc = sc.masked_fill(m, float('-inf'))
    dead = torch.isinf(sc).all(-1, keepdim=True)
    pr = torch.softmax(sc.masked_fill(dead, 0.0), -1) * (~dead)
    (pr @ vf).permute(0, 2, 1, 3).backward(do.float())
    for path, (dq, dk, dv) in grads.items():
        for name, g, gr in (('dq', dq, qr.grad), ('dk', dk, kr.grad), ('dv', dv, vr.grad)):
            err = (g.float() - gr).abs().max().item()
            assert err < 8e-2 * max(1.0, gr.abs().max().item()), (path, name, err)
    a, b = grads['ds'], grads['sweep']
    torch.testing.assert_close(a[2], b[2], atol=0, rtol=0)
    torch.testing.assert_close(a[1].float(), b[1].float(), atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(a[0].float(), b[0].float(), atol=2e-2, rtol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize('case', ['frozen_w', 'nonleaf_w'])
def test_linear_grads_frozen_or_nonleaf_weight(case):
    """A frozen weight with a trainable input, and a non-leaf (computed) weight, still get
    correct gradients through the fused linear / linear_nt paths."""
    from paddle_ray_amd.ops import fused as K
    torch.manual_seed(11)
    x = torch.randn(64, 128, device='cuda', dtype=torch.bfloat16, requires_grad=True)
    w0 = torch.randn(128, 256, device='cuda', dtype=torch.bfloat16, requires_grad=(case == 'nonleaf_w'))
    w = w0 * 2 if case == 'nonleaf_w' else w0
    gy = torch.randn(64, 256, device='cuda', dtype=torch.bfloat16)
    K.linear(x, w).backward(gy)
    xf = x.detach().float().requires_grad_(True)
    wf = w0.detach().float().requires_grad_(True)
    (xf @ (wf * 2 if case == 'nonleaf_w' else wf)).backward(gy.float())
    torch.testing.assert_close(x.grad.float(), xf.grad, atol=0.5, rtol=3e-2)
    if case == 'nonleaf_w':
        torch.testing.assert_close(w0.grad.float(), wf.grad, atol=1.0, rtol=3e-2)
    x.grad = None
    e = torch.randn(256, 128, device='cuda', dtype=torch.bfloat16)   # frozen tied embedding
    K.linear_nt(x, e).backward(gy)
    torch.testing.assert_close(x.grad.float(), gy.float() @ e.float(), atol=0.5, rtol=3e-2)


@pytest.mark.gpu
@pytest.mark.parametrize('ty', [False, True])
def test_paddle_matmul_device_gemm(ty):
    """paddle.matmul with a 2-D right operand in bf16 runs the framework GEMM (registry 'gemm'
    dispatches) with correct values and gradients, transpose_y included."""
    import paddle_ray_amd as paddle
    torch.manual_seed(12)
    a = torch.randn(4, 64, 128, device='cuda', dtype=torch.bfloat16, requires_grad=True)
    b = torch.randn(256, 128, device='cuda', dtype=torch.bfloat16) if ty else \
        torch.randn(128, 256, device='cuda', dtype=torch.bfloat16)
    b.requires_grad_(True)
    R.reset_stats()
    y = paddle.matmul(paddle.Tensor(a), paddle.Tensor(b), transpose_y=ty)._t
    assert sum(v for (op, _), v in R.stats().items() if op == 'gemm') >= 1
    gy = torch.randn_like(y)
    y.backward(gy)
    af, bf = a.detach().float().requires_grad_(True), b.detach().float().requires_grad_(True)
    yf = af @ (bf.t() if ty else bf)
    yf.backward(gy.float())
    torch.testing.assert_close(y.float(), yf, atol=0.5, rtol=3e-2)
    torch.testing.assert_close(a.grad.float(), af.grad, atol=0.5, rtol=3e-2)
    torch.testing.assert_close(b.grad.float(), bf.grad, atol=1.0, rtol=3e-2)


@pytest.mark.parametrize('path', ['plain', 'ext'])
@pytest.mark.parametrize('S,D', [(384, 64), (256, 128)])
def test_qkv_bias_grad_from_flash_partials(path, S, D):
    """The QKV projection's bias gradient taken from the flash backward's column-sum partials
    equals the column sum of the packed dQKV it wrote (fp32 sum of the rounded values), also for
    a sequence that leaves the last dQ block half empty (S = 384)."""
    torch.manual_seed(11)
    B, H = 2, 4
    HD = H * D
    x = (torch.randn(B, S, HD, device='cuda') * 0.5).to(torch.bfloat16).requires_grad_(True)
    w = (torch.randn(HD, 3 * HD, device='cuda') * 0.05).to(torch.bfloat16).requires_grad_(True)
    b = torch.zeros(3 * HD, device='cuda', dtype=torch.bfloat16, requires_grad=True)
    seen = {}
    qkv = F.linear(x, w, b)
    def keep(g):
        seen['g'] = g.detach().float().clone()
    qkv.register_hook(keep)
    q5 = qkv.view(B, S, 3, H, D)
    if path == 'plain':
        o = F.flash_attention_qkvpacked(q5, causal=True)
    else:
        mask = torch.zeros(B, 1, 1, S, device='cuda', dtype=torch.bfloat16)
        mask[1, ..., S - 40:] = float('-inf')
        o = F.flash_attention_ext_qkvpacked(q5, attn_mask=mask, dropout=0.1)
    o.float().square().sum().backward()
    ref = seen['g'].reshape(-1, 3 * HD).sum(0)
    err = (b.grad.float() - ref).abs().max().item()
    assert err <= 2e-2 * max(ref.abs().max().item(), 1e-3), (err, ref.abs().max().item())
    # the partials path was taken (the tagged gradient reached bias_grad)
    F._FA_BIAS_PART = False
    try:
        b2 = b.detach().clone().requires_grad_(True)
        qkv2 = F.linear(x.detach(), w.detach(), b2)
        q52 = qkv2.view(B, S, 3, H, D)
        if path == 'plain':
            o2 = F.flash_attention_qkvpacked(q52, causal=True)
            o2.float().square().sum().backward()
            err2 = (b2.grad.float() - b.grad.float()).abs().max().item()
            assert err2 <= 1e-2 * max(ref.abs().max().item(), 1e-3), err2
    finally:
        F._FA_BIAS_PART = True
