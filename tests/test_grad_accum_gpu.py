"""Parameter gradients accumulated inside the kernels (BN finalize, conv1x1 wgrad beta=1
epilogue) match autograd's own accumulation over two backward passes, and the
post-accumulate hooks still fire."""
import pytest
import torch

from paddle_ray_amd.ops import fused as K


@pytest.mark.gpu
def test_bn_grad_accumulates_in_kernel():
    torch.manual_seed(0)
    M, C = 4096, 64
    x = torch.randn(M, C, device='cuda', dtype=torch.bfloat16)
    w = torch.randn(C, device='cuda', requires_grad=True)
    b = torch.randn(C, device='cuda', requires_grad=True)
    fired = []
    w.register_post_accumulate_grad_hook(lambda t: fired.append('w'))
    rm, rv = torch.zeros(C, device='cuda'), torch.ones(C, device='cuda')
    dys = [torch.randn(M, C, device='cuda', dtype=torch.bfloat16) for _ in range(2)]
    for dy in dys:
        K.batch_norm_act(x, None, w, b, rm, rv, True, relu=True).backward(dy)
    assert fired == ['w', 'w']
    wr, br = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    for dy in dys:
        xf = x.float()
        y = torch.relu((xf - xf.mean(0)) / torch.sqrt(xf.var(0, unbiased=False) + 1e-5) * wr + br)
        y.backward(dy.float())
    torch.testing.assert_close(w.grad, wr.grad, rtol=2e-2, atol=2e-1)
    torch.testing.assert_close(b.grad, br.grad, rtol=2e-2, atol=2e-1)


@pytest.mark.gpu
def test_conv1x1_wgrad_accumulates_in_kernel():
    torch.manual_seed(0)
    x = torch.randn(4, 16, 16, 64, device='cuda', dtype=torch.bfloat16)
    w = (torch.randn(128, 64, 1, 1, device='cuda') * 0.1).to(torch.bfloat16).requires_grad_()
    fired = []
    w.register_post_accumulate_grad_hook(lambda t: fired.append(1))
    dys = [torch.randn(4, 16, 16, 128, device='cuda', dtype=torch.bfloat16) for _ in range(2)]
    for dy in dys:
        K.conv1x1_nhwc(x, w).backward(dy)
    assert len(fired) == 2
    ref = sum(torch.einsum('nhwo,nhwi->oi', dy.float(), x.float()) for dy in dys)
    err = (w.grad.float().view(128, 64) - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item() + 0.5, err


@pytest.mark.gpu
@pytest.mark.parametrize("stride,down", [(1, False), (2, True), (1, True)])
def test_bottleneck_grad_join_matches_autograd_sum(stride, down, monkeypatch):
    """Block-input gradient joined in-kernel (GradJoin) == autograd's own sum of branches."""
    import contextlib
    import paddle_ray_amd as paddle
    from paddle_ray_amd.vision.models import resnet as R
    paddle.seed(0)
    inpl, planes = (64, 16) if not down else (64, 32)
    ds = None
    if down:
        ds = paddle.nn.Sequential(
            paddle.nn.Conv2D(inpl, planes * 4, 1, stride=stride, bias_attr=False, data_format='NHWC'),
            paddle.nn.BatchNorm2D(planes * 4, data_format='NHWC'))
    blk = R.BottleneckBlock(inpl, planes, stride=stride, downsample=ds, data_format='NHWC')
    blk = paddle.amp.decorate(blk, level='O2', dtype='bfloat16')
    x0 = torch.randn(4, 16, 16, inpl, device='cuda', dtype=torch.bfloat16)
    # both runs start from the same BN running statistics (the conv-epilogue statistics are
    # shifted by the running mean, so a changed shift would change bf16 rounding, not the join)
    bufs0 = [b._t.clone() for b in blk.buffers()]
    outs = []
    for joined in (True, False):
        for b, b0 in zip(blk.buffers(), bufs0):
            b._t.copy_(b0)
        if not joined:
            monkeypatch.setattr(R, '_grad_join', lambda t: contextlib.nullcontext())
        for p in blk.parameters():
            p._t.grad = None
        x = paddle.Tensor(x0.clone().requires_grad_())
        y = blk(x)
        g = torch.randn(y.shape, device='cuda', generator=torch.Generator('cuda').manual_seed(1)).to(y._t.dtype)
        y._t.backward(g)
        outs.append((x._t.grad.float().clone(), [p._t.grad.float().clone() for p in blk.parameters()]))
    (gx1, gp1), (gx2, gp2) = outs
    torch.testing.assert_close(gx1, gx2, rtol=2e-2, atol=2e-2)
    for a, b in zip(gp1, gp2):
        torch.testing.assert_close(a, b, rtol=5e-2, atol=5e-2)


@pytest.mark.gpu
def test_add_dropout_ln_param_grads_accumulate_in_kernel():
    torch.manual_seed(0)
    R_, C = 512, 1024
    x = torch.randn(R_, C, device='cuda', dtype=torch.bfloat16)
    h = torch.randn(R_, C, device='cuda', dtype=torch.bfloat16)
    hb = torch.randn(C, device='cuda', dtype=torch.bfloat16, requires_grad=True)
    w = torch.randn(C, device='cuda', dtype=torch.bfloat16, requires_grad=True)
    b = torch.randn(C, device='cuda', dtype=torch.bfloat16, requires_grad=True)
    fired = []
    for t in (hb, w, b):
        t.register_post_accumulate_grad_hook(lambda t: fired.append(1))
    gs = [torch.randn(R_, C, device='cuda', dtype=torch.bfloat16) for _ in range(2)]
    for g in gs:
        r, y = K.add_dropout_layer_norm(x, h, hb, w, b, p=0.0)
        y.backward(g)
    assert len(fired) == 6
    refs = [t.detach().float().clone().requires_grad_() for t in (hb, w, b)]
    for g in gs:
        rr = x.float() + h.float() + refs[0]
        yr = torch.nn.functional.layer_norm(rr, (C,), refs[1], refs[2], 1e-5)
        yr.backward(g.float())
    for got, ref in zip((hb, w, b), refs):
        err = (got.grad.float() - ref.grad).abs().max().item()
        assert err <= 2e-2 * ref.grad.abs().max().item() + 0.5, err


@pytest.mark.gpu
@pytest.mark.parametrize("rows,cols", [(16384, 6144), (1000, 264), (7, 8)])
def test_linear_bias_grad_colsum_kernel(rows, cols):
    """Linear bias gradient = colsum(dy) on the HIP row-block kernel, fresh and accumulated
    into an existing .grad, vs an fp32 reference."""
    g = torch.Generator(device='cuda').manual_seed(3)
    dy = torch.randn(rows, cols, device='cuda', dtype=torch.bfloat16, generator=g)
    b = torch.zeros(cols, device='cuda', dtype=torch.bfloat16, requires_grad=True)
    ref = dy.float().sum(0)
    with torch.no_grad():
        db = K.bias_grad(dy, b)
    tol = 2e-2 * max(1.0, rows ** 0.5 / 16)
    torch.testing.assert_close(db.float(), ref, atol=tol, rtol=1e-2)
    b.grad = torch.ones(cols, device='cuda', dtype=torch.bfloat16)
    with torch.no_grad():
        assert K.bias_grad(dy, b) is None
    torch.testing.assert_close(b.grad.float(), ref + 1, atol=tol, rtol=1e-2)
    # through autograd: LinearFn's bias gradient
    x = torch.randn(rows, 16, device='cuda', dtype=torch.bfloat16, generator=g, requires_grad=True)
    w = torch.randn(16, cols, device='cuda', dtype=torch.bfloat16, generator=g, requires_grad=True)
    b2 = torch.zeros(cols, device='cuda', dtype=torch.bfloat16, requires_grad=True)
    K.linear(x, w, b2).backward(dy)
    torch.testing.assert_close(b2.grad.float(), ref, atol=tol, rtol=1e-2)


@pytest.mark.gpu
def test_residual_bn_reduce_in_join_dgrad(monkeypatch):
    """Two stacked bottlenecks: block A's output BN (+ residual + ReLU) gets its backward
    reductions from block B's joined input gradient (conv1 dgrad with the pending sum added before
    the ReLU mask, kBnG epilogue). Gradients match the unfused path."""
    import paddle_ray_amd as paddle
    from paddle_ray_amd.vision.models import resnet as R
    paddle.seed(0)
    ds = paddle.nn.Sequential(
        paddle.nn.Conv2D(64, 256, 1, stride=1, bias_attr=False, data_format='NHWC'),
        paddle.nn.BatchNorm2D(256, data_format='NHWC'))
    net = paddle.nn.Sequential(R.BottleneckBlock(64, 64, stride=1, downsample=ds, data_format='NHWC'),
                               R.BottleneckBlock(256, 64, stride=1, data_format='NHWC'))
    net = paddle.amp.decorate(net, level='O2', dtype='bfloat16')
    x0 = torch.randn(4, 16, 16, 64, device='cuda', dtype=torch.bfloat16)
    bufs0 = [b._t.clone() for b in net.buffers()]
    outs, used = [], []
    seen = []
    orig = K._BnHandoff.take

    def spy(self, dy2):
        r = orig(self, dy2)
        seen.append(r is not None)
        return r
    monkeypatch.setattr(K._BnHandoff, 'take', spy)
    for fuse in (True, False):
        monkeypatch.setattr(K, '_BN_DGRAD_FUSE', fuse)
        for b, b0 in zip(net.buffers(), bufs0):
            b._t.copy_(b0)
        for p in net.parameters():
            p._t.grad = None
        seen.clear()
        x = paddle.Tensor(x0.clone().requires_grad_())
        y = net(x)
        g = torch.randn(y.shape, device='cuda', generator=torch.Generator('cuda').manual_seed(1)).to(y._t.dtype)
        y._t.backward(g)
        used.append(sum(seen))
        outs.append((x._t.grad.float().clone(), [p._t.grad.float().clone() for p in net.parameters()]))
    # fused: block A's bn3, and both blocks' bn1 / bn2 (their conv consumers' dgrads)
    assert used[0] >= 5 and used[1] == 0, used
    (gx1, gp1), (gx2, gp2) = outs
    torch.testing.assert_close(gx1, gx2, rtol=3e-2, atol=3e-2)
    for a, b in zip(gp1, gp2):
        torch.testing.assert_close(a, b, rtol=5e-2, atol=5e-2)
