"""GPU numerics for the LDS-DMA MFMA GEMM (ops/csrc/gemm_lds.hip) against fp32 PyTorch references:
every layout (x·W, dy·Wᵀ, xᵀ·dy), ragged M/N edges, bias / GELU / ReLU epilogues with the
pre-activation output, dGELU + bias-gradient column sums, beta=1 accumulation, split-K, and the
autograd wrappers (Linear, tied LM head, fused MLP) built on it."""
import pytest
import torch

from paddle_ray_amd.ops import fused as K
from paddle_ray_amd.ops import registry as R

pytestmark = pytest.mark.gpu


_TS = (1 << 28) | (1 << 25) | (1 << 30)   # per-tile TS schedule: W8T for x·W / xᵀ·dy, W4T for dy·Wᵀ


@pytest.fixture(autouse=True, params=[(0, 0), (7, 0), (7 << 4, 0), (7 << 8, 0), (7 << 12, 0), (7 << 16, 0),
                                      (7 << 20, 0), (_TS, 0), (_TS, 7), (_TS, 7 | 16)],
                ids=['W8', 'W4', 'W8I', 'W4B', 'W8B', 'W4P', 'W8P', 'TS', 'PTS', 'PTS8'])
def _mfma_everywhere(request):
    """Exercise the in-tree kernel on every layout regardless of the 'auto' policy, in each
    wave configuration (gemm_set_w4 mask: 0 = 8 waves, 7 = 4 waves x 128x128, 7<<4 = 8 waves
    with the one-filler-per-MFMA schedule, 7<<8 / 7<<12 = W4 / W8 with MUBUF operand DMA,
    7<<16 / 7<<20 = W4 / W8 with the two-barrier early-refill schedule, TS = the default TS
    schedule) and with the persistent TS kernel (gemm_set_pts: 7 = every layout, +16 = 8 waves
    for dy·Wᵀ too)."""
    from paddle_ray_amd.ops import _native
    L = _native.lib()
    prev, prev_mask, prev_pts = K._GEMM_MODE, L.gemm_get_w4(), L.gemm_get_pts()
    K._GEMM_MODE = 'mfma'
    L.gemm_set_w4(request.param[0])
    L.gemm_set_pts(request.param[1])
    yield
    L.gemm_set_w4(prev_mask)
    L.gemm_set_pts(prev_pts)
    K._GEMM_MODE = prev


def _r(*s, scale=1.0):
    return ((torch.rand(*s, device='cuda') * 2 - 1) * scale).to(torch.bfloat16)


def _operands(layout, M, N, Kd):
    if layout == K.GEMM_FWD:
        return _r(M, Kd), _r(Kd, N)
    if layout == K.GEMM_NT:
        return _r(M, Kd), _r(N, Kd)
    return _r(Kd, M), _r(Kd, N)


def _ref(layout, a, b):
    a, b = a.float(), b.float()
    return a @ b if layout == K.GEMM_FWD else (a @ b.t() if layout == K.GEMM_NT else a.t() @ b)


def _close(x, ref, tol=2e-2):
    err = (x.float() - ref).abs().max().item()
    assert err <= tol * max(ref.abs().max().item(), 1e-3), (err, ref.abs().max().item())


@pytest.mark.parametrize('layout', [0, 1, 2])
@pytest.mark.parametrize('M,N,Kd', [(512, 512, 256), (300, 264, 128), (1000, 776, 192), (256, 2048, 1024)])
def test_layouts_and_edges(layout, M, N, Kd):
    if layout == 2 and M % 8:
        pytest.skip("wgrad needs M % 8 == 0")
    torch.manual_seed(0)
    a, b = _operands(layout, M, N, Kd)
    y = K._gemm_hip(layout, a, b)
    assert y is not None
    _close(y, _ref(layout, a, b))


@pytest.mark.parametrize('epi', ['gelu', 'gelu_tanh', 'relu'])
def test_bias_act_epilogue_with_preact(epi):
    torch.manual_seed(1)
    a, b = _operands(0, 520, 392, 256)
    bias = _r(392)
    z = torch.empty(520, 392, device='cuda', dtype=torch.bfloat16)
    y = K._gemm_hip(0, a, b, bias=bias, z=z, epi=epi)
    pre = _ref(0, a, b) + bias.float()
    _close(z, pre)
    if epi == 'relu':
        act = torch.relu(pre)
    else:
        act = torch.nn.functional.gelu(pre, approximate='tanh' if epi == 'gelu_tanh' else 'none')
    _close(y, act)


@pytest.mark.parametrize('epi', ['dgelu', 'dgelu_tanh'])
def test_dgelu_epilogue_and_bias_grad(epi):
    torch.manual_seed(2)
    dy, w = _r(600, 384), _r(264, 384)          # dz = (dy · wᵀ) * gelu'(z): [600, 264]
    z = _r(600, 264, scale=3.0)
    out, cs = K._gemm_hip(1, dy, w, z=z, epi=epi, want_colsum=True)
    zf = z.float().requires_grad_(True)
    g = torch.nn.functional.gelu(zf, approximate='tanh' if epi == 'dgelu_tanh' else 'none')
    ref, = torch.autograd.grad(g, zf, _ref(1, dy, w))
    _close(out, ref)
    _close(cs, ref.sum(0), tol=2e-2)
    _close(cs, out.float().sum(0), tol=1e-2)


@pytest.mark.parametrize('epi', ['gelu_d', 'gelu_tanh_d'])
@pytest.mark.parametrize('M,N,Kd', [(600, 264, 384), (4168, 4360, 256)])
def test_gelu_derivative_epilogue(epi, M, N, Kd):
    """x·W + b -> gelu, with z receiving gelu'(pre-activation) (the MLP forward that saves the
    derivative for its backward), ragged tiles and (4168 x 4360) more tiles than CUs."""
    torch.manual_seed(12)
    a, b = _operands(0, M, N, Kd)
    bias = _r(N)
    z = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
    y = K._gemm_hip(0, a, b, bias=bias, z=z, epi=epi)
    pre = (_ref(0, a, b) + bias.float()).requires_grad_(True)
    g = torch.nn.functional.gelu(pre, approximate='tanh' if epi == 'gelu_tanh_d' else 'none')
    d, = torch.autograd.grad(g.sum(), pre)
    _close(y, g.detach())
    _close(z, d)


@pytest.mark.parametrize('M,N,Kd', [(600, 264, 384), (4168, 4360, 256), (2048, 1280, 2048)])
def test_mulz_epilogue_and_bias_grad(M, N, Kd):
    """dz = (dy·Wᵀ) * z with the saved derivative z, plus the bias-gradient column sums."""
    torch.manual_seed(13)
    dy, w = _r(M, Kd), _r(N, Kd)
    z = _r(M, N, scale=1.2)
    out, cs = K._gemm_hip(1, dy, w, z=z, epi='mulz', want_colsum=True)
    ref = _ref(1, dy, w) * z.float()
    _close(out, ref)
    _close(cs, ref.sum(0), tol=2e-2)


def test_beta_accumulate_and_split_k():
    torch.manual_seed(3)
    # 2048 x 2048 output with K = 16384: 64 tiles -> split-K path
    a, b = _operands(2, 2048, 2048, 16384)
    c0 = _r(2048, 2048)
    c = c0.clone()
    from paddle_ray_amd.ops import _native
    assert _native.lib().gemm_lds_splits(2048, 2048, 16384) > 1
    K._gemm_hip(2, a, b, out=c, beta=1)
    _close(c, _ref(2, a, b) + c0.float())
    # no split-K for a full grid; beta with the in-kernel epilogue
    a, b = _operands(1, 1024, 512, 512)
    c0 = _r(1024, 512)
    c = c0.clone()
    K._gemm_hip(1, a, b, out=c, beta=1)
    _close(c, _ref(1, a, b) + c0.float())


@pytest.mark.parametrize('M,N,Kd', [(64, 256, 50176), (128, 512, 12544), (120, 264, 1024), (64, 1024, 256)])
def test_narrow_tn_128_row_tiles(M, N, Kd):
    """xᵀ·dy with <= 128 output rows (ResNet's 64 / 128-channel 1x1 weight gradients) on the
    128-row tile: split-K (long pixel axis) and single-pass, plain and beta=1."""
    torch.manual_seed(4)
    a, b = _operands(2, M, N, Kd)
    _close(K._gemm_hip(2, a, b), _ref(2, a, b))
    c0 = _r(M, N)
    c = c0.clone()
    K._gemm_hip(2, a, b, out=c, beta=1)
    _close(c, _ref(2, a, b) + c0.float())


def test_linear_fn_grads():
    torch.manual_seed(4)
    x = _r(4, 128, 256).requires_grad_(True)
    w = _r(256, 384).requires_grad_(True)
    bias = _r(384).requires_grad_(True)
    R.reset_stats()
    y = K.linear(x, w, bias)
    gy = _r(4, 128, 384)
    y.backward(gy)
    assert R.stats().get(('gemm', 'hip'), 0) >= 3 and ('gemm', 'fallback') not in R.stats()
    xf, wf, bf = (t.detach().float().requires_grad_(True) for t in (x, w, bias))
    yf = xf @ wf + bf
    yf.backward(gy.float())
    _close(y, yf)
    _close(x.grad, xf.grad)
    _close(w.grad, wf.grad)
    _close(bias.grad, bf.grad)


def test_linear_nt_head_grads():
    torch.manual_seed(5)
    h = _r(512, 256).requires_grad_(True)
    e = _r(1000, 256).requires_grad_(True)     # vocab 1000 (ragged N)
    e.grad = torch.zeros_like(e)               # dE accumulates in place (beta = 1)
    with torch.no_grad():
        e.grad.copy_(_r(1000, 256))
    g0 = e.grad.clone()
    y = K.linear_nt(h, e)
    gy = _r(512, 1000)
    y.backward(gy)
    hf, ef = h.detach().float().requires_grad_(True), e.detach().float().requires_grad_(True)
    (hf @ ef.t()).backward(gy.float())
    _close(y, hf.detach() @ ef.detach().t())
    _close(h.grad, hf.grad)
    _close(e.grad, ef.grad + g0.float())


@pytest.mark.parametrize('save_d', [True, False])
@pytest.mark.parametrize('mode', ['mfma', 'auto'])
@pytest.mark.parametrize('approx', [True, False])
def test_mlp_gelu_fused(approx, mode, save_d, monkeypatch):
    K._GEMM_MODE = mode
    monkeypatch.setattr(K, '_MLP_SAVE_D', save_d)
    torch.manual_seed(6)
    x = _r(2, 256, 256).requires_grad_(True)
    w1, b1, w2 = _r(256, 1024).requires_grad_(True), _r(1024).requires_grad_(True), \
        _r(1024, 256, scale=0.5).requires_grad_(True)
    R.reset_stats()
    y = K.mlp_gelu(x, w1, b1, w2, approx)
    gy = _r(2, 256, 256)
    y.backward(gy)
    st = R.stats()
    assert ('bias_gelu_fwd', 'hip') not in st and ('gemm', 'fallback') not in st
    xf, w1f, b1f, w2f = (t.detach().float().requires_grad_(True) for t in (x, w1, b1, w2))
    yf = torch.nn.functional.gelu(xf @ w1f + b1f, approximate='tanh' if approx else 'none') @ w2f
    yf.backward(gy.float())
    _close(y, yf)
    for got, ref in ((x.grad, xf.grad), (w1.grad, w1f.grad), (b1.grad, b1f.grad), (w2.grad, w2f.grad)):
        _close(got, ref, tol=3e-2)
    # second backward: every parameter gradient (fc1 bias included) accumulates in place
    K.mlp_gelu(x, w1, b1, w2, approx).backward(gy)
    for got, ref in ((w1.grad, w1f.grad), (b1.grad, b1f.grad), (w2.grad, w2f.grad)):
        _close(got, 2 * ref, tol=3e-2)


@pytest.mark.parametrize('layout', [0, 1, 2])
def test_many_tiles_per_workgroup(layout):
    """More 256x256 tiles than CUs (17 x 18 = 306 > 256): the persistent kernel's workgroups walk
    two tiles, refilling the next tile's operands under the epilogue; ragged last row / column."""
    torch.manual_seed(7)
    M, N, Kd = 4168, 4360, 384
    a, b = _operands(layout, M, N, Kd)
    ref = _ref(layout, a, b)
    _close(K._gemm_hip(layout, a, b), ref)
    c0 = _r(M, N)
    c = c0.clone()
    K._gemm_hip(layout, a, b, out=c, beta=1)
    _close(c, ref + c0.float())


def test_many_tiles_graph_replay():
    """The persistent kernel's dynamic tile counters reset themselves (the last workgroup out
    zeroes them): back-to-back launches and hipGraph replays, with no memset between them, must
    each cover every tile exactly once."""
    torch.manual_seed(9)
    M, N, Kd = 4168, 4360, 256
    a, b = _operands(0, M, N, Kd)
    ref = _ref(0, a, b)
    for _ in range(3):
        _close(K._gemm_hip(0, a, b), ref)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        out = K._gemm_hip(0, a, b)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = K._gemm_hip(0, a, b)
    for _ in range(4):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        _close(out, ref)


def test_many_tiles_epilogues():
    """bias + GELU with the pre-activation, and dGELU + column sums, over 306 tiles."""
    torch.manual_seed(8)
    M, N, Kd = 4168, 4360, 256
    a, b = _operands(0, M, N, Kd)
    bias = _r(N)
    z = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
    y = K._gemm_hip(0, a, b, bias=bias, z=z, epi='gelu_tanh')
    pre = _ref(0, a, b) + bias.float()
    _close(z, pre)
    _close(y, torch.nn.functional.gelu(pre, approximate='tanh'))
    dy, w = _r(M, Kd), _r(N, Kd)
    zz = _r(M, N, scale=3.0)
    out, cs = K._gemm_hip(1, dy, w, z=zz, epi='dgelu', want_colsum=True)
    zf = zz.float().requires_grad_(True)
    ref, = torch.autograd.grad(torch.nn.functional.gelu(zf), zf, _ref(1, dy, w))
    _close(out, ref)
    _close(cs, ref.sum(0), tol=2e-2)


@pytest.mark.parametrize('Kd,in_tree', [(768, True), (1024, True), (2048, False)])
def test_auto_policy_short_k_dgrad(Kd, in_tree):
    """'auto': dy·Wᵀ with K <= 1024 runs the in-tree persistent kernel (ahead of hipBLASLt at
    BERT-base widths), longer K goes to hipBLASLt; the dGELU epilogue path follows the same rule."""
    K._GEMM_MODE = 'auto'
    torch.manual_seed(9)
    dy, w = _r(2048, Kd), _r(1280, Kd)
    R.reset_stats()
    y = K.gemm(K.GEMM_NT, dy, w)
    st = R.stats()
    assert (st.get(('gemm', 'hipblaslt'), 0) == 0) == in_tree, st
    _close(y, _ref(1, dy, w))
    z = _r(2048, 1280, scale=3.0)
    out, cs = K.gemm(K.GEMM_NT, dy, w, z=z, epi='dgelu', want_colsum=True)
    zf = z.float().requires_grad_(True)
    ref, = torch.autograd.grad(torch.nn.functional.gelu(zf), zf, _ref(1, dy, w))
    _close(out, ref)
    _close(cs.float(), ref.sum(0), tol=2e-2)


@pytest.mark.parametrize('hidden,tokens', [(2048, 1024), (768, 512)])
def test_paired_wgrad_grouped_launch(hidden, tokens):
    """QKV + output-projection weight gradients (WgradPair): one grouped launch when the two tile
    counts fill one wave (hidden 2048: 192 + 64 tiles), separate launches otherwise; gradients
    match fp32 either way and the output projection's AccumulateGrad hook fires after the
    deferred accumulation."""
    torch.manual_seed(0)
    dev = 'cuda'
    x = (torch.randn(tokens, hidden, device=dev) * 0.5).bfloat16().requires_grad_()
    wq = (torch.randn(hidden, 3 * hidden, device=dev) * 0.02).bfloat16().requires_grad_()
    bq = torch.zeros(3 * hidden, device=dev).bfloat16().requires_grad_()
    wo = (torch.randn(hidden, hidden, device=dev) * 0.02).bfloat16().requires_grad_()
    for p in (wq, wo):
        p.grad = torch.zeros_like(p)
    seen = []
    wo.register_post_accumulate_grad_hook(lambda t: seen.append(float(t.grad.float().abs().sum())))
    pair = K.WgradPair()
    qkv = K.linear(x, wq, bq, pair=pair, w_dep=wo)
    a = qkv[:, :hidden] * qkv[:, hidden:2 * hidden] + qkv[:, 2 * hidden:]
    y = K.linear(a, wo, pair=pair)
    g = torch.randn_like(y)
    y.backward(g)
    torch.cuda.synchronize()
    assert pair.used == (1 if hidden == 2048 else 0)
    assert len(seen) == 1 and seen[0] > 0        # hook saw the accumulated gradient
    xf, wqf, bqf, wof = (t.detach().float().requires_grad_() for t in (x, wq, bq, wo))
    qf = xf @ wqf + bqf
    af = qf[:, :hidden] * qf[:, hidden:2 * hidden] + qf[:, 2 * hidden:]
    (af @ wof).backward(g.float())
    for got, want in ((wq.grad, wqf.grad), (wo.grad, wof.grad), (x.grad, xf.grad)):
        err = (got.float() - want).abs().max().item() / (want.abs().max().item() + 1e-6)
        assert err < 3e-2, err


@pytest.mark.parametrize('beta', [0, 1])
def test_tn_tail_split(beta):
    """TN weight gradient with a 40-tile tail past 6 full waves (LM-head shape, K shortened):
    the tail rows run as a separate split-K launch; result matches fp32."""
    M, N, KD = 50304, 2048, 1024
    g = torch.Generator(device='cuda').manual_seed(5)
    a = ((torch.rand(KD, M, device='cuda', generator=g) * 2 - 1) * 0.5).to(torch.bfloat16)
    b = ((torch.rand(KD, N, device='cuda', generator=g) * 2 - 1) * 0.5).to(torch.bfloat16)
    c0 = (torch.rand(M, N, device='cuda', generator=g) - 0.5).to(torch.bfloat16)
    out = c0.clone()
    K.gemm_tn_balanced(a, b, out=out, beta=beta)
    want = a.float().t() @ b.float() + (c0.float() if beta else 0)
    err = (out.float() - want).abs().max().item()
    assert err < 2e-2 * want.abs().max().item(), err
