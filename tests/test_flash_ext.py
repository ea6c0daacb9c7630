"""Flash attention extensions: additive mask, in-kernel dropout, varlen (flash_attn_unpadded).
GPU tests compare the HIP kernels with an fp32 PyTorch reference that applies the SAME dropout
bits (ops.fused.fa_dropout_mask_ref, a port of the kernel's counter hash); varlen against
per-sequence dense attention. Parity: python/paddle/nn/functional/flash_attention.py:20,121,
paddle/phi/kernels/gpu/flash_attn_kernel.cu:183,250."""
import math

import numpy as np
import pytest
import torch

import paddle_ray_amd as paddle
from paddle_ray_amd.ops import fused as K


def test_dropout_hash_statistics_cpu():
    bh = torch.arange(4).view(4, 1, 1)
    q = torch.arange(64).view(1, 64, 1)
    k = torch.arange(64).view(1, 1, 64)
    z = K.fa_dropout_mask_ref(1234, 7, bh, q, k, 0.25)
    keep = (z > 0).float().mean().item()
    assert abs(keep - 0.75) < 0.02
    np.testing.assert_allclose(z[z > 0].unique().numpy(), [1 / 0.75], rtol=1e-6)
    z2 = K.fa_dropout_mask_ref(1234, 8, bh, q, k, 0.25)
    assert (z != z2).float().mean() > 0.2  # a new offset draws new bits


def test_varlen_ref_matches_dense_per_sequence_cpu():
    torch.manual_seed(0)
    lens = [5, 9, 3]
    H, D = 2, 16
    cu = torch.tensor([0] + list(np.cumsum(lens)), dtype=torch.int32)
    q, k, v = (torch.randn(sum(lens), H, D) for _ in range(3))
    o = K.flash_attn_varlen(q, k, v, cu, cu, max(lens), max(lens), causal=True)
    for b, L in enumerate(lens):
        a, e = int(cu[b]), int(cu[b + 1])
        ref, _ = K._fa_ext_ref_dense(q[a:e][None], k[a:e][None], v[a:e][None], True, 1 / math.sqrt(D))
        np.testing.assert_allclose(o[a:e].numpy(), ref[0].numpy(), rtol=1e-5, atol=1e-6)


def test_sdpa_mask_and_dropout_api_cpu():
    import paddle_ray_amd.nn.functional as F
    q = paddle.randn([2, 8, 2, 16])
    m = paddle.zeros([2, 1, 1, 8])
    m[:, :, :, 6:] = float('-inf')
    o = F.scaled_dot_product_attention(q, q, q, attn_mask=m, training=False)
    ref, _ = K._fa_ext_ref_dense(q._t, q._t, q._t, False, 1 / 4.0, m._t)
    np.testing.assert_allclose(o.numpy(), ref.cpu().numpy(), rtol=1e-5, atol=1e-6)
    out, _ = F.flash_attention(q, q, q, dropout=0.5, causal=True)
    assert out.shape == [2, 8, 2, 16]


def _fp32_grads(fn, tensors, g):
    ts = [t.detach().float().requires_grad_(True) for t in tensors]
    out = fn(*ts)
    out.backward(g.float())
    return out.detach(), [t.grad for t in ts]


@pytest.mark.gpu
@pytest.mark.parametrize('causal', [False, True])
@pytest.mark.parametrize('D', [64, 128])
def test_flash_dropout_matches_reference_with_same_mask(causal, D):
    """Forward draws the keep bits (one hash per key pair) and stores them; the dK/dV kernel
    reads them. Same bits as the fp32 reference (fa_dropout_mask_ref)."""
    torch.manual_seed(1)
    dev = torch.device('cuda')
    B, S, H = 2, 320, 3
    p = 0.2
    q, k, v = (torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
               for _ in range(3))
    seed, off = 4321, 17
    sc = 1 / math.sqrt(D)
    o = K.FlashAttnExtFn.apply(q, k, v, None, None, None, S, S, causal, sc, p, seed, off)
    g = torch.randn_like(o)
    o.backward(g)
    ro, rg = _fp32_grads(lambda a, b, c: K._fa_ext_ref_dense(a, b, c, causal, sc, None, p, seed, off)[0],
                         (q, k, v), g)
    err = (o.float() - ro).abs().max().item() / ro.abs().max().item()
    assert err < 2e-2, err
    for got, ref, n in zip((q.grad, k.grad, v.grad), rg, 'qkv'):
        e = (got.float() - ref).abs().max().item() / ref.abs().max().item()
        assert e < 3e-2, (n, e)


@pytest.mark.gpu
@pytest.mark.parametrize('drop', [0.0, 0.1])
@pytest.mark.parametrize('mdtype', [torch.bfloat16, torch.float32])
def test_flash_key_padding_mask(drop, mdtype):
    """[B, 1, 1, Sk] key-padding mask (the XF_KMASK path: the forward's LDS mask row, the dK/dV
    kernel's per-lane value), alone and with dropout, against the fp32 reference."""
    torch.manual_seed(5)
    dev = torch.device('cuda')
    B, S, H, D = 3, 384, 2, 64
    q, k, v = (torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
               for _ in range(3))
    m = torch.zeros(B, 1, 1, S, device=dev, dtype=mdtype)
    m[0, ..., 300:] = float('-inf')
    m[2, ..., 17:] = float('-inf')
    m[1, ..., :5] = -3.0
    seed, off = 99, 3
    sc = 1 / math.sqrt(D)
    o = K.FlashAttnExtFn.apply(q, k, v, m, None, None, S, S, False, sc, drop, seed, off)
    g = torch.randn_like(o)
    o.backward(g)
    ro, rg = _fp32_grads(lambda a, b, c: K._fa_ext_ref_dense(a, b, c, False, sc, m.float(), drop, seed, off)[0],
                         (q, k, v), g)
    assert (o.float() - ro).abs().max().item() / ro.abs().max().item() < 2e-2
    for got, ref, n in zip((q.grad, k.grad, v.grad), rg, 'qkv'):
        e = (got.float() - ref).abs().max().item() / ref.abs().max().item()
        assert e < 3e-2, (n, e)


@pytest.mark.gpu
def test_flash_additive_mask_fwd_bwd():
    torch.manual_seed(2)
    dev = torch.device('cuda')
    B, S, H, D = 2, 200, 2, 64
    q, k, v = (torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
               for _ in range(3))
    # padding mask [B, 1, 1, S] (-inf past each batch's length) + a random bias [1, H, S, S]
    m = torch.zeros(B, 1, 1, S, device=dev)
    m[0, ..., 150:] = float('-inf')
    bias = (torch.randn(1, H, S, S, device=dev) * 0.5)
    mask = (m + bias).to(torch.bfloat16)
    o = K.flash_attention_ext(q, k, v, attn_mask=mask)
    g = torch.randn_like(o)
    o.backward(g)
    sc = 1 / math.sqrt(D)
    ro, rg = _fp32_grads(lambda a, b, c: K._fa_ext_ref_dense(a, b, c, False, sc, mask.float())[0], (q, k, v), g)
    assert (o.float() - ro).abs().max().item() / ro.abs().max().item() < 2e-2
    for got, ref in zip((q.grad, k.grad, v.grad), rg):
        assert (got.float() - ref).abs().max().item() / ref.abs().max().item() < 3e-2
    # fp32 mask path and bool mask path
    o32 = K.flash_attention_ext(q.detach(), k.detach(), v.detach(), attn_mask=(m + bias).float())
    assert (o32.float() - ro).abs().max().item() / ro.abs().max().item() < 2e-2
    keep = torch.ones(B, 1, S, S, dtype=torch.bool, device=dev).tril()
    ob = K.flash_attention_ext(q.detach(), k.detach(), v.detach(), attn_mask=keep)
    oc = K.flash_attention(q.detach(), k.detach(), v.detach(), causal=True)
    assert (ob.float() - oc.float()).abs().max().item() < 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize('causal', [False, True])
def test_flash_varlen_matches_per_sequence_dense(causal):
    torch.manual_seed(3)
    dev = torch.device('cuda')
    lens = [37, 300, 1, 129, 256]
    H, D = 4, 128
    cu = torch.tensor([0] + list(np.cumsum(lens)), dtype=torch.int32, device=dev)
    tot = sum(lens)
    q, k, v = (torch.randn(tot, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    o = K.flash_attn_varlen(q, k, v, cu, cu, max(lens), max(lens), causal=causal)
    g = torch.randn_like(o)
    o.backward(g)
    sc = 1 / math.sqrt(D)
    for b, L in enumerate(lens):
        a, e = int(cu[b]), int(cu[b + 1])
        qs, ks, vs = (t.detach()[a:e][None] for t in (q, k, v))
        ro, rg = _fp32_grads(lambda x, y, z: K._fa_ext_ref_dense(x, y, z, causal, sc)[0], (qs, ks, vs), g[a:e][None])
        assert (o[a:e].float() - ro[0]).abs().max().item() < 3e-2 * max(1.0, ro.abs().max().item())
        for got, ref in zip((q.grad[a:e], k.grad[a:e], v.grad[a:e]), rg):
            assert (got.float() - ref[0]).abs().max().item() < 4e-2 * max(1.0, ref.abs().max().item())
    # the paddle API + dropout through varlen
    import paddle_ray_amd.nn.functional as F
    out, _ = F.flash_attn_unpadded(paddle.Tensor(q.detach()), paddle.Tensor(k.detach()),
                                   paddle.Tensor(v.detach()), paddle.Tensor(cu), paddle.Tensor(cu),
                                   max(lens), max(lens), sc, dropout=0.1, causal=causal)
    assert out.shape == [tot, H, D] and torch.isfinite(out._t.float()).all()


@pytest.mark.gpu
def test_gpt_attention_dropout_uses_flash_kernel():
    from paddle_ray_amd.models import gpt_config, GPTForPretraining
    from paddle_ray_amd.ops import registry as R
    paddle.set_device('gpu')
    paddle.set_default_dtype('bfloat16')
    m = GPTForPretraining(gpt_config('gpt3-tiny', num_heads=2, attention_dropout=0.1))  # head_dim 64
    paddle.set_default_dtype('float32')
    ids = paddle.randint(0, 1000, [2, 65])
    R.reset_stats()
    loss = m(ids[:, :-1], ids[:, 1:])
    loss.backward()
    st = R.stats()
    assert st.get(('flash_attn_ext', 'hip'), 0) > 0, st
    assert np.isfinite(float(loss))


@pytest.mark.gpu
def test_packed_qkv_ext_matches_unpacked():
    torch.manual_seed(7)
    dev = torch.device('cuda')
    B, S, H, D = 2, 256, 3, 64
    qkv = torch.randn(B, S, 3, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    m = torch.zeros(B, 1, 1, S, device=dev, dtype=torch.bfloat16)
    m[1, ..., 200:] = float('-inf')
    o = K.flash_attention_ext_qkvpacked(qkv, attn_mask=m, dropout=0.1, seed=11)
    g = torch.randn_like(o)
    o.backward(g)
    q2 =qkv.detach().clone().requires_grad_(True)
    q, k, v = q2.unbind(2)
    o2 = K.flash_attention_ext(q, k, v, attn_mask=m, dropout=0.1, seed=11)
    o2.backward(g)
    assert torch.equal(o, o2)
    assert torch.equal(qkv.grad, q2.grad)


@pytest.mark.gpu
def test_dropout_masks_change_across_graph_replays():
    """Captured dropout launches (flash attention, add+dropout+LayerNorm) read the device step
    counter: every replay draws new masks, forward and backward agree within a replay."""
    torch.manual_seed(8)
    dev = torch.device('cuda')
    B, S, H, D = 2, 128, 2, 64
    q, k, v = (torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    x = torch.randn(B * S, 256, device=dev, dtype=torch.bfloat16)
    hh = torch.randn(B * S, 256, device=dev, dtype=torch.bfloat16, requires_grad=True)
    w = torch.ones(256, device=dev, dtype=torch.bfloat16)
    b = torch.zeros(256, device=dev, dtype=torch.bfloat16)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm up outside the capture
        K.flash_attention_ext(q, k, v, dropout=0.5).sum().backward()
        K.add_dropout_layer_norm(x, hh, None, w, b, 0.5)[0].float().sum().backward()
    torch.cuda.current_stream().wait_stream(s)
    q.grad = k.grad = v.grad = hh.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        o = K.flash_attention_ext(q, k, v, dropout=0.5)
        r, _ = K.add_dropout_layer_norm(x, hh, None, w, b, 0.5)
        (o.float().sum() + r.float().sum()).backward()
    outs = []
    for _ in range(2):
        g.replay()
        torch.cuda.synchronize()
        outs.append((o.clone(), r.clone(), v.grad.clone(), hh.grad.clone()))
    (o1, r1, gv1, gh1), (o2, r2, gv2, gh2) = outs
    assert not torch.equal(o1, o2) and not torch.equal(r1, r2)
    # within a replay the backward used the forward's masks: dh is zero exactly where r == x
    drop1 = (r1 == x)
    # (a kept x + 2h can round back to x in bf16 for tiny h: allow a few such elements)
    assert ((gh1 == 0) != drop1).float().mean().item() < 0.01
    assert ((gh1 == 0) != (gh2 == 0)).float().mean().item() > 0.2
    assert not torch.equal(gv1, gv2)


@pytest.mark.gpu
def test_framework_graph_entry_advances_dropout_per_replay():
    """The framework's own captures (jit / static Executor graph entries) advance the dropout
    step counter eagerly before each replay: successive replays draw new masks."""
    from paddle_ray_amd.framework.core import Tensor
    from paddle_ray_amd.jit.api import _GraphEntry
    torch.manual_seed(9)
    q = torch.randn(2, 128, 2, 64, device='cuda', dtype=torch.bfloat16)

    def fn(t):
        x = t._t
        return Tensor(K.flash_attention_ext(x, x, x, dropout=0.5))
    g = _GraphEntry(fn, (Tensor(q),), {})
    assert g.rng_dev is not None
    o1 = g((Tensor(q),), {})._t
    o2 = g((Tensor(q),), {})._t
    torch.cuda.synchronize()
    assert not torch.equal(o1, o2)
    assert torch.isfinite(o1.float()).all() and torch.isfinite(o2.float()).all()


def _recompute_dropout_case(dev):
    """A block of flash attention with dropout: the gradients with recompute (the segment re-runs
    in backward) must equal the gradients without it, i.e. the re-run draws the same mask."""
    from paddle_ray_amd.parallel.recompute import recompute
    dt = torch.bfloat16 if dev.type == 'cuda' else torch.float32
    B, S, H, D = 2, 64, 2, 64
    torch.manual_seed(3)
    x = torch.randn(B, S, H * D, device=dev, dtype=dt)
    w = torch.randn(H * D, 3 * H * D, device=dev, dtype=dt) * 0.05

    def block(xx, ww):
        xx, ww = getattr(xx, '_t', xx), getattr(ww, '_t', ww)  # (recompute passes paddle Tensors)
        q, k, v = (xx @ ww).view(B, S, 3, H, D).unbind(2)
        return K.flash_attention_ext(q, k, v, causal=True, dropout=0.3).reshape(B, S, H * D)

    grads = []
    for use_rc in (False, True):
        paddle.seed(11)
        xx = x.clone().requires_grad_(True)
        ww = w.clone().requires_grad_(True)
        out = recompute(block, xx, ww) if use_rc else block(xx, ww)
        out = out._t if hasattr(out, '_t') else out
        (out.float() ** 2).sum().backward()
        grads.append((out.detach().float(), xx.grad.float(), ww.grad.float()))
    for a, b in zip(*grads):
        assert torch.equal(a, b)
    # and a different seed draws a different mask
    paddle.seed(12)
    o3 = block(x, w)
    assert not torch.equal(o3.float(), grads[0][0])


def test_recompute_flash_dropout_same_mask_cpu():
    _recompute_dropout_case(torch.device('cpu'))


@pytest.mark.gpu
def test_recompute_flash_dropout_same_mask_gpu():
    _recompute_dropout_case(torch.device('cuda'))


@pytest.mark.gpu
def test_transformer_encoder_mask_dropout_on_flash_ext():
    """nn.TransformerEncoderLayer with a key-padding mask and attention dropout runs the extended
    flash kernel (registry: flash_attn_ext/hip) and matches an fp32 host copy of the same layer
    that applies the SAME dropout bits (same host seed, fa_dropout_mask_ref)."""
    from paddle_ray_amd.ops import registry as R
    import copy
    paddle.seed(21)
    d, nh, B, S = 256, 4, 2, 128
    layer = paddle.nn.TransformerEncoderLayer(d, nh, 512, dropout=0.0, attn_dropout=0.2)
    layer.train()
    ref = copy.deepcopy(layer)
    layer.to(device='gpu', dtype='bfloat16')
    x = paddle.randn([B, S, d])
    mask = np.zeros((B, 1, 1, S), 'float32')
    mask[1, ..., 100:] = -1e9
    xg = paddle.to_tensor(x.numpy(), place='gpu').astype('bfloat16')
    xg.stop_gradient = False
    R.reset_stats()
    paddle.seed(77)
    y = layer(xg, paddle.to_tensor(mask, place='gpu').astype('bfloat16'))
    assert R.stats().get(('flash_attn_ext', 'hip'), 0) > 0, R.stats()
    g = paddle.randn(y.shape)
    y.backward(paddle.to_tensor(g.numpy(), place='gpu').astype('bfloat16'))
    # the reference runs on the HOST (fp32 dense path, same host-drawn seed -> same keep bits);
    # on a GPU host the default place is the device, where fp32 would take torch SDPA instead
    ref.to(device='cpu')
    xc = paddle.to_tensor(x.numpy(), place='cpu')
    xc.stop_gradient = False
    paddle.seed(77)
    yr = ref(xc, paddle.to_tensor(mask, place='cpu'))
    yr.backward(paddle.to_tensor(g.numpy(), place='cpu'))
    yv, yrv = y.astype('float32').numpy(), yr.numpy()
    assert np.abs(yv - yrv).max() / np.abs(yrv).max() < 3e-2
    gx, gxr = xg.grad.astype('float32').numpy(), xc.grad.numpy()
    assert np.abs(gx - gxr).max() / np.abs(gxr).max() < 5e-2


@pytest.mark.gpu
@pytest.mark.parametrize('D', [80, 96])
@pytest.mark.parametrize('causal', [False, True])
def test_flash_ext_other_head_dims(D, causal):
    """Head dims outside the flash kernel (80, 96) take torch's memory-efficient SDPA: values and
    gradients match an fp32 reference, and no [B, H, S, S] fp32 score tensor is kept (the peak
    allocation stays far below one)."""
    torch.manual_seed(0)
    B, S, H = 2, 1024, 4
    q, k, v = (torch.randn(B, S, H, D, device='cuda', dtype=torch.bfloat16).requires_grad_() for _ in range(3))
    mask = torch.zeros(B, 1, 1, S, device='cuda', dtype=torch.bfloat16)
    mask[:, :, :, S - 64:] = float('-inf')            # key padding
    before = K.R._STATS[('flash_attn_ext', 'sdpa')]
    import paddle_ray_amd.device.cuda as dc    # (works with the native allocator too)
    torch.cuda.synchronize()
    dc.reset_max_memory_allocated()
    base = dc.memory_allocated()
    o = K.flash_attention_ext(q, k, v, causal=causal, attn_mask=mask)
    g = torch.randn_like(o)
    o.backward(g)
    torch.cuda.synchronize()
    peak = dc.max_memory_allocated() - base
    assert K.R._STATS[('flash_attn_ext', 'sdpa')] == before + 1
    scores_fp32 = B * H * S * S * 4
    print(f"D={D} causal={causal}: peak {peak / 2**20:.1f} MiB vs fp32 scores {scores_fp32 / 2**20:.1f} MiB")
    assert peak < scores_fp32 / 2, (peak, scores_fp32)   # measured 6-12 MiB vs 32 MiB
    qf, kf, vf = (t.detach().float().requires_grad_() for t in (q, k, v))
    s = torch.einsum('bqhd,bkhd->bhqk', qf, kf) / math.sqrt(D) + mask.float()
    if causal:
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device='cuda').triu(1), float('-inf'))
    of = torch.einsum('bhqk,bkhd->bqhd', s.softmax(-1), vf)
    of.backward(g.float())
    torch.testing.assert_close(o.float(), of, atol=2e-2, rtol=2e-2)
    for a, b in ((q.grad, qf.grad), (k.grad, kf.grad), (v.grad, vf.grad)):
        err = (a.float() - b).abs().max().item() / (b.abs().max().item() + 1e-6)
        assert err < 3e-2, err


@pytest.mark.gpu
@pytest.mark.parametrize('shape', [(16, 1024, 16, 128), (3, 77, 5, 64), (2, 512, 12, 64)])
def test_attn_delta_kernel(shape):
    """delta[b, h, s] = sum_d dO * O (the flash backward's row term) vs fp32."""
    from paddle_ray_amd.ops import _native
    B, S, H, D = shape
    torch.manual_seed(0)
    o = torch.randn(B, S, H, D, device='cuda').bfloat16()
    do = torch.randn(B, S, H, D, device='cuda').bfloat16()
    delta = torch.full((B, H, S), float('nan'), device='cuda')
    _native.lib().flash_bwd_pre(o.data_ptr(), do.data_ptr(), delta.data_ptr(), B, H, S, D, 2,
                                torch.cuda.current_stream().cuda_stream)
    want = (o.float() * do.float()).sum(-1).permute(0, 2, 1)
    torch.testing.assert_close(delta, want, atol=1e-3, rtol=1e-3)
