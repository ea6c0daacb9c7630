"""Hot fused ops: autograd Functions over the kernel registry.

Each op has a ``hip`` kernel (gfx950, ``ops/csrc/*.hip``) and a ``ref`` kernel
(PyTorch fp32 composition). Parity targets in the reference:
  layer_norm  -> paddle/phi/kernels/gpu/layer_norm_kernel.cu, layer_norm_grad_kernel.cu
  rms_norm    -> paddle/phi/kernels/fusion/gpu (rms_norm) / incubate fused_rms_norm
  softmax     -> paddle/phi/kernels/gpudnn/softmax_gpudnn.h
  softmax_ce  -> paddle/phi/kernels/gpu/cross_entropy_kernel.cu (softmax_with_cross_entropy)
  bias_gelu   -> paddle/fluid/operators/fused/fused_dropout_act_bias.h
  flash_attn  -> python/paddle/nn/functional/flash_attention.py (flash_attn / _C_ops.flash_attn)
  adamw       -> paddle/phi/kernels/gpu/adamw_kernel.cu, fused_adam_kernel.cu
"""
import math

import torch

from . import registry as R
from . import _native

_DT = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}


def _dt(t):
    return _DT[t.dtype]


def _stream(t=None):
    return torch.cuda.current_stream().cuda_stream


def _ptr(t):
    return 0 if t is None else t.data_ptr()


# =============================================================================
# LayerNorm (last-dim normalisation over `cols`)
# =============================================================================
@R.register_kernel('layer_norm_fwd', 'ref')
def _ln_fwd_ref(x2, w, b, eps):
    xf = x2.float()
    mean = xf.mean(-1)
    var = xf.var(-1, unbiased=False)
    rstd = torch.rsqrt(var + eps)
    y = (xf - mean[:, None]) * rstd[:, None]
    if w is not None:
        y = y * w.float()
    if b is not None:
        y = y + b.float()
    return y.to(x2.dtype), mean, rstd


@R.register_kernel('layer_norm_bwd', 'ref')
def _ln_bwd_ref(dy, x2, w, mean, rstd, need_dw, need_db):
    xf, dyf = x2.float(), dy.float()
    xhat = (xf - mean[:, None]) * rstd[:, None]
    g = dyf * w.float() if w is not None else dyf
    c1 = (g * xhat).mean(-1, keepdim=True)
    c2 = g.mean(-1, keepdim=True)
    dx = (g - c2 - xhat * c1) * rstd[:, None]
    dw = (dyf * xhat).sum(0).to(w.dtype) if (w is not None and need_dw) else None
    db = dyf.sum(0).to(w.dtype if w is not None else dy.dtype) if need_db else None
    return dx.to(x2.dtype), dw, db


def _colsum_nblk(rows):
    return max(1, min(rows, 256))


@R.register_kernel('layer_norm_fwd', 'hip')
def _ln_fwd_hip(x2, w, b, eps):
    L = _native.lib()
    rows, cols = x2.shape
    y = torch.empty_like(x2)
    mean = torch.empty(rows, device=x2.device, dtype=torch.float32)
    rstd = torch.empty(rows, device=x2.device, dtype=torch.float32)
    L.layernorm_fwd(_ptr(x2), _ptr(w), _ptr(b), _ptr(y), _ptr(mean), _ptr(rstd), rows, cols,
                    float(eps), _dt(x2), _dt(w) if w is not None else _dt(x2), _stream())
    return y, mean, rstd


@R.register_kernel('layer_norm_bwd', 'hip')
def _ln_bwd_hip(dy, x2, w, mean, rstd, need_dw, need_db):
    L = _native.lib()
    rows, cols = x2.shape
    dx = torch.empty_like(x2)
    nblk = _colsum_nblk(rows)
    part = torch.empty((2, nblk, cols), device=x2.device, dtype=torch.float32)
    L.layernorm_bwd(_ptr(dy.contiguous()), _ptr(x2), _ptr(w), _ptr(mean), _ptr(rstd), _ptr(dx),
                    _ptr(part[0]), _ptr(part[1]), rows, cols, nblk, _dt(x2),
                    _dt(w) if w is not None else _dt(x2), _stream())
    dw = db = None
    pdt = w.dtype if w is not None else x2.dtype
    if need_dw and w is not None:
        dw = torch.empty(cols, device=x2.device, dtype=pdt)
        L.colsum(_ptr(part[0]), _ptr(dw), nblk, cols, _DT[pdt], _stream())
    if need_db:
        db = torch.empty(cols, device=x2.device, dtype=pdt)
        L.colsum(_ptr(part[1]), _ptr(db), nblk, cols, _DT[pdt], _stream())
    return dx, dw, db


class LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        shp = x.shape
        cols = w.numel() if w is not None else shp[-1]
        x2 = x.contiguous().view(-1, cols)
        y, mean, rstd = R.dispatch('layer_norm_fwd', x2, x2, w, b, eps)
        ctx.save_for_backward(x2, w, mean, rstd)
        ctx.has_b = b is not None
        ctx.shp = shp
        return y.view(shp)

    @staticmethod
    def backward(ctx, dy):
        x2, w, mean, rstd = ctx.saved_tensors
        dy2 = dy.contiguous().view(x2.shape)
        dx, dw, db = R.dispatch('layer_norm_bwd', x2, dy2, x2, w, mean, rstd,
                                ctx.needs_input_grad[1], ctx.has_b and ctx.needs_input_grad[2])
        return dx.view(ctx.shp), dw, db, None


def layer_norm(x, w, b, eps=1e-5):
    return LayerNormFn.apply(x, w, b, eps)


# =============================================================================
# RMSNorm
# =============================================================================
@R.register_kernel('rms_norm_fwd', 'ref')
def _rms_fwd_ref(x2, w, eps):
    xf = x2.float()
    rstd = torch.rsqrt(xf.pow(2).mean(-1) + eps)
    y = xf * rstd[:, None]
    if w is not None:
        y = y * w.float()
    return y.to(x2.dtype), rstd


@R.register_kernel('rms_norm_bwd', 'ref')
def _rms_bwd_ref(dy, x2, w, rstd, need_dw):
    xf, dyf = x2.float(), dy.float()
    xhat = xf * rstd[:, None]
    g = dyf * w.float() if w is not None else dyf
    c1 = (g * xhat).mean(-1, keepdim=True)
    dx = (g - xhat * c1) * rstd[:, None]
    dw = (dyf * xhat).sum(0).to(w.dtype) if (w is not None and need_dw) else None
    return dx.to(x2.dtype), dw


@R.register_kernel('rms_norm_fwd', 'hip')
def _rms_fwd_hip(x2, w, eps):
    L = _native.lib()
    rows, cols = x2.shape
    y = torch.empty_like(x2)
    rstd = torch.empty(rows, device=x2.device, dtype=torch.float32)
    L.rmsnorm_fwd(_ptr(x2), _ptr(w), _ptr(y), _ptr(rstd), rows, cols, float(eps), _dt(x2),
                  _dt(w) if w is not None else _dt(x2), _stream())
    return y, rstd


@R.register_kernel('rms_norm_bwd', 'hip')
def _rms_bwd_hip(dy, x2, w, rstd, need_dw):
    L = _native.lib()
    rows, cols = x2.shape
    dx = torch.empty_like(x2)
    nblk = _colsum_nblk(rows)
    part = torch.empty((nblk, cols), device=x2.device, dtype=torch.float32)
    L.rmsnorm_bwd(_ptr(dy.contiguous()), _ptr(x2), _ptr(w), _ptr(rstd), _ptr(dx), _ptr(part),
                  rows, cols, nblk, _dt(x2), _dt(w) if w is not None else _dt(x2), _stream())
    dw = None
    if need_dw and w is not None:
        dw = torch.empty(cols, device=x2.device, dtype=w.dtype)
        L.colsum(_ptr(part), _ptr(dw), nblk, cols, _dt(w), _stream())
    return dx, dw


class RMSNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps):
        shp = x.shape
        x2 = x.contiguous().view(-1, shp[-1])
        y, rstd = R.dispatch('rms_norm_fwd', x2, x2, w, eps)
        ctx.save_for_backward(x2, w, rstd)
        ctx.shp = shp
        return y.view(shp)

    @staticmethod
    def backward(ctx, dy):
        x2, w, rstd = ctx.saved_tensors
        dx, dw = R.dispatch('rms_norm_bwd', x2, dy.contiguous().view(x2.shape), x2, w, rstd,
                            ctx.needs_input_grad[1])
        return dx.view(ctx.shp), dw, None


def rms_norm(x, w, eps=1e-6):
    return RMSNormFn.apply(x, w, eps)


# =============================================================================
# Softmax (last dim)
# =============================================================================
@R.register_kernel('softmax_fwd', 'ref')
def _sm_fwd_ref(x2):
    return torch.softmax(x2.float(), -1).to(x2.dtype)


@R.register_kernel('softmax_bwd', 'ref')
def _sm_bwd_ref(y2, dy2):
    yf, dyf = y2.float(), dy2.float()
    return (yf * (dyf - (yf * dyf).sum(-1, keepdim=True))).to(y2.dtype)


@R.register_kernel('softmax_fwd', 'hip')
def _sm_fwd_hip(x2):
    y = torch.empty_like(x2)
    _native.lib().softmax_fwd(_ptr(x2), _ptr(y), x2.shape[0], x2.shape[1], _dt(x2), _stream())
    return y


@R.register_kernel('softmax_bwd', 'hip')
def _sm_bwd_hip(y2, dy2):
    dx = torch.empty_like(y2)
    _native.lib().softmax_bwd(_ptr(y2), _ptr(dy2), _ptr(dx), y2.shape[0], y2.shape[1], _dt(y2),
                              _stream())
    return dx


class SoftmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x2 = x.contiguous().view(-1, x.shape[-1])
        y = R.dispatch('softmax_fwd', x2, x2)
        ctx.save_for_backward(y)
        ctx.shp = x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        return R.dispatch('softmax_bwd', y, y, dy.contiguous().view(y.shape)).view(ctx.shp)


def softmax_lastdim(x):
    if x.dtype not in _DT or x.shape[-1] == 0:
        return torch.softmax(x, -1)
    return SoftmaxFn.apply(x)


# =============================================================================
# Fused softmax + cross-entropy (hard labels, ignore_index)
# =============================================================================
@R.register_kernel('softmax_ce_fwd', 'ref')
def _ce_fwd_ref(logits, labels, ignore_index):
    lf = logits.float()
    lse = torch.logsumexp(lf, -1)
    valid = labels != ignore_index
    safe = torch.where(valid, labels, torch.zeros_like(labels))
    picked = lf.gather(-1, safe[:, None]).squeeze(-1)
    loss = torch.where(valid, lse - picked, torch.zeros_like(lse))
    return loss, lse


@R.register_kernel('softmax_ce_bwd', 'ref')
def _ce_bwd_ref(logits, labels, lse, dloss, ignore_index):
    p = torch.exp(logits.float() - lse[:, None])
    valid = labels != ignore_index
    safe = torch.where(valid, labels, torch.zeros_like(labels))
    p.scatter_add_(-1, safe[:, None], -torch.ones_like(p[:, :1]))
    g = p * (dloss * valid.float())[:, None]
    return g.to(logits.dtype)


@R.register_kernel('softmax_ce_fwd', 'hip')
def _ce_fwd_hip(logits, labels, ignore_index):
    rows, V = logits.shape
    loss = torch.empty(rows, device=logits.device, dtype=torch.float32)
    lse = torch.empty(rows, device=logits.device, dtype=torch.float32)
    _native.lib().softmax_ce_fwd(_ptr(logits), _ptr(labels), _ptr(loss), _ptr(lse), rows, V,
                                 int(ignore_index), _dt(logits), _stream())
    return loss, lse


@R.register_kernel('softmax_ce_bwd', 'hip')
def _ce_bwd_hip(logits, labels, lse, dloss, ignore_index):
    rows, V = logits.shape
    dl = torch.empty_like(logits)
    _native.lib().softmax_ce_bwd(_ptr(logits), _ptr(labels), _ptr(lse),
                                 _ptr(dloss.float().contiguous()), _ptr(dl), rows, V,
                                 int(ignore_index), _dt(logits), _stream())
    return dl


class SoftmaxCEFn(torch.autograd.Function):
    """loss[i] = logsumexp(logits[i]) - logits[i, label[i]]; one pass over the vocab row."""

    @staticmethod
    def forward(ctx, logits, labels, ignore_index):
        shp = logits.shape
        l2 = logits.contiguous().view(-1, shp[-1])
        lab = labels.contiguous().view(-1).to(torch.int64)
        loss, lse = R.dispatch('softmax_ce_fwd', l2, l2, lab, ignore_index)
        ctx.save_for_backward(l2, lab, lse)
        ctx.ignore_index = ignore_index
        ctx.shp = shp
        return loss.view(shp[:-1])

    @staticmethod
    def backward(ctx, dloss):
        l2, lab, lse = ctx.saved_tensors
        g = R.dispatch('softmax_ce_bwd', l2, l2, lab, lse, dloss.contiguous().view(-1),
                       ctx.ignore_index)
        return g.view(ctx.shp), None, None


def softmax_cross_entropy(logits, labels, ignore_index=-100):
    return SoftmaxCEFn.apply(logits, labels, ignore_index)


# =============================================================================
# bias + GELU
# =============================================================================
def _gelu_ref(x, approximate):
    return torch.nn.functional.gelu(x, approximate='tanh' if approximate else 'none')


@R.register_kernel('bias_gelu_fwd', 'ref')
def _bg_fwd_ref(x2, b, approximate):
    xf = x2.float() + (b.float() if b is not None else 0)
    return _gelu_ref(xf, approximate).to(x2.dtype)


@R.register_kernel('bias_gelu_bwd', 'ref')
def _bg_bwd_ref(dy2, x2, b, approximate):
    with torch.enable_grad():
        xf = (x2.float() + (b.float() if b is not None else 0)).detach().requires_grad_(True)
        y = _gelu_ref(xf, approximate)
        (g,) = torch.autograd.grad(y, xf, dy2.float())
    return g.to(x2.dtype)


@R.register_kernel('bias_gelu_fwd', 'hip')
def _bg_fwd_hip(x2, b, approximate):
    y = torch.empty_like(x2)
    _native.lib().bias_gelu_fwd(_ptr(x2), _ptr(b), _ptr(y), x2.shape[0], x2.shape[1], _dt(x2),
                                int(approximate), _stream())
    return y


@R.register_kernel('bias_gelu_bwd', 'hip')
def _bg_bwd_hip(dy2, x2, b, approximate):
    dx = torch.empty_like(x2)
    _native.lib().bias_gelu_bwd(_ptr(dy2), _ptr(x2), _ptr(b), _ptr(dx), x2.shape[0], x2.shape[1],
                                _dt(x2), int(approximate), _stream())
    return dx


class BiasGeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, b, approximate):
        shp = x.shape
        x2 = x.contiguous().view(-1, shp[-1])
        if b is not None and b.dtype != x.dtype:
            b = b.to(x.dtype)
        y = R.dispatch('bias_gelu_fwd', x2, x2, b, approximate)
        ctx.save_for_backward(x2, b)
        ctx.approximate = approximate
        ctx.shp = shp
        return y.view(shp)

    @staticmethod
    def backward(ctx, dy):
        x2, b = ctx.saved_tensors
        dx = R.dispatch('bias_gelu_bwd', x2, dy.contiguous().view(x2.shape), x2, b,
                        ctx.approximate)
        db = dx.sum(0) if (b is not None and ctx.needs_input_grad[1]) else None
        return dx.view(ctx.shp), db, None


def bias_gelu(x, b=None, approximate=False):
    if x.dtype not in _DT:
        return _gelu_ref(x + (b if b is not None else 0), approximate)
    return BiasGeluFn.apply(x, b, approximate)


# =============================================================================
# Flash attention (q,k,v: [B, S, H, D], D contiguous; arbitrary b/s/h strides)
# =============================================================================
@R.register_kernel('flash_attn_fwd', 'ref')
def _fa_fwd_ref(q, k, v, causal, scale):
    qf, kf, vf = (t.float().permute(0, 2, 1, 3) for t in (q, k, v))
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        Sq, Sk = s.shape[-2:]
        m = torch.ones(Sq, Sk, dtype=torch.bool, device=s.device).triu(Sk - Sq + 1)
        s = s.masked_fill(m, float('-inf'))
    lse = torch.logsumexp(s, -1)
    p = torch.exp(s - lse[..., None])
    o = torch.matmul(p, vf).permute(0, 2, 1, 3).to(q.dtype)
    return o.contiguous(), lse.contiguous()


@R.register_kernel('flash_attn_bwd', 'ref')
def _fa_bwd_ref(do, q, k, v, o, lse, causal, scale):
    qf, kf, vf, dof, of_ = (t.float().permute(0, 2, 1, 3) for t in (q, k, v, do, o))
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        Sq, Sk = s.shape[-2:]
        m = torch.ones(Sq, Sk, dtype=torch.bool, device=s.device).triu(Sk - Sq + 1)
        s = s.masked_fill(m, float('-inf'))
    p = torch.exp(s - lse[..., None])
    dv = torch.matmul(p.transpose(-1, -2), dof)
    dp = torch.matmul(dof, vf.transpose(-1, -2))
    delta = (dof * of_).sum(-1, keepdim=True)
    ds = p * (dp - delta) * scale
    dq = torch.matmul(ds, kf)
    dk = torch.matmul(ds.transpose(-1, -2), qf)
    f = lambda t, like: t.permute(0, 2, 1, 3).to(like.dtype).contiguous()
    return f(dq, q), f(dk, k), f(dv, v)


def _fa_supported(q, k, v):
    D = q.shape[-1]
    return (q.dtype in (torch.bfloat16, torch.float16) and D in (64, 128) and
            q.stride(-1) == 1 and k.stride(-1) == 1 and v.stride(-1) == 1 and
            k.shape == v.shape and q.shape[0] == k.shape[0] and q.shape[2] == k.shape[2])


@R.register_kernel('flash_attn_fwd', 'hip')
def _fa_fwd_hip(q, k, v, causal, scale):
    if not _fa_supported(q, k, v):
        return _fa_fwd_ref(q, k, v, causal, scale)
    B, Sq, H, D = q.shape
    Sk = k.shape[1]
    o = torch.empty((B, Sq, H, D), device=q.device, dtype=q.dtype)
    lse = torch.empty((B, H, Sq), device=q.device, dtype=torch.float32)
    _native.lib().flash_fwd(_ptr(q), _ptr(k), _ptr(v), _ptr(o), _ptr(lse), B, H, Sq, Sk, D,
                            q.stride(0), q.stride(1), q.stride(2),
                            k.stride(0), k.stride(1), k.stride(2),
                            v.stride(0), v.stride(1), v.stride(2),
                            float(scale), int(causal), _dt(q), _stream())
    return o, lse


@R.register_kernel('flash_attn_bwd', 'hip')
def _fa_bwd_hip(do, q, k, v, o, lse, causal, scale):
    if not _fa_supported(q, k, v):
        return _fa_bwd_ref(do, q, k, v, o, lse, causal, scale)
    L = _native.lib()
    B, Sq, H, D = q.shape
    Sk = k.shape[1]
    do = do.contiguous()
    delta = torch.empty((B, H, Sq), device=q.device, dtype=torch.float32)
    L.flash_bwd_pre(_ptr(o), _ptr(do), _ptr(delta), B, H, Sq, D, _dt(q), _stream())
    dq = torch.empty((B, Sq, H, D), device=q.device, dtype=q.dtype)
    dk = torch.empty((B, Sk, H, D), device=q.device, dtype=q.dtype)
    dv = torch.empty((B, Sk, H, D), device=q.device, dtype=q.dtype)
    L.flash_bwd(_ptr(q), _ptr(k), _ptr(v), _ptr(do), _ptr(lse), _ptr(delta), _ptr(dq), _ptr(dk),
                _ptr(dv), B, H, Sq, Sk, D,
                q.stride(0), q.stride(1), q.stride(2),
                k.stride(0), k.stride(1), k.stride(2),
                v.stride(0), v.stride(1), v.stride(2),
                float(scale), int(causal), _dt(q), _stream())
    return dq, dk, dv


class FlashAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        o, lse = R.dispatch('flash_attn_fwd', q, q, k, v, causal, scale)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        dq, dk, dv = R.dispatch('flash_attn_bwd', q, do, q, k, v, o, lse, ctx.causal, ctx.scale)
        return dq, dk, dv, None, None


def flash_attention(q, k, v, causal=False, scale=None):
    """q,k,v: [B, S, H, D] -> o [B, S, H, D]."""
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    return FlashAttnFn.apply(q, k, v, causal, scale)


# =============================================================================
# Multi-tensor fused AdamW / Adam / Momentum (one launch for all params)
# =============================================================================
def adamw_ref(params, grads, ms, vs, masters, lr, b1, b2, eps, wds, lr_muls, step, grad_scale=1.0):
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    for i, p in enumerate(params):
        master = masters[i] if masters[i] is not None else p
        g = grads[i].float() * grad_scale
        m, v = ms[i], vs[i]
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        lr_i = lr * lr_muls[i]
        mf = master.float() if master.dtype != torch.float32 else master
        mf.mul_(1 - lr_i * wds[i])
        denom = (v / bc2).sqrt_().add_(eps)
        mf.addcdiv_(m, denom, value=-lr_i / bc1)
        if mf is not master:
            master.copy_(mf)
        if masters[i] is not None:
            p.copy_(master)


def _mt_table(cols, n_list, extra_f, device, chunk=65536):
    """Pack a multi-tensor descriptor table (int64 ptrs + float params) for the HIP kernels."""
    import numpy as np
    T = len(n_list)
    tab = np.zeros((T, 8), dtype=np.int64)
    for i in range(T):
        for j, c in enumerate(cols):
            tab[i, j] = c[i]
    ftab = np.zeros((T, 4), dtype=np.float32)
    for i in range(T):
        for j, f in enumerate(extra_f):
            ftab[i, j] = f[i]
    chunks = []
    for i, n in enumerate(n_list):
        for s in range(0, n, chunk):
            chunks.append((i, s))
    ch = np.array(chunks, dtype=np.int64).reshape(-1, 2)
    dev_tab = torch.from_numpy(tab).to(device, non_blocking=False)
    dev_f = torch.from_numpy(ftab).to(device, non_blocking=False)
    dev_ch = torch.from_numpy(ch).to(device, non_blocking=False)
    return dev_tab, dev_f, dev_ch, len(chunks)


class MultiTensorAdamW:
    """Cached multi-tensor launch plan for a fixed parameter list (built once, replayed)."""

    def __init__(self, params, grads_getter, ms, vs, masters, wds, lr_muls):
        self.params, self.ms, self.vs, self.masters = params, ms, vs, masters
        self.grads_getter = grads_getter
        self.wds, self.lr_muls = wds, lr_muls
        self._plan = None
        self._gptrs = None

    def _build(self, grads):
        dev = self.params[0].device
        n = [p.numel() for p in self.params]
        cols = [[(self.masters[i] if self.masters[i] is not None else p).data_ptr()
                 for i, p in enumerate(self.params)],
                [g.data_ptr() for g in grads],
                [m.data_ptr() for m in self.ms],
                [v.data_ptr() for v in self.vs],
                [p.data_ptr() if self.masters[i] is not None else 0
                 for i, p in enumerate(self.params)],
                n,
                [_DT[g.dtype] for g in grads],
                [_DT[p.dtype] for p in self.params]]
        self._plan = _mt_table(cols, n, [self.wds, self.lr_muls], dev)
        self._gptrs = tuple(g.data_ptr() for g in grads)

    def step(self, lr, b1, b2, eps, step, grad_scale=1.0):
        grads = self.grads_getter()
        if self._plan is None or tuple(g.data_ptr() for g in grads) != self._gptrs:
            self._build(grads)
        tab, ftab, ch, nch = self._plan
        bc1 = 1 - b1 ** step
        bc2 = 1 - b2 ** step
        _native.lib().adamw_mt(_ptr(tab), _ptr(ftab), _ptr(ch), nch, float(lr), float(b1),
                               float(b2), float(eps), float(bc1), float(bc2), float(grad_scale),
                               _stream())


def momentum_ref(params, grads, vels, masters, lr, mu, wds, use_nesterov, grad_scale=1.0):
    for i, p in enumerate(params):
        master = masters[i] if masters[i] is not None else p
        g = grads[i].float() * grad_scale + wds[i] * master.float()
        v = vels[i]
        v.mul_(mu).add_(g)
        upd = g + mu * v if use_nesterov else v
        master.sub_((lr * upd).to(master.dtype))
        if masters[i] is not None:
            p.copy_(master)


def global_l2_norm_sq(tensors):
    """Sum of squares over a list of tensors (fp32 accumulate)."""
    if not tensors:
        return None
    if tensors[0].is_cuda and _native.available():
        out = torch.zeros(1, device=tensors[0].device, dtype=torch.float32)
        L = _native.lib()
        for t in tensors:
            L.sumsq_accum(_ptr(t), _ptr(out), t.numel(), _dt(t), _stream())
        return out[0]
    return sum((t.float() ** 2).sum() for t in tensors)
