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
import os

import numpy as np
import torch

from . import registry as R
from . import _native

_DT = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}


def _dt(t):
    return _DT[t.dtype]


def _stream(t=None):
    return torch.cuda.current_stream().cuda_stream


def _ptr(t):
    """Device address of a HIP kernel operand. A host or meta tensor here (e.g. a symbolic
    static-graph Variable reaching a kernel selected by another operand's device) would hand
    the kernel a host / null address and fault the GPU: refuse on the host instead."""
    if t is None:
        return 0
    if not t.is_cuda:
        raise TypeError(f"HIP kernel operand on {t.device}, expected the GPU")
    return t.data_ptr()


def _like(t, dtype):
    """Cast ``t`` to ``dtype`` when they differ (autocast regions mix bf16 activations with
    fp32 residuals / parameters; every HIP kernel reads its operands with ONE dtype code)."""
    return t if t is None or t.dtype == dtype else t.to(dtype)


def _check_dtypes(op, *pairs):
    """Host-side guard before a launch: a kernel given mismatched operand dtypes would read
    past the end of the narrower buffer."""
    for a, b in pairs:
        if a is not None and b is not None and a.dtype != b.dtype:
            raise TypeError(f"{op}: operand dtypes differ ({a.dtype} vs {b.dtype})")


# =============================================================================
# LayerNorm (last-dim normalisation over `cols`)
# kernel keys: the dtypes each HIP kernel is compiled for (registry dispatch falls back to the
# ref kernel for any other dtype instead of handing the HIP kernel a buffer it misreads)
_FLOATS = (torch.float32, torch.float16, torch.bfloat16)
_HALF = (torch.float16, torch.bfloat16)

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


def _adl_ok(cols):
    return cols % 8 == 0 and cols <= 4096


_ADL_NBLK = int(__import__('os').environ.get('PRA_ADL_NBLK', '768'))


def _adl_nblk(rows):
    # 768 workgroups of 4 waves = 3 waves per SIMD on 256 CUs (the two-pass backward's occupancy)
    return max(1, min(_ADL_NBLK, (rows + 7) // 8))


@R.register_kernel('layer_norm_fwd', 'hip', dtypes=_FLOATS)
def _ln_fwd_hip(x2, w, b, eps):
    _check_dtypes('layer_norm', (w, b))
    L = _native.lib()
    rows, cols = x2.shape
    y = torch.empty_like(x2)
    mean = torch.empty(rows, device=x2.device, dtype=torch.float32)
    rstd = torch.empty(rows, device=x2.device, dtype=torch.float32)
    dtw = _dt(w) if w is not None else _dt(x2)
    if _adl_ok(cols):
        L.adl_fwd(_ptr(x2), 0, 0, _ptr(w), _ptr(b), 0, _ptr(y), _ptr(mean), _ptr(rstd), rows, cols,
                  float(eps), 0.0, 0, 0, 0, _dt(x2), dtw, _stream())
    else:
        L.layernorm_fwd(_ptr(x2), _ptr(w), _ptr(b), _ptr(y), _ptr(mean), _ptr(rstd), rows, cols,
                        float(eps), _dt(x2), dtw, _stream())
    return y, mean, rstd


@R.register_kernel('layer_norm_bwd', 'hip', dtypes=_FLOATS)
def _ln_bwd_hip(dy, x2, w, mean, rstd, need_dw, need_db):
    L = _native.lib()
    rows, cols = x2.shape
    dx = torch.empty_like(x2)
    pdt = w.dtype if w is not None else x2.dtype
    dtw = _dt(w) if w is not None else _dt(x2)
    dy = dy.contiguous()
    if _adl_ok(cols):
        nblk = _adl_nblk(rows)
        part = torch.empty((2, nblk, cols), device=x2.device, dtype=torch.float32)
        L.adl_bwd(_ptr(dy), 0, _ptr(x2), _ptr(w), _ptr(mean), _ptr(rstd), _ptr(dx), 0,
                  _ptr(part[0]) if (need_dw and w is not None) else 0,
                  _ptr(part[1]) if need_db else 0, 0, rows, cols, nblk, 0.0, 0, 0, 0, _dt(x2), dtw,
                  _stream())
        red = L.colsum16
    else:
        nblk = _colsum_nblk(rows)
        part = torch.empty((2, nblk, cols), device=x2.device, dtype=torch.float32)
        L.layernorm_bwd(_ptr(dy), _ptr(x2), _ptr(w), _ptr(mean), _ptr(rstd), _ptr(dx),
                        _ptr(part[0]), _ptr(part[1]), rows, cols, nblk, _dt(x2), dtw, _stream())
        red = L.colsum
    dw = db = None
    if need_dw and w is not None:
        dw = torch.empty(cols, device=x2.device, dtype=pdt)
        red(_ptr(part[0]), _ptr(dw), nblk, cols, _DT[pdt], _stream())
    if need_db:
        db = torch.empty(cols, device=x2.device, dtype=pdt)
        red(_ptr(part[1]), _ptr(db), nblk, cols, _DT[pdt], _stream())
    return dx, dw, db


class LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        shp = x.shape
        cols = w.numel() if w is not None else shp[-1]
        x2 = x.contiguous().view(-1, cols)
        if w is not None:
            b = _like(b, w.dtype)
        y, mean, rstd = R.dispatch('layer_norm_fwd', x2, x2, w, b, eps)
        ctx.save_for_backward(x2, w, mean, rstd)
        ctx.has_b = b is not None
        ctx.shp = shp
        return y.view(shp)

    @staticmethod
    def backward(ctx, dy):
        x2, w, mean, rstd = ctx.saved_tensors
        dy2 = _like(dy, x2.dtype).contiguous().view(x2.shape)
        dx, dw, db = R.dispatch('layer_norm_bwd', x2, dy2, x2, w, mean, rstd,
                                ctx.needs_input_grad[1], ctx.has_b and ctx.needs_input_grad[2])
        return dx.view(ctx.shp), dw, db, None


def layer_norm(x, w, b, eps=1e-5):
    return LayerNormFn.apply(x, w, b, eps)


# =============================================================================
# Fused residual add + dropout(+bias) + LayerNorm:  r = x + drop(h + hb);  y = LN(r)
# =============================================================================
def _dropout_seed():
    # drawn from the host generator: follows paddle.seed and recompute's RNG restore
    return int(torch.randint(0, 2 ** 62, (1,)).item())


# Graph-safe dropout RNG. The kernels' seeds are host values, so a launch captured into a HIP
# graph would replay ONE mask forever. Under capture every dropout kernel also reads a device
# step counter (mixed into its seed in-kernel); the first dropout launch of each capture also
# captures `counter += 1`, so every replay advances it once and all launches of that replay --
# forward and backward, including recomputed segments -- read the same new value. Eager
# launches pass a null pointer (host seed only). The counter is created outside any pool that a
# graph could free (torch.empty under capture would come from the graph's private pool and is
# never released: it stays referenced here).
# The framework's own graph entries (jit / static Executor) capture under managed_graph_rng():
# no advance is captured; their replay advances the counter eagerly before a graph whose capture
# used it (graph_seq_advance), and a training pair advances only before the FORWARD graph, so a
# backward graph (and any recompute inside it) reads the forward's value.
_GSEQ = {}
_GSEQ_MANAGED = [None]


def _graph_seq(dev):
    """(device pointer of the step counter or 0, the counter tensor to keep alive or None)."""
    if dev.type != 'cuda' or not torch.cuda.is_current_stream_capturing():
        return 0, None
    st = _GSEQ.get(dev.index)
    if st is None:
        st = _GSEQ[dev.index] = [torch.empty(1, dtype=torch.int64, device=dev), 0]
    managed = _GSEQ_MANAGED[0]
    if managed is not None:
        managed['used'] = True
        return st[0].data_ptr(), st[0]
    cid = _native.lib().capture_id(_stream())
    if st[1] != cid:  # a user capture: its first dropout launch captures the advance
        st[0].add_(1)
        st[1] = cid
    return st[0].data_ptr(), st[0]


class managed_graph_rng:
    """Context for a capture whose replays advance the dropout step counter eagerly
    (``used`` tells whether any captured launch reads it)."""

    def __enter__(self):
        self.prev, self.state = _GSEQ_MANAGED[0], {'used': False}
        _GSEQ_MANAGED[0] = self.state
        return self.state

    def __exit__(self, *exc):
        _GSEQ_MANAGED[0] = self.prev
        return False


def graph_seq_advance(dev):
    """Advance the dropout step counter of ``dev`` (eager launch before a managed replay)."""
    st = _GSEQ.get(dev.index)
    if st is not None:
        st[0].add_(1)


def _hash_keep_ref(n, p, seed, device):
    """Reference of the kernel's counter-hash keep mask (for CPU + tests)."""
    import numpy as np
    i = np.arange(n, dtype=np.uint64)
    c = (i >> np.uint64(1)).astype(np.uint64)
    M = np.uint64(0xffffffff)

    def mix(x):
        x = x & M
        x ^= x >> np.uint64(16); x = (x * np.uint64(0x7feb352d)) & M
        x ^= x >> np.uint64(15); x = (x * np.uint64(0x846ca68b)) & M
        x ^= x >> np.uint64(16)
        return x
    s = np.uint64(seed)
    a = mix((c & M) ^ (s & M))
    r = mix(a ^ (c >> np.uint64(32)) ^ (s >> np.uint64(32)) ^ np.uint64(0x9e3779b9))
    u = np.where(i % np.uint64(2) == 0, r & np.uint64(0xffff), r >> np.uint64(16))
    thr = np.uint64(int(p * 65536 + 0.5))
    return torch.from_numpy((u >= thr).astype(np.bool_)).to(device)


@R.register_kernel('add_dropout_ln_fwd', 'ref')
def _adl_fwd_ref(x2, h2, hb, w, b, p, eps, seed):
    t = h2.float() + (hb.float() if hb is not None else 0)
    if p > 0:
        keep = _hash_keep_ref(h2.numel(), p, seed, h2.device).view(h2.shape)
        t = torch.where(keep, t / (1 - p), torch.zeros_like(t))
    r = (x2.float() + t).to(x2.dtype)
    y, mean, rstd = _ln_fwd_ref(r, w, b, eps)
    return r, y, mean, rstd


@R.register_kernel('add_dropout_ln_bwd', 'ref')
def _adl_bwd_ref(dy, dr_out, r, w, mean, rstd, p, seed, need_dw, need_db, need_dhb):
    dx, dw, db = _ln_bwd_ref(dy, r, w, mean, rstd, need_dw, need_db)
    dri = dx.float() + (dr_out.float() if dr_out is not None else 0)
    dh = dri
    if p > 0:
        keep = _hash_keep_ref(r.numel(), p, seed, r.device).view(r.shape)
        dh = torch.where(keep, dri / (1 - p), torch.zeros_like(dri))
    dhb = dh.sum(0).to(r.dtype) if need_dhb else None
    return dri.to(r.dtype), dh.to(r.dtype), dw, db, dhb


@R.register_kernel('add_dropout_ln_fwd', 'hip', dtypes=_FLOATS)
def _adl_fwd_hip(x2, h2, hb, w, b, p, eps, seed, dseq=0):
    _check_dtypes('add_dropout_layer_norm', (x2, h2), (x2, hb), (w, b))
    rows, cols = x2.shape
    if not _adl_ok(cols):
        return _adl_fwd_ref(x2, h2, hb, w, b, p, eps, seed)
    r = torch.empty_like(x2)
    y = torch.empty_like(x2)
    mean = torch.empty(rows, device=x2.device, dtype=torch.float32)
    rstd = torch.empty(rows, device=x2.device, dtype=torch.float32)
    _native.lib().adl_fwd(_ptr(x2), _ptr(h2), _ptr(hb), _ptr(w), _ptr(b), _ptr(r), _ptr(y),
                          _ptr(mean), _ptr(rstd), rows, cols, float(eps), float(p), seed, 0, dseq,
                          _dt(x2), _dt(w) if w is not None else _dt(x2), _stream())
    return r, y, mean, rstd


@R.register_kernel('add_dropout_ln_bwd', 'hip', dtypes=_FLOATS)
def _adl_bwd_hip(dy, dr_out, r, w, mean, rstd, p, seed, need_dw, need_db, need_dhb, into=None, dseq=0):
    """into: (w.grad, b.grad, hb.grad) or None per slot — those column sums are ADDED into the
    existing gradient by the reduction kernel and None is returned in their place (no
    AccumulateGrad add kernels for the LayerNorm / bias parameters)."""
    _check_dtypes('add_dropout_layer_norm_grad', (r, dy), (r, dr_out))
    rows, cols = r.shape
    if not _adl_ok(cols):
        return _adl_bwd_ref(dy, dr_out, r, w, mean, rstd, p, seed, need_dw, need_db, need_dhb)
    L = _native.lib()
    dri = torch.empty_like(r)
    dh = torch.empty_like(r)
    nblk = _adl_nblk(rows)
    part = torch.empty((3, nblk, cols), device=r.device, dtype=torch.float32)
    pdt = w.dtype if w is not None else r.dtype
    L.adl_bwd(_ptr(dy), _ptr(dr_out), _ptr(r), _ptr(w), _ptr(mean), _ptr(rstd), _ptr(dri),
              _ptr(dh), _ptr(part[0]) if need_dw else 0, _ptr(part[1]) if need_db else 0,
              _ptr(part[2]) if need_dhb else 0, rows, cols, nblk, float(p), seed, 0, dseq, _dt(r),
              _dt(w) if w is not None else _dt(r), _stream())
    outs, jobs = [], []
    into = into or (None, None, None)
    for need, i, dt in ((need_dw, 0, pdt), (need_db, 1, pdt), (need_dhb, 2, r.dtype)):
        if need and into[i] is not None:
            jobs.append((i, into[i], 1))
            outs.append(None)
        elif need:
            o = torch.empty(cols, device=r.device, dtype=dt)
            jobs.append((i, o, 0))
            outs.append(o)
        else:
            outs.append(None)
    if jobs and cols % 4 == 0 and len({o.dtype for _, o, _ in jobs}) == 1:
        # every parameter-gradient reduction of this backward in one launch
        L.colsum_multi([_ptr(part[i]) for i, _, _ in jobs], [_ptr(o) for _, o, _ in jobs],
                       [a for _, _, a in jobs], nblk, cols, _DT[jobs[0][1].dtype], _stream())
    else:
        for i, o, a in jobs:
            (L.colsum16_acc if a else L.colsum16)(_ptr(part[i]), _ptr(o), nblk, cols, _DT[o.dtype], _stream())
    return (dri, dh) + tuple(outs)


def _acc_target(p):
    """p's existing gradient when a kernel may add into it in place (see LinearFn)."""
    if p is None or not p.is_cuda or not p.requires_grad or p.grad_fn is not None:
        return None
    return p.grad if _acc_grad_ok(p.grad, p, p.dtype) else None


class AddDropoutLNFn(torch.autograd.Function):
    none_grads_ok = True   # backward takes g_r / g_y = None (static graph: no zero fill)

    @staticmethod
    def forward(ctx, x, h, hb, w, b, p, eps):
        shp = x.shape
        cols = shp[-1]
        x2 = x.contiguous().view(-1, cols)
        h2 = _like(h, x.dtype).contiguous().view(-1, cols)
        hb = _like(hb, x.dtype)
        if w is not None:
            b = _like(b, w.dtype)
        seed = _dropout_seed() if p > 0 else 0
        dseq, ctx.gseq = _graph_seq(x.device) if p > 0 else (0, None)
        if dseq and R.select_backend(x2, 'add_dropout_ln_fwd') == 'hip':
            r, y, mean, rstd = _adl_fwd_hip(x2, h2, hb, w, b, p, eps, seed, dseq)
        else:
            r, y, mean, rstd = R.dispatch('add_dropout_ln_fwd', x2, x2, h2, hb, w, b, p, eps, seed)
        ctx.save_for_backward(r, w, mean, rstd)
        ctx.params = (w, b, hb)
        ctx.p, ctx.seed, ctx.shp, ctx.dseq = p, seed, shp, dseq
        ctx.has_b, ctx.has_hb = b is not None, hb is not None
        return r.view(shp), y.view(shp)

    @staticmethod
    def backward(ctx, g_r, g_y):
        r, w, mean, rstd = ctx.saved_tensors
        cols = ctx.shp[-1]
        if g_y is None:
            g_y = torch.zeros_like(r)
        dr_out = None if g_r is None else _like(g_r, r.dtype).contiguous().view(-1, cols)
        args = (r, _like(g_y, r.dtype).contiguous().view(-1, cols), dr_out, r, w, mean, rstd,
                ctx.p, ctx.seed, w is not None and ctx.needs_input_grad[3],
                ctx.has_b and ctx.needs_input_grad[4], ctx.has_hb and ctx.needs_input_grad[2])
        if r.is_cuda and R.select_backend(r, 'add_dropout_ln_bwd') == 'hip':
            pw, pb, phb = ctx.params
            into = (_acc_target(pw), _acc_target(pb), _acc_target(phb))
            dri, dh, dw, db, dhb = _adl_bwd_hip(*args[1:], into=into, dseq=ctx.dseq)
        else:
            dri, dh, dw, db, dhb = R.dispatch('add_dropout_ln_bwd', *args)
        return dri.view(ctx.shp), dh.view(ctx.shp), dhb, dw, db, None, None


def add_dropout_layer_norm(x, h, hbias, w, b, p=0.0, eps=1e-5, training=True):
    """(r, y) with r = x + dropout(h + hbias), y = LayerNorm(r)·w + b."""
    p = p if training else 0.0
    if p > 0 and x.is_cuda and torch.cuda.is_current_stream_capturing() and not _adl_ok(x.shape[-1]):
        # a width the kernel does not take: torch's graph-aware dropout RNG under capture
        hh = h if hbias is None else h + hbias.to(h.dtype)
        r = x + torch.nn.functional.dropout(hh.to(x.dtype), p, True)
        return r, layer_norm(r, w, b, eps)
    return AddDropoutLNFn.apply(x, h, hbias, w, b, p, eps)


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


@R.register_kernel('rms_norm_fwd', 'hip', dtypes=_FLOATS)
def _rms_fwd_hip(x2, w, eps):
    L = _native.lib()
    rows, cols = x2.shape
    y = torch.empty_like(x2)
    rstd = torch.empty(rows, device=x2.device, dtype=torch.float32)
    L.rmsnorm_fwd(_ptr(x2), _ptr(w), _ptr(y), _ptr(rstd), rows, cols, float(eps), _dt(x2),
                  _dt(w) if w is not None else _dt(x2), _stream())
    return y, rstd


@R.register_kernel('rms_norm_bwd', 'hip', dtypes=_FLOATS)
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
        dx, dw = R.dispatch('rms_norm_bwd', x2, _like(dy, x2.dtype).contiguous().view(x2.shape), x2, w, rstd,
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


@R.register_kernel('softmax_fwd', 'hip', dtypes=_FLOATS)
def _sm_fwd_hip(x2):
    y = torch.empty_like(x2)
    _native.lib().softmax_fwd(_ptr(x2), _ptr(y), x2.shape[0], x2.shape[1], _dt(x2), _stream())
    return y


@R.register_kernel('softmax_bwd', 'hip', dtypes=_FLOATS)
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
        return R.dispatch('softmax_bwd', y, y, _like(dy, y.dtype).contiguous().view(y.shape)).view(ctx.shp)


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


@R.register_kernel('softmax_ce_fwd', 'hip', dtypes=_FLOATS)
def _ce_fwd_hip(logits, labels, ignore_index):
    rows, V = logits.shape
    loss = torch.empty(rows, device=logits.device, dtype=torch.float32)
    lse = torch.empty(rows, device=logits.device, dtype=torch.float32)
    _native.lib().softmax_ce_fwd(_ptr(logits), _ptr(labels), _ptr(loss), _ptr(lse), rows, V,
                                 int(ignore_index), _dt(logits), _stream())
    return loss, lse


@R.register_kernel('softmax_ce_bwd', 'hip', dtypes=_FLOATS)
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
# Vocab-parallel softmax + cross-entropy (parity: reference
# paddle/fluid/operators/collective/c_softmax_with_cross_entropy_op.cu). Each TP rank holds
# logits[:, start:start+V]; pass 1 reduces its slice to (max, sum-exp, picked) per row, the
# [rows, 3] partials are all-gathered (3 floats/row/rank instead of any [rows, V] tensor),
# pass 2 combines them into loss / lse, backward writes (softmax - onehot) * dloss for the
# local slice in one pass. No fp32 probabilities, no one-hot.
# =============================================================================
@R.register_kernel('vp_ce_part_fwd', 'ref')
def _vp_part_ref(logits, labels, start):
    lf = logits.float()
    m = lf.max(-1).values
    s = torch.exp(lf - m[:, None]).sum(-1)
    V = lf.shape[1]
    loc = labels - start
    inr = (loc >= 0) & (loc < V)
    picked = lf.gather(-1, loc.clamp(0, V - 1)[:, None]).squeeze(-1) * inr.float()
    return torch.stack([m, s, picked], -1).contiguous()


@R.register_kernel('vp_ce_part_fwd', 'hip', dtypes=_FLOATS)
def _vp_part_hip(logits, labels, start):
    rows, V = logits.shape
    st = torch.empty(rows, 3, device=logits.device, dtype=torch.float32)
    _native.lib().vp_ce_part_fwd(_ptr(logits), _ptr(labels), _ptr(st), rows, V, int(start),
                                 _dt(logits), _stream())
    return st


@R.register_kernel('vp_ce_final', 'ref')
def _vp_final_ref(stats, labels, vtot, ignore_index):
    m, s, picked = stats[..., 0], stats[..., 1], stats[..., 2]   # [world, rows]
    M = m.max(0).values
    lse = M + torch.log((s * torch.exp(m - M)).sum(0))
    valid = (labels != ignore_index) & (labels >= 0) & (labels < vtot)
    return torch.where(valid, lse - picked.sum(0), torch.zeros_like(lse)), lse


@R.register_kernel('vp_ce_final', 'hip')
def _vp_final_hip(stats, labels, vtot, ignore_index):
    world, rows = stats.shape[0], stats.shape[1]
    loss = torch.empty(rows, device=stats.device, dtype=torch.float32)
    lse = torch.empty_like(loss)
    _native.lib().vp_ce_final(_ptr(stats), _ptr(labels), _ptr(loss), _ptr(lse), rows, world,
                              int(vtot), int(ignore_index), _stream())
    return loss, lse


@R.register_kernel('vp_ce_bwd', 'ref')
def _vp_bwd_ref(logits, labels, lse, dloss, start, vtot, ignore_index):
    V = logits.shape[1]
    g = torch.exp(logits.float() - lse[:, None])
    loc = labels - start
    inr = (loc >= 0) & (loc < V)
    g.scatter_add_(-1, loc.clamp(0, V - 1)[:, None], -inr.float()[:, None])
    valid = (labels != ignore_index) & (labels >= 0) & (labels < vtot)
    return (g * (dloss.float() * valid.float())[:, None]).to(logits.dtype)


@R.register_kernel('vp_ce_bwd', 'hip', dtypes=_FLOATS)
def _vp_bwd_hip(logits, labels, lse, dloss, start, vtot, ignore_index):
    rows, V = logits.shape
    dl = torch.empty_like(logits)
    _native.lib().vp_ce_bwd(_ptr(logits), _ptr(labels), _ptr(lse), _ptr(dloss.float().contiguous()),
                            _ptr(dl), rows, V, int(start), int(vtot), int(ignore_index),
                            _dt(logits), _stream())
    return dl


class VocabParallelCEFn(torch.autograd.Function):
    """loss over a vocab dimension sharded across ``pg`` (rank r holds columns
    [r*V, (r+1)*V)); ``world == 1`` degenerates to the plain fused softmax-CE."""

    @staticmethod
    def forward(ctx, logits, labels, pg, world, rank, ignore_index):
        import torch.distributed as dist
        shp = logits.shape
        l2 = logits.contiguous().view(-1, shp[-1])
        lab = labels.contiguous().view(-1).to(torch.int64)
        V = l2.shape[1]
        start, vtot = rank * V, world * V
        part = R.dispatch('vp_ce_part_fwd', l2, l2, lab, start)
        if world > 1:
            allp = torch.empty((world,) + tuple(part.shape), dtype=part.dtype, device=part.device)
            if part.is_cuda:
                dist.all_gather_into_tensor(allp, part, group=pg)
            else:  # gloo has no all_gather_into_tensor
                dist.all_gather(list(allp.unbind(0)), part, group=pg)
        else:
            allp = part.unsqueeze(0)
        loss, lse = R.dispatch('vp_ce_final', allp, allp, lab, vtot, ignore_index)
        ctx.save_for_backward(l2, lab, lse)
        ctx.meta = (start, vtot, ignore_index, shp)
        return loss.view(shp[:-1])

    @staticmethod
    def backward(ctx, dloss):
        l2, lab, lse = ctx.saved_tensors
        start, vtot, ignore_index, shp = ctx.meta
        g = R.dispatch('vp_ce_bwd', l2, l2, lab, lse, dloss.contiguous().view(-1), start, vtot,
                       ignore_index)
        return g.view(shp), None, None, None, None, None


def vocab_parallel_cross_entropy(logits, labels, pg=None, world=1, rank=0, ignore_index=-100):
    return VocabParallelCEFn.apply(logits, labels, pg, world, rank, ignore_index)


# =============================================================================
# Decode-phase attention over a KV cache (decode_attn.hip; parity: the reference's masked
# multihead attention kernel of fused_multi_transformer). qkv [B, 3, H, D] is the current
# token's projection, cache [2, B, H, L, D]; positions [0, t) are read from the cache, the
# token's own K/V are written into it at position t. Inference only (no autograd).
# =============================================================================
@R.register_kernel('mmha_decode', 'ref')
def _mmha_ref(qkv, cache, t, mask):
    if isinstance(t, torch.Tensor):
        t = int(t.reshape(-1)[0])
    q, k, v = qkv.unbind(1)                                   # [B, H, D]
    cache[0, :, :, t] = k
    cache[1, :, :, t] = v
    K_, V_ = cache[0, :, :, :t + 1].float(), cache[1, :, :, :t + 1].float()
    s = torch.einsum('bhd,bhld->bhl', q.float(), K_) / math.sqrt(q.shape[-1])
    if mask is not None:
        s = s + mask.reshape(mask.shape[0], -1)[:, None, :t + 1].float()
    p = torch.softmax(s, -1)
    return torch.einsum('bhl,bhld->bhd', p, V_).to(qkv.dtype)


@R.register_kernel('mmha_decode', 'hip', dtypes=_FLOATS)
def _mmha_hip(qkv, cache, t, mask):
    B, _, H, D = qkv.shape
    L = cache.shape[3]
    t_dev = None
    if isinstance(t, torch.Tensor):  # device position (HIP-graph decode loops): read in-kernel
        if not (t.is_cuda and t.dtype == torch.int32 and t.is_contiguous()):
            raise ValueError("mmha_decode: a tensor time_step must be a CUDA int32 tensor")
        t_dev, t = t, 0
    if not (qkv.is_contiguous() and cache.is_contiguous() and cache.dtype == qkv.dtype and
            tuple(cache.shape) == (2, B, H, L, D) and D in (64, 128, 256) and
            (t_dev is not None or 0 <= t < L)):
        raise ValueError(f"mmha_decode: qkv {tuple(qkv.shape)} / cache {tuple(cache.shape)} / "
                         f"t={t} not supported by the HIP kernel")
    splits = _native.lib().mmha_splits(B, H, L - 1 if t_dev is not None else t)
    ws = torch.empty(B * H * splits * (2 + D) + 4 if splits > 1 else 4, device=qkv.device,
                     dtype=torch.float32)
    out = torch.empty(B, H, D, device=qkv.device, dtype=qkv.dtype)
    mlen = 0
    if mask is not None:
        mask = mask.reshape(B, -1).float().contiguous()
        mlen = mask.shape[1]
        if t_dev is None and mlen < t + 1:
            raise ValueError(f"mmha_decode: mask covers {mlen} positions, need {t + 1}")
    _native.lib().mmha_decode(_ptr(qkv), _ptr(cache), _ptr(mask) if mask is not None else 0,
                              _ptr(ws), _ptr(out), B, H, L, D, int(t),
                              _ptr(t_dev) if t_dev is not None else 0, splits, mlen,
                              1.0 / math.sqrt(D), _dt(qkv), _stream())
    return out


def mmha_decode(qkv, cache, time_step, mask=None):
    """One decode step of multi-head attention; returns [B, H, D] and appends K/V to
    ``cache`` at ``time_step`` in place. ``time_step`` may be a CUDA int32 tensor: the kernel
    reads it on the device (no host sync), so the step can live in a captured HIP graph."""
    if not isinstance(time_step, torch.Tensor):
        time_step = int(time_step)
    return R.dispatch('mmha_decode', qkv, qkv.contiguous(), cache, time_step, mask)


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


@R.register_kernel('bias_gelu_fwd', 'hip', dtypes=_FLOATS)
def _bg_fwd_hip(x2, b, approximate):
    y = torch.empty_like(x2)
    _native.lib().bias_gelu_fwd(_ptr(x2), _ptr(b), _ptr(y), x2.shape[0], x2.shape[1], _dt(x2),
                                int(approximate), _stream())
    return y


R.register_kernel('bias_gelu_bwd_db', 'hip')(lambda *a: None)  # dispatch-stats marker


@R.register_kernel('bias_gelu_bwd', 'hip', dtypes=_FLOATS)
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
        dy2 = _like(dy, x2.dtype).contiguous().view(x2.shape)
        rows, cols = x2.shape
        if (b is not None and ctx.needs_input_grad[1] and x2.is_cuda and cols % 8 == 0
                and R.select_backend(x2, 'bias_gelu_bwd_db') == 'hip'):
            # dx and d(bias) in one pass (bias grad = column sums kept in registers)
            L = _native.lib()
            nrb = max(1, min(256, rows // 16))
            part = torch.empty((nrb, cols), device=x2.device, dtype=torch.float32)
            dx = torch.empty_like(x2)
            L.bias_gelu_bwd_db(_ptr(dy2), _ptr(x2), _ptr(b), _ptr(dx), _ptr(part), rows, cols, nrb,
                               _dt(x2), int(ctx.approximate), _stream())
            db = torch.empty(cols, device=x2.device, dtype=b.dtype)
            L.colsum16(_ptr(part), _ptr(db), nrb, cols, _dt(db), _stream())
            return dx.view(ctx.shp), db, None
        dx = R.dispatch('bias_gelu_bwd', x2, dy2, x2, b, ctx.approximate)
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


@R.register_kernel('flash_attn_fwd', 'hip', dtypes=_HALF)
def _fa_fwd_hip(q, k, v, causal, scale):
    _check_dtypes('flash_attention', (q, k), (q, v))
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


# dQ path of the flash-attention backward: 'ds' = dQ = dS K from a dS^T scratch written by the
# dK/dV kernel (up to PRA_FA_DS_MAX_MB of scratch), 'sweep' = a dQ kernel recomputing S and dP
_FA_DQ = os.environ.get('PRA_FA_DQ', 'ds')
_FA_DS_MAX_BYTES = int(os.environ.get('PRA_FA_DS_MAX_MB', '4096')) << 20


@R.register_kernel('flash_attn_bwd', 'hip', dtypes=_HALF)
def _fa_bwd_hip(do, q, k, v, o, lse, causal, scale, dq=None, dk=None, dv=None, bsum=None):
    """bsum (optional, [B * ceil(S/128), 3*H*D] fp32, packed self-attention only): receives the
    column-sum partials of dQ/dK/dV, i.e. the QKV-projection bias gradient before its row
    reduction (filled only on the dS^T path; ``bsum.filled`` tells the caller)."""
    do = _like(do, q.dtype)
    _check_dtypes('flash_attention_grad', (q, k), (q, v), (q, o))
    if not _fa_supported(q, k, v):
        return _fa_bwd_ref(do, q, k, v, o, lse, causal, scale)
    L = _native.lib()
    B, Sq, H, D = q.shape
    Sk = k.shape[1]
    do = do.contiguous()
    o = o.contiguous()
    delta = torch.empty((B, H, Sq), device=q.device, dtype=torch.float32)
    ds_elems = B * H * (-(-Sk // 128) * 128) * (-(-Sq // 256) * 256)
    if _FA_DQ == 'ds' and ds_elems * 2 <= _FA_DS_MAX_BYTES:
        # dK/dV kernel stores dS^T (bf16 scratch), dQ = dS K from it: S and dP are not recomputed
        # for dQ. delta = rowsum(dO * O) comes from the preprocess kernel.
        L.flash_bwd_pre(_ptr(o), _ptr(do), _ptr(delta), B, H, Sq, D, _dt(q), _stream())
        ds = torch.empty(ds_elems, device=q.device, dtype=q.dtype)
        o_arg, ds_arg = 0, _ptr(ds)
    else:
        # delta is computed by the dQ sweep kernel itself (written for the dK/dV kernel)
        o_arg, ds_arg = _ptr(o), 0
    bs_arg = _ptr(bsum) if (bsum is not None and ds_arg and Sq == Sk) else 0
    if dq is None:
        dq = torch.empty((B, Sq, H, D), device=q.device, dtype=q.dtype)
        dk = torch.empty((B, Sk, H, D), device=q.device, dtype=q.dtype)
        dv = torch.empty((B, Sk, H, D), device=q.device, dtype=q.dtype)
    st = [q.stride(0), q.stride(1), q.stride(2), k.stride(0), k.stride(1), k.stride(2),
          v.stride(0), v.stride(1), v.stride(2), dq.stride(0), dq.stride(1), dq.stride(2),
          dk.stride(0), dk.stride(1), dk.stride(2), dv.stride(0), dv.stride(1), dv.stride(2)]
    L.flash_bwd(_ptr(q), _ptr(k), _ptr(v), _ptr(do), o_arg, _ptr(lse), _ptr(delta), _ptr(dq), _ptr(dk),
                _ptr(dv), ds_arg, B, H, Sq, Sk, D, st, float(scale), int(causal), _dt(q), _stream(), bs_arg)
    return (dq, dk, dv, bool(bs_arg)) if bsum is not None else (dq, dk, dv)


# QKV-projection bias gradient from the flash backward: the dQ / dK / dV kernels sum the rounded
# packed gradient's columns per 128-row block, so the Linear's bias_grad skips its own pass over
# the [tokens, 3*H*D] gradient (PRA_FA_BIAS_PART=0: the separate colsum kernel)
_FA_BIAS_PART = os.environ.get('PRA_FA_BIAS_PART', '1') == '1'


def _qkv_bias_part(qkv):
    """fp32 partial buffer for a packed [B, S, 3, H, D] gradient, or None when not applicable."""
    if not _FA_BIAS_PART or not qkv.is_cuda:
        return None
    B, S, _, H, D = qkv.shape
    return torch.empty((B * (-(-S // 128)), 3 * H * D), device=qkv.device, dtype=torch.float32)


def _tag_bias_part(dqkv, part):
    dqkv._pra_bias_part = (part, dqkv._version)


def _bias_part_of(dy2):
    """The flash backward's column-sum partials behind ``dy2`` (a [rows, 3*H*D] view of the
    packed dQKV it wrote), if that gradient is unmodified since; else None."""
    base = dy2 if dy2._base is None else dy2._base
    tag = getattr(base, '_pra_bias_part', None)
    if tag is None:
        return None
    part, ver = tag
    if base._version != ver or base.numel() != dy2.numel() or part.shape[1] != dy2.shape[-1] or \
            dy2.data_ptr() != base.data_ptr():
        return None
    return part


class FlashAttnQKVPackedFn(torch.autograd.Function):
    """qkv [B, S, 3, H, D] -> o [B, S, H, D]; backward writes dq/dk/dv straight into one
    packed [B, S, 3, H, D] gradient (no stack/cat of the three grads)."""

    @staticmethod
    def forward(ctx, qkv, causal, scale):
        q, k, v = qkv.unbind(2)
        o, lse = R.dispatch('flash_attn_fwd', qkv, q, k, v, causal, scale)
        ctx.save_for_backward(qkv, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        q, k, v = qkv.unbind(2)
        if R.select_backend(qkv, 'flash_attn_bwd') == 'hip' and _fa_supported(q, k, v):
            dqkv = torch.empty_like(qkv)
            dq, dk, dv = dqkv.unbind(2)
            part = _qkv_bias_part(qkv)
            r = _fa_bwd_hip(do, q, k, v, o, lse, ctx.causal, ctx.scale, dq, dk, dv, bsum=part)
            if part is not None and r[3]:
                _tag_bias_part(dqkv, part)
            return dqkv, None, None
        dq, dk, dv = _fa_bwd_ref(do, q, k, v, o, lse, ctx.causal, ctx.scale)
        return torch.stack([dq, dk, dv], 2), None, None


def flash_attention_qkvpacked(qkv, causal=False, scale=None):
    if scale is None:
        scale = 1.0 / math.sqrt(qkv.shape[-1])
    return FlashAttnQKVPackedFn.apply(qkv, causal, scale)


class FlashAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        k, v = _like(k, q.dtype), _like(v, q.dtype)
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


# -- extended flash attention: additive mask, in-kernel dropout, varlen (packed) ----------------
_M32 = 0xffffffff


def _mix32_t(x):
    x = x ^ (x >> 16)
    x = (x * 0x7feb352d) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846ca68b) & _M32
    return x ^ (x >> 16)


def fa_dropout_mask_ref(seed, offset, bh, q, kk, p_drop):
    """The keep multiplier (0 or 1/(1-thr/65536)) the flash kernels use for (head row bh, query q,
    key kk) — a torch port of flash_attn.hip fa_key / fa_drop for references and tests: one hash
    per pair of adjacent keys (kk >> 1), the low / high 16 bits as the even / odd key's uniform,
    keep iff u16 >= thr = round(p * 65536). bh/q/kk: int64 tensors (broadcastable)."""
    thr = min(65535, int(round(float(np.float32(p_drop)) * 65536.0)))  # the kernel receives a float32 p
    inv_keep = float(np.float32(65536.0 / (65536.0 - thr)))
    s0 = (seed & _M32) ^ ((((seed >> 32) & _M32) * 0x27d4eb2f) & _M32) ^ \
        (((offset & _M32) * 0x165667b1) & _M32)
    key = _mix32_t(((bh & _M32) * 0xc2b2ae3d & _M32) ^ s0)
    r = _mix32_t(key ^ (((q & _M32) * 0x9e3779b1) & _M32) ^ ((((kk >> 1) & _M32) * 0x85ebca77) & _M32))
    u = torch.where((kk & 1) == 1, r >> 16, r & 0xffff)
    return torch.where(u >= thr, inv_keep, 0.0)


def _fa_ext_ref_dense(q, k, v, causal, scale, mask=None, p_drop=0.0, seed=0, offset=0, bh0=None):
    """fp32 reference of the extended kernels for one dense batch [B, S, H, D] (autograd-able)."""
    qf, kf, vf = (t.float().permute(0, 2, 1, 3) for t in (q, k, v))
    B, H, Sq, Sk = qf.shape[0], qf.shape[1], qf.shape[2], kf.shape[2]
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if mask is not None:
        s = s + mask.float()
    if causal:
        m = torch.ones(Sq, Sk, dtype=torch.bool, device=s.device).triu(Sk - Sq + 1)
        s = s.masked_fill(m, float('-inf'))
    lse = torch.logsumexp(s, -1)
    p = torch.exp(s - lse[..., None]).nan_to_num(0.0)
    if p_drop > 0:
        dev = q.device
        bh = (torch.arange(B * H, device=dev) if bh0 is None else bh0).view(B, H, 1, 1)
        qi = torch.arange(Sq, device=dev).view(1, 1, Sq, 1)
        ki = torch.arange(Sk, device=dev).view(1, 1, 1, Sk)
        p = p * fa_dropout_mask_ref(seed, offset, bh, qi, ki, p_drop).to(p.dtype)
    o = torch.matmul(p, vf).permute(0, 2, 1, 3)
    return o, lse


def _mask_strides(mask, B, H, Sq, Sk):
    """[B|1, H|1, Sq, Sk] additive mask (any broadcastable rank <= 4, keys contiguous) ->
    (tensor, msb, msh, msq, is_fp32) with 0 strides on broadcast dims."""
    m = mask
    while m.dim() < 4:
        m = m.unsqueeze(0)
    m = m.expand(B, H, Sq, Sk)
    if m.stride(3) != 1:
        m = m.contiguous()
    return m, m.stride(0), m.stride(1), m.stride(2), m.dtype == torch.float32


def _fa_next_rng(seed=None, numel=1):
    """(seed, offset) for one dropout call. Without an explicit seed, a fresh per-call seed is
    drawn from the host generator (`_dropout_seed`), i.e. from the RNG state that paddle.seed
    sets, that recompute saves / restores around a re-run segment and that the model-parallel
    RNG tracker swaps per rank: a recomputed forward draws the same mask as the original one, and
    tensor-parallel ranks draw different masks for their local heads (the reference's flash_attn
    kernels take (seed, offset) from the same generator, paddle/phi/kernels/gpu/flash_attn_kernel.cu).
    An explicit seed is used as given with offset 0 (bit-exact replays in tests)."""
    if seed is None:
        return _dropout_seed() & ((1 << 63) - 1), 0
    return int(seed), 0


class FlashAttnExtFn(torch.autograd.Function):
    """Flash attention with an additive mask and/or in-kernel dropout, dense [B, S, H, D] or
    varlen packed [total, H, D] (cu_q / cu_k int32 [B+1]): one HIP forward, the dS^T backward."""

    @staticmethod
    def forward(ctx, q, k, v, mask, cu_q, cu_k, max_sq, max_sk, causal, scale, p_drop, seed, offset):
        L = _native.lib()
        varlen = cu_q is not None
        if varlen:
            B = cu_q.numel() - 1
            H, D = q.shape[1], q.shape[2]
            Sq, Sk = int(max_sq), int(max_sk)
            st = [0, q.stride(0), q.stride(1), 0, k.stride(0), k.stride(1), 0, v.stride(0), v.stride(1)]
            o = torch.empty((q.shape[0], H, D), device=q.device, dtype=q.dtype)
        else:
            B, Sq, H, D = q.shape
            Sk = k.shape[1]
            st = [q.stride(0), q.stride(1), q.stride(2), k.stride(0), k.stride(1), k.stride(2),
                  v.stride(0), v.stride(1), v.stride(2)]
            o = torch.empty((B, Sq, H, D), device=q.device, dtype=q.dtype)
        lse = torch.empty((B, H, Sq), device=q.device, dtype=torch.float32)
        mk, msb, msh, msq, m32 = (None, 0, 0, 0, False) if mask is None else \
            _mask_strides(mask, B, H, Sq, Sk)
        # dropout keep bits for the backward (1 bit per score: B*H*Sq*Sk/8 bytes, 12.6 MB at
        # BERT-base bs32): the dK/dV kernel reads them instead of re-hashing every score
        dbits = torch.empty(B * H * Sq * (-(-Sk // 32)), device=q.device, dtype=torch.int32) \
            if p_drop > 0 else torch.empty(0, device=q.device, dtype=torch.int32)
        dseq, ctx.gseq = _graph_seq(q.device) if p_drop > 0 else (0, None)
        L.flash_fwd_ext(_ptr(q), _ptr(k), _ptr(v), _ptr(o), _ptr(lse), B, H, Sq, Sk, D, st, float(scale),
                        int(causal), _dt(q), _ptr(cu_q) if varlen else 0, _ptr(cu_k) if varlen else 0,
                        _ptr(mk) if mk is not None else 0, msb, msh, msq, int(m32), float(p_drop),
                        int(seed), int(offset), _ptr(dbits) if dbits.numel() else 0, dseq, _stream())
        ctx.save_for_backward(q, k, v, o, lse, mk if mk is not None else torch.empty(0), cu_q if varlen else
                              torch.empty(0), cu_k if varlen else torch.empty(0), dbits)
        ctx.meta = (varlen, B, H, D, Sq, Sk, st, causal, scale, p_drop, seed, offset,
                    (msb, msh, msq, m32) if mk is not None else None)
        return o

    @staticmethod
    def backward(ctx, do):
        dq, dk, dv = _fa_ext_backward(ctx, do)
        return dq, dk, dv, None, None, None, None, None, None, None, None, None, None


def _fa_ext_backward(ctx, do, outs=None, bsum=None):
    """dq, dk, dv of FlashAttnExtFn (into ``outs`` = (dq, dk, dv) views when given, dense only;
    ``bsum``: packed-QKV bias partials as in _fa_bwd_hip, dense self-attention only)."""
    q, k, v, o, lse, mk, cu_q, cu_k, dbits = ctx.saved_tensors
    varlen, B, H, D, Sq, Sk, st, causal, scale, p_drop, seed, offset, mmeta = ctx.meta
    L = _native.lib()
    do = _like(do, q.dtype).contiguous()
    delta = torch.empty((B, H, Sq), device=q.device, dtype=torch.float32)
    if varlen:
        dd = (do.float() * o.float()).sum(-1)                     # [total, H]
        lens = (cu_q[1:] - cu_q[:-1]).long()
        bidx = torch.repeat_interleave(torch.arange(B, device=q.device), lens)
        qidx = torch.arange(q.shape[0], device=q.device) - cu_q.long()[bidx]
        delta.view(B, H, Sq).permute(0, 2, 1)[bidx, qidx] = dd
        dq = torch.empty_like(q)
        dk = torch.empty_like(k)
        dv = torch.empty_like(v)
        gst = st + [0, dq.stride(0), dq.stride(1), 0, dk.stride(0), dk.stride(1), 0, dv.stride(0),
                    dv.stride(1)]
    else:
        L.flash_bwd_pre(_ptr(o), _ptr(do), _ptr(delta), B, H, Sq, D, _dt(q), _stream())
        if outs is not None:
            dq, dk, dv = outs
        else:
            dq = torch.empty((B, Sq, H, D), device=q.device, dtype=q.dtype)
            dk = torch.empty((B, Sk, H, D), device=q.device, dtype=q.dtype)
            dv = torch.empty((B, Sk, H, D), device=q.device, dtype=q.dtype)
        gst = st + [dq.stride(0), dq.stride(1), dq.stride(2), dk.stride(0), dk.stride(1), dk.stride(2),
                    dv.stride(0), dv.stride(1), dv.stride(2)]
    ds = torch.empty(B * H * (-(-Sk // 128) * 128) * (-(-Sq // 256) * 256), device=q.device,
                     dtype=q.dtype)
    msb, msh, msq, m32 = mmeta if mmeta is not None else (0, 0, 0, False)
    L.flash_bwd_ext(_ptr(q), _ptr(k), _ptr(v), _ptr(do), _ptr(lse), _ptr(delta), _ptr(dq), _ptr(dk),
                    _ptr(dv), _ptr(ds), B, H, Sq, Sk, D, gst, float(scale), int(causal), _dt(q),
                    _ptr(cu_q) if varlen else 0, _ptr(cu_k) if varlen else 0,
                    _ptr(mk) if mmeta is not None else 0, msb, msh, msq, int(m32), float(p_drop),
                    int(seed), int(offset), _ptr(dbits) if dbits.numel() else 0, 0, _stream(),
                    _ptr(bsum) if (bsum is not None and not varlen and Sq == Sk) else 0)
    return dq, dk, dv


class FlashAttnExtQKVFn(torch.autograd.Function):
    """FlashAttnExtFn on a packed qkv [B, S, 3, H, D] (the fused QKV projection's output): the
    backward writes dq / dk / dv straight into one packed gradient (no stack of three grads)."""

    @staticmethod
    def forward(ctx, qkv, mask, causal, scale, p_drop, seed, offset):
        q, k, v = qkv.unbind(2)
        S = qkv.shape[1]
        return FlashAttnExtFn.forward(ctx, q, k, v, mask, None, None, S, S, causal, scale, p_drop, seed, offset)

    @staticmethod
    def backward(ctx, do):
        dqkv = torch.empty(ctx.saved_tensors[0].shape[:2] + (3,) + ctx.saved_tensors[0].shape[2:],
                           device=do.device, dtype=ctx.saved_tensors[0].dtype)
        part = _qkv_bias_part(dqkv)
        _fa_ext_backward(ctx, do, dqkv.unbind(2), bsum=part)
        if part is not None:
            _tag_bias_part(dqkv, part)
        return dqkv, None, None, None, None, None, None


def _fa_ext_ok(q, k, v):
    return (q.is_cuda and _native.available() and q.dtype in (torch.bfloat16, torch.float16) and
            q.shape[-1] in (64, 128) and q.stride(-1) == 1 and k.stride(-1) == 1 and
            v.stride(-1) == 1 and k.dtype == q.dtype and v.dtype == q.dtype)


def flash_attention_ext(q, k, v, causal=False, scale=None, attn_mask=None, dropout=0.0, seed=None):
    """[B, S, H, D] flash attention with an optional additive ``attn_mask`` (broadcastable to
    [B, H, Sq, Sk]; a bool mask means keep=True) and in-kernel dropout on the probabilities."""
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    B, Sq, H, _ = q.shape
    Sk = k.shape[1]
    if attn_mask is not None and attn_mask.dtype == torch.bool:
        attn_mask = torch.zeros(attn_mask.shape, dtype=q.dtype, device=q.device).masked_fill(
            ~attn_mask, float('-inf'))
    if attn_mask is not None and attn_mask.dtype not in (q.dtype, torch.float32):
        attn_mask = attn_mask.to(q.dtype)
    if _fa_ext_ok(q, k, v):
        sd, off = _fa_next_rng(seed) if dropout > 0 else (0, 0)
        R._STATS[('flash_attn_ext', 'hip')] += 1
        return FlashAttnExtFn.apply(q, k, v, attn_mask, None, None, Sq, Sk, causal, scale,
                                    float(dropout), sd, off)
    if q.is_cuda and seed is None:
        # outside what the kernel covers (head_dim not 64/128, fp32, strided inputs) and no
        # bit-exact dropout requested: torch's memory-efficient SDPA, never the O(S^2) fp32
        # reference that keeps scores, probabilities and mask alive for autograd
        R._STATS[('flash_attn_ext', 'sdpa')] += 1
        qt, kt, vt = (t.transpose(1, 2) for t in (q, k, v))
        am = None if attn_mask is None else attn_mask.to(q.dtype)
        if causal and am is not None:  # mask + causal: fold the causal part into the mask
            cm = torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).triu(Sk - Sq + 1)
            am = am.masked_fill(cm, float('-inf'))
        o = torch.nn.functional.scaled_dot_product_attention(
            qt, kt, vt, attn_mask=am, dropout_p=float(dropout), is_causal=bool(causal) and am is None,
            scale=scale)
        return o.transpose(1, 2)
    sd, off = _fa_next_rng(seed) if dropout > 0 else (0, 0)
    R._STATS[('flash_attn_ext', 'ref')] += 1
    o, _ = _fa_ext_ref_dense(q, k, v, causal, scale, attn_mask, dropout, sd, off)
    return o.to(q.dtype)


def flash_attention_ext_qkvpacked(qkv, causal=False, scale=None, attn_mask=None, dropout=0.0, seed=None):
    """flash_attention_ext on a packed qkv [B, S, 3, H, D] -> o [B, S, H, D]."""
    if scale is None:
        scale = 1.0 / math.sqrt(qkv.shape[-1])
    q, k, v = qkv.unbind(2)
    if not _fa_ext_ok(q, k, v) or (attn_mask is not None and attn_mask.dtype == torch.bool):
        return flash_attention_ext(q, k, v, causal, scale, attn_mask, dropout, seed)
    if attn_mask is not None and attn_mask.dtype not in (qkv.dtype, torch.float32):
        attn_mask = attn_mask.to(qkv.dtype)
    sd, off = _fa_next_rng(seed) if dropout > 0 else (0, 0)
    R._STATS[('flash_attn_ext', 'hip')] += 1
    return FlashAttnExtQKVFn.apply(qkv, attn_mask, causal, scale, float(dropout), sd, off)


def flash_attn_varlen(q, k, v, cu_q, cu_k, max_sq, max_sk, causal=False, scale=None, dropout=0.0,
                      seed=None):
    """Packed variable-length attention (paddle flash_attn_unpadded): q [total_q, H, D],
    k/v [total_k, H, D], cu_q/cu_k [B+1] row prefix sums; sequence b attends only inside itself."""
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    cu_q = cu_q.to(device=q.device, dtype=torch.int32).contiguous()
    cu_k = cu_k.to(device=q.device, dtype=torch.int32).contiguous()
    sd, off = _fa_next_rng(seed) if dropout > 0 else (0, 0)
    if _fa_ext_ok(q, k, v):
        R._STATS[('flash_attn_varlen', 'hip')] += 1
        return FlashAttnExtFn.apply(q, k, v, None, cu_q, cu_k, int(max_sq), int(max_sk), causal, scale,
                                    float(dropout), sd, off)
    R._STATS[('flash_attn_varlen', 'ref')] += 1
    return flash_attn_varlen_ref(q, k, v, cu_q, cu_k, causal, scale, dropout, sd, off)


def flash_attn_varlen_ref(q, k, v, cu_q, cu_k, causal, scale, dropout=0.0, seed=0, offset=0):
    """Per-sequence dense fp32 reference of the varlen kernel (same dropout bits)."""
    outs = []
    H = q.shape[1]
    cq, ck = cu_q.tolist(), cu_k.tolist()
    for b in range(len(cq) - 1):
        qs, ks, vs = q[cq[b]:cq[b + 1]], k[ck[b]:ck[b + 1]], v[ck[b]:ck[b + 1]]
        bh0 = torch.arange(b * H, (b + 1) * H, device=q.device)
        o, _ = _fa_ext_ref_dense(qs[None], ks[None], vs[None], causal, scale, None, dropout, seed, offset,
                                 bh0=bh0)
        outs.append(o[0])
    return torch.cat(outs, 0).to(q.dtype)


# =============================================================================
# MFMA GEMM (ops/csrc/gemm_lds.hip): the training GEMMs of every Linear
# =============================================================================
GEMM_FWD, GEMM_NT, GEMM_TN = 0, 1, 2  # x·W, dy·Wᵀ (or h·Eᵀ), xᵀ·dy
EPI = {None: 0, 'gelu': 1, 'gelu_tanh': 2, 'relu': 3, 'dgelu': 4, 'dgelu_tanh': 5,
       # forward GELU whose z output receives gelu'(pre-activation) (x·W only), and the dgrad
       # epilogue that multiplies by that saved derivative (dy·Wᵀ only)
       'gelu_d': 6, 'gelu_tanh_d': 7, 'mulz': 8}
# PRA_GEMM: 'auto' (default) = the in-tree MFMA kernel for every layout/epilogue where it measured
# at or above hipBLASLt on MI355X (forward x·W incl. the fused bias+GELU epilogue, wgrad xᵀ·dy with
# beta=1 accumulation), hipBLASLt for the dgrad dy·Wᵀ layout where it is still faster
# (profiles/r2_gemm/summary.md); 'mfma' = in-tree kernel everywhere; 'blas' = hipBLASLt everywhere.
_GEMM_MODE = __import__('os').environ.get('PRA_GEMM', 'auto')
_GEMM_SHAPE_POLICY = __import__('os').environ.get('PRA_GEMM_POLICY', '1') == '1'


def _gemm_operand_ok(t):
    return t.is_cuda and t.dtype in (torch.bfloat16, torch.float16) and t.dim() == 2 and \
        t.stride(1) == 1 and t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0


@R.register_kernel('gemm', 'ref')
def _gemm_ref(layout, a, b, out=None, bias=None, z=None, epi=None, beta=0, want_colsum=False):
    af, bf = a.float(), b.float()
    y = af @ bf if layout == GEMM_FWD else (af @ bf.t() if layout == GEMM_NT else af.t() @ bf)
    if bias is not None:
        y = y + bias.float()
    cs = None
    if epi == 'mulz':
        y = y * z.float()
    elif epi in ('gelu_d', 'gelu_tanh_d'):
        yf = y.detach().requires_grad_(True)
        with torch.enable_grad():
            g = torch.nn.functional.gelu(yf, approximate='tanh' if epi == 'gelu_tanh_d' else 'none')
            d, = torch.autograd.grad(g.sum(), yf)
        z.copy_(d.to(z.dtype))
        y = g.detach()
    elif epi in ('dgelu', 'dgelu_tanh'):
        zf = z.float().requires_grad_(True)
        with torch.enable_grad():
            g = torch.nn.functional.gelu(zf, approximate='tanh' if epi == 'dgelu_tanh' else 'none')
            d, = torch.autograd.grad(g, zf, y)
        y = d
    elif epi is not None:
        if z is not None:
            z.copy_(y.to(z.dtype))
        y = torch.nn.functional.gelu(y, approximate='tanh' if epi == 'gelu_tanh' else 'none') \
            if epi.startswith('gelu') else torch.relu(y)
    if beta and out is not None:
        y = y + out.float()
    yo = y.to(a.dtype)
    if want_colsum:
        cs = yo.float().sum(0)
    if out is not None:
        out.copy_(yo)
        yo = out
    return (yo, cs) if want_colsum else yo


@R.register_kernel('gemm', 'hip', dtypes=_HALF)
def _gemm_hip(layout, a, b, out=None, bias=None, z=None, epi=None, beta=0, want_colsum=False):
    """One MFMA GEMM launch (+ split-K reduce when the tile grid would leave CUs idle).
    Returns None when the shape/layout is outside what the kernel assumes (caller falls back)."""
    if _GEMM_MODE == 'blas' or not (_gemm_operand_ok(a) and _gemm_operand_ok(b)) or a.dtype != b.dtype:
        return None
    persist = (layout == GEMM_NT and ((_GEMM_MODE == 'auto' and _nt_in_tree(a, b)) or
                                      (epi == 'mulz' and _MLP_MULZ_PTS))) or \
        (layout == GEMM_FWD and epi in ('gelu_d', 'gelu_tanh_d') and _MLP_MULZ_PTS) or \
        (layout == GEMM_FWD and epi is None and _FWD_LONGK_PTS and a.shape[1] >= 4096)
    if _GEMM_MODE == 'auto' and layout == GEMM_NT and not persist and epi != 'mulz' and \
            not (_MLP_DGELU_EPI and epi in ('dgelu', 'dgelu_tanh')):
        return None
    if epi in ('gelu_d', 'gelu_tanh_d') and layout != GEMM_FWD or epi == 'mulz' and layout != GEMM_NT:
        return None
    if layout == GEMM_FWD:
        M, K = a.shape
        N = b.shape[1]
    elif layout == GEMM_NT:
        M, K = a.shape
        N = b.shape[0]
    else:
        K, M = a.shape
        N = b.shape[1]
    if _GEMM_MODE == 'auto' and _GEMM_SHAPE_POLICY and epi is None and not want_colsum:
        # per-shape policy from the measured table (profiles/r3_gemm/gemm_configs.log): the
        # in-tree kernel is at parity or ahead on the long-K forward (fc2 x·W K=8192: 407-409
        # vs 410 us; LM-head dgrad K=50304: 2435-2444 vs 2458 us) and within 2-4 % on the
        # mid-size split-K wgrad (qkv 2048x6144: 381-388 vs 374 us), so those stay in-tree;
        # skinny decode-time forwards (M < 128: a 256-row tile idles) go to the library
        if layout == GEMM_FWD and M < 128:
            return None
    if out is None:
        out = torch.empty((M, N), device=a.device, dtype=a.dtype)
    elif not _gemm_operand_ok(out) or out.dtype != a.dtype or tuple(out.shape) != (M, N):
        return None
    if z is not None and (not _gemm_operand_ok(z) or tuple(z.shape) != (M, N)):
        return None
    if bias is not None and (bias.dtype != a.dtype or not bias.is_contiguous()):
        bias = bias.to(a.dtype).contiguous()
    L = _native.lib()
    e = EPI[epi]
    part = None
    if want_colsum:
        part = torch.empty(((M + 255) // 256, N), device=a.device, dtype=torch.float32)
    splits = 1 if (want_colsum or e >= 4 or out.stride(0) != N) else L.gemm_lds_splits(M, N, K)
    ws = torch.empty((splits, M, N), device=a.device, dtype=torch.float32) if splits > 1 else None
    try:
        L.gemm_lds(layout, a.data_ptr(), b.data_ptr(), _ptr(bias), out.data_ptr(), _ptr(z), _ptr(part),
                   M, N, K, a.stride(0), b.stride(0), out.stride(0), N if z is None else z.stride(0),
                   _dt(a), e | (_PERSIST_BIT if persist else 0), int(beta), splits, _ptr(ws), _stream())
    except ValueError:
        return None
    if want_colsum == 'part':
        return out, part      # [ceil(M/256), N] fp32 per-tile-row column sums
    if want_colsum:
        cs = torch.empty(N, device=a.device, dtype=torch.float32)
        L.colsum_partials(part.data_ptr(), cs.data_ptr(), part.shape[0], N, 0, _stream())
        return out, cs
    return out


# dy·Wᵀ shape policy (PRA_GEMM_NT_SHORTK=0 turns it off): with a short contraction (K <= 1024:
# BERT-base's 768-wide dgrads and the MLM head's h·Eᵀ) the in-tree persistent kernel (one
# workgroup per CU walking its tiles, next tile's DMA under the epilogue) measured ahead of
# hipBLASLt: 22.5 / 61.6 / 98.5 us vs 24.5 / 63.6 / 130.9 us (profiles/r4/gemm_pts_bert.log);
# at GPT-1.3B's K = 2048..8192 hipBLASLt's stream-K kernel stays ahead (gemm_pts_15shapes.log).
_NT_SHORTK = __import__('os').environ.get('PRA_GEMM_NT_SHORTK', '1') == '1'
# long-K x·W (GPT's fc2 forward, K = 8192) on the persistent 4-wave kernel: 385.1 vs 394.5 us per-tile
# (scripts/r6_fwd_policy_probe.py); PRA_GEMM_FWD_LONGK_PTS=0 keeps the per-tile kernel (A/B)
_FWD_LONGK_PTS = __import__('os').environ.get('PRA_GEMM_FWD_LONGK_PTS', '1') == '1'
_PERSIST_BIT = 256


# (PRA_GEMM_NT_MAXK: the bound. Round 5 measured 3072 -- BERT's 2304 / 3072-deep dgrads and
# GPT's 2048-deep out-projection dgrad, at parity in isolation -- 0.3 % slower in both steps:
# GPT 130.80 / 130.63 vs 130.41 / 130.33 ms, BERT 16.93 / 16.95 vs 16.87 / 16.86 ms,
# profiles/r5/nt_maxk_ab.log)
_NT_MAXK = int(__import__('os').environ.get('PRA_GEMM_NT_MAXK', '1024'))


def _nt_in_tree(a, b):
    K = a.shape[1]
    return _NT_SHORTK and a.dtype == torch.bfloat16 and 256 <= K <= _NT_MAXK and K % 128 == 0


def gemm(layout, a, b, out=None, bias=None, z=None, epi=None, beta=0, want_colsum=False):
    """C (=|+=) epi(op(a)·op(b) + bias). layout: GEMM_FWD a[M,K]·b[K,N]; GEMM_NT a[M,K]·b[N,K]ᵀ;
    GEMM_TN a[K,M]ᵀ·b[K,N]. On the device this is the in-tree MFMA kernel; shapes it does not
    take (K % 64, ragged strides) go to hipBLASLt through torch and are counted as 'gemm'/'ref'."""
    if a.is_cuda and R.select_backend(a, 'gemm') == 'hip':
        r = _gemm_hip(layout, a, b, out, bias, z, epi, beta, want_colsum)
        if r is not None:
            return r
        R._STATS[('gemm', 'hipblaslt' if _GEMM_MODE == 'auto' and layout == GEMM_NT else 'fallback')] += 1
    return _gemm_ref_fast(layout, a, b, out, bias, z, epi, beta, want_colsum)


def _gemm_ref_fast(layout, a, b, out, bias, z, epi, beta, want_colsum):
    """Library path (hipBLASLt via torch on the device, BLAS on the host) for what the MFMA
    kernel does not take; epilogues composed."""
    if epi is None and not want_colsum:
        bb = b.t() if layout == GEMM_NT else b
        aa = a if layout != GEMM_TN else a.t()
        if out is not None and beta:
            if bias is not None:
                out.add_(bias)
            return out.addmm_(aa, bb)
        y = torch.addmm(bias, aa, bb) if bias is not None else torch.mm(aa, bb)
        if out is not None:
            out.copy_(y)
            return out
        return y
    return _gemm_ref(layout, a, b, out, bias, z, epi, beta, want_colsum)


# =============================================================================
# 1x1 convolution (channels-last) as GEMMs: y = x·Wᵀ (hipBLASLt NT), dx = dy·W (in-tree MFMA
# GEMM), dW = dyᵀ·x (in-tree MFMA GEMM, split-K over K = N·H·W). Parity: the reference's
# conv2d with 1x1 filters (phi conv kernels); stride-2 1x1 (ResNet downsample) reads the
# strided positions and scatters dx back.
# =============================================================================
class GradJoin:
    """Gradient join for a tensor consumed by several fused ops (a residual block's input: the
    first 1x1 conv, the downsample conv and the residual input of the last BN+add+ReLU).
    Instead of each op returning its own full-size gradient and autograd summing them with
    separate add kernels, every contributor adds into one pending buffer (1x1 dgrad through
    the GEMM's beta=1 epilogue, a strided conv into its sampled positions, BN's dz as the
    initial buffer) and only the LAST contributor to run backward returns the total; the
    others return None. Contributors register in forward, so the count is exact."""

    __slots__ = ('x', 'n', 'left', 'pending', 'deferred')

    def __init__(self, x):
        self.x, self.n, self.left, self.pending, self.deferred = x, 0, None, None, []

    def _finish(self):
        if self.left is None:
            self.left = self.n
        self.left -= 1
        if self.left == 0:
            out, self.pending = self.pending, None
            # strided contributions that arrived before any full-size buffer existed are added
            # into their sampled positions of the final buffer (no zero-filled full tensor
            # unless every contributor was strided)
            for dx2, xshape, sh, sw in self.deferred:
                if out is None:
                    out = torch.zeros(xshape, dtype=dx2.dtype, device=dx2.device)
                    out[:, ::sh, ::sw, :] = dx2
                else:
                    out[:, ::sh, ::sw, :] += dx2
            self.deferred = []
            self.left = None
            return out
        return None

    def add_gemm(self, dy2, w2, xshape):
        # the join's LAST term with a BatchNorm+ReLU (+ residual) producing x: the 1x1 dgrad runs
        # on the implicit-GEMM kernel with the kBnG epilogue, adding the pending sum first, so the
        # BN backward receives the masked total and its reductions (no reduce pass over it)
        left = self.n if self.left is None else self.left
        rec = _bn_handoff(self.x) if left == 1 and not self.deferred else None
        m, cout = dy2.shape
        cin = w2.shape[1]
        if (rec is not None and cout % 64 == 0 and cin % 8 == 0 and rec.x2.shape == (m, cin)
                and rec.x2.is_contiguous() and len(xshape) == 4
                and (self.pending is None or self.pending.is_contiguous()) and _bn_dgrad_ok(rec, m, cin, cout)):
            dy4 = dy2.view(*xshape[:3], cout)
            out = self.pending.view(xshape) if self.pending is not None else None
            self.pending = _bn_dgrad(rec, dy4, w2.t().contiguous(), 1, 1, 0, out=out).view(xshape)
            return self._finish()
        if self.pending is None:
            self.pending = gemm(GEMM_FWD, dy2, w2).view(xshape)
        else:
            gemm(GEMM_FWD, dy2, w2, out=self.pending.view(-1, w2.shape[1]), beta=1)
        return self._finish()

    def add_strided(self, dx2, xshape, sh, sw):
        if self.pending is None:
            self.deferred.append((dx2, xshape, sh, sw))
        else:
            self.pending[:, ::sh, ::sw, :] += dx2
        return self._finish()

    def add_tensor(self, g, owned):
        if self.pending is None:
            self.pending = g if owned else g.clone()
        else:
            self.pending += g
        return self._finish()


_JOIN = [None]


class grad_join:
    """``with grad_join(x):`` — fused ops inside that consume ``x`` (the same tensor object)
    join their input gradients (see GradJoin). No-op without autograd."""

    def __init__(self, x):
        self.x = x

    def __enter__(self):
        self.prev = _JOIN[0]
        x = self.x
        ok = isinstance(x, torch.Tensor) and x.requires_grad and torch.is_grad_enabled() and x.is_cuda
        _JOIN[0] = GradJoin(x) if ok else None
        return _JOIN[0]

    def __exit__(self, *exc):
        _JOIN[0] = self.prev
        return False


def _join_for(t):
    j = _JOIN[0]
    if j is not None and t is j.x:
        j.n += 1
        return j
    return None


# BatchNorm(+ReLU) -> convolution gradient handoff. The BN backward's two reductions (sum of g and
# of g * (x - mean), g = the ReLU-masked incoming gradient) are produced by the epilogue of the
# convolution dgrad that computes that gradient (gemm_core.h kBnG), so the BN backward is the
# finalize + apply kernels only. BatchNormActFn tags its output with a _BnHandoff; a consumer
# conv whose backward runs on the implicit-GEMM kernel writes g and the partial sums into it; the
# BN backward uses them only when the gradient it receives IS that g, unmodified (same storage and
# version: a second consumer's gradient summed in by autograd lands in a new buffer or bumps the
# version), and otherwise runs its own reduction (masking g again is idempotent).
_BN_DGRAD_FUSE = __import__('os').environ.get('PRA_BN_DGRAD_FUSE', '1') == '1'
_BN_DGRAD_SPLIT = __import__('os').environ.get('PRA_BN_DGRAD_SPLIT', '0') == '1'


class _BnHandoff:
    __slots__ = ('x2', 'mask', 'mean', 'g', 'gver', 'part', 'used')

    def __init__(self, x2, mask, mean):
        self.x2, self.mask, self.mean = x2, mask, mean
        self.g = self.gver = self.part = None
        self.used = 0

    def take(self, dy2):
        """The epilogue partial sums if dy2 is the produced g, else None (either way cleared)."""
        g, part, ver = self.g, self.part, self.gver
        self.g = self.part = self.gver = None
        if (part is None or dy2.data_ptr() != g.data_ptr() or dy2._version != ver
                or dy2.shape != self.x2.shape):
            return None
        self.used += 1
        return part


def _bn_handoff(x):
    rec = getattr(x, '_pra_bn', None) if _BN_DGRAD_FUSE else None
    return rec if isinstance(rec, _BnHandoff) else None


def _bn_dgrad_ok(rec, m, cout_dgrad, k):
    """The fused dgrad runs without split-K; shapes the split would have served keep the plain
    dgrad unless PRA_BN_DGRAD_SPLIT=1."""
    return (rec is not None and rec.x2.shape == (m, cout_dgrad) and rec.x2.is_contiguous()
            and (_BN_DGRAD_SPLIT or _native.lib().conv_lds_splits(m, cout_dgrad, k) == 1))


def _bn_dgrad(rec, dy4, wk, kh, kw, pad, out=None):
    """dgrad on the implicit-GEMM kernel with the kBnG epilogue; stores g + partials in rec.
    out: a pending gradient the product is added to (in place) before the mask."""
    g, part = _conv_lds(dy4, wk, None, kh, kw, 1, pad, bn=(rec.x2, rec.mask, rec.mean), out=out)
    rec.g, rec.part, rec.gver = g, part, g._version
    return g


class Conv1x1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias, sh, sw, join=None):
        ctx.join = join
        ctx.bn = _bn_handoff(x) if (join is None and (sh, sw) == (1, 1) and bias is None) else None
        xs = x if (sh, sw) == (1, 1) else x[:, ::sh, ::sw, :]
        xs = xs.contiguous()
        n, h, wd, cin = xs.shape
        cout = w.shape[0]
        x2, w2 = xs.view(-1, cin), w.reshape(cout, cin)
        y = gemm(GEMM_NT, x2, w2, bias=None if bias is None else bias.to(x.dtype))
        ctx.save_for_backward(x2, w2)
        ctx.w = w
        ctx.meta = (tuple(x.shape), tuple(xs.shape), tuple(w.shape), sh, sw, bias is not None)
        return y.view(n, h, wd, cout)

    @staticmethod
    def backward(ctx, dy):
        x2, w2 = ctx.saved_tensors
        xshape, xsshape, wshape, sh, sw, hb = ctx.meta
        dy2 = dy.reshape(-1, w2.shape[0])
        if not dy2.is_contiguous() or dy2.data_ptr() % 16:
            dy2 = dy2.contiguous()
        dy2 = _like(dy2, x2.dtype)
        dx = dw = db = None
        rec = getattr(ctx, 'bn', None)
        m, cout = dy2.shape
        if (ctx.needs_input_grad[0] and rec is not None and cout % 64 == 0 and w2.shape[1] % 8 == 0
                and _bn_dgrad_ok(rec, m, w2.shape[1], cout)):
            dx = _bn_dgrad(rec, dy2.view(*xsshape[:3], cout), w2.t().contiguous(), 1, 1, 0).view(xshape)
        elif ctx.needs_input_grad[0]:
            j = ctx.join
            if j is not None and (sh, sw) == (1, 1):
                dx = j.add_gemm(dy2, w2, xshape)
            elif j is not None:
                dx = j.add_strided(gemm(GEMM_FWD, dy2, w2).view(xsshape), xshape, sh, sw)
            else:
                dx2 = gemm(GEMM_FWD, dy2, w2)
                if (sh, sw) == (1, 1):
                    dx = dx2.view(xshape)
                else:
                    dx = torch.zeros(xshape, dtype=dx2.dtype, device=dx2.device)
                    dx[:, ::sh, ::sw, :] = dx2.view(xsshape)
        if ctx.needs_input_grad[1]:
            g = ctx.w.grad
            if _acc_grad_ok(g, ctx.w, dy2.dtype):
                # dW accumulated into the existing gradient by the beta=1 epilogue (the weight's
                # AccumulateGrad node still runs and fires its post-accumulate hooks)
                gemm(GEMM_TN, dy2, x2, out=g.view(w2.shape), beta=1)
            else:
                dw = gemm(GEMM_TN, dy2, x2).view(wshape)
        if hb and ctx.needs_input_grad[2]:
            db = dy2.sum(0, dtype=torch.float32).to(dy2.dtype)
        return dx, dw, db, None, None, None


def conv1x1_nhwc(x, w, bias=None, stride=(1, 1)):
    return Conv1x1Fn.apply(x, w, bias, int(stride[0]), int(stride[1]), _join_for(x))


class Conv1x1StatsFn(torch.autograd.Function):
    """1x1 convolution whose forward also returns the BatchNorm partial statistics of its output:
    the forward runs on the implicit-GEMM conv kernel (kh = kw = 1; its epilogue emits the per-tile
    shifted sums / sums of squares, as ConvKxKStatsFn), so the BN statistics pass over the output
    disappears; the backward is Conv1x1Fn's (dgrad GEMM joined into the block input's gradient,
    wgrad accumulated in place)."""

    @staticmethod
    def forward(ctx, x, w, sh, sw, join, shift):
        ctx.join = join
        xs = x if (sh, sw) == (1, 1) else x[:, ::sh, ::sw, :]
        xs = xs.contiguous()
        n, h, wd, cin = xs.shape
        cout = w.shape[0]
        w2 = w.reshape(cout, cin)
        y, part = _conv_lds(xs, w2, None, 1, 1, 1, 0, stats_shift=shift)
        ctx.bn = _bn_handoff(x) if (join is None and (sh, sw) == (1, 1)) else None
        ctx.save_for_backward(xs.view(-1, cin), w2)
        ctx.w = w
        ctx.meta = (tuple(x.shape), tuple(xs.shape), tuple(w.shape), sh, sw, False)
        ctx.mark_non_differentiable(part)
        ctx.set_materialize_grads(False)   # (no zero-filled [2, rows, C] gradient for part)
        return y, part

    @staticmethod
    def backward(ctx, dy, dpart):
        if dy is None:
            return None, None, None, None, None, None
        dx, dw, _, _, _, _ = Conv1x1Fn.backward(ctx, dy)
        return dx, dw, None, None, None, None


_CONV1X1_STATS = __import__('os').environ.get('PRA_CONV1X1_STATS', '1') == '1'


def conv1x1_bn_stats_ok(x, w, stride, padding, rmean, training):
    """1x1 conv + BN statistics in the conv epilogue (conv_bn_act_nhwc): channels-last half
    input with C % 64 == 0 (the implicit-GEMM kernel's K step), fp32 running mean, HIP BN."""
    return bool(_CONV1X1_STATS and _CONV_BN_STATS and training and padding == 0 and rmean is not None
                and rmean.dtype == torch.float32 and rmean.is_contiguous() and rmean.numel() == w.shape[0]
                and tuple(w.shape[2:]) == (1, 1) and x.is_cuda and x.dim() == 4 and x.dtype in _HALF
                and w.dtype == x.dtype and x.shape[3] == w.shape[1] and x.shape[3] % 64 == 0
                and w.shape[0] % 8 == 0 and x.numel() * 2 < 2 ** 31
                and _conv1x1_stats_shape(x, w, stride)
                and R.select_backend(x, 'batch_norm_fwd') == 'hip')


def _conv1x1_stats_shape(x, w, stride):
    """Shapes where the fused path measured faster forward+backward than hipBLASLt + the separate
    statistics pass (profiles/r3g/conv1x1_bn_shapes.md, ResNet-50 bs 256): the 14x14 / 7x7 stages
    and the wide (>= 512 channel) 28x28 outputs; the 56x56 stage stays on the library GEMM."""
    if _CONV1X1_STATS_ALL:
        # round 5: with the finalize pre-merge and no zero-filled stats gradients the 56x56
        # stage joins too (ResNet-50 bs 256: 9137 / 9154 vs 8936 / 8943 img/s with the 56x56
        # forwards on hipBLASLt + the separate statistics pass, profiles/r5/resnet_conv1x1_all_ab.log)
        return True
    m = x.shape[0] * ((x.shape[1] - 1) // stride + 1) * ((x.shape[2] - 1) // stride + 1)
    return m <= 65536 or (m <= 262144 and w.shape[0] >= 512)


_CONV1X1_STATS_ALL = __import__('os').environ.get('PRA_CONV1X1_STATS_ALL', '1') == '1'


# =============================================================================
# KxK convolution (channels-last, groups 1, dilation 1) as an implicit GEMM on the LDS-DMA MFMA
# kernel (gemm_lds.hip ConvDmaA): the im2col rows are gathered from the NHWC input by the
# buffer LDS-DMA (padding = its range check), never materialised. Forward for any stride; the stride-1 input gradient is the
# same kernel on the padded output gradient with the flipped, in/out-transposed filter; the
# weight gradient (and strided input gradients) use MIOpen's convolution_backward.
# Parity: the reference's conv2d (phi gpudnn conv kernels) for ResNet's 3x3 layers.
# =============================================================================
def conv_kxk_supported(x, w, stride, padding):
    """Host-side shape check before any launch (the kernel assumes these)."""
    if not (x.is_cuda and x.dim() == 4 and w.dim() == 4 and x.dtype in _HALF and w.dtype == x.dtype):
        return False
    cin, cout = x.shape[3], w.shape[0]
    return (w.shape[1] == cin and cin % 64 == 0 and cout % 8 == 0 and stride >= 1 and padding >= 0
            and x.shape[1] + 2 * padding >= w.shape[2] and x.shape[2] + 2 * padding >= w.shape[3]
            and x.numel() * 2 < 2 ** 31 and max(x.shape[1], x.shape[2]) < 32768)


def _conv_lds(x, wk, bias, kh, kw, stride, pad, relu=False, stats_shift=None, cv=None, bn=None, out=None):
    """y[N,Ho,Wo,Cout] = conv(x NHWC, wk [Cout, kh*kw*C] (OHWI)) via the implicit-GEMM kernel
    (zero padding applied by the kernel's DMA range check, the input is read in place).
    stats_shift (fp32 [Cout], e.g. the BN running mean): the epilogue also returns the per-tile
    BatchNorm partial sums part [2, rows, Cout] of (y - shift) and (y - shift)^2.
    bn = (x2, mask, mean) of a BatchNorm+ReLU whose output this conv's dgrad is the gradient of:
    y = the product masked by the ReLU keep-bits, part = per-tile sums of y and y * (x2 - mean)
    (gemm_core.h kBnG), returned as (y, part). out (bn only): y is written in place and its
    current contents (a pending gradient) are added to the product before the mask."""
    n, h, wd, c = x.shape
    cout = wk.shape[0]
    x = x.contiguous()
    pp = 0
    if cv is not None and cv != c:
        # pixel-pitch mode (gemm_lds.hip ConvGeom::PP): taps of cv columns = cv // c adjacent pixels
        pp, c = c, cv
        ho, wo = (h - kh) // stride + 1, (wd - c // pp) // stride + 1
    else:
        ho, wo = (h + 2 * pad - kh) // stride + 1, (wd + 2 * pad - kw) // stride + 1
    if out is not None:
        assert bn is not None and out.is_contiguous() and out.numel() == n * ho * wo * cout and out.dtype == x.dtype
        y = out
    else:
        y = torch.empty((n, ho, wo, cout), device=x.device, dtype=x.dtype)
    if bias is not None and (bias.dtype != x.dtype or not bias.is_contiguous()):
        bias = bias.to(x.dtype).contiguous()
    L = _native.lib()
    m = n * ho * wo
    part = None
    bnx = bnm = 0
    if bn is not None:
        bx2, bmask, stats_shift = bn
        assert bx2.shape == (n * ho * wo, cout) and bmask.numel() * 8 == bx2.numel() and bias is None
        bnx, bnm = bx2.data_ptr(), bmask.data_ptr()
    if stats_shift is not None:
        splits = 1
        part = torch.empty((2, L.conv_lds_stat_rows(m, cout), cout), device=x.device, dtype=torch.float32)
    else:
        splits = L.conv_lds_splits(m, cout, kh * kw * c)
    ws = torch.empty((splits, m, cout), device=x.device, dtype=torch.float32) if splits > 1 else None
    L.conv_lds(x.data_ptr(), wk.data_ptr(), _ptr(bias), y.data_ptr(), n, h, wd, c, cout, kh, kw,
               stride, pad, int(relu), _dt(x), splits, _ptr(ws), _ptr(part), _ptr(stats_shift), pp, _stream(),
               bnx, bnm, int(out is not None))
    return y if stats_shift is None else (y, part)


def _conv_wgrad_ok(x, dy, cout):
    n, h, wd, c = x.shape
    # Cout <= 128 runs 128-row tiles (the 256-row tile idled 1/2 - 3/4 of its MFMA rows there and
    # lost to MIOpen at Cout 64: profiles/r3j/conv3x3_wgrad_shapes.md); PRA_CONV_WGRAD_NARROW=0
    # keeps those shapes on MIOpen for A/B
    narrow_ok = cout >= 256 or (_CONV_WGRAD_NARROW and cout % 64 == 0)
    return (_CONV_WGRAD == 'mfma' and c % 64 == 0 and narrow_ok and cout % 8 == 0
            and x.numel() * 2 < 2 ** 31
            and (dy.shape[0] * dy.shape[1] * dy.shape[2]) % 64 == 0 and max(h, wd) < 32768)


def _conv_wgrad_lds(dy, x, kh, kw, stride, pad, cv=None):
    """dW [Cout, kh, kw, C] (OHWI) = dyᵀ · im2col(x) on the implicit-GEMM kernel (split-K over
    the output pixels, im2col rows gathered by the DMA). cv: pixel-pitch mode (see _conv_lds)."""
    n, h, wd, c = x.shape
    pp = 0
    if cv is not None and cv != c:
        pp, c = c, cv
    cout = dy.shape[3]
    L = _native.lib()
    mpix = dy.shape[0] * dy.shape[1] * dy.shape[2]
    nk = kh * kw * c
    # fill ONE wave of <= 256 workgroups (a 257th starts a second round), each split >= 16
    # K-steps of 64 pixels (profiles/r2_conv/conv3x3_wgrad.log)
    rows = L.conv_wgrad_rows(cout)
    tiles = ((cout + rows - 1) // rows) * ((nk + 255) // 256)
    splits = max(1, min(256 // tiles, mpix // (64 * 16), 256)) if tiles < 224 else 1
    ws = torch.empty((splits, cout, nk), device=x.device, dtype=torch.float32) if splits > 1 else None
    dw = torch.empty((cout, kh, kw, c), device=x.device, dtype=x.dtype)
    L.conv_wgrad_lds(dy.data_ptr(), x.data_ptr(), dw.data_ptr(), n, h, wd, c, cout, kh, kw, stride, pad,
                     _dt(x), splits, _ptr(ws), pp, _stream())
    return dw


# weight gradient of KxK convs: 'mfma' = implicit GEMM on the in-tree kernel, 'miopen' = MIOpen
_CONV_WGRAD = __import__('os').environ.get('PRA_CONV_WGRAD', 'mfma')
_CONV_WGRAD_NARROW = __import__('os').environ.get('PRA_CONV_WGRAD_NARROW', '1') == '1'


# Strided (stride-2, 3x3, pad 1) input gradient as four sub-pixel phases on the implicit-GEMM
# kernel (gemm_lds.hip pra_conv_dgrad_phase): the transposed convolution's output pixel
# (2i + ph, 2j + pw) only meets filter taps ky with (ph + 1 - ky) even, at dy row offset
# (ph + 1 - ky) / 2 in {0, 1}; each phase is a stride-1 conv of dy with a 1x1 / 1x2 / 2x1 / 2x2
# sub-filter whose epilogue writes the phase's pixels of dx directly (every pixel exactly once, no
# zero fill, no interleave pass). Parity: the reference's strided conv2d_grad (phi gpudnn).
# Off by default: ResNet-50 bs 256 measured 8991 vs 9178 img/s against MIOpen's igemm_bwd (the
# per-phase K of 1-4 taps x Cout leaves each launch prologue/epilogue-bound; 56x56x128: 210 vs
# 173 us, 28x28x256: 125 vs 149 us, 14x14x512: 189 vs 141 us, profiles/r5/strided_dgrad_probe.md)
_STRIDED_DGRAD = __import__('os').environ.get('PRA_STRIDED_DGRAD', '0') == '1'
_S2_TAPS = {0: [(0, 1)], 1: [(0, 2), (1, 0)]}   # phase -> [(dy offset, filter tap)]
_S2_IDX = {}


def _s2_phase_index(w):
    """Gather index over w.flatten() of the four phase sub-filters (each [Cin, khp*kwp*Cout],
    OHWI over the phase's taps) concatenated, and the phase table (ph, pw, khp, kwp, off, numel)."""
    cout, cin, kh, kw = w.shape
    key = (cout, cin, w.device)
    if key not in _S2_IDX:
        ci = torch.arange(cin).view(cin, 1, 1, 1)
        co = torch.arange(cout).view(1, 1, 1, cout)
        parts, table, off = [], [], 0
        for ph in (0, 1):
            for pw in (0, 1):
                rows, cols = _S2_TAPS[ph], _S2_TAPS[pw]
                ky = torch.tensor([k for _, k in rows]).view(1, -1, 1, 1)
                kx = torch.tensor([k for _, k in cols]).view(1, 1, -1, 1)
                idx = ((co * cin + ci) * 3 + ky) * 3 + kx          # [cin, khp, kwp, cout]
                parts.append(idx.reshape(-1))
                table.append((ph, pw, len(rows), len(cols), off, idx.numel()))
                off += idx.numel()
        _S2_IDX[key] = (torch.cat(parts).to(w.device), table)
    return _S2_IDX[key]


def strided_dgrad_ok(x, dy, w, stride, pad):
    cout, cin, kh, kw = w.shape
    return (_STRIDED_DGRAD and stride == 2 and kh == kw == 3 and pad == 1 and dy.is_cuda
            and x.shape[1] == 2 * dy.shape[1] and x.shape[2] == 2 * dy.shape[2]
            and cout % 64 == 0 and cin % 8 == 0 and dy.dtype in _HALF and w.dtype == dy.dtype
            and dy.numel() * 2 < 2 ** 31 and x.numel() * 2 < 2 ** 31 and max(dy.shape[1], dy.shape[2]) < 32768)


def _conv_dgrad_s2(dy, w, xshape, rec=None):
    """dx [N, 2Ho, 2Wo, Cin] of a 3x3 / stride 2 / pad 1 conv from dy [N, Ho, Wo, Cout].
    rec (_BnHandoff of the BatchNorm+ReLU producing the conv input): every phase's epilogue
    applies the ReLU keep-bits and emits its BN partial sums (kBnG); stored into rec."""
    idx, table = _s2_phase_index(w)
    n, h, wd, cin = xshape
    _, ho, wo, cout = dy.shape
    dy = dy.contiguous()
    wcat = w.reshape(-1)[idx]
    dx = torch.empty(xshape, device=dy.device, dtype=dy.dtype)
    L = _native.lib()
    es = dx.element_size()
    parts = []
    for ph, pw, khp, kwp, off, cnt in table:
        pix = ph * wd + pw
        part = bnx = bnm = kshift = 0
        if rec is not None:
            pt = torch.empty((2, L.conv_lds_stat_rows(n * ho * wo, cin), cin), device=dy.device, dtype=torch.float32)
            parts.append(pt)
            part, kshift = pt.data_ptr(), rec.mean.data_ptr()
            bnx = rec.x2.data_ptr() + pix * cin * es
            bnm = rec.mask.data_ptr() + pix * cin // 8
        L.conv_dgrad_phase(dy.data_ptr(), wcat[off:off + cnt].data_ptr(), dx.data_ptr() + pix * cin * es, n, ho, wo,
                           cout, cin, khp, kwp, 2, _dt(dy), part, kshift, bnx, bnm, _stream())
    if rec is not None:
        rec.g, rec.part, rec.gver = dx, torch.cat(parts, 1), dx._version
    return dx


def _flip_t(w):
    """[Cin, kh*kw*Cout] filter of the stride-1 input gradient: w flipped in both taps, IHWO."""
    cout, cin, kh, kw = w.shape
    if w.is_cuda and w.is_contiguous() and w.dtype in _HALF:
        wf = torch.empty((cin, kh * kw * cout), device=w.device, dtype=w.dtype)
        _native.lib().wflip_t(w.data_ptr(), wf.data_ptr(), cout, cin, kh, kw, _dt(w), _stream())
        return wf
    return w.flip(2, 3).permute(1, 2, 3, 0).reshape(cin, kh * kw * cout).contiguous()


class ConvKxKFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias, stride, pad):
        cout, cin, kh, kw = w.shape
        x = x.contiguous()
        wk = w.permute(0, 2, 3, 1).reshape(cout, kh * kw * cin).contiguous()  # a view for channels-last w
        y = _conv_lds(x, wk, bias, kh, kw, stride, pad)
        ctx.save_for_backward(x, w)
        ctx.meta = (stride, pad, bias is not None)
        ctx.bn = _bn_handoff(x) if stride in (1, 2) else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        stride, pad, hb = ctx.meta
        cout, cin, kh, kw = w.shape
        dy = _like(dy.contiguous(), x.dtype)
        ours_dx = (ctx.needs_input_grad[0] and stride == 1 and cout % 64 == 0 and cin % 8 == 0
                   and kh - 1 - pad >= 0 and kw - 1 - pad >= 0 and kh == kw)
        dx = dw = db = None
        if ours_dx:
            wf = _flip_t(w)
            rec = getattr(ctx, 'bn', None)
            if _bn_dgrad_ok(rec, x.shape[0] * x.shape[1] * x.shape[2], cin, kh * kw * cout):
                dx = _bn_dgrad(rec, dy, wf, kh, kw, kh - 1 - pad)
            else:
                dx = _conv_lds(dy, wf, None, kh, kw, 1, kh - 1 - pad)
        if ctx.needs_input_grad[0] and not ours_dx and strided_dgrad_ok(x, dy, w, stride, pad):
            rec = getattr(ctx, 'bn', None)
            ok = (rec is not None and rec.x2.shape == (x.shape[0] * x.shape[1] * x.shape[2], cin)
                  and rec.x2.is_contiguous())
            dx = _conv_dgrad_s2(dy, w, x.shape, rec if ok else None)
            ours_dx = True
        need_lib_dx = ctx.needs_input_grad[0] and not ours_dx
        ours_dw = ctx.needs_input_grad[1] and _conv_wgrad_ok(x, dy, cout)
        if ours_dw:
            dwk = _conv_wgrad_lds(dy, x, kh, kw, stride, pad)
            g = w.grad
            if _acc_grad_ok(g, w, dwk.dtype):
                # accumulated straight from the OHWI product (no OIHW copy before the add); the
                # AccumulateGrad node still fires its post-accumulate hooks
                g.add_(dwk.permute(0, 3, 1, 2))
            else:
                dw = dwk.permute(0, 3, 1, 2).contiguous()
        need_lib_dw = ctx.needs_input_grad[1] and not ours_dw
        if need_lib_dx or need_lib_dw:
            # NCHW-shaped views of the channels-last tensors: MIOpen runs its NHWC kernels
            gx, gw, _ = torch.ops.aten.convolution_backward(
                dy.permute(0, 3, 1, 2), x.permute(0, 3, 1, 2), w, None, [stride, stride], [pad, pad],
                [1, 1], False, [0, 0], 1, [need_lib_dx, need_lib_dw, False])
            if need_lib_dx:
                dx = gx.permute(0, 2, 3, 1).contiguous()
            if need_lib_dw:
                dw = gw
        if hb and ctx.needs_input_grad[2]:
            db = dy.reshape(-1, cout).sum(0, dtype=torch.float32).to(dy.dtype)
        return dx, dw, db, None, None


class ConvKxKStatsFn(ConvKxKFn):
    """ConvKxKFn whose forward also returns the BatchNorm partial statistics of its output
    (the implicit-GEMM epilogue's column sums around ``shift``; non-differentiable)."""

    @staticmethod
    def forward(ctx, x, w, bias, stride, pad, shift):
        cout, cin, kh, kw = w.shape
        x = x.contiguous()
        wk = w.permute(0, 2, 3, 1).reshape(cout, kh * kw * cin).contiguous()
        y, part = _conv_lds(x, wk, bias, kh, kw, stride, pad, stats_shift=shift)
        ctx.save_for_backward(x, w)
        ctx.meta = (stride, pad, bias is not None)
        ctx.bn = _bn_handoff(x) if stride in (1, 2) else None
        ctx.mark_non_differentiable(part)
        ctx.set_materialize_grads(False)   # (no zero-filled [2, rows, C] gradient for part)
        return y, part

    @staticmethod
    def backward(ctx, dy, dpart):
        if dy is None:
            return (None,) * 6
        return ConvKxKFn.backward(ctx, dy) + (None,)


# =============================================================================
# Narrow-input stride-2 convolution (the ResNet stem: 7x7/2 over 3 channels) as a stride-1
# convolution over the 2x2 space-to-depth image (16 channels, zero-padded), on the implicit-GEMM
# kernel in pixel-pitch mode: a row of ceil(K/2) taps x 16 channels is ONE contiguous 128-B
# segment, so the LDS-DMA gathers it like a 64-channel tap (gemm_lds.hip ConvGeom::PP). The
# reference runs this layer on cuDNN (phi gpudnn conv kernels); here no library conv is left.
# =============================================================================
_S2D_CO = 16


def stem_conv_supported(x, w, stride, padding):
    if not (x.is_cuda and x.dim() == 4 and w.dim() == 4 and x.dtype in _HALF and w.dtype == x.dtype):
        return False
    cout, cin, kh, kw = w.shape
    kt = (kh + 1) // 2
    n, h, wd, c = x.shape
    return (stride == 2 and kh == kw and c == cin and 4 * cin <= _S2D_CO and kt * _S2D_CO == 64
            and cout % 8 == 0 and (h + 2 * padding) % 2 == 0 and (wd + 2 * padding) % 2 == 0
            and (h + 2 * padding - kh) // 2 + 1 == (h + 2 * padding) // 2 - kt + 1
            and (wd + 2 * padding - kw) // 2 + 1 == (wd + 2 * padding) // 2 - kt + 1
            and n * ((h + 2 * padding) // 2) * ((wd + 2 * padding) // 2) * _S2D_CO * 2 < 2 ** 31)


_STEM_IDX = {}


def _stem_index(w):
    """Gather index of the stride-1 filter [Cout, kt, 1, kt*16] over w.flatten() (-1: zero tap):
    w'[o][KY][kx*16 + (2dy+dx)*Cin + c] = w[o][c][2KY+dy][2kx+dx]."""
    cout, cin, kh, kw = w.shape
    key = (cout, cin, kh, kw, w.device)
    idx = _STEM_IDX.get(key)
    if idx is None:
        kt = (kh + 1) // 2
        idx = torch.full((cout, kt, kt * _S2D_CO), -1, dtype=torch.long)
        for KY in range(kt):
            for kx in range(kt):
                for dy in range(2):
                    for dx in range(2):
                        ky, kxx = 2 * KY + dy, 2 * kx + dx
                        if ky >= kh or kxx >= kw:
                            continue
                        for c in range(cin):
                            col = kx * _S2D_CO + (2 * dy + dx) * cin + c
                            idx[:, KY, col] = torch.arange(cout) * cin * kh * kw + (c * kh + ky) * kw + kxx
        idx = _STEM_IDX[key] = idx.to(w.device)
    return idx


def _stem_inverse(idx, numel):
    """Position in idx of every filter element (each appears exactly once): the weight gradient
    is then one gather, no boolean mask (graph-capturable, no host sync)."""
    key = ('inv', idx.data_ptr(), numel)
    inv = _STEM_IDX.get(key)
    if inv is None:
        flat = idx.reshape(-1).cpu()
        pos = torch.nonzero(flat >= 0).squeeze(1)
        inv_h = torch.empty(numel, dtype=torch.long)
        inv_h[flat[pos]] = pos
        inv = _STEM_IDX[key] = inv_h.to(idx.device)
    return inv


class StemConvFn(torch.autograd.Function):
    """y = conv2d(x, w, stride 2, padding p) for a narrow channels-last input, through the
    space-to-depth stride-1 form; optional BN partial statistics of y (epilogue column sums
    around ``shift``). dx is not formed (the stem's input is data); dW = dyᵀ · im2col(s2d(x))
    on the weight-gradient kernel, scattered back to [Cout, Cin, K, K]."""

    @staticmethod
    def forward(ctx, x, w, pad, shift):
        n, h, wd, c = x.shape
        cout, cin, kh, kw = w.shape
        kt = (kh + 1) // 2
        L = _native.lib()
        hs, ws = (h + 2 * pad) // 2, (wd + 2 * pad) // 2
        xs = torch.empty((n, hs, ws, _S2D_CO), device=x.device, dtype=x.dtype)
        L.space_to_depth2(x.data_ptr(), xs.data_ptr(), n, h, wd, c, pad, _S2D_CO, _dt(x), _stream())
        idx = _stem_index(w)
        wflat = w.reshape(-1)
        wk = torch.where(idx >= 0, wflat[idx.clamp(min=0)], torch.zeros((), dtype=w.dtype, device=w.device))
        wk = wk.reshape(cout, kt * kt * _S2D_CO).contiguous()
        r = _conv_lds(xs, wk, None, kt, 1, 1, 0, stats_shift=shift, cv=kt * _S2D_CO)
        ctx.save_for_backward(xs, idx, x, w)
        ctx.inv = _stem_inverse(idx, w.numel())
        ctx.meta = (kt, w.shape, pad)
        if shift is None:
            return r, None
        y, part = r
        ctx.mark_non_differentiable(part)
        ctx.set_materialize_grads(False)   # (no zero-filled [2, rows, C] gradient for part)
        return y, part

    @staticmethod
    def backward(ctx, dy, dpart):
        if dy is None:
            return None, None, None, None
        xs, idx, x, w = ctx.saved_tensors
        kt, wshape, pad = ctx.meta
        dw = None
        if ctx.needs_input_grad[1]:
            dy = dy.contiguous()
            if (dy.shape[0] * dy.shape[1] * dy.shape[2]) % 64 == 0:
                dwk = _conv_wgrad_lds(dy, xs, kt, 1, 1, 0, cv=kt * _S2D_CO).reshape(-1)
                dw = dwk[ctx.inv].view(wshape)
            else:   # the weight-gradient kernel walks the output pixels 64 at a time
                _, dw, _ = torch.ops.aten.convolution_backward(
                    dy.permute(0, 3, 1, 2), x.permute(0, 3, 1, 2), w, None, [2, 2], [pad, pad], [1, 1],
                    False, [0, 0], 1, [False, True, False])
        assert not ctx.needs_input_grad[0], "stem conv: input gradient not supported on this path"
        return None, dw, None, None


def stem_conv_nhwc(x, w, padding):
    return StemConvFn.apply(x, w, int(padding), None)[0]


def conv_bn_act_nhwc(x, w, stride, padding, bn_w, bn_b, rmean, rvar, training, momentum=0.9,
                     eps=1e-5, z=None, relu=True):
    """act(BN(conv(x)) [+ z]) for channels-last KxK convolutions with the BatchNorm statistics
    taken in the convolution's epilogue (parity: the reference's fused conv + BN-statistics
    kernels, fluid/operators/fused/cudnn_norm_conv.cu.h / resnet_unit_op.cu): the separate
    statistics pass over the conv output disappears; finalize + apply (+ residual + ReLU
    keep-bits) run as in ``batch_norm_act``. Falls back to conv + batch_norm_act when the
    shape is outside the kernel or statistics are not needed (eval)."""
    if conv_bn_stats_ok(x, w, stride, padding, rmean, training):
        y, part = ConvKxKStatsFn.apply(x, w, None, int(stride), int(padding), rmean)
        return BatchNormActFn.apply(y, z, bn_w, bn_b, rmean, rvar, training, momentum, eps, relu,
                                    _join_for(z) if z is not None else None, (part, rmean))
    if (_STEM_S2D and not x.requires_grad and stem_conv_supported(x, w, stride, padding)
            and training and rmean is not None and rmean.dtype == torch.float32 and rmean.is_contiguous()
            and R.select_backend(x, 'batch_norm_fwd') == 'hip'):
        y, part = StemConvFn.apply(x, w, int(padding), rmean)
        return BatchNormActFn.apply(y, z, bn_w, bn_b, rmean, rvar, training, momentum, eps, relu,
                                    _join_for(z) if z is not None else None, (part, rmean))
    if conv1x1_bn_stats_ok(x, w, stride, padding, rmean, training):
        y, part = Conv1x1StatsFn.apply(x, w, int(stride), int(stride), _join_for(x), rmean)
        return BatchNormActFn.apply(y, z, bn_w, bn_b, rmean, rvar, training, momentum, eps, relu,
                                    _join_for(z) if z is not None else None, (part, rmean))
    if _STEM_S2D and not x.requires_grad and stem_conv_supported(x, w, stride, padding):
        y = stem_conv_nhwc(x, w, padding)
    elif w.shape[2] == w.shape[3] > 1 and conv_kxk_supported(x, w, stride, padding):
        y = conv_kxk_nhwc(x, w, None, stride, padding)
    elif w.shape[2:] == (1, 1) and padding == 0 and x.is_cuda and x.dtype in _HALF:
        y = conv1x1_nhwc(x, w, None, (stride, stride))
    else:
        y = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), w, None, stride, padding).permute(0, 2, 3, 1)
    return batch_norm_act(y, z, bn_w, bn_b, rmean, rvar, training, momentum, eps, relu)


_CONV_BN_STATS = __import__('os').environ.get('PRA_CONV_BN_STATS', '1') == '1'
# PRA_STEM_S2D=0: the narrow-input stride-2 stem through MIOpen instead (A/B)
_STEM_S2D = __import__('os').environ.get('PRA_STEM_S2D', '1') == '1'


def conv_bn_stats_ok(x, w, stride, padding, rmean, training):
    """Whether conv_bn_act_nhwc takes the statistics-in-epilogue path (checked on the host
    before any launch: the implicit-GEMM conv's shape contract, fp32 running mean, HIP BN).
    PRA_CONV_BN_STATS=0 turns it off (separate statistics pass, for A/B timing)."""
    return bool(_CONV_BN_STATS and training and rmean is not None and rmean.dtype == torch.float32 and rmean.is_contiguous()
                and rmean.numel() == w.shape[0] and w.shape[2] == w.shape[3] > 1
                and conv_kxk_supported(x, w, stride, padding)
                and R.select_backend(x, 'batch_norm_fwd') == 'hip' and w.shape[0] % 8 == 0)


def conv_kxk_nhwc(x, w, bias=None, stride=1, padding=0):
    """Channels-last KxK conv x[N,H,W,Cin] * w[Cout,Cin,KH,KW] -> [N,Ho,Wo,Cout]."""
    return ConvKxKFn.apply(x, w, bias, int(stride), int(padding))


# =============================================================================
# Linear with fused weight-gradient accumulation
# =============================================================================
def _acc_grad_ok(g, w, dt):
    return (g is not None and not torch.is_grad_enabled() and g.shape == w.shape
            and g.dtype == dt and g.is_contiguous())


# Weight-gradient pairing of two Linears of one block (GPT attention: the QKV projection and the
# output projection, whose weight gradients share M = hidden and K = tokens): the output
# projection's backward (which runs first) leaves its xᵀ·dy job in the pair; the QKV
# projection's backward runs both as ONE launch of the two-problem grouped kernel
# (pra_gemm_tn_grouped2) when their tile counts fill one wave of the chip (GPT-1.3B: 192 + 64 =
# 256 tiles over the full K, instead of a split-K pass + reduction each). The QKV Linear takes
# the output-projection weight as an extra (unused) input, so that weight's AccumulateGrad --
# and the post-accumulate hooks the DP / sharding reducers count on -- fires only after the
# deferred accumulation has been issued.
_WGRAD_PAIR = __import__('os').environ.get('PRA_WGRAD_PAIR', '1') == '1'


class WgradPair:
    __slots__ = ('job', 'used')

    def __init__(self):
        self.job = None
        self.used = 0


def _pair_fill(M, N1, N2):
    t = ((M + 255) // 256)
    tiles = t * ((N1 + 255) // 256) + t * ((N2 + 255) // 256)
    return 224 <= tiles <= 256


class LinearFn(torch.autograd.Function):
    """y = x @ W (+ b) with paddle's [in, out] weight, all three GEMMs on the MFMA kernel:
    forward x·W with the bias in its epilogue; dx = dy·Wᵀ; dW = xᵀ·dy accumulated straight into
    W's existing ``.grad`` (the flat DP/sharding gradient buffer) by the kernel's beta=1
    epilogue instead of materialising dW and running AccumulateGrad's separate add. W's
    AccumulateGrad node still runs (with no gradient to add) and fires the post-accumulate-grad
    hooks that trigger the bucketed all-reduce / reduce-scatter."""

    @staticmethod
    def forward(ctx, x, w, b, pair=None, w_dep=None):
        x2 = x.reshape(-1, x.shape[-1])
        y = gemm(GEMM_FWD, x2, w, bias=b)
        ctx.save_for_backward(x)
        ctx.w, ctx.b = w, b
        ctx.has_b = b is not None
        ctx.pair, ctx.collector = pair, w_dep is not None
        return y.view(*x.shape[:-1], w.shape[-1])

    @staticmethod
    def backward(ctx, dy):
        x, = ctx.saved_tensors
        w = ctx.w
        dy2 = dy.reshape(-1, dy.shape[-1])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        x2 = x.reshape(-1, x.shape[-1])
        dx = None
        if ctx.needs_input_grad[0]:
            acc = _dx_acc(ctx, x)
            dx = gemm(GEMM_NT, dy2, w, out=acc, beta=1 if acc is not None else 0).view(x.shape)
        dw = None
        pair = ctx.pair
        job = None
        if pair is not None and ctx.collector:
            job, pair.job = pair.job, None
        if ctx.needs_input_grad[1]:
            g = w.grad if w.is_leaf else None
            if _acc_grad_ok(g, w, dy2.dtype):
                if pair is not None and not ctx.collector and pair.job is None:
                    pair.job = (x2, dy2, g)      # the collector's backward runs it (grouped)
                elif job is not None and _grouped_wgrad(job, (x2, dy2, g)):
                    job = None
                    pair.used += 1
                else:
                    # returning None still runs W's AccumulateGrad node, which fires its
                    # post-accumulate hooks after this in-place accumulation
                    gemm(GEMM_TN, x2, dy2, out=g, beta=1)
            else:
                dw = gemm(GEMM_TN, x2, dy2)
        if job is not None:   # a deferred job that could not be grouped
            gemm(GEMM_TN, job[0], job[1], out=job[2], beta=1)
        db = bias_grad(dy2, ctx.b) if ctx.has_b and ctx.needs_input_grad[2] else None
        return dx, dw, db, None, None


def _grouped_wgrad(j1, j2):
    """g (+)= xᵀ·dy for two jobs in one grouped launch; False (nothing launched) if they do not
    share M / K or do not fill one wave of the chip."""
    (x1, d1, g1), (x2, d2, g2) = j1, j2
    M, K = x1.shape[1], x1.shape[0]
    if not (x2.shape == (K, M) and d1.shape[0] == K and d2.shape[0] == K and x1.dtype == torch.bfloat16
            and all(t.dtype == torch.bfloat16 and t.is_contiguous() for t in (x1, d1, g1, x2, d2, g2))
            and _pair_fill(M, d1.shape[1], d2.shape[1]) and K % 64 == 0 and M % 8 == 0
            and d1.shape[1] % 8 == 0 and d2.shape[1] % 8 == 0 and R.select_backend(x1, 'gemm') == 'hip'
            and _GEMM_MODE != 'blas'):
        return False
    _native.lib().gemm_tn_grouped2(x1.data_ptr(), d1.data_ptr(), g1.data_ptr(), d1.shape[1], M, d1.shape[1],
                                   d1.shape[1], x2.data_ptr(), d2.data_ptr(), g2.data_ptr(), d2.shape[1], M,
                                   d2.shape[1], d2.shape[1], M, K, 1, _stream())
    return True


def _dx_acc(ctx, x):
    """Static-graph gradient-sum fusion (static/graph.py _ACC_DX_OPS): the other partial
    gradient of input ``x`` as a [rows, in] buffer the dgrad GEMM accumulates into (beta=1), or
    None. Marks it consumed so the executor does not add it again."""
    acc = getattr(ctx, 'dx_acc', None)
    if acc is None or acc.dtype != x.dtype or tuple(acc.shape) != tuple(x.shape) or not acc.is_contiguous():
        return None
    ctx.dx_acc_used = True
    return acc.view(-1, acc.shape[-1])


def bias_grad(dy2, b):
    """colsum(dy2) for a Linear bias: HIP row-block partial sums + column reduction; added
    straight into ``b.grad`` when it already exists (returns None then, like the dW path)."""
    rows, cols = dy2.shape
    if not (dy2.is_cuda and cols % 8 == 0 and dy2.dtype in _DT and _native.available()):
        return dy2.sum(0)
    L = _native.lib()
    part = _bias_part_of(dy2)   # the flash backward already summed this packed dQKV's columns
    if part is not None:
        nrb = part.shape[0]
    else:
        nrb = max(1, min(256, rows // 32))
        part = torch.empty((nrb, cols), device=dy2.device, dtype=torch.float32)
        L.colsum_rows(_ptr(dy2), _ptr(part), rows, cols, nrb, _dt(dy2), _stream())
    g = b.grad if b.is_leaf else None
    if _acc_grad_ok(g, b, dy2.dtype):
        L.colsum16_acc(_ptr(part), _ptr(g), nrb, cols, _dt(g), _stream())
        return None
    db = torch.empty(cols, device=dy2.device, dtype=dy2.dtype)
    L.colsum16(_ptr(part), _ptr(db), nrb, cols, _dt(db), _stream())
    return db


def _no_autocast_change(x, w):
    """True when autocast is off, or on with both operands already in its dtype (O2 / bf16
    models: autocast would not cast anything, so the fused kernels may run)."""
    dev = x.device.type
    if not torch.is_autocast_enabled(dev):
        return True
    return x.dtype == w.dtype == torch.get_autocast_dtype(dev)


def linear(x, w, b=None, pair=None, w_dep=None):
    """[.., in] @ [in, out] (+ b) with fused dW accumulation (see LinearFn). pair / w_dep: the
    weight-gradient pairing of two Linears (WgradPair; w_dep on the one whose backward runs
    last: the other Linear's weight)."""
    if b is not None and b.dtype != x.dtype and torch.is_autocast_enabled(x.device.type):
        b = b.to(x.dtype)
    if torch.is_grad_enabled() and (x.requires_grad or w.requires_grad or (b is not None and b.requires_grad)) \
            and x.dtype == w.dtype and _no_autocast_change(x, w):
        # any operand that needs a gradient goes through the autograd Function (a frozen
        # weight with a trainable input, or a non-leaf weight, included: the raw GEMM below
        # records no graph)
        if pair is not None and _WGRAD_PAIR:
            return LinearFn.apply(x, w, b, pair, w_dep)
        return LinearFn.apply(x, w, b)
    x2 = x.reshape(-1, x.shape[-1])
    if x2.is_cuda and x.dtype == w.dtype and _no_autocast_change(x, w):
        y = gemm(GEMM_FWD, x2, w, bias=b)
    else:
        y = torch.addmm(b, x2, w) if b is not None else torch.mm(x2, w)
    return y.view(*x.shape[:-1], w.shape[-1])


# Tile-count tail of a long-K weight gradient: a TN product with a few tiles past a multiple of
# 256 (GPT's tied LM head: 50304 x 2048 -> 1576 tiles = 6 full waves + 40) runs its last tile
# rows as a separate split-K launch, so the 40 stragglers do not hold the chip for a whole
# seventh wave of the full K loop. PRA_GEMM_TN_TAIL=0 turns it off.
_TN_TAIL = __import__('os').environ.get('PRA_GEMM_TN_TAIL', '1') == '1'


def gemm_tn_balanced(a, b, out=None, beta=0):
    """gemm(GEMM_TN, a, b, out, beta) with the tile-count tail split off (see _TN_TAIL)."""
    K, M = a.shape
    N = b.shape[1]
    tm, tn = (M + 255) // 256, (N + 255) // 256
    tiles = tm * tn
    if (_TN_TAIL and a.is_cuda and tiles > 256 and 0 < tiles % 256 <= 64 and 256 % tn == 0
            and R.select_backend(a, 'gemm') == 'hip'):
        rows = (tiles // 256) * (256 // tn) * 256
        if 0 < rows < M and (M - rows) % 8 == 0:
            if out is None:
                out = torch.empty((M, N), device=a.device, dtype=a.dtype)
            gemm(GEMM_TN, a[:, :rows], b, out=out[:rows], beta=beta)
            gemm(GEMM_TN, a[:, rows:], b, out=out[rows:], beta=beta)
            return out
    return gemm(GEMM_TN, a, b, out=out, beta=beta)


class LinearNTFn(torch.autograd.Function):
    """y = x @ W^T for a [out, in] weight (the tied LM head: W is the [vocab, hidden] word
    embedding). dx = dy·W and dW += dyᵀ·x (beta=1 into W's grad) on the MFMA kernel."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x)
        ctx.w = w
        return gemm(GEMM_NT, x, w)

    @staticmethod
    def backward(ctx, dy):
        x, = ctx.saved_tensors
        w = ctx.w
        if not dy.is_contiguous():
            dy = dy.contiguous()
        dx = gemm(GEMM_FWD, dy, w) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            g = w.grad if w.is_leaf else None
            if _acc_grad_ok(g, w, dy.dtype):
                gemm_tn_balanced(dy, x, out=g, beta=1)
            else:
                dw = gemm_tn_balanced(dy, x)
        return dx, dw


def linear_nt(x2, w):
    """[T, in] @ [out, in]^T with fused dW accumulation (see LinearNTFn)."""
    if torch.is_grad_enabled() and (x2.requires_grad or w.requires_grad) and x2.dtype == w.dtype and \
            _no_autocast_change(x2, w):
        return LinearNTFn.apply(x2, w)
    if x2.is_cuda and x2.dtype == w.dtype:
        return gemm(GEMM_NT, x2, w)
    return torch.mm(x2, w.t())


# fc2 dgrad of the GELU MLP on the in-tree NT GEMM with gelu'(z) and the fc1 bias-gradient
# column sums in its epilogue (PRA_MLP_DGELU_EPI=1) instead of hipBLASLt + bias_gelu_bwd_db
# (measured on GPT-1.3B: 123.0K vs 124.4K tokens/s, twice on one box: off by default)
_MLP_DGELU_EPI = __import__('os').environ.get('PRA_MLP_DGELU_EPI', '0') == '1'
# PRA_MLP_DGELU_SHORTK=1: the same fusion only where the dgrad runs in-tree anyway (K <= 1024,
# BERT-base). Measured off by default: the persistent kernel's dGELU(erf) epilogue (Z read +
# erf-GELU' + column sums, not overlapped with MFMA) took 140 us vs 64 + 61 us for hipBLASLt +
# bias_gelu_bwd_db at [16384, 3072] x 768 (BERT 1751 vs 1771 seq/s, profiles/r4/bert_nt_policy.md)
_MLP_DGELU_SHORTK = __import__('os').environ.get('PRA_MLP_DGELU_SHORTK', '0') == '1'


# The forward GEMM's epilogue saves gelu'(z) instead of z (the backward needs nothing else from
# z), so the fc2 dgrad epilogue is one multiply + the bias-gradient column sums and runs in-tree
# (PRA_MLP_SAVE_D=0: save z, dGELU recomputed in the backward as before)
_MLP_SAVE_D = __import__('os').environ.get('PRA_MLP_SAVE_D', '1') == '1'
# kernel for that dgrad: 1 = the persistent kernel (next tile's DMA under the epilogue), 0 = per-tile
_MLP_MULZ_PTS = __import__('os').environ.get('PRA_MLP_MULZ_PTS', '1') == '1'


class MlpGeluFn(torch.autograd.Function):
    """y = gelu(x·W1 + b1)·W2 (fc2 bias left to the caller's fused residual kernel).

    Forward: ONE GEMM with bias+GELU in its epilogue that also stores the pre-activation Z, then
    the fc2 GEMM. Backward: the fc2 dgrad GEMM applies gelu'(Z) in its epilogue and emits the
    fc1 bias gradient as per-tile column sums, so no separate bias-GELU pass exists in either
    direction; both weight gradients accumulate in place (beta=1)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, approximate):
        x2 = x.reshape(-1, x.shape[-1])
        M, F = x2.shape[0], w1.shape[1]
        z = torch.empty((M, F), device=x.device, dtype=x.dtype)
        ctx.save_d = _MLP_SAVE_D and x2.is_cuda and x2.dtype == torch.bfloat16
        epi = 'gelu_tanh' if approximate else 'gelu'
        h = gemm(GEMM_FWD, x2, w1, bias=b1, z=z, epi=epi + '_d' if ctx.save_d else epi)
        y = gemm(GEMM_FWD, h, w2)
        ctx.save_for_backward(x, z, h)
        ctx.w1, ctx.w2, ctx.b1 = w1, w2, b1
        ctx.approximate = approximate
        return y.view(*x.shape[:-1], w2.shape[1])

    @staticmethod
    def backward(ctx, dy):
        x, z, h = ctx.saved_tensors
        w1, w2 = ctx.w1, ctx.w2
        dy2 = dy.reshape(-1, dy.shape[-1])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        x2 = x.reshape(-1, x.shape[-1])
        if ctx.save_d:
            # z holds gelu'(pre-activation): dz = dh * z and the fc1 bias gradient in the epilogue
            r = _gemm_hip(GEMM_NT, dy2, w2, z=z, epi='mulz', want_colsum='part') \
                if R.select_backend(dy2, 'gemm') == 'hip' else None
            if r is not None:
                # the per-tile-row partials go straight into b1.grad (one launch)
                dz, part = r
                db1 = _colsum_rows_to_grad(part, ctx.b1, dz.dtype)
            else:
                dz, db1 = gemm(GEMM_NT, dy2, w2, z=z, epi='mulz', want_colsum=True)
                db1 = db1.to(dz.dtype)
        elif _GEMM_MODE == 'auto' and not _MLP_DGELU_EPI and not (_MLP_DGELU_SHORTK and _nt_in_tree(dy2, w2)):
            # dgrad (hipBLASLt, or the in-tree persistent kernel for a short K: the gemm() shape
            # policy), then ONE fused pass for gelu'(z) and the bias gradient
            dh = gemm(GEMM_NT, dy2, w2)
            dz, db1 = _dgelu_db(dh, z, ctx.approximate, ctx.b1)
        else:
            dz, db1 = gemm(GEMM_NT, dy2, w2, z=z, epi='dgelu_tanh' if ctx.approximate else 'dgelu',
                           want_colsum=True)
            db1 = db1.to(dz.dtype)
        dw1 = dw2 = None
        g2 = w2.grad
        if _acc_grad_ok(g2, w2, dy2.dtype):
            gemm(GEMM_TN, h, dy2, out=g2, beta=1)
        else:
            dw2 = gemm(GEMM_TN, h, dy2)
        acc = _dx_acc(ctx, x)
        dx = gemm(GEMM_NT, dz, w1, out=acc, beta=1 if acc is not None else 0).view(x.shape)
        g1 = w1.grad
        if _acc_grad_ok(g1, w1, dz.dtype):
            gemm(GEMM_TN, x2, dz, out=g1, beta=1)
        else:
            dw1 = gemm(GEMM_TN, x2, dz)
        return dx, dw1, db1, dw2, None


def _colsum_rows_to_grad(part, b, dtype):
    """Bias gradient from fp32 partial rows [P, N]: added into ``b.grad`` when it exists (None
    returned), else returned in ``dtype``."""
    L = _native.lib()
    nrb, cols = part.shape
    g = b.grad if (b is not None and b.is_leaf) else None
    if b is not None and _acc_grad_ok(g, b, dtype):
        L.colsum16_acc(_ptr(part), _ptr(g), nrb, cols, _dt(g), _stream())
        return None
    db = torch.empty(cols, device=part.device, dtype=dtype)
    L.colsum16(_ptr(part), _ptr(db), nrb, cols, _dt(db), _stream())
    return db


def _dgelu_db(dh, z, approximate, b=None):
    """dz = dh * gelu'(z) and db = colsum(dz) in one pass (bias_gelu_bwd_db kernel; z is the
    pre-activation, bias already in it). db is added straight into ``b.grad`` when it exists
    (returned as None then), else returned in z's dtype."""
    rows, cols = z.shape
    L = _native.lib()
    nrb = max(1, min(256, rows // 16))
    part = torch.empty((nrb, cols), device=z.device, dtype=torch.float32)
    dz = torch.empty_like(z)
    L.bias_gelu_bwd_db(_ptr(dh), _ptr(z), 0, _ptr(dz), _ptr(part), rows, cols, nrb, _dt(z),
                       int(approximate), _stream())
    g = b.grad if (b is not None and b.is_leaf) else None
    if b is not None and _acc_grad_ok(g, b, z.dtype):
        L.colsum16_acc(_ptr(part), _ptr(g), nrb, cols, _dt(g), _stream())
        return dz, None
    db = torch.empty(cols, device=z.device, dtype=z.dtype)
    L.colsum16(_ptr(part), _ptr(db), nrb, cols, _dt(db), _stream())
    return dz, db


def mlp_gelu(x, w1, b1, w2, approximate=True):
    """gelu(x·W1 + b1)·W2 with the bias+GELU (and its backward) inside the GEMM epilogues."""
    if all(t.requires_grad for t in (w1, b1, w2)) and torch.is_grad_enabled() and \
            all(t.is_leaf for t in (w1, b1, w2)) and x.dtype == w1.dtype == w2.dtype == b1.dtype and \
            x.is_cuda and _no_autocast_change(x, w1):
        return MlpGeluFn.apply(x, w1, b1, w2, approximate)
    return linear(bias_gelu(linear(x, w1), b1, approximate), w2)


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


_ZERO_PLAN = {}


def zero_tensors(ts):
    """Zero a list of device tensors in ONE launch (multi-tensor fill over a cached device table
    of 64 KB pieces; the table is rebuilt only when the set of storages changes)."""
    ts = [t for t in ts if t.numel()]
    if not ts:
        return
    if not (ts[0].is_cuda and _native.available() and len(_ZERO_CHECKED) == 1 and
            all(t.is_contiguous() and t.is_cuda for t in ts)):
        torch._foreach_zero_(ts)
        return
    key = tuple((t.data_ptr(), t.numel() * t.element_size()) for t in ts)
    plan = _ZERO_PLAN.get(key)
    if plan is None:
        import numpy as np
        pieces = [(p + o, min(65536, n - o)) for p, n in key for o in range(0, n, 65536)]
        tab = torch.from_numpy(np.array(pieces, dtype=np.int64).reshape(-1, 2)).to(ts[0].device)
        if len(_ZERO_PLAN) > 8:
            _ZERO_PLAN.clear()
        plan = _ZERO_PLAN[key] = (tab, len(pieces))
    _native.lib().zero_mt(_ptr(plan[0]), plan[1], _stream())
    if not _ZERO_CHECKED[0]:
        # first use in the process: confirm the launch zeroed everything (one sync), else keep
        # the library fill from then on
        _ZERO_CHECKED[0] = True
        if any(int(torch.count_nonzero(t)) for t in ts):
            import warnings
            warnings.warn('zero_mt kernel left nonzeros: using torch._foreach_zero_')
            _ZERO_CHECKED.append('off')
            torch._foreach_zero_(ts)


_ZERO_CHECKED = [False]


@R.register_kernel('adamw_mt', 'hip')
def _adamw_mt_hip(tab, ftab, ch, nch, lr, b1, b2, eps, bc1, bc2, grad_scale, scale_t, outs):
    """Multi-tensor AdamW over a device pointer table (one launch for every parameter);
    returns ``outs`` (the updated fp32 masters / params) so the NaN/Inf checker sees them."""
    _native.lib().adamw_mt(_ptr(tab), _ptr(ftab), _ptr(ch), nch, float(lr), float(b1), float(b2),
                           float(eps), float(bc1), float(bc2), float(grad_scale), _stream(),
                           0 if scale_t is None else _ptr(scale_t))
    return outs


@R.register_kernel('momentum_mt', 'hip')
def _momentum_mt_hip(tab, ftab, ch, nch, lr, mu, nesterov, grad_scale, scale_t, outs):
    _native.lib().momentum_mt(_ptr(tab), _ptr(ftab), _ptr(ch), nch, float(lr), float(mu),
                              int(nesterov), float(grad_scale), _stream(),
                              0 if scale_t is None else _ptr(scale_t))
    return outs


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

    def step(self, lr, b1, b2, eps, step, grad_scale=1.0, scale_tensor=None):
        """``scale_tensor``: optional 0-d fp32 device tensor (the global-norm clip
        coefficient) multiplied into every gradient inside the kernel."""
        grads = self.grads_getter()
        if self._plan is None or tuple(g.data_ptr() for g in grads) != self._gptrs:
            self._build(grads)
        tab, ftab, ch, nch = self._plan
        bc1 = 1 - b1 ** step
        bc2 = 1 - b2 ** step
        outs = [m if m is not None else p for m, p in zip(self.masters, self.params)]
        R.dispatch('adamw_mt', tab, tab, ftab, ch, nch, lr, b1, b2, eps, bc1, bc2, grad_scale,
                   scale_tensor, outs)


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


@R.register_kernel('sumsq', 'ref')
def _sumsq_ref(tensors):
    return sum((t.float() ** 2).sum() for t in tensors)


@R.register_kernel('sumsq', 'hip', dtypes=_FLOATS)
def _sumsq_hip(tensors):
    out = torch.zeros(1, device=tensors[0].device, dtype=torch.float32)
    L = _native.lib()
    for t in tensors:
        L.sumsq_accum(_ptr(t), _ptr(out), t.numel(), _dt(t), _stream())
    return out[0]


def global_l2_norm_sq(tensors):
    """Sum of squares over a list of tensors (fp32 accumulate)."""
    if not tensors:
        return None
    return R.dispatch('sumsq', tensors[0], tensors)


# =============================================================================
# BatchNorm (+ residual add + ReLU), channels-last [M, C]
# parity: paddle/phi/kernels/gpu/batch_norm_kernel.cu, batch_norm_grad_kernel.cu,
#         paddle/fluid/operators/fused/fused_bn_add_activation_op.cu (y = act(BN(x) + z))
# =============================================================================
@R.register_kernel('batch_norm_fwd', 'ref')
def _bn_fwd_ref(x2, z2, w, b, rmean, rvar, training, momentum, eps, relu):
    xf = x2.float()
    if training:
        mean = xf.mean(0)
        var = xf.var(0, unbiased=False)
        if rmean is not None:
            m = x2.shape[0]
            with torch.no_grad():
                rmean.mul_(momentum).add_(mean, alpha=1 - momentum)
                rvar.mul_(momentum).add_(var * (m / max(m - 1, 1)), alpha=1 - momentum)
    else:
        mean, var = rmean.float(), rvar.float()
    invstd = torch.rsqrt(var + eps)
    y = (xf - mean) * invstd
    if w is not None:
        y = y * w.float()
    if b is not None:
        y = y + b.float()
    if z2 is not None:
        y = y + z2.float()
    if relu:
        y = torch.relu(y)
    return y.to(x2.dtype), mean, invstd, None


@R.register_kernel('batch_norm_bwd', 'ref')
def _bn_bwd_ref(dy, y, mask, x2, w, mean, invstd, relu, need_dz):
    g = dy.float()
    if relu:
        g = torch.where(y > 0, g, torch.zeros_like(g))
    xhat = (x2.float() - mean) * invstd
    m = x2.shape[0]
    s1 = g.sum(0)
    s2 = (g * xhat).sum(0)
    a = (w.float() if w is not None else 1.0) * invstd
    dx = a * (g - s1 / m - xhat * s2 / m)
    pdt = w.dtype if w is not None else torch.float32
    dz = g.to(x2.dtype) if need_dz else None
    return dx.to(x2.dtype), dz, s2.to(pdt), s1.to(pdt)


def _bn_hip_ok(x2):
    return x2.shape[1] % 8 == 0 and x2.numel() // 8 < 2 ** 32 and x2.is_contiguous()


@R.register_kernel('batch_norm_fwd', 'hip', dtypes=_FLOATS)
def _bn_fwd_hip(x2, z2, w, b, rmean, rvar, training, momentum, eps, relu):
    _check_dtypes('batch_norm', (x2, z2), (w, b))
    """Returns (y, mean, invstd, relu keep-mask bytes or None)."""
    if not _bn_hip_ok(x2):
        return _bn_fwd_ref(x2, z2, w, b, rmean, rvar, training, momentum, eps, relu)
    L = _native.lib()
    M, C = x2.shape
    dev = x2.device
    y = torch.empty_like(x2)
    dtw = _dt(w) if w is not None else 0
    z2 = z2.contiguous() if z2 is not None else None
    if training:
        nrb = L.bn_nrb(M, C)
        part = torch.empty((2, nrb, C), device=dev, dtype=torch.float32)
        stat = torch.empty((4, C), device=dev, dtype=torch.float32)  # mean | invstd | scale | shift
        mask = torch.empty(M * C // 8, device=dev, dtype=torch.uint8) if relu else None
        L.bn_fwd_train(_ptr(x2), _ptr(z2), _ptr(w), _ptr(b), _ptr(rmean), _ptr(rvar), _ptr(y),
                       _ptr(mask), _ptr(stat[0]), _ptr(stat[1]), _ptr(part), _ptr(stat[2]), M, C,
                       nrb, float(eps), float(momentum), int(relu), _dt(x2), dtw, _stream())
        return y, stat[0], stat[1], mask
    coef = torch.empty((2, C), device=dev, dtype=torch.float32)
    L.bn_fwd_infer(_ptr(x2), _ptr(z2), _ptr(w), _ptr(b), _ptr(rmean), _ptr(rvar), _ptr(y),
                   _ptr(coef), M, C, float(eps), int(relu), _dt(x2), dtw, _stream())
    mean = rmean.float()
    return y, mean, torch.rsqrt(rvar.float() + eps), None


_BN_PREMERGE_ROWS = 256


def _bn_premerge(part):
    """[2, rows, C] conv-epilogue partials -> [2, ceil(rows/64), C] when there are many rows
    (the finalize kernel walks the rows with one block per 64 channels)."""
    rows, C = part.shape[1], part.shape[2]
    if rows <= _BN_PREMERGE_ROWS:
        return part
    out = torch.empty((2, (rows + 63) // 64, C), device=part.device, dtype=torch.float32)
    _native.lib().bn_premerge(part.data_ptr(), out.data_ptr(), rows, C, _stream())
    return out


def _bn_fwd_parts_hip(x2, z2, w, b, rmean, rvar, momentum, eps, relu, part, kshift):
    """Training BN forward from the per-tile partial sums a convolution epilogue produced
    (part [2, rows, C] around kshift): finalize + apply kernels only."""
    _check_dtypes('batch_norm', (x2, z2), (w, b))
    L = _native.lib()
    part = _bn_premerge(part)
    M, C = x2.shape
    y = torch.empty_like(x2)
    stat = torch.empty((4, C), device=x2.device, dtype=torch.float32)  # mean | invstd | scale | shift
    mask = torch.empty(M * C // 8, device=x2.device, dtype=torch.uint8) if relu else None
    z2 = z2.contiguous() if z2 is not None else None
    L.bn_fwd_parts(_ptr(x2), _ptr(z2), _ptr(w), _ptr(b), _ptr(rmean), _ptr(rvar), _ptr(y), _ptr(mask),
                   _ptr(stat[0]), _ptr(stat[1]), _ptr(part), _ptr(kshift), _ptr(stat[2]), M, C,
                   part.shape[1], float(eps), float(momentum), int(relu), _dt(x2),
                   _dt(w) if w is not None else 0, _stream())
    return y, stat[0], stat[1], mask


@R.register_kernel('batch_norm_bwd', 'hip', dtypes=_FLOATS)
def _bn_bwd_hip(dy, y, mask, x2, w, mean, invstd, relu, need_dz, acc=None):
    """acc = (w.grad, b.grad): the scale / shift gradients are added into these in the
    finalize kernel and (None, None) is returned for them."""
    if not _bn_hip_ok(x2):
        return _bn_bwd_ref(dy, y, mask, x2, w, mean, invstd, relu, need_dz)
    L = _native.lib()
    M, C = x2.shape
    dev = x2.device
    dy = dy.contiguous()
    dx = torch.empty_like(x2)
    dz = None
    if need_dz:
        dz = torch.empty_like(x2) if relu else dy
    pdt = w.dtype if w is not None else torch.float32
    if acc is not None:
        gw, gb = acc
    else:
        dwb = torch.empty((2, C), device=dev, dtype=pdt)
        gw, gb = dwb[0], dwb[1]
    nrb = L.bn_nrb(M, C)
    part = torch.empty((2, nrb, C), device=dev, dtype=torch.float32)
    coef = torch.empty((3, C), device=dev, dtype=torch.float32)
    L.bn_bwd(_ptr(dy), _ptr(y) if relu else 0, _ptr(mask) if relu else 0, _ptr(x2), _ptr(w), _ptr(mean), _ptr(invstd),
             _ptr(dx), _ptr(dz) if (need_dz and relu) else 0, _ptr(gw), _ptr(gb),
             _ptr(part), _ptr(coef), M, C, nrb, int(relu), _dt(x2), _DT[pdt], int(acc is not None), _stream())
    if acc is not None:
        return dx, dz, None, None
    return dx, dz, gw, gb


def _bn_bwd_parts_hip(g, x2, w, mean, invstd, part, acc=None):
    """BN backward from the masked gradient g and its partial sums part [2, rows, C] (sum g,
    sum g * (x - mean)): returns (dx, dscale, dshift); with acc = (w.grad, b.grad) those are
    accumulated in place and (dx, None, None) returned."""
    L = _native.lib()
    R._STATS[('batch_norm_bwd', 'hip_parts')] += 1
    part = _bn_premerge(part)
    M, C = x2.shape
    dx = torch.empty_like(x2)
    pdt = w.dtype if w is not None else torch.float32
    if acc is not None:
        gw, gb = acc
    else:
        dwb = torch.empty((2, C), device=x2.device, dtype=pdt)
        gw, gb = dwb[0], dwb[1]
    coef = torch.empty((3, C), device=x2.device, dtype=torch.float32)
    L.bn_bwd_parts(g.data_ptr(), x2.data_ptr(), _ptr(w), mean.data_ptr(), invstd.data_ptr(), dx.data_ptr(),
                   gw.data_ptr(), gb.data_ptr(), part.data_ptr(), coef.data_ptr(), M, C, part.shape[1], _dt(x2),
                   _DT[pdt], int(acc is not None), _stream())
    if acc is not None:
        return dx, None, None
    return dx, gw, gb


class BatchNormActFn(torch.autograd.Function):
    """y = act(BN(x) + z) over channels-last x[..., C]; running stats updated in place."""

    @staticmethod
    def forward(ctx, x, z, w, b, rmean, rvar, training, momentum, eps, relu, join=None, stats=None):
        ctx.join = join
        shp = x.shape
        C = shp[-1]
        x2 = x.contiguous().view(-1, C)
        z2 = _like(z, x.dtype).reshape(-1, C) if z is not None else None
        if w is not None:
            b = _like(b, w.dtype)
        if stats is not None and training:
            # statistics already taken by the producing convolution's epilogue
            y, mean, invstd, mask = _bn_fwd_parts_hip(x2, z2, w, b, rmean, rvar, momentum, eps, relu,
                                                      *stats)
        else:
            y, mean, invstd, mask = R.dispatch('batch_norm_fwd', x2, x2, z2, w, b, rmean, rvar,
                                               training, momentum, eps, relu)
        # ReLU backward needs only the keep-bits (1 B per 8 channels) when the kernel wrote them
        ctx.save_for_backward(x2, y if (relu and mask is None) else None, mask, w, mean, invstd)
        ctx.relu, ctx.shp, ctx.has_z = relu, shp, z is not None
        ctx.has_b, ctx.training, ctx.b = b is not None, training, b
        out = y.view(shp)
        ctx.rec = None
        if (_BN_DGRAD_FUSE and training and relu and mask is not None and x2.is_cuda
                and mean.dtype == torch.float32 and x2.dtype in _HALF):
            ctx.rec = out._pra_bn = _BnHandoff(x2, mask, mean)
        return out

    @staticmethod
    def backward(ctx, dy):
        x2, y, mask, w, mean, invstd = ctx.saved_tensors
        dy2 = _like(dy, x2.dtype).contiguous().view(x2.shape)
        if not ctx.training:  # frozen statistics: dx = dy * w * invstd
            g = dy2.float()
            if ctx.relu:
                g = torch.where(y > 0, g, torch.zeros_like(g))
            a = invstd * (w.float() if w is not None else 1.0)
            pdt = w.dtype if w is not None else torch.float32
            dw = (g * (x2.float() - mean) * invstd).sum(0).to(pdt)
            dz = g.to(x2.dtype).view(ctx.shp) if ctx.has_z else None
            if dz is not None and ctx.join is not None:
                dz = ctx.join.add_tensor(dz, owned=True)
            return ((g * a).to(x2.dtype).view(ctx.shp), dz, dw if w is not None else None,
                    g.sum(0).to(pdt) if ctx.has_b else None, None, None, None, None, None, None, None,
                    None)
        acc = None
        b = ctx.b
        if (x2.is_cuda and w is not None and b is not None and ctx.needs_input_grad[2]
                and ctx.needs_input_grad[3] and w.is_leaf and b.is_leaf and _acc_grad_ok(w.grad, w, w.dtype)
                and _acc_grad_ok(b.grad, b, w.dtype) and R.select_backend(x2, 'batch_norm_bwd') == 'hip'):
            acc = (w.grad, b.grad)  # scale/shift grads accumulated in the finalize kernel
        part = ctx.rec.take(dy2) if ctx.rec is not None else None
        if part is not None:
            # dy2 is the ReLU-masked gradient and part its reductions (the consumer conv's dgrad
            # epilogue): finalize + apply only
            dx, dw, db = _bn_bwd_parts_hip(dy2, x2, w, mean, invstd, part, acc)
            dz = None
            if ctx.has_z and ctx.needs_input_grad[1]:
                # the residual's gradient IS the masked g (produced for this BN by the dgrad
                # epilogue; nothing else holds it, so the join may accumulate into it)
                dz = dy2.view(ctx.shp)
                if ctx.join is not None:
                    dz = ctx.join.add_tensor(dz, owned=True)
            return (dx.view(ctx.shp), dz, dw if (w is not None and ctx.needs_input_grad[2]) else None,
                    db if (ctx.has_b and ctx.needs_input_grad[3]) else None,
                    None, None, None, None, None, None, None, None)
        if acc is not None:
            dx, dz, dw, db = _bn_bwd_hip(dy2, y, mask, x2, w, mean, invstd, ctx.relu,
                                         ctx.has_z and ctx.needs_input_grad[1], acc=acc)
        else:
            dx, dz, dw, db = R.dispatch('batch_norm_bwd', x2, dy2, y, mask, x2, w, mean, invstd, ctx.relu,
                                        ctx.has_z and ctx.needs_input_grad[1])
        if dz is not None:
            dz = dz.view(ctx.shp)
            if ctx.join is not None:
                dz = ctx.join.add_tensor(dz, owned=dz.data_ptr() != dy2.data_ptr())
        return (dx.view(ctx.shp), dz,
                dw if (w is not None and ctx.needs_input_grad[2]) else None,
                db if (ctx.has_b and ctx.needs_input_grad[3]) else None,
                None, None, None, None, None, None, None, None)


def batch_norm_act(x, z, w, b, rmean, rvar, training, momentum=0.9, eps=1e-5, relu=False):
    """Channels-last BatchNorm with optional fused residual add and ReLU (paddle momentum
    convention: running = momentum * running + (1 - momentum) * batch)."""
    return BatchNormActFn.apply(x, z, w, b, rmean, rvar, training, momentum, eps, relu,
                                _join_for(z) if z is not None else None)


# =============================================================================
# Max pooling, channels-last (parity: paddle/phi/kernels/funcs/pooling.cu): the forward keeps
# the winning tap per output element as one byte; the backward gathers (no atomics, no
# zero-fill, no int64 index tensor)
# =============================================================================
class GlobalAvgPoolNHWCFn(torch.autograd.Function):
    """Global average pooling over H, W of a channels-last tensor -> [N, 1, 1, C]; the backward
    is one broadcast-write kernel (pool.hip gap_bwd_k). Parity: phi pool2d with adaptive=True,
    output 1x1 (paddle/phi/kernels/funcs/pooling.cu)."""

    @staticmethod
    def forward(ctx, x):
        ctx.shp = tuple(x.shape)
        return x.mean((1, 2), keepdim=True)

    @staticmethod
    def backward(ctx, dy):
        n, h, w, c = ctx.shp
        dy = dy.contiguous()
        dx = torch.empty(ctx.shp, device=dy.device, dtype=dy.dtype)
        _native.lib().gap_bwd(dy.data_ptr(), dx.data_ptr(), n, h * w, c, _dt(dy), _stream())
        return dx


def global_avg_pool_nhwc_supported(x):
    return x.is_cuda and x.dim() == 4 and x.dtype in _FLOATS and x.shape[3] % 8 == 0 and x.is_contiguous()


def max_pool_nhwc_supported(x, k, s, p):
    return (x.is_cuda and x.dim() == 4 and x.dtype in _FLOATS and x.shape[3] % 8 == 0
            and k[0] * k[1] <= 255 and p[0] < k[0] and p[1] < k[1] and min(s) >= 1 and min(p) >= 0)


class MaxPoolNHWCFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kh, kw, sh, sw, ph, pw):
        x = x.contiguous()
        n, h, w, c = x.shape
        ho, wo = (h + 2 * ph - kh) // sh + 1, (w + 2 * pw - kw) // sw + 1
        y = torch.empty((n, ho, wo, c), device=x.device, dtype=x.dtype)
        idx = torch.empty((n, ho, wo, c), device=x.device, dtype=torch.uint8)
        _native.lib().max_pool_fwd(x.data_ptr(), y.data_ptr(), idx.data_ptr(), n, h, w, c, ho, wo, kh, kw, sh,
                                   sw, ph, pw, _dt(x), _stream())
        ctx.save_for_backward(idx)
        ctx.geo = (n, h, w, c, ho, wo, kh, kw, sh, sw, ph, pw)
        return y

    @staticmethod
    def backward(ctx, dy):
        idx, = ctx.saved_tensors
        n, h, w, c = ctx.geo[:4]
        dy = dy.contiguous()
        dx = torch.empty((n, h, w, c), device=dy.device, dtype=dy.dtype)
        _native.lib().max_pool_bwd(dy.data_ptr(), idx.data_ptr(), dx.data_ptr(), *ctx.geo, _dt(dy), _stream())
        return dx, None, None, None, None, None, None


def max_pool2d_nhwc(x, kernel, stride, padding):
    return MaxPoolNHWCFn.apply(x, int(kernel[0]), int(kernel[1]), int(stride[0]), int(stride[1]),
                               int(padding[0]), int(padding[1]))


# =============================================================================
# Embedding lookup (parity: paddle/phi/kernels/gpu/embedding_kernel.cu,
# embedding_grad_kernel.cu); ids outside [0, V) or == padding_idx read as zero rows
# =============================================================================
@R.register_kernel('embedding_fwd', 'ref')
def _emb_fwd_ref(ids, w, pad):
    V = w.shape[0]
    ok = (ids >= 0) & (ids < V)
    if pad is not None and pad >= 0:
        ok = ok & (ids != pad)
    out = torch.nn.functional.embedding(torch.where(ok, ids, torch.zeros_like(ids)), w)
    return out * ok.unsqueeze(-1).to(out.dtype)


@R.register_kernel('embedding_bwd', 'ref')
def _emb_bwd_ref(ids, dy, w_shape, w_dtype, pad, into=None):
    V, D = w_shape
    flat = ids.reshape(-1)
    ok = (flat >= 0) & (flat < V)
    if pad is not None and pad >= 0:
        ok = ok & (flat != pad)
    g = torch.zeros(w_shape, dtype=torch.float32, device=dy.device)
    g.index_add_(0, flat[ok], dy.reshape(-1, D)[ok].float())
    if into is not None:
        into.add_(g.to(into.dtype))
        return into
    return g.to(w_dtype)


@R.register_kernel('embedding_fwd', 'hip', dtypes=_FLOATS)
def _emb_fwd_hip(ids, w, pad):
    D = w.shape[1]
    if D % 8 != 0 or not w.is_contiguous():
        return _emb_fwd_ref(ids, w, pad)
    ids_c = ids.reshape(-1).contiguous().long()
    out = torch.empty((ids_c.numel(), D), device=w.device, dtype=w.dtype)
    _native.lib().embedding_fwd(_ptr(ids_c), _ptr(w), _ptr(out), ids_c.numel(), D, w.shape[0],
                                -1 if pad is None else int(pad), _dt(w), _stream())
    return out.view(*ids.shape, D)


@R.register_kernel('embedding_bwd', 'hip', dtypes=_FLOATS)
def _emb_bwd_hip(ids, dy, w_shape, w_dtype, pad, into=None):
    V, D = w_shape
    tgt_dt = into.dtype if into is not None else w_dtype
    if D % 8 != 0 or D > 4096 or (dy.dtype, tgt_dt) not in (
            (torch.bfloat16, torch.bfloat16), (torch.bfloat16, torch.float32),
            (torch.float32, torch.float32), (torch.float16, torch.float16),
            (torch.float16, torch.float32)):
        return _emb_bwd_ref(ids, dy, w_shape, w_dtype, pad, into)
    flat = ids.reshape(-1).long()
    sids, perm = torch.sort(flat, stable=True)
    dy2 = dy.reshape(-1, D).contiguous()
    out = into if into is not None else torch.zeros(w_shape, dtype=w_dtype, device=dy.device)
    # segmented two-pass form: repeated ids (positions, token types) spread over many waves
    ws = torch.empty(2 * (-(-flat.numel() // 32)) * D, dtype=torch.float32, device=dy.device)
    _native.lib().embedding_bwd(_ptr(sids), _ptr(perm), _ptr(dy2), _ptr(out), flat.numel(), D, V,
                                -1 if pad is None else int(pad), _dt(dy2), _DT[out.dtype],
                                1, _ptr(ws), _stream())
    return out


class EmbeddingFn(torch.autograd.Function):
    """Lookup whose backward adds straight into the table's existing ``.grad`` (the flat
    DP/sharding grad buffer) when there is one, like LinearFn: no dense [V, D] gradient
    temporary, no AccumulateGrad add pass."""

    @staticmethod
    def forward(ctx, ids, w, pad):
        ctx.save_for_backward(ids)
        ctx.w, ctx.pad = w, pad
        return R.dispatch('embedding_fwd', ids if not ids.is_cuda else w, ids, w, pad)

    @staticmethod
    def backward(ctx, dy):
        ids, = ctx.saved_tensors
        w = ctx.w
        g = w.grad
        if (g is not None and not torch.is_grad_enabled() and g.shape == w.shape and
                g.is_contiguous()):
            R.dispatch('embedding_bwd', w, ids, dy, tuple(w.shape), w.dtype, ctx.pad, g)
            return None, None, None
        return None, R.dispatch('embedding_bwd', w, ids, dy, tuple(w.shape), w.dtype, ctx.pad), \
            None


def embedding(ids, w, padding_idx=None):
    if w.requires_grad and torch.is_grad_enabled():
        return EmbeddingFn.apply(ids, w, padding_idx)
    return R.dispatch('embedding_fwd', w, ids, w, padding_idx)


# =============================================================================
# GEMM + bias + activation (MFMA kernel, gemm.hip). Parity: reference
# paddle/phi/kernels/fusion/gpu/fused_gemm_epilogue_kernel.cu (cublasLt BIAS / GELU / RELU
# epilogues) behind python/paddle/incubate/nn/functional/fused_matmul_bias.py.
# =============================================================================
_ACT = {None: 0, 'none': 0, 'gelu': 1, 'gelu_tanh': 2, 'relu': 3}


def _act_ref(z, act):
    if act == 1:
        return torch.nn.functional.gelu(z)
    if act == 2:
        return torch.nn.functional.gelu(z, approximate='tanh')
    if act == 3:
        return torch.relu(z)
    return z


@R.register_kernel('gemm_bias_act', 'ref')
def _gba_ref(x2, w, b, act, want_z):
    z = x2.float() @ w.float()
    if b is not None:
        z = z + b.float()
    y = _act_ref(z, act).to(x2.dtype)
    return y, (z.to(x2.dtype) if want_z and act else None)


@R.register_kernel('gemm_bias_act', 'hip', dtypes=_HALF)
def _gba_hip(x2, w, b, act, want_z):
    M, K = x2.shape
    N = w.shape[1]
    y = torch.empty(M, N, dtype=x2.dtype, device=x2.device)
    z = torch.empty_like(y) if (want_z and act) else None
    _native.lib().gemm_bias_act(_ptr(x2), _ptr(w), _ptr(b), _ptr(y), _ptr(z), M, N, K, x2.stride(0),
                                w.stride(0), N, _dt(x2), act, _stream())
    return y, z


def gemm_supported(x2, w):
    """Shapes/layouts the MFMA kernel takes: 2-byte dtypes, 16-B aligned row-major rows."""
    return (x2.dtype in (torch.bfloat16, torch.float16) and w.dtype == x2.dtype and x2.dim() == 2
            and w.dim() == 2 and x2.stride(1) == 1 and w.stride(1) == 1 and x2.shape[1] == w.shape[0]
            and x2.shape[1] % 8 == 0 and w.shape[1] % 8 == 0 and x2.stride(0) % 8 == 0
            and w.stride(0) % 8 == 0 and x2.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0)


class GemmBiasActFn(torch.autograd.Function):
    """y = act(x @ w + b) with the epilogue fused into the MFMA GEMM; backward keeps the
    pre-activation the kernel wrote alongside y and runs hipBLASLt for dX / dW."""

    @staticmethod
    def forward(ctx, x, w, b, act):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        if x2.stride(-1) != 1 or x2.stride(0) % 8 or x2.data_ptr() % 16:
            x2 = x2.contiguous()  # row pitch may exceed K (lda), rows must stay 16-B aligned
        if b is not None:
            b = b.to(x.dtype).contiguous()
            if b.data_ptr() % 8:
                b = b.clone()
        need = any(ctx.needs_input_grad[:3])
        y, z = R.dispatch('gemm_bias_act', x2, x2, w, b, act, need)
        ctx.save_for_backward(x2, w, z)
        ctx.act, ctx.has_b, ctx.shp = act, b is not None, shp
        return y.view(*shp[:-1], w.shape[1])

    @staticmethod
    def backward(ctx, dy):
        x2, w, z = ctx.saved_tensors
        dy2 = dy.reshape(-1, w.shape[1])
        if ctx.act in (1, 2):  # GELU': the elementwise HIP kernel on the saved pre-activation
            dy2 = dy2.contiguous()
            dy2 = _like(dy2, z.dtype)
            dz = R.dispatch("bias_gelu_bwd", dy2, dy2, z, None, ctx.act == 2)
        elif ctx.act:
            with torch.enable_grad():
                zf = z.detach().requires_grad_(True)
                (dz,) = torch.autograd.grad(_act_ref(zf, ctx.act), zf, dy2)
        else:
            dz = dy2
        dx = (dz @ w.t()).view(ctx.shp) if ctx.needs_input_grad[0] else None
        dw = x2.t() @ dz if ctx.needs_input_grad[1] else None
        db = dz.sum(0, dtype=torch.float32).to(dz.dtype) if (ctx.has_b and ctx.needs_input_grad[2]) else None
        return dx, dw, db, None


def gemm_bias_act(x, w, b=None, act=None):
    """act(x @ w + b) for x [..., K], w [K, N] (Paddle Linear layout). On the GPU this is one
    MFMA kernel launch (gemm.hip); unsupported layouts fall back to matmul + epilogue."""
    a = _ACT[act] if not isinstance(act, int) else act
    x2 = x.reshape(-1, x.shape[-1])
    if x.is_cuda and not gemm_supported(x2 if x2.is_contiguous() else x2.contiguous(), w):
        z = torch.matmul(x, w)
        return _act_ref(z if b is None else z + b, a)
    return GemmBiasActFn.apply(x, w, b, a)
