"""LoD sequence ops (parity: python/paddle/static/nn/sequence_lod.py).

A LoD tensor here is a framework Tensor whose rows are the concatenated time steps of a batch of
variable-length sequences, with the sequence boundaries as host-side offset lists
(``Tensor.set_lod`` / ``set_recursive_sequence_lengths``, as on the reference's LoDTensor). The
ops run on the device as segment reductions / gathers built from the offsets (one index tensor
per call, no per-sequence Python loop over device data); gradients flow through torch autograd.
Only the last LoD level is interpreted (the reference's ops act on it too); higher levels are
carried to the output where the reference does so.
"""
import math

import torch

from ..framework.core import Tensor, _u


def _offsets(x, what='input'):
    lod = x.lod() if isinstance(x, Tensor) else []
    if not lod:
        raise ValueError(f"{what} must be a LoD tensor (Tensor.set_lod / set_recursive_sequence_lengths)")
    return lod[-1]


def _wrap(t, lod=None):
    out = Tensor(t)
    if lod is not None:
        out.set_lod(lod)
    return out


def _seg_ids(off, device):
    lens = torch.tensor([b - a for a, b in zip(off, off[1:])], dtype=torch.long)
    return torch.repeat_interleave(torch.arange(len(lens)), lens).to(device), lens.to(device)


def _upper(x):
    return x.lod()[:-1]


def sequence_pool(input, pool_type, is_test=False, pad_value=0.0):
    """Pool each sequence of the last LoD level: average / sum / sqrt / max / last / first.
    Empty sequences give ``pad_value``."""
    off = _offsets(input)
    t = _u(input)
    nseq = len(off) - 1
    seg, lens = _seg_ids(off, t.device)
    flat = t.reshape(t.shape[0], -1)
    pt = pool_type.lower()
    out_shape = (nseq,) + tuple(t.shape[1:])
    if pt in ('sum', 'average', 'sqrt'):
        acc = torch.zeros((nseq, flat.shape[1]), dtype=flat.dtype, device=t.device).index_add(0, seg, flat)
        if pt == 'average':
            acc = acc / lens.clamp(min=1).to(acc.dtype)[:, None]
        elif pt == 'sqrt':
            acc = acc / lens.clamp(min=1).to(acc.dtype).sqrt()[:, None]
    elif pt == 'max':
        idx = seg[:, None].expand_as(flat)
        acc = torch.full((nseq, flat.shape[1]), -math.inf, dtype=flat.dtype, device=t.device)
        acc = acc.scatter_reduce(0, idx, flat, reduce='amax', include_self=True)
    elif pt in ('first', 'last'):
        starts = torch.tensor(off[:-1] if pt == 'first' else [max(b - 1, 0) for b in off[1:]],
                              dtype=torch.long, device=t.device)
        acc = flat.index_select(0, starts.clamp(max=max(flat.shape[0] - 1, 0))) if flat.shape[0] else \
            torch.zeros((nseq, flat.shape[1]), dtype=flat.dtype, device=t.device)
    else:
        raise ValueError(f"unknown pool_type {pool_type!r}")
    empty = (lens == 0)[:, None]
    acc = torch.where(empty, torch.full_like(acc, pad_value), acc)
    up = _upper(input)
    return _wrap(acc.reshape(out_shape), up if up else None)


def sequence_first_step(input):
    return sequence_pool(input, 'first')


def sequence_last_step(input):
    return sequence_pool(input, 'last')


def sequence_softmax(input, use_cudnn=False, name=None):
    """Softmax over the time steps of each sequence (input [N, 1] or [N])."""
    off = _offsets(input)
    t = _u(input)
    flat = t.reshape(-1)
    seg, _ = _seg_ids(off, t.device)
    mx = torch.full((len(off) - 1,), -math.inf, dtype=flat.dtype, device=t.device)
    mx = mx.scatter_reduce(0, seg, flat.detach(), reduce='amax', include_self=True)
    e = torch.exp(flat - mx[seg])
    s = torch.zeros_like(mx).index_add(0, seg, e)
    return _wrap((e / s[seg]).reshape(t.shape), input.lod())


def _gather_rows(t, idx, lod):
    return _wrap(t.index_select(0, torch.tensor(idx, dtype=torch.long, device=t.device)), lod)


def sequence_concat(input, name=None):
    """Concatenate the i-th sequences of every input (same number of sequences each)."""
    offs = [_offsets(x) for x in input]
    n = len(offs[0]) - 1
    if any(len(o) - 1 != n for o in offs):
        raise ValueError("sequence_concat: inputs must hold the same number of sequences")
    ts = [_u(x) for x in input]
    base = [0]
    for t in ts[:-1]:
        base.append(base[-1] + t.shape[0])
    cat = torch.cat(ts, 0)
    idx, lod = [], [0]
    for i in range(n):
        for k, o in enumerate(offs):
            idx.extend(range(base[k] + o[i], base[k] + o[i + 1]))
        lod.append(len(idx))
    return _gather_rows(cat, idx, [lod])


def sequence_slice(input, offset, length, name=None):
    """Per sequence i keep rows [offset[i], offset[i] + length[i])."""
    off = _offsets(input)
    o = [int(v) for v in _u(offset).reshape(-1).tolist()]
    ln = [int(v) for v in _u(length).reshape(-1).tolist()]
    idx, lod = [], [0]
    for i in range(len(off) - 1):
        if o[i] < 0 or o[i] + ln[i] > off[i + 1] - off[i]:
            raise ValueError(f"sequence_slice: slice {o[i]}+{ln[i]} exceeds sequence {i}")
        idx.extend(range(off[i] + o[i], off[i] + o[i] + ln[i]))
        lod.append(len(idx))
    return _gather_rows(_u(input), idx, [lod])


def sequence_expand(x, y, ref_level=-1, name=None):
    """Repeat the i-th sequence of x (or row i when x has no LoD) by the i-th length of y's
    ``ref_level`` LoD level; every copy is a sequence of the output."""
    ylod = y.lod()
    if not ylod:
        raise ValueError("sequence_expand: y must be a LoD tensor")
    ref = ylod[ref_level]
    reps = [b - a for a, b in zip(ref, ref[1:])]
    t = _u(x)
    xoff = x.lod()[-1] if isinstance(x, Tensor) and x.lod() else list(range(t.shape[0] + 1))
    if len(xoff) - 1 != len(reps):
        raise ValueError(f"sequence_expand: x has {len(xoff) - 1} sequences, y's level has {len(reps)}")
    idx, lod = [], [0]
    for i, r in enumerate(reps):
        for _ in range(r):
            idx.extend(range(xoff[i], xoff[i + 1]))
            lod.append(len(idx))
    return _gather_rows(t, idx, [lod])


def sequence_expand_as(x, y, name=None):
    """Row i of x repeated to the length of y's i-th sequence; the output takes y's LoD."""
    yoff = _offsets(y, 'y')
    t = _u(x)
    lens = torch.tensor([b - a for a, b in zip(yoff, yoff[1:])], dtype=torch.long, device=t.device)
    if lens.numel() != t.shape[0]:
        raise ValueError("sequence_expand_as: x rows must equal the number of y's sequences")
    return _wrap(torch.repeat_interleave(t, lens, dim=0), [yoff])


def sequence_pad(x, pad_value, maxlen=None, name=None):
    """-> (Out [B, maxlen, ...], Length [B] int64); ``pad_value`` is a scalar or one time step."""
    off = _offsets(x)
    t = _u(x)
    lens = [b - a for a, b in zip(off, off[1:])]
    L = max(lens) if maxlen is None or maxlen < 0 else int(maxlen)
    if lens and max(lens) > L:
        raise ValueError(f"sequence_pad: maxlen {L} is shorter than a sequence ({max(lens)})")
    pv = _u(pad_value) if isinstance(pad_value, Tensor) else torch.as_tensor(pad_value)
    pv = pv.to(device=t.device, dtype=t.dtype)
    step = tuple(t.shape[1:])
    out = pv.reshape(-1)[0].expand((len(lens), L) + step).clone() if pv.numel() == 1 else \
        pv.reshape(step).expand((len(lens), L) + step).clone()
    seg, lt = _seg_ids(off, t.device)
    pos = torch.arange(t.shape[0], device=t.device) - torch.tensor(off[:-1], device=t.device)[seg]
    out = out.index_put((seg, pos), t)
    return Tensor(out), Tensor(lt.to(torch.int64))


def sequence_unpad(x, length, name=None):
    """Inverse of sequence_pad: keep the first length[i] steps of row i, as a LoD tensor."""
    t = _u(x)
    ln = [int(v) for v in _u(length).reshape(-1).tolist()]
    seg = torch.repeat_interleave(torch.arange(len(ln)), torch.tensor(ln, dtype=torch.long))
    pos = torch.cat([torch.arange(n) for n in ln]) if ln else torch.zeros(0, dtype=torch.long)
    lod = [0]
    for n in ln:
        lod.append(lod[-1] + n)
    return _wrap(t[seg.to(t.device), pos.to(t.device)], [lod])


def sequence_reshape(input, new_dim):
    """Re-split each sequence's (len x D) block into rows of ``new_dim``."""
    off = _offsets(input)
    t = _u(input)
    d = t.shape[1]
    lod = [0]
    for a, b in zip(off, off[1:]):
        if ((b - a) * d) % new_dim:
            raise ValueError(f"sequence_reshape: sequence of {b - a}x{d} not divisible by {new_dim}")
        lod.append(lod[-1] + (b - a) * d // new_dim)
    return _wrap(t.reshape(-1, new_dim), [lod])


def sequence_scatter(input, index, updates, name=None):
    """out = input; out[i, index[p]] += updates[p] for every p in index's i-th sequence."""
    off = _offsets(index, 'index')
    t = _u(input)
    seg, _ = _seg_ids(off, t.device)
    idx = _u(index).reshape(-1).long().to(t.device)
    upd = _u(updates).reshape(-1).to(t.dtype)
    return Tensor(t.index_put((seg, idx), upd, accumulate=True))


def sequence_enumerate(input, win_size, pad_value=0, name=None):
    """Row n -> [x[n], x[n+1], ..., x[n+win-1]] within its sequence, ``pad_value`` past its end."""
    off = _offsets(input)
    t = _u(input).reshape(-1)
    seg, _ = _seg_ids(off, t.device)
    ends = torch.tensor(off[1:], dtype=torch.long, device=t.device)[seg]
    pos = torch.arange(t.shape[0], device=t.device)[:, None] + torch.arange(win_size, device=t.device)[None]
    valid = pos < ends[:, None]
    vals = t[pos.clamp(max=max(t.shape[0] - 1, 0))]
    out = torch.where(valid, vals, torch.full_like(vals, pad_value))
    return _wrap(out, input.lod())


def sequence_reverse(x, name=None):
    """Reverse the time steps inside every sequence."""
    off = _offsets(x)
    t = _u(x)
    seg, _ = _seg_ids(off, t.device)
    st = torch.tensor(off[:-1], dtype=torch.long, device=t.device)[seg]
    en = torch.tensor(off[1:], dtype=torch.long, device=t.device)[seg]
    pos = torch.arange(t.shape[0], device=t.device)
    return _wrap(t.index_select(0, st + en - 1 - pos), x.lod())


def _context_project(t, off, filter_size, padding_start):
    """[N, D] -> [N, filter_size * D]: row n gathers rows n + padding_start + j (zero outside
    its own sequence)."""
    n, d = t.shape
    seg, _ = _seg_ids(off, t.device)
    st = torch.tensor(off[:-1], dtype=torch.long, device=t.device)[seg]
    en = torch.tensor(off[1:], dtype=torch.long, device=t.device)[seg]
    pos = torch.arange(n, device=t.device)[:, None] + padding_start + \
        torch.arange(filter_size, device=t.device)[None]
    valid = (pos >= st[:, None]) & (pos < en[:, None])
    g = t[pos.clamp(0, max(n - 1, 0))] * valid[..., None].to(t.dtype)
    return g.reshape(n, filter_size * d)


def sequence_conv(input, num_filters, filter_size=3, filter_stride=1, padding=True,
                  padding_start=None, bias_attr=None, param_attr=None, act=None, name=None):
    """Context-projection convolution over each sequence: out = proj(x) · W (+ b), act."""
    from .. import nn as _nn
    from ..nn import functional as F
    from .nn import _keep
    if filter_stride != 1:
        raise ValueError("sequence_conv supports filter_stride = 1 only (as the reference)")
    off = _offsets(input)
    t = _u(input)
    d = t.shape[1]
    ps = -int(filter_size // 2) if padding_start is None else int(padding_start)
    lin = _keep(_nn.Linear(filter_size * d, num_filters, weight_attr=param_attr,
                           bias_attr=bias_attr))
    proj = _context_project(t, off, filter_size, ps)
    out = lin(Tensor(proj))
    if act:
        out = getattr(F, act)(out)
    out.set_lod(input.lod())
    return out


def create_lod_tensor(data, recursive_seq_lens, place=None):
    """A LoD tensor from a numpy array / Tensor / nested list and per-level sequence lengths
    (parity: python/paddle/fluid/lod_tensor.py create_lod_tensor)."""
    import numpy as np
    if isinstance(data, Tensor):
        t = data._t
    elif isinstance(data, list):
        # list of sequences -> rows concatenated, lengths must agree with recursive_seq_lens
        t = torch.as_tensor(np.concatenate([np.asarray(s).reshape(len(s), -1) for s in data], 0))
    else:
        t = torch.as_tensor(np.asarray(data))
    out = Tensor(t)
    out.set_recursive_sequence_lengths(recursive_seq_lens)
    if not out.has_valid_recursive_sequence_lengths():
        raise ValueError(f"sequence lengths {recursive_seq_lens} do not match data of shape {tuple(t.shape)}")
    return out
