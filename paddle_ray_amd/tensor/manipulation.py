"""Shape / layout manipulation API (parity: python/paddle/tensor/manipulation.py)."""
import numpy as np
import torch

from ..framework.core import Tensor, _u, convert_dtype, _default_device


def _t(x):
    if isinstance(x, Tensor):
        return x._t
    if isinstance(x, torch.Tensor):
        return x
    return torch.as_tensor(np.asarray(x), device=_default_device())


def _ints(s):
    if isinstance(s, Tensor):
        return [int(v) for v in s._t.flatten().tolist()]
    if isinstance(s, (int, np.integer)):
        return [int(s)]
    return [int(v.item()) if isinstance(v, Tensor) else int(v) for v in s]


def reshape(x, shape, name=None):
    t = _t(x)
    shp = _ints(shape)
    # paddle: 0 means "copy this dim from input"
    shp = [t.shape[i] if v == 0 and i < t.dim() else v for i, v in enumerate(shp)]
    return Tensor(t.reshape(shp))


def reshape_(x, shape, name=None):
    object.__setattr__(x, '_t', reshape(x, shape)._t)
    return x


def view(x, shape_or_dtype, name=None):
    t = _t(x)
    if isinstance(shape_or_dtype, (list, tuple)):
        return Tensor(t.view(_ints(shape_or_dtype)))
    return Tensor(t.view(convert_dtype(shape_or_dtype)))


def transpose(x, perm, name=None):
    return Tensor(_t(x).permute(*_ints(perm)))


def t(input, name=None):
    x = _t(input)
    return Tensor(x.t() if x.dim() >= 2 else x)


def moveaxis(x, source, destination, name=None):
    return Tensor(torch.movedim(_t(x), source, destination))


def swapaxes(x, axis0, axis1):
    return Tensor(_t(x).transpose(axis0, axis1))


def concat(x, axis=0, name=None):
    axis = int(axis.item()) if isinstance(axis, Tensor) else axis
    return Tensor(torch.cat([_t(e) for e in x], dim=axis))


def stack(x, axis=0, name=None):
    return Tensor(torch.stack([_t(e) for e in x], dim=axis))


def hstack(x, name=None):
    return Tensor(torch.hstack([_t(e) for e in x]))


def vstack(x, name=None):
    return Tensor(torch.vstack([_t(e) for e in x]))


def split(x, num_or_sections, axis=0, name=None):
    t = _t(x)
    axis = int(axis.item()) if isinstance(axis, Tensor) else int(axis)
    if isinstance(num_or_sections, int):
        n = t.shape[axis]
        assert n % num_or_sections == 0, "split: dimension not divisible"
        return [Tensor(s) for s in torch.split(t, n // num_or_sections, dim=axis)]
    secs = _ints(num_or_sections)
    if -1 in secs:
        i = secs.index(-1)
        secs[i] = t.shape[axis] - (sum(secs) + 1)
    return [Tensor(s) for s in torch.split(t, secs, dim=axis)]


def vsplit(x, num_or_sections, name=None):
    return split(x, num_or_sections, 0)


def hsplit(x, num_or_sections, name=None):
    return split(x, num_or_sections, 1)


def chunk(x, chunks, axis=0, name=None):
    return split(x, chunks, axis)


def unbind(input, axis=0):
    return [Tensor(s) for s in torch.unbind(_t(input), axis)]


def unstack(x, axis=0, num=None):
    return unbind(x, axis)


def squeeze(x, axis=None, name=None):
    t = _t(x)
    if axis is None:
        return Tensor(t.squeeze())
    axes = [a % max(t.dim(), 1) for a in _ints(axis)]
    axes = [a for a in axes if t.dim() and t.shape[a] == 1]
    return Tensor(t.squeeze(tuple(axes)) if axes else t)


def squeeze_(x, axis=None, name=None):
    object.__setattr__(x, '_t', squeeze(x, axis)._t)
    return x


def unsqueeze(x, axis, name=None):
    t = _t(x)
    for a in sorted(_ints(axis)):
        a = a if a >= 0 else a + t.dim() + 1
        t = t.unsqueeze(a)
    return Tensor(t)


def unsqueeze_(x, axis, name=None):
    object.__setattr__(x, '_t', unsqueeze(x, axis)._t)
    return x


def flatten(x, start_axis=0, stop_axis=-1, name=None):
    t = _t(x)
    if t.dim() == 0:
        return Tensor(t.reshape(1))
    return Tensor(t.flatten(start_axis, stop_axis))


def flatten_(x, start_axis=0, stop_axis=-1, name=None):
    object.__setattr__(x, '_t', flatten(x, start_axis, stop_axis)._t)
    return x


def expand(x, shape, name=None):
    return Tensor(_t(x).expand(*_ints(shape)))


def broadcast_to(x, shape, name=None):
    return Tensor(torch.broadcast_to(_t(x), _ints(shape)))


def expand_as(x, y, name=None):
    return Tensor(_t(x).expand_as(_t(y)))


def broadcast_tensors(input, name=None):
    return [Tensor(e) for e in torch.broadcast_tensors(*[_t(i) for i in input])]


def tile(x, repeat_times, name=None):
    return Tensor(_t(x).repeat(*_ints(repeat_times)) if len(_ints(repeat_times)) >= _t(x).dim()
                  else torch.tile(_t(x), tuple(_ints(repeat_times))))


def repeat_interleave(x, repeats, axis=None, name=None):
    r = _t(repeats) if isinstance(repeats, Tensor) else repeats
    return Tensor(torch.repeat_interleave(_t(x), r, dim=axis))


def flip(x, axis, name=None):
    return Tensor(torch.flip(_t(x), _ints(axis)))


reverse = flip


def rot90(x, k=1, axes=[0, 1], name=None):
    return Tensor(torch.rot90(_t(x), k, axes))


def roll(x, shifts, axis=None, name=None):
    return Tensor(torch.roll(_t(x), shifts if not isinstance(shifts, Tensor) else _ints(shifts),
                             axis))


def cast(x, dtype):
    return Tensor(_t(x).to(convert_dtype(dtype)))


def gather(x, index, axis=None, name=None):
    t = _t(x)
    axis = 0 if axis is None else (int(axis.item()) if isinstance(axis, Tensor) else axis)
    idx = _t(index)
    if idx.dim() == 0:
        idx = idx.reshape(1)
    return Tensor(torch.index_select(t, axis, idx.flatten().long()))


def gather_nd(x, index, name=None):
    t = _t(x)
    idx = _t(index).long()
    k = idx.shape[-1]
    flat = idx.reshape(-1, k)
    out = t[tuple(flat[:, i] for i in range(k))]
    return Tensor(out.reshape(list(idx.shape[:-1]) + list(t.shape[k:])))


def scatter(x, index, updates, overwrite=True, name=None):
    t = _t(x).clone()
    idx = _t(index).long().flatten()
    u = _t(updates)
    if overwrite:
        t[idx] = u.to(t.dtype)
    else:
        t[idx] = 0
        t.index_add_(0, idx, u.to(t.dtype))
    return Tensor(t)


def scatter_(x, index, updates, overwrite=True, name=None):
    r = scatter(x, index, updates, overwrite)
    with torch.no_grad():
        x._t.copy_(r._t)
    return x


def scatter_nd_add(x, index, updates, name=None):
    t = _t(x).clone()
    idx = _t(index).long()
    k = idx.shape[-1]
    flat = idx.reshape(-1, k)
    u = _t(updates).reshape([flat.shape[0]] + list(t.shape[k:]))
    t.index_put_(tuple(flat[:, i] for i in range(k)), u.to(t.dtype), accumulate=True)
    return Tensor(t)


def scatter_nd(index, updates, shape, name=None):
    z = torch.zeros(_ints(shape), dtype=_t(updates).dtype, device=_t(updates).device)
    return scatter_nd_add(Tensor(z), index, updates)


def index_select(x, index, axis=0, name=None):
    return Tensor(torch.index_select(_t(x), axis, _t(index).long()))


def index_add(x, index, axis, value, name=None):
    return Tensor(torch.index_add(_t(x), axis, _t(index).long(), _t(value)))


def index_add_(x, index, axis, value, name=None):
    """In-place index_add (parity: python/paddle/tensor/manipulation.py:4723)."""
    t = _t(x)
    t.index_add_(axis, _t(index).long(), _t(value).to(t.dtype))
    return x


def index_put(x, indices, value, accumulate=False, name=None):
    return Tensor(torch.index_put(_t(x), tuple(_t(i) for i in indices), _t(value), accumulate))


def take_along_axis(arr, indices, axis, broadcast=True):
    a, i = _t(arr), _t(indices).long()
    if broadcast:
        shp = list(a.shape)
        shp[axis] = i.shape[axis]
        i = i.expand(shp) if i.dim() == a.dim() else i
    return Tensor(torch.take_along_dim(a, i, axis))


def put_along_axis(arr, indices, values, axis, reduce='assign', include_self=True,
                   broadcast=True):
    a, i = _t(arr), _t(indices).long()
    v = _t(values) if isinstance(values, (Tensor, torch.Tensor)) else \
        torch.full(i.shape, values, dtype=a.dtype, device=a.device)
    if v.dim() == 0:
        v = v.expand(i.shape)
    v = v.to(a.dtype).expand(i.shape) if v.shape != i.shape else v.to(a.dtype)
    if reduce == 'assign':
        return Tensor(a.scatter(axis, i, v))
    red = {'add': 'sum', 'mul': 'prod', 'multiply': 'prod', 'mean': 'mean', 'amax': 'amax',
           'amin': 'amin'}[reduce]
    return Tensor(a.scatter_reduce(axis, i, v, red, include_self=include_self))


def put_along_axis_(arr, indices, values, axis, reduce='assign', include_self=True,
                    broadcast=True):
    """In-place put_along_axis (parity: python/paddle/tensor/manipulation.py put_along_axis_)."""
    arr._t.copy_(_t(put_along_axis(arr, indices, values, axis, reduce, include_self, broadcast)))
    return arr


def take(x, index, mode='raise', name=None):
    t, i = _t(x).flatten(), _t(index).long()
    n = t.numel()
    if mode == 'wrap':
        i = i % n
    elif mode == 'clip':
        i = i.clamp(0, n - 1)
    return Tensor(t[i])


def slice(input, axes, starts, ends):
    t = _t(input)
    idx = [builtins_slice(None)] * t.dim()
    for a, s, e in zip(axes, _ints(starts), _ints(ends)):
        n = t.shape[a]
        s = max(s + n, 0) if s < 0 else min(s, n)
        e = max(e + n, 0) if e < 0 else min(e, n)
        idx[a] = builtins_slice(s, e)
    return Tensor(t[tuple(idx)])


def strided_slice(x, axes, starts, ends, strides, name=None):
    t = _t(x)
    idx = [builtins_slice(None)] * t.dim()
    flips = []
    for a, s, e, st in zip(axes, _ints(starts), _ints(ends), _ints(strides)):
        n = t.shape[a]
        if st > 0:
            s = max(s + n, 0) if s < 0 else min(s, n)
            e = max(e + n, 0) if e < 0 else min(e, n)
            idx[a] = builtins_slice(s, e, st)
        else:
            s = s + n if s < 0 else min(s, n - 1)
            e = e + n if e < -1 or (e < 0 and e != -n - 1) else e
            rng = list(range(s, max(e, -1), st))
            idx[a] = torch.tensor(rng, dtype=torch.long, device=t.device)
            flips.append(a)
    out = t
    for a, ix in enumerate(idx):
        if isinstance(ix, torch.Tensor):
            out = out.index_select(a, ix)
        else:
            sl = [builtins_slice(None)] * out.dim()
            sl[a] = ix
            out = out[tuple(sl)]
    return Tensor(out)


import builtins as _b  # noqa: E402
builtins_slice = _b.slice


def crop(x, shape=None, offsets=None, name=None):
    t = _t(x)
    shape = _ints(shape) if shape is not None else list(t.shape)
    offsets = _ints(offsets) if offsets is not None else [0] * t.dim()
    idx = tuple(builtins_slice(o, o + (s if s != -1 else t.shape[i] - o))
                for i, (o, s) in enumerate(zip(offsets, shape)))
    return Tensor(t[idx])


def shard_index(input, index_num, nshards, shard_id, ignore_value=-1):
    t = _t(input)
    size = (index_num + nshards - 1) // nshards
    in_shard = (t // size) == shard_id
    return Tensor(torch.where(in_shard, t % size, torch.full_like(t, ignore_value)))


def tolist(x):
    return _t(x).tolist()


def shape(input):
    return Tensor(torch.tensor(list(_t(input).shape), dtype=torch.int32))


def unfold(x, axis, size, step, name=None):
    return Tensor(_t(x).unfold(axis, size, step))


def as_strided(x, shape, stride, offset=0, name=None):
    return Tensor(torch.as_strided(_t(x), shape, stride, offset))


def tensordot(x, y, axes=2, name=None):
    if isinstance(axes, Tensor):
        axes = axes.tolist()
    return Tensor(torch.tensordot(_t(x), _t(y), dims=axes))


def atleast_1d(*inputs, name=None):
    r = [Tensor(torch.atleast_1d(_t(i))) for i in inputs]
    return r[0] if len(r) == 1 else r


def atleast_2d(*inputs, name=None):
    r = [Tensor(torch.atleast_2d(_t(i))) for i in inputs]
    return r[0] if len(r) == 1 else r
