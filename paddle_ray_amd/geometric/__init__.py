"""paddle.geometric (parity: python/paddle/geometric/{math.py,reindex.py,sampling/,
message_passing/send_recv.py}): graph message passing, segment reductions, neighbor
sampling and reindexing. Scatter-reductions map onto torch's index_add / scatter_reduce
(atomic-free segmented kernels on the HIP device)."""
import numpy as np
import torch

from ..framework.core import Tensor, _u


def _w(t):
    return Tensor(t)


def _reduce_into(msg, dst, n, op):
    shape = (n,) + tuple(msg.shape[1:])
    idx = dst.long().view(-1, *([1] * (msg.dim() - 1))).expand_as(msg)
    if op == 'sum':
        return torch.zeros(shape, dtype=msg.dtype, device=msg.device).index_add_(0, dst.long(), msg)
    if op == 'mean':
        s = torch.zeros(shape, dtype=msg.dtype, device=msg.device).index_add_(0, dst.long(), msg)
        c = torch.zeros(n, dtype=msg.dtype, device=msg.device).index_add_(
            0, dst.long(), torch.ones(len(dst), dtype=msg.dtype, device=msg.device))
        return s / c.clamp(min=1).view(-1, *([1] * (msg.dim() - 1)))
    if op in ('max', 'min'):
        out = torch.zeros(shape, dtype=msg.dtype, device=msg.device)
        out = out.scatter_reduce(0, idx, msg, 'amax' if op == 'max' else 'amin', include_self=False)
        return out
    raise ValueError(f"unsupported reduce_op {op}")


def _n_out(x, dst, out_size):
    if out_size is None:
        return x.shape[0]
    n = int(out_size.item()) if isinstance(out_size, (torch.Tensor, Tensor)) else int(out_size)
    return x.shape[0] if n <= 0 else n


def send_u_recv(x, src_index, dst_index, reduce_op='sum', out_size=None, name=None):
    xt, s, d = _u(x), _u(src_index), _u(dst_index)
    return _w(_reduce_into(xt[s.long()], d, _n_out(xt, d, out_size), reduce_op))


def _message(a, b, op):
    return {'add': a + b, 'sub': a - b, 'mul': a * b, 'div': a / b}[op]


def send_ue_recv(x, y, src_index, dst_index, message_op='add', reduce_op='sum', out_size=None,
                 name=None):
    xt, yt, s, d = _u(x), _u(y), _u(src_index), _u(dst_index)
    return _w(_reduce_into(_message(xt[s.long()], yt, message_op), d, _n_out(xt, d, out_size),
                           reduce_op))


def send_uv(x, y, src_index, dst_index, message_op='add', name=None):
    xt, yt = _u(x), _u(y)
    return _w(_message(xt[_u(src_index).long()], yt[_u(dst_index).long()], message_op))


def _segment(data, segment_ids, op):
    t, ids = _u(data), _u(segment_ids).long()
    n = int(ids.max().item()) + 1 if ids.numel() else 0
    return _w(_reduce_into(t, ids, n, op))


def segment_sum(data, segment_ids, name=None):
    return _segment(data, segment_ids, 'sum')


def segment_mean(data, segment_ids, name=None):
    return _segment(data, segment_ids, 'mean')


def segment_max(data, segment_ids, name=None):
    return _segment(data, segment_ids, 'max')


def segment_min(data, segment_ids, name=None):
    return _segment(data, segment_ids, 'min')


def reindex_graph(x, neighbors, count, value_buffer=None, index_buffer=None, name=None):
    """Renumber nodes: input nodes x first (0..len(x)-1), then new neighbors in order of
    first appearance. Returns (reindex_src, reindex_dst, out_nodes)."""
    xs = _u(x).cpu().numpy()
    nb = _u(neighbors).cpu().numpy()
    cnt = _u(count).cpu().numpy()
    mapping = {int(v): i for i, v in enumerate(xs)}
    out_nodes = list(int(v) for v in xs)
    src = np.empty(len(nb), dtype=np.int64)
    for i, v in enumerate(nb):
        v = int(v)
        if v not in mapping:
            mapping[v] = len(out_nodes)
            out_nodes.append(v)
        src[i] = mapping[v]
    dst = np.repeat(np.arange(len(xs), dtype=np.int64), cnt)
    dev = _u(x).device
    mk = lambda a: _w(torch.as_tensor(a, dtype=_u(x).dtype, device=dev))  # noqa: E731
    return mk(src), mk(dst), mk(np.array(out_nodes, dtype=np.int64))


def reindex_heter_graph(x, neighbors, count, value_buffer=None, index_buffer=None, name=None):
    nb = torch.cat([_u(n) for n in neighbors])
    xs = _u(x)
    src_all, dst_all = [], []
    mapping = {int(v): i for i, v in enumerate(xs.cpu().numpy())}
    out_nodes = [int(v) for v in xs.cpu().numpy()]
    for n, c in zip(neighbors, count):
        nbn = _u(n).cpu().numpy()
        for v in nbn:
            v = int(v)
            if v not in mapping:
                mapping[v] = len(out_nodes)
                out_nodes.append(v)
            src_all.append(mapping[v])
        dst_all.append(np.repeat(np.arange(len(xs)), _u(c).cpu().numpy()))
    dev = xs.device
    mk = lambda a: _w(torch.as_tensor(np.asarray(a, dtype=np.int64), dtype=xs.dtype, device=dev))  # noqa
    del nb
    return mk(src_all), mk(np.concatenate(dst_all)), mk(out_nodes)


def sample_neighbors(row, colptr, input_nodes, sample_size=-1, eids=None, return_eids=False,
                     perm_buffer=None, name=None):
    """CSC neighbor sampling without replacement (sample_size=-1: all neighbors)."""
    r = _u(row).cpu().numpy()
    cp = _u(colptr).cpu().numpy()
    nodes = _u(input_nodes).cpu().numpy()
    e = _u(eids).cpu().numpy() if eids is not None else None
    rng = np.random.default_rng(int(torch.randint(0, 2 ** 31 - 1, (1,)).item()))
    outs, cnts, oe = [], [], []
    for v in nodes:
        lo, hi = int(cp[v]), int(cp[v + 1])
        idx = np.arange(lo, hi)
        if 0 <= sample_size < len(idx):
            idx = np.sort(rng.choice(idx, sample_size, replace=False))
        outs.append(r[idx])
        cnts.append(len(idx))
        if e is not None:
            oe.append(e[idx])
    dev = _u(row).device
    mk = lambda a, dt: _w(torch.as_tensor(np.asarray(a), dtype=dt, device=dev))  # noqa: E731
    res = (mk(np.concatenate(outs) if outs else np.zeros(0), _u(row).dtype),
           mk(np.array(cnts), torch.int32))
    if return_eids:
        return res + (mk(np.concatenate(oe) if oe else np.zeros(0), torch.int64),)
    return res


def weighted_sample_neighbors(row, colptr, edge_weight, input_nodes, sample_size=-1, eids=None,
                              return_eids=False, name=None):
    r = _u(row).cpu().numpy()
    cp = _u(colptr).cpu().numpy()
    wts = _u(edge_weight).float().cpu().numpy()
    nodes = _u(input_nodes).cpu().numpy()
    rng = np.random.default_rng(int(torch.randint(0, 2 ** 31 - 1, (1,)).item()))
    outs, cnts = [], []
    for v in nodes:
        lo, hi = int(cp[v]), int(cp[v + 1])
        idx = np.arange(lo, hi)
        if 0 <= sample_size < len(idx):
            p = wts[lo:hi] / wts[lo:hi].sum()
            idx = np.sort(rng.choice(idx, sample_size, replace=False, p=p))
        outs.append(r[idx])
        cnts.append(len(idx))
    dev = _u(row).device
    return (_w(torch.as_tensor(np.concatenate(outs), dtype=_u(row).dtype, device=dev)),
            _w(torch.as_tensor(np.array(cnts), dtype=torch.int32, device=dev)))
