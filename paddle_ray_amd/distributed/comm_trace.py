"""Per-rank collective schedule recorder.

``CommTrace`` records, in issue order, every ``torch.distributed`` collective and point-to-point
call this rank makes (the framework's DP / TP / PP / sharding layers all issue through the
``torch.distributed`` module attributes, so wrapping those attributes sees every call), together
with compute markers the caller places (``mark``) or hooks onto layers (``hook_layers``). Each
record carries the op, the payload bytes, the communicator's global ranks, async-ness and the
issuing stream, so a test can assert a whole step's schedule -- op order, byte counts, which
communicator carries what, and that a prefetch all-gather / gradient reduce-scatter is ISSUED
before the compute that depends on it (the overlap the RCCL streams need to get at all).

There is no reference counterpart to copy: Paddle checks its collectives with the
comm-task watchdog (``paddle/fluid/distributed/collective/process_group_nccl.cc``) and the
``CommunicateTopology`` group lists; this is the test-side view of the same schedule.

    with CommTrace() as tr:
        tr.hook_layers({'blk0': model.blocks[0], ...})
        step()
    tr.ops('all_gather_into_tensor')    # -> [Record, ...]
"""
import contextlib
import dataclasses

import torch
import torch.distributed as dist

__all__ = ['CommTrace', 'Record']

_OPS = ('all_reduce', 'all_gather_into_tensor', 'reduce_scatter_tensor', 'all_gather', 'broadcast',
        'reduce', 'reduce_scatter', 'all_to_all_single', 'all_to_all', 'isend', 'irecv', 'send', 'recv',
        'barrier', 'batch_isend_irecv')


@dataclasses.dataclass
class Record:
    seq: int
    kind: str              # 'comm' or 'mark'
    op: str                # collective name, or the marker label
    bytes: int = 0         # payload bytes this rank contributes (input side)
    out_bytes: int = 0     # bytes this rank receives into (output side)
    ranks: tuple = ()      # global ranks of the communicator
    comm: str = ''         # the communicator's name (distinguishes twin groups on equal ranks)
    peer: int = -1         # p2p peer (global rank)
    async_op: bool = False
    stream: int = 0        # issuing HIP stream id (0 on the host)


def _nbytes(x):
    if isinstance(x, torch.Tensor):
        return x.numel() * x.element_size()
    if isinstance(x, (list, tuple)):
        return sum(_nbytes(t) for t in x)
    return 0


def _comm_name(group):
    try:
        return str((group if group is not None else dist.group.WORLD).group_name)
    except Exception:
        return ''


def _ranks(group):
    try:
        return tuple(dist.get_process_group_ranks(group if group is not None else dist.group.WORLD))
    except Exception:
        return ()


class CommTrace(contextlib.AbstractContextManager):
    def __init__(self):
        self.records = []
        self._saved = {}
        self._hooks = []

    # -- recording -----------------------------------------------------------------------------
    def _add(self, **kw):
        self.records.append(Record(seq=len(self.records), **kw))

    def mark(self, label):
        self._add(kind='mark', op=label)

    def _wrap(self, name, fn):
        tr = self

        def w(*a, **k):
            group = k.get('group')
            ins, outs, peer = 0, 0, -1
            if name in ('all_gather_into_tensor', 'reduce_scatter_tensor'):
                outs, ins = _nbytes(a[0] if a else k.get('output_tensor')), _nbytes(a[1] if len(a) > 1 else k.get('input_tensor'))
                group = group if group is not None else (a[3] if len(a) > 3 else None)
            elif name in ('all_gather', 'reduce_scatter', 'all_to_all'):
                outs, ins = _nbytes(a[0] if a else None), _nbytes(a[1] if len(a) > 1 else None)
            elif name == 'all_to_all_single':
                outs, ins = _nbytes(a[0] if a else None), _nbytes(a[1] if len(a) > 1 else None)
            elif name in ('isend', 'send', 'irecv', 'recv'):
                t = a[0] if a else k.get('tensor')
                peer = a[1] if len(a) > 1 else k.get('dst', k.get('src', -1))
                group = group if group is not None else (a[2] if len(a) > 2 else None)
                if name in ('isend', 'send'):
                    ins = _nbytes(t)
                else:
                    outs = _nbytes(t)
            elif name != 'barrier' and name != 'batch_isend_irecv':
                ins = outs = _nbytes(a[0] if a else k.get('tensor'))
            async_op = bool(k.get('async_op', False)) or name in ('isend', 'irecv', 'batch_isend_irecv')
            st = 0
            if torch.cuda.is_available() and torch.cuda.is_initialized():
                st = torch.cuda.current_stream().stream_id
            tr._add(kind='comm', op=name, bytes=ins, out_bytes=outs, ranks=_ranks(group),
                    comm=_comm_name(group),
                    peer=int(peer) if peer is not None else -1, async_op=async_op, stream=st)
            return fn(*a, **k)
        return w

    def __enter__(self):
        for n in _OPS:
            f = getattr(dist, n, None)
            if f is not None:
                self._saved[n] = f
                setattr(dist, n, self._wrap(n, f))
        return self

    def __exit__(self, *exc):
        for n, f in self._saved.items():
            setattr(dist, n, f)
        self._saved.clear()
        for h in self._hooks:
            h.remove()
        self._hooks.clear()
        return False

    # -- compute markers ---------------------------------------------------------------------------
    def hook_layers(self, named):
        """Mark 'fwd:<name>' when each layer's forward starts and 'bwd:<name>' when the gradient
        of its output first arrives (its backward starts)."""
        from ..framework.core import _u
        for name, layer in named.items():
            def pre(l, inputs, name=name):
                self.mark(f'fwd:{name}')

            def post(l, inputs, outputs, name=name):
                fired = [False]
                outs = outputs if isinstance(outputs, (list, tuple)) else [outputs]
                for o in outs:
                    t = _u(o) if not isinstance(o, torch.Tensor) else o
                    if isinstance(t, torch.Tensor) and t.requires_grad:
                        def g(grad, fired=fired, name=name):
                            if not fired[0]:
                                fired[0] = True
                                self.mark(f'bwd:{name}')
                        t.register_hook(g)
            self._hooks.append(layer.register_forward_pre_hook(pre))
            self._hooks.append(layer.register_forward_post_hook(post))

    # -- queries -----------------------------------------------------------------------------------
    def ops(self, *names):
        return [r for r in self.records if r.kind == 'comm' and (not names or r.op in names)]

    def index(self, label):
        for r in self.records:
            if r.kind == 'mark' and r.op == label:
                return r.seq
        raise KeyError(label)

    def summary(self):
        """[(op, bytes, out_bytes, ranks, comm)] of the comm records, in order."""
        return [(r.op, r.bytes, r.out_bytes, r.ranks, r.comm) for r in self.ops()]
