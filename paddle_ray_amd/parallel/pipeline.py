"""Pipeline parallelism (parity: python/paddle/distributed/fleet/meta_parallel/
{parallel_layers/pp_layers.py, pipeline_parallel.py, pp_utils/p2p_communication.py}).

* ``PipelineLayer`` builds only this stage's layers from ``LayerDesc`` lists (uniform,
  ``layer:<Name>`` or parameter-balanced segmentation). With
  ``num_virtual_pipeline_stages = V`` the model is cut into ``stages * V`` chunks and stage
  ``s`` holds chunks ``s, s + stages, ...`` (interleaved placement, pp_layers.py
  ``_construct_shared_comm`` / virtual stages).
* ``SharedLayerDesc``: a layer used on several stages (tied input embedding / LM head) is
  built on every owning stage, broadcast from the first owning stage at construction and its
  gradient is all-reduced over the owning stages after each batch
  (pp_layers.py ``_synchronize_shared_weights`` :485, ``allreduce_shared_weight_gradients`` :498).
* ``PipelineParallel.train_batch``: 1F1B (V = 1) or the interleaved schedule over virtual
  chunks (V > 1, ``PipelineParallelWithInterleave``); activations may be tuples of tensors;
  point-to-point isend/irecv over RCCL (xGMI peer links), every transfer registered with the
  collective watchdog. Data-parallel gradients live in flat buckets: with 1F1B the bucket
  all-reduces are launched from the gradient hooks of the LAST micro-batch's backward, so they
  overlap the rest of it; the interleaved schedule reduces all buckets after the schedule.
"""
import math

import torch
import torch.distributed as dist

from ..framework.core import Tensor, _u
from ..nn.layer.layers import Layer
from ..nn.layer.common import LayerList
from ..distributed import watchdog as _watchdog
from .recompute import recompute


class LayerDesc:
    def __init__(self, layer_func, *inputs, **kwargs):
        self.layer_func, self.inputs, self.kwargs = layer_func, inputs, kwargs

    def build_layer(self):
        return self.layer_func(*self.inputs, **self.kwargs)

    def __repr__(self):
        return f'LayerDesc({self.layer_func.__name__})'


class SharedLayerDesc(LayerDesc):
    def __init__(self, key, layer_func, forward_func=None, shared_weight_attr='weight', *inputs,
                 **kwargs):
        super().__init__(layer_func, *inputs, **kwargs)
        self.layer_name, self.forward_func, self.shared_weight_attr = key, forward_func, \
            shared_weight_attr


class SegmentLayers:
    def __init__(self, layers_desc, num_parts, method="uniform"):
        self._descs, self.num_parts, self.method = layers_desc, num_parts, method

    def do_segment(self):
        n = len(self._descs)
        if self.method.startswith('layer:'):
            name = self.method.split(':')[1]
            idx = [i for i, d in enumerate(self._descs)
                   if isinstance(d, LayerDesc) and d.layer_func.__name__ == name]
            per = math.ceil(len(idx) / self.num_parts)
            bounds = [0]
            for p in range(1, self.num_parts):
                bounds.append(idx[min(p * per, len(idx) - 1)])
            bounds.append(n)
            return bounds
        per = n / self.num_parts
        return [int(round(per * i)) for i in range(self.num_parts)] + [n]


def _as_list(x):
    if x is None:
        return []
    if isinstance(x, (list, tuple)):
        return [_u(t) if isinstance(t, Tensor) else t for t in x]
    return [_u(x) if isinstance(x, Tensor) else x]


def _wrap_acts(ts):
    ts = [Tensor(t) if isinstance(t, torch.Tensor) else t for t in ts]
    return ts[0] if len(ts) == 1 else tuple(ts)


class PipelineLayer(Layer):
    def __init__(self, layers, num_stages=None, topology=None, loss_fn=None, seg_method="uniform",
                 recompute_interval=0, recompute_ctx=None, num_virtual_pipeline_stages=None):
        super().__init__()
        from ..distributed import fleet
        hcg = fleet.get_hybrid_communicate_group() if fleet.fleet._hcg is not None else None
        self._hcg = hcg
        self._num_stages = num_stages or (hcg.get_pipe_parallel_world_size() if hcg else 1)
        self._stage_id = hcg.get_stage_id() if hcg else 0
        self._num_virtual = max(1, int(num_virtual_pipeline_stages or 1))
        self._loss_fn = loss_fn
        self._recompute_interval = recompute_interval
        self._layers_desc = list(layers)
        nparts = self._num_stages * self._num_virtual
        self.segment_parts = SegmentLayers(self._layers_desc, nparts, seg_method).do_segment()
        self.shared_layers = {}
        self._chunks = []          # run functions per local virtual chunk
        built = LayerList()
        for v in range(self._num_virtual):
            part = v * self._num_stages + self._stage_id
            lo, hi = self.segment_parts[part], self.segment_parts[part + 1]
            fns = []
            for i in range(lo, hi):
                d = self._layers_desc[i]
                if isinstance(d, SharedLayerDesc):
                    if d.layer_name not in self.shared_layers:
                        self.shared_layers[d.layer_name] = d.build_layer()
                        built.append(self.shared_layers[d.layer_name])
                    l = self.shared_layers[d.layer_name]
                    fns.append((lambda layer, f: (lambda x: f(layer, x)))(l, d.forward_func)
                               if d.forward_func else l)
                elif isinstance(d, LayerDesc):
                    l = d.build_layer()
                    built.append(l)
                    fns.append(l)
                elif isinstance(d, Layer):
                    built.append(d)
                    fns.append(d)
                else:
                    fns.append(d)
            self._chunks.append(fns)
        self.run_function = [f for c in self._chunks for f in c]
        self.run_layers = built
        self._shared_comm = {}
        if self._num_stages > 1 and hcg is not None:
            self._build_shared_comm(hcg)
            self._synchronize_shared_weights()

    # -- shared (tied) layers across stages -----------------------------------------------------
    def _owning_stages(self):
        owners = {}
        for part in range(len(self.segment_parts) - 1):
            stage = part % self._num_stages
            for i in range(self.segment_parts[part], self.segment_parts[part + 1]):
                d = self._layers_desc[i]
                if isinstance(d, SharedLayerDesc):
                    owners.setdefault(d.layer_name, set()).add(stage)
        return {k: sorted(v) for k, v in owners.items()}

    def _build_shared_comm(self, hcg):
        """One group per shared key and per pipe group, over the stages owning that key;
        every rank creates every group in the same order (collective new_group)."""
        from ..distributed import collective as C
        me = C.get_rank()
        attr_of = {d.layer_name: d.shared_weight_attr for d in self._layers_desc
                   if isinstance(d, SharedLayerDesc)}
        for key, stages in sorted(self._owning_stages().items()):
            if len(stages) < 2:
                continue
            for pipe_ranks in hcg.topology().get_comm_list('pipe'):
                ranks = [pipe_ranks[s] for s in stages]
                g = C.new_group(ranks)
                if me in ranks and key in self.shared_layers:
                    self._shared_comm[key] = (g, ranks, attr_of[key])

    def _shared_params(self, key):
        _, _, attr = self._shared_comm[key]
        layer = self.shared_layers[key]
        names = attr if isinstance(attr, (list, tuple)) else [attr]
        out = []
        for n in names:  # dotted paths reach into sublayers ('word_embeddings.weight')
            obj = layer
            for part in n.split('.'):
                obj = getattr(obj, part)
            out.append(obj)
        return out

    def _synchronize_shared_weights(self):
        from ..distributed import collective as C
        me = C.get_rank()
        for key, (g, ranks, _) in self._shared_comm.items():
            for p in self._shared_params(key):
                dist.broadcast(p._t.data, ranks[0], group=g.process_group)
            # the global-norm clip counts a tied weight once: on its first owner only
            # (parity: pp_layers.py:485-496 is_firstly_shared)
            for p in self.shared_layers[key].parameters():
                p.is_firstly_shared = me == ranks[0]

    def allreduce_shared_weight_gradients(self):
        for key, (g, ranks, _) in self._shared_comm.items():
            for p in self._shared_params(key):
                if p._t.grad is not None:
                    _watchdog.track(f'pp.shared[{key}]', dist.all_reduce(
                        p._t.grad, group=g.process_group, async_op=True), len(ranks)).wait()

    # -- forward -------------------------------------------------------------------------------
    def get_stage_from_index(self, idx):
        for part in range(len(self.segment_parts) - 1):
            if self.segment_parts[part] <= idx < self.segment_parts[part + 1]:
                return part % self._num_stages

    def _run(self, fns, x):
        if self._recompute_interval > 0 and self.training:
            k = self._recompute_interval
            for lo in range(0, len(fns), k):
                seg = fns[lo:lo + k]

                def run(*xs, seg=seg):
                    y = xs[0] if len(xs) == 1 else xs
                    for f in seg:
                        y = f(y)
                    return y
                x = recompute(run, *(x if isinstance(x, tuple) else (x,)))
            return x
        for f in fns:
            x = f(x)
        return x

    def forward(self, input, chunk_id=None):
        if chunk_id is not None:
            return self._run(self._chunks[chunk_id], input)
        return self._run(self.run_function, input)


_DT_CODES = [torch.float32, torch.float16, torch.bfloat16, torch.int64, torch.int32, torch.bool,
             torch.uint8, torch.float64]
_META_LEN = 64


class _P2P:
    """Point-to-point activation / gradient exchange between pipeline stages.

    Every DIRECTED channel has its own 2-rank communicator: activations s -> s+1, gradients
    s+1 -> s, and (interleaved schedule only) the ring wrap: activations from the last stage
    to the first and gradients back (parity: the send_next / recv_prev groups of
    pp_utils/p2p_communication.py). On RCCL a communicator is one stream per rank and
    transfers on it are matched in issue order, so a channel with exactly one sender and one
    receiver, both walking the same schedule, can never pair a send with the wrong receive,
    and an activation send never queues behind (or waits for) a gradient transfer travelling
    the other way — the cycle a shared per-pair communicator forms once a message is larger
    than the RCCL staging buffer. Sends are asynchronous (the host never blocks on them);
    receives make the compute stream wait for the transfer. A sent tensor is released as
    soon as its send has completed (checked at every new send), not at batch end.
    Activations may be tuples; only floating tensors carry gradients back."""

    def __init__(self, hcg, virtual=1, partial=True):
        from ..distributed import collective as C
        self.hcg = hcg
        # partial send/recv (parity: pp_utils/p2p_communication.py:180-295): the activation at a
        # stage boundary is identical on every tensor-parallel rank, so each mp rank moves only
        # its 1/mp slice over its own pipe channel and the receiving stage all-gathers the
        # slices over the mp group (xGMI point-to-point bytes / mp; the all-gather rides the
        # mp group's links, which sit idle at the pipeline boundary)
        mg = hcg.get_model_parallel_group() if hasattr(hcg, 'get_model_parallel_group') else None
        self.mp = mg.nranks if (partial and mg is not None) else 1
        self.mp_rank = hcg.get_model_parallel_rank() if self.mp > 1 else 0
        self.mp_pg = mg.process_group if self.mp > 1 else None
        self.bytes_sent = 0   # activation / gradient payload bytes this rank has sent (stats)
        self.stage = hcg.get_stage_id()
        self.nstages = hcg.get_pipe_parallel_world_size()
        g = hcg.get_pipe_parallel_group()
        self.pg = g.process_group
        self.ranks = g.ranks
        self.prev = g.ranks[(self.stage - 1) % self.nstages]
        self.next = g.ranks[(self.stage + 1) % self.nstages]
        self.dev = torch.device('cuda', torch.cuda.current_device()) \
            if torch.cuda.is_available() and dist.get_backend(self.pg) == 'nccl' else \
            torch.device('cpu')
        # channels: (kind, src_stage, dst_stage) -> process group; created by every rank for
        # every pipe group in one global order (new_group is collective)
        n = self.nstages
        edges = [('act', s, s + 1) for s in range(n - 1)] + [('grad', s + 1, s) for s in range(n - 1)]
        if virtual > 1:
            edges += [('act', n - 1, 0), ('grad', 0, n - 1)]
        self.chan = {}
        me = C.get_rank()
        for pipe_ranks in hcg.topology().get_comm_list('pipe'):
            for kind, a, b in edges:
                grp = C.new_group([pipe_ranks[a], pipe_ranks[b]])
                if me in (pipe_ranks[a], pipe_ranks[b]):
                    self.chan[(kind, a, b)] = grp.process_group
        self.meta_from = {}   # channel -> [(shape, dtype)] of what arrives on it
        self.meta_sent = set()
        self.pending = []     # (work, tensor) isends not yet known to be complete
        self.peak_pending = 0

    def _ch(self, kind, a, b):
        return self.chan[(kind, a % self.nstages, b % self.nstages)]

    def _prune(self):
        self.pending = [(w, t) for w, t in self.pending if not w.is_completed()]

    def _partial_ok(self, t):
        return self.mp > 1 and t.numel() > 0 and t.numel() % self.mp == 0

    def _isend(self, t, peer, pg, what, partial=False):
        t = t.detach().contiguous()
        if partial and self._partial_ok(t):
            t = t.view(-1).chunk(self.mp)[self.mp_rank]   # this mp rank's slice (contiguous)
            what = what + '.partial'
        self._prune()
        w = _watchdog.track(f'pp.{what}', dist.isend(t, peer, group=pg), 2)
        if what != 'meta':
            self.bytes_sent += t.numel() * t.element_size()
        self.pending.append((w, t))
        self.peak_pending = max(self.peak_pending, len(self.pending))

    def _recv(self, t, peer, pg, what, partial=False):
        if partial and self._partial_ok(t):
            flat = t.view(-1)
            mine = flat.chunk(self.mp)[self.mp_rank]
            _watchdog.track(f'pp.{what}.partial', dist.irecv(mine, peer, group=pg), 2).wait()
            # every mp rank received its own slice: gather the whole activation
            _watchdog.track(f'pp.{what}.allgather', dist.all_gather_into_tensor(
                flat, mine.clone(), group=self.mp_pg, async_op=True), self.mp).wait()
            return t
        _watchdog.track(f'pp.{what}', dist.irecv(t, peer, group=pg), 2).wait()
        return t

    def send_acts(self, acts, dst_stage):
        pg = self._ch('act', self.stage, dst_stage)
        peer = self.ranks[dst_stage % self.nstages]
        ts = [t for t in acts if isinstance(t, torch.Tensor)]
        if pg not in self.meta_sent:
            m = torch.zeros(_META_LEN, dtype=torch.int64)
            m[0] = len(ts)
            k = 1
            for t in ts:
                m[k], m[k + 1] = t.dim(), _DT_CODES.index(t.dtype)
                m[k + 2:k + 2 + t.dim()] = torch.tensor(list(t.shape))
                k += 2 + t.dim()
            self._isend(m.to(self.dev), peer, pg, 'meta')
            self.meta_sent.add(pg)
        for t in ts:
            self._isend(t, peer, pg, 'send_fwd', partial=True)

    def recv_acts(self, src_stage):
        pg = self._ch('act', src_stage, self.stage)
        peer = self.ranks[src_stage % self.nstages]
        if pg not in self.meta_from:
            m = self._recv(torch.zeros(_META_LEN, dtype=torch.int64, device=self.dev), peer, pg,
                           'meta').cpu()
            n, k, meta = int(m[0]), 1, []
            for _ in range(n):
                nd, dt = int(m[k]), _DT_CODES[int(m[k + 1])]
                meta.append((tuple(int(v) for v in m[k + 2:k + 2 + nd]), dt))
                k += 2 + nd
            self.meta_from[pg] = meta
        out = []
        for shp, dt in self.meta_from[pg]:
            t = self._recv(torch.empty(shp, dtype=dt, device=self.dev), peer, pg, 'recv_fwd',
                           partial=True)
            out.append(t.requires_grad_(t.is_floating_point()))
        return out

    def send_grads(self, grads, dst_stage):
        pg = self._ch('grad', self.stage, dst_stage)
        peer = self.ranks[dst_stage % self.nstages]
        for g in grads:
            self._isend(g, peer, pg, 'send_bwd', partial=True)

    def recv_grads(self, like, src_stage):
        pg = self._ch('grad', src_stage, self.stage)
        peer = self.ranks[src_stage % self.nstages]
        return [self._recv(torch.empty_like(t), peer, pg, 'recv_bwd', partial=True) for t in like
                if t.is_floating_point()]

    def new_batch(self):
        self.meta_from.clear()
        self.meta_sent.clear()  # both sides re-exchange activation meta every batch

    def flush(self):
        for w, _ in self.pending:
            w.wait()
        self.pending.clear()


def interleaved_order(M, nstages, V, stage):
    """The interleaved 1F1B schedule of one stage (parity: pipeline_parallel.py:535-760,
    PipelineParallelWithInterleave): forward unit k runs chunk ``(k // nstages) % V`` on
    micro-batch ``(k // (nstages * V)) * nstages + k % nstages``; backward unit k runs the
    mirrored chunk ``V - 1 - (k // nstages) % V`` on the same micro-batch formula. Returns
    (warmup, [('F'|'B', k), ...]): ``warmup`` forward units first (startup), then one
    forward + one backward per step (steady), then the remaining backwards (cooldown)."""
    total = M * V
    if M == nstages:
        warmup = total
    else:
        warmup = min((nstages - stage - 1) * 2 + (V - 1) * nstages, total)
    seq = [('F', k) for k in range(warmup)]
    for i in range(total - warmup):
        seq += [('F', warmup + i), ('B', i)]
    seq += [('B', k) for k in range(total - warmup, total)]
    return warmup, seq


class PipelineParallel(Layer):
    def __init__(self, layers, hcg, strategy, sharded_state=None):
        super().__init__()
        self._layers = layers
        self._hcg = hcg
        cfg = (strategy.pipeline_configs if strategy is not None else {}) or {}
        self.micro_batch_size = cfg.get('micro_batch_size', 1)
        self.accumulate_steps = cfg.get('accumulate_steps', 1)
        self.is_first = hcg.is_first_stage()
        self.is_last = hcg.is_last_stage()
        V = layers._num_virtual if isinstance(layers, PipelineLayer) else 1
        self._p2p = _P2P(hcg, V, partial=bool(cfg.get('enable_partial_send_recv', True))) \
            if hcg.get_pipe_parallel_world_size() > 1 else None
        self.total_loss = None
        self.peak_live_units = 0
        self._dp_group = hcg.get_data_parallel_group()
        self._dp_reducer = None
        self._state = sharded_state
        if sharded_state is not None:
            # pipeline x sharding (stage 1): the sharding state's bucket reducer all-reduces
            # this stage's gradients over the sharding group (+ dp), the sharded optimizer
            # updates the owned shards and all-gathers the new parameters
            self._dp_reducer = sharded_state.reducer
        elif self._dp_group is not None and self._dp_group.nranks > 1:
            self._build_dp_buckets(strategy)
        if self._dp_reducer is not None:
            self._dp_reducer.enabled = False
            self._dp_reducer.auto_finalize = False  # the schedule decides when to finalize

    def _build_dp_buckets(self, strategy):
        """Flat gradient buckets over this stage's parameters, all-reduced over the dp group
        (GradBucketReducer: one RCCL call per bucket, watchdog-tracked)."""
        from .data_parallel import GradBucketReducer
        from .flat import FlatGroup, group_params_into_buckets
        g = self._dp_group
        params = [p for p in self._layers.parameters() if not p.stop_gradient]
        for p in self._layers.parameters():
            dist.broadcast(p._t.data, g.ranks[0], group=g.process_group)
        mb = getattr(strategy, 'fuse_grad_size_in_MB', 64) if strategy is not None else 64
        self._dp_groups = [FlatGroup(b) for b in group_params_into_buckets(params, int(mb) << 20)]
        self._dp_reducer = GradBucketReducer(self._dp_groups, g.process_group, g.nranks,
                                             'allreduce', name='pp.dp_bucket')

    def forward(self, *a, **k):
        return self._layers(*a, **k)

    def _micro(self, data, i):
        if data is None:
            return None
        mb = self.micro_batch_size
        if isinstance(data, (list, tuple)):
            return tuple(self._micro(d, i) for d in data)
        t = _u(data)
        return t[i * mb:(i + 1) * mb]

    def _run_chunk(self, acts, labels, chunk, last_chunk):
        out = self._layers(_wrap_acts(acts), chunk_id=chunk) if self._layers._num_virtual > 1 \
            else self._layers(_wrap_acts(acts))
        if self.is_last and last_chunk:
            loss = self._layers._loss_fn(out, Tensor(labels) if isinstance(labels, torch.Tensor)
                                         else labels)
            lt = _u(loss)
            if lt.dim():
                lt = lt.mean()
            return [lt / self.accumulate_steps]
        return _as_list(out)

    @staticmethod
    def _backward(xs, ys, gys):
        outs, grads = [], []
        for y, g in zip([y for y in ys if y.is_floating_point()], gys):
            if y.requires_grad:
                outs.append(y)
                grads.append(g)
        if outs:
            torch.autograd.backward(outs, grads if any(g is not None for g in grads) else None)
        return [x.grad if (x.requires_grad and x.grad is not None) else torch.zeros_like(x)
                for x in xs if isinstance(x, torch.Tensor) and x.is_floating_point()]

    def _first_inputs(self, inputs, i):
        x = self._micro(inputs, i)
        return [t for t in (x if isinstance(x, tuple) else (x,))]

    def forward_backward_pipeline(self, data, scaler=None):
        inputs, labels = data if isinstance(data, (list, tuple)) and len(data) == 2 else (data, None)
        M = self.accumulate_steps
        p2p = self._p2p
        if p2p is None:
            losses = []
            for i in range(M):
                if self._dp_reducer is not None:
                    self._dp_reducer.enabled = i == M - 1
                y = self._run_chunk(self._first_inputs(inputs, i), self._micro(labels, i), 0, True)[0]
                if scaler is not None:
                    y = _u(scaler.scale(Tensor(y)))
                y.backward()
                losses.append(y.detach())
            self.peak_live_units = 1
            self.total_loss = torch.stack(losses).sum()
            return self.total_loss
        p2p.new_batch()
        if self._layers._num_virtual > 1:
            losses = self._interleaved(inputs, labels, M, scaler)
        else:
            losses = self._one_f_one_b(inputs, labels, M, scaler)
        p2p.flush()
        loss = torch.stack(losses).sum() if losses else torch.zeros((), device=p2p.dev)
        loss = loss.to(p2p.dev).float()
        if scaler is not None and losses:
            loss = loss / scaler.get_loss_scaling()
        dist.broadcast(loss, p2p.ranks[-1], group=p2p.pg)
        self.total_loss = loss
        return loss

    # -- 1F1B ----------------------------------------------------------------------------------
    def _one_f_one_b(self, inputs, labels, M, scaler):
        p2p = self._p2p
        nst, st = p2p.nstages, p2p.stage
        warmup = min(nst - st - 1, M)
        pending, losses = [], []
        nb = [0]
        self.peak_live_units = 0

        def fwd(i):
            xs = self._first_inputs(inputs, i) if self.is_first else p2p.recv_acts(st - 1)
            ys = self._run_chunk(xs, self._micro(labels, i), 0, True)
            if self.is_last:
                if scaler is not None:
                    ys = [_u(scaler.scale(Tensor(ys[0])))]
                losses.append(ys[0].detach())
            else:
                p2p.send_acts(ys, st + 1)
            pending.append((xs, ys))
            self.peak_live_units = max(self.peak_live_units, len(pending))

        def bwd():
            xs, ys = pending.pop(0)
            gys = [None] if self.is_last else p2p.recv_grads(ys, st + 1)
            nb[0] += 1
            if self._dp_reducer is not None:
                self._dp_reducer.enabled = nb[0] == M  # last micro-batch: launch bucket reduces
            dxs = self._backward(xs, ys, gys)
            if not self.is_first:
                p2p.send_grads(dxs, st - 1)

        for i in range(warmup):
            fwd(i)
        for i in range(M - warmup):
            fwd(warmup + i)
            bwd()
        for _ in range(warmup):
            bwd()
        return losses

    # -- interleaved 1F1B (virtual stages) -----------------------------------------------------
    def _interleaved(self, inputs, labels, M, scaler):
        """Interleaved 1F1B over V virtual chunks per stage (``interleaved_order``): startup
        forwards, then alternating one forward / one backward, then the cooldown backwards.
        Chunk v of the last stage feeds chunk v+1 of the first stage over the ring-wrap
        channel (and gradients travel back the same way). At most ``warmup + 1`` units keep
        their activations alive at once, independent of the number of micro-batches."""
        p2p = self._p2p
        V = self._layers._num_virtual
        nst, st = p2p.nstages, p2p.stage
        if M % nst:
            raise ValueError(f"interleaved pipeline needs accumulate_steps ({M}) to be a "
                             f"multiple of the pipeline degree ({nst})")
        bufs, losses = {}, []
        self.peak_live_units = 0

        def chunk(k, fwd):
            v = (k // nst) % V
            return v if fwd else V - 1 - v

        def micro(k):
            return (k // (nst * V)) * nst + k % nst

        def fwd(k):
            v, m = chunk(k, True), micro(k)
            if st == 0 and v == 0:
                xs = self._first_inputs(inputs, m)
            else:
                xs = p2p.recv_acts(st - 1)   # stage 0 (v > 0): from the last stage, ring wrap
            ys = self._run_chunk(xs, self._micro(labels, m), v, v == V - 1)
            if st == nst - 1 and v == V - 1:
                if scaler is not None:
                    ys = [_u(scaler.scale(Tensor(ys[0])))]
                losses.append(ys[0].detach())
            else:
                p2p.send_acts(ys, st + 1)
            bufs[(v, m)] = (xs, ys)
            self.peak_live_units = max(self.peak_live_units, len(bufs))

        def bwd(k):
            v, m = chunk(k, False), micro(k)
            xs, ys = bufs.pop((v, m))
            last = st == nst - 1 and v == V - 1
            gys = [None] if last else p2p.recv_grads(ys, st + 1)
            if self._dp_reducer is not None:
                # the last micro-batch of each chunk completes that chunk's gradients
                self._dp_reducer.enabled = m == M - 1
            dxs = self._backward(xs, ys, gys)
            if not (st == 0 and v == 0):
                p2p.send_grads(dxs, st - 1)

        _, seq = interleaved_order(M, nst, V, st)
        for op, k in seq:
            fwd(k) if op == 'F' else bwd(k)
        return losses

    # -- gradient reduction + step --------------------------------------------------------------
    def _reduce_dp(self):
        r = self._dp_reducer
        if r is None:
            return
        r.enabled = True
        r.finalize()

    def train_batch(self, data, optimizer, lr_scheduler=None, scaler=None):
        self._layers.train()
        if self._state is not None:
            self._state.before_forward()
        elif self._dp_reducer is not None:
            for g in self._dp_groups:
                if g.grads_missing():
                    g.grad_buf.zero_()
                    g.reattach_grads()
        loss = self.forward_backward_pipeline(data, scaler)
        self._reduce_dp()  # launches what the hooks did not and waits for every bucket
        self._layers.allreduce_shared_weight_gradients()
        if self._dp_reducer is not None:
            self._dp_reducer.enabled = False
        if scaler is not None:
            scaler.step(optimizer)
            scaler.update()
        else:
            optimizer.step()
        optimizer.clear_grad()
        if lr_scheduler is not None:
            lr_scheduler.step()
        return Tensor(loss)

    def eval_batch(self, data, compute_loss=False):
        self._layers.eval()
        with torch.no_grad():
            inputs, labels = data
            out = self._layers(inputs)
            if compute_loss and self._layers._loss_fn is not None:
                return self._layers._loss_fn(out, labels)
            return out


PipelineParallelWithInterleave = PipelineParallel
