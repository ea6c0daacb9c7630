"""Pipeline parallelism (parity: python/paddle/distributed/fleet/meta_parallel/
{parallel_layers/pp_layers.py, pipeline_parallel.py, pp_utils/p2p_communication.py}).

PipelineLayer builds only the local stage's layers from LayerDesc lists
(uniform or parameter-balanced segmentation, SharedLayerDesc for tied
embeddings). PipelineParallel.train_batch runs the 1F1B schedule; the steady
state pairs send/recv with batched isend/irecv so neighbouring stages never
deadlock; activations go point-to-point over RCCL (xGMI peer link).
"""
import math

import numpy as np
import torch
import torch.distributed as dist

from ..framework.core import Tensor, _u
from ..nn.layer.layers import Layer
from ..nn.layer.common import LayerList
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


class PipelineLayer(Layer):
    def __init__(self, layers, num_stages=None, topology=None, loss_fn=None, seg_method="uniform",
                 recompute_interval=0, recompute_ctx=None, num_virtual_pipeline_stages=None):
        super().__init__()
        from ..distributed import fleet
        hcg = fleet.get_hybrid_communicate_group() if fleet.fleet._hcg is not None else None
        self._num_stages = num_stages or (hcg.get_pipe_parallel_world_size() if hcg else 1)
        self._stage_id = hcg.get_stage_id() if hcg else 0
        self._loss_fn = loss_fn
        self._recompute_interval = recompute_interval
        self._layers_desc = list(layers)
        self.segment_parts = SegmentLayers(self._layers_desc, self._num_stages,
                                           seg_method).do_segment()
        lo, hi = self.segment_parts[self._stage_id], self.segment_parts[self._stage_id + 1]
        self.run_function = []
        self.shared_layers = {}
        built = LayerList()
        for i in range(lo, hi):
            d = self._layers_desc[i]
            if isinstance(d, SharedLayerDesc):
                if d.layer_name not in self.shared_layers:
                    self.shared_layers[d.layer_name] = d.build_layer()
                    built.append(self.shared_layers[d.layer_name])
                l = self.shared_layers[d.layer_name]
                fn = (lambda layer, f: (lambda x: f(layer, x)))(l, d.forward_func) \
                    if d.forward_func else l
                self.run_function.append(fn)
            elif isinstance(d, LayerDesc):
                l = d.build_layer()
                built.append(l)
                self.run_function.append(l)
            elif isinstance(d, Layer):
                built.append(d)
                self.run_function.append(d)
            else:
                self.run_function.append(d)
        self.run_layers = built

    def get_stage_from_index(self, idx):
        for s in range(self._num_stages):
            if self.segment_parts[s] <= idx < self.segment_parts[s + 1]:
                return s

    def forward(self, input):
        x = input
        fns = self.run_function
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


_DT_CODES = [torch.float32, torch.float16, torch.bfloat16, torch.int64, torch.int32, torch.bool]


class _P2P:
    def __init__(self, hcg):
        self.hcg = hcg
        self.stage = hcg.get_stage_id()
        self.nstages = hcg.get_pipe_parallel_world_size()
        g = hcg.get_pipe_parallel_group()
        self.pg = g.process_group
        self.prev = g.ranks[self.stage - 1] if self.stage > 0 else None
        self.next = g.ranks[self.stage + 1] if self.stage < self.nstages - 1 else None
        self.dev = torch.device('cuda', torch.cuda.current_device()) \
            if torch.cuda.is_available() and dist.get_backend(self.pg) == 'nccl' else \
            torch.device('cpu')
        self.recv_meta = None
        self.sent_meta = False

    def _send_meta(self, t):
        m = torch.zeros(16, dtype=torch.int64, device=self.dev)
        m[0] = t.dim()
        m[1] = _DT_CODES.index(t.dtype)
        m[2:2 + t.dim()] = torch.tensor(list(t.shape))
        dist.send(m, self.next, group=self.pg)

    def _recv_meta(self):
        m = torch.zeros(16, dtype=torch.int64, device=self.dev)
        dist.recv(m, self.prev, group=self.pg)
        nd = int(m[0])
        self.recv_meta = (tuple(int(v) for v in m[2:2 + nd]), _DT_CODES[int(m[1])])

    def send_fwd(self, t):
        if self.next is None:
            return
        if not self.sent_meta:
            self._send_meta(t)
            self.sent_meta = True
        dist.send(t.detach().contiguous(), self.next, group=self.pg)

    def recv_fwd(self):
        if self.prev is None:
            return None
        if self.recv_meta is None:
            self._recv_meta()
        shp, dt = self.recv_meta
        t = torch.empty(shp, dtype=dt, device=self.dev)
        dist.recv(t, self.prev, group=self.pg)
        return t.requires_grad_(t.is_floating_point())

    def send_bwd(self, g):
        if self.prev is None or g is None:
            return
        dist.send(g.contiguous(), self.prev, group=self.pg)

    def recv_bwd(self, like):
        if self.next is None:
            return None
        t = torch.empty_like(like)
        dist.recv(t, self.next, group=self.pg)
        return t

    def send_fwd_recv_bwd(self, y):
        if self.next is None:
            return None
        g = torch.empty_like(y)
        ops = [dist.P2POp(dist.isend, y.detach().contiguous(), self.next, self.pg),
               dist.P2POp(dist.irecv, g, self.next, self.pg)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        return g

    def send_bwd_recv_fwd(self, dx):
        if self.prev is None:
            return None
        shp, dt = self.recv_meta
        x = torch.empty(shp, dtype=dt, device=self.dev)
        ops = [dist.P2POp(dist.isend, dx.contiguous(), self.prev, self.pg),
               dist.P2POp(dist.irecv, x, self.prev, self.pg)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        return x.requires_grad_(x.is_floating_point())


class PipelineParallel(Layer):
    def __init__(self, layers, hcg, strategy):
        super().__init__()
        self._layers = layers
        self._hcg = hcg
        cfg = (strategy.pipeline_configs if strategy is not None else {}) or {}
        self.micro_batch_size = cfg.get('micro_batch_size', 1)
        self.accumulate_steps = cfg.get('accumulate_steps', 1)
        self.is_first = hcg.is_first_stage()
        self.is_last = hcg.is_last_stage()
        self._p2p = _P2P(hcg) if hcg.get_pipe_parallel_world_size() > 1 else None
        self.total_loss = None
        # DP over the data-parallel axis: gradient all-reduce after the schedule
        self._dp_group = hcg.get_data_parallel_group()

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

    def _fwd(self, x, labels):
        out = self._layers(Tensor(x) if isinstance(x, torch.Tensor) else x)
        if self.is_last:
            loss = self._layers._loss_fn(out, Tensor(labels) if isinstance(labels, torch.Tensor)
                                         else labels)
            lt = _u(loss)
            if lt.dim():
                lt = lt.mean()
            return lt / self.accumulate_steps
        return _u(out)

    def _bwd(self, x, y, dy):
        if self.is_last:
            y.backward()
        else:
            torch.autograd.backward(y, dy)
        return x.grad if isinstance(x, torch.Tensor) and x.requires_grad else None

    def forward_backward_pipeline(self, data, scaler=None):
        inputs, labels = data if isinstance(data, (list, tuple)) and len(data) == 2 else (data, None)
        M = self.accumulate_steps
        p2p = self._p2p
        if p2p is None:
            losses = []
            for i in range(M):
                x = self._micro(inputs, i)
                y = self._fwd(x, self._micro(labels, i))
                y.backward()
                losses.append(y.detach())
            self.total_loss = torch.stack(losses).sum()
            return self.total_loss
        p2p.sent_meta = False
        p2p.recv_meta = None  # both sides re-exchange activation meta every batch
        nst, st = p2p.nstages, p2p.stage
        warmup = min(nst - st - 1, M)
        remaining = M - warmup
        pending, losses = [], []

        def get_x(i):
            if self.is_first:
                x = self._micro(inputs, i)
                return x
            return None

        for i in range(warmup):
            x = get_x(i) if self.is_first else p2p.recv_fwd()
            y = self._fwd(x, self._micro(labels, i))
            p2p.send_fwd(y)
            pending.append((x, y))
            if self.is_last:
                losses.append(y.detach())
        x = None
        if remaining > 0:
            x = get_x(warmup) if self.is_first else p2p.recv_fwd()
        for i in range(remaining):
            y = self._fwd(x, self._micro(labels, warmup + i))
            if self.is_last:
                losses.append(y.detach())
                dy = None
            else:
                dy = p2p.send_fwd_recv_bwd(y)
            pending.append((x, y))
            x0, y0 = pending.pop(0)
            dx = self._bwd(x0, y0, dy if not self.is_last else None) if True else None
            if i == remaining - 1:
                p2p.send_bwd(dx)
            else:
                if self.is_first:
                    x = get_x(warmup + i + 1)
                else:
                    x = p2p.send_bwd_recv_fwd(dx)
                if self.is_first:
                    pass
        for i in range(warmup):
            x0, y0 = pending.pop(0)
            dy = p2p.recv_bwd(y0) if not self.is_last else None
            dx = self._bwd(x0, y0, dy)
            p2p.send_bwd(dx)
        # last stage owns the loss; broadcast it over the pipe group for reporting
        loss = torch.stack(losses).sum() if losses else torch.zeros((), device=p2p.dev)
        loss = loss.to(p2p.dev).float()
        dist.broadcast(loss, p2p.hcg.get_pipe_parallel_group().ranks[-1], group=p2p.pg)
        self.total_loss = loss
        return loss

    def _dp_allreduce(self):
        g = self._dp_group
        if g is None or g.nranks <= 1:
            return
        for p in self._layers.parameters():
            if p._t.grad is not None:
                dist.all_reduce(p._t.grad, group=g.process_group)
                p._t.grad.div_(g.nranks)

    def train_batch(self, data, optimizer, lr_scheduler=None, scaler=None):
        self._layers.train()
        loss = self.forward_backward_pipeline(data, scaler)
        self._dp_allreduce()
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
