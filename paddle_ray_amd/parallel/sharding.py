"""ZeRO sharding stages 1/2/3 over RCCL (parity:
python/paddle/distributed/sharding/group_sharded.py (group_sharded_parallel,
save_group_sharded_model), python/paddle/distributed/fleet/meta_parallel/sharding/
group_sharded_stage2.py, group_sharded_stage3.py, group_sharded_optimizer_stage2.py,
python/paddle/distributed/fleet/meta_optimizers/dygraph_optimizer/dygraph_sharding_optimizer.py).

One mechanism, three schedules (MI355X-first):
  * parameters of a bucket ("unit", default 128 MB) live in one flat buffer
    (``FlatGroup``); rank r OWNS the r-th contiguous shard of every bucket;
  * optimizer state (fp32 master, Adam moments) exists only for the owned shard;
    ONE fused multi-tensor AdamW launch updates every owned shard piece and
    writes the new bf16 values straight into the owned slice of the flat param
    buffer (the all-gather source, in place);
  * level 'os'    (stage 1): grads all-reduced (full), update own shard, all-gather params after step;
    level 'os_g'  (stage 2): grads reduce-scattered into the owner shard as each bucket completes
                             in backward, update, all-gather params after step;
    level 'p_g_os'(stage 3): as stage 2 but params are kept sharded after the step and all-gathered
                             lazily at the next forward: every bucket's all-gather is issued up front
                             on the RCCL stream and each layer waits only for its own bucket, so the
                             gather overlaps the forward compute. With 288 GB HBM the gathered
                             buffers stay resident through backward (no backward re-gather traffic).
"""
import contextlib
import math

import torch
import torch.distributed as dist

from ..framework.core import Tensor, Parameter, _u
from ..nn.layer.layers import Layer
from ..ops import fused as K
from ..ops import _native
from ..ops import registry as R
from .data_parallel import GradBucketReducer, _avg_supported
from .flat import FlatGroup, group_params_into_buckets
from ..distributed import watchdog as _watchdog

LEVELS = {'os': 1, 'os_g': 2, 'p_g_os': 3}


def _find_units(layer, exclude=()):
    """ZeRO-3 units: the members of the outermost LayerList / Sequential containers (the
    repeated blocks), in forward order. Parameters outside every unit (embeddings, heads,
    final norms) belong to the root and stay gathered for the whole step (FSDP-root style)."""
    from ..nn.layer.common import LayerList, Sequential
    units = []

    def walk(m):
        for child in m.children():
            if isinstance(child, exclude):
                continue
            if isinstance(child, (LayerList, Sequential)):
                units.extend(c for c in child.children() if not isinstance(c, exclude))
            else:
                walk(child)
    if isinstance(layer, (LayerList, Sequential)):
        units.extend(layer.children())
    else:
        walk(layer)
    return units


def _tensors_in(obj):
    if isinstance(obj, torch.Tensor):
        yield obj
    elif isinstance(obj, Tensor):
        yield obj._t
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            yield from _tensors_in(o)
    elif isinstance(obj, dict):
        for o in obj.values():
            yield from _tensors_in(o)


def _in_backward():
    return torch._C._current_graph_task_id() != -1


class _Unit:
    __slots__ = ('index', 'layer', 'gids')

    def __init__(self, index, layer, gids):
        self.index, self.layer, self.gids = index, layer, gids


class ShardedState:
    """Flat buckets + owned-shard optimizer state for one model.

    Stage 3 (``p_g_os``) with more than one rank is real ZeRO-3 (parity:
    group_sharded_stage3.py ``_release_param`` :925, ``_allgather_buffer`` :985,
    ``_register_forward_hooks`` / ``_register_backward_hooks``):
      * every parameter of a unit (a repeated block) larger than ``segment_size`` elements
        lives in a per-unit flat buffer of which a rank keeps ONLY its owned shard; the
        full buffer exists only while the unit runs;
      * forward: the unit's pre-hook waits for its all-gather and prefetches the next unit's
        on the RCCL stream; its post-hook frees the gathered buffer again and hooks the
        unit's outputs so that, in backward, the gradient arriving at them re-gathers the
        unit (prefetching the previous one) before the unit's backward kernels run;
      * backward: once the unit's gradients are accumulated the reduce-scatter is launched
        and the gathered buffer is freed; after the reduce-scatter completes the full
        gradient buffer is freed too — only owned shards stay resident between steps.
    Small parameters (biases, norms, ``<= segment_size``), parameters outside units and those of
    sublayers flagged ``_zero3_resident`` (read outside their unit's forward) stay resident
    (gathered once per step after the optimizer update, like stage 2).
    ``dp_group``: hybrid dp x sharding — shard gradients are then averaged over the replicas.
    """

    def __init__(self, layer, level, group=None, segment_bytes=128 << 20, grad_fp32=False,
                 dp_group=None, segment_size=2 ** 20, exclude_layer=None,
                 release_after_forward=True):
        from ..distributed import collective as C
        self.layer = layer
        self.stage = LEVELS[level] if isinstance(level, str) else int(level)
        self.group = group
        self.pg = None if group is None else group.process_group
        self.world = C.get_world_size(group)
        self.rank = C.get_rank(group)
        self.dp_group = dp_group
        self.dp_pg = None if dp_group is None else dp_group.process_group
        self.dp_world = 1 if dp_group is None else dp_group.nranks
        params = [p for p in layer.parameters() if not p.stop_gradient]
        if self.world > 1 or self.dp_world > 1:
            # the sharding group (None = the whole job) and, in hybrid dp x sharding, the dp
            # group (None = no dp replicas: nothing to broadcast there)
            for i, (grp, pg, n) in enumerate(((group, self.pg, self.world),
                                              (dp_group, self.dp_pg, self.dp_world))):
                if n == 1 or (i == 1 and dp_group is None):
                    continue
                src = grp.ranks[0] if grp is not None else 0
                for t in [p._t for p in layer.parameters()] + [b._t for b in layer.buffers()]:
                    dist.broadcast(t.data, src, group=pg)
        self.zero3 = self.stage == 3 and self.world > 1
        self.units = []
        unit_of = {}
        if self.zero3:
            excl = tuple(exclude_layer) if exclude_layer else ()
            for u in _find_units(layer, excl):
                # sublayers flagged _zero3_resident are read outside the unit's forward (e.g.
                # GPT's next-block LayerNorm fused into the previous block): never released
                shared = {id(p) for m in u.sublayers(include_self=True)
                          if getattr(m, '_zero3_resident', False) for p in m.parameters()}
                for p in u.parameters():
                    if not p.stop_gradient and p._t.numel() > segment_size and id(p) not in shared:
                        unit_of.setdefault(id(p), len(self.units))
                self.units.append(u)
        resident = [p for p in params if id(p) not in unit_of]
        buckets = group_params_into_buckets(resident, segment_bytes)
        unit_buckets = []
        for ui in range(len(self.units)):
            ps = [p for p in params if unit_of.get(id(p)) == ui]
            # one bucket per unit (or a few when a unit exceeds the bucket size)
            unit_buckets.append(group_params_into_buckets(ps, max(segment_bytes, 1), reverse=False)
                                if ps else [])
        self.groups = [FlatGroup(b, self.world, self.rank) for b in buckets]
        self.n_resident = len(self.groups)
        self.unit_meta = []
        for ui, ub in enumerate(unit_buckets):
            gids = []
            for b in ub:
                g = FlatGroup(b, self.world, self.rank)
                g.own_shard()
                gids.append(len(self.groups))
                self.groups.append(g)
            self.unit_meta.append(_Unit(ui, self.units[ui], gids))
        self.unit_meta = [u for u in self.unit_meta if u.gids]
        for i, u in enumerate(self.unit_meta):
            u.index = i
        self.release_after_forward = self._resolve_release(release_after_forward)
        # ZeRO-3 all-gathers run on their own communicator (own RCCL stream), so the backward
        # prefetch of unit i-1 is not queued behind unit i's gradient reduce-scatter
        self.ag_pg = self.pg
        if self.zero3:
            from ..distributed import collective as C
            self.ag_group = C.twin_group(group)
            self.ag_pg = self.ag_group.process_group
        self.shard_grads = [g.shard(g.grad_buf) if self.world == 1 else
                            torch.zeros(g.shard_numel, dtype=g.grad_dtype, device=g.device)
                            for g in self.groups]
        if self.stage == 1:
            # stage 1 reduces the full grad buffer; the owned slice of it is the shard grad
            self.shard_grads = [g.shard(g.grad_buf) for g in self.groups]
        mode = 'allreduce' if self.stage == 1 else 'reduce_scatter'
        self.reducer = GradBucketReducer(
            self.groups, self.pg, self.world, mode, self.shard_grads, dp_pg=self.dp_pg,
            dp_world=self.dp_world, on_launch=self._on_grads_launched if self.zero3 else None,
            on_finalize=self._on_backward_done if self.zero3 else None,
            name=f'sharding{self.stage}', accumulate=self.zero3) \
            if self.stage > 1 or self.world > 1 or self.dp_world > 1 else None
        self.gather_works = {}
        self.params_stale = False
        self._param_bucket = {}
        for gi, g in enumerate(self.groups):
            for p in g.params:
                self._param_bucket[id(p)] = gi
        self._unit_gid = {}
        for u in self.unit_meta:
            for gi in u.gids:
                self._unit_gid[gi] = u
        self._hooks = []
        self._rs_window = []
        self.peak_resident_bytes = 0
        self.on_params_loaded = []
        self.step_overlap = None  # _StepOverlap, set by a one-rank ShardedOptimizer
        if self.zero3:
            for u in self.unit_meta:
                self._hooks.append(u.layer.register_forward_pre_hook(self._make_pre(u)))
                self._hooks.append(u.layer.register_forward_post_hook(self._make_post(u)))
                for gi in u.gids:
                    self.groups[gi].release_params()
                    self.groups[gi].release_grads()

    def _resolve_release(self, mode):
        """``release_after_forward``: True (the default, as the reference's ForwardPostHooks,
        group_sharded_stage3.py:828) frees every unit after its forward and re-gathers it in
        backward (minimum memory); False keeps the gathered units resident from their forward to
        their gradient reduce-scatter (no backward re-gather traffic); 'auto' (opt-in) keeps
        them when the full unit parameters fit in ``PRA_ZERO3_RESIDENT_FRAC`` (default 0.25) of
        the device memory LEFT FREE at wrap time — SURVEY §3: with 288 GB per MI355X a 1.3B
        model's gathered bf16 weights (2.6 GB) are about 1 % of HBM. ``PRA_ZERO3_RESIDENT=1``
        turns the resident mode on (0: off) whatever the argument."""
        env = __import__('os').environ.get('PRA_ZERO3_RESIDENT')
        if env is not None:
            return env in ('0', 'false', 'False')
        if mode != 'auto':
            return bool(mode)
        if not self.zero3 or not self.groups or self.groups[0].device.type != 'cuda':
            return True
        unit_bytes = sum(self.groups[gi].numel * self.groups[gi].param_buf.element_size()
                         for u in self.unit_meta for gi in u.gids)
        total = torch.cuda.mem_get_info(self.groups[0].device)[0]
        frac = float(__import__('os').environ.get('PRA_ZERO3_RESIDENT_FRAC', '0.25'))
        return unit_bytes > frac * total

    # -- memory accounting ----------------------------------------------------------------
    def resident_bytes(self):
        return sum(g.resident_bytes() for g in self.groups)

    def _note_peak(self):
        b = self.resident_bytes()
        if b > self.peak_resident_bytes:
            self.peak_resident_bytes = b

    def full_bytes(self):
        return sum(g.numel * (g.param_buf.element_size() + g.grad_buf.element_size())
                   for g in self.groups)

    # -- ZeRO-3 unit residency -----------------------------------------------------------------
    def _gather_group(self, gi):
        g = self.groups[gi]
        if not g.params_released or gi in self.gather_works:
            return
        g.materialize_params()
        self.gather_works[gi] = _watchdog.track(f'sharding3.all_gather[{gi}]', dist.all_gather_into_tensor(
            g.param_buf, g.param_shard, group=self.ag_pg, async_op=True), self.world)
        self._note_peak()

    def _gather_unit(self, u, wait):
        for gi in u.gids:
            self._gather_group(gi)
        if wait:
            for gi in u.gids:
                w = self.gather_works.pop(gi, None)
                if w is not None:
                    w.wait()

    def _release_unit(self, u):
        for gi in u.gids:
            w = self.gather_works.pop(gi, None)
            if w is not None:
                w.wait()
            self.groups[gi].release_params()

    def _prepare_backward(self, u):
        self._gather_unit(u, wait=True)
        for gi in u.gids:
            self.groups[gi].materialize_grads()
            self.groups[gi].reattach_grads()
        if u.index > 0:
            self._gather_unit(self.unit_meta[u.index - 1], wait=False)
        self._note_peak()

    def _make_pre(self, u):
        def hook(layer, inputs):
            if _in_backward():  # recompute re-running the unit inside backward
                self._prepare_backward(u)
                return
            self._gather_unit(u, wait=True)
            if u.index + 1 < len(self.unit_meta):
                self._gather_unit(self.unit_meta[u.index + 1], wait=False)
        return hook

    def _make_post(self, u):
        def hook(layer, inputs, outputs):
            if _in_backward():
                return
            if torch.is_grad_enabled():
                fired = [False]

                def grad_hook(grad, u=u, fired=fired):
                    if not fired[0]:
                        fired[0] = True
                        self._prepare_backward(u)
                for t in _tensors_in(outputs):
                    if t.requires_grad:
                        t.register_hook(grad_hook)
            if self.release_after_forward:
                self._note_peak()
                self._release_unit(u)
        return hook

    def _on_grads_launched(self, gi):
        if gi in self._unit_gid and _in_backward():
            # every gradient of this bucket is final: its gathered parameters are dead
            self.groups[gi].release_params()
            # keep at most two reduce-scatters in flight; older ones are complete on the
            # compute stream's timeline (wait = stream dependency, no host sync), so their
            # full gradient buffers can go back to the allocator
            self._rs_window.append(gi)
            while len(self._rs_window) > 2:
                old = self._rs_window.pop(0)
                for g2, w in self.reducer.works:
                    if g2 == old:
                        w.wait()
                self._note_peak()
                self.groups[old].release_grads()

    def _on_backward_done(self):
        self._rs_window = []
        self._note_peak()
        for u in self.unit_meta:
            for gi in u.gids:
                self.groups[gi].release_params()
                self.groups[gi].release_grads()

    # -- params all-gather (resident groups) ------------------------------------------------
    def launch_gathers(self, order=None):
        if self.world == 1:
            self.params_stale = False
            return
        n = self.n_resident
        order = range(n - 1, -1, -1) if order is None else order
        for gi in order:  # buckets are in backward order: gather forward-first buckets first
            g = self.groups[gi]
            self.gather_works[gi] = _watchdog.track(f'sharding.all_gather[{gi}]', dist.all_gather_into_tensor(
                g.param_buf, g.param_shard, group=self.pg, async_op=True), self.world)
        self.params_stale = False

    def wait_gathers(self):
        for gi in list(self.gather_works):
            self.gather_works.pop(gi).wait()

    def before_forward(self):
        ov = self.step_overlap
        if ov is not None:
            if any(not g.grads_released and g.grads_missing() for g in self.groups):
                ov.sync()
            else:
                ov.before_forward()
        for g in self.groups:
            if not g.grads_released and g.grads_missing():
                g.grad_buf.zero_()
                g.reattach_grads()
        if self.params_stale:
            self.launch_gathers()
            self.wait_gathers()
        if self.zero3 and self.unit_meta:
            self._gather_unit(self.unit_meta[0], wait=False)  # prefetch the first unit

    def after_step(self):
        self.params_stale = True
        if self.zero3:
            for u in self.unit_meta:  # gathered copies (e.g. from state_dict) are stale now
                self._release_unit(u)
        if self.stage in (1, 2):
            self.launch_gathers()
            self.wait_gathers()

    def sync_params(self):
        """Make every parameter hold its full current value (resident and unit groups)."""
        if self.step_overlap is not None:
            self.step_overlap.sync()
        if self.params_stale:
            self.launch_gathers()
        for u in self.unit_meta:
            self._gather_unit(u, wait=False)
        self.wait_gathers()

    def release_all(self):
        for u in self.unit_meta:
            self._release_unit(u)

    def zero_grad(self):
        """Zero the flat gradient slabs in ONE multi-tensor launch. (Running the fill on a side
        stream under the next forward measured 131.0 vs 126.2 ms per GPT-1.3B step: the fill's
        workgroups take CU slots from the one-workgroup-per-CU persistent GEMMs,
        profiles/r6/zero_side_stream_ab.md.)"""
        bufs = [g.grad_buf for g in self.groups if not g.grads_released]
        if self.stage > 1 and self.world > 1:
            bufs += list(self.shard_grads)
        if bufs:
            K.zero_tensors(bufs)
        for g in self.groups:
            if not g.grads_released:
                g.reattach_grads()
        if self.reducer is not None:
            self.reducer.reset_accumulation()

    def params_loaded(self):
        """Full parameter values were written into the gathered buffers (set_state_dict):
        refresh the owned shards and the optimizer's fp32 masters from them."""
        for gi in range(self.n_resident, len(self.groups)):
            g = self.groups[gi]
            if not g.params_released:
                g.param_shard.copy_(g.shard(g.param_buf))
        for cb in self.on_params_loaded:
            cb()


class _StepOverlap:
    """One-GPU optimizer / next-forward overlap (``PRA_OPT_OVERLAP=1``, opt-in; applies with one
    rank, no dp replicas, no offload, device update kernels).

    The update of step t is queued on a side HIP stream in the NEXT forward's order: the root
    parameters (embeddings, final norm, head) first, then unit 0, 1, ... (the repeated blocks,
    ``_find_units``), one multi-tensor launch per phase with an event after each. The next
    forward waits for the root and unit-0 phases before it starts and each unit waits, in its
    forward pre-hook, for its own phase and the next unit's (GPT applies block 0's LayerNorm
    before calling it and fuses the next block's LayerNorm into the previous block); the last
    unit waits for everything. Gradient zeroing from ``clear_grad`` follows the updates on the same
    stream. The update is an HBM-bound stream over 28 B per parameter (fp32 master + moments,
    bf16 grad and copy) while the forward GEMMs are MFMA-bound, so the two share the chip
    instead of running back to back. Anything that reads parameters, gradients or optimizer
    state from outside a forward (state dicts, a second optimizer step) first joins the side
    stream (``sync``). Units must only read their own, earlier units' or the next unit's
    parameters.

    Measured on GPT-3 1.3B (profiles/r3j/opt_overlap_ab.md): the phases do run under the
    forward, but sharing the CUs slows both sides (forward GEMMs 2-3x, the update 1.5x) and the
    forward is gated on the update's progress, so the step is ~1 ms slower than the serial
    update (132.1 vs 131.1 ms): off by default."""

    @classmethod
    def maybe(cls, opt):
        import os
        st = opt.state
        if os.environ.get('PRA_OPT_OVERLAP', '0') != '1' or opt._offload or st.world != 1 \
                or st.dp_world != 1 or not st.groups or st.groups[0].device.type != 'cuda' \
                or not _native.available() or opt._kind not in ('AdamW', 'Momentum', 'SGD') \
                or opt._mp_pg is not None or opt._norm_pgs:
            return None
        units = _find_units(st.layer)
        if len(units) < 2:
            return None
        return cls(opt, units)

    def __init__(self, opt, units):
        st = opt.state
        unit_of = {}
        for ui, u in enumerate(units):
            for p in u.parameters():
                unit_of.setdefault(id(p), ui)
        nph = len(units) + 1
        self.phase_pieces = [[] for _ in range(nph)]
        for i, (gi, p, lo, hi, plo) in enumerate(opt._pieces):
            self.phase_pieces[unit_of.get(id(p), -1) + 1].append(i)
        self.plans = [None] * nph
        self.device = st.groups[0].device
        self.stream = torch.cuda.Stream(device=self.device)
        self.events = [None] * nph
        self.final = None
        self.hooks = [u.register_forward_pre_hook(self._make_wait(ui, len(units)))
                      for ui, u in enumerate(units)]

    def _make_wait(self, ui, n):
        def hook(layer, inputs):
            if ui == n - 1:
                self.sync()
            else:
                self._wait(ui + 2)
        return hook

    def _wait(self, ph):
        # the latest recorded event at or before phase ph: a phase with no trainable pieces
        # records none, and must not let the reader skip an earlier phase still being written
        for i in range(min(ph, len(self.events) - 1), -1, -1):
            ev = self.events[i]
            if ev is not None:
                torch.cuda.current_stream(self.device).wait_event(ev)
                return

    def before_forward(self):
        self._wait(1)  # root and unit 0 (GPT applies block 0's ln1 before calling the block)

    def sync(self):
        """The caller's stream waits for every queued update and zeroing."""
        if self.final is not None:
            torch.cuda.current_stream(self.device).wait_event(self.final)
            self.final = None
            self.events = [None] * len(self.events)

    def run(self, opt, lr, scale_t, launch):
        """Queue the update: ``launch(plan)`` issues one phase's multi-tensor kernel."""
        main = torch.cuda.current_stream(self.device)
        s = self.stream
        s.wait_stream(main)
        if scale_t is not None:
            scale_t.record_stream(s)
        with torch.cuda.stream(s):
            for ph, idx in enumerate(self.phase_pieces):
                if not idx:
                    continue
                if self.plans[ph] is None:
                    self.plans[ph] = opt._build_plan(idx)
                launch(self.plans[ph])
                ev = torch.cuda.Event()
                ev.record(s)
                self.events[ph] = ev
        self.final = torch.cuda.Event()
        self.final.record(s)

    def zero_grads(self, st):
        """clear_grad after a queued update: zero on the side stream, behind the updates."""
        if self.final is None:
            return False
        s = self.stream
        with torch.cuda.stream(s):
            K.zero_tensors([g.grad_buf for g in st.groups if not g.grads_released])
        for g in st.groups:
            if not g.grads_released:
                g.reattach_grads()
        self.final = torch.cuda.Event()
        self.final.record(s)
        # the last phase's event now also covers the zeroing (the backward runs after it)
        self.events[-1] = self.final
        return True


class _ShardPiece:
    """Stand-in parameter for one owned shard piece, handed to an element-wise inner optimizer's
    ``_update`` (its accumulators are keyed by ``name``; ``_t`` is the fp32 target slice)."""

    def __init__(self, name, t, param):
        self.name = name
        self._t = t
        self.optimize_attr = getattr(param, 'optimize_attr', {'learning_rate': 1.0})
        self.stop_gradient = False
        self.param = param


class ShardedOptimizer:
    """Owned-shard optimizer driving the fused multi-tensor HIP kernel.

    Hyper-parameters (lr / scheduler, betas, eps, weight decay incl.
    apply_decay_param_fun, grad_clip) are taken from the user's optimizer.
    """

    def __init__(self, optimizer, state: ShardedState, offload=False, mp_group=None,
                 norm_groups=()):
        self._inner = optimizer
        self.state = state
        self._kind = type(optimizer).__name__
        # Adam / AdamW / Momentum / SGD run the multi-tensor HIP kernels over the flat shards;
        # every other optimizer (Lamb, Adagrad, Adadelta, Adamax, RMSProp: the reference wraps
        # any inner optimizer, dygraph_sharding_optimizer.py:29-212) runs its own per-element
        # update on this rank's shard pieces, with its accumulators kept as flat per-group
        # shards (so checkpoints gather / re-slice them like the moments); Lamb's trust ratio
        # needs whole-parameter norms: one all-reduce of the per-parameter partial sums
        from ..optimizer.optimizer import _ForeachOpt
        self._generic = self._kind not in ('Adam', 'AdamW', 'Momentum', 'SGD')
        if self._generic and not isinstance(optimizer, _ForeachOpt):
            raise NotImplementedError(f"sharding does not support {self._kind}")
        if self._generic and offload:
            raise NotImplementedError(f"sharding offload supports Adam/AdamW/Momentum/SGD, not {self._kind}")
        self._offload = bool(offload)
        self._mp_pg = None if mp_group is None or mp_group.nranks == 1 else mp_group.process_group
        self._norm_pgs = [g.process_group for g in norm_groups if g is not None and g.nranks > 1]
        self._pieces = []
        self._masters, self._m, self._v = [], [], []
        for gi, g in enumerate(state.groups):
            shard = g.param_shard
            sdev = torch.device('cpu') if self._offload else g.device
            master = shard.detach().float().clone().to(sdev) \
                if (shard.dtype != torch.float32 or self._offload) else None
            self._masters.append(master)
            self._m.append(torch.zeros(g.shard_numel, dtype=torch.float32, device=sdev)
                           if not self._generic else None)
            self._v.append(torch.zeros(g.shard_numel, dtype=torch.float32, device=sdev)
                           if self._kind in ('Adam', 'AdamW') else None)
            for (p, lo, hi, plo) in g.params_in_shard():
                self._pieces.append((gi, p, lo, hi, plo))
        self._gen_acc = {}
        self._shadows = []
        if self._generic:
            init = {'moment': getattr(optimizer, '_init_acc', 0.0)} if self._kind == 'Adagrad' else {}
            for name in type(optimizer)._acc_names:
                if name == 'mean_grad' and not getattr(optimizer, '_centered', False):
                    continue
                self._gen_acc[name] = [torch.full((g.shard_numel,), float(init.get(name, 0.0)),
                                                  dtype=torch.float32, device=g.device)
                                       for g in state.groups]
            for i, (gi, p, lo, hi, plo) in enumerate(self._pieces):
                sh = _ShardPiece(f'{p.name}@{gi}.{lo}', self._target(gi, lo, hi), p)
                for name, bufs in self._gen_acc.items():
                    optimizer._accumulators.setdefault(name, {})[sh.name] = bufs[gi][lo:hi]
                self._shadows.append(sh)
        self._plan = None
        self._step = 0
        state.on_params_loaded.append(self._refresh_masters)
        self._overlap = _StepOverlap.maybe(self)
        state.step_overlap = self._overlap

    def _target(self, gi, lo, hi):
        """The fp32 tensor the update writes for a piece: its master slice, else its shard."""
        m = self._masters[gi] if gi < len(self._masters) else None
        return m[lo:hi] if m is not None else self.state.groups[gi].param_shard[lo:hi]

    def _step_generic(self, lr, coef):
        """Per-piece update of any element-wise inner optimizer (its own ``_update``) on this
        rank's owned shard pieces; Lamb with whole-parameter trust ratios."""
        st, o = self.state, self._inner
        c = None if coef is None else coef.to(torch.float32)
        lamb = self._kind == 'Lamb'
        upds, wsq, usq = [], {}, {}
        for (gi, p, lo, hi, plo), sh in zip(self._pieces, self._shadows):
            grad = st.shard_grads[gi][lo:hi].float()
            if c is not None:
                grad = grad * c
            w = self._target(gi, lo, hi)
            lrp = lr * p.optimize_attr.get('learning_rate', 1.0)
            if lamb:
                m = o._accumulators['moment1'][sh.name]
                v = o._accumulators['moment2'][sh.name]
                m.mul_(o._beta1).add_((1 - o._beta1) * grad)
                v.mul_(o._beta2).add_((1 - o._beta2) * grad * grad)
                mh = m / (1 - o._beta1 ** self._step)
                vh = v / (1 - o._beta2 ** self._step)
                wd = 0.0 if (o._exclude is not None and o._exclude(p)) else o._wd
                r = mh / (vh.sqrt() + o._epsilon) + wd * w.float()
                key = id(p)
                wsq[key] = wsq.get(key, 0.0) + (w.float() * w.float()).sum()
                usq[key] = usq.get(key, 0.0) + (r * r).sum()
                upds.append((w, r, lrp, key))
            else:
                wd = self._wd(p)
                if wd:
                    grad = grad + wd * w.float()
                w.add_(o._update(sh, grad, w.float(), lrp).to(w.dtype))
        if lamb:
            # the pieces of one parameter may sit on several ranks: whole-parameter norms from
            # one all-reduce of [n_params, 2] partial sums (same parameter order on every rank)
            allp = [id(q) for g in st.groups for q in g.params]
            pos = {k: i for i, k in enumerate(allp)}
            dev = st.groups[0].device
            sums = torch.zeros(len(allp), 2, dtype=torch.float32, device=dev)
            for k in wsq:
                sums[pos[k], 0] += wsq[k]
                sums[pos[k], 1] += usq[k]
            if st.world > 1:
                dist.all_reduce(sums, group=st.pg)
            norms = {k: sums[pos[k]].sqrt() for k in wsq}
            for w, r, lrp, key in upds:
                wn, rn = norms[key][0], norms[key][1]
                trust = torch.where((wn > 0) & (rn > 0), wn / rn, torch.ones_like(wn))
                w.add_((-lrp * trust * r).to(w.dtype))
        with torch.no_grad():
            for gi, g in enumerate(st.groups):
                if self._masters[gi] is not None:
                    g.param_shard.copy_(self._masters[gi].to(g.param_shard.device, g.param_shard.dtype))

    def _acc_bufs(self, gi):
        """[(checkpoint accumulator name, flat shard buffer)] of group gi."""
        if self._generic:
            return [(n, bufs[gi]) for n, bufs in self._gen_acc.items()]
        k1, k2 = self._acc_keys()
        return [(k, b) for k, b in ((k1, self._m[gi]), (k2, self._v[gi])) if k is not None and b is not None]

    def _refresh_masters(self):
        with torch.no_grad():
            for gi, g in enumerate(self.state.groups):
                if self._masters[gi] is not None:
                    self._masters[gi].copy_(g.param_shard.float())

    # -- paddle optimizer surface ----------------------------------------------------------
    def get_lr(self):
        return self._inner.get_lr()

    def set_lr(self, v):
        self._inner.set_lr(v)

    @property
    def _learning_rate(self):
        return self._inner._learning_rate

    @property
    def _parameter_list(self):
        return self._inner._parameter_list

    def clear_grad(self, set_to_zero=True):
        ov = self._overlap
        if ov is not None and set_to_zero and ov.zero_grads(self.state):
            if self.state.reducer is not None:
                self.state.reducer.reset_accumulation()
            return
        if ov is not None:
            ov.sync()
        self.state.zero_grad()

    def _scaler_grads(self):
        return list(self.state.shard_grads)

    def _found_inf_groups(self):
        st = self.state
        return [pg for pg, n in ((st.pg, st.world), (st.dp_pg, st.dp_world)) if n > 1] + \
            ([self._mp_pg] if self._mp_pg is not None else []) + list(self._norm_pgs)

    clear_gradients = clear_grad

    def _wd(self, p):
        o = self._inner
        wd = o._weight_decay
        wd = float(wd) if wd is not None else 0.0
        fn = getattr(o, '_apply_decay_param_fun', None)
        if fn is not None and not fn(p.name):
            return 0.0
        return wd

    def _clip_local(self):
        """ClipGradByValue / ClipGradByNorm on the owned gradient shards (reference
        python/paddle/nn/clip.py semantics). By value is element-wise: each rank clamps its own
        pieces. By norm is per parameter: the squared norms of every parameter's pieces are
        summed in one vector all-reduce over the sharding group (a TP-split parameter keeps its
        mp-local norm, as the reference's per-tensor clip), then each piece is scaled by
        clip_norm / max(||g_p||, clip_norm). Returns True when it handled the clip."""
        from ..nn.clip import ClipGradByValue, ClipGradByNorm
        clip = self._inner._grad_clip
        st = self.state
        gs = st.shard_grads
        if isinstance(clip, ClipGradByValue):
            for gi, p, lo, hi, _ in self._pieces:
                if getattr(p, 'need_clip', True):
                    gs[gi][lo:hi].clamp_(clip.min, clip.max)
            return True
        if not isinstance(clip, ClipGradByNorm):
            return False
        params = [p for g in st.groups for p in g.params]  # same order on every rank
        index = {id(p): i for i, p in enumerate(params)}
        dev = gs[0].device if gs else torch.device('cpu')
        sq = torch.zeros(len(params), dtype=torch.float32, device=dev)
        for gi, p, lo, hi, _ in self._pieces:
            if hi > lo:
                sq[index[id(p)]] += gs[gi][lo:hi].float().square().sum()
        if st.world > 1:
            dist.all_reduce(sq, group=st.pg)
        # (no model-parallel reduction: the reference's ClipGradByNorm clips each LOCAL tensor by
        # its own norm -- HybridParallelClipGrad wraps only ClipGradByGlobalNorm -- so a
        # TP-split parameter is clipped by the norm of this mp rank's slice)
        scale = clip.clip_norm / torch.clamp(torch.sqrt(sq), min=clip.clip_norm)
        for gi, p, lo, hi, _ in self._pieces:
            if getattr(p, 'need_clip', True) and hi > lo:
                gs[gi][lo:hi].mul_(scale[index[id(p)]].to(gs[gi].dtype))
        return True

    def _clip_coef(self):
        from ..nn.clip import ClipGradByGlobalNorm
        clip = self._inner._grad_clip
        if clip is None:
            return None
        if self._clip_local():
            return None
        if not isinstance(clip, ClipGradByGlobalNorm):
            raise NotImplementedError("sharding supports ClipGradByGlobalNorm / ClipGradByNorm / ClipGradByValue")
        st = self.state
        dev = st.shard_grads[0].device if st.shard_grads else torch.device('cpu')

        def nsq(ts):
            return K.global_l2_norm_sq(ts).reshape(1).float() if ts else \
                torch.zeros(1, device=dev)
        # owned shards partition the gradients: local sum of squares + one all-reduce. A
        # pipeline-tied weight (is_firstly_shared False on all but its first owner stage) is
        # counted once, so its pieces are left out on the other stages.
        tied = [pc for pc in self._pieces if not getattr(pc[1], 'is_firstly_shared', True)]
        if self._mp_pg is None and tied:
            gs = st.shard_grads
            sq = nsq([gs[gi][lo:hi] for gi, p, lo, hi, _ in self._pieces
                      if getattr(p, 'is_firstly_shared', True)])
            if st.world > 1:
                dist.all_reduce(sq, group=st.pg)
        elif self._mp_pg is None:
            sq = nsq(st.shard_grads)
            if st.world > 1:
                dist.all_reduce(sq, group=st.pg)
        else:
            # TP-split parameters are summed over the mp group, replicated ones counted once
            gs = st.shard_grads
            d = [gs[gi][lo:hi] for gi, p, lo, hi, _ in self._pieces
                 if getattr(p, 'is_distributed', False) and getattr(p, 'is_firstly_shared', True)]
            r = [gs[gi][lo:hi] for gi, p, lo, hi, _ in self._pieces
                 if not getattr(p, 'is_distributed', False) and getattr(p, 'is_firstly_shared', True)]
            both = torch.cat([nsq(d), nsq(r)])
            if st.world > 1:
                dist.all_reduce(both, group=st.pg)
            sd = both[:1].contiguous()
            dist.all_reduce(sd, group=self._mp_pg)
            sq = sd + both[1:]
        for pg in self._norm_pgs:  # pipeline stages own disjoint parameters
            dist.all_reduce(sq, group=pg)
        sq = sq.reshape(())
        return clip.clip_norm / torch.clamp(torch.sqrt(sq), min=clip.clip_norm)

    @torch.no_grad()
    def step(self):
        st = self.state
        self._step += 1
        o = self._inner
        o._step_count = self._step
        ov = self._overlap
        if ov is not None:
            ov.sync()  # a second step before the next forward: the previous update comes first
        coef = self._clip_coef()
        lr = o.get_lr()
        dev = st.groups[0].device if st.groups else None
        coupled = self._kind == 'Adam' and o._weight_decay
        if self._generic:
            if ov is not None:
                ov.sync()
            self._step_generic(lr, coef)
            st.after_step()
            return
        if ov is not None:
            scale_t = None if coef is None else coef.to(torch.float32).reshape(()).contiguous()
            ov.run(self, lr, scale_t, lambda plan: self._launch(plan, lr, scale_t))
            st.after_step()
            return
        if self._offload:
            self._step_offload(lr, coef)
        elif dev is not None and dev.type == 'cuda' and _native.available() and not coupled:
            # the clip coefficient is read by the update kernel: no extra pass over the grads
            self._step_hip(lr, None if coef is None else
                           coef.to(torch.float32).reshape(()).contiguous())
        else:
            if coef is not None:
                for s in st.shard_grads:
                    s.mul_(coef.to(s.dtype))
            if dev is not None and dev.type == 'cuda' and _native.available():
                self._step_hip(lr)
            else:
                self._step_ref(lr)
        st.after_step()

    def _step_offload(self, lr, coef):
        """Host-resident master/moments (group_sharded offload=True): owned grads go to the
        host, the update runs there, the new low-precision shard is copied back."""
        st = self.state
        o = self._inner
        c = None if coef is None else float(coef)
        for gi, g in enumerate(st.groups):
            gh = st.shard_grads[gi].detach().to('cpu', torch.float32)
            if c is not None:
                gh.mul_(c)
            master = self._masters[gi]
            for gj, p, lo, hi, plo in self._pieces:
                if gj != gi:
                    continue
                lrm = p.optimize_attr.get('learning_rate', 1.0)
                if self._kind in ('Adam', 'AdamW'):
                    wd = self._wd(p)
                    grad = gh[lo:hi]
                    if self._kind == 'Adam' and wd:
                        grad = grad + wd * master[lo:hi]
                        wd = 0.0
                    K.adamw_ref([master[lo:hi]], [grad], [self._m[gi][lo:hi]], [self._v[gi][lo:hi]],
                                [None], lr, o._beta1, o._beta2, o._epsilon, [wd], [lrm], self._step)
                else:
                    K.momentum_ref([master[lo:hi]], [gh[lo:hi]], [self._m[gi][lo:hi]], [None],
                                   lr * lrm, getattr(o, '_momentum', 0.0), [self._wd(p)],
                                   getattr(o, '_use_nesterov', False))
            g.param_shard.copy_(master.to(g.dtype), non_blocking=False)

    def _piece_views(self, gi, lo, hi):
        g = self.state.groups[gi]
        shard = g.param_shard
        master = self._masters[gi]
        return (master[lo:hi] if master is not None else shard[lo:hi], self.state.shard_grads[gi][lo:hi],
                self._m[gi][lo:hi], None if self._v[gi] is None else self._v[gi][lo:hi],
                shard[lo:hi] if master is not None else None)

    def _step_ref(self, lr):
        o = self._inner
        for gi, p, lo, hi, plo in self._pieces:
            master, grad, m, v, lowp = self._piece_views(gi, lo, hi)
            lrm = p.optimize_attr.get('learning_rate', 1.0)
            if self._kind in ('Adam', 'AdamW'):
                wd = self._wd(p)
                if self._kind == 'Adam' and wd:
                    grad = grad.float() + wd * master.float()
                    wd = 0.0
                K.adamw_ref([master if lowp is None else lowp], [grad], [m], [v],
                            [None if lowp is None else master], lr, o._beta1, o._beta2, o._epsilon,
                            [wd], [lrm], self._step)
            else:
                mu = getattr(o, '_momentum', 0.0)
                K.momentum_ref([master if lowp is None else lowp], [grad], [m],
                               [None if lowp is None else master], lr * lrm, mu, [self._wd(p)],
                               getattr(o, '_use_nesterov', False))

    def _updated_shards(self):
        """The tensors the multi-tensor kernel writes (fp32 masters, else the param shards)."""
        return [m if m is not None else g.param_shard
                for m, g in zip(self._masters, self.state.groups)]

    def _build_plan(self, idx=None):
        """Multi-tensor descriptor tables for the pieces ``idx`` (default: all)."""
        cols = [[], [], [], [], [], [], [], []]
        wds, lrms = [], []
        for i in (range(len(self._pieces)) if idx is None else idx):
            gi, p, lo, hi, plo = self._pieces[i]
            master, grad, m, v, lowp = self._piece_views(gi, lo, hi)
            cols[0].append(master.data_ptr())
            cols[1].append(grad.data_ptr())
            cols[2].append(m.data_ptr())
            cols[3].append(0 if v is None else v.data_ptr())
            cols[4].append(0 if lowp is None else lowp.data_ptr())
            cols[5].append(hi - lo)
            cols[6].append(K._DT[grad.dtype])
            cols[7].append(K._DT[(lowp if lowp is not None else master).dtype])
            wd = self._wd(p)
            if self._kind == 'Adam':
                wd = 0.0  # coupled L2 handled in _step_hip (rare); AdamW decoupled in-kernel
            wds.append(wd)
            lrms.append(p.optimize_attr.get('learning_rate', 1.0))
        return K._mt_table(cols, cols[5], [wds, lrms], self.state.groups[0].device)

    def _launch(self, plan, lr, scale_t):
        o = self._inner
        tab, ftab, ch, nch = plan
        if self._kind in ('Adam', 'AdamW'):
            b1, b2 = o._beta1, o._beta2
            R.dispatch('adamw_mt', tab, tab, ftab, ch, nch, lr, b1, b2, o._epsilon,
                       1 - b1 ** self._step, 1 - b2 ** self._step, 1.0, scale_t,
                       self._updated_shards())
        else:
            R.dispatch('momentum_mt', tab, tab, ftab, ch, nch, lr, getattr(o, '_momentum', 0.0),
                       getattr(o, '_use_nesterov', False), 1.0, scale_t,
                       self._updated_shards())

    def _step_hip(self, lr, scale_t=None):
        o = self._inner
        if self._plan is None:
            self._plan = self._build_plan()
        if self._kind == 'Adam' and o._weight_decay:
            for gi, p, lo, hi, plo in self._pieces:
                w = self._wd(p)
                if w:
                    master, grad, m, v, lowp = self._piece_views(gi, lo, hi)
                    grad.add_(master.to(grad.dtype), alpha=w)
        self._launch(self._plan, lr, scale_t)

    def minimize(self, loss, *a, **k):
        loss.backward()
        self.step()

    # -- checkpoint ------------------------------------------------------------------------
    def _acc_keys(self):
        return ('moment1', 'moment2') if self._kind in ('Adam', 'AdamW') else ('velocity', None)

    def _gather_full(self, buf, g):
        """All-gather one group's owned shards into the full flat buffer (host copy)."""
        st = self.state
        if st.world == 1:
            return buf.detach().float().cpu()
        dev = g.device if (g.device.type == 'cuda' and dist.get_backend(st.pg) == 'nccl') \
            else torch.device('cpu')
        src = buf.detach().float().to(dev).contiguous()
        out = torch.empty(src.numel() * st.world, dtype=src.dtype, device=dev)
        _watchdog.track('sharding.ckpt_gather', dist.all_gather_into_tensor(
            out, src, group=st.pg, async_op=True), st.world).wait()
        return out.cpu()

    def state_dict(self, full=True):
        """Optimizer state in the reference's per-parameter layout (``{param}_moment1_0``,
        ``{param}_moment2_0`` / ``{param}_velocity_0``, ``{param}_beta{1,2}_pow_acc_0``,
        ``master_weights``, ``LR_Scheduler``), gathered from every rank's owned shard: a
        ``.pdopt`` written here resumes under ANY sharding degree (or none: the plain optimizer
        reads the same keys). ``full=False`` returns this rank's raw shards only."""
        st = self.state
        if self._overlap is not None:
            self._overlap.sync()
        sd = {}
        if not full:
            for gi in range(len(st.groups)):
                if self._generic:
                    for key, buf in self._acc_bufs(gi):
                        sd[f'shard{gi}_{key}'] = Tensor(buf)
                else:
                    sd[f'shard{gi}_moment1'] = Tensor(self._m[gi])
                if self._v[gi] is not None:
                    sd[f'shard{gi}_moment2'] = Tensor(self._v[gi])
                if self._masters[gi] is not None:
                    sd[f'shard{gi}_master'] = Tensor(self._masters[gi])
            sd['@rank'], sd['@world'] = st.rank, st.world
        else:
            masters = {}
            for gi, g in enumerate(st.groups):
                bufs = self._acc_bufs(gi) + [('master', self._masters[gi])]
                for key, buf in bufs:
                    if key is None or buf is None:
                        continue
                    flat = self._gather_full(buf, g)
                    for p, o, n, shp in zip(g.params, g.offsets, g.numels, g.shapes):
                        v = Tensor(flat[o:o + n].view(shp).clone())
                        if key == 'master':
                            masters[p.name] = v
                        else:
                            sd[f'{p.name}_{key}_0'] = v
                if self._kind in ('Adam', 'AdamW'):
                    o = self._inner
                    for p in g.params:
                        # reference convention: beta**(t+1) after t updates (adamw.py:343-348)
                        sd[f'{p.name}_beta1_pow_acc_0'] = Tensor(
                            torch.tensor([o._beta1 ** (self._step + 1)], dtype=torch.float32))
                        sd[f'{p.name}_beta2_pow_acc_0'] = Tensor(
                            torch.tensor([o._beta2 ** (self._step + 1)], dtype=torch.float32))
            if masters:
                sd['master_weights'] = masters
        sd['@step'] = self._step
        from ..optimizer.lr import LRScheduler
        if isinstance(self._inner._learning_rate, LRScheduler):
            sd['LR_Scheduler'] = self._inner._learning_rate.state_dict()
        return sd

    def set_state_dict(self, sd):
        st = self.state
        if self._overlap is not None:
            self._overlap.sync()
        knames = [k for k, _ in self._acc_bufs(0)] if st.groups else []
        per_param = any(isinstance(k, str) and any(k.endswith(f'_{n}_0') for n in knames) for k in sd)
        masters_sd = sd.get('master_weights', {})
        with torch.no_grad():
            for gi, g in enumerate(st.groups):
                if per_param:
                    # slice this rank's owned pieces out of the full per-parameter tensors
                    for p, lo, hi, plo in g.params_in_shard():
                        for key, buf in self._acc_bufs(gi):
                            name = f'{p.name}_{key}_0'
                            if key is None or buf is None or name not in sd:
                                continue
                            src = _u(sd[name]).reshape(-1)[plo:plo + (hi - lo)]
                            buf[lo:hi].copy_(src.to(device=buf.device, dtype=buf.dtype))
                        if self._masters[gi] is not None and p.name in masters_sd:
                            src = _u(masters_sd[p.name]).reshape(-1)[plo:plo + (hi - lo)]
                            self._masters[gi][lo:hi].copy_(src.to(self._masters[gi].device,
                                                                  torch.float32))
                else:
                    shard_bufs = [(f'shard{gi}_{k}', b) for k, b in self._acc_bufs(gi)] if self._generic else \
                        [(f'shard{gi}_moment1', self._m[gi]), (f'shard{gi}_moment2', self._v[gi])]
                    for key, buf in shard_bufs + [(f'shard{gi}_master', self._masters[gi])]:
                        if key in sd and buf is not None:
                            buf.copy_(_u(sd[key]).to(buf.device))
        step = sd.get('@step')
        if step is None and self._kind in ('Adam', 'AdamW'):
            b1 = [v for k, v in sd.items() if isinstance(k, str) and k.endswith('_beta1_pow_acc_0')]
            if b1:
                from ..optimizer.optimizer import beta_pow_to_step
                step = beta_pow_to_step(b1[0], self._inner._beta1)
        if step is not None:
            self._step = int(step)
        if 'LR_Scheduler' in sd:
            self._inner._learning_rate.set_state_dict(sd['LR_Scheduler'])
        # refresh the owned low-precision shard from the restored master
        for gi, g in enumerate(st.groups):
            if self._masters[gi] is not None:
                g.param_shard.copy_(self._masters[gi].to(g.param_shard.device))
        st.params_stale = True
        st.sync_params()
        if st.zero3:
            st.release_all()


class ShardedModel(Layer):
    """Model wrapper returned by group_sharded_parallel (GroupShardedStage2/3 parity)."""

    def __init__(self, layer, state: ShardedState):
        super().__init__()
        self._layer = layer
        self.__dict__['_state'] = state

    def forward(self, *inputs, **kwargs):
        self._state.before_forward()
        return self._layer(*inputs, **kwargs)

    def state_dict(self, *a, **k):
        st = self._state
        st.sync_params()
        sd = self._layer.state_dict(*a, **k)
        if st.zero3:
            # unit parameters are freed again after this call: hand out copies
            unit_ids = {id(p) for u in st.unit_meta for gi in u.gids for p in st.groups[gi].params}
            for key, v in list(sd.items()):
                if id(v) in unit_ids:
                    c = Parameter(v._t.detach().clone())
                    c.name = v.name
                    sd[key] = c
            st.release_all()
        return sd

    def set_state_dict(self, sd, use_structured_name=True):
        st = self._state
        st.sync_params()
        r = self._layer.set_state_dict(sd, use_structured_name)
        st.params_loaded()
        if st.zero3:
            st.release_all()
        return r

    set_dict = set_state_dict
    load_dict = set_state_dict

    def parameters(self, include_sublayers=True):
        return self._layer.parameters(include_sublayers)

    def named_parameters(self, prefix='', include_sublayers=True):
        return self._layer.named_parameters(prefix, include_sublayers)

    def get_all_parameters(self, convert2cpu=False):
        """Gather every parameter (stays gathered until the next forward/step releases it)."""
        self._state.sync_params()
        ps = self._layer.parameters()
        if convert2cpu:
            return [Parameter(p._t.detach().cpu()) for p in ps]
        return ps


def group_sharded_parallel(model, optimizer, level, scaler=None, group=None, offload=False,
                           sync_buffers=False, buffer_max_size=2 ** 23, segment_size=2 ** 20,
                           sync_comm=False, dp_group=None, exclude_layer=None,
                           bucket_mb=128, release_after_forward=True):
    """paddle.distributed.sharding.group_sharded_parallel (parity:
    python/paddle/distributed/sharding/group_sharded.py). ``offload=True`` keeps the fp32
    master weights and optimizer moments in host memory (the update runs on the CPU)."""
    if level not in LEVELS:
        raise ValueError(f"level must be one of {list(LEVELS)}")
    st = ShardedState(model, level, group, segment_bytes=bucket_mb << 20, dp_group=dp_group,
                      segment_size=segment_size, exclude_layer=exclude_layer,
                      release_after_forward=release_after_forward)
    # the (bucketed, flat) params were re-pointed in place: the inner optimizer's list stays valid
    sopt = ShardedOptimizer(optimizer, st, offload=offload)
    if scaler is not None:
        from ..amp import ShardedGradScaler
        scaler = ShardedGradScaler.wrap(scaler, st)
    return ShardedModel(model, st), sopt, scaler


def save_group_sharded_model(model, output, optimizer=None):
    """Save the FULL model (``model.pdparams``) and the FULL, per-parameter optimizer state
    (``model.pdopt``) from rank 0 (parity: distributed/sharding/group_sharded.py
    save_group_sharded_model); every rank takes part in the gathers. The files load into
    a sharded run of any degree or into a plain single-process optimizer."""
    import os
    from ..framework.io import save
    from ..distributed import collective as C
    os.makedirs(output, exist_ok=True)
    sd = model.state_dict()
    osd = optimizer.state_dict() if optimizer is not None else None
    if C.get_rank() == 0:
        save(sd, os.path.join(output, 'model.pdparams'))
        if osd is not None:
            save(osd, os.path.join(output, 'model.pdopt'))
