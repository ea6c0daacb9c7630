"""Static-graph pipeline parallelism: a program split by ``static.device_guard('gpu:k')`` into
stages, one stage per rank, micro-batched (parity: python/paddle/fluid/optimizer.py:4494
PipelineOptimizer -- ``_add_op_device_attr`` / section split by op_device, the send_v2 /
recv_v2 pairs between sections, gradient accumulation over ``accumulate_steps`` micro-batches
-- and distributed/fleet/meta_optimizers/pipeline_optimizer.py:198; fluid/device_worker.py
Section + framework/section_worker.cc for the F-then-B / 1F1B schedules).

MI355X design: one process per GPU, no per-section sub-programs. Every rank keeps the whole
program; minimize builds the full backward once and labels every op with its stage:

* forward ops: the stage of their ``device_guard`` ('gpu:k' -> k), else the latest stage among
  their inputs' producers (a loss head written after the last guard stays on the last stage);
* grad ops: the stage of their forward op; gradient ``sum`` ops: the stage that produced the
  summed variable (the gradient is needed where the activation came from); the seed: the
  loss's stage; each parameter's optimizer update: the stage that uses the parameter.

Every edge between stages becomes a point-to-point transfer (``torch.distributed`` send /
recv: RCCL over xGMI, gloo on CPU), forward activations from lower to higher stages in the
forward phase and their gradients back from higher to lower stages in the backward phase.
Receivers take their inputs in increasing (forward) / decreasing (backward) source-stage
order, which keeps the blocking transfers free of wait cycles for any DAG of stage edges, skip
connections included. A step splits the fed batch into ``n_micro`` micro-batches, runs the
schedule (F-then-B: every forward, then every backward; 1F1B: after ``stages - stage - 1``
warm-up forwards each forward is followed by one backward, bounding the live activations to the
pipeline depth), accumulates the parameter gradients (the backward seed is 1 / n_micro, so the
sum is the gradient of the mean loss), all-reduces them over the data-parallel group when there
is one, and steps this stage's optimizer. A global-norm clip sums the squared norms of every
stage (one all-reduce over the pipeline group). The fetched loss is the micro-batch mean from
the last stage, broadcast to every stage.

Not supported (raise): parameters shared by two stages, recompute checkpoints and fp16 loss
scaling together with the pipeline."""
import numpy as np
import torch
import torch.distributed as dist

from ..framework.core import Tensor, _u
from . import graph as G

__all__ = ['PipelineOptimizer', 'build_pipeline']

_DT = [torch.float32, torch.float16, torch.bfloat16, torch.float64, torch.int64, torch.int32, torch.bool,
       torch.uint8, torch.int8]
_HDR = 10


def _stage_of_device(dev):
    k = G._device_index(dev)
    if k is None or k[0] not in ('gpu', 'cuda', 'npu', 'xpu'):
        return None
    return int(k[1]) if k[1] not in (None, '') else 0


class _Pipeline:
    def __init__(self, prog, loss, opt, n_micro, schedule, stage, n_stages, pp_group, pp_ranks, dp_group):
        self.prog, self.loss, self.opt = prog, loss, opt
        self.n_micro, self.schedule = int(n_micro), schedule
        self.stage, self.n_stages = stage, n_stages
        self.pp_group, self.pp_ranks, self.dp_group = pp_group, pp_ranks, dp_group
        self._shapes = {}   # feed signature -> received (shape, dtype) per direction
        blk = prog.global_block()
        fwd = [op for op in blk.ops if op.role == 'forward']
        # -- forward stages --------------------------------------------------------------------
        producer, st = {}, {}
        for op in fwd:
            s = _stage_of_device(op.attrs.get('device'))
            if s is None:
                ins = [st[id(producer[v])] for v in op.in_vids if v in producer and id(producer[v]) in st]
                s = max(ins) if ins else None
            if s is not None:
                st[id(op)] = s
            for v in op.out_vids:
                producer[v] = op
        for op in reversed(fwd):      # input-less unguarded ops: their first consumer's stage
            if id(op) not in st:
                cons = [st[id(c)] for c in fwd if id(c) in st and any(v in c.in_vids for v in op.out_vids)]
                st[id(op)] = min(cons) if cons else 0
        for op in fwd:
            for v in op.in_vids:
                if v in producer and st[id(producer[v])] > st[id(op)]:
                    raise ValueError(f"pipeline: op {op.type} on stage {st[id(op)]} reads a variable "
                                     f"produced on the later stage {st[id(producer[v])]}")
        n_used = max(st.values()) + 1 if st else 1
        if n_used != n_stages:
            raise ValueError(f"pipeline: the program uses {n_used} stages (device_guard gpu:0..gpu:"
                             f"{n_used - 1}) but the pipeline group has {n_stages} ranks")
        self.loss_stage = st[id(producer[loss.vid])]
        # -- parameters ------------------------------------------------------------------------
        pstage = {}
        for op in fwd:
            for p in op.attrs.get('params', []):
                if p.stop_gradient:
                    continue
                if pstage.get(p.name, st[id(op)]) != st[id(op)]:
                    raise NotImplementedError(
                        f"pipeline: parameter {p.name} is used on stages {pstage[p.name]} and "
                        f"{st[id(op)]}; parameters shared across pipeline stages are not supported")
                pstage[p.name] = st[id(op)]
        self.fwd_stage = st
        self.producer = producer
        self.pstage = pstage

    # -- backward ----------------------------------------------------------------------------------
    def build_backward(self, parameters=None, checkpoints=None):
        """checkpoints (RecomputeOptimizer / strategy.recompute): the recompute segments' clones
        run on their forward ops' stages; a segment's intermediates are dropped from the micro-
        batch's state after its forward (only what the stage's backward reads stays)."""
        prog, blk = self.prog, self.prog.global_block()
        before = {id(op) for op in blk.ops}
        pg = G.append_backward(self.loss, parameters, loss_scale=1.0 / self.n_micro, checkpoints=checkpoints)
        st = dict(self.fwd_stage)
        # forward ops the backward builder inserted (each recompute segment's RNG snapshot, placed
        # right before the segment's first op): the stage of the next forward op
        ops = blk.ops
        for k in range(len(ops) - 1, -1, -1):
            op = ops[k]
            if op.role == 'forward' and id(op) not in st:
                nxt = next((st[id(o)] for o in ops[k + 1:] if o.role == 'forward' and id(o) in st), 0)
                st[id(op)] = nxt
        grad_of = {}   # grad-op output vid -> ('v', forward vid) | ('p', param name)
        bwd = [op for op in blk.ops if id(op) not in before and op.role != 'forward']
        producer_any = {}
        for op in blk.ops:
            for v in op.out_vids:
                producer_any[v] = op
        for op in bwd:
            if op.role == 'recompute':
                st[id(op)] = st[id(op.attrs['recompute_of'])]
                continue
            if op.type in ('recompute_rng_swap', 'recompute_rng_restore'):
                # swap: its RNG-snapshot input's stage (the segment's); restore: the swap's
                st[id(op)] = st[id(producer_any[op.in_vids[0]])]
                continue
            f = op.attrs.get('fwd')
            if f is not None:
                st[id(op)] = st[id(f)]
                din = f.attrs.get('diff_in', [])
                dps = f.attrs.get('diff_params', [])
                keys = [('v', v) for v in din] + [('p', p.name) for p in dps]
                for vid, key in zip(op.out_vids, keys):
                    grad_of[vid] = key
            elif op.type == 'fill_grad_seed':
                st[id(op)] = self.loss_stage
                grad_of[op.out_vids[0]] = ('v', self.loss.vid)
            elif op.type == 'sum':
                key = next((grad_of[v] for v in op.in_vids if v in grad_of), None)
                if key is None:
                    raise NotImplementedError("pipeline: cannot place a gradient sum")
                grad_of[op.out_vids[0]] = key
                st[id(op)] = self.pstage[key[1]] if key[0] == 'p' else \
                    self.fwd_stage[id(self.producer[key[1]])] if key[1] in self.producer else 0
            else:
                raise NotImplementedError(f"pipeline: unexpected backward op {op.type}")
        self.st = st
        me = self.stage
        self.fwd_ops = [op for op in blk.ops if op.role == 'forward' and st[id(op)] == me]
        self.bwd_ops = [op for op in bwd if st[id(op)] == me]
        # -- transfers ----------------------------------------------------------------------------
        prod_all = {}
        for op in blk.ops:
            for v in op.all_outputs():
                prod_all[v] = op
        fsend, frecv, bsend, brecv = set(), set(), set(), set()
        for op in blk.ops:
            if id(op) not in st:
                continue
            t = st[id(op)]
            for v in op.in_vids:
                p = prod_all.get(v)
                if p is None or id(p) not in st or st[id(p)] == t:
                    continue
                s = st[id(p)]
                if op.role == 'forward' and p.role == 'forward':
                    edge = (s, t, v)
                    if s == me:
                        fsend.add(edge)
                    if t == me:
                        frecv.add(edge)
                elif op.role == 'recompute' and p.role == 'forward':
                    continue   # a segment input from another stage: received in the forward, kept
                elif op.role in ('backward', 'recompute') and p.role in ('backward', 'recompute') and s > t:
                    edge = (s, t, v)
                    if s == me:
                        bsend.add(edge)
                    if t == me:
                        brecv.add(edge)
                else:
                    raise NotImplementedError(
                        f"pipeline: {op.role} op {op.type} on stage {t} reads a {p.role} value of stage {s}")
        self.fsend = sorted(fsend, key=lambda e: (e[1], e[2]))
        self.frecv = sorted(frecv, key=lambda e: (e[0], e[2]))
        self.bsend = sorted(bsend, key=lambda e: (-e[1], e[2]))
        self.brecv = sorted(brecv, key=lambda e: (-e[0], e[2]))
        # -- this stage's parameters and their gradient variables ----------------------------------
        self.params = [p for p, _ in pg if self.pstage.get(p.name) == me]
        self.grad_vid = {p.name: g.vid for p, g in pg}
        self.ctx_needed = {id(op) for op in self.fwd_ops if op.ctx_vid is not None and
                           any(op.ctx_vid in b.in_vids for b in self.bwd_ops)}
        # recompute clones whose autograd contexts the segment's grad ops read
        self.bctx_needed = {id(op) for op in self.bwd_ops if op.role == 'recompute' and op.ctx_vid is not None
                            and any(op.ctx_vid in b.in_vids for b in self.bwd_ops)}
        # a recomputed segment's forward outputs no later op of this stage reads: dropped per micro-batch
        seg = {id(op.attrs['recompute_of']) for op in self.bwd_ops if op.role == 'recompute'}
        keep = {v for op in self.bwd_ops for v in op.in_vids} | {v for _, _, v in self.fsend} | {self.loss.vid}
        self.drop_after_fwd = [v for op in self.fwd_ops if id(op) in seg for v in op.out_vids if v not in keep]
        data = {v.vid: v for v in blk.vars.values() if v.__dict__.get('is_data')}
        used = {v for op in self.fwd_ops + self.bwd_ops for v in op.in_vids}
        self.feeds = {data[v].name: v for v in used if v in data}
        opt = self.opt
        opt._param_groups = []
        opt._add_param_group({'params': list(self.params)})
        return pg

    # -- transport ---------------------------------------------------------------------------------------
    def _peer(self, stage):
        return self.pp_ranks[stage]

    def _exchange(self, sends, recvs, dev, shapes=None):
        """One point-to-point round: ``sends`` [(tensor, dst stage)], ``recvs`` [src stage] ->
        (received tensors, their (shape, dtype)). With ``shapes`` known (cached from an earlier
        step) it is ONE grouped batch_isend_irecv (an RCCL group on the GPU), so a stage's send
        of a forward output and its receive of a backward gradient progress together (the 1F1B
        steady state). Without, a header round carries the shapes first; that two-round form is
        only used under the F-then-B order, whose transfers all point one way per phase."""
        if not sends and not recvs:
            return [], []
        grp = self.pp_group
        outs = [_u(t).detach().contiguous() for t, _ in sends]
        if shapes is None:
            hin = [torch.zeros(_HDR, dtype=torch.int64, device=dev) for _ in recvs]
            ops = []
            for t, (_, dst) in zip(outs, sends):
                h = torch.zeros(_HDR, dtype=torch.int64)
                h[0], h[1] = t.dim(), _DT.index(t.dtype)
                h[2:2 + t.dim()] = torch.tensor(list(t.shape), dtype=torch.int64)
                ops.append(dist.P2POp(dist.isend, h.to(dev), self._peer(dst), grp))
            for h, src in zip(hin, recvs):
                ops.append(dist.P2POp(dist.irecv, h, self._peer(src), grp))
            for w in dist.batch_isend_irecv(ops):
                w.wait()
            shapes = []
            for h in hin:
                hv = h.tolist()
                shapes.append((tuple(hv[2:2 + hv[0]]), _DT[hv[1]]))
        bufs = [torch.empty(shp, dtype=dt, device=dev) for shp, dt in shapes]
        ops = [dist.P2POp(dist.isend, t, self._peer(dst), grp) for t, (_, dst) in zip(outs, sends)]
        ops += [dist.P2POp(dist.irecv, b_, self._peer(src), grp) for b_, src in zip(bufs, recvs)]
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        return bufs, shapes

    # -- one micro-batch (transfers are done by the schedule around these) ------------------------------
    def _fwd_sends(self, env):
        return [(env[v], t) for _, t, v in self.fsend]

    def _bwd_sends(self, env):
        return [(env[v], t) for _, t, v in self.bsend]

    def _put(self, env, edges, tensors):
        for (_, _, v), t in zip(edges, tensors):
            env[v] = Tensor(t)

    def _forward(self, exe, env):
        for op in self.fwd_ops:
            self._apply(exe, op, env, id(op) in self.ctx_needed)

    def _backward(self, exe, env, acc):
        for op in self.bwd_ops:
            self._apply(exe, op, env, id(op) in self.bctx_needed)
        for p in self.params:
            g = env.get(self.grad_vid[p.name])
            if g is None:
                continue
            g = _u(g)
            if p.name in acc:
                acc[p.name].add_(g.to(acc[p.name].dtype))
            else:
                acc[p.name] = g.to(torch.float32 if g.dtype in (torch.float16, torch.bfloat16) else g.dtype).clone()

    @staticmethod
    def _apply(exe, op, env, ctx_needed):
        res = exe._run_op(op, env, ctx_needed, True)
        if op.out_vids:
            flat, _ = G._flatten_out(res)
            for vid, t in zip(op.out_vids, flat):
                env[vid] = t

    # -- a training step -------------------------------------------------------------------------------
    def run(self, exe, feed, fetch_list, return_numpy=True):
        blk = self.prog.global_block()
        M = self.n_micro
        dev = G._default_device()
        chunks = {}
        for name, vid in self.feeds.items():
            if name not in feed:
                raise ValueError(f"pipeline: feed {name!r} missing")
            a = feed[name]
            t = a._t if isinstance(a, Tensor) else torch.as_tensor(np.asarray(a))
            if t.shape[0] % M:
                raise ValueError(f"pipeline: the batch of {name!r} ({t.shape[0]}) is not divisible by "
                                 f"{M} micro-batches")
            var = blk.vars[vid]
            chunks[vid] = [G._as_tensor_feed(Tensor(c), var) for c in torch.chunk(t, M, 0)]
        loss_vals = []
        fetch_vars = [blk.var(f) if isinstance(f, str) else f for f in fetch_list]
        fetched = {id(f): [] for f in fetch_vars}
        envs = {}
        acc = {}
        prev = G._STATIC[0]
        G._STATIC[0] = False

        fsrc = [e[0] for e in self.frecv]
        bsrc = [e[0] for e in self.brecv]

        def new_env(i):
            return {vid: chunks[vid][i] for vid in chunks}

        def fwd(i, env):
            self._forward(exe, env)
            if self.stage == self.loss_stage:
                loss_vals.append(_u(env[self.loss.vid]).detach().float().reshape(()))
            for f in fetch_vars:
                if f.vid in env and f.vid != self.loss.vid:
                    fetched[id(f)].append(_u(env[f.vid]).detach())
            for v in self.drop_after_fwd:   # recomputed segments' intermediates
                env.pop(v, None)
            envs[i] = env
        sig = tuple((vid, tuple(chunks[vid][0]._t.shape), str(chunks[vid][0]._t.dtype)) for vid in sorted(chunks))
        known = self._shapes.get(sig)
        fsh = known['f'] if known else None
        bsh = known['b'] if known else None
        seen = {'f': None, 'b': None}

        disc = known is None   # this step discovers the transfer shapes (header rounds)

        def xf(sends, srcs, which, sh):
            # a transfer round; records the received shapes of this direction (first step)
            bufs, shp = self._exchange(sends, srcs, dev, None if disc else (sh if srcs else []))
            if srcs:
                seen[which] = shp
            return bufs
        try:
            if self.schedule == '1F1B' and known is not None:
                # warm-up forwards, then one forward + one backward per step (the forward output
                # leaves in the same grouped round that brings the backward gradient in), then the
                # cool-down backwards (reference section_worker.cc 1F1B). Needs the transfer
                # shapes: the first step of a new feed shape runs F-then-B and records them.
                warm = min(self.n_stages - self.stage - 1, M)
                for i in range(warm):
                    env = new_env(i)
                    self._put(env, self.frecv, xf([], fsrc, 'f', fsh))
                    fwd(i, env)
                    xf(self._fwd_sends(env), [], 'f', [])
                nxt = None
                if M - warm > 0:
                    nxt = new_env(warm)
                    self._put(nxt, self.frecv, xf([], fsrc, 'f', fsh))
                for k in range(M - warm):
                    i, j = warm + k, k
                    env = nxt
                    fwd(i, env)
                    self._put(envs[j], self.brecv, xf(self._fwd_sends(env), bsrc, 'b', bsh))
                    benv = envs.pop(j)
                    self._backward(exe, benv, acc)
                    if k + 1 < M - warm:
                        nxt = new_env(i + 1)
                        self._put(nxt, self.frecv, xf(self._bwd_sends(benv), fsrc, 'f', fsh))
                    else:
                        xf(self._bwd_sends(benv), [], 'b', [])
                    del benv
                for j in range(M - warm, M):
                    benv = envs.pop(j)
                    self._put(benv, self.brecv, xf([], bsrc, 'b', bsh))
                    self._backward(exe, benv, acc)
                    xf(self._bwd_sends(benv), [], 'b', [])
                    del benv
            else:
                for i in range(M):
                    env = new_env(i)
                    self._put(env, self.frecv, xf([], fsrc, 'f', fsh))
                    fwd(i, env)
                    xf(self._fwd_sends(env), [], 'f', [])
                for j in range(M):
                    benv = envs.pop(j)
                    self._put(benv, self.brecv, xf([], bsrc, 'b', bsh))
                    self._backward(exe, benv, acc)
                    xf(self._bwd_sends(benv), [], 'b', [])
                    del benv
                if known is None:
                    self._shapes[sig] = {'f': seen['f'] or [], 'b': seen['b'] or []}
            self._merge_or_step(acc, dev)
        finally:
            G._STATIC[0] = prev
        # the loss: micro-batch mean on the last stage, broadcast over the pipeline
        lt = torch.stack(loss_vals).mean() if loss_vals else torch.zeros((), device=dev)
        lt = lt.to(dev)
        if self.n_stages > 1:
            dist.broadcast(lt, self._peer(self.loss_stage), group=self.pp_group)
        outs = []
        for f in fetch_vars:
            if f.vid == self.loss.vid:
                outs.append(Tensor(lt))
            elif fetched[id(f)]:
                parts = fetched[id(f)]
                outs.append(Tensor(torch.cat(parts, 0) if parts[0].dim() else torch.stack(parts).mean()))
            else:
                outs.append(None)
        return [(o.numpy() if return_numpy else o) if o is not None else None for o in outs]

    def _merge_or_step(self, acc, dev):
        """Gradient merge (strategy.gradient_merge over the pipeline): the micro-batch-accumulated
        gradients of gm_k consecutive runs are summed (averaged with gm_avg) and the optimizer
        steps on the k-th run only (reference gradient_merge_optimizer.py / pipeline: the merge
        window spans whole pipeline runs)."""
        k = getattr(self, 'gm_k', 1)
        if k <= 1:
            self._step(acc, dev)
            return
        gm = self.__dict__.setdefault('_gm', {})
        for name, g in acc.items():
            if name in gm:
                gm[name].add_(g)
            else:
                gm[name] = g
        self._gm_n = getattr(self, '_gm_n', 0) + 1
        if self._gm_n < k:
            return
        if getattr(self, 'gm_avg', True):
            for g in gm.values():
                g.div_(k)
        self._gm, self._gm_n = {}, 0
        self._step(gm, dev)

    def _step(self, acc, dev):
        from ..nn.clip import ClipGradByGlobalNorm
        ps = [p for p in self.params if p.name in acc]
        grads = [acc[p.name] for p in ps]
        local = getattr(self, 'localsgd', None)
        if local is None and self.dp_group is not None and dist.get_world_size(self.dp_group) > 1:
            n = dist.get_world_size(self.dp_group)
            for g in grads:
                dist.all_reduce(g, group=self.dp_group)
                g.div_(n)
        opt = self.opt
        clip = getattr(opt, '_grad_clip', None)
        prev = None
        is_gn = isinstance(clip, ClipGradByGlobalNorm)
        plan = getattr(self, 'shard_plan', None)
        hook = is_gn and (self.n_stages > 1 or plan is not None)
        if hook:
            # every stage joins the one all-reduce of the squared norms (a stage without
            # gradients contributes zero), the clip then uses the pipeline-wide norm
            from ..ops.fused import global_l2_norm_sq
            gs = [g for p, g in zip(ps, grads) if getattr(p, 'need_clip', True)]
            sq = global_l2_norm_sq(gs) if gs else None
            tot = sq.reshape(()).float().clone() if sq is not None else torch.zeros((), device=dev)
            if self.n_stages > 1:
                dist.all_reduce(tot, group=self.pp_group)
            prev = clip._norm_hook
            clip._norm_hook = lambda _sq: tot
        try:
            if plan is not None:
                # sharding stage 1 over the stage's data-parallel replicas: each steps the
                # parameters it owns (the norm above covered every gradient), then the owners
                # broadcast them
                own = {p.name for p in plan.owned(ps)}
                sel = [(p, g) for p, g in zip(ps, grads) if p.name in own]
                if sel:
                    G._optimize_fn(opt, [p for p, _ in sel], *[Tensor(g) for _, g in sel])
                plan.broadcast(self.params)
            elif ps:
                G._optimize_fn(opt, ps, *[Tensor(g) for g in grads])
        finally:
            if hook:
                clip._norm_hook = prev
        if local is not None and self.dp_group is not None and dist.get_world_size(self.dp_group) > 1:
            # localsgd over the stage's data-parallel replicas (no gradient all-reduce): parameters
            # averaged after every step through begin_step, then k_steps after the last averaging
            # (reference localsgd_optimizer.py:206)
            k, begin = local
            self._ls_steps = getattr(self, '_ls_steps', 0) + 1
            last = getattr(self, '_ls_last', 0)
            if self._ls_steps <= begin or self._ls_steps - last >= k:
                n = dist.get_world_size(self.dp_group)
                ts = [_u(p) for p in self.params]
                flat = torch.cat([t.detach().reshape(-1) for t in ts])
                dist.all_reduce(flat, group=self.dp_group)
                flat.div_(n)
                off = 0
                with torch.no_grad():
                    for t in ts:
                        t.copy_(flat[off:off + t.numel()].view(t.shape))
                        off += t.numel()
                self._ls_last = self._ls_steps


def build_pipeline(opt, loss, n_micro=1, schedule='1F1B', parameters=None, pp_group=None, dp_group=None,
                   checkpoints=None, gradient_merge=None, shard=False, localsgd=None):
    """Turn ``loss``'s program into this rank's pipeline stage (see the module docstring).
    checkpoints / a RecomputeOptimizer ``opt``: recompute segments inside the stages."""
    prog = loss.block.program
    if isinstance(opt, G.RecomputeOptimizer):
        checkpoints = opt._resolve(prog)
        opt = opt._optimizer
    if checkpoints:
        blk = prog.global_block()
        checkpoints = [blk.var(c) if isinstance(c, str) else c for c in checkpoints]
    from .amp import OptimizerWithMixedPrecision
    if isinstance(opt, OptimizerWithMixedPrecision):
        if opt._use_scaling:
            raise NotImplementedError("pipeline with fp16 loss scaling is not supported (use bfloat16)")
        opt._tag_program(prog)
        opt = opt._optimizer
    if schedule not in ('1F1B', 'F-then-B', 'FThenB'):
        raise ValueError(f"pipeline schedule_mode must be '1F1B' or 'F-then-B', got {schedule!r}")
    if not dist.is_initialized():
        raise RuntimeError("the static pipeline needs torch.distributed (one rank per stage): "
                           "call paddle.distributed.init_parallel_env() / fleet.init()")
    if pp_group is None:
        pp_ranks = list(range(dist.get_world_size()))
        pg = None
    else:
        pp_ranks = list(pp_group.ranks)
        pg = pp_group.process_group
    stage = pp_ranks.index(dist.get_rank())
    pipe = _Pipeline(prog, loss, opt, n_micro, '1F1B' if schedule == '1F1B' else 'FThenB', stage,
                     len(pp_ranks), pg, pp_ranks, dp_group.process_group if dp_group is not None else None)
    pg_list = pipe.build_backward(parameters, checkpoints)
    if gradient_merge is not None:
        pipe.gm_k, pipe.gm_avg = int(gradient_merge[0]), bool(gradient_merge[1])
    if localsgd is not None:
        pipe.localsgd = (max(1, int(localsgd[0])), max(1, int(localsgd[1])))
    if shard and dp_group is not None and dp_group.nranks > 1:
        # sharding stage 1 inside each stage, over its data-parallel replicas
        from ..distributed.fleet.meta_optimizers import _ShardPlan
        pipe.shard_plan = _ShardPlan(pipe.params, dp_group)
    prog.__dict__['_pipeline'] = pipe
    prog.__dict__['_no_graph'] = True
    prog._bump()
    return None, pg_list


class PipelineOptimizer:
    """paddle.static / fluid PipelineOptimizer(optimizer, num_microbatches): minimize splits the
    program by device_guard into one stage per rank of the world (see the module docstring)."""

    def __init__(self, optimizer, num_microbatches=1, start_cpu_core_id=0, schedule_mode='1F1B'):
        from . import _static_mode_enabled
        if not _static_mode_enabled():
            raise Exception("In dygraph, don't support PipelineOptimizer.")
        if int(num_microbatches) < 1:
            raise ValueError("num_microbatches must be >= 1")
        self._optimizer = optimizer
        self._num_microbatches = int(num_microbatches)
        self._schedule = schedule_mode

    def minimize(self, loss, startup_program=None, parameter_list=None, no_grad_set=None):
        return build_pipeline(self._optimizer, loss, self._num_microbatches, self._schedule, parameter_list)

    def __getattr__(self, k):
        return getattr(self.__dict__['_optimizer'], k)
