"""auto_parallel.Engine (parity: reference python/paddle/distributed/auto_parallel/engine.py:
Engine(model, loss, optimizer, metrics, cluster, strategy) with fit/evaluate/predict/save/load).

Static mode (``paddle.enable_static()`` before the model is built, so ``shard_tensor`` only
annotates; reference engine.py:513 _build, :670 _plan, :698 _parallel, :1272 prepare):
``prepare(inputs_spec, labels_spec)`` records the serial program from the model and
loss, completes and partitions it for this rank (static_passes.parallelize: local parameter
shards, reshard, the implied all-reduces -- the reference's static flow), binds the optimizer to
the local parameters and appends backward + update; fit / evaluate then feed every rank the
whole batch and the program slices what each rank owns.

Eager MI355X design: no program completion/partitioning. Batches are split over mesh axis 0
(DistributedBatchSampler with that axis' size/coordinate); after backward every gradient is
all-reduced (mean) over the mesh axes its parameter is replicated on and data is split over —
one flat bucket per step so RCCL sees a single large collective; sharded (tensor-parallel)
parameters keep their shard-local gradient on the other axes. Strategy sections honoured:
amp (bf16/fp16 auto_cast + GradScaler for fp16), recompute (whole-model recompute),
gradient_merge (k_steps accumulation), seed.
"""
import numpy as np
import torch

from ...framework.core import Tensor, _u
from .. import collective as C
from . import ProcessMesh, dist_attr, _fetches, _world_mesh
from .strategy import Strategy


def _to_list(x):
    if x is None:
        return []
    return list(x) if isinstance(x, (list, tuple)) else [x]


class Engine:
    def __init__(self, model=None, loss=None, optimizer=None, metrics=None, cluster=None, strategy=None):
        self._model, self._loss, self._optimizer = model, loss, optimizer
        self._metrics = _to_list(metrics)
        self._strategy = strategy if strategy is not None else Strategy()
        self._mesh = None
        self._scaler = None
        self.history = None
        self._merge_count = 0
        if self._strategy.seed is not None:
            from ... import seed as _seed
            _seed(self._strategy.seed)

    # ------------------------------------------------------------------ placement
    def _resolve_mesh(self):
        if self._mesh is not None:
            return self._mesh
        for p in self._model.parameters():
            a = dist_attr(p)
            if a is not None:
                self._mesh = a.process_mesh
                break
        if self._mesh is None:
            self._mesh = _world_mesh()
        return self._mesh

    def _dp(self):
        """(group, size, coordinate) of mesh axis 0, the data-parallel axis."""
        mesh = self._resolve_mesh()
        coord = mesh.coord()
        if coord is None or C.get_world_size() == 1:
            return None, 1, 0
        return mesh.axis_group(0), mesh.shape[0], coord[0]

    def _sync_grads(self):
        group, n, _ = self._dp()
        if n == 1:
            return
        grads = []
        for p in self._model.parameters():
            g = p._t.grad
            if g is None:
                continue
            a = dist_attr(p)
            if a is not None and a.process_mesh == self._mesh and 0 in a.dims_mapping:
                continue  # sharded over the batch axis: its gradient is already shard-local
            grads.append(g)
        if not grads:
            return
        flat = torch.cat([g.reshape(-1).float() for g in grads])
        torch.distributed.all_reduce(flat, group=group.process_group)
        flat /= n
        off = 0
        for g in grads:
            k = g.numel()
            g.copy_(flat[off:off + k].view_as(g).to(g.dtype))
            off += k

    # ------------------------------------------------------------------ data
    def _loader(self, data, batch_size, shuffle, collate_fn, drop_last=False):
        from ...io import DataLoader, DistributedBatchSampler, Dataset
        if data is None:
            return None
        if not isinstance(data, Dataset) and hasattr(data, '__iter__') and not hasattr(data, '__getitem__'):
            return data
        _, n, r = self._dp()
        if not self._strategy.split_data:
            n, r = 1, 0
        bs = DistributedBatchSampler(data, batch_size, num_replicas=n, rank=r, shuffle=shuffle,
                                     drop_last=drop_last)
        return DataLoader(data, batch_sampler=bs, collate_fn=collate_fn)

    @staticmethod
    def _split(batch, sample_split):
        batch = _to_list(batch)
        if sample_split is None:
            sample_split = len(batch) - 1 if len(batch) > 1 else len(batch)
        return batch[:sample_split], batch[sample_split:]

    # ------------------------------------------------------------------ steps
    def _forward(self, inputs):
        amp = self._strategy.amp
        fwd = self._model
        if self._strategy.recompute.enable:
            from . import recompute
            fwd = recompute(self._model)
        if amp.enable:
            from ...amp import auto_cast
            with auto_cast(True, level=amp.level.upper(), dtype=amp.dtype):
                return fwd(*inputs)
        return fwd(*inputs)

    def _compute_loss(self, outs, labels):
        if self._loss is None:
            return outs[0] if isinstance(outs, (list, tuple)) else outs
        return self._loss(*(_to_list(outs) + labels))

    def _update_metrics(self, outs, labels):
        res = {}
        for m in self._metrics:
            r = m.compute(*(_to_list(outs) + labels))
            m.update(*[x.numpy() if isinstance(x, Tensor) else x for x in _to_list(r)])
            acc = m.accumulate()
            names = _to_list(m.name())
            for nme, v in zip(names, _to_list(acc)):
                res[nme] = v
        return res

    def _train_step(self, inputs, labels):
        gm = self._strategy.gradient_merge
        k = gm.k_steps if gm.enable else 1
        outs = self._forward(inputs)
        loss = self._compute_loss(outs, labels)
        scaled = loss / k if (k > 1 and gm.avg) else loss
        if self._strategy.amp.enable and self._strategy.amp.dtype == 'float16':
            if self._scaler is None:
                from ...amp import GradScaler
                self._scaler = GradScaler(init_loss_scaling=self._strategy.amp.init_loss_scaling)
            self._scaler.scale(scaled).backward()
        else:
            scaled.backward()
        self._merge_count += 1
        if self._merge_count % k == 0:
            self._sync_grads()
            if self._scaler is not None:
                self._scaler.step(self._optimizer)
                self._scaler.update()
            else:
                self._optimizer.step()
            self._optimizer.clear_grad()
        return loss, outs

    def _fetch_logs(self):
        out = {}
        for name, (t, _) in _fetches.items():
            out[name] = t.numpy() if isinstance(t, Tensor) else t
        return out

    # ------------------------------------------------------------------ static programs
    @staticmethod
    def _static_on():
        from ...static import _STATIC
        return _STATIC[0]

    def _build_static(self, inputs_spec, labels_spec):
        """Serial program from the model + loss, completed and partitioned for this rank."""
        from ... import static
        from .static_passes import parallelize
        assert inputs_spec, "a static Engine needs inputs_spec (paddle.static.InputSpec list)"
        st = self._strategy
        serial = static.Program()
        with static.program_guard(serial):
            ins = [static.data(sp.name or f'input{i}', list(sp.shape), sp.dtype)
                   for i, sp in enumerate(_to_list(inputs_spec))]
            lbs = [static.data(sp.name or f'label{i}', list(sp.shape), sp.dtype)
                   for i, sp in enumerate(_to_list(labels_spec))]
            outs = self._model(*ins)
            loss = self._compute_loss(outs, lbs)
        dist, vmap, part = parallelize(serial)
        local = [part.local_param(p) for p in self._model.parameters() if id(p) in part.params]
        if self._optimizer is not None:
            self._apply_passes(dist, serial, vmap, part, ins, outs)
        self._dist = {'program': dist, 'feeds': [v.name for v in ins + lbs], 'n_in': len(ins),
                      'label_specs': list(_to_list(labels_spec)),
                      'loss': vmap[loss], 'outs': [vmap[o] for o in _to_list(outs)],
                      'partitioner': part, 'serial': serial, 'params': local}
        eval_prog = dist.clone(for_test=True)
        if self._optimizer is not None:
            opt = self._optimizer
            opt._param_groups = []                     # update this rank's shards
            opt._add_param_group({'params': [p for p in local if not p.stop_gradient]})
            with static.program_guard(dist):
                opt.minimize(vmap[loss], parameters=[p for p in local if not p.stop_gradient])
        self._dist['eval_program'] = eval_prog
        self._exe = static.Executor()

    def _apply_passes(self, dist, serial, vmap, part, ins, outs):
        """strategy.{amp, recompute, gradient_merge, sharding, fused_passes} as program passes on
        the partitioned program, before its minimize (reference engine.py _apply_pre_optimization
        / _apply_post_optimization -> distributed/passes); the distributed global-norm clip
        whenever the optimizer clips by global norm."""
        from ..passes import new_pass, PassManager
        from ...nn.clip import ClipGradByGlobalNorm
        st = self._strategy
        passes = []
        if st is not None and st.amp.enable:
            lvl = str(st.amp.level).lower()
            passes.append(new_pass('auto_parallel_fp16' if lvl in ('o2', 'o3') else 'auto_parallel_amp', {
                'dtype': st.amp.dtype, 'custom_white_list': st.amp.custom_white_list,
                'custom_black_list': st.amp.custom_black_list,
                'init_loss_scaling': st.amp.init_loss_scaling,
                'use_dynamic_loss_scaling': st.amp.use_dynamic_loss_scaling,
                'incr_every_n_steps': st.amp.incr_every_n_steps,
                'decr_every_n_nan_or_inf': st.amp.decr_every_n_nan_or_inf,
                'incr_ratio': st.amp.incr_ratio, 'decr_ratio': st.amp.decr_ratio,
                'use_optimizer_fp16': lvl == 'o3'}))
        if st is not None and st.recompute.enable:
            blk = serial.global_block()
            ck = [vmap[blk.var(c) if isinstance(c, str) else c].name for c in st.recompute.checkpoints or []]
            if not ck and not any('recompute_id' in op.attrs for op in dist.global_block().ops):
                # no checkpoints, no auto_parallel.recompute regions: the whole model is one
                # segment (what the dygraph Engine's recompute(model) does)
                ck = [vmap[o].name for o in _to_list(outs)]
            passes.append(new_pass('auto_parallel_recompute', {
                'checkpoints': ck or None, 'no_recompute_segments': st.recompute.no_recompute_segments}))
        if st is not None and st.gradient_merge.enable and int(st.gradient_merge.k_steps) > 1:
            passes.append(new_pass('auto_parallel_gradient_merge_pass', {
                'k_steps': int(st.gradient_merge.k_steps), 'avg': bool(st.gradient_merge.avg)}))
        if st is not None and st.sharding.enable:
            group = None
            if ins:
                m = part.ctx.get(ins[0])
                if m and m[0] >= 0:
                    group = part.ctx.mesh.axis_group(m[0])
            passes.append(new_pass('auto_parallel_sharding', {'stage': int(st.sharding.stage), 'group': group}))
        if isinstance(getattr(self._optimizer, '_grad_clip', None), ClipGradByGlobalNorm):
            passes.append(new_pass('auto_parallel_grad_clip'))
        if st is not None and st.fused_passes.enable:
            passes += [new_pass(n) for n in st.fused_passes.fused_passes_list or []]
        if passes:
            self._pass_context = PassManager(passes).apply([dist], [None])

    def _static_feed(self, batch, split):
        inputs, labels = self._split(batch, split)
        vals = [x.numpy() if isinstance(x, Tensor) else np.asarray(x) for x in inputs + labels]
        return dict(zip(self._dist['feeds'], vals))

    def local_parameters(self):
        """This rank's parameter shards of the partitioned static program."""
        return list(self._dist['params']) if getattr(self, '_dist', None) else list(self._model.parameters())

    # ------------------------------------------------------------------ public API
    def prepare(self, inputs_spec=None, labels_spec=None, inputs=None, labels=None, main_program=None,
                startup_program=None, mode='train'):
        if self._static_on():
            self._build_static(inputs_spec, labels_spec)
            return self
        self._resolve_mesh()
        return self

    def fit(self, train_data, train_sample_split=None, batch_size=1, epochs=1, steps_per_epoch=None,
            log_freq=10, save_dir=None, save_freq=1, valid_data=None, valid_sample_split=None, valid_freq=1,
            valid_steps=None, collate_fn=None, callbacks=None, verbose=2, nvprof_range=None):
        assert self._optimizer is not None, "fit() needs an optimizer"
        if getattr(self, '_dist', None) is not None:
            return self._fit_static(train_data, train_sample_split, batch_size, epochs, steps_per_epoch,
                                    log_freq, collate_fn, verbose)
        self._model.train()
        loader = self._loader(train_data, batch_size, False, collate_fn)
        history = {'loss': []}
        for epoch in range(epochs):
            for m in self._metrics:
                m.reset()
            for step, batch in enumerate(loader):
                if steps_per_epoch is not None and step >= steps_per_epoch:
                    break
                inputs, labels = self._split(batch, train_sample_split)
                loss, outs = self._train_step(inputs, labels)
                history['loss'].append(float(loss))
                logs = self._update_metrics(outs, labels) if self._metrics else {}
                logs.update(self._fetch_logs())
                for kk, v in logs.items():
                    history.setdefault(kk, []).append(v)
                if verbose and log_freq and step % log_freq == 0 and C.get_rank() == 0:
                    print(f"[Engine] epoch {epoch} step {step} loss {float(loss):.6f}")
            if save_dir is not None and (epoch + 1) % save_freq == 0:
                self.save(f"{save_dir}/epoch{epoch}")
            if valid_data is not None and (epoch + 1) % valid_freq == 0:
                ev = self.evaluate(valid_data, valid_sample_split, batch_size, valid_steps,
                                   collate_fn=collate_fn, verbose=0)
                for kk, v in ev.items():
                    history.setdefault('eval_' + kk, []).append(v)
                self._model.train()
        self.history = history
        return history

    def _static_loader(self, data, batch_size, collate_fn):
        from ...io import DataLoader, BatchSampler, Dataset
        if not isinstance(data, Dataset) and hasattr(data, '__iter__') and not hasattr(data, '__getitem__'):
            return data
        # every rank is fed the whole batch: the partitioned program slices its own share
        return DataLoader(data, batch_sampler=BatchSampler(data, batch_size=batch_size, shuffle=False),
                          collate_fn=collate_fn)

    def _fit_static(self, data, split, batch_size, epochs, steps_per_epoch, log_freq, collate_fn, verbose):
        d = self._dist
        history = {'loss': []}
        for epoch in range(epochs):
            for step, batch in enumerate(self._static_loader(data, batch_size, collate_fn)):
                if steps_per_epoch is not None and step >= steps_per_epoch:
                    break
                loss, = self._exe.run(d['program'], feed=self._static_feed(batch, split), fetch_list=[d['loss']])
                history['loss'].append(float(loss))
                if verbose and log_freq and step % log_freq == 0 and C.get_rank() == 0:
                    print(f"[Engine] epoch {epoch} step {step} loss {float(loss):.6f}")
        self.history = history
        return history

    @torch.no_grad()
    def evaluate(self, valid_data, valid_sample_split=None, batch_size=1, steps=None, log_freq=10,
                 collate_fn=None, callbacks=None, verbose=2):
        if getattr(self, '_dist', None) is not None:
            d, losses = self._dist, []
            for step, batch in enumerate(self._static_loader(valid_data, batch_size, collate_fn)):
                if steps is not None and step >= steps:
                    break
                loss, = self._exe.run(d['eval_program'], feed=self._static_feed(batch, valid_sample_split),
                                      fetch_list=[d['loss']])
                losses.append(float(loss))
            return {'loss': float(np.mean(losses))} if losses else {}
        self._model.eval()
        loader = self._loader(valid_data, batch_size, False, collate_fn)
        for m in self._metrics:
            m.reset()
        losses, logs = [], {}
        for step, batch in enumerate(loader):
            if steps is not None and step >= steps:
                break
            inputs, labels = self._split(batch, valid_sample_split)
            outs = self._forward(inputs)
            if self._loss is not None:
                losses.append(float(self._compute_loss(outs, labels)))
            if self._metrics:
                logs = self._update_metrics(outs, labels)
        res = dict(logs)
        if losses:
            res['loss'] = float(np.mean(losses))
        return res

    @torch.no_grad()
    def predict(self, test_data, test_sample_split=None, batch_size=1, steps=None, collate_fn=None,
                callbacks=None, verbose=2):
        if getattr(self, '_dist', None) is not None:
            # the partitioned eval program, fetching the model outputs (whole on every rank)
            d, outputs = self._dist, []
            n_in = d['n_in']
            for step, batch in enumerate(self._static_loader(test_data, batch_size, collate_fn)):
                if steps is not None and step >= steps:
                    break
                inputs, _ = self._split(batch, test_sample_split if test_sample_split is not None
                                        else len(_to_list(batch)))
                vals = [x.numpy() if isinstance(x, Tensor) else np.asarray(x) for x in inputs[:n_in]]
                feed = dict(zip(d['feeds'][:n_in], vals))   # labels: not on the outputs' path
                outs = self._exe.run(d['eval_program'], feed=feed, fetch_list=d['outs'])
                outputs.append([np.asarray(o) for o in outs])
            return outputs
        self._model.eval()
        loader = self._loader(test_data, batch_size, False, collate_fn)
        outputs = []
        for step, batch in enumerate(loader):
            if steps is not None and step >= steps:
                break
            inputs, _ = self._split(batch, test_sample_split if test_sample_split is not None
                                    else len(_to_list(batch)))
            outs = self._forward(inputs)
            outputs.append([o.numpy() for o in _to_list(outs)])
        return outputs

    # -- checkpoints of a partitioned static program: the trained values live in this rank's
    # parameter shards (Partitioner.local_param), not in the serial model. save() gathers every
    # shard along its dims_mapping into the FULL tensor (serial names, reference .pdparams /
    # .pdopt layout; rank 0 writes), load() slices the full tensors back into the shards (and
    # the serial parameters), so a checkpoint resumes on any mesh (parity: the reference Engine's
    # save/load + auto_parallel/dist_saver.py merge of the per-rank files).
    def _shard_of(self, p):
        part = self._dist['partitioner']
        return part.params.get(id(p))

    def _gather_full(self, t, mapping):
        from . import _GatherAxis
        mesh = self._dist['partitioner'].ctx.mesh
        for i, d in enumerate(mapping or []):
            if d >= 0:
                g = mesh.axis_group(d)
                if g is not None:
                    t = _GatherAxis.apply(t.contiguous(), i, g)
        return t

    def _slice_local(self, t, mapping):
        mesh = self._dist['partitioner'].ctx.mesh
        coord = mesh.coord()
        for i, d in enumerate(mapping or []):
            if d >= 0:
                n = t.shape[i] // mesh.shape[d]
                t = t.narrow(i, coord[d] * n, n)
        return t.contiguous()

    def _dist_state(self, training):
        model_sd, by_name = {}, {}
        for k, p in self._model.state_dict().items():
            lp = self._shard_of(p)
            if lp is None:
                model_sd[k] = p
                continue
            full = self._gather_full(_u(lp).detach(), lp.__dict__.get('_dist_mapping'))
            model_sd[k] = Tensor(full)
            by_name[lp.name] = lp
        opt_sd = None
        if training and self._optimizer is not None:
            opt_sd = {}
            for k, v in self._optimizer.state_dict().items():
                if k == 'master_weights':
                    opt_sd[k] = {pn: Tensor(self._gather_full(_u(t), by_name[pn].__dict__.get('_dist_mapping')))
                                 if pn in by_name else t for pn, t in v.items()}
                    continue
                pn = next((n for n in by_name if isinstance(v, Tensor) and k.startswith(n + '_') and
                           tuple(_u(v).shape) == tuple(_u(by_name[n]).shape)), None)
                opt_sd[k] = Tensor(self._gather_full(_u(v), by_name[pn].__dict__.get('_dist_mapping'))) \
                    if pn is not None else v
        return model_sd, opt_sd

    def save(self, path, training=True):
        from ...framework.io import save
        if getattr(self, '_dist', None) is not None:
            model_sd, opt_sd = self._dist_state(training)   # collective: every rank gathers
            if C.get_rank() == 0:
                save(model_sd, path + '.pdparams')
                if opt_sd is not None:
                    save(opt_sd, path + '.pdopt')
            if C.get_world_size() > 1:
                C.barrier()
            return
        save(self._model.state_dict(), path + '.pdparams')
        if training and self._optimizer is not None:
            save(self._optimizer.state_dict(), path + '.pdopt')

    def load(self, path, strict=True, load_optimizer=True):
        import os
        from ...framework.io import load
        sd = load(path + '.pdparams')
        self._model.set_state_dict(sd)
        if getattr(self, '_dist', None) is not None:
            by_name, full_shape = {}, {}
            with torch.no_grad():
                for k, p in self._model.state_dict().items():
                    lp = self._shard_of(p)
                    if lp is None:
                        continue
                    full = _u(p).detach()
                    _u(lp).copy_(self._slice_local(full, lp.__dict__.get('_dist_mapping')))
                    by_name[lp.name] = lp
                    full_shape[lp.name] = tuple(full.shape)
            if load_optimizer and self._optimizer is not None and os.path.exists(path + '.pdopt'):
                osd = load(path + '.pdopt')
                local = {}
                for k, v in osd.items():
                    if k == 'master_weights':
                        local[k] = {pn: Tensor(self._slice_local(_u(t), by_name[pn].__dict__.get('_dist_mapping')))
                                    if pn in by_name else t for pn, t in v.items()}
                        continue
                    # the LONGEST parameter name that prefixes the key ('w_1_moment1_0' belongs to
                    # 'w_1', not 'w'), and only an accumulator with the parameter's FULL shape is
                    # sliced like it (beta-pow scalars and foreign shapes pass through)
                    pn = max((n for n in by_name if k.startswith(n + '_')), key=len, default=None)
                    if pn is not None and isinstance(v, Tensor) and _u(v).dim() > 0 and \
                            tuple(_u(v).shape) == full_shape[pn]:
                        v = Tensor(self._slice_local(_u(v), by_name[pn].__dict__.get('_dist_mapping')))
                    local[k] = v
                self._optimizer.set_state_dict(local)
            return
        if load_optimizer and self._optimizer is not None and os.path.exists(path + '.pdopt'):
            self._optimizer.set_state_dict(load(path + '.pdopt'))

    @property
    def main_program(self):
        return None

    @property
    def mode(self):
        return 'train' if self._model.training else 'eval'
