"""Optimizers (parity: python/paddle/optimizer/{optimizer,sgd,momentum,adam,adamw,lamb,...}.py).

On the HIP device, SGD/Momentum/Adam/AdamW update ALL parameters in ONE
multi-tensor kernel launch (``ops.fused.MultiTensorAdamW`` / momentum_mt) with
fp32 master weights for bf16/fp16 params (``multi_precision``), and the
global-norm clip coefficient folded into the update as ``grad_scale``.
State-dict keys follow the reference: ``{param}_moment1_0``, ``{param}_moment2_0``,
``{param}_beta1_pow_acc_0``, ``{param}_velocity_0``, ``master_weights``, ``LR_Scheduler``.
"""
import math

import numpy as np
import torch

from ..framework.core import Tensor, Parameter, _u
from ..ops import fused as K
from ..ops import _native
from .lr import LRScheduler


class L2Decay:
    def __init__(self, coeff=0.0):
        self._coeff = float(coeff)

    def __float__(self):
        return self._coeff


class L1Decay(L2Decay):
    pass


def _wd_value(wd):
    if wd is None:
        return 0.0
    if isinstance(wd, (L2Decay,)):
        return float(wd)
    return float(wd)


class Optimizer:
    _acc_names = ()

    def __init__(self, learning_rate=0.001, parameters=None, weight_decay=None, grad_clip=None,
                 name=None, multi_precision=False):
        if parameters is not None and not isinstance(parameters, (list, tuple)):
            parameters = list(parameters)
        self._learning_rate = learning_rate
        self._grad_clip = grad_clip
        self._multi_precision = multi_precision
        self._param_groups = []
        self._weight_decay = weight_decay
        self.regularization = weight_decay if isinstance(weight_decay, L1Decay) else None
        if parameters is None:
            parameters = []
        if parameters and isinstance(parameters[0], dict):
            for g in parameters:
                self._add_param_group(dict(g))
        else:
            self._add_param_group({'params': list(parameters)})
        self._accumulators = {}     # acc_name -> {param_name: torch.Tensor}
        self._master_weights = {}   # param_name -> fp32 torch.Tensor
        self._step_count = 0
        self._fused_plan = None
        self.helper = None

    # -- groups --------------------------------------------------------------------
    def _add_param_group(self, group):
        group.setdefault('learning_rate', 1.0)
        group.setdefault('weight_decay', self._weight_decay)
        group.setdefault('grad_clip', self._grad_clip)
        group['params'] = list(group['params'])
        self._param_groups.append(group)
        self._fused_plan = None

    @property
    def _parameter_list(self):
        return [p for g in self._param_groups for p in g['params']]

    # -- lr ---------------------------------------------------------------------------
    def get_lr(self):
        lr = self._learning_rate
        return float(lr()) if isinstance(lr, LRScheduler) else float(lr)

    def set_lr(self, value):
        if isinstance(self._learning_rate, LRScheduler):
            raise RuntimeError("cannot set_lr when learning rate is an LRScheduler")
        self._learning_rate = float(value)

    def set_lr_scheduler(self, scheduler):
        self._learning_rate = scheduler

    # -- accumulators -------------------------------------------------------------------
    def _acc(self, name, p, init=0.0, dtype=torch.float32, shape=None):
        d = self._accumulators.setdefault(name, {})
        key = p.name
        if key not in d:
            t = _u(p)
            d[key] = torch.full(t.shape if shape is None else shape, init, dtype=dtype,
                                device=t.device)
        return d[key]

    def _master(self, p):
        t = _u(p)
        if not (self._multi_precision and t.dtype in (torch.float16, torch.bfloat16)):
            return None
        if p.name not in self._master_weights:
            self._master_weights[p.name] = t.detach().float().clone()
        return self._master_weights[p.name]

    # -- step ----------------------------------------------------------------------------
    def _params_grads(self):
        out = []
        for g in self._param_groups:
            for p in g['params']:
                if p.stop_gradient or p._t.grad is None:
                    continue
                out.append((p, g))
        return out

    def _clip_coef(self, pgs):
        clip = self._grad_clip
        if clip is None:
            return None
        from ..nn.clip import ClipGradByGlobalNorm
        if hasattr(clip, 'coefficient_from_params'):  # e.g. MoE clip: needs param identity
            return clip.coefficient_from_params([(p, p._t.grad) for p, g in pgs])
        if isinstance(clip, ClipGradByGlobalNorm):
            grads = [p._t.grad for p, g in pgs if getattr(p, 'need_clip', True)]
            return clip.coefficient(grads)
        clip([(p, Tensor(p._t.grad)) for p, g in pgs])
        return None

    @torch.no_grad()
    def step(self):
        pgs = self._params_grads()
        if not pgs:
            return
        self._step_count += 1
        coef = self._clip_coef(pgs)
        self._apply(pgs, coef)
        if self.regularization is not None:
            pass

    def _apply(self, pgs, coef):
        raise NotImplementedError

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        from ..static import _static_mode_enabled
        if _static_mode_enabled():
            from ..static.graph import _static_minimize
            return _static_minimize(self, loss, parameters)
        loss.backward()
        self.step()
        return None, None

    def clear_grad(self, set_to_zero=True):
        if set_to_zero:
            gs = [p._t.grad for p in self._parameter_list if p._t.grad is not None]
            if gs:
                from ..ops.fused import zero_tensors
                zero_tensors(gs)  # one multi-tensor launch, not one fill per parameter
            return
        for p in self._parameter_list:
            p._t.grad = None

    clear_gradients = clear_grad

    # -- state ---------------------------------------------------------------------------
    def state_dict(self):
        sd = {}
        for acc, d in self._accumulators.items():
            for pname, t in d.items():
                sd[f'{pname}_{acc}_0'] = Tensor(t)
        if self._master_weights:
            sd['master_weights'] = {k: Tensor(v) for k, v in self._master_weights.items()}
        if isinstance(self._learning_rate, LRScheduler):
            sd['LR_Scheduler'] = self._learning_rate.state_dict()
        sd['@step'] = self._step_count
        return sd

    def set_state_dict(self, state_dict):
        names = {p.name: p for p in self._parameter_list}
        for k, v in state_dict.items():
            if k == 'master_weights':
                for pn, t in v.items():
                    src = _u(t) if isinstance(t, Tensor) else torch.as_tensor(np.asarray(t))
                    dev = names[pn]._t.device if pn in names else src.device
                    self._master_weights[pn] = src.to(device=dev, dtype=torch.float32).clone()
                continue
            if k == 'LR_Scheduler':
                if isinstance(self._learning_rate, LRScheduler):
                    self._learning_rate.set_state_dict(v)
                continue
            if k == '@step':
                self._step_count = int(v)
                continue
            accs = [(a, a) for a in self._acc_names] + list(getattr(self, '_acc_aliases', {}).items())
            for stored, acc in sorted(accs, key=lambda x: -len(x[0])):   # longest suffix first
                suf = f'_{stored}_0'
                if k.endswith(suf):
                    pn = k[:-len(suf)]
                    src = _u(v) if isinstance(v, Tensor) else torch.as_tensor(np.asarray(v))
                    dev = names[pn]._t.device if pn in names else src.device
                    self._accumulators.setdefault(acc, {})[pn] = src.to(dev).float().clone()
                    break
        self._fused_plan = None

    set_dict = set_state_dict

    def _lr_for(self, p, group):
        lr = self.get_lr() * group.get('learning_rate', 1.0)
        return lr * p.optimize_attr.get('learning_rate', 1.0) if hasattr(p, 'optimize_attr') else lr


class SGD(Optimizer):
    def __init__(self, learning_rate=0.001, parameters=None, weight_decay=None, grad_clip=None,
                 multi_precision=False, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, multi_precision)

    def _apply(self, pgs, coef):
        for p, g in pgs:
            t = p._t
            grad = t.grad.float() if coef is None else t.grad.float() * coef
            wd = _wd_value(g.get('weight_decay'))
            m = self._master(p)
            tgt = m if m is not None else t
            if wd:
                grad = grad + wd * tgt.float()
            tgt.sub_((self._lr_for(p, g) * grad).to(tgt.dtype))
            if m is not None:
                t.copy_(m)


class Momentum(Optimizer):
    _acc_names = ('velocity',)

    def __init__(self, learning_rate=0.001, momentum=0.9, parameters=None, use_nesterov=False,
                 weight_decay=None, grad_clip=None, multi_precision=False, rescale_grad=1.0,
                 use_multi_tensor=False, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, multi_precision)
        self._momentum, self._use_nesterov = momentum, use_nesterov
        self._rescale_grad = rescale_grad

    def _apply(self, pgs, coef):
        ps = [p for p, g in pgs]
        vels = [self._acc('velocity', p) for p in ps]
        masters = [self._master(p) for p in ps]
        wds = [_wd_value(g.get('weight_decay')) for p, g in pgs]
        lr = self.get_lr()
        lrm = [self._lr_for(p, g) / lr if lr else 1.0 for p, g in pgs]
        gs = 1.0 * self._rescale_grad
        if ps[0]._t.is_cuda and _native.available():
            scale_t = None if coef is None else coef.to(torch.float32).reshape(()).contiguous()
            self._mt_momentum(ps, vels, masters, wds, lrm, lr, gs, scale_t)
        else:
            grads = [p._t.grad * (coef if coef is not None else 1.0) for p in ps]
            K.momentum_ref([p._t for p in ps], grads, vels, masters, lr, self._momentum,
                           [w for w in wds], self._use_nesterov, gs)

    def _mt_momentum(self, ps, vels, masters, wds, lrm, lr, gs, scale_t=None):
        key = tuple(p._t.grad.data_ptr() for p in ps) + tuple(p._t.data_ptr() for p in ps)
        if self._fused_plan is None or self._fused_plan[0] != key:
            n = [p._t.numel() for p in ps]
            cols = [[(m if m is not None else p._t).data_ptr() for p, m in zip(ps, masters)],
                    [p._t.grad.data_ptr() for p in ps],
                    [v.data_ptr() for v in vels],
                    [0] * len(ps),
                    [p._t.data_ptr() if m is not None else 0 for p, m in zip(ps, masters)],
                    n,
                    [K._DT[p._t.grad.dtype] for p in ps],
                    [K._DT[p._t.dtype] for p in ps]]
            self._fused_plan = (key, K._mt_table(cols, n, [wds, lrm], ps[0]._t.device))
        tab, ftab, ch, nch = self._fused_plan[1]
        from ..ops import registry as R
        R.dispatch('momentum_mt', tab, tab, ftab, ch, nch, lr, self._momentum, self._use_nesterov,
                   gs, scale_t, [m if m is not None else p._t for p, m in zip(ps, masters)])


class Adam(Optimizer):
    _acc_names = ('moment1', 'moment2', 'beta1_pow_acc', 'beta2_pow_acc')
    _decoupled = False

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-08, parameters=None,
                 weight_decay=None, grad_clip=None, lazy_mode=False, multi_precision=False,
                 use_multi_tensor=False, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, multi_precision)
        self._beta1, self._beta2, self._epsilon = beta1, beta2, epsilon
        self._apply_decay_param_fun = None
        self._lr_ratio = None

    def _wd_for(self, p, g):
        wd = _wd_value(g.get('weight_decay'))
        if self._apply_decay_param_fun is not None and not self._apply_decay_param_fun(p.name):
            return 0.0
        return wd

    def _apply(self, pgs, coef):
        ps = [p for p, g in pgs]
        ms = [self._acc('moment1', p) for p in ps]
        vs = [self._acc('moment2', p) for p in ps]
        masters = [self._master(p) for p in ps]
        wds = [self._wd_for(p, g) for p, g in pgs]
        lr = self.get_lr()
        lrm = []
        for p, g in pgs:
            r = self._lr_for(p, g) / lr if lr else 1.0
            if self._lr_ratio is not None:
                r *= self._lr_ratio(p)
            lrm.append(r)
        b1, b2 = self._beta1, self._beta2
        b1 = float(b1.item()) if isinstance(b1, Tensor) else b1
        b2 = float(b2.item()) if isinstance(b2, Tensor) else b2
        step = self._step_count
        coupled = not self._decoupled and any(wds)
        if coupled:
            # Adam + L2: clip first, then the coupled decay folded into the gradient
            if coef is not None:
                for p in ps:
                    p._t.grad.mul_(coef.to(p._t.grad.dtype))
                coef = None
            for p, w, m in zip(ps, wds, masters):
                if w:
                    p._t.grad.add_((m if m is not None else p._t).to(p._t.grad.dtype), alpha=w)
            wds = [0.0] * len(ps)
        if ps[0]._t.is_cuda and _native.available():
            gscale = 1.0
            scale_t = None
            if coef is not None:  # the clip coefficient is applied inside the update kernel
                scale_t = coef.to(torch.float32).reshape(()).contiguous()
            key = tuple(p._t.grad.data_ptr() for p in ps) + tuple(p._t.data_ptr() for p in ps) + \
                tuple(wds) + tuple(lrm)
            if self._fused_plan is None or self._fused_plan[0] != key:
                plan = K.MultiTensorAdamW([p._t for p in ps], lambda: [p._t.grad for p in ps], ms, vs,
                                          masters, wds, lrm)
                self._fused_plan = (key, plan)
            plan = self._fused_plan[1]
            plan.grads_getter = lambda: [p._t.grad for p in ps]
            plan.step(lr, b1, b2, self._epsilon, step, gscale, scale_t)
        else:
            grads = [p._t.grad if coef is None else p._t.grad * coef for p in ps]
            K.adamw_ref([p._t for p in ps], grads, ms, vs, masters, lr, b1, b2, self._epsilon, wds,
                        lrm, step)


    def _betas(self):
        b1, b2 = self._beta1, self._beta2
        return (float(b1.item()) if isinstance(b1, Tensor) else b1,
                float(b2.item()) if isinstance(b2, Tensor) else b2)

    def state_dict(self):
        """Adds the reference's ``{param}_beta{1,2}_pow_acc_0``: the accumulator starts at beta
        and is multiplied after every update (adamw.py:343-348), so after t steps it holds
        beta**(t+1). They are derived from the step count here, not kept per parameter (no
        per-step fill launches)."""
        sd = super().state_dict()
        b1, b2 = self._betas()
        t = self._step_count
        for pn in self._accumulators.get('moment1', {}):
            sd[f'{pn}_beta1_pow_acc_0'] = Tensor(torch.tensor([b1 ** (t + 1)], dtype=torch.float32))
            sd[f'{pn}_beta2_pow_acc_0'] = Tensor(torch.tensor([b2 ** (t + 1)], dtype=torch.float32))
        return sd

    def set_state_dict(self, state_dict):
        super().set_state_dict(state_dict)
        for acc in ('beta1_pow_acc', 'beta2_pow_acc'):
            self._accumulators.pop(acc, None)
        if '@step' not in state_dict:  # a reference file: recover t from beta1**(t+1)
            pw = [v for k, v in state_dict.items() if k.endswith('_beta1_pow_acc_0')]
            if pw:
                self._step_count = beta_pow_to_step(pw[0], self._betas()[0])


def beta_pow_to_step(pw, beta):
    """Steps taken, from a reference ``beta_pow_acc`` (= beta**(t+1) after t updates)."""
    import math
    v = float(_u(pw).reshape(-1)[0]) if isinstance(pw, Tensor) else float(np.asarray(pw).reshape(-1)[0])
    return max(0, int(round(math.log(v) / math.log(beta))) - 1)


class AdamW(Adam):
    _decoupled = True

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, parameters=None,
                 weight_decay=0.01, lr_ratio=None, apply_decay_param_fun=None, grad_clip=None,
                 lazy_mode=False, multi_precision=False, name=None):
        super().__init__(learning_rate, beta1, beta2, epsilon, parameters, weight_decay, grad_clip,
                         lazy_mode, multi_precision, name=name)
        self._apply_decay_param_fun = apply_decay_param_fun
        self._lr_ratio = lr_ratio


class _ForeachOpt(Optimizer):
    """Optimizers without a dedicated HIP kernel: vectorised torch composition."""

    def _apply(self, pgs, coef):
        for p, g in pgs:
            t = p._t
            grad = t.grad.float()
            if coef is not None:
                grad = grad * coef
            m = self._master(p)
            tgt = m if m is not None else t
            wd = _wd_value(g.get('weight_decay'))
            if wd:
                grad = grad + wd * tgt.float()
            upd = self._update(p, grad, tgt.float(), self._lr_for(p, g))
            tgt.copy_((tgt.float() + upd).to(tgt.dtype))
            if m is not None:
                t.copy_(m)


class Adagrad(_ForeachOpt):
    _acc_names = ('moment',)

    def __init__(self, learning_rate, epsilon=1.0e-6, parameters=None, weight_decay=None,
                 grad_clip=None, name=None, initial_accumulator_value=0.0, multi_precision=False):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, multi_precision)
        self._epsilon, self._init_acc = epsilon, initial_accumulator_value

    def _update(self, p, g, w, lr):
        m = self._acc('moment', p, self._init_acc)
        m.add_(g * g)
        return -lr * g / (m.sqrt() + self._epsilon)


class Adadelta(_ForeachOpt):
    # the reference's accumulator names (adadelta.py:109-110): keys `{param}__avg_squared_grad_0`
    _acc_names = ('_avg_squared_grad', '_avg_squared_update')
    # checkpoints written before the rename used the names without the leading underscore
    _acc_aliases = {'avg_squared_grad': '_avg_squared_grad', 'avg_squared_update': '_avg_squared_update'}

    def __init__(self, learning_rate=0.001, epsilon=1.0e-6, rho=0.95, parameters=None,
                 weight_decay=None, grad_clip=None, name=None, multi_precision=False):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, multi_precision)
        self._epsilon, self._rho = epsilon, rho

    def _update(self, p, g, w, lr):
        a = self._acc('_avg_squared_grad', p)
        u = self._acc('_avg_squared_update', p)
        a.mul_(self._rho).add_((1 - self._rho) * g * g)
        upd = -torch.sqrt((u + self._epsilon) / (a + self._epsilon)) * g
        u.mul_(self._rho).add_((1 - self._rho) * upd * upd)
        return lr * upd


class Adamax(_ForeachOpt):
    _acc_names = ('moment', 'inf_norm')

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, parameters=None,
                 weight_decay=None, grad_clip=None, name=None, multi_precision=False):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, multi_precision)
        self._beta1, self._beta2, self._epsilon = beta1, beta2, epsilon

    def _update(self, p, g, w, lr):
        m = self._acc('moment', p)
        u = self._acc('inf_norm', p)
        m.mul_(self._beta1).add_((1 - self._beta1) * g)
        torch.maximum(u * self._beta2, g.abs() + self._epsilon, out=u)
        return -lr / (1 - self._beta1 ** self._step_count) * m / u


class RMSProp(_ForeachOpt):
    _acc_names = ('momentum', 'mean_square', 'mean_grad')

    def __init__(self, learning_rate, rho=0.95, epsilon=1.0e-6, momentum=0.0, centered=False,
                 parameters=None, weight_decay=None, grad_clip=None, name=None,
                 multi_precision=False):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, multi_precision)
        self._rho, self._epsilon, self._momentum, self._centered = rho, epsilon, momentum, centered

    def _update(self, p, g, w, lr):
        ms = self._acc('mean_square', p)
        mom = self._acc('momentum', p)
        ms.mul_(self._rho).add_((1 - self._rho) * g * g)
        if self._centered:
            mg = self._acc('mean_grad', p)
            mg.mul_(self._rho).add_((1 - self._rho) * g)
            denom = torch.sqrt(ms - mg * mg + self._epsilon)
        else:
            denom = torch.sqrt(ms + self._epsilon)
        mom.mul_(self._momentum).add_(lr * g / denom)
        return -mom


class Lamb(_ForeachOpt):
    _acc_names = ('moment1', 'moment2')

    def __init__(self, learning_rate=0.001, lamb_weight_decay=0.01, beta1=0.9, beta2=0.999,
                 epsilon=1e-6, parameters=None, grad_clip=None, exclude_from_weight_decay_fn=None,
                 multi_precision=False, name=None):
        super().__init__(learning_rate, parameters, None, grad_clip, name, multi_precision)
        self._wd, self._beta1, self._beta2, self._epsilon = lamb_weight_decay, beta1, beta2, epsilon
        self._exclude = exclude_from_weight_decay_fn

    def _update(self, p, g, w, lr):
        m = self._acc('moment1', p)
        v = self._acc('moment2', p)
        m.mul_(self._beta1).add_((1 - self._beta1) * g)
        v.mul_(self._beta2).add_((1 - self._beta2) * g * g)
        mh = m / (1 - self._beta1 ** self._step_count)
        vh = v / (1 - self._beta2 ** self._step_count)
        wd = 0.0 if (self._exclude is not None and self._exclude(p)) else self._wd
        r = mh / (vh.sqrt() + self._epsilon) + wd * w
        wn, rn = w.norm(), r.norm()
        trust = torch.where((wn > 0) & (rn > 0), wn / rn, torch.ones_like(wn))
        return -lr * trust * r


class LarsMomentum(_ForeachOpt):
    """Momentum with layer-wise adaptive rate scaling (parity: fluid/optimizer.py:1786
    LarsMomentumOptimizer; the `strategy.lars` meta-optimizer's replacement of Momentum):

        local_lr = lr * lars_coeff * ||w|| / (||g|| + lars_weight_decay * ||w|| + epsilon)
        v = mu * v + local_lr * (g + lars_weight_decay * w);   w -= v

    (local_lr = lr when ||w|| or ||g|| is 0; parameters whose name contains an entry of
    ``exclude_from_weight_decay`` get lars_weight_decay = 0). Accumulator key: velocity."""
    _acc_names = ('velocity',)

    def __init__(self, learning_rate=0.001, momentum=0.9, lars_coeff=0.001, lars_weight_decay=0.0005,
                 parameters=None, grad_clip=None, name=None, exclude_from_weight_decay=None,
                 epsilon=0.0, multi_precision=False, rescale_grad=1.0):
        super().__init__(learning_rate, parameters, None, grad_clip, name, multi_precision)
        self._momentum, self._lars_coeff, self._lars_wd = momentum, lars_coeff, lars_weight_decay
        self._exclude = list(exclude_from_weight_decay or [])
        self._epsilon, self._rescale_grad = epsilon, rescale_grad

    def _update(self, p, g, w, lr):
        g = g * self._rescale_grad
        wd = 0.0 if any(n in p.name for n in self._exclude) else self._lars_wd
        v = self._acc('velocity', p)
        pn, gn = w.norm(), g.norm()
        local = torch.where((pn > 0) & (gn > 0),
                            lr * self._lars_coeff * pn / (gn + wd * pn + self._epsilon),
                            torch.full_like(pn, lr))
        v.mul_(self._momentum).add_(local * (g + wd * w))
        return -v
