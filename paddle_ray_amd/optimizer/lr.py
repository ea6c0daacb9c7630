"""Learning-rate schedulers (parity: python/paddle/optimizer/lr.py)."""
import math
import warnings

import numpy as np


class LRScheduler:
    def __init__(self, learning_rate=0.1, last_epoch=-1, verbose=False):
        self.base_lr = float(learning_rate)
        self.last_lr = float(learning_rate)
        self.last_epoch = last_epoch
        self.verbose = verbose
        self.step()

    def __call__(self):
        return self.last_lr

    def step(self, epoch=None):
        if epoch is None:
            self.last_epoch += 1
            self.last_lr = self.get_lr()
        else:
            self.last_epoch = epoch
            self.last_lr = self._get_closed_form_lr() if hasattr(self, '_get_closed_form_lr') \
                else self.get_lr()
        if self.verbose:
            print(f'Epoch {self.last_epoch}: {type(self).__name__} set learning rate to {self.last_lr}.')

    def get_lr(self):
        raise NotImplementedError

    def state_keys(self):
        self.keys = ['last_epoch', 'last_lr']

    def state_dict(self):
        self.state_keys()
        return {k: getattr(self, k) for k in self.keys}

    def set_state_dict(self, state_dict):
        self.state_keys()
        for k in self.keys:
            if k in state_dict:
                setattr(self, k, state_dict[k])

    set_dict = set_state_dict


class NoamDecay(LRScheduler):
    def __init__(self, d_model, warmup_steps, learning_rate=1.0, last_epoch=-1, verbose=False):
        self.d_model, self.warmup_steps = d_model, warmup_steps
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        a = 1 if self.last_epoch == 0 else self.last_epoch ** -0.5
        b = self.warmup_steps ** -1.5 * self.last_epoch
        return self.base_lr * (self.d_model ** -0.5) * min(a, b)


class PiecewiseDecay(LRScheduler):
    def __init__(self, boundaries, values, last_epoch=-1, verbose=False):
        self.boundaries, self.values = boundaries, values
        super().__init__(values[0], last_epoch, verbose)

    def get_lr(self):
        for i, b in enumerate(self.boundaries):
            if self.last_epoch < b:
                return self.values[i]
        return self.values[len(self.values) - 1]


class NaturalExpDecay(LRScheduler):
    def __init__(self, learning_rate, gamma, last_epoch=-1, verbose=False):
        self.gamma = gamma
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.base_lr * math.exp(-self.gamma * self.last_epoch)


class InverseTimeDecay(LRScheduler):
    def __init__(self, learning_rate, gamma, last_epoch=-1, verbose=False):
        self.gamma = gamma
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.base_lr / (1 + self.gamma * self.last_epoch)


class PolynomialDecay(LRScheduler):
    def __init__(self, learning_rate, decay_steps, end_lr=0.0001, power=1.0, cycle=False,
                 last_epoch=-1, verbose=False):
        self.decay_steps, self.end_lr, self.power, self.cycle = decay_steps, end_lr, power, cycle
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        t = self.last_epoch
        ds = self.decay_steps
        if self.cycle:
            div = math.ceil(t / float(ds)) if t > 0 else 1
            ds = ds * div
        else:
            t = min(t, ds)
        return (self.base_lr - self.end_lr) * ((1 - float(t) / float(ds)) ** self.power) + self.end_lr


class LinearWarmup(LRScheduler):
    def __init__(self, learning_rate, warmup_steps, start_lr, end_lr, last_epoch=-1, verbose=False):
        self.learning_rate = learning_rate
        self.warmup_steps, self.start_lr, self.end_lr = warmup_steps, start_lr, end_lr
        base = learning_rate if isinstance(learning_rate, (int, float)) else learning_rate.base_lr
        super().__init__(base if not isinstance(learning_rate, LRScheduler) else end_lr, last_epoch,
                         verbose)

    def get_lr(self):
        if self.last_epoch < self.warmup_steps:
            return (self.end_lr - self.start_lr) * float(self.last_epoch) / float(
                self.warmup_steps) + self.start_lr
        if isinstance(self.learning_rate, LRScheduler):
            self.learning_rate.step(self.last_epoch - self.warmup_steps)
            return self.learning_rate()
        return self.learning_rate

    def state_dict(self):
        d = super().state_dict()
        if isinstance(self.learning_rate, LRScheduler):
            d['LinearWarmup_LR'] = self.learning_rate.state_dict()
        return d

    def set_state_dict(self, sd):
        super().set_state_dict(sd)
        if isinstance(self.learning_rate, LRScheduler) and 'LinearWarmup_LR' in sd:
            self.learning_rate.set_state_dict(sd['LinearWarmup_LR'])


class ExponentialDecay(LRScheduler):
    def __init__(self, learning_rate, gamma, last_epoch=-1, verbose=False):
        self.gamma = gamma
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.base_lr * (self.gamma ** self.last_epoch)


class MultiStepDecay(LRScheduler):
    def __init__(self, learning_rate, milestones, gamma=0.1, last_epoch=-1, verbose=False):
        self.milestones, self.gamma = milestones, gamma
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        for i, m in enumerate(self.milestones):
            if self.last_epoch < m:
                return self.base_lr * (self.gamma ** i)
        return self.base_lr * (self.gamma ** len(self.milestones))


class StepDecay(LRScheduler):
    def __init__(self, learning_rate, step_size, gamma=0.1, last_epoch=-1, verbose=False):
        self.step_size, self.gamma = step_size, gamma
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.base_lr * (self.gamma ** (self.last_epoch // self.step_size))


class LambdaDecay(LRScheduler):
    def __init__(self, learning_rate, lr_lambda, last_epoch=-1, verbose=False):
        self.lr_lambda = lr_lambda
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.base_lr * self.lr_lambda(self.last_epoch)


class MultiplicativeDecay(LRScheduler):
    def __init__(self, learning_rate, lr_lambda, last_epoch=-1, verbose=False):
        self.lr_lambda = lr_lambda
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        if self.last_epoch > 0:
            return self.last_lr * self.lr_lambda(self.last_epoch)
        return self.base_lr


class CosineAnnealingDecay(LRScheduler):
    def __init__(self, learning_rate, T_max, eta_min=0, last_epoch=-1, verbose=False):
        self.T_max, self.eta_min = T_max, eta_min
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        if self.last_epoch == 0:
            return self.base_lr
        if (self.last_epoch - 1 - self.T_max) % (2 * self.T_max) == 0:
            return self.last_lr + (self.base_lr - self.eta_min) * (
                1 - math.cos(math.pi / self.T_max)) / 2
        return (1 + math.cos(math.pi * self.last_epoch / self.T_max)) / (
            1 + math.cos(math.pi * (self.last_epoch - 1) / self.T_max)) * (
            self.last_lr - self.eta_min) + self.eta_min

    def _get_closed_form_lr(self):
        return self.eta_min + (self.base_lr - self.eta_min) * (
            1 + math.cos(math.pi * self.last_epoch / self.T_max)) / 2


class ReduceOnPlateau(LRScheduler):
    def __init__(self, learning_rate, mode='min', factor=0.1, patience=10, threshold=1e-4,
                 threshold_mode='rel', cooldown=0, min_lr=0, epsilon=1e-8, verbose=False):
        self.mode, self.factor, self.patience = mode, factor, patience
        self.threshold, self.threshold_mode = threshold, threshold_mode
        self.cooldown, self.min_lr, self.epsilon = cooldown, min_lr, epsilon
        self.cooldown_counter = 0
        self.best = None
        self.num_bad_epochs = 0
        self.last_epoch = 0
        self.base_lr = self.last_lr = float(learning_rate)
        self.verbose = verbose

    def state_keys(self):
        self.keys = ['cooldown_counter', 'best', 'num_bad_epochs', 'last_epoch', 'last_lr']

    def step(self, metrics=None, epoch=None):
        if metrics is None:
            return
        self.last_epoch = self.last_epoch + 1 if epoch is None else epoch
        m = float(metrics.item() if hasattr(metrics, 'item') else np.asarray(metrics).reshape(-1)[0])
        if self.cooldown_counter > 0:
            self.cooldown_counter -= 1
        else:
            if self.best is None or self._better(m, self.best):
                self.best = m
                self.num_bad_epochs = 0
            else:
                self.num_bad_epochs += 1
            if self.num_bad_epochs > self.patience:
                self.cooldown_counter = self.cooldown
                self.num_bad_epochs = 0
                new = max(self.last_lr * self.factor, self.min_lr)
                if self.last_lr - new > self.epsilon:
                    self.last_lr = new

    def _better(self, cur, best):
        if self.mode == 'min' and self.threshold_mode == 'rel':
            return cur < best - best * self.threshold
        if self.mode == 'min':
            return cur < best - self.threshold
        if self.threshold_mode == 'rel':
            return cur > best + best * self.threshold
        return cur > best + self.threshold


class OneCycleLR(LRScheduler):
    def __init__(self, max_learning_rate, total_steps, divide_factor=25., end_learning_rate=0.0001,
                 phase_pct=0.3, anneal_strategy='cos', three_phase=False, last_epoch=-1,
                 verbose=False):
        self.max_lr, self.total_steps = max_learning_rate, total_steps
        self.initial_lr = max_learning_rate / divide_factor
        self.end_lr = end_learning_rate
        self.anneal = anneal_strategy
        if three_phase:
            self.phases = [(float(phase_pct * total_steps) - 1, self.initial_lr, self.max_lr),
                           (float(2 * phase_pct * total_steps) - 2, self.max_lr, self.initial_lr),
                           (total_steps - 1, self.initial_lr, self.end_lr)]
        else:
            self.phases = [(float(phase_pct * total_steps) - 1, self.initial_lr, self.max_lr),
                           (total_steps - 1, self.max_lr, self.end_lr)]
        super().__init__(self.initial_lr, last_epoch, verbose)

    def _interp(self, start, end, pct):
        if self.anneal == 'cos':
            return end + (start - end) / 2.0 * (math.cos(math.pi * pct) + 1)
        return (end - start) * pct + start

    def get_lr(self):
        step = self.last_epoch
        start_step = 0
        for i, (end_step, s, e) in enumerate(self.phases):
            if step <= end_step or i == len(self.phases) - 1:
                pct = (step - start_step) / max(end_step - start_step, 1e-12)
                return self._interp(s, e, min(max(pct, 0.0), 1.0))
            start_step = end_step
        return self.end_lr


class CyclicLR(LRScheduler):
    def __init__(self, base_learning_rate, max_learning_rate, step_size_up, step_size_down=None,
                 mode='triangular', exp_gamma=1., scale_fn=None, scale_mode='cycle', last_epoch=-1,
                 verbose=False):
        self.max_lr = max_learning_rate
        step_size_down = step_size_up if step_size_down is None else step_size_down
        self.cycle_size = step_size_up + step_size_down
        self.step_up_pct = step_size_up / self.cycle_size
        self.mode, self.exp_gamma = mode, exp_gamma
        if scale_fn is None:
            if mode == 'triangular':
                scale_fn, scale_mode = (lambda x: 1.), 'cycle'
            elif mode == 'triangular2':
                scale_fn, scale_mode = (lambda x: 1 / (2. ** (x - 1))), 'cycle'
            else:
                scale_fn, scale_mode = (lambda x: exp_gamma ** x), 'iterations'
        self.scale_fn, self.scale_mode = scale_fn, scale_mode
        super().__init__(base_learning_rate, last_epoch, verbose)

    def get_lr(self):
        it = self.last_epoch
        cycle = 1 + it // self.cycle_size
        pct = 1. + it / self.cycle_size - cycle
        scale = pct / self.step_up_pct if pct <= self.step_up_pct else (1 - pct) / (
            1 - self.step_up_pct)
        amp = (self.max_lr - self.base_lr) * scale
        s = self.scale_fn(cycle if self.scale_mode == 'cycle' else it)
        return self.base_lr + amp * s
