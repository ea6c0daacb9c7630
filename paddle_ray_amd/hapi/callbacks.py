"""Training callbacks (parity: python/paddle/hapi/callbacks.py)."""
import os
import time

import numpy as np


class Callback:
    def __init__(self):
        self.model, self.params = None, {}

    def set_params(self, params):
        self.params = params

    def set_model(self, model):
        self.model = model

    def on_train_begin(self, logs=None): pass
    def on_train_end(self, logs=None): pass
    def on_eval_begin(self, logs=None): pass
    def on_eval_end(self, logs=None): pass
    def on_predict_begin(self, logs=None): pass
    def on_predict_end(self, logs=None): pass
    def on_epoch_begin(self, epoch, logs=None): pass
    def on_epoch_end(self, epoch, logs=None): pass
    def on_train_batch_begin(self, step, logs=None): pass
    def on_train_batch_end(self, step, logs=None): pass
    def on_eval_batch_begin(self, step, logs=None): pass
    def on_eval_batch_end(self, step, logs=None): pass
    def on_predict_batch_begin(self, step, logs=None): pass
    def on_predict_batch_end(self, step, logs=None): pass


class CallbackList:
    def __init__(self, callbacks=None):
        self.callbacks = list(callbacks or [])

    def append(self, c):
        self.callbacks.append(c)

    def set_params(self, p):
        for c in self.callbacks:
            c.set_params(p)

    def set_model(self, m):
        for c in self.callbacks:
            c.set_model(m)

    def __getattr__(self, name):
        def call(*a, **k):
            for c in self.callbacks:
                getattr(c, name)(*a, **k)
        return call


class ProgBarLogger(Callback):
    def __init__(self, log_freq=1, verbose=2):
        super().__init__()
        self.log_freq, self.verbose = log_freq, verbose

    def on_epoch_begin(self, epoch, logs=None):
        self._epoch, self._t0 = epoch, time.time()

    def on_train_batch_end(self, step, logs=None):
        if self.verbose and step % self.log_freq == 0:
            items = ', '.join(f'{k}: {v:.4f}' if isinstance(v, float) else f'{k}: {v}'
                              for k, v in (logs or {}).items())
            print(f'Epoch {self._epoch + 1} step {step}: {items}')

    def on_eval_end(self, logs=None):
        if self.verbose:
            print('Eval:', logs)


class ModelCheckpoint(Callback):
    def __init__(self, save_freq=1, save_dir=None):
        super().__init__()
        self.save_freq, self.save_dir = save_freq, save_dir

    def on_epoch_end(self, epoch, logs=None):
        if self.save_dir and (epoch + 1) % self.save_freq == 0:
            self.model.save(os.path.join(self.save_dir, str(epoch)))

    def on_train_end(self, logs=None):
        if self.save_dir:
            self.model.save(os.path.join(self.save_dir, 'final'))


class LRScheduler(Callback):
    def __init__(self, by_step=True, by_epoch=False):
        super().__init__()
        self.by_step, self.by_epoch = by_step, by_epoch

    def _step(self):
        opt = self.model._optimizer
        from ..optimizer.lr import LRScheduler as S
        if opt is not None and isinstance(opt._learning_rate, S):
            opt._learning_rate.step()

    def on_train_batch_end(self, step, logs=None):
        if self.by_step:
            self._step()

    def on_epoch_end(self, epoch, logs=None):
        if self.by_epoch:
            self._step()


class EarlyStopping(Callback):
    def __init__(self, monitor='loss', mode='auto', patience=0, verbose=1, min_delta=0,
                 baseline=None, save_best_model=True):
        super().__init__()
        self.monitor, self.patience, self.min_delta = monitor, patience, abs(min_delta)
        self.baseline, self.save_best_model = baseline, save_best_model
        if mode == 'auto':
            mode = 'max' if 'acc' in monitor else 'min'
        self.op = np.greater if mode == 'max' else np.less
        if mode == 'min':
            self.min_delta *= -1
        self.wait_epoch, self.best_value, self.stopped_epoch = 0, None, 0

    def on_train_begin(self, logs=None):
        self.wait_epoch = 0
        self.best_value = self.baseline if self.baseline is not None else (
            -np.inf if self.op == np.greater else np.inf)

    def on_eval_end(self, logs=None):
        if logs is None or self.monitor not in logs:
            return
        cur = logs[self.monitor]
        cur = cur[0] if isinstance(cur, (list, tuple)) else cur
        if self.op(cur - self.min_delta, self.best_value):
            self.best_value, self.wait_epoch = cur, 0
            if self.save_best_model and self.params.get('save_dir'):
                self.model.save(os.path.join(self.params['save_dir'], 'best_model'))
        else:
            self.wait_epoch += 1
        if self.wait_epoch >= self.patience:
            self.model.stop_training = True


class VisualDL(Callback):
    def __init__(self, log_dir):
        super().__init__()
        self.log_dir = log_dir


class ReduceLROnPlateau(Callback):
    def __init__(self, monitor='loss', factor=0.1, patience=10, verbose=1, mode='auto',
                 min_delta=1e-4, cooldown=0, min_lr=0):
        super().__init__()
        self.monitor, self.factor, self.patience = monitor, factor, patience
        self.min_lr, self.min_delta = min_lr, min_delta
        self.best, self.wait = None, 0

    def on_eval_end(self, logs=None):
        if not logs or self.monitor not in logs:
            return
        cur = logs[self.monitor]
        cur = cur[0] if isinstance(cur, (list, tuple)) else cur
        if self.best is None or cur < self.best - self.min_delta:
            self.best, self.wait = cur, 0
        else:
            self.wait += 1
            if self.wait >= self.patience:
                opt = self.model._optimizer
                opt.set_lr(max(opt.get_lr() * self.factor, self.min_lr))
                self.wait = 0


class WandbCallback(Callback):
    """Weights & Biases logging (wandb is not installed here: logs into ``self.history``)."""

    def __init__(self, project=None, entity=None, name=None, dir=None, mode=None, job_type=None,
                 **kwargs):
        super().__init__()
        self.history = []

    def on_train_batch_end(self, step, logs=None):
        self.history.append(dict(logs or {}))

    def on_eval_end(self, logs=None):
        self.history.append({'eval': dict(logs or {})})
