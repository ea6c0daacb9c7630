"""paddle.Model high-level API (parity: python/paddle/hapi/model.py, dynamic-graph adapter)."""
import os

import numpy as np
import torch

from ..framework.core import Tensor, _u, to_tensor
from ..framework.io import save as _save, load as _load
from ..io import DataLoader, Dataset
from .callbacks import CallbackList, ProgBarLogger, ModelCheckpoint, LRScheduler


def _to_list(x):
    if x is None:
        return []
    return list(x) if isinstance(x, (list, tuple)) else [x]


def _as_tensor(x):
    if isinstance(x, Tensor):
        return x
    return to_tensor(np.asarray(x))


class Model:
    def __init__(self, network, inputs=None, labels=None):
        self.network = network
        self._inputs, self._labels = inputs, labels
        self._optimizer = self._loss = None
        self._metrics = []
        self._amp = None
        self.stop_training = False

    def prepare(self, optimizer=None, loss=None, metrics=None, amp_configs=None):
        self._optimizer, self._loss = optimizer, loss
        self._metrics = _to_list(metrics)
        self._amp = amp_configs

    def parameters(self, *a, **k):
        return self.network.parameters(*a, **k)

    def _split(self, data):
        data = _to_list(data)
        n_in = len(_to_list(self._inputs)) or (len(data) - 1 if len(data) > 1 else 1)
        return [_as_tensor(d) for d in data[:n_in]], [_as_tensor(d) for d in data[n_in:]]

    def train_batch(self, inputs, labels=None, update=True):
        self.network.train()
        inputs = [_as_tensor(i) for i in _to_list(inputs)]
        labels = [_as_tensor(l) for l in _to_list(labels)]
        if self._amp:
            from ..amp import auto_cast
            ctx = auto_cast(level=self._amp.get('level', 'O1') if isinstance(self._amp, dict)
                            else self._amp, dtype='bfloat16')
        else:
            import contextlib
            ctx = contextlib.nullcontext()
        with ctx:
            outs = _to_list(self.network(*inputs))
            losses = _to_list(self._loss(*(outs + labels)))
        total = losses[0]
        for l in losses[1:]:
            total = total + l
        total.backward()
        if update:
            self._optimizer.step()
            self._optimizer.clear_grad()
        metrics = []
        for m in self._metrics:
            r = m.update(*_to_list(m.compute(*(outs + labels))))
            metrics.append(r)
        lv = [float(l.numpy().mean()) for l in losses]
        return (lv, metrics) if metrics else lv

    def eval_batch(self, inputs, labels=None):
        self.network.eval()
        with torch.no_grad():
            inputs = [_as_tensor(i) for i in _to_list(inputs)]
            labels = [_as_tensor(l) for l in _to_list(labels)]
            outs = _to_list(self.network(*inputs))
            losses = _to_list(self._loss(*(outs + labels))) if self._loss and labels else []
            metrics = [m.update(*_to_list(m.compute(*(outs + labels)))) for m in self._metrics]
        lv = [float(l.numpy().mean()) for l in losses]
        return (lv, metrics) if metrics else lv

    def predict_batch(self, inputs):
        self.network.eval()
        with torch.no_grad():
            outs = _to_list(self.network(*[_as_tensor(i) for i in _to_list(inputs)]))
        return [o.numpy() for o in outs]

    def _loader(self, data, batch_size, shuffle, drop_last, num_workers):
        if data is None or isinstance(data, DataLoader):
            return data
        return DataLoader(data, batch_size=batch_size, shuffle=shuffle, drop_last=drop_last,
                          num_workers=num_workers)

    def fit(self, train_data=None, eval_data=None, batch_size=1, epochs=1, eval_freq=1, log_freq=10,
            save_dir=None, save_freq=1, verbose=2, drop_last=False, shuffle=True, num_workers=0,
            callbacks=None, accumulate_grad_batches=1, num_iters=None):
        loader = self._loader(train_data, batch_size, shuffle, drop_last, num_workers)
        eval_loader = self._loader(eval_data, batch_size, False, False, num_workers)
        cbs = CallbackList(_to_list(callbacks))
        if not any(isinstance(c, ProgBarLogger) for c in cbs.callbacks):
            cbs.append(ProgBarLogger(log_freq, verbose))
        if save_dir and not any(isinstance(c, ModelCheckpoint) for c in cbs.callbacks):
            cbs.append(ModelCheckpoint(save_freq, save_dir))
        if not any(isinstance(c, LRScheduler) for c in cbs.callbacks):
            cbs.append(LRScheduler())
        cbs.set_model(self)
        cbs.set_params({'epochs': epochs, 'save_dir': save_dir, 'verbose': verbose})
        cbs.on_train_begin()
        self.stop_training = False
        it = 0
        for ep in range(epochs):
            cbs.on_epoch_begin(ep)
            for m in self._metrics:
                m.reset()
            logs = {}
            for step, data in enumerate(loader):
                cbs.on_train_batch_begin(step)
                ins, labs = self._split(data)
                upd = (step + 1) % accumulate_grad_batches == 0
                r = self.train_batch(ins, labs, update=upd)
                lv = r[0] if isinstance(r, tuple) else r
                logs = {'loss': lv[0] if len(lv) == 1 else lv, 'step': step}
                for m in self._metrics:
                    a = m.accumulate()
                    for n, v in zip(_to_list(m.name()), _to_list(a)):
                        logs[n] = v
                cbs.on_train_batch_end(step, logs)
                it += 1
                if num_iters is not None and it >= num_iters:
                    break
            cbs.on_epoch_end(ep, logs)
            if eval_loader is not None and (ep + 1) % eval_freq == 0:
                self.evaluate(eval_loader, callbacks=cbs, verbose=verbose)
            if self.stop_training or (num_iters is not None and it >= num_iters):
                break
        cbs.on_train_end()

    def evaluate(self, eval_data, batch_size=1, log_freq=10, verbose=2, num_workers=0,
                 callbacks=None, num_iters=None):
        loader = self._loader(eval_data, batch_size, False, False, num_workers)
        cbs = callbacks if isinstance(callbacks, CallbackList) else CallbackList(
            _to_list(callbacks))
        for m in self._metrics:
            m.reset()
        cbs.on_eval_begin()
        losses = []
        for step, data in enumerate(loader):
            ins, labs = self._split(data)
            r = self.eval_batch(ins, labs)
            lv = r[0] if isinstance(r, tuple) else r
            losses.extend(lv[:1])
            if num_iters is not None and step + 1 >= num_iters:
                break
        logs = {}
        if losses:
            logs['loss'] = [float(np.mean(losses))]
        for m in self._metrics:
            for n, v in zip(_to_list(m.name()), _to_list(m.accumulate())):
                logs[n] = v
        cbs.on_eval_end(logs)
        return logs

    def predict(self, test_data, batch_size=1, num_workers=0, stack_outputs=False, verbose=1,
                callbacks=None):
        loader = self._loader(test_data, batch_size, False, False, num_workers)
        outs = []
        for data in loader:
            ins, _ = self._split(data)
            outs.append(self.predict_batch(ins))
        res = list(zip(*outs))
        if stack_outputs:
            res = [np.concatenate(r, 0) for r in res]
        return res

    def save(self, path, training=True):
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        _save(self.network.state_dict(), path + '.pdparams')
        if training and self._optimizer is not None:
            _save(self._optimizer.state_dict(), path + '.pdopt')

    def load(self, path, skip_mismatch=False, reset_optimizer=False):
        self.network.set_state_dict(_load(path + '.pdparams'))
        if not reset_optimizer and self._optimizer is not None and os.path.exists(path + '.pdopt'):
            self._optimizer.set_state_dict(_load(path + '.pdopt'))

    def summary(self, input_size=None, dtype=None):
        from .summary import summary
        return summary(self.network, input_size, dtype)
