"""ModelAverage (parity: python/paddle/incubate/optimizer/modelaverage.py): sliding-window
average of the parameters for evaluation; ``apply()`` swaps the averages in, ``restore()``
puts the trained values back. The window follows the reference's accumulator scheme:
current sums (sum_1 + sum_2) and the previous window (sum_3), restarted when the window
length min(max_average_window, max(min_average_window, num_updates * rate)) is reached."""
import contextlib

import torch

from ...framework.core import _u
from ...optimizer.optimizer import Optimizer


class ModelAverage(Optimizer):
    def __init__(self, average_window_rate, parameters=None, min_average_window=10000,
                 max_average_window=10000, name=None):
        super().__init__(learning_rate=0.0, parameters=parameters, weight_decay=None,
                         grad_clip=None, name=name)
        self.average_window = average_window_rate
        self.min_average_window = min_average_window
        self.max_average_window = max_average_window
        ps = self._params()
        self._sum_cur = [torch.zeros_like(p, dtype=torch.float32) for p in ps]
        self._sum_old = [torch.zeros_like(p, dtype=torch.float32) for p in ps]
        self._num_acc = 0
        self._old_num_acc = 0
        self._num_updates = 0
        self._backup = None

    def _params(self):
        return [_u(p) for p in self._parameter_list if not p.stop_gradient]

    @torch.no_grad()
    def step(self):
        ps = self._params()
        self._num_updates += 1
        self._num_acc += 1
        torch._foreach_add_(self._sum_cur, [p.float() for p in ps])
        window = min(self.max_average_window,
                     max(self.min_average_window, int(self._num_updates * self.average_window)))
        if self._num_acc >= window:
            self._sum_old = [s.clone() for s in self._sum_cur]
            for s in self._sum_cur:
                s.zero_()
            self._old_num_acc = self._num_acc
            self._num_acc = 0

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        self.step()
        return None, None

    @torch.no_grad()
    def _average(self):
        n = self._num_acc + self._old_num_acc
        if n == 0:
            return None
        return [(c + o) / n for c, o in zip(self._sum_cur, self._sum_old)]

    @contextlib.contextmanager
    def apply(self, executor=None, need_restore=True):
        ps = self._params()
        avg = self._average()
        with torch.no_grad():
            self._backup = [p.detach().clone() for p in ps]
            if avg is not None:
                for p, a in zip(ps, avg):
                    p.copy_(a)
        try:
            yield
        finally:
            if need_restore:
                self.restore()

    @torch.no_grad()
    def restore(self, executor=None):
        if self._backup is None:
            return
        for p, b in zip(self._params(), self._backup):
            p.copy_(b)
        self._backup = None
