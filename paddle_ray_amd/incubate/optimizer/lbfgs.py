"""LBFGS optimizer (parity: python/paddle/incubate/optimizer/lbfgs.py): closure-driven
limited-memory BFGS with optional strong-Wolfe line search, over the layer's parameters
(runs on whatever device they live on)."""
import torch

from ...framework.core import _u
from ...optimizer.optimizer import Optimizer


class LBFGS(Optimizer):
    def __init__(self, learning_rate=1.0, max_iter=20, max_eval=None, tolerance_grad=1e-7,
                 tolerance_change=1e-9, history_size=100, line_search_fn=None, parameters=None,
                 weight_decay=None, grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        if line_search_fn not in (None, 'strong_wolfe'):
            raise ValueError("only 'strong_wolfe' is supported")
        self._impl = torch.optim.LBFGS([_u(p) for p in self._parameter_list],
                                       lr=float(learning_rate), max_iter=max_iter,
                                       max_eval=max_eval, tolerance_grad=tolerance_grad,
                                       tolerance_change=tolerance_change,
                                       history_size=history_size, line_search_fn=line_search_fn)

    def step(self, closure):
        if closure is None:
            raise ValueError("LBFGS.step needs a closure that re-evaluates the loss")

        def _c():
            with torch.enable_grad():
                loss = closure()
            return _u(loss)
        return self._impl.step(_c)

    def state_dict(self):
        return self._impl.state_dict()

    def set_state_dict(self, state_dict):
        self._impl.load_state_dict(state_dict)
