"""LookAhead (parity: python/paddle/incubate/optimizer/lookahead.py): every ``k`` inner
steps, slow += alpha * (fast - slow); fast = slow. One fused foreach update per sync."""
import torch

from ...framework.core import _u
from ...optimizer.optimizer import Optimizer


class LookAhead(Optimizer):
    def __init__(self, inner_optimizer, alpha=0.5, k=5, name=None):
        assert inner_optimizer is not None, "inner optimizer can not be None"
        assert 0.0 <= alpha <= 1.0, \
            "alpha should be larger or equal to 0.0, and less or equal than 1.0"
        assert isinstance(k, int) and k > 0, "k should be a positive integer"
        self.inner_optimizer = inner_optimizer
        super().__init__(learning_rate=alpha, parameters=inner_optimizer._parameter_list,
                         weight_decay=None, grad_clip=None, name=name)
        self.alpha, self.k = alpha, k
        self.type = "lookahead"
        self._slow = None
        self._la_step = 0

    @torch.no_grad()
    def step(self):
        self.inner_optimizer.step()
        self._la_step += 1
        params = [_u(p) for p in self._parameter_list if not p.stop_gradient]
        if self._slow is None:  # slow weights start at the parameters after the first step
            self._slow = [p.detach().float().clone() for p in params]
        if self._la_step % self.k == 0:
            fast = [p.float() for p in params]
            torch._foreach_add_(self._slow, torch._foreach_sub(fast, self._slow),
                                alpha=self.alpha)
            for p, s in zip(params, self._slow):
                p.copy_(s)

    def clear_grad(self, set_to_zero=True):
        self.inner_optimizer.clear_grad(set_to_zero)

    clear_gradients = clear_grad

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        loss.backward()
        self.step()
        return None, None

    def state_dict(self):
        sd = self.inner_optimizer.state_dict()
        sd['lookahead_step'] = self._la_step
        if self._slow is not None:
            for p, s in zip([p for p in self._parameter_list if not p.stop_gradient], self._slow):
                sd[p.name + '_slow'] = s.cpu().numpy()
        return sd

    def set_state_dict(self, state_dict):
        import numpy as np
        sd = dict(state_dict)
        self._la_step = int(sd.pop('lookahead_step', 0))
        ps = [p for p in self._parameter_list if not p.stop_gradient]
        slows = [sd.pop(p.name + '_slow', None) for p in ps]
        if all(s is not None for s in slows) and slows:
            self._slow = [torch.as_tensor(np.asarray(s), device=_u(p).device)
                          for p, s in zip(ps, slows)]
        self.inner_optimizer.set_state_dict(sd)
