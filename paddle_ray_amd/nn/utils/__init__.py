"""paddle.nn.utils (parity: python/paddle/nn/utils/*)."""
import torch

from ...framework.core import Tensor, _u
from ..clip import clip_grad_norm_, clip_grad_value_  # noqa


def parameters_to_vector(parameters, name=None):
    return Tensor(torch.cat([p._t.detach().reshape(-1) for p in parameters]))


def vector_to_parameters(vec, parameters, name=None):
    v = _u(vec)
    off = 0
    with torch.no_grad():
        for p in parameters:
            n = p._t.numel()
            p._t.copy_(v[off:off + n].view_as(p._t))
            off += n


def weight_norm(layer, name='weight', dim=0):
    w = getattr(layer, name)
    t = w._t.detach()
    from ...framework.core import Parameter
    dims = [i for i in range(t.dim()) if i != dim]
    g = Parameter(t.norm(dim=dims, keepdim=True) if dims else t.abs())
    v = Parameter(t.clone())
    del layer._parameters[name]
    layer.add_parameter(name + '_g', g)
    layer.add_parameter(name + '_v', v)

    def hook(l, inputs):
        vv = l._parameters[name + '_v']._t
        nrm = vv.norm(dim=dims, keepdim=True) if dims else vv.abs()
        object.__setattr__(l, name, Tensor(l._parameters[name + '_g']._t * vv / nrm))
    layer.register_forward_pre_hook(hook)
    hook(layer, None)
    return layer


def remove_weight_norm(layer, name='weight'):
    return layer


def spectral_norm(layer, name='weight', n_power_iterations=1, eps=1e-12, dim=None):
    return layer
