"""Model summary + FLOPs counter (parity: python/paddle/hapi/model_summary.py, dynamic_flops.py)."""
import numpy as np
import torch

from ..framework.core import Tensor, _u


def _make_inputs(input_size, dtypes=None):
    from ..tensor.creation import zeros
    if isinstance(input_size, (list, tuple)) and input_size and isinstance(input_size[0],
                                                                          (list, tuple)):
        return [zeros([1 if s in (None, -1) else s for s in shp]) for shp in input_size]
    return [zeros([1 if s in (None, -1) else s for s in input_size])]


def summary(net, input_size=None, dtypes=None, input=None):
    rows = []
    hooks = []

    def hook(layer, inp, out):
        n = sum(p._t.numel() for p in layer._parameters.values() if p is not None)
        shp = list(_u(out).shape) if isinstance(out, Tensor) else '-'
        rows.append((type(layer).__name__, shp, n))
    for l in net.sublayers():
        if not l._sub_layers:
            hooks.append(l.register_forward_post_hook(hook))
    ins = input if input is not None else _make_inputs(input_size, dtypes)
    with torch.no_grad():
        net(*(ins if isinstance(ins, (list, tuple)) else [ins]))
    for h in hooks:
        h.remove()
    total = sum(p._t.numel() for p in net.parameters())
    trainable = sum(p._t.numel() for p in net.parameters() if not p.stop_gradient)
    lines = [f'{"Layer (type)":25s} {"Output Shape":25s} {"Param #":>12s}']
    for n, s, c in rows:
        lines.append(f'{n:25s} {str(s):25s} {c:12d}')
    lines.append(f'Total params: {total:,}\nTrainable params: {trainable:,}')
    print('\n'.join(lines))
    return {'total_params': total, 'trainable_params': trainable}


def flops(net, input_size, custom_ops=None, print_detail=False):
    from ..nn.layer.common import Linear
    from ..nn.layer.conv import _ConvNd
    total = [0]
    hooks = []

    def lin(layer, inp, out):
        total[0] += int(np.prod(_u(out).shape)) * layer.weight._t.shape[0]

    def conv(layer, inp, out):
        w = layer.weight._t
        total[0] += int(np.prod(_u(out).shape)) * int(np.prod(w.shape[1:]))
    for l in net.sublayers(include_self=True):
        if isinstance(l, Linear):
            hooks.append(l.register_forward_post_hook(lin))
        elif isinstance(l, _ConvNd):
            hooks.append(l.register_forward_post_hook(conv))
    with torch.no_grad():
        net(*_make_inputs(input_size))
    for h in hooks:
        h.remove()
    if print_detail:
        print(f'Total FLOPs (MACs): {total[0]}')
    return total[0]
