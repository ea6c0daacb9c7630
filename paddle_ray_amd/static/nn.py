"""paddle.static.nn (parity: python/paddle/static/nn/common.py): layer-building functions
usable in static programs (parameters created eagerly, ops recorded)."""
from .. import nn as _nn
from ..nn import functional as F

_layers = []  # keep created layers alive (their params are referenced by the program)


def _keep(l):
    _layers.append(l)
    return l


def fc(x, size, num_flatten_dims=1, weight_attr=None, bias_attr=None, activation=None, name=None):
    in_f = 1
    for s in x.shape[num_flatten_dims:]:
        in_f *= s
    lin = _keep(_nn.Linear(in_f, size, weight_attr, bias_attr))
    if len(x.shape) > num_flatten_dims + 1:
        x = x.flatten(num_flatten_dims)
    out = lin(x)
    if activation:
        out = getattr(F, activation)(out)
    return out


def embedding(input, size, is_sparse=False, is_distributed=False, padding_idx=None,
              param_attr=None, dtype='float32'):
    return _keep(_nn.Embedding(size[0], size[1], padding_idx, weight_attr=param_attr))(input)


sparse_embedding = embedding


def conv2d(input, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=None,
           param_attr=None, bias_attr=None, use_cudnn=True, act=None, name=None,
           data_format="NCHW"):
    cin = input.shape[1] if data_format == 'NCHW' else input.shape[-1]
    out = _keep(_nn.Conv2D(cin, num_filters, filter_size, stride, padding, dilation, groups or 1,
                           weight_attr=param_attr, bias_attr=bias_attr,
                           data_format=data_format))(input)
    return getattr(F, act)(out) if act else out


def conv2d_transpose(input, num_filters, output_size=None, filter_size=None, padding=0,
                     stride=1, dilation=1, groups=None, param_attr=None, bias_attr=None,
                     use_cudnn=True, act=None, name=None, data_format='NCHW'):
    cin = input.shape[1]
    out = _keep(_nn.Conv2DTranspose(cin, num_filters, filter_size, stride, padding,
                                    dilation=dilation, groups=groups or 1,
                                    weight_attr=param_attr, bias_attr=bias_attr))(input)
    return getattr(F, act)(out) if act else out


def conv3d(input, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=None,
           param_attr=None, bias_attr=None, use_cudnn=True, act=None, name=None,
           data_format="NCDHW"):
    out = _keep(_nn.Conv3D(input.shape[1], num_filters, filter_size, stride, padding, dilation,
                           groups or 1, weight_attr=param_attr, bias_attr=bias_attr))(input)
    return getattr(F, act)(out) if act else out


def conv3d_transpose(input, num_filters, output_size=None, filter_size=None, padding=0,
                     stride=1, dilation=1, groups=None, param_attr=None, bias_attr=None,
                     use_cudnn=True, act=None, name=None, data_format='NCDHW'):
    out = _keep(_nn.Conv3DTranspose(input.shape[1], num_filters, filter_size, stride,
                                    padding))(input)
    return getattr(F, act)(out) if act else out


def batch_norm(input, act=None, is_test=False, momentum=0.9, epsilon=1e-05, param_attr=None,
               bias_attr=None, data_layout='NCHW', in_place=False, name=None,
               moving_mean_name=None, moving_variance_name=None,
               do_model_average_for_mean_and_var=True, use_global_stats=False):
    c = input.shape[1] if data_layout == 'NCHW' else input.shape[-1]
    bn = _keep(_nn.BatchNorm(c, act, is_test, momentum, epsilon, param_attr, bias_attr,
                             data_layout=data_layout, use_global_stats=use_global_stats))
    return bn(input)


def layer_norm(input, scale=True, shift=True, begin_norm_axis=1, epsilon=1e-05, param_attr=None,
               bias_attr=None, act=None, name=None):
    shp = input.shape[begin_norm_axis:]
    out = _keep(_nn.LayerNorm(shp, epsilon, param_attr if scale else False,
                              bias_attr if shift else False))(input)
    return getattr(F, act)(out) if act else out


def group_norm(input, groups, epsilon=1e-05, param_attr=None, bias_attr=None, act=None,
               data_layout='NCHW', name=None):
    out = _keep(_nn.GroupNorm(groups, input.shape[1], epsilon, param_attr, bias_attr))(input)
    return getattr(F, act)(out) if act else out


def instance_norm(input, epsilon=1e-05, param_attr=None, bias_attr=None, name=None):
    return _keep(_nn.InstanceNorm2D(input.shape[1], epsilon))(input)


def prelu(x, mode='all', param_attr=None, data_format="NCHW", name=None):
    n = 1 if mode == 'all' else x.shape[1]
    return _keep(_nn.PReLU(n, weight_attr=param_attr, data_format=data_format))(x)


def bilinear_tensor_product(x, y, size, act=None, name=None, param_attr=None, bias_attr=None):
    out = _keep(_nn.Bilinear(x.shape[-1], y.shape[-1], size, param_attr, bias_attr))(x, y)
    return getattr(F, act)(out) if act else out


def spectral_norm(weight, dim=0, power_iters=1, eps=1e-12, name=None):
    return _keep(_nn.SpectralNorm(weight.shape, dim, power_iters, eps))(weight)


def data_norm(input, act=None, epsilon=1e-05, param_attr=None, **kw):
    return layer_norm(input, epsilon=epsilon)


def deform_conv2d(*a, **k):
    raise NotImplementedError("deform_conv2d is not available in the MI355X build yet")


def nce(*a, **k):
    raise NotImplementedError("nce is not available in the MI355X build yet")


def row_conv(*a, **k):
    raise NotImplementedError


def cond(pred, true_fn=None, false_fn=None, name=None, return_names=None):
    """Data-dependent branch: both branches are recorded and selected with paddle.where."""
    from .. import where
    t = true_fn() if true_fn else None
    f = false_fn() if false_fn else None
    if t is None or f is None:
        return t if t is not None else f
    if isinstance(t, (list, tuple)):
        return type(t)(where(pred, a, b) for a, b in zip(t, f))
    return where(pred, t, f)


def case(pred_fn_pairs, default=None, name=None):
    out = default() if default else None
    for pred, fn in reversed(pred_fn_pairs):
        r = fn()
        out = r if out is None else cond(pred, lambda r=r: r, lambda o=out: o)
    return out


def switch_case(branch_index, branch_fns, default=None, name=None):
    from .. import equal, full
    items = branch_fns.items() if isinstance(branch_fns, dict) else enumerate(branch_fns)
    pairs = [(equal(branch_index, full([1], k, 'int64')), fn) for k, fn in items]
    return case(pairs, default)


def while_loop(cond, body, loop_vars, is_test=False, name=None):
    """Eager-unrolled while loop (the trip count is evaluated at graph-build time)."""
    vs = list(loop_vars)
    while bool(cond(*vs)):
        vs = list(body(*vs))
    return vs


class StaticRNN:
    def __init__(self, name=None):
        raise NotImplementedError("StaticRNN: use paddle.nn.RNN in the MI355X build")


def py_func(func, x, out, backward_func=None, skip_vars_in_backward_input=None):
    from .graph import py_func as pf
    return pf(func, x, out, backward_func, skip_vars_in_backward_input)


def _seq(*a, **k):
    raise NotImplementedError("LoD sequence ops are not part of the MI355X build")


sequence_conv = sequence_softmax = sequence_pool = sequence_concat = sequence_first_step = _seq
sequence_last_step = sequence_slice = sequence_expand = sequence_expand_as = sequence_pad = _seq
sequence_unpad = sequence_reshape = sequence_scatter = sequence_enumerate = sequence_reverse = _seq
