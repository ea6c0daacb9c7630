"""nn.Layer base class + ParamAttr (parity: python/paddle/nn/layer/layers.py, python/paddle/fluid/param_attr.py)."""
import collections
import copy
import re

import numpy as np
import torch

from ...framework.core import (Tensor, Parameter, _u, convert_dtype, get_default_dtype,
                               _default_device, _to_torch_device, _unique_name)
from .. import initializer as I
from ...profiler import _hooks as _prof_hooks


class ParamAttr:
    def __init__(self, name=None, initializer=None, learning_rate=1.0, regularizer=None,
                 trainable=True, do_model_average=True, need_clip=True):
        self.name = name
        self.initializer = initializer
        self.learning_rate = learning_rate
        self.regularizer = regularizer
        self.trainable = trainable
        self.do_model_average = do_model_average
        self.need_clip = need_clip

    @staticmethod
    def _to_attr(arg):
        if arg is None:
            return ParamAttr()
        if isinstance(arg, ParamAttr):
            return arg
        if isinstance(arg, str):
            return ParamAttr(name=arg)
        if isinstance(arg, I.Initializer):
            return ParamAttr(initializer=arg)
        if arg is False:
            return False
        raise TypeError(f"bad param attr {arg!r}")


class WeightNormParamAttr(ParamAttr):
    def __init__(self, dim=None, **kw):
        super().__init__(**kw)
        self.dim = dim


class HookRemoveHelper:
    def __init__(self, hooks, hid):
        self._hooks, self._hid = hooks, hid

    def remove(self):
        self._hooks.pop(self._hid, None)


_layer_name_counts = collections.defaultdict(int)


class Layer:
    """Base class of all layers (parity: paddle.nn.Layer)."""

    def __init__(self, name_scope=None, dtype='float32'):
        d = self.__dict__
        d['training'] = True
        d['_dtype'] = convert_dtype(dtype) if dtype is not None else get_default_dtype()
        if convert_dtype(dtype) == torch.float32 and get_default_dtype() != torch.float32:
            d['_dtype'] = get_default_dtype()
        d['_parameters'] = collections.OrderedDict()
        d['_sub_layers'] = collections.OrderedDict()
        d['_buffers'] = collections.OrderedDict()
        d['_non_persistable_buffer_names_set'] = set()
        d['_forward_pre_hooks'] = collections.OrderedDict()
        d['_forward_post_hooks'] = collections.OrderedDict()
        d['_hook_id'] = 0
        scope = name_scope or re.sub(r'(?<!^)(?=[A-Z])', '_', type(self).__name__).lower()
        d['_full_name'] = _unique_name(scope)

    # -- construction ----------------------------------------------------------
    def full_name(self):
        return self._full_name

    def create_parameter(self, shape, attr=None, dtype=None, is_bias=False,
                         default_initializer=None):
        attr = ParamAttr._to_attr(attr)
        if attr is False:
            return None
        dt = convert_dtype(dtype) or self._dtype
        t = torch.empty([int(s) for s in shape], dtype=dt, device=_default_device())
        p = Parameter(t, trainable=attr.trainable,
                      name=attr.name or _unique_name(self._full_name + ('.b' if is_bias else '.w')),
                      regularizer=attr.regularizer, need_clip=attr.need_clip,
                      optimize_attr={'learning_rate': attr.learning_rate},
                      do_model_average=attr.do_model_average)
        I._init_param(p, attr, default_initializer, is_bias)
        return p

    def create_variable(self, name=None, persistable=None, dtype=None):
        return Tensor(torch.empty(0, dtype=convert_dtype(dtype) or self._dtype))

    create_tensor = create_variable

    def add_parameter(self, name, parameter):
        if parameter is None:
            self._parameters[name] = None
        else:
            assert isinstance(parameter, Parameter)
            self._parameters[name] = parameter
        return parameter

    def add_sublayer(self, name, sublayer):
        assert isinstance(sublayer, Layer) or sublayer is None
        self._sub_layers[str(name)] = sublayer
        return sublayer

    def register_buffer(self, name, tensor, persistable=True):
        if tensor is not None and not isinstance(tensor, Tensor):
            tensor = Tensor(tensor)
        self._buffers[name] = tensor
        if persistable:
            self._non_persistable_buffer_names_set.discard(name)
        else:
            self._non_persistable_buffer_names_set.add(name)

    def __setattr__(self, name, value):
        d = self.__dict__
        params = d.get('_parameters')
        if isinstance(value, Parameter):
            if params is None:
                raise RuntimeError("super().__init__() must be called before assigning parameters")
            d.pop(name, None)
            self._sub_layers.pop(name, None) if '_sub_layers' in d else None
            params[name] = value
            return
        if isinstance(value, Layer):
            if '_sub_layers' not in d:
                raise RuntimeError("super().__init__() must be called before assigning sublayers")
            d.pop(name, None)
            params.pop(name, None)
            self._sub_layers[name] = value
            return
        if params is not None and name in params:
            if value is not None:
                raise TypeError(f"cannot assign {type(value)} to parameter {name}")
            params[name] = None
            return
        subs = d.get('_sub_layers')
        if subs is not None and name in subs:
            subs[name] = value
            return
        bufs = d.get('_buffers')
        if bufs is not None and name in bufs:
            if value is not None and not isinstance(value, Tensor):
                value = Tensor(value) if isinstance(value, torch.Tensor) else value
            bufs[name] = value
            return
        object.__setattr__(self, name, value)

    def __getattr__(self, name):
        d = self.__dict__
        if '_parameters' in d:
            p = d['_parameters']
            if name in p:
                return p[name]
            s = d['_sub_layers']
            if name in s:
                return s[name]
            b = d['_buffers']
            if name in b:
                return b[name]
        raise AttributeError(f"'{type(self).__name__}' object has no attribute '{name}'")

    def __delattr__(self, name):
        for k in ('_parameters', '_sub_layers', '_buffers'):
            if name in self.__dict__[k]:
                del self.__dict__[k][name]
                return
        object.__delattr__(self, name)

    def __dir__(self):
        return list(super().__dir__()) + list(self._parameters) + list(self._sub_layers) + \
            list(self._buffers)

    # -- traversal ---------------------------------------------------------------
    def named_parameters(self, prefix='', include_sublayers=True):
        seen = set()
        layers = self.named_sublayers(prefix=prefix, include_self=True) if include_sublayers \
            else [(prefix, self)]
        for lp, layer in layers:
            for n, p in layer._parameters.items():
                if p is None or id(p) in seen:
                    continue
                seen.add(id(p))
                yield (lp + '.' + n if lp else n), p

    def parameters(self, include_sublayers=True):
        return [p for _, p in self.named_parameters(include_sublayers=include_sublayers)]

    def named_sublayers(self, prefix='', include_self=False, layers_set=None):
        if layers_set is None:
            layers_set = set()
        if include_self and id(self) not in layers_set:
            layers_set.add(id(self))
            yield prefix, self
        for n, l in self._sub_layers.items():
            if l is None:
                continue
            p = prefix + '.' + n if prefix else n
            if id(l) in layers_set:
                continue
            layers_set.add(id(l))
            yield p, l
            yield from l.named_sublayers(prefix=p, include_self=False, layers_set=layers_set)

    def sublayers(self, include_self=False):
        return [l for _, l in self.named_sublayers(include_self=include_self)]

    def named_children(self):
        seen = set()
        for n, l in self._sub_layers.items():
            if l is not None and id(l) not in seen:
                seen.add(id(l))
                yield n, l

    def children(self):
        return [l for _, l in self.named_children()]

    def named_buffers(self, prefix='', include_sublayers=True):
        seen = set()
        layers = self.named_sublayers(prefix=prefix, include_self=True) if include_sublayers \
            else [(prefix, self)]
        for lp, layer in layers:
            for n, b in layer._buffers.items():
                if b is None or id(b) in seen:
                    continue
                seen.add(id(b))
                yield (lp + '.' + n if lp else n), b

    def buffers(self, include_sublayers=True):
        return [b for _, b in self.named_buffers(include_sublayers=include_sublayers)]

    def apply(self, fn):
        for l in self.children():
            l.apply(fn)
        fn(self)
        return self

    # -- modes ------------------------------------------------------------------
    def train(self):
        for l in self.sublayers(include_self=True):
            l.__dict__['training'] = True
        return self

    def eval(self):
        for l in self.sublayers(include_self=True):
            l.__dict__['training'] = False
        return self

    # -- hooks / call -------------------------------------------------------------
    def register_forward_pre_hook(self, hook):
        hid = self._hook_id
        self.__dict__['_hook_id'] += 1
        self._forward_pre_hooks[hid] = hook
        return HookRemoveHelper(self._forward_pre_hooks, hid)

    def register_forward_post_hook(self, hook):
        hid = self._hook_id
        self.__dict__['_hook_id'] += 1
        self._forward_post_hooks[hid] = hook
        return HookRemoveHelper(self._forward_post_hooks, hid)

    def forward(self, *inputs, **kwargs):
        raise NotImplementedError

    def __call__(self, *inputs, **kwargs):
        from ...static import _STATIC
        if _STATIC[0]:
            from ...static.graph import _has_var, record_layer_call
            if _has_var(inputs) or _has_var(kwargs):
                return record_layer_call(self, inputs, kwargs)
        if _prof_hooks.ACTIVE and not _prof_hooks.layer_depth():
            # the outermost layer call of a recording profiler is the step's Forward range
            from ...profiler import RecordEvent, TracerEventType
            _prof_hooks.enter_layer()
            try:
                with RecordEvent(type(self).__name__, TracerEventType.Forward):
                    return self._call_impl(*inputs, **kwargs)
            finally:
                _prof_hooks.exit_layer()
        return self._call_impl(*inputs, **kwargs)

    def _call_impl(self, *inputs, **kwargs):
        if self._forward_pre_hooks:
            for h in list(self._forward_pre_hooks.values()):
                r = h(self, inputs)
                if r is not None:
                    inputs = r if isinstance(r, tuple) else (r,)
        out = self.forward(*inputs, **kwargs)
        if self._forward_post_hooks:
            for h in list(self._forward_post_hooks.values()):
                r = h(self, inputs, out)
                if r is not None:
                    out = r
        return out

    # -- state --------------------------------------------------------------------
    def state_dict(self, destination=None, include_sublayers=True, structured_name_prefix='',
                   use_hook=True, keep_vars=True):
        dest = collections.OrderedDict() if destination is None else destination
        for n, p in self.named_parameters(include_sublayers=include_sublayers):
            dest[structured_name_prefix + n] = p
        for lp, layer in (self.named_sublayers(include_self=True) if include_sublayers
                          else [('', self)]):
            for n, b in layer._buffers.items():
                if b is None or n in layer._non_persistable_buffer_names_set:
                    continue
                dest[structured_name_prefix + (lp + '.' + n if lp else n)] = b
        return dest

    def set_state_dict(self, state_dict, use_structured_name=True):
        own = self.state_dict()
        missing, unexpected = [], []
        name_map = {}
        if not use_structured_name:
            name_map = {v.name: k for k, v in own.items()}
        for k, v in state_dict.items():
            key = name_map.get(k, k)
            if key not in own:
                unexpected.append(k)
                continue
            tgt = own[key]
            src = _u(v) if isinstance(v, Tensor) else torch.as_tensor(np.asarray(v))
            tt = tgt._t
            if list(src.shape) != list(tt.shape):
                raise ValueError(f"shape mismatch for {key}: {list(src.shape)} vs {list(tt.shape)}")
            with torch.no_grad():
                tt.copy_(src.to(device=tt.device, dtype=tt.dtype))
        for k in own:
            if k not in state_dict and not (not use_structured_name and own[k].name in state_dict):
                missing.append(k)
        return missing, unexpected

    set_dict = set_state_dict
    load_dict = set_state_dict

    def to(self, device=None, dtype=None, blocking=None):
        dev = _to_torch_device(device) if device is not None else None
        dt = convert_dtype(dtype)
        for t in self.parameters() + self.buffers():
            x = t._t
            if dt is not None and x.is_floating_point():
                x = x.to(dt)
            if dev is not None:
                x = x.to(dev)
            if x is not t._t:
                rg = t._t.requires_grad
                object.__setattr__(t, '_t', x.detach().requires_grad_(rg) if rg else x.detach())
        if dt is not None:
            for l in self.sublayers(include_self=True):
                l.__dict__['_dtype'] = dt
        return self

    def _to_impl(self, *a, **k):
        return self.to(*a, **k)

    def float(self):
        return self.to(dtype='float32')

    def half(self):
        return self.to(dtype='float16')

    def bfloat16(self):
        return self.to(dtype='bfloat16')

    def clear_gradients(self, set_to_zero=True):
        for p in self.parameters():
            if p._t.grad is not None:
                p.clear_gradient(set_to_zero)

    # -- repr ------------------------------------------------------------------------
    def extra_repr(self):
        return ''

    def __repr__(self):
        lines = []
        for n, l in self._sub_layers.items():
            r = repr(l).replace('\n', '\n  ')
            lines.append(f'({n}): {r}')
        main = type(self).__name__ + '(' + self.extra_repr()
        if lines:
            main += '\n  ' + '\n  '.join(lines) + '\n'
        return main + ')'

    def __deepcopy__(self, memo):
        cls = type(self)
        new = cls.__new__(cls)
        memo[id(self)] = new
        for k, v in self.__dict__.items():
            new.__dict__[k] = copy.deepcopy(v, memo)
        return new
