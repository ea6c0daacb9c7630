"""paddle.onnx: ONNX export of a Layer (parity: python/paddle/onnx/export.py, which delegates to
the external paddle2onnx package; here the exporter is self-contained).

``export(layer, path, input_spec)`` runs the layer once on CPU in fp32 under a PyTorch
``TorchDispatchMode`` that records every aten operation with its concrete arguments, maps the
recorded operations to ONNX nodes (opset >= 13 semantics), folds everything that depends only on
parameters or constants into initializers (shapes are static: the spec's sizes, -1 / None taken
as 1), and writes ``path + '.onnx'`` as an ONNX ``ModelProto`` with its own protobuf writer (no
``onnx`` package needed). ``run(path_or_bytes, inputs)`` evaluates such a model with NumPy
(the op subset the exporter emits) so exports are checkable without onnxruntime.
Unsupported aten operations raise ``NotImplementedError`` naming the operation.
"""
import copy
import struct
import warnings

import numpy as np
import torch

from ..static.program_desc import _varint, _read_varint

__all__ = ['export', 'run', 'to_model_proto']

# -- minimal ONNX protobuf schema (field numbers of onnx.proto) -------------------------------------
_SCHEMA = {
    'ModelProto': {1: ('ir_version', 'int64', False), 2: ('producer_name', 'string', False),
                   3: ('producer_version', 'string', False), 7: ('graph', 'm:GraphProto', False),
                   8: ('opset_import', 'm:OperatorSetIdProto', True)},
    'OperatorSetIdProto': {1: ('domain', 'string', False), 2: ('version', 'int64', False)},
    'GraphProto': {1: ('node', 'm:NodeProto', True), 2: ('name', 'string', False),
                   5: ('initializer', 'm:TensorProto', True), 11: ('input', 'm:ValueInfoProto', True),
                   12: ('output', 'm:ValueInfoProto', True)},
    'NodeProto': {1: ('input', 'string', True), 2: ('output', 'string', True), 3: ('name', 'string', False),
                  4: ('op_type', 'string', False), 5: ('attribute', 'm:AttributeProto', True)},
    'AttributeProto': {1: ('name', 'string', False), 2: ('f', 'float', False), 3: ('i', 'int64', False),
                       4: ('s', 'bytes', False), 7: ('floats', 'float', True), 8: ('ints', 'int64', True),
                       20: ('type', 'int32', False)},
    'TensorProto': {1: ('dims', 'int64', True), 2: ('data_type', 'int32', False), 8: ('name', 'string', False),
                    9: ('raw_data', 'bytes', False)},
    'ValueInfoProto': {1: ('name', 'string', False), 2: ('type', 'm:TypeProto', False)},
    'TypeProto': {1: ('tensor_type', 'm:TypeTensor', False)},
    'TypeTensor': {1: ('elem_type', 'int32', False), 2: ('shape', 'm:TensorShapeProto', False)},
    'TensorShapeProto': {1: ('dim', 'm:Dimension', True)},
    'Dimension': {1: ('dim_value', 'int64', False), 2: ('dim_param', 'string', False)},
}
_VARINT, _I64, _LEN, _I32 = 0, 1, 2, 5
_WIRE = {'int32': _VARINT, 'int64': _VARINT, 'float': _I32, 'string': _LEN, 'bytes': _LEN}
_ONNX_DT = {np.dtype('float32'): 1, np.dtype('uint8'): 2, np.dtype('int8'): 3, np.dtype('int32'): 6,
            np.dtype('int64'): 7, np.dtype('bool'): 9, np.dtype('float16'): 10, np.dtype('float64'): 11}
_NP_DT = {v: k for k, v in _ONNX_DT.items()}


def _enc(msg, d):
    out = bytearray()
    for num, (name, kind, rep) in sorted(_SCHEMA[msg].items()):
        if name not in d or d[name] is None:
            continue
        for v in (d[name] if rep else [d[name]]):
            if kind.startswith('m:'):
                body = _enc(kind[2:], v)
                out += _varint(num << 3 | _LEN) + _varint(len(body)) + body
            elif kind == 'float':
                out += _varint(num << 3 | _I32) + struct.pack('<f', float(v))
            elif kind in ('string', 'bytes'):
                b = v.encode() if isinstance(v, str) else bytes(v)
                out += _varint(num << 3 | _LEN) + _varint(len(b)) + b
            else:
                out += _varint(num << 3 | _VARINT) + _varint(int(v))
    return bytes(out)


def _dec(msg, buf):
    schema, d, i = _SCHEMA[msg], {}, 0
    while i < len(buf):
        key, i = _read_varint(buf, i)
        num, wt = key >> 3, key & 7
        if wt == _VARINT:
            payload, i = _read_varint(buf, i)
        elif wt == _I32:
            payload, i = buf[i:i + 4], i + 4
        elif wt == _I64:
            payload, i = buf[i:i + 8], i + 8
        else:
            ln, i = _read_varint(buf, i)
            payload, i = buf[i:i + ln], i + ln
        if num not in schema:
            continue
        name, kind, rep = schema[num]
        if kind.startswith('m:'):
            vals = [_dec(kind[2:], payload)]
        elif kind == 'float':
            vals = list(struct.unpack('<%df' % (len(payload) // 4), payload)) if wt == _LEN else \
                [struct.unpack('<f', payload)[0]]
        elif kind == 'string':
            vals = [bytes(payload).decode()]
        elif kind == 'bytes':
            vals = [bytes(payload)]
        elif wt == _LEN:  # packed repeated varints
            vals, j = [], 0
            while j < len(payload):
                v, j = _read_varint(payload, j)
                vals.append(v - (1 << 64) if v >= 1 << 63 else v)
        else:
            vals = [payload - (1 << 64) if payload >= 1 << 63 else payload]
        if rep:
            d.setdefault(name, []).extend(vals)
        else:
            d[name] = vals[-1]
    return d


def _tensor_proto(name, arr):
    arr = np.ascontiguousarray(arr)
    if arr.dtype not in _ONNX_DT:
        arr = arr.astype(np.float32)
    return {'name': name, 'dims': list(arr.shape), 'data_type': _ONNX_DT[arr.dtype], 'raw_data': arr.tobytes()}


def _value_info(name, arr):
    return {'name': name, 'type': {'tensor_type': {'elem_type': _ONNX_DT.get(np.dtype(arr.dtype), 1),
                                                   'shape': {'dim': [{'dim_value': int(s)} for s in arr.shape]}}}}


def _attr(name, v):
    if isinstance(v, float):
        return {'name': name, 'f': v, 'type': 1}
    if isinstance(v, (bool, int, np.integer)):
        return {'name': name, 'i': int(v), 'type': 2}
    if isinstance(v, str):
        return {'name': name, 's': v.encode(), 'type': 3}
    v = list(v)
    if v and isinstance(v[0], float):
        return {'name': name, 'floats': v, 'type': 6}
    return {'name': name, 'ints': [int(x) for x in v], 'type': 7}


# -- recording -------------------------------------------------------------------------------------
class _Recorder(torch.utils._python_dispatch.TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.log = []

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        out = func(*args, **kwargs)
        self.log.append((func, args, kwargs, out))
        return out


def _np(t):
    return t.detach().cpu().numpy()


class _Builder:
    def __init__(self):
        self.nodes, self.inits, self.names, self.const = [], [], {}, {}
        self.n = 0

    def fresh(self, base='t'):
        self.n += 1
        return f'{base}_{self.n}'

    def name_of(self, t):
        """ONNX value name of tensor t (an initializer when it is a constant)."""
        k = id(t)
        if k in self.names:
            return self.names[k]
        nm = self.fresh('c')
        self.inits.append(_tensor_proto(nm, _np(t)))
        self.names[k] = nm
        self.const[k] = t
        return nm

    def scalar(self, v, like):
        nm = self.fresh('s')
        dt = np.float32 if like is None or like.dtype.is_floating_point else np.int64
        self.inits.append(_tensor_proto(nm, np.array(v, dtype=dt)))
        return nm

    def ints(self, vals):
        nm = self.fresh('i')
        self.inits.append(_tensor_proto(nm, np.array(list(vals), dtype=np.int64)))
        return nm

    def node(self, op, ins, outs=None, **attrs):
        outs = outs or [self.fresh(op.lower())]
        self.nodes.append({'op_type': op, 'input': list(ins), 'output': list(outs), 'name': self.fresh('n'),
                           'attribute': [_attr(k, v) for k, v in attrs.items()]})
        return outs[0]


def _is_const(b, x):
    return isinstance(x, torch.Tensor) and id(x) not in b.names or id(x) in b.const


def _emit(b, func, args, kwargs, out):
    """Append the ONNX nodes of one aten op; returns the output name (or list of names)."""
    op = func.overloadpacket.__name__
    if op.endswith('_') and not op.startswith('_'):
        op = op[:-1]  # in-place form (relu_, add_, ...): same node, the result is rebound
    a = list(args)
    t = lambda x: b.name_of(x)  # noqa: E731
    rank = out.dim() if isinstance(out, torch.Tensor) else None

    def operand(x, like):
        return t(x) if isinstance(x, torch.Tensor) else b.scalar(x, like)
    if op in ('clone', 'contiguous', 'alias', 'detach', 'lift_fresh', 'lift_fresh_copy'):
        return b.node('Identity', [t(a[0])])
    if op in ('_to_copy', 'to'):
        dt = kwargs.get('dtype', out.dtype)
        return b.node('Cast', [t(a[0])], to=_ONNX_DT[np.dtype(torch.empty(0, dtype=dt).numpy().dtype)])
    if op in ('add', 'sub', 'mul', 'div', 'rsub'):
        x, y = a[0], a[1]
        alpha = kwargs.get('alpha', a[2] if len(a) > 2 else 1)
        if op == 'rsub':
            x, y, op = y, x, 'sub'
        yn = operand(y, x)
        if alpha != 1:
            yn = b.node('Mul', [yn, b.scalar(alpha, x)])
        onnx_op = {'add': 'Add', 'sub': 'Sub', 'mul': 'Mul', 'div': 'Div'}[op]
        return b.node(onnx_op, [operand(x, y if isinstance(y, torch.Tensor) else None), yn])
    unary = {'relu': 'Relu', 'sigmoid': 'Sigmoid', 'tanh': 'Tanh', 'exp': 'Exp', 'log': 'Log', 'sqrt': 'Sqrt',
             'neg': 'Neg', 'abs': 'Abs', 'erf': 'Erf', 'reciprocal': 'Reciprocal', 'floor': 'Floor', 'ceil': 'Ceil'}
    if op in unary:
        return b.node(unary[op], [t(a[0])])
    cmp = {'ge': 'GreaterOrEqual', 'gt': 'Greater', 'le': 'LessOrEqual', 'lt': 'Less', 'eq': 'Equal'}
    if op in cmp:
        return b.node(cmp[op], [t(a[0]), operand(a[1], a[0])])
    if op == 'ne':
        return b.node('Not', [b.node('Equal', [t(a[0]), operand(a[1], a[0])])])
    if op in ('logical_not', 'bitwise_not') and out.dtype == torch.bool:
        return b.node('Not', [t(a[0])])
    if op in ('logical_and', 'bitwise_and', 'logical_or', 'bitwise_or') and out.dtype == torch.bool:
        return b.node('And' if 'and' in op else 'Or', [t(a[0]), t(a[1])])
    if op == 'rsqrt':
        return b.node('Reciprocal', [b.node('Sqrt', [t(a[0])])])
    if op == 'pow':
        return b.node('Pow', [t(a[0]), operand(a[1], a[0])])
    if op == 'gelu':
        x = t(a[0])
        if kwargs.get('approximate', a[1] if len(a) > 1 else 'none') == 'tanh':
            x3 = b.node('Mul', [b.node('Mul', [x, x]), x])
            inner = b.node('Mul', [b.node('Add', [x, b.node('Mul', [x3, b.scalar(0.044715, a[0])])]),
                                   b.scalar(0.7978845608028654, a[0])])
            return b.node('Mul', [b.node('Mul', [x, b.scalar(0.5, a[0])]),
                                  b.node('Add', [b.node('Tanh', [inner]), b.scalar(1.0, a[0])])])
        e = b.node('Erf', [b.node('Mul', [x, b.scalar(0.7071067811865476, a[0])])])
        return b.node('Mul', [b.node('Mul', [x, b.scalar(0.5, a[0])]), b.node('Add', [e, b.scalar(1.0, a[0])])])
    if op in ('hardswish', 'hardsigmoid'):
        x = t(a[0])
        hs = b.node('Div', [b.node('Clip', [b.node('Add', [x, b.scalar(3.0, a[0])]), b.scalar(0.0, a[0]),
                                           b.scalar(6.0, a[0])]), b.scalar(6.0, a[0])])
        return b.node('Mul', [x, hs]) if op == 'hardswish' else hs
    if op == 'silu':
        x = t(a[0])
        return b.node('Mul', [x, b.node('Sigmoid', [x])])
    if op in ('hardtanh', 'clamp'):
        lo = a[1] if len(a) > 1 else kwargs.get('min')
        hi = a[2] if len(a) > 2 else kwargs.get('max')
        ins = [t(a[0]), '' if lo is None else b.scalar(lo, a[0]), '' if hi is None else b.scalar(hi, a[0])]
        return b.node('Clip', ins)
    if op in ('_softmax', 'softmax'):
        return b.node('Softmax', [t(a[0])], axis=int(a[1]) % a[0].dim())
    if op in ('_log_softmax', 'log_softmax'):
        return b.node('LogSoftmax', [t(a[0])], axis=int(a[1]) % a[0].dim())
    if op == 'addmm':
        bias, m1, m2 = a[0], a[1], a[2]
        beta, alpha = kwargs.get('beta', 1), kwargs.get('alpha', 1)
        return b.node('Gemm', [t(m1), t(m2), t(bias)], alpha=float(alpha), beta=float(beta))
    if op in ('mm', 'bmm', 'matmul'):
        return b.node('MatMul', [t(a[0]), t(a[1])])
    if op == 't':
        return b.node('Transpose', [t(a[0])], perm=[1, 0]) if a[0].dim() == 2 else b.node('Identity', [t(a[0])])
    if op == 'transpose':
        perm = list(range(a[0].dim()))
        d0, d1 = int(a[1]) % a[0].dim(), int(a[2]) % a[0].dim()
        perm[d0], perm[d1] = perm[d1], perm[d0]
        return b.node('Transpose', [t(a[0])], perm=perm)
    if op == 'permute':
        return b.node('Transpose', [t(a[0])], perm=[int(d) % a[0].dim() for d in a[1]])
    if op in ('view', '_unsafe_view', 'reshape', 'flatten', 'unsqueeze', 'squeeze', '_reshape_alias', 'expand'):
        if op == 'expand':
            return b.node('Expand', [t(a[0]), b.ints(out.shape)])
        return b.node('Reshape', [t(a[0]), b.ints(out.shape)])
    if op == 'slice':
        dim = int(a[1]) if len(a) > 1 else 0
        start = a[2] if len(a) > 2 and a[2] is not None else 0
        end = a[3] if len(a) > 3 and a[3] is not None else a[0].shape[dim]
        step = a[4] if len(a) > 4 else 1
        end = min(int(end), a[0].shape[dim])
        return b.node('Slice', [t(a[0]), b.ints([start]), b.ints([end]), b.ints([dim]), b.ints([step])])
    if op == 'select':
        dim, idx = int(a[1]) % a[0].dim(), int(a[2])
        g = b.node('Gather', [t(a[0]), b.ints([idx % a[0].shape[dim]])], axis=dim)
        return b.node('Reshape', [g, b.ints(out.shape)])
    if op in ('unbind', 'split', 'split_with_sizes'):
        x = a[0]
        outs_t = list(out)
        dim = int(a[1] if op == 'unbind' else (a[2] if len(a) > 2 else kwargs.get('dim', 0))) % x.dim()
        sizes = [o.shape[dim] if op != 'unbind' else 1 for o in outs_t]
        names = [b.fresh('split') for _ in outs_t]
        b.node('Split', [t(x), b.ints(sizes)], names, axis=dim)
        if op == 'unbind':
            names = [b.node('Reshape', [nm, b.ints(o.shape)]) for nm, o in zip(names, outs_t)]
        return names
    if op == 'masked_fill':
        return b.node('Where', [t(a[1]), operand(a[2], a[0]), t(a[0])])
    if op == 'cat':
        dim = int(a[1]) if len(a) > 1 else kwargs.get('dim', 0)
        return b.node('Concat', [t(x) for x in a[0]], axis=dim % out.dim())
    if op == 'embedding':
        return b.node('Gather', [t(a[0]), t(a[1])], axis=0)
    if op == 'index_select':
        return b.node('Gather', [t(a[0]), t(a[2])], axis=int(a[1]) % a[0].dim())
    if op == 'where':
        return b.node('Where', [t(a[0]), operand(a[1], out), operand(a[2], out)])
    if op in ('mean', 'sum', 'amax'):
        dims = a[1] if len(a) > 1 else list(range(a[0].dim()))
        keep = bool(a[2]) if len(a) > 2 else kwargs.get('keepdim', False)
        onnx_op = {'mean': 'ReduceMean', 'sum': 'ReduceSum', 'amax': 'ReduceMax'}[op]
        axes = [int(d) % a[0].dim() for d in (dims if isinstance(dims, (list, tuple)) else [dims])]
        if onnx_op == 'ReduceSum':
            return b.node(onnx_op, [t(a[0]), b.ints(axes)], keepdims=int(keep))
        return b.node(onnx_op, [t(a[0])], axes=axes, keepdims=int(keep))
    if op == 'logsumexp':
        dims = a[1] if len(a) > 1 else kwargs.get('dim')
        keep = bool(a[2]) if len(a) > 2 else kwargs.get('keepdim', False)
        axes = [int(d) % a[0].dim() for d in (dims if isinstance(dims, (list, tuple)) else [dims])]
        return b.node('ReduceLogSumExp', [t(a[0])], axes=axes, keepdims=int(keep))
    if op == 'nan_to_num':
        x = t(a[0])
        return b.node('Where', [b.node('IsNaN', [x]), b.scalar(0.0, a[0]), x])
    if op in ('var', 'std'):
        x = a[0]
        dims = a[1] if len(a) > 1 and a[1] is not None else kwargs.get('dim', list(range(x.dim())))
        dims = [int(d) % x.dim() for d in (dims if isinstance(dims, (list, tuple)) else [dims])]
        corr = kwargs.get('correction', 1 if kwargs.get('unbiased', True) else 0)
        corr = 0 if corr is None else corr
        keep = kwargs.get('keepdim', False)
        n = int(np.prod([x.shape[d] for d in dims]))
        xn = t(x)
        d = b.node('Sub', [xn, b.node('ReduceMean', [xn], axes=dims, keepdims=1)])
        v = b.node('ReduceMean', [b.node('Mul', [d, d])], axes=dims, keepdims=int(keep))
        if corr:
            v = b.node('Mul', [v, b.scalar(n / max(1, n - corr), x)])
        return b.node('Sqrt', [v]) if op == 'std' else v
    if op == 'convolution':
        x, w, bias, stride, pad, dil, transposed, opad, groups = a[:9]
        ins = [t(x), t(w)] + ([t(bias)] if bias is not None else [])
        nd = w.dim() - 2
        if transposed:
            # weight [Cin, Cout/groups, k...]: ONNX ConvTranspose's W layout as is
            return b.node('ConvTranspose', ins, strides=list(stride), pads=list(pad) * 2, dilations=list(dil),
                          group=int(groups), kernel_shape=list(w.shape[2:2 + nd]),
                          output_padding=[int(v) for v in opad])
        return b.node('Conv', ins, strides=list(stride), pads=list(pad) * 2, dilations=list(dil), group=int(groups),
                      kernel_shape=list(w.shape[2:2 + nd]))
    if op in ('_native_batch_norm_legit_no_training', 'native_batch_norm', '_native_batch_norm_legit'):
        x, w, bias, rm, rv = a[:5]
        eps = a[-1]
        y = b.node('BatchNormalization', [t(x), t(w), t(bias), t(rm), t(rv)], epsilon=float(eps))
        return [y, None, None]
    if op in ('max_pool2d_with_indices', 'max_pool2d'):
        x, k = a[0], list(a[1])
        s = list(a[2]) if len(a) > 2 and a[2] else k
        p = list(a[3]) if len(a) > 3 else [0, 0]
        ceil = bool(a[5]) if len(a) > 5 else False
        y = b.node('MaxPool', [t(x)], kernel_shape=k, strides=s, pads=p * 2, ceil_mode=int(ceil))
        return [y, None] if op == 'max_pool2d_with_indices' else y
    if op == 'avg_pool2d':
        x, k = a[0], list(a[1])
        s = list(a[2]) if len(a) > 2 and a[2] else k
        p = list(a[3]) if len(a) > 3 else [0, 0]
        incl = bool(a[5]) if len(a) > 5 else True
        return b.node('AveragePool', [t(x)], kernel_shape=k, strides=s, pads=p * 2,
                      count_include_pad=int(incl))
    if op in ('_adaptive_avg_pool2d', 'adaptive_avg_pool2d'):
        if tuple(out.shape[-2:]) == (1, 1):
            return b.node('GlobalAveragePool', [t(a[0])])
        ih, iw = a[0].shape[-2:]
        oh, ow = out.shape[-2:]
        if ih % oh or iw % ow:
            raise NotImplementedError('onnx export: adaptive_avg_pool2d with a non-divisible output size')
        k = [ih // oh, iw // ow]
        return b.node('AveragePool', [t(a[0])], kernel_shape=k, strides=k, pads=[0, 0, 0, 0])
    if op == 'native_layer_norm':
        x, shape, w, bias, eps = a[:5]
        axes = list(range(x.dim() - len(shape), x.dim()))
        xn = t(x)
        mu = b.node('ReduceMean', [xn], axes=axes, keepdims=1)
        d = b.node('Sub', [xn, mu])
        var = b.node('ReduceMean', [b.node('Mul', [d, d])], axes=axes, keepdims=1)
        y = b.node('Div', [d, b.node('Sqrt', [b.node('Add', [var, b.scalar(float(eps), x)])])])
        if w is not None:
            y = b.node('Mul', [y, t(w)])
        if bias is not None:
            y = b.node('Add', [y, t(bias)])
        return [y, None, None]
    raise NotImplementedError(f'onnx export: aten.{op} is not supported')


_SHAPE_ONLY = {'zeros_like', 'ones_like', 'full_like', 'empty_like', 'new_zeros', 'new_ones', 'new_full',
               'new_empty', 'empty_strided', 'sym_size', 'size'}


def to_model_proto(layer, input_spec, opset_version=13):
    """Record ``layer`` on example inputs from ``input_spec`` and build the ModelProto dict."""
    from ..framework.core import Tensor, _u
    from ..static.input import InputSpec
    if opset_version < 13:
        warnings.warn(f'onnx export: opset {opset_version} requested; the exporter emits opset 13 '
                      'semantics (Softmax axis, ReduceSum axes input)')
        opset_version = 13
    model = copy.deepcopy(layer)
    for p in list(model.parameters()) + list(model.buffers()):
        p._t = _u(p).detach().to('cpu', torch.float32 if _u(p).is_floating_point() else _u(p).dtype)
    if hasattr(model, 'eval'):
        model.eval()
    examples = []
    for s in input_spec or []:
        if isinstance(s, InputSpec):
            shp = [1 if d is None or d < 0 else int(d) for d in s.shape]
            dt = s.dtype if isinstance(s.dtype, torch.dtype) else _u(Tensor(torch.zeros(1))).dtype
            examples.append(torch.randn(shp) if torch.empty(0, dtype=dt).is_floating_point()
                            else torch.zeros(shp, dtype=dt))
        else:
            x = _u(s).detach().cpu()
            examples.append(x.float() if x.is_floating_point() else x)
    rec = _Recorder()
    with torch.no_grad(), rec:
        out = model(*[Tensor(x) for x in examples])
    outs = [_u(o) for o in (out if isinstance(out, (list, tuple)) else [out])]
    b = _Builder()
    inputs = []
    for i, x in enumerate(examples):
        nm = f'x{i}'
        b.names[id(x)] = nm
        inputs.append(_value_info(nm, _np(x)))
    def tensors_in(args, kwargs):
        return [x for x in list(args) + list(kwargs.values()) for x in (x if isinstance(x, (list, tuple)) else [x])
                if isinstance(x, torch.Tensor)]
    # only the operations the outputs depend on (index bound checks, asserts and other host-side
    # reads of device values are dead code for the graph)
    # which recorded values depend on the inputs (everything else folds into initializers)
    derived = {id(x) for x in examples}
    producer = {}
    for k, (func, args, kwargs, res) in enumerate(rec.log):
        live = any(id(x) in derived for x in tensors_in(args, kwargs))
        for r in (res if isinstance(res, (list, tuple)) else [res]):
            if isinstance(r, torch.Tensor):
                if live:
                    derived.add(id(r))
                # an in-place op returns its input: the value keeps its producer chain, the op joins it
                producer.setdefault(id(r), k) if func.overloadpacket.__name__.endswith('_') else \
                    producer.__setitem__(id(r), k)
    inplace_of = {}
    for k, (func, args, kwargs, res) in enumerate(rec.log):
        if func.overloadpacket.__name__.endswith('_') and isinstance(res, torch.Tensor):
            inplace_of.setdefault(producer.get(id(res)), []).append(k)
    needed, stack = set(), [producer[id(o)] for o in outs if id(o) in producer]
    while stack:
        k = stack.pop()
        if k in needed:
            continue
        needed.add(k)
        stack.extend(inplace_of.get(k, []))
        stack.extend(producer[id(x)] for x in tensors_in(rec.log[k][1], rec.log[k][2]) if id(x) in producer)
    for k, (func, args, kwargs, res) in enumerate(rec.log):
        if k not in needed:
            continue
        flat_in = tensors_in(args, kwargs)
        res_list = list(res) if isinstance(res, (list, tuple)) else [res]
        opname = func.overloadpacket.__name__
        if opname in _SHAPE_ONLY:
            derived.difference_update(id(r) for r in res_list if isinstance(r, torch.Tensor))
            continue  # reads only its input's (static) shape: the output is a constant
        if not any(id(x) in derived for x in flat_in):
            continue  # depends only on parameters / constants: its outputs fold into initializers
        if opname == 'as_strided_' and isinstance(res, torch.Tensor):
            src = b.names[id(args[0])]
            b.names[id(res)] = b.node('Reshape', [src, b.ints(res.shape)])
            continue
        names = _emit(b, func, args, kwargs, res)
        names = names if isinstance(names, list) else [names]
        for r, nm in zip(res_list, names):
            if isinstance(r, torch.Tensor) and nm is not None:
                b.names[id(r)] = nm
    out_infos = []
    for j, o in enumerate(outs):
        src = b.name_of(o)
        nm = f'y{j}'
        b.node('Identity', [src], [nm])
        out_infos.append(_value_info(nm, _np(o)))
    graph = {'name': type(layer).__name__, 'node': b.nodes, 'initializer': b.inits, 'input': inputs,
             'output': out_infos}
    return {'ir_version': 8, 'producer_name': 'paddle_ray_amd', 'producer_version': '3',
            'opset_import': [{'domain': '', 'version': int(opset_version)}], 'graph': graph}


def export(layer, path, input_spec=None, opset_version=9, **configs):
    """Write ``path + '.onnx'`` (see the module docstring). Returns the file name."""
    if not input_spec:
        raise ValueError('onnx export needs input_spec (InputSpec or example tensors)')
    proto = to_model_proto(layer, input_spec, opset_version)
    fn = path + '.onnx'
    with open(fn, 'wb') as f:
        f.write(_enc('ModelProto', proto))
    return fn


# -- NumPy evaluator of the emitted op subset ------------------------------------------------------
def _conv2d(x, w, b, strides, pads, dil, group):
    n, c, h, wd = x.shape
    oc, icg, kh, kw = w.shape
    x = np.pad(x, ((0, 0), (0, 0), (pads[0], pads[2]), (pads[1], pads[3])))
    ho = (x.shape[2] - dil[0] * (kh - 1) - 1) // strides[0] + 1
    wo = (x.shape[3] - dil[1] * (kw - 1) - 1) // strides[1] + 1
    y = np.zeros((n, oc, ho, wo), dtype=np.float32)
    ocg = oc // group
    for g in range(group):
        xs = x[:, g * icg:(g + 1) * icg]
        for i in range(kh):
            for j in range(kw):
                patch = xs[:, :, i * dil[0]:i * dil[0] + strides[0] * ho:strides[0],
                           j * dil[1]:j * dil[1] + strides[1] * wo:strides[1]]
                y[:, g * ocg:(g + 1) * ocg] += np.einsum('nchw,oc->nohw', patch, w[g * ocg:(g + 1) * ocg, :, i, j])
    if b is not None:
        y += b[None, :, None, None]
    return y


def _conv_transpose2d(x, w, b, strides, pads, dil, group, opad):
    """ONNX ConvTranspose (2-D) as a stride-1 convolution of the zero-upsampled input with the
    flipped, in/out-swapped filter: w [Cin, Cout/group, kh, kw]."""
    n, c, h, wd = x.shape
    cin, ocg, kh, kw = w.shape
    up = np.zeros((n, c, (h - 1) * strides[0] + 1, (wd - 1) * strides[1] + 1), dtype=np.float32)
    up[:, :, ::strides[0], ::strides[1]] = x
    # per side: dil*(k-1) - pad (+ output_padding at the end); a negative amount crops
    amounts = [(dil[0] * (kh - 1) - pads[0], dil[0] * (kh - 1) - pads[2] + opad[0]),
               (dil[1] * (kw - 1) - pads[1], dil[1] * (kw - 1) - pads[3] + opad[1])]
    for ax, (lo, hi) in zip((2, 3), amounts):
        if lo < 0:
            up = np.take(up, range(-lo, up.shape[ax]), axis=ax)
            lo = 0
        if hi < 0:
            up = np.take(up, range(0, up.shape[ax] + hi), axis=ax)
            hi = 0
        pw = [(0, 0)] * 4
        pw[ax] = (lo, hi)
        up = np.pad(up, pw)
    icg = cin // group
    wc = w.reshape(group, icg, ocg, kh, kw).transpose(0, 2, 1, 3, 4).reshape(group * ocg, icg, kh, kw)
    wc = np.ascontiguousarray(wc[:, :, ::-1, ::-1])
    return _conv2d(up, wc, b, [1, 1], [0, 0, 0, 0], dil, group)


def _pool(x, k, s, p, kind, ceil=0, incl=1):
    n, c, h, w = x.shape
    fill = -np.inf if kind == 'max' else 0.0
    xp = np.pad(x, ((0, 0), (0, 0), (p[0], p[2]), (p[1], p[3])), constant_values=fill)
    rnd = np.ceil if ceil else np.floor
    ho = int(rnd((h + p[0] + p[2] - k[0]) / s[0])) + 1
    wo = int(rnd((w + p[1] + p[3] - k[1]) / s[1])) + 1
    xp = np.pad(xp, ((0, 0), (0, 0), (0, max(0, (ho - 1) * s[0] + k[0] - xp.shape[2])),
                     (0, max(0, (wo - 1) * s[1] + k[1] - xp.shape[3]))), constant_values=fill)
    out = np.full((n, c, ho, wo), fill, dtype=np.float32) if kind == 'max' else np.zeros((n, c, ho, wo), np.float32)
    for i in range(k[0]):
        for j in range(k[1]):
            v = xp[:, :, i:i + s[0] * ho:s[0], j:j + s[1] * wo:s[1]]
            out = np.maximum(out, v) if kind == 'max' else out + v
    return out if kind == 'max' else out / (k[0] * k[1])


def run(model, inputs):
    """Evaluate an exported model (file name or bytes) on a list of NumPy inputs with NumPy."""
    from math import erf as _erf
    buf = open(model, 'rb').read() if isinstance(model, str) else model
    m = _dec('ModelProto', buf)
    g = m['graph']
    env = {}
    for tp in g.get('initializer', []):
        dt = _NP_DT[tp['data_type']]
        env[tp['name']] = np.frombuffer(tp.get('raw_data', b''), dtype=dt).reshape(tp.get('dims', [])).copy()
    for vi, x in zip(g.get('input', []), inputs):
        env[vi['name']] = np.asarray(x)
    erf = np.vectorize(_erf, otypes=[np.float32])
    for nd in g.get('node', []):
        at = {a['name']: a for a in nd.get('attribute', [])}
        A = lambda k, d=None: (at[k].get('i', at[k].get('f', at[k].get('ints', at[k].get('floats')))) if k in at else d)  # noqa: E731
        ins = [env[i] if i else None for i in nd.get('input', [])]
        op = nd['op_type']
        x = ins[0] if ins else None
        if op == 'Identity':
            y = x
        elif op == 'Cast':
            y = x.astype(_NP_DT[A('to')])
        elif op in ('Add', 'Sub', 'Mul', 'Div', 'Pow'):
            f = {'Add': np.add, 'Sub': np.subtract, 'Mul': np.multiply, 'Div': np.divide, 'Pow': np.power}[op]
            y = f(x, ins[1])
        elif op in ('Relu', 'Sigmoid', 'Tanh', 'Exp', 'Log', 'Sqrt', 'Neg', 'Abs', 'Erf', 'Reciprocal', 'Floor', 'Ceil'):
            y = {'Relu': lambda v: np.maximum(v, 0), 'Sigmoid': lambda v: 1 / (1 + np.exp(-v)), 'Tanh': np.tanh,
                 'Exp': np.exp, 'Log': np.log, 'Sqrt': np.sqrt, 'Neg': np.negative, 'Abs': np.abs, 'Erf': erf,
                 'Reciprocal': lambda v: 1 / v, 'Floor': np.floor, 'Ceil': np.ceil}[op](x)
        elif op == 'Clip':
            y = np.clip(x, ins[1] if len(ins) > 1 and ins[1] is not None else None,
                        ins[2] if len(ins) > 2 and ins[2] is not None else None)
        elif op in ('Softmax', 'LogSoftmax'):
            ax = A('axis', -1)
            e = np.exp(x - x.max(axis=ax, keepdims=True))
            s = e / e.sum(axis=ax, keepdims=True)
            y = s if op == 'Softmax' else np.log(s)
        elif op == 'Gemm':
            y = A('alpha', 1.0) * (x @ ins[1]) + (A('beta', 1.0) * ins[2] if len(ins) > 2 else 0)
        elif op == 'MatMul':
            y = np.matmul(x, ins[1])
        elif op == 'Transpose':
            y = np.transpose(x, A('perm'))
        elif op == 'Reshape':
            y = x.reshape([int(v) for v in ins[1]])
        elif op == 'Expand':
            y = np.broadcast_to(x, [int(v) for v in ins[1]]).copy()
        elif op == 'Slice':
            sl = [slice(None)] * x.ndim
            sl[int(ins[3][0])] = slice(int(ins[1][0]), int(ins[2][0]), int(ins[4][0]))
            y = x[tuple(sl)]
        elif op == 'Gather':
            y = np.take(x, ins[1].astype(np.int64), axis=A('axis', 0))
        elif op == 'Split':
            ax = A('axis', 0)
            cuts = np.cumsum([int(v) for v in ins[1]])[:-1]
            parts = np.split(x, cuts, axis=ax)
            for nm, part in zip(nd['output'], parts):
                env[nm] = part
            continue
        elif op == 'Concat':
            y = np.concatenate(ins, axis=A('axis'))
        elif op in ('GreaterOrEqual', 'Greater', 'LessOrEqual', 'Less', 'Equal', 'And', 'Or'):
            f = {'GreaterOrEqual': np.greater_equal, 'Greater': np.greater, 'LessOrEqual': np.less_equal,
                 'Less': np.less, 'Equal': np.equal, 'And': np.logical_and, 'Or': np.logical_or}[op]
            y = f(x, ins[1])
        elif op == 'Not':
            y = np.logical_not(x)
        elif op == 'Where':
            y = np.where(x, ins[1], ins[2])
        elif op in ('ReduceMean', 'ReduceMax'):
            f = np.mean if op == 'ReduceMean' else np.max
            y = f(x, axis=tuple(A('axes')), keepdims=bool(A('keepdims', 1)))
        elif op == 'ReduceLogSumExp':
            ax = tuple(A('axes'))
            mx = np.max(x, axis=ax, keepdims=True)
            mx = np.where(np.isfinite(mx), mx, 0)
            y = np.log(np.sum(np.exp(x - mx), axis=ax, keepdims=True)) + mx
            if not A('keepdims', 1):
                y = np.squeeze(y, axis=ax)
        elif op == 'IsNaN':
            y = np.isnan(x)
        elif op == 'ReduceSum':
            y = np.sum(x, axis=tuple(int(v) for v in ins[1]), keepdims=bool(A('keepdims', 1)))
        elif op == 'Conv':
            y = _conv2d(x, ins[1], ins[2] if len(ins) > 2 else None, A('strides'), A('pads'), A('dilations'),
                        A('group', 1))
        elif op == 'ConvTranspose':
            y = _conv_transpose2d(x, ins[1], ins[2] if len(ins) > 2 else None, A('strides'), A('pads'),
                                  A('dilations'), A('group', 1), A('output_padding', [0, 0]))
        elif op == 'BatchNormalization':
            sh = (1, -1) + (1,) * (x.ndim - 2)
            y = (x - ins[3].reshape(sh)) / np.sqrt(ins[4].reshape(sh) + A('epsilon', 1e-5)) * ins[1].reshape(sh) + \
                ins[2].reshape(sh)
        elif op in ('MaxPool', 'AveragePool'):
            y = _pool(x, A('kernel_shape'), A('strides'), A('pads'), 'max' if op == 'MaxPool' else 'avg',
                      A('ceil_mode', 0))
        elif op == 'GlobalAveragePool':
            y = x.mean(axis=tuple(range(2, x.ndim)), keepdims=True)
        else:
            raise NotImplementedError(f'onnx run: {op}')
        env[nd['output'][0]] = np.asarray(y, dtype=y.dtype if hasattr(y, 'dtype') else np.float32)
    return [env[o['name']] for o in g.get('output', [])]
