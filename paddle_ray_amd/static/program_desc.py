"""``.pdmodel`` as a Paddle ``ProgramDesc`` protobuf (parity: paddle/fluid/framework/
framework.proto:23-246 — Version, OpDesc{Attr, Var}, VarType{TensorDesc, LoDTensorDesc},
VarDesc, BlockDesc, ProgramDesc).

A self-contained proto2 wire codec (varint / fixed32 / fixed64 / length-delimited; repeated
scalars written unpacked as proto2 does, read packed or unpacked) over a field table that
mirrors framework.proto's field numbers, so the bytes are a genuine ProgramDesc that
protobuf tooling built from framework.proto parses.

Mapping of a ``static.Program``:

* block 0 holds every variable as a VarDesc (LOD_TENSOR, TensorDesc dtype/dims; parameters
  ``persistable`` + ``is_parameter``), Paddle's ``feed`` / ``fetch`` ops with their ``col``
  attribute around the program's ops (the inference-model convention), and one OpDesc per op;
* an op's ``type`` is its registered op type; its ``inputs`` / ``outputs`` name the variables
  it reads / writes (slots ``X`` / ``Out``); scalar arguments also appear as typed attributes
  (INT/LONG/FLOAT/STRING/BOOLEAN and their lists) for readers, and the exact call structure
  (positional/keyword layout, tuples, dtypes, slices, parameter references) is kept in the
  STRING attribute ``__pra_call__`` from which the loader rebuilds the op;
* a control-flow sub-block (``cond`` / ``while_loop`` bodies) becomes its own BlockDesc with
  ``parent_idx``; the op refers to it through a BLOCK attribute (``sub_block``).
"""
import json
import struct

# ----------------------------------------------------------------------------- wire codec
_VARINT, _I64, _LEN, _I32 = 0, 1, 2, 5

# message -> {field number: (name, kind, repeated)}; kind: a scalar kind or 'm:<Message>'
_SCHEMA = {
    'Version': {1: ('version', 'int64', False)},
    'Attr': {1: ('name', 'string', False), 2: ('type', 'enum', False), 3: ('i', 'int32', False),
             4: ('f', 'float', False), 5: ('s', 'string', False), 6: ('ints', 'int32', True),
             7: ('floats', 'float', True), 8: ('strings', 'string', True), 10: ('b', 'bool', False),
             11: ('bools', 'bool', True), 12: ('block_idx', 'int32', False),
             13: ('l', 'int64', False), 14: ('blocks_idx', 'int32', True),
             15: ('longs', 'int64', True), 16: ('float64s', 'double', True),
             17: ('var_name', 'string', False), 18: ('vars_name', 'string', True),
             19: ('float64', 'double', False)},
    'OpVar': {1: ('parameter', 'string', False), 2: ('arguments', 'string', True)},
    'OpDesc': {3: ('type', 'string', False), 1: ('inputs', 'm:OpVar', True),
               2: ('outputs', 'm:OpVar', True), 4: ('attrs', 'm:Attr', True),
               5: ('is_target', 'bool', False)},
    'TensorDesc': {1: ('data_type', 'enum', False), 2: ('dims', 'int64', True)},
    'LoDTensorDesc': {1: ('tensor', 'm:TensorDesc', False), 2: ('lod_level', 'int32', False)},
    'VarType': {1: ('type', 'enum', False), 2: ('selected_rows', 'm:TensorDesc', False),
                3: ('lod_tensor', 'm:LoDTensorDesc', False),
                4: ('tensor_array', 'm:LoDTensorDesc', False)},
    'VarDesc': {1: ('name', 'string', False), 2: ('type', 'm:VarType', False),
                3: ('persistable', 'bool', False), 4: ('need_check_feed', 'bool', False),
                5: ('is_parameter', 'bool', False), 6: ('stop_gradient', 'bool', False)},
    'BlockDesc': {1: ('idx', 'int32', False), 2: ('parent_idx', 'int32', False),
                  3: ('vars', 'm:VarDesc', True), 4: ('ops', 'm:OpDesc', True),
                  5: ('forward_block_idx', 'int32', False)},
    'ProgramDesc': {1: ('blocks', 'm:BlockDesc', True), 4: ('version', 'm:Version', False)},
}
_WIRE = {'int32': _VARINT, 'int64': _VARINT, 'enum': _VARINT, 'bool': _VARINT, 'float': _I32,
         'double': _I64, 'string': _LEN}


def _varint(v):
    v &= (1 << 64) - 1  # negative int32/int64: two's complement in 10 bytes (proto2)
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _scalar(kind, v):
    if kind in ('int32', 'int64', 'enum'):
        return _varint(int(v))
    if kind == 'bool':
        return _varint(1 if v else 0)
    if kind == 'float':
        return struct.pack('<f', float(v))
    if kind == 'double':
        return struct.pack('<d', float(v))
    b = v.encode() if isinstance(v, str) else bytes(v)
    return _varint(len(b)) + b


def encode(msg, d):
    """dict -> bytes for message type ``msg`` (fields in field-number order)."""
    out = bytearray()
    for num, (name, kind, rep) in sorted(_SCHEMA[msg].items()):
        if name not in d or d[name] is None:
            continue
        vals = d[name] if rep else [d[name]]
        for v in vals:
            if kind.startswith('m:'):
                body = encode(kind[2:], v)
                out += _varint(num << 3 | _LEN) + _varint(len(body)) + body
            else:
                out += _varint(num << 3 | _WIRE[kind]) + _scalar(kind, v)
    return bytes(out)


def _read_varint(buf, i):
    v = shift = 0
    while True:
        b = buf[i]
        i += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            return v, i
        shift += 7


def _signed(v, bits=64):
    return v - (1 << 64) if v >= 1 << 63 else v


def decode(msg, buf):
    """bytes -> dict for message type ``msg``; unknown fields are skipped."""
    schema = _SCHEMA[msg]
    d, i, n = {}, 0, len(buf)
    while i < n:
        key, i = _read_varint(buf, i)
        num, wt = key >> 3, key & 7
        if wt == _VARINT:
            raw, i = _read_varint(buf, i)
            payload = raw
        elif wt == _I64:
            payload, i = buf[i:i + 8], i + 8
        elif wt == _I32:
            payload, i = buf[i:i + 4], i + 4
        elif wt == _LEN:
            ln, i = _read_varint(buf, i)
            payload, i = buf[i:i + ln], i + ln
        else:
            raise ValueError(f"ProgramDesc: unsupported wire type {wt}")
        if num not in schema:
            continue
        name, kind, rep = schema[num]
        if kind.startswith('m:'):
            vals = [decode(kind[2:], payload)]
        elif wt == _LEN and kind != 'string':  # packed repeated scalars
            vals, j = [], 0
            while j < len(payload):
                if kind == 'float':
                    vals.append(struct.unpack('<f', payload[j:j + 4])[0]); j += 4
                elif kind == 'double':
                    vals.append(struct.unpack('<d', payload[j:j + 8])[0]); j += 8
                else:
                    r, j = _read_varint(payload, j)
                    vals.append(_conv(kind, r))
        elif kind == 'string':
            vals = [bytes(payload).decode()]
        elif kind == 'float':
            vals = [struct.unpack('<f', payload)[0]]
        elif kind == 'double':
            vals = [struct.unpack('<d', payload)[0]]
        else:
            vals = [_conv(kind, payload)]
        if rep:
            d.setdefault(name, []).extend(vals)
        else:
            d[name] = vals[-1]
    return d


def _conv(kind, raw):
    if kind == 'bool':
        return bool(raw)
    if kind == 'int32':
        v = _signed(raw)
        return v - (1 << 32) if v >= 1 << 31 else v
    return _signed(raw)


# ----------------------------------------------------------------------------- enums
ATTR = dict(INT=0, FLOAT=1, STRING=2, INTS=3, FLOATS=4, STRINGS=5, BOOLEAN=6, BOOLEANS=7,
            BLOCK=8, LONG=9, BLOCKS=10, LONGS=11, FLOAT64S=12, VAR=13, VARS=14, FLOAT64=15)
VT_LOD_TENSOR, VT_FEED_MINIBATCH, VT_FETCH_LIST = 7, 9, 10
_DT2VT = {'bool': 0, 'int16': 1, 'int32': 2, 'int64': 3, 'float16': 4, 'float32': 5,
          'float64': 6, 'uint8': 20, 'int8': 21, 'bfloat16': 22, 'complex64': 23,
          'complex128': 24}
_VT2DT = {v: k for k, v in _DT2VT.items()}
PROGRAM_VERSION = 2005000  # a 2.5-era ProgramDesc version stamp


def var_desc(name, shape, dtype, persistable=False, is_parameter=False, stop_gradient=False,
             need_check_feed=False):
    return {'name': name, 'persistable': persistable, 'is_parameter': is_parameter,
            'stop_gradient': stop_gradient, 'need_check_feed': need_check_feed or None,
            'type': {'type': VT_LOD_TENSOR,
                     'lod_tensor': {'tensor': {'data_type': _DT2VT.get(dtype, 5),
                                               'dims': [int(s) for s in shape]},
                                    'lod_level': 0}}}


def var_info(vd):
    """(name, shape, dtype str) of a decoded VarDesc (None dtype for feed/fetch holders)."""
    t = vd.get('type', {})
    lt = t.get('lod_tensor')
    if t.get('type') != VT_LOD_TENSOR or lt is None:
        return vd['name'], None, None
    td = lt.get('tensor', {})
    return vd['name'], list(td.get('dims', [])), _VT2DT.get(td.get('data_type', 5), 'float32')


def scalar_attr(name, v):
    """A typed OpDesc.Attr for a plain Python value, or None if it has no attr type."""
    if isinstance(v, bool):
        return {'name': name, 'type': ATTR['BOOLEAN'], 'b': v}
    if isinstance(v, int):
        if -2 ** 31 <= v < 2 ** 31:
            return {'name': name, 'type': ATTR['INT'], 'i': v}
        return {'name': name, 'type': ATTR['LONG'], 'l': v}
    if isinstance(v, float):
        return {'name': name, 'type': ATTR['FLOAT64'], 'float64': v}
    if isinstance(v, str):
        return {'name': name, 'type': ATTR['STRING'], 's': v}
    if isinstance(v, (list, tuple)) and v:
        if all(isinstance(e, bool) for e in v):
            return {'name': name, 'type': ATTR['BOOLEANS'], 'bools': list(v)}
        if all(isinstance(e, int) and not isinstance(e, bool) for e in v):
            if all(-2 ** 31 <= e < 2 ** 31 for e in v):
                return {'name': name, 'type': ATTR['INTS'], 'ints': list(v)}
            return {'name': name, 'type': ATTR['LONGS'], 'longs': list(v)}
        if all(isinstance(e, (int, float)) and not isinstance(e, bool) for e in v):
            return {'name': name, 'type': ATTR['FLOAT64S'], 'float64s': [float(e) for e in v]}
        if all(isinstance(e, str) for e in v):
            return {'name': name, 'type': ATTR['STRINGS'], 'strings': list(v)}
    return None


def attr_value(a):
    t = a.get('type')
    key = {0: 'i', 1: 'f', 2: 's', 3: 'ints', 4: 'floats', 5: 'strings', 6: 'b', 7: 'bools',
           8: 'block_idx', 9: 'l', 10: 'blocks_idx', 11: 'longs', 12: 'float64s',
           13: 'var_name', 14: 'vars_name', 15: 'float64'}.get(t)
    default = [] if t in (3, 4, 5, 7, 10, 11, 12, 14) else None
    return a.get(key, default)


def is_program_desc(data):
    """A .pdmodel written by this module (protobuf) vs the round-1/2 JSON op list."""
    return not (data[:1] == b'{' or data[:1] == '{')


def dumps_call(obj):
    return json.dumps(obj, separators=(',', ':'))


def loads_call(s):
    return json.loads(s)
