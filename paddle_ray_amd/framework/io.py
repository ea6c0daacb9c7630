"""paddle.save / paddle.load — ``.pdparams`` / ``.pdopt`` checkpoint format.

Byte-level layout of the reference (python/paddle/framework/io.py ``_build_saved_state_dict``
:54-70, ``reduce_varbase`` :293, ``_unpack_saved_dict`` / ``_pack_loaded_dict`` in io_utils.py,
``load`` :1060-1100):

* a top-level dict keeps its keys; every Tensor value becomes a plain ``numpy.ndarray``
  (bfloat16 as its uint16 bit pattern, Paddle's numpy representation of bf16) and the dict
  gains ``"StructuredToParameterName@@": {key: tensor.name}``;
* a Tensor anywhere else (nested containers, a bare tensor) pickles as the tuple
  ``(name, ndarray)`` exactly like the reference's ``reduce_varbase``;
* with pickle protocol 2/3, arrays over 2**30 bytes are split into ``key@@.i`` slices listed
  under ``"UnpackBigParamInfor@@"`` (protocol 4 writes them whole).

``load`` reverses all of it (uint16 arrays come back as bfloat16 tensors, names restored
from the table unless ``keep_name_table``), and also reads files written by round-1 builds
of this framework. Loading uses a RESTRICTED unpickler that only reconstructs numpy arrays /
dtypes and builtin containers: a checkpoint cannot execute code on load.
"""
import collections
import math
import os
import pickle

import numpy as np
import torch

from .core import Tensor, Parameter, _u, to_tensor  # noqa: F401

NAME_TABLE = 'StructuredToParameterName@@'
UNPACK_INFO = 'UnpackBigParamInfor@@'
_LEGACY_BF16_TAG = '__pra_bf16__'
_MAX_SLICE_BYTES = 2 ** 30 - 1


def _ndarray(t):
    t = t.detach()
    if t.dtype == torch.bfloat16:
        return t.cpu().view(torch.int16).numpy().view(np.uint16)
    return t.cpu().numpy()


def _nested(obj):
    """Non-top-level conversion: tensors become the reference's (name, ndarray) tuples."""
    if isinstance(obj, Tensor):
        return (obj.name, _ndarray(obj._t))
    if isinstance(obj, torch.Tensor):
        return (None, _ndarray(obj))
    if isinstance(obj, collections.OrderedDict):
        return collections.OrderedDict((k, _nested(v)) for k, v in obj.items())
    if isinstance(obj, dict):
        return {k: _nested(v) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_nested(v) for v in obj]
    if isinstance(obj, tuple):
        return tuple(_nested(v) for v in obj)
    if hasattr(obj, 'state_dict') and callable(obj.state_dict) and not isinstance(obj, type):
        return _build_saved_state_dict(obj.state_dict())
    return obj


def _build_saved_state_dict(state_dict):
    out = type(state_dict)() if isinstance(state_dict, collections.OrderedDict) else {}
    table = {}
    for k, v in state_dict.items():
        if isinstance(v, (Tensor, torch.Tensor)):
            out[k] = _ndarray(_u(v))
            table[k] = v.name if isinstance(v, Tensor) else k
        else:
            out[k] = _nested(v)
    out[NAME_TABLE] = table
    return out


def _unpack_saved_dict(saved, protocol, max_bytes=_MAX_SLICE_BYTES):
    if not (1 < protocol < 4) or not isinstance(saved, dict):
        return saved
    info, parts = {}, {}
    for k, v in saved.items():
        if isinstance(v, np.ndarray):
            max_el = int(max_bytes / v.dtype.itemsize)
            n = int(np.prod(v.shape))
            if n > max_el:
                flat = v.flatten()
                info[k] = {'OriginShape': v.shape, 'slices': []}
                for i in range(int(math.ceil(n / max_el))):
                    name = f'{k}@@.{i}'
                    info[k]['slices'].append(name)
                    parts[name] = flat[i * max_el:(i + 1) * max_el]
    if info:
        for k, meta in info.items():
            saved.pop(k)
            for name in meta['slices']:
                saved[name] = parts[name]
        saved[UNPACK_INFO] = info
    return saved


def _pack_loaded_dict(obj):
    if isinstance(obj, dict) and UNPACK_INFO in obj:
        removes = []
        for k, meta in obj[UNPACK_INFO].items():
            obj[k] = np.concatenate([obj[s] for s in meta['slices']]).reshape(meta['OriginShape'])
            removes += meta['slices']
        for s in removes:
            obj.pop(s)
        obj.pop(UNPACK_INFO)
    return obj


def save(obj, path, protocol=4, **configs):
    if isinstance(path, (str, os.PathLike)):
        d = os.path.dirname(os.fspath(path))
        if d:
            os.makedirs(d, exist_ok=True)
    if not (1 < protocol < 5):
        raise ValueError(f"Expected 1<'protocol'<5, but received protocol={protocol}")
    if isinstance(obj, dict):
        data = _build_saved_state_dict(obj)
    else:
        data = _nested(obj)
    data = _unpack_saved_dict(data, protocol, configs.get('_max_slice_bytes', _MAX_SLICE_BYTES))
    if hasattr(path, 'write'):
        pickle.dump(data, path, protocol=protocol)
        return
    tmp = os.fspath(path) + '.tmp'
    with open(tmp, 'wb') as f:
        pickle.dump(data, f, protocol=protocol)
    os.replace(tmp, path)  # atomic: a crash mid-save never corrupts the previous checkpoint


class _SafeUnpickler(pickle.Unpickler):
    _ALLOWED = {
        ('numpy.core.multiarray', '_reconstruct'), ('numpy._core.multiarray', '_reconstruct'),
        ('numpy', 'ndarray'), ('numpy', 'dtype'), ('numpy.core.multiarray', 'scalar'),
        ('numpy._core.multiarray', 'scalar'), ('collections', 'OrderedDict'),
        ('builtins', 'set'), ('builtins', 'frozenset'), ('builtins', 'complex'),
        ('builtins', 'slice'), ('builtins', 'range'), ('builtins', 'tuple'),
        ('__builtin__', 'tuple'), ('__builtin__', 'set'),
        ('_codecs', 'encode'),  # protocol-2 pickles carry ndarray bytes as latin-1 strings
    }

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            import importlib
            return getattr(importlib.import_module(module.replace('__builtin__', 'builtins')), name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from checkpoint")


def _to_tensor(arr, name=None):
    if arr.dtype == np.uint16:  # Paddle's numpy form of bfloat16
        t = torch.from_numpy(arr.view(np.int16).copy()).view(torch.bfloat16)
    else:
        t = torch.from_numpy(np.ascontiguousarray(arr))
    out = Tensor(t)
    if name is not None:
        out.name = name
    return out


def _is_named_tensor(obj):
    return isinstance(obj, tuple) and len(obj) == 2 and isinstance(obj[1], np.ndarray) and \
        (obj[0] is None or isinstance(obj[0], str))


def _parse(obj, return_numpy):
    if isinstance(obj, dict):
        if _LEGACY_BF16_TAG in obj:  # round-1 files of this framework
            arr = obj[_LEGACY_BF16_TAG]
            return arr if return_numpy else _to_tensor(arr, obj.get('name'))
        res = type(obj)() if isinstance(obj, collections.OrderedDict) else {}
        if NAME_TABLE in obj:
            obj = _parse_state_dict(obj, return_numpy, keep_name_table=True)
        for k, v in obj.items():
            res[k] = _parse(v, return_numpy) if not isinstance(v, Tensor) else v
        return res
    if _is_named_tensor(obj):
        return obj[1] if return_numpy else _to_tensor(obj[1], obj[0])
    if isinstance(obj, np.ndarray):
        return obj if return_numpy else _to_tensor(obj)
    if isinstance(obj, list):
        return [_parse(v, return_numpy) for v in obj]
    if isinstance(obj, tuple):
        return tuple(_parse(v, return_numpy) for v in obj)
    return obj


def _parse_state_dict(obj, return_numpy, keep_name_table):
    obj = _pack_loaded_dict(obj)
    table = obj.get(NAME_TABLE, {})
    for k, name in table.items():
        v = obj.get(k)
        if isinstance(v, np.ndarray):
            obj[k] = v if return_numpy else _to_tensor(v, name)
    if not keep_name_table:
        obj.pop(NAME_TABLE, None)
    return obj


def load(path, **configs):
    return_numpy = configs.get('return_numpy', False)
    keep = configs.get('keep_name_table', False)
    if hasattr(path, 'read'):
        data = _SafeUnpickler(path, encoding='latin1').load()
    else:
        with open(path, 'rb') as f:
            data = _SafeUnpickler(f, encoding='latin1').load()
    if isinstance(data, dict):
        data = _pack_loaded_dict(data)
        if NAME_TABLE in data:
            data = _parse_state_dict(data, return_numpy, keep)
    return _parse(data, return_numpy)
