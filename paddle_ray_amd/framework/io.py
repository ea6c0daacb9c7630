"""paddle.save / paddle.load — ``.pdparams`` / ``.pdopt`` checkpoint format.

Parity: python/paddle/framework/io.py (``_build_saved_state_dict``, ``_pickle_save``,
``_parse_load_result``). The on-disk format matches the reference: a pickle
(protocol 2..4) of nested dicts/lists whose tensors are stored as
``numpy.ndarray`` (bf16 as uint16 bit patterns, like the reference). Loading
uses a RESTRICTED unpickler that only reconstructs numpy arrays/dtypes and
builtin containers — a checkpoint cannot execute code on load.
"""
import collections
import io
import os
import pickle

import numpy as np
import torch

from .core import Tensor, Parameter, _u, to_tensor

_BF16_TAG = '__pra_bf16__'


def _to_saveable(obj):
    if isinstance(obj, Tensor):
        t = obj._t.detach()
        if t.dtype == torch.bfloat16:
            arr = t.cpu().view(torch.int16).numpy().view(np.uint16)
            return {_BF16_TAG: arr, 'name': obj.name}
        return t.cpu().numpy()
    if isinstance(obj, torch.Tensor):
        return _to_saveable(Tensor(obj))
    if isinstance(obj, dict):
        return type(obj)((k, _to_saveable(v)) for k, v in obj.items()) \
            if isinstance(obj, collections.OrderedDict) else {k: _to_saveable(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_saveable(v) for v in obj)
    if hasattr(obj, 'state_dict') and callable(obj.state_dict):
        return _to_saveable(obj.state_dict())
    return obj


def save(obj, path, protocol=4, **configs):
    if isinstance(path, (str, os.PathLike)):
        d = os.path.dirname(os.fspath(path))
        if d:
            os.makedirs(d, exist_ok=True)
    if not (2 <= protocol <= 4):
        raise ValueError("protocol must be in [2, 4]")
    data = _to_saveable(obj)
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
        ('builtins', 'slice'), ('builtins', 'range'),
    }

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            import importlib
            return getattr(importlib.import_module(module), name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from checkpoint")


def _from_saved(obj, return_numpy=False):
    if isinstance(obj, dict):
        if _BF16_TAG in obj:
            arr = obj[_BF16_TAG]
            if return_numpy:
                return arr
            t = torch.from_numpy(arr.view(np.int16).copy()).view(torch.bfloat16)
            out = Tensor(t)
            out.name = obj.get('name')
            return out
        res = type(obj)() if isinstance(obj, collections.OrderedDict) else {}
        for k, v in obj.items():
            res[k] = _from_saved(v, return_numpy)
        return res
    if isinstance(obj, np.ndarray):
        if return_numpy:
            return obj
        return Tensor(torch.from_numpy(np.ascontiguousarray(obj)))
    if isinstance(obj, (list, tuple)):
        return type(obj)(_from_saved(v, return_numpy) for v in obj)
    return obj


def load(path, **configs):
    return_numpy = configs.get('return_numpy', False)
    if hasattr(path, 'read'):
        data = _SafeUnpickler(path).load()
    else:
        with open(path, 'rb') as f:
            data = _SafeUnpickler(f).load()
    return _from_saved(data, return_numpy)
