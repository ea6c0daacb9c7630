"""InputSpec (parity: python/paddle/static/input.py)."""
import numpy as np

from ..framework.core import convert_dtype


class InputSpec:
    def __init__(self, shape, dtype='float32', name=None, stop_gradient=False):
        self.shape = tuple(-1 if s is None else int(s) for s in shape)
        self.dtype = convert_dtype(dtype)
        self.name = name
        self.stop_gradient = stop_gradient

    @classmethod
    def from_tensor(cls, tensor, name=None):
        return cls(tensor.shape, tensor.dtype, name or getattr(tensor, '_name', None))

    @classmethod
    def from_numpy(cls, ndarray, name=None):
        return cls(ndarray.shape, ndarray.dtype, name)

    def batch(self, batch_size):
        self.shape = (batch_size,) + self.shape
        return self

    def unbatch(self):
        self.shape = self.shape[1:]
        return self

    def __repr__(self):
        return f'InputSpec(shape={self.shape}, dtype={self.dtype}, name={self.name})'

    def __eq__(self, o):
        return isinstance(o, InputSpec) and (self.shape, self.dtype, self.name) == (o.shape, o.dtype,
                                                                                   o.name)

    def __hash__(self):
        return hash((self.shape, self.dtype, self.name))
