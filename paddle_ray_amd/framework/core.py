"""Tensor core: dtypes, places, device selection and the eager ``Tensor``.

Parity: ``python/paddle/fluid/dygraph/varbase_patch_methods.py`` (Tensor methods),
``python/paddle/framework/dtype.py`` (dtypes), ``python/paddle/device/__init__.py``
(set_device/get_device) and ``paddle/fluid/pybind/eager.cc`` (Tensor object).

Design (MI355X-first): a ``Tensor`` is a thin Python handle over a PyTorch-ROCm
``torch.Tensor`` (HBM storage + caching allocator + autograd tape). Swapping the
handle's storage (``_t``) is O(1), which sharding stage-3 and static-graph
replay rely on. Paddle semantics (``stop_gradient``, list ``shape``, ``place``)
live here; all math dispatches through ``paddle_ray_amd.ops`` to HIP kernels or
library calls.
"""
from __future__ import annotations

import numbers
import threading

import numpy as np
import torch

# ----------------------------------------------------------------------------
# dtypes: paddle dtype objects ARE torch dtypes (cheap equality, no mapping).
# ----------------------------------------------------------------------------
bool_ = torch.bool
uint8 = torch.uint8
int8 = torch.int8
int16 = torch.int16
int32 = torch.int32
int64 = torch.int64
float16 = torch.float16
bfloat16 = torch.bfloat16
float32 = torch.float32
float64 = torch.float64
complex64 = torch.complex64
complex128 = torch.complex128

_STR2DT = {
    'bool': torch.bool, 'uint8': torch.uint8, 'int8': torch.int8, 'int16': torch.int16,
    'int32': torch.int32, 'int64': torch.int64, 'float16': torch.float16, 'fp16': torch.float16,
    'half': torch.float16, 'bfloat16': torch.bfloat16, 'bf16': torch.bfloat16,
    'float32': torch.float32, 'fp32': torch.float32, 'float': torch.float32,
    'float64': torch.float64, 'fp64': torch.float64, 'double': torch.float64,
    'complex64': torch.complex64, 'complex128': torch.complex128, 'uint16': torch.bfloat16,
    'int': torch.int64, 'long': torch.int64,
}
_DT2STR = {v: k for k, v in _STR2DT.items() if k in (
    'bool', 'uint8', 'int8', 'int16', 'int32', 'int64', 'float16', 'bfloat16', 'float32',
    'float64', 'complex64', 'complex128')}
_NP2DT = {
    np.dtype('bool'): torch.bool, np.dtype('uint8'): torch.uint8, np.dtype('int8'): torch.int8,
    np.dtype('int16'): torch.int16, np.dtype('int32'): torch.int32, np.dtype('int64'): torch.int64,
    np.dtype('float16'): torch.float16, np.dtype('float32'): torch.float32,
    np.dtype('float64'): torch.float64, np.dtype('complex64'): torch.complex64,
    np.dtype('complex128'): torch.complex128,
}


def convert_dtype(dtype):
    """Any dtype spelling (str / numpy / torch / paddle) -> torch dtype."""
    if dtype is None:
        return None
    if isinstance(dtype, torch.dtype):
        return dtype
    if isinstance(dtype, str):
        d = _STR2DT.get(dtype.lower().replace('paddle.', ''))
        if d is None:
            raise TypeError(f"unsupported dtype {dtype!r}")
        return d
    if dtype is bool:
        return torch.bool
    if dtype is int:
        return torch.int64
    if dtype is float:
        return get_default_dtype()
    try:
        return _NP2DT[np.dtype(dtype)]
    except Exception:
        raise TypeError(f"unsupported dtype {dtype!r}")


def dtype_to_str(dtype):
    return _DT2STR.get(convert_dtype(dtype), str(dtype))


def is_floating_dtype(dt):
    return dt in (torch.float16, torch.bfloat16, torch.float32, torch.float64)


_default_dtype = torch.float32


def set_default_dtype(d):
    global _default_dtype
    d = convert_dtype(d)
    if d not in (torch.float16, torch.bfloat16, torch.float32, torch.float64):
        raise TypeError("default dtype must be a floating type")
    _default_dtype = d


def get_default_dtype():
    return _default_dtype


class iinfo:
    def __init__(self, dtype):
        i = torch.iinfo(convert_dtype(dtype))
        self.min, self.max, self.bits, self.dtype = i.min, i.max, i.bits, dtype_to_str(dtype)


class finfo:
    def __init__(self, dtype):
        i = torch.finfo(convert_dtype(dtype))
        self.min, self.max, self.eps, self.tiny = i.min, i.max, i.eps, i.tiny
        self.smallest_normal, self.resolution, self.bits = i.smallest_normal, i.resolution, i.bits
        self.dtype = dtype_to_str(dtype)


# ----------------------------------------------------------------------------
# places / devices
# ----------------------------------------------------------------------------
class Place:
    __slots__ = ('_dev',)

    def __init__(self, dev):
        self._dev = torch.device(dev)

    def is_gpu_place(self):
        return self._dev.type == 'cuda'

    def is_cpu_place(self):
        return self._dev.type == 'cpu'

    def gpu_device_id(self):
        return self._dev.index or 0

    def get_device_id(self):
        return self._dev.index or 0

    def __eq__(self, o):
        return isinstance(o, Place) and o._dev == self._dev

    def __hash__(self):
        return hash(self._dev)

    def __repr__(self):
        if self._dev.type == 'cpu':
            return 'Place(cpu)'
        return f'Place(gpu:{self._dev.index or 0})'


def CPUPlace():
    return Place('cpu')


def CUDAPlace(i=0):
    return Place(f'cuda:{int(i)}')


def CUDAPinnedPlace():
    return Place('cpu')


def _foreign_place(kind):
    def make(i=0):  # no such device on an MI355X build; kept for API surface
        raise RuntimeError(f"{kind} is not available in the MI355X build (devices: CPUPlace, CUDAPlace = HIP)")
    make.__name__ = kind
    return make


XPUPlace = _foreign_place('XPUPlace')
IPUPlace = _foreign_place('IPUPlace')
MLUPlace = _foreign_place('MLUPlace')


NPUPlace = XPUPlace


_dev_state = threading.local()
_global_device = None


def _gpu_available():
    return torch.cuda.is_available()


def _default_device():
    global _global_device
    if _global_device is None:
        _global_device = torch.device('cuda', 0) if _gpu_available() else torch.device('cpu')
    return _global_device


def set_device(device):
    """paddle.set_device('gpu'|'gpu:N'|'cpu') — 'gpu' means the HIP device."""
    global _global_device
    if isinstance(device, Place):
        _global_device = device._dev
    else:
        s = str(device).lower()
        if s.startswith('gpu') or s.startswith('cuda') or s.startswith('hip'):
            idx = int(s.split(':')[1]) if ':' in s else 0
            if not _gpu_available():
                raise ValueError("no HIP device available")
            _global_device = torch.device('cuda', idx)
            torch.cuda.set_device(idx)
        elif s.startswith('cpu'):
            _global_device = torch.device('cpu')
        else:
            raise ValueError(f"unknown device {device!r}")
    return Place(_global_device)


def get_device():
    d = _default_device()
    return 'cpu' if d.type == 'cpu' else f'gpu:{d.index or 0}'


def _get_place():
    return Place(_default_device())


def _to_torch_device(place):
    if place is None:
        return _default_device()
    if isinstance(place, Place):
        return place._dev
    if isinstance(place, torch.device):
        return place
    s = str(place).lower()
    if s.startswith('gpu'):
        s = 'cuda' + s[3:]
    return torch.device(s)


def is_compiled_with_cuda():
    # HIP device visible through the torch "cuda" namespace on ROCm.
    return torch.cuda.is_available()


def is_compiled_with_rocm():
    return torch.version.hip is not None


def is_compiled_with_xpu():
    return False


# ----------------------------------------------------------------------------
# grad mode
# ----------------------------------------------------------------------------
class no_grad:
    """Context manager / decorator disabling the tape (paddle.no_grad)."""

    def __enter__(self):
        self._prev = torch.is_grad_enabled()
        torch.set_grad_enabled(False)

    def __exit__(self, *a):
        torch.set_grad_enabled(self._prev)

    def __call__(self, fn):
        def wrapper(*a, **k):
            with no_grad():
                return fn(*a, **k)
        wrapper.__name__ = getattr(fn, '__name__', 'wrapped')
        wrapper.__doc__ = getattr(fn, '__doc__', None)
        return wrapper


class enable_grad(no_grad):
    def __enter__(self):
        self._prev = torch.is_grad_enabled()
        torch.set_grad_enabled(True)

    def __call__(self, fn):
        def wrapper(*a, **k):
            with enable_grad():
                return fn(*a, **k)
        return wrapper


class set_grad_enabled:
    def __init__(self, mode):
        self._prev = torch.is_grad_enabled()
        torch.set_grad_enabled(bool(mode))
        self.mode = mode

    def __enter__(self):
        return self

    def __exit__(self, *a):
        torch.set_grad_enabled(self._prev)


def is_grad_enabled():
    return torch.is_grad_enabled()


# ----------------------------------------------------------------------------
# Tensor
# ----------------------------------------------------------------------------
# per-prefix counters, like the reference's paddle.utils.unique_name (``linear_0.w_0``);
# ``paddle.utils.unique_name.guard()`` swaps in a fresh table
_NAME_COUNTERS = [__import__('collections').defaultdict(int)]


def _unique_name(prefix='generated_tensor'):
    c = _NAME_COUNTERS[0]
    n = c[prefix]
    c[prefix] += 1
    return f'{prefix}_{n}'


class Tensor:
    """Eager tensor handle (parity: paddle.Tensor / core.eager.Tensor).

    ``_t`` is the backing torch.Tensor. ``stop_gradient`` maps to
    ``not requires_grad``; setting it True on a non-leaf detaches the handle,
    which is exactly Paddle's "stop the gradient here" semantics.
    """
    __slots__ = ('_t', '_name', 'persistable', '__weakref__', '__dict__')
    __array_priority__ = 100

    def __init__(self, data=None, dtype=None, place=None, stop_gradient=True, name=None):
        if data is None:
            t = torch.empty(0)
        elif isinstance(data, torch.Tensor):
            t = data
        elif isinstance(data, Tensor):
            t = data._t
        else:
            t = _as_torch(data, dtype, place)
        if dtype is not None and t.dtype != convert_dtype(dtype):
            t = t.to(convert_dtype(dtype))
        object.__setattr__(self, '_t', t)
        self._name = name
        self.persistable = False
        if not stop_gradient and t.is_floating_point() and not t.requires_grad:
            t.requires_grad_(True)

    # -- identity ------------------------------------------------------------
    @property
    def name(self):
        if self._name is None:
            self._name = _unique_name()
        return self._name

    @name.setter
    def name(self, v):
        self._name = v

    def __hash__(self):
        return id(self)

    # -- meta ----------------------------------------------------------------
    @property
    def shape(self):
        return list(self._t.shape)

    @property
    def ndim(self):
        return self._t.dim()

    def dim(self):
        return self._t.dim()

    def ndimension(self):
        return self._t.dim()

    @property
    def size(self):
        return self._t.numel()

    def numel(self):
        return Tensor(torch.tensor(self._t.numel(), dtype=torch.int64))

    @property
    def dtype(self):
        return self._t.dtype

    @property
    def place(self):
        return Place(self._t.device)

    @property
    def is_leaf(self):
        return self._t.is_leaf

    @property
    def T(self):
        t = self._t
        return Tensor(t.permute(*reversed(range(t.dim()))))

    @property
    def mT(self):
        return Tensor(self._t.transpose(-1, -2))

    @property
    def stop_gradient(self):
        return not self._t.requires_grad

    @stop_gradient.setter
    def stop_gradient(self, v):
        t = self._t
        if v:
            if t.requires_grad:
                if t.is_leaf:
                    t.requires_grad_(False)
                else:
                    object.__setattr__(self, '_t', t.detach())
        else:
            if not t.requires_grad:
                if t.is_leaf:
                    t.requires_grad_(True)
                else:  # non-leaf without history: becomes a new leaf
                    object.__setattr__(self, '_t', t.detach().requires_grad_(True))

    # -- autograd --------------------------------------------------------------
    @property
    def grad(self):
        g = self._t.grad
        return None if g is None else Tensor(g)

    @grad.setter
    def grad(self, v):
        self._t.grad = None if v is None else _u(v)

    def gradient(self):
        g = self._t.grad
        return None if g is None else g.detach().cpu().float().numpy() if g.dtype == torch.bfloat16 \
            else g.detach().cpu().numpy()

    def backward(self, grad_tensor=None, retain_graph=False):
        g = None if grad_tensor is None else _u(grad_tensor)
        if g is None and self._t.numel() != 1:
            g = torch.ones_like(self._t)
        from ..profiler import _hooks
        if _hooks.ACTIVE:
            from ..profiler import RecordEvent, TracerEventType
            with RecordEvent('backward', TracerEventType.Backward):
                self._t.backward(g, retain_graph=retain_graph)
            return
        self._t.backward(g, retain_graph=retain_graph)

    def clear_gradient(self, set_to_zero=True):
        g = self._t.grad
        if g is not None:
            if set_to_zero:
                g.zero_()
            else:
                self._t.grad = None

    clear_grad = clear_gradient

    def detach(self):
        return Tensor(self._t.detach())

    def detach_(self):
        object.__setattr__(self, '_t', self._t.detach())
        return self

    def register_hook(self, hook):
        def _h(g):
            r = hook(Tensor(g))
            return None if r is None else _u(r)
        h = self._t.register_hook(_h)
        return h

    def retain_grads(self):
        self._t.retain_grad()

    # -- conversion --------------------------------------------------------------
    def numpy(self):
        t = self._t.detach()
        if t.dtype == torch.bfloat16:
            t = t.float()
        return t.cpu().numpy()

    def __array__(self, dtype=None, copy=None):
        a = self.numpy()
        return a.astype(dtype) if dtype is not None else a

    def tolist(self):
        return self._t.tolist()

    def item(self, *args):
        if args:
            return self._t[args].item() if len(args) > 1 else self._t.flatten()[args[0]].item()
        return self._t.item()

    def __float__(self):
        return float(self._t.item())

    def __int__(self):
        return int(self._t.item())

    def __index__(self):
        return int(self._t.item())

    def __bool__(self):
        return bool(self._t.item()) if self._t.numel() == 1 else bool(self._t.numel())

    def __len__(self):
        return self._t.shape[0] if self._t.dim() else 0

    def __iter__(self):
        for i in range(len(self)):
            yield Tensor(self._t[i])

    def astype(self, dtype):
        return Tensor(self._t.to(convert_dtype(dtype)))

    cast = astype

    def cpu(self):
        return Tensor(self._t.cpu())

    def cuda(self, device_id=None, blocking=True):
        return Tensor(self._t.cuda(device_id))

    def pin_memory(self):
        return Tensor(self._t.pin_memory()) if torch.cuda.is_available() else self

    def to(self, *args, **kwargs):
        dev, dt = None, kwargs.get('dtype')
        if 'device' in kwargs:
            dev = _to_torch_device(kwargs['device'])
        for a in args:
            if isinstance(a, (str, Place, torch.device)) and not (isinstance(a, str) and a in _STR2DT):
                dev = _to_torch_device(a)
            else:
                dt = a
        t = self._t
        if dev is not None:
            t = t.to(dev)
        if dt is not None:
            t = t.to(convert_dtype(dt))
        return Tensor(t)

    def clone(self):
        return Tensor(self._t.clone())

    def value(self):
        return self

    def get_tensor(self):
        return self

    # --- LoD (level-of-detail) sequence info, as on the reference's LoDTensor
    # (paddle/fluid/framework/lod_tensor.h): offset lists per level, host-side metadata -----
    def set_lod(self, lod):
        lod = [[int(v) for v in level] for level in lod]
        for level in lod:
            if not level or level[0] != 0 or any(b < a for a, b in zip(level, level[1:])):
                raise ValueError(f"invalid LoD level {level}: offsets must start at 0 and not decrease")
        if lod and lod[-1][-1] != (self._t.shape[0] if self._t.dim() else 1):
            raise ValueError(f"LoD {lod} does not cover the tensor's first dimension {tuple(self._t.shape)}")
        self.__dict__['_lod'] = lod

    def lod(self):
        return [list(level) for level in self.__dict__.get('_lod', [])]

    def set_recursive_sequence_lengths(self, lengths):
        lod = []
        for level in lengths:
            off = [0]
            for n in level:
                off.append(off[-1] + int(n))
            lod.append(off)
        self.set_lod(lod)

    def recursive_sequence_lengths(self):
        return [[b - a for a, b in zip(level, level[1:])] for level in self.lod()]

    def has_valid_recursive_sequence_lengths(self):
        lod = self.__dict__.get('_lod')
        if not lod:
            return True
        for upper, lower in zip(lod, lod[1:]):
            if upper[-1] != len(lower) - 1:
                return False
        return lod[-1][-1] == self._t.shape[0]

    def set_value(self, value):
        v = value._t if isinstance(value, Tensor) else torch.as_tensor(np.asarray(value))
        with torch.no_grad():
            self._t.copy_(v.to(self._t.dtype).reshape(self._t.shape))

    def copy_(self, src, blocking=True):
        with torch.no_grad():
            self._t.copy_(_u(src))
        return self

    def _share_buffer_to(self, other):
        object.__setattr__(other, '_t', self._t)

    def data_ptr(self):
        return self._t.data_ptr()

    def is_contiguous(self):
        return self._t.is_contiguous()

    def contiguous(self):
        return Tensor(self._t.contiguous())

    def element_size(self):
        return self._t.element_size()

    @property
    def data(self):
        return Tensor(self._t.detach())

    @data.setter
    def data(self, v):
        self._t.data = _u(v)

    def is_dense(self):
        return self._t.layout == torch.strided

    def is_sparse(self):
        return self._t.layout in (torch.sparse_coo, torch.sparse_csr)

    # -- sparse tensor surface (parity: SparseCooTensor / SparseCsrTensor methods) ---------------
    def is_sparse_coo(self):
        return self._t.layout == torch.sparse_coo

    def is_sparse_csr(self):
        return self._t.layout == torch.sparse_csr

    def indices(self):
        t = self._t.coalesce() if self._t.layout == torch.sparse_coo else self._t.to_sparse_coo().coalesce()
        return Tensor(t.indices())

    def values(self):
        t = self._t
        if t.layout == torch.sparse_coo:
            return Tensor(t.coalesce().values())
        return Tensor(t.values())

    def crows(self):
        return Tensor(self._t.crow_indices())

    def cols(self):
        return Tensor(self._t.col_indices())

    def nnz(self):
        t = self._t
        return int(t.coalesce()._nnz() if t.layout == torch.sparse_coo else t._nnz())

    def to_dense(self):
        return Tensor(self._t.to_dense() if self.is_sparse() else self._t)

    def to_sparse_coo(self, sparse_dim=None):
        t = self._t
        if t.layout == torch.sparse_csr:
            return Tensor(t.to_sparse_coo().coalesce())
        if t.layout == torch.sparse_coo:
            return Tensor(t)
        return Tensor(t.to_sparse(sparse_dim if sparse_dim is not None else t.dim()).coalesce())

    def to_sparse_csr(self):
        t = self._t
        if t.layout == torch.sparse_csr:
            return Tensor(t)
        return Tensor(t.to_dense().to_sparse_csr() if t.dim() > 2 and t.layout == torch.sparse_coo
                      else t.to_sparse_csr())

    def _is_initialized(self):
        return True

    def __repr__(self):
        t = self._t
        body = np.array2string(self.numpy(), separator=', ', prefix='       ')
        return (f"Tensor(shape={list(t.shape)}, dtype={dtype_to_str(t.dtype)}, place={self.place}, "
                f"stop_gradient={self.stop_gradient},\n       {body})")

    __str__ = __repr__

    def __deepcopy__(self, memo):
        n = type(self).__new__(type(self))
        object.__setattr__(n, '_t', self._t.detach().clone().requires_grad_(self._t.requires_grad))
        n._name = self._name
        n.persistable = self.persistable
        for k, v in self.__dict__.items():
            n.__dict__[k] = v
        return n

    # -- indexing --------------------------------------------------------------
    def __getitem__(self, idx):
        return Tensor(self._t[_index(idx)])

    def __setitem__(self, idx, value):
        v = _u(value)
        t = self._t
        if isinstance(v, torch.Tensor) and v.dtype != t.dtype:
            v = v.to(t.dtype)
        if t.requires_grad and t.is_leaf:
            with torch.no_grad():
                t[_index(idx)] = v
        else:
            t[_index(idx)] = v


class Parameter(Tensor):
    """Trainable parameter (parity: paddle.fluid.framework.EagerParamBase)."""

    def __init__(self, data, trainable=True, name=None, **kwargs):
        super().__init__(data, stop_gradient=not trainable, name=name)
        self.persistable = True
        self.trainable = trainable
        self.optimize_attr = kwargs.get('optimize_attr', {'learning_rate': 1.0})
        self.regularizer = kwargs.get('regularizer', None)
        self.need_clip = kwargs.get('need_clip', True)
        self.is_distributed = kwargs.get('is_distributed', False)
        self.do_model_average = kwargs.get('do_model_average', None)

    @property
    def trainable(self):
        return self.__dict__.get('_trainable', True)

    @trainable.setter
    def trainable(self, v):
        self.__dict__['_trainable'] = bool(v)
        self.stop_gradient = not v

    def __repr__(self):
        return 'Parameter containing:\n' + super().__repr__()


EagerParamBase = Parameter


# ----------------------------------------------------------------------------
# wrap / unwrap helpers
# ----------------------------------------------------------------------------
def _u(x):
    """Unwrap Tensor -> torch.Tensor (recursively for lists/tuples)."""
    if isinstance(x, Tensor):
        return x._t
    if isinstance(x, (list, tuple)):
        if x and any(isinstance(e, Tensor) for e in x):
            return type(x)(_u(e) for e in x)
    return x


def _w(t):
    """Wrap torch.Tensor -> Tensor (recursively)."""
    if isinstance(t, torch.Tensor):
        return Tensor(t)
    if isinstance(t, (list, tuple)):
        return type(t)(_w(e) for e in t)
    return t


def _index(idx):
    if isinstance(idx, Tensor):
        t = idx._t
        return t
    if isinstance(idx, tuple):
        return tuple(_index(i) for i in idx)
    if isinstance(idx, list):
        if any(isinstance(i, Tensor) for i in idx):
            return [_index(i) for i in idx]
        return idx
    return idx


def _as_torch(data, dtype=None, place=None):
    dev = _to_torch_device(place)
    dt = convert_dtype(dtype)
    if isinstance(data, Tensor):
        t = data._t
    elif isinstance(data, torch.Tensor):
        t = data
    elif isinstance(data, np.ndarray):
        if data.dtype == np.float64 and dt is None:
            t = torch.from_numpy(np.ascontiguousarray(data))
        elif data.dtype.kind in 'fciub':
            t = torch.from_numpy(np.ascontiguousarray(data))
        else:
            t = torch.as_tensor(data.astype(np.float32))
    elif isinstance(data, (bool, np.bool_)):
        t = torch.tensor(bool(data))
    elif isinstance(data, numbers.Integral):
        t = torch.tensor(int(data), dtype=torch.int64)
    elif isinstance(data, numbers.Real):
        t = torch.tensor(float(data), dtype=get_default_dtype())
    elif isinstance(data, numbers.Complex):
        t = torch.tensor(complex(data))
    elif isinstance(data, (list, tuple)):
        if any(isinstance(e, Tensor) for e in _flatten_list(data)):
            t = torch.stack([_as_torch(e, dtype, place) for e in data])
        else:
            a = np.array(data)
            if a.dtype == np.float64:
                a = a.astype(np.dtype(str(get_default_dtype()).split('.')[-1])
                             if get_default_dtype() != torch.bfloat16 else np.float32)
            t = torch.from_numpy(a)
    else:
        t = torch.as_tensor(data)
    if dt is not None and t.dtype != dt:
        t = t.to(dt)
    if t.device != dev:
        t = t.to(dev)
    return t


def _flatten_list(x):
    for e in x:
        if isinstance(e, (list, tuple)):
            yield from _flatten_list(e)
        else:
            yield e


def to_tensor(data, dtype=None, place=None, stop_gradient=True):
    """paddle.to_tensor (parity: python/paddle/tensor/creation.py:to_tensor)."""
    if isinstance(data, Tensor):
        t = data._t.detach().clone()
        if dtype is not None:
            t = t.to(convert_dtype(dtype))
        if place is not None:
            t = t.to(_to_torch_device(place))
    else:
        t = _as_torch(data, dtype, place)
        if isinstance(data, torch.Tensor):
            t = t.detach().clone() if t is data else t
    out = Tensor(t)
    if not stop_gradient:
        out.stop_gradient = False
    return out


def is_tensor(x):
    return isinstance(x, Tensor)


_in_dynamic = [True]


def in_dynamic_mode():
    return _in_dynamic[0]


in_dygraph_mode = in_dynamic_mode
