"""paddle.utils.cpp_extension for MI355X (parity: python/paddle/utils/cpp_extension/
cpp_extension.py ``setup`` :79, ``CppExtension`` :239, ``CUDAExtension`` :289, ``load`` :800,
and the custom-op registration of paddle/extension.h / PD_BUILD_OP).

A custom operator is C++ (host) or HIP (gfx950 device) source written against the small C ABI
in ``include/pra_extension.h`` — tensors arrive as ``PraTensor`` views, the caller's HIP
stream as ``void*`` — and registered with ``PRA_REGISTER_OP(name, n_in, n_out, forward,
infer, backward)``. ``load()`` compiles it in-process-free fashion (g++ for ``.cc/.cpp``,
``hipcc --offload-arch=gfx950`` for ``.hip``; content-hashed, so an unchanged extension is
not rebuilt), loads the library with ctypes and returns a module whose attributes are the
ops: each call allocates its outputs from ``infer``, runs ``forward`` on the current HIP
stream, and records an autograd node whose backward runs the op's ``backward`` kernel. Every
op is also entered into the kernel registry as ``custom.<name>`` (backend 'hip' for device
builds, 'ref' for host builds), so a host and a HIP build of the same op dispatch by tensor
placement like the built-in kernels.

No hipify and no CUDA headers: the ABI is framework-independent C, compiled for gfx950 only.
"""
import ctypes
import hashlib
import json
import os
import subprocess
import sys
import types

import torch

INCLUDE_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'include')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = os.environ.get('PRA_ARCH', 'gfx950')
MAX_DIMS = 8

_DT = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2, torch.float64: 3, torch.int32: 4,
       torch.int64: 5, torch.uint8: 6, torch.bool: 7}
_DT_INV = {v: k for k, v in _DT.items()}


class PraTensor(ctypes.Structure):
    _fields_ = [('data', ctypes.c_void_p), ('numel', ctypes.c_int64), ('ndim', ctypes.c_int32),
                ('dtype', ctypes.c_int32), ('shape', ctypes.c_int64 * MAX_DIMS)]


_OpFn = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.POINTER(PraTensor), ctypes.c_int,
                         ctypes.POINTER(PraTensor), ctypes.c_int, ctypes.c_void_p)
_InferFn = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.POINTER(PraTensor), ctypes.c_int,
                            ctypes.POINTER(PraTensor), ctypes.c_int)


class PraOpDef(ctypes.Structure):
    _fields_ = [('name', ctypes.c_char_p), ('n_in', ctypes.c_int), ('n_out', ctypes.c_int),
                ('forward', ctypes.c_void_p), ('infer', ctypes.c_void_p),
                ('backward', ctypes.c_void_p)]


def get_build_directory(verbose=False):
    d = os.environ.get('PADDLE_EXTENSION_DIR') or os.path.join(
        os.path.expanduser('~'), '.cache', 'paddle_ray_amd_extensions')
    os.makedirs(d, exist_ok=True)
    return d


# -- build ---------------------------------------------------------------------------------------
def _is_device(src):
    return src.endswith(('.hip', '.cu'))


def _compile_cmds(name, sources, build_dir, cflags, hipflags, ldflags, include_paths):
    incs = sum((['-I', p] for p in [INCLUDE_DIR] + list(include_paths or [])), [])
    objs, cmds = [], []
    device = any(_is_device(s) for s in sources)
    for s in sources:
        base = os.path.splitext(os.path.basename(s))[0]
        obj = os.path.join(build_dir, f'{base}.{"hip" if _is_device(s) else "cc"}.o')
        if _is_device(s):
            cmd = [HIPCC, f'--offload-arch={ARCH}', '-O3', '-fPIC', '-std=c++17', '-x', 'hip', '-c', s,
                   '-o', obj] + incs + list(hipflags or [])
        else:
            cmd = ['g++', '-O2', '-fPIC', '-std=c++17', '-c', s, '-o', obj] + incs + list(cflags or [])
        objs.append(obj)
        cmds.append(cmd)
    so = os.path.join(build_dir, f'{name}.so')
    link = ([HIPCC, '-shared', '-fPIC', f'--offload-arch={ARCH}'] if device else
            ['g++', '-shared', '-fPIC']) + ['-o', so] + objs + list(ldflags or [])
    return cmds, link, so


def _build(name, sources, build_dir, cflags=None, hipflags=None, ldflags=None, include_paths=None,
           verbose=False):
    sources = [os.path.abspath(s) for s in sources]
    os.makedirs(build_dir, exist_ok=True)
    cmds, link, so = _compile_cmds(name, sources, build_dir, cflags, hipflags, ldflags,
                                   include_paths)
    h = hashlib.sha256()
    for s in sources + [os.path.join(INCLUDE_DIR, 'pra_extension.h')]:
        with open(s, 'rb') as f:
            h.update(f.read())
    h.update(json.dumps([cmds, link]).encode())
    key = h.hexdigest()
    stamp = so + '.sha256'
    if os.path.exists(so) and os.path.exists(stamp) and open(stamp).read() == key:
        return so
    for c in cmds + [link]:
        if verbose:
            print(' '.join(c), file=sys.stderr)
        r = subprocess.run(c, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"building custom op '{name}' failed:\n{' '.join(c)}\n{r.stdout}{r.stderr}")
    with open(stamp, 'w') as f:
        f.write(key)
    return so


# -- runtime -------------------------------------------------------------------------------------
def _view(t):
    v = PraTensor()
    if t is None:
        return v
    v.data = t.data_ptr()
    v.numel = t.numel()
    v.ndim = t.dim()
    v.dtype = _DT[t.dtype]
    for i, s in enumerate(t.shape):
        v.shape[i] = s
    return v


def _views(ts):
    arr = (PraTensor * max(1, len(ts)))()
    for i, t in enumerate(ts):
        arr[i] = _view(t)
    return arr


def _stream_ptr(ts):
    for t in ts:
        if t is not None and t.is_cuda:
            return torch.cuda.current_stream(t.device).cuda_stream
    return None


class CustomOp:
    """One registered op of a loaded extension: ``op(*tensors)`` -> output tensor(s)."""

    def __init__(self, lib, d, device_build):
        self.name = d.name.decode()
        self.n_in, self.n_out = d.n_in, d.n_out
        self._lib = lib
        self._fwd = _OpFn(d.forward)
        self._infer = _InferFn(d.infer) if d.infer else None
        self._bwd = _OpFn(d.backward) if d.backward else None
        self.device_build = device_build
        op = self

        class _Fn(torch.autograd.Function):
            @staticmethod
            def forward(ctx, *xs):
                outs = op._run_forward(xs)
                ctx.save_for_backward(*xs, *outs)
                ctx.mark_non_differentiable(*[o for o in outs if not o.is_floating_point()])
                return outs[0] if len(outs) == 1 else tuple(outs)

            @staticmethod
            def backward(ctx, *gouts):
                saved = ctx.saved_tensors
                xs, outs = saved[:op.n_in], saved[op.n_in:]
                return tuple(op._run_backward(xs, outs, gouts))
        self._autograd = _Fn

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"custom op '{self.name}' {what} returned {rc}")

    def _run_forward(self, xs):
        xs = [x.contiguous() for x in xs]
        if len(xs) != self.n_in:
            raise TypeError(f"custom op '{self.name}' takes {self.n_in} inputs, got {len(xs)}")
        ins = _views(xs)
        meta = (PraTensor * self.n_out)()
        if self._infer is not None:
            self._check(self._infer(ins, self.n_in, meta, self.n_out), 'infer')
        else:
            for i in range(self.n_out):
                meta[i] = ins[0]
        outs = []
        for m in meta:
            shape = [m.shape[i] for i in range(m.ndim)]
            outs.append(torch.empty(shape, dtype=_DT_INV[m.dtype], device=xs[0].device))
        if xs[0].is_cuda and not self.device_build:
            raise RuntimeError(f"custom op '{self.name}' was built for the host; its inputs are "
                               "on the GPU (build it from a .hip source)")
        st = _stream_ptr(xs)
        self._check(self._fwd(ins, self.n_in, _views(outs), self.n_out, st), 'forward')
        return outs

    def _run_backward(self, xs, outs, gouts):
        if self._bwd is None:
            raise RuntimeError(f"custom op '{self.name}' has no backward kernel")
        gouts = [torch.zeros_like(o) if g is None else g.contiguous() for o, g in zip(outs, gouts)]
        gins = [torch.empty_like(x) if x.is_floating_point() else None for x in xs]
        ins = list(xs) + list(outs) + gouts
        res = _views([g if g is not None else torch.empty(0) for g in gins])
        for i, g in enumerate(gins):
            if g is None:
                res[i].data = None
        self._check(self._bwd(_views(ins), len(ins), res, len(gins), _stream_ptr(ins)), 'backward')
        return gins

    def __call__(self, *xs):
        from ...framework.core import Tensor, _u
        ts = [_u(x) if isinstance(x, Tensor) else x for x in xs]
        out = self._autograd.apply(*ts)
        if isinstance(out, tuple):
            return tuple(Tensor(o) for o in out)
        return Tensor(out)


def _register(op):
    from ...ops import registry as R
    backend = 'hip' if op.device_build else 'ref'

    def kern(*xs):
        return op(*xs)
    R.register_kernel(f'custom.{op.name}', backend)(kern)


def _dispatcher(name):
    """``module.<op>``: routes through the kernel registry (host / HIP build by placement)."""
    from ...framework.core import Tensor, _u
    from ...ops import registry as R

    def call(*xs):
        t = _u(xs[0]) if isinstance(xs[0], Tensor) else xs[0]
        return R.dispatch(f'custom.{name}', t, *xs)
    call.__name__ = name
    return call


def _load_library(name, so, device_build):
    lib = ctypes.CDLL(so)
    lib.pra_ext_num_ops.restype = ctypes.c_int
    lib.pra_ext_op.restype = ctypes.POINTER(PraOpDef)
    lib.pra_ext_op.argtypes = [ctypes.c_int]
    mod = types.ModuleType(name)
    mod.__file__ = so
    mod._ops = {}
    for i in range(lib.pra_ext_num_ops()):
        op = CustomOp(lib, lib.pra_ext_op(i).contents, device_build)
        mod._ops[op.name] = op
        _register(op)
        setattr(mod, op.name, _dispatcher(op.name))
    mod._lib = lib
    return mod


def load(name, sources, extra_cxx_cflags=None, extra_cuda_cflags=None, extra_ldflags=None,
         extra_include_paths=None, build_directory=None, interpreter=None, verbose=False,
         extra_hip_cflags=None):
    """Compile ``sources`` into a custom-op library and return its module (JIT mode).
    ``extra_cuda_cflags`` is accepted for signature compatibility and passed to hipcc."""
    bdir = os.path.join(build_directory or get_build_directory(), name)
    hipflags = list(extra_hip_cflags or []) + list(extra_cuda_cflags or [])
    so = _build(name, sources, bdir, extra_cxx_cflags, hipflags, extra_ldflags,
                extra_include_paths, verbose)
    return _load_library(name, so, any(_is_device(s) for s in sources))


class _Extension:
    def __init__(self, sources, *args, include_dirs=None, extra_compile_args=None, **kwargs):
        self.sources = list(sources)
        self.include_dirs = list(include_dirs or [])
        eca = extra_compile_args or {}
        if isinstance(eca, dict):
            self.cxx_flags = list(eca.get('cxx', []))
            self.hip_flags = list(eca.get('hipcc', [])) + list(eca.get('nvcc', []))
        else:
            self.cxx_flags, self.hip_flags = list(eca), []
        self.name = kwargs.get('name')


def CppExtension(sources, *args, **kwargs):
    """A host (g++) custom-op extension."""
    return _Extension(sources, *args, **kwargs)


def CUDAExtension(sources, *args, **kwargs):
    """A device extension: ``.hip`` sources compiled by hipcc for gfx950 (the reference's
    CUDAExtension role; CUDA sources are not translated)."""
    return _Extension(sources, *args, **kwargs)


HIPExtension = CUDAExtension


class BuildExtension:
    @classmethod
    def with_options(cls, **options):
        return cls


def setup(**attr):
    """Build the extension(s) ahead of time into ``build_directory`` (default ``./build``) and
    write an importable loader module ``<name>.py`` next to it, so ``import <name>`` returns
    the ops (the reference's ``setup`` + install, without touching site-packages)."""
    name = attr['name']
    exts = attr.get('ext_modules')
    exts = exts if isinstance(exts, (list, tuple)) else [exts]
    out_dir = attr.get('build_directory') or os.path.join(os.getcwd(), 'build')
    sos = []
    for i, e in enumerate(exts):
        en = e.name or (name if len(exts) == 1 else f'{name}_{i}')
        so = _build(en, e.sources, os.path.join(out_dir, en), e.cxx_flags, e.hip_flags, None,
                    e.include_dirs, attr.get('verbose', False))
        sos.append((en, so, any(_is_device(s) for s in e.sources)))
    stub = os.path.join(attr.get('stub_directory') or os.getcwd(), f'{name}.py')
    with open(stub, 'w') as f:
        f.write('"""Generated by paddle_ray_amd.utils.cpp_extension.setup."""\n'
                'from paddle_ray_amd.utils.cpp_extension import _load_library as _ld\n'
                f'_mods = [_ld(n, so, dev) for n, so, dev in {sos!r}]\n'
                'for _m in _mods:\n'
                '    for _k in _m._ops:\n'
                '        globals()[_k] = getattr(_m, _k)\n')
    return [_load_library(en, so, dev) for en, so, dev in sos]
