"""paddle.fft (parity: python/paddle/fft.py; kernels paddle/phi/kernels/gpu/fft_kernel.cu,
fft_grad_kernel.cu over cuFFT plans).

Every public transform reduces to one of three primitive ops, as in the reference:

* ``fft_c2c(x, axes, norm, forward)``                 complex -> complex
* ``fft_r2c(x, axes, norm, forward, onesided)``       real -> complex (half spectrum if onesided)
* ``fft_c2r(x, axes, norm, forward, last_dim_size)``  Hermitian half spectrum -> real

``forward`` picks the exponent sign (e^{-i..} when True); ``norm`` says which direction carries the
1/n ('backward': the inverse, 'forward': the forward, 'ortho': 1/sqrt(n) both ways). The inverse-sign
real transforms (ihfft = r2c with forward=False, hfft = c2r with forward=True) are the conjugate of
the opposite-sign transform with the normalisation direction swapped, so all three primitives run
on the rocFFT plans behind ``torch.fft`` (the library FFT, like the reference's cuFFT) and inherit
their autograd. The primitives are static-graph ops (``fft_c2c`` / ``fft_r2c`` / ``fft_c2r`` OpDescs)
and dispatch through the kernel registry (``stats()`` shows them).

The public layer owns the reference's argument semantics: norm/n/s/axes validation with the same
error conditions, integer inputs promoted to the default dtype, zero-pad / crop of the input to
``n`` / ``s`` BEFORE the transform (for c2r the Hermitian input is resized to n//2+1), the n-D axes
sorted with the last real axis kept last, and fft2-family shape checks.
"""
from collections.abc import Sequence

import torch

from .framework.core import Tensor, _u
from .ops import registry as R
from .static import graph as _G

__all__ = ['fft', 'ifft', 'rfft', 'irfft', 'hfft', 'ihfft', 'fft2', 'ifft2', 'rfft2', 'irfft2', 'hfft2',
           'ihfft2', 'fftn', 'ifftn', 'rfftn', 'irfftn', 'hfftn', 'ihfftn', 'fftfreq', 'rfftfreq',
           'fftshift', 'ifftshift']

_NORMS = ('forward', 'backward', 'ortho')
_SWAP = {'forward': 'backward', 'backward': 'forward', 'ortho': 'ortho'}


# ----------------------------------------------------------------------------- primitives

def _resize(t, sizes, axes):
    """Crop / zero-pad ``t`` along ``axes`` to ``sizes`` (the reference pads at the end)."""
    if sizes is None:
        return t
    for a, n in zip(axes, sizes):
        cur = t.shape[a]
        if cur > n:
            t = t.narrow(a, 0, n)
        elif cur < n:
            pad = list(t.shape)
            pad[a] = n - cur
            t = torch.cat([t, t.new_zeros(pad)], a)
    return t


def _default_real():
    from .framework.core import get_default_dtype
    d = get_default_dtype()
    return getattr(torch, d) if isinstance(d, str) else d


def _as_complex(t):
    if t.is_complex():
        return t
    if not t.is_floating_point():
        t = t.to(_default_real())
    return t.to(torch.complex128 if t.dtype == torch.float64 else torch.complex64)


def _as_real(t):
    if t.is_complex():
        raise TypeError("this transform expects a real input, got a complex tensor")
    return t if t.is_floating_point() else t.to(_default_real())


@R.register_kernel('fft_c2c', 'ref')
@R.register_kernel('fft_c2c', 'hip')
def _c2c_kernel(x, axes, sizes, norm, forward):
    x = _resize(_as_complex(x), sizes, axes)
    f = torch.fft.fftn if forward else torch.fft.ifftn
    return f(x, dim=tuple(axes), norm=norm)


@R.register_kernel('fft_r2c', 'ref')
@R.register_kernel('fft_r2c', 'hip')
def _r2c_kernel(x, axes, sizes, norm, forward, onesided):
    x = _resize(_as_real(x), sizes, axes)
    axes = tuple(axes)
    f = torch.fft.rfftn if onesided else torch.fft.fftn
    if forward:
        return f(x, dim=axes, norm=norm)
    # e^{+i..} on a real input = conj of the e^{-i..} transform with 1/n on the other side
    return torch.conj(f(x, dim=axes, norm=_SWAP[norm])).resolve_conj()


@R.register_kernel('fft_c2r', 'ref')
@R.register_kernel('fft_c2r', 'hip')
def _c2r_kernel(x, axes, sizes, norm, forward, last_dim_size):
    """``sizes`` = the real output sizes (None: input sizes, last 2*(m-1)); the half-spectrum
    input is resized to sizes[:-1] + [sizes[-1]//2 + 1] first."""
    x = _as_complex(x)
    if sizes is not None:
        x = _resize(x, list(sizes[:-1]) + [sizes[-1] // 2 + 1], axes)
    axes = tuple(axes)
    s = [x.shape[a] for a in axes]
    s[-1] = last_dim_size if last_dim_size else 2 * (x.shape[axes[-1]] - 1)
    if not forward:
        return torch.fft.irfftn(x, s=s, dim=axes, norm=norm)
    return torch.fft.irfftn(torch.conj(x).resolve_conj(), s=s, dim=axes, norm=_SWAP[norm])


def _prim(op):
    def run(x, *attrs):
        t = _u(x)
        return Tensor(R.dispatch(op, t, t, *attrs))
    run.__name__ = op
    return _G.static_op(op, run)


fft_c2c_op, fft_r2c_op, fft_c2r_op = _prim('fft_c2c'), _prim('fft_r2c'), _prim('fft_c2r')


# ----------------------------------------------------------------------------- argument checks

def _check_norm(norm):
    if norm not in _NORMS:
        raise ValueError(f"Unexpected norm: {norm}. Norm should be forward, backward or ortho")


def _check_n(n):
    if not isinstance(n, int) or isinstance(n, bool):
        raise ValueError(f"Invalid FFT argument n({n}), it should be an integer.")
    if n <= 0:
        raise ValueError(f"Invalid FFT argument n({n}), it should be positive.")


def _check_axis(nd, axis):
    if not isinstance(axis, int) or not -nd <= axis < nd:
        raise ValueError(f"Invalid FFT axis ({axis}), it should be an integer in range [-{nd}, {nd})")


def _check_s(nd, s):
    if not isinstance(s, Sequence):
        raise ValueError(f"Invalid FFT argument s({s}), it should be a sequence of integers.")
    if len(s) > nd:
        raise ValueError(f"Length of FFT argument s should not be larger than the rank of input. "
                         f"Received s: {s}, rank of x: {nd}")
    for v in s:
        if not isinstance(v, int) or v <= 0:
            raise ValueError(f"FFT sizes {s} contains invalid value ({v})")


def _check_axes(nd, axes):
    if not isinstance(axes, Sequence):
        raise ValueError(f"Invalid FFT axes ({axes}), it should be a sequence of integers.")
    if len(axes) > nd:
        raise ValueError(f"Length of fft axes should not be larger than the rank of input. "
                         f"Received, len of axes: {len(axes)}, rank of x: {nd}")
    for a in axes:
        if not isinstance(a, int) or not -nd <= a < nd:
            raise ValueError(f"FFT axes {axes} contains invalid value ({a}), it should be in range "
                             f"[-{nd}, {nd})")


def _is_complex(x):
    if isinstance(x, _G.Variable):
        return 'complex' in str(x.dtype)
    return _u(x).is_complex()


def _one_axis(x, n, axis, norm):
    nd = len(x.shape)
    _check_norm(norm)
    axis = -1 if axis is None else axis
    _check_axis(nd, axis)
    if n is not None:
        _check_n(n)
    return [axis % nd], (None if n is None else [n])


def _fft_1d(x, n, axis, norm, forward):
    axes, s = _one_axis(x, n, axis, norm)
    if not _is_complex(x):
        return fft_r2c_op(x, axes, s, norm, forward, False)
    return fft_c2c_op(x, axes, s, norm, forward)


def _r2c_1d(x, n, axis, norm, forward, onesided):
    axes, s = _one_axis(x, n, axis, norm)
    return fft_r2c_op(x, axes, s, norm, forward, onesided)


def _c2r_1d(x, n, axis, norm, forward):
    axes, s = _one_axis(x, n, axis, norm)
    return fft_c2r_op(x, axes, s, norm, forward, n or 0)


def _nd_axes(x, s, axes, norm, real_last):
    """Validated (s, axes) for an n-D transform: axes sorted (the last one pinned for real
    transforms, whose last axis is the half-spectrum one), s permuted alike."""
    nd = len(x.shape)
    _check_norm(norm)
    if s is not None:
        _check_s(nd, s)
    if axes is None:
        axes = list(range(nd)) if s is None else list(range(nd - len(s), nd))
    else:
        _check_axes(nd, axes)
        axes = [a % nd for a in axes]
        if len(set(axes)) != len(axes):
            raise ValueError(f"FFT axes {axes} contains duplicated axes")
        if s is not None and len(s) != len(axes):
            raise ValueError(f"Length of s ({len(s)}) and length of axes ({len(axes)}) does not match.")
        head = axes[:-1] if real_last else axes
        order = sorted(range(len(head)), key=lambda i: head[i])
        axes = [head[i] for i in order] + ([axes[-1]] if real_last else [])
        if s is not None:
            s = [s[i] for i in order] + ([s[-1]] if real_last else [])
    return (list(s) if s is not None else None), axes


def _fftn(x, s, axes, norm, forward):
    if not _is_complex(x):
        return _r2cn(x, s, axes, norm, forward, False)
    s, axes = _nd_axes(x, s, axes, norm, False)
    return fft_c2c_op(x, axes, s, norm, forward)


def _r2cn(x, s, axes, norm, forward, onesided):
    s, axes = _nd_axes(x, s, axes, norm, True)
    return fft_r2c_op(x, axes, s, norm, forward, onesided)


def _c2rn(x, s, axes, norm, forward):
    s, axes = _nd_axes(x, s, axes, norm, True)
    return fft_c2r_op(x, axes, s, norm, forward, s[-1] if s is not None else 0)


def _check_2d(x, s, axes):
    if len(x.shape) < 2:
        raise ValueError(f"The rank of the input ({len(x.shape)}) should >= 2")
    if s is not None and (not isinstance(s, Sequence) or len(s) != 2):
        raise ValueError(f"Invalid FFT argument s ({s}), it should be a sequence of 2 integers.")
    if axes is not None and (not isinstance(axes, Sequence) or len(axes) != 2):
        raise ValueError(f"Invalid FFT argument axes ({axes}), it should be a sequence of 2 integers.")


# ----------------------------------------------------------------------------- public 1-D

def fft(x, n=None, axis=-1, norm='backward', name=None):
    return _fft_1d(x, n, axis, norm, True)


def ifft(x, n=None, axis=-1, norm='backward', name=None):
    return _fft_1d(x, n, axis, norm, False)


def rfft(x, n=None, axis=-1, norm='backward', name=None):
    return _r2c_1d(x, n, axis, norm, True, True)


def irfft(x, n=None, axis=-1, norm='backward', name=None):
    return _c2r_1d(x, n, axis, norm, False)


def hfft(x, n=None, axis=-1, norm='backward', name=None):
    return _c2r_1d(x, n, axis, norm, True)


def ihfft(x, n=None, axis=-1, norm='backward', name=None):
    return _r2c_1d(x, n, axis, norm, False, True)


# ----------------------------------------------------------------------------- public n-D

def fftn(x, s=None, axes=None, norm='backward', name=None):
    return _fftn(x, s, axes, norm, True)


def ifftn(x, s=None, axes=None, norm='backward', name=None):
    return _fftn(x, s, axes, norm, False)


def rfftn(x, s=None, axes=None, norm='backward', name=None):
    return _r2cn(x, s, axes, norm, True, True)


def irfftn(x, s=None, axes=None, norm='backward', name=None):
    return _c2rn(x, s, axes, norm, False)


def hfftn(x, s=None, axes=None, norm='backward', name=None):
    return _c2rn(x, s, axes, norm, True)


def ihfftn(x, s=None, axes=None, norm='backward', name=None):
    return _r2cn(x, s, axes, norm, False, True)


def _two(fn):
    def f(x, s=None, axes=(-2, -1), norm='backward', name=None):
        _check_2d(x, s, axes)
        return fn(x, s, axes, norm, name)
    f.__name__ = fn.__name__ + '2'
    f.__doc__ = f"2-D ``{fn.__name__}`` over ``axes`` (default the last two)."
    return f


fft2, ifft2, rfft2, irfft2, hfft2, ihfft2 = (_two(f) for f in (fftn, ifftn, rfftn, irfftn, hfftn, ihfftn))


# ----------------------------------------------------------------------------- helpers

def _freq_dtype(dtype):
    if dtype is None:
        return _default_real()
    from .framework.core import convert_dtype
    return convert_dtype(dtype)


def fftfreq(n, d=1.0, dtype=None, name=None):
    """Sample frequencies [0, 1, ..., ceil(n/2)-1, -floor(n/2), ..., -1] / (d n)."""
    if d * n == 0:
        raise ValueError("d or n should not be 0.")
    idx = torch.arange(-(n // 2), (n + 1) // 2, dtype=_freq_dtype(dtype))
    return Tensor(torch.roll(idx, -(n // 2)) * (1.0 / (n * d)))


def rfftfreq(n, d=1.0, dtype=None, name=None):
    """Non-negative sample frequencies [0, 1, ..., n//2] / (d n)."""
    if d * n == 0:
        raise ValueError("d or n should not be 0.")
    return Tensor(torch.arange(0, n // 2 + 1, dtype=_freq_dtype(dtype)) * (1.0 / (n * d)))


def _shift(x, axes, sign):
    t = _u(x)
    if axes is None:
        axes = list(range(t.dim()))
    elif isinstance(axes, int):
        axes = [axes]
    shifts = [sign * (t.shape[a] // 2) for a in axes]
    return Tensor(torch.roll(t, shifts, list(axes)))


def _fftshift(x, axes=None, name=None):
    """Move the zero-frequency term to the centre (roll by n//2 along each axis)."""
    return _shift(x, axes, 1)


def _ifftshift(x, axes=None, name=None):
    """Inverse of ``fftshift`` (roll by -(n//2)); differs from it for odd lengths."""
    return _shift(x, axes, -1)


fftshift = _G.static_op('fftshift', _fftshift)
ifftshift = _G.static_op('ifftshift', _ifftshift)
