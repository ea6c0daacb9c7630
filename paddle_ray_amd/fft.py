"""paddle.fft (parity: python/paddle/fft.py) — rocFFT through PyTorch-ROCm."""
import torch

from .framework.core import Tensor, _u


def _mk(fn, nd=False):
    if nd:
        def f(x, s=None, axes=None, norm='backward', name=None):
            return Tensor(fn(_u(x), s=s, dim=axes, norm=norm))
    else:
        def f(x, n=None, axis=-1, norm='backward', name=None):
            return Tensor(fn(_u(x), n=n, dim=axis, norm=norm))
    return f


fft, ifft, rfft, irfft, hfft, ihfft = (_mk(getattr(torch.fft, n)) for n in
                                       ('fft', 'ifft', 'rfft', 'irfft', 'hfft', 'ihfft'))
fftn, ifftn, rfftn, irfftn, hfftn, ihfftn = (_mk(getattr(torch.fft, n), True) for n in
                                             ('fftn', 'ifftn', 'rfftn', 'irfftn', 'hfftn', 'ihfftn'))


def _mk2(fn):
    def f(x, s=None, axes=(-2, -1), norm='backward', name=None):
        return Tensor(fn(_u(x), s=s, dim=axes, norm=norm))
    return f


fft2, ifft2, rfft2, irfft2, hfft2, ihfft2 = (_mk2(getattr(torch.fft, n)) for n in
                                             ('fft2', 'ifft2', 'rfft2', 'irfft2', 'hfft2', 'ihfft2'))


def fftfreq(n, d=1.0, dtype=None, name=None):
    return Tensor(torch.fft.fftfreq(n, d))


def rfftfreq(n, d=1.0, dtype=None, name=None):
    return Tensor(torch.fft.rfftfreq(n, d))


def fftshift(x, axes=None, name=None):
    return Tensor(torch.fft.fftshift(_u(x), axes))


def ifftshift(x, axes=None, name=None):
    return Tensor(torch.fft.ifftshift(_u(x), axes))
