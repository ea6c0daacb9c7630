"""paddle.signal (parity: python/paddle/signal.py)."""
import torch

from .framework.core import Tensor, _u


def stft(x, n_fft, hop_length=None, win_length=None, window=None, center=True, pad_mode='reflect',
         normalized=False, onesided=True, name=None):
    return Tensor(torch.stft(_u(x), n_fft, hop_length, win_length,
                             None if window is None else _u(window), center, pad_mode, normalized,
                             onesided, return_complex=True))


def istft(x, n_fft, hop_length=None, win_length=None, window=None, center=True, normalized=False,
          onesided=True, length=None, return_complex=False, name=None):
    return Tensor(torch.istft(_u(x), n_fft, hop_length, win_length,
                              None if window is None else _u(window), center, normalized, onesided,
                              length, return_complex))


def frame(x, frame_length, hop_length, axis=-1, name=None):
    t = _u(x)
    return Tensor(t.unfold(axis, frame_length, hop_length).movedim(-1, axis - 1 if axis < 0 else axis))


def overlap_add(x, hop_length, axis=-1, name=None):
    t = _u(x)
    fl, nf = t.shape[-2], t.shape[-1]
    n = (nf - 1) * hop_length + fl
    out = torch.zeros(t.shape[:-2] + (n,), dtype=t.dtype, device=t.device)
    for i in range(nf):
        out[..., i * hop_length:i * hop_length + fl] += t[..., :, i]
    return Tensor(out)
