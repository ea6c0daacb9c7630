"""Mel / DCT helpers (parity: python/paddle/audio/functional/functional.py; librosa's Slaney
and HTK mel scales). Tensors are built with torch ops on the default device."""
import math

import torch

from ...framework.core import Tensor, _u


def _dt(dtype):
    from ...framework.core import convert_dtype
    return convert_dtype(dtype) if dtype is not None else torch.float32


def _is_t(x):
    return isinstance(x, Tensor) or torch.is_tensor(x)


_F_SP = 200.0 / 3            # Slaney: linear region slope (Hz per mel)
_MIN_LOG_HZ = 1000.0         # start of the log region
_MIN_LOG_MEL = _MIN_LOG_HZ / _F_SP
_LOGSTEP = math.log(6.4) / 27.0


def hz_to_mel(freq, htk=False):
    """Hz -> mel (HTK: 2595 log10(1 + f/700); Slaney: linear below 1 kHz, log above)."""
    if _is_t(freq):
        f = _u(freq)
        if htk:
            return Tensor(2595.0 * torch.log10(1.0 + f / 700.0))
        lin = f / _F_SP
        log = _MIN_LOG_MEL + torch.log(f / _MIN_LOG_HZ + 1e-10) / _LOGSTEP
        return Tensor(torch.where(f > _MIN_LOG_HZ, log, lin))
    if htk:
        return 2595.0 * math.log10(1.0 + freq / 700.0)
    if freq >= _MIN_LOG_HZ:
        return _MIN_LOG_MEL + math.log(freq / _MIN_LOG_HZ + 1e-10) / _LOGSTEP
    return freq / _F_SP


def mel_to_hz(mel, htk=False):
    """mel -> Hz, inverse of :func:`hz_to_mel`."""
    if _is_t(mel):
        m = _u(mel)
        if htk:
            return Tensor(700.0 * (10.0 ** (m / 2595.0) - 1.0))
        lin = _F_SP * m
        log = _MIN_LOG_HZ * torch.exp(_LOGSTEP * (m - _MIN_LOG_MEL))
        return Tensor(torch.where(m > _MIN_LOG_MEL, log, lin))
    if htk:
        return 700.0 * (10.0 ** (mel / 2595.0) - 1.0)
    if mel >= _MIN_LOG_MEL:
        return _MIN_LOG_HZ * math.exp(_LOGSTEP * (mel - _MIN_LOG_MEL))
    return _F_SP * mel


def mel_frequencies(n_mels=64, f_min=0.0, f_max=11025.0, htk=False, dtype='float32'):
    """n_mels frequencies (Hz) uniformly spaced on the mel scale."""
    lo, hi = hz_to_mel(f_min, htk=htk), hz_to_mel(f_max, htk=htk)
    mels = torch.linspace(lo, hi, n_mels, dtype=torch.float64)
    return Tensor(_u(mel_to_hz(Tensor(mels), htk=htk)).to(_dt(dtype)))


def fft_frequencies(sr, n_fft, dtype='float32'):
    """Center frequencies of the n_fft//2 + 1 one-sided FFT bins."""
    return Tensor(torch.linspace(0, float(sr) / 2, int(1 + n_fft // 2), dtype=_dt(dtype)))


def compute_fbank_matrix(sr, n_fft, n_mels=64, f_min=0.0, f_max=None, htk=False, norm='slaney',
                         dtype='float32'):
    """Triangular mel filterbank [n_mels, n_fft//2 + 1] (Slaney area normalisation by
    default, or p-norm rows for a numeric ``norm``)."""
    if f_max is None:
        f_max = float(sr) / 2
    fft_f = _u(fft_frequencies(sr, n_fft, 'float64'))
    mel_f = _u(mel_frequencies(n_mels + 2, f_min, f_max, htk, 'float64'))
    fdiff = mel_f[1:] - mel_f[:-1]
    ramps = mel_f[:, None] - fft_f[None, :]
    lower = -ramps[:-2] / fdiff[:-1, None]
    upper = ramps[2:] / fdiff[1:, None]
    w = torch.clamp(torch.minimum(lower, upper), min=0.0)
    if norm == 'slaney':
        w = w * (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, None]
    elif isinstance(norm, (int, float)):
        w = torch.nn.functional.normalize(w, p=float(norm), dim=-1)
    return Tensor(w.to(_dt(dtype)))


def power_to_db(spect, ref_value=1.0, amin=1e-10, top_db=80.0):
    """10 log10(max(S, amin) / ref), floored at ``top_db`` below the peak."""
    if amin <= 0:
        raise ValueError("amin must be strictly positive")
    if ref_value <= 0:
        raise ValueError("ref_value must be strictly positive")
    s = _u(spect) if _is_t(spect) else torch.as_tensor(spect)
    log_spec = 10.0 * torch.log10(torch.clamp(s, min=amin))
    log_spec = log_spec - 10.0 * math.log10(max(ref_value, amin))
    if top_db is not None:
        if top_db < 0:
            raise ValueError("top_db must be non-negative")
        log_spec = torch.maximum(log_spec, log_spec.max() - top_db)
    return Tensor(log_spec)


def create_dct(n_mfcc, n_mels, norm='ortho', dtype='float32'):
    """DCT-II basis [n_mels, n_mfcc] (orthonormal with ``norm='ortho'``)."""
    n = torch.arange(n_mels, dtype=torch.float64)
    k = torch.arange(n_mfcc, dtype=torch.float64)[:, None]
    dct = torch.cos(math.pi / float(n_mels) * (n + 0.5) * k)
    if norm is None:
        dct = dct * 2.0
    else:
        if norm != 'ortho':
            raise ValueError("norm must be None or 'ortho'")
        dct[0] *= 1.0 / math.sqrt(2.0)
        dct = dct * math.sqrt(2.0 / float(n_mels))
    return Tensor(dct.t().contiguous().to(_dt(dtype)))
