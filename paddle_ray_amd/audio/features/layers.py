"""Audio feature layers (parity: python/paddle/audio/features/layers.py). The STFT runs on
the tensor's device (rocFFT on MI355X); filterbank / DCT projections are GEMMs over the
frequency axis, batched over the (N, frames) dimensions."""
import torch

from ... import nn
from ...framework.core import Tensor, _u
from ..functional import compute_fbank_matrix, create_dct, power_to_db
from ..functional.window import get_window


class Spectrogram(nn.Layer):
    """|STFT(x)|^power : (N, T) -> (N, n_fft//2 + 1, frames)."""

    def __init__(self, n_fft=512, hop_length=512, win_length=None, window='hann', power=1.0,
                 center=True, pad_mode='reflect', dtype='float32'):
        super().__init__()
        if power <= 0:
            raise ValueError('Power of spectrogram must be > 0.')
        self.power = power
        win_length = n_fft if win_length is None else win_length
        self.n_fft, self.hop_length, self.win_length = n_fft, hop_length, win_length
        self.center, self.pad_mode = center, pad_mode
        self.register_buffer('fft_window', get_window(window, win_length, fftbins=True,
                                                      dtype=dtype))

    def forward(self, x):
        t = _u(x)
        w = _u(self.fft_window).to(t.device)
        hop = self.hop_length if self.hop_length is not None else self.win_length // 4
        st = torch.stft(t, self.n_fft, hop, self.win_length, w, self.center, self.pad_mode,
                         False, True, return_complex=True)
        return Tensor(st.abs().pow(self.power))


class MelSpectrogram(nn.Layer):
    def __init__(self, sr=22050, n_fft=2048, hop_length=512, win_length=None, window='hann',
                 power=2.0, center=True, pad_mode='reflect', n_mels=64, f_min=50.0, f_max=None,
                 htk=False, norm='slaney', dtype='float32'):
        super().__init__()
        self._spectrogram = Spectrogram(n_fft, hop_length, win_length, window, power, center,
                                        pad_mode, dtype)
        self.n_mels, self.f_min, self.f_max, self.htk, self.norm = n_mels, f_min, f_max, htk, norm
        if f_max is None:
            f_max = sr // 2
        self.register_buffer('fbank_matrix', compute_fbank_matrix(sr, n_fft, n_mels, f_min, f_max,
                                                                  htk, norm, dtype))

    def forward(self, x):
        spec = _u(self._spectrogram(x))
        fb = _u(self.fbank_matrix).to(spec.device, spec.dtype)
        return Tensor(torch.matmul(fb, spec))


class LogMelSpectrogram(nn.Layer):
    def __init__(self, sr=22050, n_fft=512, hop_length=None, win_length=None, window='hann',
                 power=2.0, center=True, pad_mode='reflect', n_mels=64, f_min=50.0, f_max=None,
                 htk=False, norm='slaney', ref_value=1.0, amin=1e-10, top_db=None,
                 dtype='float32'):
        super().__init__()
        self._melspectrogram = MelSpectrogram(sr, n_fft, hop_length, win_length, window, power,
                                              center, pad_mode, n_mels, f_min, f_max, htk, norm,
                                              dtype)
        self.ref_value, self.amin, self.top_db = ref_value, amin, top_db

    def forward(self, x):
        return power_to_db(self._melspectrogram(x), self.ref_value, self.amin, self.top_db)


class MFCC(nn.Layer):
    def __init__(self, sr=22050, n_mfcc=40, n_fft=512, hop_length=None, win_length=None,
                 window='hann', power=2.0, center=True, pad_mode='reflect', n_mels=64,
                 f_min=50.0, f_max=None, htk=False, norm='slaney', ref_value=1.0, amin=1e-10,
                 top_db=None, dtype='float32'):
        super().__init__()
        if n_mfcc > n_mels:
            raise ValueError(f'n_mfcc cannot be larger than n_mels: {n_mfcc} vs {n_mels}')
        self._log_melspectrogram = LogMelSpectrogram(sr, n_fft, hop_length, win_length, window,
                                                     power, center, pad_mode, n_mels, f_min,
                                                     f_max, htk, norm, ref_value, amin, top_db,
                                                     dtype)
        self.register_buffer('dct_matrix', create_dct(n_mfcc, n_mels, dtype=dtype))

    def forward(self, x):
        lm = _u(self._log_melspectrogram(x))                     # (N, n_mels, frames)
        dct = _u(self.dct_matrix).to(lm.device, lm.dtype)         # (n_mels, n_mfcc)
        return Tensor(torch.matmul(lm.transpose(-1, -2), dct).transpose(-1, -2))
