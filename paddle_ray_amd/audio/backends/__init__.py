"""Audio I/O backends (parity: python/paddle/audio/backends/): a built-in PCM16 WAV backend
(Python ``wave`` + numpy); other backends can be registered with :func:`register_backend`."""
import wave

import numpy as np
import torch

from ...framework.core import Tensor, _u

__all__ = ['get_current_backend', 'list_available_backends', 'set_backend', 'info', 'load',
           'save', 'AudioInfo']


class AudioInfo:
    """Audio file metadata."""

    def __init__(self, sample_rate, num_frames, num_channels, bits_per_sample, encoding):
        self.sample_rate = sample_rate
        self.num_frames = num_frames
        self.num_channels = num_channels
        self.bits_per_sample = bits_per_sample
        self.encoding = encoding

    def __repr__(self):
        return (f"AudioInfo(sample_rate={self.sample_rate}, num_frames={self.num_frames}, "
                f"num_channels={self.num_channels}, bits_per_sample={self.bits_per_sample}, "
                f"encoding={self.encoding})")


def _open(filepath, mode):
    return filepath if hasattr(filepath, 'read' if mode == 'rb' else 'write') else \
        open(filepath, mode)


def _wave_info(filepath):
    f = _open(filepath, 'rb')
    try:
        w = wave.open(f)
    except wave.Error as e:
        raise NotImplementedError("only PCM16 WAV is supported by the 'wave_backend'") from e
    out = AudioInfo(w.getframerate(), w.getnframes(), w.getnchannels(), w.getsampwidth() * 8,
                    'PCM_S')
    w.close()
    return out


def _wave_load(filepath, frame_offset=0, num_frames=-1, normalize=True, channels_first=True):
    f = _open(filepath, 'rb')
    try:
        w = wave.open(f)
    except wave.Error as e:
        raise NotImplementedError("only PCM16 WAV is supported by the 'wave_backend'") from e
    ch, sr, n = w.getnchannels(), w.getframerate(), w.getnframes()
    if w.getsampwidth() != 2:
        raise NotImplementedError("only 16-bit PCM WAV is supported")
    w.setpos(min(frame_offset, n))
    count = n - frame_offset if num_frames == -1 else min(num_frames, n - frame_offset)
    raw = w.readframes(max(count, 0))
    w.close()
    data = np.frombuffer(raw, dtype='<i2').reshape(-1, ch)
    if normalize:
        data = data.astype(np.float32) / 32768.0
    t = torch.from_numpy(np.ascontiguousarray(data.T if channels_first else data))
    return Tensor(t), sr


def _wave_save(filepath, src, sample_rate, channels_first=True, encoding=None,
               bits_per_sample=16):
    if bits_per_sample not in (None, 16):
        raise NotImplementedError("the 'wave_backend' writes 16-bit PCM only")
    a = _u(src).detach().cpu().numpy() if isinstance(src, Tensor) or torch.is_tensor(src) \
        else np.asarray(src)
    if a.ndim == 1:
        a = a[None, :] if channels_first else a[:, None]
    if channels_first:
        a = a.T
    if a.dtype.kind == 'f':
        a = np.clip(a, -1.0, 1.0 - 1.0 / 32768.0) * 32768.0
    pcm = a.astype('<i2')
    f = _open(filepath, 'wb')
    w = wave.open(f, 'wb')
    w.setnchannels(pcm.shape[1])
    w.setsampwidth(2)
    w.setframerate(int(sample_rate))
    w.writeframes(pcm.tobytes())
    w.close()


_BACKENDS = {'wave_backend': (_wave_info, _wave_load, _wave_save)}
_current = ['wave_backend']


def register_backend(name, info_fn, load_fn, save_fn):
    _BACKENDS[name] = (info_fn, load_fn, save_fn)


def list_available_backends():
    return list(_BACKENDS)


def get_current_backend():
    return _current[0]


def set_backend(backend_name):
    if backend_name not in _BACKENDS:
        raise NotImplementedError(f"audio backend {backend_name!r} is not available "
                                  f"(available: {list(_BACKENDS)})")
    _current[0] = backend_name


def info(filepath):
    return _BACKENDS[_current[0]][0](filepath)


def load(filepath, frame_offset=0, num_frames=-1, normalize=True, channels_first=True):
    return _BACKENDS[_current[0]][1](filepath, frame_offset, num_frames, normalize,
                                     channels_first)


def save(filepath, src, sample_rate, channels_first=True, encoding=None, bits_per_sample=16):
    return _BACKENDS[_current[0]][2](filepath, src, sample_rate, channels_first, encoding,
                                     bits_per_sample)
