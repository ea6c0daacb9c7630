"""paddle.audio (parity: python/paddle/audio/): window functions, mel/DCT filterbanks,
spectrogram feature layers (STFT on the device via paddle.signal.stft), WAV I/O backend
and audio-classification datasets read from local files."""
from . import functional  # noqa: F401
from . import features  # noqa: F401
from . import backends  # noqa: F401
from . import datasets  # noqa: F401
from .backends import info, load, save  # noqa: F401

__all__ = ["functional", "features", "datasets", "backends", "load", "info", "save"]
