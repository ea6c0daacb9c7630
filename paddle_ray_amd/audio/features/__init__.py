from .layers import Spectrogram, MelSpectrogram, LogMelSpectrogram, MFCC  # noqa: F401

__all__ = ['Spectrogram', 'MelSpectrogram', 'LogMelSpectrogram', 'MFCC']
