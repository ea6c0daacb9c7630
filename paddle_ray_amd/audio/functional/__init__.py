from .functional import (hz_to_mel, mel_to_hz, mel_frequencies, fft_frequencies,  # noqa: F401
                         compute_fbank_matrix, power_to_db, create_dct)
from .window import get_window  # noqa: F401

__all__ = ['compute_fbank_matrix', 'create_dct', 'fft_frequencies', 'hz_to_mel', 'mel_frequencies',
           'mel_to_hz', 'power_to_db', 'get_window']
