"""Window functions (parity: python/paddle/audio/functional/window.py; definitions follow
scipy.signal.windows, which computes them here in float64 before the cast)."""
import numpy as np
import torch

from ...framework.core import Tensor

_SUPPORTED = ('hamming', 'hann', 'gaussian', 'general_gaussian', 'exponential', 'triang',
              'bohman', 'blackman', 'cosine', 'tukey', 'taylor', 'general_cosine',
              'general_hamming', 'kaiser')


def get_window(window, win_length, fftbins=True, dtype='float64'):
    """Window of ``win_length`` samples; ``fftbins=True`` gives the periodic (DFT-even)
    form. Parameterised windows are passed as tuples, e.g. ``('gaussian', 7)``."""
    from ...framework.core import convert_dtype
    if isinstance(window, tuple):
        name, args = window[0], tuple(window[1:])
    elif isinstance(window, str):
        if window in ('gaussian', 'exponential'):
            raise ValueError(f"The '{window}' window needs one or more parameters -- pass a tuple.")
        name, args = window, ()
    else:
        raise ValueError(f"{type(window)} as window type is not supported.")
    if name not in _SUPPORTED:
        raise ValueError("Unknown window type.")
    import scipy.signal
    spec = (name,) + args if args else name
    if name == 'exponential' and args:  # (center, tau) ; scipy: exponential(M, center, tau)
        spec = ('exponential',) + args
    w = scipy.signal.get_window(spec, int(win_length), fftbins=fftbins)
    return Tensor(torch.from_numpy(np.asarray(w, dtype=np.float64)).to(convert_dtype(dtype)))
