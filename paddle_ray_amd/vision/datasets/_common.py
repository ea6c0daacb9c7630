"""Shared helpers for the vision datasets: data-home lookup, safe CIFAR unpickling, image
decoding."""
import io
import os
import pickle

import numpy as np

DATA_HOME = os.path.expanduser(os.environ.get('PADDLE_DATA_HOME', '~/.cache/paddle/dataset'))


def find_local(module, filename):
    """``DATA_HOME/module/filename`` if it exists (no network: nothing is downloaded)."""
    p = os.path.join(DATA_HOME, module, filename)
    return p if os.path.exists(p) else None


def require(path, what, download):
    if path is None or not os.path.exists(path):
        raise FileNotFoundError(
            f"{what}: file {path!r} not found. This environment has no network access, so "
            f"datasets are never downloaded (download={download}); pass the local file path.")
    return path


class _NumpyOnlyUnpickler(pickle.Unpickler):
    """Unpickler for the CIFAR python batches: only builtin containers and plain numpy
    array reconstruction are allowed, so a crafted file cannot run code."""

    _ALLOWED = {('numpy.core.multiarray', '_reconstruct'),
                ('numpy._core.multiarray', '_reconstruct'), ('numpy', 'ndarray'),
                ('numpy', 'dtype'), ('copyreg', '_reconstructor'), ('builtins', 'object')}

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from a dataset file")


def load_numpy_pickle(fileobj):
    return _NumpyOnlyUnpickler(fileobj, encoding='bytes').load()


def decode_image(data, backend, mode='RGB'):
    """Bytes -> PIL image ('pil') or HWC uint8 array ('cv2': BGR channel order like cv2)."""
    from PIL import Image
    img = Image.open(io.BytesIO(data))
    img = img.convert(mode) if mode else img
    if backend == 'pil':
        return img
    arr = np.asarray(img)
    if arr.ndim == 3 and arr.shape[2] == 3:
        arr = arr[:, :, ::-1]
    return np.ascontiguousarray(arr)


def check_backend(backend):
    if backend is None:
        from .. import get_image_backend
        backend = get_image_backend()
    if backend not in ('pil', 'cv2'):
        raise ValueError(f"Expected backend are one of ['pil', 'cv2'], but got {backend}")
    return backend
