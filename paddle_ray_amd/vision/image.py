"""Image backend selection and loading (parity: python/paddle/vision/image.py). 'cv2'
(OpenCV is not installed here) is served by PIL returning HWC uint8 BGR arrays like
cv2.imread."""
import numpy as np

_image_backend = 'pil'


def set_image_backend(backend):
    global _image_backend
    if backend not in ('pil', 'cv2', 'tensor'):
        raise ValueError(f"Expected backend are one of ['pil', 'cv2', 'tensor'], but got {backend}")
    _image_backend = backend


def get_image_backend():
    return _image_backend


def image_load(path, backend=None):
    from PIL import Image
    backend = backend or _image_backend
    if backend == 'pil':
        return Image.open(path)
    arr = np.asarray(Image.open(path).convert('RGB'))[:, :, ::-1]
    return np.ascontiguousarray(arr)
