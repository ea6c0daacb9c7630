"""paddle.vision (parity: python/paddle/vision/__init__.py)."""
from . import models, transforms, datasets, ops  # noqa
from .models import *  # noqa


def set_image_backend(backend):
    pass


def get_image_backend():
    return 'cv2'
