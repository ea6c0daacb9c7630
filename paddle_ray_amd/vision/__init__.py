"""paddle.vision (parity: python/paddle/vision/__init__.py)."""
from .image import set_image_backend, get_image_backend, image_load  # noqa: F401
from . import models, transforms, datasets, ops  # noqa
from .models import *  # noqa
