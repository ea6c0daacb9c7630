"""paddle.vision.transforms (parity: python/paddle/vision/transforms/__init__.py)."""
from . import functional  # noqa: F401
from .transforms import (BaseTransform, Compose, ToTensor, Normalize, Transpose, Resize,  # noqa
                         RandomResizedCrop, CenterCrop, RandomCrop, RandomHorizontalFlip,
                         RandomVerticalFlip, BrightnessTransform, ContrastTransform,
                         SaturationTransform, HueTransform, ColorJitter, Pad, RandomRotation,
                         RandomAffine, RandomPerspective, Grayscale, RandomErasing)
from .functional import (to_tensor, normalize, resize, crop, center_crop, hflip, vflip,  # noqa
                         pad, affine, rotate, perspective, to_grayscale, adjust_brightness,
                         adjust_contrast, adjust_saturation, adjust_hue, erase)
