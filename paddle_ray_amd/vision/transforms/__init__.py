"""paddle.vision.transforms (parity: python/paddle/vision/transforms/transforms.py) — numpy HWC."""
import numbers
import random

import numpy as np

from ...framework.core import Tensor


class BaseTransform:
    def __call__(self, img):
        return self._apply_image(img)


class Compose:
    def __init__(self, transforms):
        self.transforms = transforms

    def __call__(self, data):
        for t in self.transforms:
            data = t(data)
        return data


class ToTensor(BaseTransform):
    def __init__(self, data_format='CHW', keys=None):
        self.data_format = data_format

    def _apply_image(self, img):
        a = np.asarray(img)
        if a.ndim == 2:
            a = a[:, :, None]
        a = a.astype(np.float32)
        if np.asarray(img).dtype == np.uint8:
            a = a / 255.0
        if self.data_format == 'CHW':
            a = a.transpose(2, 0, 1)
        return Tensor(a)


class Normalize(BaseTransform):
    def __init__(self, mean=0.0, std=1.0, data_format='CHW', to_rgb=False, keys=None):
        self.mean = np.asarray(mean, dtype=np.float32)
        self.std = np.asarray(std, dtype=np.float32)
        self.data_format = data_format

    def _apply_image(self, img):
        a = img.numpy() if isinstance(img, Tensor) else np.asarray(img, dtype=np.float32)
        shp = (-1, 1, 1) if self.data_format == 'CHW' else (1, 1, -1)
        out = (a - self.mean.reshape(shp)) / self.std.reshape(shp)
        return Tensor(out.astype(np.float32)) if isinstance(img, Tensor) else out.astype(np.float32)


class Transpose(BaseTransform):
    def __init__(self, order=(2, 0, 1), keys=None):
        self.order = order

    def _apply_image(self, img):
        return np.asarray(img).transpose(self.order)


class Resize(BaseTransform):
    def __init__(self, size, interpolation='bilinear', keys=None):
        self.size = size

    def _apply_image(self, img):
        import torch
        a = np.asarray(img, dtype=np.float32)
        hw = (self.size, self.size) if isinstance(self.size, int) else tuple(self.size)
        t = torch.from_numpy(a.transpose(2, 0, 1)[None] if a.ndim == 3 else a[None, None])
        out = torch.nn.functional.interpolate(t, size=hw, mode='bilinear', align_corners=False)
        o = out[0].numpy()
        return o.transpose(1, 2, 0) if a.ndim == 3 else o[0]


class CenterCrop(BaseTransform):
    def __init__(self, size, keys=None):
        self.size = (size, size) if isinstance(size, int) else size

    def _apply_image(self, img):
        a = np.asarray(img)
        h, w = a.shape[:2]
        th, tw = self.size
        i, j = (h - th) // 2, (w - tw) // 2
        return a[i:i + th, j:j + tw]


class RandomCrop(CenterCrop):
    def __init__(self, size, padding=None, pad_if_needed=False, keys=None):
        super().__init__(size)
        self.padding = padding

    def _apply_image(self, img):
        a = np.asarray(img)
        if self.padding:
            p = self.padding
            a = np.pad(a, ((p, p), (p, p)) + ((0, 0),) * (a.ndim - 2))
        h, w = a.shape[:2]
        th, tw = self.size
        i, j = random.randint(0, h - th), random.randint(0, w - tw)
        return a[i:i + th, j:j + tw]


class RandomHorizontalFlip(BaseTransform):
    def __init__(self, prob=0.5, keys=None):
        self.prob = prob

    def _apply_image(self, img):
        a = np.asarray(img)
        return a[:, ::-1].copy() if random.random() < self.prob else a


class RandomVerticalFlip(RandomHorizontalFlip):
    def _apply_image(self, img):
        a = np.asarray(img)
        return a[::-1].copy() if random.random() < self.prob else a


def to_tensor(pic, data_format='CHW'):
    return ToTensor(data_format)(pic)


def normalize(img, mean, std, data_format='CHW', to_rgb=False):
    return Normalize(mean, std, data_format)(img)
