"""paddle.vision.transforms classes (parity: python/paddle/vision/transforms/transforms.py).

Every transform accepts a PIL image, an HWC numpy array or a CHW Tensor (see
``functional``). ``keys`` lets a transform receive a tuple such as (image, label): entries
named 'image' are transformed, everything else passes through unchanged.
"""
import math
import numbers
import random

import numpy as np

from ...framework.core import Tensor, _u
from . import functional as F


def _setup_size(size):
    return (int(size), int(size)) if isinstance(size, numbers.Number) else tuple(size)


class BaseTransform:
    def __init__(self, keys=None):
        self.keys = keys if keys is not None else ('image',)
        self.params = None

    def _get_params(self, inputs):
        return None

    def _apply_image(self, img):
        raise NotImplementedError

    def __call__(self, inputs):
        if isinstance(inputs, tuple):
            self.params = self._get_params(inputs)
            out = []
            for key, data in zip(self.keys, inputs):
                fn = getattr(self, f'_apply_{key}', None)
                out.append(fn(data) if fn is not None else data)
            out += list(inputs[len(self.keys):])
            return tuple(out)
        self.params = self._get_params((inputs,))
        return self._apply_image(inputs)


class Compose:
    def __init__(self, transforms):
        self.transforms = transforms

    def __call__(self, data):
        for t in self.transforms:
            data = t(data)
        return data

    def __repr__(self):
        return 'Compose(' + ', '.join(type(t).__name__ for t in self.transforms) + ')'


class ToTensor(BaseTransform):
    def __init__(self, data_format='CHW', keys=None):
        super().__init__(keys)
        self.data_format = data_format

    def _apply_image(self, img):
        return F.to_tensor(img, self.data_format)


class Normalize(BaseTransform):
    def __init__(self, mean=0.0, std=1.0, data_format='CHW', to_rgb=False, keys=None):
        super().__init__(keys)
        n = lambda v: [v] * 3 if isinstance(v, numbers.Number) else list(v)  # noqa: E731
        self.mean, self.std = n(mean), n(std)
        self.data_format, self.to_rgb = data_format, to_rgb

    def _apply_image(self, img):
        c = (_u(img).shape[0 if self.data_format == 'CHW' else -1] if isinstance(img, Tensor)
             else np.asarray(img).shape[0 if self.data_format == 'CHW' else -1])
        return F.normalize(img, self.mean[:c], self.std[:c], self.data_format, self.to_rgb)


class Transpose(BaseTransform):
    def __init__(self, order=(2, 0, 1), keys=None):
        super().__init__(keys)
        self.order = order

    def _apply_image(self, img):
        if isinstance(img, Tensor):
            return img.transpose(list(self.order))
        a = np.asarray(img)
        if a.ndim == 2:
            a = a[..., None]
        return a.transpose(self.order)


class Resize(BaseTransform):
    def __init__(self, size, interpolation='bilinear', keys=None):
        super().__init__(keys)
        self.size, self.interpolation = size, interpolation

    def _apply_image(self, img):
        return F.resize(img, self.size, self.interpolation)


class RandomResizedCrop(BaseTransform):
    def __init__(self, size, scale=(0.08, 1.0), ratio=(3.0 / 4, 4.0 / 3),
                 interpolation='bilinear', keys=None):
        super().__init__(keys)
        self.size = _setup_size(size)
        self.scale, self.ratio, self.interpolation = scale, ratio, interpolation

    def _crop_params(self, img):
        h, w = F._size_hw(img)
        area = h * w
        for _ in range(10):
            target = random.uniform(*self.scale) * area
            log_r = (math.log(self.ratio[0]), math.log(self.ratio[1]))
            ar = math.exp(random.uniform(*log_r))
            cw = int(round(math.sqrt(target * ar)))
            ch = int(round(math.sqrt(target / ar)))
            if 0 < cw <= w and 0 < ch <= h:
                return random.randint(0, h - ch), random.randint(0, w - cw), ch, cw
        in_ratio = w / h
        if in_ratio < min(self.ratio):
            cw, ch = w, int(round(w / min(self.ratio)))
        elif in_ratio > max(self.ratio):
            ch, cw = h, int(round(h * max(self.ratio)))
        else:
            cw, ch = w, h
        return (h - ch) // 2, (w - cw) // 2, ch, cw

    def _apply_image(self, img):
        i, j, h, w = self._crop_params(img)
        return F.resize(F.crop(img, i, j, h, w), self.size, self.interpolation)


class CenterCrop(BaseTransform):
    def __init__(self, size, keys=None):
        super().__init__(keys)
        self.size = _setup_size(size)

    def _apply_image(self, img):
        return F.center_crop(img, self.size)


class RandomCrop(BaseTransform):
    def __init__(self, size, padding=None, pad_if_needed=False, fill=0, padding_mode='constant',
                 keys=None):
        super().__init__(keys)
        self.size = _setup_size(size)
        self.padding, self.pad_if_needed = padding, pad_if_needed
        self.fill, self.padding_mode = fill, padding_mode

    def _apply_image(self, img):
        if self.padding is not None:
            img = F.pad(img, self.padding, self.fill, self.padding_mode)
        h, w = F._size_hw(img)
        th, tw = self.size
        if self.pad_if_needed and w < tw:
            img = F.pad(img, (tw - w, 0), self.fill, self.padding_mode)
        if self.pad_if_needed and h < th:
            img = F.pad(img, (0, th - h), self.fill, self.padding_mode)
        h, w = F._size_hw(img)
        i, j = random.randint(0, h - th), random.randint(0, w - tw)
        return F.crop(img, i, j, th, tw)


class RandomHorizontalFlip(BaseTransform):
    def __init__(self, prob=0.5, keys=None):
        super().__init__(keys)
        self.prob = prob

    def _apply_image(self, img):
        return F.hflip(img) if random.random() < self.prob else img


class RandomVerticalFlip(BaseTransform):
    def __init__(self, prob=0.5, keys=None):
        super().__init__(keys)
        self.prob = prob

    def _apply_image(self, img):
        return F.vflip(img) if random.random() < self.prob else img


class _ColorBase(BaseTransform):
    def __init__(self, value, keys=None, center=1.0, bound=(0, float('inf'))):
        super().__init__(keys)
        if isinstance(value, numbers.Number):
            if value < 0:
                raise ValueError("value must be non-negative")
            value = [center - value, center + value]
        self.value = [max(bound[0], value[0]), min(bound[1], value[1])]

    def _factor(self):
        return random.uniform(*self.value)


class BrightnessTransform(_ColorBase):
    def _apply_image(self, img):
        return F.adjust_brightness(img, self._factor()) if self.value != [1, 1] else img


class ContrastTransform(_ColorBase):
    def _apply_image(self, img):
        return F.adjust_contrast(img, self._factor()) if self.value != [1, 1] else img


class SaturationTransform(_ColorBase):
    def _apply_image(self, img):
        return F.adjust_saturation(img, self._factor()) if self.value != [1, 1] else img


class HueTransform(_ColorBase):
    def __init__(self, value, keys=None):
        super().__init__(value, keys, center=0.0, bound=(-0.5, 0.5))

    def _apply_image(self, img):
        return F.adjust_hue(img, self._factor()) if self.value != [0, 0] else img


class ColorJitter(BaseTransform):
    """Brightness / contrast / saturation / hue jitter applied in random order."""

    def __init__(self, brightness=0, contrast=0, saturation=0, hue=0, keys=None):
        super().__init__(keys)
        self.ts = [BrightnessTransform(brightness), ContrastTransform(contrast),
                   SaturationTransform(saturation), HueTransform(hue)]

    def _apply_image(self, img):
        order = list(range(4))
        random.shuffle(order)
        for i in order:
            img = self.ts[i]._apply_image(img)
        return img


class Pad(BaseTransform):
    def __init__(self, padding, fill=0, padding_mode='constant', keys=None):
        super().__init__(keys)
        self.padding, self.fill, self.padding_mode = padding, fill, padding_mode

    def _apply_image(self, img):
        return F.pad(img, self.padding, self.fill, self.padding_mode)


class RandomRotation(BaseTransform):
    def __init__(self, degrees, interpolation='nearest', expand=False, center=None, fill=0,
                 keys=None):
        super().__init__(keys)
        self.degrees = (-degrees, degrees) if isinstance(degrees, numbers.Number) else degrees
        self.interpolation, self.expand, self.center, self.fill = interpolation, expand, \
            center, fill

    def _apply_image(self, img):
        return F.rotate(img, random.uniform(*self.degrees), self.interpolation, self.expand,
                        self.center, self.fill)


class RandomAffine(BaseTransform):
    def __init__(self, degrees, translate=None, scale=None, shear=None, interpolation='nearest',
                 fill=0, center=None, keys=None):
        super().__init__(keys)
        self.degrees = (-degrees, degrees) if isinstance(degrees, numbers.Number) else degrees
        self.translate, self.scale, self.interpolation = translate, scale, interpolation
        if shear is not None and isinstance(shear, numbers.Number):
            shear = (-shear, shear)
        self.shear, self.fill, self.center = shear, fill, center

    def _apply_image(self, img):
        h, w = F._size_hw(img)
        angle = random.uniform(*self.degrees)
        if self.translate is not None:
            tx = round(random.uniform(-self.translate[0] * w, self.translate[0] * w))
            ty = round(random.uniform(-self.translate[1] * h, self.translate[1] * h))
        else:
            tx = ty = 0
        sc = random.uniform(*self.scale) if self.scale is not None else 1.0
        sh = (0.0, 0.0)
        if self.shear is not None:
            sh = (random.uniform(self.shear[0], self.shear[1]),
                  random.uniform(self.shear[2], self.shear[3]) if len(self.shear) == 4 else 0.0)
        return F.affine(img, angle, (tx, ty), sc, sh, self.interpolation, self.fill,
                        self.center)


class RandomPerspective(BaseTransform):
    def __init__(self, prob=0.5, distortion_scale=0.5, interpolation='nearest', fill=0,
                 keys=None):
        super().__init__(keys)
        self.prob, self.distortion_scale = prob, distortion_scale
        self.interpolation, self.fill = interpolation, fill

    def _apply_image(self, img):
        if random.random() >= self.prob:
            return img
        h, w = F._size_hw(img)
        dw, dh = int(self.distortion_scale * w / 2), int(self.distortion_scale * h / 2)
        start = [[0, 0], [w - 1, 0], [w - 1, h - 1], [0, h - 1]]
        end = [[random.randint(0, dw), random.randint(0, dh)],
               [w - 1 - random.randint(0, dw), random.randint(0, dh)],
               [w - 1 - random.randint(0, dw), h - 1 - random.randint(0, dh)],
               [random.randint(0, dw), h - 1 - random.randint(0, dh)]]
        return F.perspective(img, start, end, self.interpolation, self.fill)


class Grayscale(BaseTransform):
    def __init__(self, num_output_channels=1, keys=None):
        super().__init__(keys)
        self.num_output_channels = num_output_channels

    def _apply_image(self, img):
        return F.to_grayscale(img, self.num_output_channels)


class RandomErasing(BaseTransform):
    """Erase a random rectangle of a CHW Tensor / HWC array (Zhong et al. 2017)."""

    def __init__(self, prob=0.5, scale=(0.02, 0.33), ratio=(0.3, 3.3), value=0, inplace=False,
                 keys=None):
        super().__init__(keys)
        self.prob, self.scale, self.ratio = prob, scale, ratio
        self.value, self.inplace = value, inplace

    def _apply_image(self, img):
        if random.random() >= self.prob:
            return img
        if isinstance(img, Tensor):
            c, h, w = _u(img).shape[-3:]
        else:
            h, w = np.asarray(img).shape[:2]
            c = np.asarray(img).shape[2] if np.asarray(img).ndim == 3 else 1
        area = h * w
        for _ in range(10):
            ea = random.uniform(*self.scale) * area
            ar = math.exp(random.uniform(math.log(self.ratio[0]), math.log(self.ratio[1])))
            eh, ew = int(round(math.sqrt(ea * ar))), int(round(math.sqrt(ea / ar)))
            if eh < h and ew < w:
                i, j = random.randint(0, h - eh), random.randint(0, w - ew)
                if self.value == 'random':
                    v = np.random.normal(size=(c, eh, ew) if isinstance(img, Tensor)
                                         else (eh, ew, c)).astype(np.float32)
                    if not isinstance(img, Tensor) and np.asarray(img).ndim == 2:
                        v = v[..., 0]
                else:
                    v = self.value
                return F.erase(img, i, j, eh, ew, v, self.inplace)
        return img
