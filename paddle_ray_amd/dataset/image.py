"""Legacy image helpers (parity: python/paddle/dataset/image.py): HWC numpy images, PIL
decoding (OpenCV is not installed here)."""
import io

import numpy as np

__all__ = []


def load_image_bytes(bytes, is_color=True):  # noqa: A002 (reference signature)
    from PIL import Image
    img = Image.open(io.BytesIO(bytes)).convert('RGB' if is_color else 'L')
    a = np.asarray(img)
    return a[:, :, ::-1].copy() if is_color else a  # BGR like cv2.imdecode


def load_image(file, is_color=True):
    with open(file, 'rb') as f:
        return load_image_bytes(f.read(), is_color)


def resize_short(im, size):
    from ..vision.transforms import functional as F
    return F.resize(im, size, 'bilinear')


def to_chw(im, order=(2, 0, 1)):
    assert len(im.shape) == len(order)
    return im.transpose(order)


def center_crop(im, size, is_color=True):
    h, w = im.shape[:2]
    hs, ws = (h - size) // 2, (w - size) // 2
    return im[hs:hs + size, ws:ws + size]


def random_crop(im, size, is_color=True):
    h, w = im.shape[:2]
    hs, ws = np.random.randint(0, h - size + 1), np.random.randint(0, w - size + 1)
    return im[hs:hs + size, ws:ws + size]


def left_right_flip(im, is_color=True):
    return im[:, ::-1]


def simple_transform(im, resize_size, crop_size, is_train, is_color=True, mean=None):
    im = resize_short(im, resize_size)
    if is_train:
        im = random_crop(im, crop_size, is_color)
        if np.random.randint(2) == 0:
            im = left_right_flip(im, is_color)
    else:
        im = center_crop(im, crop_size, is_color)
    if im.ndim == 3:
        im = to_chw(im)
    im = im.astype('float32')
    if mean is not None:
        mean = np.array(mean, dtype=np.float32)
        if mean.ndim == 1 and is_color:
            mean = mean[:, None, None]
        im -= mean
    return im


def load_and_transform(filename, resize_size, crop_size, is_train, is_color=True, mean=None):
    return simple_transform(load_image(filename, is_color), resize_size, crop_size, is_train,
                            is_color, mean)
