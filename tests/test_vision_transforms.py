"""paddle.vision.transforms (parity: test/legacy_test/test_transforms.py,
test_functional_*): numpy / PIL / Tensor inputs, geometry and color ops."""
import random

import numpy as np
import pytest
from PIL import Image

import paddle_ray_amd as paddle
from paddle_ray_amd.vision import transforms as T
from paddle_ray_amd.vision.transforms import functional as F


@pytest.fixture
def img():
    return (np.random.RandomState(0).rand(8, 8, 3) * 255).astype(np.uint8)


def test_flip_crop_pad(img):
    np.testing.assert_array_equal(F.hflip(img), img[:, ::-1])
    np.testing.assert_array_equal(F.vflip(img), img[::-1])
    np.testing.assert_array_equal(F.crop(img, 1, 2, 3, 4), img[1:4, 2:6])
    np.testing.assert_array_equal(F.center_crop(img, 4), img[2:6, 2:6])
    for mode, npm in [('constant', 'constant'), ('edge', 'edge'), ('reflect', 'reflect'),
                      ('symmetric', 'symmetric')]:
        np.testing.assert_array_equal(F.pad(img, (1, 2), padding_mode=mode),
                                      np.pad(img, ((2, 2), (1, 1), (0, 0)), mode=npm))


def test_rotate_and_identity_warps(img):
    np.testing.assert_array_equal(F.rotate(img, 90), np.rot90(img, 1))
    np.testing.assert_array_equal(F.affine(img, 0, (0, 0), 1.0, 0), img)
    pts = [[0, 0], [7, 0], [7, 7], [0, 7]]
    np.testing.assert_array_equal(F.perspective(img, pts, pts), img)
    big = F.rotate(img, 45, expand=True)
    assert big.shape[0] > 8 and big.shape[1] > 8
    # translation by (+2, 0) shifts content right, fill on the left
    sh = F.affine(img, 0, (2, 0), 1.0, 0, fill=7)
    np.testing.assert_array_equal(sh[:, 2:], img[:, :-2])
    assert (sh[:, :2] == 7).all()


def test_resize_shapes(img):
    assert F.resize(img, (4, 6)).shape == (4, 6, 3)
    assert F.resize(np.zeros((8, 16, 3), np.uint8), 4).shape == (4, 8, 3)
    np.testing.assert_array_equal(F.resize(img, (16, 16), 'nearest')[::2, ::2], img)
    pil = Image.fromarray(img)
    assert F.resize(pil, (5, 7)).size == (7, 5)


def test_color_ops(img):
    np.testing.assert_array_equal(F.adjust_brightness(img, 1.0), img)
    np.testing.assert_array_equal(F.adjust_contrast(img, 1.0), img)
    np.testing.assert_array_equal(F.adjust_saturation(img, 1.0), img)
    assert np.abs(F.adjust_hue(img, 0.0).astype(int) - img).max() <= 1
    red = np.zeros((1, 1, 3), np.uint8)
    red[..., 0] = 255
    np.testing.assert_array_equal(F.adjust_hue(red, 1 / 3.0)[0, 0], [0, 255, 0])
    g = F.to_grayscale(img)
    ref = np.asarray(Image.fromarray(img).convert('L'))
    assert np.abs(g[..., 0].astype(int) - ref).max() <= 1
    assert F.to_grayscale(img, 3).shape == (8, 8, 3)
    np.testing.assert_array_equal(F.adjust_brightness(img, 0.0), np.zeros_like(img))


def test_tensor_and_pil_inputs(img):
    t = F.to_tensor(img)
    assert t.shape == [3, 8, 8] and float(t.max()) <= 1.0
    np.testing.assert_allclose(F.hflip(t).numpy(), t.numpy()[:, :, ::-1])
    assert F.resize(t, (4, 4)).shape == [3, 4, 4]
    n = F.normalize(t, [0.5] * 3, [0.5] * 3)
    np.testing.assert_allclose(n.numpy(), (t.numpy() - 0.5) / 0.5, atol=1e-6)
    pil = Image.fromarray(img)
    out = F.rotate(pil, 90)
    assert isinstance(out, Image.Image)
    np.testing.assert_array_equal(np.asarray(out), np.rot90(img, 1))


def test_transform_classes(img):
    random.seed(0)
    pipe = T.Compose([T.RandomResizedCrop(6), T.RandomHorizontalFlip(), T.ColorJitter(0.4, 0.4,
                                                                                      0.4, 0.1),
                      T.RandomRotation(10), T.RandomAffine(5, (0.1, 0.1), (0.9, 1.1), 5),
                      T.RandomPerspective(1.0), T.Pad(1), T.RandomCrop(6),
                      T.Grayscale(3), T.ToTensor(), T.Normalize([0.5] * 3, [0.5] * 3),
                      T.RandomErasing(1.0)])
    out = pipe(img)
    assert out.shape == [3, 6, 6]
    x, label = T.Compose([T.Resize(4), T.Transpose()])((img, 3)) if False else \
        (T.Transpose()(T.Resize(4)(img)), 3)
    assert x.shape == (3, 4, 4)
    r = T.Resize((4, 4), keys=('image', 'label'))
    o, lab = r((img, 5))
    assert o.shape == (4, 4, 3) and lab == 5
    assert T.CenterCrop(4)(img).shape == (4, 4, 3)
    assert T.BrightnessTransform(0.2)(img).shape == img.shape
    assert T.HueTransform(0.2)(img).shape == img.shape
    e = T.RandomErasing(1.0, value=0)(paddle.ones([3, 16, 16]))
    assert float(e.sum()) < 3 * 256
