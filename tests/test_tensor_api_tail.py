"""Tensor-API names the reference exports that were missing (parity:
python/paddle/tensor/__init__.py tensor_method_func, python/paddle/__init__.py __all__):
rank, create_tensor and the in-place erfinv_ / remainder_ / lerp_ / put_along_axis_."""
import re

import numpy as np
import torch

import paddle_ray_amd as paddle


def test_rank_and_create_tensor():
    x = paddle.to_tensor(np.zeros((2, 3, 4), np.float32))
    r = paddle.rank(x)
    assert int(r) == 3 and r.dtype in (paddle.int32, torch.int32)
    t = paddle.create_tensor('float32')
    assert t.shape == [0] or tuple(t.shape) == (0,)
    paddle.assign(paddle.to_tensor([1.0, 2.0]), t)
    np.testing.assert_allclose(t.numpy(), [1.0, 2.0])


def test_inplace_variants_match_out_of_place():
    a = np.array([0.1, -0.5, 0.9], np.float32)
    ref = torch.erfinv(torch.tensor(a.copy())).numpy()
    x = paddle.to_tensor(a.copy())
    y = x.erfinv_()
    assert y is x
    np.testing.assert_allclose(x.numpy(), ref, rtol=1e-6)
    x = paddle.to_tensor(np.array([5.0, -5.0, 7.5], np.float32))
    x.remainder_(paddle.to_tensor(np.array([3.0, 3.0, 2.0], np.float32)))
    np.testing.assert_allclose(x.numpy(), [2.0, 1.0, 1.5])          # floor-mod sign rule
    x = paddle.to_tensor(np.array([0.0, 10.0], np.float32))
    x.lerp_(paddle.to_tensor(np.array([10.0, 20.0], np.float32)), 0.25)
    np.testing.assert_allclose(x.numpy(), [2.5, 12.5])
    arr = paddle.to_tensor(np.zeros((2, 3), np.float32))
    idx = paddle.to_tensor(np.array([[2], [0]], np.int64))
    out = arr.put_along_axis_(idx, 7.0, 1)
    assert out is arr
    np.testing.assert_allclose(arr.numpy(), [[0, 0, 7], [7, 0, 0]])


def test_reference_tensor_method_names_present():
    src = open('/root/reference/python/paddle/tensor/__init__.py').read() \
        if __import__('os').path.exists('/root/reference/python/paddle/tensor/__init__.py') else None
    if src is None:
        return
    m = re.search(r"tensor_method_func\s*=\s*\[(.*?)\]", src, re.S)
    names = re.findall(r"'(\w+)'", m.group(1))
    missing = [n for n in names if not hasattr(paddle, n) and not hasattr(paddle.Tensor, n)]
    assert missing == [], missing
