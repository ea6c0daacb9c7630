"""paddle.utils.cpp_extension: build user operators (host C++ and gfx950 HIP), call them with
autograd and through the kernel registry (parity: python/paddle/utils/cpp_extension/
cpp_extension.py load :800 / setup :79; test/custom_op/test_custom_relu_op_jit.py)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import paddle_ray_amd as paddle
from paddle_ray_amd.utils import cpp_extension

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, 'custom_ops')


def test_host_custom_op_forward_backward(tmp_path):
    mod = cpp_extension.load('pra_test_relu_host', [os.path.join(SRC, 'relu_host.cc')],
                             build_directory=str(tmp_path))
    x = paddle.to_tensor(np.random.RandomState(0).randn(3, 5).astype('float32'), stop_gradient=False)
    y = mod.custom_relu(x)
    np.testing.assert_allclose(y.numpy(), np.maximum(x.numpy(), 0))
    (y * paddle.arange(15, dtype='float32').reshape([3, 5])).sum().backward()
    np.testing.assert_allclose(x.grad.numpy(), (x.numpy() > 0) * np.arange(15).reshape(3, 5))
    # two inputs, two outputs, gradients through both outputs
    a = paddle.to_tensor([1.0, 2.0, 3.0], stop_gradient=False)
    b = paddle.to_tensor([4.0, 5.0, 6.0], stop_gradient=False)
    p, s = mod.custom_mul_add(a, b)
    (p.sum() * 2 + s.sum()).backward()
    np.testing.assert_allclose(a.grad.numpy(), 2 * b.numpy() + 1)
    np.testing.assert_allclose(b.grad.numpy(), 2 * a.numpy() + 1)
    from paddle_ray_amd.ops import registry as R
    assert R.has_kernel('custom.custom_relu', 'ref')
    # rebuilding an unchanged extension reuses the library
    so = mod.__file__
    t0 = os.path.getmtime(so)
    cpp_extension.load('pra_test_relu_host', [os.path.join(SRC, 'relu_host.cc')],
                       build_directory=str(tmp_path))
    assert os.path.getmtime(so) == t0


def test_setup_writes_importable_module(tmp_path):
    cpp_extension.setup(name='pra_test_setup_ops',
                        ext_modules=cpp_extension.CppExtension([os.path.join(SRC, 'relu_host.cc')]),
                        build_directory=str(tmp_path / 'build'), stub_directory=str(tmp_path))
    code = ("import sys; sys.path.insert(0, %r); import numpy as np, paddle_ray_amd as paddle;"
            "import pra_test_setup_ops as m;"
            "print(m.custom_relu(paddle.to_tensor([-1.0, 2.0])).numpy().tolist())") % str(tmp_path)
    r = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True,
                       cwd=os.path.dirname(HERE), env=dict(os.environ, PYTHONPATH=os.path.dirname(HERE)))
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().splitlines()[-1] == '[0.0, 2.0]'


def test_device_extension_builds_for_gfx950(tmp_path):
    """The HIP build compiles for gfx950 on a GPU-less host (hipcc cross-compiles)."""
    mod = cpp_extension.load('pra_test_relu_hip_build', [os.path.join(SRC, 'relu_hip.hip')],
                             build_directory=str(tmp_path))
    assert mod._ops['custom_relu'].device_build
    out = subprocess.run(['/opt/rocm/lib/llvm/bin/llvm-objdump', '--offloading', mod.__file__],
                         capture_output=True, text=True)
    assert 'gfx950' in out.stdout + out.stderr or out.returncode != 0


@pytest.mark.gpu
def test_hip_custom_op_forward_backward(tmp_path):
    paddle.set_device('gpu')
    mod = cpp_extension.load('pra_test_relu_hip', [os.path.join(SRC, 'relu_hip.hip')],
                             build_directory=str(tmp_path))
    for dt in ('float32', 'bfloat16'):
        x = paddle.randn([64, 33]).astype(dt)
        x.stop_gradient = False
        y = mod.custom_relu(x)
        ref = np.maximum(x.astype('float32').numpy(), 0)
        np.testing.assert_allclose(y.astype('float32').numpy(), ref)
        g = paddle.randn([64, 33]).astype(dt)
        (y * g).sum().backward()
        np.testing.assert_allclose(x.grad.astype('float32').numpy(),
                                   (ref > 0) * g.astype('float32').numpy(), rtol=1e-6)
    from paddle_ray_amd.ops import registry as R
    assert R.has_kernel('custom.custom_relu', 'hip')
