"""paddle.fft against numpy.fft / scipy.fft (parity targets: python/paddle/fft.py and the
reference's test_fft.py / test_fft_with_static_graph.py: every transform x norm, n/s/axes
padding and cropping, argument errors, frequency helpers, shifts, gradients, static recording)."""
import numpy as np
import pytest
import scipy.fft as sf
import torch

import paddle_ray_amd as paddle
from paddle_ray_amd import fft as F

RS = np.random.RandomState(0)
XR = RS.randn(4, 6, 5)
XC = XR + 1j * RS.randn(4, 6, 5)
NORMS = ['backward', 'forward', 'ortho']


def _t(a):
    return paddle.to_tensor(a)


@pytest.mark.parametrize('norm', NORMS)
@pytest.mark.parametrize('name,x,kw', [
    ('fft', XC, dict(n=7, axis=1)), ('fft', XR, dict(n=4, axis=0)), ('ifft', XC, dict(n=3, axis=-1)),
    ('rfft', XR, dict(n=8, axis=1)), ('irfft', XC, dict(n=7, axis=-1)), ('irfft', XC, dict()),
    ('hfft', XC, dict(n=9, axis=0)), ('ihfft', XR, dict(axis=2)),
])
def test_1d_against_numpy(name, x, kw, norm):
    got = getattr(F, name)(_t(x), norm=norm, **kw).numpy()
    ref = getattr(np.fft, name)(x, norm=norm, **kw)
    np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize('norm', NORMS)
@pytest.mark.parametrize('name,x,kw', [
    ('fftn', XC, dict()), ('fftn', XC, dict(s=(3, 8), axes=(2, 0))), ('ifftn', XC, dict(s=(5, 4))),
    ('rfftn', XR, dict(axes=(0, 2))), ('rfftn', XR, dict(s=(3, 8), axes=(2, 0))),
    ('irfftn', XC, dict(s=(6, 7))), ('irfftn', XC, dict(axes=(1, 0))),
    ('hfftn', XC, dict(s=(4, 6), axes=(0, 1))), ('ihfftn', XR, dict(axes=(0, 1, 2))),
    ('fft2', XC, dict()), ('ifft2', XC, dict(s=(3, 3))), ('rfft2', XR, dict(axes=(0, 1))),
    ('irfft2', XC, dict(s=(5, 8))), ('hfft2', XC, dict()), ('ihfft2', XR, dict(axes=(1, 2))),
])
def test_nd_against_scipy(name, x, kw, norm):
    got = getattr(F, name)(_t(x), norm=norm, **kw).numpy()
    ref = getattr(sf, name)(x, norm=norm, **kw)
    np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-9)


def test_integer_and_float32_promotion():
    xi = np.arange(8)
    y = F.fft(_t(xi))
    assert y.dtype == paddle.complex64 or 'complex64' in str(y.dtype)
    np.testing.assert_allclose(y.numpy(), np.fft.fft(xi), rtol=1e-5, atol=1e-4)
    y32 = F.rfft(_t(XR.astype('float32')))
    assert 'complex64' in str(y32.dtype)


@pytest.mark.parametrize('call,msg', [
    (lambda: F.fft(_t(XC), norm='bad'), 'Unexpected norm'),
    (lambda: F.fft(_t(XC), n=0), 'positive'),
    (lambda: F.fft(_t(XC), n=2.5), 'integer'),
    (lambda: F.fft(_t(XC), axis=3), 'axis'),
    (lambda: F.fftn(_t(XC), s=(1, 2, 3, 4)), 'larger than the rank'),
    (lambda: F.fftn(_t(XC), s=(2, -1)), 'invalid value'),
    (lambda: F.fftn(_t(XC), axes=(0, 5)), 'invalid value'),
    (lambda: F.fftn(_t(XC), s=(2, 3), axes=(0,)), 'does not match'),
    (lambda: F.fft2(_t(XC[0, 0])), 'should >= 2'),
    (lambda: F.fft2(_t(XC), s=(2,)), 'sequence of 2'),
    (lambda: F.fftfreq(0), 'should not be 0'),
])
def test_argument_errors(call, msg):
    with pytest.raises(ValueError, match=msg):
        call()


def test_rfft_rejects_complex():
    with pytest.raises(TypeError):
        F.rfft(_t(XC))


def test_freq_and_shift():
    for n in (5, 8):
        np.testing.assert_allclose(F.fftfreq(n, 0.3).numpy(), np.fft.fftfreq(n, 0.3), rtol=1e-6)
        np.testing.assert_allclose(F.rfftfreq(n, 0.3).numpy(), np.fft.rfftfreq(n, 0.3), rtol=1e-6)
        v = np.fft.fftfreq(n)
        np.testing.assert_allclose(F.fftshift(_t(v)).numpy(), np.fft.fftshift(v))
        np.testing.assert_allclose(F.ifftshift(_t(v)).numpy(), np.fft.ifftshift(v))
        np.testing.assert_allclose(F.ifftshift(F.fftshift(_t(v))).numpy(), v)
    assert F.fftfreq(4, dtype='float64').numpy().dtype == np.float64
    np.testing.assert_allclose(F.fftshift(_t(XR), axes=(0, 2)).numpy(), np.fft.fftshift(XR, axes=(0, 2)))
    np.testing.assert_allclose(F.ifftshift(_t(XR), axes=1).numpy(), np.fft.ifftshift(XR, axes=1))


def test_gradients_through_primitives():
    """d/dx sum(|rfft(x)|^2) by autograd through fft_r2c equals the analytic Parseval weights."""
    x = torch.tensor(RS.randn(8), dtype=torch.float64, requires_grad=True)
    xp = paddle.to_tensor(x.detach().numpy(), stop_gradient=False)
    y = F.fft(xp)
    (y.abs() ** 2).sum().backward()
    # sum |fft(x)|^2 = n * sum x^2  ->  grad = 2 n x
    np.testing.assert_allclose(xp.grad.numpy(), 2 * 8 * x.detach().numpy(), rtol=1e-10)
    xc = paddle.to_tensor(XC[0], stop_gradient=False)
    z = F.irfft(F.rfft(F.ifft(F.fft(xc)).real()))
    z.sum().backward()
    assert xc.grad is not None


def test_registry_dispatch_and_static_recording():
    from paddle_ray_amd.ops import registry as R
    R.reset_stats()
    F.hfft(_t(XC))
    F.ihfftn(_t(XR))
    F.fft2(_t(XC))
    st = R.stats()
    assert st[('fft_c2r', 'ref')] == 1 and st[('fft_r2c', 'ref')] == 1 and st[('fft_c2c', 'ref')] == 1
    paddle.enable_static()
    try:
        main, start = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, start):
            x = paddle.static.data('x', [4, 6, 5], 'float64')
            y = F.rfftn(x, s=(3, 8), axes=(2, 0), norm='ortho')
            z = F.irfft(y, n=6)
        types = [op.type for op in main.global_block().ops]
        assert 'fft_r2c' in types and 'fft_c2r' in types
        exe = paddle.static.Executor()
        exe.run(start)
        out_y, out_z = exe.run(main, feed={'x': XR}, fetch_list=[y, z])
    finally:
        paddle.disable_static()
    ref_y = sf.rfftn(XR, s=(3, 8), axes=(2, 0), norm='ortho')
    np.testing.assert_allclose(out_y, ref_y, rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(out_z, np.fft.irfft(ref_y, n=6), rtol=1e-9, atol=1e-9)
