"""paddle.signal: frame / overlap_add layouts from the reference's docstring examples, stft vs
torch.stft, istft round trips, gradients and argument errors (parity targets:
python/paddle/signal.py, test_signal.py / test_stft_op.py)."""
import numpy as np
import pytest
import torch

import paddle_ray_amd as paddle
from paddle_ray_amd import signal as S


def test_frame_layouts():
    x = paddle.to_tensor(np.arange(8))
    np.testing.assert_array_equal(S.frame(x, 4, 2, axis=-1).numpy(), [[0, 2, 4], [1, 3, 5], [2, 4, 6], [3, 5, 7]])
    np.testing.assert_array_equal(S.frame(x, 4, 2, axis=0).numpy(), [[0, 1, 2, 3], [2, 3, 4, 5], [4, 5, 6, 7]])
    x0 = paddle.to_tensor(np.arange(16).reshape(2, 8))
    y0 = S.frame(x0, 4, 2, axis=-1).numpy()
    assert y0.shape == (2, 4, 3) and y0[1, 2, 0] == 10
    x1 = paddle.to_tensor(np.arange(16).reshape(8, 2))
    y1 = S.frame(x1, 4, 2, axis=0).numpy()
    assert y1.shape == (3, 4, 2)
    np.testing.assert_array_equal(y1[1], [[4, 5], [6, 7], [8, 9], [10, 11]])
    assert S.frame(paddle.to_tensor(np.arange(32).reshape(8, 2, 2)), 4, 2, axis=0).shape == [3, 4, 2, 2]


def test_overlap_add_layouts():
    x0 = paddle.to_tensor(np.arange(16).reshape(8, 2))
    np.testing.assert_array_equal(S.overlap_add(x0, 2, axis=-1).numpy(), [0, 2, 5, 9, 13, 17, 21, 25, 13, 15])
    x1 = paddle.to_tensor(np.arange(16).reshape(2, 8))
    np.testing.assert_array_equal(S.overlap_add(x1, 2, axis=0).numpy(), [0, 1, 10, 12, 14, 16, 18, 20, 14, 15])
    assert S.overlap_add(paddle.to_tensor(np.arange(32).reshape(2, 1, 8, 2)), 2, axis=-1).shape == [2, 1, 10]
    assert S.overlap_add(paddle.to_tensor(np.arange(32).reshape(2, 8, 1, 2)), 2, axis=0).shape == [10, 1, 2]


def test_overlap_add_is_adjoint_of_frame():
    torch.manual_seed(0)
    x = torch.randn(3, 50, dtype=torch.float64, requires_grad=True)
    f = S.frame(paddle.Tensor(x), 8, 3)._t
    g = torch.randn_like(f)
    (f * g).sum().backward()
    np.testing.assert_allclose(x.grad.numpy(), S.overlap_add(paddle.Tensor(g), 3).numpy()[:, :50], rtol=1e-12)


@pytest.mark.parametrize('center,pad_mode,normalized,onesided,win', [
    (True, 'reflect', False, True, None), (False, 'constant', True, False, 'hann'), (True, 'constant', False, True, 'short')])
def test_stft_matches_torch(center, pad_mode, normalized, onesided, win):
    torch.manual_seed(1)
    x = torch.randn(2, 400, dtype=torch.float64)
    n_fft, hop = 64, 16
    wl = 48 if win == 'short' else n_fft
    w = None if win is None else torch.hann_window(wl, dtype=torch.float64)
    got = S.stft(paddle.Tensor(x), n_fft, hop, wl, None if w is None else paddle.Tensor(w), center, pad_mode,
                 normalized, onesided).numpy()
    ref = torch.stft(x, n_fft, hop, wl, w, center, pad_mode, normalized, onesided, return_complex=True).numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-9)


def test_stft_complex_and_1d():
    torch.manual_seed(2)
    xc = torch.randn(300, dtype=torch.complex128)
    got = S.stft(paddle.Tensor(xc), 32, 8, center=False, onesided=False).numpy()
    ref = torch.stft(xc, 32, 8, center=False, onesided=False, return_complex=True).numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-9)
    with pytest.raises(AssertionError):
        S.stft(paddle.Tensor(xc), 32, 8, center=False, onesided=True)


@pytest.mark.parametrize('onesided,center,length', [(True, True, None), (False, True, 390), (True, False, None)])
def test_istft_round_trip(onesided, center, length):
    torch.manual_seed(3)
    x = torch.randn(2, 400, dtype=torch.float64)
    w = torch.hann_window(64, dtype=torch.float64) + 0.1
    spec = S.stft(paddle.Tensor(x), 64, 16, window=paddle.Tensor(w), center=center, onesided=onesided)
    y = S.istft(spec, 64, 16, window=paddle.Tensor(w), center=center, onesided=onesided, length=length).numpy()
    n = y.shape[-1]
    if center:
        np.testing.assert_allclose(y, x.numpy()[:, :n], rtol=1e-9, atol=1e-9)
    else:  # without centre padding the reconstruction covers the framed span
        np.testing.assert_allclose(y[:, 64:n - 64], x.numpy()[:, 64:n - 64], rtol=1e-9, atol=1e-9)
    ref = torch.istft(torch.as_tensor(spec.numpy()), 64, 16, window=w, center=center, onesided=onesided,
                      length=length).numpy()
    if center:
        np.testing.assert_allclose(y, ref[:, :n], rtol=1e-9, atol=1e-9)


def test_istft_nola_and_argument_errors():
    spec = S.stft(paddle.Tensor(torch.randn(200, dtype=torch.float64)), 32, 8)
    with pytest.raises(ValueError, match='NOLA'):
        S.istft(spec, 32, 8, window=paddle.Tensor(torch.zeros(32, dtype=torch.float64)))
    with pytest.raises(ValueError):
        S.frame(paddle.to_tensor(np.arange(8)), 9, 2)
    with pytest.raises(ValueError):
        S.frame(paddle.to_tensor(np.arange(8)), 4, 2, axis=1)
    with pytest.raises(ValueError):
        S.overlap_add(paddle.to_tensor(np.arange(8).reshape(4, 2)), 0)
