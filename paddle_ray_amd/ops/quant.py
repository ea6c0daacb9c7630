"""Fake-quantization primitives shared by paddle.nn.quant and paddle.quantization
(parity: paddle/phi/kernels/funcs/fake_quantize_functor.cu: fake_quantize_dequantize_abs_max,
..._moving_average_abs_max, fake_channel_wise_quantize_dequantize_abs_max,
quantize_linear / dequantize_linear).

Symmetric uniform quantization with range = 2^(bits-1) - 1:
    q = clip(round(x / scale * range), -range - 1, range),  x_hat = q * scale / range
The backward of a quantize-dequantize is the straight-through estimator (dx = dout), as in
the reference. ``fp8=True`` simulates OCP float8 e4m3 (the MI355X MFMA fp8 format: scale so
that absmax maps to 448, cast through torch.float8_e4m3fn).
"""
import torch

FP8_E4M3_MAX = 448.0


def qrange(bits):
    return float((1 << (bits - 1)) - 1)


def absmax(x, axis=None):
    """max |x| (per channel along ``axis`` if given), fp32, floored at a tiny value."""
    a = x.detach().abs().float()
    if axis is None:
        return a.max().clamp_min(1e-9)
    dims = [d for d in range(x.dim()) if d != axis % x.dim()]
    return a.amax(dim=dims).clamp_min(1e-9)


def _bcast(scale, x, axis):
    if axis is None or scale.dim() == 0 or scale.numel() == 1:
        return scale.reshape(())
    shape = [1] * x.dim()
    shape[axis % x.dim()] = -1
    return scale.reshape(shape)


class _QDQ(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, scale, bits, axis, fp8):
        s = _bcast(scale.to(torch.float32), x, axis)
        xf = x.float()
        if fp8:
            y = (xf / s * FP8_E4M3_MAX).clamp(-FP8_E4M3_MAX, FP8_E4M3_MAX)
            y = y.to(torch.float8_e4m3fn).float() * s / FP8_E4M3_MAX
        else:
            r = qrange(bits)
            y = torch.clamp(torch.round(xf / s * r), -r - 1, r) * s / r
        return y.to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g, None, None, None, None


def fake_quant_dequant(x, scale, bits=8, axis=None, fp8=False):
    """Quantize-dequantize ``x`` with the given scale (straight-through gradient)."""
    if not torch.is_tensor(scale):
        scale = torch.tensor(float(scale), device=x.device)
    return _QDQ.apply(x, scale.to(x.device), int(bits), axis, bool(fp8))


def quantize_linear(x, scale, bits=8, axis=None):
    r = qrange(bits)
    s = _bcast(scale.to(x.device, torch.float32), x, axis)
    return torch.clamp(torch.round(x.float() / s * r), -r - 1, r)


def dequantize_linear(q, scale, bits=8, axis=None):
    r = qrange(bits)
    s = _bcast(scale.to(q.device, torch.float32), q, axis)
    return q.float() * s / r


def moving_average_update(state, accum, cur_absmax, rate):
    """state = rate*state + 1; accum = rate*accum + absmax; returns scale = accum/state."""
    with torch.no_grad():
        state.mul_(rate).add_(1.0)
        accum.mul_(rate).add_(cur_absmax.to(accum.dtype))
        return accum / state
