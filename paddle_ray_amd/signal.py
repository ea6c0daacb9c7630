"""paddle.signal (parity: python/paddle/signal.py; kernels paddle/phi/kernels/funcs/frame_functor.h,
overlap_add_kernel).

Built on the framework's own pieces rather than torch.stft:

* ``frame`` is a strided view (no copy): frame ``f`` of axis ``-1`` starts at ``f * hop``; the
  output is ``[..., frame_length, num_frames]`` for ``axis=-1`` and ``[num_frames, frame_length,
  ...]`` for ``axis=0``, as the reference lays it out.
* ``overlap_add`` is its adjoint: one scatter-add of every frame sample into its output position
  (a single index_add over a precomputed position table, differentiable).
* ``stft`` = optional centre padding (reflect / constant) -> frame -> window -> the ``fft_r2c``
  (real input) or ``fft_c2c`` (complex input) primitive of ``paddle.fft``; ``istft`` = inverse
  ``fft_c2r`` / ``fft_c2c`` -> window -> overlap_add, divided by the overlap-added squared window
  (least-squares inverse), with the reference's NOLA check.
"""
import torch

from .framework.core import Tensor, _u
from . import fft as _fft

__all__ = ['frame', 'overlap_add', 'stft', 'istft']


def _check_axis(axis):
    if axis not in (0, -1):
        raise ValueError(f'Unexpected axis: {axis}. It should be 0 or -1.')


def _frame(t, frame_length, hop_length, axis):
    if axis == 0:
        # [seq, ...] -> [num_frames, frame_length, ...]
        return _frame(t.movedim(0, -1), frame_length, hop_length, -1).movedim(-1, 0).movedim(-1, 1)
    n = t.shape[-1]
    nf = 1 + (n - frame_length) // hop_length
    st = list(t.stride())
    # [..., num_frames, frame_length] as a view, then frame_length before num_frames
    v = t.as_strided(tuple(t.shape[:-1]) + (nf, frame_length), tuple(st[:-1]) + (st[-1] * hop_length, st[-1]),
                     t.storage_offset())
    return v.transpose(-1, -2)


def frame(x, frame_length, hop_length, axis=-1, name=None):
    """Slice ``x`` into overlapping frames of ``frame_length`` every ``hop_length`` samples."""
    _check_axis(axis)
    if not isinstance(frame_length, int) or frame_length <= 0:
        raise ValueError(f'Unexpected frame_length: {frame_length}. It should be an positive integer.')
    if not isinstance(hop_length, int) or hop_length <= 0:
        raise ValueError(f'Unexpected hop_length: {hop_length}. It should be an positive integer.')
    t = _u(x)
    if frame_length > t.shape[axis]:
        raise ValueError(f'Attribute frame_length should be less equal than sequence length, '
                         f'but got ({frame_length}) > ({t.shape[axis]}).')
    return Tensor(_frame(t, frame_length, hop_length, axis))


def _overlap_add(t, hop_length, axis):
    if axis == 0:
        # [num_frames, frame_length, ...] -> [seq, ...]
        return _overlap_add(t.movedim(1, -1).movedim(0, -1), hop_length, -1).movedim(-1, 0)
    fl, nf = t.shape[-2], t.shape[-1]
    n = (nf - 1) * hop_length + fl
    pos = (torch.arange(nf, device=t.device) * hop_length)[None, :] + torch.arange(fl, device=t.device)[:, None]
    lead = t.shape[:-2]
    flat = t.reshape(-1, fl * nf)
    out = flat.new_zeros(flat.shape[0], n).index_add(1, pos.reshape(-1), flat)
    return out.reshape(tuple(lead) + (n,))


def overlap_add(x, hop_length, axis=-1, name=None):
    """Sum overlapping frames back into a sequence (the adjoint of ``frame``)."""
    _check_axis(axis)
    if not isinstance(hop_length, int) or hop_length <= 0:
        raise ValueError(f'Unexpected hop_length: {hop_length}. It should be an positive integer.')
    return Tensor(_overlap_add(_u(x), hop_length, axis))


def _center_window(w, win_length, n_fft):
    if win_length < n_fft:
        left = (n_fft - win_length) // 2
        w = torch.nn.functional.pad(w, (left, n_fft - win_length - left))
    return w


def stft(x, n_fft, hop_length=None, win_length=None, window=None, center=True, pad_mode='reflect',
         normalized=False, onesided=True, name=None):
    """Short-time Fourier transform: ``[..., seq]`` (1-D or 2-D) -> ``[..., n_fft//2+1 | n_fft,
    num_frames]`` complex."""
    t = _u(x)
    rank = t.dim()
    assert rank in (1, 2), f'x should be a 1D or 2D real tensor, but got rank of x is {rank}'
    if rank == 1:
        t = t.unsqueeze(0)
    hop_length = n_fft // 4 if hop_length is None else hop_length
    assert hop_length > 0, f'hop_length should be > 0, but got {hop_length}.'
    win_length = n_fft if win_length is None else win_length
    assert 0 < n_fft <= t.shape[-1], f'n_fft should be in (0, seq_length({t.shape[-1]})], but got {n_fft}.'
    assert 0 < win_length <= n_fft, f'win_length should be in (0, n_fft({n_fft})], but got {win_length}.'
    if window is not None:
        w = _u(window)
        assert w.dim() == 1 and w.shape[0] == win_length, \
            f'expected a 1D window tensor of size equal to win_length({win_length}), but got window with shape {list(w.shape)}.'
    else:
        w = torch.ones(win_length, dtype=t.real.dtype if t.is_complex() else t.dtype, device=t.device)
    w = _center_window(w.to(t.device), win_length, n_fft)
    if center:
        assert pad_mode in ('constant', 'reflect'), \
            f'pad_mode should be "reflect" or "constant", but got "{pad_mode}".'
        p = n_fft // 2
        if t.is_complex():
            t = torch.complex(*(torch.nn.functional.pad(c.unsqueeze(1), (p, p), mode=pad_mode).squeeze(1)
                                for c in (t.real, t.imag)))
        else:
            t = torch.nn.functional.pad(t.unsqueeze(1), (p, p), mode=pad_mode).squeeze(1)
    frames = _frame(t, n_fft, hop_length, -1).transpose(-1, -2) * w      # [batch, num_frames, n_fft]
    norm = 'ortho' if normalized else 'backward'
    if frames.is_complex():
        assert not onesided, 'onesided should be False when input or window is a complex Tensor.'
        out = _fft.fft_c2c_op(Tensor(frames), [frames.dim() - 1], None, norm, True)
    else:
        out = _fft.fft_r2c_op(Tensor(frames), [frames.dim() - 1], None, norm, True, onesided)
    o = _u(out).transpose(-1, -2)
    return Tensor(o.squeeze(0) if rank == 1 else o)


def istft(x, n_fft, hop_length=None, win_length=None, window=None, center=True, normalized=False,
          onesided=True, length=None, return_complex=False, name=None):
    """Least-squares inverse of ``stft`` (requires the NOLA condition of the window / hop)."""
    t = _u(x)
    assert t.is_complex(), "istft expects a complex STFT tensor"
    rank = t.dim()
    assert rank in (2, 3), f'x should be a 2D or 3D complex tensor, but got rank of x is {rank}'
    if rank == 2:
        t = t.unsqueeze(0)
    hop_length = n_fft // 4 if hop_length is None else hop_length
    win_length = n_fft if win_length is None else win_length
    assert 0 < hop_length <= win_length, \
        f'hop_length should be in (0, win_length({win_length})], but got {hop_length}.'
    assert 0 < win_length <= n_fft, f'win_length should be in (0, n_fft({n_fft})], but got {win_length}.'
    n_frames, fft_size = t.shape[-1], t.shape[-2]
    if onesided:
        assert fft_size == n_fft // 2 + 1, \
            f'fft_size should be equal to n_fft // 2 + 1({n_fft // 2 + 1}) when onesided is True, but got {fft_size}.'
    else:
        assert fft_size == n_fft, f'fft_size should be equal to n_fft({n_fft}) when onesided is False, but got {fft_size}.'
    if window is not None:
        w = _u(window)
        assert w.dim() == 1 and w.shape[0] == win_length, \
            f'expected a 1D window tensor of size equal to win_length({win_length}), but got window with shape {list(w.shape)}.'
    else:
        w = torch.ones(win_length, dtype=torch.float32 if t.dtype == torch.complex64 else torch.float64,
                       device=t.device)
    w = _center_window(w.to(t.device), win_length, n_fft)
    fr = t.transpose(-1, -2)                                             # [batch, num_frames, fft_size]
    norm = 'ortho' if normalized else 'backward'
    if return_complex:
        assert not onesided, 'onesided should be False when input(output of istft) or window is a complex Tensor.'
        out = _u(_fft.fft_c2c_op(Tensor(fr), [2], None, norm, False))
    else:
        assert not w.is_complex(), 'Data type of window should not be complex when return_complex is False.'
        if not onesided:
            fr = fr[:, :, :n_fft // 2 + 1]
        out = _u(_fft.fft_c2r_op(Tensor(fr), [2], None, norm, False, n_fft))
    out = _overlap_add((out * w).transpose(-1, -2), hop_length, -1)      # [batch, seq]
    env = _overlap_add((w * w)[:, None].expand(n_fft, n_frames), hop_length, -1)
    start = n_fft // 2 if center else 0
    if length is None:
        if center:
            out, env = out[:, start:-start], env[start:-start]
    else:
        out, env = out[:, start:start + length], env[start:start + length]
    if float(env.abs().min()) < 1e-11:
        raise ValueError('Abort istft because Nonzero Overlap Add (NOLA) condition failed.')
    out = out / env
    return Tensor(out.squeeze(0) if rank == 2 else out)
