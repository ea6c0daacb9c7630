"""Viterbi decoding of a linear-chain CRF (parity: python/paddle/text/viterbi_decode.py,
paddle/phi/kernels/cpu/viterbi_decode_kernel.cc). Batched on the tensor's device: one
[B, N, N] max/argmax per time step, then a gather back-trace; sequences shorter than the
batch maximum keep their scores frozen after their last step and pad the path with 0.

With ``include_bos_eos_tag`` the last row of ``transition_params`` is the start (BOS)
transition and the second-to-last row the stop (EOS) transition."""
import torch

from ..framework.core import Tensor, _u
from .. import nn


def viterbi_decode(potentials, transition_params, lengths, include_bos_eos_tag=True, name=None):
    pot, trans = _u(potentials), _u(transition_params)
    left = _u(lengths).to(device=pot.device, dtype=torch.int64).clone()
    B, L, N = pot.shape
    max_len = int(left.max().item()) if B else 0
    x = pot.transpose(0, 1)
    stop = trans[N - 2] if include_bos_eos_tag else None
    if include_bos_eos_tag:
        alpha = x[0] + trans[N - 1]
        alpha = alpha + stop * (left == 1).unsqueeze(1).to(alpha.dtype)
    else:
        alpha = x[0].clone()
    left = left - 1
    hist = []
    for i in range(1, max_len):
        cand = alpha.unsqueeze(2) + trans.unsqueeze(0)        # [B, from, to]
        best, arg = cand.max(1)
        hist.append(arg)
        m = (left > 0).unsqueeze(1).to(alpha.dtype)
        alpha = (best + x[i]) * m + alpha * (1 - m)
        if include_bos_eos_tag:
            alpha = alpha + stop * (left == 1).unsqueeze(1).to(alpha.dtype)
        left = left - 1
    scores, last = alpha.max(1)
    actual = min(L, max_len)
    path = torch.zeros(max(max_len, 0), B, dtype=torch.int64, device=pot.device)
    if actual > 0:
        path[actual - 1] = last * (left >= 0).to(torch.int64)
    pos = actual - 1
    for h in reversed(hist):
        pos -= 1
        left = left + 1
        upd = h.gather(1, last.unsqueeze(1)).squeeze(1) * (left > 0).to(torch.int64)
        zero = (left == 0).to(torch.int64)
        upd = upd * (1 - zero) + last * zero
        path[pos] = upd
        # still past this sequence's end: keep its final tag for the step that reaches it
        last = last * (left < 0).to(torch.int64) + upd
    return Tensor(scores), Tensor(path.t().contiguous())


class ViterbiDecoder(nn.Layer):
    def __init__(self, transitions, include_bos_eos_tag=True, name=None):
        super().__init__()
        self.transitions = transitions
        self.include_bos_eos_tag = include_bos_eos_tag
        self.name = name

    def forward(self, potentials, lengths):
        return viterbi_decode(potentials, self.transitions, lengths, self.include_bos_eos_tag,
                              self.name)
