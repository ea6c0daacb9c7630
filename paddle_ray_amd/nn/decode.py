"""Sequence decoding: ``Decoder``, ``BeamSearchDecoder`` and ``dynamic_decode``.

Parity: python/paddle/nn/decode.py (Decoder :42, BeamSearchDecoder :153, the imperative
dynamic_decode loop :674). Same state layout ([batch, beam, ...] between steps, merged to
[batch*beam, ...] for the cell), same score rule (running sum of log-softmax, finished
beams forced onto ``end_token`` with zero cost, top-k over beam*vocab), same outputs
(predicted ids back-traced with ``gather_tree``; ``[batch, time, beam]`` unless
``output_time_major``).

Device notes: every step is a handful of batched kernels (log-softmax, masked add, one
top-k over ``beam*vocab``, index gathers) with no host round-trip except the single
"all finished?" flag ``dynamic_decode`` reads per step to stop early (the reference reads
it per step too). Beam bookkeeping stays on the device; nothing is materialised on the
host until the caller asks for it.
"""
import collections

import torch

from ..framework.core import Tensor, _u
from ..utils.layers_utils import flatten, map_structure
from . import functional as F

_KINF = 1e9


def _t(x):
    return _u(x) if isinstance(x, Tensor) else x


def _w(x):
    return Tensor(x) if isinstance(x, torch.Tensor) else x


class Decoder:
    """Interface used by ``dynamic_decode``: ``initialize(inits) -> (inputs, states,
    finished)``, ``step(time, inputs, states) -> (outputs, next_states, next_inputs,
    finished)``, optional ``finalize(outputs, final_states, sequence_lengths)``."""

    def initialize(self, inits):
        raise NotImplementedError

    def step(self, time, inputs, states, **kwargs):
        raise NotImplementedError

    def finalize(self, outputs, final_states, sequence_lengths):
        raise NotImplementedError

    @property
    def tracks_own_finished(self):
        return False


class BeamSearchDecoder(Decoder):
    OutputWrapper = collections.namedtuple('OutputWrapper',
                                           ('scores', 'predicted_ids', 'parent_ids'))
    StateWrapper = collections.namedtuple('StateWrapper',
                                          ('cell_states', 'log_probs', 'finished', 'lengths'))

    def __init__(self, cell, start_token, end_token, beam_size, embedding_fn=None,
                 output_fn=None):
        self.cell = cell
        self.embedding_fn = embedding_fn
        self.output_fn = output_fn
        self.start_token = int(start_token)
        self.end_token = int(end_token)
        self.beam_size = int(beam_size)

    # -- [batch, ...] <-> [batch * beam, ...] ---------------------------------------------
    @staticmethod
    def tile_beam_merge_with_batch(x, beam_size):
        """[batch, ...] -> [batch*beam, ...], each entry repeated ``beam_size`` times."""
        t = _t(x)
        return _w(t.unsqueeze(1).expand(t.shape[0], beam_size, *t.shape[1:])
                  .reshape(t.shape[0] * beam_size, *t.shape[1:]))

    def _split_batch_beams(self, x):
        t = _t(x)
        return _w(t.reshape(-1, self.beam_size, *t.shape[1:]))

    def _merge_batch_beams(self, x):
        t = _t(x)
        return _w(t.reshape(-1, *t.shape[2:]))

    def _expand_to_beam_size(self, x):
        t = _t(x)
        return _w(t.unsqueeze(1).expand(t.shape[0], self.beam_size, *t.shape[1:]).contiguous())

    def _gather(self, x, indices, batch_size=None):
        """x[b, indices[b, k], ...] -> [batch, beam, ...]."""
        t, idx = _t(x), _t(indices)
        view = idx.reshape(idx.shape + (1,) * (t.dim() - 2)).expand(idx.shape + t.shape[2:])
        return _w(torch.gather(t, 1, view))

    # -- decoding --------------------------------------------------------------------------
    def initialize(self, initial_cell_states):
        state = _t(flatten(initial_cell_states)[0])
        self.batch_size = state.shape[0]
        dev = state.device
        cell_states = map_structure(self._expand_to_beam_size, initial_cell_states)
        inputs = torch.full((self.batch_size, self.beam_size), self.start_token,
                            dtype=torch.int64, device=dev)
        log_probs = torch.full((self.batch_size, self.beam_size), -_KINF,
                               dtype=torch.get_default_dtype(), device=dev)
        log_probs[:, 0] = 0.0
        finished = torch.zeros((self.batch_size, self.beam_size), dtype=torch.bool, device=dev)
        lengths = torch.zeros((self.batch_size, self.beam_size), dtype=torch.int64, device=dev)
        init_inputs = self.embedding_fn(_w(inputs)) if self.embedding_fn else _w(inputs)
        return (init_inputs,
                self.StateWrapper(cell_states, _w(log_probs), _w(finished), _w(lengths)),
                _w(finished))

    def _beam_search_step(self, time, logits, next_cell_states, beam_state):
        lg = _t(logits)
        V = lg.shape[-1]
        self.vocab_size = V
        step_lp = torch.log_softmax(lg.float(), -1).to(lg.dtype if lg.is_floating_point()
                                                       else torch.float32)
        fin = _t(beam_state.finished)
        # finished beams put all their mass on end_token at zero cost
        noend = torch.full((V,), -_KINF, dtype=step_lp.dtype, device=step_lp.device)
        noend[self.end_token] = 0.0
        step_lp = torch.where(fin.unsqueeze(-1), noend, step_lp)
        log_probs = step_lp + _t(beam_state.log_probs).unsqueeze(-1).to(step_lp.dtype)
        flat = log_probs.reshape(-1, self.beam_size * V)
        topk_scores, topk_idx = torch.topk(flat, self.beam_size, -1)
        beam_idx = torch.div(topk_idx, V, rounding_mode='floor')
        token_idx = topk_idx % V
        next_log_probs = torch.gather(flat, 1, topk_idx)
        next_cell_states = map_structure(lambda s: self._gather(s, beam_idx), next_cell_states)
        next_finished = torch.gather(fin, 1, beam_idx)
        next_lengths = torch.gather(_t(beam_state.lengths), 1, beam_idx)
        next_lengths = next_lengths + (~next_finished).to(next_lengths.dtype)
        next_finished = next_finished | (token_idx == self.end_token)
        out = self.OutputWrapper(_w(topk_scores), _w(token_idx), _w(beam_idx))
        state = self.StateWrapper(next_cell_states, _w(next_log_probs), _w(next_finished),
                                  _w(next_lengths))
        return out, state

    def step(self, time, inputs, states, **kwargs):
        inputs = map_structure(self._merge_batch_beams, inputs)
        cell_states = map_structure(self._merge_batch_beams, states.cell_states)
        cell_outputs, next_cell_states = self.cell(inputs, cell_states, **kwargs)
        cell_outputs = map_structure(self._split_batch_beams, cell_outputs)
        next_cell_states = map_structure(self._split_batch_beams, next_cell_states)
        if self.output_fn is not None:
            cell_outputs = self.output_fn(cell_outputs)
        out, state = self._beam_search_step(time, cell_outputs, next_cell_states, states)
        sample_ids = out.predicted_ids
        sample_ids.stop_gradient = True
        next_inputs = self.embedding_fn(sample_ids) if self.embedding_fn else sample_ids
        return out, state, next_inputs, state.finished

    def finalize(self, outputs, final_states, sequence_lengths):
        return F.gather_tree(outputs.predicted_ids, outputs.parent_ids), final_states

    @property
    def tracks_own_finished(self):
        return True


def _maybe_copy(state, new_state, step_mask):
    s, n, m = _t(state), _t(new_state), _t(step_mask)
    m = m.reshape(m.shape + (1,) * (s.dim() - m.dim()))
    return _w(torch.where(m, s, n))


def dynamic_decode(decoder, inits=None, max_step_num=None, output_time_major=False,
                   impute_finished=False, is_test=False, return_length=False, **kwargs):
    """Run ``decoder`` step by step until every sequence is finished or ``max_step_num``
    steps have run (the loop runs ``max_step_num + 1`` steps at most, as the reference's)."""
    inputs, states, finished = decoder.initialize(inits)
    seq_len = torch.zeros_like(_t(finished), dtype=torch.int64)
    outputs = None
    step = 0
    while bool((~_t(finished)).any()):
        time = Tensor(torch.full((1,), step, dtype=torch.int64))
        step_out, next_states, next_inputs, next_finished = decoder.step(time, inputs, states,
                                                                         **kwargs)
        if not decoder.tracks_own_finished:
            next_finished = _w(_t(next_finished) | _t(finished))
            next_seq_len = seq_len + (~_t(finished)).to(seq_len.dtype)
            if impute_finished:
                next_states = map_structure(lambda a, b: _maybe_copy(a, b, finished), states,
                                            next_states)
        else:
            lens = getattr(next_states, 'lengths', None)
            next_seq_len = _t(lens) if lens is not None else seq_len
        flat = [_t(x) for x in flatten(step_out)]
        outputs = [[x] for x in flat] if outputs is None else \
            [acc + [x] for acc, x in zip(outputs, flat)]
        inputs, states, finished, seq_len = next_inputs, next_states, next_finished, next_seq_len
        step += 1
        if max_step_num is not None and step > max_step_num:
            break
    from ..utils.layers_utils import pack_sequence_as
    final = pack_sequence_as(step_out, [Tensor(torch.stack(xs, 0)) for xs in outputs])
    final_states = states
    try:
        final, final_states = decoder.finalize(final, final_states, Tensor(seq_len))
    except NotImplementedError:
        pass
    if not output_time_major:
        final = map_structure(lambda x: Tensor(_t(x).transpose(0, 1)), final)
    if return_length:
        return final, final_states, Tensor(seq_len)
    return final, final_states
