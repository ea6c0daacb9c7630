"""Recurrent layers (parity: python/paddle/nn/layer/rnn.py).

Multi-layer SimpleRNN/LSTM/GRU run the fused MIOpen RNN path of PyTorch-ROCm
(``torch._VF``) over paddle-layout parameters (weight_ih_l{k}, weight_hh_l{k},
bias_ih_l{k}, bias_hh_l{k}; gate order i,f,c,o / r,z,c as in the reference).
Cells are explicit compositions.
"""
import math

import torch

from ...framework.core import Tensor, _u
from .. import functional as F
from .. import initializer as I
from .layers import Layer


class RNNCellBase(Layer):
    def get_initial_states(self, batch_ref, shape=None, dtype=None, init_value=0.0, batch_dim_idx=0):
        b = _u(batch_ref).shape[batch_dim_idx]
        shp = self.state_shape
        if isinstance(shp[0], (list, tuple)):
            return tuple(Tensor(torch.full((b,) + tuple(s), init_value, device=_u(batch_ref).device))
                         for s in shp)
        return Tensor(torch.full((b,) + tuple(shp), init_value, device=_u(batch_ref).device))


class SimpleRNNCell(RNNCellBase):
    def __init__(self, input_size, hidden_size, activation="tanh", weight_ih_attr=None,
                 weight_hh_attr=None, bias_ih_attr=None, bias_hh_attr=None, name=None):
        super().__init__()
        std = 1.0 / math.sqrt(hidden_size)
        u = I.Uniform(-std, std)
        self.weight_ih = self.create_parameter([hidden_size, input_size], weight_ih_attr,
                                               default_initializer=u)
        self.weight_hh = self.create_parameter([hidden_size, hidden_size], weight_hh_attr,
                                               default_initializer=u)
        self.bias_ih = self.create_parameter([hidden_size], bias_ih_attr, is_bias=True,
                                             default_initializer=u)
        self.bias_hh = self.create_parameter([hidden_size], bias_hh_attr, is_bias=True,
                                             default_initializer=u)
        self.hidden_size, self.activation = hidden_size, activation
        self.state_shape = (hidden_size,)

    def forward(self, inputs, states=None):
        if states is None:
            states = self.get_initial_states(inputs)
        x, h = _u(inputs), _u(states)
        pre = x @ self.weight_ih._t.t() + self.bias_ih._t + h @ self.weight_hh._t.t() + self.bias_hh._t
        hn = torch.tanh(pre) if self.activation == 'tanh' else torch.relu(pre)
        return Tensor(hn), Tensor(hn)


class LSTMCell(RNNCellBase):
    def __init__(self, input_size, hidden_size, weight_ih_attr=None, weight_hh_attr=None,
                 bias_ih_attr=None, bias_hh_attr=None, proj_size=0, name=None):
        super().__init__()
        std = 1.0 / math.sqrt(hidden_size)
        u = I.Uniform(-std, std)
        self.weight_ih = self.create_parameter([4 * hidden_size, input_size], weight_ih_attr,
                                               default_initializer=u)
        self.weight_hh = self.create_parameter([4 * hidden_size, hidden_size], weight_hh_attr,
                                               default_initializer=u)
        self.bias_ih = self.create_parameter([4 * hidden_size], bias_ih_attr, is_bias=True,
                                             default_initializer=u)
        self.bias_hh = self.create_parameter([4 * hidden_size], bias_hh_attr, is_bias=True,
                                             default_initializer=u)
        self.hidden_size = hidden_size
        self.state_shape = ((hidden_size,), (hidden_size,))

    def forward(self, inputs, states=None):
        if states is None:
            states = self.get_initial_states(inputs)
        x = _u(inputs)
        h, c = _u(states[0]), _u(states[1])
        g = x @ self.weight_ih._t.t() + self.bias_ih._t + h @ self.weight_hh._t.t() + self.bias_hh._t
        i, f, cc, o = g.chunk(4, -1)
        c2 = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(cc)
        h2 = torch.sigmoid(o) * torch.tanh(c2)
        return Tensor(h2), (Tensor(h2), Tensor(c2))


class GRUCell(RNNCellBase):
    def __init__(self, input_size, hidden_size, weight_ih_attr=None, weight_hh_attr=None,
                 bias_ih_attr=None, bias_hh_attr=None, name=None):
        super().__init__()
        std = 1.0 / math.sqrt(hidden_size)
        u = I.Uniform(-std, std)
        self.weight_ih = self.create_parameter([3 * hidden_size, input_size], weight_ih_attr,
                                               default_initializer=u)
        self.weight_hh = self.create_parameter([3 * hidden_size, hidden_size], weight_hh_attr,
                                               default_initializer=u)
        self.bias_ih = self.create_parameter([3 * hidden_size], bias_ih_attr, is_bias=True,
                                             default_initializer=u)
        self.bias_hh = self.create_parameter([3 * hidden_size], bias_hh_attr, is_bias=True,
                                             default_initializer=u)
        self.hidden_size = hidden_size
        self.state_shape = (hidden_size,)

    def forward(self, inputs, states=None):
        if states is None:
            states = self.get_initial_states(inputs)
        x, h = _u(inputs), _u(states)
        xg = x @ self.weight_ih._t.t() + self.bias_ih._t
        hg = h @ self.weight_hh._t.t() + self.bias_hh._t
        xr, xz, xc = xg.chunk(3, -1)
        hr, hz, hc = hg.chunk(3, -1)
        r = torch.sigmoid(xr + hr)
        z = torch.sigmoid(xz + hz)
        c = torch.tanh(xc + r * hc)
        h2 = z * h + (1 - z) * c
        return Tensor(h2), Tensor(h2)


class RNN(Layer):
    """Wraps a cell and unrolls it over time (parity: paddle.nn.RNN)."""

    def __init__(self, cell, is_reverse=False, time_major=False):
        super().__init__()
        self.cell, self.is_reverse, self.time_major = cell, is_reverse, time_major

    def forward(self, inputs, initial_states=None, sequence_length=None, **kwargs):
        x = _u(inputs)
        if not self.time_major:
            x = x.transpose(0, 1)
        T = x.shape[0]
        states = initial_states
        outs = []
        steps = range(T - 1, -1, -1) if self.is_reverse else range(T)
        for t in steps:
            o, new_states = self.cell(Tensor(x[t]), states)
            if sequence_length is not None:
                mask = (_u(sequence_length) > t).to(x.dtype).unsqueeze(-1)
                if states is not None:
                    def _sel(n, s):
                        return Tensor(_u(n) * mask + _u(s) * (1 - mask))
                    if isinstance(new_states, (tuple, list)):
                        new_states = type(new_states)(_sel(n, s) for n, s in zip(new_states, states))
                    else:
                        new_states = _sel(new_states, states)
                o = Tensor(_u(o) * mask)
            states = new_states
            outs.append(_u(o))
        if self.is_reverse:
            outs = outs[::-1]
        y = torch.stack(outs, 0)
        if not self.time_major:
            y = y.transpose(0, 1)
        return Tensor(y), states


class BiRNN(Layer):
    def __init__(self, cell_fw, cell_bw, time_major=False):
        super().__init__()
        self.rnn_fw = RNN(cell_fw, False, time_major)
        self.rnn_bw = RNN(cell_bw, True, time_major)

    def forward(self, inputs, initial_states=None, sequence_length=None, **kwargs):
        s_fw, s_bw = (None, None) if initial_states is None else initial_states
        o1, st1 = self.rnn_fw(inputs, s_fw, sequence_length)
        o2, st2 = self.rnn_bw(inputs, s_bw, sequence_length)
        return Tensor(torch.cat([_u(o1), _u(o2)], -1)), (st1, st2)


class _RNNBase(Layer):
    _mode = 'RNN_TANH'
    _gates = 1

    def __init__(self, input_size, hidden_size, num_layers=1, direction="forward", time_major=False,
                 dropout=0., activation='tanh', weight_ih_attr=None, weight_hh_attr=None,
                 bias_ih_attr=None, bias_hh_attr=None, name=None):
        super().__init__()
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        self.bidirect = direction in ('bidirect', 'bidirectional')
        self.num_directions = 2 if self.bidirect else 1
        self.time_major, self.dropout = time_major, dropout
        if self._mode.startswith('RNN'):
            self._mode = 'RNN_TANH' if activation == 'tanh' else 'RNN_RELU'
        std = 1.0 / math.sqrt(hidden_size)
        u = I.Uniform(-std, std)
        G = self._gates * hidden_size
        self._flat = []
        for layer in range(num_layers):
            for d in range(self.num_directions):
                insz = input_size if layer == 0 else hidden_size * self.num_directions
                sfx = f'_l{layer}' + ('_reverse' if d == 1 else '')
                ws = [self.create_parameter([G, insz], weight_ih_attr, default_initializer=u),
                      self.create_parameter([G, hidden_size], weight_hh_attr, default_initializer=u),
                      self.create_parameter([G], bias_ih_attr, is_bias=True, default_initializer=u),
                      self.create_parameter([G], bias_hh_attr, is_bias=True, default_initializer=u)]
                for n, w in zip(['weight_ih', 'weight_hh', 'bias_ih', 'bias_hh'], ws):
                    self.add_parameter(n + sfx, w)
                self._flat += ws

    def forward(self, inputs, initial_states=None, sequence_length=None):
        x = _u(inputs)
        if self.time_major:
            x = x.transpose(0, 1)
        B = x.shape[0]
        L = self.num_layers * self.num_directions
        ws = [p._t for p in self._flat]
        if self._mode == 'LSTM':
            if initial_states is None:
                h0 = torch.zeros(L, B, self.hidden_size, dtype=x.dtype, device=x.device)
                c0 = torch.zeros_like(h0)
            else:
                h0, c0 = _u(initial_states[0]), _u(initial_states[1])
            out, h, c = torch._VF.lstm(x, (h0, c0), ws, True, self.num_layers, self.dropout,
                                       self.training, self.bidirect, True)
            final = (Tensor(h), Tensor(c))
        else:
            h0 = torch.zeros(L, B, self.hidden_size, dtype=x.dtype, device=x.device) \
                if initial_states is None else _u(initial_states)
            fn = torch._VF.gru if self._mode == 'GRU' else (
                torch._VF.rnn_tanh if self._mode == 'RNN_TANH' else torch._VF.rnn_relu)
            out, h = fn(x, h0, ws, True, self.num_layers, self.dropout, self.training, self.bidirect,
                        True)
            final = Tensor(h)
        if sequence_length is not None:
            sl = _u(sequence_length)
            mask = (torch.arange(out.shape[1], device=out.device)[None, :] < sl[:, None]).to(out.dtype)
            out = out * mask.unsqueeze(-1)
        if self.time_major:
            out = out.transpose(0, 1)
        return Tensor(out), final


class SimpleRNN(_RNNBase):
    _mode = 'RNN_TANH'
    _gates = 1


class LSTM(_RNNBase):
    _mode = 'LSTM'
    _gates = 4


class GRU(_RNNBase):
    _mode = 'GRU'
    _gates = 3
