"""Auto-parallel tuner: tunable spaces, trials and an analytic parallel-strategy search.

Parity: python/paddle/distributed/auto_parallel/tuner/ -- tunable_variable.py (Fixed, Boolean,
Choice, IntRange, FloatRange), tunable_space.py (TunableSpace: fixed/boolean/choice/int_range/
float_range, get_state/from_state), trial.py (Trial, TrialStatus) and the parallel / rule-based
tuners that search dp x mp x pp x sharding for a program. The reference profiles candidate
programs or prices them with its op cost model; this tuner prices a transformer training step
analytically for ONE MI355X node (or several) instead:

* compute: 6 * params * tokens dense FLOPs (+ one extra forward under recompute) at a sustained
  fraction of the 2.5 PF/s dense bf16 peak (default 0.45, the measured GPT-1.3B step MFU);
* pipeline bubble: (pp - 1) / (micro_batches + pp - 1) of the pipelined compute (1F1B);
* collectives on xGMI: every GPU reaches each peer through its own link (~64 GB/s per direction),
  so a ring over n ranks moves 2 (n - 1) / n * B bytes per rank at ~7 links' worth of bus
  bandwidth when the group spans the node (fewer links for smaller groups); TP all-reduces the
  [micro_batch, seq, hidden] activations 4x per layer (2 forward + 2 backward), DP all-reduces
  (or sharding reduce-scatters + all-gathers) the gradients once per step and is overlapped with
  the backward except for the last bucket;
* memory (288 GB HBM3E per GPU): bf16 weights + grads + fp32 master/moments (16 B / param)
  divided over mp * pp and, per sharding stage, over dp; activations ~ 34 * s * b * h bytes per
  layer (/ mp, ~2 * s * b * h with recompute); configurations above ``mem_fraction`` of HBM are
  rejected.

``ParallelTuner(model, cluster).tune()`` returns the trials sorted by estimated step time; the
first is the recommended strategy (``Trial.strategy()`` gives the Fleet hybrid_configs)."""
import itertools
import math
import random as _random

__all__ = ['TunableVariable', 'Fixed', 'Boolean', 'Choice', 'IntRange', 'FloatRange', 'TunableSpace',
           'TrialStatus', 'Trial', 'ModelSpec', 'ClusterSpec', 'ParallelTuner']


class TunableVariable:
    def __init__(self, name, default=None):
        self.name = name
        self._default = default

    @property
    def default(self):
        return self._default

    def get_state(self):
        return {'class_name': type(self).__name__, 'name': self.name, 'default': self._default}


class Fixed(TunableVariable):
    def random(self, seed=None):
        return self._default

    def get_state(self):
        return dict(super().get_state(), default=self._default)

    def __repr__(self):
        return f'Fixed(name: {self.name}, value: {self._default})'


class Boolean(TunableVariable):
    def __init__(self, name, default=False):
        if default not in (True, False):
            raise ValueError(f"Boolean {name}: default must be a bool, got {default!r}")
        super().__init__(name, default)
        self.values = [False, True]

    def random(self, seed=None):
        return _random.Random(seed).choice(self.values)

    def __repr__(self):
        return f'Boolean(name: {self.name}, default: {self._default})'


class Choice(TunableVariable):
    def __init__(self, name, values, default=None):
        values = list(values)
        if not values:
            raise ValueError(f"Choice {name}: values must be non-empty")
        if len({type(v) for v in values}) > 1:
            raise TypeError(f"Choice {name}: values must share one type, got {values}")
        if default is not None and default not in values:
            raise ValueError(f"Choice {name}: default {default!r} not among {values}")
        super().__init__(name, values[0] if default is None else default)
        self.values = values

    def random(self, seed=None):
        return _random.Random(seed).choice(self.values)

    def get_state(self):
        return dict(super().get_state(), values=list(self.values))

    def __repr__(self):
        return f'Choice(name: {self.name}, values: {self.values}, default: {self._default})'


class IntRange(TunableVariable):
    def __init__(self, name, start, stop, step=1, default=None, endpoint=False):
        super().__init__(name, start if default is None else int(default))
        self.start, self.stop, self.step, self.endpoint = int(start), int(stop), int(step), endpoint
        self.values = list(range(self.start, self.stop + (1 if endpoint else 0), self.step))

    def random(self, seed=None):
        return _random.Random(seed).choice(self.values)

    def get_state(self):
        return dict(super().get_state(), start=self.start, stop=self.stop, step=self.step, endpoint=self.endpoint)

    def __repr__(self):
        return f'IntRange(name: {self.name}, start: {self.start}, stop: {self.stop}, step: {self.step})'


class FloatRange(TunableVariable):
    def __init__(self, name, start, stop, step=None, default=None, endpoint=False):
        super().__init__(name, float(start) if default is None else float(default))
        self.start, self.stop, self.step, self.endpoint = float(start), float(stop), step, endpoint

    def random(self, seed=None):
        r = _random.Random(seed)
        if self.step is None:
            return r.uniform(self.start, self.stop)
        n = int((self.stop - self.start) / self.step) + (1 if self.endpoint else 0)
        return self.start + self.step * r.randrange(max(n, 1))

    def get_state(self):
        return dict(super().get_state(), start=self.start, stop=self.stop, step=self.step, endpoint=self.endpoint)

    def __repr__(self):
        return f'FloatRange(name: {self.name}, start: {self.start}, stop: {self.stop}, step: {self.step})'


_CLASSES = {c.__name__: c for c in (Fixed, Boolean, Choice, IntRange, FloatRange)}


class TunableSpace:
    """Named tunable variables and their current values."""

    def __init__(self):
        self._variables = {}
        self._values = {}

    @property
    def variables(self):
        return self._variables

    @property
    def values(self):
        return self._values

    def get_value(self, name):
        if name not in self._values:
            raise KeyError(f"{name} does not exist in the tunable space")
        return self._values[name]

    def set_value(self, name, value):
        if name not in self._variables:
            raise KeyError(f"{name} does not exist in the tunable space")
        self._values[name] = value

    def __getitem__(self, name):
        return self.get_value(name)

    def __setitem__(self, name, value):
        self.set_value(name, value)

    def __contains__(self, name):
        return name in self._variables

    def _register(self, tv):
        if tv.name in self._variables:
            return self._values[tv.name]   # first registration wins (reference _retrieve)
        self._variables[tv.name] = tv
        self._values[tv.name] = tv.default
        return tv.default

    def fixed(self, name, default):
        return self._register(Fixed(name, default))

    def boolean(self, name, default=False):
        return self._register(Boolean(name, default))

    def choice(self, name, values, default=None):
        return self._register(Choice(name, values, default))

    def int_range(self, name, start, stop, step=1, default=None):
        return self._register(IntRange(name, start, stop, step, default))

    def float_range(self, name, start, stop, step=None, default=None):
        return self._register(FloatRange(name, start, stop, step, default))

    def get_state(self):
        return {'variables': [v.get_state() for v in self._variables.values()], 'values': dict(self._values)}

    @classmethod
    def from_state(cls, state):
        ts = cls()
        for st in state['variables']:
            st = dict(st)
            c = _CLASSES[st.pop('class_name')]
            name = st.pop('name')
            if c is Fixed:
                tv = Fixed(name, st['default'])
            elif c is Boolean:
                tv = Boolean(name, st['default'])
            elif c is Choice:
                tv = Choice(name, st['values'], st['default'])
            elif c is IntRange:
                tv = IntRange(name, st['start'], st['stop'], st['step'], st['default'], st['endpoint'])
            else:
                tv = FloatRange(name, st['start'], st['stop'], st['step'], st['default'], st['endpoint'])
            ts._register(tv)
        ts._values.update(state['values'])
        return ts


class TrialStatus:
    RUNNING = 'RUNNING'
    COMPLETED = 'COMPLETED'
    STOPPED = 'STOPPED'
    INVALID = 'INVALID'


class Trial:
    _next = 0

    def __init__(self, space, trial_id=None, status=TrialStatus.RUNNING):
        if trial_id is None:
            trial_id = f'trial_{Trial._next:05d}'
            Trial._next += 1
        self.id, self.space, self.status = trial_id, space, status
        self.metrics = {}
        self.reason = None

    def summary(self):
        return {'id': self.id, 'status': self.status, 'values': dict(self.space.values), 'metrics': dict(self.metrics),
                'reason': self.reason}

    def strategy(self):
        """Fleet hybrid_configs + the sharding / recompute switches of this trial."""
        v = self.space.values
        stage = int(v['sharding_stage'])
        # evaluate() models optimizer state / gradients / parameters sharded over the data-parallel
        # ranks when sharding_stage > 0: those ranks then form fleet's SHARDING group (sharding
        # degree = dp, dp degree 1), so the emitted strategy shards exactly what was priced
        dp = int(v['dp_degree'])
        return {'hybrid_configs': {'dp_degree': 1 if stage > 0 else dp, 'mp_degree': v['mp_degree'],
                                   'pp_degree': v['pp_degree'], 'sharding_degree': dp if stage > 0 else 1},
                'sharding': stage > 0, 'sharding_configs': {'stage': stage} if stage > 0 else {},
                'sharding_stage': stage, 'micro_batch_size': v['micro_batch_size'],
                'recompute': v['recompute']}

    def __repr__(self):
        return f'Trial({self.id}, {self.status}, {self.space.values}, {self.metrics})'


class ModelSpec:
    """A decoder/encoder transformer to place: layers, hidden, heads, seq, vocab, global batch."""

    def __init__(self, num_layers, hidden, num_heads, seq_len, vocab_size, global_batch, ffn_mult=4):
        self.num_layers, self.hidden, self.num_heads = num_layers, hidden, num_heads
        self.seq_len, self.vocab_size, self.global_batch, self.ffn_mult = seq_len, vocab_size, global_batch, ffn_mult

    @property
    def params(self):
        h, L = self.hidden, self.num_layers
        per_layer = (4 + 2 * self.ffn_mult) * h * h + (9 + 2 * self.ffn_mult) * h   # qkv/out/fc1/fc2 + biases/LN
        return L * per_layer + self.vocab_size * h + self.seq_len * h


class ClusterSpec:
    """GPUs of one job on MI355X nodes (8 per node on xGMI)."""

    def __init__(self, n_gpus=8, gpus_per_node=8, hbm_gb=288.0, peak_tflops=2500.0, mfu=0.45,
                 link_gbs=64.0, links_per_gpu=7, internode_gbs=50.0, mem_fraction=0.9):
        self.n_gpus, self.gpus_per_node, self.hbm_gb = n_gpus, gpus_per_node, hbm_gb
        self.peak_tflops, self.mfu, self.link_gbs, self.links_per_gpu = peak_tflops, mfu, link_gbs, links_per_gpu
        self.internode_gbs, self.mem_fraction = internode_gbs, mem_fraction

    def bus_gbs(self, group):
        """Per-rank ring bandwidth of a collective over ``group`` consecutive ranks."""
        if group <= 1:
            return float('inf')
        if group > self.gpus_per_node:
            return self.internode_gbs
        return self.link_gbs * min(self.links_per_gpu, group - 1)


def _ring_s(nbytes, group, cluster, alpha_us=30.0):
    if group <= 1:
        return 0.0
    return alpha_us * 1e-6 + 2.0 * (group - 1) / group * nbytes / (cluster.bus_gbs(group) * 1e9)


class ParallelTuner:
    """Enumerates dp x mp x pp x sharding stage x micro batch x recompute for ``model`` on
    ``cluster`` and ranks the feasible ones by the analytic step time (module docstring)."""

    def __init__(self, model, cluster=None, micro_batch_sizes=(1, 2, 4, 8, 16)):
        self.model, self.cluster = model, cluster or ClusterSpec()
        self.micro_batch_sizes = tuple(micro_batch_sizes)
        self.trials = []

    def _divisors(self, n):
        return [d for d in range(1, n + 1) if n % d == 0]

    def space(self):
        ts = TunableSpace()
        n = self.cluster.n_gpus
        ts.choice('dp_degree', self._divisors(n))
        ts.choice('mp_degree', self._divisors(n))
        ts.choice('pp_degree', self._divisors(n))
        ts.choice('sharding_stage', [0, 1, 2, 3])
        ts.choice('micro_batch_size', list(self.micro_batch_sizes))
        ts.boolean('recompute')
        return ts

    def evaluate(self, values):
        """(step_seconds, memory_gb) or raises ValueError with the reason the config is invalid."""
        m, c = self.model, self.cluster
        dp, mp, pp = values['dp_degree'], values['mp_degree'], values['pp_degree']
        st, mb, rc = values['sharding_stage'], values['micro_batch_size'], values['recompute']
        if dp * mp * pp != c.n_gpus:
            raise ValueError('dp * mp * pp != n_gpus')
        if m.num_heads % mp or m.hidden % mp or (m.ffn_mult * m.hidden) % mp:
            raise ValueError('heads / hidden not divisible by mp')
        if m.num_layers % pp:
            raise ValueError('layers not divisible by pp')
        if mp > c.gpus_per_node:
            raise ValueError('tensor parallel across nodes')
        if st and dp == 1:
            raise ValueError('sharding needs dp > 1')
        if m.global_batch % (dp * mb):
            raise ValueError('global batch not divisible by dp * micro batch')
        n_micro = m.global_batch // (dp * mb)
        if pp > 1 and n_micro < pp:
            raise ValueError('fewer micro batches than pipeline stages')
        P = m.params
        s, h, L = m.seq_len, m.hidden, m.num_layers
        # memory per GPU (GB)
        p_local = P / (mp * pp)
        w_b, g_b, o_b = 2.0, 2.0, 12.0   # bf16 weights, bf16 grads, fp32 master + 2 moments
        shard = dp if st else 1
        mem = p_local * (o_b / shard + (g_b / dp if st >= 2 else g_b) + (w_b / dp if st >= 3 else w_b))
        act_layer = (2.0 if rc else 34.0) * s * mb * h / mp
        in_flight = min(pp, n_micro) if pp > 1 else 1
        mem += act_layer * (L / pp) * in_flight + 4.0 * s * mb * m.vocab_size / mp * (1 if pp == 1 else 1 / pp)
        mem_gb = mem / 1e9
        if mem_gb > c.hbm_gb * c.mem_fraction:
            raise ValueError(f'needs {mem_gb:.0f} GB > {c.hbm_gb * c.mem_fraction:.0f} GB')
        # time
        tokens = m.global_batch * s
        flops = 6.0 * P * tokens * (4.0 / 3.0 if rc else 1.0)
        t_comp = flops / (c.n_gpus * c.peak_tflops * 1e12 * c.mfu)
        if mp > 1:   # smaller per-GPU GEMMs run less efficiently
            t_comp *= 1.0 + 0.04 * math.log2(mp)
        t_bubble = t_comp * (pp - 1) / (n_micro + pp - 1) if pp > 1 else 0.0
        t_tp = 4 * L / pp * n_micro * _ring_s(2.0 * s * mb * h, mp, c) if mp > 1 else 0.0
        t_pp = 2 * (pp - 1) * n_micro * (2.0 * s * mb * h / mp) / (c.link_gbs * 1e9) if pp > 1 else 0.0
        grad_bytes = 2.0 * p_local
        t_dp = 0.0
        if dp > 1:
            t_dp = _ring_s(grad_bytes, dp, c)
            if st >= 3:   # parameter all-gathers in forward and backward
                t_dp += 2 * 0.5 * _ring_s(2.0 * p_local, dp, c)
            t_dp = min(t_dp, 0.15 * t_dp + max(0.0, t_dp - 0.85 * t_comp))   # overlapped with backward
        return t_comp + t_bubble + t_tp + t_pp + t_dp, mem_gb

    def tune(self, max_trials=None):
        base = self.space()
        names = list(base.variables)
        combos = itertools.product(*[base.variables[k].values for k in names])
        self.trials = []
        for vals in combos:
            ts = TunableSpace.from_state(base.get_state())
            for k, v in zip(names, vals):
                ts[k] = v
            t = Trial(ts)
            try:
                step, mem = self.evaluate(ts.values)
                t.metrics = {'step_time_s': step, 'memory_gb': mem,
                             'tokens_per_s': self.model.global_batch * self.model.seq_len / step}
                t.status = TrialStatus.COMPLETED
            except ValueError as e:
                t.status, t.reason = TrialStatus.INVALID, str(e)
            self.trials.append(t)
        done = sorted((t for t in self.trials if t.status == TrialStatus.COMPLETED),
                      key=lambda t: (round(t.metrics['step_time_s'], 6), t.metrics['memory_gb']))
        return done[:max_trials] if max_trials else done

    def best(self):
        done = self.tune(1)
        if not done:
            raise RuntimeError('no feasible parallel configuration for this model on this cluster')
        return done[0]
