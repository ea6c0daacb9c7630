"""paddle.jit (parity: python/paddle/jit/api.py, python/paddle/jit/translated_layer.py,
python/paddle/jit/dy2static/program_translator.py).

MI355X design — no AST transcription. ``to_static`` keeps eager semantics for training
(the PyTorch-ROCm autograd tape already drives our HIP kernels) and adds two things the
reference's dy2static is used for:

* **HIP-graph replay** for gradient-free calls on the GPU: the first call for a given
  input signature captures the whole forward into a ``torch.cuda.CUDAGraph`` (= hipGraph
  on ROCm) with static input buffers; later calls copy inputs in and replay the graph —
  one launch instead of hundreds (launch-bound serving / small-batch inference).
* **Program export**: ``concrete_program`` / ``jit.save`` record the layer into a static
  ``Program`` (static/graph.py) from ``InputSpec``s and write ``.pdmodel`` (JSON op list)
  + ``.pdiparams``; ``jit.load`` returns a ``TranslatedLayer`` that replays the program
  eagerly, so it can run inference or be fine-tuned.
"""
import functools
import os

import torch

from ..framework.core import Tensor, _u
from ..static.input import InputSpec

_enabled = [True]
_graph_default = [os.environ.get('PRA_TO_STATIC_HIP_GRAPH', '1') == '1']


def enable_to_static(flag):
    _enabled[0] = bool(flag)


def set_code_level(level=100, also_to_stdout=False):
    pass


def set_verbosity(level=0, also_to_stdout=False):
    pass


def not_to_static(fn):
    fn._not_to_static = True
    return fn


def ignore_module(modules):
    pass


def _flat_tensors(obj, out):
    if isinstance(obj, Tensor):
        out.append(obj)
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            _flat_tensors(o, out)
    elif isinstance(obj, dict):
        for o in obj.values():
            _flat_tensors(o, out)
    return out


def _signature(args, kwargs):
    def sig(o):
        if isinstance(o, Tensor):
            t = o._t
            return ('T', tuple(t.shape), t.dtype, str(t.device))
        if isinstance(o, (list, tuple)):
            return tuple(sig(x) for x in o)
        if isinstance(o, dict):
            return tuple((k, sig(v)) for k, v in sorted(o.items()))
        return ('C', repr(o))
    return (sig(args), sig(kwargs))


class _GraphEntry:
    """One captured HIP graph: static input buffers, the graph, and static outputs."""

    def __init__(self, fn, args, kwargs):
        ins = _flat_tensors((args, kwargs), [])
        self.static_in = [t._t.clone() for t in ins]
        it = iter(self.static_in)

        def swap(o):
            if isinstance(o, Tensor):
                return Tensor(next(it))
            if isinstance(o, list):
                return [swap(x) for x in o]
            if isinstance(o, tuple):
                return tuple(swap(x) for x in o)
            if isinstance(o, dict):
                return {k: swap(v) for k, v in o.items()}
            return o
        sargs, skw = swap(args), swap(kwargs)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):  # warm up allocator / lazy inits outside the capture
                fn(*sargs, **skw)
        torch.cuda.current_stream().wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = fn(*sargs, **skw)

    def __call__(self, args, kwargs):
        for buf, t in zip(self.static_in, _flat_tensors((args, kwargs), [])):
            buf.copy_(t._t, non_blocking=True)
        self.graph.replay()
        return self.out


class StaticFunction:
    """Callable returned by ``to_static``."""

    def __init__(self, fn, input_spec=None, build_strategy=None, layer=None, **kwargs):
        self._fn = fn
        self._input_spec = list(input_spec) if input_spec is not None else None
        self._build_strategy = build_strategy
        self._layer = layer
        self._graphs = {}
        self._programs = {}
        functools.update_wrapper(self, fn)

    def __get__(self, instance, owner):
        if instance is None:
            return self
        key = '_pra_sf_' + self._fn.__name__
        bound = instance.__dict__.get(key)
        if bound is None:
            bound = StaticFunction(self._fn.__get__(instance, owner), self._input_spec,
                                   self._build_strategy, layer=instance)
            instance.__dict__[key] = bound
        return bound

    @property
    def dygraph_function(self):
        return self._fn

    def _use_graph(self, args, kwargs):
        bs = self._build_strategy
        want = getattr(bs, 'use_hip_graph', None) if bs is not None else None
        if want is None:
            want = _graph_default[0]
        if not want or not torch.cuda.is_available() or torch.is_grad_enabled() and \
                self._needs_grad(args, kwargs):
            return False
        ins = _flat_tensors((args, kwargs), [])
        return bool(ins) and all(t._t.is_cuda for t in ins)

    def _needs_grad(self, args, kwargs):
        if any(t._t.requires_grad for t in _flat_tensors((args, kwargs), [])):
            return True
        if self._layer is not None:
            return any(not p.stop_gradient for p in self._layer.parameters())
        return True

    def __call__(self, *args, **kwargs):
        from ..static import _STATIC
        if not _enabled[0] or _STATIC[0]:
            return self._fn(*args, **kwargs)
        if self._use_graph(args, kwargs):
            key = _signature(args, kwargs)
            g = self._graphs.get(key)
            if g is None:
                g = self._graphs[key] = _GraphEntry(self._fn, args, kwargs)
            return g(args, kwargs)
        return self._fn(*args, **kwargs)

    # -- program export --------------------------------------------------------------
    def get_concrete_program(self, *input_spec, **kwargs):
        specs = list(input_spec) or self._input_spec
        if specs is None:
            raise ValueError("input_spec is required to build a concrete program")
        key = tuple(repr(s) for s in specs)
        if key not in self._programs:
            self._programs[key] = _record_program(self._fn, specs, self._layer)
        return self._programs[key]

    @property
    def concrete_program(self):
        return self.get_concrete_program()

    @property
    def main_program(self):
        return self.concrete_program[0]

    def rollback(self):
        return self._fn


def _to_spec(s, i):
    if isinstance(s, InputSpec):
        return s
    if isinstance(s, Tensor):
        return InputSpec(s.shape, s.dtype, f'x{i}')
    raise TypeError(f"unsupported input_spec entry {s!r}")


def _record_program(fn, specs, layer=None):
    """Trace ``fn`` on symbolic inputs -> (Program, feed Variables, fetch Variables)."""
    from .. import static
    from ..static import graph as G
    specs = [_to_spec(s, i) for i, s in enumerate(specs)]
    was_static = static._STATIC[0]
    was_training = layer.training if layer is not None else None
    static.enable_static()
    try:
        if layer is not None:
            layer.eval()
        prog = G.Program()
        with G.program_guard(prog, G.Program()):
            feeds = [G.data(s.name or f'x{i}', list(s.shape), s.dtype)
                     for i, s in enumerate(specs)]
            out = fn(*feeds)
        fetches = [v for v in _flat_tensors(out, []) if isinstance(v, G.Variable)]
    finally:
        if not was_static:
            static.disable_static()
        if layer is not None and was_training:
            layer.train()
    return prog, feeds, fetches


def to_static(function=None, input_spec=None, build_strategy=None, backend=None, **kwargs):
    def deco(fn):
        from ..nn.layer.layers import Layer
        if isinstance(fn, Layer):
            fwd = fn.forward
            if not isinstance(fwd, StaticFunction):
                inner = getattr(fwd, '__func__', None)
                sf = StaticFunction(inner if inner is not None else fwd, input_spec,
                                    build_strategy)
                fn.__dict__['forward'] = sf.__get__(fn, type(fn)) if inner is not None else sf
            return fn
        if getattr(fn, '_not_to_static', False):
            return fn
        return StaticFunction(fn, input_spec, build_strategy)
    return deco(function) if function is not None else deco


# =============================================================================
# save / load
# =============================================================================
def save(layer, path, input_spec=None, **configs):
    """Export ``layer`` (or a StaticFunction / plain function) as ``path.pdmodel`` +
    ``path.pdiparams`` (parity: paddle.jit.save)."""
    from ..static import graph as G
    from ..nn.layer.layers import Layer
    if isinstance(layer, Layer):
        fwd = layer.forward
        specs = input_spec
        if isinstance(fwd, StaticFunction):
            specs = specs or fwd._input_spec
            fn = fwd._fn
        else:
            fn = fwd
        owner = layer
    elif isinstance(layer, StaticFunction):
        fn, specs, owner = layer._fn, input_spec or layer._input_spec, layer._layer
    else:
        fn, specs, owner = layer, input_spec, None
    if specs is None:
        raise ValueError("jit.save needs input_spec (or a to_static function with one)")
    prog, feeds, fetches = _record_program(fn, specs, owner)
    output_spec = configs.get('output_spec')
    if output_spec is not None:
        fetches = [fetches[i] for i in range(len(output_spec))]
    G.save_inference_model(path, feeds, fetches, program=prog)


class TranslatedLayer:
    """Layer that replays a loaded program (inference or fine-tuning)."""


def _make_translated_layer():
    from ..nn.layer.layers import Layer
    from ..static import graph as G

    class _TranslatedLayer(Layer, TranslatedLayer):
        def __init__(self, program, feed_names, fetch_vars):
            super().__init__()
            self._program = program
            self._feed_names = feed_names
            self._fetch_vars = fetch_vars
            for name, p in program._params.items():
                p.stop_gradient = False
                p.trainable = True
                self._parameters[name.replace('.', '_')] = p
            self._exe = G.Executor()

        def forward(self, *inputs):
            feed = dict(zip(self._feed_names, inputs))
            outs = self._exe.run(self._program, feed=feed, fetch_list=self._fetch_vars,
                                 return_numpy=False)
            return outs[0] if len(outs) == 1 else outs

        def program(self, method_name='forward'):
            return self._program

    return _TranslatedLayer


def load(path, **configs):
    from ..static import graph as G
    prog, feed_names, fetch_vars = G.load_inference_model(path)
    return _make_translated_layer()(prog, feed_names, fetch_vars)
