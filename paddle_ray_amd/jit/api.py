"""paddle.jit (parity: python/paddle/jit/api.py, python/paddle/jit/translated_layer.py,
python/paddle/jit/dy2static/program_translator.py).

MI355X design. ``to_static`` keeps eager semantics for training (the PyTorch-ROCm autograd
tape already drives our HIP kernels); tensor-valued ``if`` / ``while`` are transcribed only for
program export (``jit/dy2static.py``, applied by ``jit.save`` / ``concrete_program``). It adds
the things the reference's dy2static is used for:

* **HIP-graph replay** for gradient-free calls on the GPU: the first call for a given
  input signature captures the whole forward into a ``torch.cuda.CUDAGraph`` (= hipGraph
  on ROCm) with static input buffers; later calls copy inputs in and replay the graph —
  one launch instead of hundreds (launch-bound serving / small-batch inference).
* **Training capture** (``build_strategy.use_hip_graph = True`` on a call that needs
  gradients): the forward AND its backward are captured as two graphs sharing one memory
  pool; the call becomes one autograd node whose forward replays the first graph and whose
  backward replays the second, returning input and parameter gradients (accumulated into
  ``.grad`` as usual). Parameters must keep their storage (optimizers update in place).
* **Program export**: ``concrete_program`` / ``jit.save`` record the layer into a static
  ``Program`` (static/graph.py) from ``InputSpec``s and write ``.pdmodel`` (a ProgramDesc
  protobuf, static/program_desc.py) + ``.pdiparams``; ``jit.load`` returns a ``TranslatedLayer`` that replays the program
  eagerly, so it can run inference or be fine-tuned. Before recording, the function's
  tensor-valued ``if`` / ``while`` statements are converted (``dy2static.py``) into
  ``static.nn.cond`` / ``while_loop`` sub-blocks, which serialize as sub-BlockDescs.
* Graph replay hands out fresh output tensors on every call, and a function that cannot be
  captured (host read of device data, data-dependent shapes) runs eagerly instead.
"""
import functools
import os

import torch

from ..framework.core import Tensor, _u
from ..static.input import InputSpec

_enabled = [True]
_TRAIN_GRAPH_ACCUMULATE = os.environ.get('PRA_TRAIN_GRAPH_ACCUMULATE', '1') == '1'
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
        from ..ops.fused import managed_graph_rng
        with managed_graph_rng() as rng:
            with torch.cuda.graph(self.graph):
                self.out = fn(*sargs, **skw)
        self.rng_dev = torch.device('cuda', torch.cuda.current_device()) if rng['used'] else None

    def replay_static(self, args, kwargs):
        """Replay and return the graph's STATIC output buffers (rewritten by the next replay):
        for callers that consume them before replaying again (the static Executor's optimizer
        step reads the captured gradients in place)."""
        for buf, t in zip(self.static_in, _flat_tensors((args, kwargs), [])):
            buf.copy_(t._t, non_blocking=True)
        if self.rng_dev is not None:  # new dropout masks for this replay
            from ..ops.fused import graph_seq_advance
            graph_seq_advance(self.rng_dev)
        self.graph.replay()
        return self.out

    def __call__(self, args, kwargs):
        # the captured outputs are the graph's static buffers, rewritten by the next replay:
        # every call hands out its own copies (y1 = f(x1); y2 = f(x2) keeps y1)
        return _clone_struct(self.replay_static(args, kwargs))


def _clone_struct(o):
    if isinstance(o, Tensor):
        c = Tensor(o._t.clone())
        c.stop_gradient = o.stop_gradient
        return c
    if isinstance(o, torch.Tensor):
        return o.clone()
    if isinstance(o, list):
        return [_clone_struct(x) for x in o]
    if isinstance(o, tuple):
        return tuple(_clone_struct(x) for x in o)
    if isinstance(o, dict):
        return {k: _clone_struct(v) for k, v in o.items()}
    return o


class _Eager:
    """Marks a signature whose capture failed (a host read of device data, a data-dependent
    shape, a synchronising op): it runs eagerly from then on."""
    reason = None


class _TrainGraph:
    """Forward + backward of ``fn`` captured as two HIP graphs (parity in spirit with the
    reference's to_static training programs run by the standalone executor)."""

    def __init__(self, fn, params, args, kwargs):
        ins = _flat_tensors((args, kwargs), [])
        self.params = [p for p in params if not p.stop_gradient]
        self.static_in = [t._t.detach().clone().requires_grad_(t._t.requires_grad) for t in ins]
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
        ptens = [p._t for p in self.params]
        diff_in = [t for t in self.static_in if t.requires_grad]
        wrt = diff_in + ptens
        # Accumulate mode (no differentiable inputs, no post-accumulate hooks on the parameters):
        # the backward graph adds straight into the parameters' .grad buffers -- the fused
        # kernels' in-place beta=1 / finalize accumulation and autograd's AccumulateGrad are
        # captured -- so a replay hands no per-parameter gradient copies back to autograd. The
        # .grad buffers must keep their storage (clear_grad(set_to_zero=True) zeroes in place).
        self.accumulate = (_TRAIN_GRAPH_ACCUMULATE and not diff_in and all(
            not getattr(p, '_post_accumulate_grad_hooks', None) for p in ptens))
        saved_grads = [p.grad for p in ptens]
        if self.accumulate:
            for p in ptens:
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
            saved_grads = [p.grad.clone() for p in ptens]
        else:
            for p in ptens:   # fused kernels add into an existing .grad in place: keep them pure
                p.grad = None
        try:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):  # warm up allocator / lazy inits / autotuning
                    outs = [o._t for o in _flat_tensors(fn(*sargs, **skw), [])]
                    if self.accumulate:
                        torch.autograd.backward(outs, [torch.ones_like(o) for o in outs], inputs=ptens)
                    else:
                        torch.autograd.grad(outs, wrt, [torch.ones_like(o) for o in outs],
                                            allow_unused=True)
            torch.cuda.current_stream().wait_stream(s)
            pool = torch.cuda.graph_pool_handle()
            self.fwd_graph = torch.cuda.CUDAGraph()
            from ..ops.fused import managed_graph_rng
            with managed_graph_rng() as rng:
                with torch.cuda.graph(self.fwd_graph, pool=pool):
                    out = fn(*sargs, **skw)
            self.rng_dev = torch.device('cuda', torch.cuda.current_device()) if rng['used'] else None
            self.out_struct = out
            self.static_out = [o._t for o in _flat_tensors(out, [])]
            self.static_gout = [torch.empty_like(o) for o in self.static_out]
            self.bwd_graph = torch.cuda.CUDAGraph()
            with managed_graph_rng():  # reads the forward's counter value, never advances it
                with torch.cuda.graph(self.bwd_graph, pool=pool):
                    if self.accumulate:
                        torch.autograd.backward(self.static_out, self.static_gout, inputs=ptens)
                        grads = [None] * len(wrt)
                    else:
                        grads = torch.autograd.grad(self.static_out, wrt, self.static_gout,
                                                    allow_unused=True)
            self.static_grads = [g if g is not None else None for g in grads]
        finally:
            if self.accumulate:   # the warm-up added into the buffers: restore their values
                for p, g in zip(ptens, saved_grads):
                    p.grad.copy_(g)
            else:
                for p, g in zip(ptens, saved_grads):
                    p.grad = g
        self.diff_mask = [t.requires_grad for t in self.static_in]
        entry = self

        class _Graphed(torch.autograd.Function):
            @staticmethod
            def forward(ctx, *tensors):
                n_in = len(entry.static_in)
                for buf, t in zip(entry.static_in, tensors[:n_in]):
                    buf.detach().copy_(t, non_blocking=True)
                if entry.rng_dev is not None:  # new dropout masks for this step
                    from ..ops.fused import graph_seq_advance
                    graph_seq_advance(entry.rng_dev)
                entry.fwd_graph.replay()
                return tuple(o.detach() for o in entry.static_out)

            @staticmethod
            def backward(ctx, *gouts):
                for buf, g in zip(entry.static_gout, gouts):
                    if g is None:
                        buf.zero_()
                    else:
                        buf.copy_(g, non_blocking=True)
                entry.bwd_graph.replay()
                if entry.accumulate:   # already added into the parameters' .grad
                    return tuple(None for _ in range(len(entry.static_in) + len(entry.params)))
                gi = iter(entry.static_grads)
                res = []
                for m in entry.diff_mask:
                    res.append(next(gi).clone() if m else None)
                for _ in entry.params:
                    g = next(gi)
                    res.append(None if g is None else g.clone())
                return tuple(res)
        self._fn = _Graphed

    def __call__(self, args, kwargs):
        ins = [t._t for t in _flat_tensors((args, kwargs), [])]
        outs = self._fn.apply(*ins, *[p._t for p in self.params])
        it = iter(outs)

        def rebuild(o):
            if isinstance(o, Tensor):
                return Tensor(next(it))
            if isinstance(o, list):
                return [rebuild(x) for x in o]
            if isinstance(o, tuple):
                return tuple(rebuild(x) for x in o)
            if isinstance(o, dict):
                return {k: rebuild(v) for k, v in o.items()}
            return o
        return rebuild(self.out_struct)


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

    def _use_train_graph(self, args, kwargs):
        bs = self._build_strategy
        if not (bs is not None and getattr(bs, 'use_hip_graph', False)):
            return False  # training capture is opt-in: parameters must keep their storage
        if not torch.cuda.is_available() or not torch.is_grad_enabled():
            return False
        ins = _flat_tensors((args, kwargs), [])
        return bool(ins) and all(t._t.is_cuda for t in ins) and self._needs_grad(args, kwargs)

    def __call__(self, *args, **kwargs):
        from ..static import _STATIC
        if not _enabled[0] or _STATIC[0]:
            return self._fn(*args, **kwargs)
        if self._use_train_graph(args, kwargs):
            key = ('train',) + _signature(args, kwargs)
            g = self._graphs.get(key)
            if g is None:
                params = self._layer.parameters() if self._layer is not None else []
                g = self._capture(key, lambda: _TrainGraph(self._fn, params, args, kwargs))
            if not isinstance(g, _Eager):
                return g(args, kwargs)
        elif self._use_graph(args, kwargs):
            key = _signature(args, kwargs)
            g = self._graphs.get(key)
            if g is None:
                g = self._capture(key, lambda: _GraphEntry(self._fn, args, kwargs))
            if not isinstance(g, _Eager):
                return g(args, kwargs)
        return self._fn(*args, **kwargs)

    def _capture(self, key, build):
        """Capture a graph for ``key``; if the function cannot be captured the error is
        swallowed, the half-built graph discarded, and the signature runs eagerly in this
        process from then on (no restart, no retry per call)."""
        try:
            g = build()
        except Exception as e:  # noqa: BLE001 - any capture failure means: not capturable
            torch.cuda.synchronize()
            g = _Eager()
            g.reason = f'{type(e).__name__}: {e}'
        self._graphs[key] = g
        return g

    def graph_status(self):
        """{signature: 'graph' | 'eager (<why the capture failed>)'} for the calls seen so far."""
        return {k: ('eager (' + v.reason + ')') if isinstance(v, _Eager) else 'graph'
                for k, v in self._graphs.items()}

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
    """Trace ``fn`` on symbolic inputs -> (Program, feed Variables, fetch Variables).
    ``fn`` is first control-flow converted (dy2static.convert_function): an ``if`` / ``while``
    on a tensor value records both branches / the loop as sub-blocks decided at run time."""
    from .. import static
    from ..static import graph as G
    from .dy2static import convert_function
    fn = convert_function(fn)
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
