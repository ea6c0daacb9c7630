"""paddle.profiler.Profiler (parity: python/paddle/profiler/profiler.py -- scheduler states,
targets, on_trace_ready exporters, step / step_info / summary / export).

Recording: the framework's host tracer keeps typed ranges (RecordEvent, profiler steps, and the
Forward / Backward / Optimization / Dataloader / Communication ranges the framework opens on its
own hot paths while a profiler records). Unless ``timer_only``, the PyTorch-ROCm profiler runs
alongside for the device side (kernels of the in-tree HIP library, library kernels, copies) and
aten operators; ``result.merge_torch_events`` folds both into one ProfilerResult."""
import datetime
import os
import socket
import threading
import time
from enum import Enum

import torch

from . import _hooks
from .result import ProfilerResult, HostEvent, TracerEventType, merge_torch_events
from .statistic import SortedKeys, StatisticData, build_table
from .timer import benchmark


class ProfilerState(Enum):
    CLOSED = 0
    READY = 1
    RECORD = 2
    RECORD_AND_RETURN = 3


class ProfilerTarget(Enum):
    CPU = 0
    GPU = 1
    XPU = 2
    CUSTOM_DEVICE = 3


class SummaryView(Enum):
    DeviceView = 0
    OverView = 1
    ModelView = 2
    DistributedView = 3
    KernelView = 4
    OperatorView = 5
    MemoryView = 6
    MemoryManipulationView = 7
    UDFView = 8


def make_scheduler(*, closed, ready, record, repeat=0, skip_first=0):
    """Step -> state: skip_first CLOSED steps, then cycles of closed / ready / record steps (the
    last record step of a cycle is RECORD_AND_RETURN), ``repeat`` cycles (0: forever)."""
    def sched(step):
        s = step - skip_first
        if s < 0:
            return ProfilerState.CLOSED
        period = closed + ready + record
        if period <= 0 or (repeat > 0 and s // period >= repeat):
            return ProfilerState.CLOSED
        m = s % period
        if m < closed:
            return ProfilerState.CLOSED
        if m < closed + ready:
            return ProfilerState.READY
        return ProfilerState.RECORD_AND_RETURN if m == period - 1 else ProfilerState.RECORD
    return sched


def _default_scheduler(step):
    return ProfilerState.RECORD


def _worker_name(worker_name):
    return worker_name or f'host_{socket.gethostname()}pid_{os.getpid()}'


def export_chrome_tracing(dir_name, worker_name=None):
    """on_trace_ready handler writing ``<worker>_time_<stamp>.paddle_trace.json`` (Chrome trace)."""
    os.makedirs(dir_name, exist_ok=True)

    def handler(prof):
        stamp = datetime.datetime.now().strftime('%Y_%m_%d_%H_%M_%S_%f')
        prof.export(os.path.join(dir_name, f'{_worker_name(worker_name)}_time_{stamp}.paddle_trace.json'), 'json')
    return handler


def export_protobuf(dir_name, worker_name=None):
    """on_trace_ready handler writing ``<worker>_time_<stamp>.paddle_trace.pb`` (a protobuf
    ProfilerResult; load_profiler_result reads it back)."""
    os.makedirs(dir_name, exist_ok=True)

    def handler(prof):
        stamp = datetime.datetime.now().strftime('%Y_%m_%d_%H_%M_%S_%f')
        prof.export(os.path.join(dir_name, f'{_worker_name(worker_name)}_time_{stamp}.paddle_trace.pb'), 'pb')
    return handler


class RecordEvent:
    """A user range (parity: python/paddle/profiler/utils.py:37). Recorded only while a
    Profiler records; also forwarded to the PyTorch profiler so its device kernels correlate."""

    def __init__(self, name, event_type=TracerEventType.PythonUserDefined):
        self.name = name
        self.event_type = event_type
        self._t0 = None
        self._rf = None

    def begin(self):
        if not _hooks.ACTIVE:
            return
        self._t0 = time.perf_counter_ns()
        if any(p._tp is not None for p in _hooks.ACTIVE):
            self._rf = torch.profiler.record_function(self.name)
            self._rf.__enter__()

    def end(self):
        if self._t0 is None:
            return
        t1 = time.perf_counter_ns()
        if self._rf is not None:
            self._rf.__exit__(None, None, None)
            self._rf = None
        tid = threading.get_ident()
        for p in _hooks.ACTIVE:
            p._add(HostEvent(self.name, self.event_type, self._t0, t1, tid))
        self._t0 = None

    def __enter__(self):
        self.begin()
        return self

    def __exit__(self, *a):
        self.end()

    def __call__(self, fn):
        import functools

        @functools.wraps(fn)
        def wrapped(*a, **k):
            with RecordEvent(self.name, self.event_type):
                return fn(*a, **k)
        return wrapped


_wrapped_optimizers = set()


def wrap_optimizers():
    """Optimizer.step of every optimizer class opens an Optimization range while a profiler
    records (parity: profiler/utils.py wrap_optimizers)."""
    from ..optimizer.optimizer import Optimizer
    todo = [Optimizer]
    seen = []
    while todo:
        c = todo.pop()
        seen.append(c)
        todo += c.__subclasses__()
    for cls in seen:
        if cls in _wrapped_optimizers or 'step' not in cls.__dict__:
            continue
        fn = cls.__dict__['step']

        def make(fn, cls):
            def step(self, *a, **k):
                if not _hooks.ACTIVE:
                    return fn(self, *a, **k)
                with RecordEvent(f'{cls.__name__}.step', TracerEventType.Optimization):
                    return fn(self, *a, **k)
            step.__wrapped__ = fn
            step.__doc__ = fn.__doc__
            return step
        cls.step = make(fn, cls)
        _wrapped_optimizers.add(cls)


class Profiler:
    def __init__(self, *, targets=None, scheduler=None, on_trace_ready=None, record_shapes=False,
                 profile_memory=False, timer_only=False, emit_nvtx=False, custom_device_types=[],
                 with_flops=False):
        if targets is None:
            targets = [ProfilerTarget.CPU] + ([ProfilerTarget.GPU] if torch.cuda.is_available() else [])
        self.targets = list(targets)
        if isinstance(scheduler, (tuple, list)):
            lo, hi = scheduler
            if not (0 <= lo < hi):
                raise ValueError(f"scheduler=(start_batch, end_batch) needs 0 <= start < end, got {scheduler}")
            scheduler = make_scheduler(closed=max(lo - 1, 0), ready=1 if lo > 0 else 0, record=hi - lo, repeat=1)
        self.scheduler = scheduler or _default_scheduler
        self.on_trace_ready = on_trace_ready
        self.timer_only = timer_only
        self.record_shapes, self.profile_memory, self.with_flops = record_shapes, profile_memory, with_flops
        self.step_num = 0
        self.previous_state = ProfilerState.CLOSED
        self.current_state = self.scheduler(0)
        self.profiler_result = None
        self._events = []
        self._own_names = set()
        self._steps = []
        self._step_open = None
        self._step_rf = None
        self._tp = None
        self._recording = False
        self._span = 0
        self._lock = threading.Lock()

    # -- recording ---------------------------------------------------------------------------------------
    def _add(self, ev):
        with self._lock:
            self._events.append(ev)
            self._own_names.add(ev.name)

    def _open_step(self):
        self._step_open = (self.step_num, time.perf_counter_ns())
        if self._tp is not None:
            self._step_rf = torch.profiler.record_function(f'ProfileStep#{self.step_num}')
            self._step_rf.__enter__()

    def _close_step(self):
        if self._step_open is None:
            return
        n, t0 = self._step_open
        t1 = time.perf_counter_ns()
        if self._step_rf is not None:
            self._step_rf.__exit__(None, None, None)
            self._step_rf = None
        self._add(HostEvent(f'ProfileStep#{n}', TracerEventType.ProfileStep, t0, t1, threading.get_ident()))
        self._steps.append((n, t0, t1))
        self._step_open = None

    def _open(self):
        if self._recording:
            return
        self._recording = True
        self._events, self._steps, self._own_names = [], [], set()
        wrap_optimizers()
        if not self.timer_only:
            acts = [torch.profiler.ProfilerActivity.CPU]
            if ProfilerTarget.GPU in self.targets and torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self._tp = torch.profiler.profile(activities=acts, record_shapes=self.record_shapes,
                                              profile_memory=self.profile_memory, with_flops=self.with_flops)
            self._tp.__enter__()
        _hooks.ACTIVE.append(self)
        self._open_step()

    def _close(self):
        if not self._recording:
            return
        self._close_step()
        if self in _hooks.ACTIVE:
            _hooks.ACTIVE.remove(self)
        self._recording = False
        res = ProfilerResult(self._events, steps=self._steps, span_index=self._span)
        self._span += 1
        if self._tp is not None:
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            self._tp.__exit__(None, None, None)
            try:
                merge_torch_events(res, self._tp.events(), self._own_names)
            except Exception as e:   # a torch-side trace problem must not lose the host tracer's data
                res.extra_info['device_trace_error'] = repr(e)
        if torch.cuda.is_available():
            try:
                res.extra_info['peak_allocated'] = torch.cuda.max_memory_allocated()
                res.extra_info['peak_reserved'] = torch.cuda.max_memory_reserved()
            except Exception:
                pass
        res.extra_info.setdefault('targets', ','.join(t.name for t in self.targets))
        self.profiler_result = res
        if self.on_trace_ready is not None:
            self.on_trace_ready(self)
        self._tp = None

    # -- public -----------------------------------------------------------------------------------------
    def start(self):
        benchmark().begin()
        if self.timer_only:
            return
        if self.current_state in (ProfilerState.RECORD, ProfilerState.RECORD_AND_RETURN):
            self._open()

    def stop(self):
        benchmark().end()
        if self.timer_only:
            return
        self._close()

    def step(self, num_samples=None):
        benchmark().step(num_samples)
        if self.timer_only:
            return
        if self._recording:
            self._close_step()
        self.previous_state = self.current_state
        self.step_num += 1
        self.current_state = self.scheduler(self.step_num)
        rec = (ProfilerState.RECORD, ProfilerState.RECORD_AND_RETURN)
        if self._recording:
            if self.previous_state == ProfilerState.RECORD_AND_RETURN or self.current_state not in rec:
                self._close()
                if self.current_state in rec:
                    self._open()
            else:
                self._open_step()
        elif self.current_state in rec:
            self._open()

    def step_info(self, unit=None):
        """' reader_cost: .. s batch_cost: .. s ips: ..' averaged since the previous call (the
        reader cost comes from the DataLoader's before/after-reader hooks)."""
        return benchmark().step_info(unit)

    def export(self, path='', format='json'):
        if self.profiler_result is None:
            raise RuntimeError("Profiler.export: nothing recorded yet (call it from on_trace_ready or after stop)")
        self.profiler_result.save(path, 'pb' if format in ('pb', 'protobuf') else 'json')

    def summary(self, sorted_by=SortedKeys.CPUTotal, op_detail=True, thread_sep=False, time_unit='ms',
                views=None):
        """Print (and return) the summary tables of the last recorded span; ``views`` limits
        them, ``sorted_by`` ranks the operator / kernel / user-defined rows, ``time_unit`` in
        ('s', 'ms', 'us', 'ns')."""
        if self.profiler_result is None:
            return ''
        s = build_table(StatisticData(self.profiler_result), sorted_by=sorted_by, op_detail=op_detail,
                        thread_sep=thread_sep, time_unit=time_unit, views=views)
        print(s)
        return s

    def __enter__(self):
        self.start()
        return self

    def __exit__(self, *a):
        self.stop()


def in_profiler_mode():
    return bool(_hooks.ACTIVE)
