"""paddle.profiler (parity: python/paddle/profiler/{profiler.py,timer.py,utils.py}).

Host ranges (RecordEvent) are recorded by our own tracer AND forwarded to the
PyTorch-ROCm profiler (roctracer/rocprofiler-sdk) so device kernels of the
hand-written HIP library appear in the same Chrome trace; summary tables are
aggregated per event name.
"""
import collections
import contextlib
import json
import os
import threading
import time
from enum import Enum

import torch


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


class SortedKeys(Enum):
    CPUTotal = 0
    CPUAvg = 1
    CPUMax = 2
    CPUMin = 3
    GPUTotal = 4
    GPUAvg = 5
    GPUMax = 6
    GPUMin = 7


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


_tls = threading.local()
_active = []


class RecordEvent:
    def __init__(self, name, event_type=None):
        self.name = name
        self._t0 = None
        self._rf = None

    def begin(self):
        self._t0 = time.perf_counter_ns()
        if _active:
            self._rf = torch.profiler.record_function(self.name)
            self._rf.__enter__()

    def end(self):
        if self._t0 is None:
            return
        t1 = time.perf_counter_ns()
        if self._rf is not None:
            self._rf.__exit__(None, None, None)
            self._rf = None
        for p in _active:
            p._host_events.append((self.name, self._t0, t1, threading.get_ident()))
        self._t0 = None

    def __enter__(self):
        self.begin()
        return self

    def __exit__(self, *a):
        self.end()


def make_scheduler(*, closed, ready, record, repeat=0, skip_first=0):
    def sched(step):
        s = step - skip_first
        if s < 0:
            return ProfilerState.CLOSED
        period = closed + ready + record
        if repeat > 0 and s // period >= repeat:
            return ProfilerState.CLOSED
        m = s % period
        if m < closed:
            return ProfilerState.CLOSED
        if m < closed + ready:
            return ProfilerState.READY
        return ProfilerState.RECORD_AND_RETURN if m == period - 1 else ProfilerState.RECORD
    return sched


def export_chrome_tracing(dir_name, worker_name=None):
    def handler(prof):
        os.makedirs(dir_name, exist_ok=True)
        name = worker_name or f'host_{os.getpid()}'
        prof.export(os.path.join(dir_name, f'{name}.pt.trace.json'), 'json')
    return handler


def export_protobuf(dir_name, worker_name=None):
    return export_chrome_tracing(dir_name, worker_name)


class Profiler:
    def __init__(self, *, targets=None, scheduler=None, on_trace_ready=None, record_shapes=False,
                 profile_memory=False, timer_only=False, emit_nvtx=False, custom_device_types=[],
                 with_flops=False):
        self.targets = targets or [ProfilerTarget.CPU] + (
            [ProfilerTarget.GPU] if torch.cuda.is_available() else [])
        if isinstance(scheduler, (tuple, list)):
            lo, hi = scheduler
            scheduler = make_scheduler(closed=max(lo, 0), ready=0, record=hi - lo, repeat=1)
        self.scheduler = scheduler
        self.on_trace_ready = on_trace_ready
        self.timer_only = timer_only
        self.record_shapes, self.profile_memory = record_shapes, profile_memory
        self._host_events = []
        self._tp = None
        self._recording = False
        self.step_num = 0
        self._step_times = []
        self._t_step = None

    def _want_record(self):
        if self.scheduler is None:
            return True
        return self.scheduler(self.step_num) in (ProfilerState.RECORD,
                                                 ProfilerState.RECORD_AND_RETURN)

    def _open(self):
        if self._recording:
            return
        self._recording = True
        _active.append(self)
        if self.timer_only:
            return
        acts = [torch.profiler.ProfilerActivity.CPU]
        if ProfilerTarget.GPU in self.targets and torch.cuda.is_available():
            acts.append(torch.profiler.ProfilerActivity.CUDA)
        self._tp = torch.profiler.profile(activities=acts, record_shapes=self.record_shapes,
                                          profile_memory=self.profile_memory)
        self._tp.__enter__()

    def _close(self):
        if not self._recording:
            return
        self._recording = False
        if self in _active:
            _active.remove(self)
        if self._tp is not None:
            self._tp.__exit__(None, None, None)
        if self.on_trace_ready is not None:
            self.on_trace_ready(self)

    def start(self):
        self._t_step = time.perf_counter()
        if self._want_record():
            self._open()

    def stop(self):
        self._close()

    def step(self, num_samples=None):
        now = time.perf_counter()
        if self._t_step is not None:
            self._step_times.append((now - self._t_step, num_samples))
        self._t_step = now
        self.step_num += 1
        rec = self._want_record()
        if rec and not self._recording:
            self._open()
        elif not rec and self._recording:
            self._close()

    def step_info(self, unit=None):
        if not self._step_times:
            return ''
        ts = [t for t, _ in self._step_times]
        avg = sum(ts) / len(ts)
        s = f'reader_cost: 0.0 s batch_cost: {avg:.5f} s ips: {1.0 / avg:.3f} steps/s'
        ns = [n for _, n in self._step_times if n]
        if ns:
            s += f' {sum(ns) / sum(ts):.3f} {unit or "samples"}/s'
        return s

    def export(self, path, format='json'):
        if self._tp is not None:
            self._tp.export_chrome_trace(path)
        else:
            evs = [{'name': n, 'ph': 'X', 'ts': a / 1000, 'dur': (b - a) / 1000, 'pid': os.getpid(),
                    'tid': tid} for n, a, b, tid in self._host_events]
            with open(path, 'w') as f:
                json.dump({'traceEvents': evs}, f)

    def summary(self, sorted_by=SortedKeys.CPUTotal, op_detail=True, thread_sep=False,
                time_unit='ms', views=None):
        agg = collections.defaultdict(lambda: [0, 0.0, 0.0, float('inf')])
        for n, a, b, _ in self._host_events:
            d = (b - a) / 1e6
            r = agg[n]
            r[0] += 1
            r[1] += d
            r[2] = max(r[2], d)
            r[3] = min(r[3], d)
        lines = [f'{"Name":40s} {"Calls":>8s} {"Total(ms)":>12s} {"Avg(ms)":>10s} {"Max(ms)":>10s}']
        for n, (c, tot, mx, mn) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            lines.append(f'{n[:40]:40s} {c:8d} {tot:12.3f} {tot / c:10.3f} {mx:10.3f}')
        if self._tp is not None:
            try:
                lines.append(self._tp.key_averages().table(
                    sort_by='cuda_time_total' if torch.cuda.is_available() else 'cpu_time_total',
                    row_limit=30))
            except Exception:
                pass
        out = '\n'.join(lines)
        print(out)
        return out

    def __enter__(self):
        self.start()
        return self

    def __exit__(self, *a):
        self.stop()


def load_profiler_result(filename):
    with open(filename) as f:
        return json.load(f)


@contextlib.contextmanager
def _nvprof_range(iter_id, start, end, exit_after_prof=True):
    yield


from . import timer  # noqa: E402,F401
