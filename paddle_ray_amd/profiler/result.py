"""Profiling result: host ranges, device activities, memory events and steps on one clock (ns),
serialisable to a protobuf file and to a Chrome trace (parity: the C++ ProfilerResult of
paddle/fluid/platform/profiler/profiler_result.h and its dump/serialization_logger.cc; the
field layout below is this framework's own ``ProfilerResultProto``).

Sources (``collect``): the framework's own host tracer (RecordEvent ranges with their
TracerEventType, profiler steps) and, unless the profiler is timer-only, the PyTorch-ROCm
profiler's event tree -- aten operators with the device time of the kernels they launched, the
device kernels / copies themselves (roctracer / rocprofiler-sdk activity records of the
hand-written HIP kernels and the library ones), and allocator events with ``profile_memory``.
The two clocks are aligned on the profiler's own step / RecordEvent ranges, which both record."""
import enum
import json
import os


class TracerEventType(enum.Enum):
    """parity: paddle/phi/api/profiler/trace_event.h TracerEventType"""
    Operator = 0
    Dataloader = 1
    ProfileStep = 2
    CudaRuntime = 3
    Kernel = 4
    Memcpy = 5
    Memset = 6
    UserDefined = 7
    OperatorInner = 8
    Forward = 9
    Backward = 10
    Optimization = 11
    Communication = 12
    PythonOp = 13
    PythonUserDefined = 14
    MluRuntime = 15


class TracerMemEventType(enum.Enum):
    Allocate = 0
    Free = 1
    ReservedAllocate = 2
    ReservedFree = 3


class HostEvent:
    __slots__ = ('name', 'type', 'start_ns', 'end_ns', 'tid', 'gpu_ns', 'kernels')

    def __init__(self, name, type, start_ns, end_ns, tid=0, gpu_ns=0, kernels=None):
        self.name, self.type = name, type
        self.start_ns, self.end_ns, self.tid = int(start_ns), int(end_ns), int(tid)
        self.gpu_ns = int(gpu_ns)
        self.kernels = kernels or []     # [(kernel name, device ns)] launched by this range

    @property
    def dur_ns(self):
        return self.end_ns - self.start_ns


class DeviceEvent:
    __slots__ = ('name', 'type', 'start_ns', 'end_ns', 'device', 'stream')

    def __init__(self, name, type, start_ns, end_ns, device=0, stream=0):
        self.name, self.type = name, type
        self.start_ns, self.end_ns = int(start_ns), int(end_ns)
        self.device, self.stream = int(device), int(stream)

    @property
    def dur_ns(self):
        return self.end_ns - self.start_ns

    # a kernel's "thread" in the statistics tables is its stream; its device time is itself
    @property
    def tid(self):
        return self.stream

    @property
    def gpu_ns(self):
        return self.end_ns - self.start_ns

    kernels = None


class MemEvent:
    __slots__ = ('name', 'place', 'bytes', 'type', 'ts_ns')

    def __init__(self, name, place, nbytes, type, ts_ns):
        self.name, self.place, self.bytes, self.type, self.ts_ns = name, place, int(nbytes), type, int(ts_ns)


# -- protobuf schema (registered with the in-tree proto2 codec of static/program_desc.py) ----------
_SCHEMA = {
    'PraHostEvent': {1: ('name', 'string', False), 2: ('type', 'enum', False), 3: ('start_ns', 'int64', False),
                     4: ('end_ns', 'int64', False), 5: ('thread_id', 'int64', False),
                     6: ('gpu_ns', 'int64', False), 7: ('kernels', 'm:PraKernelRef', True)},
    'PraKernelRef': {1: ('name', 'string', False), 2: ('dur_ns', 'int64', False)},
    'PraDeviceEvent': {1: ('name', 'string', False), 2: ('type', 'enum', False), 3: ('start_ns', 'int64', False),
                       4: ('end_ns', 'int64', False), 5: ('device_id', 'int32', False),
                       6: ('stream_id', 'int64', False)},
    'PraMemEvent': {1: ('name', 'string', False), 2: ('place', 'string', False), 3: ('bytes', 'int64', False),
                    4: ('type', 'enum', False), 5: ('ts_ns', 'int64', False)},
    'PraStep': {1: ('step', 'int32', False), 2: ('start_ns', 'int64', False), 3: ('end_ns', 'int64', False)},
    'PraKV': {1: ('key', 'string', False), 2: ('value', 'string', False)},
    'PraProfilerResult': {1: ('version', 'string', False), 2: ('span_index', 'int64', False),
                          3: ('host_events', 'm:PraHostEvent', True),
                          4: ('device_events', 'm:PraDeviceEvent', True),
                          5: ('mem_events', 'm:PraMemEvent', True), 6: ('steps', 'm:PraStep', True),
                          7: ('extra_info', 'm:PraKV', True)},
}
def _codec():
    from ..static import program_desc as pd
    if 'PraProfilerResult' not in pd._SCHEMA:
        pd._SCHEMA.update(_SCHEMA)
    return pd


class ProfilerResult:
    """What one recording span produced (``Profiler.profiler_result``)."""

    def __init__(self, host_events=None, device_events=None, mem_events=None, steps=None, extra_info=None,
                 span_index=0):
        self.host_events = list(host_events or [])
        self.device_events = list(device_events or [])
        self.mem_events = list(mem_events or [])
        self.steps = list(steps or [])          # [(step number, start ns, end ns)]
        self.extra_info = dict(extra_info or {})
        self.span_index = span_index

    # reference ProfilerResult accessors
    def get_data(self):
        return self

    def get_extra_info(self):
        return dict(self.extra_info)

    def get_span_indx(self):
        return self.span_index

    def has_device(self):
        return bool(self.device_events)

    # -- protobuf ---------------------------------------------------------------------------------------
    def to_proto_dict(self):
        return {
            'version': '1', 'span_index': self.span_index,
            'host_events': [{'name': e.name, 'type': e.type.value, 'start_ns': e.start_ns, 'end_ns': e.end_ns,
                             'thread_id': e.tid, 'gpu_ns': e.gpu_ns,
                             'kernels': [{'name': k, 'dur_ns': int(d)} for k, d in e.kernels]}
                            for e in self.host_events],
            'device_events': [{'name': e.name, 'type': e.type.value, 'start_ns': e.start_ns, 'end_ns': e.end_ns,
                               'device_id': e.device, 'stream_id': e.stream} for e in self.device_events],
            'mem_events': [{'name': m.name, 'place': m.place, 'bytes': m.bytes, 'type': m.type.value,
                            'ts_ns': m.ts_ns} for m in self.mem_events],
            'steps': [{'step': s, 'start_ns': a, 'end_ns': b} for s, a, b in self.steps],
            'extra_info': [{'key': str(k), 'value': str(v)} for k, v in self.extra_info.items()],
        }

    def save(self, path, format='pb'):
        if format in ('pb', 'protobuf'):
            with open(path, 'wb') as f:
                f.write(_codec().encode('PraProfilerResult', self.to_proto_dict()))
        else:
            with open(path, 'w') as f:
                json.dump(self.chrome_trace(), f)

    @classmethod
    def from_proto_bytes(cls, data):
        d = _codec().decode('PraProfilerResult', data)
        hes = [HostEvent(h.get('name', ''), TracerEventType(h.get('type', 7)), h.get('start_ns', 0),
                         h.get('end_ns', 0), h.get('thread_id', 0), h.get('gpu_ns', 0),
                         [(k.get('name', ''), k.get('dur_ns', 0)) for k in h.get('kernels', [])])
               for h in d.get('host_events', [])]
        des = [DeviceEvent(e.get('name', ''), TracerEventType(e.get('type', 4)), e.get('start_ns', 0),
                           e.get('end_ns', 0), e.get('device_id', 0), e.get('stream_id', 0))
               for e in d.get('device_events', [])]
        mes = [MemEvent(m.get('name', ''), m.get('place', ''), m.get('bytes', 0),
                        TracerMemEventType(m.get('type', 0)), m.get('ts_ns', 0)) for m in d.get('mem_events', [])]
        steps = [(s.get('step', 0), s.get('start_ns', 0), s.get('end_ns', 0)) for s in d.get('steps', [])]
        extra = {kv.get('key', ''): kv.get('value', '') for kv in d.get('extra_info', [])}
        return cls(hes, des, mes, steps, extra, d.get('span_index', 0))

    # -- chrome trace -----------------------------------------------------------------------------------
    def chrome_trace(self):
        pid = os.getpid()
        evs = []
        for e in self.host_events:
            evs.append({'name': e.name, 'ph': 'X', 'cat': e.type.name, 'ts': e.start_ns / 1e3,
                        'dur': e.dur_ns / 1e3, 'pid': pid, 'tid': e.tid})
        for e in self.device_events:
            evs.append({'name': e.name, 'ph': 'X', 'cat': e.type.name, 'ts': e.start_ns / 1e3,
                        'dur': e.dur_ns / 1e3, 'pid': f'GPU:{e.device}', 'tid': f'stream {e.stream}'})
        for m in self.mem_events:
            evs.append({'name': f'[memory] {m.name}', 'ph': 'i', 's': 't', 'cat': 'Memory', 'ts': m.ts_ns / 1e3,
                        'pid': pid, 'tid': 0, 'args': {'bytes': m.bytes, 'place': m.place, 'type': m.type.name}})
        return {'traceEvents': evs, 'displayTimeUnit': 'ms', 'extra_info': self.extra_info}


def load_profiler_result(filename):
    """A ProfilerResult from a protobuf dump (export_protobuf), or the parsed JSON of a Chrome
    trace (export_chrome_tracing)."""
    with open(filename, 'rb') as f:
        data = f.read()
    if filename.endswith('.json') or data.lstrip()[:1] == b'{':
        return json.loads(data.decode())
    return ProfilerResult.from_proto_bytes(data)


# -- collection from the PyTorch profiler ------------------------------------------------------------
_COMM_PAT = ('nccl', 'rccl', 'allreduce', 'all_reduce', 'allgather', 'all_gather', 'reducescatter',
             'reduce_scatter', 'broadcast', 'sendrecv', 'alltoall', 'c10d::')


def is_comm_kernel(name):
    n = name.lower()
    return any(p in n for p in _COMM_PAT)


def _device_type(name):
    n = name.lower()
    if 'memcpy' in n or 'copybuffer' in n or 'copy_buffer' in n:
        return TracerEventType.Memcpy
    if 'memset' in n or 'fillbuffer' in n:
        return TracerEventType.Memset
    return TracerEventType.Kernel


def merge_torch_events(res, tp_events, own_names):
    """Fold the PyTorch profiler's event tree into ``res`` (in place). ``own_names`` are the names
    our tracer recorded (RecordEvent / steps), which torch saw as user annotations: matching
    them occurrence by occurrence gives the clock offset and each range's device time."""
    import torch
    cuda = torch.autograd.DeviceType.CUDA
    cpu_evs, dev_evs, mem_evs, dev_ann = [], [], [], {}
    for e in tp_events:
        if e.name == '[memory]':
            mem_evs.append(e)
        elif getattr(e, 'device_type', None) == cuda:
            if e.name in own_names:
                # the device-side mirror of one of our ranges (gpu_user_annotation): the span of
                # the kernels launched inside it, natively launched ones included
                dev_ann.setdefault(e.name, []).append(e)
            else:
                dev_evs.append(e)
        else:
            cpu_evs.append(e)
    # 1) clock: pair our ranges with torch's annotation events of the same name, k-th with k-th
    ours = {}
    for h in res.host_events:
        ours.setdefault(h.name, []).append(h)
    for v in ours.values():
        v.sort(key=lambda h: h.start_ns)
    theirs = {}
    for e in cpu_evs:
        if e.name in own_names:
            theirs.setdefault(e.name, []).append(e)
    offsets = []
    for name, tl in theirs.items():
        tl.sort(key=lambda e: e.time_range.start)
        for h, e in zip(ours.get(name, []), tl):
            offsets.append(h.start_ns - int(e.time_range.start * 1000))
            h.gpu_ns = int(e.device_time_total * 1000)
            h.kernels = _kernels_of(e)
    offsets.sort()
    off = offsets[len(offsets) // 2] if offsets else 0
    for name, dl in dev_ann.items():
        dl.sort(key=lambda e: e.time_range.start)
        for h, e in zip(sorted(ours.get(name, []), key=lambda h: h.start_ns), dl):
            g = int(getattr(e, 'device_time_total', 0) * 1000) or int((e.time_range.end - e.time_range.start) * 1000)
            h.gpu_ns = max(h.gpu_ns, g)
    # 1b) kernels launched straight through the HIP runtime (the in-tree kernels: no aten op
    # around them) are credited to every one of our ranges their launch call falls in, by the
    # runtime API event's time (its .kernels are linked by correlation id)
    own = sorted(res.host_events, key=lambda h: h.start_ns)
    starts = [h.start_ns for h in own]
    launched = {}
    import bisect
    for e in cpu_evs:
        ks = getattr(e, 'kernels', None)
        if not ks or e.name.startswith('aten::') or e.name in own_names:
            continue
        t = int(e.time_range.start * 1000) + off
        dur = sum(int(getattr(k, 'duration', 0) * 1000) for k in ks)
        for h in own[:bisect.bisect_right(starts, t)]:
            if h.end_ns >= t:
                launched[id(h)] = launched.get(id(h), 0) + dur
    for h in own:
        if launched.get(id(h), 0) > h.gpu_ns:
            h.gpu_ns = launched[id(h)]
    # 2) operators: top-level aten ops (an op nested in another aten op is its inner detail)
    for e in cpu_evs:
        if not e.name.startswith('aten::'):
            continue
        p = e.cpu_parent
        if p is not None and p.name.startswith('aten::'):
            continue
        res.host_events.append(HostEvent(e.name, TracerEventType.Operator, int(e.time_range.start * 1000) + off,
                                         int(e.time_range.end * 1000) + off, e.thread,
                                         int(e.device_time_total * 1000), _kernels_of(e)))
    # 3) device activities
    for e in dev_evs:
        res.device_events.append(DeviceEvent(e.name, _device_type(e.name), int(e.time_range.start * 1000) + off,
                                             int(e.time_range.end * 1000) + off, getattr(e, 'device_index', 0) or 0,
                                             getattr(e, 'thread', 0) or 0))
    # 4) allocator events (profile_memory)
    for e in mem_evs:
        nb = getattr(e, 'device_memory_usage', 0) or 0
        place = 'gpu' if nb else 'cpu'
        if not nb:
            nb = getattr(e, 'cpu_memory_usage', 0) or 0
        if not nb:
            continue
        parent = e.cpu_parent.name if e.cpu_parent is not None else 'unknown'
        res.mem_events.append(MemEvent(parent, place, abs(nb), TracerMemEventType.Allocate if nb > 0
                                       else TracerMemEventType.Free, int(e.time_range.start * 1000) + off))


def _kernels_of(e):
    out = []
    for k in getattr(e, 'kernels', []) or []:
        out.append((k.name, int(getattr(k, 'duration', 0) * 1000)))
    return out
