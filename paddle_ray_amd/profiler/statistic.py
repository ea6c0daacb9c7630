"""Summary tables of a ProfilerResult (parity: python/paddle/profiler/profiler_statistic.py:857
StatisticData, :875 _build_table -- Device / Overview / Model / Distributed / Operator / Kernel /
Memory-manipulation / User-defined / Memory views, rows ranked by SortedKeys, times in a chosen
unit).

Time accounting (this framework's own formulation):
* a category's time is the UNION of its ranges (nested or overlapping ranges of one type are
  not counted twice);
* steps are the profiler's ProfileStep ranges (one pseudo-step spanning the recording when the
  loop never called ``step``); the Model view's "Others" is the step time no Dataloader /
  Forward / Backward / Optimization range covers;
* device time of a host range is the time of the kernels it launched (PyTorch-profiler
  correlation); device utilisation is the union of kernel intervals over the step time;
* Distributed view: communication = union of collective kernels (RCCL) and Communication
  ranges, computation = union of the other kernels, overlap = their intersection.
"""
import collections
from enum import Enum

from .result import TracerEventType as TT, TracerMemEventType, is_comm_kernel


class SortedKeys(Enum):
    CPUTotal = 0
    CPUAvg = 1
    CPUMax = 2
    CPUMin = 3
    GPUTotal = 4
    GPUAvg = 5
    GPUMax = 6
    GPUMin = 7


_UNIT = {'s': 1e9, 'ms': 1e6, 'us': 1e3, 'ns': 1.0}


def _union(ranges):
    """Total length of the union of [a, b) ranges, and the merged list."""
    rs = sorted((a, b) for a, b in ranges if b > a)
    merged = []
    for a, b in rs:
        if merged and a <= merged[-1][1]:
            if b > merged[-1][1]:
                merged[-1][1] = b
        else:
            merged.append([a, b])
    return sum(b - a for a, b in merged), merged


def _intersect(m1, m2):
    i = j = tot = 0
    while i < len(m1) and j < len(m2):
        a, b = max(m1[i][0], m2[j][0]), min(m1[i][1], m2[j][1])
        if b > a:
            tot += b - a
        if m1[i][1] < m2[j][1]:
            i += 1
        else:
            j += 1
    return tot


def _clip(ranges, lo, hi):
    return [(max(a, lo), min(b, hi)) for a, b in ranges if b > lo and a < hi]


class _Item:
    """Per-name statistics (calls, cpu / gpu total, max, min)."""
    __slots__ = ('name', 'calls', 'cpu', 'cpu_max', 'cpu_min', 'gpu', 'gpu_max', 'gpu_min', 'children', 'tid')

    def __init__(self, name, tid=0):
        self.name, self.tid = name, tid
        self.calls, self.cpu, self.gpu = 0, 0, 0
        self.cpu_max, self.gpu_max = 0, 0
        self.cpu_min, self.gpu_min = float('inf'), float('inf')
        self.children = None

    def add(self, cpu_ns, gpu_ns):
        self.calls += 1
        self.cpu += cpu_ns
        self.cpu_max = max(self.cpu_max, cpu_ns)
        self.cpu_min = min(self.cpu_min, cpu_ns)
        self.gpu += gpu_ns
        self.gpu_max = max(self.gpu_max, gpu_ns)
        self.gpu_min = min(self.gpu_min, gpu_ns)

    def key(self, k):
        c = max(self.calls, 1)
        return {SortedKeys.CPUTotal: self.cpu, SortedKeys.CPUAvg: self.cpu / c, SortedKeys.CPUMax: self.cpu_max,
                SortedKeys.CPUMin: self.cpu_min, SortedKeys.GPUTotal: self.gpu, SortedKeys.GPUAvg: self.gpu / c,
                SortedKeys.GPUMax: self.gpu_max, SortedKeys.GPUMin: self.gpu_min}[k]


def _rank(items, sorted_by):
    asc = sorted_by in (SortedKeys.CPUMin, SortedKeys.GPUMin)
    return sorted(items, key=lambda it: (it.key(sorted_by) if asc else -it.key(sorted_by), it.name))


class StatisticData:
    """Aggregates of one ProfilerResult, consumed by ``build_table``."""

    def __init__(self, result, extra_info=None):
        self.result = result
        self.extra_info = dict(extra_info or getattr(result, 'extra_info', {}) or {})
        hes, des = result.host_events, result.device_events
        self.steps = [(n, a, b) for n, a, b in result.steps if b > a]
        if not self.steps:
            ends = [e.end_ns for e in hes] + [e.end_ns for e in des]
            starts = [e.start_ns for e in hes] + [e.start_ns for e in des]
            if starts:
                self.steps = [(0, min(starts), max(ends))]
        self.step_ns = sum(b - a for _, a, b in self.steps)
        self.kernels = [e for e in des if e.type == TT.Kernel]
        self.memops = [e for e in des if e.type in (TT.Memcpy, TT.Memset)]
        self.devices = sorted({e.device for e in des})
        by_type = collections.defaultdict(list)
        for e in hes:
            by_type[e.type].append(e)
        self.by_type = by_type

        def items(events, detail=False):
            d = {}
            for e in events:
                it = d.get((e.name, e.tid))
                if it is None:
                    it = d[(e.name, e.tid)] = _Item(e.name, e.tid)
                it.add(e.dur_ns, e.gpu_ns)
                if detail and e.kernels:
                    if it.children is None:
                        it.children = {}
                    for kn, kd in e.kernels:
                        c = it.children.get(kn)
                        if c is None:
                            c = it.children[kn] = _Item(kn)
                        c.add(0, kd)
            return d
        self.op_items = items(by_type[TT.Operator] + by_type[TT.PythonOp], detail=True)
        self.udf_items = items(by_type[TT.UserDefined] + by_type[TT.PythonUserDefined], detail=True)
        self.kernel_items = items(self.kernels)
        for it in self.kernel_items.values():      # device items: the time is GPU time
            it.gpu, it.gpu_max, it.gpu_min = it.cpu, it.cpu_max, it.cpu_min
        self.memop_items = items(self.memops)
        for it in self.memop_items.values():
            it.gpu, it.gpu_max, it.gpu_min = it.cpu, it.cpu_max, it.cpu_min

    # -- per-type / per-step aggregates ------------------------------------------------------------------
    def cpu_union(self, types, lo=None, hi=None):
        rs = [(e.start_ns, e.end_ns) for t in types for e in self.by_type.get(t, [])]
        if lo is not None:
            rs = _clip(rs, lo, hi)
        return _union(rs)

    def gpu_of(self, types, lo=None, hi=None):
        tot = 0
        for t in types:
            for e in self.by_type.get(t, []):
                if lo is None or (e.start_ns >= lo and e.start_ns < hi):
                    tot += e.gpu_ns
        return tot

    def device_union(self, events, lo=None, hi=None):
        rs = [(e.start_ns, e.end_ns) for e in events]
        if lo is not None:
            rs = _clip(rs, lo, hi)
        return _union(rs)


# -- table rendering -----------------------------------------------------------------------------------
class _Table:
    def __init__(self, title, headers, widths):
        self.title, self.headers, self.widths = title, headers, widths
        self.rows = []

    def add(self, *cells):
        self.rows.append([str(c) for c in cells])

    def render(self):
        w = list(self.widths)
        for r in self.rows + [self.headers]:
            for i, c in enumerate(r):
                w[i] = max(w[i], len(c))
        total = sum(w) + 2 * (len(w) - 1)
        line = '-' * total
        out = [self.title.center(total, '-'), line,
               '  '.join(h.ljust(w[i]) if i == 0 else h.rjust(w[i]) for i, h in enumerate(self.headers)), line]
        for r in self.rows:
            out.append('  '.join(c.ljust(w[i]) if i == 0 else c.rjust(w[i]) for i, c in enumerate(r)))
        out.append(line)
        return '\n'.join(out)


def build_table(data, sorted_by=SortedKeys.CPUTotal, op_detail=True, thread_sep=False, time_unit='ms',
                views=None, row_limit=100):
    from .profiler import SummaryView
    if time_unit not in _UNIT:
        raise ValueError(f"time_unit must be one of {list(_UNIT)}, got {time_unit!r}")
    if isinstance(views, SummaryView):
        views = [views]
    want = (lambda v: True) if views is None else (lambda v: v in views)
    div = _UNIT[time_unit]
    ft = lambda ns: f'{ns / div:.3f}' if ns != float('inf') else '-'  # noqa: E731
    fr = lambda x, tot: f'{100.0 * x / tot:.2f}%' if tot else '0.00%'  # noqa: E731
    u = time_unit
    out = []
    total = data.step_ns

    if want(SummaryView.DeviceView):
        t = _Table('Device Summary', ['Device', 'Utilization(%)', f'Busy({u})', f'Total({u})'], [20, 14, 12, 12])
        cpu_busy, _ = data.cpu_union(list(TT))
        t.add('CPU(host tracer)', fr(cpu_busy, total), ft(cpu_busy), ft(total))
        for d in data.devices:
            busy, _ = data.device_union([k for k in data.kernels if k.device == d])
            t.add(f'GPU{d}', fr(busy, total), ft(busy), ft(total))
        out.append(t.render())

    if want(SummaryView.OverView):
        t = _Table('Overview Summary', ['Event Type', 'Calls', f'CPU Time({u})', 'Ratio(%)', f'GPU Time({u})'],
                   [26, 8, 14, 10, 14])
        t.add('ProfileStep', len(data.steps), ft(total), '100.00%', ft(data.device_union(data.kernels)[0]))
        for ty in (TT.Dataloader, TT.Forward, TT.Backward, TT.Optimization, TT.Communication, TT.Operator,
                   TT.PythonOp, TT.UserDefined, TT.PythonUserDefined, TT.OperatorInner):
            evs = data.by_type.get(ty, [])
            if not evs:
                continue
            cpu, _ = data.cpu_union([ty])
            t.add(ty.name, len(evs), ft(cpu), fr(cpu, total), ft(data.gpu_of([ty])))
        for name, evs in (('Kernel', data.kernels), ('Memcpy', [e for e in data.memops if e.type == TT.Memcpy]),
                          ('Memset', [e for e in data.memops if e.type == TT.Memset])):
            if evs:
                g, _ = data.device_union(evs)
                t.add(f'{name}(device)', len(evs), '-', '-', ft(g))
        out.append(t.render())

    if want(SummaryView.ModelView):
        t = _Table('Model Summary', ['Name', 'Calls', f'CPU Total({u})', f'Avg({u})', f'Max({u})', f'Min({u})',
                                     'Ratio(%)', f'GPU Total({u})', 'Ratio(%)'], [14, 6, 12, 10, 10, 10, 9, 12, 9])
        durs = [b - a for _, a, b in data.steps]
        gpu_steps = [data.device_union(data.kernels, a, b)[0] for _, a, b in data.steps]
        gtot = sum(gpu_steps)
        if durs:
            t.add('ProfileStep', len(durs), ft(total), ft(total / len(durs)), ft(max(durs)), ft(min(durs)),
                  '100.00%', ft(gtot), '100.00%' if gtot else '0.00%')
        covered = []
        for ty in (TT.Dataloader, TT.Forward, TT.Backward, TT.Optimization):
            per, calls, g = [], 0, 0
            for _, a, b in data.steps:
                c, m = data.cpu_union([ty], a, b)
                per.append(c)
                covered += [tuple(x) for x in m]
                calls += sum(1 for e in data.by_type.get(ty, []) if a <= e.start_ns < b)
                g += data.gpu_of([ty], a, b)
            if calls:
                tot = sum(per)
                t.add(ty.name, calls, ft(tot), ft(tot / len(per)), ft(max(per)), ft(min(per)), fr(tot, total),
                      ft(g), fr(g, gtot))
        cov, _ = _union(covered)
        others = max(total - cov, 0)
        t.add('Others', '-', ft(others), '-', '-', '-', fr(others, total), '-', '-')
        out.append(t.render())

    if want(SummaryView.DistributedView):
        comm_k = [k for k in data.kernels if is_comm_kernel(k.name)]
        comp_k = [k for k in data.kernels if not is_comm_kernel(k.name)]
        comm_h = [(e.start_ns, e.end_ns) for e in data.by_type.get(TT.Communication, [])]
        if comm_k or comm_h:
            ct, cm = _union([(k.start_ns, k.end_ns) for k in comm_k] + comm_h)
            pt, pm = _union([(k.start_ns, k.end_ns) for k in comp_k])
            ov = _intersect(cm, pm)
            t = _Table('Distribution Summary', ['Name', f'Total Time({u})', 'Ratio(%)'], [26, 14, 10])
            t.add('ProfileStep', ft(total), '100.00%')
            t.add('  Communication', ft(ct), fr(ct, total))
            t.add('  Computation', ft(pt), fr(pt, total))
            t.add('  Overlap', ft(ov), fr(ov, total))
            out.append(t.render())

    def item_view(title, items, detail, gpu_only=False, sort=sorted_by):
        if not items:
            return
        if gpu_only:
            if sort in (SortedKeys.CPUTotal, SortedKeys.CPUAvg, SortedKeys.CPUMax, SortedKeys.CPUMin):
                sort = SortedKeys.GPUTotal
            t = _Table(title, ['Name', 'Calls', f'GPU Total({u})', f'Avg({u})', f'Max({u})', f'Min({u})',
                               'Ratio(%)'], [48, 6, 12, 10, 10, 10, 9])
            gt = sum(it.gpu for it in items.values())
            for it in _rank(items.values(), sort)[:row_limit]:
                t.add(it.name[:90], it.calls, ft(it.gpu), ft(it.gpu / it.calls), ft(it.gpu_max), ft(it.gpu_min),
                      fr(it.gpu, gt))
            out.append(t.render())
            return
        groups = collections.defaultdict(dict)
        for k, it in items.items():
            merged_key = k if thread_sep else k[0]
            g = groups[k[1] if thread_sep else 0]
            cur = g.get(merged_key)
            if cur is None:
                g[merged_key] = it
            else:        # same name on several threads, merged
                m = _Item(it.name)
                for src in (cur, it):
                    m.calls += src.calls
                    m.cpu += src.cpu
                    m.gpu += src.gpu
                    m.cpu_max, m.gpu_max = max(m.cpu_max, src.cpu_max), max(m.gpu_max, src.gpu_max)
                    m.cpu_min, m.gpu_min = min(m.cpu_min, src.cpu_min), min(m.gpu_min, src.gpu_min)
                    m.children = src.children or m.children
                g[merged_key] = m
        t = _Table(title, ['Name', 'Calls', f'CPU Total({u})', f'Avg({u})', f'Max({u})', f'Min({u})', 'Ratio(%)',
                           f'GPU Total({u})', f'Avg({u})', 'Ratio(%)'], [40, 6, 12, 10, 10, 10, 9, 12, 10, 9])
        for tid, g in sorted(groups.items()):
            if thread_sep:
                t.add(f'Thread: {tid}', '', '', '', '', '', '', '', '', '')
            ct = sum(it.cpu for it in g.values())
            gt = sum(it.gpu for it in g.values())
            for it in _rank(g.values(), sort)[:row_limit]:
                c = max(it.calls, 1)
                t.add(it.name[:80], it.calls, ft(it.cpu), ft(it.cpu / c), ft(it.cpu_max), ft(it.cpu_min),
                      fr(it.cpu, ct), ft(it.gpu), ft(it.gpu / c), fr(it.gpu, gt))
                if detail and op_detail and it.children:
                    for ch in _rank(it.children.values(), SortedKeys.GPUTotal)[:10]:
                        t.add('  ' + ch.name[:78], ch.calls, '-', '-', '-', '-', '-', ft(ch.gpu),
                              ft(ch.gpu / max(ch.calls, 1)), fr(ch.gpu, it.gpu or 1))
        out.append(t.render())

    if want(SummaryView.OperatorView):
        item_view('Operator Summary', data.op_items, True)
    if want(SummaryView.KernelView):
        item_view('Kernel Summary', data.kernel_items, False, gpu_only=True)
    if want(SummaryView.MemoryManipulationView):
        item_view('Memory Manipulation Summary', data.memop_items, False, gpu_only=True)
    if want(SummaryView.UDFView):
        item_view('UserDefined Summary', data.udf_items, True)

    if want(SummaryView.MemoryView) and (data.result.mem_events or 'peak_allocated' in data.extra_info):
        t = _Table('Memory Summary', ['Event / Place', 'Alloc Calls', 'Alloc Size(MB)', 'Free Calls',
                                      'Free Size(MB)', 'Net(MB)'], [40, 11, 14, 10, 13, 10])
        per = collections.defaultdict(lambda: [0, 0, 0, 0])
        for m in data.result.mem_events:
            r = per[(m.name, m.place)]
            if m.type in (TracerMemEventType.Allocate, TracerMemEventType.ReservedAllocate):
                r[0] += 1
                r[1] += m.bytes
            else:
                r[2] += 1
                r[3] += m.bytes
        for (name, place), (ac, asz, fc, fsz) in sorted(per.items(), key=lambda kv: -kv[1][1])[:row_limit]:
            t.add(f'{name[:30]} ({place})', ac, f'{asz / 2**20:.3f}', fc, f'{fsz / 2**20:.3f}',
                  f'{(asz - fsz) / 2**20:.3f}')
        for k in ('peak_allocated', 'peak_reserved'):
            if k in data.extra_info:
                t.add(k, '-', f'{float(data.extra_info[k]) / 2**20:.3f}', '-', '-', '-')
        out.append(t.render())
    return '\n\n'.join(out)
