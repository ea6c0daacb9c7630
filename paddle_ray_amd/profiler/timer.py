"""Benchmark timer: reader cost, batch cost and ips per step (parity: python/paddle/profiler/
timer.py:51-222 -- Event / TimerHook / Benchmark; the DataLoader calls ``before_reader`` /
``after_reader`` around every batch it hands out, the Profiler calls ``begin`` / ``step`` /
``end``). Nested tasks (an evaluation loop with its own DataLoader inside training) pause the
outer task's timing until its own reader is used again.
"""
import timeit

_SKIP = 10   # the first iterations are excluded from the max / min / summary records


class _Stat:
    __slots__ = ('total', 'n', 'max', 'min')

    def __init__(self):
        self.total, self.n, self.max, self.min = 0.0, 0, 0.0, float('inf')

    def add(self, v):
        self.total += v
        self.n += 1
        self.max = max(self.max, v)
        self.min = min(self.min, v)


class Event:
    """The timing state of one task (training, or a nested evaluation)."""

    def __init__(self):
        self.reader_window, self.batch_window = [], []   # since the last step_info()
        self.samples_window = []
        self.reader = _Stat()                           # records after the skipped iterations
        self.batch = _Stat()
        self.speed = _Stat()
        self.iters = 0
        self.total_samples = 0
        self.reader_obj = None
        self.need_record = True
        self.speed_mode = 'samples/s'
        self.speed_unit = 'samples/s'

    def reset(self):
        self.reader_window, self.batch_window, self.samples_window = [], [], []

    def record_reader(self, t):
        self.reader_window.append(t)
        if self.iters >= _SKIP:
            self.reader.add(t)

    def record_batch(self, t, num_samples=None):
        if num_samples is None:
            self.speed_mode = self.speed_unit = 'steps/s'
        self.batch_window.append(t)
        self.samples_window.append(num_samples)
        self.iters += 1
        if self.iters >= _SKIP:
            self.batch.add(t)
            if num_samples is not None:
                self.total_samples += num_samples
                self.speed.add(num_samples / t if t > 0 else 0.0)
            else:
                self.speed.add(1.0 / t if t > 0 else 0.0)

    def reader_average(self):
        return sum(self.reader_window) / len(self.reader_window) if self.reader_window else 0.0

    def batch_average(self):
        return sum(self.batch_window) / len(self.batch_window) if self.batch_window else 0.0

    def speed_average(self):
        tot = sum(self.batch_window)
        if not tot:
            return 0.0
        if self.speed_mode == 'samples/s':
            return sum(s or 0 for s in self.samples_window) / tot
        return len(self.batch_window) / tot

    def get_summary(self):
        if self.iters <= _SKIP:
            return {}
        rd = self.reader.total / self.reader.n if self.reader.n else 0.0
        bt = self.batch.total / self.batch.n if self.batch.n else 0.0
        if self.speed_mode == 'samples/s':
            ips = self.total_samples / self.batch.total if self.batch.total else 0.0
        else:
            ips = self.batch.n / self.batch.total if self.batch.total else 0.0
        return {'reader_summary': {'avg': rd, 'max': self.reader.max, 'min': self.reader.min if self.reader.n else 0.0},
                'batch_summary': {'avg': bt, 'max': self.batch.max, 'min': self.batch.min if self.batch.n else 0.0},
                'ips_summary': {'avg': ips, 'max': self.speed.max, 'min': self.speed.min if self.speed.n else 0.0},
                'reader_ratio': 100.0 * rd / bt if bt else 0.0}


class Hook:
    def begin(self, benchmark):
        pass

    def end(self, benchmark):
        pass

    def before_reader(self, benchmark):
        pass

    def after_reader(self, benchmark):
        pass

    def after_step(self, benchmark):
        pass


class TimerHook(Hook):
    def __init__(self):
        self.start_time = timeit.default_timer()
        self.start_reader = self.start_time

    def begin(self, benchmark):
        benchmark.events.append(Event())
        benchmark.current_event = benchmark.events[-1]
        self.start_time = timeit.default_timer()

    def before_reader(self, benchmark):
        self.start_reader = timeit.default_timer()

    def after_reader(self, benchmark):
        cost = timeit.default_timer() - self.start_reader
        ev = benchmark.current_event
        if ev is None or not ev.need_record or cost == 0:
            return
        ev.record_reader(cost)

    def after_step(self, benchmark):
        ev = benchmark.current_event
        if ev is None or not ev.need_record:
            return
        now = timeit.default_timer()
        ev.record_batch(now - self.start_time, benchmark.num_samples)
        self.start_time = now

    def end(self, benchmark):
        if not benchmark.events:
            return
        self.print_summary(benchmark)
        benchmark.events.pop()
        benchmark.current_event = benchmark.events[-1] if benchmark.events else None
        self.start_time = timeit.default_timer()

    @staticmethod
    def print_summary(benchmark):
        s = benchmark.current_event.get_summary()
        if not s:
            return
        print(' Perf Summary '.center(100, '='))
        if s['reader_ratio']:
            print(f"Reader Ratio: {s['reader_ratio']:.3f}%")
        print(f'Time Unit: s, IPS Unit: {benchmark.current_event.speed_unit}')
        print('|' + ''.center(17) + '|' + 'avg'.center(17) + '|' + 'max'.center(17) + '|' + 'min'.center(17) + '|')
        rows = [('batch_cost', s['batch_summary']), ('ips', s['ips_summary'])]
        if s['reader_summary']['avg']:
            rows.insert(0, ('reader_cost', s['reader_summary']))
        for name, d in rows:
            print('|' + name.center(17) + '|' + f"{d['avg']:.5f}".center(17) + '|' +
                  f"{d['max']:.5f}".center(17) + '|' + f"{d['min']:.5f}".center(17) + '|')


class Benchmark:
    def __init__(self):
        self.num_samples = None
        self.hooks = {'timer_hook': TimerHook()}
        self.current_event = None
        self.events = []

    def begin(self):
        for h in self.hooks.values():
            h.begin(self)

    def end(self):
        for h in self.hooks.values():
            h.end(self)

    def before_reader(self):
        for h in self.hooks.values():
            h.before_reader(self)

    def after_reader(self):
        for h in self.hooks.values():
            h.after_reader(self)

    def after_step(self):
        for h in self.hooks.values():
            h.after_step(self)

    def step(self, num_samples=None):
        self.num_samples = num_samples
        self.after_step()

    def step_info(self, unit=None):
        ev = self.current_event
        if ev is None:
            return ''
        msg = ''
        r, b = ev.reader_average(), ev.batch_average()
        if r:
            msg += f' reader_cost: {r:.5f} s'
        if b:
            ev.speed_unit = 'steps/s' if ev.speed_mode == 'steps/s' else f'{unit or "samples"}/s'
            msg += f' batch_cost: {b:.5f} s'
        sp = ev.speed_average()
        if sp:
            msg += f' ips: {sp:.3f} {ev.speed_unit}'
        ev.reset()
        return msg

    def check_if_need_record(self, reader):
        """A DataLoader is about to produce a batch: pause the current task's timing while a
        different reader (a nested evaluation) runs, resume when its own reader comes back."""
        ev = self.current_event
        if ev is None:
            return
        ds = getattr(reader, 'dataset', None)
        if ev.need_record:
            if ev.reader_obj is None:
                ev.reader_obj = reader
            elif getattr(ev.reader_obj, 'dataset', None) is not ds:
                ev.need_record = False
        elif getattr(ev.reader_obj, 'dataset', None) is ds:
            ev.need_record = True
            self.hooks['timer_hook'].start_time = timeit.default_timer()


_bm = Benchmark()


def benchmark():
    return _bm
