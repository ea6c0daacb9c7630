"""Benchmark timer (parity: python/paddle/profiler/timer.py)."""
import time


class Benchmark:
    def __init__(self):
        self.reset()

    def reset(self):
        self._t0 = None
        self._costs = []
        self._samples = []

    def begin(self):
        self._t0 = time.perf_counter()

    def step(self, num_samples=None):
        t = time.perf_counter()
        if self._t0 is not None:
            self._costs.append(t - self._t0)
            self._samples.append(num_samples or 0)
        self._t0 = t

    def end(self):
        self._t0 = None

    def step_info(self, unit='samples'):
        if not self._costs:
            return ''
        avg = sum(self._costs) / len(self._costs)
        ips = sum(self._samples) / sum(self._costs) if any(self._samples) else 1 / avg
        return f'batch_cost: {avg:.5f} s, ips: {ips:.3f} {unit}/s'


_bm = Benchmark()


def benchmark():
    return _bm
