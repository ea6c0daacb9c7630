"""paddle.profiler (parity: python/paddle/profiler/{profiler.py,profiler_statistic.py,timer.py,
utils.py}). See profiler.py (recording), result.py (the ProfilerResult and its protobuf /
Chrome-trace forms), statistic.py (summary views) and timer.py (reader / batch cost)."""
import contextlib

from .result import TracerEventType, TracerMemEventType, ProfilerResult, load_profiler_result  # noqa: F401
from .statistic import SortedKeys, StatisticData, build_table  # noqa: F401
from .profiler import (ProfilerState, ProfilerTarget, SummaryView, Profiler, RecordEvent,  # noqa: F401
                       make_scheduler, export_chrome_tracing, export_protobuf, wrap_optimizers,
                       in_profiler_mode)
from . import timer  # noqa: F401

__all__ = ['ProfilerState', 'ProfilerTarget', 'make_scheduler', 'export_chrome_tracing', 'export_protobuf',
           'Profiler', 'RecordEvent', 'load_profiler_result', 'SortedKeys', 'SummaryView']


@contextlib.contextmanager
def _nvprof_range(iter_id, start, end, exit_after_prof=True):
    yield
