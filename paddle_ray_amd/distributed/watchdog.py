"""Collective watchdog + rank heartbeat (failure detection).

Parity: the reference's comm-task watchdog / timeouts in
paddle/fluid/distributed/collective/process_group_nccl.cc (per-task timeout checks) and the
elastic/heartbeat failure detection in python/paddle/distributed/fleet/elastic/manager.py.

* ``CommWatchdog``: every collective issued through ``paddle_ray_amd.distributed`` is
  registered (op name, group size, issue time) until it completes. A daemon thread polls
  the in-flight set; a task older than ``PRA_COMM_WATCHDOG_S`` (default 600 s) is reported
  once with rank, op, elapsed time and ALL Python thread stacks (``faulthandler``), so a
  hang shows which collective and which code path each rank was in. With
  ``PRA_COMM_WATCHDOG_ABORT=1`` the process then exits (non-zero) so the launcher can
  restart the job from its last checkpoint instead of hanging until the RCCL timeout.
* ``Heartbeat``: each rank bumps ``pra_hb/<rank>`` in the rendezvous TCPStore every
  ``interval`` seconds; ``dead_ranks()`` lists peers whose heartbeat is stale.
"""
import faulthandler
import itertools
import logging
import os
import sys
import threading
import time

_log = logging.getLogger('paddle_ray_amd.watchdog')


class CommWatchdog:
    def __init__(self, timeout_s=None, poll_s=1.0, abort=None):
        self.timeout_s = float(timeout_s if timeout_s is not None
                               else os.environ.get('PRA_COMM_WATCHDOG_S', 600))
        self.abort = (os.environ.get('PRA_COMM_WATCHDOG_ABORT', '0') == '1') if abort is None \
            else abort
        self.poll_s = poll_s
        self._tasks = {}
        self._ids = itertools.count()
        self._lock = threading.Lock()
        self._thread = None
        self.reports = []
        self.on_timeout = None

    def _ensure_thread(self):
        if self._thread is None or not self._thread.is_alive():
            self._thread = threading.Thread(target=self._loop, name='pra-comm-watchdog',
                                            daemon=True)
            self._thread.start()

    def track(self, name, work, nranks=None):
        tid = next(self._ids)
        with self._lock:
            self._tasks[tid] = [name, work, time.monotonic(), nranks, False]
        self._ensure_thread()
        return tid

    def done(self, tid):
        with self._lock:
            self._tasks.pop(tid, None)

    def in_flight(self):
        with self._lock:
            return [(v[0], time.monotonic() - v[2]) for v in self._tasks.values()]

    def _loop(self):
        while True:
            time.sleep(self.poll_s)
            now = time.monotonic()
            expired = []
            with self._lock:
                for tid, rec in list(self._tasks.items()):
                    name, work, t0, nranks, reported = rec
                    try:
                        if work is not None and work.is_completed():
                            del self._tasks[tid]
                            continue
                    except Exception:  # noqa: BLE001 - a failed work is reported below
                        pass
                    if not reported and now - t0 > self.timeout_s:
                        rec[4] = True
                        expired.append((name, now - t0, nranks))
            for name, el, nranks in expired:
                self._report(name, el, nranks)

    def _report(self, name, elapsed, nranks):
        rank = os.environ.get('RANK', os.environ.get('PADDLE_TRAINER_ID', '0'))
        msg = (f"[comm watchdog] rank {rank}: collective '{name}' (group of {nranks}) "
               f"not complete after {elapsed:.1f}s (limit {self.timeout_s:.0f}s)")
        self.reports.append(msg)
        _log.error(msg)
        print(msg, file=sys.stderr, flush=True)
        try:
            faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
        except Exception:  # noqa: BLE001
            pass
        if self.on_timeout is not None:
            self.on_timeout(name, elapsed)
        if self.abort:
            os._exit(17)


_WATCHDOG = [None]


def get_watchdog():
    if _WATCHDOG[0] is None:
        _WATCHDOG[0] = CommWatchdog()
    return _WATCHDOG[0]


def enabled():
    return os.environ.get('PRA_COMM_WATCHDOG', '1') != '0'


class Heartbeat:
    """Per-rank liveness in the rendezvous store."""

    def __init__(self, store=None, rank=None, world_size=None, interval=5.0, prefix='pra_hb'):
        import torch.distributed as dist
        if store is None:
            from torch.distributed import distributed_c10d as c10d
            store = c10d._get_default_store()
        self.store = store
        self.rank = dist.get_rank() if rank is None else rank
        self.world = dist.get_world_size() if world_size is None else world_size
        self.interval = interval
        self.prefix = prefix
        self._stop = threading.Event()
        self._thread = None

    def beat(self):
        self.store.set(f'{self.prefix}/{self.rank}', repr(time.time()))

    def start(self):
        self.beat()

        def loop():
            while not self._stop.wait(self.interval):
                try:
                    self.beat()
                except Exception:  # noqa: BLE001 - store gone: job is ending
                    return
        self._thread = threading.Thread(target=loop, name='pra-heartbeat', daemon=True)
        self._thread.start()
        return self

    def stop(self):
        self._stop.set()

    def last_seen(self):
        out = {}
        for r in range(self.world):
            try:
                self.store.wait([f'{self.prefix}/{r}'], __import__('datetime').timedelta(
                    milliseconds=10))
                out[r] = float(self.store.get(f'{self.prefix}/{r}').decode())
            except Exception:  # noqa: BLE001 - never seen
                out[r] = None
        return out

    def dead_ranks(self, stale_s=None):
        stale_s = stale_s if stale_s is not None else 3 * self.interval
        now = time.time()
        return [r for r, t in self.last_seen().items() if t is None or now - t > stale_s]


class TrackedWork:
    """An async RCCL work registered with the watchdog until ``wait()`` returns — used by the
    hot-path reducers (DataParallel buckets, sharding reduce-scatter / all-gather, pipeline
    p2p) that call ``torch.distributed`` directly."""

    __slots__ = ('work', 'tid')

    def __init__(self, name, work, nranks=None):
        self.work = work
        self.tid = get_watchdog().track(name, work, nranks) if (work is not None and enabled()) \
            else None

    def wait(self):
        if self.work is not None:
            self.work.wait()
        if self.tid is not None:
            get_watchdog().done(self.tid)
            self.tid = None
        return True

    def is_completed(self):
        return self.work is None or self.work.is_completed()


def track(name, work, nranks=None):
    return TrackedWork(name, work, nranks)
