"""Reader decorators (parity: python/paddle/reader/decorator.py).

A *reader* is a zero-argument callable returning an iterable of samples; a decorator
takes readers and returns a new reader. Thread-based decorators (buffered, xmap_readers)
overlap sample production with consumption; multiprocess_reader runs each reader in its
own forked process and merges their samples through one queue.
"""
import itertools
import multiprocessing
import queue as _queue
import random
import sys
import threading

__all__ = []


def cache(reader):
    """Materialize the reader once; the returned reader replays the cached samples."""
    data = tuple(reader())

    def cached():
        yield from data
    return cached


def map_readers(func, *readers):
    """Reader of func(s1, s2, ...) over the zipped outputs of ``readers``."""
    def mapped():
        yield from map(func, *[r() for r in readers])
    return mapped


def shuffle(reader, buf_size):
    """Shuffle within consecutive windows of ``buf_size`` samples."""
    def shuffled():
        buf = []
        for e in reader():
            buf.append(e)
            if len(buf) >= buf_size:
                random.shuffle(buf)
                yield from buf
                buf = []
        if buf:
            random.shuffle(buf)
            yield from buf
    return shuffled


def chain(*readers):
    """Outputs of the readers one after another."""
    def chained():
        yield from itertools.chain(*[r() for r in readers])
    return chained


class ComposeNotAligned(ValueError):
    pass


def compose(*readers, **kwargs):
    """Zip readers into flat tuples: (1, 2), 3, (4, 5) -> (1, 2, 3, 4, 5). With
    ``check_alignment`` (default) readers of different lengths raise ComposeNotAligned."""
    check = kwargs.pop('check_alignment', True)
    as_tuple = lambda x: x if isinstance(x, tuple) else (x,)  # noqa: E731
    _missing = object()

    def composed():
        its = [r() for r in readers]
        rows = itertools.zip_longest(*its, fillvalue=_missing) if check else zip(*its)
        for outs in rows:
            if check and any(o is _missing for o in outs):
                raise ComposeNotAligned("outputs of readers are not aligned.")
            yield sum((as_tuple(o) for o in outs), ())
    return composed


class _End:
    pass


def buffered(reader, size):
    """Produce samples on a background thread into a queue of at most ``size``."""
    def buffered_reader():
        q = _queue.Queue(maxsize=size)
        end = _End()
        err = []

        def work():
            try:
                for d in reader():
                    q.put(d)
            except BaseException as e:  # surfaced in the consumer
                err.append(e)
            q.put(end)
        threading.Thread(target=work, daemon=True).start()
        while True:
            e = q.get()
            if e is end:
                if err:
                    raise err[0]
                return
            yield e
    return buffered_reader


def firstn(reader, n):
    """At most the first ``n`` samples."""
    def limited():
        yield from itertools.islice(reader(), n)
    return limited


XmapEndSignal = _End


def xmap_readers(mapper, reader, process_num, buffer_size, order=False):
    """Map samples with ``process_num`` worker threads; ``order`` keeps input order."""
    def xreader():
        in_q = _queue.Queue(buffer_size)
        out_q = _queue.Queue(buffer_size)
        end = _End()

        def feed():
            for i, s in enumerate(reader()):
                in_q.put((i, s))
            for _ in range(process_num):
                in_q.put(end)

        def work():
            while True:
                item = in_q.get()
                if item is end:
                    out_q.put(end)
                    return
                i, s = item
                out_q.put((i, mapper(s)))
        threading.Thread(target=feed, daemon=True).start()
        for _ in range(process_num):
            threading.Thread(target=work, daemon=True).start()
        done, nxt, pending = 0, 0, {}
        while done < process_num:
            item = out_q.get()
            if item is end:
                done += 1
                continue
            if not order:
                yield item[1]
                continue
            pending[item[0]] = item[1]
            while nxt in pending:
                yield pending.pop(nxt)
                nxt += 1
        while order and nxt in pending:
            yield pending.pop(nxt)
            nxt += 1
    return xreader


def _mp_worker(reader, q):
    try:
        for sample in reader():
            if sample is None:
                raise ValueError("sample has None")
            q.put(sample)
        q.put(None)
    except Exception:
        q.put('')
        raise


def multiprocess_reader(readers, use_pipe=True, queue_size=1000):
    """Run every reader in a forked process and merge their samples (order between
    readers is not defined). ``use_pipe`` is accepted for API parity; one queue is used."""
    if sys.platform == 'win32':
        raise NotImplementedError("The multiprocess_reader method is not supported on windows.")
    if not isinstance(readers, (list, tuple)) or not readers:
        raise ValueError("`readers` must be a non-empty list or tuple.")
    ctx = multiprocessing.get_context('fork')

    def merged():
        q = ctx.Queue(queue_size)
        procs = [ctx.Process(target=_mp_worker, args=(r, q), daemon=True) for r in readers]
        for p in procs:
            p.start()
        finished = 0
        try:
            while finished < len(readers):
                s = q.get()
                if s is None:
                    finished += 1
                elif isinstance(s, str) and s == '':
                    raise ValueError("multiprocess_reader: a reader process failed")
                else:
                    yield s
        finally:
            for p in procs:
                p.join(timeout=5)
    return merged
