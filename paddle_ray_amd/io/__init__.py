"""paddle.io — datasets, samplers, DataLoader (parity: python/paddle/io/__init__.py,
python/paddle/fluid/dataloader/{dataset,batch_sampler,sampler,dataloader_iter}.py).

DataLoader: worker processes (``num_workers``) produce numpy batches; the main
process pins them and issues non-blocking H2D copies on a side HIP stream one
batch ahead (``use_buffer_reader``), so the copy overlaps the previous step.
"""
import bisect
import itertools
import math
import queue
import threading

import numpy as np
import torch

from ..framework.core import Tensor, _u, _default_device


class Dataset:
    def __getitem__(self, idx):
        raise NotImplementedError

    def __len__(self):
        raise NotImplementedError


class IterableDataset(Dataset):
    def __iter__(self):
        raise NotImplementedError


class TensorDataset(Dataset):
    def __init__(self, tensors):
        self.tensors = tensors
        n = len(tensors[0])
        assert all(len(t) == n for t in tensors)

    def __getitem__(self, i):
        return tuple(t[i] for t in self.tensors)

    def __len__(self):
        return len(self.tensors[0])


class ComposeDataset(Dataset):
    def __init__(self, datasets):
        self.datasets = list(datasets)

    def __len__(self):
        return len(self.datasets[0])

    def __getitem__(self, i):
        out = []
        for d in self.datasets:
            s = d[i]
            out.extend(s if isinstance(s, (list, tuple)) else [s])
        return tuple(out)


class ChainDataset(IterableDataset):
    def __init__(self, datasets):
        self.datasets = list(datasets)

    def __iter__(self):
        for d in self.datasets:
            yield from d


class Subset(Dataset):
    def __init__(self, dataset, indices):
        self.dataset, self.indices = dataset, list(indices)

    def __getitem__(self, i):
        return self.dataset[self.indices[i]]

    def __len__(self):
        return len(self.indices)


class ConcatDataset(Dataset):
    def __init__(self, datasets):
        self.datasets = list(datasets)
        self.cum = list(itertools.accumulate(len(d) for d in self.datasets))

    def __len__(self):
        return self.cum[-1]

    def __getitem__(self, i):
        di = bisect.bisect_right(self.cum, i)
        prev = self.cum[di - 1] if di else 0
        return self.datasets[di][i - prev]


def random_split(dataset, lengths, generator=None):
    n = len(dataset)
    if all(0 < l < 1 for l in lengths) and abs(sum(lengths) - 1) < 1e-6:
        lengths = [int(math.floor(n * f)) for f in lengths]
        for i in range(n - sum(lengths)):
            lengths[i % len(lengths)] += 1
    perm = np.random.permutation(n).tolist()
    out, off = [], 0
    for l in lengths:
        out.append(Subset(dataset, perm[off:off + l]))
        off += l
    return out


class Sampler:
    def __init__(self, data_source=None):
        self.data_source = data_source

    def __iter__(self):
        raise NotImplementedError


class SequenceSampler(Sampler):
    def __iter__(self):
        return iter(range(len(self.data_source)))

    def __len__(self):
        return len(self.data_source)


class RandomSampler(Sampler):
    def __init__(self, data_source, replacement=False, num_samples=None, generator=None):
        super().__init__(data_source)
        self.replacement, self._num_samples = replacement, num_samples
        self.generator = generator

    @property
    def num_samples(self):
        return len(self.data_source) if self._num_samples is None else self._num_samples

    def __iter__(self):
        n = len(self.data_source)
        if self.generator is not None:
            yield from (next(self.generator) for _ in range(self.num_samples))
            return
        if self.replacement:
            yield from np.random.randint(0, n, self.num_samples).tolist()
        else:
            yield from np.random.permutation(n).tolist()[:self.num_samples]

    def __len__(self):
        return self.num_samples


class WeightedRandomSampler(Sampler):
    def __init__(self, weights, num_samples, replacement=True):
        self.weights = np.asarray(weights, dtype=np.float64)
        self.num_samples, self.replacement = num_samples, replacement

    def __iter__(self):
        p = self.weights / self.weights.sum()
        yield from np.random.choice(len(p), self.num_samples, self.replacement, p).tolist()

    def __len__(self):
        return self.num_samples


class SubsetRandomSampler(Sampler):
    def __init__(self, indices):
        self.indices = list(indices)

    def __iter__(self):
        return iter([self.indices[i] for i in np.random.permutation(len(self.indices))])

    def __len__(self):
        return len(self.indices)


class BatchSampler(Sampler):
    def __init__(self, dataset=None, sampler=None, shuffle=False, batch_size=1, drop_last=False):
        if sampler is None:
            sampler = RandomSampler(dataset) if shuffle else SequenceSampler(dataset)
        self.sampler, self.batch_size, self.drop_last = sampler, batch_size, drop_last

    def __iter__(self):
        b = []
        for i in self.sampler:
            b.append(i)
            if len(b) == self.batch_size:
                yield b
                b = []
        if b and not self.drop_last:
            yield b

    def __len__(self):
        n = len(self.sampler)
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size


class DistributedBatchSampler(BatchSampler):
    """Each rank sees a disjoint 1/nranks slice (parity: paddle.io.DistributedBatchSampler)."""

    def __init__(self, dataset, batch_size, num_replicas=None, rank=None, shuffle=False,
                 drop_last=False):
        from ..distributed.collective import get_rank, get_world_size
        self.dataset, self.batch_size = dataset, batch_size
        self.nranks = num_replicas if num_replicas is not None else get_world_size()
        self.local_rank = rank if rank is not None else get_rank()
        self.shuffle, self.drop_last = shuffle, drop_last
        self.epoch = 0
        self.num_samples = int(math.ceil(len(dataset) * 1.0 / self.nranks))
        self.total_size = self.num_samples * self.nranks

    def __iter__(self):
        n = len(self.dataset)
        idx = np.arange(n).tolist()
        if self.shuffle:
            np.random.RandomState(self.epoch).shuffle(idx)
            self.epoch += 1
        idx += idx[:(self.total_size - len(idx))]
        idx = idx[self.local_rank * self.num_samples:(self.local_rank + 1) * self.num_samples]
        b = []
        for i in idx:
            b.append(i)
            if len(b) == self.batch_size:
                yield b
                b = []
        if b and not self.drop_last:
            yield b

    def __len__(self):
        n = self.num_samples
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size

    def set_epoch(self, epoch):
        self.epoch = epoch


def default_collate_fn(batch):
    s = batch[0]
    if isinstance(s, Tensor):
        return np.stack([b.numpy() for b in batch])
    if isinstance(s, np.ndarray):
        return _stack_native(batch)
    if isinstance(s, (int, np.integer)):
        return np.array(batch, dtype=np.int64)
    if isinstance(s, (float, np.floating)):
        return np.array(batch, dtype=np.float32)
    if isinstance(s, (str, bytes)):
        return batch
    if isinstance(s, dict):
        return {k: default_collate_fn([b[k] for b in batch]) for k in s}
    if isinstance(s, (list, tuple)):
        return [default_collate_fn(list(x)) for x in zip(*batch)]
    return batch


def _stack_native(arrs):
    """np.stack via the native multi-threaded row copy for large same-shape batches."""
    s = arrs[0]
    nbytes = s.nbytes * len(arrs)
    if nbytes < (4 << 20) or not all(a.shape == s.shape and a.dtype == s.dtype for a in arrs):
        return np.stack(arrs)
    from ..native import runtime
    rt = runtime()
    if rt is None:
        return np.stack(arrs)
    arrs = [np.ascontiguousarray(a) for a in arrs]
    out = np.empty((len(arrs),) + s.shape, dtype=s.dtype)
    rt.stack_rows([a.ctypes.data for a in arrs], s.nbytes, out.ctypes.data, 8)
    return out


def default_convert_fn(batch):
    return batch


class _WorkerInfo:
    def __init__(self, id, num_workers, dataset, seed=0):
        self.id, self.num_workers, self.dataset, self.seed = id, num_workers, dataset, seed


_worker_info = None


def get_worker_info():
    return _worker_info


def _to_device_tree(x, dev, stream=None):
    if isinstance(x, np.ndarray):
        t = torch.from_numpy(x)
        if dev.type == 'cuda':
            t = t.pin_memory().to(dev, non_blocking=True)
        return Tensor(t)
    if isinstance(x, torch.Tensor):
        return Tensor(x.to(dev, non_blocking=True))
    if isinstance(x, Tensor):
        return x
    if isinstance(x, dict):
        return {k: _to_device_tree(v, dev) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_to_device_tree(v, dev) for v in x]
    return x


class _TorchDS(torch.utils.data.Dataset):
    def __init__(self, ds):
        self.ds = ds

    def __len__(self):
        return len(self.ds)

    def __getitem__(self, i):
        return self.ds[i]


class _TorchIterDS(torch.utils.data.IterableDataset):
    def __init__(self, ds):
        self.ds = ds

    def __iter__(self):
        return iter(self.ds)


def _np_tree(x):
    if isinstance(x, Tensor):
        return x.numpy()
    if isinstance(x, dict):
        return {k: _np_tree(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_np_tree(v) for v in x]
    return x


class DataLoader:
    def __init__(self, dataset, feed_list=None, places=None, return_list=True, batch_sampler=None,
                 batch_size=1, shuffle=False, drop_last=False, collate_fn=None, num_workers=0,
                 use_buffer_reader=True, prefetch_factor=2, use_shared_memory=True, timeout=0,
                 worker_init_fn=None, persistent_workers=False):
        self.dataset = dataset
        self.return_list = return_list
        self.collate_fn = collate_fn or default_collate_fn
        self.num_workers = num_workers
        self.use_buffer_reader = use_buffer_reader
        self.prefetch_factor = prefetch_factor
        self.worker_init_fn = worker_init_fn
        self.timeout = timeout
        self._iterable = isinstance(dataset, IterableDataset)
        if self._iterable:
            self.batch_sampler = None
            self.batch_size, self.drop_last = batch_size, drop_last
        elif batch_sampler is not None:
            self.batch_sampler = batch_sampler
        elif batch_size is None:
            self.batch_sampler = None
        else:
            self.batch_sampler = BatchSampler(dataset, shuffle=shuffle, batch_size=batch_size,
                                              drop_last=drop_last)
        self.places = places

    def __len__(self):
        if self._iterable:
            raise TypeError("IterableDataset has no len()")
        return len(self.batch_sampler) if self.batch_sampler is not None else len(self.dataset)

    def _device(self):
        if self.places is not None:
            from ..framework.core import _to_torch_device
            p = self.places[0] if isinstance(self.places, (list, tuple)) else self.places
            return _to_torch_device(p)
        return _default_device()

    def _host_batches(self):
        collate = self.collate_fn
        if self.num_workers > 0:
            if self._iterable:
                tds = _TorchIterDS(self.dataset)
                dl = torch.utils.data.DataLoader(
                    tds, batch_size=self.batch_size, drop_last=self.drop_last,
                    collate_fn=lambda b: collate([_np_tree(e) for e in b]),
                    num_workers=self.num_workers, prefetch_factor=self.prefetch_factor,
                    worker_init_fn=self.worker_init_fn)
            else:
                tds = _TorchDS(self.dataset)
                dl = torch.utils.data.DataLoader(
                    tds, batch_sampler=self.batch_sampler if self.batch_sampler is not None else None,
                    batch_size=None if self.batch_sampler is None else 1,
                    collate_fn=(lambda b: collate([_np_tree(e) for e in b])) if
                    self.batch_sampler is not None else _np_tree,
                    num_workers=self.num_workers, prefetch_factor=self.prefetch_factor,
                    worker_init_fn=self.worker_init_fn)
                if self.batch_sampler is not None:
                    dl = torch.utils.data.DataLoader(
                        tds, batch_sampler=self.batch_sampler,
                        collate_fn=lambda b: collate([_np_tree(e) for e in b]),
                        num_workers=self.num_workers, prefetch_factor=self.prefetch_factor,
                        worker_init_fn=self.worker_init_fn)
            yield from dl
            return
        if self._iterable:
            b = []
            for s in self.dataset:
                b.append(_np_tree(s))
                if len(b) == self.batch_size:
                    yield collate(b)
                    b = []
            if b and not self.drop_last:
                yield collate(b)
            return
        if self.batch_sampler is None:
            for i in range(len(self.dataset)):
                yield _np_tree(self.dataset[i])
            return
        for idx in self.batch_sampler:
            yield collate([_np_tree(self.dataset[i]) for i in idx])

    def __iter__(self):
        return _ReaderTimed(self, self._iter_batches())

    def _iter_batches(self):
        dev = self._device()
        src = self._host_batches()
        if not (self.use_buffer_reader and dev.type == 'cuda'):
            for b in src:
                yield _to_device_tree(b, dev)
            return
        # one-ahead prefetch: H2D of batch i+1 on a side stream while step i runs
        side = torch.cuda.Stream(device=dev)
        nxt = None
        for b in src:
            with torch.cuda.stream(side):
                cur = _to_device_tree(b, dev)
            ev = side.record_event()
            if nxt is not None:
                yield nxt
            torch.cuda.current_stream(dev).wait_event(ev)
            nxt = cur
        if nxt is not None:
            yield nxt

    @staticmethod
    def from_generator(feed_list=None, capacity=None, use_double_buffer=True, iterable=True,
                       return_list=False, use_multiprocess=False, drop_last=True):
        return _GeneratorLoader(return_list)


class _ReaderTimed:
    """Iterator over a DataLoader's batches that reports each batch's reader time to the
    profiler benchmark (reader_cost in step_info; parity: fluid/dataloader/dataloader_iter.py
    benchmark().before_reader / after_reader) and, while a profiler records, opens a
    Dataloader range around it."""

    def __init__(self, loader, it):
        self._loader, self._it = loader, it

    def __iter__(self):
        return self

    def __next__(self):
        from ..profiler import _hooks
        from ..profiler.timer import benchmark
        bm = benchmark()
        bm.check_if_need_record(self._loader)
        bm.before_reader()
        if _hooks.ACTIVE:
            from ..profiler import RecordEvent, TracerEventType
            with RecordEvent('Dataloader', TracerEventType.Dataloader):
                b = next(self._it)
        else:
            b = next(self._it)
        bm.after_reader()
        return b

    def __len__(self):
        return len(self._loader)


class _GeneratorLoader:
    def __init__(self, return_list):
        self._gen = None
        self.return_list = return_list

    def set_sample_list_generator(self, reader, places=None):
        self._gen = lambda: (default_collate_fn(b) for b in reader())

    def set_batch_generator(self, reader, places=None):
        self._gen = reader

    def set_sample_generator(self, reader, batch_size, drop_last=True, places=None):
        def g():
            b = []
            for s in reader():
                b.append(s)
                if len(b) == batch_size:
                    yield default_collate_fn(b)
                    b = []
        self._gen = g

    def __iter__(self):
        dev = _default_device()
        for b in self._gen():
            yield _to_device_tree(b, dev)


from .gpt_dataset import GPTDataset, NativeTokenLoader, write_token_dataset  # noqa: E402
