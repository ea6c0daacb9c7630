"""GPT pretraining token dataset + native prefetch loader.

Parity: the reference Fleet GPT benchmarks' dataset (documents concatenated into one token
stream, fixed seq_len+1 windows, per-epoch document shuffle, global sample shuffle) and
paddle/fluid/operators/reader/buffered_reader.cc (ring of prefetched batches + async H2D).

Data files: ``<prefix>_ids.npy`` (1-D token ids, uint16/int32/int64, memory-mapped) and
``<prefix>_idx.npz`` with ``lens`` (int32 tokens per document) — the same pair layout the
reference's preprocessing emits. ``write_token_dataset`` produces it.
"""
import os

import numpy as np
import torch

from ..framework.core import Tensor, _default_device


def write_token_dataset(prefix, docs, dtype=np.uint16):
    """docs: iterable of 1-D int arrays -> <prefix>_ids.npy + <prefix>_idx.npz."""
    docs = [np.asarray(d, dtype=dtype) for d in docs]
    ids = np.concatenate(docs) if docs else np.zeros(0, dtype)
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    np.save(prefix + '_ids.npy', ids)
    np.savez(prefix + '_idx.npz', lens=np.array([len(x) for x in docs], dtype=np.int32))


def _native():
    from ..native import runtime
    rt = runtime()
    if rt is None:
        raise RuntimeError("native runtime (_pra_runtime) not built: "
                           "python -m paddle_ray_amd.native.build")
    return rt


class GPTDataset:
    """Map-style dataset of [seq_len+1] int64 token windows (input = [:-1], label = [1:])."""

    def __init__(self, prefix, seq_len, num_samples=None, seed=1234, num_epochs=None):
        self.tokens = np.load(prefix + '_ids.npy', mmap_mode='r', allow_pickle=False)
        self.lens = np.load(prefix + '_idx.npz', allow_pickle=False)['lens'].astype(np.int32)
        self.doc_off = np.zeros(len(self.lens) + 1, dtype=np.int64)
        np.cumsum(self.lens, out=self.doc_off[1:])
        self.seq_len = seq_len
        tokens_per_epoch = int(self.lens.sum())
        if num_epochs is None:
            need = (num_samples or tokens_per_epoch // seq_len) * seq_len + 1
            num_epochs = max(1, -(-need // tokens_per_epoch))
        rng = np.random.RandomState(seed)
        doc_idx = np.concatenate([rng.permutation(len(self.lens)).astype(np.int32)
                                  for _ in range(num_epochs)])
        self.doc_idx = doc_idx
        self.sample_idx = _native().build_sample_idx(self.lens, doc_idx, seq_len, num_epochs,
                                                     tokens_per_epoch)
        n = len(self.sample_idx) - 1
        if num_samples is not None:
            n = min(n, num_samples)
        self.shuffle_idx = rng.permutation(n).astype(np.int64)

    def __len__(self):
        return len(self.shuffle_idx)

    def __getitem__(self, i):
        s = int(self.shuffle_idx[i])
        (p0, o0), (p1, o1) = self.sample_idx[s], self.sample_idx[s + 1]
        parts = []
        for p in range(p0, p1 + 1):
            d = self.doc_idx[p]
            a = self.doc_off[d] + (o0 if p == p0 else 0)
            b = self.doc_off[d] + o1 + 1 if p == p1 else self.doc_off[d + 1]
            parts.append(self.tokens[a:b])
        return np.concatenate(parts).astype(np.int64)


class NativeTokenLoader:
    """Iterates (input_ids, labels) device batches; C++ threads gather windows from the
    memory-mapped token file into a ring of pinned host slots, each copied to HBM with a
    non_blocking DMA on a side stream that overlaps the previous step's compute."""

    def __init__(self, dataset, batch_size, num_slots=4, num_threads=4, device=None,
                 drop_last=True, rank=0, world_size=1):
        self.ds = dataset
        self.batch = batch_size
        self.dev = torch.device(device) if device is not None else _default_device()
        shuffle = dataset.shuffle_idx
        if world_size > 1:  # contiguous per-rank shards of each global batch
            nb = len(shuffle) // (batch_size * world_size)
            shuffle = shuffle[:nb * batch_size * world_size].reshape(nb, world_size, batch_size)
            shuffle = np.ascontiguousarray(shuffle[:, rank].reshape(-1))
        self._shuffle = shuffle
        pin = self.dev.type == 'cuda'
        S1 = dataset.seq_len + 1
        self.slots = [torch.empty((batch_size, S1), dtype=torch.int64, pin_memory=pin)
                      for _ in range(num_slots)]
        tok = dataset.tokens
        self._tok = tok  # keep the mmap alive
        self._loader = _native().TokenLoader(
            tok.ctypes.data, tok.dtype.itemsize, dataset.doc_off, dataset.doc_idx,
            dataset.sample_idx, shuffle, batch_size, dataset.seq_len,
            [t.data_ptr() for t in self.slots], num_threads)
        self._stream = torch.cuda.Stream(self.dev) if pin else None
        self._pending = []  # (slot, event) waiting for their H2D copy to finish

    def __len__(self):
        return self._loader.num_batches()

    def _recycle(self, wait_all=False):
        keep = []
        for slot, ev in self._pending:
            if ev is None or wait_all or ev.query():
                if ev is not None and wait_all:
                    ev.synchronize()
                self._loader.release(slot)
            else:
                keep.append((slot, ev))
        self._pending = keep

    def __iter__(self, first_batch=0):
        self._loader.start(first_batch)
        try:
            while True:
                self._recycle()
                slot, b = self._loader.acquire()
                if slot < 0:
                    break
                host = self.slots[slot]
                if self._stream is not None:
                    with torch.cuda.stream(self._stream):
                        dev = host.to(self.dev, non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record(self._stream)
                    torch.cuda.current_stream(self.dev).wait_stream(self._stream)
                    dev.record_stream(torch.cuda.current_stream(self.dev))
                else:
                    dev, ev = host.clone(), None
                self._pending.append((slot, ev))
                yield Tensor(dev[:, :-1]), Tensor(dev[:, 1:])
        finally:
            self._recycle(wait_all=True)
            self._loader.stop()

    def resume_from(self, batch_no):
        """Iterator starting at global batch ``batch_no`` (checkpoint resume)."""
        return self.__iter__(first_batch=batch_no)
