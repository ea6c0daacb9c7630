"""Parameter-server style datasets (parity: python/paddle/distributed/fleet/dataset/dataset.py).
In-memory / queue datasets over local files (slot-based text format), usable
with paddle.io.DataLoader."""
from ..io import IterableDataset


class _FileDataset(IterableDataset):
    def __init__(self):
        self._files, self._batch_size, self._parse = [], 1, None
        self._data = []

    def init(self, batch_size=1, thread_num=1, use_var=None, pipe_command=None, input_type=0,
             fs_name='', fs_ugi='', download_cmd='cat', **kw):
        self._batch_size = batch_size

    def set_filelist(self, filelist):
        self._files = list(filelist)

    def set_parse_fn(self, fn):
        self._parse = fn

    def _iter_lines(self):
        for f in self._files:
            with open(f) as fh:
                for line in fh:
                    yield self._parse(line) if self._parse else line.rstrip('\n')

    def __iter__(self):
        yield from (self._data if self._data else self._iter_lines())


class InMemoryDataset(_FileDataset):
    def load_into_memory(self, is_shuffle=False):
        self._data = list(self._iter_lines())

    def local_shuffle(self):
        import random
        random.shuffle(self._data)

    def global_shuffle(self, fleet=None, thread_num=12):
        self.local_shuffle()

    def release_memory(self):
        self._data = []

    def get_memory_data_size(self, fleet=None):
        return len(self._data)


class QueueDataset(_FileDataset):
    pass
