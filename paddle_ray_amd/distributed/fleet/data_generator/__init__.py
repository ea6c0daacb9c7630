"""Data generators that turn raw text lines into the MultiSlot data-feed format (parity:
python/paddle/distributed/fleet/data_generator/data_generator.py -- DataGenerator,
MultiSlotDataGenerator, MultiSlotStringDataGenerator).

A user subclass overrides ``generate_sample(line)`` (returning a generator factory of
``[(slot name, [feasign, ...]), ...]`` samples) and optionally ``generate_batch(samples)``;
``run_from_stdin`` / ``run_from_memory`` write one ``<n> v1 .. vn <m> w1 .. wm ...`` line per
sample to stdout (what ``InMemoryDataset`` / ``QueueDataset`` pipe commands consume)."""
import sys

__all__ = ['DataGenerator', 'MultiSlotDataGenerator', 'MultiSlotStringDataGenerator']


class DataGenerator:
    def __init__(self):
        self._proto_info = None
        self.batch_size_ = 32

    def set_batch(self, batch_size):
        self.batch_size_ = int(batch_size)

    def _emit(self, samples, out):
        for s in self.generate_batch(samples)():
            out.write(self._gen_str(s))

    def _run(self, lines, out=None):
        out = out or sys.stdout
        batch = []
        for line in lines:
            for s in self.generate_sample(line)():
                if s is None:
                    continue
                batch.append(s)
                if len(batch) == self.batch_size_:
                    self._emit(batch, out)
                    batch = []
        if batch:
            self._emit(batch, out)

    def run_from_memory(self):
        """Samples from ``generate_sample(None)`` (debugging / benchmarking)."""
        self._run([None])

    def run_from_stdin(self):
        self._run(sys.stdin)

    def _gen_str(self, line):
        raise NotImplementedError("use MultiSlotDataGenerator or MultiSlotStringDataGenerator")

    def generate_sample(self, line):
        raise NotImplementedError("override generate_sample(line) to return a generator factory of "
                                  "[(name, [feasign, ...]), ...] samples")

    def generate_batch(self, samples):
        def local_iter():
            yield from samples
        return local_iter


def _fields(line):
    if isinstance(line, zip):
        line = list(line)
    if not isinstance(line, (list, tuple)):
        raise ValueError("the output of generate_sample must be a list or tuple of (name, [feasign, ...]), "
                         "e.g. [('words', [1926, 8, 17]), ('label', [1])]")
    return line


class MultiSlotStringDataGenerator(DataGenerator):
    """Feasigns already strings: ``<count> f1 f2 ...`` per slot, no type tracking."""

    def _gen_str(self, line):
        parts = []
        for name, elements in _fields(line):
            parts.append(' '.join([str(len(elements))] + [str(e) for e in elements]))
        return ' '.join(parts) + '\n'


class MultiSlotDataGenerator(DataGenerator):
    """Integer / float feasigns; the slot list (names, order) is fixed by the first sample and
    ``_proto_info`` records each slot's type (uint64 until a float appears)."""

    def _gen_str(self, line):
        line = _fields(line)
        first = self._proto_info is None
        if first:
            self._proto_info = []
        elif len(line) != len(self._proto_info):
            raise ValueError("the complete field set of two given line are inconsistent.")
        parts = []
        for idx, item in enumerate(line):
            name, elements = item
            if not isinstance(name, str):
                raise ValueError(f"name{type(name)} must be in str type")
            if not isinstance(elements, list):
                raise ValueError(f"elements{type(elements)} must be in list type")
            if not elements:
                raise ValueError("the elements of each field can not be empty, you need padding it in process().")
            if first:
                self._proto_info.append((name, 'uint64'))
            elif name != self._proto_info[idx][0]:
                raise ValueError(f"the field name of two given line are not match: require<"
                                 f"{self._proto_info[idx][0]}>, get<{name}>.")
            for e in elements:
                if isinstance(e, float):
                    self._proto_info[idx] = (name, 'float')
                elif not isinstance(e, int):
                    raise ValueError(f"the type of element{type(e)} must be in int or float")
            parts.append(' '.join([str(len(elements))] + [str(e) for e in elements]))
        return ' '.join(parts) + '\n'
