"""paddle.batch (parity: python/paddle/batch.py)."""


def batch(reader, batch_size, drop_last=False):
    def batch_reader():
        b = []
        for instance in reader():
            b.append(instance)
            if len(b) == batch_size:
                yield b
                b = []
        if not drop_last and b:
            yield b
    return batch_reader
