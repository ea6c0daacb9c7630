"""Reader creators over the map-style datasets (the legacy paddle.dataset.* modules)."""


def from_dataset(make, convert=lambda s: s, cycle=False):
    """Reader creator: iterate ``make()``'s samples through ``convert``; the dataset is
    built lazily on the first read."""
    def reader():
        ds = make()
        while True:
            for i in range(len(ds)):
                yield convert(ds[i])
            if not cycle:
                return
    return reader
