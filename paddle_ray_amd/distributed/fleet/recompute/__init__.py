from ....parallel.recompute import recompute, recompute_sequential, recompute_hybrid  # noqa
