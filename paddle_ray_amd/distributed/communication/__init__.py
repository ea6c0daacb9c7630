"""paddle.distributed.communication (parity: python/paddle/distributed/communication/): the
collectives, plus the ``stream`` variants that take ``use_calc_stream``."""
from ..collective import (all_reduce, broadcast, reduce, all_gather, reduce_scatter, scatter,  # noqa: F401
                          alltoall, alltoall_single, send, recv)
from . import stream  # noqa: F401
