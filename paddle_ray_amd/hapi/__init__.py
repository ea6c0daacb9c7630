"""paddle.hapi (parity: python/paddle/hapi/{model.py,callbacks.py,model_summary.py,dynamic_flops.py})."""
from .model import Model  # noqa
from .summary import summary, flops  # noqa
from . import callbacks  # noqa
