"""paddle.callbacks (parity: python/paddle/callbacks.py) -> hapi callbacks."""
from .hapi.callbacks import *  # noqa: F401,F403
from .hapi import callbacks as _cb

Callback = _cb.Callback
ProgBarLogger = _cb.ProgBarLogger
ModelCheckpoint = _cb.ModelCheckpoint
LRScheduler = _cb.LRScheduler
EarlyStopping = _cb.EarlyStopping
ReduceLROnPlateau = getattr(_cb, 'ReduceLROnPlateau', None)
VisualDL = getattr(_cb, 'VisualDL', None)
WandbCallback = getattr(_cb, 'WandbCallback', None)
