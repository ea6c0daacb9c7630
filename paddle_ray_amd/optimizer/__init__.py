"""paddle.optimizer (parity: python/paddle/optimizer/__init__.py)."""
from .optimizer import (Optimizer, SGD, Momentum, Adam, AdamW, Adagrad, Adadelta, Adamax,  # noqa
                        RMSProp, Lamb, LarsMomentum, L1Decay, L2Decay)
from . import lr  # noqa
