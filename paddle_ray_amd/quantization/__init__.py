"""paddle.quantization (parity: python/paddle/quantization/__init__.py): the config-driven
QAT / PTQ API (QuantConfig, quanters, observers) and the legacy imperative API
(ImperativeQuantAware, ImperativePTQ with Absmax/PerChannel/KL/Hist calibration)."""
from .base import (BaseQuanter, BaseObserver, QuanterFactory, ObserverFactory,  # noqa: F401
                   quanter, ObserveWrapper)
from .config import QuantConfig, SingleLayerConfig  # noqa: F401
from .quantize import Quantization, QAT, PTQ  # noqa: F401
from . import quanters, observers, imperative  # noqa: F401
from .imperative import (ImperativeQuantAware, ImperativePTQ, PTQConfig,  # noqa: F401
                         default_ptq_config, BaseQuantizer, AbsmaxQuantizer,
                         PerChannelAbsmaxQuantizer, KLQuantizer, HistQuantizer,
                         SUPPORT_ACT_QUANTIZERS, SUPPORT_WT_QUANTIZERS, PTQRegistry)
from .imperative.fuse_utils import fuse_layers  # noqa: F401
