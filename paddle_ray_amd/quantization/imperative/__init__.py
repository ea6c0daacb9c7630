"""Legacy imperative quantization API (parity: python/paddle/quantization/imperative/
{qat,ptq,ptq_config,ptq_quantizer,ptq_registry}.py)."""
from .ptq_quantizer import (BaseQuantizer, AbsmaxQuantizer, PerChannelAbsmaxQuantizer,  # noqa
                            KLQuantizer, HistQuantizer, SUPPORT_ACT_QUANTIZERS,
                            SUPPORT_WT_QUANTIZERS, cal_kl_threshold)
from .ptq_config import PTQConfig, default_ptq_config  # noqa: F401
from .ptq_registry import PTQRegistry  # noqa: F401
from .ptq import ImperativePTQ  # noqa: F401
from .qat import ImperativeQuantAware  # noqa: F401
