"""paddle.static.amp: mixed precision for static programs = the dygraph AMP machinery
applied during Executor replay."""
from ..amp import auto_cast, decorate as _decorate, GradScaler  # noqa


def decorate(optimizer, amp_lists=None, init_loss_scaling=2 ** 15, use_dynamic_loss_scaling=True,
             use_pure_fp16=False, use_fp16_guard=None, use_bf16=False, **kw):
    optimizer._multi_precision = True
    return optimizer


class AutoMixedPrecisionLists:
    def __init__(self, custom_white_list=None, custom_black_list=None, custom_black_varnames=None):
        self.white_list = set(custom_white_list or [])
        self.black_list = set(custom_black_list or [])


CustomOpLists = AutoMixedPrecisionLists
