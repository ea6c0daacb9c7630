"""paddle.amp.debugging: tensor checker API over the NaN/Inf checker
(framework/nan_inf.py)."""
import enum

import torch

from ..framework import nan_inf as _ni
from ..framework.core import _u


class DebugMode(enum.Enum):
    CHECK_NAN_INF_AND_ABORT = 0
    CHECK_NAN_INF = 1
    CHECK_ALL_FOR_OVERFLOW = 2
    CHECK_ALL = 3
    DUMP_ALL = 4


class TensorCheckerConfig:
    def __init__(self, enable, debug_mode=DebugMode.CHECK_NAN_INF_AND_ABORT, output_dir=None,
                 checked_op_list=None, skipped_op_list=None, debug_step=None, stack_height_limit=1):
        self.enable = enable
        self.debug_mode = debug_mode
        self.skipped_op_list = list(skipped_op_list or [])


def enable_tensor_checker(checker_config):
    if checker_config.enable:
        level = 0 if checker_config.debug_mode == DebugMode.CHECK_NAN_INF_AND_ABORT else 1
        _ni.enable(level, checker_config.skipped_op_list)


def disable_tensor_checker():
    _ni.disable()


def check_numerics(tensor, op_type='', var_name='', debug_mode=DebugMode.CHECK_NAN_INF_AND_ABORT):
    t = _u(tensor)
    n_nan = int(torch.isnan(t).sum())
    n_inf = int(torch.isinf(t).sum())
    if (n_nan or n_inf) and debug_mode == DebugMode.CHECK_NAN_INF_AND_ABORT:
        raise RuntimeError(f"[check_numerics] {op_type} {var_name}: {n_nan} NaN, {n_inf} Inf")
    return n_nan, n_inf


def enable_operator_stats_collection():
    pass


def disable_operator_stats_collection():
    pass
