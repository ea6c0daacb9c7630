"""paddle.device (parity: python/paddle/device/__init__.py). 'gpu' == the HIP device."""
import torch

from ..framework.core import (set_device, get_device, is_compiled_with_cuda, is_compiled_with_rocm,  # noqa
                              is_compiled_with_xpu)
from ..framework.core import XPUPlace, IPUPlace, MLUPlace  # noqa: F401
from . import cuda  # noqa
from . import xpu  # noqa: F401


def get_all_device_type():
    return ['cpu'] + (['gpu'] if torch.cuda.is_available() else [])


def get_all_custom_device_type():
    return []


def get_available_device():
    return ['cpu'] + [f'gpu:{i}' for i in range(torch.cuda.device_count())]


def get_cudnn_version():
    return None


def synchronize(device=None):
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def is_compiled_with_cinn():
    return False


def is_compiled_with_ipu():
    return False


def is_compiled_with_npu():
    return False


def is_compiled_with_mlu():
    return False


def is_compiled_with_custom_device(device_type):
    return False


def get_available_custom_device():
    return []


Stream = cuda.Stream
Event = cuda.Event
current_stream = cuda.current_stream
set_stream = cuda.set_stream
stream_guard = cuda.stream_guard
