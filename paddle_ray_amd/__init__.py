"""paddle_ray_amd — an MI355X-native deep-learning framework with the Paddle API.

``import paddle_ray_amd as paddle`` gives the ``paddle.*`` surface
(parity: python/paddle/__init__.py). Compute path: PyTorch-ROCm tensors +
hand-written gfx950 HIP kernels (``paddle_ray_amd.ops``) + RCCL over xGMI.
"""
__version__ = '0.1.0'

import torch as _torch

from .native import allocator as _allocator  # noqa: E402
_allocator.maybe_enable_from_env()  # PRA_ALLOCATOR=auto_growth: before any device allocation

from .framework.core import (Tensor, Parameter, EagerParamBase, Place, CPUPlace, CUDAPlace,  # noqa
                             CUDAPinnedPlace, XPUPlace, NPUPlace, to_tensor, is_tensor, no_grad,
                             enable_grad, set_grad_enabled, is_grad_enabled, set_device, get_device,
                             set_default_dtype, get_default_dtype, iinfo, finfo, in_dynamic_mode,
                             is_compiled_with_cuda, is_compiled_with_rocm, is_compiled_with_xpu,
                             convert_dtype as _convert_dtype,
                             bool_ as bool, uint8, int8, int16, int32, int64, float16, bfloat16,
                             float32, float64, complex64, complex128)
from .framework.core import _u, _w  # noqa
from .tensor import *  # noqa
from .tensor import creation, math, manipulation, linalg as _tlinalg, random as _trandom  # noqa
from .tensor.random import (seed, get_rng_state, set_rng_state, get_cuda_rng_state,  # noqa
                            set_cuda_rng_state)
from .framework.io import save, load  # noqa
from .framework import flags as _flags  # noqa
from .framework.flags import set_flags, get_flags  # noqa
from . import nn, optimizer, autograd, amp, io, static, jit, distributed, incubate, vision, metric  # noqa
from . import audio, text, quantization, reader, dataset, cost_model  # noqa: E402
from . import linalg, fft, device, utils, profiler, hapi, sparse, distribution, signal, models  # noqa
from . import framework, inference, geometric, regularizer, callbacks, sysconfig, hub, onnx  # noqa
from .autograd import grad, PyLayer  # noqa
from .hapi import Model, summary, flops  # noqa
from .distributed.parallel import DataParallel  # noqa
from .nn.layer.layers import ParamAttr  # noqa
from .framework.lazy import LazyGuard  # noqa
from .static import enable_static, disable_static  # noqa
from .batch import batch  # noqa

dtype = _torch.dtype
tolist = manipulation.tolist
CUDAPlace = CUDAPlace


def disable_signal_handler():
    pass


def set_printoptions(precision=None, threshold=None, edgeitems=None, sci_mode=None,
                     linewidth=None):
    import numpy as np
    kw = {k: v for k, v in dict(precision=precision, threshold=threshold, edgeitems=edgeitems,
                                linewidth=linewidth).items() if v is not None}
    np.set_printoptions(**kw)


def check_shape(shape):
    return shape


def is_compiled_with_cinn():
    return False


def is_compiled_with_ipu():
    return False


def is_compiled_with_npu():
    return False


def is_compiled_with_mlu():
    return False


def is_compiled_with_custom_device(name):
    return False
