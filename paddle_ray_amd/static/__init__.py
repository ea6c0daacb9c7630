"""paddle.static (parity: python/paddle/static/__init__.py)."""
_STATIC = [False]


def _static_mode_enabled():
    return _STATIC[0]


def enable_static():
    from .graph import install_static_hooks
    install_static_hooks()
    _STATIC[0] = True
    import importlib
    _core = importlib.import_module("paddle_ray_amd.framework.core")
    _core._in_dynamic[0] = False


def disable_static(place=None):
    _STATIC[0] = False
    import importlib
    _core = importlib.import_module("paddle_ray_amd.framework.core")
    _core._in_dynamic[0] = True


from .input import InputSpec  # noqa: E402
from .graph import (Program, Block, Variable, Executor, global_scope, scope_guard,  # noqa: E402
                    program_guard, name_scope, device_guard, default_main_program,
                    default_startup_program, data, append_backward, gradients, BuildStrategy,
                    ExecutionStrategy, CompiledProgram, ParallelExecutor, save_inference_model,
                    load_inference_model, serialize_program, serialize_persistables,
                    deserialize_program, deserialize_persistables, save_to_file, load_from_file,
                    normalize_program, load_program_state, set_program_state, save, load,
                    create_parameter, create_global_var, Print, py_func, cpu_places, cuda_places,
                    xpu_places, npu_places, mlu_places, accuracy, auc, WeightNormParamAttr,
                    ExponentialMovingAverage, ipu_shard_guard, set_ipu_shard, IpuStrategy,
                    IpuCompiledProgram, exponential_decay, ctr_metric_bundle, _static_minimize,
                    Scope, RecomputeOptimizer)
from . import nn  # noqa: E402
from .sequence_lod import create_lod_tensor  # noqa: E402,F401
from . import amp  # noqa: E402
from .pipeline import PipelineOptimizer  # noqa: E402,F401
