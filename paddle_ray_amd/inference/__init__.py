"""paddle.inference (parity: python/paddle/inference/__init__.py, paddle/fluid/inference/api/
analysis_predictor.cc): Config / create_predictor / Predictor with zero-copy-style
input/output handles over a ``.pdmodel`` + ``.pdiparams`` pair.

MI355X design: the predictor replays the saved Program (static/graph.py) under
``no_grad``; with ``Config.enable_use_gpu`` + ``enable_hip_graph`` (default on GPU) each
new input signature is captured once into a hipGraph and then replayed with one launch.
"""
import enum
import os

import numpy as np
import torch

from ..framework.core import Tensor


class PrecisionType(enum.IntEnum):
    Float32 = 0
    Int8 = 1
    Half = 2
    Bfloat16 = 3


class PlaceType(enum.IntEnum):
    UNK = -1
    CPU = 0
    GPU = 1


DataType = enum.IntEnum('DataType', 'FLOAT32 INT64 INT32 UINT8 INT8 FLOAT16 BFLOAT16 BOOL')


class Config:
    def __init__(self, model_file=None, params_file=None):
        if model_file is not None and params_file is None and not model_file.endswith('.pdmodel'):
            model_file, params_file = model_file + '.pdmodel', model_file + '.pdiparams'
        self._model, self._params = model_file, params_file
        self._gpu = False
        self._device_id = 0
        self._hip_graph = True
        self._precision = PrecisionType.Float32

    def set_model(self, model_file, params_file):
        self._model, self._params = model_file, params_file

    def model_dir(self):
        return os.path.dirname(self._model or '')

    def prog_file(self):
        return self._model

    def params_file(self):
        return self._params

    def enable_use_gpu(self, memory_pool_init_size_mb=100, device_id=0, precision=None):
        self._gpu, self._device_id = True, device_id
        if precision is not None:
            self._precision = precision

    def disable_gpu(self):
        self._gpu = False

    def use_gpu(self):
        return self._gpu

    def gpu_device_id(self):
        return self._device_id

    def enable_hip_graph(self, flag=True):
        self._hip_graph = bool(flag)

    enable_cuda_graph = enable_hip_graph

    def switch_ir_optim(self, flag=True):
        pass

    def enable_memory_optim(self, flag=True):
        pass

    def switch_use_feed_fetch_ops(self, flag=True):
        pass

    def set_cpu_math_library_num_threads(self, n):
        torch.set_num_threads(int(n))

    def enable_mkldnn(self):
        pass

    def disable_glog_info(self):
        pass

    def summary(self):
        return f'Config(model={self._model}, gpu={self._gpu}, hip_graph={self._hip_graph})'


class _Handle:
    def __init__(self, name, predictor, is_input):
        self.name, self._p, self._in = name, predictor, is_input

    def copy_from_cpu(self, arr):
        self._p._inputs[self.name] = np.asarray(arr)

    def share_external_data(self, t):
        self._p._inputs[self.name] = t

    def reshape(self, shape):
        pass

    def copy_to_cpu(self):
        return self._p._outputs[self.name]

    def shape(self):
        src = self._p._inputs if self._in else self._p._outputs
        return list(np.shape(src[self.name]))

    def type(self):
        return DataType.FLOAT32


class Predictor:
    def __init__(self, config):
        from ..static import graph as G
        self._cfg = config
        if config._gpu and torch.cuda.is_available():
            torch.cuda.set_device(config._device_id)
            from ..device import set_device
            set_device(f'gpu:{config._device_id}')
        prefix = config._model[:-len('.pdmodel')] if config._model.endswith('.pdmodel') \
            else config._model
        self._prog, self._feed_names, self._fetch = G.load_inference_model(prefix)
        self._fetch_names = [v.name for v in self._fetch]
        self._exe = G.Executor()
        self._inputs, self._outputs = {}, {}
        self._graphs = {}

    def get_input_names(self):
        return list(self._feed_names)

    def get_output_names(self):
        return list(self._fetch_names)

    def get_input_handle(self, name):
        return _Handle(name, self, True)

    def get_output_handle(self, name):
        return _Handle(name, self, False)

    def _replay(self, *ins):
        outs = self._exe.run(self._prog, feed=dict(zip(self._feed_names, ins)),
                             fetch_list=self._fetch, return_numpy=False)
        return outs

    def _run_tensors(self, ins):
        use_graph = (self._cfg._hip_graph and self._cfg._gpu and torch.cuda.is_available())
        with torch.no_grad():
            if use_graph:
                from ..jit.api import _GraphEntry, _signature
                key = _signature(tuple(ins), {})
                g = self._graphs.get(key)
                if g is None:
                    g = self._graphs[key] = _GraphEntry(self._replay, tuple(ins), {})
                return [Tensor(o._t.clone()) for o in g(tuple(ins), {})]
            return self._replay(*ins)

    def _io_types(self, outs):
        mp = self._prog.__dict__.get('_mixed_precision')
        if mp and mp.get('keep_io_types', True):
            outs = [Tensor(o._t.float()) if o._t.dtype in (torch.float16, torch.bfloat16) else o
                    for o in outs]
        return outs

    def run(self, inputs=None):
        from ..framework.core import to_tensor
        if inputs is not None:  # new-style API: list of tensors in, list out
            return self._io_types(self._run_tensors([x if isinstance(x, Tensor) else to_tensor(x)
                                                     for x in inputs]))
        ins = [to_tensor(self._inputs[n]) if not isinstance(self._inputs[n], Tensor)
               else self._inputs[n] for n in self._feed_names]
        outs = self._io_types(self._run_tensors(ins))
        self._outputs = {n: o.numpy() for n, o in zip(self._fetch_names, outs)}
        return True

    def clone(self):
        return Predictor(self._cfg)

    def clear_intermediate_tensor(self):
        pass

    def try_shrink_memory(self):
        if torch.cuda.is_available():
            torch.cuda.empty_cache()


def create_predictor(config):
    return Predictor(config)


class PredictorPool:
    """``size`` predictors over one config (parity: paddle.inference.PredictorPool): one per
    serving thread, sharing nothing but the model files."""

    def __init__(self, config, size=1):
        if size < 1:
            raise ValueError("PredictorPool size must be >= 1")
        first = Predictor(config)
        self._preds = [first] + [first.clone() for _ in range(size - 1)]

    def retrive(self, idx):
        return self._preds[idx]

    retrieve = retrive

    def __len__(self):
        return len(self._preds)


def convert_to_mixed_precision(model_file, params_file, mixed_model_file, mixed_params_file,
                               mixed_precision, backend, keep_io_types=True, black_list=None):
    """fp32 ``.pdmodel`` / ``.pdiparams`` -> a mixed-precision pair (parity:
    python/paddle/inference/wrapper.py convert_to_mixed_precision): floating parameters are stored
    in the half type (bf16 for PrecisionType.Bfloat16, fp16 for Half) except those read by an
    op type in ``black_list``, which stay fp32, and the program is marked so that it replays
    under O2 autocast with ``black_list`` op types in fp32; ``keep_io_types``: the predictor still
    takes and returns fp32."""
    import json
    from ..framework.io import load, save
    from ..static import program_desc as PD
    from ..static.graph import MIXED_PRECISION_OP
    if int(mixed_precision) not in (int(PrecisionType.Half), int(PrecisionType.Bfloat16)):
        raise ValueError(f"mixed_precision must be PrecisionType.Half or Bfloat16, got {mixed_precision!r}")
    if int(backend) != int(PlaceType.GPU):
        raise ValueError("convert_to_mixed_precision targets PlaceType.GPU")
    half = 'bfloat16' if int(mixed_precision) == int(PrecisionType.Bfloat16) else 'float16'
    tdt = torch.bfloat16 if half == 'bfloat16' else torch.float16
    black = sorted(set(black_list or ()))
    with open(model_file, 'rb') as f:
        desc = PD.decode('ProgramDesc', f.read())
    ops = desc['blocks'][0].setdefault('ops', [])
    def param_refs(obj, out):
        if isinstance(obj, dict):
            if '__param__' in obj:
                out.add(obj['__param__'])
            for v in obj.values():
                param_refs(v, out)
        elif isinstance(obj, list):
            for v in obj:
                param_refs(v, out)
        return out
    keep32 = set()
    for od in ops:
        if od.get('type') in black:
            for slot in od.get('inputs', []):
                keep32.update(slot.get('arguments', []))
            for a in od.get('attrs', []):
                if a.get('name') == '__pra_call__':
                    param_refs(PD.loads_call(PD.attr_value(a)), keep32)
    cfg = {'dtype': half, 'black_list': black, 'keep_io_types': bool(keep_io_types)}
    marker = {'type': MIXED_PRECISION_OP, 'inputs': [], 'outputs': [],
              'attrs': [{'name': 'config', 'type': PD.ATTR['STRING'], 's': json.dumps(cfg)}]}
    nfeed = sum(1 for od in ops if od.get('type') == 'feed')
    ops.insert(nfeed, marker)
    params = load(params_file)
    out = {}
    for k, v in params.items():
        t = v._t if isinstance(v, Tensor) else torch.as_tensor(v)
        if t.is_floating_point() and k not in keep32:
            t = t.to(tdt)
        out[k] = Tensor(t)
    for d in (os.path.dirname(mixed_model_file), os.path.dirname(mixed_params_file)):
        if d:
            os.makedirs(d, exist_ok=True)
    with open(mixed_model_file, 'wb') as f:
        f.write(PD.encode('ProgramDesc', desc))
    save(out, mixed_params_file)


def get_num_bytes_of_data_type(dtype):
    """Bytes per element of an inference DataType."""
    return {DataType.FLOAT32: 4, DataType.INT64: 8, DataType.INT32: 4, DataType.UINT8: 1, DataType.INT8: 1,
            DataType.FLOAT16: 2, DataType.BFLOAT16: 2, DataType.BOOL: 1}[DataType(int(dtype))]


def get_trt_compile_version():
    """TensorRT is not part of an MI355X build: (0, 0, 0) as the reference reports without it."""
    return (0, 0, 0)


def get_trt_runtime_version():
    return (0, 0, 0)


def _get_phi_kernel_name(op_name):
    """The kernel-registry name an op type dispatches to (ops/registry.py keys)."""
    from ..ops import registry as R
    names = {k[0] for k in R.list_kernels()}
    return op_name if op_name in names else op_name


def get_version():
    from .. import __version__
    return __version__
