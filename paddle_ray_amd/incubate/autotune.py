"""paddle.incubate.autotune (parity: python/paddle/incubate/autotune.py ``set_config``).

Kernel auto-tuning on MI355X maps onto the two library searches the compute path uses:

* GEMMs (hipBLASLt / rocBLAS under ``torch.mm``/``addmm``): PyTorch-ROCm TunableOp
  benchmarks every candidate solution per (op, transpose, M, N, K, dtype) and keeps the
  fastest. Results persist in a CSV; the in-tree ``tuning/gemm_gfx950.csv`` holds the
  solutions measured on MI355X for the flagship shapes and is loaded read-only by
  :func:`use_tuned_gemms` (no tuning at run time).
* convolutions (MIOpen): find-mode algorithm search, ``torch.backends.cudnn.benchmark``.

``layout`` tuning is accepted and recorded (the vision models already run NHWC on the
device); ``dataloader`` tuning is accepted and recorded (the native ring loader sizes its
own prefetch depth).
"""
import json
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
TUNED_GEMM_FILE = os.path.join(os.path.dirname(_HERE), 'tuning', 'gemm_gfx950.csv')

_config = {'kernel': {'enable': False, 'tuning_range': [1, 10]},
           'layout': {'enable': False}, 'dataloader': {'enable': False}}


def get_config():
    return json.loads(json.dumps(_config))


def _tunable():
    import torch
    if not torch.cuda.is_available():
        return None
    return torch.cuda.tunable


def enable_gemm_tuning(filename=None, tune=True, max_duration_ms=30, max_iterations=100):
    """Turn on TunableOp GEMM search (``tune=True``) or replay of a results file
    (``tune=False``). Returns False when there is no device."""
    t = _tunable()
    if t is None:
        return False
    t.enable(True)
    t.tuning_enable(bool(tune))
    t.set_max_tuning_duration(int(max_duration_ms))
    t.set_max_tuning_iterations(int(max_iterations))
    if filename is not None:
        t.set_filename(filename, insert_device_ordinal=False)
        if os.path.exists(filename):
            t.read_file(filename)
    return True


def use_tuned_gemms(filename=None):
    """Replay the committed MI355X GEMM solutions (read-only; untuned shapes fall back
    to the hipBLASLt heuristic). No-op without a device or results file."""
    filename = filename or os.environ.get('PRA_GEMM_TUNING_FILE', TUNED_GEMM_FILE)
    if not os.path.exists(filename):
        return False
    t = _tunable()
    if t is None:
        return False
    t.enable(True)
    t.tuning_enable(False)
    # never write the shared file back: point the writer at a scratch path
    t.set_filename(os.path.join(os.environ.get('TMPDIR', '/tmp'), 'pra_tunableop_unused.csv'),
                   insert_device_ordinal=True)
    return bool(t.read_file(filename))


def write_gemm_results(filename):
    """Write every tuned GEMM solution of this process (validators first) as a TunableOp
    CSV that :func:`use_tuned_gemms` / ``torch.cuda.tunable.read_file`` accept."""
    t = _tunable()
    if t is None:
        return 0
    vals = t.get_validators()
    res = t.get_results()
    os.makedirs(os.path.dirname(os.path.abspath(filename)), exist_ok=True)
    with open(filename, 'w') as f:
        for k, v in vals:
            f.write(f"Validator,{k},{v}\n")
        for op_sig, param_sig, solution, ms in res:
            f.write(f"{op_sig},{param_sig},{solution},{ms}\n")
    return len(res)


def set_config(config=None):
    """Configure kernel / layout / dataloader auto-tuning (dict, JSON path, or None = all on)."""
    global _config
    if config is None:
        cfg = {'kernel': {'enable': True}, 'layout': {'enable': True},
               'dataloader': {'enable': True}}
    elif isinstance(config, str):
        with open(config) as f:
            cfg = json.load(f)
    elif isinstance(config, dict):
        cfg = config
    else:
        raise TypeError("set_config expects a dict, a JSON file path or None")
    for key, val in cfg.items():
        if key not in _config:
            import warnings
            warnings.warn(f"autotune: unknown tuning type {key!r} ignored")
            continue
        if not isinstance(val, dict):
            raise TypeError(f"autotune config for {key!r} must be a dict")
        _config[key].update(val)
    if _config['kernel'].get('enable'):
        import torch
        if torch.cuda.is_available():
            torch.backends.cudnn.benchmark = True
            if not use_tuned_gemms():
                enable_gemm_tuning(tune=True)
        from ..framework import flags
        flags._FLAGS['FLAGS_cudnn_exhaustive_search'] = True
        flags._FLAGS['FLAGS_use_autotune'] = True
    else:
        import torch
        from ..framework import flags
        flags._FLAGS['FLAGS_cudnn_exhaustive_search'] = False
        flags._FLAGS['FLAGS_use_autotune'] = False
        if torch.cuda.is_available():
            torch.backends.cudnn.benchmark = False
            torch.cuda.tunable.enable(False)
    return get_config()
