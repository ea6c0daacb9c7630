"""Loader for the in-tree gfx950 kernel library ``_pra_hip`` (built by ``ops/build.py``)."""
import glob
import importlib.util
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None
_err = None


def _load():
    global _lib, _err
    if _lib is not None or _err is not None:
        return _lib
    cands = sorted(glob.glob(os.path.join(_HERE, '_pra_hip*.so')))
    if not cands:
        _err = ImportError(f"_pra_hip extension not built in {_HERE}; run "
                           f"`python -m paddle_ray_amd.ops.build`")
        return None
    try:
        spec = importlib.util.spec_from_file_location('paddle_ray_amd.ops._pra_hip', cands[0])
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        _check_provenance(mod)
        _lib = mod
    except Exception as e:  # pragma: no cover - depends on runtime libs
        _err = e
    return _lib


def build_info():
    import json
    return json.loads(lib().build_info())


def _check_provenance(mod):
    """Refuse a library that was not built from the sources beside it (a stale build or a
    foreign binary): the hash compiled into the .so must match csrc/ as it is now. Set
    PRA_SKIP_PROVENANCE=1 to bypass (e.g. an installed wheel without sources)."""
    import json
    if os.environ.get('PRA_SKIP_PROVENANCE') == '1' or not os.path.isdir(os.path.join(_HERE, 'csrc')):
        return
    from .build import sources_hash
    info = json.loads(mod.build_info())
    want = sources_hash()
    if info.get('sources_sha256') != want:
        raise ImportError(f"_pra_hip was built from different sources (library "
                          f"{info.get('sources_sha256', '?')[:12]}, csrc/ {want[:12]}); rebuild "
                          f"with `python -m paddle_ray_amd.ops.build`")


def available():
    import torch
    if not torch.cuda.is_available():
        return False
    return _load() is not None


def lib():
    l = _load()
    if l is None:
        raise RuntimeError(f"paddle_ray_amd native HIP library unavailable: {_err}")
    return l


def require():
    lib()


def load_error():
    _load()
    return _err
