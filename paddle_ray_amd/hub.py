"""paddle.hub (parity: python/paddle/hapi/hub.py): list/help/load entry points from a
``hubconf.py``. Only ``source='local'`` works here (no network)."""
import importlib.util
import os
import sys


def _load_hubconf(repo_dir, source):
    if source != 'local':
        raise RuntimeError("paddle.hub: only source='local' is available (no network access)")
    path = os.path.join(repo_dir, 'hubconf.py')
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    sys.path.insert(0, repo_dir)
    try:
        spec = importlib.util.spec_from_file_location('hubconf', path)
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
    finally:
        sys.path.remove(repo_dir)
    return m


def list(repo_dir, source='github', force_reload=False):  # noqa: A001
    m = _load_hubconf(repo_dir, source)
    return [n for n in dir(m) if callable(getattr(m, n)) and not n.startswith('_')]


def help(repo_dir, model, source='github', force_reload=False):  # noqa: A001
    return getattr(_load_hubconf(repo_dir, source), model).__doc__


def load(repo_dir, model, source='github', force_reload=False, **kwargs):
    return getattr(_load_hubconf(repo_dir, source), model)(**kwargs)
