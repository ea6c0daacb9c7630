"""Build provenance: the HIP library embeds the SHA-256 of the sources it was compiled from
and the loader refuses a library whose hash does not match csrc/ as it is now."""
import os

import pytest

from paddle_ray_amd.ops import _native, build


def test_loaded_library_matches_sources():
    mod = _native._load()
    if mod is None:
        pytest.skip(f"library not loadable here: {_native.load_error()}")
    assert _native.build_info()['sources_sha256'] == build.sources_hash()
    assert _native.build_info()['arch'] == 'gfx950'


def test_stale_library_is_refused(monkeypatch):
    mod = _native._load()
    if mod is None:
        pytest.skip(f"library not loadable here: {_native.load_error()}")
    monkeypatch.setattr(build, 'sources_hash', lambda: '0' * 64)
    with pytest.raises(ImportError, match='different sources'):
        _native._check_provenance(mod)


@pytest.mark.gpu
def test_gpu_runs_the_in_tree_library():
    import torch
    assert torch.cuda.is_available()
    mod = _native.lib()
    assert os.path.dirname(mod.__file__) == os.path.dirname(_native.__file__)
    assert _native.build_info()['sources_sha256'] == build.sources_hash()
