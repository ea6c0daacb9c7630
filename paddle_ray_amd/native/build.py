"""Build the native runtime extension in-tree: python -m paddle_ray_amd.native.build"""
import os
import subprocess
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))


def build_allocator(force=False, verbose=True):
    """The auto-growth allocator twice: against the HIP runtime (hipcc, host code) and against
    malloc (-DPRA_ALLOC_HOST) for CPU unit tests of its bookkeeping."""
    src = os.path.join(HERE, 'alloc', 'auto_growth_allocator.cpp')
    outs = []
    for name, cmd in (
            ('_pra_alloc_host.so', ['g++', '-O2', '-std=c++17', '-shared', '-fPIC', '-pthread',
                                    '-DPRA_ALLOC_HOST', src]),
            ('_pra_alloc_hip.so', [os.environ.get('HIPCC', '/opt/rocm/bin/hipcc'), '-O2',
                                   '-std=c++17', '-shared', '-fPIC', src])):
        out = os.path.join(HERE, name)
        outs.append(out)
        if not force and os.path.exists(out) and os.path.getmtime(out) > os.path.getmtime(src):
            continue
        r = subprocess.run(cmd + ['-o', out], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(r.stderr)
        if verbose:
            print(f'built {out}')
    return outs


def build_torch_hooks(force=False, verbose=True):
    """The PyTorch integration of the allocator (alloc/torch_hooks.cpp): host C++ against the
    installed torch (g++; the HIP headers only for the c10 stream types)."""
    import torch
    src = os.path.join(HERE, 'alloc', 'torch_hooks.cpp')
    out = os.path.join(HERE, '_pra_alloc_torch' + sysconfig.get_config_var('EXT_SUFFIX'))
    if not force and os.path.exists(out) and os.path.getmtime(out) > os.path.getmtime(src):
        return out
    ti = os.path.dirname(torch.__file__)
    libs = ['torch', 'torch_cpu', 'c10', 'torch_python'] + \
        (['torch_hip', 'c10_hip'] if torch.version.hip else [])
    cmd = ['g++', '-O2', '-std=c++17', '-shared', '-fPIC', '-pthread', '-D__HIP_PLATFORM_AMD__=1',
           '-DUSE_ROCM=1', '-I', os.path.join(ti, 'include'),
           '-I', os.path.join(ti, 'include', 'torch', 'csrc', 'api', 'include'),
           '-I', '/opt/rocm/include', '-I', sysconfig.get_paths()['include'], src, '-o', out,
           '-L', os.path.join(ti, 'lib'), '-Wl,-rpath,' + os.path.join(ti, 'lib')] + ['-l' + x for x in libs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stderr[-4000:])
    if verbose:
        print(f'built {out}')
    return out


def build(force=False, verbose=True):
    build_allocator(force, verbose)
    try:
        build_torch_hooks(force, verbose)
    except Exception as e:  # the allocator stays usable through ctypes (no graph pools)
        print(f'warning: allocator torch hooks not built: {e}')
    import pybind11
    import glob
    srcs = sorted(glob.glob(os.path.join(HERE, 'src', '*.cpp')))
    out = os.path.join(HERE, '_pra_runtime' + sysconfig.get_config_var('EXT_SUFFIX'))
    if not force and os.path.exists(out) and \
            os.path.getmtime(out) > max(os.path.getmtime(s) for s in srcs):
        return out
    cmd = ['g++', '-O2', '-std=c++17', '-shared', '-fPIC', '-pthread', *srcs, '-o', out, '-I',
           pybind11.get_include(), '-I', sysconfig.get_paths()['include']]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stderr)
    if verbose:
        print(f'built {out}')
    return out


if __name__ == '__main__':
    build(force=True)
