"""Build the native runtime extension in-tree: python -m paddle_ray_amd.native.build"""
import os
import subprocess
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))


def build(force=False, verbose=True):
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
