"""Build the in-tree gfx950 kernel library ``_pra_hip`` (hipcc, no hipify, no JIT cache).

    python -m paddle_ray_amd.ops.build [--force]

Each ``csrc/*.hip`` is compiled with ``hipcc --offload-arch=gfx950 -O3``; the
pybind11 binding is compiled by hipcc as host code; everything is linked into
``paddle_ray_amd/ops/_pra_hip<EXT_SUFFIX>`` which travels with the repo
snapshot to the GPU box (built .so files are git-ignored).
"""
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
BUILD = os.path.join(HERE, '..', '..', 'build', 'pra_hip')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = os.environ.get('PRA_ARCH', 'gfx950')


def _out_path():
    return os.path.join(HERE, '_pra_hip' + sysconfig.get_config_var('EXT_SUFFIX'))


def _needs(obj, srcs):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(s) > t for s in srcs)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def build(force=False, verbose=True):
    import pybind11
    os.makedirs(BUILD, exist_ok=True)
    common = os.path.join(CSRC, 'common.h')
    hip_srcs = sorted(f for f in os.listdir(CSRC) if f.endswith('.hip'))
    jobs = []
    objs = []
    for f in hip_srcs:
        src = os.path.join(CSRC, f)
        obj = os.path.join(BUILD, f.replace('.hip', '.o'))
        objs.append(obj)
        if force or _needs(obj, [src, common]):
            jobs.append([HIPCC, f'--offload-arch={ARCH}', '-O3', '-fPIC', '-std=c++17', '-c', src, '-o', obj,
                         '-I', CSRC, '-munsafe-fp-atomics'])
    bsrc = os.path.join(CSRC, 'bindings.cpp')
    bobj = os.path.join(BUILD, 'bindings.o')
    objs.append(bobj)
    if force or _needs(bobj, [bsrc]):
        jobs.append([HIPCC, '-O2', '-fPIC', '-std=c++17', '-c', bsrc, '-o', bobj,
                     '-I', pybind11.get_include(), '-I', sysconfig.get_paths()['include']])
    with cf.ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        for j in ex.map(_run, jobs):
            pass
    out = _out_path()
    if force or jobs or not os.path.exists(out):
        _run([HIPCC, '-shared', '-fPIC', f'--offload-arch={ARCH}', '-o', out] + objs)
    if verbose:
        print(f"built {out} ({len(jobs)} objects recompiled)")
    return out


if __name__ == '__main__':
    build(force='--force' in sys.argv)
