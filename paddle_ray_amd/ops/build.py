"""Build the in-tree gfx950 kernel library ``_pra_hip`` (hipcc, no hipify, no JIT cache).

    python -m paddle_ray_amd.ops.build [--force]

Each ``csrc/*.hip`` is compiled with ``hipcc --offload-arch=gfx950 -O3``; the
pybind11 binding is compiled by hipcc as host code; everything is linked into
``paddle_ray_amd/ops/_pra_hip<EXT_SUFFIX>`` which travels with the repo
snapshot to the GPU box (built .so files are git-ignored).

Provenance: objects are rebuilt when the SHA-256 of their source (+ common.h + the exact
compile command) changes — content, not mtimes — and the linked library embeds
``pra_build_info()`` = {sources hash, arch, hipcc version}. ``_native`` compares that hash
with the sources next to it at load time, so a stale or foreign binary is refused instead
of silently running.
"""
import concurrent.futures as cf
import hashlib
import json
import os
import re
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


def _digest(paths, cmd=()):
    h = hashlib.sha256()
    for p in paths:
        h.update(os.path.basename(p).encode())
        with open(p, 'rb') as f:
            h.update(f.read())
    h.update('\0'.join(cmd).encode())
    return h.hexdigest()


def sources_hash():
    """Hash of every source that goes into the library (what build_info() must match)."""
    files = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC)
                   if f.endswith(('.hip', '.h', '.cpp')))
    return _digest(files, (ARCH,))


def _manifest_path():
    return os.path.join(BUILD, 'manifest.json')


def _needs(obj, key, manifest):
    return not os.path.exists(obj) or manifest.get(os.path.basename(obj)) != key


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


@__import__('functools').lru_cache(None)
def _hipcc_version():
    try:
        r = subprocess.run([HIPCC, '--version'], capture_output=True, text=True)
        for line in r.stdout.splitlines():
            if 'HIP version' in line:
                return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return 'unknown'


def _stamp_path():
    return _out_path() + '.sources'


_HIP_FLAGS = ('-O3', '-fPIC', '-std=c++17', '-munsafe-fp-atomics')


def _toolchain_key():
    """hipcc version + compile flags: part of the library stamp, so a ROCm / flag change
    rebuilds instead of keeping a library compiled by another toolchain."""
    return hashlib.sha256((_hipcc_version() + '\0' + ' '.join(_HIP_FLAGS) + '\0' + ARCH).encode()).hexdigest()[:16]


def _stamp():
    return sources_hash() + ' ' + _toolchain_key()


_INC = re.compile(r'^\s*#\s*include\s+"([^"]+)"')


def _header_closure(src, seen=None):
    """The in-tree headers ``src`` includes, transitively (per-object rebuild keys: a header
    edit recompiles only the translation units that include it)."""
    seen = set() if seen is None else seen
    with open(src) as f:
        for line in f:
            m = _INC.match(line)
            if m:
                h = os.path.join(CSRC, m.group(1))
                if os.path.exists(h) and h not in seen:
                    seen.add(h)
                    _header_closure(h, seen)
    return sorted(seen)


def build(force=False, verbose=True):
    # fast path: the library next to the sources was linked from exactly these sources (the
    # sidecar travels with the .so; the object cache under build/ does not reach the GPU box)
    if not force and os.path.exists(_out_path()) and os.path.exists(_stamp_path()):
        with open(_stamp_path()) as f:
            if f.read().strip() == _stamp():
                if verbose:
                    print(f"up to date {_out_path()} (sources {sources_hash()[:12]})")
                return _out_path()
    import pybind11
    os.makedirs(BUILD, exist_ok=True)
    try:
        with open(_manifest_path()) as f:
            manifest = json.load(f)
    except (OSError, ValueError):
        manifest = {}
    hip_srcs = sorted(f for f in os.listdir(CSRC) if f.endswith('.hip'))
    jobs, keys, objs = [], {}, []
    for f in hip_srcs:
        src = os.path.join(CSRC, f)
        obj = os.path.join(BUILD, f.replace('.hip', '.o'))
        objs.append(obj)
        cmd = [HIPCC, f'--offload-arch={ARCH}', *_HIP_FLAGS, '-c', src, '-o', obj, '-I', CSRC]
        keys[os.path.basename(obj)] = _digest([src] + _header_closure(src), cmd + [_hipcc_version()])
        if force or _needs(obj, keys[os.path.basename(obj)], manifest):
            jobs.append(cmd)
    bsrc = os.path.join(CSRC, 'bindings.cpp')
    bobj = os.path.join(BUILD, 'bindings.o')
    objs.append(bobj)
    bcmd = [HIPCC, '-O2', '-fPIC', '-std=c++17', '-c', bsrc, '-o', bobj,
            '-I', pybind11.get_include(), '-I', sysconfig.get_paths()['include']]
    keys['bindings.o'] = _digest([bsrc], bcmd)
    if force or _needs(bobj, keys['bindings.o'], manifest):
        jobs.append(bcmd)
    with cf.ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        for j in ex.map(_run, jobs):
            pass
    # provenance record compiled into the library itself
    info = {'sources_sha256': sources_hash(), 'arch': ARCH, 'hipcc': _hipcc_version()}
    isrc = os.path.join(BUILD, 'build_info.cpp')
    iobj = os.path.join(BUILD, 'build_info.o')
    text = ('extern "C" const char* pra_build_info() { return R"PRA(' + json.dumps(info) +
            ')PRA"; }\n')
    old = open(isrc).read() if os.path.exists(isrc) else None
    if old != text or not os.path.exists(iobj):
        with open(isrc, 'w') as f:
            f.write(text)
        _run([HIPCC, '-O2', '-fPIC', '-c', isrc, '-o', iobj])
        jobs.append('build_info')
    objs.append(iobj)
    out = _out_path()
    if force or jobs or not os.path.exists(out):
        _run([HIPCC, '-shared', '-fPIC', f'--offload-arch={ARCH}', '-o', out] + objs)
    manifest.update(keys)
    with open(_manifest_path(), 'w') as f:
        json.dump(manifest, f, indent=1)
    with open(_stamp_path(), 'w') as f:
        f.write(_stamp() + '\n')
    if verbose:
        print(f"built {out} ({len(jobs)} objects recompiled, sources {info['sources_sha256'][:12]})")
    return out


if __name__ == '__main__':
    build(force='--force' in sys.argv)
