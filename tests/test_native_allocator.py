"""Native auto-growth best-fit allocator (parity: auto_growth_best_fit_allocator.cc +
stream_safe_cuda_allocator.cc). CPU: the block bookkeeping, built against malloc, under
random alloc/free traffic on several streams. GPU: a training step with every tensor coming
from the HIP build through torch's pluggable-allocator hook."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

from paddle_ray_amd.native import allocator as A

MB = 1 << 20


@pytest.fixture
def lib():
    path = A.library_path(host=True)
    if not os.path.exists(path):
        from paddle_ray_amd.native.build import build_allocator
        build_allocator()
    return A.load(host=True)


def _alloc(lib, dev, n, stream=0):
    p = lib.pra_alloc(n, dev, ctypes.c_void_p(stream))
    assert p, n
    return p


def test_random_traffic_keeps_invariants(lib):
    dev = 11
    lib.pra_alloc_set_growth(dev, 8 * MB)
    rs = np.random.RandomState(0)
    live = {}
    for step in range(3000):
        if live and (rs.rand() < 0.45 or len(live) > 200):
            p = list(live)[rs.randint(len(live))]
            n, s = live.pop(p)
            lib.pra_free(p, n, dev, ctypes.c_void_p(s))
        else:
            n = int(rs.choice([rs.randint(1, 4096), rs.randint(4096, 2 * MB), rs.randint(MB, 12 * MB)]))
            s = int(rs.randint(0, 3))
            p = _alloc(lib, dev, n, s)
            live[p] = (n, s)
        if step % 97 == 0:
            assert lib.pra_alloc_check(dev) == 1, step
            spans = sorted((p, p + ((n + 255) // 256) * 256) for p, (n, _) in live.items())
            assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:])), "live blocks overlap"
            st = A.stats(dev, lib)
            want = sum(((n + 255) // 256) * 256 for n, _ in live.values())
            # a block keeps a remainder smaller than the split threshold (<= 256 B extra)
            assert 0 <= st['allocated'] - want <= 256 * len(live)
    for p, (n, s) in list(live.items()):
        lib.pra_free(p, n, dev, ctypes.c_void_p(s))
    assert lib.pra_alloc_check(dev) == 1
    st = A.stats(dev, lib)
    assert st['allocated'] == 0 and st['num_allocs'] == st['num_frees']
    released = A.empty_cache(dev, lib)
    assert released > 0 and A.stats(dev, lib)['reserved'] == 0   # every chunk coalesced back


def test_best_fit_split_and_coalesce(lib):
    dev = 12
    lib.pra_alloc_set_growth(dev, 16 * MB)
    a = _alloc(lib, dev, 1 * MB)
    b = _alloc(lib, dev, 3 * MB)
    c = _alloc(lib, dev, 1 * MB)
    d = _alloc(lib, dev, 2 * MB)
    assert b == a + MB and c == b + 3 * MB            # split from one chunk, address order
    lib.pra_free(b, 3 * MB, dev, None)
    lib.pra_free(d, 2 * MB, dev, None)                 # d merges with the chunk's tail
    e = _alloc(lib, dev, 2 * MB + 17)                  # best fit: b's 3 MB hole, not the tail
    assert e == b
    lib.pra_free(e, 0, dev, None)
    lib.pra_free(a, MB, dev, None)
    lib.pra_free(c, MB, dev, None)                     # a|b|c|tail coalesce into one block
    st = A.stats(dev, lib)
    assert st['num_chunks'] == 1 and st['allocated'] == 0
    f = _alloc(lib, dev, 16 * MB)                      # whole chunk again: no new backend alloc
    assert f == a and A.stats(dev, lib)['num_backend_allocs'] == 1
    lib.pra_free(f, 0, dev, None)
    assert lib.pra_alloc_check(dev) == 1


_GPU_SCRIPT = r'''
import paddle_ray_amd as paddle
from paddle_ray_amd.native import allocator as A
from paddle_ray_amd.models import gpt_config, GPTForPretraining
assert A.enabled()
paddle.set_device('gpu:0')
m = GPTForPretraining(gpt_config('gpt3-tiny'))
opt = paddle.optimizer.AdamW(1e-3, parameters=m.parameters())
ids = paddle.randint(0, 1024, [4, 65])
losses = []
for _ in range(4):
    loss = m(ids[:, :-1], ids[:, 1:])
    loss.backward(); opt.step(); opt.clear_grad()
    losses.append(float(loss))
st = A.stats(0)
print('STATS', st['num_allocs'], st['allocated'], st['reserved'], paddle.device.cuda.memory_allocated())
assert st['num_allocs'] > 50 and st['reserved'] >= st['allocated'] > 0
assert paddle.device.cuda.memory_allocated() == st['allocated']
assert losses[-1] < losses[0], losses
print('OK', losses)
'''


@pytest.mark.gpu
def test_training_on_native_allocator_gpu():
    env = dict(os.environ, PRA_ALLOCATOR='auto_growth')
    r = subprocess.run([sys.executable, '-c', _GPU_SCRIPT], env=env, capture_output=True, text=True,
                       timeout=300, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0 and 'OK' in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]


def test_split_remainder_keeps_pending_gate(lib):
    """A block reused by its own stream while its free-time event is still pending is split:
    the remainder must stay gated (another stream may not take it until that work is done)."""
    dev = 41
    lib.pra_alloc_set_growth(dev, 2 * MB)
    s1, s2 = 0x1000, 0x2000
    a = _alloc(lib, dev, 2 * MB, s1)           # chunk 1 is exactly a
    warm = _alloc(lib, dev, 1 * MB, s2)        # second stream (chunk 2): events recorded from now on
    lib.pra_alloc_host_set_pending(1)
    try:
        lib.pra_free(a, 2 * MB, dev, ctypes.c_void_p(s1))   # pending: s1 work may still use it
        b = _alloc(lib, dev, 256 << 10, s1)                # same stream: reuses a, splits it
        assert b == a
        # 1.5 MB fits only in a's 1.75 MB remainder among existing free blocks
        c = _alloc(lib, dev, 3 * MB // 2, s2)
        assert not (a <= c < a + 2 * MB), "remainder handed to another stream before its event"
        lib.pra_alloc_host_complete_events()
        d = _alloc(lib, dev, 3 * MB // 2, s2)                # gate passed: now it may
        assert a <= d < a + 2 * MB
        assert lib.pra_alloc_check(dev) == 1
        for p, n, s in ((b, 256 << 10, s1), (c, 3 * MB // 2, s2), (d, 3 * MB // 2, s2),
                        (warm, MB, s2)):
            lib.pra_free(p, n, dev, ctypes.c_void_p(s))
    finally:
        lib.pra_alloc_host_set_pending(0)
        lib.pra_alloc_host_complete_events()


def test_record_stream_defers_reuse(lib):
    """Tensor.record_stream: a block used by a second stream is not reused -- by any stream,
    its own included -- until the work that stream had queued at free time is done."""
    dev = 42
    lib.pra_alloc_set_growth(dev, 4 * MB)
    s1, s2 = 0x1000, 0x2000
    a = _alloc(lib, dev, 1 * MB, s1)
    warm = _alloc(lib, dev, 1 * MB, s2)       # second stream: events from now on
    lib.pra_record_stream(ctypes.c_void_p(a), ctypes.c_void_p(s2))
    lib.pra_alloc_host_set_pending(1)
    try:
        lib.pra_free(a, MB, dev, ctypes.c_void_p(s1))
        assert A.stats(dev, lib)['allocated'] == 2 * MB     # held back, still counted
        b = _alloc(lib, dev, 1 * MB, s1)                    # same stream: may NOT reuse a
        assert b != a
        assert lib.pra_alloc_check(dev) == 1
        lib.pra_alloc_host_complete_events()
        c = _alloc(lib, dev, 1 * MB, s1)                    # s2's work done: a is free again
        assert c == a
        for p, s in ((b, s1), (c, s1), (warm, s2)):
            lib.pra_free(p, MB, dev, ctypes.c_void_p(s))
        assert lib.pra_alloc_check(dev) == 1 and A.stats(dev, lib)['allocated'] == 0
    finally:
        lib.pra_alloc_host_set_pending(0)
        lib.pra_alloc_host_complete_events()


def test_pool_arena_host_bookkeeping(lib):
    """Graph-capture arenas (host build): pool blocks come from their own chunks, are reused
    inside the pool, never mix with the device arena, and the pool's memory goes back once it
    is released and its last block freed."""
    dev = 51
    lib.pra_alloc_pool.restype = ctypes.c_void_p
    lib.pra_alloc_pool.argtypes = [ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                                   ctypes.c_uint64]
    lib.pra_pool_release.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64]
    lib.pra_pool_check.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64]
    e = _alloc(lib, dev, MB)
    p1 = lib.pra_alloc_pool(MB, dev, None, 7, 0)
    p2 = lib.pra_alloc_pool(3 * MB, dev, None, 7, 0)
    assert p1 and p2 and not (e <= p1 < e + MB)
    st = A.stats(dev, lib)
    assert st['num_pools'] == 1 and st['pool_allocated'] >= 4 * MB and st['allocated'] == MB
    lib.pra_free(p1, MB, dev, None)                       # freed inside the pool ...
    p3 = lib.pra_alloc_pool(MB, dev, None, 7, 0)            # ... and reused by it (best fit)
    assert p3 == p1
    e2 = _alloc(lib, dev, 512 << 10)                       # the device arena never gets pool memory
    assert not (p1 <= e2 < p1 + 4 * MB)
    assert lib.pra_pool_check(dev, 7, 0) == 1
    lib.pra_pool_release(dev, 7, 0)                         # graph gone, blocks still live
    assert A.stats(dev, lib)['num_pools'] == 1
    lib.pra_free(p2, 3 * MB, dev, None)
    lib.pra_free(p3, MB, dev, None)                         # last block: the arena is dropped
    st = A.stats(dev, lib)
    assert st['num_pools'] == 0 and st['pool_reserved'] == 0
    for p, n in ((e, MB), (e2, 512 << 10)):
        lib.pra_free(p, n, dev, None)
    assert lib.pra_alloc_check(dev) == 1


_GPU_GRAPH_SCRIPT = r'''
import torch
import paddle_ray_amd as paddle
from paddle_ray_amd.native import allocator as A
assert A.enabled()
x = torch.randn(1024, 1024, device='cuda')
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(2):
        y = (x @ x).relu() @ x
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    t = (x @ x).relu()        # an intermediate freed inside the capture
    y = t @ x
    del t
st = A.stats(0)
assert st['num_pools'] == 1 and st['pool_allocated'] > 0, st
eager = [torch.empty(1024, 1024, device='cuda') for _ in range(8)]   # never inside the pool
g.replay()
ref = (x @ x).relu() @ x
torch.cuda.synchronize()
assert torch.allclose(y, ref, rtol=1e-3, atol=1e-2)
for e in eager:
    e.fill_(7.0)
g.replay(); torch.cuda.synchronize()
assert torch.allclose(y, ref, rtol=1e-3, atol=1e-2)   # eager writes did not land in graph memory
before = A.stats(0)['pool_allocated']
del g, y
import gc; gc.collect(); torch.cuda.synchronize()
st = A.stats(0)
# the graph's blocks went back (its arena stays while the BLAS workspace it created lives)
assert st['pool_allocated'] < before, (before, st)
# a jit.to_static training graph (forward + backward captured) on the native allocator
from paddle_ray_amd.models import gpt_config, GPTForPretraining
paddle.set_device('gpu:0')
paddle.seed(0)
m = GPTForPretraining(gpt_config('gpt3-tiny', hidden_dropout=0.0, attention_dropout=0.0))
opt = paddle.optimizer.AdamW(1e-3, parameters=m.parameters())
st = paddle.static.BuildStrategy(); st.use_hip_graph = True
mg = paddle.jit.to_static(m, build_strategy=st)
ids = paddle.randint(0, 1024, [4, 65])
losses = []
for _ in range(5):
    loss = mg(ids[:, :-1], ids[:, 1:])
    loss.backward(); opt.step(); opt.clear_grad()
    losses.append(float(loss))
assert losses[-1] < losses[0], losses
print('OK', losses, A.stats(0)['num_pools'])
'''


@pytest.mark.gpu
def test_graph_capture_pools_on_native_allocator_gpu():
    env = dict(os.environ, PRA_ALLOCATOR='auto_growth')
    r = subprocess.run([sys.executable, '-c', _GPU_GRAPH_SCRIPT], env=env, capture_output=True, text=True,
                       timeout=300, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0 and 'OK' in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
