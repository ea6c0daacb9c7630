"""MI355X op benchmark table for paddle.cost_model (reference schema:
python/paddle/cost_model/static_op_benchmark.json). Times forward and forward+backward of
the framework's ops on the GPT / ResNet shapes and writes
paddle_ray_amd/cost_model/static_op_benchmark_gfx950.json (or --out)."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import paddle_ray_amd as paddle  # noqa: E402
import paddle_ray_amd.nn.functional as F  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--out', default=os.path.join(os.path.dirname(paddle.__file__), 'cost_model',
                                              'static_op_benchmark_gfx950.json'))
ap.add_argument('--iters', type=int, default=20)
a = ap.parse_args()
paddle.set_device('gpu')


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def rnd(shape, dtype, grad=True):
    x = paddle.randn(shape, dtype='float32').astype(dtype)
    x.stop_gradient = not grad
    return x


CASES = []


def case(op, dtype, desc, make, fn):
    CASES.append((op, dtype, desc, make, fn))


for dt in ('bfloat16', 'float32'):
    case('matmul', dt, 'x: [16384, 2048], y: [2048, 8192]',
         lambda dt=dt: (rnd([16384, 2048], dt), rnd([2048, 8192], dt)), paddle.matmul)
    case('layer_norm', dt, 'x: [16384, 2048]',
         lambda dt=dt: (rnd([16384, 2048], dt), rnd([2048], dt), rnd([2048], dt)),
         lambda x, w, b: F.layer_norm(x, [2048], w, b))
    case('softmax', dt, 'x: [256, 1024, 1024]', lambda dt=dt: (rnd([256, 1024, 1024], dt),),
         lambda x: F.softmax(x, -1))
    case('gelu', dt, 'x: [16384, 8192]', lambda dt=dt: (rnd([16384, 8192], dt),), F.gelu)
    case('elementwise_add', dt, 'x: [16384, 2048], y: [16384, 2048]',
         lambda dt=dt: (rnd([16384, 2048], dt), rnd([16384, 2048], dt)), paddle.add)
    case('conv2d', dt, 'x: [256, 64, 56, 56], w: [64, 64, 3, 3], NCHW',
         lambda dt=dt: (rnd([256, 64, 56, 56], dt), rnd([64, 64, 3, 3], dt)),
         lambda x, w: F.conv2d(x, w, padding=1))
    case('cross_entropy', dt, 'logits: [16384, 50304], label: [16384]',
         lambda dt=dt: (rnd([16384, 50304], dt), paddle.randint(0, 50304, [16384])),
         lambda x, y: F.cross_entropy(x, y))
case('flash_attention', 'bfloat16', 'q/k/v: [16, 1024, 16, 128], causal',
     lambda: tuple(rnd([16, 1024, 16, 128], 'bfloat16') for _ in range(3)),
     lambda q, k, v: F.scaled_dot_product_attention(q, k, v, is_causal=True))
case('embedding', 'bfloat16', 'ids: [16, 1024], w: [50304, 2048]',
     lambda: (paddle.randint(0, 50304, [16, 1024]), rnd([50304, 2048], 'bfloat16')),
     lambda i, w: F.embedding(i, w))

rows = []
for op, dt, desc, make, fn in CASES:
    args = make()
    fwd = timeit(lambda: fn(*args), a.iters)

    def fb():
        out = fn(*args)
        out.sum().backward() if out.dtype != paddle.int64 else None
    tot = timeit(fb, a.iters)
    for t in args:
        if hasattr(t, 'clear_gradient'):
            t.clear_gradient()
    rows.append({'name': f'{op}_{dt}', 'op': op, 'config': f'{desc}, dtype: {dt}\n',
                 'device': torch.cuda.get_device_name(0), 'paddle_gpu_time': round(fwd, 4),
                 'paddle_gpu_time_backward': round(max(tot - fwd, 0.0), 4)})
    print(f'{op:16s} {dt:9s} fwd {fwd:8.3f} ms  bwd {tot - fwd:8.3f} ms', flush=True)
with open(a.out, 'w') as f:
    json.dump(rows, f, indent=1)
print('wrote', a.out)
