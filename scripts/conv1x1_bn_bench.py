"""ResNet-50 (bs 256, NHWC bf16) 1x1 conv + BatchNorm(+ReLU) forward and forward+backward:
hipBLASLt NT GEMM + separate BN statistics pass (PRA_CONV1X1_STATS=0 path) vs the implicit-GEMM
conv kernel with the statistics in its epilogue. Interleaved in one process, median of rounds."""
import statistics
import sys

import torch

sys.path.insert(0, '.')
from paddle_ray_amd.ops import fused as K  # noqa: E402

SHAPES = [  # (name, H=W of input, cin, cout, stride)
    ('l1.conv1a', 56, 64, 64, 1), ('l1.conv1', 56, 256, 64, 1), ('l1.conv3', 56, 64, 256, 1),
    ('l2.conv1a', 56, 256, 128, 1), ('l2.conv1', 28, 512, 128, 1), ('l2.conv3', 28, 128, 512, 1),
    ('l2.ds', 56, 256, 512, 2),
    ('l3.conv1a', 28, 512, 256, 1), ('l3.conv1', 14, 1024, 256, 1), ('l3.conv3', 14, 256, 1024, 1),
    ('l3.ds', 28, 512, 1024, 2),
    ('l4.conv1a', 14, 1024, 512, 1), ('l4.conv1', 7, 2048, 512, 1), ('l4.conv3', 7, 512, 2048, 1),
    ('l4.ds', 14, 1024, 2048, 2),
]
COUNT = {'l1.conv1a': 1, 'l1.conv1': 2, 'l1.conv3': 3, 'l2.conv1a': 1, 'l2.conv1': 3, 'l2.conv3': 4, 'l2.ds': 1,
         'l3.conv1a': 1, 'l3.conv1': 5, 'l3.conv3': 6, 'l3.ds': 1, 'l4.conv1a': 1, 'l4.conv1': 2, 'l4.conv3': 3,
         'l4.ds': 1}


def timeit(fn, it=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


def main():
    torch.manual_seed(0)
    dev = 'cuda'
    print('| conv | M | cin | cout | s | fwd blas+stats us | fwd fused us | f+b blas+stats us | f+b fused us | x/step |')
    print('|---|---|---|---|---|---|---|---|---|---|')
    tot = [0.0] * 4
    for name, hw, cin, cout, st in SHAPES:
        x = torch.randn(256, hw, hw, cin, device=dev).bfloat16().requires_grad_()
        w = (torch.randn(cout, cin, 1, 1, device=dev) * (2.0 / cin) ** 0.5).bfloat16().requires_grad_()
        s = torch.ones(cout, device=dev, requires_grad=True)
        b = torch.zeros(cout, device=dev, requires_grad=True)
        rm, rv = torch.zeros(cout, device=dev), torch.ones(cout, device=dev)
        ho = (hw - 1) // st + 1
        g = torch.randn(256, ho, ho, cout, device=dev).bfloat16()

        def fwd(flag):
            K._CONV1X1_STATS = flag
            with torch.no_grad():
                return K.conv_bn_act_nhwc(x, w, st, 0, s, b, rm, rv, True, 0.9, 1e-5, None, True)

        def fb(flag):
            K._CONV1X1_STATS = flag
            y = K.conv_bn_act_nhwc(x, w, st, 0, s, b, rm, rv, True, 0.9, 1e-5, None, True)
            y.backward(g)
            x.grad = w.grad = s.grad = b.grad = None
        r = [[] for _ in range(4)]
        for _ in range(5):
            r[0].append(timeit(lambda: fwd(False)))
            r[1].append(timeit(lambda: fwd(True)))
            r[2].append(timeit(lambda: fb(False)))
            r[3].append(timeit(lambda: fb(True)))
        m = [statistics.median(v) for v in r]
        n = COUNT[name]
        for i in range(4):
            tot[i] += m[i] * n
        print(f'| {name} | {256 * ho * ho} | {cin} | {cout} | {st} | {m[0]:.1f} | {m[1]:.1f} | {m[2]:.1f} | {m[3]:.1f} | {n} |',
              flush=True)
    print(f'\nper ResNet-50 step (x count): fwd {tot[0] / 1e3:.2f} vs {tot[1] / 1e3:.2f} ms, '
          f'fwd+bwd {tot[2] / 1e3:.2f} vs {tot[3] / 1e3:.2f} ms')


if __name__ == '__main__':
    main()
