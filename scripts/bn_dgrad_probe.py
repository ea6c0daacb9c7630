"""Per-shape cost of the BN+ReLU backward with its reductions in the consumer conv's dgrad
epilogue (kBnG) vs the plain dgrad + the 3-kernel BN backward, on the ResNet-50 (bs 256) shapes
where a BN output feeds a stride-1 conv: 3x3 conv2 dgrad -> bn1, 1x1 conv3 dgrad -> bn2.
Interleaved timing in one process.

    python scripts/bn_dgrad_probe.py [batch]
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_ray_amd.ops import fused as F, _native  # noqa: E402

NB = int(sys.argv[1]) if len(sys.argv) > 1 else 256


def timeit(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    L = _native.lib()
    dev = 'cuda'
    print(f"batch {NB}\n| conv | H | C | dgrad plain | BN bwd plain | sum | dgrad kBnG | BN parts | sum | gain |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for kind, hw, c in [('3x3', 56, 64), ('3x3', 28, 128), ('3x3', 14, 256), ('3x3', 7, 512),
                        ('1x1', 56, 64), ('1x1', 28, 128), ('1x1', 14, 256), ('1x1', 7, 512)]:
        torch.manual_seed(0)
        m = NB * hw * hw
        co = c if kind == '3x3' else 4 * c
        x2 = torch.randn(m, c, device=dev).bfloat16()
        s = torch.rand(c, device=dev) + 0.5
        b = torch.randn(c, device=dev) * 0.1
        y, mean, invstd, mask = F._bn_fwd_hip(x2, None, s, b, None, None, True, 0.9, 1e-5, True)
        dy = torch.randn(NB, hw, hw, co, device=dev).bfloat16()
        if kind == '3x3':
            w = (torch.randn(co, c, 3, 3, device=dev) * 0.05).bfloat16()
            wf = w.flip(2, 3).permute(1, 2, 3, 0).reshape(c, 9 * co).contiguous()
            plain = lambda: F._conv_lds(dy, wf, None, 3, 3, 1, 1)  # noqa: E731
            fused = lambda: F._conv_lds(dy, wf, None, 3, 3, 1, 1, bn=(x2, mask, mean))  # noqa: E731
        else:
            w2 = (torch.randn(co, c, device=dev) * 0.05).bfloat16()
            wt = w2.t().contiguous()
            dy2 = dy.view(m, co)
            plain = lambda: F.gemm(F.GEMM_FWD, dy2, w2)  # noqa: E731
            fused = lambda: F._conv_lds(dy, wt, None, 1, 1, 1, 0, bn=(x2, mask, mean))  # noqa: E731
        g0 = plain().reshape(m, c)
        gf, part = fused()
        gf = gf.reshape(m, c)
        bn_plain = lambda: F._bn_bwd_hip(g0, None, mask, x2, s, mean, invstd, True, False)  # noqa: E731
        bn_parts = lambda: F._bn_bwd_parts_hip(gf, x2, s, mean, invstd, part)  # noqa: E731
        # sanity: same dx
        d0 = bn_plain()[0].float()
        d1 = bn_parts()[0].float()
        err = (d0 - d1).abs().max().item() / (d0.abs().max().item() + 1e-6)
        fns = [plain, bn_plain, fused, bn_parts]
        for f in fns:
            f()
        torch.cuda.synchronize()
        ts = [[] for _ in fns]
        for _ in range(5):
            for i, f in enumerate(fns):
                ts[i].append(timeit(f))
        t = [statistics.median(v) for v in ts]
        print(f"| {kind} | {hw} | {c} | {t[0]:.1f} | {t[1]:.1f} | {t[0] + t[1]:.1f} | {t[2]:.1f} | {t[3]:.1f} | "
              f"{t[2] + t[3]:.1f} | {t[0] + t[1] - t[2] - t[3]:+.1f} (err {err:.1e}, splits "
              f"{L.conv_lds_splits(m, c, (9 if kind == '3x3' else 1) * co)}) |", flush=True)


if __name__ == '__main__':
    main()
