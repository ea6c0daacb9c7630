"""LDS-DMA MFMA GEMM (ops/csrc/gemm_lds.hip) vs hipBLASLt (torch.mm) on the GPT-3 1.3B training
GEMMs (M = 16 x 1024 tokens): correctness vs an fp32 reference, then interleaved timing rounds in
one process (median of per-round means).

    python scripts/gemm_lds_bench.py [--quick]
"""
import statistics
import sys
import time

import torch

sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from paddle_ray_amd.ops import _native  # noqa: E402

L = _native.lib()
T = 16384
SHAPES = [  # (name, layout, M, N, K)
    ('qkv.fwd', 0, T, 6144, 2048), ('out.fwd', 0, T, 2048, 2048), ('fc1.fwd', 0, T, 8192, 2048),
    ('fc2.fwd', 0, T, 2048, 8192),
    ('qkv.dgrad', 1, T, 2048, 6144), ('out.dgrad', 1, T, 2048, 2048), ('fc1.dgrad', 1, T, 2048, 8192),
    ('fc2.dgrad', 1, T, 8192, 2048),
    ('qkv.wgrad', 2, 2048, 6144, T), ('out.wgrad', 2, 2048, 2048, T), ('fc1.wgrad', 2, 2048, 8192, T),
    ('fc2.wgrad', 2, 8192, 2048, T),
    ('head.fwd', 1, T, 50304, 2048), ('head.dgrad', 0, T, 2048, 50304), ('head.wgrad', 2, 50304, 2048, T),
]

# BERT-base (hidden 768, FFN 3072, bs 32 x 512 tokens; MLM head on 32 x 80 masked rows): --bert
SHAPES_BERT = [
    ('qkv.fwd', 0, T, 2304, 768), ('out.fwd', 0, T, 768, 768), ('fc1.fwd', 0, T, 3072, 768),
    ('fc2.fwd', 0, T, 768, 3072),
    ('qkv.dgrad', 1, T, 768, 2304), ('out.dgrad', 1, T, 768, 768), ('fc1.dgrad', 1, T, 768, 3072),
    ('fc2.dgrad', 1, T, 3072, 768),
    ('qkv.wgrad', 2, 768, 2304, T), ('out.wgrad', 2, 768, 768, T), ('fc1.wgrad', 2, 768, 3072, T),
    ('fc2.wgrad', 2, 3072, 768, T),
    ('mlm.fwd', 1, 2560, 30522 // 8 * 8, 768),
]
if '--bert' in sys.argv:
    SHAPES = SHAPES_BERT


def operands(layout, M, N, K, dev):
    g = torch.Generator(device=dev).manual_seed(M * 7 + N * 3 + K)
    def r(*s):
        return (torch.rand(*s, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    if layout == 0:
        return r(M, K), r(K, N)
    if layout == 1:
        return r(M, K), r(N, K)
    return r(K, M), r(K, N)


def ref_mm(layout, a, b):
    if layout == 0:
        return torch.mm(a, b)
    if layout == 1:
        return torch.mm(a, b.t())
    return torch.mm(a.t(), b)


def ours(layout, a, b, c, M, N, K, bias=None, z=None, colsum=None, epi=0, beta=0):
    from paddle_ray_amd.ops import fused as F
    F._GEMM_MODE = 'mfma'  # the in-tree kernel on every layout (auto routes dy·Wᵀ to hipBLASLt)
    r = F._gemm_hip(layout, a, b, out=c)  # includes the split-K choice for small grids
    assert r is not None


def check(name, layout, M, N, K, dev):
    a, b = operands(layout, M, N, K, dev)
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ours(layout, a, b, c, M, N, K)
    ref = ref_mm(layout, a.float(), b.float())
    err = (c.float() - ref).abs().max().item()
    scale = ref.abs().max().item()
    return err / scale


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main_w4():
    """Kernel configurations vs hipBLASLt, interleaved in one process. A configuration is
    (name, alt-config mask for pra_gemm_set_w4, persistent-kernel mask for pra_gemm_set_pts)."""
    dev = torch.device('cuda')
    cfgs = [('W8', 0, 0), ('W4', 7, 0), ('W8I', 7 << 4, 0), ('W4B', 7 << 8, 0), ('W8B', 7 << 12, 0),
            ('W4P', 7 << 16, 0), ('W8P', 7 << 20, 0), ('W4T', 7 << 24, 0), ('W8T', 7 << 28, 0)]
    if '--ts' in sys.argv:  # the TS schedule against the default configurations only
        cfgs = [('W8', 0, 0), ('W4', 7, 0), ('W4T', 7 << 24, 0), ('W8T', 7 << 28, 0)]
    if '--pts' in sys.argv:  # persistent TS kernel vs per-tile TS (default alt mask) vs the W8 baseline
        ts = (1 << 28) | (1 << 25) | (1 << 30)
        cfgs = [('W8', 0, 0), ('TS', ts, 0), ('PTS', ts, 7), ('PTS8', ts, 7 | 16)]
    hdr = ' | '.join(f'err {c[0]}' for c in cfgs) + ' | ' + ' | '.join(f'{c[0]} us' for c in cfgs)
    print(f"| GEMM | layout | M | N | K | {hdr} | hipBLASLt us | best | best PF/s | best vs hipBLASLt |")
    print("|---|---|---|---|---|" + "---|" * (2 * len(cfgs) + 4), flush=True)
    tot = [0.0] * (len(cfgs) + 1)

    def setc(c):
        L.gemm_set_w4(c[1])
        L.gemm_set_pts(c[2])
    for name, layout, M, N, K in SHAPES:
        errs = []
        for c in cfgs:
            setc(c)
            errs.append(check(name, layout, M, N, K, dev))
        a, b = operands(layout, M, N, K, dev)
        c_out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

        def mk(cf):
            def f():
                setc(cf)
                ours(layout, a, b, c_out, M, N, K)
            return f
        fs = [mk(c) for c in cfgs] + [lambda: ref_mm(layout, a, b)]
        for f in fs:
            f()
        torch.cuda.synchronize()
        it = 5 if M * N * K > 1e12 else 20
        ts_ = [[] for _ in fs]
        for _ in range(5):
            for i, f in enumerate(fs):
                ts_[i].append(timeit(f, it))
        m = [statistics.median(t) for t in ts_]
        for i in range(len(fs)):
            tot[i] += m[i]
        fl = 2.0 * M * N * K
        bi = min(range(len(cfgs)), key=lambda i: m[i])
        print(f"| {name} | {layout} | {M} | {N} | {K} | " + ' | '.join(f'{e:.1e}' for e in errs) + ' | '
              + ' | '.join(f'{x * 1e3:.1f}' for x in m[:-1]) + f" | {m[-1] * 1e3:.1f} | {cfgs[bi][0]} | "
              f"{fl / m[bi] / 1e12:.3f} | {m[-1] / m[bi]:.3f} |", flush=True)
    print('\ntotal ' + ', '.join(f'{c[0]} {t:.3f} ms' for c, t in zip(cfgs, tot)) + f', hipBLASLt {tot[-1]:.3f} ms')
    L.gemm_set_w4(0)


def main():
    dev = torch.device('cuda')
    quick = '--quick' in sys.argv
    shapes = SHAPES[:1] + SHAPES[4:5] + SHAPES[8:9] if quick else SHAPES
    print("| GEMM | layout | M | N | K | rel err | ours us | ours PF/s | hipBLASLt us | hipBLASLt PF/s | ratio |")
    print("|---|---|---|---|---|---|---|---|---|---|---|", flush=True)
    tot_o = tot_h = 0.0
    for name, layout, M, N, K in shapes:
        rel = check(name, layout, M, N, K, dev)
        a, b = operands(layout, M, N, K, dev)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        fo = lambda: ours(layout, a, b, c, M, N, K)  # noqa: E731
        fh = lambda: ref_mm(layout, a, b)  # noqa: E731
        for f in (fo, fh):
            f()
        torch.cuda.synchronize()
        it = 5 if M * N * K > 1e12 else 20
        to, th = [], []
        for _ in range(5):
            to.append(timeit(fo, it))
            th.append(timeit(fh, it))
        mo, mh = statistics.median(to), statistics.median(th)
        fl = 2.0 * M * N * K
        tot_o += mo
        tot_h += mh
        print(f"| {name} | {layout} | {M} | {N} | {K} | {rel:.1e} | {mo * 1e3:.1f} | {fl / mo / 1e12:.3f} | "
              f"{mh * 1e3:.1f} | {fl / mh / 1e12:.3f} | {mh / mo:.3f} |", flush=True)
    print(f"\ntotal ours {tot_o:.3f} ms, hipBLASLt {tot_h:.3f} ms")


if __name__ == '__main__' and '--w4' in sys.argv:
    main_w4()
elif __name__ == '__main__' and '--fused' not in sys.argv:
    main()


def fused_main():
    """fc1 forward with bias+GELU(+pre-act) epilogue and fc2 dgrad with dGELU + bias-grad epilogue
    vs hipBLASLt GEMM + the separate bias-GELU kernels they replace."""
    from paddle_ray_amd.ops import fused as F
    dev = torch.device('cuda')
    x, w1 = operands(0, T, 8192, 2048, dev)
    b1 = (torch.rand(8192, device=dev) - 0.5).to(torch.bfloat16)
    z = torch.empty(T, 8192, device=dev, dtype=torch.bfloat16)
    dy, w2t = operands(1, T, 8192, 2048, dev)  # dy [T, 2048], W2 [8192, 2048] as [N][K]

    def ours_fwd():
        F._gemm_hip(0, x, w1, bias=b1, z=z, epi='gelu_tanh')

    def blas_fwd():
        F.bias_gelu(torch.mm(x, w1), b1, True)

    def ours_bwd():
        F._gemm_hip(1, dy, w2t, z=z, epi='dgelu_tanh', want_colsum=True)

    zz = z.clone().requires_grad_(False)

    def blas_bwd():
        dh = torch.mm(dy, w2t.t())
        F.BiasGeluFn.backward(type('C', (), {'saved_tensors': (zz, b1), 'needs_input_grad': (True, True, False),
                                             'approximate': True, 'shp': zz.shape})(), dh)

    if '--w4' in sys.argv:
        _native.lib().gemm_set_w4(7)
    F._GEMM_MODE = 'mfma'   # the in-tree kernel for the NT dGELU GEMM too (the 'auto' policy would skip it)
    if '--pts' in sys.argv:
        _native.lib().gemm_set_pts(2)
    print("\n| fused op | ours us | hipBLASLt + separate kernel us | ratio |\n|---|---|---|---|")
    for name, fo, fh in (('fc1 fwd +bias+GELU+Z', ours_fwd, blas_fwd), ('fc2 dgrad +dGELU+db', ours_bwd, blas_bwd)):
        fo(); fh()
        torch.cuda.synchronize()
        to, th = [], []
        for _ in range(5):
            to.append(timeit(fo, 10))
            th.append(timeit(fh, 10))
        mo, mh = statistics.median(to), statistics.median(th)
        print(f"| {name} | {mo * 1e3:.1f} | {mh * 1e3:.1f} | {mh / mo:.3f} |", flush=True)


if __name__ == '__main__' and '--fused' in sys.argv:
    fused_main()
