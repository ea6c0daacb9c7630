"""GELU-MLP GEMM epilogues: the derivative-saving forward (z <- gelu'(pre-activation)) and the
multiply-by-z fc2 dgrad (+ fc1 bias-gradient column sums) against the round-4 pair (forward saving
the pre-activation; hipBLASLt dgrad + the bias_gelu_bwd_db pass). Correctness vs fp32, then
interleaved timing in one process.

    python scripts/gemm_mlp_bench.py [--bert]
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_ray_amd.ops import fused as F  # noqa: E402

T = 16384
H, FF, APPROX = (768, 3072, False) if '--bert' in sys.argv else (2048, 8192, True)


def timeit(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    dev = torch.device('cuda')
    g = torch.Generator(device=dev).manual_seed(0)

    def r(*s, sc=1.0):
        return ((torch.rand(*s, device=dev, generator=g) * 2 - 1) * sc).to(torch.bfloat16)
    x, w1, b1 = r(T, H), r(H, FF, sc=0.05), r(FF, sc=0.5)
    w2, dy = r(FF, H, sc=0.05), r(T, H)
    gname = 'gelu_tanh' if APPROX else 'gelu'
    z_pre = torch.empty(T, FF, device=dev, dtype=torch.bfloat16)
    z_d = torch.empty_like(z_pre)

    # ---- correctness vs fp32 --------------------------------------------------------------
    pre = x.float() @ w1.float() + b1.float()
    pre_r = pre.detach().requires_grad_(True)
    hr = torch.nn.functional.gelu(pre_r, approximate='tanh' if APPROX else 'none')
    dref, = torch.autograd.grad(hr.sum(), pre_r)
    h = F._gemm_hip(F.GEMM_FWD, x, w1, bias=b1, z=z_d, epi=gname + '_d')
    assert h is not None
    torch.cuda.synchronize()
    eh = ((h.float() - hr.detach()).abs().max() / hr.abs().max()).item()
    ed = ((z_d.float() - dref).abs().max() / dref.abs().max()).item()
    dh = dy.float() @ w2.float().t()
    dz_ref = dh * z_d.float()
    dz, cs = F._gemm_hip(F.GEMM_NT, dy, w2, z=z_d, epi='mulz', want_colsum=True)
    torch.cuda.synchronize()
    edz = ((dz.float() - dz_ref).abs().max() / dz_ref.abs().max()).item()
    ecs = ((cs - dz.float().sum(0)).abs().max() / dz.float().sum(0).abs().max()).item()
    print(f"shape T={T} H={H} FF={FF} {gname}: rel err h {eh:.1e}  gelu' {ed:.1e}  dz {edz:.1e}  db {ecs:.1e}",
          flush=True)
    assert max(eh, ed, edz, ecs) < 2e-2

    # ---- timing ---------------------------------------------------------------------------
    def fwd_old():
        F._gemm_hip(F.GEMM_FWD, x, w1, bias=b1, z=z_pre, epi=gname)

    def fwd_new():
        F._gemm_hip(F.GEMM_FWD, x, w1, bias=b1, z=z_d, epi=gname + '_d')

    F._gemm_hip(F.GEMM_FWD, x, w1, bias=b1, z=z_pre, epi=gname)

    def bwd_old():
        dhh = torch.mm(dy, w2.t())
        F._dgelu_db(dhh, z_pre, APPROX)

    def bwd_pts():
        F._MLP_MULZ_PTS = True
        F._gemm_hip(F.GEMM_NT, dy, w2, z=z_d, epi='mulz', want_colsum=True)

    def bwd_ts():
        F._MLP_MULZ_PTS = False
        F._gemm_hip(F.GEMM_NT, dy, w2, z=z_d, epi='mulz', want_colsum=True)

    def plain_nt():
        torch.mm(dy, w2.t())

    fns = [('fwd +bias+GELU, z = pre-activation', fwd_old), ('fwd +bias+GELU, z = gelu\'', fwd_new),
           ('dgrad hipBLASLt + bias_gelu_bwd_db', bwd_old), ('dgrad in-tree PTS *z + db', bwd_pts),
           ('dgrad in-tree TS *z + db', bwd_ts), ('plain hipBLASLt dy·W2ᵀ (reference)', plain_nt)]
    for _, f in fns:
        f()
    torch.cuda.synchronize()
    ts = [[] for _ in fns]
    for _ in range(7):
        for i, (_, f) in enumerate(fns):
            ts[i].append(timeit(f))
    print("| op | us (median of 7 x 10) |\n|---|---|")
    for (name, _), t in zip(fns, ts):
        print(f"| {name} | {statistics.median(t):.1f} |", flush=True)
    F._MLP_MULZ_PTS = True


if __name__ == '__main__':
    main()
