"""Where a GEMM tile's time goes: per-workgroup phase stamps of the diagnostic build
(ops/csrc/gemm_probe.hip). Prints, per configuration, the median / p90 shader-clock cycles of the
prologue (entry -> first fragment read), the K loop and the epilogue, the in-kernel clock, and
the gap between consecutive workgroups on the same CU (launch / drain cost).

    python scripts/gemm_stamps.py [layout M N K]
"""
import collections
import statistics
import sys

import torch

sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from paddle_ray_amd.ops import _native  # noqa: E402
from scripts.gemm_lds_bench import operands  # noqa: E402

L = _native.lib()


def run(cfg, layout, M, N, K, reps=6):
    a, b = operands(layout, M, N, K, torch.device('cuda'))
    c = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
    tiles = (M // 256) * (N // 256)
    st = torch.zeros(tiles * 16, dtype=torch.int64, device='cuda')
    lda = K
    ldb = N if layout == 0 else K
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(reps):
        n = L.gemm_probe(cfg, layout, a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, lda, ldb, N,
                         st.data_ptr(), s)
        assert n == tiles
    torch.cuda.synchronize()
    w = st.view(tiles, 16).cpu().tolist()
    pro = [r[1] - r[0] for r in w]
    loop = [r[2] - r[1] for r in w]
    epi = [r[3] - r[2] for r in w]
    clk = [(r[3] - r[0]) / max(1, (r[5] - r[4])) * 0.1 for r in w]  # GHz (realtime is 100 MHz)
    # per-CU timelines: (xcc, se/sh/cu bits of HW_ID)
    by_cu = collections.defaultdict(list)
    for r in w:
        hw = r[6]
        key = (r[7] & 0xf, (hw >> 8) & 0xf, (hw >> 12) & 0x1, (hw >> 13) & 0x7)
        by_cu[key].append((r[4], r[5]))
    gaps = []
    for ev in by_cu.values():
        ev.sort()
        for (s0, e0), (s1, e1) in zip(ev, ev[1:]):
            gaps.append((s1 - e0) * 10.0)  # ns
    span = (max(r[5] for r in w) - min(r[4] for r in w)) * 10.0 / 1e3
    q = lambda v, p: sorted(v)[int(p * (len(v) - 1))]  # noqa: E731
    print(f"cfg {cfg} layout {layout} {M}x{N}x{K}: {tiles} tiles on {len(by_cu)} CUs, span {span:.1f} us, "
          f"clock {statistics.median(clk):.2f} GHz")
    for name, v in (('prologue', pro), ('loop', loop), ('epilogue', epi)):
        print(f"   {name:9s} cycles median {statistics.median(v):9.0f}  p10 {q(v, .1):9.0f}  p90 {q(v, .9):9.0f}")
    if gaps:
        print(f"   gap between workgroups on one CU: median {statistics.median(gaps):.0f} ns, "
              f"p90 {q(gaps, .9):.0f} ns, n={len(gaps)}")
    nk = K // 64
    secs = [statistics.median([r[8 + i] for r in w]) / nk for i in range(3)]
    print(f"   loop cycles per K-step {statistics.median(loop) / nk:.0f} (MFMA-bound: 2048); default body "
          f"sections per K-step: half0 {secs[0]:.0f}, wait+barrier {secs[1]:.0f}, half1 {secs[2]:.0f}",
          flush=True)


if __name__ == '__main__':
    shapes = [(1, 16384, 2048, 8192), (1, 16384, 8192, 2048), (0, 16384, 8192, 2048), (0, 16384, 2048, 8192)]
    if len(sys.argv) > 4:
        shapes = [tuple(int(x) for x in sys.argv[1:5])]
    for sh in shapes:
        for cfg in (0, 1, 2):
            run(cfg, *sh)
