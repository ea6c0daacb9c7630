"""Sharded DistributedFusedLamb (reference: paddle/fluid/operators/optimizers/
distributed_fused_lamb_op.cu:922-1000 reduce-scatter, :1595-1641 sharded moments / masters):
2- and 4-rank gloo jobs match single-process Lamb on the union of the ranks' batches, per-rank
optimizer state is 1/nranks, and the HIP shard kernels match the fp32 reference."""
import numpy as np
import pytest
import torch

from dist_utils import run_ranks

D_IN, D_H, D_OUT, B = 12, 24, 5, 4


def _model():
    import paddle_ray_amd as paddle
    paddle.seed(9)
    return paddle.nn.Sequential(paddle.nn.Linear(D_IN, D_H), paddle.nn.Tanh(), paddle.nn.Linear(D_H, D_OUT))


def _data(world, steps, acc):
    rs = np.random.RandomState(5)
    return (rs.randn(steps, acc, world, B, D_IN).astype('float32'),
            rs.randn(steps, acc, world, B, D_OUT).astype('float32'))


def _excl(p):
    return p.name.endswith('bias') or len(p.shape) == 1


def _run_dfl(rank, world, steps, acc, clip):
    import paddle_ray_amd as paddle
    from paddle_ray_amd.incubate.optimizer import DistributedFusedLamb
    m = _model()
    opt = DistributedFusedLamb(0.02, lamb_weight_decay=0.05, parameters=m.parameters(),
                               grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5) if clip else None,
                               exclude_from_weight_decay_fn=_excl, gradient_accumulation_steps=acc)
    xs, ys = _data(world, steps, acc)
    for s in range(steps):
        for a in range(acc):
            loss = ((m(paddle.to_tensor(xs[s, a, rank])) - paddle.to_tensor(ys[s, a, rank])) ** 2).mean()
            loss.backward()
            opt.step()
            opt.clear_grad()
    total = sum(int(np.prod(p.shape)) for p in m.parameters())
    return [p.numpy().copy() for p in m.parameters()], opt.state_bytes(), total


def _serial(world, steps, acc, clip):
    import paddle_ray_amd as paddle
    m = _model()
    opt = paddle.optimizer.Lamb(0.02, lamb_weight_decay=0.05, parameters=m.parameters(),
                                grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5) if clip else None,
                                exclude_from_weight_decay_fn=_excl)
    xs, ys = _data(world, steps, acc)
    for s in range(steps):
        x = xs[s].reshape(acc * world * B, D_IN)
        y = ys[s].reshape(acc * world * B, D_OUT)
        loss = ((m(paddle.to_tensor(x)) - paddle.to_tensor(y)) ** 2).mean()
        loss.backward()
        opt.step()
        opt.clear_grad()
    return [p.numpy().copy() for p in m.parameters()]


@pytest.mark.parametrize('world,acc,clip', [(2, 1, True), (4, 1, False), (2, 2, True)])
def test_dist_fused_lamb_matches_serial_lamb(tmp_path, world, acc, clip):
    res = run_ranks(_run_dfl, world, tmp_path, args=(3, acc, clip))
    ref = _serial(world, 3, acc, clip)
    for r in res[1:]:
        for a, b in zip(res[0][0], r[0]):
            assert np.array_equal(a, b), "ranks diverged"
    for a, b in zip(res[0][0], ref):
        np.testing.assert_allclose(a, b, rtol=2e-5, atol=2e-6)
    state, total = res[0][1], res[0][2]
    # moments + fp32 masters of this rank's shard only (padding rounds up slightly)
    assert state <= 12 * total / world * 1.5 + 12 * 128 * 3, (state, total)
    assert state < 12 * total


def test_dist_fused_lamb_single_process_matches_lamb():
    got = _run_dfl(0, 1, 3, 1, True)[0]
    ref = _serial(1, 3, 1, True)
    for a, b in zip(got, ref):
        np.testing.assert_allclose(a, b, rtol=2e-5, atol=2e-6)


@pytest.mark.gpu
def test_lamb_shard_kernels_match_fp32_reference():
    from paddle_ray_amd.ops import _native
    from paddle_ray_amd.ops.fused import _dt
    from paddle_ray_amd.incubate.optimizer.distributed_fused_lamb import lamb_stage1_ref, lamb_stage2_ref
    L = _native.lib()
    dev = torch.device('cuda')
    g = torch.Generator().manual_seed(0)
    n, P = 50000, 3
    pieces = [(0, 0, 8192), (0, 8192, 10000), (1, 10240, 30000), (2, 30016, 49990)]
    pt = torch.tensor(pieces, dtype=torch.int64, device=dev)
    for gdt in (torch.bfloat16, torch.float32):
        grad = torch.randn(n, generator=g).to(gdt)
        w = torch.randn(n, generator=g)
        m, v = torch.randn(n, generator=g) * 0.1, torch.rand(n, generator=g) * 0.01
        wd = torch.tensor([0.01, 0.0, 0.05])
        args = dict(b1=0.9, b2=0.999, eps=1e-6, bc1=1 - 0.9 ** 3, bc2=1 - 0.999 ** 3)
        # reference (fp32, CPU)
        rw, rm, rv, rr, rn = w.clone(), m.clone(), v.clone(), torch.zeros(n), torch.zeros(2 * P)
        lamb_stage1_ref(pieces, grad, rw, rm, rv, rr, wd, rn, P, args['b1'], args['b2'], args['eps'],
                        args['bc1'], args['bc2'], 0.5 * 0.7)
        rout = torch.zeros(n, dtype=torch.bfloat16)
        lamb_stage2_ref(pieces, rw, rr, rn, P, 0.01, rout)
        # HIP
        dg, dw, dm, dv = grad.to(dev), w.to(dev), m.to(dev), v.to(dev)
        dr, dn = torch.zeros(n, device=dev), torch.zeros(2 * P, device=dev)
        dwd = wd.to(dev)
        coef = torch.tensor([0.7], device=dev)
        dout = torch.zeros(n, dtype=torch.bfloat16, device=dev)
        s = torch.cuda.current_stream().cuda_stream
        L.lamb_shard_stage1(pt.data_ptr(), len(pieces), dg.data_ptr(), _dt(dg), dw.data_ptr(), dm.data_ptr(),
                            dv.data_ptr(), dr.data_ptr(), dwd.data_ptr(), dn.data_ptr(), P, args['b1'], args['b2'],
                            args['eps'], args['bc1'], args['bc2'], 0.5, coef.data_ptr(), s)
        L.lamb_shard_stage2(pt.data_ptr(), len(pieces), dw.data_ptr(), dr.data_ptr(), dn.data_ptr(), P, 0.01,
                            dout.data_ptr(), _dt(dout), s)
        torch.cuda.synchronize()
        np.testing.assert_allclose(dn.cpu().numpy(), rn.numpy(), rtol=1e-4)
        np.testing.assert_allclose(dm.cpu().numpy(), rm.numpy(), rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(dv.cpu().numpy(), rv.numpy(), rtol=5e-5, atol=1e-9)
        np.testing.assert_allclose(dw.cpu().numpy(), rw.numpy(), rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(dout.cpu().float().numpy(), rout.float().numpy(), rtol=1e-2, atol=1e-2)
        untouched = torch.ones(n, dtype=torch.bool)
        for _, lo, hi in pieces:
            untouched[lo:hi] = False
        assert torch.equal(dw.cpu()[untouched], w[untouched])      # padding between params kept
