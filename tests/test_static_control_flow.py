"""Static control flow executes at RUN time (parity: static/nn/control_flow.py while_loop /
cond / StaticRNN over while_op.cc, conditional_block_op.cc, recurrent_op.cc): the same
program takes a fed-value-dependent trip count / branch, and append_backward differentiates
through the iterations that actually ran. Plus data_norm, nce and row_conv semantics."""
import numpy as np
import pytest

import paddle_ray_amd as paddle
import paddle_ray_amd.nn.functional as F
from paddle_ray_amd import static


@pytest.fixture
def static_mode():
    paddle.enable_static()
    yield
    paddle.disable_static()


def test_while_loop_trip_count_is_runtime(static_mode):
    main = static.Program()
    with static.program_guard(main):
        n = static.data('n', [1], 'int64')
        x = static.data('x', [2, 3], 'float32')
        i = paddle.zeros([1], 'int64')
        acc = paddle.zeros([2, 3], 'float32')
        i_out, acc_out = static.nn.while_loop(lambda i, a: i < n,
                                              lambda i, a: [i + 1, a + x * 2.0], [i, acc])
    exe = static.Executor()
    xv = np.random.RandomState(0).rand(2, 3).astype('float32')
    for trips in (0, 3, 7):
        iv, av = exe.run(main, feed={'n': np.array([trips]), 'x': xv}, fetch_list=[i_out, acc_out])
        assert int(iv[0]) == trips
        np.testing.assert_allclose(av, xv * 2.0 * trips, rtol=1e-6)
    assert [op.type for op in main.global_block().ops].count('while') == 1


def test_while_loop_gradient_through_runtime_iterations(static_mode):
    paddle.seed(3)
    main = static.Program()
    with static.program_guard(main):
        n = static.data('n', [1], 'int64')
        h0 = static.data('h0', [4, 8], 'float32')
        i = paddle.zeros([1], 'int64')
        lin = paddle.nn.Linear(8, 8)

        def body(i, h):
            return [i + 1, paddle.tanh(lin(h))]
        _, h = static.nn.while_loop(lambda i, h: i < n, body, [i, h0])
        loss = paddle.mean(h * h)
        pg = static.append_backward(loss)
    exe = static.Executor()
    hv = np.random.RandomState(1).randn(4, 8).astype('float32')
    got = exe.run(main, feed={'n': np.array([3]), 'h0': hv}, fetch_list=[loss] + [g for _, g in pg])
    paddle.disable_static()
    h = paddle.to_tensor(hv)
    for _ in range(3):
        h = paddle.tanh(lin(h))
    ref = paddle.mean(h * h)
    ref.backward()
    paddle.enable_static()
    np.testing.assert_allclose(got[0], ref.numpy(), rtol=1e-5)
    by_name = {p.name: g for (p, _), g in zip(pg, got[1:])}
    np.testing.assert_allclose(by_name[lin.weight.name], lin.weight.grad.numpy(), rtol=1e-4,
                               atol=1e-6)


def test_cond_runs_only_the_taken_branch(static_mode):
    main = static.Program()
    with static.program_guard(main):
        p = static.data('p', [1], 'bool')
        x = static.data('x', [3], 'float32')
        x.stop_gradient = False
        y = static.nn.cond(p, lambda: paddle.exp(x), lambda: x * -3.0)
        gx, = static.gradients([paddle.sum(y)], [x])
    assert [op.type for op in main.global_block().ops].count('conditional_block') == 1
    exe = static.Executor()
    xv = np.array([0.5, -1.0, 2.0], 'float32')
    yt, gt = exe.run(main, feed={'p': np.array([True]), 'x': xv}, fetch_list=[y, gx])
    yf, gf = exe.run(main, feed={'p': np.array([False]), 'x': xv}, fetch_list=[y, gx])
    np.testing.assert_allclose(yt, np.exp(xv), rtol=1e-6)
    np.testing.assert_allclose(gt, np.exp(xv), rtol=1e-6)
    np.testing.assert_allclose(yf, xv * -3.0, rtol=1e-6)
    np.testing.assert_allclose(gf, np.full(3, -3.0), rtol=1e-6)


def test_switch_case_runtime(static_mode):
    main = static.Program()
    with static.program_guard(main):
        k = static.data('k', [1], 'int64')
        x = static.data('x', [2], 'float32')
        y = static.nn.switch_case(k, {0: lambda: x + 1.0, 1: lambda: x * 10.0,
                                      2: lambda: x - 5.0})
    exe = static.Executor()
    xv = np.array([1.0, 2.0], 'float32')
    for k, want in ((0, xv + 1), (1, xv * 10), (2, xv - 5)):
        out, = exe.run(main, feed={'k': np.array([k]), 'x': xv}, fetch_list=[y])
        np.testing.assert_allclose(out, want)


def test_static_rnn_matches_unrolled(static_mode):
    paddle.seed(5)
    main = static.Program()
    T, B, D, Hd = 5, 3, 4, 6
    with static.program_guard(main):
        x = static.data('x', [T, B, D], 'float32')
        h0 = static.data('h0', [B, Hd], 'float32')
        lx = paddle.nn.Linear(D, Hd)
        lh = paddle.nn.Linear(Hd, Hd)
        rnn = static.nn.StaticRNN()
        with rnn.step():
            xt = rnn.step_input(x)
            h = rnn.memory(init=h0)
            hn = paddle.tanh(lx(xt) + lh(h))
            rnn.update_memory(h, hn)
            rnn.step_output(hn)
        out = rnn()
        loss = paddle.mean(out)
        pg = static.append_backward(loss)
    exe = static.Executor()
    rs = np.random.RandomState(0)
    xv, hv = rs.randn(T, B, D).astype('float32'), rs.randn(B, Hd).astype('float32')
    got = exe.run(main, feed={'x': xv, 'h0': hv}, fetch_list=[out, loss] + [g for _, g in pg])
    paddle.disable_static()
    h = paddle.to_tensor(hv)
    outs = []
    for t in range(T):
        h = paddle.tanh(lx(paddle.to_tensor(xv[t])) + lh(h))
        outs.append(h)
    ref = paddle.stack(outs)
    paddle.mean(ref).backward()
    paddle.enable_static()
    np.testing.assert_allclose(got[0], ref.numpy(), rtol=1e-5, atol=1e-6)
    by_name = {p.name: g for (p, _), g in zip(pg, got[2:])}
    np.testing.assert_allclose(by_name[lh.weight.name], lh.weight.grad.numpy(), rtol=1e-4,
                               atol=1e-6)


def test_data_norm_uses_accumulated_stats():
    from paddle_ray_amd.static.nn import _DataNorm
    dn = _DataNorm(3, 1e-5, None, -1, 0.5, False)
    x = np.random.RandomState(0).randn(4, 3).astype('float32')
    y = dn(paddle.to_tensor(x)).numpy()
    np.testing.assert_allclose(y, x, rtol=1e-6)   # init: mean 0, scale sqrt(1e4/1e4)
    bs = 1e4 * 0.5 + 4
    su = x.sum(0)
    sq = 1e4 * 0.5 + (x ** 2).sum(0) + 4 * 1e-5
    np.testing.assert_allclose(dn.batch_size.numpy(), bs, rtol=1e-6)
    np.testing.assert_allclose(dn.batch_sum.numpy(), su, rtol=1e-5)
    np.testing.assert_allclose(dn.batch_square_sum.numpy(), sq, rtol=1e-6)
    dn.eval()
    y2 = dn(paddle.to_tensor(x)).numpy()
    np.testing.assert_allclose(y2, (x - su / bs) * np.sqrt(bs / sq), rtol=1e-5)


def test_nce_formula_with_deterministic_sampler():
    from paddle_ray_amd.static.nn import _NCE
    C, D, k = 6, 4, 3
    dist = [0.0, 0.0, 0.0, 1.0, 0.0, 0.0]         # every negative sample is class 3
    layer = _NCE(D, C, k, 'custom_dist', dist, 1, None, None)
    rs = np.random.RandomState(2)
    x = rs.randn(5, D).astype('float32')
    lab = np.array([[0], [1], [2], [4], [5]])
    cost = layer(paddle.to_tensor(x), paddle.to_tensor(lab)).numpy()
    W, b = layer.weight.numpy(), layer.bias.numpy()[:, 0]
    sig = lambda z: 1 / (1 + np.exp(-z))  # noqa
    for i in range(5):
        o_t = sig(x[i] @ W[lab[i, 0]] + b[lab[i, 0]])
        bt = k * dist[lab[i, 0]]
        o_n = sig(x[i] @ W[3] + b[3])
        bn = k * 1.0
        want = -np.log(o_t / (o_t + bt)) - k * np.log(bn / (o_n + bn))
        np.testing.assert_allclose(cost[i, 0], want, rtol=1e-5)


def test_row_conv_lookahead():
    from paddle_ray_amd.static.nn import _RowConv
    rc = _RowConv(3, 2, None)
    x = np.random.RandomState(4).randn(2, 5, 3).astype('float32')
    W = rc.weight.numpy()
    got = rc(paddle.to_tensor(x)).numpy()
    want = np.zeros_like(x)
    for t in range(5):
        for i in range(3):
            if t + i < 5:
                want[:, t] += x[:, t + i] * W[i]
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-6)
