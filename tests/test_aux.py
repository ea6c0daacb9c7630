"""Aux subsystems: NaN/Inf checker, flags (parity: test/legacy_test/test_nan_inf.py)."""
import numpy as np
import pytest

import paddle_ray_amd as paddle


def test_check_nan_inf_flag_raises_with_op_name():
    paddle.set_flags({'FLAGS_check_nan_inf': True})
    try:
        x = paddle.to_tensor([1.0, 0.0])
        with pytest.raises(RuntimeError, match='log'):
            paddle.log(x - 1.0)
        # finite math is unaffected
        assert float(paddle.exp(x).sum()) > 0
    finally:
        paddle.set_flags({'FLAGS_check_nan_inf': False})
    # disabled: produces NaN silently
    assert np.isnan(paddle.log(paddle.to_tensor([-1.0])).numpy()).all()


def test_check_nan_inf_backward():
    paddle.set_flags({'FLAGS_check_nan_inf': True})
    try:
        x = paddle.to_tensor([0.0, 1.0], stop_gradient=False)
        y = paddle.sqrt(x).sum()
        with pytest.raises(RuntimeError, match='check_nan_inf'):
            y.backward()  # d sqrt(x)/dx at 0 = inf
    finally:
        paddle.set_flags({'FLAGS_check_nan_inf': False})


def test_tensor_checker_log_level():
    from paddle_ray_amd.amp import debugging
    cfg = debugging.TensorCheckerConfig(True, debugging.DebugMode.CHECK_NAN_INF)
    debugging.enable_tensor_checker(cfg)
    try:
        paddle.log(paddle.to_tensor([-1.0]))  # logs, does not raise
    finally:
        debugging.disable_tensor_checker()
    assert debugging.check_numerics(paddle.to_tensor([np.inf]),
                                    debug_mode=debugging.DebugMode.CHECK_NAN_INF) == (0, 1)


def test_flags_roundtrip():
    paddle.set_flags({'FLAGS_cudnn_deterministic': True})
    assert paddle.get_flags('FLAGS_cudnn_deterministic')['FLAGS_cudnn_deterministic']
    paddle.set_flags({'FLAGS_cudnn_deterministic': False})
