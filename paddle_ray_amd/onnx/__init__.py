"""paddle.onnx.export (parity: python/paddle/onnx/export.py). Exports through
``torch.onnx`` when the ``onnx`` package is importable; otherwise raises (no install
possible here). The framework's own portable format is ``paddle.jit.save``."""


def export(layer, path, input_spec=None, opset_version=9, **configs):
    try:
        import onnx  # noqa: F401
    except ImportError as e:
        raise RuntimeError("paddle.onnx.export needs the 'onnx' package; use paddle.jit.save "
                           "for the native .pdmodel/.pdiparams format") from e
    import torch
    from ..framework.core import Tensor, _u
    from ..static.input import InputSpec
    args = []
    for s in input_spec or []:
        if isinstance(s, InputSpec):
            shp = [1 if d is None or d < 0 else d for d in s.shape]
            args.append(torch.zeros(shp, dtype=s.dtype))
        else:
            args.append(_u(s))

    class _Wrap(torch.nn.Module):
        def forward(self, *a):
            out = layer(*[Tensor(t) for t in a])
            return _u(out) if isinstance(out, Tensor) else tuple(_u(o) for o in out)
    torch.onnx.export(_Wrap(), tuple(args), path + '.onnx', opset_version=opset_version)
