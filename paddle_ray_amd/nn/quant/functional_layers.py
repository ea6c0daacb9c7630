"""Layer wrappers of functional ops so that quantization passes can attach observers to
them (parity: python/paddle/nn/quant/functional_layers.py)."""
from ..layer.layers import Layer


class FloatFunctionalLayer(Layer):
    def __init__(self):
        super().__init__()


def _make(name, fn_name, doc):
    def forward(self, *args, **kwargs):
        import paddle_ray_amd as paddle
        fn = getattr(paddle, fn_name)
        return fn(*args, **kwargs)
    return type(name, (FloatFunctionalLayer,), {'forward': forward, '__doc__': doc})


add = _make('add', 'add', 'x + y as a layer')
subtract = _make('subtract', 'subtract', 'x - y as a layer')
multiply = _make('multiply', 'multiply', 'x * y as a layer')
divide = _make('divide', 'divide', 'x / y as a layer')
reshape = _make('reshape', 'reshape', 'reshape as a layer')
transpose = _make('transpose', 'transpose', 'transpose as a layer')
concat = _make('concat', 'concat', 'concat as a layer')
flatten = _make('flatten', 'flatten', 'flatten as a layer')
matmul = _make('matmul', 'matmul', 'matmul as a layer')
