"""Vision model zoo breadth (parity: test/legacy_test/test_vision_models.py): architecture
checked by exact parameter counts of the published models, plus forward shapes."""
import pytest

import paddle_ray_amd as paddle
from paddle_ray_amd.vision import models as Mz

COUNTS = [('densenet121', 7978856), ('densenet161', 28681000), ('inception_v3', 23834568),
          ('mobilenet_v3_large', 5483032), ('mobilenet_v3_small', 2542856),
          ('shufflenet_v2_x1_0', 2278604), ('squeezenet1_0', 1248424),
          ('squeezenet1_1', 1235496)]


@pytest.mark.parametrize('name,count', COUNTS)
def test_param_counts(name, count):
    m = getattr(Mz, name)()
    assert sum(int(p.numel()) for p in m.parameters()) == count


@pytest.mark.parametrize('name,size', [('densenet121', 64), ('inception_v3', 299),
                                       ('mobilenet_v3_small', 64), ('mobilenet_v3_large', 64),
                                       ('shufflenet_v2_x0_5', 64), ('shufflenet_v2_swish', 64),
                                       ('squeezenet1_1', 96)])
def test_forward_shapes(name, size):
    paddle.seed(0)
    m = getattr(Mz, name)(num_classes=7)
    m.eval()
    assert m(paddle.randn([2, 3, size, size])).shape == [2, 7]
    feat = getattr(Mz, name)(num_classes=0, with_pool=True)
    feat.eval()
    assert feat(paddle.randn([1, 3, size, size])).shape[0] == 1


def test_googlenet_aux_heads_and_train_step():
    paddle.seed(0)
    m = Mz.googlenet(num_classes=5)
    out, a1, a2 = m(paddle.randn([2, 3, 224, 224]))
    assert out.shape == a1.shape == a2.shape == [2, 5]
    loss = out.sum() + 0.3 * (a1.sum() + a2.sum())
    loss.backward()
    assert m.fc.weight.grad is not None and m.aux1.fc2.weight.grad is not None
