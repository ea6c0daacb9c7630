"""paddle.vision.models (parity: python/paddle/vision/models/__init__.py)."""
from .lenet import LeNet  # noqa
from .resnet import (ResNet, resnet18, resnet34, resnet50, resnet101, resnet152,  # noqa
                     resnext50_32x4d, resnext50_64x4d, resnext101_32x4d, resnext101_64x4d,
                     resnext152_32x4d, resnext152_64x4d, wide_resnet50_2, wide_resnet101_2)
from .vgg import VGG, vgg11, vgg13, vgg16, vgg19  # noqa
from .mobilenet import MobileNetV1, MobileNetV2, mobilenet_v1, mobilenet_v2  # noqa
from .alexnet import AlexNet, alexnet  # noqa
