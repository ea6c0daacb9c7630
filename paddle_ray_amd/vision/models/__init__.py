"""paddle.vision.models (parity: python/paddle/vision/models/__init__.py)."""
from .lenet import LeNet  # noqa
from .resnet import (ResNet, resnet18, resnet34, resnet50, resnet101, resnet152,  # noqa
                     resnext50_32x4d, resnext50_64x4d, resnext101_32x4d, resnext101_64x4d,
                     resnext152_32x4d, resnext152_64x4d, wide_resnet50_2, wide_resnet101_2)
from .vgg import VGG, vgg11, vgg13, vgg16, vgg19  # noqa
from .mobilenet import MobileNetV1, MobileNetV2, mobilenet_v1, mobilenet_v2  # noqa
from .alexnet import AlexNet, alexnet  # noqa
from .densenet import (DenseNet, densenet121, densenet161, densenet169, densenet201,  # noqa
                       densenet264)
from .googlenet import GoogLeNet, googlenet  # noqa
from .inceptionv3 import InceptionV3, inception_v3  # noqa
from .mobilenetv3 import (MobileNetV3Small, MobileNetV3Large, mobilenet_v3_small,  # noqa
                          mobilenet_v3_large)
from .shufflenetv2 import (ShuffleNetV2, shufflenet_v2_x0_25, shufflenet_v2_x0_33,  # noqa
                           shufflenet_v2_x0_5, shufflenet_v2_x1_0, shufflenet_v2_x1_5,
                           shufflenet_v2_x2_0, shufflenet_v2_swish)
from .squeezenet import SqueezeNet, squeezenet1_0, squeezenet1_1  # noqa
