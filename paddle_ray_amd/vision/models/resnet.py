"""ResNet family (parity: python/paddle/vision/models/resnet.py).

``data_format='NHWC'`` keeps activations channels-last end to end, the layout
MIOpen's fast bf16 conv kernels want on MI355X (no NCHW<->NHWC transposes).
"""
from ... import nn
from ...nn import functional as F
from ...ops.fused import grad_join as _grad_join


def _bn_act(bn, x, z=None, act='relu'):
    """act(bn(x) + z) through the fused BN(+add)(+ReLU) op (one read of x, one write of y on
    the gfx950 channels-last path; parity: fused_bn_add_activation_op)."""
    if isinstance(bn, nn.SyncBatchNorm) or not isinstance(bn, nn.layer.norm._BatchNormBase):
        out = bn(x)
        if z is not None:
            out = out + z
        return F.relu(out) if act == 'relu' else out
    return F.fused_bn_add_act(x, z, bn._mean, bn._variance, bn.weight, bn.bias,
                              bn.training and not bn._use_global_stats, bn._momentum, bn._epsilon,
                              act, bn._data_format)


def _conv_bn_act(conv, bn, x, z=None, act='relu'):
    """act(bn(conv(x)) + z); for a channels-last KxK convolution in training mode the BatchNorm
    statistics come from the convolution's epilogue (ops.fused.conv_bn_act_nhwc), so the
    separate statistics pass over the conv output is skipped."""
    import torch
    from ...framework.core import Tensor, _u
    from ...ops import fused as K
    xt = _u(x)
    st, pd, dl = conv._stride, conv._padding, conv._dilation
    st = st if isinstance(st, int) else (st[0] if len(set(st)) == 1 else None)
    pd = pd if isinstance(pd, int) else (pd[0] if not isinstance(pd, str) and len(set(pd)) == 1 else None)
    dl = dl if isinstance(dl, int) else (dl[0] if len(set(dl)) == 1 else None)
    if (conv._data_format == 'NHWC' and conv._groups == 1 and conv.bias is None and dl == 1
            and st is not None and pd is not None and isinstance(bn, nn.layer.norm._BatchNormBase)
            and not isinstance(bn, nn.SyncBatchNorm) and bn.training and not bn._use_global_stats
            and xt.is_cuda and xt.dtype == _u(conv.weight).dtype and xt.dtype in (torch.bfloat16, torch.float16)
            and act in ('relu', None)):
        y = K.conv_bn_act_nhwc(xt, _u(conv.weight), st, pd, _u(bn.weight), _u(bn.bias), _u(bn._mean),
                               _u(bn._variance), True, bn._momentum, bn._epsilon,
                               _u(z) if z is not None else None, act == 'relu')
        return Tensor(y)
    return _bn_act(bn, conv(x), z, act)


class BasicBlock(nn.Layer):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64,
                 dilation=1, norm_layer=None, data_format='NCHW'):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2D
        df = data_format
        self.conv1 = nn.Conv2D(inplanes, planes, 3, padding=1, stride=stride, bias_attr=False,
                               data_format=df)
        self.bn1 = norm_layer(planes, data_format=df)
        self.relu = nn.ReLU()
        self.conv2 = nn.Conv2D(planes, planes, 3, padding=1, bias_attr=False, data_format=df)
        self.bn2 = norm_layer(planes, data_format=df)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        out = _conv_bn_act(self.conv1, self.bn1, x)
        if self.downsample is not None:
            identity = self.downsample(x)
        return _conv_bn_act(self.conv2, self.bn2, out, identity)


class BottleneckBlock(nn.Layer):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64,
                 dilation=1, norm_layer=None, data_format='NCHW'):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2D
        df = data_format
        width = int(planes * (base_width / 64.)) * groups
        self.conv1 = nn.Conv2D(inplanes, width, 1, bias_attr=False, data_format=df)
        self.bn1 = norm_layer(width, data_format=df)
        self.conv2 = nn.Conv2D(width, width, 3, padding=dilation, stride=stride, groups=groups,
                               dilation=dilation, bias_attr=False, data_format=df)
        self.bn2 = norm_layer(width, data_format=df)
        self.conv3 = nn.Conv2D(width, planes * self.expansion, 1, bias_attr=False, data_format=df)
        self.bn3 = norm_layer(planes * self.expansion, data_format=df)
        self.relu = nn.ReLU()
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        # the block input's gradient is joined in-kernel across its consumers (conv1, the
        # downsample conv or the residual add) instead of summed by separate add kernels
        with _grad_join(x._t):
            identity = x
            # every conv + BN pair takes its BN statistics from the conv epilogue (1x1 and 3x3)
            out = _conv_bn_act(self.conv1, self.bn1, x)
            out = _conv_bn_act(self.conv2, self.bn2, out)
            if self.downsample is not None:
                ds = self.downsample
                if len(ds) == 2 and isinstance(ds[0], nn.Conv2D):
                    identity = _conv_bn_act(ds[0], ds[1], x, act=None)
                else:
                    identity = ds(x)
            return _conv_bn_act(self.conv3, self.bn3, out, identity)


class ResNet(nn.Layer):
    def __init__(self, block, depth=50, width=64, num_classes=1000, with_pool=True, groups=1,
                 data_format='NCHW'):
        super().__init__()
        layer_cfg = {18: [2, 2, 2, 2], 34: [3, 4, 6, 3], 50: [3, 4, 6, 3], 101: [3, 4, 23, 3],
                     152: [3, 8, 36, 3]}
        layers = layer_cfg[depth]
        self.groups, self.base_width = groups, width
        self.num_classes, self.with_pool = num_classes, with_pool
        self._norm_layer = nn.BatchNorm2D
        self.data_format = df = data_format
        self.inplanes, self.dilation = 64, 1
        self.conv1 = nn.Conv2D(3, self.inplanes, 7, stride=2, padding=3, bias_attr=False,
                               data_format=df)
        self.bn1 = self._norm_layer(self.inplanes, data_format=df)
        self.relu = nn.ReLU()
        self.maxpool = nn.MaxPool2D(3, stride=2, padding=1, data_format=df)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        if with_pool:
            self.avgpool = nn.AdaptiveAvgPool2D((1, 1), data_format=df)
        if num_classes > 0:
            self.fc = nn.Linear(512 * block.expansion, num_classes)

    def _make_layer(self, block, planes, blocks, stride=1, dilate=False):
        df = self.data_format
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                nn.Conv2D(self.inplanes, planes * block.expansion, 1, stride=stride,
                          bias_attr=False, data_format=df),
                self._norm_layer(planes * block.expansion, data_format=df))
        layers = [block(self.inplanes, planes, stride, downsample, self.groups, self.base_width,
                        1, self._norm_layer, df)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, groups=self.groups,
                                base_width=self.base_width, norm_layer=self._norm_layer,
                                data_format=df))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(_conv_bn_act(self.conv1, self.bn1, x))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        if self.with_pool:
            x = self.avgpool(x)
        if self.num_classes > 0:
            x = x.flatten(1)
            x = self.fc(x)
        return x


def _resnet(block, depth, pretrained=False, **kw):
    if pretrained:
        raise ValueError("pretrained weights are not downloadable in this environment")
    return ResNet(block, depth, **kw)


def resnet18(pretrained=False, **kw):
    return _resnet(BasicBlock, 18, pretrained, **kw)


def resnet34(pretrained=False, **kw):
    return _resnet(BasicBlock, 34, pretrained, **kw)


def resnet50(pretrained=False, **kw):
    return _resnet(BottleneckBlock, 50, pretrained, **kw)


def resnet101(pretrained=False, **kw):
    return _resnet(BottleneckBlock, 101, pretrained, **kw)


def resnet152(pretrained=False, **kw):
    return _resnet(BottleneckBlock, 152, pretrained, **kw)


def resnext50_32x4d(pretrained=False, **kw):
    return _resnet(BottleneckBlock, 50, pretrained, groups=32, width=4, **kw)


def resnext50_64x4d(pretrained=False, **kw):
    return _resnet(BottleneckBlock, 50, pretrained, groups=64, width=4, **kw)


def resnext101_32x4d(pretrained=False, **kw):
    return _resnet(BottleneckBlock, 101, pretrained, groups=32, width=4, **kw)


def resnext101_64x4d(pretrained=False, **kw):
    return _resnet(BottleneckBlock, 101, pretrained, groups=64, width=4, **kw)


def resnext152_32x4d(pretrained=False, **kw):
    return _resnet(BottleneckBlock, 152, pretrained, groups=32, width=4, **kw)


def resnext152_64x4d(pretrained=False, **kw):
    return _resnet(BottleneckBlock, 152, pretrained, groups=64, width=4, **kw)


def wide_resnet50_2(pretrained=False, **kw):
    return _resnet(BottleneckBlock, 50, pretrained, width=128, **kw)


def wide_resnet101_2(pretrained=False, **kw):
    return _resnet(BottleneckBlock, 101, pretrained, width=128, **kw)
