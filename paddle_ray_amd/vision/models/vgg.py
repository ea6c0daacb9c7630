"""VGG (parity: python/paddle/vision/models/vgg.py)."""
from ... import nn

_CFG = {'A': [64, 'M', 128, 'M', 256, 256, 'M', 512, 512, 'M', 512, 512, 'M'],
        'B': [64, 64, 'M', 128, 128, 'M', 256, 256, 'M', 512, 512, 'M', 512, 512, 'M'],
        'D': [64, 64, 'M', 128, 128, 'M', 256, 256, 256, 'M', 512, 512, 512, 'M', 512, 512, 512, 'M'],
        'E': [64, 64, 'M', 128, 128, 'M', 256, 256, 256, 256, 'M', 512, 512, 512, 512, 'M', 512, 512,
              512, 512, 'M']}


def make_layers(cfg, batch_norm=False):
    layers, c = [], 3
    for v in cfg:
        if v == 'M':
            layers.append(nn.MaxPool2D(2, 2))
        else:
            layers.append(nn.Conv2D(c, v, 3, padding=1))
            if batch_norm:
                layers.append(nn.BatchNorm2D(v))
            layers.append(nn.ReLU())
            c = v
    return nn.Sequential(*layers)


class VGG(nn.Layer):
    def __init__(self, features, num_classes=1000, with_pool=True):
        super().__init__()
        self.features = features
        self.num_classes, self.with_pool = num_classes, with_pool
        if with_pool:
            self.avgpool = nn.AdaptiveAvgPool2D((7, 7))
        if num_classes > 0:
            self.classifier = nn.Sequential(nn.Linear(512 * 7 * 7, 4096), nn.ReLU(), nn.Dropout(),
                                            nn.Linear(4096, 4096), nn.ReLU(), nn.Dropout(),
                                            nn.Linear(4096, num_classes))

    def forward(self, x):
        x = self.features(x)
        if self.with_pool:
            x = self.avgpool(x)
        if self.num_classes > 0:
            x = self.classifier(x.flatten(1))
        return x


def _vgg(cfg, batch_norm, **kw):
    return VGG(make_layers(_CFG[cfg], batch_norm), **kw)


def vgg11(pretrained=False, batch_norm=False, **kw):
    return _vgg('A', batch_norm, **kw)


def vgg13(pretrained=False, batch_norm=False, **kw):
    return _vgg('B', batch_norm, **kw)


def vgg16(pretrained=False, batch_norm=False, **kw):
    return _vgg('D', batch_norm, **kw)


def vgg19(pretrained=False, batch_norm=False, **kw):
    return _vgg('E', batch_norm, **kw)
