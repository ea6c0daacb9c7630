"""GoogLeNet / Inception-v1 (parity: python/paddle/vision/models/googlenet.py): returns
[main logits, aux logits from inception 4a, aux logits from inception 4d]."""
from ... import nn
from ...tensor import manipulation as M


def _conv(cin, cout, k, stride=1):
    return nn.Conv2D(cin, cout, k, stride, (k - 1) // 2, bias_attr=False)


class _Inception(nn.Layer):
    """Four parallel branches (1x1 | 1x1-3x3 | 1x1-5x5 | maxpool-1x1), concat, ReLU."""

    def __init__(self, cin, c1, c3r, c3, c5r, c5, proj):
        super().__init__()
        self.b1 = _conv(cin, c1, 1)
        self.b3 = nn.Sequential(_conv(cin, c3r, 1), _conv(c3r, c3, 3))
        self.b5 = nn.Sequential(_conv(cin, c5r, 1), _conv(c5r, c5, 5))
        self.bp = nn.Sequential(nn.MaxPool2D(3, 1, 1), _conv(cin, proj, 1))
        self.relu = nn.ReLU()
        self.out_channels = c1 + c3 + c5 + proj

    def forward(self, x):
        return self.relu(M.concat([self.b1(x), self.b3(x), self.b5(x), self.bp(x)], axis=1))


class _AuxHead(nn.Layer):
    def __init__(self, cin, num_classes, with_pool):
        super().__init__()
        self.with_pool = with_pool
        self.pool = nn.AvgPool2D(5, 3)
        self.conv = _conv(cin, 128, 1)
        self.fc1 = nn.Linear(1152, 1024)
        self.drop = nn.Dropout(0.7, mode='downscale_in_infer')
        self.fc2 = nn.Linear(1024, num_classes)
        self.relu = nn.ReLU()

    def forward(self, x):
        if self.with_pool:
            x = self.pool(x)
        x = self.relu(self.fc1(self.conv(x).flatten(1)))
        return self.fc2(self.drop(x))


class GoogLeNet(nn.Layer):
    def __init__(self, num_classes=1000, with_pool=True):
        super().__init__()
        self.num_classes, self.with_pool = num_classes, with_pool
        self.stem = nn.Sequential(_conv(3, 64, 7, 2), nn.MaxPool2D(3, 2), _conv(64, 64, 1),
                                  _conv(64, 192, 3), nn.MaxPool2D(3, 2))
        cfg3 = [(192, 64, 96, 128, 16, 32, 32), (256, 128, 128, 192, 32, 96, 64)]
        cfg4 = [(480, 192, 96, 208, 16, 48, 64), (512, 160, 112, 224, 24, 64, 64),
                (512, 128, 128, 256, 24, 64, 64), (512, 112, 144, 288, 32, 64, 64),
                (528, 256, 160, 320, 32, 128, 128)]
        cfg5 = [(832, 256, 160, 320, 32, 128, 128), (832, 384, 192, 384, 48, 128, 128)]
        self.inc3 = nn.Sequential(*[_Inception(*c) for c in cfg3])
        self.inc4 = nn.LayerList([_Inception(*c) for c in cfg4])
        self.inc5 = nn.Sequential(*[_Inception(*c) for c in cfg5])
        self.maxpool = nn.MaxPool2D(3, 2)
        if with_pool:
            self.pool = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.drop = nn.Dropout(0.4, mode='downscale_in_infer')
            self.fc = nn.Linear(1024, num_classes)
            self.aux1 = _AuxHead(512, num_classes, with_pool)
            self.aux2 = _AuxHead(528, num_classes, with_pool)

    def forward(self, x):
        x = self.maxpool(self.inc3(self.stem(x)))
        taps = []
        for i, blk in enumerate(self.inc4):
            x = blk(x)
            if i in (0, 3):
                taps.append(x)
        out = self.inc5(self.maxpool(x))
        o1, o2 = taps
        if self.with_pool:
            out = self.pool(out)
        if self.num_classes > 0:
            out = self.fc(self.drop(out).flatten(1))
            o1, o2 = self.aux1(o1), self.aux2(o2)
        elif self.with_pool:
            o1, o2 = nn.functional.avg_pool2d(o1, 5, 3), nn.functional.avg_pool2d(o2, 5, 3)
        return [out, o1, o2]


def googlenet(pretrained=False, **kwargs):
    if pretrained:
        raise ValueError("pretrained weights are not available offline")
    return GoogLeNet(**kwargs)
