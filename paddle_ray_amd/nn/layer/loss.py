"""Loss layers (parity: python/paddle/nn/layer/loss.py)."""
from .. import functional as F
from .layers import Layer


class CrossEntropyLoss(Layer):
    def __init__(self, weight=None, ignore_index=-100, reduction='mean', soft_label=False, axis=-1,
                 use_softmax=True, label_smoothing=0.0, name=None):
        super().__init__()
        self.weight, self.ignore_index, self.reduction = weight, ignore_index, reduction
        self.soft_label, self.axis, self.use_softmax = soft_label, axis, use_softmax
        self.label_smoothing = label_smoothing

    def forward(self, input, label):
        return F.cross_entropy(input, label, self.weight, self.ignore_index, self.reduction,
                               self.soft_label, self.axis, self.use_softmax, self.label_smoothing)


def _simple(name, fn, *argnames, **defaults):
    def __init__(self, *args, name=None, **kwargs):
        Layer.__init__(self)
        p = dict(defaults)
        for k, a in zip(list(defaults), args):
            p[k] = a
        p.update({k: v for k, v in kwargs.items() if k in defaults})
        self._p = p

    def forward(self, *inputs):
        return fn(*inputs, **self._p)

    return type(name, (Layer,), {'__init__': __init__, 'forward': forward})


MSELoss = _simple('MSELoss', F.mse_loss, reduction='mean')
L1Loss = _simple('L1Loss', F.l1_loss, reduction='mean')
SmoothL1Loss = _simple('SmoothL1Loss', F.smooth_l1_loss, reduction='mean', delta=1.0)
BCELoss = _simple('BCELoss', F.binary_cross_entropy, weight=None, reduction='mean')
KLDivLoss = _simple('KLDivLoss', F.kl_div, reduction='mean')
MarginRankingLoss = _simple('MarginRankingLoss', F.margin_ranking_loss, margin=0.0, reduction='mean')
HingeEmbeddingLoss = _simple('HingeEmbeddingLoss', F.hinge_embedding_loss, margin=1.0,
                             reduction='mean')
CosineEmbeddingLoss = _simple('CosineEmbeddingLoss', F.cosine_embedding_loss, margin=0,
                              reduction='mean')
SoftMarginLoss = _simple('SoftMarginLoss', F.soft_margin_loss, reduction='mean')
MultiLabelSoftMarginLoss = _simple('MultiLabelSoftMarginLoss', F.multi_label_soft_margin_loss,
                                   weight=None, reduction='mean')
MultiMarginLoss = _simple('MultiMarginLoss', F.multi_margin_loss, p=1, margin=1.0, weight=None,
                          reduction='mean')
TripletMarginLoss = _simple('TripletMarginLoss', F.triplet_margin_loss, margin=1.0, p=2,
                            epsilon=1e-6, swap=False, reduction='mean')
TripletMarginWithDistanceLoss = _simple('TripletMarginWithDistanceLoss',
                                        F.triplet_margin_with_distance_loss, distance_function=None,
                                        margin=1.0, swap=False, reduction='mean')
CTCLoss = _simple('CTCLoss', F.ctc_loss, blank=0, reduction='mean')


class BCEWithLogitsLoss(Layer):
    def __init__(self, weight=None, reduction='mean', pos_weight=None, name=None):
        super().__init__()
        self.weight, self.reduction, self.pos_weight = weight, reduction, pos_weight

    def forward(self, logit, label):
        return F.binary_cross_entropy_with_logits(logit, label, self.weight, self.reduction,
                                                  self.pos_weight)


class NLLLoss(Layer):
    def __init__(self, weight=None, ignore_index=-100, reduction='mean', name=None):
        super().__init__()
        self.weight, self.ignore_index, self.reduction = weight, ignore_index, reduction

    def forward(self, input, label):
        return F.nll_loss(input, label, self.weight, self.ignore_index, self.reduction)


class RNNTLoss(Layer):
    """parity: python/paddle/nn/layer/loss.py RNNTLoss."""

    def __init__(self, blank=0, fastemit_lambda=0.001, reduction='mean', name=None):
        super().__init__()
        self.blank, self.fastemit_lambda, self.reduction = blank, fastemit_lambda, reduction

    def forward(self, input, label, input_lengths, label_lengths):
        return F.rnnt_loss(input, label, input_lengths, label_lengths, blank=self.blank,
                           fastemit_lambda=self.fastemit_lambda, reduction=self.reduction)


class HSigmoidLoss(Layer):
    """parity: python/paddle/nn/layer/loss.py HSigmoidLoss — weight [C, feature_size],
    bias [C, 1] with C = num_classes - 1 (default tree) or num_classes (custom tree)."""

    def __init__(self, feature_size, num_classes, weight_attr=None, bias_attr=None,
                 is_custom=False, is_sparse=False, name=None):
        super().__init__()
        if num_classes < 2 and not is_custom:
            raise ValueError("num_classes must not be less than 2 with default tree")
        self._num_classes, self._is_custom, self._is_sparse = num_classes, is_custom, is_sparse
        C = num_classes if is_custom else num_classes - 1
        self.weight = self.create_parameter([C, feature_size], attr=weight_attr)
        self.bias = None if bias_attr is False else \
            self.create_parameter([C, 1], attr=bias_attr, is_bias=True)

    def forward(self, input, label, path_table=None, path_code=None):
        return F.hsigmoid_loss(input, label, self._num_classes, self.weight, self.bias,
                               path_table=path_table, path_code=path_code,
                               is_sparse=self._is_sparse)
