"""paddle.metric (parity: python/paddle/metric/metrics.py)."""
import numpy as np
import torch

from ..framework.core import Tensor, _u


def _np(x):
    return x.numpy() if isinstance(x, Tensor) else np.asarray(x)


class Metric:
    def __init__(self):
        pass

    def reset(self):
        raise NotImplementedError

    def update(self, *args):
        raise NotImplementedError

    def accumulate(self):
        raise NotImplementedError

    def name(self):
        return self._name

    def compute(self, *args):
        return args


class Accuracy(Metric):
    def __init__(self, topk=(1,), name=None, *args, **kwargs):
        super().__init__()
        self.topk = topk
        self.maxk = max(topk)
        self._init_name(name)
        self.reset()

    def _init_name(self, name):
        name = name or 'acc'
        self._name = [f'{name}_top{k}' for k in self.topk] if self.maxk != 1 else [name]

    def compute(self, pred, label, *args):
        p, l = _u(pred), _u(label)
        idx = torch.topk(p, self.maxk, -1).indices
        if l.dim() == p.dim() and l.shape[-1] != 1:
            l = l.argmax(-1, keepdim=True)
        elif l.dim() < p.dim():
            l = l.unsqueeze(-1)
        return Tensor((idx == l).float())

    def update(self, correct, *args):
        c = _np(correct)
        accs = []
        for i, k in enumerate(self.topk):
            nc = c[..., :k].sum()
            n = int(np.prod(c.shape[:-1]))
            accs.append(float(nc) / n if n else 0.0)
            self.total[i] += nc
            self.count[i] += n
        return accs[0] if len(self.topk) == 1 else accs

    def reset(self):
        self.total = [0.] * len(self.topk)
        self.count = [0] * len(self.topk)

    def accumulate(self):
        res = [float(t) / c if c else 0.0 for t, c in zip(self.total, self.count)]
        return res[0] if len(self.topk) == 1 else res


class Precision(Metric):
    def __init__(self, name='precision', *args, **kwargs):
        super().__init__()
        self._name = name
        self.reset()

    def update(self, preds, labels):
        p = np.rint(_np(preds)).astype('int32').reshape(-1)
        l = _np(labels).astype('int32').reshape(-1)
        self.tp += int(((p == 1) & (l == 1)).sum())
        self.fp += int(((p == 1) & (l != 1)).sum())

    def reset(self):
        self.tp = self.fp = 0

    def accumulate(self):
        ap = self.tp + self.fp
        return float(self.tp) / ap if ap else 0.0


class Recall(Metric):
    def __init__(self, name='recall', *args, **kwargs):
        super().__init__()
        self._name = name
        self.reset()

    def update(self, preds, labels):
        p = np.rint(_np(preds)).astype('int32').reshape(-1)
        l = _np(labels).astype('int32').reshape(-1)
        self.tp += int(((p == 1) & (l == 1)).sum())
        self.fn += int(((p != 1) & (l == 1)).sum())

    def reset(self):
        self.tp = self.fn = 0

    def accumulate(self):
        r = self.tp + self.fn
        return float(self.tp) / r if r else 0.0


class Auc(Metric):
    def __init__(self, curve='ROC', num_thresholds=4095, name='auc', *args, **kwargs):
        super().__init__()
        self._name, self._num_thresholds, self._curve = name, num_thresholds, curve
        self.reset()

    def update(self, preds, labels):
        p = _np(preds)
        l = _np(labels).reshape(-1)
        pos = p[:, 1] if p.ndim == 2 else p.reshape(-1)
        idx = np.clip((pos * self._num_thresholds).astype(int), 0, self._num_thresholds)
        for i, lab in zip(idx, l):
            if lab:
                self._stat_pos[i] += 1
            else:
                self._stat_neg[i] += 1

    def reset(self):
        self._stat_pos = np.zeros(self._num_thresholds + 1)
        self._stat_neg = np.zeros(self._num_thresholds + 1)

    def accumulate(self):
        tot_pos = tot_neg = auc = 0.0
        for i in range(self._num_thresholds, -1, -1):
            np_, nn_ = self._stat_pos[i], self._stat_neg[i]
            auc += nn_ * (tot_pos + tot_pos + np_) / 2.0
            tot_pos += np_
            tot_neg += nn_
        return auc / (tot_pos * tot_neg) if tot_pos > 0 and tot_neg > 0 else 0.0


def accuracy(input, label, k=1, correct=None, total=None, name=None):
    p, l = _u(input), _u(label)
    idx = torch.topk(p, k, -1).indices
    if l.dim() == 1:
        l = l.unsqueeze(-1)
    acc = (idx == l).any(-1).float().mean()
    return Tensor(acc)
