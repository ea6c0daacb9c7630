"""Cross-rank metric reduction (parity: python/paddle/distributed/fleet/metrics/metric.py:26-378 --
sum / max / min / auc / mae / rmse / mse / acc over every worker).

Inputs are numpy arrays, or static Variables / variable names whose values live in a Scope (the
reference's persistable accumulator vars); the reduction is ``fleet.util.all_reduce`` (a host
all-reduce over the world's process group: gloo on CPU, RCCL through the device otherwise)."""
import math

import numpy as np

__all__ = ['sum', 'max', 'min', 'auc', 'mae', 'rmse', 'mse', 'acc']

_builtin_sum = sum


def _util(util):
    if util is None:
        from .. import util as u
        return u
    return util


def _value(x, scope):
    """A metric input as a numpy array."""
    from ....static.graph import Variable, global_scope
    if isinstance(x, (Variable, str)):
        name = x if isinstance(x, str) else x.name
        v = (scope or global_scope()).find_var(name)
        if v is None:
            raise ValueError(f"fleet.metrics: variable {name!r} not found in the scope")
        x = v
    if hasattr(x, 'numpy'):
        x = x.numpy()
    elif hasattr(x, 'get_tensor'):
        x = np.array(x.get_tensor())
    return np.asarray(x)


def _reduce(x, mode, scope, util):
    a = _value(x, scope)
    out = np.asarray(_util(util).all_reduce(np.array(a, copy=True), mode))
    return out.reshape(a.shape)


def sum(input, scope=None, util=None):  # noqa: A001
    """Element-wise sum of ``input`` over every worker."""
    return _reduce(input, 'sum', scope, util)


def max(input, scope=None, util=None):  # noqa: A001
    return _reduce(input, 'max', scope, util)


def min(input, scope=None, util=None):  # noqa: A001
    return _reduce(input, 'min', scope, util)


def auc(stat_pos, stat_neg, scope=None, util=None):
    """Global ROC AUC from the per-bucket positive / negative counts of ``static.auc`` (each
    [1, num_buckets]), summed over the workers; trapezoids swept from the highest bucket."""
    pos = _reduce(stat_pos, 'sum', scope, util).reshape(-1).astype(np.float64)
    neg = _reduce(stat_neg, 'sum', scope, util).reshape(-1).astype(np.float64)
    # cumulative counts from the top threshold down; area = sum of trapezoids in (fp, tp) space
    tp = np.concatenate([[0.0], np.cumsum(pos[::-1])])
    fp = np.concatenate([[0.0], np.cumsum(neg[::-1])])
    area = float(np.sum((fp[1:] - fp[:-1]) * (tp[1:] + tp[:-1]) / 2.0))
    P, N = tp[-1], fp[-1]
    if P * N == 0 or P + N == 0:
        return 0.5
    return area / (P * N)


def _count(total_ins_num, scope, util):
    return float(np.asarray(_reduce(total_ins_num, 'sum', scope, util)).reshape(-1)[0])


def mae(abserr, total_ins_num, scope=None, util=None):
    """Mean absolute error from the workers' summed |error| and instance counts."""
    e = float(np.asarray(_reduce(abserr, 'sum', scope, util)).reshape(-1)[0])
    n = _count(total_ins_num, scope, util)
    return e / n if n else 0.0


def mse(sqrerr, total_ins_num, scope=None, util=None):
    e = float(np.asarray(_reduce(sqrerr, 'sum', scope, util)).reshape(-1)[0])
    n = _count(total_ins_num, scope, util)
    return e / n if n else 0.0


def rmse(sqrerr, total_ins_num, scope=None, util=None):
    return math.sqrt(mse(sqrerr, total_ins_num, scope, util))


def acc(correct, total, scope=None, util=None):
    """Global accuracy = sum of correct / sum of totals over the workers."""
    c = float(np.asarray(_reduce(correct, 'sum', scope, util)).reshape(-1)[0])
    t = float(np.asarray(_reduce(total, 'sum', scope, util)).reshape(-1)[0])
    return c / t if t else 0.0
