"""fleet.metrics cross-rank reductions (reference: distributed/fleet/metrics/metric.py:26-378) and
the MultiSlot data generators (fleet/data_generator/data_generator.py)."""
import io
import sys

import numpy as np
import pytest

from dist_utils import run_ranks


def _metrics(rank, world):
    from paddle_ray_amd.distributed import fleet
    from paddle_ray_amd.distributed.fleet import metrics as M
    fleet.init(is_collective=True)
    a = np.array([[1.0 + rank, 2.0 * rank]], 'float32')
    # static.auc-style bucket stats: [1, num_buckets]
    pos = np.array([[0, 1, 2 + rank, 4]], 'int64')
    neg = np.array([[3 + rank, 2, 1, 0]], 'int64')
    return {'sum': M.sum(a), 'max': M.max(a), 'min': M.min(a), 'auc': M.auc(pos, neg),
            'mae': M.mae(np.array([1.5 * (rank + 1)]), np.array([10.0])),
            'mse': M.mse(np.array([4.0 * (rank + 1)]), np.array([10.0])),
            'rmse': M.rmse(np.array([4.0 * (rank + 1)]), np.array([10.0])),
            'acc': M.acc(np.array([7 + rank]), np.array([10])), 'a_after': a}


def _auc_ref(pos, neg):
    # brute force over (positive, negative) pairs: P(score_pos > score_neg) + 0.5 P(tie)
    num = den = 0.0
    for i, p in enumerate(pos):
        for j, n in enumerate(neg):
            w = p * n
            den += w
            num += w * (1.0 if i > j else 0.5 if i == j else 0.0)
    return num / den


def test_fleet_metrics_two_ranks(tmp_path):
    r = run_ranks(_metrics, 2, tmp_path)
    for k in ('sum', 'max', 'min', 'auc', 'mae', 'mse', 'rmse', 'acc'):
        np.testing.assert_allclose(r[0][k], r[1][k])
    np.testing.assert_allclose(r[0]['sum'], [[3.0, 2.0]])
    np.testing.assert_allclose(r[0]['max'], [[2.0, 2.0]])
    np.testing.assert_allclose(r[0]['min'], [[1.0, 0.0]])
    np.testing.assert_allclose(r[0]['a_after'], [[1.0, 0.0]])      # inputs are not reduced in place
    pos = np.array([0, 2, 5, 8], float)
    neg = np.array([7, 4, 2, 0], float)
    np.testing.assert_allclose(r[0]['auc'], _auc_ref(pos, neg), rtol=1e-9)
    np.testing.assert_allclose(r[0]['mae'], 4.5 / 20)
    np.testing.assert_allclose(r[0]['mse'], 12.0 / 20)
    np.testing.assert_allclose(r[0]['rmse'], np.sqrt(12.0 / 20))
    np.testing.assert_allclose(r[0]['acc'], 15 / 20)


def test_fleet_metrics_single_process_and_scope():
    from paddle_ray_amd.distributed.fleet import metrics as M
    from paddle_ray_amd import static
    sc = static.Scope()
    sc.vars['cnt'] = np.array([5.0], 'float32')
    np.testing.assert_allclose(M.sum('cnt', scope=sc), [5.0])
    with pytest.raises(ValueError):
        M.sum('missing', scope=sc)
    assert M.auc(np.array([[0, 0]]), np.array([[1, 1]])) == 0.5


def test_multislot_data_generators():
    from paddle_ray_amd.distributed import fleet

    class G(fleet.MultiSlotDataGenerator):
        def generate_sample(self, line):
            def it():
                ws = [int(x) for x in line.split()]
                yield [('words', ws), ('label', [ws[0] % 2])]
            return it

    g = G()
    g.set_batch(2)
    old = sys.stdout
    sys.stdout = buf = io.StringIO()
    try:
        g._run(['3 4 5', '7 8'])
    finally:
        sys.stdout = old
    assert buf.getvalue() == '3 3 4 5 1 1\n2 7 8 1 1\n'
    assert g._proto_info == [('words', 'uint64'), ('label', 'uint64')]
    assert g._gen_str([('words', [1.5]), ('label', [0])]) == '1 1.5 1 0\n'
    assert g._proto_info[0] == ('words', 'float')
    with pytest.raises(ValueError):
        g._gen_str([('other', [1]), ('label', [0])])
    with pytest.raises(ValueError):
        g._gen_str([('words', []), ('label', [0])])

    class S(fleet.MultiSlotStringDataGenerator):
        def generate_sample(self, line):
            def it():
                yield [('q', line.split()), ('y', ['1'])]
            return it
    assert S()._gen_str([('q', ['a1', 'b2']), ('y', ['0'])]) == '2 a1 b2 1 0\n'
    with pytest.raises(NotImplementedError):
        fleet.data_generator.DataGenerator()._gen_str([])
