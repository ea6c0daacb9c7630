"""Auto-parallel tuner (distributed/auto_parallel/tuner.py): tunable spaces / trials with the
reference's interface (auto_parallel/tuner/tunable_space.py, tunable_variable.py, trial.py) and the
analytic MI355X strategy search."""
import pytest

from paddle_ray_amd.distributed.auto_parallel import tuner as T


def test_tunable_space_roundtrip():
    ts = T.TunableSpace()
    assert ts.choice('mp', [1, 2, 4], default=2) == 2
    assert ts.boolean('recompute') is False
    assert ts.int_range('mb', 1, 9, 2) == 1
    ts.fixed('seed', 7)
    ts.float_range('lr', 0.1, 1.0)
    assert ts.choice('mp', [8]) == 2               # first registration wins
    ts['mp'] = 4
    back = T.TunableSpace.from_state(ts.get_state())
    assert back.values == ts.values and set(back.variables) == {'mp', 'recompute', 'mb', 'seed', 'lr'}
    assert back.variables['mb'].values == [1, 3, 5, 7]
    with pytest.raises(KeyError):
        ts['nope']
    with pytest.raises(ValueError):
        T.Choice('x', [1, 2], default=3)


def test_gpt13b_on_one_node_prefers_data_parallel():
    gpt = T.ModelSpec(24, 2048, 16, 1024, 50304, global_batch=128)
    assert abs(gpt.params - 1.31e9) / 1.31e9 < 0.02
    tuner = T.ParallelTuner(gpt, T.ClusterSpec(n_gpus=8))
    best = tuner.best()
    v = best.space.values
    assert (v['dp_degree'], v['mp_degree'], v['pp_degree']) == (8, 1, 1)
    assert best.metrics['memory_gb'] < 288
    # every trial is either priced or carries the reason it was rejected
    assert all((t.status == T.TrialStatus.COMPLETED) == (t.reason is None) for t in tuner.trials)
    hc = best.strategy()['hybrid_configs']
    # the 8 data-parallel ranks: plain dp, or fleet's sharding group when the trial shards
    if v['sharding_stage'] > 0:
        assert (hc['dp_degree'], hc['sharding_degree']) == (1, 8)
        assert best.strategy()['sharding_configs'] == {'stage': v['sharding_stage']}
    else:
        assert (hc['dp_degree'], hc['sharding_degree']) == (8, 1)


def test_175b_needs_more_than_one_node():
    m = T.ModelSpec(96, 12288, 96, 2048, 50304, global_batch=256)
    with pytest.raises(RuntimeError):
        T.ParallelTuner(m, T.ClusterSpec(n_gpus=8)).best()
    best = T.ParallelTuner(m, T.ClusterSpec(n_gpus=64), micro_batch_sizes=(1, 2)).best()
    v = best.space.values
    assert v['mp_degree'] <= 8                      # tensor parallel stays inside a node
    assert v['mp_degree'] * v['pp_degree'] > 1 or v['sharding_stage'] >= 2
    assert best.metrics['memory_gb'] <= 288 * 0.9
