"""paddle.profiler statistics and benchmark timer (reference: python/paddle/profiler/
profiler_statistic.py:857-875 views + SortedKeys, profiler/timer.py:51-222 reader cost,
profiler.py:838 summary, export_protobuf / load_profiler_result)."""
import os
import re
import time

import numpy as np
import pytest

import paddle_ray_amd as paddle
import paddle_ray_amd.profiler as profiler


def _rows(table, title):
    """Row names of one view of a summary string, in printed order."""
    lines = table.splitlines()
    start = next(i for i, l in enumerate(lines) if title in l)
    out, seps = [], 0
    for l in lines[start + 1:]:
        if l.startswith('---'):
            seps += 1
            if seps == 3:
                break
            continue
        if seps == 2 and l.strip():
            out.append(l.split('  ')[0].strip())
    return out


def _udf_profile():
    prof = profiler.Profiler(targets=[profiler.ProfilerTarget.CPU])
    prof.start()
    for _ in range(2):
        for _ in range(3):
            with profiler.RecordEvent('many_short'):
                time.sleep(0.002)
        with profiler.RecordEvent('one_long'):
            time.sleep(0.004)
        prof.step()
    prof.stop()
    return prof


def test_summary_sorted_by_changes_order_and_views_filter():
    prof = _udf_profile()
    tot = prof.summary(sorted_by=profiler.SortedKeys.CPUTotal, views=[profiler.SummaryView.UDFView])
    mx = prof.summary(sorted_by=profiler.SortedKeys.CPUMax, views=profiler.SummaryView.UDFView)
    assert _rows(tot, 'UserDefined Summary')[:2] == ['many_short', 'one_long']     # 12 ms vs 8 ms total
    assert _rows(mx, 'UserDefined Summary')[:2] == ['one_long', 'many_short']      # 4 ms vs 2 ms max
    assert 'Operator Summary' not in tot and 'Model Summary' not in tot
    full = prof.summary()
    for title in ('Device Summary', 'Overview Summary', 'Model Summary', 'UserDefined Summary'):
        assert title in full


def test_summary_time_unit():
    prof = _udf_profile()
    ms = prof.summary(views=[profiler.SummaryView.UDFView], time_unit='ms')
    us = prof.summary(views=[profiler.SummaryView.UDFView], time_unit='us')
    row = lambda s: next(l for l in s.splitlines() if l.startswith('one_long'))  # noqa: E731
    v_ms = float(row(ms).split()[2])
    v_us = float(row(us).split()[2])
    assert 7.5 < v_ms < 40 and abs(v_us / v_ms - 1000) < 1e-3 * 1000
    assert 'CPU Total(us)' in us
    with pytest.raises(ValueError):
        prof.summary(time_unit='minutes')


class _SlowDS(paddle.io.Dataset):
    def __getitem__(self, i):
        time.sleep(0.003)
        return np.full([4], i, 'float32'), np.array([i % 2], 'int64')

    def __len__(self):
        return 64


def test_model_view_and_reader_cost_with_dataloader():
    model = paddle.nn.Sequential(paddle.nn.Linear(4, 8), paddle.nn.ReLU(), paddle.nn.Linear(8, 2))
    opt = paddle.optimizer.Adam(1e-3, parameters=model.parameters())
    loader = paddle.io.DataLoader(_SlowDS(), batch_size=4)
    prof = profiler.Profiler(targets=[profiler.ProfilerTarget.CPU], scheduler=(1, 4))
    prof.start()
    infos = []
    for i, (x, y) in enumerate(loader):
        loss = paddle.nn.functional.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        opt.clear_grad()
        prof.step(num_samples=4)
        infos.append(prof.step_info(unit='samples'))
        if i == 5:
            break
    prof.stop()
    m = re.search(r'reader_cost: ([0-9.]+) s', infos[-1])
    assert m and float(m.group(1)) > 0.005, infos[-1]     # 4 samples x 3 ms
    assert 'ips:' in infos[-1] and 'samples/s' in infos[-1]
    res = prof.profiler_result
    assert [s for s, _, _ in res.steps] == [1, 2, 3]       # scheduler (1, 4): steps 1..3 recorded
    s = prof.summary(views=[profiler.SummaryView.ModelView, profiler.SummaryView.OperatorView])
    rows = _rows(s, 'Model Summary')
    for r in ('ProfileStep', 'Dataloader', 'Forward', 'Backward', 'Optimization', 'Others'):
        assert r in rows, (r, rows)
    ops = _rows(s, 'Operator Summary')
    assert any(o.startswith('aten::') for o in ops), ops


def test_export_protobuf_roundtrip_and_chrome(tmp_path):
    prof = profiler.Profiler(targets=[profiler.ProfilerTarget.CPU],
                             on_trace_ready=profiler.export_protobuf(str(tmp_path / 'pb')))
    prof.start()
    with profiler.RecordEvent('roundtrip'):
        paddle.matmul(paddle.randn([16, 16]), paddle.randn([16, 16]))
    prof.step()
    prof.stop()
    files = os.listdir(tmp_path / 'pb')
    assert len(files) == 1 and files[0].endswith('.pb')
    res = profiler.load_profiler_result(str(tmp_path / 'pb' / files[0]))
    assert isinstance(res, profiler.ProfilerResult)
    names = {e.name for e in res.host_events}
    assert 'roundtrip' in names and 'ProfileStep#0' in names
    orig = prof.profiler_result
    assert len(res.host_events) == len(orig.host_events)
    a = sorted((e.name, e.start_ns, e.end_ns, e.type) for e in orig.host_events)
    b = sorted((e.name, e.start_ns, e.end_ns, e.type) for e in res.host_events)
    assert a == b
    # genuine protobuf wire format: the first field is 'version' (field 1, length-delimited)
    raw = open(tmp_path / 'pb' / files[0], 'rb').read()
    assert raw[0] == (1 << 3 | 2)
    # the reloaded result summarises like the live one
    t = profiler.build_table(profiler.StatisticData(res), views=[profiler.SummaryView.UDFView])
    assert 'roundtrip' in t
    prof.export(str(tmp_path / 'trace.json'), 'json')
    tr = profiler.load_profiler_result(str(tmp_path / 'trace.json'))
    assert any(e['name'] == 'roundtrip' for e in tr['traceEvents'])


def test_timer_only_and_nested_reader_pause():
    from paddle_ray_amd.profiler.timer import benchmark
    prof = profiler.Profiler(timer_only=True)
    prof.start()
    for _ in range(3):
        time.sleep(0.002)
        prof.step(num_samples=2)
    info = prof.step_info()
    prof.stop()
    assert 'batch_cost' in info and 'reader_cost' not in info
    assert prof.profiler_result is None and prof.summary() == ''
    assert benchmark().current_event is None


def test_statistics_with_device_events_synthetic():
    """Kernel / Device / Distributed views over device records (what a GPU run merges in):
    kernel totals, GPU sort keys and the communication overlap, checked on synthetic events."""
    from paddle_ray_amd.profiler.result import ProfilerResult, HostEvent, DeviceEvent, TracerEventType as TT
    from paddle_ray_amd.profiler.statistic import StatisticData, build_table, SortedKeys
    host = [HostEvent('ProfileStep#0', TT.ProfileStep, 0, 1000, 1)]
    dev = [DeviceEvent('pra::gemm_a', TT.Kernel, 0, 300), DeviceEvent('pra::gemm_a', TT.Kernel, 400, 500),
           DeviceEvent('pra::small', TT.Kernel, 500, 520), DeviceEvent('ncclDevKernel_AllReduce', TT.Kernel, 250, 450)]
    res = ProfilerResult(host, dev, steps=[(0, 0, 1000)])
    data = StatisticData(res)
    tot = {k[0]: it.gpu for k, it in data.kernel_items.items()}
    assert tot == {'pra::gemm_a': 400, 'pra::small': 20, 'ncclDevKernel_AllReduce': 200}
    busy, _ = data.device_union(data.kernels)
    assert busy == 520
    t_total = build_table(data, SortedKeys.GPUTotal, views=[profiler.SummaryView.KernelView], time_unit='ns')
    t_min = build_table(data, SortedKeys.GPUMin, views=[profiler.SummaryView.KernelView], time_unit='ns')
    rows = lambda t: [l.split()[0] for l in t.splitlines() if l.startswith(('pra::', 'nccl'))]  # noqa: E731
    assert rows(t_total)[0] == 'pra::gemm_a' and rows(t_min)[0] == 'pra::small'
    dist = build_table(data, SortedKeys.CPUTotal, views=[profiler.SummaryView.DistributedView], time_unit='ns')
    assert 'Communication' in dist or 'communication' in dist.lower()
