"""Profiler device side on the MI355X: a GPT-tiny training step's KernelView lists the in-tree
HIP kernels (pra::...) with totals matching the device trace, GPU sort keys rank them, and the
Model view attributes device time to Forward / Backward / Optimization (reference:
python/paddle/profiler/profiler_statistic.py KernelView / ModelView)."""
import json

import pytest

pytestmark = pytest.mark.gpu


def _gpt_step_profile(tmp_path):
    import torch
    import paddle_ray_amd as paddle
    import paddle_ray_amd.profiler as profiler
    from paddle_ray_amd.models import gpt_config, GPTForPretraining
    paddle.set_device('gpu:0')
    paddle.set_default_dtype('bfloat16')
    model = GPTForPretraining(gpt_config('gpt3-tiny'))
    paddle.set_default_dtype('float32')
    opt = paddle.optimizer.AdamW(1e-3, parameters=model.parameters(), multi_precision=True)
    ids = paddle.randint(0, 1024, [4, 129])

    def step():
        loss = model(ids[:, :-1], ids[:, 1:])
        loss.backward()
        opt.step()
        opt.clear_grad()
    step()
    torch.cuda.synchronize()
    prof = profiler.Profiler(targets=[profiler.ProfilerTarget.CPU, profiler.ProfilerTarget.GPU],
                             scheduler=(1, 3))
    prof.start()
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(3):
        if i == 1:
            s0.record()
        step()
        if i == 2:
            s1.record()
        prof.step()
    prof.stop()
    torch.cuda.synchronize()
    return prof, s0.elapsed_time(s1) * 1e6


def test_kernel_view_lists_hip_kernels_and_matches_trace(tmp_path):
    import paddle_ray_amd.profiler as profiler
    from paddle_ray_amd.profiler.statistic import StatisticData
    prof, wall_ns = _gpt_step_profile(tmp_path)
    res = prof.profiler_result
    assert res.device_events, res.extra_info
    data = StatisticData(res)
    pra = {k: it for k, it in data.kernel_items.items() if 'pra::' in k[0] or 'WCfg' in k[0]}
    assert pra, sorted(k[0] for k in data.kernel_items)[:20]
    s = prof.summary(views=[profiler.SummaryView.KernelView], sorted_by=profiler.SortedKeys.GPUTotal)
    top = [l for l in s.splitlines() if 'pra::' in l or 'WCfg' in l]
    assert top
    # KernelView totals == the exported Chrome trace's device events (same kernels, same time)
    prof.export(str(tmp_path / 't.json'), 'json')
    tr = json.load(open(tmp_path / 't.json'))
    dev = [e for e in tr['traceEvents'] if str(e.get('pid', '')).startswith('GPU')]
    tot_trace = sum(e['dur'] for e in dev if e.get('cat') == 'Kernel') * 1e3
    tot_view = sum(it.gpu for it in data.kernel_items.values())
    assert abs(tot_trace - tot_view) <= 0.05 * tot_view
    # the recorded steps' device time is bounded by the measured wall time (GPT-tiny is
    # launch-bound: the device is busy for only a fraction of it)
    busy, _ = data.device_union(data.kernels)
    assert busy <= wall_ns * 1.05 and busy > 0.02 * wall_ns, (busy, wall_ns)
    # GPU sort keys change the ranking
    mn = prof.summary(views=[profiler.SummaryView.KernelView], sorted_by=profiler.SortedKeys.GPUMin)
    first = lambda t: next(l for l in t.splitlines()[4:] if l.strip()).split('  ')[0]  # noqa: E731
    assert first(s) != first(mn)
    # the Model view attributes device time to the training phases
    mv = prof.summary(views=[profiler.SummaryView.ModelView])
    for r in ('Forward', 'Backward', 'Optimization'):
        line = next(l for l in mv.splitlines() if l.startswith(r))
        assert float(line.split()[7]) > 0, line
