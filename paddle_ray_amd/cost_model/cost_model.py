"""Op cost model (parity: python/paddle/cost_model/cost_model.py).

Two sources of cost, both measured on MI355X rather than carried over from other GPUs:
  * profile_measure(): runs a static Program through the Executor with per-op timing
    (device-synchronized around every op) and returns total / per-op-type milliseconds;
  * static_cost_data() / get_static_op_time(): a benchmark table of the framework's ops
    (forward and backward time per op and config) in the reference's JSON schema, produced
    on the GPU by ``scripts/op_benchmark.py`` into ``static_op_benchmark_gfx950.json``.
"""
import json
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
STATIC_DATA = os.path.join(_HERE, 'static_op_benchmark_gfx950.json')


class CostModel:
    def __init__(self):
        self._static_cost_data = None

    def build_program(self):
        """A small fc + mean + SGD program (the reference's example program)."""
        import paddle_ray_amd as paddle
        from paddle_ray_amd import static
        paddle.enable_static()
        main_program, startup_program = static.Program(), static.Program()
        with static.program_guard(main_program, startup_program):
            data = static.data(name='X', shape=[None, 1], dtype='float32')
            hidden = static.nn.fc(data, 10)
            loss = paddle.mean(hidden)
            paddle.optimizer.SGD(learning_rate=0.01).minimize(loss)
        return startup_program, main_program

    def profile_measure(self, startup_program, main_program, device='gpu',
                        fetch_cost_list=('time',), feed=None, warmup=1):
        """Execute ``main_program`` (after ``startup_program``) and measure it.

        Returns {'time': total ms, 'op_time': {op type: summed ms}, 'ops': [(type, ms)]}.
        ``feed`` defaults to random data for every ``static.data`` variable (None dims -> 10).
        """
        import paddle_ray_amd as paddle
        from paddle_ray_amd import static
        if device == 'gpu':
            try:
                paddle.set_device('gpu')
            except Exception:  # no device: measure on the CPU
                paddle.set_device('cpu')
        else:
            paddle.set_device(device)
        exe = static.Executor()
        exe.run(startup_program)
        if feed is None:
            feed = {}
            for v in main_program.global_block().vars.values():
                if getattr(v, 'is_data', False):
                    shape = [10 if (d is None or d < 0) else d for d in v.shape]
                    feed[v.name] = np.random.random(shape).astype(str(v.dtype).replace(
                        'paddle.', '').replace('torch.', ''))
        for _ in range(warmup):
            exe.run(main_program, feed=feed, fetch_list=[])
        exe.enable_op_timing(True)
        exe.run(main_program, feed=feed, fetch_list=[])
        ops = exe.op_costs
        exe.enable_op_timing(False)
        per = {}
        for t, ms in ops:
            per[t] = per.get(t, 0.0) + ms
        out = {'ops': ops, 'op_time': per}
        if 'time' in fetch_cost_list:
            out['time'] = sum(ms for _, ms in ops)
        return out

    def static_cost_data(self, path=None):
        path = path or STATIC_DATA
        if not os.path.exists(path):
            raise FileNotFoundError(
                f"{path} not found: generate it on the GPU with scripts/op_benchmark.py")
        with open(path) as f:
            self._static_cost_data = json.load(f)
        return self._static_cost_data

    def get_static_op_time(self, op_name, forward=True, dtype='float32'):
        """{'op_time': ms, 'config': str} of the last matching entry (fwd or bwd time)."""
        if op_name is None:
            raise ValueError('op_name should not be empty when you want to get static op time')
        if self._static_cost_data is None:
            self.static_cost_data()
        op_cost = {}
        for d in self._static_cost_data:
            if d['op'] == op_name and dtype in d['config']:
                op_cost['op_time'] = d['paddle_gpu_time' if forward else
                                       'paddle_gpu_time_backward']
                op_cost['config'] = d['config']
        return op_cost
