"""paddle.distributed.fleet (parity: python/paddle/distributed/fleet/{fleet.py,
base/distributed_strategy.py, model.py, optimizer.py}).

``fleet.init(is_collective=True, strategy)`` builds the hybrid topology
(dp × pp × sharding × mp) over RCCL; ``distributed_model`` wraps the model for
the active mode (PipelineParallel / TensorParallel / sharded / DataParallel);
``distributed_optimizer`` returns the matching optimizer wrapper
(HybridParallelOptimizer semantics: TP-aware global-norm clipping, sharding).
"""
import copy

import torch
import torch.distributed as dist

from .. import collective as C
from ...parallel.topology import CommunicateTopology, HybridCommunicateGroup, ParallelMode  # noqa
from ...parallel import tensor_parallel as _tp
from ...parallel import pipeline as _pp
from ...parallel.recompute import recompute as _recompute
from ...framework.core import Tensor, _u


class DistributedStrategy:
    def __init__(self):
        self.hybrid_configs = {'dp_degree': -1, 'mp_degree': 1, 'pp_degree': 1,
                               'sharding_degree': 1}
        self.pipeline_configs = {'micro_batch_size': 1, 'accumulate_steps': 1,
                                 'schedule_mode': '1F1B'}
        self.sharding = False
        self.sharding_configs = {'sharding_degree': 1, 'stage': 1, 'segment_broadcast_MB': 32}
        self.amp = False
        self.amp_configs = {'init_loss_scaling': 32768, 'use_pure_fp16': False,
                            'use_bf16': False}
        self.recompute = False
        self.recompute_configs = {'checkpoints': []}
        self.gradient_merge = False
        self.gradient_merge_configs = {'k_steps': 1, 'avg': True}
        self.lamb = False
        self.lars = False
        self.dgc = False
        self.localsgd = False
        self.fuse_all_reduce_ops = True
        self.fuse_grad_size_in_MB = 64
        self.find_unused_parameters = False
        self.tensor_parallel = False
        self.tensor_parallel_configs = {'tensor_parallel_degree': 1}
        self.without_graph_optimization = True
        self.a_sync = False
        self.a_sync_configs = {}
        self.heter_ccl_mode = False
        self.build_strategy = None
        self.execution_strategy = None

    def __setattr__(self, k, v):
        if k.endswith('_configs') and k in self.__dict__ and isinstance(v, dict):
            d = dict(self.__dict__[k])
            d.update(v)
            v = d
        object.__setattr__(self, k, v)

    def __repr__(self):
        return f'DistributedStrategy(hybrid_configs={self.hybrid_configs})'


class UtilBase:
    def all_reduce(self, input, mode="sum", comm_world="worker"):
        t = torch.as_tensor(input)
        if C.is_initialized() and C.get_world_size() > 1:
            op = {'sum': dist.ReduceOp.SUM, 'max': dist.ReduceOp.MAX,
                  'min': dist.ReduceOp.MIN}[mode]
            dist.all_reduce(t, op)
        return t.numpy()

    def barrier(self, comm_world="worker"):
        C.barrier()

    def all_gather(self, input, comm_world="worker"):
        out = []
        C.all_gather_object(out, input)
        return out

    def get_file_shard(self, files):
        r, n = C.get_rank(), C.get_world_size()
        return files[r::n]

    def print_on_rank(self, message, rank_id):
        if C.get_rank() == rank_id:
            print(message)


class Role:
    WORKER = 1
    SERVER = 2
    HETER_WORKER = 3
    ALL = 4
    COORDINATOR = 5


class PaddleCloudRoleMaker:
    def __init__(self, is_collective=False, **kwargs):
        self._is_collective = is_collective

    def _worker_index(self):
        return C.get_rank()

    def _worker_num(self):
        return C.get_world_size()

    def _is_worker(self):
        return True

    def _is_server(self):
        return False


class UserDefinedRoleMaker(PaddleCloudRoleMaker):
    def __init__(self, is_collective=False, init_gloo=False, **kwargs):
        super().__init__(is_collective)
        self._kw = kwargs


class Fleet:
    def __init__(self):
        self._hcg = None
        self._strategy = None
        self._topology = None
        self._is_collective = True
        self.util = UtilBase()

    def init(self, role_maker=None, is_collective=False, strategy=None, log_level="INFO"):
        self._strategy = strategy or DistributedStrategy()
        self._is_collective = True
        C.init_parallel_env()
        ws = C.get_world_size()
        hc = dict(self._strategy.hybrid_configs)
        mp, pp = hc.get('mp_degree', 1), hc.get('pp_degree', 1)
        sh = hc.get('sharding_degree', 1)
        dp = hc.get('dp_degree', -1)
        if dp in (-1, None):
            dp = ws // (mp * pp * sh)
        assert dp * mp * pp * sh == ws, \
            f"dp({dp})*mp({mp})*pp({pp})*sharding({sh}) != world_size({ws})"
        self._topology = CommunicateTopology(["data", "pipe", "sharding", "model"], [dp, pp, sh, mp])
        self._hcg = HybridCommunicateGroup(self._topology)
        if mp > 1:
            _tp.model_parallel_random_seed()
        return self

    # -- info ----------------------------------------------------------------------------
    def is_first_worker(self):
        return C.get_rank() == 0

    def worker_index(self):
        return C.get_rank()

    def worker_num(self):
        return C.get_world_size()

    def is_worker(self):
        return True

    def is_server(self):
        return False

    def worker_endpoints(self, to_string=False):
        eps = C.ParallelEnv().trainer_endpoints
        return ','.join(eps) if to_string else eps

    def barrier_worker(self):
        C.barrier()

    def init_worker(self):
        pass

    def init_server(self, *a, **k):
        pass

    def run_server(self):
        pass

    def stop_worker(self):
        pass

    def get_hybrid_communicate_group(self):
        return self._hcg

    # -- wrapping ----------------------------------------------------------------------------
    def distributed_model(self, model):
        hcg, st = self._hcg, self._strategy
        if hcg is None:
            self.init(is_collective=True)
            hcg, st = self._hcg, self._strategy
        mode = hcg.get_parallel_mode()
        if mode == ParallelMode.PIPELINE_PARALLEL:
            return _pp.PipelineParallel(model, hcg, st)
        if mode == ParallelMode.TENSOR_PARALLEL:
            return TensorParallel(model, hcg, st)
        if mode == ParallelMode.SHARDING_PARALLEL:
            return model  # sharding wrapper is applied together with the optimizer
        from ...parallel.data_parallel import DataParallel
        if C.get_world_size() > 1:
            return DataParallel(model, comm_buffer_size=st.fuse_grad_size_in_MB,
                                find_unused_parameters=st.find_unused_parameters,
                                group=hcg.get_data_parallel_group())
        return model

    def distributed_optimizer(self, optimizer, strategy=None):
        if strategy is not None:
            self._strategy = strategy
        if self._hcg is None:
            return optimizer
        return HybridParallelOptimizer(optimizer, self._hcg, self._strategy)

    # -- checkpoints ---------------------------------------------------------------------------
    def save_persistables(self, executor, dirname, main_program=None, mode=0):
        from ..io import save_persistables
        save_persistables(executor, dirname, main_program)

    def state_dict(self):
        return {}


class TensorParallel(torch.nn.Module if False else object):
    pass


from ...nn.layer.layers import Layer  # noqa: E402


class TensorParallel(Layer):  # noqa: F811
    """Broadcast non-distributed params inside the mp group; DP all-reduce over dp group."""

    def __init__(self, layers, hcg, strategy=None):
        super().__init__()
        self._layers = layers
        self._hcg = hcg
        mpg = hcg.get_model_parallel_group()
        if mpg.nranks > 1:
            for p in layers.parameters():
                if not getattr(p, 'is_distributed', False):
                    dist.broadcast(p._t.data, mpg.ranks[0], group=mpg.process_group)
        dpg = hcg.get_data_parallel_group()
        self._dp = None
        if dpg.nranks > 1:
            from ...parallel.data_parallel import DataParallel
            self._dp = DataParallel(layers, group=dpg)

    def forward(self, *a, **k):
        return (self._dp or self._layers)(*a, **k)

    def state_dict(self, *a, **k):
        return self._layers.state_dict(*a, **k)

    def set_state_dict(self, *a, **k):
        return self._layers.set_state_dict(*a, **k)

    def parameters(self, include_sublayers=True):
        return self._layers.parameters(include_sublayers)


class HybridParallelOptimizer:
    """Global-norm clip over the full (TP-sharded + replicated) parameter set, then step."""

    def __init__(self, optimizer, hcg, strategy):
        self._inner_opt = optimizer
        self._hcg = hcg
        self._strategy = strategy
        from ...nn.clip import ClipGradByGlobalNorm
        clip = optimizer._grad_clip
        mpg = hcg.get_model_parallel_group()
        ppg = hcg.get_pipe_parallel_group()
        if isinstance(clip, ClipGradByGlobalNorm) and (mpg.nranks > 1 or ppg.nranks > 1):
            params = optimizer._parameter_list
            dist_ids = {id(p._t.grad) for p in params if getattr(p, 'is_distributed', False)}

            def hook(sq_local, params=params):
                # recompute split: distributed params are summed over mp ranks, replicated once
                d = [p._t.grad for p in params if p._t.grad is not None and
                     getattr(p, 'is_distributed', False)]
                r = [p._t.grad for p in params if p._t.grad is not None and
                     not getattr(p, 'is_distributed', False)]
                from ...ops.fused import global_l2_norm_sq
                sd = global_l2_norm_sq(d) if d else torch.zeros((), device=sq_local.device)
                sr = global_l2_norm_sq(r) if r else torch.zeros((), device=sq_local.device)
                sd = sd.reshape(1).float()
                if mpg.nranks > 1:
                    dist.all_reduce(sd, group=mpg.process_group)
                tot = (sd + sr.reshape(1).float())
                if ppg.nranks > 1:
                    dist.all_reduce(tot, group=ppg.process_group)
                return tot[0]
            clip._norm_hook = hook

    def step(self):
        self._inner_opt.step()

    def clear_grad(self, set_to_zero=True):
        self._inner_opt.clear_grad(set_to_zero)

    def minimize(self, loss, *a, **k):
        return self._inner_opt.minimize(loss, *a, **k)

    def __getattr__(self, k):
        return getattr(self._inner_opt, k)


fleet = Fleet()
init = fleet.init
distributed_model = fleet.distributed_model
distributed_optimizer = fleet.distributed_optimizer
get_hybrid_communicate_group = fleet.get_hybrid_communicate_group
is_first_worker = fleet.is_first_worker
worker_index = fleet.worker_index
worker_num = fleet.worker_num
barrier_worker = fleet.barrier_worker
util = fleet.util

from . import meta_parallel, utils, layers, recompute  # noqa: E402,F401
from .meta_parallel import (LayerDesc, SharedLayerDesc, PipelineLayer,  # noqa: E402,F401
                            ColumnParallelLinear, RowParallelLinear, VocabParallelEmbedding,
                            ParallelCrossEntropy, get_rng_state_tracker)
