"""paddle.distributed.fleet (parity: python/paddle/distributed/fleet/{fleet.py,
base/distributed_strategy.py, model.py, optimizer.py}).

``fleet.init(is_collective=True, strategy)`` builds the hybrid topology
(dp × pp × sharding × mp) over RCCL; ``distributed_model`` wraps the model for
the active mode (PipelineParallel / TensorParallel / sharded / DataParallel);
``distributed_optimizer`` returns the matching optimizer wrapper
(HybridParallelOptimizer semantics: TP-aware global-norm clipping, sharding).
"""
import os
import copy

import numpy as np
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
                                 'schedule_mode': '1F1B', 'enable_partial_send_recv': True}
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
        self.lamb_configs = {'lamb_weight_decay': 0.01, 'exclude_from_weight_decay': []}
        self.lars = False
        self.lars_configs = {'lars_coeff': 0.001, 'lars_weight_decay': 0.0005, 'epsilon': 0.0,
                             'exclude_from_weight_decay': []}
        self.dgc = False
        self.dgc_configs = {'rampup_begin_step': 0, 'rampup_step': 1, 'sparsity': [0.999]}
        self.localsgd = False
        self.localsgd_configs = {'k_steps': 1, 'begin_step': 1}
        self.adaptive_localsgd = False
        self.fuse_all_reduce_ops = True
        self.fuse_grad_size_in_MB = 64
        self.find_unused_parameters = False
        self.tensor_parallel = False
        self.tensor_parallel_configs = {'tensor_parallel_degree': 1}
        self.without_graph_optimization = True
        self.a_sync = True      # parameter-server mode: asynchronous updates (reference default)
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
        """Host all-reduce of a numpy array (a copy: the input is not modified); over RCCL the
        values travel through the device."""
        a = np.asarray(input)
        t = torch.from_numpy(np.array(a, copy=True))
        if C.is_initialized() and C.get_world_size() > 1:
            op = {'sum': dist.ReduceOp.SUM, 'max': dist.ReduceOp.MAX,
                  'min': dist.ReduceOp.MIN}[mode]
            if dist.get_backend() == 'nccl':
                d = t.to(f'cuda:{torch.cuda.current_device()}')
                dist.all_reduce(d, op)
                t = d.cpu()
            else:
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
        self._ps_role = None
        if not is_collective and os.environ.get('TRAINING_ROLE') and os.environ.get('PADDLE_PSERVERS_IP_PORT_LIST'):
            # parameter-server mode (reference role_maker.py PaddleCloudRoleMaker environment):
            # servers hold the tables, trainers pull / push over distributed.rpc (distributed/ps)
            from .. import ps as _ps
            self._ps_role = _ps.role_from_env()
            self._is_collective = False
            _ps.set_mode('async' if getattr(self._strategy, 'a_sync', True) else 'sync')
            return self
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
        r = getattr(self, '_ps_role', None)
        if r is not None:
            return not r.is_server and r.index == 0
        return C.get_rank() == 0

    def worker_index(self):
        r = getattr(self, '_ps_role', None)
        return r.index if r is not None and not r.is_server else C.get_rank()

    def worker_num(self):
        r = getattr(self, '_ps_role', None)
        return r.n_trainers if r is not None else C.get_world_size()

    def is_worker(self):
        r = getattr(self, '_ps_role', None)
        return r is None or not r.is_server

    def is_server(self):
        r = getattr(self, '_ps_role', None)
        return r is not None and r.is_server

    def server_num(self):
        r = getattr(self, '_ps_role', None)
        return r.n_servers if r is not None else 0

    def server_index(self):
        r = getattr(self, '_ps_role', None)
        return r.index if r is not None and r.is_server else -1

    def worker_endpoints(self, to_string=False):
        eps = C.ParallelEnv().trainer_endpoints
        return ','.join(eps) if to_string else eps

    def barrier_worker(self):
        C.barrier()

    def init_worker(self):
        if getattr(self, '_ps_role', None) is not None:
            from .. import ps as _ps
            _ps.init_worker(self._ps_role)

    def init_server(self, dirname=None, var_names=None, **kwargs):
        """PS mode: join as a server; ``dirname`` preloads the tables save_persistables wrote
        (the_one_ps.py:1340 _init_server)."""
        if getattr(self, '_ps_role', None) is not None:
            from .. import ps as _ps
            _ps.init_server(self._ps_role, dirname=dirname)

    def run_server(self):
        if getattr(self, '_ps_role', None) is not None:
            from .. import ps as _ps
            _ps.run_server()

    def stop_worker(self):
        if getattr(self, '_ps_role', None) is not None:
            from .. import ps as _ps
            _ps.stop_worker()

    def get_hybrid_communicate_group(self):
        return self._hcg

    # -- job geometry (fleet.py rank / nranks / world_size / local_rank / node_num ...) -------
    def rank(self):
        return self.worker_index()

    def nranks(self):
        return self.worker_num()

    world_size = nranks

    def local_rank(self):
        return int(os.environ.get('PADDLE_LOCAL_RANK', os.environ.get('LOCAL_RANK', self.rank())))

    def local_device_ids(self):
        ids = os.environ.get('FLAGS_selected_gpus') or os.environ.get('PADDLE_LOCAL_DEVICE_IDS')
        if ids:
            return [int(i) for i in ids.split(',') if i != '']
        return [self.local_rank()]

    def world_device_ids(self):
        ids = os.environ.get('PADDLE_WORLD_DEVICE_IDS')
        if ids:
            return [[int(i) for i in node.split(',') if i != ''] for node in ids.split(':')]
        return [self.local_device_ids()]

    def node_num(self):
        r = getattr(self, '_ps_role', None)
        if r is not None:
            return len({e.split(':')[0] for e in r.server_endpoints})
        n = os.environ.get('PADDLE_NNODES') or os.environ.get('PADDLE_TRAINERS_NUM_NODES')
        if n:
            return int(n)
        eps = [e for e in os.environ.get('PADDLE_TRAINER_ENDPOINTS', '').split(',') if e]
        return max(1, len({e.split(':')[0] for e in eps}))

    def server_endpoints(self, to_string=False):
        r = getattr(self, '_ps_role', None)
        eps = list(r.server_endpoints) if r is not None else []
        return ','.join(eps) if to_string else eps

    def is_coordinator(self):
        return False

    def init_coordinator(self, *a, **k):
        raise NotImplementedError("federated-learning coordinator (fleet.init_coordinator) is not supported")

    def make_fl_strategy(self, *a, **k):
        raise NotImplementedError("federated-learning strategies (fleet.make_fl_strategy) are not supported")

    def get_fl_client(self, *a, **k):
        raise NotImplementedError("federated-learning clients (fleet.get_fl_client) are not supported")

    def _final_strategy(self):
        return self._strategy

    def _get_applied_meta_list(self):
        return list(getattr(self, '_applied_meta', []))

    def _get_applied_graph_list(self):
        return []

    # -- PS-mode table persistence (fleet.py:695,934; the_one_ps.py) ----------------------------
    def _ps(self):
        if getattr(self, '_ps_role', None) is None:
            return None
        from .. import ps as _ps
        return _ps

    def save_cache_model(self, dirname, **configs):
        ps = self._ps()
        if ps is None:
            raise RuntimeError("save_cache_model is a parameter-server API")
        return ps.save(dirname, int(configs.get('mode', 0)))

    save_cache_table = save_cache_model

    def check_save_pre_patch_done(self):
        return True

    def save_one_table(self, table_id, path, mode):
        ps = self._ps()
        if ps is None:
            raise RuntimeError("save_one_table is a parameter-server API")
        return ps.save(path, mode, table=str(table_id))

    def save_dense_params(self, executor, dirname, scope, program, var_names=None):
        ps = self._ps()
        if ps is None:
            from ..io import save_persistables
            return save_persistables(executor, dirname, program)
        return ps.save(dirname, 0)

    def load_model(self, path, mode=0):
        ps = self._ps()
        if ps is None:
            from ...framework.io import load
            return load(path)
        return ps.load(path)

    def load_one_table(self, table_id, path, mode=0):
        ps = self._ps()
        if ps is None:
            raise RuntimeError("load_one_table is a parameter-server API")
        return ps.load(path, table=str(table_id))

    def shrink(self, threshold=None):
        raise NotImplementedError("fleet.shrink needs per-feature show/click statistics, which this "
                                  "framework's sparse tables do not keep")

    def save_inference_model(self, executor, dirname, feeded_var_names=None, target_vars=None,
                             main_program=None, export_for_deployment=True, mode=0):
        from ...static import save_inference_model, default_main_program
        from ...static.graph import Variable
        prog = main_program or default_main_program()
        blk = prog.global_block()
        feeds = [blk.var(n) if isinstance(n, str) else n for n in (feeded_var_names or [])]
        fetches = list(target_vars or [])
        os.makedirs(dirname, exist_ok=True)
        save_inference_model(os.path.join(dirname, 'model'), feeds, fetches, executor, program=prog)
        ps = self._ps()
        if ps is not None:
            ps.save(os.path.join(dirname, 'tables'), mode)

    def load_inference_model(self, path, mode=0):
        from ...static import load_inference_model
        ps = self._ps()
        if ps is not None and os.path.isdir(os.path.join(path, 'tables')):
            ps.load(os.path.join(path, 'tables'))
        return load_inference_model(os.path.join(path, 'model'))

    # -- wrapping ----------------------------------------------------------------------------
    def _sharding_level(self):
        st = self._strategy
        stage = int(st.sharding_configs.get('stage', 1)) if st.sharding_configs else 1
        return {1: 'os', 2: 'os_g', 3: 'p_g_os'}[stage]

    def distributed_model(self, model):
        out = self._distributed_model(model)
        self._wrapped_model = out
        return out

    def _distributed_model(self, model):
        """Wrap ``model`` for the active hybrid mode (parity: fleet/model.py:30-140).

        * sharding_degree > 1 (alone, with dp, or with mp): ``ShardedModel`` over the sharding
          group (stage from ``sharding_configs['stage']``, default 1 as in the reference's
          DygraphShardingOptimizer), gradients additionally averaged over the dp group;
        * ``strategy.recompute``: every repeated block (LayerList / Sequential member, or the
          sublayers named in ``recompute_configs['checkpoints']``) runs under recompute;
        * ``strategy.amp``: forward under ``auto_cast`` (O2 decorate with use_pure_fp16)."""
        hcg, st = self._hcg, self._strategy
        if hcg is None:
            self.init(is_collective=True)
            hcg, st = self._hcg, self._strategy
        self._sharded_state = None
        if st.amp:
            model = _apply_amp(model, st)
        if st.recompute:
            _apply_recompute(model, st.recompute_configs.get('checkpoints') or [])
        mode = hcg.get_parallel_mode()
        sh = hcg.get_sharding_parallel_world_size()
        if mode == ParallelMode.PIPELINE_PARALLEL:
            state = None
            if sh > 1:
                # pipeline x sharding (parity: pipeline_parallel.py:40-89 with the
                # DygraphShardingOptimizer of hybrid_parallel_optimizer.py:243-313): optimizer
                # state sharded over the sharding group inside each stage (stage 1)
                if self._sharding_level() != 'os':
                    raise NotImplementedError("pipeline x sharding supports sharding stage 1")
                from ...parallel.sharding import ShardedState
                dpg = hcg.get_data_parallel_group()
                state = ShardedState(model, 'os', hcg.get_sharding_parallel_group(),
                                     dp_group=dpg if dpg.nranks > 1 else None,
                                     segment_bytes=int(st.fuse_grad_size_in_MB) << 20)
                self._sharded_state = state
            return _wrap_amp(_pp.PipelineParallel(model, hcg, st, sharded_state=state), st)
        if sh > 1:
            from ...parallel.sharding import ShardedState, ShardedModel
            if hcg.get_model_parallel_world_size() > 1:
                _broadcast_mp_replicated(model, hcg)
            dpg = hcg.get_data_parallel_group()
            state = ShardedState(model, self._sharding_level(), hcg.get_sharding_parallel_group(),
                                 dp_group=dpg if dpg.nranks > 1 else None,
                                 segment_bytes=int(st.fuse_grad_size_in_MB) << 20)
            self._sharded_state = state
            return _wrap_amp(ShardedModel(model, state), st)
        if mode == ParallelMode.TENSOR_PARALLEL:
            return _wrap_amp(TensorParallel(model, hcg, st), st)
        from ...parallel.data_parallel import DataParallel
        if C.get_world_size() > 1:
            return _wrap_amp(DataParallel(model, comm_buffer_size=st.fuse_grad_size_in_MB,
                                          find_unused_parameters=st.find_unused_parameters,
                                          group=hcg.get_data_parallel_group()), st)
        return _wrap_amp(model, st)

    def distributed_optimizer(self, optimizer, strategy=None):
        """HybridParallelOptimizer / sharding optimizer (parity:
        hybrid_parallel_optimizer.py:243-313); ``strategy.gradient_merge`` wraps the result."""
        if strategy is not None:
            self._strategy = strategy
        if getattr(self, '_ps_role', None) is not None:
            # PS mode: the strategy picks async / sync tables; dense parameters are trained on the
            # servers through distributed.ps.DistributedOptimizer
            from .. import ps as _ps
            _ps.set_mode('async' if getattr(self._strategy, 'a_sync', True) else 'sync')
            return optimizer
        if self._hcg is None:
            from ...static import _static_mode_enabled
            if not _static_mode_enabled():
                return optimizer
            self.init(is_collective=True, strategy=self._strategy)
        hcg, st = self._hcg, self._strategy
        from .meta_optimizers import apply_optimizer_swaps
        from ...static import _static_mode_enabled
        if _static_mode_enabled():
            # static programs: the meta-optimizer chain runs at minimize() (meta_optimizers.py)
            opt = StaticFleetOptimizer(optimizer, hcg, st)
            self._wrapped_optimizer = opt
            return opt
        if st.localsgd:
            raise NotImplementedError("strategy.localsgd is a static-graph meta optimizer "
                                      "(reference localsgd_optimizer.py); in dygraph use DataParallel")
        optimizer = apply_optimizer_swaps(optimizer, st)
        state = getattr(self, '_sharded_state', None)
        if state is not None:
            from ...parallel.sharding import ShardedOptimizer
            ppg = hcg.get_pipe_parallel_group()
            opt = ShardedOptimizer(optimizer, state, mp_group=hcg.get_model_parallel_group(),
                                   norm_groups=[ppg])
        else:
            opt = HybridParallelOptimizer(optimizer, hcg, st)
        if st.gradient_merge and int(st.gradient_merge_configs.get('k_steps', 1)) > 1:
            opt = GradientMergeOptimizer(opt, int(st.gradient_merge_configs['k_steps']),
                                         bool(st.gradient_merge_configs.get('avg', True)),
                                         reducer=self._grad_reducer())
        self._wrapped_optimizer = opt
        return opt

    def _grad_reducer(self):
        """The bucket reducer whose collectives gradient merge may skip on non-final
        micro-steps: DataParallel's all-reduce and sharding stage 1/2's all-reduce /
        reduce-scatter (their full gradient buffers accumulate locally). Stage 3 frees its
        full gradients after every backward and accumulates into the owned shard instead."""
        m = getattr(self, '_wrapped_model', None)
        while m is not None and not hasattr(m, '_reducer') and not hasattr(m, '_state') \
                and hasattr(m, '_layers') and isinstance(getattr(m, '_layers'), Layer):
            m = m._layers
        if m is None:
            return None
        state = m.__dict__.get('_state')
        if state is not None:
            return state.reducer if state.stage in (1, 2) else None
        return getattr(m, '_reducer', None)

    def minimize(self, loss, startup_program=None, parameter_list=None, no_grad_set=None):
        """fleet.minimize (reference fleet.py:1216): the distributed optimizer's minimize."""
        opt = getattr(self, '_wrapped_optimizer', None)
        if opt is None:
            raise RuntimeError("call fleet.distributed_optimizer(optimizer) before fleet.minimize")
        return opt.minimize(loss, startup_program, parameter_list, no_grad_set)

    def distributed_scaler(self, scaler):
        """HybridParallelGradScaler: found_inf is MAX-reduced over every hybrid group."""
        hcg = self._hcg
        if hcg is None:
            return scaler
        from ...amp import _uniq
        pgs = [g.process_group for g in (hcg.get_data_parallel_group(), hcg.get_model_parallel_group(),
                                         hcg.get_pipe_parallel_group(),
                                         hcg.get_sharding_parallel_group()) if g.nranks > 1]
        scaler._extra_pgs = _uniq(list(scaler._extra_pgs) + pgs)
        return scaler

    # -- checkpoints ---------------------------------------------------------------------------
    def save_persistables(self, executor, dirname, main_program=None, mode=0):
        """Collective: the program's persistables. PS mode (from a trainer): every server
        writes its dense and sparse tables (mode 0 with optimizer state, 2 parameters only;
        the_one_ps.py:1730 _save_persistables, :1459 _save_sparse_params)."""
        if getattr(self, '_ps_role', None) is not None:
            from .. import ps as _ps
            if self._ps_role.is_server:
                raise RuntimeError("fleet.save_persistables in PS mode is called on a trainer")
            return _ps.save(dirname, mode)
        from ..io import save_persistables
        save_persistables(executor, dirname, main_program)

    def state_dict(self):
        """Checkpoint of the job as this rank sees it: the wrapped model's FULL parameters (a
        sharded model gathers them) and, once ``distributed_optimizer`` ran, the optimizer state
        in the reference's per-parameter layout (a sharded optimizer gathers every shard, so the
        file resumes at any sharding degree). Every rank of the hybrid groups must call it."""
        sd = {}
        m = getattr(self, '_wrapped_model', None)
        if m is not None:
            sd['model'] = m.state_dict()
        o = getattr(self, '_wrapped_optimizer', None)
        if o is not None:
            sd['optimizer'] = o.state_dict()
        return sd

    def set_state_dict(self, sd):
        m = getattr(self, '_wrapped_model', None)
        if m is not None and 'model' in sd:
            m.set_state_dict(sd['model'])
        o = getattr(self, '_wrapped_optimizer', None)
        if o is not None and 'optimizer' in sd:
            o.set_state_dict(sd['optimizer'])


from ...nn.layer.layers import Layer  # noqa: E402


def _broadcast_mp_replicated(layers, hcg):
    mpg = hcg.get_model_parallel_group()
    if mpg.nranks > 1:
        for p in layers.parameters():
            if not getattr(p, 'is_distributed', False):
                dist.broadcast(p._t.data, mpg.ranks[0], group=mpg.process_group)


def _apply_recompute(model, checkpoints):
    """strategy.recompute for dygraph: run the chosen blocks under activation recompute."""
    from ...parallel.sharding import _find_units
    if checkpoints:
        named = dict(model.named_sublayers())
        blocks = [named[n] for n in checkpoints if n in named]
    else:
        blocks = _find_units(model)
    for blk in blocks:
        if getattr(blk, '_pra_recompute', False):
            continue
        fwd = blk.forward

        def run(*a, _f=fwd, **k):
            if not blk.training or not torch.is_grad_enabled():
                return _f(*a, **k)
            return _recompute(_f, *a, **k)
        blk.__dict__['forward'] = run
        blk.__dict__['_pra_recompute'] = True


def _apply_amp(model, st):
    cfg = st.amp_configs
    if cfg.get('use_pure_fp16') or cfg.get('use_fp16_guard') is False and cfg.get('level') == 'O2':
        from ... import amp
        amp.decorate(model, level='O2', dtype='bfloat16' if cfg.get('use_bf16') else 'float16')
    return model


class _AmpForward(Layer):
    def __init__(self, inner, st):
        super().__init__()
        self._layers = inner
        cfg = st.amp_configs
        self.__dict__['_amp_kw'] = dict(
            level='O2' if cfg.get('use_pure_fp16') else 'O1',
            dtype='bfloat16' if cfg.get('use_bf16') else 'float16',
            custom_white_list=cfg.get('custom_white_list'),
            custom_black_list=cfg.get('custom_black_list'))

    def forward(self, *a, **k):
        from ... import amp
        with amp.auto_cast(True, **self._amp_kw):
            return self._layers(*a, **k)

    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            return getattr(self.__dict__['_sub_layers']['_layers'], name)

    def state_dict(self, *a, **k):
        return self._layers.state_dict(*a, **k)

    def set_state_dict(self, *a, **k):
        return self._layers.set_state_dict(*a, **k)

    def parameters(self, include_sublayers=True):
        return self._layers.parameters(include_sublayers)


def _wrap_amp(model, st):
    return _AmpForward(model, st) if st.amp else model


class GradientMergeOptimizer:
    """strategy.gradient_merge (parity: meta_optimizers/gradient_merge_optimizer.py): gradients
    accumulate over ``k_steps`` backward passes; the inner step runs on every k-th call
    (grads averaged when ``avg``) and only then are grads cleared."""

    def __init__(self, inner, k_steps, avg=True, reducer=None):
        self._inner_opt = inner
        self.k_steps = k_steps
        self.avg = avg
        self._calls = 0
        # no_sync for the k-1 non-final backward passes: the gradient collectives run once per
        # k micro-steps, on the locally accumulated buffers (parity: the reference merges
        # gradients before its allreduce ops)
        self._reducer = reducer
        self._arm()

    def _arm(self):
        if self._reducer is not None:
            self._reducer.enabled = (self._calls + 1) % self.k_steps == 0

    def _grads(self):
        g = getattr(self._inner_opt, '_scaler_grads', None)
        if g is not None:
            return g()
        return [p._t.grad for p in self._inner_opt._parameter_list if p._t.grad is not None]

    def step(self):
        self._calls += 1
        self._arm()  # the NEXT backward reduces only if it completes a merge window
        if self._calls % self.k_steps:
            return
        if self.avg:
            with torch.no_grad():
                for g in self._grads():
                    g.div_(self.k_steps)
        self._inner_opt.step()
        self._merged_ready = True

    def clear_grad(self, set_to_zero=True):
        if self._calls % self.k_steps == 0:
            self._inner_opt.clear_grad(set_to_zero)

    clear_gradients = clear_grad

    def minimize(self, loss, *a, **k):
        loss.backward()
        self.step()

    def __getattr__(self, k):
        return getattr(self._inner_opt, k)


class TensorParallel(Layer):
    """Broadcast non-distributed params inside the mp group; DP all-reduce over dp group."""

    def __init__(self, layers, hcg, strategy=None):
        super().__init__()
        self._layers = layers
        self._hcg = hcg
        _broadcast_mp_replicated(layers, hcg)
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
                ps = [p for p in params if p._t.grad is not None and
                      getattr(p, 'is_firstly_shared', True)]  # tied weights counted once
                d = [p._t.grad for p in ps if getattr(p, 'is_distributed', False)]
                r = [p._t.grad for p in ps if not getattr(p, 'is_distributed', False)]
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

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        from ...static import _static_mode_enabled
        if _static_mode_enabled():
            from .meta_optimizers import static_minimize
            return static_minimize(self._inner_opt, loss, self._strategy, self._hcg, parameters)
        return self._inner_opt.minimize(loss, startup_program, parameters, no_grad_set)

    def __getattr__(self, k):
        return getattr(self._inner_opt, k)


class StaticFleetOptimizer:
    """``fleet.distributed_optimizer`` in static mode: ``minimize`` appends the backward and the
    collective-training rewrite of meta_optimizers.static_minimize (bucketed async gradient
    all-reduce, gradient merge, sharding stage 1, localsgd, lamb / lars swaps, amp)."""

    def __init__(self, optimizer, hcg, strategy):
        from .meta_optimizers import apply_optimizer_swaps
        from ...static.amp import OptimizerWithMixedPrecision
        if isinstance(optimizer, OptimizerWithMixedPrecision):
            optimizer._optimizer = apply_optimizer_swaps(optimizer._optimizer, strategy)
            self._inner_opt = optimizer
        else:
            self._inner_opt = apply_optimizer_swaps(optimizer, strategy)
        self._hcg, self._strategy = hcg, strategy

    def minimize(self, loss, startup_program=None, parameter_list=None, no_grad_set=None):
        from .meta_optimizers import static_minimize
        return static_minimize(self._inner_opt, loss, self._strategy, self._hcg, parameter_list)

    def __getattr__(self, k):
        return getattr(self._inner_opt, k)


fleet = Fleet()
init = fleet.init
distributed_model = fleet.distributed_model
distributed_optimizer = fleet.distributed_optimizer
get_hybrid_communicate_group = fleet.get_hybrid_communicate_group
state_dict = fleet.state_dict
set_state_dict = fleet.set_state_dict
distributed_scaler = fleet.distributed_scaler
is_first_worker = fleet.is_first_worker
worker_index = fleet.worker_index
worker_num = fleet.worker_num
barrier_worker = fleet.barrier_worker
is_worker = fleet.is_worker
is_server = fleet.is_server
server_num = fleet.server_num
server_index = fleet.server_index
init_worker = fleet.init_worker
init_server = fleet.init_server
run_server = fleet.run_server
stop_worker = fleet.stop_worker
worker_endpoints = fleet.worker_endpoints
util = fleet.util
_final_strategy = fleet._final_strategy
_get_applied_meta_list = fleet._get_applied_meta_list
_get_applied_graph_list = fleet._get_applied_graph_list
node_num = fleet.node_num
rank = fleet.rank
nranks = fleet.nranks
world_size = fleet.world_size
local_device_ids = fleet.local_device_ids
world_device_ids = fleet.world_device_ids
local_rank = fleet.local_rank
is_coordinator = fleet.is_coordinator
init_coordinator = fleet.init_coordinator
make_fl_strategy = fleet.make_fl_strategy
get_fl_client = fleet.get_fl_client
server_endpoints = fleet.server_endpoints
save_inference_model = fleet.save_inference_model
save_persistables = fleet.save_persistables
save_cache_model = fleet.save_cache_model
save_cache_table = fleet.save_cache_table
check_save_pre_patch_done = fleet.check_save_pre_patch_done
save_one_table = fleet.save_one_table
save_dense_params = fleet.save_dense_params
load_model = fleet.load_model
load_inference_model = fleet.load_inference_model
load_one_table = fleet.load_one_table
minimize = fleet.minimize
shrink = fleet.shrink

from . import meta_parallel, utils, layers, recompute, metrics, data_generator  # noqa: E402,F401
from .data_generator import MultiSlotDataGenerator, MultiSlotStringDataGenerator  # noqa: E402,F401
from .meta_parallel import (LayerDesc, SharedLayerDesc, PipelineLayer,  # noqa: E402,F401
                            ColumnParallelLinear, RowParallelLinear, VocabParallelEmbedding,
                            ParallelCrossEntropy, get_rng_state_tracker)
