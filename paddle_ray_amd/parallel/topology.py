"""Hybrid-parallel topology (parity: python/paddle/distributed/fleet/base/topology.py).

Rank layout order is [dp, pp, sharding, mp] (mp fastest-varying), exactly like
the reference, so TP groups are the adjacent GPUs of a node: on MI355X the TP
all-reduces then stay on direct xGMI links between neighbouring GPUs.
"""
import collections
import itertools

import numpy as np

from ..distributed import collective as C


class ParallelMode:
    DATA_PARALLEL = 0
    TENSOR_PARALLEL = 1
    PIPELINE_PARALLEL = 2
    SHARDING_PARALLEL = 3


class CommunicateTopology:
    def __init__(self, hybrid_group_names=("data", "pipe", "sharding", "model"),
                 dims=(1, 1, 1, 1)):
        self._parallel_names = list(hybrid_group_names)
        self._dims = list(dims)
        self.coordinate = collections.namedtuple('Coordinate', self._parallel_names)
        self._world_size = int(np.prod(self._dims))
        ranges = [range(d) for d in self._dims]
        all_coords = [self.coordinate(*c) for c in itertools.product(*ranges)]
        self._coord2rank = {c: i for i, c in enumerate(all_coords)}
        self._rank2coord = {i: c for c, i in self._coord2rank.items()}

    def get_hybrid_group_names(self):
        return self._parallel_names

    def get_dim(self, axis_name):
        return self._dims[self._parallel_names.index(axis_name)]

    def world_size(self):
        return self._world_size

    def get_rank(self, **kwargs):
        return self._coord2rank[self.coordinate(**kwargs)]

    def get_coord(self, rank):
        return self._rank2coord[rank]

    def get_axis_list(self, axis_name, index):
        ai = self._parallel_names.index(axis_name)
        return sorted(r for c, r in self._coord2rank.items() if c[ai] == index)

    def get_dim_size(self, axis_name):
        return self.get_dim(axis_name)

    def get_comm_list(self, axis_name):
        """All rank lists that communicate along ``axis_name``."""
        ai = self._parallel_names.index(axis_name)
        other = [range(d) for i, d in enumerate(self._dims) if i != ai]
        out = []
        for oc in itertools.product(*other):
            ranks = []
            for k in range(self._dims[ai]):
                c = list(oc)
                c.insert(ai, k)
                ranks.append(self._coord2rank[self.coordinate(*c)])
            out.append(ranks)
        return out

    def get_rank_from_stage(self, global_rank, **kwargs):
        c = self._rank2coord[global_rank]._asdict()
        c.update(kwargs)
        return self._coord2rank[self.coordinate(**c)]


class HybridCommunicateGroup:
    def __init__(self, topology):
        self._topo = topology
        self.global_rank = C.get_rank()
        self.nranks = topology.world_size()
        self._dp_degree = topology.get_dim('data')
        self._mp_degree = topology.get_dim('model')
        self._pp_degree = topology.get_dim('pipe')
        self._sharding_degree = topology.get_dim('sharding')
        coord = topology.get_coord(self.global_rank) if self.global_rank < self.nranks else None
        self._groups = {}
        for axis in ('data', 'model', 'pipe', 'sharding'):
            mine = None
            for ranks in topology.get_comm_list(axis):
                g = C.new_group(ranks) if C.is_initialized() and C.get_world_size() > 1 and \
                    len(ranks) > 1 else C.Group(ranks, None, -1)
                if self.global_rank in ranks:
                    mine = g
            self._groups[axis] = mine
        # pipeline neighbours for p2p
        self.stage_id = coord.pipe if coord else 0
        self._check_group = self._groups['data']

    # -- parallel mode ---------------------------------------------------------------
    def get_parallel_mode(self):
        if self._pp_degree > 1:
            return ParallelMode.PIPELINE_PARALLEL
        if self._mp_degree > 1:
            return ParallelMode.TENSOR_PARALLEL
        if self._sharding_degree > 1:
            return ParallelMode.SHARDING_PARALLEL
        return ParallelMode.DATA_PARALLEL

    def topology(self):
        return self._topo

    def get_global_rank(self):
        return self.global_rank

    # data
    def get_data_parallel_rank(self):
        return self._groups['data'].rank

    def get_data_parallel_world_size(self):
        return self._dp_degree

    def get_data_parallel_group(self):
        return self._groups['data']

    def get_data_parallel_group_src_rank(self):
        return self._groups['data'].ranks[0]

    # model
    def get_model_parallel_rank(self):
        return self._groups['model'].rank

    def get_model_parallel_world_size(self):
        return self._mp_degree

    def get_model_parallel_group(self):
        return self._groups['model']

    def get_model_parallel_group_src_rank(self):
        return self._groups['model'].ranks[0]

    # pipe
    def get_stage_id(self):
        return self.stage_id

    def get_pipe_parallel_world_size(self):
        return self._pp_degree

    def get_pipe_parallel_group(self):
        return self._groups['pipe']

    def is_first_stage(self):
        return self.stage_id == 0

    def is_last_stage(self):
        return self.stage_id == self._pp_degree - 1

    def get_rank_from_stage(self, stage_id, **kwargs):
        return self._topo.get_rank_from_stage(self.global_rank, pipe=stage_id, **kwargs)

    # sharding
    def get_sharding_parallel_rank(self):
        return self._groups['sharding'].rank

    def get_sharding_parallel_world_size(self):
        return self._sharding_degree

    def get_sharding_parallel_group(self):
        return self._groups['sharding']

    def get_sharding_parallel_group_src_rank(self):
        return self._groups['sharding'].ranks[0]

    def get_check_parallel_group(self, sharding=False):
        return self._check_group
