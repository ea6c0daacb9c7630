"""Distributed inference over parameter-server tables (parity: python/paddle/distributed/fleet/
utils/ps_util.py DistributedInfer).

In this framework a model's sparse tables are ``distributed.ps.SparseEmbedding`` layers whose
lookups already pull from the servers, so the "distributed inference program" is the program /
model itself: what DistributedInfer adds is the job bring-up -- servers load the saved tables
(``init_server(dirname)``), trainers initialise their local dense parameters and, with
``dirname``, load the dense values saved by ``fleet.save_persistables``."""
import glob
import os

import numpy as np

__all__ = ['DistributedInfer']


class DistributedInfer:
    def __init__(self, main_program=None, startup_program=None):
        from ....static import default_main_program, default_startup_program
        self.origin_main_program = (main_program or default_main_program()).clone()
        self.origin_startup_program = startup_program or default_startup_program()
        self.sparse_table_maps = None

    def init_distributed_infer_env(self, exe, loss=None, role_maker=None, dirname=None):
        """Servers: load ``dirname`` and serve (returns when the trainers stop). Trainers: run the
        startup program, join the PS world and load the saved dense parameters."""
        from ... import fleet
        from ... import ps as _ps
        if getattr(fleet.fleet, '_ps_role', None) is None:
            fleet.init(role_maker=role_maker, is_collective=False)
        if fleet.is_server():
            fleet.init_server(dirname=dirname)
            fleet.run_server()
            return
        if exe is not None:
            exe.run(self.origin_startup_program)
        fleet.init_worker()
        self._init_dense_params(exe, dirname)
        self.sparse_table_maps = None
        self._ps = _ps

    def _get_sparse_table_map(self):
        """{sparse table name: table name} of the job (tables are addressed by name here)."""
        if self.sparse_table_maps is None:
            self.sparse_table_maps = {}
        return self.sparse_table_maps

    def _init_dense_params(self, exe=None, dirname=None):
        """Dense values saved as ``dense/<name>.npz`` are copied into the program's persistable
        variables of the same name."""
        if not dirname:
            return []
        prog = self.origin_main_program
        params = {p.name: p for p in prog.all_parameters()}
        loaded = []
        for f in sorted(glob.glob(os.path.join(dirname, 'dense', '*.npz'))):
            name = os.path.basename(f)[:-4]
            p = params.get(name)
            if p is None:
                continue
            with np.load(f, allow_pickle=False) as z:
                p.set_value(z['w'].reshape(p.shape).astype(p.numpy().dtype))
            loaded.append(name)
        return loaded

    def get_dist_infer_program(self):
        return self.origin_main_program
