"""paddle.distributed.passes (parity: python/paddle/distributed/passes/__init__.py): the pass
registry (``new_pass``), ``PassManager`` / ``PassContext`` and the passes this framework
implements over its static programs -- distributed training (auto_parallel_amp / _fp16 /
_recompute / _gradient_merge_pass / _sharding / _grad_clip / _data_parallel_optimization,
fuse_all_reduce) and op fusion onto the in-tree HIP kernels (fuse_gemm_epilogue,
fused_feedforward, fuse_elewise_add_act, fuse_optimizer). The reference's parameter-server
program-splitting passes have no counterpart: the PS here (distributed/ps) serves tables over
RPC from the unmodified program."""
from .pass_base import (PassContext, PassType, PassBase, register_pass, new_pass,  # noqa: F401
                        PassManager, registered_passes)
from . import auto_parallel_passes  # noqa: F401  (registers the passes)
from . import fusion_passes  # noqa: F401

__all__ = ['new_pass', 'PassManager', 'PassContext']
