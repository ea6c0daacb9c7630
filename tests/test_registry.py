"""Kernel registry keys (op, backend, dtype) — parity: paddle/phi/core/kernel_factory.cc
KernelKey selection with a fallback kernel."""
import torch

from paddle_ray_amd.ops import registry as R
from paddle_ray_amd.ops import fused as K  # noqa: F401  (registers the kernels)


def test_dtype_keys_and_fallback():
    R.register_kernel('t_op', 'ref')(lambda x: ('ref', x.dtype))
    R.register_kernel('t_op', 'hip', dtypes=(torch.bfloat16,))(lambda x: ('hip', x.dtype))
    assert R.has_kernel('t_op', 'hip', torch.bfloat16)
    assert not R.has_kernel('t_op', 'hip', torch.float32)
    assert R.get_kernel('t_op', 'ref', torch.float64)(torch.zeros(1))[0] == 'ref'
    tab = R.kernel_table()
    assert tab[('t_op', 'hip')] == ['bfloat16'] and tab[('t_op', 'ref')] == ['any']
    # host tensors always take the ref kernel
    assert R.dispatch('t_op', torch.zeros(1, dtype=torch.bfloat16),
                      torch.zeros(1, dtype=torch.bfloat16))[0] == 'ref'


def test_hot_kernels_declare_dtypes():
    tab = R.kernel_table()
    assert tab[('gemm', 'hip')] == ['bfloat16', 'float16']
    assert tab[('flash_attn_fwd', 'hip')] == ['bfloat16', 'float16']
    assert set(tab[('layer_norm_fwd', 'hip')]) == {'bfloat16', 'float16', 'float32'}
    for op in ('adamw_mt', 'momentum_mt', 'sumsq', 'vp_ce_bwd', 'mmha_decode'):
        assert (op, 'hip') in tab, op
