"""paddle.linalg (parity: python/paddle/linalg.py)."""
from .tensor.linalg import (cholesky, norm, cond, cov, corrcoef, inv, eig, eigvals, multi_dot,  # noqa
                            matrix_rank, svd, qr, lu, lu_unpack, matrix_power, det, slogdet, eigh,
                            eigvalsh, pinv, solve, cholesky_solve, triangular_solve, lstsq,
                            vector_norm, matrix_norm, matrix_exp)
