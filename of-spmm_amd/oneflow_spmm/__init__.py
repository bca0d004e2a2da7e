"""oneflow_spmm — MI355X-native `spmm_csr` operator with OneFlow's user-op surface.

    import oneflow_spmm as flow_spmm
    out = flow_spmm.spmm(row_ptr, col_idx, values, num_rows, num_cols, b)   # oneflow.spmm
    out = flow_spmm._C.spmm_csr(...)                                          # oneflow._C.spmm_csr
`spmm` is differentiable in the values and in b (autograd.py: SDDMM and A^T @ dC).
Graph mode (UserKernel's CUDA-graph branch) is the compiled job's native hipGraph executable:
`ccl.SpmmJob(..., graph=True)` over `ofx_spmm_job_set_graph`.

Re-exports mirror python/oneflow/__init__.py:158-160 (`from oneflow._C import ... as mv`).
"""
from . import _C, _lib, autograd, build, ops, synth  # noqa: F401
from ._C import spmm_csr
from ._lib import OfxError
from .autograd import csr_transpose, fused_spmm, sddmm, spmm
from .build import coo_to_csr

__version__ = _lib.LIB.ofx_version().decode()

__all__ = ["spmm", "fused_spmm", "spmm_csr", "sddmm", "csr_transpose", "OfxError", "ops", "synth", "autograd", "coo_to_csr", "_C"]
