"""Docstrings of oneflow.spmm / oneflow._C.fused_spmm_csr, in the add_docstr form of
python/oneflow/framework/docstr/math_ops.py (oneflow.mv, :1306).  A maintainer appends these
entries to math_ops.py; this file is not imported here (OneFlow is not installed)."""
import oneflow
from oneflow.framework.docstr.utils import add_docstr

add_docstr(
    oneflow.spmm,
    r"""
    spmm(a_csr_row_ptr, a_csr_col_idx, a_csr_values, a_num_rows, a_num_cols, b, static_csr=0) -> Tensor

    Multiplies the sparse matrix :math:`A` (:attr:`a_num_rows` :math:`\times` :attr:`a_num_cols`,
    CSR) by the dense matrix :attr:`b` (:attr:`a_num_cols` :math:`\times N`):
    :math:`out[r, :] = \sum_{j=rp[r]}^{rp[r+1]-1} values[j] \cdot b[col[j], :]`, summed in
    ascending :math:`j` (the order of gather -> multiply -> unsorted_segment_sum).

    Rows with more than ``T = clamp(65536 / N, 128, 512)`` nonzeros (rounded down to a power of
    two: 512 for N <= 128, 256 at N = 256, 128 from N = 512) are summed in chunks of ``T``
    nonzeros, the last chunk taking the remainder, and the chunk sums are then added in chunk
    order; the result is deterministic and identical on CPU and GPU.

    Column indices outside ``[0, a_num_cols)``: a column ``>= a_num_cols`` contributes
    ``value * 0`` in its place of the order (the gather's zero fill) on every device; a negative
    column raises on the CPU (the gather's CHECK) and contributes ``value * 0`` on the GPU (the
    CUDA gather's zero fill of any index outside the table).

    Args:
        a_csr_row_ptr (oneflow.Tensor): int32 or int64, shape ``[a_num_rows + 1]``
        a_csr_col_idx (oneflow.Tensor): same dtype as ``a_csr_row_ptr``, shape ``[nnz]``
        a_csr_values (oneflow.Tensor): float, double, float16 or bfloat16, shape ``[nnz]``
        a_num_rows (int): M
        a_num_cols (int): K
        b (oneflow.Tensor): dtype of ``a_csr_values``, shape ``[K, N]``
        static_csr (int, optional): 0 (default) plans the row work list on every call.  A non-zero
            value promises that the CSR tensors are not modified while calls carry that value;
            the GPU kernel then keeps the plan in its state and later calls skip the planning
            kernel.  Give a new CSR built in reused memory a new value.  No numeric effect.
    Returns:
        oneflow.Tensor: shape ``[M, N]``, dtype of ``b``

    Differentiable in ``a_csr_values`` (SDDMM) and ``b`` (:math:`A^T \cdot grad`).

    For example:

    .. code-block:: python

        >>> import oneflow as flow
        >>> row_ptr = flow.tensor([0, 2, 3], dtype=flow.int32)
        >>> col_idx = flow.tensor([0, 2, 1], dtype=flow.int32)
        >>> values = flow.tensor([1.0, 2.0, 3.0])
        >>> b = flow.tensor([[1.0, 0.0], [0.0, 1.0], [1.0, 1.0]])
        >>> flow.spmm(row_ptr, col_idx, values, 2, 3, b)
        tensor([[3., 2.],
                [0., 3.]], dtype=oneflow.float32)

    """,
)

add_docstr(
    oneflow._C.fused_spmm_csr,
    r"""
    fused_spmm_csr(a_csr_row_ptr, a_csr_col_idx, a_csr_values, a_num_rows, a_num_cols, b, bias=None, relu=False, static_csr=0) -> Tensor

    ``relu(spmm(...) + bias)`` in one kernel, with the bits of the three ops run separately
    (spmm, then bias_add over dim 1, then relu). ``bias`` has shape ``[N]``. ``static_csr`` as
    for ``oneflow.spmm``: a non-zero value keeps the plan of an unchanged CSR across calls.
    """,
)
