"""COO (edge_index) -> CSR construction: HIP kernels on GPU tensors
(csrc/csr_build.hip: stable radix sort + run merge + row_ptr by search), the C++ host version on
CPU tensors; both give the same arrays and the same summed values."""
from __future__ import annotations

import ctypes

import torch

from ._C import current_stream_handle, dtype_code
from ._lib import LIB, check


def coo_to_csr(row: torch.Tensor, col: torch.Tensor, values: torch.Tensor | None, m: int, k: int,
               merge_duplicates: bool = True):
    """Returns (row_ptr [m+1], col_idx [nnz'], values [nnz'] or None) in canonical CSR order.
    Duplicates (same row and col) are summed in input order when merge_duplicates."""
    if row.shape != col.shape or row.dim() != 1:
        raise RuntimeError("coo_to_csr: row and col must be 1-D tensors of equal length")
    if row.dtype != col.dtype:
        raise TypeError("coo_to_csr: row and col must have the same index dtype")
    row, col = row.contiguous(), col.contiguous()
    nnz = row.numel()
    it, dev = row.dtype, row.device
    idt = dtype_code(it)
    vdt = dtype_code(values.dtype) if values is not None else dtype_code(torch.float32)
    if values is not None:
        values = values.contiguous()
        if values.shape != row.shape:
            raise RuntimeError("coo_to_csr: values must match row/col")
    out_rp = torch.empty(m + 1, dtype=it, device=dev)
    out_ci = torch.empty(nnz, dtype=it, device=dev)
    out_v = torch.empty(nnz, dtype=values.dtype, device=dev) if values is not None else None
    ptr = lambda t: t.data_ptr() if t is not None and t.numel() else None  # noqa: E731
    if dev.type == "cpu":
        cnt = ctypes.c_int64(0)
        check(LIB.ofx_coo_to_csr_cpu(idt, vdt, m, k, nnz, ptr(row), ptr(col), ptr(values),
                                     int(merge_duplicates), out_rp.data_ptr(), ptr(out_ci),
                                     ptr(out_v), ctypes.byref(cnt)), "coo_to_csr")
        n_out = cnt.value
    else:
        ws_bytes = ctypes.c_size_t(0)
        check(LIB.ofx_coo_to_csr_workspace_size(idt, m, k, nnz, ctypes.byref(ws_bytes)), "coo_to_csr")
        ws = torch.empty(max(ws_bytes.value, 1), dtype=torch.uint8, device=dev)
        scalars = torch.zeros(2, dtype=torch.int64, device=dev)  # [nnz', bad flag]
        check(LIB.ofx_coo_to_csr(current_stream_handle(row), idt, vdt, m, k, nnz, ptr(row), ptr(col),
                                 ptr(values), int(merge_duplicates), out_rp.data_ptr(), ptr(out_ci),
                                 ptr(out_v), scalars.data_ptr(), scalars.data_ptr() + 8,
                                 ws.data_ptr(), ws_bytes.value), "coo_to_csr")
        n_out, bad = (int(x) for x in scalars.tolist())
        if bad:
            raise RuntimeError(f"coo_to_csr: entries outside the {m} x {k} matrix")
    return out_rp, out_ci[:n_out], (out_v[:n_out] if out_v is not None else None)
