"""Direct C-ABI entry points (below the op layer): the device kernel with explicit schedule
options and workspace, the CPU kernel, CSR validation and row slicing.  Used by the row-split
wrapper, the benchmark and the parity tests; `oneflow_spmm.spmm` is the op-level API.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._C import current_stream_handle, dtype_code
from ._lib import LIB, Options, check

INT64_MAX = (1 << 63) - 1


def make_options(split: int = 0, chunk: int = 0, ordered: bool = False, variant: int = 0,
                 heavy: int = 0, planned: bool = False, range_nnz: int = 0) -> Options:
    """heavy: rows longer than this (not split) are scheduled first; 0 = default, <0 = off.
    planned: the workspace holds ofx_spmm_csr_plan's work list (see SpmmCsrKernel.plan).
    range_nnz: the launch's row range holds this many nonzeros (0 = estimated as its share of
    nnz); picks the kernel form only."""
    return Options(int(split), int(chunk), 1 if ordered else 0, int(variant), int(heavy),
                   1 if planned else 0, 0, int(range_nnz))


def _with(o: Options | None, **fields) -> Options:
    """A copy of options `o` (None: the defaults) with `fields` replaced."""
    c = Options()
    if o is not None:
        ctypes.memmove(ctypes.addressof(c), ctypes.addressof(o), ctypes.sizeof(Options))
    for key, val in fields.items():
        setattr(c, key, val)
    return c


def default_split(n: int) -> int:
    return int(LIB.ofx_spmm_default_split(int(n)))


def workspace_size(idx_dtype: torch.dtype, val_dtype: torch.dtype, m: int, k: int, n: int, nnz: int,
                   options: Options | None = None) -> int:
    out = ctypes.c_size_t(0)
    check(LIB.ofx_spmm_csr_workspace_size(dtype_code(idx_dtype), dtype_code(val_dtype), m, k, n, nnz,
                                          ctypes.byref(options) if options else None,
                                          ctypes.byref(out)), "workspace_size")
    return out.value


class SpmmCsrKernel:
    """Holds the workspace for repeated launches of one problem shape (the OneFlow tmp buffer).

    plan(row_ptr, row_begin, row_end) builds the work list once (ofx_spmm_csr_plan) for a static
    graph; launches with planned=True on that same row_ptr tensor and row range then skip the
    planning kernel.  The caller promises row_ptr's contents have not changed (a bound
    CSR); the tensor identity and range are checked here."""

    def __init__(self, m: int, k: int, n: int, nnz: int, idx_dtype: torch.dtype,
                 val_dtype: torch.dtype, device, options: Options | None = None):
        self.m, self.k, self.n, self.nnz = m, k, n, nnz
        self.idx_dt, self.val_dt = dtype_code(idx_dtype), dtype_code(val_dtype)
        self.options = options
        ws = workspace_size(idx_dtype, val_dtype, m, k, n, nnz, options)
        self.workspace = torch.empty(max(ws, 1), dtype=torch.uint8, device=device)
        self.ws_bytes = ws
        self._planned_for = None
        self._planned_opts = None

    def plan(self, row_ptr, row_begin=0, row_end=None, stream=None, range_nnz: int = 0):
        row_end = self.m if row_end is None else row_end
        s = stream if stream is not None else current_stream_handle(row_ptr)
        o = _with(self.options, range_nnz=int(range_nnz)) if range_nnz else self.options
        check(LIB.ofx_spmm_csr_plan(s, self.idx_dt, self.val_dt, self.m, self.k, self.n, self.nnz,
                                    row_ptr.data_ptr(), row_begin, row_end,
                                    self.workspace.data_ptr(), self.ws_bytes,
                                    ctypes.byref(o) if o else None),
              "spmm_csr_plan")
        self._planned_opts = _with(o, planned=1)
        self._planned_for = (row_ptr.data_ptr(), row_ptr.numel(), row_begin, row_end, int(range_nnz))
        return self

    def launch_options(self, row_ptr, row_begin, row_end, planned: bool, range_nnz: int = 0):
        """The options struct of one launch (the planned form after a matching plan())."""
        if not planned:
            return _with(self.options, range_nnz=int(range_nnz)) if range_nnz else self.options
        if self._planned_for != (row_ptr.data_ptr(), row_ptr.numel(), row_begin, row_end,
                                 int(range_nnz)):
            raise RuntimeError("SpmmCsrKernel: planned launch without a plan() of this row_ptr, "
                               "row range and range_nnz")
        return self._planned_opts

    def __call__(self, row_ptr, col_idx, values, b, out, row_begin=0, row_end=None, stream=None,
                 bias=None, relu=False, planned: bool = False, range_nnz: int = 0):
        """bias / relu: the fused epilogue (ofx_spmm_csr_fused); none = the plain op.
        range_nnz: nonzeros of [row_begin, row_end) if known (the form choice; 0 = estimated)."""
        row_end = self.m if row_end is None else row_end
        s = stream if stream is not None else current_stream_handle(b)
        opts = self.launch_options(row_ptr, row_begin, row_end, planned, range_nnz)
        check(LIB.ofx_spmm_csr_fused(s, self.idx_dt, self.val_dt, self.m, self.k, self.n, self.nnz,
                                     row_ptr.data_ptr(), col_idx.data_ptr() if col_idx.numel() else None,
                                     values.data_ptr() if values.numel() else None,
                                     b.data_ptr() if b.numel() else None, b.stride(0), out.data_ptr(),
                                     out.stride(0), row_begin, row_end,
                                     bias.data_ptr() if bias is not None else None, 1 if relu else 0,
                                     self.workspace.data_ptr(), self.ws_bytes,
                                     ctypes.byref(opts) if opts else None),
              "spmm_csr")
        return out


def spmm_csr_device(row_ptr, col_idx, values, b, m, k, *, out=None, row_begin=0, row_end=None,
                    options: Options | None = None):
    """One launch of the HIP kernel (C-ABI ofx_spmm_csr) on torch's current stream."""
    if b.device.type != "cuda":
        raise RuntimeError("spmm_csr_device: HIP kernel needs device tensors")
    row_end = m if row_end is None else row_end
    if out is None:
        out = torch.empty((row_end - row_begin, b.shape[1]), dtype=b.dtype, device=b.device)
    kern = SpmmCsrKernel(m, k, b.shape[1], col_idx.numel(), row_ptr.dtype, b.dtype, b.device, options)
    return kern(row_ptr, col_idx, values, b, out, row_begin, row_end)


def describe(m: int, k: int, n: int, nnz: int, val_dtype: torch.dtype,
             idx_dtype: torch.dtype = torch.int32, *, row_begin: int = 0, row_end: int | None = None,
             ldb: int | None = None, ldc: int | None = None, b_addr: int = 256, c_addr: int = 256,
             options: Options | None = None) -> dict:
    """The configuration an ofx_spmm_csr launch with these arguments takes (ofx_spmm_csr_describe):
    {"form": "small"|"mid"|"narrow"|"prefetch"|"bandwidth", "kernel": ..., "VEC": .., "LPR": ..,
    "U": .., flags ...}.  Nothing is launched; b_addr / c_addr only set the pointer alignment the
    width dispatch sees (256: aligned)."""
    row_end = m if row_end is None else row_end
    buf = ctypes.create_string_buffer(512)
    check(LIB.ofx_spmm_csr_describe(dtype_code(idx_dtype), dtype_code(val_dtype), m, k, n, nnz,
                                    b_addr, ldb or n, c_addr, ldc or n, row_begin, row_end,
                                    ctypes.byref(options) if options else None, buf, len(buf)),
          "spmm_csr_describe")
    out = {}
    for kv in buf.value.decode().split():
        key, val = kv.split("=")
        out[key] = int(val) if val.lstrip("-").isdigit() else val
    return out


def spmm_csr_gathered(row_ptr, col_idx, values, values_perm, b, m, k, *, out=None,
                      options: Options | None = None):
    """out = A @ b where nonzero j's value is values[values_perm[j]] (ofx_spmm_csr_gathered):
    the backward's A^T @ d(out) on A's values without writing values[perm].  Same bits as
    spmm_csr on the gathered values."""
    if b.device.type != "cuda":
        return spmm_csr_cpu(row_ptr, col_idx, values[values_perm.long()], b, m, k, out=out,
                            options=options)
    if values_perm.dtype != row_ptr.dtype or values_perm.numel() != col_idx.numel():
        raise RuntimeError("spmm_csr_gathered: values_perm must be [nnz] in the index dtype")
    if out is None:
        out = torch.empty((m, b.shape[1]), dtype=b.dtype, device=b.device)
    n, nnz = b.shape[1], col_idx.numel()
    ws = workspace_size(row_ptr.dtype, b.dtype, m, k, n, nnz, options)
    wbuf = torch.empty(max(ws, 1), dtype=torch.uint8, device=b.device)
    nz = lambda t: t.data_ptr() if t.numel() else None  # noqa: E731
    check(LIB.ofx_spmm_csr_gathered(current_stream_handle(b), dtype_code(row_ptr.dtype),
                                    dtype_code(b.dtype), m, k, n, nnz, row_ptr.data_ptr(),
                                    nz(col_idx), nz(values), nz(values_perm), nz(b), b.stride(0),
                                    out.data_ptr(), out.stride(0), 0, m, wbuf.data_ptr(), ws,
                                    ctypes.byref(options) if options else None),
          "spmm_csr_gathered")
    return out


def relu_bias_grad(y, dy, *, relu: bool, bias_grad: bool, num_threads: int = 0):
    """Backward of the fused epilogue (ofx_relu_bias_grad[_cpu]): returns (dx, d_bias).
    dx = relu ? where(y > 0, dy, 0) : dy (dy itself when relu is off); d_bias = column sum of dx
    in the contract's fixed order, or None."""
    m, n = dy.shape
    dt = dtype_code(dy.dtype)
    dx = torch.empty_like(dy) if relu else dy
    db = torch.empty(n, dtype=dy.dtype, device=dy.device) if bias_grad else None
    if not relu and not bias_grad:
        return dx, db
    nz = lambda t: t.data_ptr() if t is not None and t.numel() else None  # noqa: E731
    yy = y if relu else None
    args = (m, n, nz(yy), yy.stride(0) if yy is not None else n, nz(dy), dy.stride(0),
            nz(dx) if relu else None, dx.stride(0) if relu else n, nz(db), 1 if relu else 0)
    if dy.device.type == "cpu":
        check(LIB.ofx_relu_bias_grad_cpu(int(num_threads), dt, *args), "relu_bias_grad")
        return dx, db
    size = ctypes.c_size_t(0)
    check(LIB.ofx_relu_bias_grad_workspace_size(dt, m, n, ctypes.byref(size)), "relu_bias_grad")
    ws = torch.empty(max(size.value, 1), dtype=torch.uint8, device=dy.device)
    check(LIB.ofx_relu_bias_grad(current_stream_handle(dy), dt, *args, ws.data_ptr(), size.value),
          "relu_bias_grad")
    return dx, db


def spmm_csr_cpu(row_ptr, col_idx, values, b, m, k, *, out=None, row_begin=0, row_end=None,
                 options: Options | None = None, num_threads: int = 0, bias=None, relu=False):
    """The DeviceType::kCPU kernel (C-ABI ofx_spmm_csr_fused_cpu), host tensors."""
    row_end = m if row_end is None else row_end
    if out is None:
        out = torch.empty((row_end - row_begin, b.shape[1]), dtype=b.dtype)
    check(LIB.ofx_spmm_csr_fused_cpu(int(num_threads), dtype_code(row_ptr.dtype), dtype_code(b.dtype),
                                     m, k, b.shape[1], col_idx.numel(), row_ptr.data_ptr(),
                                     col_idx.data_ptr() if col_idx.numel() else None,
                                     values.data_ptr() if values.numel() else None,
                                     b.data_ptr() if b.numel() else None, b.stride(0), out.data_ptr(),
                                     out.stride(0), row_begin, row_end,
                                     bias.data_ptr() if bias is not None else None, 1 if relu else 0,
                                     ctypes.byref(options) if options else None), "spmm_csr_cpu")
    return out


def validate_csr(row_ptr, col_idx, m, k) -> int:
    """Device-side CSR check; returns 0 ok, 1 bad row_ptr, 2 column out of range (syncs)."""
    flag = torch.zeros(1, dtype=torch.int32, device=row_ptr.device)
    check(LIB.ofx_csr_validate(current_stream_handle(row_ptr), dtype_code(row_ptr.dtype), m, k,
                               col_idx.numel(), row_ptr.data_ptr(),
                               col_idx.data_ptr() if col_idx.numel() else None, flag.data_ptr()),
          "csr_validate")
    return int(flag.item())


def csr_row_slice(row_ptr, row_begin: int, row_end: int):
    """Rebased row_ptr of rows [row_begin, row_end) (+ the nnz range it covers)."""
    out = torch.empty(row_end - row_begin + 1, dtype=row_ptr.dtype, device=row_ptr.device)
    if row_ptr.device.type == "cpu":
        lo, hi = ctypes.c_int64(), ctypes.c_int64()
        check(LIB.ofx_csr_row_slice_host(dtype_code(row_ptr.dtype), row_ptr.data_ptr(), row_begin,
                                         row_end, out.data_ptr(), ctypes.byref(lo), ctypes.byref(hi)),
              "csr_row_slice")
        return out, lo.value, hi.value
    check(LIB.ofx_csr_row_slice(current_stream_handle(row_ptr), dtype_code(row_ptr.dtype),
                                row_ptr.data_ptr(), row_begin, row_end, out.data_ptr()),
          "csr_row_slice")
    return out, None, None


__all__ = ["make_options", "default_split", "workspace_size", "SpmmCsrKernel", "spmm_csr_device",
           "describe",
           "spmm_csr_gathered",
           "spmm_csr_cpu", "validate_csr", "csr_row_slice", "INT64_MAX", "_lib"]
