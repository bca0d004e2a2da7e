"""oneflow_spmm._C — the functional binding `spmm_csr`, mirroring `oneflow._C.spmm_csr`.

Signature (functional YAML entry, pattern oneflow/core/functional/functional_api.yaml:1062-1065):
    "Tensor (Tensor a_csr_row_ptr, Tensor a_csr_col_idx, Tensor a_csr_values,
             Int64 a_num_rows, Int64 a_num_cols, Tensor b) => SpmmCsr"
Tensors are torch tensors (PyTorch-ROCm supplies device memory and streams); the call goes
through the C-ABI into the C++ op registry (oneflow/user/ops/spmm_op.cpp inference, kernel
choice, Compute) and launches the HIP kernel on torch's current stream.  CPU tensors run the
op's DeviceType::kCPU kernel (the reference registers CPU kernels the same way); GPU tensors run
only the HIP kernel — there is no fallback between them.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import LIB, TensorDesc, check

_TORCH_TO_DT = {
    torch.float32: _lib.DT_FLOAT,
    torch.float64: _lib.DT_DOUBLE,
    torch.float16: _lib.DT_FLOAT16,
    torch.bfloat16: _lib.DT_BFLOAT16,
    torch.int32: _lib.DT_INT32,
    torch.int64: _lib.DT_INT64,
}
_DT_TO_TORCH = {v: k for k, v in _TORCH_TO_DT.items()}


def dtype_code(dt: torch.dtype) -> int:
    try:
        return _TORCH_TO_DT[dt]
    except KeyError:
        raise TypeError(f"spmm_csr: unsupported dtype {dt}") from None


def _device_index(t: torch.Tensor) -> int:
    if t.device.type == "cpu":
        return -1
    if t.device.type != "cuda":  # PyTorch-ROCm names HIP devices "cuda"
        raise RuntimeError(f"spmm_csr: unsupported device {t.device}")
    return t.device.index if t.device.index is not None else torch.cuda.current_device()


def _prep(t: torch.Tensor, name: str, matrix: bool = False) -> torch.Tensor:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"spmm_csr: {name} must be a tensor, got {type(t).__name__}")
    if matrix and t.dim() == 2 and t.stride(1) == 1 and t.stride(0) >= t.shape[1]:
        return t  # row-strided views are consumed in place (ldb)
    return t.contiguous()


def desc(t: torch.Tensor) -> TensorDesc:
    d = TensorDesc()
    d.dtype = dtype_code(t.dtype)
    d.device = _device_index(t)
    d.ndim = t.dim()
    if d.ndim > 2:
        raise RuntimeError(f"spmm_csr: tensors must be 1-D or 2-D, got {t.dim()}-D")
    for i in range(t.dim()):
        d.shape[i] = t.shape[i]
        d.stride[i] = t.stride(i)
    d.data = t.data_ptr() if t.numel() > 0 else None
    return d


def current_stream_handle(t: torch.Tensor):
    if t.device.type == "cpu":
        return None
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _placement(_parallel, _placement_nd):
    """(hierarchy dims, out split axis per hierarchy axis, parallel_id, logical N or -1)."""
    if _placement_nd is not None:
        pl = dict(_placement_nd)
        hier = tuple(int(x) for x in pl["hierarchy"])
        axes = tuple(-1 if a in (None, "B") else (int(a[2:-1]) if isinstance(a, str) else int(a))
                     for a in pl["nd_sbp"])
        return hier, axes, int(pl["parallel_id"]), int(pl.get("logical_n", -1))
    if _parallel is None:
        return (1,), (-1,), 0, -1
    pid, pnum, axis = _parallel[:3]
    logical_n = _parallel[3] if len(_parallel) > 3 else -1
    return (int(pnum),), (int(axis),), int(pid), int(logical_n)


def spmm_csr(a_csr_row_ptr: torch.Tensor, a_csr_col_idx: torch.Tensor,
             a_csr_values: torch.Tensor, a_num_rows: int, a_num_cols: int, b: torch.Tensor, *,
             out: torch.Tensor | None = None, _parallel=None, _placement_nd=None,
             num_threads: int = 0, static_csr: int = 0) -> torch.Tensor:
    """out[M, N] = CSR(a_csr_row_ptr, a_csr_col_idx, a_csr_values; M x K) @ b[K, N].

    static_csr (op attr, include/ofx_spmm.h ofx_spmm_attrs): non-zero (True = 1) promises that
    the CSR at these addresses is not rewritten while the process calls the op with this value;
    the HIP kernel's state then plans its work list once and every later call launches planned
    (no planner kernel).  A caller that frees a static CSR and builds another one gives the new
    one another value.  No numeric effect.

    Global form (one rank of a placement; `b` and `out` are this rank's physical tensors):
      `_parallel=(parallel_id, parallel_num, out_split_axis[, logical_n])` for a 1-D placement
      (out_split_axis 0: this rank's BalancedSplitter rows; 1: a column slice of width b.shape[1]
      out of logical_n; -1: broadcast), or
      `_placement_nd=dict(hierarchy=(R, C), nd_sbp=("S(0)", "S(1)"), parallel_id=p, logical_n=N)`
      for an N-D one.  The op's physical inference shapes `out`; the kernel's cache takes the row
      range from out's NdSbp (GetTensorSliceView4ParallelId) and the hub schedule from logical N.
    """
    rp = _prep(a_csr_row_ptr, "a_csr_row_ptr")
    ci = _prep(a_csr_col_idx, "a_csr_col_idx")
    vals = _prep(a_csr_values, "a_csr_values")
    bb = _prep(b, "b", matrix=True)
    d_rp, d_ci, d_v, d_b = desc(rp), desc(ci), desc(vals), desc(bb)
    hier, axes, pid, logical_n = _placement(_parallel, _placement_nd)
    c_hier = (ctypes.c_int64 * len(hier))(*hier)
    c_axes = (ctypes.c_int32 * len(axes))(*axes)
    common = (ctypes.byref(d_rp), ctypes.byref(d_ci), ctypes.byref(d_v), int(a_num_rows),
              int(a_num_cols), ctypes.byref(d_b), logical_n)
    tail = (len(hier), c_hier, c_axes, pid, int(num_threads))
    # Out shape and tmp size depend only on the signature (shapes, dtypes, strides, device,
    # attrs, placement): memoised after the first successful call, as OneFlow's eager path keeps
    # its inferred descs per op signature.  The launch below still runs the full inference.
    key = (tuple(d.shape[i] for d in (d_rp, d_ci, d_v, d_b) for i in range(2)), d_rp.dtype,
           d_ci.dtype, d_v.dtype, d_b.dtype, d_b.stride[0], d_b.device, int(a_num_rows),
           int(a_num_cols), hier, axes, pid, logical_n, int(num_threads))
    memo = _SIG_MEMO.get(key)
    if out is None and memo is not None:
        out = torch.empty(memo[0], dtype=memo[1], device=bb.device)
    if out is None:
        # the physical out of this rank: the op's physical inference, through a dry run on an
        # empty descriptor (tmp size query) would not return the shape, so ask the infer entry
        # for the logical shape and apply the placement like GetPhysicalShape
        od = TensorDesc()
        check(LIB.ofx_functional_spmm_csr_infer(ctypes.byref(d_rp), ctypes.byref(d_ci),
                                                ctypes.byref(d_v), int(a_num_rows), int(a_num_cols),
                                                ctypes.byref(d_b), ctypes.byref(od)), "spmm_csr")
        rows, n = od.shape[0], od.shape[1]
        for i, (h, a) in enumerate(zip(hier, axes)):
            if a == 0 and h > 1 and rows > 0:
                idx = pid
                for hh in hier[i + 1:]:
                    idx //= hh
                lo, hi = balanced_range(rows, h, idx % h)
                rows = hi - lo
        out = torch.empty((rows, n), dtype=_DT_TO_TORCH[od.dtype], device=bb.device)
    d_o = desc(out)
    tmp_bytes = ctypes.c_size_t(0)
    if memo is not None:
        tmp_bytes.value = memo[2]
    else:
        check(LIB.ofx_functional_spmm_csr_global(None, *common, None, None, 0, *tail,
                                                 ctypes.byref(tmp_bytes)), "spmm_csr")
    tmp = None
    if tmp_bytes.value:
        tmp = torch.empty(tmp_bytes.value, dtype=torch.uint8, device=bb.device)
    if static_csr:
        attrs = _lib.SpmmAttrs()
        attrs.static_csr = int(static_csr)
        check(LIB.ofx_functional_spmm_csr_global_attrs(
            current_stream_handle(bb), *common, ctypes.byref(d_o),
            tmp.data_ptr() if tmp is not None else None, tmp_bytes.value, *tail, None,
            ctypes.byref(attrs)), "spmm_csr")
    else:
        check(LIB.ofx_functional_spmm_csr_global(current_stream_handle(bb), *common,
                                                 ctypes.byref(d_o),
                                                 tmp.data_ptr() if tmp is not None else None,
                                                 tmp_bytes.value, *tail, None), "spmm_csr")
    if memo is None and len(_SIG_MEMO) < 4096:
        _SIG_MEMO[key] = (tuple(out.shape), out.dtype, tmp_bytes.value)
    return out


_SIG_MEMO: dict = {}


def static_plans(release: bool = False) -> dict:
    """The static-CSR plans the eager op states hold (ofx_spmm_static_plans): live entries,
    planner launches and calls that reused a plan; release=True frees them first -- the plans
    graph captures used included, so destroy those graphs before releasing."""
    e, p, h = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    check(LIB.ofx_spmm_static_plans(ctypes.byref(e), ctypes.byref(p), ctypes.byref(h),
                                    1 if release else 0), "spmm_static_plans")
    return {"entries": e.value, "plans": p.value, "hits": h.value}


def fused_spmm_csr(a_csr_row_ptr: torch.Tensor, a_csr_col_idx: torch.Tensor,
                   a_csr_values: torch.Tensor, a_num_rows: int, a_num_cols: int, b: torch.Tensor,
                   bias: torch.Tensor | None = None, *, relu: bool = False,
                   out: torch.Tensor | None = None, static_csr: int = 0) -> torch.Tensor:
    """Op "fused_spmm_csr": relu?(A @ b + bias?) in one kernel, the same bits as
    spmm_csr -> bias_add -> relu run separately.  `static_csr` as for
    spmm_csr: the plan of an unchanged CSR is kept in the op's kernel state."""
    rp = _prep(a_csr_row_ptr, "a_csr_row_ptr")
    ci = _prep(a_csr_col_idx, "a_csr_col_idx")
    vals = _prep(a_csr_values, "a_csr_values")
    bb = _prep(b, "b", matrix=True)
    bs = _prep(bias, "bias") if bias is not None else None
    d_rp, d_ci, d_v, d_b = desc(rp), desc(ci), desc(vals), desc(bb)
    d_bias = ctypes.byref(desc(bs)) if bs is not None else None
    od = TensorDesc()
    check(LIB.ofx_functional_spmm_csr_infer(ctypes.byref(d_rp), ctypes.byref(d_ci), ctypes.byref(d_v),
                                            int(a_num_rows), int(a_num_cols), ctypes.byref(d_b),
                                            ctypes.byref(od)), "fused_spmm_csr")
    if out is None:
        out = torch.empty((od.shape[0], od.shape[1]), dtype=_DT_TO_TORCH[od.dtype], device=bb.device)
    d_o = desc(out)
    args = (ctypes.byref(d_rp), ctypes.byref(d_ci), ctypes.byref(d_v), ctypes.byref(d_b), d_bias,
            int(a_num_rows), int(a_num_cols), 1 if relu else 0, ctypes.byref(d_o))
    size = ctypes.c_size_t(0)
    check(LIB.ofx_functional_fused_spmm_csr(None, *args, None, 0, ctypes.byref(size)), "fused_spmm_csr")
    tmp = None
    if size.value and bb.device.type != "cpu":
        tmp = torch.empty(size.value, dtype=torch.uint8, device=bb.device)
    attrs = None
    if static_csr:
        attrs = _lib.SpmmAttrs()
        attrs.static_csr = int(static_csr)
        attrs = ctypes.byref(attrs)
    check(LIB.ofx_functional_fused_spmm_csr_attrs(current_stream_handle(bb), *args,
                                                  tmp.data_ptr() if tmp is not None else None,
                                                  size.value if tmp is not None else 0, None,
                                                  attrs),
          "fused_spmm_csr")
    return out


def _run_grad_op(fn, stream_of, ins, outs, extra, attrs=()):
    """Two-phase call of a functional gradient entry: tmp size, then the run.  `attrs`: trailing
    arguments of an `_attrs` entry (an ofx_spmm_attrs pointer)."""
    size = ctypes.c_size_t(0)
    descs_in = [ctypes.byref(desc(t)) for t in ins]
    descs_out = [ctypes.byref(desc(t)) for t in outs]
    check(fn(None, *descs_in, *extra, *descs_out, None, 0, ctypes.byref(size), *attrs),
          fn.__name__)
    tmp = None
    if size.value:  # the op's tmp_buffer, on the op's device (host memory for kCPU kernels)
        tmp = torch.empty(size.value, dtype=torch.uint8, device=stream_of.device)
    check(fn(current_stream_handle(stream_of), *descs_in, *extra, *descs_out,
             tmp.data_ptr() if tmp is not None else None, size.value if tmp is not None else 0,
             None, *attrs), fn.__name__)


def sddmm_csr(a_csr_row_ptr: torch.Tensor, a_csr_col_idx: torch.Tensor, a: torch.Tensor,
              b: torch.Tensor, a_num_rows: int, a_num_cols: int, *,
              static_csr: int = 0) -> torch.Tensor:
    """out[j] = <a[row(j), :], b[col(j), :]> (op "sddmm_csr": the values-gradient of spmm_csr).
    `static_csr` as for spmm_csr: the SDDMM's plan of an unchanged CSR is kept."""
    rp, ci = _prep(a_csr_row_ptr, "a_csr_row_ptr"), _prep(a_csr_col_idx, "a_csr_col_idx")
    a, b = _prep(a, "a", matrix=True), _prep(b, "b", matrix=True)
    if b.dim() == 2 and b.shape[1] == 0:  # empty inner dimension: every dot product is 0
        out = torch.zeros(ci.numel(), dtype=b.dtype, device=b.device)
    else:
        out = torch.empty(ci.numel(), dtype=b.dtype, device=b.device)
    if b.dim() == 2 and b.shape[1] == 0 and a.dim() == 2 and a.shape[1] == 0:
        return out
    if static_csr:
        attrs = _lib.SpmmAttrs()
        attrs.static_csr = int(static_csr)
        _run_grad_op(LIB.ofx_functional_sddmm_csr_attrs, b, [rp, ci, a, b], [out],
                     [int(a_num_rows), int(a_num_cols)], (ctypes.byref(attrs),))
    else:
        _run_grad_op(LIB.ofx_functional_sddmm_csr, b, [rp, ci, a, b], [out],
                     [int(a_num_rows), int(a_num_cols)])
    return out


def spmm_csr_gathered(a_csr_row_ptr: torch.Tensor, a_csr_col_idx: torch.Tensor,
                      a_csr_values: torch.Tensor, values_perm: torch.Tensor, a_num_rows: int,
                      a_num_cols: int, b: torch.Tensor, *, out: torch.Tensor | None = None,
                      static_csr: int = 0):
    """Op "spmm_csr_gathered": A @ b with nonzero j's value a_csr_values[values_perm[j]] (the
    d(b) gradient of spmm_csr with learnable values: A^T's structure, A's values, A^T's perm).
    `static_csr` as for spmm_csr (the autograd's cached A^T passes its entry's value)."""
    rp, ci = _prep(a_csr_row_ptr, "a_csr_row_ptr"), _prep(a_csr_col_idx, "a_csr_col_idx")
    vals, perm = _prep(a_csr_values, "a_csr_values"), _prep(values_perm, "values_perm")
    bb = _prep(b, "b", matrix=True)
    if out is None:
        out = torch.empty((int(a_num_rows), bb.shape[1] if bb.dim() == 2 else 0), dtype=bb.dtype,
                          device=bb.device)
    if out.numel() == 0:
        return out
    if static_csr:
        attrs = _lib.SpmmAttrs()
        attrs.static_csr = int(static_csr)
        _run_grad_op(LIB.ofx_functional_spmm_csr_gathered_attrs, bb, [rp, ci, vals, perm, bb],
                     [out], [int(a_num_rows), int(a_num_cols)], (ctypes.byref(attrs),))
    else:
        _run_grad_op(LIB.ofx_functional_spmm_csr_gathered, bb, [rp, ci, vals, perm, bb], [out],
                     [int(a_num_rows), int(a_num_cols)])
    return out


def csr_transpose(a_csr_row_ptr: torch.Tensor, a_csr_col_idx: torch.Tensor, a_num_rows: int,
                  a_num_cols: int):
    """Structure of A^T (op "csr_transpose"): (row_ptr [K+1], col_idx [nnz], perm [nnz])."""
    rp, ci = _prep(a_csr_row_ptr, "a_csr_row_ptr"), _prep(a_csr_col_idx, "a_csr_col_idx")
    it, dev = rp.dtype, rp.device
    rp_t = torch.empty(int(a_num_cols) + 1, dtype=it, device=dev)
    ci_t = torch.empty(ci.numel(), dtype=it, device=dev)
    perm = torch.empty(ci.numel(), dtype=it, device=dev)
    _run_grad_op(LIB.ofx_functional_csr_transpose, rp, [rp, ci], [rp_t, ci_t, perm],
                 [int(a_num_rows), int(a_num_cols)])
    return rp_t, ci_t, perm


def balanced_range(total: int, parts: int, idx: int) -> tuple[int, int]:
    lo, hi = ctypes.c_int64(), ctypes.c_int64()
    check(LIB.ofx_balanced_range(total, parts, idx, ctypes.byref(lo), ctypes.byref(hi)),
          "balanced_range")
    return lo.value, hi.value


def sbp_signatures(op: str = "spmm_csr", optional_inputs: str = "") -> str:
    buf = ctypes.create_string_buffer(4096)
    check(LIB.ofx_op_sbp_signatures(op.encode(), optional_inputs.encode(), buf, len(buf)), "sbp")
    return buf.value.decode()
