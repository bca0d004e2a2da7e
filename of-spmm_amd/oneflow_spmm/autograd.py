"""Gradients of `spmm_csr`: d(values) by SDDMM, d(b) by SpMM with A^T.

Mirrors what a OneFlow gradient function for the op would do (pattern
oneflow/core/autograd/gradient_funcs/matrix_vector_product.cpp:26-91: capture what the backward
needs, then call the grad functors): for out = A @ b,
    d(values)[j] = <d(out)[row(j), :], b[col(j), :]>      ofx_sddmm_csr
    d(b)         = A^T @ d(out)                            ofx_csr_transpose (cached per graph)
                                                           + ofx_spmm_csr_gathered (values read
                                                           through perm), or ofx_gather_values
                                                           once + ofx_spmm_csr for constant values
The index inputs never get gradients (spmm_op.cpp ModifyInputArg).  All device work runs in the
HIP kernels; CPU tensors run the kCPU kernels.  Both give the same bits (contracts in
include/ofx_spmm.h).
"""
from __future__ import annotations

from collections import OrderedDict

import torch

from . import _C, ops
from ._C import current_stream_handle, dtype_code, spmm_csr
from ._lib import LIB, check


# ---- building blocks ----------------------------------------------------------------------------
def csr_transpose(row_ptr: torch.Tensor, col_idx: torch.Tensor, k: int):
    """Structure of A^T: (row_ptr_T [k+1], col_idx_T [nnz] = rows of A, perm [nnz]).
    Op "csr_transpose" through the op layer (CPU or HIP kernel by device)."""
    return _C.csr_transpose(row_ptr, col_idx, row_ptr.numel() - 1, k)


def gather_values(perm: torch.Tensor, values: torch.Tensor) -> torch.Tensor:
    """values[perm] (device kernel on GPU)."""
    if values.device.type == "cpu":
        return values[perm.long()]
    out = torch.empty_like(values)
    check(LIB.ofx_gather_values(current_stream_handle(values), dtype_code(perm.dtype),
                                dtype_code(values.dtype), values.numel(),
                                perm.data_ptr() if perm.numel() else None,
                                values.data_ptr() if values.numel() else None,
                                out.data_ptr() if out.numel() else None), "gather_values")
    return out


def sddmm(row_ptr: torch.Tensor, col_idx: torch.Tensor, a: torch.Tensor, b: torch.Tensor,
          static_csr: int = 0) -> torch.Tensor:
    """out[j] = <a[row(j), :], b[col_idx[j], :]>: op "sddmm_csr" through the op layer
    (`static_csr`: the forward's promise that the CSR is unchanged; its SDDMM plan is kept)."""
    return _C.sddmm_csr(row_ptr, col_idx, a, b, row_ptr.numel() - 1, b.shape[0],
                        static_csr=static_csr)


# ---- transpose cache (the sparsity pattern of a GNN graph is static across layers/steps) -------
class _TransposeCache:
    def __init__(self, capacity: int = 4):
        self.capacity = capacity
        self.static_ids: dict = {}  # id(row_ptr_T) -> its static_csr value (while cached)
        self._next_id = 1 << 40  # clear of the small values callers pass
        self.entries: OrderedDict = OrderedDict()
        self.value_entries: OrderedDict = OrderedDict()
        self.seen: OrderedDict = OrderedDict()  # value keys met once (not yet worth a copy)

    def get(self, row_ptr, col_idx, k):
        key = (row_ptr.data_ptr(), col_idx.data_ptr(), row_ptr._version, col_idx._version,
               row_ptr.numel(), col_idx.numel(), k, str(row_ptr.device))
        hit = self.entries.get(key)
        if hit is not None:
            self.entries.move_to_end(key)
            return hit[2]
        t = csr_transpose(row_ptr, col_idx, k)
        # keep the source tensors alive so their storage (and so the key) cannot be reused; the
        # entry's A^T is static while it lives, so its SpMMs run with static_csr = a value no
        # other entry ever had (a later transpose at recycled addresses gets a new one)
        self._next_id += 1
        self.static_ids[id(t[0])] = self._next_id
        self.entries[key] = (row_ptr, col_idx, t)
        while len(self.entries) > self.capacity:
            _, (_, _, old) = self.entries.popitem(last=False)
            self.static_ids.pop(id(old[0]), None)
        return t

    def static_id(self, rp_t) -> int:
        """The static_csr value of a cached A^T (0 if it is not cached any more)."""
        return self.static_ids.get(id(rp_t), 0)


    def values_t(self, row_ptr, col_idx, values, k):
        """A^T's values = values[perm].  Edge weights of a GNN (e.g. GCN normalisation) are
        usually constant across steps, so the gathered copy is kept too, keyed on the values
        tensor's storage and version (an in-place update invalidates it)."""
        rp_t, ci_t, perm = self.get(row_ptr, col_idx, k)
        key = (row_ptr.data_ptr(), col_idx.data_ptr(), row_ptr._version, col_idx._version, k,
               values.data_ptr(), values._version, values.dtype, values.numel(), str(values.device))
        hit = self.value_entries.get(key)
        if hit is not None:
            self.value_entries.move_to_end(key)
            return rp_t, ci_t, hit[1]
        vals_t = gather_values(perm, values)
        self.value_entries[key] = (values, vals_t)  # holds values: its storage cannot be reused
        while len(self.value_entries) > self.capacity:
            self.value_entries.popitem(last=False)
        return rp_t, ci_t, vals_t


    def grad_b(self, row_ptr, col_idx, values, m, k, d_out):
        """d(b) = A^T @ d(out).  Values met for the first time (e.g. learnable edge weights,
        new every step) are read through the transpose's perm inside the SpMM
        (ofx_spmm_csr_gathered: no values[perm] copy written); values met again unchanged
        (constant GCN weights) are gathered once and cached, then the plain SpMM runs on them.
        Every route gives the same bits."""
        rp_t, ci_t, perm = self.get(row_ptr, col_idx, k)
        key = (row_ptr.data_ptr(), col_idx.data_ptr(), row_ptr._version, col_idx._version, k,
               values.data_ptr(), values._version, values.dtype, values.numel(), str(values.device))
        if key not in self.value_entries and values.device.type == "cuda" and key not in self.seen:
            self.seen[key] = values  # holds values: its storage cannot be reused under the key
            while len(self.seen) > self.capacity:
                self.seen.popitem(last=False)
            # the cached A^T's structure is static while its entry lives: its plan is kept too
            return _C.spmm_csr_gathered(rp_t, ci_t, values, perm, k, m, d_out,
                                        static_csr=self.static_id(rp_t))
        _, _, vals_t = self.values_t(row_ptr, col_idx, values, k)
        # the cached A^T: its plan is kept across steps (static_csr, a value unique to the entry)
        return spmm_csr(rp_t, ci_t, vals_t, k, m, d_out, static_csr=self.static_id(rp_t))


TRANSPOSE_CACHE = _TransposeCache()


class SpmmCsrFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, row_ptr, col_idx, values, m, k, b, static_csr=0):
        out = spmm_csr(row_ptr, col_idx, values, m, k, b, static_csr=static_csr)
        ctx.save_for_backward(row_ptr, col_idx, values, b)
        ctx.m, ctx.k, ctx.static_csr = m, k, static_csr
        return out

    @staticmethod
    def backward(ctx, d_out):
        row_ptr, col_idx, values, b = ctx.saved_tensors
        d_out = d_out.contiguous()
        d_values = d_b = None
        if ctx.needs_input_grad[2]:
            d_values = sddmm(row_ptr, col_idx, d_out, b, ctx.static_csr)
        if ctx.needs_input_grad[5]:
            d_b = TRANSPOSE_CACHE.grad_b(row_ptr, col_idx, values.detach(), ctx.m, ctx.k, d_out)
        return None, None, d_values, None, None, d_b, None


def spmm(a_csr_row_ptr, a_csr_col_idx, a_csr_values, a_num_rows, a_num_cols, b, *, out=None,
         static_csr=0):
    """`oneflow.spmm` with autograd: differentiable in `a_csr_values` and `b`.
    `out=` (a preallocated result) is only accepted when no gradient is being recorded.
    `static_csr` (op attr; True = 1): the CSR is not rewritten while calls carry this value, so
    the forward plans its work list once (_C.spmm_csr)."""
    if torch.is_grad_enabled() and (a_csr_values.requires_grad or b.requires_grad):
        if out is not None:
            raise RuntimeError("spmm: out= is not supported when gradients are required")
        return SpmmCsrFunction.apply(a_csr_row_ptr, a_csr_col_idx, a_csr_values, int(a_num_rows),
                                     int(a_num_cols), b, int(static_csr))
    return spmm_csr(a_csr_row_ptr, a_csr_col_idx, a_csr_values, a_num_rows, a_num_cols, b, out=out,
                    static_csr=int(static_csr))


class FusedSpmmCsrFunction(torch.autograd.Function):
    """relu?(A @ b + bias?).  Backward as the unfused graph's: relu_grad from the output
    (dy where y > 0, oneflow/core/autograd/gradient_funcs/activation.cpp:195-205), bias_add
    grad = column sum of the masked gradient (gradient_funcs/bias_add.cpp:62), then the
    spmm_csr gradients."""

    @staticmethod
    def forward(ctx, row_ptr, col_idx, values, m, k, b, bias, relu, static_csr=0):
        out = _C.fused_spmm_csr(row_ptr, col_idx, values, m, k, b, bias, relu=relu,
                                static_csr=static_csr)
        ctx.save_for_backward(row_ptr, col_idx, values, b, out if relu else None)
        ctx.m, ctx.k, ctx.relu, ctx.has_bias = m, k, relu, bias is not None
        ctx.static_csr = static_csr
        return out

    @staticmethod
    def backward(ctx, d_out):
        row_ptr, col_idx, values, b, out = ctx.saved_tensors
        # relu_grad and the bias column sum in one HIP pass (ofx_relu_bias_grad)
        g, d_bias = ops.relu_bias_grad(out, d_out.contiguous(), relu=ctx.relu,
                                       bias_grad=ctx.has_bias and ctx.needs_input_grad[6])
        d_values = d_b = None
        if ctx.needs_input_grad[2]:
            d_values = sddmm(row_ptr, col_idx, g, b, ctx.static_csr)
        if ctx.needs_input_grad[5]:
            d_b = TRANSPOSE_CACHE.grad_b(row_ptr, col_idx, values.detach(), ctx.m, ctx.k, g)
        return None, None, d_values, None, None, d_b, d_bias, None, None


def fused_spmm(a_csr_row_ptr, a_csr_col_idx, a_csr_values, a_num_rows, a_num_cols, b, bias=None,
               *, relu=False, out=None, static_csr=0):
    """A GCN layer's aggregation + bias + activation: relu?(A @ b + bias?) with autograd.
    `static_csr` as for `spmm`: the forward plans an unchanged CSR once."""
    needs = (a_csr_values.requires_grad or b.requires_grad or
             (bias is not None and bias.requires_grad))
    if torch.is_grad_enabled() and needs:
        if out is not None:
            raise RuntimeError("fused_spmm: out= is not supported when gradients are required")
        return FusedSpmmCsrFunction.apply(a_csr_row_ptr, a_csr_col_idx, a_csr_values,
                                          int(a_num_rows), int(a_num_cols), b, bias, bool(relu),
                                          int(static_csr))
    return _C.fused_spmm_csr(a_csr_row_ptr, a_csr_col_idx, a_csr_values, a_num_rows, a_num_cols, b,
                             bias, relu=relu, out=out, static_csr=int(static_csr))


__all__ = ["csr_transpose", "gather_values", "sddmm", "SpmmCsrFunction", "spmm", "TRANSPOSE_CACHE", "ops",
           "FusedSpmmCsrFunction", "fused_spmm"]
