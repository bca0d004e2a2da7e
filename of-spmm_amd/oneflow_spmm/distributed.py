"""Row-split SpMM across the GPUs of a node: one process per GPU, RCCL all-gather of B.

SBP view (oneflow/user/ops/spmm_op.cpp GetSbp): the CSR rows are split by
BalancedSplitter (oneflow/core/common/balanced_splitter.cpp:20-40, the rows OneFlow's S(0) gives,
oneflow/core/job/nd_sbp_util.cpp:68-78), `b` arrives Split(0) and is boxed to Broadcast by an
all-gather (ccl-s-to-b, oneflow/core/boxing/ccl_boxing_function.cpp:185-215 -> ncclAllGather,
oneflow/user/kernels/collective_communication/cuda/cuda_all_gather.cpp:38), `out` is Split(0).

Layout choices (MI355X-first):
  * ncclAllGather needs equal counts, and OneFlow's S->B check wants K % G == 0
    (ccl_boxing_function.cpp:114).  Shards are therefore padded to P = ceil(K/G) rows in the
    gathered buffer, and the local column indices are remapped ONCE at setup (the graph is static
    across layers/iterations) so the hot path needs no compaction copy.
  * The gather is in place: each rank writes its B shard straight into its slot of the gathered
    buffer (`shard_view()`), so no send-buffer copy either.
  * Communication backend: native RCCL through the C-ABI (ofx_comm_*/ofx_allgather) on GPUs;
    torch.distributed (gloo) on CPU for the multi-process CPU tests.
"""
from __future__ import annotations

import ctypes
import math

import torch
import torch.distributed as dist

from . import ops
from ._C import balanced_range, current_stream_handle, dtype_code
from ._lib import LIB, UNIQUE_ID_BYTES, check


def padded_owner_remap(col_idx: torch.Tensor, k: int, world: int) -> torch.Tensor:
    """Column index c of B -> its row in the padded gathered buffer [world * P, n].
    Rank r owns BalancedSplitter(k, world).At(r) and lands at rows [r*P, r*P + size_r)."""
    base, extra = divmod(k, world)
    if extra == 0:
        return col_idx
    c = col_idx.to(torch.int64)
    big = extra * (base + 1)
    owner = torch.where(c < big, c // (base + 1), extra + (c - big) // max(base, 1))
    shift = torch.clamp(owner - extra, min=0)
    return (c + shift).to(col_idx.dtype)


class RowSplitSpmm:
    """out[rows of this rank] = A[rows of this rank, :] @ all_gather(b shards).

    Call with this rank's *local* CSR slice (row_ptr rebased to 0, columns already remapped with
    `remap_columns`) — or construct with `local_csr=False` and pass the full CSR (Broadcast SBP);
    the kernel then computes the row range itself (the OpKernelCache path)."""

    def __init__(self, m: int, k: int, n: int, nnz_local: int, dtype: torch.dtype,
                 idx_dtype: torch.dtype, device: torch.device, group=None,
                 comm: str = "auto", local_csr: bool = True):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.m, self.k, self.n = m, k, n
        self.dtype, self.device = dtype, torch.device(device)
        self.row_range = balanced_range(m, self.world, self.rank)
        self.k_range = balanced_range(k, self.world, self.rank)
        self.pad = math.ceil(k / self.world) if k else 0
        self.k_padded = self.pad * self.world
        self.local_csr = local_csr
        self.gathered = torch.zeros((self.k_padded, n), dtype=dtype, device=self.device)
        rows_local = self.row_range[1] - self.row_range[0]
        m_kernel = rows_local if local_csr else m
        self.kernel = None
        if self.device.type == "cuda":
            self.kernel = ops.SpmmCsrKernel(m_kernel, self.k_padded, n, nnz_local, idx_dtype, dtype,
                                            self.device)
        if comm == "auto":
            comm = "rccl" if self.device.type == "cuda" else "torch"
        if comm not in ("rccl", "rccl-p2p", "torch"):
            raise ValueError(f"RowSplitSpmm: unknown comm {comm!r}")
        self.comm_kind = comm
        self._comm = None
        if comm.startswith("rccl"):
            self._init_rccl()
        self.ev = None

    # -- communicator (EagerNcclCommMgr::CreateNcclComm pattern: rank 0 makes the id) --------
    def _init_rccl(self):
        uid = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
        if self.rank == 0:
            check(LIB.ofx_comm_get_unique_id(uid), "comm_get_unique_id")
        obj = [bytes(uid.raw) if self.rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=self.group)
        uid = ctypes.create_string_buffer(obj[0], UNIQUE_ID_BYTES)
        comm = ctypes.c_void_p()
        check(LIB.ofx_set_device(self.device.index if self.device.index is not None else 0), "set_device")
        check(LIB.ofx_comm_init_rank(ctypes.byref(comm), self.world, uid, self.rank), "comm_init_rank")
        self._comm = comm

    def tune_comm(self, reps: int = 3) -> dict:
        """Times the ring all-gather and the point-to-point one on this node (same bytes) and
        keeps the faster; the timings are max-reduced over ranks, so every rank makes the
        same choice.  Returns the timings (ms)."""
        if not self.comm_kind.startswith("rccl") or self.world == 1:
            return {}
        times = {}
        for kind in ("rccl", "rccl-p2p"):
            self.comm_kind = kind
            self.all_gather_b()
            torch.cuda.synchronize(self.device)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                self.all_gather_b()
            e1.record()
            torch.cuda.synchronize(self.device)
            t = torch.tensor([e0.elapsed_time(e1) / reps], dtype=torch.float64, device=self.device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
            times[kind] = float(t.item())
        self.comm_kind = min(times, key=times.get)
        return times

    def close(self):
        if self._comm is not None:
            check(LIB.ofx_comm_destroy(self._comm), "comm_destroy")
            self._comm = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- layout helpers ----------------------------------------------------------------------
    def shard_view(self) -> torch.Tensor:
        """This rank's B shard inside the gathered buffer (write b here: in-place all-gather)."""
        lo, hi = self.k_range
        return self.gathered[self.rank * self.pad: self.rank * self.pad + (hi - lo)]

    def remap_columns(self, col_idx: torch.Tensor) -> torch.Tensor:
        return padded_owner_remap(col_idx, self.k, self.world)

    # -- the collective ------------------------------------------------------------------------
    def all_gather_b(self, b_shard: torch.Tensor | None = None):
        slot = self.gathered[self.rank * self.pad:(self.rank + 1) * self.pad]
        if b_shard is not None and b_shard.data_ptr() != slot.data_ptr():
            slot[: b_shard.shape[0]].copy_(b_shard)
        count = self.pad * self.n
        if self.comm_kind == "rccl":
            s = current_stream_handle(self.gathered)
            check(LIB.ofx_allgather(s, slot.data_ptr(), self.gathered.data_ptr(), count,
                                    dtype_code(self.dtype), self._comm), "allgather")
        elif self.comm_kind == "rccl-p2p":
            s = current_stream_handle(self.gathered)
            check(LIB.ofx_allgather_p2p(s, self.gathered.data_ptr(), count, dtype_code(self.dtype),
                                        self._comm), "allgather_p2p")
        else:
            parts = list(self.gathered.view(self.world, self.pad, self.n).unbind(0))
            dist.all_gather(parts, slot.clone(), group=self.group)  # views: lands in place

    # -- one step ------------------------------------------------------------------------------
    def __call__(self, row_ptr, col_idx, values, b_shard=None, out=None, events=None):
        """events: optional (start, mid, end) torch.cuda.Event to time gather / SpMM."""
        lo, hi = self.row_range
        if out is None:
            out = torch.empty((hi - lo, self.n), dtype=self.dtype, device=self.device)
        if events:
            events[0].record()
        self.all_gather_b(b_shard)
        if events:
            events[1].record()
        rb, re = (0, hi - lo) if self.local_csr else (lo, hi)
        if self.kernel is not None:
            self.kernel(row_ptr, col_idx, values, self.gathered, out, rb, re)
        else:
            m_kernel = hi - lo if self.local_csr else self.m
            ops.spmm_csr_cpu(row_ptr, col_idx, values, self.gathered, m_kernel, self.k_padded,
                             out=out, row_begin=rb, row_end=re)
        if events:
            events[2].record()
        return out
