"""Collectives of the OneFlow mirror and the lazy (graph) path of the row-split op.

- `install_control_plane()` hands the library the host's control plane: torch.distributed's store
  for the RCCL unique id (what OneFlow's EagerNcclCommMgr pulls from its CtrlClient KV store,
  oneflow/core/job/eager_nccl_comm_manager.cpp:57-131) and gloo point-to-point moves for the
  kCPU ring all-gather (collective_communication/cpu/cpu_all_gather.cpp:27-80);
- `ccl_s2b()` is OneFlow's eager boxing "ccl-s-to-b" (oneflow/core/boxing/ccl_boxing_function.cpp:
  104-122, 185-215): op eager_ccl_all_gather through the op and kernel registries, RCCL on kHIP;
- `nccl_logical_all_gather()` runs the lazy compiler's `_nccl_logical_all_gather` through its kHIP
  kernel, `insert_nccl_logical_op()` is the pass's choice for one edge
  (insert_nccl_logical_op_pass.cpp:150-240);
- `SpmmJob` is the compiled row-split layer of an nn.Graph: b (S(0)) -> _nccl_logical_all_gather
  -> spmm_csr (a_csr_*: B, b: B) -> out (S(0)), compiled once, run as stream-ordered launches.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

from ._C import current_stream_handle, desc, dtype_code
from ._lib import DEV_CPU, DEV_HIP, KV_PULL_FN, KV_PUSH_FN, LIB, SENDRECV_FN, Placement, check

__all__ = ["PlacementSpec", "install_control_plane", "ccl_registered", "check_ccl_s2b", "ccl_s2b",
           "nccl_logical_all_gather", "insert_nccl_logical_op", "rccl_comm_key", "SpmmJob"]

_INSTALLED = {}  # keeps the ctypes callbacks alive for the library's lifetime


def _host_bytes(ptr: int, nbytes: int) -> torch.Tensor:
    """A uint8 CPU tensor viewing `nbytes` at a raw host address (no copy)."""
    buf = (ctypes.c_uint8 * nbytes).from_address(ptr)
    return torch.from_numpy(np.frombuffer(buf, dtype=np.uint8))


def install_control_plane(group=None):
    """Installs the calling process's rank, world size, KV store and point-to-point transport in
    the library (ofx_process_ctx_init).  Without torch.distributed the process is rank 0 of 1 with a
    local store (enough for single-rank communicators)."""
    if dist.is_available() and dist.is_initialized():
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        store = dist.distributed_c10d._get_default_store()
    else:
        rank, world, store = 0, 1, None
    local = {}

    def push(_user, key, val, n):
        try:
            data = ctypes.string_at(val, n)
            if store is None:
                local[key] = data
            else:
                store.set("ofx/" + key.decode(), data)
            return 0
        except Exception:  # noqa: BLE001  (a failed callback is reported as a status)
            return 1

    def pull(_user, key, val, cap, lenp):
        try:
            data = local[key] if store is None else store.get("ofx/" + key.decode())
            if len(data) > cap:
                return 1
            ctypes.memmove(val, data, len(data))
            lenp[0] = len(data)
            return 0
        except Exception:  # noqa: BLE001
            return 1

    def sendrecv(_user, send, send_bytes, to, recv, recv_bytes, frm):
        try:
            ops = []
            if send_bytes:
                ops.append(dist.P2POp(dist.isend, _host_bytes(send, send_bytes), int(to), group))
            if recv_bytes:
                ops.append(dist.P2POp(dist.irecv, _host_bytes(recv, recv_bytes), int(frm), group))
            if ops:
                for req in dist.batch_isend_irecv(ops):
                    req.wait()
            return 0
        except Exception:  # noqa: BLE001
            return 1

    cbs = (KV_PUSH_FN(push), KV_PULL_FN(pull), SENDRECV_FN(sendrecv))
    check(LIB.ofx_process_ctx_init(rank, world, *cbs, None), "process_ctx_init")
    _INSTALLED["callbacks"] = cbs
    return rank, world


@dataclass
class PlacementSpec:
    """A placement (oneflow/core/job/parallel_desc.h): device type "cpu" or "hip", this process's
    parallel id, and per parallel id its machine (process rank) and local device."""
    device_type: str
    parallel_num: int
    parallel_id: int
    machine_ids: tuple | None = None
    device_ids: tuple | None = None

    def c(self) -> Placement:
        p = Placement()
        p.device_type = {"cpu": DEV_CPU, "hip": DEV_HIP}[self.device_type]
        p.parallel_num, p.parallel_id = self.parallel_num, self.parallel_id
        keep = []
        for field, ids in (("machine_ids", self.machine_ids), ("device_ids", self.device_ids)):
            if ids is not None:
                arr = (ctypes.c_int64 * self.parallel_num)(*ids)
                keep.append(arr)
                setattr(p, field, ctypes.cast(arr, ctypes.POINTER(ctypes.c_int64)))
        p._keep = keep  # the arrays live as long as the struct
        return p

    @staticmethod
    def of_process_group(device_type: str, device_ids=None) -> "PlacementSpec":
        """Every rank of the default group, parallel id = rank, device = local device."""
        world, rank = dist.get_world_size(), dist.get_rank()
        return PlacementSpec(device_type, world, rank, tuple(range(world)),
                             tuple(device_ids) if device_ids is not None else tuple(range(world)))


def ccl_registered(device_type: str) -> tuple[bool, bool]:
    ag, cc = ctypes.c_int(), ctypes.c_int()
    check(LIB.ofx_ccl_registered({"cpu": DEV_CPU, "hip": DEV_HIP}[device_type], ctypes.byref(ag),
                                 ctypes.byref(cc)), "ccl_registered")
    return bool(ag.value), bool(cc.value)


def check_ccl_s2b(placement: PlacementSpec, logical_shape, in_sbp="S(0)", out_sbp="B"):
    """The boxing's applicability check; raises OfxError with the failed condition."""
    shape = (ctypes.c_int64 * len(logical_shape))(*logical_shape)
    check(LIB.ofx_boxing_check_ccl_s2b(ctypes.byref(placement.c()), len(logical_shape), shape,
                                       in_sbp.encode(), out_sbp.encode()), "ccl-s-to-b")


def ccl_s2b(shard: torch.Tensor, placement: PlacementSpec, logical_dim0: int,
            out: torch.Tensor | None = None) -> torch.Tensor:
    """S(0) -> B of a tensor whose rank-local slice is `shard` (eager boxing; every rank calls)."""
    shard = shard.contiguous()
    if out is None:
        out = torch.empty((logical_dim0, *shard.shape[1:]), dtype=shard.dtype, device=shard.device)
    stream = current_stream_handle(shard) if shard.is_cuda else None
    check(LIB.ofx_boxing_ccl_s2b(stream, ctypes.byref(placement.c()), ctypes.byref(desc(shard)),
                                 ctypes.byref(desc(out)), logical_dim0), "ccl-s-to-b")
    return out


def nccl_logical_all_gather(shard: torch.Tensor, placement: PlacementSpec,
                            out: torch.Tensor | None = None, stream_name: str = "") -> torch.Tensor:
    shard = shard.contiguous()
    if out is None:
        out = torch.empty((shard.shape[0] * placement.parallel_num, *shard.shape[1:]),
                          dtype=shard.dtype, device=shard.device)
    stream = current_stream_handle(shard) if shard.is_cuda else None
    check(LIB.ofx_nccl_logical_all_gather(stream, ctypes.byref(placement.c()), ctypes.byref(desc(shard)),
                                          ctypes.byref(desc(out)), stream_name.encode()),
          "_nccl_logical_all_gather")
    return out


def insert_nccl_logical_op(src_sbp: str, dst_sbp: str, logical_shape, parallel_num: int) -> str:
    shape = (ctypes.c_int64 * len(logical_shape))(*logical_shape)
    buf = ctypes.create_string_buffer(128)
    check(LIB.ofx_insert_nccl_logical_op(src_sbp.encode(), dst_sbp.encode(), len(logical_shape),
                                         shape, parallel_num, buf, len(buf)), "insert_nccl_logical_op")
    return buf.value.decode()


def rccl_comm_key(placement: PlacementSpec, machine: int, device: int, stream_name=None):
    buf = ctypes.create_string_buffer(4096)
    rank = ctypes.c_int()
    check(LIB.ofx_rccl_comm_key(ctypes.byref(placement.c()),
                                stream_name.encode() if stream_name else None, machine, device, buf,
                                len(buf), ctypes.byref(rank)), "rccl_comm_key")
    return buf.value.decode(), rank.value


class SpmmJob:
    """The compiled row-split spmm_csr layer (nn.Graph form): every rank holds the whole CSR
    (Broadcast) and its K/P rows of b (S(0)); a run all-gathers b with the logical collective and
    computes this rank's BalancedSplitter rows of out (S(0)).  Bits equal the single-device op."""

    def __init__(self, placement: PlacementSpec, m: int, k: int, n: int, nnz: int,
                 idx_dtype: torch.dtype, dtype: torch.dtype, device, stream_name: str = "",
                 graph: bool = False, static_csr: int = 0):
        self.placement, self.m, self.k, self.n, self.nnz = placement, m, k, n, nnz
        self.dtype, self.idx_dtype, self.device = dtype, idx_dtype, torch.device(device)
        self._job = ctypes.c_void_p()
        check(LIB.ofx_spmm_job_create(ctypes.byref(placement.c()), dtype_code(idx_dtype),
                                      dtype_code(dtype), m, k, n, nnz, stream_name.encode(),
                                      ctypes.byref(self._job)), "spmm_job_create")
        buf = ctypes.create_string_buffer(4096)
        size = ctypes.c_size_t()
        check(LIB.ofx_spmm_job_describe(self._job, buf, len(buf), ctypes.byref(size)), "describe")
        self.plan, self.tmp_bytes = buf.value.decode(), size.value
        self._tmp = torch.empty(max(self.tmp_bytes, 1), dtype=torch.uint8, device=self.device)
        lo, hi = _balanced(m, placement.parallel_num, placement.parallel_id)
        self.row_range = (lo, hi)
        if graph:
            self.set_graph(True)
        if static_csr:
            self.set_static(static_csr)

    def set_static(self, static_csr: int = 1):
        """Attr static_csr of the job's spmm_csr (include/ofx_spmm.h ofx_spmm_attrs): the caller
        promises the CSR it runs on is not rewritten; the job's kernel state keeps its work-list
        plan, so only the first run launches the planner (0 turns it off)."""
        check(LIB.ofx_spmm_job_set_static(self._job, int(static_csr)), "spmm_job_set_static")

    @property
    def static_stats(self):
        """{"plans", "hits"}: planner launches of the static CSR and runs that reused a plan."""
        p, h = ctypes.c_int64(), ctypes.c_int64()
        check(LIB.ofx_spmm_job_static_stats(self._job, ctypes.byref(p), ctypes.byref(h)),
              "spmm_job_static_stats")
        return {"plans": p.value, "hits": h.value}

    def set_graph(self, enable: bool = True):
        """Graph mode (user_kernel.cpp:676-707): after one eager run, a run is captured into a
        hipGraph and every later run with the same tensor addresses (pass `out=` to keep them)
        is one graph launch on the current stream; host placements ignore it."""
        check(LIB.ofx_spmm_job_set_graph(self._job, 1 if enable else 0), "spmm_job_set_graph")

    @property
    def graph_stats(self):
        """{"captures", "replays", "updates"}: captured runs, graph launches without re-capture,
        and captures that patched the executable in place."""
        c, r, u = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        check(LIB.ofx_spmm_job_graph_stats(self._job, ctypes.byref(c), ctypes.byref(r),
                                           ctypes.byref(u)), "spmm_job_graph_stats")
        return {"captures": c.value, "replays": r.value, "updates": u.value}

    def __call__(self, row_ptr, col_idx, values, b_shard, out=None) -> torch.Tensor:
        if out is None:
            out = torch.empty((self.row_range[1] - self.row_range[0], self.n), dtype=self.dtype,
                              device=self.device)
        # the compiled job trusts these shapes (raw pointers cross the C-ABI): check them here
        p = self.placement.parallel_num
        want = {"row_ptr": ((self.m + 1,), self.idx_dtype), "col_idx": ((self.nnz,), self.idx_dtype),
                "values": ((self.nnz,), self.dtype),
                "b_shard": ((self.k // p if p > 1 else self.k, self.n), self.dtype),
                "out": ((self.row_range[1] - self.row_range[0], self.n), self.dtype)}
        for t, name in ((row_ptr, "row_ptr"), (col_idx, "col_idx"), (values, "values"),
                        (b_shard, "b_shard"), (out, "out")):
            shape, dt = want[name]
            if tuple(t.shape) != shape or t.dtype != dt:
                raise ValueError(f"SpmmJob: {name} must be {shape} {dt}, got {tuple(t.shape)} "
                                 f"{t.dtype}")
            if not t.is_contiguous() or t.device != self.device:
                raise ValueError(f"SpmmJob: {name} must be contiguous on {self.device}")
        ptr = lambda t: t.data_ptr() if t.numel() else None  # noqa: E731
        check(LIB.ofx_spmm_job_run(self._job, current_stream_handle(out), ptr(row_ptr), ptr(col_idx),
                                   ptr(values), ptr(b_shard), ptr(out), self._tmp.data_ptr(),
                                   self._tmp.numel()), "spmm_job_run")
        return out

    def close(self):
        if self._job:
            LIB.ofx_spmm_job_destroy(self._job)
            self._job = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


def _balanced(total, parts, idx):
    lo, hi = ctypes.c_int64(), ctypes.c_int64()
    check(LIB.ofx_balanced_range(total, parts, idx, ctypes.byref(lo), ctypes.byref(hi)), "balanced")
    return lo.value, hi.value

