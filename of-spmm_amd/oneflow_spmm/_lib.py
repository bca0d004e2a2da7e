"""Loader of libofx_spmm.so (the C-ABI of include/ofx_spmm.h) with ctypes signatures.

There is deliberately no fallback: if the native library is missing the import fails loudly.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# OFX_SPMM_LIB: A/B timing of alternative builds of the same sources (scripts/); the default is
# the in-tree library next to this file.
LIB_PATH = os.environ.get("OFX_SPMM_LIB") or os.path.join(_HERE, "libofx_spmm.so")

# OneFlow DataType codes (oneflow/core/common/data_type.proto:4-26)
DT_FLOAT, DT_DOUBLE, DT_INT32, DT_INT64, DT_FLOAT16, DT_BFLOAT16 = 2, 3, 5, 6, 9, 11

(OFX_OK, OFX_EINVAL, OFX_EDEVICE, OFX_ENOMEM, OFX_EUNSUPPORTED, OFX_ECOMM, OFX_EWORKSPACE, OFX_EPLAN,
 OFX_EINTERNAL) = range(9)
# test knobs of ofx_debug_set (include/ofx_spmm.h)
DEBUG_PLAN_SPIN_LIMIT, DEBUG_THROW_IN_COMPUTE, DEBUG_EXCHANGE_STALL = 1, 2, 3
MEMCPY_H2D, MEMCPY_D2H, MEMCPY_D2D, MEMCPY_DEFAULT = 1, 2, 3, 4
UNIQUE_ID_BYTES = 128
PEER_HANDLE_BYTES = 96   # OFX_PEER_HANDLE_BYTES
PEER_MAX_RANKS = 16      # OFX_PEER_MAX_RANKS


class OfxError(RuntimeError):
    """A failed C-ABI call; `code` is the ofx status."""

    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


STRUCT_MAGIC = 0x4F465831  # OFX_STRUCT_MAGIC, "OFX1"


class _Versioned(ctypes.Structure):
    """A versioned C-ABI struct: struct_size and magic (its first two fields) are set to this
    layout's size and OFX_STRUCT_MAGIC, as the OFX_*_INIT initialisers of include/ofx_spmm.h do;
    positional fields start after them."""

    def __init__(self, *args, **kw):
        super().__init__(ctypes.sizeof(type(self)), STRUCT_MAGIC, *args, **kw)


class Options(_Versioned):
    _fields_ = [("struct_size", ctypes.c_uint32), ("magic", ctypes.c_uint32),
                ("split_threshold", ctypes.c_int64), ("chunk", ctypes.c_int64),
                ("ordered", ctypes.c_int32), ("variant", ctypes.c_int32),
                ("heavy_threshold", ctypes.c_int64), ("planned", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("range_nnz", ctypes.c_int64)]


class SpmmAttrs(_Versioned):
    """ofx_spmm_attrs: op "spmm_csr"'s attributes beyond a_num_rows / a_num_cols."""
    _fields_ = [("struct_size", ctypes.c_uint32), ("magic", ctypes.c_uint32),
                ("static_csr", ctypes.c_int64)]


class Placement(_Versioned):
    _fields_ = [("struct_size", ctypes.c_uint32), ("magic", ctypes.c_uint32),
                ("device_type", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("parallel_num", ctypes.c_int64), ("parallel_id", ctypes.c_int64),
                ("machine_ids", ctypes.POINTER(ctypes.c_int64)),
                ("device_ids", ctypes.POINTER(ctypes.c_int64))]


# control-plane callbacks of ofx_process_ctx_init (include/ofx_spmm.h)
KV_PUSH_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p,
                              ctypes.c_size_t)
KV_PULL_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p,
                              ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t))
SENDRECV_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                               ctypes.c_int64, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int64)
DEV_CPU, DEV_HIP = 1, 4


class TensorDesc(_Versioned):
    _fields_ = [("struct_size", ctypes.c_uint32), ("magic", ctypes.c_uint32),
                ("dtype", ctypes.c_int32), ("device", ctypes.c_int32), ("ndim", ctypes.c_int32),
                ("reserved", ctypes.c_int32),
                ("shape", ctypes.c_int64 * 2), ("stride", ctypes.c_int64 * 2),
                ("data", ctypes.c_void_p)]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"oneflow_spmm: native library {LIB_PATH} is missing; build it with "
            "`make -C of-spmm_amd` or `python -c 'import __graft_entry__ as g; g.build()'`. "
            "There is no CPU/torch fallback for the HIP path.")
    lib = ctypes.CDLL(LIB_PATH)
    i32, i64, u64, p, sz = ctypes.c_int, ctypes.c_int64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t
    popt = ctypes.POINTER(Options)
    pdesc = ctypes.POINTER(TensorDesc)
    ppl = ctypes.POINTER(Placement)
    pattrs = ctypes.POINTER(SpmmAttrs)
    sigs = {
        "ofx_last_error": ([], ctypes.c_char_p),
        "ofx_device_error_check": ([], i32),
        "ofx_debug_set": ([i32, i64], i32),
        "ofx_version": ([], ctypes.c_char_p),
        "ofx_spmm_default_split": ([i64], i64),
        "ofx_spmm_csr_workspace_size": ([i32, i32, i64, i64, i64, i64, popt, ctypes.POINTER(sz)], i32),
        "ofx_spmm_csr": ([p, i32, i32, i64, i64, i64, i64, p, p, p, p, i64, p, i64, i64, i64, p, sz,
                          popt], i32),
        "ofx_spmm_csr_gathered": ([p, i32, i32, i64, i64, i64, i64, p, p, p, p, p, i64, p, i64, i64,
                                   i64, p, sz, popt], i32),
        "ofx_relu_bias_grad_workspace_size": ([i32, i64, i64, ctypes.POINTER(sz)], i32),
        "ofx_relu_bias_grad": ([p, i32, i64, i64, p, i64, p, i64, p, i64, p, i32, p, sz], i32),
        "ofx_relu_bias_grad_cpu": ([i32, i32, i64, i64, p, i64, p, i64, p, i64, p, i32], i32),
        "ofx_spmm_csr_plan": ([p, i32, i32, i64, i64, i64, i64, p, i64, i64, p, sz, popt], i32),
        "ofx_debug_bounds_read": ([ctypes.POINTER(u64), i32], i32),
        "ofx_spmm_csr_describe": ([i32, i32, i64, i64, i64, i64, p, i64, p, i64, i64, i64, popt,
                                   ctypes.c_char_p, sz], i32),
        "ofx_spmm_csr_fused": ([p, i32, i32, i64, i64, i64, i64, p, p, p, p, i64, p, i64, i64, i64,
                                p, i32, p, sz, popt], i32),
        "ofx_spmm_csr_fused_cpu": ([i32, i32, i32, i64, i64, i64, i64, p, p, p, p, i64, p, i64, i64,
                                    i64, p, i32, popt], i32),
        "ofx_functional_fused_spmm_csr": ([p, pdesc, pdesc, pdesc, pdesc, pdesc, i64, i64, i32, pdesc,
                                           p, sz, ctypes.POINTER(sz)], i32),
        "ofx_functional_fused_spmm_csr_attrs": ([p, pdesc, pdesc, pdesc, pdesc, pdesc, i64, i64, i32,
                                                 pdesc, p, sz, ctypes.POINTER(sz), pattrs], i32),
        "ofx_csr_validate": ([p, i32, i64, i64, i64, p, p, p], i32),
        "ofx_spmm_csr_cpu": ([i32, i32, i32, i64, i64, i64, i64, p, p, p, p, i64, p, i64, i64, i64,
                              popt], i32),
        "ofx_csr_transpose_workspace_size": ([i32, i64, i64, i64, ctypes.POINTER(sz)], i32),
        "ofx_csr_transpose": ([p, i32, i64, i64, i64, p, p, p, p, p, p, sz], i32),
        "ofx_csr_transpose_cpu": ([i32, i64, i64, i64, p, p, p, p, p], i32),
        "ofx_gather_values": ([p, i32, i32, i64, p, p, p], i32),
        "ofx_copy_blocks": ([p, i64, i64, i64, i64, p, i64, i64, i64, p, i64, i64, i64], i32),
        "ofx_gather_values_host": ([i32, i32, i64, p, p, p], i32),
        "ofx_sddmm_csr_workspace_size": ([i32, i32, i64, i64, i64, ctypes.POINTER(sz)], i32),
        "ofx_sddmm_csr": ([p, i32, i32, i64, i64, i64, i64, p, p, p, i64, p, i64, p, i64, i64, p, sz], i32),
        "ofx_sddmm_csr_ex": ([p, i32, i32, i64, i64, i64, i64, p, p, p, i64, p, i64, p, i64, i64, p, sz,
                              popt], i32),
        "ofx_sddmm_csr_plan": ([p, i32, i32, i64, i64, i64, p, i64, i64, p, sz], i32),
        "ofx_sddmm_csr_cpu": ([i32, i32, i32, i64, i64, i64, i64, p, p, p, i64, p, i64, p, i64, i64], i32),
        "ofx_coo_to_csr_workspace_size": ([i32, i64, i64, i64, ctypes.POINTER(sz)], i32),
        "ofx_coo_to_csr": ([p, i32, i32, i64, i64, i64, p, p, p, i32, p, p, p, p, p, p, sz], i32),
        "ofx_coo_to_csr_cpu": ([i32, i32, i64, i64, i64, p, p, p, i32, p, p, p, ctypes.POINTER(i64)], i32),
        "ofx_balanced_range": ([i64, i64, i64, ctypes.POINTER(i64), ctypes.POINTER(i64)], i32),
        "ofx_csr_row_slice": ([p, i32, p, i64, i64, p], i32),
        "ofx_csr_row_slice_host": ([i32, p, i64, i64, p, ctypes.POINTER(i64), ctypes.POINTER(i64)], i32),
        "ofx_device_count": ([ctypes.POINTER(i32)], i32),
        "ofx_set_device": ([i32], i32),
        "ofx_get_device": ([ctypes.POINTER(i32)], i32),
        "ofx_device_synchronize": ([], i32),
        "ofx_malloc": ([ctypes.POINTER(p), sz], i32),
        "ofx_free": ([p], i32),
        "ofx_host_malloc": ([ctypes.POINTER(p), sz], i32),
        "ofx_host_free": ([p], i32),
        "ofx_stream_create": ([ctypes.POINTER(p)], i32),
        "ofx_stream_destroy": ([p], i32),
        "ofx_stream_sync": ([p], i32),
        "ofx_memcpy_async": ([p, p, p, sz, i32], i32),
        "ofx_memset_async": ([p, p, i32, sz], i32),
        "ofx_event_create": ([ctypes.POINTER(p), i32], i32),
        "ofx_event_destroy": ([p], i32),
        "ofx_event_record": ([p, p], i32),
        "ofx_event_sync": ([p], i32),
        "ofx_event_elapsed_ms": ([p, p, ctypes.POINTER(ctypes.c_float)], i32),
        "ofx_stream_wait_event": ([p, p], i32),
        "ofx_graph_exec_create": ([ctypes.POINTER(p)], i32),
        "ofx_graph_exec_destroy": ([p], i32),
        "ofx_graph_exec_stats": ([p, ctypes.POINTER(i32), ctypes.POINTER(i64), ctypes.POINTER(i64),
                                  ctypes.POINTER(i64)], i32),
        "ofx_stream_begin_capture": ([p], i32),
        "ofx_stream_is_capturing": ([p, ctypes.POINTER(i32)], i32),
        "ofx_stream_end_capture": ([p, p], i32),
        "ofx_graph_launch": ([p, p], i32),
        "ofx_comm_get_unique_id": ([p], i32),
        "ofx_comm_init_rank": ([ctypes.POINTER(p), i32, p, i32], i32),
        "ofx_comm_init_rank_deadline": ([ctypes.POINTER(p), i32, p, i32, ctypes.c_double], i32),
        "ofx_comm_set_timeouts": ([p, ctypes.c_double, ctypes.c_double], i32),
        "ofx_comm_abort": ([p], i32),
        "ofx_comm_destroy": ([p], i32),
        "ofx_comm_count": ([p, ctypes.POINTER(i32), ctypes.POINTER(i32)], i32),
        "ofx_allgather": ([p, p, p, sz, i32, p], i32),
        "ofx_allgather_p2p": ([p, p, sz, i32, p], i32),
        "ofx_peer_export": ([p, p], i32),
        "ofx_peer_open": ([p, ctypes.POINTER(p)], i32),
        "ofx_peer_close": ([p], i32),
        "ofx_peer_publish": ([p], i32),
        "ofx_peer_pull": ([p, i32, i32, p, p, u64], i32),
        "ofx_peer_pull_host": ([i32, i32, p, p, u64], i32),
        "ofx_allgather_pull": ([p, p, p, p, sz, i32], i32),
        "ofx_exchange_rows": ([p, p, i32, i64, p, p, p, p, p, p], i32),
        "ofx_spmm_rowsplit": ([p, p, i32, i32, i64, i64, i64, i64, p, p, p, p, p, i64, p, sz, popt], i32),
        "ofx_padded_owner_remap": ([p, i32, i64, i64, i64, p, p], i32),
        "ofx_gather_rows": ([p, i32, i64, i64, p, p, i64, p, i64], i32),
        "ofx_synth_row_ptr": ([i64, i64, i64, ctypes.c_double, u64, p], i32),
        "ofx_synth_columns": ([i64, i64, ctypes.c_double, u64, p, i64, i64, i32, p, i32], i32),
        "ofx_synth_values_host": ([i32, i64, i64, u64, i32, p], i32),
        "ofx_synth_dense": ([p, i32, i64, i64, i64, i64, u64, i32, p], i32),
        "ofx_synth_dense_host": ([i32, i64, i64, i64, i64, u64, i32, p], i32),
        "ofx_functional_spmm_csr_infer": ([pdesc, pdesc, pdesc, i64, i64, pdesc, pdesc], i32),
        "ofx_functional_spmm_csr_tmp_size": ([pdesc, pdesc, pdesc, i64, i64, pdesc,
                                              ctypes.POINTER(sz)], i32),
        "ofx_functional_spmm_csr": ([p, pdesc, pdesc, pdesc, i64, i64, pdesc, pdesc, p, sz], i32),
        "ofx_functional_spmm_csr_ex": ([p, pdesc, pdesc, pdesc, i64, i64, pdesc, pdesc, p, sz, i64,
                                        i64, i32, i32], i32),
        "ofx_functional_spmm_csr_global": ([p, pdesc, pdesc, pdesc, i64, i64, pdesc, i64, pdesc, p,
                                            sz, i32, ctypes.POINTER(i64), ctypes.POINTER(i32), i64,
                                            i32, ctypes.POINTER(sz)], i32),
        "ofx_functional_spmm_csr_global_attrs": ([p, pdesc, pdesc, pdesc, i64, i64, pdesc, i64, pdesc,
                                                  p, sz, i32, ctypes.POINTER(i64),
                                                  ctypes.POINTER(i32), i64, i32, ctypes.POINTER(sz),
                                                  pattrs], i32),
        "ofx_spmm_static_plans": ([ctypes.POINTER(i64), ctypes.POINTER(i64), ctypes.POINTER(i64),
                                   i32], i32),
        "ofx_functional_sddmm_csr": ([p, pdesc, pdesc, pdesc, pdesc, i64, i64, pdesc, p, sz,
                                      ctypes.POINTER(sz)], i32),
        "ofx_functional_sddmm_csr_attrs": ([p, pdesc, pdesc, pdesc, pdesc, i64, i64, pdesc, p, sz,
                                            ctypes.POINTER(sz), pattrs], i32),
        "ofx_functional_spmm_csr_gathered": ([p, pdesc, pdesc, pdesc, pdesc, pdesc, i64, i64, pdesc,
                                              p, sz, ctypes.POINTER(sz)], i32),
        "ofx_functional_spmm_csr_gathered_attrs": ([p, pdesc, pdesc, pdesc, pdesc, pdesc, i64, i64,
                                                    pdesc, p, sz, ctypes.POINTER(sz), pattrs], i32),
        "ofx_functional_csr_transpose": ([p, pdesc, pdesc, i64, i64, pdesc, pdesc, pdesc, p, sz,
                                          ctypes.POINTER(sz)], i32),
        "ofx_op_spmm_csr_sbp_signatures": ([ctypes.c_char_p, sz], i32),
        "ofx_process_ctx_init": ([i64, i64, KV_PUSH_FN, KV_PULL_FN, SENDRECV_FN, p], i32),
        "ofx_ccl_registered": ([i32, ctypes.POINTER(i32), ctypes.POINTER(i32)], i32),
        "ofx_boxing_check_ccl_s2b": ([ppl, i32, ctypes.POINTER(i64), ctypes.c_char_p,
                                      ctypes.c_char_p], i32),
        "ofx_boxing_ccl_s2b": ([p, ppl, pdesc, pdesc, i64], i32),
        "ofx_nccl_logical_all_gather": ([p, ppl, pdesc, pdesc, ctypes.c_char_p], i32),
        "ofx_insert_nccl_logical_op": ([ctypes.c_char_p, ctypes.c_char_p, i32, ctypes.POINTER(i64),
                                        i64, p, sz], i32),
        "ofx_rccl_comm_key": ([ppl, ctypes.c_char_p, i64, i64, p, sz, ctypes.POINTER(i32)], i32),
        "ofx_spmm_job_create": ([ppl, i32, i32, i64, i64, i64, i64, ctypes.c_char_p,
                                 ctypes.POINTER(p)], i32),
        "ofx_spmm_job_describe": ([p, p, sz, ctypes.POINTER(sz)], i32),
        "ofx_spmm_job_run": ([p, p, p, p, p, p, p, p, sz], i32),
        "ofx_spmm_job_destroy": ([p], i32),
        "ofx_spmm_job_set_graph": ([p, i32], i32),
        "ofx_spmm_job_set_static": ([p, i64], i32),
        "ofx_spmm_job_static_stats": ([p, ctypes.POINTER(i64), ctypes.POINTER(i64)], i32),
        "ofx_spmm_job_graph_stats": ([p, ctypes.POINTER(i64), ctypes.POINTER(i64),
                                      ctypes.POINTER(i64)], i32),
        "ofx_op_sbp_signatures": ([ctypes.c_char_p, ctypes.c_char_p, p, sz], i32),
    }
    # an alternative build selected with OFX_SPMM_LIB (A/B timing against an older library) may
    # predate some entry points: those are left out; the in-tree library must export them all
    alt = bool(os.environ.get("OFX_SPMM_LIB"))
    found = []
    for name, (args, res) in sigs.items():
        if alt and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
        found.append(name)
    return lib, tuple(found)


LIB, EXPORTED = _load()


def last_error() -> str:
    return LIB.ofx_last_error().decode(errors="replace")


def check(rc: int, what: str = "") -> None:
    if rc == OFX_OK:
        return
    msg = last_error()
    if msg.startswith("TypeError"):
        raise TypeError(msg)
    raise OfxError(rc, f"{what}: {msg}" if what else msg)
