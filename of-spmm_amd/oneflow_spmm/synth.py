"""Synthetic power-law CSR / dense inputs (generator in csrc/synth.cpp; spec in DESIGN.md §5).

The BASELINE configs are dataset-shaped; the datasets are not available offline, so the bench
and tests use these deterministic Chung–Lu-style matrices.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from ._C import dtype_code
from ._lib import LIB, check

SEED_GRAPH, SEED_VALUES, SEED_DENSE = 0, 1, 2

# BASELINE.json configs (dataset-shaped, public statistics).
CONFIGS = {
    "cora": dict(m=2708, k=2708, nnz=10556, n=16, dtype=torch.float32),
    "plaw1m": dict(m=1_000_000, k=1_000_000, nnz=20_000_000, n=64, dtype=torch.float32),
    "products": dict(m=2_449_029, k=2_449_029, nnz=123_718_280, n=128, dtype=torch.float32),
    "reddit": dict(m=232_965, k=232_965, nnz=114_615_892, n=256, dtype=torch.bfloat16),
    "papers": dict(m=111_059_956, k=111_059_956, nnz=1_615_685_872, n=128, dtype=torch.float32),
}
# Not a BASELINE config: the maximum-size case of the int64 index path (nnz > 2^31 - 1, so
# row_ptr offsets and every nonzero position past 2^31 need 64-bit indices end to end).
EXTRA_CONFIGS = {
    "int64_max": dict(m=40_000_000, k=40_000_000, nnz=2_300_000_000, n=16, dtype=torch.float32),
    # the CPU rehearsal of the multi-rank bench path (bench.py --device cpu, tests)
    "tiny": dict(m=20_000, k=20_000, nnz=200_000, n=32, dtype=torch.float32),
}


@dataclass
class HostCsr:
    m: int
    k: int
    row_ptr: np.ndarray  # int64 [rows+1] (global offsets unless rebased)
    col_idx: np.ndarray  # idx dtype [nnz_local]
    row_begin: int
    row_end: int


def row_ptr(m: int, k: int, nnz: int, gamma: float = 2.5, seed: int = SEED_GRAPH) -> np.ndarray:
    rp = np.empty(m + 1, dtype=np.int64)
    check(LIB.ofx_synth_row_ptr(m, k, nnz, gamma, seed, rp.ctypes.data), "synth_row_ptr")
    return rp


def columns(m: int, k: int, rp: np.ndarray, row_begin: int = 0, row_end: int | None = None,
            gamma: float = 2.5, seed: int = SEED_GRAPH, idx_dtype=np.int32,
            threads: int = 0) -> np.ndarray:
    row_end = m if row_end is None else row_end
    cnt = int(rp[row_end] - rp[row_begin])
    out = np.empty(cnt, dtype=idx_dtype)
    dt = 5 if np.dtype(idx_dtype) == np.int32 else 6
    check(LIB.ofx_synth_columns(m, k, gamma, seed, rp.ctypes.data, row_begin, row_end, dt,
                                out.ctypes.data if cnt else None, threads), "synth_columns")
    return out


def values(j_begin: int, j_end: int, dtype: torch.dtype = torch.float32, seed: int = SEED_VALUES,
           exact: bool = False) -> torch.Tensor:
    t = torch.empty(j_end - j_begin, dtype=dtype)
    check(LIB.ofx_synth_values_host(dtype_code(dtype), j_begin, j_end, seed, int(exact),
                                    t.data_ptr() if t.numel() else None), "synth_values")
    return t


def dense(r_begin: int, r_end: int, n: int, dtype: torch.dtype = torch.float32, device="cpu",
          seed: int = SEED_DENSE, exact: bool = False, ld: int | None = None) -> torch.Tensor:
    """Rows [r_begin, r_end) of the K x n dense operand (generated on the device for GPU)."""
    ld = n if ld is None else ld
    t = torch.empty((r_end - r_begin, ld), dtype=dtype, device=device)
    if t.device.type == "cpu":
        check(LIB.ofx_synth_dense_host(dtype_code(dtype), r_begin, r_end, n, ld, seed, int(exact),
                                       t.data_ptr() if t.numel() else None), "synth_dense")
    else:
        s = ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)
        check(LIB.ofx_synth_dense(s, dtype_code(dtype), r_begin, r_end, n, ld, seed, int(exact),
                                  t.data_ptr() if t.numel() else None), "synth_dense")
    return t[:, :n] if ld != n else t


def csr(m: int, k: int, nnz: int, *, idx_dtype=torch.int32, val_dtype=torch.float32,
        gamma: float = 2.5, exact: bool = False, row_begin: int = 0, row_end: int | None = None,
        rebase: bool = False, threads: int = 0):
    """Synthetic CSR rows [row_begin, row_end) as torch CPU tensors (row_ptr, col_idx, values).
    With rebase=True the row_ptr is local (starts at 0); otherwise the full global row_ptr is
    returned together with the global nonzeros of the whole matrix (row_begin must be 0)."""
    row_end = m if row_end is None else row_end
    rp = row_ptr(m, k, nnz, gamma)
    np_idx = np.int32 if idx_dtype == torch.int32 else np.int64
    if not rebase and (row_begin != 0 or row_end != m):
        raise ValueError("synth.csr: a partial row range needs rebase=True")
    ci = columns(m, k, rp, row_begin, row_end, gamma, idx_dtype=np_idx, threads=threads)
    j0, j1 = int(rp[row_begin]), int(rp[row_end])
    vals = values(j0, j1, val_dtype, exact=exact)
    local_rp = rp[row_begin:row_end + 1] - rp[row_begin]
    return (torch.from_numpy(local_rp.astype(np_idx)), torch.from_numpy(ci), vals)
