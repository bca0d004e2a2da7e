"""CPU: the C-ABI library loads and exports every symbol include/ofx_spmm.h declares; the op
layer's inference / SBP / error behaviour mirrors the reference's user-op conventions."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

import oneflow_spmm as fs
from oneflow_spmm import _lib, ops
from tests.helpers import random_csr, random_dense

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    text = open(os.path.join(ROOT, "include", "ofx_spmm.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ofx_[a-z0-9_]+)\s*\(", text)))


def test_every_declared_symbol_is_exported():
    names = declared_functions()
    assert len(names) >= 40
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and the Python binding declares a signature for each of them
    assert set(names) <= set(_lib.EXPORTED), set(names) - set(_lib.EXPORTED)


def test_version_and_default_split():
    assert fs.__version__.startswith("ofx-spmm")
    for n in (1, 16, 64, 128, 256, 1000):
        from oracle import oracle
        assert ops.default_split(n) == oracle.default_split(n)


def test_sbp_signatures_and_no_grad_inputs():
    s = fs._C.sbp_signatures()
    sigs, mods = s.split("|")
    rows = [dict(kv.split(":") for kv in sig.split(",")) for sig in sigs.split(";")]
    assert {"a_csr_row_ptr": "B", "a_csr_col_idx": "B", "a_csr_values": "B", "b": "B", "out": "S(0)"} in rows
    assert {"a_csr_row_ptr": "B", "a_csr_col_idx": "B", "a_csr_values": "B", "b": "S(1)", "out": "S(1)"} in rows
    assert mods == "no_grad:a_csr_col_idx,a_csr_row_ptr"


def test_fused_op_sbp_with_and_without_bias():
    def parse(s):
        sigs, mods = s.split("|")
        return [dict(kv.split(":") for kv in sig.split(",")) for sig in sigs.split(";")], mods
    rows, mods = parse(fs._C.sbp_signatures("fused_spmm_csr", "bias"))
    base = {"a_csr_row_ptr": "B", "a_csr_col_idx": "B", "a_csr_values": "B"}
    assert {**base, "b": "B", "bias": "B", "out": "S(0)"} in rows
    assert {**base, "b": "S(1)", "bias": "S(0)", "out": "S(1)"} in rows
    assert mods == "no_grad:a_csr_col_idx,a_csr_row_ptr"
    rows, _ = parse(fs._C.sbp_signatures("fused_spmm_csr", ""))
    assert all("bias" not in r for r in rows) and {**base, "b": "B", "out": "S(0)"} in rows
    with pytest.raises(fs.OfxError, match="not registered"):
        fs._C.sbp_signatures("no_such_op")


def _small():
    rng = np.random.default_rng(0)
    rp, ci, v = random_csr(6, 9, rng.integers(0, 4, size=6), rng)
    return rp, ci, v, random_dense(9, 5, rng)


def test_op_shape_and_dtype_errors():
    rp, ci, v, b = _small()
    with pytest.raises(RuntimeError, match="a_num_rows"):
        fs.spmm(rp, ci, v, 5, 9, b)
    with pytest.raises(RuntimeError, match="Dim K"):
        fs.spmm(rp, ci, v, 6, 8, b)
    with pytest.raises(RuntimeError, match="nnz"):
        fs.spmm(rp, ci, v[:-1] if v.numel() else torch.ones(1), 6, 9, b)
    with pytest.raises(RuntimeError, match="b should be 2-D"):
        fs.spmm(rp, ci, v, 6, 9, b.reshape(-1))
    with pytest.raises(TypeError, match="a_csr_values"):
        fs.spmm(rp, ci, v.double(), 6, 9, b)
    with pytest.raises(TypeError, match="int32 or int64"):
        fs.spmm(rp.float(), ci, v, 6, 9, b)
    with pytest.raises(TypeError, match="dtype of a_csr_row_ptr"):
        fs.spmm(rp, ci.long(), v, 6, 9, b)
    with pytest.raises(TypeError):
        fs.spmm(rp, ci, v.to(torch.uint8), 6, 9, b.to(torch.uint8))


def test_op_cpu_global_form_rows():
    rng = np.random.default_rng(1)
    m, k, n = 103, 50, 8
    rp, ci, v = random_csr(m, k, rng.integers(0, 10, size=m), rng)
    b = random_dense(k, n, rng)
    full = fs.spmm(rp, ci, v, m, k, b)
    for parts in (2, 5):
        chunks = [fs._C.spmm_csr(rp, ci, v, m, k, b, _parallel=(r, parts, 0)) for r in range(parts)]
        assert torch.equal(torch.cat(chunks), full)
    # column split (S(1)): local b columns -> local out columns
    left = fs._C.spmm_csr(rp, ci, v, m, k, b[:, :3].contiguous(), _parallel=(0, 2, 1))
    assert torch.equal(left, full[:, :3])


def test_out_argument_validation():
    rp, ci, v, b = _small()
    with pytest.raises(RuntimeError, match="out must be"):
        fs.spmm(rp, ci, v, 6, 9, b, out=torch.empty(6, 4))
    out = torch.empty(6, 5)
    r = fs.spmm(rp, ci, v, 6, 9, b, out=out)
    assert r is out


def test_direct_abi_argument_checks():
    L = _lib.LIB
    sz = ctypes.c_size_t()
    assert L.ofx_spmm_csr_workspace_size(7, 2, 1, 1, 1, 1, None, ctypes.byref(sz)) == _lib.OFX_EUNSUPPORTED
    assert L.ofx_spmm_csr_workspace_size(5, 2, -1, 1, 1, 1, None, ctypes.byref(sz)) == _lib.OFX_EINVAL
    assert L.ofx_spmm_csr_workspace_size(5, 2, 10, 10, 128, 6, None, ctypes.byref(sz)) == 0
    assert sz.value == 0  # every row is in the lightest degree bin: no plan, no workspace
    assert L.ofx_spmm_csr_workspace_size(5, 2, 10, 10, 128, 100000, None, ctypes.byref(sz)) == 0
    assert sz.value > 0
    rc = L.ofx_spmm_csr(None, 5, 2, 4, 4, 4, 0, None, None, None, None, 4, None, 4, 3, 2, None, 0, None)
    assert rc == _lib.OFX_EINVAL and "row range" in _lib.last_error()
    rc = L.ofx_spmm_csr_cpu(0, 5, 2, 4, 4, 4, 0, None, None, None, None, 2, None, 4, 0, 4, None)
    assert rc == _lib.OFX_EINVAL
    lo, hi = ctypes.c_int64(), ctypes.c_int64()
    assert L.ofx_balanced_range(10, 0, 0, ctypes.byref(lo), ctypes.byref(hi)) == _lib.OFX_EINVAL


def test_kernel_registry_and_device_dispatch_without_gpu():
    """GPU tensors never reach the CPU kernel: a CPU tensor runs kCPU; the HIP kernel is chosen
    only for device tensors (checked on the GPU box in test_gpu_parity)."""
    rp, ci, v, b = _small()
    out = fs.spmm(rp, ci, v, 6, 9, b)
    assert out.device.type == "cpu"
