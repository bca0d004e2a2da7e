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
    # column split (S(1)): this rank's b columns (BalancedSplitter of the logical N) -> its out
    # columns; the logical width is passed, as a global tensor knows it
    for r in range(2):
        lo, hi = fs._C.balanced_range(n, 2, r)
        part = fs._C.spmm_csr(rp, ci, v, m, k, b[:, lo:hi].contiguous(), _parallel=(r, 2, 1, n))
        assert torch.equal(part, full[:, lo:hi])
    with pytest.raises(fs.OfxError, match="physical b"):  # b slice inconsistent with logical N
        fs._C.spmm_csr(rp, ci, v, m, k, b[:, :3].contiguous(), _parallel=(0, 2, 1, n))


def _hub_problem(n=128, seed=3):
    """Rows between default_split(N) and default_split(N/4) nonzeros: chunked under the logical
    width's schedule, not under the physical slice's, so a rank that used its own width would
    compute other bits."""
    rng = np.random.default_rng(seed)
    m, k = 24, 4000
    deg = rng.integers(0, 40, size=m)
    deg[[2, 9, 17]] = [fs.ops.default_split(n) + 300, 3 * fs.ops.default_split(n) + 5, 1900]
    rp, ci, v = random_csr(m, k, deg, rng)
    return m, k, rp, ci, v, random_dense(k, n, rng)


def test_op_column_split_keeps_logical_schedule():
    """under S(1) every rank runs the hub schedule of the logical N (split =
    default_split(512) = 128, not default_split(128) = 512): each slice is bit-identical to the
    single-device op's columns."""
    n = 512
    m, k, rp, ci, v, b = _hub_problem(n)
    full = fs.spmm(rp, ci, v, m, k, b)
    assert fs.ops.default_split(n // 4) != fs.ops.default_split(n)
    for r in range(4):
        lo, hi = fs._C.balanced_range(n, 4, r)
        part = fs._C.spmm_csr(rp, ci, v, m, k, b[:, lo:hi].contiguous(), _parallel=(r, 4, 1, n))
        assert torch.equal(part.view(torch.int32), full[:, lo:hi].contiguous().view(torch.int32))
    # a rank that planned with its own width differs somewhere (the schedule is visible)
    own = fs.spmm(rp, ci, v, m, k, b[:, :32].contiguous())
    assert not torch.equal(own.view(torch.int32), full[:, :32].contiguous().view(torch.int32))


@pytest.mark.parametrize("hier", [(2, 2), (2, 4), (4, 2)])
def test_op_2d_placement_rows_x_columns(hier):
    """(S(0), S(1)) over a 2-D hierarchy: physical inference gives each rank (M/R) x (N/C) and the
    kernel cache the row range of GetTensorSliceView4ParallelId (nd_sbp_util.cpp:58-104); the
    tiles reassemble the single-device result bit for bit."""
    n = 128
    m, k, rp, ci, v, b = _hub_problem(n, seed=7)
    full = fs.spmm(rp, ci, v, m, k, b)
    R, C = hier
    got = torch.empty_like(full)
    for pid in range(R * C):
        r, c = divmod(pid, C)
        rlo, rhi = r * m // R, (r + 1) * m // R
        clo, chi = c * n // C, (c + 1) * n // C
        tile = fs._C.spmm_csr(rp, ci, v, m, k, b[:, clo:chi].contiguous(),
                              _placement_nd=dict(hierarchy=hier, nd_sbp=("S(0)", "S(1)"),
                                                 parallel_id=pid, logical_n=n))
        assert tile.shape == (rhi - rlo, chi - clo)
        got[rlo:rhi, clo:chi] = tile
    assert torch.equal(got.view(torch.int32), full.view(torch.int32))
    # the transposed placement (S(1), S(0)) splits columns first, rows second
    pid = R * C - 1
    c, r = divmod(pid, R)
    tile = fs._C.spmm_csr(rp, ci, v, m, k, b[:, c * n // C:(c + 1) * n // C].contiguous(),
                          _placement_nd=dict(hierarchy=(C, R), nd_sbp=("S(1)", "S(0)"),
                                             parallel_id=pid, logical_n=n))
    assert torch.equal(tile, full[r * m // R:(r + 1) * m // R, c * n // C:(c + 1) * n // C])


def test_op_physical_out_under_row_split_and_refusals():
    """the physical out under S(0) is the rank's BalancedSplitter slice (an out of
    the logical shape is refused); rows not divisible by a 2-D hierarchy axis are refused by the
    slice view's CHECK, as in the reference."""
    rng = np.random.default_rng(2)
    m, k, n = 10, 12, 4
    rp, ci, v = random_csr(m, k, rng.integers(0, 6, size=m), rng)
    b = random_dense(k, n, rng)
    with pytest.raises(RuntimeError, match="out must be"):
        fs._C.spmm_csr(rp, ci, v, m, k, b, out=torch.empty(m, n), _parallel=(1, 3, 0))
    o = fs._C.spmm_csr(rp, ci, v, m, k, b, out=torch.empty(3, n), _parallel=(2, 3, 0))
    assert torch.equal(o, fs.spmm(rp, ci, v, m, k, b)[7:])
    with pytest.raises(fs.OfxError, match="divisible"):
        fs._C.spmm_csr(rp, ci, v, m, k, b[:, :2].contiguous(),
                       _placement_nd=dict(hierarchy=(4, 2), nd_sbp=("S(0)", "S(1)"),
                                          parallel_id=1, logical_n=n))


def test_strided_out_and_b_column_stride_refused():
    """a 2-D out/b whose column stride is not 1 cannot be expressed to the kernel
    (it takes the row stride only) and is refused instead of written to the wrong elements;
    row-strided views stay accepted."""
    rp, ci, v, b = _small()
    buf = torch.zeros(6, 10)
    with pytest.raises(RuntimeError, match="unit column stride"):
        fs.spmm(rp, ci, v, 6, 9, b, out=buf[:, ::2])
    assert torch.count_nonzero(buf) == 0
    wide = torch.zeros(6, 8)
    r = fs.spmm(rp, ci, v, 6, 9, b, out=wide[:, 1:6])
    assert torch.equal(r, fs.spmm(rp, ci, v, 6, 9, b)) and torch.count_nonzero(wide[:, 6:]) == 0
    desc_b = fs._C.desc(b.t().contiguous().t())  # column-major b, passed raw to the C-ABI
    from oneflow_spmm._lib import LIB, TensorDesc
    import ctypes
    d = [fs._C.desc(x) for x in (rp, ci, v)]
    o = torch.empty(6, 5)
    d_o = fs._C.desc(o)
    rc = LIB.ofx_functional_spmm_csr(None, *[ctypes.byref(x) for x in d], 6, 9,
                                     ctypes.byref(desc_b), ctypes.byref(d_o), None, 0)
    assert rc != 0 and "unit column stride" in fs._lib.last_error()
    # fused op path: the same refusal
    with pytest.raises(RuntimeError, match="unit column stride"):
        fs._C.fused_spmm_csr(rp, ci, v, 6, 9, b, torch.zeros(5), out=buf[:, ::2])
    assert TensorDesc is not None


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
    # the small form (one launch, no plan): <= 32768 rows, <= 2^17 nonzeros and <= 2^23
    # products nnz * n (spmm_launch.h)
    for m, n, nnz, small in [(32768, 16, 65536, True), (32769, 16, 65536, False),
                             (2708, 16, 10556, True), (2708, 128, 10556, True),
                             (19717, 64, 88648, True), (19717, 128, 88648, False),
                             (20000, 16, 131072, True), (20000, 16, 131073, False),
                             (1000, 300, 27962, True), (1000, 300, 27963, False)]:
        assert L.ofx_spmm_csr_workspace_size(5, 2, m, m, n, nnz, None, ctypes.byref(sz)) == 0
        assert (sz.value == 0) == small, (m, n, nnz)
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
