"""Op "fused_spmm_csr" (SURVEY.md §8f row 4): relu?(A @ b + bias?) in one kernel must give the
bits of spmm_csr -> bias_add -> relu run as separate ops (oracle.bias_act over oracle.spmm), on
the CPU kernel and the HIP kernel, including hub rows (their epilogue runs in the reduce
kernel), int64 indices and strided outputs; autograd matches an fp64 dense composition."""
import numpy as np
import pytest
import torch

import oneflow_spmm as fs
from oneflow_spmm import _C, ops
from oracle import oracle

from helpers import (DTYPES, assert_bitwise, from_f32, oracle_spmm, power_law_degrees, random_csr,
                     random_dense, to_oracle)


def _problem(seed, m, k, n, dtype, idx=torch.int32, hubs=False):
    rng = np.random.default_rng(seed)
    deg = power_law_degrees(m, 60 * m, k, rng) if hubs else rng.integers(0, 30, size=m)
    if not hubs:
        deg[::7] = 0  # empty rows: the epilogue still runs (out = relu?(0 + bias))
    rp, ci, v = random_csr(m, k, deg, rng, idx_dtype=idx, val_dtype=DTYPES[dtype])
    b = random_dense(k, n, rng, dtype=DTYPES[dtype])
    bias = from_f32(rng.uniform(-0.5, 0.5, n).astype(np.float32), DTYPES[dtype])
    if n > 3:  # signed zeros in the bias: -0 + +0 sums, relu(-0) -> +0
        bias[1] = -0.0
        bias[2] = 0.0
    return rp, ci, v, b, bias


def _ref(rp, ci, v, b, bias, relu, dtype):
    c = oracle_spmm(rp, ci, v, b)
    return oracle.bias_act(c, None if bias is None else to_oracle(bias),
                           "relu" if relu else "none", dtype=dtype)


@pytest.mark.parametrize("dtype", ["f32", "f64", "bf16", "f16"])
@pytest.mark.parametrize("with_bias,relu", [(True, True), (True, False), (False, True)])
def test_cpu_fused_matches_composition(dtype, with_bias, relu):
    rp, ci, v, b, bias = _problem(11, 90, 70, 24, dtype)
    bias = bias if with_bias else None
    got = _C.fused_spmm_csr(rp, ci, v, 90, 70, b, bias, relu=relu)
    assert_bitwise(got, _ref(rp, ci, v, b, bias, relu, dtype), f"cpu fused {dtype}")


def test_fused_without_epilogue_is_spmm():
    rp, ci, v, b, _ = _problem(12, 50, 40, 16, "f32")
    assert torch.equal(_C.fused_spmm_csr(rp, ci, v, 50, 40, b).view(torch.int32),
                       fs.spmm(rp, ci, v, 50, 40, b).view(torch.int32))


def test_cpu_fused_static_csr_is_accepted_and_exact():
    """The kCPU kernel has no work list: static_csr changes nothing but must be accepted, through
    the op (_C) and its autograd binding."""
    rp, ci, v, b, bias = _problem(13, 90, 70, 24, "f32")
    ref = _ref(rp, ci, v, b, bias, True, "f32")
    assert_bitwise(_C.fused_spmm_csr(rp, ci, v, 90, 70, b, bias, relu=True, static_csr=3), ref,
                   "cpu fused static")
    bb = b.clone().requires_grad_(True)
    y = fs.fused_spmm(rp, ci, v, 90, 70, bb, bias, relu=True, static_csr=3)
    assert_bitwise(y.detach(), ref, "cpu fused static (autograd)")
    y.sum().backward()
    assert bb.grad is not None and torch.isfinite(bb.grad).all()


def test_oracle_bias_act_by_hand():
    c = np.array([[1.5, -0.0, -2.0, 0.25]], dtype=np.float32)
    bias = np.array([-1.5, 0.0, 1.0, -1.0], dtype=np.float32)
    y = oracle.bias_act(c, bias, "relu")
    assert y.tolist() == [[0.0, 0.0, 0.0, 0.0]] and not np.signbit(y).any()
    y = oracle.bias_act(c, bias, "none")
    assert y.tolist() == [[0.0, 0.0, -1.0, -0.75]]
    assert not np.signbit(y[0, 1])  # -0 + +0 = +0 (round to nearest)
    # relu keeps NaN and maps -0 to +0
    y = oracle.bias_act(np.array([[np.nan, -0.0]], dtype=np.float32), None, "relu")
    assert np.isnan(y[0, 0]) and y[0, 1] == 0 and not np.signbit(y[0, 1])


def test_fused_op_errors():
    rp, ci, v, b, bias = _problem(13, 20, 40, 8, "f32")
    with pytest.raises(fs.OfxError, match="bias length"):
        _C.fused_spmm_csr(rp, ci, v, 20, 40, b, bias[:5])
    with pytest.raises(TypeError, match="bias datatype"):
        _C.fused_spmm_csr(rp, ci, v, 20, 40, b, bias.double())


def test_cpu_fused_autograd_matches_fp64_dense():
    rng = np.random.default_rng(14)
    m, k, n = 60, 45, 20
    rp, ci, v = random_csr(m, k, rng.integers(0, 9, size=m), rng)
    b = random_dense(k, n, rng)
    bias = torch.from_numpy(rng.uniform(-0.5, 0.5, n).astype(np.float32))
    vv, bb, bs = (t.clone().requires_grad_(True) for t in (v, b, bias))
    out = fs.fused_spmm(rp, ci, vv, m, k, bb, bs, relu=True)
    g = torch.from_numpy(rng.uniform(-1, 1, (m, n)).astype(np.float32))
    out.backward(g)
    v64, b64, s64 = (t.double().requires_grad_(True) for t in (v, b, bias))
    rows = torch.repeat_interleave(torch.arange(m), torch.diff(rp.long()))
    a64 = torch.zeros(m, k, dtype=torch.float64).index_put((rows, ci.long()), v64)
    torch.relu(a64 @ b64 + s64).backward(g.double())
    for got, want in ((vv.grad, v64.grad), (bb.grad, b64.grad), (bs.grad, s64.grad)):
        torch.testing.assert_close(got.double(), want, rtol=0, atol=1e-5)


# ---- HIP kernel ------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f32", "f64", "bf16", "f16"])
@pytest.mark.parametrize("n", [1, 24, 128, 130])
def test_gpu_fused_bitexact(device, dtype, n):
    rp, ci, v, b, bias = _problem(21, 400, 300, n, dtype)
    for with_bias, relu in ((True, True), (True, False), (False, True)):
        bs = bias if with_bias else None
        got = _C.fused_spmm_csr(rp.to(device), ci.to(device), v.to(device), 400, 300, b.to(device),
                                None if bs is None else bs.to(device), relu=relu)
        torch.cuda.synchronize()
        assert_bitwise(got, _ref(rp, ci, v, b, bs, relu, dtype), f"gpu fused {dtype} n={n}")


@pytest.mark.gpu
@pytest.mark.parametrize("idx", [torch.int32, torch.int64])
def test_gpu_fused_hub_rows_and_strided_out(device, idx):
    """Hub rows > 2 x default_split(128): their epilogue runs in the reduce kernel."""
    m, k, n = 700, 4000, 128
    rp, ci, v, b, bias = _problem(22, m, k, n, "f32", idx=idx, hubs=True)
    assert int(torch.diff(rp.long()).max()) > 2 * ops.default_split(n)
    big = torch.full((m, n + 8), float("nan"), device=device)
    out = big[:, 4:4 + n]  # row stride n + 8, offset 16 B
    kern = ops.SpmmCsrKernel(m, k, n, ci.numel(), idx, torch.float32, device)
    kern(rp.to(device), ci.to(device), v.to(device), b.to(device), out, bias=bias.to(device),
         relu=True)
    torch.cuda.synchronize()
    assert_bitwise(out, _ref(rp, ci, v, b, bias, True, "f32"), "hub rows fused")
    assert torch.isnan(big[:, :4]).all() and torch.isnan(big[:, 4 + n:]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_gpu_fused_static_csr_plans_once(device, dtype):
    """static_csr on the fused op: its kernel state plans the CSR once (hub rows: a real work
    list), later calls reuse the plan, and every call keeps the composition's bits."""
    m, k, n = 20_000, 20_000, 64
    rp, ci, v, b, bias = _problem(24, m, k, n, dtype, hubs=True)
    ref = _ref(rp, ci, v, b, bias, True, dtype)
    d = [rp.to(device), ci.to(device), v.to(device)]
    db, dbias = b.to(device), bias.to(device)
    _C.static_plans(release=True)
    s0 = _C.static_plans()
    outs = [_C.fused_spmm_csr(*d, m, k, db, dbias, relu=True, static_csr=5) for _ in range(3)]
    torch.cuda.synchronize()
    s1 = _C.static_plans()
    assert (s1["plans"] - s0["plans"], s1["hits"] - s0["hits"]) == (1, 2), (s0, s1)
    for i, o in enumerate(outs):
        assert_bitwise(o, ref, f"fused static call {i}")
    _C.static_plans(release=True)


@pytest.mark.gpu
def test_gpu_fused_autograd_matches_cpu(device):
    rng = np.random.default_rng(23)
    m, k, n = 300, 250, 32
    rp, ci, v = random_csr(m, k, rng.integers(0, 20, size=m), rng)
    b = random_dense(k, n, rng)
    bias = torch.from_numpy(rng.uniform(-0.5, 0.5, n).astype(np.float32))
    g = torch.from_numpy(rng.uniform(-1, 1, (m, n)).astype(np.float32))
    grads = []
    for dev in ("cpu", device):
        vv, bb, bs = (t.to(dev).clone().requires_grad_(True) for t in (v, b, bias))
        out = fs.fused_spmm(rp.to(dev), ci.to(dev), vv, m, k, bb, bs, relu=True)
        out.backward(g.to(dev))
        grads.append([out.detach().cpu(), vv.grad.cpu(), bb.grad.cpu()])
    for a, c in zip(*grads):  # forward, d values (SDDMM) and dB are bit-identical CPU vs GPU
        assert torch.equal(a.view(torch.int32), c.view(torch.int32))


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f64"])
@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("m", [0, 5, 2048, 2049, 40000])
def test_cpu_relu_bias_grad_bitexact(dtype, relu, m):
    """The fused epilogue's backward on the host (ofx_relu_bias_grad_cpu): dx and the bias
    column sum equal the oracle's restatement of the stated order bit for bit (chunk edges at
    2048 rows, more than 8 chunks at 40000 rows, an empty batch)."""
    from oneflow_spmm import ops
    rng = np.random.default_rng(m + 3)
    n = 13
    y = random_dense(m, n, rng, DTYPES[dtype])
    dy = random_dense(m, n, rng, DTYPES[dtype])
    dx, db = ops.relu_bias_grad(y, dy, relu=relu, bias_grad=True)
    ref_dx, ref_db = oracle.relu_bias_grad(to_oracle(y), to_oracle(dy), relu=relu, dtype=dtype)
    assert_bitwise(dx, ref_dx, "dx")
    assert_bitwise(db, ref_db, "d_bias")
    if m:
        exact = (torch.where(y > 0, dy, torch.zeros_like(dy)) if relu else dy).double().sum(0)
        assert torch.allclose(db.double(), exact, rtol=1e-2 if dtype == "bf16" else 1e-5, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16", "f64"])
@pytest.mark.parametrize("m,n", [(0, 7), (3, 300), (2049, 64), (70001, 129)])
def test_gpu_relu_bias_grad_bitexact(device, dtype, m, n):
    """ofx_relu_bias_grad on the device: same bits as the oracle and as the CPU kernel."""
    from oneflow_spmm import ops
    rng = np.random.default_rng(m + n)
    y = random_dense(m, n, rng, DTYPES[dtype])
    dy = random_dense(m, n, rng, DTYPES[dtype])
    dx, db = ops.relu_bias_grad(y.to(device), dy.to(device), relu=True, bias_grad=True)
    _, db_only = ops.relu_bias_grad(y.to(device), dy.to(device), relu=False, bias_grad=True)
    torch.cuda.synchronize()
    ref_dx, ref_db = oracle.relu_bias_grad(to_oracle(y), to_oracle(dy), relu=True, dtype=dtype)
    assert_bitwise(dx, ref_dx, "dx")
    assert_bitwise(db, ref_db, "d_bias")
    assert_bitwise(db_only, oracle.relu_bias_grad(to_oracle(y), to_oracle(dy), relu=False,
                                                  dtype=dtype)[1], "d_bias without relu")
    cdx, cdb = ops.relu_bias_grad(y, dy, relu=True, bias_grad=True)
    assert_bitwise(dx, to_oracle(cdx), "dx vs the CPU kernel")
    assert_bitwise(db, to_oracle(cdb), "d_bias vs the CPU kernel")
