"""Gradient path: CSR transpose, SDDMM and autograd through `spmm`.

CPU tests pin the kCPU kernels and the oracle against independent references (numpy stable sort,
scipy, fp64 dense torch autograd); GPU tests check the HIP kernels bit-for-bit against the oracle.
"""
import numpy as np
import pytest
import torch

import oneflow_spmm as fs
from oracle import oracle
from tests.helpers import (DTYPES, assert_bitwise, oracle_spmm, power_law_degrees, random_csr,
                           random_dense, to_oracle)


def _dense64(rp, ci, vals, m, k):
    rows = torch.repeat_interleave(torch.arange(m), torch.diff(rp.long()))
    a = torch.zeros(m, k, dtype=torch.float64)
    return a.index_put((rows, ci.long()), vals.double(), accumulate=False), rows


# ---- oracle pinned against independent references ---------------------------------------------
def test_oracle_transpose_matches_scipy():
    import scipy.sparse as sp
    rng = np.random.default_rng(0)
    m, k = 80, 50
    rp, ci, v = random_csr(m, k, rng.integers(0, 12, size=m), rng)
    rt, ct, perm = oracle.transpose(rp.numpy(), ci.numpy(), k)
    at = sp.csr_matrix((v.numpy(), ci.numpy(), rp.numpy()), shape=(m, k)).T.tocsr()
    at.sort_indices()
    np.testing.assert_array_equal(rt, at.indptr)
    np.testing.assert_array_equal(ct, at.indices)
    np.testing.assert_array_equal(v.numpy()[perm], at.data)


def test_oracle_sddmm_close_to_fp64_and_exact_on_integers():
    rng = np.random.default_rng(1)
    m, k = 60, 70
    for n in (1, 7, 8, 9, 64, 100, 600):
        rp, ci, v = random_csr(m, k, rng.integers(0, 8, size=m), rng)
        a = rng.uniform(-1, 1, (m, n)).astype(np.float32)
        b = rng.uniform(-1, 1, (k, n)).astype(np.float32)
        got = oracle.sddmm(rp.numpy(), ci.numpy(), a, b)
        rows = np.repeat(np.arange(m), np.diff(rp.numpy()))
        ref = np.einsum("jn,jn->j", a[rows].astype(np.float64), b[ci.numpy()].astype(np.float64))
        absum = np.einsum("jn,jn->j", np.abs(a[rows]).astype(np.float64), np.abs(b[ci.numpy()]).astype(np.float64))
        assert np.all(np.abs(got - ref) <= 1e-6 * absum + 1e-30), n
        ai = rng.integers(-8, 9, (m, n)).astype(np.float32)
        bi = rng.integers(-8, 9, (k, n)).astype(np.float32)
        got = oracle.sddmm(rp.numpy(), ci.numpy(), ai, bi)
        np.testing.assert_array_equal(got, np.einsum("jn,jn->j", ai[rows], bi[ci.numpy()]))


def test_oracle_sddmm_pairwise_order_by_hand():
    rng = np.random.default_rng(2)
    rp = np.array([0, 1], dtype=np.int64)
    ci = np.array([0], dtype=np.int64)
    n = 40  # 5 leaves -> padded to 8
    a = rng.uniform(-1, 1, (1, n)).astype(np.float32)
    b = rng.uniform(-1, 1, (1, n)).astype(np.float32)
    leaves = []
    for l in range(8):
        s = np.float32(0)
        for e in range(8 * l, min(8 * l + 8, n)):
            s = np.float32(s + np.float32(a[0, e] * b[0, e]))
        leaves.append(s)
    while len(leaves) > 1:
        leaves = [np.float32(leaves[i] + leaves[i + 1]) for i in range(0, len(leaves), 2)]
    assert oracle.sddmm(rp, ci, a, b)[0] == leaves[0]


# ---- kCPU kernels vs oracle ------------------------------------------------------------------
@pytest.mark.parametrize("idx", [torch.int32, torch.int64])
def test_cpu_transpose_bitexact(idx):
    rng = np.random.default_rng(3)
    m, k = 300, 211
    rp, ci, v = random_csr(m, k, power_law_degrees(m, 3000, k, rng), rng, idx)
    rt, ct, perm = fs.csr_transpose(rp, ci, k)
    ort, oct_, opt = oracle.transpose(rp.numpy(), ci.numpy(), k)
    assert rt.dtype == idx
    np.testing.assert_array_equal(rt.numpy(), ort)
    np.testing.assert_array_equal(ct.numpy(), oct_)
    np.testing.assert_array_equal(perm.numpy(), opt)


@pytest.mark.parametrize("dtype", ["f32", "f64", "bf16", "f16"])
@pytest.mark.parametrize("n", [3, 16, 128])
def test_cpu_sddmm_bitexact(dtype, n):
    rng = np.random.default_rng(n)
    m, k = 120, 90
    rp, ci, v = random_csr(m, k, rng.integers(0, 20, size=m), rng)
    a = random_dense(m, n, rng, DTYPES[dtype])
    b = random_dense(k, n, rng, DTYPES[dtype])
    got = fs.sddmm(rp, ci, a, b)
    ref = oracle.sddmm(rp.numpy(), ci.numpy(), to_oracle(a), to_oracle(b), dtype=dtype)
    assert_bitwise(got, ref, f"cpu sddmm {dtype}")


def test_cpu_autograd_matches_fp64_dense():
    rng = np.random.default_rng(4)
    m, k, n = 70, 55, 24
    rp, ci, v = random_csr(m, k, rng.integers(0, 9, size=m), rng)
    b = random_dense(k, n, rng)
    vv, bb = v.clone().requires_grad_(True), b.clone().requires_grad_(True)
    out = fs.spmm(rp, ci, vv, m, k, bb)
    g = torch.from_numpy(rng.uniform(-1, 1, (m, n)).astype(np.float32))
    out.backward(g)
    v64 = v.double().requires_grad_(True)
    b64 = b.double().requires_grad_(True)
    rows = torch.repeat_interleave(torch.arange(m), torch.diff(rp.long()))
    a64 = torch.zeros(m, k, dtype=torch.float64).index_put((rows, ci.long()), v64)
    (a64 @ b64).backward(g.double())
    torch.testing.assert_close(vv.grad.double(), v64.grad, rtol=0, atol=1e-5)
    torch.testing.assert_close(bb.grad.double(), b64.grad, rtol=0, atol=1e-5)
    # the dB path is exactly the forward contract on A^T
    rt, ct, perm = oracle.transpose(rp.numpy(), ci.numpy(), k)
    ref_db = oracle.spmm(rt, ct, v.numpy()[perm], g.numpy())
    assert_bitwise(bb.grad, ref_db, "dB = A^T dC")


def test_spmm_out_argument_with_grad_is_rejected():
    rng = np.random.default_rng(5)
    rp, ci, v = random_csr(5, 5, rng.integers(0, 3, size=5), rng)
    b = random_dense(5, 4, rng).requires_grad_(True)
    with pytest.raises(RuntimeError, match="out="):
        fs.spmm(rp, ci, v, 5, 5, b, out=torch.empty(5, 4))


# ---- HIP kernels vs oracle -----------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("idx", [torch.int32, torch.int64])
def test_gpu_transpose_bitexact(device, idx):
    rng = np.random.default_rng(6)
    m, k = 5000, 3000
    rp, ci, v = random_csr(m, k, power_law_degrees(m, 80000, k, rng), rng, idx)
    rt, ct, perm = fs.csr_transpose(rp.to(device), ci.to(device), k)
    torch.cuda.synchronize()
    ort, oct_, opt = oracle.transpose(rp.numpy(), ci.numpy(), k)
    np.testing.assert_array_equal(rt.cpu().numpy(), ort)
    np.testing.assert_array_equal(ct.cpu().numpy(), oct_)
    np.testing.assert_array_equal(perm.cpu().numpy(), opt)
    vt = fs.autograd.gather_values(perm, v.to(device))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(vt.cpu().numpy(), v.numpy()[opt])


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16", "f64"])
@pytest.mark.parametrize("n", [1, 5, 8, 16, 64, 128, 256, 520, 1024])
def test_gpu_sddmm_bitexact(device, dtype, n):
    rng = np.random.default_rng(100 + n)
    m, k = 400, 300
    deg = rng.integers(0, 25, size=m)
    deg[17] = 290
    rp, ci, v = random_csr(m, k, deg, rng)
    a = random_dense(m, n, rng, DTYPES[dtype])
    b = random_dense(k, n, rng, DTYPES[dtype])
    got = fs.sddmm(rp.to(device), ci.to(device), a.to(device), b.to(device))
    torch.cuda.synchronize()
    ref = oracle.sddmm(rp.numpy(), ci.numpy(), to_oracle(a), to_oracle(b), dtype=dtype)
    assert_bitwise(got, ref, f"gpu sddmm {dtype} n={n}")


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,n", [("f32", 2049), ("f32", 4096), ("bf16", 5000), ("f64", 3000),
                                     ("f32", 20003), ("f16", 8192)])
def test_gpu_sddmm_wide_rows_bitexact(device, dtype, n):
    """n > 2048: 256-leaf tiles whose pairwise trees are added pairwise (the same order as one
    tree over all padded leaves), including a hub row split by the planner and unaligned n."""
    rng = np.random.default_rng(200 + n)
    m, k = 60, 900
    deg = rng.integers(0, 30, size=m)
    deg[5] = 850
    rp, ci, v = random_csr(m, k, deg, rng)
    a = random_dense(m, n, rng, DTYPES[dtype])
    b = random_dense(k, n, rng, DTYPES[dtype])
    got = fs.sddmm(rp.to(device), ci.to(device), a.to(device), b.to(device))
    torch.cuda.synchronize()
    ref = oracle.sddmm(rp.numpy(), ci.numpy(), to_oracle(a), to_oracle(b), dtype=dtype)
    assert_bitwise(got, ref, f"gpu wide sddmm {dtype} n={n}")
    cpu = fs.sddmm(rp, ci, a, b)  # the CPU kernel: same bits
    assert_bitwise(cpu, ref, f"cpu wide sddmm {dtype} n={n}")


@pytest.mark.gpu
def test_gpu_sddmm_hub_rows_and_unaligned(device):
    rng = np.random.default_rng(7)
    m, k, n = 30, 70000, 128
    deg = rng.integers(0, 50, size=m)
    deg[2] = 60000  # hub row: split into chunks by the planner (no numeric effect)
    rp, ci, v = random_csr(m, k, deg, rng)
    a = random_dense(m, n, rng)
    b = random_dense(k, n, rng)
    ref = oracle.sddmm(rp.numpy(), ci.numpy(), a.numpy(), b.numpy())
    got = fs.sddmm(rp.to(device), ci.to(device), a.to(device), b.to(device))
    torch.cuda.synchronize()
    assert_bitwise(got, ref, "hub sddmm")
    big = torch.zeros(k * n + 1)
    big[1:] = b.reshape(-1)
    b_un = big.to(device)[1:].view(k, n)  # not 16-B aligned -> scalar leaf loads
    got = fs.sddmm(rp.to(device), ci.to(device), a.to(device), b_un)
    torch.cuda.synchronize()
    assert_bitwise(got, ref, "unaligned sddmm")


@pytest.mark.gpu
def test_gpu_autograd_bitexact_vs_oracle(device):
    rng = np.random.default_rng(8)
    m, k, n = 20000, 15000, 64
    rp, ci, v = random_csr(m, k, power_law_degrees(m, 300000, k, rng), rng)
    b = random_dense(k, n, rng)
    g = random_dense(m, n, rng)
    vv = v.to(device).requires_grad_(True)
    bb = b.to(device).requires_grad_(True)
    rp_d, ci_d = rp.to(device), ci.to(device)
    out = fs.spmm(rp_d, ci_d, vv, m, k, bb)
    out.backward(g.to(device))
    torch.cuda.synchronize()
    assert_bitwise(out, oracle_spmm(rp, ci, v, b), "forward")
    assert_bitwise(vv.grad, oracle.sddmm(rp.numpy(), ci.numpy(), g.numpy(), b.numpy()), "d values")
    rt, ct, perm = oracle.transpose(rp.numpy(), ci.numpy(), k)
    assert_bitwise(bb.grad, oracle.spmm(rt, ct, v.numpy()[perm], g.numpy()), "d b")
    # second backward reuses the cached transpose
    vv.grad = None
    bb.grad = None
    n_cached = len(fs.autograd.TRANSPOSE_CACHE.entries)
    fs.spmm(rp_d, ci_d, vv, m, k, bb).backward(g.to(device))
    assert len(fs.autograd.TRANSPOSE_CACHE.entries) == n_cached
    torch.cuda.synchronize()
    assert_bitwise(bb.grad, oracle.spmm(rt, ct, v.numpy()[perm], g.numpy()), "d b (cached)")


def test_grad_ops_through_op_layer_errors_and_sbp():
    rng = np.random.default_rng(9)
    m, k, n = 10, 12, 6
    rp, ci, v = random_csr(m, k, rng.integers(0, 4, size=m), rng)
    a = random_dense(m, n, rng)
    b = random_dense(k, n, rng)
    with pytest.raises(RuntimeError, match="same number of columns"):
        fs._C.sddmm_csr(rp, ci, a[:, :4].contiguous(), b, m, k)
    with pytest.raises(RuntimeError, match="a_num_rows rows"):
        fs._C.sddmm_csr(rp, ci, a[:5].contiguous(), b, m, k)
    with pytest.raises(TypeError, match="a datatype"):
        fs._C.sddmm_csr(rp, ci, a.double(), b, m, k)
    with pytest.raises(RuntimeError, match="a_num_rows"):
        fs._C.csr_transpose(rp, ci, m + 1, k)
    assert fs._C.sddmm_csr(rp, ci, a[:, :0], b[:, :0], m, k).abs().sum() == 0
    rt, ct, perm = fs._C.csr_transpose(rp, ci, m, k)
    assert rt.shape == (k + 1,) and ct.shape == ci.shape and perm.dtype == rp.dtype


def test_transposed_values_cache_follows_inplace_updates():
    """dB uses A^T's values from a cache keyed on the values' storage and version: an in-place
    update of the values (an optimizer step on edge weights) must be seen by the next backward."""
    from oneflow_spmm.autograd import TRANSPOSE_CACHE
    rng = np.random.default_rng(31)
    m, k, n = 40, 30, 8
    rp, ci, v = random_csr(m, k, rng.integers(0, 6, size=m), rng)
    b = random_dense(k, n, rng)
    g = torch.from_numpy(rng.uniform(-1, 1, (m, n)).astype(np.float32))
    vv = v.clone().requires_grad_(True)
    rt, ct, perm = oracle.transpose(rp.numpy(), ci.numpy(), k)
    for step in range(3):
        bb = b.clone().requires_grad_(True)
        fs.spmm(rp, ci, vv, m, k, bb).backward(g)
        ref_db = oracle.spmm(rt, ct, vv.detach().numpy()[perm], g.numpy())
        assert_bitwise(bb.grad, ref_db, f"dB step {step}")
        with torch.no_grad():
            vv.mul_(0.5).add_(0.25)
    assert len(TRANSPOSE_CACHE.value_entries) <= TRANSPOSE_CACHE.capacity


@pytest.mark.gpu
@pytest.mark.parametrize("idx", [torch.int32, torch.int64])
@pytest.mark.parametrize("dtype,n", [("f32", 64), ("f32", 256), ("bf16", 128), ("f64", 17)])
def test_gpu_spmm_gathered_values(device, idx, dtype, n):
    """ofx_spmm_csr_gathered (values read through perm inside the SpMM) equals the SpMM on the
    gathered copy, bit for bit: on A^T of a hub-heavy graph (LPR < 64 and the wave-uniform
    LPR = 64 path, hub chunks)."""
    from oneflow_spmm import ops
    rng = np.random.default_rng(40 + n)
    m, k = 6000, 5000
    rp, ci, v = random_csr(m, k, power_law_degrees(m, 200000, k, rng), rng, idx, DTYPES[dtype])
    npi = np.int32 if idx == torch.int32 else np.int64
    rt, ct, perm = (x.astype(npi) for x in oracle.transpose(rp.numpy(), ci.numpy(), k))
    g = random_dense(m, n, rng, DTYPES[dtype])
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
    out = ops.spmm_csr_gathered(d(rt), d(ct), v.to(device), d(perm), g.to(device), k, m)
    out_op = fs._C.spmm_csr_gathered(d(rt), d(ct), v.to(device), d(perm), k, m, g.to(device))
    torch.cuda.synchronize()
    vals = to_oracle(v)[perm]
    ref = oracle.spmm(rt, ct, vals, to_oracle(g), dtype=dtype)
    assert_bitwise(out, ref, f"{dtype} n={n}")
    assert_bitwise(out_op, ref, f"op layer {dtype} n={n}")


@pytest.mark.gpu
def test_gpu_learnable_values_backward(device):
    """Edge weights updated in place every step: each backward reads them through perm
    (no stale cached copy), bit-exact against the oracle on the current values."""
    from oneflow_spmm.autograd import TRANSPOSE_CACHE
    rng = np.random.default_rng(44)
    m, k, n = 3000, 2500, 32
    rp, ci, v = random_csr(m, k, power_law_degrees(m, 60000, k, rng), rng)
    b = random_dense(k, n, rng)
    g = random_dense(m, n, rng)
    rt, ct, perm = oracle.transpose(rp.numpy(), ci.numpy(), k)
    rp_d, ci_d, g_d = rp.to(device), ci.to(device), g.to(device)
    vv = v.to(device).requires_grad_(True)
    for step in range(3):
        bb = b.to(device).requires_grad_(True)
        fs.spmm(rp_d, ci_d, vv, m, k, bb).backward(g_d)
        torch.cuda.synchronize()
        ref = oracle.spmm(rt, ct, vv.detach().cpu().numpy()[perm], g.numpy())
        assert_bitwise(bb.grad, ref, f"dB step {step}")
        with torch.no_grad():
            vv.mul_(0.5).add_(0.25)
    assert len(TRANSPOSE_CACHE.seen) <= TRANSPOSE_CACHE.capacity


@pytest.mark.parametrize("idx", [torch.int32, torch.int64])
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_cpu_spmm_csr_gathered_op(idx, dtype):
    """Op "spmm_csr_gathered" through the op layer on CPU (its kCPU kernel gathers the values
    into the tmp buffer and runs the CPU SpMM): bit-exact vs the oracle on values[perm]; shape
    and dtype errors from the op's inference; SBP signatures with values_perm broadcast."""
    rng = np.random.default_rng(12)
    m, k, n = 120, 90, 9
    rp, ci, v = random_csr(m, k, power_law_degrees(m, 3000, k, rng), rng, idx, DTYPES[dtype])
    rt, ct, perm = fs.csr_transpose(rp, ci, k)
    g = random_dense(m, n, rng, DTYPES[dtype])
    out = fs._C.spmm_csr_gathered(rt, ct, v, perm, k, m, g)
    ref = oracle.spmm(rt.numpy(), ct.numpy(), to_oracle(v)[perm.numpy()], to_oracle(g), dtype=dtype)
    assert_bitwise(out, ref, f"gathered op {dtype}/{idx}")
    with pytest.raises(RuntimeError, match="values_perm should have nnz"):
        fs._C.spmm_csr_gathered(rt, ct, v, perm[:-1].contiguous(), k, m, g)
    with pytest.raises(TypeError, match="values_perm should have the dtype"):
        other = torch.int64 if idx == torch.int32 else torch.int32
        fs._C.spmm_csr_gathered(rt, ct, v, perm.to(other), k, m, g)
    sig = fs._C.sbp_signatures("spmm_csr_gathered")
    assert "values_perm:B" in sig and "out:S(0)" in sig and "out:S(1)" in sig
    assert "values_perm" in sig.split("|no_grad:")[1]
