"""COO (edge_index) -> CSR construction against the oracle (numpy stable
sort + sequential duplicate sums) and scipy; CPU kernel here, HIP kernel on the GPU box."""
import numpy as np
import pytest
import torch

import oneflow_spmm as fs
from oracle import oracle
from tests.helpers import DTYPES, from_f32, to_oracle


def _coo(m, k, nnz, rng, dup_frac=0.3, dtype=torch.float32, idx=torch.int32):
    row = rng.integers(0, m, nnz)
    col = rng.integers(0, k, nnz)
    nd = int(nnz * dup_frac)
    if nd:  # force duplicates
        src = rng.integers(0, nnz, nd)
        dst = rng.integers(0, nnz, nd)
        row[dst], col[dst] = row[src], col[src]
    vals = from_f32(rng.uniform(-1, 1, nnz).astype(np.float32), dtype)
    np_idx = np.int32 if idx == torch.int32 else np.int64
    return torch.from_numpy(row.astype(np_idx)), torch.from_numpy(col.astype(np_idx)), vals


def _check(got, ref, dtype):
    rp, ci, v = got
    orp, oci, ov = ref
    np.testing.assert_array_equal(rp.cpu().numpy(), orp)
    np.testing.assert_array_equal(ci.cpu().numpy(), oci)
    if ov is not None:
        g = to_oracle(v)
        assert np.array_equal(np.ascontiguousarray(g).view(np.uint8), np.ascontiguousarray(ov).view(np.uint8))


@pytest.mark.parametrize("merge", [True, False])
@pytest.mark.parametrize("dtype", ["f32", "bf16", "f64"])
def test_cpu_coo_to_csr(merge, dtype):
    rng = np.random.default_rng(1)
    m, k = 50, 40
    row, col, v = _coo(m, k, 600, rng, dtype=DTYPES[dtype])
    got = fs.coo_to_csr(row, col, v, m, k, merge)
    ref = oracle.coo_to_csr(row.numpy(), col.numpy(), to_oracle(v), m, k, merge, dtype)
    _check(got, ref, dtype)


def test_oracle_coo_to_csr_matches_scipy():
    import scipy.sparse as sp
    rng = np.random.default_rng(2)
    m, k = 30, 20
    row, col, v = _coo(m, k, 300, rng)
    rp, ci, vals = oracle.coo_to_csr(row.numpy(), col.numpy(), v.numpy(), m, k, True)
    a = sp.coo_matrix((v.numpy().astype(np.float64), (row.numpy(), col.numpy())), shape=(m, k)).tocsr()
    a.sum_duplicates()
    np.testing.assert_array_equal(rp, a.indptr)
    np.testing.assert_array_equal(ci, a.indices)
    np.testing.assert_allclose(vals, a.data, rtol=0, atol=1e-5)


def test_cpu_coo_errors_and_structure_only():
    row = torch.tensor([0, 5], dtype=torch.int32)
    col = torch.tensor([0, 1], dtype=torch.int32)
    with pytest.raises(RuntimeError, match="outside"):
        fs.coo_to_csr(row, col, None, 3, 3)
    rp, ci, v = fs.coo_to_csr(torch.tensor([2, 0, 2], dtype=torch.int32),
                              torch.tensor([1, 1, 1], dtype=torch.int32), None, 3, 3)
    assert rp.tolist() == [0, 1, 1, 2] and ci.tolist() == [1, 1] and v is None
    rp, ci, v = fs.coo_to_csr(torch.zeros(0, dtype=torch.int64), torch.zeros(0, dtype=torch.int64),
                              torch.zeros(0), 4, 4)
    assert rp.tolist() == [0] * 5 and ci.numel() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("merge", [True, False])
@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16", "f64"])
@pytest.mark.parametrize("idx", [torch.int32, torch.int64])
def test_gpu_coo_to_csr(device, merge, dtype, idx):
    rng = np.random.default_rng(3)
    m, k = 3000, 2000
    row, col, v = _coo(m, k, 40000, rng, dtype=DTYPES[dtype], idx=idx)
    got = fs.coo_to_csr(row.to(device), col.to(device), v.to(device), m, k, merge)
    torch.cuda.synchronize()
    ref = oracle.coo_to_csr(row.numpy(), col.numpy(), to_oracle(v), m, k, merge, dtype)
    _check(got, ref, dtype)


@pytest.mark.gpu
def test_gpu_coo_to_csr_feeds_spmm_and_flags_bad(device):
    rng = np.random.default_rng(4)
    m, k, n = 5000, 4000, 64
    row, col, v = _coo(m, k, 60000, rng)
    rp, ci, vals = fs.coo_to_csr(row.to(device), col.to(device), v.to(device), m, k)
    b = torch.from_numpy(rng.uniform(-1, 1, (k, n)).astype(np.float32))
    out = fs.spmm(rp, ci, vals, m, k, b.to(device))
    torch.cuda.synchronize()
    orp, oci, ov = oracle.coo_to_csr(row.numpy(), col.numpy(), v.numpy(), m, k, True)
    ref = oracle.spmm(orp, oci, ov, b.numpy())
    assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    bad_row = row.clone()
    bad_row[7] = m
    with pytest.raises(RuntimeError, match="outside"):
        fs.coo_to_csr(bad_row.to(device), col.to(device), None, m, k)
